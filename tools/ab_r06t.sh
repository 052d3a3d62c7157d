# r06t: fused task + QP kernel above 8 192 instances (DRC_FUSE_MAX) on the current build
set -e
cd $GRAFT_REPO_ROOT
bash tools/env_ab.sh fuse_husky "husky_fr3" "base DRC_FUSE_MAX=16384" 3
bash tools/env_ab.sh fuse_65k "fr3 ur5e xls_fr3 caster_fr3" "base DRC_FUSE_MAX=65536" 2
BENCH_ARGS="--batch 16384" bash tools/env_ab.sh fuse_16k "fr3 ur5e xls_fr3" "base DRC_FUSE_MAX=16384" 2

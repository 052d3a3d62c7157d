# r06y: fused + EPA-first order for manipulator calls of 32 768 / 65 536
set -e
cd $GRAFT_REPO_ROOT
BENCH_ARGS="--batch 32768" bash tools/env_ab.sh man_fuse32k "fr3 ur5e" "base DRC_FUSE_MAX=65536" 2
bash tools/env_ab.sh man_fuse65k "fr3 ur5e" "base DRC_FUSE_MAX=65536" 2

# r06x: UR5e fused (with the EPA-first order) vs pipeline above 8 192
set -e
cd $GRAFT_REPO_ROOT
BENCH_ARGS="--batch 12288" bash tools/env_ab.sh ur5e_fuse12k "ur5e" "base DRC_FUSE_MAX=16384" 2
BENCH_ARGS="--batch 16384" bash tools/env_ab.sh ur5e_fuse16k "ur5e" "base DRC_FUSE_MAX=16384" 2
BENCH_ARGS="--batch 32768" bash tools/env_ab.sh fuse32k "fr3 xls_fr3" "base DRC_FUSE_MAX=32768" 2

# r06v: EPA-first order for fused FR3 / UR5e calls above 8 192 instances
set -e
cd $GRAFT_REPO_ROOT
BENCH_ARGS="--batch 16384" bash tools/env_ab.sh order16k "fr3" "base DRC_ORDER_MAX=16384" 3
BENCH_ARGS="--batch 12288" bash tools/env_ab.sh order12k "fr3" "base DRC_ORDER_MAX=16384" 2

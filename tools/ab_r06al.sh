# r06al: one Ruiz pass in exact mode for the manipulators, on the final build
set -e
cd $GRAFT_REPO_ROOT
bash tools/env_ab.sh scal1 "fr3 ur5e" "base DRC_EXACT_SCALING=1" 3
BENCH_ARGS="--batch 4096" bash tools/env_ab.sh scal1_b4096 "fr3" "base DRC_EXACT_SCALING=1" 3

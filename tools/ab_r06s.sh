# r06s: Husky-FR3 16 384 launch-shape knobs on the current build
set -e
cd $GRAFT_REPO_ROOT
bash tools/env_ab.sh husky_shape "husky_fr3" "base DRC_FUSE_MAX=16384 DRC_TASK_W3=1 DRC_GRID_TASK=1024 DRC_GRID_QP=1024 DRC_MIN_SUBBATCH=8192" 2
BENCH_ARGS="--chunks 2" bash tools/env_ab.sh husky_chunks2 "husky_fr3" "base" 2

# r06aj: task build (two / three waves per SIMD) re-checked on the final grids
set -e
cd $GRAFT_REPO_ROOT
bash tools/env_ab.sh taskw "fr3 ur5e xls_fr3" "base DRC_TASK_W3=0 DRC_TASK_W3=1" 2

# r06af: persistent-grid combinations (QP 3 072 / 4 096 x task 1 024 / 1 536 / 2 048)
set -e
cd $GRAFT_REPO_ROOT
bash tools/env_ab.sh grid2 "fr3 ur5e xls_fr3" "base DRC_GRID_QP=3072,DRC_GRID_TASK=1536 DRC_GRID_QP=4096 DRC_GRID_QP=4096,DRC_GRID_TASK=1536 DRC_GRID_QP=4096,DRC_GRID_TASK=1024" 2

# r06ae: persistent-grid sizes re-swept on the final kernels (B = 65 536)
set -e
cd $GRAFT_REPO_ROOT
bash tools/env_ab.sh grid "fr3 ur5e" "base DRC_GRID_QP=1536 DRC_GRID_QP=3072 DRC_GRID_TASK=1536 DRC_GRID_TASK=3072" 2

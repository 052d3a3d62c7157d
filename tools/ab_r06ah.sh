# r06ah: grid edges beyond the new defaults (QP 6 144 / 8 192, task 512 / 768)
set -e
cd $GRAFT_REPO_ROOT
bash tools/env_ab.sh grid3 "fr3 ur5e caster_fr3" "base DRC_GRID_QP=8192 DRC_GRID_QP=6144 DRC_GRID_TASK=512 DRC_GRID_TASK=768" 2

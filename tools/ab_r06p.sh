# r06p: exact-mode first-polish iteration re-swept after the call-free ADMM loop (iterations ~4x cheaper)
set -e
cd $GRAFT_REPO_ROOT
bash tools/env_ab.sh check_man "fr3 ur5e" "base DRC_EXACT_CHECK=10 DRC_EXACT_CHECK=12 DRC_EXACT_CHECK=16" 2
bash tools/env_ab.sh check_moma "xls_fr3 husky_fr3" "base DRC_EXACT_CHECK=3 DRC_EXACT_CHECK=4" 2

# r06n: QP kernel at 4 waves per SIMD (128 VGPRs) vs 3 (168), after the call-free ADMM loop
set -e
cd $GRAFT_REPO_ROOT
bash tools/ab_bench.sh qw4_exact "libdrc_amd.so libdrc_amd_qw4.so" "fr3 ur5e xls_fr3" 2
BENCH_ARGS="--solver osqp_default" bash tools/ab_bench.sh qw4_ref "libdrc_amd.so libdrc_amd_qw4.so" "fr3" 2

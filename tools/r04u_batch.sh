set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 bash tools/ab_bench.sh r04u_st3 "libdrc_amd.so libdrc_amd_st.so" "fr3 ur5e xls_fr3" 2 || exit 1
BENCH_ARGS="--chunks 4" timeout -k 10 300 bash tools/ab_bench.sh r04u_st4 "libdrc_amd_st.so" "fr3 ur5e xls_fr3" 2 || exit 1

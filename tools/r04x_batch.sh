set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 bash tools/ab_bench.sh r04x_g32 "libdrc_amd.so libdrc_amd_g32.so libdrc_amd_g32w2.so" "fr3 ur5e xls_fr3" 2 || exit 1

set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/lib_bits.py main > gpurun_out/r04roles_bits.log 2>&1 || exit 1
DRC_AMD_LIB=libdrc_amd_roles.so timeout -k 10 300 python3 tools/lib_bits.py roles >> gpurun_out/r04roles_bits.log 2>&1 || exit 1
python3 tools/lib_bits.py --compare main roles >> gpurun_out/r04roles_bits.log 2>&1; tail -5 gpurun_out/r04roles_bits.log
timeout -k 10 600 bash tools/ab_bench.sh r04roles "libdrc_amd.so libdrc_amd_roles.so" "xls_fr3 fr3 ur5e" 2 || exit 1

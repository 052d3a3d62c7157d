set -o pipefail
mkdir -p gpurun_out
timeout -k 10 250 python3 tools/check_sweep.py fr3 long > gpurun_out/r04h_long_fr3.jsonl 2>&1 || exit 1
timeout -k 10 250 python3 tools/check_sweep.py fr3 scaling > gpurun_out/r04h_scaling_fr3.jsonl 2>&1 || exit 1
timeout -k 10 500 bash tools/ab_bench.sh r04h_inl "libdrc_amd.so libdrc_amd_inl.so" "fr3 ur5e xls_fr3" 2 || exit 1
timeout -k 10 200 bash tools/pmc_pass.sh r04h_base || exit 1
DRC_AMD_LIB=libdrc_amd_inl.so timeout -k 10 200 bash tools/pmc_pass.sh r04h_inl || exit 1
cat gpurun_out/r04h_*.jsonl

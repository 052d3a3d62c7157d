set -o pipefail
mkdir -p gpurun_out
# where the final build's extra writes come from: the pre-Ruiz build (two-wave FR3 task kernel) and the final
# build with the two-wave task build forced
DRC_AMD_LIB=libdrc_amd_base.so timeout -k 10 300 bash tools/pmc_pass.sh r04p_base --robot fr3 || exit 1
DRC_TASK_W3=0 timeout -k 10 300 bash tools/pmc_pass.sh r04p_w2 --robot fr3 || exit 1
# the bench line of the final build with its committed same-build summaries
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extras > gpurun_out/r04p_bench_fr3.json 2> gpurun_out/r04p_bench_fr3.err || exit 1
cut -c1-400 gpurun_out/r04p_bench_fr3.json
DRC_AMD_LIB=libdrc_amd_ws.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r04q_ws.log 2>&1
rc=$?; tail -3 gpurun_out/gputest_r04q_ws.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/lib_bits.py final > gpurun_out/r04q_bits.log 2>&1 || exit 1
DRC_AMD_LIB=libdrc_amd_ws.so timeout -k 10 300 python3 tools/lib_bits.py ws >> gpurun_out/r04q_bits.log 2>&1 || exit 1
python3 tools/lib_bits.py --compare final ws >> gpurun_out/r04q_bits.log 2>&1; tail -5 gpurun_out/r04q_bits.log
timeout -k 10 600 bash tools/ab_bench.sh r04q_ws "libdrc_amd.so libdrc_amd_ws.so" "fr3 ur5e xls_fr3" 2 || exit 1

set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r04j.log 2>&1
rc=$?; tail -3 gpurun_out/gputest_r04j.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash tools/ab_bench.sh r04j_lds "libdrc_amd_ldsb.so libdrc_amd.so libdrc_amd_t3.so" "fr3 ur5e xls_fr3 husky_fr3" 3 || exit 1
timeout -k 10 120 python3 tools/phase_timing.py fr3 > gpurun_out/r04j_phase_fr3.txt 2>&1 || exit 1
timeout -k 10 120 python3 tools/phase_timing.py ur5e > gpurun_out/r04j_phase_ur5e.txt 2>&1 || exit 1

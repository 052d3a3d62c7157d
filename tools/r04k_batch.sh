set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > gpurun_out/gputest_r04k.log 2>&1
rc=$?; tail -3 gpurun_out/gputest_r04k.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash tools/ab_bench.sh r04k_w3 "libdrc_amd_ldsb.so libdrc_amd.so" "ur5e fr3 caster_fr3" 3 || exit 1
timeout -k 10 60 rocprofv3 -L > gpurun_out/r04k_rocprof_L.txt 2>&1 || true

set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r04m.log 2>&1
rc=$?; tail -3 gpurun_out/gputest_r04m.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash tools/ab_bench.sh r04m_ruiz "libdrc_amd_base.so libdrc_amd.so" "fr3 xls_fr3 ur5e husky_fr3" 3 || exit 1

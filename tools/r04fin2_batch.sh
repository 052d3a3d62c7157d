set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r04fin2.log 2>&1
rc=$?; tail -3 gpurun_out/gputest_r04fin2.log; [ $rc -eq 0 ] || exit $rc
bash tools/final_round.sh r04end fr3 ur5e husky_fr3

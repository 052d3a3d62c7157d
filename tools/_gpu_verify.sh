set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/v_pytest.log 2>&1; rc=$?; echo "pytest rc $rc"; tail -3 gpurun_out/v_pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py > gpurun_out/v_bench.json 2> gpurun_out/v_bench.err; echo "bench rc $?"; cat gpurun_out/v_bench.json

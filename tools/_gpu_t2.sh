set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t2_pytest.log 2>&1; rc=$?
echo "all pytest rc $rc"; tail -25 gpurun_out/t2_pytest.log | grep -E "passed|failed|Error|assert|FAIL" | head -20

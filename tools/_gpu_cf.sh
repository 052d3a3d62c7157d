set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_closed_form.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/cf_pytest.log 2>&1; rc=$?
echo "cf pytest rc $rc"; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/cf_pytest.log | head -30

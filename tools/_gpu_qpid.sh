set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_qpid.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/qpid_pytest.log 2>&1; rc=$?
echo "qpid pytest rc $rc"; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/qpid_pytest.log | head -30
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/all_pytest.log 2>&1; rc=$?
echo "all pytest rc $rc"; tail -3 gpurun_out/all_pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/q_bench.json 2> gpurun_out/q_bench.err; echo "bench rc $?"; python -c "
import json; d=json.load(open('gpurun_out/q_bench.json')); r=d['roofline']
print('value %.4g ms %.3f task %.3f qp %.3f' % (d['value'], d['ms_per_step'], r['task_kernel_ms_sum'], r['qp_kernel_ms_sum']))"

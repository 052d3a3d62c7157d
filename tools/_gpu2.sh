set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q -s > gpurun_out/t4_pytest.log 2>&1; echo "pytest rc $?"; grep -E "instances outside|passed|failed|Error" gpurun_out/t4_pytest.log | head
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/t4_bench.json 2> gpurun_out/t4_bench.err && python -c "
import json; d=json.load(open('gpurun_out/t4_bench.json')); r=d['roofline']
print('value %.4g ms/step %.3f task %.3f qp %.3f iters %.1f nonsolved %d' % (d['value'], d['ms_per_step'], r['task_kernel_ms_sum'], r['qp_kernel_ms_sum'], d['admm_iters_mean'], d['non_solved']))"

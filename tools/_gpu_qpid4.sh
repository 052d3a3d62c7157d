set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/all_pytest.log 2>&1; rc=$?
echo "all pytest rc $rc"; tail -3 gpurun_out/all_pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u tools/bench_qpid.py --cpu 0 --steps 5 > gpurun_out/bq5.jsonl 2> gpurun_out/bq5.err; echo "bench rc $?"; cut -c1-130,300-520 gpurun_out/bq5.jsonl
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b5.json 2> gpurun_out/b5.err; echo "bench rc $?"; python -c "
import json; d=json.load(open('gpurun_out/b5.json')); r=d['roofline']
print('value %.4g ms %.3f task %.3f qp %.3f iters %.2f' % (d['value'], d['ms_per_step'], r['task_kernel_ms_sum'], r['qp_kernel_ms_sum'], d['admm_iters_mean']))"

cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/t6.log 2>&1; echo "pytest rc $?"; tail -1 gpurun_out/t6.log
for c in 1 2 4; do
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --chunks $c > gpurun_out/c$c.json 2>/dev/null && python -c "
import json; d=json.load(open('gpurun_out/c$c.json')); r=d['roofline']
print('chunks $c value %.4g ms/step %.3f call %.3f task_sum %.3f qp_sum %.3f' % (d['value'], d['ms_per_step'], r['kernel_ms'], r['task_kernel_ms_sum'], r['qp_kernel_ms_sum']))"
done

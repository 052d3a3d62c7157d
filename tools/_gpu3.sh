cd $GRAFT_REPO_ROOT
for g in 2048 4096 8192 16384; do
  DRC_TASK_GRID=$g timeout -k 10 120 python bench.py --no-cpu-baseline --steps 5 > gpurun_out/g$g.json 2>/dev/null && python -c "
import json; d=json.load(open('gpurun_out/g$g.json')); r=d['roofline']
print('grid $g value %.4g task %.3f qp %.3f' % (d['value'], r['task_kernel_ms'], r['qp_kernel_ms']))"
done

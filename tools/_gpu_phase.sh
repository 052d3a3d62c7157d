cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b6.json 2> gpurun_out/b6.err; echo "bench rc $?"; python -c "
import json; d=json.load(open('gpurun_out/b6.json')); r=d['roofline']
print('value %.4g ms %.3f task %.3f qp %.3f iters %.2f tail %s' % (d['value'], d['ms_per_step'], r['task_kernel_ms_sum'], r['qp_kernel_ms_sum'], d['admm_iters_mean'], d['admm_iters_p99_max']))"
timeout -k 10 300 python tools/phase_timing.py fr3 65536 > gpurun_out/phase.log 2>&1; echo "phase rc $?"; cat gpurun_out/phase.log | grep -v amdgpu.ids

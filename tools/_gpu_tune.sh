set -o pipefail
# Sweep: concurrent sub-batches (product library) and task-kernel occupancy builds.
cd $GRAFT_REPO_ROOT
run() {  # lib chunks
  DRC_AMD_LIB=$1 timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --chunks $2 > gpurun_out/tune_$1_$2.json 2>gpurun_out/tune_$1_$2.err || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/tune_$1_$2.json')); r=d['roofline']
print('$1 chunks $2 value %.4g ms %.3f task_sum %.3f qp_sum %.3f' % (d['value'], d['ms_per_step'], r['task_kernel_ms_sum'], r['qp_kernel_ms_sum']))"
}
for c in 2 3 4 5 6 8; do run libdrc_amd.so $c; done
for w in 1 3 4; do run libdrc_amd_w$w.so 3; done

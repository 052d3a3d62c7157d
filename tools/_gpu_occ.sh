set -o pipefail
cd $GRAFT_REPO_ROOT
for v in libdrc_amd.so libdrc_amd_t2q1.so libdrc_amd_t1q1.so; do
DRC_AMD_LIB=$v timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/occ_$v.json 2>gpurun_out/occ_$v.err || exit 1
python -c "
import json; d=json.load(open('gpurun_out/occ_$v.json')); r=d['roofline']
print('$v value %.4g ms %.3f task_sum %.3f qp_sum %.3f' % (d['value'], d['ms_per_step'], r['task_kernel_ms_sum'], r['qp_kernel_ms_sum']))"
done

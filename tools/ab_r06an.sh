# r06an: fused task record inside the task plan's dead overlay region (whole-body fused plans: 8 waves per CU)
set -e
cd $GRAFT_REPO_ROOT
export DRC_BITS_DIR=/tmp/bits; mkdir -p $DRC_BITS_DIR
for v in base new; do lib=libdrc_amd_$v.so; [ $v = new ] && lib=libdrc_amd.so; DRC_AMD_LIB=$lib timeout -k 10 300 python3 -u tools/lib_bits.py $v husky_fr3; done
python3 tools/lib_bits.py --compare base new husky_fr3
timeout -k 10 300 python -u -m pytest tests/test_gpu_cycle.py -k lds_plan -m gpu -q -s --timeout 120 --timeout-method thread 2>&1 | grep 'task'
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_fullsize.py tests/test_gpu_golden.py tests/test_gpu_order.py tests/test_gpu_moma.py -m gpu -q --timeout 200 --timeout-method thread 2>&1 | tail -1
bash tools/ab_bench.sh fusedrec "libdrc_amd_base.so libdrc_amd.so" "husky_fr3" 3
BENCH_ARGS="--batch 16384" bash tools/ab_bench.sh fusedrec16k "libdrc_amd_base.so libdrc_amd.so" "xls_fr3" 2

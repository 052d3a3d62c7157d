# r06ak: 8-bit EPA vertex / free-list slots (UR5e task plan 14 000 -> 13 488 B: 12 waves per CU): bits, A/B, LDS plans
set -e
cd $GRAFT_REPO_ROOT
export DRC_BITS_DIR=/tmp/bits; mkdir -p $DRC_BITS_DIR
R="fr3 ur5e husky_fr3 xls_fr3 caster_fr3"
for v in base new; do lib=libdrc_amd_$v.so; [ $v = new ] && lib=libdrc_amd.so; DRC_AMD_LIB=$lib timeout -k 10 300 python3 -u tools/lib_bits.py $v $R; done
python3 tools/lib_bits.py --compare base new $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_cycle.py -k lds_plan -m gpu -q -s --timeout 120 --timeout-method thread 2>&1 | grep 'task'
timeout -k 10 300 python -u -m pytest tests/test_gpu_narrow.py tests/test_gpu_many_candidates.py -m gpu -q --timeout 200 --timeout-method thread 2>&1 | tail -1
bash tools/ab_bench.sh epa8 "libdrc_amd_base.so libdrc_amd.so" "ur5e fr3" 3

# r06o: register EQP setup / pivot scaling stop at the KKT size N; then the GPU suite and the bench line
set -e
cd $GRAFT_REPO_ROOT
export DRC_BITS_DIR=/tmp/bits; mkdir -p $DRC_BITS_DIR
R="fr3 ur5e husky_fr3 xls_fr3 caster_fr3"
for v in base new; do lib=libdrc_amd_$v.so; [ $v = new ] && lib=libdrc_amd.so; DRC_AMD_LIB=$lib timeout -k 10 300 python3 -u tools/lib_bits.py $v $R; done
python3 tools/lib_bits.py --compare base new $R
bash tools/ab_bench.sh eqpn_exact "libdrc_amd_base.so libdrc_amd.so" "fr3 ur5e" 2
bash tools/gpu_suite.sh r06o

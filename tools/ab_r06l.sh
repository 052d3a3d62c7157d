# r06l: ADMM iterations as a call-free loop between checks (leaf = out of line, inl = inlined) vs the HEAD build
set -e
cd $GRAFT_REPO_ROOT
export DRC_BITS_DIR=/tmp/bits; mkdir -p $DRC_BITS_DIR
R="fr3 ur5e husky_fr3 xls_fr3 caster_fr3"
for v in base leaf inl; do DRC_AMD_LIB=libdrc_amd_$v.so timeout -k 10 300 python3 -u tools/lib_bits.py $v $R; done
python3 tools/lib_bits.py --compare base leaf $R
python3 tools/lib_bits.py --compare base inl $R
for v in base inl; do DRC_SOLVER=osqp_default DRC_AMD_LIB=libdrc_amd_$v.so timeout -k 10 300 python3 -u tools/lib_bits.py ref$v fr3 ur5e xls_fr3; done
python3 tools/lib_bits.py --compare refbase refinl fr3 ur5e xls_fr3
bash tools/ab_bench.sh leaf_exact "libdrc_amd_base.so libdrc_amd_leaf.so libdrc_amd_inl.so" "fr3 ur5e xls_fr3" 2
BENCH_ARGS="--solver osqp_default" bash tools/ab_bench.sh leaf_ref "libdrc_amd_base.so libdrc_amd_leaf.so libdrc_amd_inl.so" "fr3 ur5e" 2

# r06m: mixed build (iterations inlined in exact mode, out of line in reference mode) vs the HEAD build
set -e
cd $GRAFT_REPO_ROOT
export DRC_BITS_DIR=/tmp/bits; mkdir -p $DRC_BITS_DIR
R="fr3 ur5e husky_fr3 xls_fr3 caster_fr3"
for v in base mix; do DRC_AMD_LIB=libdrc_amd_$v.so timeout -k 10 300 python3 -u tools/lib_bits.py $v $R; done
python3 tools/lib_bits.py --compare base mix $R
for v in base mix; do DRC_SOLVER=osqp_default DRC_AMD_LIB=libdrc_amd_$v.so timeout -k 10 300 python3 -u tools/lib_bits.py ref$v fr3 ur5e xls_fr3; done
python3 tools/lib_bits.py --compare refbase refmix fr3 ur5e xls_fr3
bash tools/ab_bench.sh mix_exact "libdrc_amd_base.so libdrc_amd_inl.so libdrc_amd_mix.so" "fr3 ur5e xls_fr3 husky_fr3" 2
BENCH_ARGS="--solver osqp_default" bash tools/ab_bench.sh mix_ref "libdrc_amd_base.so libdrc_amd_mix.so" "fr3 ur5e" 2
timeout -k 10 200 python3 tools/phase_timing.py fr3 > gpurun_out/r06m_phase_fr3.txt 2>&1
DRC_SOLVER=osqp_default timeout -k 10 200 python3 tools/phase_timing.py fr3 > gpurun_out/r06m_phase_fr3_reference_mode.txt 2>&1

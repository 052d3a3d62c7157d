# r06ap / r06aq: EQP loops (register Gauss-Jordan, range-space Schur) run a
# fixed trip count with a uniform skip past N instead of a break, so they fully
# unroll and the Ki / K0 register rows are indexed by constants (no
# s_set_gpr_idx moves).  r06ap also unrolled the polish / EQP right-hand-side
# loops over a G row (skip past the slack columns): bit-identical, FR3 -4.9 %
# (profiles/r06ap_ab_eqp_unroll.jsonl); r06aq (TAG=eqpunroll_only) is the EQP
# loops alone.
# One call: bits against the previous build on every robot, targeted GPU tests,
# A/B throughput; then (only if the new build is bit-identical and not slower)
# the GPU suite, the FR3 profile round and the FR3 SQ counters of the new build.
set -e -o pipefail
cd $GRAFT_REPO_ROOT
export DRC_BITS_DIR=/tmp/bits; mkdir -p $DRC_BITS_DIR
for v in base new; do lib=libdrc_amd_$v.so; [ $v = new ] && lib=libdrc_amd.so; DRC_AMD_LIB=$lib timeout -k 10 300 python3 -u tools/lib_bits.py $v; done
python3 tools/lib_bits.py --compare base new | tee gpurun_out/bits_${TAG:-eqpunroll}.txt
for v in base new; do lib=libdrc_amd_$v.so; [ $v = new ] && lib=libdrc_amd.so; DRC_SOLVER=osqp_default DRC_AMD_LIB=$lib timeout -k 10 300 python3 -u tools/lib_bits.py ref_$v fr3; done
python3 tools/lib_bits.py --compare ref_base ref_new fr3 | tee -a gpurun_out/bits_${TAG:-eqpunroll}.txt
bash tools/ab_bench.sh ${TAG:-eqpunroll} "libdrc_amd_base.so libdrc_amd.so" "fr3 ur5e xls_fr3" 1
python3 - <<'PY'
import json, sys
rows = [json.loads(l) for l in open("gpurun_out/ab_%s.jsonl" % __import__("os").environ.get("TAG", "eqpunroll"))]
v = {(r["robot"], r["lib"]): r["value"] for r in rows}
for rb in ("fr3", "ur5e", "xls_fr3"):
    a, b = v[(rb, "libdrc_amd_base.so")], v[(rb, "libdrc_amd.so")]
    print(rb, "%.3f -> %.3f M (%+.1f %%)" % (a / 1e6, b / 1e6, 100 * (b / a - 1)))
if v[("fr3", "libdrc_amd.so")] < 1.005 * v[("fr3", "libdrc_amd_base.so")] or \
   v[("ur5e", "libdrc_amd.so")] < v[("ur5e", "libdrc_amd_base.so")]:
    sys.exit("new build not faster: stop")
PY
bash tools/gpu_suite.sh r06fin6 > gpurun_out/suite_r06fin6.log 2>&1 || { tail -20 gpurun_out/suite_r06fin6.log; exit 1; }
tail -3 gpurun_out/gputest_r06fin6.log
bash tools/final_round.sh r06fin6 fr3
timeout -k 10 400 bash tools/sq_pass.sh r06fin6_fr3 > gpurun_out/sq_r06fin6.log 2>&1
echo "sq done"

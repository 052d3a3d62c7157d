#!/bin/bash
# One GPU lease, a sequence of steps (replaces the per-iteration batch files):
#   bash tools/lease.sh <tag> <step> [<step> ...]
# Steps (each under its own time limit; the first failure ends the lease):
#   test[:<k expr>]            pytest -m gpu [-k expr, commas become spaces] (gpurun_out/gputest_<tag>.log)
#   smoke                      __graft_entry__.smoke()
#   bench:<robot>[,<robot>]    one bench line per robot, no CPU baseline (tools/gpu_check.sh's summary)
#   line[:<args>]              the default bench line (with CPU baseline), extra bench.py args after ':'
#                              (commas become spaces), into gpurun_out/line_<tag>.json
#   ab:<lib>,<lib>:<robot>,<robot>[:reps]   library A/B (tools/ab_bench.sh)
#   env:<E=V+E2=V>,base:<robot>,..[:reps]   environment A/B (tools/env_ab.sh; '+' joins variables)
#   bits:<lib>,<lib>           bit-for-bit comparison of two builds on all five robots (tools/lib_bits.py)
#   phase:<robot>[,<batch>]    DRC_PHASE_TIMING build's phase shares (tools/phase_timing.py)
#   gpus2                      two-rank rehearsal on the one GPU (gloo), gpurun_out/gpus2_<tag>.json
#   gpus:<n>[:<args>]          n-rank gloo rehearsal on the one GPU, extra bench.py args (commas become spaces)
#   final[:<robot>,..]         round-end measurement (tools/final_round.sh)
#   refcensus[:bench]          reference-settings census (tools/reference_census.py [--bench])
#   stamps:<robot>:<batch>[:<fusion>[:<concurrency>]]  small-batch makespan study (tools/stamp_study.py)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $ROOT
TAG=$1; shift
mkdir -p gpurun_out
summ() {
  python3 - "$1" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); ro = d["roofline"]
print(d["config"]["robot"], "B", d["config"].get("batch_per_gpu"), "%.3fM" % (d["value"] / 1e6), "ms",
      round(d["ms_per_step"], 3), "task", round(ro["task_kernel_ms_sum"], 3), "qp", round(ro["qp_kernel_ms_sum"], 3),
      "nonsolved", d["non_solved"], "iters", round(d["admm_iters_mean"], 3), d["admm_iters_p99_max"])
for k in ("reference_settings", "batch_4096", "latency_b1", "latency_cycle"):
    if k in d:
        v = d[k]
        print("  %s: %s" % (k, {a: v[a] for a in v if a in ("value", "non_solved", "admm_iters_p99_max", "p50_us",
                                                             "p99_us", "max_us", "ms_per_call")}))
PY
}
for step in "$@"; do
  kind=${step%%:*}; rest=${step#*:}; [ "$rest" = "$step" ] && rest=""
  echo "== $step"
  case $kind in
    test)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
        ${rest:+-k "${rest//,/ }"} > gpurun_out/gputest_$TAG.log 2>&1
      rc=$?; tail -3 gpurun_out/gputest_$TAG.log; [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 \
        || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
      tail -2 gpurun_out/smoke_$TAG.log ;;
    bench)
      for r in ${rest//,/ }; do
        timeout -k 10 300 python3 bench.py --no-cpu-baseline --robot $r > gpurun_out/bench_${TAG}_$r.json \
          2> gpurun_out/bench_${TAG}_$r.err || { tail -5 gpurun_out/bench_${TAG}_$r.err; exit 1; }
        summ gpurun_out/bench_${TAG}_$r.json
      done ;;
    line)
      timeout -k 10 400 python3 bench.py ${rest//,/ } > gpurun_out/line_$TAG.json 2> gpurun_out/line_$TAG.err \
        || { tail -5 gpurun_out/line_$TAG.err; exit 1; }
      summ gpurun_out/line_$TAG.json ;;
    ab)
      IFS=: read -r libs robots reps <<< "$rest"
      timeout -k 10 900 bash tools/ab_bench.sh $TAG "${libs//,/ }" "${robots//,/ }" ${reps:-2} || exit 1 ;;
    env)
      IFS=: read -r envs robots reps <<< "$rest"
      e=${envs//,/ }
      timeout -k 10 900 bash tools/env_ab.sh $TAG "${robots//,/ }" "${e//+/,}" ${reps:-2} || exit 1 ;;
    bits)
      IFS=, read -r la lb <<< "$rest"
      DRC_AMD_LIB=$la timeout -k 10 300 python3 tools/lib_bits.py ${TAG}_a > gpurun_out/bits_$TAG.log 2>&1 || exit 1
      DRC_AMD_LIB=$lb timeout -k 10 300 python3 tools/lib_bits.py ${TAG}_b >> gpurun_out/bits_$TAG.log 2>&1 || exit 1
      python3 tools/lib_bits.py --compare ${TAG}_a ${TAG}_b >> gpurun_out/bits_$TAG.log 2>&1
      tail -6 gpurun_out/bits_$TAG.log ;;
    phase)
      timeout -k 10 300 python3 tools/phase_timing.py ${rest//,/ } > gpurun_out/phase_${TAG}_${rest//,/_}.txt 2>&1 || exit 1
      cat gpurun_out/phase_${TAG}_${rest//,/_}.txt ;;
    gpus2)
      DRC_DIST_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline \
        > gpurun_out/gpus2_$TAG.json 2> gpurun_out/gpus2_$TAG.err || { tail -5 gpurun_out/gpus2_$TAG.err; exit 1; }
      grep -h '^{' gpurun_out/gpus2_$TAG.json | cut -c1-240 ;;
    gpus)
      IFS=: read -r n args <<< "$rest"
      DRC_DIST_BACKEND=gloo timeout -k 10 600 python3 bench.py --gpus $n --steps 5 --warmup 2 --no-cpu-baseline ${args//,/ } \
        > gpurun_out/gpus${n}_$TAG.json 2> gpurun_out/gpus${n}_$TAG.err || { tail -5 gpurun_out/gpus${n}_$TAG.err; exit 1; }
      grep -h '^{' gpurun_out/gpus${n}_$TAG.json | cut -c1-300 ;;
    final)
      timeout -k 10 3000 bash tools/final_round.sh $TAG ${rest//,/ } || exit 1 ;;
    refcensus)
      timeout -k 10 600 python3 -u tools/reference_census.py ${rest:+--$rest} > gpurun_out/refcensus_$TAG$rest.log 2>&1 \
        || { tail -20 gpurun_out/refcensus_$TAG$rest.log; exit 1; }
      cut -c1-400 gpurun_out/refcensus_$TAG$rest.log ;;
    stamps)
      IFS=: read -r robot batch fz cc <<< "$rest"
      timeout -k 10 300 python3 tools/stamp_study.py --robot $robot --batch $batch --fusion ${fz:--1} \
        --concurrency ${cc:-0} >> gpurun_out/stamps_$TAG.jsonl 2> gpurun_out/stamps_$TAG.err \
        || { tail -5 gpurun_out/stamps_$TAG.err; exit 1; }
      tail -3 gpurun_out/stamps_$TAG.jsonl | cut -c1-1500 ;;
    *) echo "lease.sh: unknown step $step" >&2; exit 2 ;;
  esac
done

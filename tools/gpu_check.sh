#!/bin/bash
# GPU-box iteration check: the -m gpu suite, then one bench line per robot
# (no CPU baseline) summarised.  usage: bash tools/gpu_check.sh <tag> robot...
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $ROOT
TAG=$1; shift
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/gputest_$TAG.log
[ $rc -eq 0 ] || exit $rc
for r in "$@"; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --robot $r > gpurun_out/bench_${TAG}_$r.json 2> gpurun_out/bench_${TAG}_$r.err || exit 1
  python3 - gpurun_out/bench_${TAG}_$r.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); ro = d["roofline"]
print(d["config"]["robot"], "%.3fM" % (d["value"] / 1e6), "ms", round(d["ms_per_step"], 3), "task",
      round(ro["task_kernel_ms_sum"], 3), "qp", round(ro["qp_kernel_ms_sum"], 3), "nonsolved", d["non_solved"],
      "iters", round(d["admm_iters_mean"], 3), d["admm_iters_p99_max"])
if "latency_b1" in d:
    rs, sb, lb, lr = d["reference_settings"], d["batch_4096"], d["latency_b1"], ro["latency_roof"]
    print("  osqp_default %.3fM nonsolved %d iters %s | B=4096 %.3fM | B=1 p50 %.0f us p99 %.0f us | "
          "instance latency %.0f us, roof %.2fM (frac %.2f)" % (rs["value"] / 1e6, rs["non_solved"],
          rs["admm_iters_p99_max"], sb["value"] / 1e6, lb["p50_us"], lb["p99_us"], lr["instance_latency_us"],
          lr["solves_per_s"] / 1e6, lr["frac"]))
PY
done

#!/bin/bash
# A/B throughput of library variants on one box (DRC_AMD_LIB selects the .so):
#   bash tools/ab_bench.sh <tag> "<lib1> <lib2> ..." "<robot1> <robot2> ..." [reps]
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $ROOT
TAG=$1; LIBS=$2; ROBOTS=$3; REPS=${4:-2}
mkdir -p gpurun_out
out=gpurun_out/ab_$TAG.jsonl
: > $out
for rep in $(seq $REPS); do
  for r in $ROBOTS; do
    for lib in $LIBS; do
      DRC_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-extras --robot $r --steps 20 --warmup 5 $BENCH_ARGS \
        > gpurun_out/ab_tmp.json 2> gpurun_out/ab_tmp.err || { tail -5 gpurun_out/ab_tmp.err; exit 1; }
      python3 - "$lib" "$r" gpurun_out/ab_tmp.json >> $out <<'PY'
import json, sys
d = json.load(open(sys.argv[3])); ro = d["roofline"]
print(json.dumps({"lib": sys.argv[1], "robot": sys.argv[2], "value": d["value"], "task": ro["task_kernel_ms_sum"],
                  "qp": ro["qp_kernel_ms_sum"], "ms": d["ms_per_step"]}))
PY
    done
  done
done
python3 - $out <<'PY'
import json, sys, collections
rows = [json.loads(l) for l in open(sys.argv[1])]
agg = collections.defaultdict(list)
for r in rows: agg[(r["robot"], r["lib"])].append(r)
for (rb, lib), rs in sorted(agg.items()):
    print(rb, lib, "%.3fM" % (max(x["value"] for x in rs) / 1e6), "task %.3f qp %.3f" % (min(x["task"] for x in rs), min(x["qp"] for x in rs)))
PY

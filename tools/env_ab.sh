#!/bin/bash
# A/B throughput of environment settings on one box:
#   bash tools/env_ab.sh <tag> "<robot> ..." "<ENV=VAL,ENV2=VAL>|base ..." [reps]
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $ROOT
TAG=$1; ROBOTS=$2; ENVS=$3; REPS=${4:-2}
mkdir -p gpurun_out
out=gpurun_out/envab_$TAG.jsonl
: > $out
for rep in $(seq $REPS); do
  for r in $ROBOTS; do
    for e in $ENVS; do
      envs=""; [ "$e" != base ] && envs=$(echo $e | tr ',' ' ')
      env $envs timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-extras --robot $r --steps 20 --warmup 5 $BENCH_ARGS \
        > gpurun_out/envab_tmp.json 2> gpurun_out/envab_tmp.err || { tail -5 gpurun_out/envab_tmp.err; exit 1; }
      python3 - "$e" "$r" gpurun_out/envab_tmp.json >> $out <<'PY'
import json, sys
d = json.load(open(sys.argv[3])); ro = d["roofline"]
print(json.dumps({"env": sys.argv[1], "robot": sys.argv[2], "value": d["value"], "task": ro["task_kernel_ms_sum"],
                  "qp": ro["qp_kernel_ms_sum"], "ms": d["ms_per_step"]}))
PY
    done
  done
done
python3 - $out <<'PY'
import json, sys, collections
rows = [json.loads(l) for l in open(sys.argv[1])]
agg = collections.defaultdict(list)
for r in rows: agg[(r["robot"], r["env"])].append(r)
for (rb, e), rs in sorted(agg.items()):
    print(rb, e, "%.3fM" % (max(x["value"] for x in rs) / 1e6), "ms %.3f" % min(x["ms"] for x in rs))
PY

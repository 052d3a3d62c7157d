#!/bin/bash
# Launch-shape sweep of the two-kernel pipeline on one box: persistent grid
# sizes (DRC_GRID_TASK / DRC_GRID_QP) and concurrent sub-batches (--chunks).
#   bash tools/launch_sweep.sh <tag> <robot>   -> gpurun_out/sweep_<tag>.jsonl
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $ROOT
TAG=$1; R=${2:-fr3}
out=gpurun_out/sweep_$TAG.jsonl
: > $out
for cfg in "2048 2048 3" "4096 2048 3" "2048 4096 3" "4096 4096 3" "2048 2048 2" "2048 2048 4" "1024 2048 3" "2048 1024 3"; do
  set -- $cfg
  DRC_GRID_TASK=$1 DRC_GRID_QP=$2 timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-extras --robot $R --steps 20 --warmup 5 --chunks $3 \
    > gpurun_out/sweep_tmp.json 2> gpurun_out/sweep_tmp.err || { tail -3 gpurun_out/sweep_tmp.err; exit 1; }
  python3 -c "
import json,sys; d=json.load(open('gpurun_out/sweep_tmp.json'))
print(json.dumps({'grid_task': $1, 'grid_qp': $2, 'chunks': $3, 'robot': '$R', 'value': d['value']}))" >> $out
  tail -1 $out
done

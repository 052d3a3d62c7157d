#!/bin/bash
# Library A/B at one batch size (FR3 unless --robot is among the extra args):
#   bash tools/ab_batch.sh <tag> <libA> <libB> <reps> [bench args...]
# one JSON summary line per run into gpurun_out/abb_<tag>.jsonl
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $ROOT
TAG=$1; LA=$2; LB=$3; REPS=$4; shift 4
for r in $(seq $REPS); do
  for lib in $LA $LB; do
    DRC_AMD_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extras "$@" > gpurun_out/abb_tmp.json 2> gpurun_out/abb_tmp.err \
      || { tail -5 gpurun_out/abb_tmp.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('gpurun_out/abb_tmp.json').read().strip().splitlines()[-1])
print(json.dumps({'lib': '$lib', 'args': '$*', 'value': d['value'], 'ms_per_step': d['ms_per_step']}))" | tee -a gpurun_out/abb_$TAG.jsonl
  done
done

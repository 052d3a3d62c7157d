#!/bin/bash
# Instruction-fetch counters per kernel over a short bench run (one rocprofv3
# --pmc pass per group):  bash tools/icache_pass.sh <tag> [bench args...]
set -e -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
OUT=$ROOT/gpurun_out/ic_$TAG
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
A="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ"
B="SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY"
i=0
for G in "$A" "$B"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $G -f csv -d $OUT/p$i -o p$i -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras "$@" > $OUT/p$i.log 2>&1
  echo "pass $i done"
done

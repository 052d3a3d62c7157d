#!/bin/bash
# SQ counter passes (instruction mix and stall split per kernel) over a short
# bench run; one rocprofv3 --pmc pass per counter group (<= 8 SQ counters).
#   usage: bash tools/sq_pass.sh <tag> [bench args...]
set -e -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
OUT=$ROOT/gpurun_out/sq_$TAG
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
B="SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS"
i=0
for G in "$A" "$B"; do
  i=$((i+1))
  timeout -k 10 150 rocprofv3 --pmc $G -f csv -d $OUT/p$i -o p$i -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras "$@" > $OUT/p$i.log 2>&1
  echo "pass $i done"
done

#!/bin/bash
# FP64 VALU counter passes (SQ block, <= 8 counters per rocprofv3 --pmc run)
# over a short bench run, for tools/valu_summary.py.
#   usage: bash tools/valu_pass.sh <tag> [bench args...]
set -e -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
OUT=$ROOT/gpurun_out/valu_$TAG
mkdir -p $OUT
# the library build these counters belong to (drc_build_id; no GPU call)
python3 -c "import sys; sys.path.insert(0, '$ROOT'); from dyros_robot_controller_amd import _capi; print(_capi.build_id())" > $OUT/build_id
cd /tmp
export TMPDIR=/tmp
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS"
B="SQ_WAVES SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY"
i=0
for G in "$A" "$B"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $G -f csv -d $OUT/p$i -o p$i -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras "$@" > $OUT/p$i.log 2>&1
  echo "valu pass $i done"
done

#!/bin/bash
# WRITE_SIZE per task / QP dispatch against the persistent grid size (per-wave
# prologue spills scale with the grid, per-instance spills do not).
set -e -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/wgrid
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
for g in 1024 2048 4096; do
  DRC_GRID_TASK=$g DRC_GRID_QP=$g timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/g$g -o w -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras "$@" > $OUT/g$g.log 2>&1
  echo "grid $g done"
done

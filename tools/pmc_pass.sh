#!/bin/bash
# FETCH_SIZE and WRITE_SIZE passes (separate rocprofv3 runs) over a short
# bench run, for tools/pmc_summary.py-style summaries of a library variant.
#   usage: DRC_AMD_LIB=<lib> bash tools/pmc_pass.sh <tag> [bench args...]
set -e -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C -f csv -d $OUT/$C -o $C -- python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras "$@" > $OUT/$C.log 2>&1
  echo "pmc $C done"
done

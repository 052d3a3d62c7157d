#!/bin/bash
# Cache-hierarchy counters per kernel over a short bench run (one rocprofv3
# --pmc pass per group): scalar data cache, vector L1, L2.
#   bash tools/cache_pass.sh <tag> [bench args...]  -> gpurun_out/cache_<tag>/
set -e -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
OUT=$ROOT/gpurun_out/cache_$TAG
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
i=0
for G in "SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_MISSES_DUPLICATE" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $G -f csv -d $OUT/p$i -o p$i -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras "$@" > $OUT/p$i.log 2>&1
  echo "cache pass $i done"
done

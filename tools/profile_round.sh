#!/bin/bash
# GPU-box profiling pass for one round: bench line, rocprofv3 kernel-trace
# stats, and the two PMC passes (FETCH_SIZE, WRITE_SIZE: they do not fit in
# one pass on gfx950).  Summaries land in gpurun_out/prof_<tag>/; run
# tools/pmc_summary.py on them afterwards to produce profiles/<tag>_*.
#   usage: bash tools/profile_round.sh <tag> [bench args...]
set -e -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
ARGS="$@"
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 420 python3 bench.py $ARGS > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
cd /tmp
export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats -f csv -d $OUT/kt -o kt -- python3 $ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras $ARGS > $OUT/kt.log 2>&1
echo "kernel trace done"
timeout -k 10 420 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/fetch -o fetch -- python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras $ARGS > $OUT/fetch.log 2>&1
echo "fetch pass done"
timeout -k 10 420 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/write -o write -- python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras $ARGS > $OUT/write.log 2>&1
echo "write pass done"
# L2 hit / miss of the same dispatches (is the spill stream served by L2?)
timeout -k 10 420 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -f csv -d $OUT/tcc -o tcc -- python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras $ARGS > $OUT/tcc.log 2>&1
echo "tcc pass done"
bash $ROOT/tools/valu_pass.sh $TAG $ARGS

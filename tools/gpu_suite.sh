#!/bin/bash
# GPU suite (verbose per-test timing) and the default bench line.
#   usage: bash tools/gpu_suite.sh <tag> [pytest selection...]
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -x -v --durations=25 --timeout 300 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1
rc=$?; tail -30 gpurun_out/gputest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
cut -c1-300 gpurun_out/bench_$TAG.json

#!/bin/bash
# Phase-timing shares (libdrc_amd_timing.so) and the B = 1 / small-batch
# latency census of the current build, per robot, into gpurun_out/census_<tag>/.
#   usage: bash tools/census_pass.sh <tag> "<robot1> <robot2> ..."
set -e -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $ROOT
OUT=gpurun_out/census_$1
mkdir -p $OUT
for r in $2; do
  timeout -k 10 240 python3 tools/phase_timing.py $r > $OUT/phase_$r.txt 2> $OUT/phase_$r.err
  echo "phase $r done"
  timeout -k 10 300 python3 tools/latency_probe.py --robot $r --n 128 > $OUT/latency_$r.json 2> $OUT/latency_$r.err
  echo "latency $r done"
done

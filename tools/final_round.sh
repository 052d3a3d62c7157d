#!/bin/bash
# Round-end measurement on the final build (one MI355X): for every BASELINE
# robot, tools/profile_round.sh (the bench line with its CPU baseline, the
# rocprofv3 kernel-trace stats, the FETCH_SIZE / WRITE_SIZE passes and the
# FP64 VALU passes) into gpurun_out/prof_<tag>_<robot>/ and valu_<tag>_<robot>/;
# then the FR3 B = 4 096 line.  Summarise afterwards on the build host with
#   python tools/pmc_summary.py <tag>_<robot> <robot> <B> 4
#   python tools/valu_summary.py <tag>_<robot> <robot> <B> 4
#   usage: bash tools/final_round.sh <tag> [robot ...]
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $ROOT
TAG=$1; shift
ROBOTS=${@:-fr3 ur5e husky_fr3 xls_fr3 caster_fr3}
mkdir -p gpurun_out
for r in $ROBOTS; do
  timeout -k 10 900 bash tools/profile_round.sh ${TAG}_$r --robot $r > gpurun_out/final_${TAG}_$r.log 2>&1 || { tail -5 gpurun_out/final_${TAG}_$r.log; exit 1; }
  echo "$r: $(grep -m1 '^{' gpurun_out/prof_${TAG}_$r/bench.json | cut -c1-200)"
done
timeout -k 10 300 python3 bench.py --batch 4096 > gpurun_out/final_${TAG}_fr3_b4096.json 2> gpurun_out/final_${TAG}_fr3_b4096.err || exit 1
echo "fr3 B=4096: $(cut -c1-200 gpurun_out/final_${TAG}_fr3_b4096.json)"

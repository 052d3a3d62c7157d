#!/bin/bash
# Every BASELINE config on one MI355X with the CPU baseline (bench.py lines
# into gpurun_out/final_<tag>/), then the rocprofv3 rounds for FR3 and UR5e.
#   usage: bash tools/final_benches.sh <tag>
set -e -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $ROOT
TAG=$1
OUT=gpurun_out/final_$TAG
mkdir -p $OUT
run() {
  local name=$1; shift
  timeout -k 10 300 python3 bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err
  echo "$name: $(cut -c1-160 $OUT/$name.json)"
}
run fr3
run fr3_b4096 --batch 4096
run ur5e --robot ur5e
run husky_fr3 --robot husky_fr3
run xls_fr3 --robot xls_fr3
run caster_fr3 --robot caster_fr3
run xls_fr3_global --robot xls_fr3 --global-batch 65536 --no-cpu-baseline
bash tools/profile_round.sh ${TAG} > /dev/null
echo "profile fr3 done"
bash tools/profile_round.sh ${TAG}_ur5e --robot ur5e > /dev/null
echo "profile ur5e done"

#!/bin/bash
# Round-4 iteration check: GPU suite, then fused-vs-pipeline bits and an A/B
# of the -ffp-contract=on build, then the default bench line.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gputest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/fused_bits.py fr3 ur5e xls_fr3 > gpurun_out/${TAG}_bits_base.log 2>&1 || exit 1
DRC_AMD_LIB=libdrc_amd_fpon.so timeout -k 10 300 python3 -u tools/fused_bits.py fr3 ur5e xls_fr3 > gpurun_out/${TAG}_bits_fpon.log 2>&1 || exit 1
timeout -k 10 600 bash tools/ab_bench.sh ${TAG}_fpon "libdrc_amd.so libdrc_amd_fpon.so" "fr3 ur5e xls_fr3" 2 || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
cut -c1-300 gpurun_out/bench_$TAG.json

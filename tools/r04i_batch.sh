set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r04i.log 2>&1
rc=$?; tail -3 gpurun_out/gputest_r04i.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash tools/ab_bench.sh r04i_as "libdrc_amd_prev.so libdrc_amd.so libdrc_amd_ldsb.so" "fr3 ur5e xls_fr3" 3 || exit 1
# bench.py's own N-rank path on the box's one GPU (gloo transport; the driver's 8-GPU run uses RCCL)
DRC_DIST_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r04i_gpus2.json 2> gpurun_out/r04i_gpus2.err || exit 1
grep '^{' gpurun_out/r04i_gpus2.json | cut -c1-300

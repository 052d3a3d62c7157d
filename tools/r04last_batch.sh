set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04end_smoke.log 2>&1 || { cat gpurun_out/r04end_smoke.log; exit 1; }
tail -1 gpurun_out/r04end_smoke.log
DRC_DIST_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r04end_gpus2.json 2> gpurun_out/r04end_gpus2.err || exit 1
grep -h '^{' gpurun_out/r04end_gpus2.json | cut -c1-200

set -o pipefail
mkdir -p gpurun_out
for r in fr3 ur5e xls_fr3; do
  timeout -k 10 120 python3 tools/phase_timing.py $r > gpurun_out/r04z_phase_$r.txt 2>&1 || exit 1
done
DRC_DIST_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r04z_gpus2.json 2> gpurun_out/r04z_gpus2.err || exit 1
grep -h '^{' gpurun_out/r04z_gpus2.json | cut -c1-300
timeout -k 10 600 bash tools/env_ab.sh r04z_grid "fr3 ur5e" "base DRC_GRID_TASK=1024 DRC_GRID_TASK=4096 DRC_GRID_QP=1024 DRC_GRID_QP=4096" 2 || exit 1

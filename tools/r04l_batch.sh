set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 bash tools/ab_bench.sh r04l_lds "libdrc_amd_ldsb.so libdrc_amd.so" "husky_fr3 xls_fr3" 2 || exit 1
timeout -k 10 300 bash tools/env_ab.sh r04l_w3 "fr3" "base DRC_TASK_W3=1" 3 || exit 1
BENCH_ARGS="--batch 4096" timeout -k 10 300 bash tools/env_ab.sh r04l_b4k "fr3" "base DRC_GRID_FUSED=1024 DRC_GRID_FUSED=512" 3 || exit 1
timeout -k 10 120 python3 tools/phase_timing.py fr3 > gpurun_out/r04l_phase_fr3.txt 2>&1 || exit 1
timeout -k 10 120 python3 tools/phase_timing.py ur5e > gpurun_out/r04l_phase_ur5e.txt 2>&1 || exit 1
timeout -k 10 120 python3 tools/phase_timing.py xls_fr3 > gpurun_out/r04l_phase_xls_fr3.txt 2>&1 || exit 1

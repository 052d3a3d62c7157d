# r06aa: fused kernel at 3 waves per SIMD (168 VGPRs) at 16 384 / 65 536; EPA-first order on pipeline calls of 65 536
set -e
cd $GRAFT_REPO_ROOT
BENCH_ARGS="--batch 16384" bash tools/ab_bench.sh fw3_16k "libdrc_amd.so libdrc_amd_fw3.so" "fr3 ur5e xls_fr3" 2
DRC_FUSE_MAX=65536 bash tools/ab_bench.sh fw3_65k_fused "libdrc_amd.so libdrc_amd_fw3.so" "fr3 ur5e" 1
bash tools/env_ab.sh order65k "fr3 ur5e" "base DRC_ORDER_MAX=65536" 2

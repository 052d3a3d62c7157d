set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r04r.log 2>&1
rc=$?; tail -3 gpurun_out/gputest_r04r.log; [ $rc -eq 0 ] || exit $rc
# QP write attribution: the ADMM passes' vectors by v_readlane instead of LDS
DRC_AMD_LIB=libdrc_amd_rl.so timeout -k 10 300 bash tools/pmc_pass.sh r04r_rl --robot fr3 || exit 1
bash tools/final_round.sh r04g fr3 ur5e

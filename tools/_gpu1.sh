set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t1_pytest.log 2>&1; echo "pytest rc $?" >> gpurun_out/t1_pytest.log
tail -3 gpurun_out/t1_pytest.log
for w in 1 3 4; do
  DRC_AMD_LIB=libdrc_amd_w$w.so timeout -k 10 300 python tools/gpu_quick.py fr3 65536 5 > gpurun_out/t1_quick_w$w.log 2>&1 || { echo "quick w$w failed"; cat gpurun_out/t1_quick_w$w.log | tail -5; exit 1; }
  echo "w$w"; grep -E "solves|err" gpurun_out/t1_quick_w$w.log
done
timeout -k 10 300 python tools/gpu_quick.py fr3 65536 5 > gpurun_out/t1_quick_w2.log 2>&1 && echo w2 && grep -E "solves|err" gpurun_out/t1_quick_w2.log
timeout -k 10 300 python tools/phase_timing.py fr3 65536 > gpurun_out/t1_phase.log 2>&1 && cat gpurun_out/t1_phase.log

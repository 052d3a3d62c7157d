set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r04v.log 2>&1
rc=$?; tail -3 gpurun_out/gputest_r04v.log; [ $rc -eq 0 ] || exit $rc
DRC_AMD_LIB=libdrc_amd_db5c.so timeout -k 10 300 python3 tools/lib_bits.py db5c > gpurun_out/r04v_bits.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/lib_bits.py final4 >> gpurun_out/r04v_bits.log 2>&1 || exit 1
python3 tools/lib_bits.py --compare db5c final4 >> gpurun_out/r04v_bits.log 2>&1; tail -5 gpurun_out/r04v_bits.log
bash tools/final_round.sh r04h fr3 ur5e

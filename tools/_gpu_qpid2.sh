set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_qpid.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/qpid_pytest.log 2>&1; rc=$?
echo "qpid pytest rc $rc"; tail -3 gpurun_out/qpid_pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u tools/bench_qpid.py --cpu 0 > gpurun_out/bq2.jsonl 2> gpurun_out/bq2.err; echo "bench rc $?"; cut -c1-200 gpurun_out/bq2.jsonl

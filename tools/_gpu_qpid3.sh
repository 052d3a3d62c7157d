set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/bench_qpid.py --cpu 0 --robots fr3,xls_fr3 --steps 3 > gpurun_out/bq3.jsonl 2> gpurun_out/bq3.err; echo "bench rc $?"; cut -c1-120,300-520 gpurun_out/bq3.jsonl
timeout -k 10 400 python -u tools/bench_qpid.py --cpu 0 --robots fr3,xls_fr3 --steps 3 --osqp-default > gpurun_out/bq4.jsonl 2> gpurun_out/bq4.err; echo "bench rc $?"; cut -c1-120,300-520 gpurun_out/bq4.jsonl

set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/bench_qpid.py > gpurun_out/bq.jsonl 2> gpurun_out/bq.err; echo "bench rc $?"; cat gpurun_out/bq.jsonl
mkdir -p gpurun_out/prof_qpid
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_qpid -o qpid -- python3 $GRAFT_REPO_ROOT/tools/bench_qpid.py --robots fr3 --steps 5 --cpu 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_qpid/run.log 2>&1; echo "prof rc $?"
find $GRAFT_REPO_ROOT/gpurun_out/prof_qpid -name "*kernel_stats.csv" | head -3

set -e
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -f csv -d $GRAFT_REPO_ROOT/gpurun_out/kt4096 -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --batch 4096 --steps 20 --warmup 3 --no-cpu-baseline --no-extras > $GRAFT_REPO_ROOT/gpurun_out/kt4096.log 2>&1
echo done

cd $GRAFT_REPO_ROOT
for mi in 100 400 1000; do
timeout -k 10 200 python -u tools/bench_qpid.py --cpu 0 --robots fr3 --steps 3 --max-iter $mi > gpurun_out/bqm$mi.jsonl 2>&1 || exit 1
echo "max_iter $mi"; cut -c1-130 gpurun_out/bqm$mi.jsonl
done

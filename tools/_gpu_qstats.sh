cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/qpid_parity_stats.py > gpurun_out/qstats.log 2>&1; echo rc $?; cat gpurun_out/qstats.log | tail -30

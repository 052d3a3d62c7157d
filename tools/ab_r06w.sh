# r06w: EPA-first order on fused manipulator calls above 8 192: tests and bench lines
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_order.py tests/test_gpu_fused.py tests/test_gpu_fullsize.py tests/test_gpu_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r06w.log 2>&1
tail -2 gpurun_out/gputest_r06w.log
for b in 12288 16384; do for r in fr3 ur5e; do echo "$r $b: $(timeout -k 10 300 python3 bench.py --robot $r --batch $b --no-cpu-baseline --no-extras --steps 20 --warmup 5 | cut -c90-140)"; done; done

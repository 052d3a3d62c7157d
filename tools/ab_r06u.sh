# r06u: occupancy-based fusion threshold (16 384 except UR5e): GPU tests it touches and the bench lines it moves
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_dist.py tests/test_gpu_fused.py tests/test_gpu_order.py tests/test_gpu_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r06u.log 2>&1
tail -3 gpurun_out/gputest_r06u.log
for r in husky_fr3; do timeout -k 10 300 python3 bench.py --robot $r --no-cpu-baseline --no-extras --steps 20 --warmup 5 | cut -c1-160; done
for r in fr3 ur5e xls_fr3; do timeout -k 10 300 python3 bench.py --robot $r --batch 16384 --no-cpu-baseline --no-extras --steps 20 --warmup 5 | cut -c1-160; done

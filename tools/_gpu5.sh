cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/b1.json 2> gpurun_out/b1.err && tail -c 400 gpurun_out/b1.json && echo
DRC_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/b2.json 2> gpurun_out/b2.err; echo "rc $?"; cat gpurun_out/b2.json | head -c 600; tail -3 gpurun_out/b2.err

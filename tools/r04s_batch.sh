set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04s_smoke.log 2>&1 || { cat gpurun_out/r04s_smoke.log; exit 1; }
tail -1 gpurun_out/r04s_smoke.log
# bench.py's N-rank path on the box's one GPU (gloo transport; the driver's 8-GPU run uses RCCL)
DRC_DIST_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r04s_gpus2.json 2> gpurun_out/r04s_gpus2.err || exit 1
DRC_DIST_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --robot xls_fr3 --global-batch 131072 > gpurun_out/r04s_gpus2_xls_strong.json 2> gpurun_out/r04s_gpus2_xls_strong.err || exit 1
grep -h '^{' gpurun_out/r04s_gpus2.json gpurun_out/r04s_gpus2_xls_strong.json | cut -c1-300
# concurrent sub-batches per call on the final build
out=gpurun_out/r04s_chunks.jsonl; : > $out
for r in fr3 ur5e xls_fr3; do for c in 2 3 4; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-extras --robot $r --steps 20 --warmup 5 --chunks $c > gpurun_out/c_tmp.json 2> gpurun_out/c_tmp.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/c_tmp.json')); print(json.dumps({'robot':'$r','chunks':$c,'value':d['value']}))" >> $out
done; done
cat $out

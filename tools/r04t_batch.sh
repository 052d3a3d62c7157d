set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r04t_queues.jsonl; : > $out
for r in fr3 xls_fr3; do for q in 4 8; do for c in 3 6; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-extras --robot $r --steps 20 --warmup 5 --chunks $c > gpurun_out/c_tmp.json 2> gpurun_out/c_tmp.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/c_tmp.json')); print(json.dumps({'robot':'$r','queues':$q,'chunks':$c,'value':d['value']}))" >> $out
done; done; done
cat $out
timeout -k 10 500 bash tools/ab_bench.sh r04u_st3 "libdrc_amd.so libdrc_amd_st.so" "fr3 ur5e xls_fr3" 2 || exit 1
BENCH_ARGS="--chunks 4" timeout -k 10 300 bash tools/ab_bench.sh r04u_st4 "libdrc_amd_st.so" "fr3 ur5e xls_fr3" 2 || exit 1

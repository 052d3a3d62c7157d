cd $GRAFT_REPO_ROOT
out=gpurun_out/chunks_ab.jsonl; : > $out
for rep in 1 2; do for r in fr3 ur5e xls_fr3 husky_fr3; do for c in 2 3; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-extras --robot $r --steps 20 --warmup 5 --chunks $c > gpurun_out/c_tmp.json 2> gpurun_out/c_tmp.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/c_tmp.json')); print(json.dumps({'robot':'$r','chunks':$c,'value':d['value']}))" >> $out
done; done; done
cat $out


set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  for a in "" "--no-kernel-events"; do
    for b in 65536 4096; do
      timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-extras --batch $b $a > gpurun_out/evab_tmp.json 2> gpurun_out/evab_tmp.err || { tail -3 gpurun_out/evab_tmp.err; exit 1; }
      python3 -c "
import json; d=json.loads(open('gpurun_out/evab_tmp.json').read().strip().splitlines()[-1]); print(json.dumps({'batch': $b, 'args': '$a', 'value': d['value'], 'ms': d['ms_per_step']}))" | tee -a gpurun_out/evab.jsonl
    done
  done
done

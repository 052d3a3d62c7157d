set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extras > gpurun_out/r04check_bench.json 2> gpurun_out/r04check_bench.err || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/r04check_bench.json')); r=d['roofline']
print(d['value'], d['build_id'], r['traffic'], r['traffic_source'])
print({k: v for k, v in r.get('fp64_valu', {}).items() if k != 'note'})
print({k: v for k, v in r.get('valu_issue_roof', {}).items() if k != 'note'})"

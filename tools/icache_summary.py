"""Summarise tools/icache_pass.sh output: per kernel family (task / qp /
fused), the instruction-cache hit rate and the share of wave cycles spent
waiting for instruction fetch (SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES) next to all
waits (SQ_WAIT_ANY / SQ_WAVE_CYCLES).
    python tools/icache_summary.py gpurun_out/ic_<tag>"""
import collections
import csv
import glob
import json
import sys


def family(name):
    for k in ("fused_kernel", "task_kernel", "qp_kernel"):
        if k in name:
            return k
    return None


def main(d):
    acc = collections.defaultdict(lambda: collections.Counter())
    for f in glob.glob(d + "/p*/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            fam = family(r["Kernel_Name"])
            if fam:
                acc[fam][r["Counter_Name"]] += float(r["Counter_Value"])
    out = {}
    for fam, c in acc.items():
        hits, miss = c["SQC_ICACHE_HITS"], c["SQC_ICACHE_MISSES"]
        out[fam] = {
            "icache_hit_rate": hits / max(hits + miss, 1),
            "icache_misses": miss,
            "wait_inst_frac": c["SQ_WAIT_INST_ANY"] / max(c["SQ_WAVE_CYCLES"], 1),
            "wait_any_frac": c["SQ_WAIT_ANY"] / max(c["SQ_WAVE_CYCLES"], 1),
            "ifetch": c["SQ_IFETCH"],
        }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])

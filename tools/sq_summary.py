"""Per-kernel SQ counter summary of a tools/sq_pass.sh run.

    python tools/sq_summary.py <tag> [instances_per_dispatch]

Counters are averaged over dispatches and divided by the waves of the
dispatch (one wave = one instance for the task and QP kernels).  Cycle
counters (SQ_WAVE_CYCLES, SQ_WAIT_*, SQ_ACTIVE_*) count quad-cycles on gfx950
(MI355X_MICROARCH.md), so they are multiplied by 4 into shader cycles.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    for k in ("task_kernel", "qpid_kernel", "qp_kernel", "dyn_kernel", "fused_kernel"):
        if k in name:
            return k
    return name[:40]


def main():
    tag = sys.argv[1]
    src = os.path.join(ROOT, "gpurun_out", "sq_" + tag)
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                vals[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {}
    for k, cs in vals.items():
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        waves = avg.get("SQ_WAVES")
        if not waves:
            continue
        per = {}
        for c, v in avg.items():
            q = 4.0 if ("CYCLES" in c or "WAIT" in c or "ACTIVE" in c) and c != "SQ_BUSY_CYCLES" else 1.0
            per[c] = v * q / waves
        out[k] = dict(waves_per_dispatch=waves, per_wave=per)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

"""Summarise a tools/profile_round.sh run into committed profiles.

    python tools/pmc_summary.py <tag> [robot batch chunks]

Reads gpurun_out/prof_<tag>/ and writes
  profiles/<tag>_bench.json          the bench line of that run
  profiles/<tag>_kernel_stats.csv    rocprofv3 --kernel-trace --stats summary
  profiles/<tag>_pmc.json            per-kernel FETCH_SIZE / WRITE_SIZE per launch
  profiles/pmc_traffic_<robot>.json  the same, as read by bench.py (latest run of that robot)

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE
are in KiB; on gfx950 FETCH_SIZE counts half the bytes of a streaming read,
so it is doubled.  Our loads are 8 B/lane gathers, an access width the guide
leaves uncalibrated, so the raw values are kept next to the corrected ones.
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    for k in ("task_kernel", "qp_kernel", "fused_kernel"):
        if k in name:
            return k
    return None


MAIN_GRID = None   # (r06: the task / QP / fused grids differ; the dispatch order selects the bench's rows)


def bench_rows(rows, grid_key, grid=MAIN_GRID):
    """The bench's own task/QP dispatches: the workload generator's stage
    launches (task kernel only) all precede the first QP dispatch, and the
    bench's first task dispatch immediately precedes it (a call enqueues task,
    QP, task, QP, ... for its sub-batches).  `grid` (work-items) additionally
    keeps only dispatches of that size when given."""
    rows = [r for r in rows if short(r.get("Kernel_Name", "")) and (grid is None or int(r.get(grid_key, grid)) == grid)]
    ids = [int(r["Dispatch_Id"]) for r in rows if short(r["Kernel_Name"]) == "qp_kernel" and "Dispatch_Id" in r]
    if not ids:   # a fused call (B <= 16 384): its own dispatches only
        fid = [int(r["Dispatch_Id"]) for r in rows if short(r["Kernel_Name"]) == "fused_kernel" and "Dispatch_Id" in r]
        return [r for r in rows if short(r["Kernel_Name"]) == "fused_kernel"] if fid else rows
    first = min(ids) - 1
    return [r for r in rows if int(r.get("Dispatch_Id", first)) >= first]


def counters(d, cname, grid=MAIN_GRID):
    """Per-kernel average of a counter over the bench's own dispatches (the
    workload generator's stage launches are excluded, bench_rows)."""
    per = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in bench_rows(list(csv.DictReader(fh)), "Grid_Size", grid):
                if row.get("Counter_Name") != cname:
                    continue
                k = short(row.get("Kernel_Name", ""))
                if k:
                    per[k].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in per.items()}, {k: len(v) for k, v in per.items()}


def trace_durations(d, grid=MAIN_GRID):
    """Per-kernel average duration (ns) of the bench's dispatches from the kernel trace."""
    per = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for row in bench_rows(list(csv.DictReader(fh)), "Grid_Size_X", grid):
                k = short(row.get("Kernel_Name", ""))
                if k:
                    per[k].append(float(row["End_Timestamp"]) - float(row["Start_Timestamp"]))
    return {k: sum(v) / len(v) for k, v in per.items()}, {k: len(v) for k, v in per.items()}


def main():
    tag = sys.argv[1]
    robot = sys.argv[2] if len(sys.argv) > 2 else "fr3"
    batch = int(sys.argv[3]) if len(sys.argv) > 3 else 65536
    chunks = int(sys.argv[4]) if len(sys.argv) > 4 else 4   # sub-batches per drc_qpik_batch call (bench default)
    src = os.path.join(ROOT, "gpurun_out", "prof_" + tag)
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "bench.json"), os.path.join(dst, tag + "_bench.json"))
    stats = glob.glob(os.path.join(src, "kt", "**", "*kernel_stats.csv"), recursive=True)
    shutil.copy(stats[0], os.path.join(dst, tag + "_kernel_stats.csv"))
    avg, ndisp = trace_durations(os.path.join(src, "kt"))
    fetch, nf = counters(os.path.join(src, "fetch"), "FETCH_SIZE")
    write, nw = counters(os.path.join(src, "write"), "WRITE_SIZE")
    hit, _ = counters(os.path.join(src, "tcc"), "TCC_HIT_sum")
    miss, _ = counters(os.path.join(src, "tcc"), "TCC_MISS_sum")
    kern = {}
    for k in sorted(set(fetch) | set(write)):
        kern[k] = {"FETCH_SIZE_KiB_raw": fetch.get(k), "WRITE_SIZE_KiB_raw": write.get(k),
                   "fetch_bytes": 2 * 1024 * fetch.get(k, 0.0), "write_bytes": 1024 * write.get(k, 0.0),
                   "dispatches": [nf.get(k, 0), nw.get(k, 0)], "avg_duration_ns": avg.get(k)}
        if k in hit and k in miss and hit[k] + miss[k] > 0:
            kern[k]["TCC_HIT"] = hit[k]
            kern[k]["TCC_MISS"] = miss[k]
            kern[k]["l2_hit_rate"] = hit[k] / (hit[k] + miss[k])
    per_dispatch = sum(v["fetch_bytes"] + v["write_bytes"] for v in kern.values())
    # each dispatch pair covers one sub-batch (batch / chunks instances); a step is one call
    with open(os.path.join(src, "bench.json")) as fh:
        build = json.loads(fh.read().strip().splitlines()[-1]).get("build_id")
    out = {"robot": robot, "batch": batch, "chunks": chunks, "tag": tag, "build_id": build, "kernels": kern,
           "hbm_bytes_per_step": chunks * per_dispatch,
           "hbm_bytes_per_instance": chunks * per_dispatch / batch,
           "corrections": "FETCH_SIZE KiB x1024 x2 (gfx950 half-count), WRITE_SIZE KiB x1024",
           "main_dispatch_avg_ns": avg, "main_dispatches_traced": ndisp,
           "note": "averages over the bench's own dispatches (grid %s work-items); the kernel_stats csv "
                   "also counts the workload generator's stage launches" % "task 1024 x 64, QP 4096 x 64 / fused 2048 x 64"}
    for name in (tag + "_pmc.json", "pmc_traffic_%s.json" % robot):
        with open(os.path.join(dst, name), "w") as fh:
            json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

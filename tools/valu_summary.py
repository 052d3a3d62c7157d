"""Counter-based FP64 work of one drc_qpik_batch call from a tools/valu_pass.sh
run; writes profiles/valu_counters_<robot>.json (read by bench.py as
roofline.fp64_valu) and profiles/<tag>_valu.json.

    python tools/valu_summary.py <tag> <robot> <batch> [chunks]

FP64 FLOP per dispatch = 64 x (2 FMA + ADD + MUL) instructions (rocprofv3's
own FLOPS expression; every lane counted, as the instruction occupies the
SIMD for a full wave) and, separately, SQ_INSTS_VALU_FLOPS_FP64 as the
hardware reports it.  Lane efficiency = SQ_THREAD_CYCLES_VALU /
(64 x SQ_ACTIVE_INST_VALU): the fraction of issued VALU lane-slots that had an
active lane.  A step is one call = `chunks` dispatches of each kernel.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import bench_rows  # noqa: E402


def short(name):
    for k in ("task_kernel", "qpid_kernel", "qp_kernel", "dyn_kernel", "fused_kernel"):
        if k in name:
            return k
    return None


def main():
    tag, robot, batch = sys.argv[1], sys.argv[2], int(sys.argv[3])
    chunks = int(sys.argv[4]) if len(sys.argv) > 4 else 4
    src = os.path.join(ROOT, "gpurun_out", "valu_" + tag)
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in bench_rows(list(csv.DictReader(fh)), "Grid_Size"):   # the bench's own dispatches
                k = short(row["Kernel_Name"])
                if k:
                    vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    kern = {}
    for k, cs in vals.items():
        a = {c: sum(v) / len(v) for c, v in cs.items()}
        fl = 64 * (2 * a.get("SQ_INSTS_VALU_FMA_F64", 0) + a.get("SQ_INSTS_VALU_ADD_F64", 0)
                   + a.get("SQ_INSTS_VALU_MUL_F64", 0))
        eff = a.get("SQ_THREAD_CYCLES_VALU", 0) / max(64 * a.get("SQ_ACTIVE_INST_VALU", 0), 1)
        kern[k] = {"per_dispatch": a, "fp64_flops_per_dispatch": fl,
                   "fp64_flops_hw_per_dispatch": a.get("SQ_INSTS_VALU_FLOPS_FP64"),
                   "lane_efficiency": eff,
                   "fp64_share_of_valu": (a.get("SQ_INSTS_VALU_FMA_F64", 0) + a.get("SQ_INSTS_VALU_ADD_F64", 0)
                                          + a.get("SQ_INSTS_VALU_MUL_F64", 0) + a.get("SQ_INSTS_VALU_TRANS_F64", 0))
                   / max(a.get("SQ_INSTS_VALU", 0), 1)}
    qp = [k for k in ("task_kernel", "qp_kernel", "fused_kernel") if k in kern]
    step = chunks * sum(kern[k]["fp64_flops_per_dispatch"] for k in qp)
    step_hw = chunks * sum(kern[k]["fp64_flops_hw_per_dispatch"] or 0 for k in qp)
    tc = sum(kern[k]["per_dispatch"].get("SQ_THREAD_CYCLES_VALU", 0) for k in qp)
    ac = sum(kern[k]["per_dispatch"].get("SQ_ACTIVE_INST_VALU", 0) for k in qp)
    # VALU issue cycles on the SIMD: a wave64 FP64 instruction (16 FP64 lanes per
    # cycle: the 78.6 TFLOP/s vector peak = 1 024 SIMDs x 2.4 GHz x 16 FMA) takes
    # 4 cycles, any other VALU instruction 2 (32 lanes per cycle, MI355X_MICROARCH.md)
    def f64(a):
        return sum(a.get(c, 0) for c in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                                          "SQ_INSTS_VALU_TRANS_F64"))
    issue = chunks * sum(4 * f64(kern[k]["per_dispatch"]) + 2 * (kern[k]["per_dispatch"].get("SQ_INSTS_VALU", 0)
                                                                   - f64(kern[k]["per_dispatch"])) for k in qp)
    valu_insts = chunks * sum(kern[k]["per_dispatch"].get("SQ_INSTS_VALU", 0) for k in qp)
    with open(os.path.join(src, "build_id")) as fh:
        build = fh.read().strip()
    out = {"robot": robot, "batch": batch, "chunks": chunks, "tag": tag, "build_id": build, "kernels": kern,
           "fp64_flops_per_step": step, "fp64_flops_hw_per_step": step_hw,
           "fp64_flops_per_solve": step / batch, "lane_efficiency": tc / max(64 * ac, 1),
           "valu_insts_per_solve": valu_insts / batch, "valu_issue_cycles_per_solve": issue / batch,
           "note": "FLOP = 64 x (2 FMA + ADD + MUL) FP64 instructions per dispatch, summed over the task and QP "
                   "kernels of one call (chunks dispatches each); lane efficiency = thread-cycles / (64 x active "
                   "VALU quad-cycles) over both kernels"}
    dst = os.path.join(ROOT, "profiles")
    for name in (tag + "_valu.json", "valu_counters_%s.json" % robot):
        with open(os.path.join(dst, name), "w") as fh:
            json.dump(out, fh, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "kernels"}, indent=1))


if __name__ == "__main__":
    main()

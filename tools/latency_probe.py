"""Latency census (GPU box): per-instance task / QP kernel durations of B = 1
calls over the first N instances of the bench workload, and the split of a
small-batch call (B = 512 ... 8192) into its task and QP kernels.

    python tools/latency_probe.py [--robot fr3] [--n 256] > gpurun_out/latency_<robot>.json
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--robot", default="fr3")
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--solver", default="exact")
    ap.add_argument("--batches", default="512,1024,2048,4096,8192")
    args = ap.parse_args()
    import torch
    import bench
    from dyros_robot_controller_amd import BUNDLED, _capi, make_robot, manipulator, mobile_manipulator
    dev = torch.device("cuda", 0)
    rd = make_robot(args.robot, dev)
    spec = BUNDLED[args.robot]
    mod = manipulator if spec["kind"] == "manipulator" else mobile_manipulator
    ctrl = mod.RobotController(0.001, rd, solver_mode=args.solver)
    B = 8192
    _, (dq, dqd, dxt, dxdt), _ = bench.make_inputs(rd, args.robot, B, 12345, 0, dev)
    link = spec["link"]
    lib, h = _capi.lib(), rd.model.handle

    def times(fn, reps):
        fn()
        torch.cuda.synchronize()
        _capi.check(lib.drc_debug_kernel_timing(h, 1))
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        tw, tk, tq, nc = C.c_double(), C.c_double(), C.c_double(), C.c_int()
        _capi.check(lib.drc_debug_kernel_times(h, C.byref(tw), C.byref(tk), C.byref(tq), C.byref(nc)))
        _capi.check(lib.drc_debug_kernel_timing(h, 0))
        n = max(nc.value, 1)
        return tw.value / n, tk.value / n, tq.value / n

    res = {"robot": args.robot, "solver": args.solver}
    per = []
    it1 = torch.zeros(1, dtype=torch.int32, device=dev)
    for b in range(args.n):
        one = [t[:, b:b + 1].contiguous() for t in (dq, dqd, dxt, dxdt)]
        w, tk, tq = times(lambda: ctrl.QPIK_step_batch(*one, link, iters=it1), 3)
        per.append((tk * 1e3, tq * 1e3, int(it1.item())))
    a = np.array(per)
    q = lambda v: {"p50": float(np.percentile(v, 50)), "p90": float(np.percentile(v, 90)),
                   "p99": float(np.percentile(v, 99)), "max": float(v.max()), "mean": float(v.mean())}
    res["b1_task_us"], res["b1_qp_us"] = q(a[:, 0]), q(a[:, 1])
    res["b1_total_us"] = q(a[:, 0] + a[:, 1])
    res["b1_worst"] = [[int(i), float(a[i, 0]), float(a[i, 1]), int(a[i, 2])]
                       for i in np.argsort(-(a[:, 0] + a[:, 1]))[:8]]
    for nb in [int(v) for v in args.batches.split(",")]:
        sub = [t[:, :nb].contiguous() for t in (dq, dqd, dxt, dxdt)]
        it = torch.zeros(nb, dtype=torch.int32, device=dev)
        w, tk, tq = times(lambda: ctrl.QPIK_step_batch(*sub, link, iters=it), 10)
        res["batch_%d" % nb] = {"call_ms": w, "task_ms": tk, "qp_ms": tq, "solves_per_s": nb / (w * 1e-3),
                                "iters_max": int(it.max().item())}
        if nb <= args.n:  # the slowest of these instances alone on the GPU
            res["batch_%d" % nb]["max_isolated_ms"] = float((a[:nb, 0] + a[:nb, 1]).max()) * 1e-3
    print(json.dumps(res))


if __name__ == "__main__":
    main()

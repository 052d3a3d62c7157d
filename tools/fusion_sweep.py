"""Fused task + QP kernel vs the two-kernel pipeline across batch sizes (GPU):
solves/s of drc_qpik_batch (QPIKStep, exact, bench workload) with
drc_set_fusion(1) and (0).   python tools/fusion_sweep.py [--robot fr3]"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--robot", default="fr3")
    ap.add_argument("--sizes", default="1,512,2048,4096,8192,16384,32768,65536")
    a = ap.parse_args()
    import torch
    import bench
    from dyros_robot_controller_amd import BUNDLED, _capi, make_robot, manipulator, mobile_manipulator
    dev = torch.device("cuda", 0)
    rd = make_robot(a.robot, dev)
    spec = BUNDLED[a.robot]
    mod = manipulator if spec["kind"] == "manipulator" else mobile_manipulator
    ctrl = mod.RobotController(0.001, rd, solver_mode="exact")
    _, (dq, dqd, dxt, dxdt), _ = bench.make_inputs(rd, a.robot, 65536, 12345, 0, dev)
    res = {"robot": a.robot}
    for n in [int(x) for x in a.sizes.split(",")]:
        sub = [t[:, :n].contiguous() for t in (dq, dqd, dxt, dxdt)]
        for f in (1, 0):
            _capi.check(_capi.lib().drc_set_fusion(rd.model.handle, C.c_int(f)))
            reps = max(5, min(200, 200000 // max(n, 1)))
            s = bench.timed_steps(torch, lambda: ctrl.QPIK_step_batch(*sub, spec["link"]), reps, 3)
            res["%d_%s" % (n, "fused" if f else "pipeline")] = n / s
    print(json.dumps(res))


if __name__ == "__main__":
    main()

"""Throughput of drc_dynamics_batch on one GPU.

Times K launches of the batched updateDynamics (M, M_inv, g, nle, c) with
inputs resident in HBM, with HIP events on the launch stream, and prints one
JSON line per robot with the roofline numbers DESIGN.md quotes:
algorithmic bytes per robot = 8 * (2*D inputs + 2*n^2 + 3*n outputs),
n = D (actuated = 0) or A (actuated = 1)."""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from dyros_robot_controller_amd import _batch, workload  # noqa: E402

HBM_PEAK_GBS = 8000.0


def run(robot, B, steps, warmup, actuated, dev):
    import oracle as O   # robot specs only (paths, index layout); not timed
    from _common import make_manipulator, make_moma
    pm, _, spec = O.load(robot)
    rd = make_moma(robot, dev) if spec["kind"] == 1 else make_manipulator(robot, dev)
    lo, hi, vel = np.array(pm.lower), np.array(pm.upper), np.array(pm.vel)
    if spec["kind"] == 1:
        q, qd = workload.mobile_states(lo, hi, vel, spec["joint_index"], spec["n_arm"], spec["n_wheel"], 1, B)
    else:
        q, qd = workload.joint_states(lo, hi, vel, 1, B)
    q, qd = _batch.as_device(q, dev), _batch.as_device(qd, dev)
    D = pm.nv
    n = (spec["n_arm"] + spec["n_wheel"]) if actuated else D
    outs = {k: torch.empty((n * n if k in ("M", "Minv") else n, B), dtype=torch.float64, device=dev)
            for k in _batch.DYN_FIELDS}
    st = torch.cuda.current_stream(dev)
    import ctypes as C
    from dyros_robot_controller_amd import _capi
    lib = _capi.lib()
    p = lambda t: C.c_void_p(t.data_ptr())

    def call():
        _capi.check(lib.drc_dynamics_batch(rd.model.handle, C.c_int(1 if actuated else 0), C.c_int64(B), p(q), p(qd),
                                           p(outs["M"]), p(outs["Minv"]), p(outs["g"]), p(outs["nle"]), p(outs["c"]),
                                           C.c_void_p(st.cuda_stream)))
    for _ in range(warmup):
        call()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(steps):
        call()
    e1.record(st)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / steps
    byts = 8 * (2 * D + 2 * n * n + 3 * n)
    gbs = byts * B / (ms * 1e-3) / 1e9
    return dict(robot=robot, actuated=bool(actuated), B=B, ms_per_call=ms, robots_per_s=B / (ms * 1e-3),
                bytes_per_robot=byts, achieved_GBs=gbs, hbm_frac=gbs / HBM_PEAK_GBS)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--robots", default="fr3,ur5e,husky_fr3,xls_fr3")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for r in a.robots.split(","):
        print(json.dumps(run(r, a.B, a.steps, a.warmup, False, dev)), flush=True)
        if r in ("husky_fr3", "xls_fr3"):
            print(json.dumps(run(r, a.B, a.steps, a.warmup, True, dev)), flush=True)


if __name__ == "__main__":
    main()

"""Throughput of the batched QPID path on one GPU.

One step = one drc_qpid_batch call in QPIDStep mode over B robots with the
inputs resident in HBM: device dynamics (M, g of the equality rows) ->
QPID task kernel -> QPID QP kernel, timed with HIP events on the launch
stream.  Prints one JSON line per robot:
  algorithmic HBM bytes per solve = 8 * (2 D + 12 + 6) in + (8 * 2 A + 4) out;
  cpu_sample: the oracle's QPIDStep (C restatement, exact mode) on one core
  for a bounded sample, dynamics precomputed (not timed) — a reported
  baseline, not the target.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

from dyros_robot_controller_amd import _batch, _capi  # noqa: E402

HBM_PEAK_GBS = 8000.0


def run(robot, B, steps, warmup, dev, cpu_n, exact, max_iter=None):
    import oracle as O
    from _common import LINK, make_manipulator, make_moma, moma_step_inputs, step_inputs
    from dyros_robot_controller_amd import manipulator, mobile_manipulator as MM
    pm, om, spec = O.load(robot)
    if spec["kind"] == 1:
        rd = make_moma(robot, dev)
        q, qd, xt, xdt = moma_step_inputs(rd, robot, 12345, B, dev)
        ctrl = MM.RobotController(0.001, rd, solver_mode="exact" if exact else "osqp_default")
    else:
        rd = make_manipulator(robot, dev)
        q, qd, xt, xdt = step_inputs(rd, robot, 12345, B, dev)
        ctrl = manipulator.RobotController(0.001, rd, solver_mode="exact" if exact else "osqp_default")
    p = ctrl._pbd.params(LINK[robot], _capi.MODE_QPID_STEP, ctrl.Kp_task_, ctrl.Kv_task_)
    if max_iter:
        p.solver.max_iter = max_iter
    a = lambda v: _batch.as_device(v, dev)
    dq, dqd, dxt, dxdt = a(q), a(qd), a(xt), a(xdt)
    na, D = rd.model.actuated_dof, rd.model.dof
    qdd = torch.empty((na, B), dtype=torch.float64, device=dev)
    tau = torch.empty((na, B), dtype=torch.float64, device=dev)
    status = torch.empty(B, dtype=torch.int32, device=dev)
    iters = torch.empty(B, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev)

    def call():
        _batch.qpid_batch(rd.model, p, dq, dqd, dxt, dxdt, qddot=qdd, tau=tau, status=status, iters=iters,
                          stream=st.cuda_stream)
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
    bytes_per = 8 * (2 * D + 18) + 8 * 2 * na + 4
    stv = status.cpu().numpy()
    out = dict(robot=robot, B=B, mode="exact" if exact else "osqp_default", ms_per_call=ms,
               solves_per_s=B / (ms * 1e-3), bytes_per_solve=bytes_per,
               achieved_GBs=B * bytes_per / (ms * 1e-3) / 1e9, hbm_frac=B * bytes_per / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
               solved_frac=float(np.mean(stv == _capi.STATUS_SOLVED)), admm_iters_mean=float(iters.float().mean()),
               admm_iters_p99=float(np.percentile(iters.cpu().numpy(), 99)), admm_iters_max=int(iters.max()))
    if cpu_n:
        par = O.default_qpid_params(om.kind, exact=exact)
        par.mode = 1
        dyn = [O.qpid_dynamics(pm, om, spec, q[:, b], qd[:, b]) for b in range(cpu_n)]
        t0 = time.perf_counter()
        for b in range(cpu_n):
            O.qpid_one(om, par, q[:, b], qd[:, b], *dyn[b], xt[:, b], xdt[:, b])
        dt = time.perf_counter() - t0
        out["cpu_sample"] = dict(solves_per_s=cpu_n / dt, cores=1, kind="port", n=cpu_n,
                                 note="oracle QPIDStep (C) per instance, dynamics precomputed, Python call loop")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--robots", default="fr3,ur5e,husky_fr3,xls_fr3")
    ap.add_argument("--B", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--cpu", type=int, default=300)
    ap.add_argument("--osqp-default", action="store_true")
    ap.add_argument("--max-iter", type=int, default=0, help="diagnostic: override OSQP max_iter")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    for r in args.robots.split(","):
        print(json.dumps(run(r, args.B, args.steps, args.warmup, dev, args.cpu, not args.osqp_default, args.max_iter)), flush=True)


if __name__ == "__main__":
    main()

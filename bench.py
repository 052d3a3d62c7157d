#!/usr/bin/env python3
"""Headline benchmark: batched QP-IK solves/s (FR3 7-DoF QPIKStep, 65 536
instances per GPU) + achieved HBM GB/s vs peak (BASELINE.json "metric").

One "step" = one control cycle of the whole batch through the product path
(drc_qpik_batch: task-space kernel + QP kernel), inputs resident in HBM.
Multi-GPU: one process per GPU (torchrun), instances sharded across ranks
with no data-path collective (weak scaling: 65 536 per GPU); a barrier and a
max-reduction of the timed region are the only collectives.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--robot fr3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
FP64_VECTOR_PEAK_TFS = 78.6    # AMD spec, FP64 vector
LINKS = {"fr3": "fr3_link8", "ur5e": "tool0"}


def algorithmic_bytes(nv):
    """per solve, HBM in (q, qdot [nv], x_target [12], xdot_target [6])
    + out (qdot* [nv] f64, status i32).  FR3: 256 + 60 = 316 B."""
    return (2 * nv + 12 + 6) * 8 + nv * 8 + 4


def flops_per_solve(nv, iters):
    """SURVEY §8(d) static estimate for FR3-sized problems: 52k setup +
    1.3k per ADMM iteration (reported as an estimate, not measured)."""
    return 52e3 + 1.3e3 * iters


def make_inputs(rd, robot, B, seed, offset, dev):
    import torch
    from dyros_robot_controller_amd import _batch, _capi, manipulator, workload
    lo, hi = rd.getJointPositionLimit()
    _, vmax = rd.getJointVelocityLimit()
    q, qd = workload.joint_states(lo, hi, vmax, seed, B, offset)
    # SURVEY §8d stress tiers (10 % each: joint limit, near-singular, CBF-active
    # self-collision), judged by the product's own stage kernel
    workload.apply_stress(q, lo, hi, list(range(len(lo))), seed, offset,
                          workload.device_evaluator(rd.model, LINKS[robot], dev))
    pb = manipulator.QPIKParamsBuilder(rd.model, exact=True)
    p = pb.params(LINKS[robot], _capi.MODE_QPIK)
    dq, dqd = _batch.as_device(q, dev), _batch.as_device(qd, dev)
    st = _batch.stages_batch(rd.model, p, dq, dqd, None, _batch.as_device(np.zeros((6, B)), dev))
    xt, xdt = workload.perturb_targets(st["pose"].cpu().numpy(), seed, B, offset)
    return q, qd, xt, xdt, dq, dqd, _batch.as_device(xt, dev), _batch.as_device(xdt, dev)


def cpu_baseline(robot, q, qd, xt, xdt, budget_s=1.5):
    """Oracle restatement of the reference CPU path (OSQP-default settings,
    fresh setup per solve) on this host's cores, bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    _, om, spec = O.load(robot)
    par = O.default_params(spec["kind"], exact=False)
    threads = max(1, min(16, os.cpu_count() or 1))   # box CPU share is 16
    n = min(q.shape[1], 2048)
    t0 = time.time()
    O.qpik_batch(om, par, q[:, :n], qd[:, :n], xt[:, :n], xdt[:, :n], nthreads=threads)
    dt = time.time() - t0
    per = dt / n
    n2 = int(min(q.shape[1], max(n, budget_s / max(per, 1e-9))))
    t0 = time.time()
    O.qpik_batch(om, par, q[:, :n2], qd[:, :n2], xt[:, :n2], xdt[:, :n2], nthreads=threads)
    dt = time.time() - t0
    return {"value": n2 / dt, "unit": "solves/s", "cores": threads, "kind": "port",
            "sample": "first %d instances of the same batch, oracle/drc_oracle.c QPIKStep with the "
                      "reference OSQP settings (eps 1e-3, no polish, fresh setup per solve), "
                      "%d pthreads, %.2f s wall" % (n2, threads, dt)}


def load_traffic(robot, B):
    """HBM bytes per drc_qpik_batch call (both kernels) from the committed
    rocprofv3 PMC summary (tools/pmc_summary.py), if it matches this workload
    and this build; else None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as fh:
            d = json.load(fh)
        if d.get("robot") == robot and int(d.get("batch")) == B:
            return d.get("hbm_bytes_per_step")
    except Exception:
        pass
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=65536, help="instances per GPU")
    ap.add_argument("--robot", default="fr3", choices=sorted(LINKS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--chunks", type=int, default=3, help="concurrent sub-batches per call")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from dyros_robot_controller_amd import dist as ddist
    rank, world, local = ddist.env_rank()
    backend = os.environ.get("DRC_DIST_BACKEND", "nccl")   # gloo: rehearse N ranks on one GPU
    if world > 1:
        torch.cuda.set_device(local % max(torch.cuda.device_count(), 1))
        ddist.init(backend, torch.device("cuda", local) if backend == "nccl" else None)
    dev = torch.device("cuda", local % max(torch.cuda.device_count(), 1))
    torch.cuda.set_device(dev)

    from dyros_robot_controller_amd import manipulator, robot_path
    robot, B = args.robot, args.batch
    rd = manipulator.RobotData(robot_path(robot), robot_path(robot, "srdf"), device=dev)
    ctrl = manipulator.RobotController(0.001, rd, solver_mode="exact")
    offset, _ = ddist.shard(rank, B)   # contiguous instance range of this rank
    q, qd, xt, xdt, dq, dqd, dxt, dxdt = make_inputs(rd, robot, B, 12345, offset, dev)
    iters = torch.zeros(B, dtype=torch.int32, device=dev)
    link = LINKS[robot]

    def step():
        return ctrl.QPIK_step_batch(dq, dqd, dxt, dxdt, link, iters=iters)

    from dyros_robot_controller_amd import _capi
    import ctypes as C
    handle = rd.model.handle
    _capi.check(_capi.lib().drc_set_concurrency(handle, args.chunks))
    for _ in range(args.warmup):
        out, status = step()
    torch.cuda.synchronize()
    # per-kernel durations: HIP events recorded by the library on the launch
    # stream around task_kernel and qp_kernel of every timed step
    _capi.check(_capi.lib().drc_debug_kernel_timing(handle, 1))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        out, status = step()
    ev1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    step_event_ms = ev0.elapsed_time(ev1) / args.steps   # HIP events on the launch stream
    tw, tk, tq, nc = C.c_double(), C.c_double(), C.c_double(), C.c_int()
    _capi.check(_capi.lib().drc_debug_kernel_times(handle, C.byref(tw), C.byref(tk), C.byref(tq), C.byref(nc)))
    _capi.check(_capi.lib().drc_debug_kernel_timing(handle, 0))
    ncall = max(nc.value, 1)
    # kernel_ms: one drc_qpik_batch call on its stream (fork -> join of the
    # concurrent sub-batches); task/qp: summed per-sub-batch kernel durations
    kernel_ms, task_ms, qp_ms = tw.value / ncall, tk.value / ncall, tq.value / ncall
    wall, n_bad, it_mean = ddist.reduce_stats(wall, float((status != 1).sum().item()),
                                              float(iters.double().mean().item()), world,
                                              dev if backend == "nccl" else "cpu")

    if rank == 0:
        nv = rd.getDof()
        total = B * world * args.steps
        value = total / wall
        ms_per_step = 1e3 * wall / args.steps
        per_launch_bytes = algorithmic_bytes(nv) * B
        achieved = per_launch_bytes / (kernel_ms * 1e-3) / 1e9
        traffic = load_traffic(robot, B)
        fl = flops_per_solve(nv, it_mean) * B / (kernel_ms * 1e-3) / 1e12
        line = {
            "metric": "QP-IK solves/s (FR3 7-DoF, batch 65k) + achieved HBM GB/s vs peak",
            "value": value, "unit": "solves/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f64", "data": "synthetic",
            "config": {"workload": "%s QPIKStep (exact: certified OSQP polish), %d instances per GPU"
                                   % (robot.upper(), B),
                       "robot": robot, "batch_per_gpu": B, "global_batch": B * world,
                       "parallelism": "dp%d (instances sharded, no data-path collective)" % world},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "drc_qpik_batch call (task_kernel + qp_kernel per sub-batch, %d concurrent "
                                   "sub-batches)" % args.chunks,
                         "bytes_per_solve": algorithmic_bytes(nv), "bytes_per_launch": per_launch_bytes,
                         "kernel_ms": kernel_ms, "task_kernel_ms_sum": task_ms, "qp_kernel_ms_sum": qp_ms,
                         "step_event_ms": step_event_ms,
                         "fp64_valu_estimate": {"achieved_tflops": fl, "peak_tflops": FP64_VECTOR_PEAK_TFS,
                                                "frac": fl / FP64_VECTOR_PEAK_TFS,
                                                "flops_per_solve": flops_per_solve(nv, it_mean)}},
            "non_solved": int(n_bad), "admm_iters_mean": it_mean,
            "admm_iters_p99_max": [float(np.percentile(iters.cpu().numpy(), 99)), int(iters.max().item())],
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(robot, q, qd, xt, xdt)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

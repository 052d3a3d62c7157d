#!/usr/bin/env python3
"""Headline benchmark: batched QP-IK solves/s + achieved HBM GB/s vs peak
(BASELINE.json "metric"), on the configurations BASELINE.json names:

  default       FR3 7-DoF QPIKStep, 65 536 instances per GPU (the metric's config)
  --robot ur5e                     UR5e 6-DoF, 65 536 per GPU (HBM-roofline / counter run)
  --robot husky_fr3 --batch 16384  Husky-FR3 whole-body QPIKStep
  --robot xls_fr3 --global-batch 524288   XLS-FR3 whole-body, fixed global batch over N GPUs
  (also caster_fr3)

One "step" = one control cycle of the batch through the product path
(drc_qpik_batch: task-space kernel + QP kernel), inputs resident in HBM,
SURVEY §8d's workload including the three 10 % stress tiers.  Multi-GPU: one
process per GPU, instances sharded as contiguous ranges with no data-path
collective; weak scaling by default (--batch per GPU), strong scaling with
--global-batch.  A barrier and a max-reduction of the timed region are the
only collectives.  ``--gpus N`` without a torchrun environment starts the N
ranks itself (dist.launch_if_needed); under torchrun, WORLD_SIZE must equal N.

Besides the headline line (exact mode), a single-GPU run reports, outside the
timed region: the same batch at the reference's OSQP settings
(``reference_settings``), the BASELINE config-2 batch of 4 096
(``batch_4096``), and the latency of the reference's per-cycle call — one
synchronous QPIKCubic through the host entry (``latency_b1``, p50 / p99).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--robot fr3] [--batch B | --global-batch G]
                    [--solver exact|osqp_default] [--no-extras] [--no-cpu-baseline]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from dyros_robot_controller_amd import dist as ddist  # noqa: E402  (no torch / GPU at import)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
FP64_VECTOR_PEAK_TFS = 78.6    # AMD spec, FP64 vector
SIMDS = 256 * 4                # CUs x SIMDs (MI355X_MICROARCH.md)
CLOCK_HZ = 2.4e9               # max engine clock (MI355X_MICROARCH.md chip table)
CLOCK_GHZ = 2.4                # MI355X peak engine clock (MI355X_MICROARCH.md)
CUS = 256                      # MI355X compute units (MI355X_MICROARCH.md)
LDS_PER_CU = 160 * 1024        # bytes
DEFAULT_BATCH = {"fr3": 65536, "ur5e": 65536, "husky_fr3": 16384, "xls_fr3": 65536, "caster_fr3": 65536}
METRIC = "QP-IK solves/s (FR3 7-DoF, batch 65k) + achieved HBM GB/s vs peak"


def algorithmic_bytes(dof, actuated):
    """per solve, HBM in (q, qdot [dof], x_target [12],
    xdot_target [6]) + out (qdot* [actuated] f64, status i32).
    FR3 316 B, UR5e 292 B, Husky-FR3 412 B, XLS-FR3 460 B."""
    return (2 * dof + 12 + 6) * 8 + actuated * 8 + 4


def algorithmic_flops(robot, solver, q, qd, xt, xdt, n=256):
    """FP64 operations per solve of the algorithm itself, counted, not
    estimated: the oracle's C restatement built with every double replaced by
    a counting type (oracle/flopcount.hpp, count_build.cpp) runs a strided
    sample of the same batch with the same settings and the kernels' pruned
    narrow phase (oracle min_distance_pruned -- same argmin as all pairs).
    + - * / sqrt count 1 each; sin / cos / atan2 / acos are reported apart.
    ``flops_per_solve`` counts only the operations whose operands are all
    nonzero: the oracle's QP linear algebra is dense (P^T P + A^T rho A at
    n^2 m, dense 39 x 23 products per ADMM iteration), and its work on
    structural zeros -- which OSQP's sparse KKT never does -- drops out.  The
    dense count is reported beside it (``dense_flops_per_solve``)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    _, om, spec = O.load(robot)
    par = O.default_params(spec["kind"], exact=(solver == "exact"))
    idx = np.unique(np.linspace(0, q.shape[1] - 1, n).astype(np.int64))
    pick = lambda a: np.ascontiguousarray(a[:, idx])
    with O.counting_build():
        O.set_pruned_narrow_phase(True)
        try:
            O.flop_counts(reset=True)
            O.qpik_batch(om, par, pick(q), pick(qd), pick(xt), pick(xdt), nthreads=1)
            fl, tr, nz = O.flop_counts(reset=True, nonzero=True)
        finally:
            O.set_pruned_narrow_phase(False)
    return {"flops_per_solve": nz / len(idx), "dense_flops_per_solve": fl / len(idx),
            "transcendentals_per_solve": tr / len(idx),
            "rule": "operations with all operands nonzero (structural zeros of the dense restatement excluded)",
            "sample": "%d instances, every %d-th of the batch" % (len(idx), max(1, q.shape[1] // n)),
            "source": "oracle/count_build.cpp (counting build of oracle/drc_oracle.c, pruned narrow phase)"}


def make_inputs(rd, robot, B, seed, offset, dev):
    """States (with the stress tiers, judged by the product's stage kernel) and
    targets near the current pose, [field][B] numpy + device copies."""
    from dyros_robot_controller_amd import BUNDLED, _batch, _capi, manipulator, workload
    spec = BUNDLED[robot]
    link = spec["link"]
    ev = workload.device_evaluator(rd.model, link, dev)
    if spec["kind"] == "manipulator":
        lo, hi = rd.getJointPositionLimit()
        _, vmax = rd.getJointVelocityLimit()
        q, qd = workload.joint_states(lo, hi, vmax, seed, B, offset)
        arm = list(range(len(lo)))
    else:
        lo, hi = rd.get_joint_position_limit()
        _, vmax = rd.get_joint_velocity_limit()
        ji = rd.get_joint_index()
        q, qd = workload.mobile_states(lo, hi, vmax, (ji.virtual_start, ji.mani_start, ji.mobi_start),
                                       rd.get_manipulator_dof(), rd.get_mobile_dof(), seed, B, offset)
        arm = list(range(ji.mani_start, ji.mani_start + rd.get_manipulator_dof()))
    tier, stats = workload.apply_stress(q, lo, hi, arm, seed, offset, ev)
    p = manipulator.QPIKParamsBuilder(rd.model, exact=True).params(link, _capi.MODE_QPIK)
    dq, dqd = _batch.as_device(q, dev), _batch.as_device(qd, dev)
    st = _batch.stages_batch(rd.model, p, dq, dqd, None, _batch.as_device(np.zeros((6, B)), dev))
    xt, xdt = workload.perturb_targets(st["pose"].cpu().numpy(), seed, B, offset)
    return (q, qd, xt, xdt), (dq, dqd, _batch.as_device(xt, dev), _batch.as_device(xdt, dev)), stats


def cpu_baseline(robot, q, qd, xt, xdt, target_s=4.0, warmups=3, runs=5, sequential=10000):
    """Oracle restatement of the reference CPU path (OSQP-default settings,
    fresh setup per solve) on this host's cores: 1 thread and all threads
    (capped at 16, the box's CPU share), median of 5 timed runs after 3
    warm-ups (BASELINE.md plan).  1 thread: ``sequential`` (10 000, BASELINE.md's
    "FR3 single instance, 10 000 sequential solves") solves one after another
    per timed run, warm-ups on a 256-instance sample; all threads: a bounded
    sample of about target_s / 8 s per run."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    _, om, spec = O.load(robot)
    par = O.default_params(spec["kind"], exact=False)
    cores = max(1, min(16, os.cpu_count() or 1))

    def timed(n, threads):
        t0 = time.perf_counter()
        O.qpik_batch(om, par, q[:, :n], qd[:, :n], xt[:, :n], xdt[:, :n], nthreads=threads)
        return time.perf_counter() - t0

    out = {}
    for threads in (1, cores):
        if threads == 1:
            n = min(q.shape[1], sequential)
            for _ in range(warmups):
                timed(min(n, 256), 1)
        else:
            n = min(q.shape[1], 256 * threads)
            per = timed(n, threads) / n                      # calibration run
            n = int(min(q.shape[1], max(64, target_s / (warmups + runs) / max(per, 1e-9))))
            for _ in range(warmups):
                timed(n, threads)
        ts = sorted(timed(n, threads) for _ in range(runs))
        out[threads] = (n / ts[len(ts) // 2], n)
    (v1, n1), (vc, nc) = out[1], out[cores]
    return {"value": vc, "unit": "solves/s", "cores": cores, "kind": "port",
            "single_thread": {"value": v1, "cores": 1, "sample_instances": n1,
                              "note": "%d sequential solves per timed run (BASELINE.md config 1)" % n1},
            "sample": "first %d instances of the same batch (1 thread: %d sequential), oracle/drc_oracle.c QPIKStep "
                      "with the reference OSQP settings (eps 1e-3, no polish, fresh setup per solve), %d pthreads; "
                      "median of %d timed runs after %d warm-ups" % (nc, n1, cores, runs, warmups)}


def load_profile(name, robot, B, build_id):
    """A committed profiles/ counter summary for this workload and batch,
    measured on THIS library build (its ``build_id`` equals drc_build_id()),
    or None: a summary of another build is never attributed to this one."""
    try:
        with open(os.path.join(ROOT, "profiles", name)) as fh:
            d = json.load(fh)
        if d.get("robot") == robot and int(d.get("batch")) == B and d.get("build_id") == build_id:
            return d
    except Exception:
        pass
    return None


def valu_issue_roof(valu, value, world=1):
    """A hardware roof from a same-build VALU counter summary: every SIMD of
    the job's GPUs issuing VALU work back to back at the maximum clock, over
    the counted issue cycles per solve (None without the count)."""
    cyc = valu.get("valu_issue_cycles_per_solve")
    if not cyc:
        return None
    roof = world * SIMDS * CLOCK_HZ / cyc
    return {"issue_cycles_per_solve": cyc, "valu_insts_per_solve": valu.get("valu_insts_per_solve"),
            "solves_per_s": roof, "frac": value / roof, "n_gpus": world,
            "note": "n_gpus x 1 024 SIMDs x 2.4 GHz over the VALU issue cycles per solve counted on this build "
                    "(SQ_INSTS_VALU and its FP64 classes, task + QP kernels: 4 cycles per wave64 FP64 instruction, "
                    "2 per other VALU instruction); SALU, LDS and memory instructions issue beside it and are not "
                    "charged"}


def timed_steps(torch, step, steps, warmup):
    """Warm-up, then ``steps`` calls bracketed by synchronisation: seconds per
    call (host wall clock over the whole run)."""
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def iter_stats(iters, status):
    it = iters.cpu().numpy()
    return {"non_solved": int((status != 1).sum().item()), "admm_iters_mean": float(it.mean()),
            "admm_iters_p99_max": [float(np.percentile(it, 99)), int(it.max())]}


def latency_b1(rd, robot, q, qd, xt, xdt, solver, calls=400, warmup=20):
    """The reference's per-cycle call (examples/C++/src/fr3_controller.cpp:122-134,
    one QPIKCubic per 1 kHz control cycle): one instance through the
    synchronous host entry drc_qpik_host (what the C++ facade's QPIKCubic
    calls), wall time per call on the host, p50 / p99 / max."""
    import ctypes as C
    from dyros_robot_controller_amd import BUNDLED, _capi, manipulator
    link = BUNDLED[robot]["link"]
    p = manipulator.QPIKParamsBuilder(rd.model, exact=(solver == "exact")).params(
        link, _capi.MODE_QPIK_CUBIC, t=0.3, t0=0.0, duration=1.0)
    col = lambda a: np.ascontiguousarray(a[:, :1])
    q1, qd1, xt1, xdt1 = col(q), col(qd), col(xt), col(xdt)
    xi1, xdi1 = xt1.copy(), np.zeros_like(xdt1)
    xi1[9:] -= 0.02                                  # start 2 cm away: the cubic is mid-profile at t = 0.3
    out = np.zeros((rd.model.actuated_dof, 1))
    st, it = np.zeros(1, np.int32), np.zeros(1, np.int32)
    dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))
    ip = lambda a: a.ctypes.data_as(C.POINTER(C.c_int))
    lib, h = _capi.lib(), rd.model.handle
    ts = []
    import gc
    gc_was = gc.isenabled()
    gc.disable()      # a 1 kHz control loop does not let the collector run inside a cycle
    for k in range(warmup + calls):
        if k == warmup:   # host-side phase stamps of the timed calls (drc_debug_host_timeline)
            _capi.check(lib.drc_debug_host_timeline(h, 1, None, 0, None))
        t0 = time.perf_counter()
        rc = lib.drc_qpik_host(h, C.byref(p), C.c_int64(1), dp(q1), dp(qd1), dp(xt1), dp(xdt1), dp(xi1), dp(xdi1),
                               dp(out), ip(st), ip(it))
        t1 = time.perf_counter()
        _capi.check(rc)
        if k >= warmup:
            ts.append(t1 - t0)
    if gc_was:
        gc.enable()
    tl = np.zeros((calls, 5), np.int64)
    n = C.c_int64()
    _capi.check(lib.drc_debug_host_timeline(h, 0, tl.ctypes.data_as(C.POINTER(C.c_int64)), calls, C.byref(n)))
    ts = np.array(ts) * 1e6
    ph = np.diff(tl[:n.value], axis=1) / 1e3            # pack, enqueue, wait, unpack (us)
    names = ["pack_inputs", "enqueue_copy_launch_copy", "wait_completion", "unpack_outputs"]
    worst = int(np.argmax(ts))
    breakdown = {"p50_us": {k: float(np.percentile(ph[:, i], 50)) for i, k in enumerate(names)},
                 "max_us": {k: float(ph[:, i].max()) for i, k in enumerate(names)},
                 "slowest_call_us": {k: float(ph[worst, i]) for i, k in enumerate(names)} if len(ph) == calls else None,
                 "outside_library_slowest_us": float(ts[worst] - (tl[worst, 4] - tl[worst, 0]) / 1e3)
                 if len(ph) == calls else None,
                 "library_max_us": float((tl[:n.value, 4] - tl[:n.value, 0]).max() / 1e3) if n.value else None,
                 "host_wait": ("poll up to %s us, then block" % os.environ.get("DRC_HOST_WAIT", "300"))
                 if int(os.environ.get("DRC_HOST_WAIT", "300")) else "block",
                 "calls_over_us": {str(t): int(np.sum(ts > t)) for t in (200, 300, 500)}}
    return {"call": "QPIKCubic, B = 1, drc_qpik_host (host buffers in and out, synchronous)",
            "p50_us": float(np.percentile(ts, 50)), "p99_us": float(np.percentile(ts, 99)),
            "max_us": float(ts.max()), "calls": calls, "status": int(st[0]), "admm_iters": int(it[0]),
            "cycle_budget_us": 1000.0, "phases": breakdown}


def BUNDLED_KIND(robot):
    from dyros_robot_controller_amd import BUNDLED
    return BUNDLED[robot]["kind"]


def whole_job(ranks, tier_keys, backend):
    """Whole-job fields of the bench line from the gathered per-rank rows
    [rank, device, pci bus, wall, iters p99, iters max, non-solved,
    instances, tier counts...]: iteration p99 / max are the max over ranks,
    counts are sums; with more than one rank, each rank's row and the
    transport."""
    out = {"admm_iters_p99_max": [float(ranks[:, 4].max()), int(ranks[:, 5].max())],
           "stress_tiers": {k: int(ranks[:, 8 + i].sum()) for i, k in enumerate(tier_keys)}}
    if len(ranks) > 1:
        out["ranks"] = [{"rank": int(r[0]), "device": int(r[1]), "pci_bus_id": int(r[2]), "wall_s": float(r[3]),
                         "instances": int(r[7]), "non_solved": int(r[6]),
                         "admm_iters_p99_max": [float(r[4]), int(r[5])]} for r in ranks]
        out["backend"] = backend
    return out


def latency_cycle(robot, q, qd, solver, cycles=400, warmup=20):
    """The reference's whole per-cycle call chain at B = 1
    (examples/C++/src/fr3_controller.cpp:66-68,123-134 at 1 kHz,
    examples/README.md:55): updateState -> getPose -> getVelocity ->
    QPIKCubic -> moveJointTorqueStep(q + qdot* dt, qdot*), through the
    pybind11 module with the reference's binding names (its C++ facade: the
    getters share one drc_state_host round trip per state, the torque step
    reads the cached M and g, QPIKCubic is one drc_qpik_host call).  Host wall
    time per cycle: p50 / p99 / max; each cycle takes the next instance's state."""
    sys.path.insert(0, os.path.join(ROOT, "dyros_robot_controller_amd", "python"))
    import dyros_robot_controller_cpp_wrapper as drc
    from dyros_robot_controller_amd import BUNDLED, robot_path
    link, dt = BUNDLED[robot]["link"], 0.001
    rd = drc.ManipulatorRobotData(robot_path(robot), robot_path(robot, "srdf"), "")
    rc = drc.ManipulatorRobotController(dt, rd)
    if solver != "exact":
        rc.setExact(False)
    ts, bad = [], 0
    n = q.shape[1]
    for k in range(warmup + cycles):
        qk, qdk = np.ascontiguousarray(q[:, k % n]), np.ascontiguousarray(qd[:, k % n])
        t0 = time.perf_counter()
        rd.updateState(qk, qdk)
        x = rd.getPose(link)
        xdot = rd.getVelocity(link)
        xt = x.copy()
        xt[:3, 3] += (0.0, 0.1, 0.1)                      # fr3_controller.cpp:123-131
        qdot_star = rc.QPIKCubic(xt, np.zeros(6), x, xdot, 0.3, 0.0, 3.0, link)
        tau = rc.moveJointTorqueStep(qk + qdot_star * dt, qdot_star)
        t1 = time.perf_counter()
        if k >= warmup:
            ts.append(t1 - t0)
            bad += int(not np.all(np.isfinite(tau)))
    ts = np.array(ts) * 1e6
    return {"call": "updateState, getPose, getVelocity, QPIKCubic, moveJointTorqueStep (B = 1, pybind11 module "
                    "dyros_robot_controller_cpp_wrapper over the C++ facade)",
            "p50_us": float(np.percentile(ts, 50)), "p99_us": float(np.percentile(ts, 99)),
            "max_us": float(ts.max()), "cycles": cycles, "nonfinite_tau": bad, "cycle_budget_us": 1000.0,
            "round_trips_per_cycle": 2}


def dry_run(args):
    """Launcher / sharding / reduction rehearsal without a GPU (tests): every
    rank reports its shard through the same collectives the bench uses."""
    import torch.distributed as dist
    rank, world, _ = ddist.env_rank()
    backend = os.environ.get("DRC_DIST_BACKEND", "gloo")
    if world > 1:
        ddist.init(backend)
    B = args.batch or DEFAULT_BATCH[args.robot]
    offset, cnt = ddist.shard_global(rank, world, args.global_batch) if args.global_batch else ddist.shard(rank, B)
    wall, n_cnt, off_mean = ddist.reduce_stats(0.001 * (rank + 1), cnt, offset, world)
    # the same per-rank rows and whole-job reduction as the GPU path, with
    # rank-dependent stand-in values: iters p99 = rank + 1, max = 10 (rank + 1),
    # non-solved = rank, tier counts (rank, 2 rank)
    tier_keys = ["collision", "singular"]
    ranks = ddist.gather_stats([rank, rank, -1, 0.001 * (rank + 1), rank + 1.0, 10.0 * (rank + 1), float(rank),
                                float(cnt), float(rank), 2.0 * rank], world)
    if rank == 0:
        line = {"dry_run": True, "n_gpus": world, "ranks_reporting": world, "instances": int(n_cnt),
                "max_wall": wall, "mean_offset": off_mean}
        line.update(whole_job(ranks, tier_keys, backend))
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--robot", default="fr3", choices=sorted(DEFAULT_BATCH))
    ap.add_argument("--batch", type=int, default=None, help="instances per GPU (weak scaling)")
    ap.add_argument("--global-batch", type=int, default=None, help="fixed total instances (strong scaling)")
    ap.add_argument("--solver", default="exact", choices=("exact", "osqp_default"),
                    help="exact: certified optimum (parity contract); osqp_default: the reference's OSQP settings")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip reference_settings / batch_4096 / latency_b1")
    ap.add_argument("--chunks", type=int, default=4, help="concurrent sub-batches per call")
    ap.add_argument("--task-stage", type=int, default=0, choices=(0, 1, 2),
                    help="0 wave-per-instance task kernel (default), 1 lane stage + side-stream hand-backs, "
                         "2 lane stage + serial hand-backs (drc_debug_lane_stage)")
    ap.add_argument("--dry-run", action="store_true", help="launcher and collectives only (no GPU)")
    ap.add_argument("--no-kernel-events", action="store_true",
                    help="study: no per-kernel HIP events in the timed region (roofline kernel times then null)")
    args = ap.parse_args()

    rc = ddist.launch_if_needed(args.gpus, os.path.abspath(__file__), sys.argv[1:])
    if rc is not None:          # this process launched the ranks; it never touched the GPU
        sys.exit(rc)
    if args.dry_run:
        return dry_run(args)

    import torch
    import torch.distributed as dist

    from dyros_robot_controller_amd import BUNDLED, _capi, make_robot
    from dyros_robot_controller_amd import manipulator, mobile_manipulator
    rank, world, local = ddist.env_rank()
    backend = os.environ.get("DRC_DIST_BACKEND", "nccl")   # gloo: rehearse N ranks on one GPU
    ndev = max(torch.cuda.device_count(), 1)
    dev = torch.device("cuda", local % ndev)
    torch.cuda.set_device(dev)
    if world > 1:
        ddist.init(backend, dev if backend == "nccl" else None)
    red_dev = dev if backend == "nccl" else "cpu"

    robot = args.robot
    spec = BUNDLED[robot]
    if args.global_batch:
        offset, B = ddist.shard_global(rank, world, args.global_batch)
        scaling, total_per_step = "strong", args.global_batch
    else:
        B = args.batch or DEFAULT_BATCH[robot]
        offset, _ = ddist.shard(rank, B)   # contiguous instance range of this rank
        scaling, total_per_step = "weak", B * world
    rd = make_robot(robot, dev)
    mod = manipulator if spec["kind"] == "manipulator" else mobile_manipulator
    ctrl = mod.RobotController(0.001, rd, solver_mode=args.solver)
    (q, qd, xt, xdt), (dq, dqd, dxt, dxdt), tiers = make_inputs(rd, robot, B, 12345, offset, dev)
    iters = torch.zeros(B, dtype=torch.int32, device=dev)
    link = spec["link"]

    def step():
        return ctrl.QPIK_step_batch(dq, dqd, dxt, dxdt, link, iters=iters)

    import ctypes as C
    handle = rd.model.handle
    _capi.check(_capi.lib().drc_set_concurrency(handle, args.chunks))
    _capi.check(_capi.lib().drc_debug_lane_stage(handle, args.task_stage))
    for _ in range(args.warmup):
        out, status = step()
    torch.cuda.synchronize()
    # per-kernel durations: HIP events recorded by the library on the launch
    # stream around task_kernel and qp_kernel of every timed step
    _capi.check(_capi.lib().drc_debug_kernel_timing(handle, 0 if args.no_kernel_events else 1))
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
    wall_local = wall
    step_event_ms = ev0.elapsed_time(ev1) / args.steps   # HIP events on the launch stream
    tw, tk, tq, nc = C.c_double(), C.c_double(), C.c_double(), C.c_int()
    _capi.check(_capi.lib().drc_debug_kernel_times(handle, C.byref(tw), C.byref(tk), C.byref(tq), C.byref(nc)))
    _capi.check(_capi.lib().drc_debug_kernel_timing(handle, 0))
    ncall = max(nc.value, 1)
    # kernel_ms: one drc_qpik_batch call on its stream (fork -> join of the
    # concurrent sub-batches); task/qp: summed per-sub-batch kernel durations
    kernel_ms, task_ms, qp_ms = tw.value / ncall, tk.value / ncall, tq.value / ncall
    if nc.value == 0:   # --no-kernel-events (study): the call's own stream events stand in
        kernel_ms = step_event_ms
    wall, n_bad, it_mean = ddist.reduce_stats(wall, float((status != 1).sum().item()),
                                              float(iters.double().mean().item()), world, red_dev)
    # per-rank statistics, gathered whole-job: iteration p99 / max (max over
    # ranks), stress-tier counts (sums), each rank's device and its timed wall
    it_np = iters.cpu().numpy()
    tier_keys = sorted(tiers)
    props = torch.cuda.get_device_properties(dev)
    per_rank = [rank, dev.index, getattr(props, "pci_bus_id", -1), wall_local,
                float(np.percentile(it_np, 99)), float(it_np.max()), float((status != 1).sum().item()),
                float(B)] + [float(tiers[k]) for k in tier_keys]
    ranks = ddist.gather_stats(per_rank, world, red_dev)

    if rank == 0:
        build = _capi.build_id()
        dof, act = rd.model.dof, rd.model.actuated_dof
        total = total_per_step * args.steps
        value = total / wall
        ms_per_step = 1e3 * wall / args.steps
        bps = algorithmic_bytes(dof, act)
        per_launch_bytes = bps * B
        # the library runs calls of up to DRC_FUSE_MAX (default 16 384) instances
        # of the compiled (bundled) shapes as one fused task + QP launch
        fuse_max = int(os.environ.get("DRC_FUSE_MAX", "16384"))
        fused = B <= fuse_max
        achieved = per_launch_bytes / (kernel_ms * 1e-3) / 1e9
        # counter summaries are used only when measured on this very build
        traffic = load_profile("pmc_traffic_%s.json" % robot, robot, B, build)
        alg = algorithmic_flops(robot, args.solver, q, qd, xt, xdt)
        fl = alg["flops_per_solve"] * B / (kernel_ms * 1e-3) / 1e12
        roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic.get("hbm_bytes_per_step") if traffic else None,
                "traffic_source": ("profiles/pmc_traffic_%s.json (build %s)" % (robot, build)) if traffic else
                                  "no PMC summary of this build (%s) for this robot and batch" % build,
                "kernel": ("drc_qpik_batch call (one fused_kernel launch: B <= DRC_FUSE_MAX = %d; "
                           "task_kernel_ms_sum is its duration)" % fuse_max) if fused else
                          ("drc_qpik_batch call (task_kernel + qp_kernel per sub-batch, %d concurrent sub-batches)"
                           % args.chunks),
                "bytes_per_solve": bps, "bytes_per_launch": per_launch_bytes,
                "kernel_ms": kernel_ms, "task_kernel_ms_sum": task_ms, "qp_kernel_ms_sum": qp_ms,
                "step_event_ms": step_event_ms,
                "fp64_algorithmic": dict(alg, achieved_tflops=fl, peak_tflops=FP64_VECTOR_PEAK_TFS,
                                         frac=fl / FP64_VECTOR_PEAK_TFS)}
        valu = load_profile("valu_counters_%s.json" % robot, robot, B, build)
        if valu:   # counter-based FP64 work per call (tools/valu_summary.py over rocprofv3 --pmc passes)
            f = valu["fp64_flops_per_step"]
            eff = valu.get("lane_efficiency") or 0.0
            issued = f / (kernel_ms * 1e-3) / 1e12
            roof["fp64_valu"] = {"issued_tflops": issued, "executed_tflops": issued * eff,
                                 "peak_tflops": FP64_VECTOR_PEAK_TFS,
                                 "issued_frac": issued / FP64_VECTOR_PEAK_TFS,
                                 "executed_frac": issued * eff / FP64_VECTOR_PEAK_TFS,
                                 "fp64_flops_issued_per_step": f, "lane_efficiency": eff,
                                 "executed_flops_per_solve": f * eff / B,
                                 "algorithmic_over_executed": alg["flops_per_solve"] / max(f * eff / B, 1e-30),
                                 "note": "issued counts 64 lanes per FP64 instruction; executed = issued x lane "
                                         "efficiency (active lanes); neither is algorithmic work",
                                 "source": "profiles/valu_counters_%s.json (build %s)" % (robot, build)}
            ir = valu_issue_roof(valu, value, world)
            if ir:
                roof["valu_issue_roof"] = dict(ir, source="profiles/valu_counters_%s.json (build %s)" % (robot, build))
        line = {
            "metric": METRIC, "value": value, "unit": "solves/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": scaling,
            "vs_baseline": None, "dtype": "f64", "data": "synthetic (SURVEY 8d workload with the stress tiers)",
            "config": {"workload": "%s QPIKStep (%s), %d instances per GPU%s"
                                   % (robot.upper(), "exact: certified OSQP polish" if args.solver == "exact"
                                      else "reference OSQP settings: eps 1e-3, no polish", B,
                                      ", global batch %d" % args.global_batch if args.global_batch else ""),
                       "robot": robot, "batch_per_gpu": B, "global_batch": total_per_step, "solver": args.solver,
                       "parallelism": "dp%d (instances sharded, no data-path collective)" % world,
                       "task_stage": ["wave-per-instance", "lane-per-instance + side-stream hand-backs",
                                      "lane-per-instance + serial hand-backs"][args.task_stage]},
            "roofline": roof,
            "build_id": build,
            # whole-job counters over every rank's instances
            "non_solved": int(n_bad), "admm_iters_mean": it_mean,
        }
        line.update(whole_job(ranks, tier_keys, backend))
        if world == 1 and not args.no_extras:
            extras(torch, args, rd, mod, robot, link, q, qd, xt, xdt, dq, dqd, dxt, dxdt, line)
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(robot, q, qd, xt, xdt)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def extras(torch, args, rd, mod, robot, link, q, qd, xt, xdt, dq, dqd, dxt, dxdt, line):
    """Single-GPU side measurements, outside the headline's timed region."""
    B = dq.shape[1]
    other = "osqp_default" if args.solver == "exact" else "exact"
    ctrl_o = mod.RobotController(0.001, rd, solver_mode=other)
    it_o = torch.zeros(B, dtype=torch.int32, device=dq.device)
    res = {}
    s = timed_steps(torch, lambda: res.update(r=ctrl_o.QPIK_step_batch(dq, dqd, dxt, dxdt, link, iters=it_o)),
                    args.steps, 2)
    line["reference_settings" if other == "osqp_default" else "exact_settings"] = dict(
        solver=other, value=B / s, unit="solves/s", ms_per_step=1e3 * s, **iter_stats(it_o, res["r"][1]))
    # BASELINE config 2: batch 4 096 (first instances of the same workload)
    nb = min(4096, B)
    sub = [t[:, :nb].contiguous() for t in (dq, dqd, dxt, dxdt)]
    ctrl = mod.RobotController(0.001, rd, solver_mode=args.solver)
    it_s = torch.zeros(nb, dtype=torch.int32, device=dq.device)
    s = timed_steps(torch, lambda: res.update(r=ctrl.QPIK_step_batch(*sub, link, iters=it_s)), max(args.steps, 20), 3)
    line["batch_%d" % nb] = dict(value=nb / s, unit="solves/s", ms_per_step=1e3 * s, **iter_stats(it_s, res["r"][1]))
    line["latency_b1"] = latency_b1(rd, robot, q, qd, xt, xdt, args.solver)
    if BUNDLED_KIND(robot) == "manipulator":
        line["latency_cycle"] = latency_cycle(robot, q, qd, args.solver)
    # latency roof: one instance alone on the chip (B = 1 device time) bounds a
    # wave-per-instance design at WAVE_SLOTS / latency solves/s
    import ctypes as C
    from dyros_robot_controller_amd import _capi
    # mean over the first 32 instances, each alone on the GPU (B = 1 calls)
    lib, h = _capi.lib(), rd.model.handle
    it1 = torch.zeros(1, dtype=torch.int32, device=dq.device)
    ones = [[t[:, k:k + 1].contiguous() for t in (dq, dqd, dxt, dxdt)] for k in range(32)]
    # the two-kernel pipeline (what a full batch runs): task and QP kernel apart
    # (the params builder fills the model kind's defaults: manipulator or whole-body)
    from dyros_robot_controller_amd import manipulator as _man
    p1 = _man.QPIKParamsBuilder(rd.model, exact=(args.solver == "exact")).params(link, _capi.MODE_QPIK_STEP)
    _capi.check(lib.drc_set_fusion(h, C.c_int(0)))
    try:
        for one in ones:
            ctrl.QPIK_step_batch(*one, link, iters=it1)
        torch.cuda.synchronize()
        _capi.check(lib.drc_debug_kernel_timing(h, 1))
        for one in ones:
            for _ in range(3):
                ctrl.QPIK_step_batch(*one, link, iters=it1)
        torch.cuda.synchronize()
        tw, tk, tq, nc = C.c_double(), C.c_double(), C.c_double(), C.c_int()
        _capi.check(lib.drc_debug_kernel_times(h, C.byref(tw), C.byref(tk), C.byref(tq), C.byref(nc)))
        _capi.check(lib.drc_debug_kernel_timing(h, 0))
        # task / QP latency (seconds) from the kernels' own per-instance stamps
        # (drc_debug_qpik_stamps: task start -> end, QP start -> stored); HIP events
        # between two back-to-back kernels on one stream put most of the QP
        # kernel's time into the task kernel's on this stack (r05 stamp study)
        dpp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))
        ipp = lambda a: a.ctypes.data_as(C.POINTER(C.c_int))
        nout = rd.model.actuated_dof
        lts, lqs = [], []
        for one in ones:
            cols = [np.ascontiguousarray(t.cpu().numpy()) for t in one]
            o1, s1, i1 = np.zeros((nout, 1)), np.zeros(1, np.int32), np.zeros(1, np.int32)
            stp = np.zeros((8, 1), np.uint64)
            for _ in range(2):
                _capi.check(lib.drc_debug_qpik_stamps(h, C.byref(p1), C.c_int64(1), dpp(cols[0]), dpp(cols[1]),
                                                      dpp(cols[2]), dpp(cols[3]), dpp(cols[2]), dpp(cols[3]), dpp(o1),
                                                      ipp(s1), ipp(i1), stp.ctypes.data_as(C.POINTER(C.c_uint64))))
            t = stp[:6, 0].astype(np.int64)
            lts.append((t[1] - t[0]) * 1e-8)
            lqs.append((t[5] - t[2]) * 1e-8)
    finally:
        _capi.check(lib.drc_set_fusion(h, C.c_int(1)))
    lt, lq = float(np.mean(lts)), float(np.mean(lqs))
    # waves per CU of each kernel as the call launches it: the register build's
    # waves per SIMD (drc_debug_waves) x 4, capped by the LDS plan (drc_debug_lds_plan)
    p = p1
    wt, wq, bt, bq, bf = C.c_int(), C.c_int(), C.c_int(), C.c_int(), C.c_int()
    _capi.check(lib.drc_debug_waves(h, C.byref(p), C.byref(wt), C.byref(wq)))
    _capi.check(lib.drc_debug_lds_plan(h, C.byref(p), 0, C.byref(bt), C.byref(bq), C.byref(bf)))
    cu_t = min(4 * wt.value, LDS_PER_CU // max(bt.value, 1))
    cu_q = min(4 * wq.value, LDS_PER_CU // max(bq.value, 1))
    # an instance holds a task-wave slot for lt and a QP-wave slot for lq:
    # CUS / (lt / cu_t + lq / cu_q) instances per second with every slot busy
    roof = CUS / (lt / cu_t + lq / cu_q)
    line["roofline"]["latency_roof"] = {
        "instance_latency_us": 1e6 * (lt + lq), "task_latency_us": 1e6 * lt, "qp_latency_us": 1e6 * lq,
        "call_us": 1e3 * tw.value / max(nc.value, 1), "task_waves_per_cu": cu_t, "qp_waves_per_cu": cu_q,
        "solves_per_s": roof, "frac": line["value"] / roof,
        "note": "design-relative, not a hardware limit (the hardware roof is valu_issue_roof): task and QP kernel "
                "latency of one instance alone on the GPU (mean over the batch's first 32 instances, B = 1 calls "
                "through the two-kernel pipeline, the kernels' own stage stamps; call_us from HIP events); with the "
                "waves per CU each kernel is launched at (register build x 4 SIMDs, capped "
                "by its LDS plan), 256 CUs complete 256 / (t_task / w_task + t_qp / w_qp) instances per second "
                "if every wave slot stays busy at the isolated latency"}


if __name__ == "__main__":
    main()

"""Small-batch makespan study (diagnostic): where one QPIKStep call's time goes,
from the kernels' per-instance stage stamps (drc_debug_qpik_stamps: clock at
task start / end, QP start / assembled / solved / stored, and the workgroup,
CU and SIMD each stage ran on).  For each case: the call's span on the device,
per-instance task and QP durations, the mean number of instances in flight
per stage against the wave slots, when the in-flight count falls off (the
tail), the busiest wave's chain and the slowest instances.  Also the isolated
B = 1 task / QP durations (the latency roof's inputs) from the same stamps.
JSON lines on stdout.

    python tools/stamp_study.py [--robot fr3] [--batch 4096] [--fusion -1|0|1] [--single 32]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
TICK_US = 0.01          # s_memrealtime: 100 MHz


def run(lib, h, p, cols, B, nrow):
    dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))
    ip = lambda a: a.ctypes.data_as(C.POINTER(C.c_int))
    q, qd, xt, xdt = cols
    out = np.zeros((nrow, B))
    st, it = np.zeros(B, np.int32), np.zeros(B, np.int32)
    stamps = np.zeros((8, B), np.uint64)
    from dyros_robot_controller_amd import _capi
    _capi.check(lib.drc_debug_qpik_stamps(h, C.byref(p), C.c_int64(B), dp(q), dp(qd), dp(xt), dp(xdt), dp(xt),
                                          dp(xdt), dp(out), ip(st), ip(it),
                                          stamps.ctypes.data_as(C.POINTER(C.c_uint64))))
    return stamps, st, it


def analyse(stamps, st, it, slots):
    s = stamps[:6].astype(np.int64)
    ok = np.all(s > 0, axis=0) & np.all(np.diff(s, axis=0) >= 0, axis=0)
    s = s[:, ok]
    t0 = s[0].min()
    s = (s - t0) * TICK_US                                  # us from the first task start
    span = s[5].max()
    task, wait, qp = s[1] - s[0], s[2] - s[1], s[5] - s[2]
    pct = lambda a: {k: round(float(np.percentile(a, v)), 2) for k, v in (("p50", 50), ("p99", 99))} | {
        "mean": round(float(a.mean()), 2), "max": round(float(a.max()), 2)}
    # instances in flight over the span (1 us bins)
    nb = int(np.ceil(span)) + 1
    grid = np.arange(nb)
    fl_t = np.zeros(nb)
    fl_q = np.zeros(nb)
    for a, b, fl in ((s[0], s[1], fl_t), (s[2], s[5], fl_q)):
        np.add.at(fl, np.clip(np.floor(a).astype(int), 0, nb - 1), 1)
        np.add.at(fl, np.clip(np.floor(b).astype(int), 0, nb - 1), -1)
    fl_t, fl_q = np.cumsum(fl_t), np.cumsum(fl_q)
    busy = fl_t + fl_q
    peak = busy.max()
    half = grid[busy >= 0.5 * peak]
    tail_from = float(half.max()) if len(half) else 0.0
    # chains: instances per workgroup of the stage that ran them (fused: one wave does both)
    wt = (stamps[6, ok] >> np.uint64(32)).astype(np.int64)
    wq = (stamps[7, ok] >> np.uint64(32)).astype(np.int64)
    simd = (stamps[7, ok] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    chain = {}
    for w, a, b in zip(wq, s[2], s[5]):
        c = chain.setdefault(int(w), [0.0, 0, 1e30, 0.0])
        c[0] += b - a
        c[1] += 1
        c[2] = min(c[2], a)
        c[3] = max(c[3], b)
    busiest = max(chain.items(), key=lambda kv: kv[1][3])
    order = np.argsort(-(s[5] - s[0]))[:5]
    return {
        "instances": int(ok.sum()), "span_us": round(float(span), 2),
        "task_us": pct(task), "record_wait_us": pct(wait), "qp_us": pct(qp),
        "mean_in_flight": {"task": round(float(task.sum() / span), 1), "qp": round(float(qp.sum() / span), 1),
                           "slots": slots},
        "peak_in_flight": int(peak), "below_half_peak_from_us": tail_from,
        "waves_used": len(chain), "simds_used": int(len(np.unique(simd))),
        "latest_wave": {"instances": busiest[1][1], "busy_us": round(busiest[1][0], 2),
                        "first_us": round(busiest[1][2], 2), "last_us": round(busiest[1][3], 2)},
        "slowest_instances": [{"b": int(np.nonzero(ok)[0][k]), "task_us": round(float(task[k]), 2), "qp_us": round(float(qp[k]), 2),
                               "start_us": round(float(s[0][k]), 2), "iters": int(it[ok][k]),
                               "status": int(st[ok][k])} for k in order],
        "iters": {"mean": round(float(it[ok].mean()), 2), "max": int(it[ok].max())},
        "in_flight_profile_us": [[int(g), int(busy[g])] for g in grid[:: max(1, nb // 24)]],
    }


def main():
    import torch
    import bench
    from dyros_robot_controller_amd import BUNDLED, _capi, make_robot, manipulator
    ap = argparse.ArgumentParser()
    ap.add_argument("--robot", default="fr3")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--fusion", type=int, default=-1, help="-1: the library's choice, 0 pipeline, 1 fused")
    ap.add_argument("--concurrency", type=int, default=0)
    ap.add_argument("--single", type=int, default=32)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--order", default="",
                    help="comma list of scheduling orders to compare with the queue order (drc_debug_instance_order): "
                         "lpt (longest task + QP first, from this run's stamps: the perfect-knowledge bound), "
                         "task (longest task first), hint (instances a cheap narrow-phase bound flags first: "
                         "oracle_epa_predict's lower bound, host-side)")
    ap.add_argument("--subbatches", type=int, default=1, help="sub-batches the call runs as (orders stay inside each)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    rd = make_robot(a.robot, dev)
    link = BUNDLED[a.robot]["link"]
    lib, h = _capi.lib(), rd.model.handle
    p = manipulator.QPIKParamsBuilder(rd.model, exact=True).params(link, _capi.MODE_QPIK_STEP)
    host, _, _ = bench.make_inputs(rd, a.robot, max(a.batch, a.single), 12345, 0, dev)
    cols = [np.ascontiguousarray(x, dtype=np.float64) for x in host]
    nrow = rd.model.actuated_dof
    wt, wq = C.c_int(), C.c_int()
    _capi.check(lib.drc_debug_waves(h, C.byref(p), C.byref(wt), C.byref(wq)))
    if a.fusion >= 0:
        _capi.check(lib.drc_set_fusion(h, C.c_int(a.fusion)))
    if a.concurrency > 0:
        _capi.check(lib.drc_set_concurrency(h, C.c_int(a.concurrency)))
    sub = [np.ascontiguousarray(c[:, :a.batch]) for c in cols]
    for _ in range(a.reps):
        stamps, st, it = run(lib, h, p, sub, a.batch, nrow)
    fused = a.fusion == 1 or (a.fusion < 0 and a.batch <= 8192 and a.robot != "caster_fr3")
    slots = {"task_waves_per_simd": wt.value, "qp_waves_per_simd": wq.value, "fused": fused}
    r = analyse(stamps, st, it, slots)
    # the slowest instances' inputs and outputs, for the oracle on the CPU
    slow = [row["b"] for row in r["slowest_instances"]] + [int(b) for b in np.nonzero(it > 40)[0][:16]]
    slow = sorted(set(slow))
    np.savez(os.path.join(ROOT, "gpurun_out", "stamps_slow_%s_%d.npz" % (a.robot, a.batch)), b=np.array(slow),
             q=sub[0][:, slow], qd=sub[1][:, slow], xt=sub[2][:, slow], xdt=sub[3][:, slow], iters=it[slow],
             status=st[slow])
    r.update(robot=a.robot, batch=a.batch, fusion=a.fusion, concurrency=a.concurrency)
    print(json.dumps(r), flush=True)
    if a.order:
        s6 = stamps[:6].astype(np.int64)
        dur_all = (s6[5] - s6[0]).astype(np.float64)
        dur_task = (s6[1] - s6[0]).astype(np.float64)
        flags = None
        S = a.subbatches
        cuts = [a.batch * c // S for c in range(S + 1)]
        for name in a.order.split(","):
            if name == "hint" and flags is None:
                sys.path.insert(0, os.path.join(ROOT, "oracle"))
                import oracle as O
                om = O.load(a.robot)[1]
                t_, lb_, co_ = C.c_int(), C.c_int(), C.c_int()
                flags = np.zeros(a.batch, bool)
                for b in range(a.batch):
                    O.lib().oracle_epa_predict(C.byref(om), np.ascontiguousarray(sub[0][:, b]).ctypes.data_as(
                        C.POINTER(C.c_double)), C.byref(t_), C.byref(lb_), C.byref(co_))
                    flags[b] = lb_.value != 0
            key = {"lpt": -dur_all, "task": -dur_task, "hint": None}[name]
            order = np.zeros(a.batch, np.int32)
            for c in range(S):
                lo_, hi_ = cuts[c], cuts[c + 1]
                idx = np.arange(lo_, hi_)
                if name == "hint":
                    k = np.argsort(~flags[lo_:hi_], kind="stable")
                else:
                    k = np.argsort(key[lo_:hi_], kind="stable")
                order[lo_:hi_] = idx[k]
            _capi.check(lib.drc_debug_instance_order(h, order.ctypes.data_as(C.POINTER(C.c_int32)),
                                                     C.c_int64(a.batch)))
            for _ in range(a.reps):
                st2, s2, i2 = run(lib, h, p, sub, a.batch, nrow)
            assert np.array_equal(s2, st) and np.array_equal(i2, it)
            r2 = analyse(st2, s2, i2, slots)
            print(json.dumps({"robot": a.robot, "batch": a.batch, "order": name,
                              "flagged": float(flags.mean()) if name == "hint" else None,
                              "span_us": r2["span_us"], "below_half_peak_from_us": r2["below_half_peak_from_us"],
                              "task_us": r2["task_us"], "qp_us": r2["qp_us"],
                              "slowest_instances": r2["slowest_instances"][:3]}), flush=True)
        _capi.check(lib.drc_debug_instance_order(h, None, C.c_int64(0)))
    # isolated instances: B = 1 calls through the two-kernel pipeline and the fused kernel
    for fz in (0, 1):
        _capi.check(lib.drc_set_fusion(h, C.c_int(fz)))
        tk, tq = [], []
        for k in range(a.single):
            one = [np.ascontiguousarray(c[:, k:k + 1]) for c in cols]
            for _ in range(2):
                stamps, st, it = run(lib, h, p, one, 1, nrow)
            s = stamps[:6, 0].astype(np.int64)
            tk.append((s[1] - s[0]) * TICK_US)
            tq.append((s[5] - s[2]) * TICK_US)
        print(json.dumps({"robot": a.robot, "single_instances": a.single, "fusion": fz,
                          "task_us_mean": round(float(np.mean(tk)), 2), "qp_us_mean": round(float(np.mean(tq)), 2),
                          "task_us_max": round(float(np.max(tk)), 2), "qp_us_max": round(float(np.max(tq)), 2)}),
              flush=True)
    _capi.check(lib.drc_set_fusion(h, C.c_int(1)))


if __name__ == "__main__":
    main()

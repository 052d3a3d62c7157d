"""QP stragglers on the CPU (diagnostic; test infrastructure): the bench
workload's instances whose exact-mode QPIKStep needs the most ADMM
iterations, each re-run alone through the oracle with the polish census on
(oracle_polish_census), so their polish attempts, EQP solves and active-set
steps can be set against a typical instance's.  These instances are the
makespan of a small batch (tools/stamp_study.py).

    python tools/straggler_study.py [--robot fr3] [--batch 4096] [--seed 12345] [--top 8]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tools")]


def one(O, om, par, inputs, b):
    L = O.lib()
    out = (C.c_longlong * (8 + 8 + 3 * 16))()
    t = (C.c_double * 16)(*([1e-6] * 16))
    L.oracle_polish_census(C.c_int(1), t, out, C.c_int(1))
    _, st, it = O.qpik_batch(om, par, *[x[:, b:b + 1].copy() for x in inputs], nthreads=1)
    L.oracle_polish_census(C.c_int(0), None, out, C.c_int(1))
    v = list(out)
    return {"b": int(b), "iters": int(it[0]), "status": int(st[0]), "polish_calls": v[0], "certified": v[1],
            "eqp": v[2], "add_steps": v[3], "drop_steps": v[4], "ratio_blocks": v[5], "eqp_hist": v[8:16]}


def main():
    import oracle as O
    from polish_census import workload
    ap = argparse.ArgumentParser()
    ap.add_argument("--robot", default="fr3")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--seed", type=int, default=12345)
    ap.add_argument("--top", type=int, default=8)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--npz", help="instances dumped by tools/stamp_study.py (the device's inputs and iterations)")
    a = ap.parse_args()
    _, om, spec = O.load(a.robot)
    par = O.default_params(spec["kind"], exact=True)
    if a.npz:
        d = np.load(a.npz)
        inputs = [np.ascontiguousarray(d[k]) for k in ("q", "qd", "xt", "xdt")]
        for k, b in enumerate(d["b"]):
            r = one(O, om, par, inputs, k)
            r.update(b=int(b), device_iters=int(d["iters"][k]), device_status=int(d["status"][k]))
            print(json.dumps(r))
        return
    inputs = workload(om, a.robot, a.batch, a.seed)
    _, st, it = O.qpik_batch(om, par, *inputs, nthreads=a.threads)
    vals, cnt = np.unique(it, return_counts=True)
    print(json.dumps({"robot": a.robot, "batch": a.batch, "iters_hist": {int(k): int(c) for k, c in zip(vals, cnt)}}))
    for b in np.argsort(-it, kind="stable")[:a.top]:
        print(json.dumps(one(O, om, par, inputs, b)))
    typ = [b for b in range(a.batch) if it[b] == np.median(it)][:3]
    for b in typ:
        print(json.dumps(dict(one(O, om, par, inputs, b), typical=True)))


if __name__ == "__main__":
    main()

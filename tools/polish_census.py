"""Certified-polish census on the CPU (diagnostic; test infrastructure).

Builds the bench workload of one robot on the host (the stress tiers judged by
the oracle's manipulability / min distance, targets around the oracle's FK
pose -- the same generator as bench.py, with the oracle as stage evaluator),
runs the oracle's exact-mode QPIKStep and reports the polish's step counts and
how well alternative first guesses of the active set match the set each
successful polish certifies (oracle/drc_oracle.c: oracle_polish_census).

    python tools/polish_census.py [--robot fr3] [--batch 2048] [--seed 1]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

RULES = ["osqp z", "osqp Ax", "dual sign", "primal near", "osqp z + violated", "osqp z widened",
         "osqp Ax widened", "primal near & dual sign | violated", "bound: diag Newton trial", "bound: diag Newton | osqp", "r10", "pGS 1", "pGS 2", "pGS 4", "pJacobi 3"]


def workload(om, robot, B, seed):
    import oracle as O
    from dyros_robot_controller_amd import workload as W
    lo = np.array(om.lower[:om.nv])
    hi = np.array(om.upper[:om.nv])
    v = np.array(om.vel[:om.nv])
    q, qd = W.joint_states(lo, hi, v, seed, B, 0)

    def ev(qs):
        m = [O.manipulability(om, qs[:, b])[0] for b in range(qs.shape[1])]
        d = [O.min_distance(om, qs[:, b])[0] for b in range(qs.shape[1])]
        return np.array(m), np.array(d)
    W.apply_stress(q, lo, hi, list(range(om.nv)), seed, 0, ev)
    pose = np.zeros((12, B))
    for b in range(B):
        p, _ = O.fk_pose(om, q[:, b])
        R = p[:9].reshape(3, 3)            # row-major
        pose[:9, b] = R.T.reshape(-1)       # col-major (x_target layout)
        pose[9:, b] = p[9:]
    xt, xdt = W.perturb_targets(pose, seed, B, 0)
    return q, qd, xt, xdt


def census(om, par, inputs, tol, nthreads):
    import oracle as O
    L = O.lib()
    n = 8 + 8 + 3 * 16
    out = (C.c_longlong * n)()
    t = (C.c_double * 16)(*tol)
    L.oracle_polish_census(C.c_int(1), t, out, C.c_int(1))
    t0 = time.perf_counter()
    _, status, iters = O.qpik_batch(om, par, *inputs, nthreads=nthreads)
    dt = time.perf_counter() - t0
    L.oracle_polish_census(C.c_int(0), None, out, C.c_int(1))
    v = list(out)
    return v, status, iters, dt


def main():
    import oracle as O
    ap = argparse.ArgumentParser()
    ap.add_argument("--robot", default="fr3")
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--tol", type=float, nargs="*", default=[1e-6, 1e-4, 1e-3, 1e-2])
    ap.add_argument("--guess", type=int, default=-1, help="first-guess rule of the polish (-1: OSQP's)")
    ap.add_argument("--check", type=int, default=0, help="check_termination (0: the default 25)")
    ap.add_argument("--feas-drop", type=int, default=5, help="study: infeasible-phase drop mode (oracle_polish_feas)")
    ap.add_argument("--feas-att", type=int, default=6, help="study: infeasible-phase attempts")
    ap.add_argument("--npz", help="inputs from a device dump (tools/dump_batch.py) instead of the CPU generator")
    ap.add_argument("--refine", type=int, default=-1, help="polish_refine_iter (-1: the default 3)")
    a = ap.parse_args()
    _, om, spec = O.load(a.robot)
    par = O.default_params(spec["kind"], exact=True)
    if a.check:
        par.solver.check_termination = a.check
    if a.refine >= 0:
        par.solver.polish_refine_iter = a.refine
    if a.npz:
        d = np.load(a.npz)
        inputs = tuple(np.ascontiguousarray(d[k]) for k in ("q", "qd", "xt", "xdt"))
        a.batch = inputs[0].shape[1]
    else:
        inputs = workload(om, a.robot, a.batch, a.seed)
    O.lib().oracle_polish_guess(C.c_int(a.guess))
    O.lib().oracle_polish_feas(C.c_int(a.feas_drop), C.c_int(a.feas_att))
    res = {"robot": a.robot, "batch": a.batch, "seed": a.seed, "by_tol": []}
    for tol in a.tol:
        v, status, iters, dt = census(om, par, inputs, [tol] * 16, a.threads)
        calls, ok = v[0], v[1]
        row = {"tol": tol, "polish_calls": calls, "certified": ok, "eqp": v[2], "eqp_per_instance": v[2] / a.batch,
               "add_steps": v[3], "drop_steps": v[4], "ratio_blocks": v[5], "certified_on_first_eqp": v[6],
               "eqp_hist": v[8:16], "non_solved": int(np.sum(status != 1)), "iters_mean": float(iters.mean()),
               "iters_hist": {int(k): int(c) for k, c in zip(*np.unique(iters, return_counts=True))},
               "seconds": dt, "rules": {}}
        for r, name in enumerate(RULES):
            row["rules"][name] = {"match": v[16 + r], "false_neg": v[32 + r], "false_pos": v[48 + r]}
        res["by_tol"].append(row)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

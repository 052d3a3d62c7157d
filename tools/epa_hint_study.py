"""Small-batch scheduling study (diagnostic, CPU): how well cheap per-instance
tests predict the instances whose narrow phase runs EPA (the small-batch
makespan's tail, DESIGN.md "Small batches").  For the bench workload (stress
tiers, seed 12345) of each robot: the fraction of instances that run EPA
(truth: some GJK candidate intersects) and, for the predictors of
oracle_epa_predict, the fraction flagged and the recall.

    python tools/epa_hint_study.py [--robots fr3,ur5e] [--batch 4096]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import oracle as O  # noqa: E402
from dyros_robot_controller_amd import workload  # noqa: E402


def batch(robot, B, seed=12345):
    pm, om, spec = O.load(robot)
    nv = om.nv
    lo, hi, v = (np.array(a[:nv]) for a in (om.lower, om.upper, om.vel))

    def ev(qs):
        m = np.array([O.manipulability(om, qs[:, b])[0] for b in range(qs.shape[1])])
        d = np.array([O.min_distance(om, qs[:, b])[0] for b in range(qs.shape[1])])
        return m, d
    if spec["kind"] == 0:
        q, _ = workload.joint_states(lo, hi, v, seed, B)
        arm = list(range(nv))
    else:
        vs, ms, ws = spec["joint_index"]
        q, _ = workload.mobile_states(lo, hi, v, (vs, ms, ws), spec["n_arm"], spec["n_wheel"], seed, B, 0)
        arm = list(range(ms, ms + spec["n_arm"]))
    workload.apply_stress(q, lo, hi, arm, seed, 0, ev)
    return om, q


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--robots", default="fr3,ur5e,husky_fr3,xls_fr3,caster_fr3")
    ap.add_argument("--batch", type=int, default=4096)
    a = ap.parse_args()
    L = O.lib()
    for robot in a.robots.split(","):
        om, q = batch(robot, a.batch)
        t, lb, core = C.c_int(), C.c_int(), C.c_int()
        res = np.zeros((3, q.shape[1]), bool)
        for b in range(q.shape[1]):
            L.oracle_epa_predict(C.byref(om), q[:, b].ctypes.data_as(C.POINTER(C.c_double)), C.byref(t), C.byref(lb),
                                 C.byref(core))
            res[:, b] = (t.value, lb.value, core.value)
        tr = res[0]
        out = {"robot": robot, "B": int(q.shape[1]), "epa": float(tr.mean())}
        for k, name in ((1, "lower_bound"), (2, "swept_core")):
            p = res[k]
            out[name] = {"flagged": float(p.mean()), "recall": float((p & tr).sum() / max(tr.sum(), 1))}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

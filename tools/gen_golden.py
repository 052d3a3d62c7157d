#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

Inputs: counter-based synthetic batches (workload.py, fixture seeds 0, 1, 2)
with targets built from the numpy FK (oracle/pyref.py).  Expected outputs:
the C restatement (oracle/drc_oracle.c) in exact mode, each QP solution
cross-checked against the independent numpy interior-point solver with a
KKT certificate before it is written.  Run in the build container:

    python tools/gen_golden.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402
import pyref as R  # noqa: E402
from dyros_robot_controller_amd import workload  # noqa: E402

LINK = {"fr3": "fr3_link8", "ur5e": "tool0"}


def pose12(T):
    v = np.zeros(12)
    v[:9] = T[:3, :3].T.reshape(-1)
    v[9:] = T[:3, 3]
    return v


def certify_distance(pm, om, q):
    """The narrow-phase certificate of DESIGN.md D17 for one instance whose
    argmin pair ran GJK / EPA (tests/test_oracle_witness.py): with
    n = (pB - pA) / d the refined witness pA attains A's support in n and pB
    attains B's support in -n (1e-12), so a separated distance is exact and a
    penetration depth is an attained support overlap.  Witnesses the
    refinement keeps (parallel flat features) are exempt.  Returns 1 when the
    instance was certified, 0 when it needed none."""
    d, _, pair = O.min_distance(om, q)
    d0, pA0, pB0, how = O.pair_distance_raw(om, q, pair)
    if how == 0:
        return 0
    dd, pA, pB = O.pair_distance(om, q, pair)
    if np.array_equal(pA, pA0) and np.array_equal(pB, pB0):
        return 0
    a, c = pm.pairs[pair]
    Tg = R.geom_poses(pm, R.fk(pm, q))
    n = (pB - pA) / dd
    assert abs(np.linalg.norm(pB - pA) - abs(dd)) <= 1e-12
    assert abs(n @ pA - n @ R.support(pm.geoms[a], Tg[a], n)) <= 1e-12
    assert abs(-n @ pB + n @ R.support(pm.geoms[c], Tg[c], -n)) <= 1e-12
    return 1


def gen(robot, seed, B):
    pm, om, spec = O.load(robot)
    q, qd = workload.joint_states(pm.lower, pm.upper, pm.vel, seed, B)
    poses = np.stack([pose12(R.frame_pose(pm, R.fk(pm, q[:, b]), LINK[robot])) for b in range(B)], axis=1)
    xt, xdt = workload.perturb_targets(poses, seed, B)
    par = O.default_params(0, exact=True)
    out, status, iters = O.qpik_batch(om, par, q, qd, xt, xdt, nthreads=8)
    man = np.zeros((1 + pm.nv, B))
    dist = np.zeros((1 + pm.nv, B))
    pair = np.zeros(B, np.int32)
    xdd = np.zeros((6, B))
    for b in range(B):
        st, o, dg = O.qpik_one(om, par, q[:, b], qd[:, b], xt[:, b], xdt[:, b])
        man[0, b], man[1:, b] = dg.man, np.array(dg.man_grad[:pm.nv])
        dist[0, b], dist[1:, b] = dg.dist, np.array(dg.dist_grad[:pm.nv])
        pair[b] = dg.pair
        xdd[:, b] = np.array(dg.xdot_des)
        # independent certificate of the QP solution
        P, qv, A, l, u = R.build_qp_manipulator(pm, q[:, b], xdd[:, b], LINK[robot],
                                                man=(man[0, b], man[1:, b]), dist=(dist[0, b], dist[1:, b]))
        x, y, s2 = R.solve_qp_exact(P, qv, A, l, u)
        assert st == 1 and s2 == 1
        assert np.max(np.abs(x[:pm.nv] - o)) < 1e-7, (robot, seed, b, np.max(np.abs(x[:pm.nv] - o)))
        # the distance stage the QP was built on rests on its own certificate
        certify_distance(pm, om, q[:, b])
    path = os.path.join(ROOT, "tests", "golden", "%s_qpik_step_seed%d.npz" % (robot, seed))
    np.savez_compressed(path, q=q, qdot=qd, x_target=xt, xdot_target=xdt, poses=poses, qdot_opt=out,
                        status=status, man=man, dist=dist, pair=pair, xdot_des=xdd)
    print("wrote", path, "B =", B)


if __name__ == "__main__":
    for robot in ("fr3", "ur5e"):
        for seed in (0, 1, 2):
            gen(robot, seed, 96)

"""Witness refinement in the oracle: the GJK / EPA witness
points of the winning pair are sharpened to the exact critical point of
|pA - pB|^2 on their surface features.

- certificate: with n = (pB - pA) / d the refined pA attains A's support in
  n and pB attains B's support in -n (both to 1e-12), so for a separated
  pair d is the exact distance, and a penetration depth is an attained value
  of the support overlap (never above a direct minimisation of it);
- path independence: a 1e-13 perturbation of q moves the raw GJK / EPA
  witnesses (GJK and EPA gap 1e-6, hpp-fcl's defaults: up to ~1e-3 from the
  exact points) by up to ~1e-5 where it changes their iteration path (UR5e,
  Caster-FR3 samples below; with the r05 GJK gap the FR3 / XLS-FR3 samples
  no longer hit a path change), but the refined ones by rounding only -- the
  property that makes two implementations agree.
"""
import numpy as np
import pytest

import oracle as O
import pyref as R
from dyros_robot_controller_amd import workload
from test_oracle_distance import _true_pd


def _batch(robot, seed, B):
    pm, om, spec = O.load(robot)
    nv = om.nv
    lo, hi, v = (np.array(x[:nv]) for x in (om.lower, om.upper, om.vel))
    if om.kind == 0:
        q, _ = workload.joint_states(lo, hi, v, seed, B)
        arm = list(range(nv))
    else:
        vs, ms, ws = spec["joint_index"]
        q, _ = workload.mobile_states(lo, hi, v, (vs, ms, ws), spec["n_arm"], spec["n_wheel"], seed, B, 0)
        arm = list(range(ms, ms + spec["n_arm"]))

    def ev(qs):
        return (np.array([O.manipulability(om, qs[:, b])[0] for b in range(qs.shape[1])]),
                np.array([O.min_distance(om, qs[:, b])[0] for b in range(qs.shape[1])]))
    workload.apply_stress(q, lo, hi, arm, seed, 0, ev)
    return pm, om, q


def _winners(om, q):
    """(b, pair, raw, refined) for every instance whose argmin pair ran GJK / EPA."""
    out = []
    for b in range(q.shape[1]):
        _, _, pair = O.min_distance(om, q[:, b])
        d0, pA0, pB0, how = O.pair_distance_raw(om, q[:, b], pair)
        if how == 0:
            continue
        out.append((b, pair, how, (d0, pA0, pB0), O.pair_distance(om, q[:, b], pair)))
    return out


@pytest.mark.parametrize("robot,seed", [("ur5e", 1), ("fr3", 2), ("xls_fr3", 2)])
def test_refined_witnesses_certified(robot, seed):
    pm, om, q = _batch(robot, seed, 160)
    refined = pen = 0
    for b, pair, how, raw, (d, pA, pB) in _winners(om, q):
        a, c = pm.pairs[pair]
        Tg = R.geom_poses(pm, R.fk(pm, q[:, b]))
        assert abs(d - raw[0]) <= 1e-6
        if np.array_equal(pA, raw[1]) and np.array_equal(pB, raw[2]):
            continue                      # kept (degenerate features) -- or already exact
        refined += 1
        n = (pB - pA) / d
        assert abs(np.linalg.norm(pB - pA) - abs(d)) <= 1e-12
        hA = n @ R.support(pm.geoms[a], Tg[a], n)
        hB = -n @ R.support(pm.geoms[c], Tg[c], -n)
        assert abs(n @ pA - hA) <= 1e-12 and abs(-n @ pB - hB) <= 1e-12, (b, n @ pA - hA, -n @ pB - hB)
        if d < 0 and pen < 4:
            # the certificate makes -d = h_A(n) + h_B(-n) an attained value of the
            # support overlap, so it can only be at or below a direct
            # minimisation (which stalls at the kinks of box / cap features)
            assert -d <= _true_pd(pm.geoms[a], Tg[a], pm.geoms[c], Tg[c]) + 1e-9
            pen += 1
    assert refined >= 10


# seeds whose batch holds a GJK / EPA winner whose raw witness moves under the
# 1e-13 perturbation (a GJK stop one iteration apart).  Since GJK stops at
# hpp-fcl's 1e-6 support gap the raw witness can move by up to ~sqrt(gap * d)
# (~1e-5 here: XLS-FR3 seeds 7 and 10 move 9.4e-6 / 1.2e-5; seed 2 no longer
# changes path), so each robot is held at a seed that does
@pytest.mark.parametrize("robot,seed", [("ur5e", 1), ("caster_fr3", 2), ("xls_fr3", 7), ("xls_fr3", 10)])
def test_refinement_removes_path_dependence(robot, seed):
    pm, om, q = _batch(robot, seed, 160)
    raw_move, ref_move = [], []
    for b, pair, how, raw, ref in _winners(om, q):
        qp = q[:, b] + 1e-13 * np.sin(np.arange(om.nv) + 1.0)
        d1, pA1, pB1, _ = O.pair_distance_raw(om, qp, pair)
        e1, qA1, qB1 = O.pair_distance(om, qp, pair)
        raw_move.append(max(np.abs(pA1 - raw[1]).max(), np.abs(pB1 - raw[2]).max()))
        ref_move.append(max(np.abs(qA1 - ref[1]).max(), np.abs(qB1 - ref[2]).max()))
    assert max(raw_move) > 1e-10         # the footprint the refinement removes ...
    assert max(ref_move) <= 1e-11, max(ref_move)   # ... down to rounding

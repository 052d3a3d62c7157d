"""Synthetic workload (dyros_robot_controller_amd/workload.py): SURVEY §8d's
stress tiers, judged by the oracle's manipulability and min distance, and
independence of every instance from the batch size / shard offset."""
import numpy as np

import oracle as O
from dyros_robot_controller_amd import workload


def _oracle_evaluator(om):
    def ev(qs):
        m = [O.manipulability(om, qs[:, b])[0] for b in range(qs.shape[1])]
        d = [O.min_distance(om, qs[:, b])[0] for b in range(qs.shape[1])]
        return np.array(m), np.array(d)
    return ev


def _states(om, seed, B, offset):
    lo = np.array(om.lower[:om.nv])
    hi = np.array(om.upper[:om.nv])
    v = np.array(om.vel[:om.nv])
    q, qd = workload.joint_states(lo, hi, v, seed, B, offset)
    tier, stats = workload.apply_stress(q, lo, hi, list(range(om.nv)), seed, offset, _oracle_evaluator(om))
    return q, tier, stats, lo, hi


def test_stress_tiers_fr3():
    _, om, _ = O.load("fr3")
    B = 200
    q, tier, stats, lo, hi = _states(om, 7, B, 0)
    assert np.all(q >= lo[:, None] - 1e-15) and np.all(q <= hi[:, None] + 1e-15)
    frac = [np.mean(tier == t) for t in (1, 2, 3)]
    assert all(0.04 <= f <= 0.17 for f in frac), frac
    for b in np.nonzero(tier == workload.TIER_JOINT_LIMIT)[0]:
        gap = np.minimum(q[:, b] - lo, hi - q[:, b])
        assert gap.min() <= workload.STRESS_MARGIN
    assert stats["singular_unmet"] == 0 and stats["collision_unmet"] == 0, stats
    for b in np.nonzero(tier == workload.TIER_SINGULAR)[0]:
        assert O.manipulability(om, q[:, b])[0] < workload.STRESS_MAN
    for b in np.nonzero(tier == workload.TIER_COLLISION)[0]:
        assert O.min_distance(om, q[:, b])[0] < workload.STRESS_DIST


def test_stress_instances_independent_of_batch():
    _, om, _ = O.load("ur5e")
    qa, ta, _, _, _ = _states(om, 3, 96, 0)
    qb, tb, _, _, _ = _states(om, 3, 40, 50)
    np.testing.assert_array_equal(qa[:, 50:90], qb)
    np.testing.assert_array_equal(ta[50:90], tb)

"""Golden fixtures (tests/golden/*.npz, written by tools/gen_golden.py with
an independent KKT certificate): the C oracle must keep reproducing them."""
import glob
import os

import numpy as np
import pytest

import oracle as O

GOLD = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*_qpik_step_seed*.npz")))


@pytest.mark.parametrize("path", GOLD, ids=[os.path.basename(p) for p in GOLD])
def test_oracle_reproduces_golden(path):
    g = np.load(path)
    robot = os.path.basename(path).split("_qpik")[0]
    pm, om, spec = O.load(robot)
    out, status, _ = O.qpik_batch(om, O.default_params(spec["kind"], exact=True), g["q"], g["qdot"],
                                  g["x_target"], g["xdot_target"], nthreads=4)
    assert np.array_equal(status, g["status"])
    np.testing.assert_allclose(out, g["qdot_opt"], atol=1e-9)


def test_golden_present():
    assert len(GOLD) == 15   # FR3, UR5e, Husky-FR3, XLS-FR3, Caster-FR3 x seeds 0, 1, 2


@pytest.mark.parametrize("path", GOLD, ids=[os.path.basename(p) for p in GOLD])
def test_golden_distance_stage_certified(path):
    """Every fixture instance whose argmin pair ran GJK / EPA: the refined
    witnesses attain both supports (the D17 certificate, tools/gen_golden.py
    certify_distance), so the fixtures' distance stage -- which the QP rows and
    the KKT certificate of the fixtures are built from -- is exact, not only
    the oracle agreeing with itself."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from gen_golden import certify_distance
    g = np.load(path)
    robot = os.path.basename(path).split("_qpik")[0]
    pm, om, spec = O.load(robot)
    certified = 0
    for b in range(g["q"].shape[1]):
        d, _, _ = O.min_distance(om, g["q"][:, b])
        assert abs(d - g["dist"][0, b]) <= 1e-12
        certified += certify_distance(pm, om, g["q"][:, b])
    assert certified >= 5   # 8-25 of the 96 instances per fixture have a GJK / EPA winner

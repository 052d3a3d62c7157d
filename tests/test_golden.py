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
    assert len(GOLD) == 6

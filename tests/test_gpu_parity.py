"""GPU parity: the HIP kernel (through the C-ABI) vs the oracle restatement.

Tolerances (FP64 throughout; the code is tests/_common.py):
  pose / Jacobian        1e-12 abs        (same formulas, different op order)
  manipulability         1e-10 rel; grad 1e-8 abs
  min distance           1e-9 abs separated, 1e-6 penetrating (EPA stops at
                         hpp-fcl's default 1e-6 face gap; the winner's
                         witnesses are then refined to the exact critical
                         point on both sides);
                         grad 1e-6 abs, or the oracle's min distance is
                         non-smooth at q (one-sided derivatives differ: the
                         reference's gradient is ill-defined)
                         (narrow_phase_close)
  argmin pair            the oracle's, or a pair at the same distance
  QP-IK qdot* (exact)    assert_qpik_parity:
                         on the device's distance stage: EVERY instance within
                         1e-6 abs and task residual |J dq|_inf <= 1e-6
                         (north_star bound 1e-4), status identical;
                         end to end (the oracle's own narrow phase): status
                         identical, median |dq| <= 1e-9, and EVERY instance
                         within 1e-4 in q-dot and in the task residual
                         (EXPECTED_OFF = 0 for every robot and seed).
                         Inputs include the SURVEY §8d stress tiers (ids
                         "stress").
"""
import numpy as np
import pytest

import oracle as O
from _common import LINK, assert_qpik_parity, make_manipulator, narrow_phase_close, oracle_batch, stage_pose, step_inputs
from dyros_robot_controller_amd import manipulator

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("robot", ["fr3", "ur5e"])
def test_stages_match_oracle(cuda, robot):
    rd = make_manipulator(robot, cuda)
    B = 256
    q, qd, xt, xdt = step_inputs(rd, robot, 1, B, cuda, stress=True)
    st = stage_pose(rd.model, cuda, q, qd, LINK[robot])
    pm, om, spec = O.load(robot)
    n = om.nv
    for b in range(B):
        pose, J = O.fk_pose(om, q[:, b])
        Rrm = pose[:9].reshape(3, 3)
        np.testing.assert_allclose(st["pose"][:9, b], Rrm.T.reshape(-1), atol=1e-12)
        np.testing.assert_allclose(st["pose"][9:, b], pose[9:], atol=1e-12)
        np.testing.assert_allclose(st["jac"][:, b].reshape(6, n), J, atol=1e-12)
        m, mg = O.manipulability(om, q[:, b])
        assert abs(st["man"][0, b] - m) <= 1e-10 * max(1.0, m)
        np.testing.assert_allclose(st["man"][1:, b], mg, atol=1e-8)
        d, dg, pair = O.min_distance(om, q[:, b])
        if st["pair"][b] != pair:  # exact tie in distance only
            dk, _, _ = O.pair_distance(om, q[:, b], int(st["pair"][b]))
            assert abs(dk - d) <= (1e-9 if d > 0 else 1e-6)
        assert narrow_phase_close(om, q[:, b], st["dist"][0, b], st["dist"][1:, b]), (b, st["dist"][0, b], d)


# end-to-end instances beyond 1e-4 at these seeds (measured; see assert_qpik_parity)
EXPECTED_OFF = {("fr3", False): 0, ("ur5e", False): 0, ("fr3", True): 0, ("ur5e", True): 0}


@pytest.mark.parametrize("stress", [False, True], ids=["nominal", "stress"])
@pytest.mark.parametrize("robot", ["fr3", "ur5e"])
def test_qpik_step_exact_matches_oracle(cuda, robot, stress):
    rd = make_manipulator(robot, cuda)
    ctrl = manipulator.RobotController(0.001, rd, solver_mode="exact")
    B = 512
    q, qd, xt, xdt = step_inputs(rd, robot, 2, B, cuda, stress=stress)
    out, status = ctrl.QPIK_step_batch(q, qd, xt, xdt, LINK[robot])
    out, status = out.cpu().numpy(), status.cpu().numpy()
    assert_qpik_parity(robot, rd.model, q, qd, xt, xdt, out, status, EXPECTED_OFF[robot, stress])

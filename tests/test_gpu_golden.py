"""The HIP path against the committed golden fixtures, with no live oracle in
the loop (tests/golden/*_qpik_step_seed*.npz, written by tools/gen_golden.py
and certified there by the numpy interior point / HiGHS, independently of the
C oracle).  The CPU test_golden.py holds the C oracle to the same files, so a
change that moved the oracle and the kernel together would fail one of the
two.

Per fixture (FR3, UR5e, Husky-FR3, XLS-FR3, Caster-FR3 x seeds 0, 1, 2; 96
instances; the whole-body fixtures hold 12-13 PrimalInfeasible instances
each), through the C-ABI, in the exact (parity) mode:
  - statuses identical to the fixture's; non-Solved instances return zeros
    (QP_IK.cpp:56-61);
  - q-dot* / eta*: median |d| <= 1e-9 and every instance within 1e-4 (the
    north_star tolerance; manipulators: also the task residual |J d|_inf with
    the device's own J);
  - the stage data the QP was built on: xdot_des (1e-9 relative),
    manipulability and its gradient (1e-10 / 1e-8), the min self-distance
    (1e-9 separated, 1e-6 penetrating: GJK / EPA tolerances,
    tests/test_gpu_parity.py header);
  - the fused kernel (B = 96 runs fused by default) and the two-kernel
    pipeline return the same bits."""
import ctypes as C
import glob
import os

import numpy as np
import pytest

from _common import LINK, make_manipulator, make_moma, stage_step
from dyros_robot_controller_amd import _capi, manipulator, mobile_manipulator

pytestmark = pytest.mark.gpu

GOLD = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*_qpik_step_seed*.npz")))
MOMA = ("husky_fr3", "xls_fr3", "caster_fr3")


@pytest.mark.parametrize("path", GOLD, ids=[os.path.basename(p)[:-4] for p in GOLD])
def test_hip_matches_golden(cuda, path):
    import torch
    g = np.load(path)
    robot = os.path.basename(path).split("_qpik")[0]
    moma = robot in MOMA
    rd = make_moma(robot, cuda) if moma else make_manipulator(robot, cuda)
    ctrl = (mobile_manipulator if moma else manipulator).RobotController(0.001, rd, solver_mode="exact")
    q, qd, xt, xdt = g["q"], g["qdot"], g["x_target"], g["xdot_target"]
    outs = []
    for fused in (1, 0):
        _capi.check(_capi.lib().drc_set_fusion(rd.model.handle, C.c_int(fused)))
        out, st = ctrl.QPIK_step_batch(q, qd, xt, xdt, LINK[robot])
        torch.cuda.synchronize()
        outs.append((out.cpu().numpy(), st.cpu().numpy()))
    _capi.check(_capi.lib().drc_set_fusion(rd.model.handle, C.c_int(1)))
    (out, st), (out0, st0) = outs
    np.testing.assert_array_equal(st, st0)
    np.testing.assert_array_equal(out, out0)

    np.testing.assert_array_equal(st, g["status"])
    assert np.all(out[:, st != 1] == 0.0)
    err = np.abs(out - g["qdot_opt"]).max(axis=0)
    assert np.median(err) <= 1e-9, np.median(err)
    assert err.max() <= 1e-4, (err.max(), int(np.argmax(err)))

    s = stage_step(rd.model, cuda, q, qd, xt, xdt, LINK[robot])
    xdd = g["xdot_des"]
    assert np.max(np.abs(s["xdot_des"] - xdd)) <= 1e-9 * max(1.0, np.abs(xdd).max())
    m = g["man"]
    assert np.max(np.abs(s["man"][0] - m[0]) / np.maximum(1.0, m[0])) <= 1e-10
    assert np.max(np.abs(s["man"][1:] - m[1:])) <= 1e-8
    d = g["dist"][0]
    dd = np.abs(s["dist"][0] - d)
    assert np.all(dd <= np.where(d > 0, 1e-9, 1e-6)), (dd.max(), int(np.argmax(dd)))
    if not moma:
        n = q.shape[0]
        for b in range(q.shape[1]):
            J = s["jac"][:, b].reshape(6, n)
            assert np.max(np.abs(J @ (out[:, b] - g["qdot_opt"][:, b]))) <= 1e-4, b
    print("%s: max |d qdot| %.2e, median %.2e, %d non-Solved" % (os.path.basename(path), err.max(), np.median(err),
                                                                 int(np.sum(st != 1))))

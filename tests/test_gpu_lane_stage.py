"""Lane-per-instance task stage (csrc/lane_task.hpp) against the
wave-per-instance task_kernel on identical inputs (drc_debug_lane_stage).

Both compute the same formulas (FK, LWA Jacobian, task velocity, JJ^T
manipulability and gradient, self-distance with the same closed forms, GJK
and candidate rule); they differ in instruction order (registers vs LDS,
FMA contraction), so the stage data agree to rounding and the QP optimum
to the solver's certification tolerance.  Instances the lane stage hands
back (EPA, many GJK candidates) are computed by the wave kernel in both runs.
"""
import numpy as np
import pytest

from _common import LINK, make_manipulator, stage_pose, step_inputs
from dyros_robot_controller_amd import _batch, _capi, manipulator

pytestmark = pytest.mark.gpu
T0, T = 1.0, 2.0


def _run(rd, p, args, lane):
    import torch
    lib = _capi.lib()
    _capi.check(lib.drc_debug_lane_stage(rd.model.handle, lane))
    try:
        st = _batch.stages_batch(rd.model, p, *args)
        out, status = _batch.qpik_batch(rd.model, p, *args[:4], *args[4:])
        torch.cuda.synchronize()
    finally:
        _capi.check(lib.drc_debug_lane_stage(rd.model.handle, 0))
    st = {k: v.cpu().numpy() for k, v in st.items()}
    return st, out.cpu().numpy(), status.cpu().numpy()


@pytest.mark.parametrize("robot", ["fr3", "ur5e"])
@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("stress", [False, True])
@pytest.mark.parametrize("lane_mode", [1, 2])
def test_lane_stage_matches_wave_kernel(cuda, robot, mode, stress, lane_mode):
    rd = make_manipulator(robot, cuda)
    B = 4096
    q, qd, xt, xdt = step_inputs(rd, robot, 21 + mode, B, cuda, stress=stress)
    dev = lambda a: _batch.as_device(a, cuda)
    pb = manipulator.QPIKParamsBuilder(rd.model, exact=True)
    if mode == 2:
        xi = stage_pose(rd.model, cuda, q, qd, LINK[robot])["pose"]
        xdi = 0.1 * xdt
        p = pb.params(LINK[robot], mode, t=T0 + 0.37 * T, t0=T0, duration=T)
        args = [dev(q), dev(qd), dev(xt), dev(xdt), dev(xi), dev(xdi)]
    else:
        p = pb.params(LINK[robot], mode)
        args = [dev(q), dev(qd), dev(xt) if mode else None, dev(xdt)]
    sl, ol, tl = _run(rd, p, args, lane_mode)
    sw, ow, tw = _run(rd, p, args, 0)
    for k in ("pose", "jac", "xdot_des", "man"):
        np.testing.assert_allclose(sl[k], sw[k], rtol=1e-12, atol=1e-12, err_msg=k)
    same = sl["pair"] == sw["pair"]
    assert same.mean() >= 0.999, "argmin pair differs on %d instances" % (~same).sum()
    np.testing.assert_allclose(sl["dist"][0], sw["dist"][0], rtol=0, atol=1e-9)
    # GJK stops at a 1e-12 gap, which fixes the witness points on curved
    # surfaces only to ~sqrt of it: one-ulp differences in the joint frames
    # move them (and so grad d) by up to ~1e-6
    gd = np.abs(sl["dist"][1:] - sw["dist"][1:]).max(axis=0)
    assert gd[same].max() <= 1e-5
    assert (tl == tw).mean() >= 0.999
    dq = np.abs(ol - ow).max(axis=0)
    # identical stage data -> identical QP solution
    other = np.max([np.abs(sl[k] - sw[k]).max(axis=0) for k in ("pose", "jac", "xdot_des", "man")], axis=0)
    ident = same & (gd == 0) & (other == 0) & (sl["dist"][0] == sw["dist"][0])
    assert dq[ident].max() <= 1e-12, "q_dot differs with identical stage data"
    # a grad d moved within the witness tolerance moves q_dot by at most the
    # QP's sensitivity to an active distance row
    assert dq[same & ~ident].max(initial=0) <= 1e-3

"""The reference's per-control-cycle call chain on the drop-in
(examples/C++/src/fr3_controller.cpp:66-68,123-134): updateState -> getPose ->
getVelocity -> QPIKCubic -> moveJointTorqueStep.

  * drc_kinematics_batch (getPose / getJacobian / getVelocity without the
    manipulability and self-collision stages) against the QPIK task stage's
    own pose and Jacobian (drc_qpik_stages_batch) and J qdot;
  * drc_state_host (kinematics + updateDynamics in one round trip) against
    drc_kinematics_batch and drc_dynamics_host;
  * drc_qpik_host_timed against drc_qpik_host (same outputs, bit for bit) and
    its QP::TimeDuration fields;
  * the whole cycle through the pybind11 module (the reference's Python
    binding names) against the oracle: pose = FK(q), J qdot, QPIKCubic's q-dot*,
    and tau = M (Kp (q + dt qdot* - q) + Kv (qdot* - qdot)) + g."""
import ctypes as C
import os
import sys

import numpy as np
import pytest

from _common import LINK, make_manipulator, make_moma, moma_step_inputs, oracle_batch, step_inputs
from dyros_robot_controller_amd import _batch, _capi, manipulator

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))
ip = lambda a: a.ctypes.data_as(C.POINTER(C.c_int))


def _frame(rd, robot):
    fid = C.c_int()
    _capi.check(_capi.lib().drc_model_find_frame(rd.model.handle, LINK[robot].encode(), C.byref(fid)))
    return fid.value


@pytest.mark.parametrize("robot", ["fr3", "ur5e", "xls_fr3"])
def test_kinematics_batch_matches_task_stage(cuda, robot):
    import torch
    moma = robot == "xls_fr3"
    rd = make_moma(robot, cuda) if moma else make_manipulator(robot, cuda)
    B = 300
    q, qd, xt, xdt = (moma_step_inputs if moma else step_inputs)(rd, robot, 31, B, cuda)
    dof = rd.model.dof
    st = _batch.stages_batch(rd.model, manipulator.QPIKParamsBuilder(rd.model, exact=True).params(
        LINK[robot], _capi.MODE_QPIK), _batch.as_device(q, cuda), _batch.as_device(qd, cuda), None,
        _batch.as_device(np.zeros((6, B)), cuda))
    pose = torch.empty((12, B), dtype=torch.float64, device=cuda)
    jac = torch.empty((6 * dof, B), dtype=torch.float64, device=cuda)
    xdot = torch.empty((6, B), dtype=torch.float64, device=cuda)
    dq, dqd = _batch.as_device(q, cuda), _batch.as_device(qd, cuda)
    _capi.check(_capi.lib().drc_kinematics_batch(rd.model.handle, _frame(rd, robot), C.c_int64(B),
                                                 C.c_void_p(dq.data_ptr()), C.c_void_p(dqd.data_ptr()),
                                                 C.c_void_p(pose.data_ptr()), C.c_void_p(jac.data_ptr()),
                                                 C.c_void_p(xdot.data_ptr()),
                                                 C.c_void_p(torch.cuda.current_stream(cuda).cuda_stream)))
    torch.cuda.synchronize()
    np.testing.assert_allclose(pose.cpu().numpy(), st["pose"].cpu().numpy(), rtol=0, atol=1e-14)
    J = jac.cpu().numpy()
    np.testing.assert_allclose(J, st["jac"].cpu().numpy(), rtol=0, atol=1e-14)
    ref = np.stack([J[:, b].reshape(6, dof) @ qd[:, b] for b in range(B)], 1)
    np.testing.assert_allclose(xdot.cpu().numpy(), ref, rtol=0, atol=1e-12)


def test_state_host_one_round_trip(cuda):
    rd = make_manipulator("fr3", cuda)
    B, n = 5, rd.model.dof
    q, qd, _, _ = step_inputs(rd, "fr3", 32, B, cuda)
    outs = [np.zeros((12, B)), np.zeros((6 * n, B)), np.zeros((6, B)), np.zeros((n * n, B)), np.zeros((n * n, B)),
            np.zeros((n, B)), np.zeros((n, B)), np.zeros((n, B))]
    _capi.check(_capi.lib().drc_state_host(rd.model.handle, _frame(rd, "fr3"), B, dp(q), dp(qd), *[dp(o) for o in outs]))
    dyn = [np.zeros((n * n, B)), np.zeros((n * n, B)), np.zeros((n, B)), np.zeros((n, B)), np.zeros((n, B))]
    _capi.check(_capi.lib().drc_dynamics_host(rd.model.handle, 0, B, dp(q), dp(qd), *[dp(o) for o in dyn]))
    for a, b in zip(outs[3:], dyn):
        np.testing.assert_array_equal(a, b)
    import oracle as O
    _, om, _ = O.load("fr3")
    for b in range(B):
        pose, J = O.fk_pose(om, q[:, b])
        R = pose[:9].reshape(3, 3)
        np.testing.assert_allclose(outs[0][:9, b], R.T.reshape(-1), atol=1e-12)   # column-major R
        np.testing.assert_allclose(outs[0][9:, b], pose[9:], atol=1e-12)
        np.testing.assert_allclose(outs[1][:, b].reshape(6, n), J, atol=1e-12)
        np.testing.assert_allclose(outs[2][:, b], J @ qd[:, b], atol=1e-12)


def test_qpik_host_timed(cuda):
    rd = make_manipulator("fr3", cuda)
    B = 3
    q, qd, xt, xdt = step_inputs(rd, "fr3", 33, B, cuda, stress=True)
    p = manipulator.QPIKParamsBuilder(rd.model, exact=True).params(LINK["fr3"], _capi.MODE_QPIK_STEP)
    n = rd.model.dof
    o1, s1, i1 = np.zeros((n, B)), np.zeros(B, np.int32), np.zeros(B, np.int32)
    o2, s2, i2 = np.zeros((n, B)), np.zeros(B, np.int32), np.zeros(B, np.int32)
    lib, h = _capi.lib(), rd.model.handle
    _capi.check(lib.drc_qpik_host(h, C.byref(p), B, dp(q), dp(qd), dp(xt), dp(xdt), None, None, dp(o1), ip(s1), ip(i1)))
    t = _capi.TimeDuration()
    _capi.check(lib.drc_qpik_host_timed(h, C.byref(p), B, dp(q), dp(qd), dp(xt), dp(xdt), None, None, dp(o2), ip(s2),
                                        ip(i2), C.byref(t)))
    np.testing.assert_array_equal(o1, o2)
    np.testing.assert_array_equal(s1, s2)
    np.testing.assert_array_equal(i1, i2)
    assert t.set_ineq > 0 and t.set_constraint > 0 and t.set_solver > 0 and t.solve_qp > 0
    assert t.set_cost == 0 and t.set_bound == 0 and t.set_eq == 0
    assert abs(t.set_qp - t.set_ineq - t.set_constraint) < 1e-15
    assert t.set_ineq + t.set_constraint + t.set_solver < 0.05       # seconds: one instance's stages


def test_cycle_through_module_matches_oracle(cuda):
    """fr3_controller.cpp's cycle with the reference's Python binding names."""
    sys.path.insert(0, os.path.join(ROOT, "dyros_robot_controller_amd", "python"))
    import dyros_robot_controller_cpp_wrapper as drc
    import oracle as O
    import pyref as R
    from dyros_robot_controller_amd import robot_path
    rd = drc.ManipulatorRobotData(robot_path("fr3"), robot_path("fr3", "srdf"), "")
    rc = drc.ManipulatorRobotController(0.001, rd)
    pm, om, _ = O.load("fr3")
    q, qd, _, _ = step_inputs(make_manipulator("fr3", cuda), "fr3", 34, 6, cuda, stress=True)
    link, dt = "fr3_link8", 0.001
    for b in range(q.shape[1]):
        assert rd.updateState(q[:, b], qd[:, b])
        x = rd.getPose(link)
        xdot = rd.getVelocity(link)
        pose, J = O.fk_pose(om, q[:, b])
        np.testing.assert_allclose(x[:3, :3], pose[:9].reshape(3, 3), atol=1e-12)
        np.testing.assert_allclose(x[:3, 3], pose[9:], atol=1e-12)
        np.testing.assert_allclose(xdot, J @ qd[:, b], atol=1e-12)
        xt = x.copy()
        xt[:3, 3] += [0.0, 0.1, 0.1]                         # fr3_controller.cpp:123-131: target = x_init + (0, .1, .1)
        qdot_star = rc.QPIKCubic(xt, np.zeros(6), x, xdot, 0.4, 0.0, 3.0, link)
        tau = rc.moveJointTorqueStep(q[:, b] + qdot_star * dt, qdot_star)
        # the oracle's QPIKCubic on the same instance
        xt12 = np.concatenate([xt[:3, :3].T.reshape(-1), xt[:3, 3]])
        xi12 = np.concatenate([x[:3, :3].T.reshape(-1), x[:3, 3]])
        ref, st, _, _ = oracle_batch("fr3", q[:, b:b + 1], qd[:, b:b + 1], xt12[:, None], np.zeros((6, 1)), exact=True,
                                     xi=xi12[:, None], xdi=xdot[:, None], mode=2, t=0.4, t0=0.0, T=3.0)
        if st[0] == 1:
            np.testing.assert_allclose(qdot_star, ref[:, 0], atol=1e-6)
        else:   # QP_IK.cpp:56-61: a failed solve returns zeros on both sides
            assert np.all(qdot_star == 0.0) and np.all(ref[:, 0] == 0.0), (qdot_star, ref[:, 0])
        d = R.dynamics(pm, q[:, b], qd[:, b])
        qdd = 400 * (qdot_star * dt) + 40 * (qdot_star - qd[:, b])
        np.testing.assert_allclose(tau, d["M"] @ qdd + d["g"], rtol=1e-10, atol=1e-8)


@pytest.mark.parametrize("robot", ["fr3", "ur5e", "husky_fr3", "xls_fr3", "caster_fr3"])
def test_lds_plan(cuda, robot):
    """Per-wave LDS of the three QPIK kernels (drc_debug_lds_plan): the QP
    kernel's plan fits three waves per SIMD (12 per CU in 160 KB), the task
    kernel's at least one (its VGPRs allow two; DESIGN.md "Occupancy"), and the
    fused plan holds the larger of the two and the task record -- inside the
    task plan's dead overlay region where it fits there (kernel_common.hpp
    fused_rec_offset: the whole-body plans), else past both plans."""
    moma = robot in ("husky_fr3", "xls_fr3", "caster_fr3")
    rd = make_moma(robot, cuda) if moma else make_manipulator(robot, cuda)
    p = manipulator.QPIKParamsBuilder(rd.model, exact=True).params(LINK[robot], _capi.MODE_QPIK_STEP)
    t, q, f = C.c_int(), C.c_int(), C.c_int()
    _capi.check(_capi.lib().drc_debug_lds_plan(rd.model.handle, C.byref(p), 0, C.byref(t), C.byref(q), C.byref(f)))
    print(robot, "task", t.value, "qp", q.value, "fused", f.value)
    assert 0 < q.value <= 160 * 1024 // 12
    assert 0 < t.value <= 160 * 1024 // 4
    assert max(t.value, q.value) <= f.value <= max(t.value, q.value) + 8 * 128
    if moma:   # the whole-body record fits in the task plan's overlay region
        assert f.value == t.value


def test_host_timeline_and_waves(cuda):
    """drc_debug_host_timeline: one row of five ordered steady-clock stamps per
    synchronous call while enabled; drc_debug_waves: the task build the call
    launches (two or three waves per SIMD) and the QP kernel's three."""
    rd = make_manipulator("fr3", cuda)
    B = 2
    q, qd, xt, xdt = step_inputs(rd, "fr3", 35, B, cuda)
    p = manipulator.QPIKParamsBuilder(rd.model, exact=True).params(LINK["fr3"], _capi.MODE_QPIK_STEP)
    n = rd.model.dof
    o, s, it = np.zeros((n, B)), np.zeros(B, np.int32), np.zeros(B, np.int32)
    lib, h = _capi.lib(), rd.model.handle
    _capi.check(lib.drc_debug_host_timeline(h, 1, None, 0, None))
    for _ in range(3):
        _capi.check(lib.drc_qpik_host(h, C.byref(p), B, dp(q), dp(qd), dp(xt), dp(xdt), None, None, dp(o), ip(s), ip(it)))
    tl = np.zeros((8, 5), np.int64)
    cnt = C.c_int64()
    _capi.check(lib.drc_debug_host_timeline(h, 0, tl.ctypes.data_as(C.POINTER(C.c_int64)), 8, C.byref(cnt)))
    assert cnt.value == 3
    assert np.all(np.diff(tl[:3], axis=1) >= 0) and np.all(tl[:3, 0] > 0)
    assert np.all(tl[1:3, 0] >= tl[0:2, 4])
    _capi.check(lib.drc_qpik_host(h, C.byref(p), B, dp(q), dp(qd), dp(xt), dp(xdt), None, None, dp(o), ip(s), ip(it)))
    _capi.check(lib.drc_debug_host_timeline(h, 0, None, 0, C.byref(cnt)))
    assert cnt.value == 0                                   # disabled: nothing recorded
    wt, wq = C.c_int(), C.c_int()
    _capi.check(lib.drc_debug_waves(h, C.byref(p), C.byref(wt), C.byref(wq)))
    assert wt.value in (2, 3) and wq.value == 3


def test_qpik_stamps_diagnostic(cuda):
    """drc_debug_qpik_stamps: the same outputs as drc_qpik_host, plus per
    instance six ordered clock stamps (task start / end, QP start / assembled /
    solved / stored) and where each stage ran (workgroup << 32 | CU << 2 |
    SIMD), for the fused kernel and the two-kernel pipeline."""
    rd = make_manipulator("fr3", cuda)
    B = 96
    q, qd, xt, xdt = step_inputs(rd, "fr3", 36, B, cuda)
    p = manipulator.QPIKParamsBuilder(rd.model, exact=True).params(LINK["fr3"], _capi.MODE_QPIK_STEP)
    n = rd.model.dof
    lib, h = _capi.lib(), rd.model.handle
    o0, s0, i0 = np.zeros((n, B)), np.zeros(B, np.int32), np.zeros(B, np.int32)
    _capi.check(lib.drc_qpik_host(h, C.byref(p), B, dp(q), dp(qd), dp(xt), dp(xdt), None, None, dp(o0), ip(s0), ip(i0)))
    try:
        for fused in (1, 0):
            _capi.check(lib.drc_set_fusion(h, C.c_int(fused)))
            o, s, it = np.zeros((n, B)), np.zeros(B, np.int32), np.zeros(B, np.int32)
            st = np.zeros((8, B), np.uint64)
            _capi.check(lib.drc_debug_qpik_stamps(h, C.byref(p), B, dp(q), dp(qd), dp(xt), dp(xdt), dp(xt), dp(xdt),
                                                  dp(o), ip(s), ip(it), st.ctypes.data_as(C.POINTER(C.c_uint64))))
            assert np.array_equal(o, o0) and np.array_equal(s, s0) and np.array_equal(it, i0)
            t = st[:6].astype(np.int64)
            assert np.all(t > 0) and np.all(np.diff(t, axis=0) >= 0)
            assert np.all((t[5] - t[0]) * 1e-8 < 0.05)        # < 50 ms per instance (100 MHz ticks)
            for k in (6, 7):                                   # CU id << 2 | SIMD, workgroup in the high word
                assert np.all(((st[k] & np.uint64(0xFFFFFFFF)) >> np.uint64(2)) < 4096)
                assert np.all((st[k] >> np.uint64(32)) < 1 << 20)
            if fused:                                          # one wave runs both stages of an instance
                assert np.array_equal(st[6] >> np.uint64(32), st[7] >> np.uint64(32))
    finally:
        _capi.check(lib.drc_set_fusion(h, C.c_int(1)))

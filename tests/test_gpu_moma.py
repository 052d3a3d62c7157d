"""GPU parity for the mobile-manipulator whole-body QP-IK (SURVEY §8a
a18-a22): Husky-FR3 (differential, A = 9) and XLS-FR3 (mecanum, A = 11) vs
the oracle restatement, through the C-ABI.

Tolerances and the parity contract as tests/test_gpu_parity.py (assert_qpik_parity).  The MoMa QP has no slack variables
(QP_IK.cpp:85-128), so instances can be primal infeasible: the status must
match the oracle's and such instances return zeros (QP_IK.cpp:56-61)."""
import numpy as np
import pytest

import oracle as O
from _common import LINK, assert_qpik_parity, make_moma, moma_step_inputs, narrow_phase_close, stage_pose
from dyros_robot_controller_amd import mobile_manipulator as MM

pytestmark = pytest.mark.gpu
ROBOTS = ["husky_fr3", "xls_fr3", "caster_fr3"]


@pytest.mark.parametrize("robot", ROBOTS)
def test_moma_model_and_mobile_jacobian(cuda, robot):
    rd = make_moma(robot, cuda)
    pm, om, spec = O.load(robot)
    assert rd.get_dof() == om.nv
    assert rd.get_manipulator_dof() == 7 and rd.get_mobile_dof() == spec["n_wheel"]
    assert rd.get_actuator_dof() == 7 + spec["n_wheel"]
    rng = np.random.default_rng(3)
    for _ in range(8):   # caster: J_mobile follows the steer angles (mobile/robot_data.cpp:179-204)
        wp = rng.uniform(-np.pi, np.pi, spec["n_wheel"])
        ref = spec["J_mobile"](wp) if spec.get("drive") == 2 else spec["J_mobile"]()
        np.testing.assert_allclose(rd.compute_mobile_FK_jacobian(wp), ref, atol=1e-12)


@pytest.mark.parametrize("robot", ROBOTS)
def test_moma_stages_match_oracle(cuda, robot):
    rd = make_moma(robot, cuda)
    B = 128
    q, qd, xt, xdt = moma_step_inputs(rd, robot, 1, B, cuda, stress=True)
    st = stage_pose(rd.model, cuda, q, qd, LINK[robot])
    pm, om, spec = O.load(robot)
    n = om.nv
    for b in range(B):
        pose, J = O.fk_pose(om, q[:, b])
        np.testing.assert_allclose(st["pose"][:9, b], pose[:9].reshape(3, 3).T.reshape(-1), atol=1e-12)
        np.testing.assert_allclose(st["pose"][9:, b], pose[9:], atol=1e-12)
        np.testing.assert_allclose(st["jac"][:, b].reshape(6, n), J, atol=1e-12)
        m, mg = O.manipulability(om, q[:, b])
        assert abs(st["man"][0, b] - m) <= 1e-10 * max(1.0, m)
        np.testing.assert_allclose(st["man"][1:, b], mg, atol=1e-8)
        assert narrow_phase_close(om, q[:, b], st["dist"][0, b], st["dist"][1:, b]), b


EXPECTED_OFF = {"husky_fr3": 0, "xls_fr3": 0, "caster_fr3": 0}   # measured end-to-end count beyond 1e-4 (assert_qpik_parity)


@pytest.mark.parametrize("robot", ROBOTS)
def test_moma_qpik_step_exact_matches_oracle(cuda, robot):
    rd = make_moma(robot, cuda)
    ctrl = MM.RobotController(0.001, rd, solver_mode="exact")
    B = 512
    q, qd, xt, xdt = moma_step_inputs(rd, robot, 2, B, cuda, stress=True)
    out, status = ctrl.QPIK_step_batch(q, qd, xt, xdt, LINK[robot])
    out, status = out.cpu().numpy(), status.cpu().numpy()
    assert np.all(out[:, status != 1] == 0)
    assert_qpik_parity(robot, rd.model, q, qd, xt, xdt, out, status, EXPECTED_OFF[robot])


def test_moma_single_instance_split(cuda):
    """QPIK_step returns (qdot_mobile, qdot_mani) split by ActuatorIndex
    (mobile_manipulator/robot_controller.cpp:182-196)."""
    robot = "xls_fr3"
    rd = make_moma(robot, cuda)
    ctrl = MM.RobotController(0.001, rd)
    q, qd, xt, xdt = moma_step_inputs(rd, robot, 5, 1, cuda)
    ji = rd.get_joint_index()
    W = rd.get_mobile_dof()
    rd.update_state(q[ji.virtual_start:ji.virtual_start + 3, 0], q[ji.mobi_start:ji.mobi_start + W, 0],
                    q[ji.mani_start:ji.mani_start + 7, 0], qd[ji.virtual_start:ji.virtual_start + 3, 0],
                    qd[ji.mobi_start:ji.mobi_start + W, 0], qd[ji.mani_start:ji.mani_start + 7, 0])
    from dyros_robot_controller_amd.manipulator import pose_from12
    vm, va = ctrl.QPIK_step(pose_from12(xt[:, 0]), xdt[:, 0], LINK[robot])
    eta, st = ctrl.QPIK_step_batch(q, qd, xt, xdt, LINK[robot])
    eta = eta.cpu().numpy()[:, 0]
    a = rd.get_actuator_index()
    if int(st.cpu().numpy()[0]) == 1:
        np.testing.assert_array_equal(vm, eta[a.mobi_start:a.mobi_start + W])
        np.testing.assert_array_equal(va, eta[a.mani_start:a.mani_start + 7])
    assert vm.shape == (W,) and va.shape == (7,)


@pytest.mark.parametrize("robot", ["husky_fr3", "xls_fr3"])
def test_moma_lp_certificate_on_device(cuda, robot):
    """D15 on the device: the whole-body instances the oracle's Farkas
    certificate proves infeasible come back PrimalInfeasible after 0 ADMM
    iterations with zero output, the same instances as the oracle's (fed the
    device's distance stage, so both judge the same rows); every other
    instance runs the ADMM (iterations > 0) and no instance runs past 100
    iterations (D16: no polish-cap tail)."""
    import torch
    rd = make_moma(robot, cuda)
    ctrl = MM.RobotController(0.001, rd, solver_mode="exact")
    B = 2048
    q, qd, xt, xdt = moma_step_inputs(rd, robot, 12, B, cuda, stress=True)
    iters = torch.zeros(B, dtype=torch.int32, device=cuda)
    out, status = ctrl.QPIK_step_batch(q, qd, xt, xdt, LINK[robot], iters=iters)
    out, status, iters = out.cpu().numpy(), status.cpu().numpy(), iters.cpu().numpy()
    st = stage_pose(rd.model, cuda, q, qd, LINK[robot])
    pm, om, spec = O.load(robot)
    par = O.default_params(1, exact=True)
    _, ost, oit = O.qpik_batch_dist(om, par, q, qd, xt, xdt, np.ascontiguousarray(st["dist"]), nthreads=8)
    cert_dev = (status == O.PRIMAL_INFEASIBLE) & (iters == 0)
    cert_orc = (ost == O.PRIMAL_INFEASIBLE) & (oit == 0)
    assert cert_dev.sum() >= 3
    np.testing.assert_array_equal(cert_dev, cert_orc)
    assert np.all(out[:, cert_dev] == 0)
    assert np.all(iters[~cert_dev] > 0)
    assert iters.max() <= 100, iters.max()

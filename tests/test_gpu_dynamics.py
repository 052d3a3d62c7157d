"""GPU parity of drc_dynamics_batch against the numpy
restatement (oracle/pyref.py: dynamics, dynamics_actuated), which
tests/test_oracle_dynamics.py pins.  FP64 on both sides; tolerances are
relative to each quantity's scale, and M_inv's scales with cond(M) (up to ~1e6
for the mobile manipulators, whose base mass sits beside the hand's 1e-4
inertias)."""
import numpy as np
import pytest

import oracle as O
import pyref as R
from pyref_model import load_urdf
from _dyn_models import two_link, two_link_closed_form, rank_deficient
from dyros_robot_controller_amd import manipulator, _batch, workload
from _common import make_manipulator, make_moma

pytestmark = pytest.mark.gpu


def _states(pm, B, seed):
    rng = np.random.default_rng(seed)
    lo, hi = np.array(pm.lower), np.array(pm.upper)
    q = np.where((hi > lo)[:, None], rng.uniform(lo[:, None], hi[:, None], (pm.nv, B)),
                 rng.uniform(-3, 3, (pm.nv, B)))
    return q, rng.uniform(-1.5, 1.5, (pm.nv, B))


def _check(dev, ref, b, cond_tol=True):
    n = ref["M"].shape[0]
    sM = max(1.0, np.abs(ref["M"]).max())
    np.testing.assert_allclose(dev["M"][:, :, b], ref["M"], atol=1e-12 * sM, err_msg="M b=%d" % b)
    sX = np.abs(ref["Minv"]).max()
    kappa = sM * sX
    np.testing.assert_allclose(dev["Minv"][:, :, b], ref["Minv"], atol=1e-14 * kappa * sX + 1e-12,
                               err_msg="Minv b=%d" % b)
    for k in ("g", "nle", "c"):
        s = max(1.0, np.abs(ref[k]).max())
        np.testing.assert_allclose(dev[k][:, b], ref[k], atol=1e-11 * s, err_msg="%s b=%d" % (k, b))
    assert dev["M"].shape == (n, n, dev["M"].shape[2])


def _run(rd, q, qd, actuated=False):
    out = _batch.dynamics_batch(rd.model, _batch.as_device(q, rd.device), _batch.as_device(qd, rd.device),
                                actuated=actuated)
    return {k: v.cpu().numpy() for k, v in out.items()}


@pytest.mark.parametrize("robot", ["fr3", "ur5e"])
def test_manipulator_dynamics_match_oracle(cuda, robot):
    pm, _, _ = O.load(robot)
    rd = make_manipulator(robot, cuda)
    B = 203                                     # ragged: not a multiple of the 16-robot block
    q, qd = _states(pm, B, 11)
    dev = _run(rd, q, qd)
    for b in range(B):
        _check(dev, R.dynamics(pm, q[:, b], qd[:, b]), b)


@pytest.mark.parametrize("robot", ["husky_fr3", "xls_fr3", "caster_fr3"])
def test_moma_dynamics_match_oracle(cuda, robot):
    pm, _, spec = O.load(robot)
    rd = make_moma(robot, cuda)
    lo, hi = np.array(pm.lower), np.array(pm.upper)
    B = 97
    q, qd = workload.mobile_states(lo, hi, np.array(pm.vel), spec["joint_index"], spec["n_arm"], spec["n_wheel"],
                                   5, B, 0)
    full, act = _run(rd, q, qd), _run(rd, q, qd, actuated=True)
    for b in range(B):
        _check(full, R.dynamics(pm, q[:, b], qd[:, b]), b)
        ws = spec["joint_index"][2]
        Jm = spec["J_mobile"](q[ws:ws + spec["n_wheel"], b]) if spec.get("drive") == 2 else spec["J_mobile"]()
        S = R.selection_matrix(pm.nv, spec["n_arm"], spec["n_wheel"], spec["joint_index"], spec["actuator_index"],
                               Jm, q[spec["joint_index"][0] + 2, b])
        _check(act, R.dynamics_actuated(pm, q[:, b], qd[:, b], S), b)


def test_two_link_known_answer(cuda, tmp_path):
    rd = manipulator.RobotData(two_link(str(tmp_path)), "", device=cuda)
    rng = np.random.default_rng(7)
    q, qd = rng.uniform(-3, 3, (2, 40)), rng.uniform(-2, 2, (2, 40))
    dev = _run(rd, q, qd)
    for b in range(40):
        M, g, c = two_link_closed_form(q[:, b], qd[:, b])
        np.testing.assert_allclose(dev["M"][:, :, b], M, atol=1e-13)
        np.testing.assert_allclose(dev["g"][:, b], g, atol=1e-12)
        np.testing.assert_allclose(dev["c"][:, b], c, atol=1e-12)
        np.testing.assert_allclose(dev["Minv"][:, :, b], np.linalg.inv(M), rtol=1e-11, atol=1e-12)


def test_rank_deficient_pinv_cod_fallback(cuda, tmp_path):
    """Massless last link: M is rank 2, the full-rank certificate fails for every
    instance and the serial COD pseudo-inverse (second launch) must match PinvCOD."""
    path = rank_deficient(str(tmp_path))
    pm = load_urdf(path)
    rd = manipulator.RobotData(path, "", device=cuda)
    rng = np.random.default_rng(8)
    B = 37
    q, qd = rng.uniform(-3, 3, (3, B)), rng.uniform(-1, 1, (3, B))
    dev = _run(rd, q, qd)
    for b in range(B):
        ref = R.dynamics(pm, q[:, b], qd[:, b])
        np.testing.assert_allclose(dev["Minv"][:, :, b], ref["Minv"], atol=1e-9 * np.abs(ref["Minv"]).max())
        assert np.abs(dev["Minv"][2, :, b]).max() < 1e-12


def test_host_entry_and_getters(cuda):
    pm, _, _ = O.load("fr3")
    rd = make_manipulator("fr3", cuda)
    q, qd = _states(pm, 5, 9)
    host = _batch.dynamics_host(rd.model, q, qd)
    dev = _run(rd, q, qd)
    for k in ("M", "Minv", "g", "nle", "c"):
        np.testing.assert_array_equal(host[k], dev[k])
    rd.updateState(q[:, 2], qd[:, 2])
    ref = R.dynamics(pm, q[:, 2], qd[:, 2])
    np.testing.assert_allclose(rd.getMassMatrix(), ref["M"], atol=1e-12)
    np.testing.assert_allclose(rd.getGravity(), ref["g"], atol=1e-11)
    np.testing.assert_allclose(rd.getCoriolis(), ref["c"], atol=1e-11)
    np.testing.assert_allclose(rd.getNonlinearEffects(), ref["nle"], atol=1e-11)
    np.testing.assert_allclose(rd.computeGravity(q[:, 2]), ref["g"], atol=1e-11)
    # empty batch is a no-op
    assert _batch.dynamics_batch(rd.model, _batch.as_device(np.zeros((7, 0)), cuda))["M"].shape == (7, 7, 0)


def _torque_ref(d, q, qd, qt, qdt, kp, kv, s, n):
    acc = kp * (qt - q[s:s + n]) + kv * (qdt - qd[s:s + n])
    return d["M"][s:s + n, s:s + n] @ acc + d["g"][s:s + n]


@pytest.mark.parametrize("robot", ["fr3", "xls_fr3"])
def test_joint_torque_step_matches_oracle(cuda, robot):
    """moveJointTorqueStep (robot_controller.cpp:115-125) / the MoMa arm block
    (mobile_manipulator/robot_controller.cpp:103-118), including the QPIK
    example's Euler target q + dt qdot* (fr3_controller.cpp:133)."""
    pm, _, spec = O.load(robot)
    moma = spec["kind"] == 1
    rd = make_moma(robot, cuda) if moma else make_manipulator(robot, cuda)
    B = 45
    if moma:
        q, qd = workload.mobile_states(np.array(pm.lower), np.array(pm.upper), np.array(pm.vel),
                                       spec["joint_index"], spec["n_arm"], spec["n_wheel"], 3, B, 0)
        s, n = spec["joint_index"][1], spec["n_arm"]
    else:
        q, qd = _states(pm, B, 12)
        s, n = 0, pm.nv
    rng = np.random.default_rng(13)
    qt, qdt, qddt = rng.uniform(-1, 1, (n, B)), rng.uniform(-1, 1, (n, B)), rng.uniform(-3, 3, (n, B))
    kp, kv = rng.uniform(100, 500, n), rng.uniform(10, 50, n)
    dt = 0.001
    A = lambda t: _batch.as_device(t, cuda)
    t1 = _batch.joint_torque_step_batch(rd.model, A(q), A(qd), A(qt), A(qdt), None, dt, kp, kv).cpu().numpy()
    t2 = _batch.joint_torque_step_batch(rd.model, A(q), A(qd), None, A(qdt), None, dt, kp, kv).cpu().numpy()
    t3 = _batch.joint_torque_step_batch(rd.model, A(q), A(qd), None, None, A(qddt), dt).cpu().numpy()
    t4 = _batch.joint_torque_step_batch(rd.model, A(q), A(qd), A(qt), A(qdt), None, dt).cpu().numpy()
    for b in range(B):
        d = R.dynamics(pm, q[:, b], qd[:, b])
        scale = lambda r: 1e-11 * max(1.0, np.abs(r).max())
        r1 = _torque_ref(d, q[:, b], qd[:, b], qt[:, b], qdt[:, b], kp, kv, s, n)
        r2 = _torque_ref(d, q[:, b], qd[:, b], q[s:s + n, b] + dt * qdt[:, b], qdt[:, b], kp, kv, s, n)
        r3 = d["M"][s:s + n, s:s + n] @ qddt[:, b] + d["g"][s:s + n]
        r4 = _torque_ref(d, q[:, b], qd[:, b], qt[:, b], qdt[:, b], 400.0, 40.0, s, n)
        for t, r in ((t1, r1), (t2, r2), (t3, r3), (t4, r4)):
            np.testing.assert_allclose(t[:, b], r, atol=scale(r))
    # single-instance mirror signatures
    if not moma:
        ctrl = manipulator.RobotController(dt, rd)
        rd.updateState(q[:, 0], qd[:, 0])
        ctrl.setJointGain(kp, kv)
        np.testing.assert_allclose(ctrl.move_joint_torque_step(q_target=qt[:, 0], qdot_target=qdt[:, 0]), t1[:, 0],
                                   rtol=0, atol=1e-12 * max(1, np.abs(t1[:, 0]).max()))

"""Mobile base Jacobians through the C-ABI (host code, no GPU):
drc_mobile_fk_jacobian = Mobile::RobotData::computeFKJacobian
(src/mobile/robot_data.cpp:123-204) and drc_mobile_ik_jacobian =
Mobile::RobotController::computeIKJacobian (src/mobile/robot_controller.cpp:55-125),
against the oracle's restatements (C and numpy) for all three drives.

Reference quirk, restated as written: the caster IK row of the steer joint
(robot_controller.cpp:120) is not the inverse of the FK map
(robot_data.cpp:193-198) — its constant term is (px cos + py sin)/b - 1 where
inverting Jq^-1 Jp~ gives (px cos + py sin)/b + 1.  The drive rows agree."""
import ctypes as C

import numpy as np

import oracle as O
from dyros_robot_controller_amd import _capi, mobile_manipulator as MM


def _c(kp):
    return kp.c_struct()


def _fk(kp, wp):
    p = _c(kp)
    J = np.zeros(3 * 8)
    n = C.c_int()
    dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))
    _capi.check(_capi.lib().drc_mobile_fk_jacobian(C.byref(p), dp(np.ascontiguousarray(wp, float)), dp(J), C.byref(n)))
    return J[:3 * n.value].reshape(3, n.value)


def _ik(kp, wp):
    p = _c(kp)
    J = np.zeros(8 * 3)
    n = C.c_int()
    dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))
    _capi.check(_capi.lib().drc_mobile_ik_jacobian(C.byref(p), dp(np.ascontiguousarray(wp, float)), dp(J), C.byref(n)))
    return J[:3 * n.value].reshape(n.value, 3)


DIFF = MM.KinematicParam(MM.DriveType.Differential, 0.165, base_width=0.555)
MEC = MM.KinematicParam(MM.DriveType.Mecanum, 0.120, roller_angles=[-np.pi / 4, np.pi / 4, np.pi / 4, -np.pi / 4],
                        base2wheel_positions=[(0.2225, 0.2045), (0.2225, -0.2045), (-0.2225, 0.2045),
                                              (-0.2225, -0.2045)], base2wheel_angles=[0, 0, 0, 0])
CAS = MM.KinematicParam(MM.DriveType.Caster, O.CASTER_FR3["radius"], base2wheel_positions=O.CASTER_FR3["positions"],
                        wheel_offset=O.CASTER_FR3["offset"])


def test_fk_differential_and_mecanum():
    np.testing.assert_allclose(_fk(DIFF, np.zeros(2)), O.differential_fk_jacobian(0.165, 0.555), atol=1e-15)
    np.testing.assert_allclose(_fk(MEC, np.zeros(4)), O.ROBOTS["xls_fr3"]["J_mobile"](), atol=1e-12)
    # mecanum: FK o IK = I (J_fk = PinvCOD of the full-column-rank IK map, robot_data.cpp:175)
    np.testing.assert_allclose(_fk(MEC, np.zeros(4)) @ _ik(MEC, np.zeros(4)), np.eye(3), atol=1e-12)
    # differential: the reachable twists (vy = 0) round-trip
    for v in ([0.3, 0.0, 0.2], [-0.1, 0.0, 1.0]):
        np.testing.assert_allclose(_fk(DIFF, np.zeros(2)) @ (_ik(DIFF, np.zeros(2)) @ v), v, atol=1e-12)


def test_fk_caster_matches_oracles():
    _, om, spec = O.load("caster_fr3")
    rng = np.random.default_rng(11)
    for _ in range(50):
        wp = rng.uniform(-np.pi, np.pi, 4)
        q = np.zeros(om.nv)
        q[spec["joint_index"][2]:spec["joint_index"][2] + 4] = wp
        J = _fk(CAS, wp)
        np.testing.assert_allclose(J, spec["J_mobile"](wp), atol=1e-12)       # numpy (pyref.pinv_cod)
        np.testing.assert_allclose(J, O.mobile_fk_jacobian(om, q), atol=1e-12)  # C oracle (pinv_cod_sym)


def test_ik_caster_formula():
    c = O.CASTER_FR3
    r, b = c["radius"], c["offset"]
    rng = np.random.default_rng(5)
    for _ in range(20):
        wp = rng.uniform(-np.pi, np.pi, 4)
        J = _ik(CAS, wp)
        for i, (px, py) in enumerate(c["positions"]):
            phi = wp[2 * i]
            np.testing.assert_allclose(J[2 * i], [-np.sin(phi) / b, np.cos(phi) / b,
                                                  (px * np.cos(phi) + py * np.sin(phi)) / b - 1], atol=1e-12)
            np.testing.assert_allclose(J[2 * i + 1], [np.cos(phi) / r, np.sin(phi) / r,
                                                      (px * np.sin(phi) - py * np.cos(phi)) / r], atol=1e-12)

"""Pins of the QPID restatement (oracle/drc_oracle.c: point_jacobian_dot,
manip_graddot, mindist_graddot, oracle_qpid_one) — SURVEY §8f row 2.

The reference's QPID (src/manipulator/QP_ID.cpp, src/mobile_manipulator/
QP_ID.cpp) consumes Pinocchio's Jacobian time variation and the grad_dot
terms of getManipulability / getMinDistance (robot_data.cpp:496-512,555-569).
No reference test holds values for them (parity unpinned at Pinocchio), so
they are pinned here by:
  * finite differences along qdot of the frame Jacobian and of the point
    Jacobian of a material point (what Pinocchio's LWA dJ is: d/dt J);
  * an independent numpy restatement of the reference grad_dot formulas
    built from pyref's dJ/dq and finite-difference Jdot;
  * optimality of the exact-mode QPID solution against an independent numpy
    assembly + interior-point solve (objective, feasibility, task
    acceleration J qdd + Jdot qdot)."""
import numpy as np
import pytest

import oracle as O
import pyref as R
from dyros_robot_controller_amd import workload

LINK = "fr3_link8"


def _states(robot, seed, B):
    pm, om, spec = O.load(robot)
    if om.kind == 0:
        q, qd = workload.joint_states(pm.lower, pm.upper, pm.vel, seed, B)
    else:
        q, qd = workload.mobile_states(pm.lower, pm.upper, pm.vel, spec["joint_index"], spec["n_arm"],
                                       spec["n_wheel"], seed, B)
    return pm, om, spec, q, qd


def _arm(om):
    return (np.arange(om.mani_start, om.mani_start + om.n_arm) if om.kind == 1 else np.arange(om.nv))


@pytest.mark.parametrize("robot", ["fr3", "ur5e", "xls_fr3"])
def test_frame_jdot_matches_finite_difference(robot):
    pm, om, spec, q, qd = _states(robot, 3, 6)
    h = 1e-6
    for b in range(q.shape[1]):
        Jd, _, _ = O.qpid_stages(om, q[:, b], qd[:, b])
        Jp = O.fk_pose(om, q[:, b] + h * qd[:, b])[1]
        Jm = O.fk_pose(om, q[:, b] - h * qd[:, b])[1]
        np.testing.assert_allclose(Jd, (Jp - Jm) / (2 * h), atol=2e-7)


@pytest.mark.parametrize("robot", ["fr3", "husky_fr3"])
def test_point_jdot_matches_material_point_fd(robot):
    """getJointJacobianTimeVariation at a point carried by the body: d/dt of
    the point Jacobian with the point moving rigidly (what JA_dot in
    robot_data.cpp:501-509 assumes)."""
    pm, om, spec, q, qd = _states(robot, 5, 4)
    h = 1e-6
    rng = np.random.default_rng(1)
    for b in range(q.shape[1]):
        for jid in (om.nv // 2, om.nv):
            T = O.joint_placement(om, q[:, b], jid)
            p = T[:3, 3] + rng.normal(0, 0.1, 3)
            _, Jd = O.point_jacobian_dot(om, q[:, b], qd[:, b], jid, p)
            fd = []
            for sgn in (1, -1):
                qq = q[:, b] + sgn * h * qd[:, b]
                T2 = O.joint_placement(om, qq, jid)
                p2 = T2[:3, :3] @ T[:3, :3].T @ (p - T[:3, 3]) + T2[:3, 3]
                fd.append(O.point_jacobian_dot(om, qq, qd[:, b], jid, p2)[0])
            np.testing.assert_allclose(Jd, (fd[0] - fd[1]) / (2 * h), atol=2e-7)


@pytest.mark.parametrize("robot", ["fr3", "xls_fr3"])
def test_manipulability_graddot_restatement(robot):
    """grad_dot (robot_data.cpp:555-569, MoMa :477-492) against a numpy
    restatement of the same formula from pyref's dJ/dq and an FD Jdot."""
    pm, om, spec, q, qd = _states(robot, 7, 5)
    arm = _arm(om)
    h = 1e-6
    for b in range(q.shape[1]):
        qb, qdb = q[:, b], qd[:, b]
        _, mgd, _ = O.qpid_stages(om, qb, qdb)
        oMi = R.fk(pm, qb)
        J = R.frame_jacobian(pm, oMi, LINK)[:, arm]
        Jd = ((R.frame_jacobian(pm, R.fk(pm, qb + h * qdb), LINK) -
               R.frame_jacobian(pm, R.fk(pm, qb - h * qdb), LINK)) / (2 * h))[:, arm]
        dJ = R.frame_jacobian_dq(pm, oMi, LINK)
        m = np.sqrt(np.linalg.det(J @ J.T))
        Ai = R.pinv_cod(J @ J.T)
        mani_dot = m * np.trace(Jd @ J.T @ Ai)
        Aid = -(Ai @ (2 * Jd @ J.T) @ Ai)
        ref = np.array([mani_dot * np.trace(dJ[i][:, arm] @ J.T @ Ai) +
                        m * np.trace(dJ[i][:, arm] @ Jd.T @ Ai + dJ[i][:, arm] @ J.T @ Aid) for i in arm])
        np.testing.assert_allclose(mgd, ref, rtol=1e-5, atol=1e-7)
        # mani_dot itself is the exact time derivative of m
        mp = O.manipulability(om, qb + h * qdb)[0]
        mm = O.manipulability(om, qb - h * qdb)[0]
        assert abs(mani_dot - (mp - mm) / (2 * h)) < 1e-6


@pytest.mark.parametrize("robot", ["fr3", "ur5e"])
def test_min_distance_graddot_restatement(robot):
    """grad_dot = n^T (JB_dot - JA_dot) (robot_data.cpp:496-512) with the
    point-Jacobian derivatives taken by finite differences of material points."""
    pm, om, spec, q, qd = _states(robot, 9, 5)
    h = 1e-6
    for b in range(q.shape[1]):
        qb, qdb = q[:, b], qd[:, b]
        _, _, dgd = O.qpid_stages(om, qb, qdb)
        d, grad, pair = O.min_distance(om, qb)
        _, pA, pB = O.pair_distance(om, qb, pair)
        n = (pB - pA) / np.linalg.norm(pB - pA)
        JXd = []
        for g, p in ((om.pair_a[pair], pA), (om.pair_b[pair], pB)):
            jid = om.gparent[g]
            T = O.joint_placement(om, qb, jid)
            fd = []
            for sgn in (1, -1):
                qq = qb + sgn * h * qdb
                T2 = O.joint_placement(om, qq, jid)
                p2 = T2[:3, :3] @ T[:3, :3].T @ (p - T[:3, 3]) + T2[:3, 3]
                fd.append(O.point_jacobian_dot(om, qq, qdb, jid, p2)[0][:3])
            JXd.append((fd[0] - fd[1]) / (2 * h))
        np.testing.assert_allclose(dgd, n @ (JXd[1] - JXd[0]), atol=2e-6)


def _qpid_case(robot, seed, B, exact=True):
    pm, om, spec, q, qd = _states(robot, seed, B)
    poses = np.zeros((12, B))
    for b in range(B):
        T = R.frame_pose(pm, R.fk(pm, q[:, b]), LINK)
        poses[:9, b] = T[:3, :3].T.reshape(-1)
        poses[9:, b] = T[:3, 3]
    xt, xdt = workload.perturb_targets(poses, seed, B)
    par = O.default_qpid_params(om.kind, exact=exact)
    par.mode = 1
    return pm, om, spec, q, qd, xt, xdt, par


@pytest.mark.parametrize("robot", ["fr3", "xls_fr3"])
def test_qpid_exact_mode_is_optimal(robot):
    pm, om, spec, q, qd, xt, xdt, par = _qpid_case(robot, 21, 24)
    arm = _arm(om)
    na = om.nv if om.kind == 0 else om.n_arm + om.n_wheel
    solved = 0
    for b in range(q.shape[1]):
        qb, qdb = q[:, b], qd[:, b]
        M, g, gf = O.qpid_dynamics(pm, om, spec, qb, qdb)
        st, qdd, tau, dg = O.qpid_one(om, par, qb, qdb, M, g, gf, xt[:, b], xdt[:, b])
        J = np.array(dg.J[:6 * om.nv]).reshape(6, om.nv)
        if om.kind == 1:
            Jm = np.array([[om.J_mobile[r][c] for c in range(om.n_wheel)] for r in range(3)])
            S = R.selection_matrix(om.nv, om.n_arm, om.n_wheel, spec["joint_index"], spec["actuator_index"], Jm,
                                   qb[om.virtual_start + 2])
            Jt, col = J @ S, om.act_mani_start
        else:
            Jt, col = J, 0
        n = len(arm)
        man = (dg.man, np.array(dg.man_grad[:n]), dg.man_gd)
        dist = (dg.dist, np.array(dg.dist_grad[:om.nv])[arm], dg.dist_gd)
        P, qv, A, l, u = R.build_qp_qpid(pm, qb, qdb, Jt, np.array(dg.xdot_des), np.array(dg.jdot_v), M, g,
                                         man, dist, arm, col, slacks=om.kind == 0)
        x, y, s2 = R.solve_qp_exact(P, qv, A, l, u)
        assert s2 in (1, 3), "interior-point certificate produced no finite iterate (instance %d)" % b
        assert x is None or np.all(np.isfinite(x))
        if s2 != 1:
            assert st != O.SOLVED          # reference: status != Solved -> gravity torque
            assert np.all(qdd == 0)
            np.testing.assert_array_equal(tau, gf[:na] if om.kind == 1 else g)
            continue
        assert st == O.SOLVED
        solved += 1
        # reconstruct the slacks (minimal: linear cost 1000 > 0)
        xo = np.zeros(P.shape[0])
        xo[:na], xo[na:2 * na] = qdd, tau
        if om.kind == 0:
            G = A[P.shape[0]:P.shape[0] + 4 * n + 2]
            lg = l[P.shape[0]:P.shape[0] + 4 * n + 2]
            xo[2 * na:] = np.maximum(0.0, lg - G[:, :2 * na] @ xo[:2 * na])
        f = lambda v: 0.5 * v @ P @ v + qv @ v
        Ax = A @ xo
        tol = 1e-7 * (1 + np.abs(l[np.abs(l) < 1e20]).max())
        assert np.all(Ax >= l - tol) and np.all(Ax <= u + tol)
        # never worse than the independent solver ...
        assert f(xo) <= f(x) + 1e-7 * (1 + abs(f(x)))
        if max(R.kkt_residuals(P, qv, A, l, u, x, y)) < 1e-6:   # ... and equal where it certifies itself
            assert abs(f(xo) - f(x)) <= 1e-7 * (1 + abs(f(x)))
            # the task acceleration is unique even where qdd is not (P singular on null(J))
            np.testing.assert_allclose(Jt @ qdd, Jt @ x[:na], rtol=1e-6, atol=1e-6)
    assert solved >= q.shape[1] // 2


def test_qpid_reference_settings_band():
    """OSQP defaults stop far from the optimum on QPID as on QPIK (slack
    weight 1000 in the relative dual tolerance): the reference's own band."""
    pm, om, spec, q, qd, xt, xdt, par = _qpid_case("fr3", 22, 12)
    p0 = O.default_qpid_params(0, exact=False)
    p0.mode = 1
    errs = []
    for b in range(q.shape[1]):
        M, g, gf = O.qpid_dynamics(pm, om, spec, q[:, b], qd[:, b])
        s1, a1, t1, _ = O.qpid_one(om, par, q[:, b], qd[:, b], M, g, gf, xt[:, b], xdt[:, b])
        s0, a0, t0, _ = O.qpid_one(om, p0, q[:, b], qd[:, b], M, g, gf, xt[:, b], xdt[:, b])
        if s0 == s1 == O.SOLVED:
            errs.append(np.abs(t0 - t1).max())
    assert len(errs) > 6 and np.median(errs) > 1e-4


def test_ipm_certificate_keeps_best_iterate():
    """Regression (round-1 verdict): on FR3 seed 21 instance 11 the Mehrotra
    iteration converged to ~1e-10 and then diverged to NaN because P (QPID's
    2 J^T J on the qdd block) is singular and the Newton matrix reached cond
    1e22; the certificate reported the NaN point as solved.  The best iterate
    is now kept and a non-finite result is never status 1."""
    pm, om, spec, q, qd, xt, xdt, par = _qpid_case("fr3", 21, 24)
    arm = _arm(om)
    b = 11
    qb, qdb = q[:, b], qd[:, b]
    M, g, gf = O.qpid_dynamics(pm, om, spec, qb, qdb)
    st, qdd, tau, dg = O.qpid_one(om, par, qb, qdb, M, g, gf, xt[:, b], xdt[:, b])
    J = np.array(dg.J[:6 * om.nv]).reshape(6, om.nv)
    n = len(arm)
    man = (dg.man, np.array(dg.man_grad[:n]), dg.man_gd)
    dist = (dg.dist, np.array(dg.dist_grad[:om.nv])[arm], dg.dist_gd)
    P, qv, A, l, u = R.build_qp_qpid(pm, qb, qdb, J, np.array(dg.xdot_des), np.array(dg.jdot_v), M, g,
                                     man, dist, arm, 0, slacks=True)
    x, y, s2 = R.solve_qp_exact(P, qv, A, l, u)
    assert s2 == 1 and np.all(np.isfinite(x)) and np.all(np.isfinite(y))
    assert max(R.kkt_residuals(P, qv, A, l, u, x, y)) < 1e-6

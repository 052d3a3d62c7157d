"""QP pins: the restated OSQP (ADMM + certified polish) against an
independent numpy interior-point solver with a KKT certificate; the
reference-settings band; infeasibility detection."""
import numpy as np

import oracle as O
import pyref as R
from dyros_robot_controller_amd import workload


def _instances(robot, seed, B):
    pm, om, spec = O.load(robot)
    q, qd = workload.joint_states(pm.lower, pm.upper, pm.vel, seed, B)
    link = "fr3_link8" if robot == "fr3" else "tool0"
    poses = np.zeros((12, B))
    for b in range(B):
        T = R.frame_pose(pm, R.fk(pm, q[:, b]), link)
        poses[:9, b] = T[:3, :3].T.reshape(-1)
        poses[9:, b] = T[:3, 3]
    xt, xdt = workload.perturb_targets(poses, seed, B)
    return pm, om, q, qd, xt, xdt, link


def test_exact_mode_is_kkt_optimal():
    pm, om, q, qd, xt, xdt, link = _instances("fr3", 11, 40)
    par = O.default_params(0, exact=True)
    for b in range(40):
        st, out, dg = O.qpik_one(om, par, q[:, b], qd[:, b], xt[:, b], xdt[:, b])
        assert st == O.SOLVED
        P, qv, A, l, u = R.build_qp_manipulator(pm, q[:, b], np.array(dg.xdot_des), link,
                                                man=(dg.man, np.array(dg.man_grad[:7])),
                                                dist=(dg.dist, np.array(dg.dist_grad[:7])))
        x, y, s2 = R.solve_qp_exact(P, qv, A, l, u)
        stat, prim, comp = R.kkt_residuals(P, qv, A, l, u, x, y)
        assert max(stat, prim, comp) < 1e-8
        np.testing.assert_allclose(out, x[:7], atol=1e-8)


def test_reference_settings_band():
    """OSQP defaults (eps 1e-3, slack weight 1000 in the relative dual
    tolerance) stop far from the optimum: the reference's own output band."""
    pm, om, q, qd, xt, xdt, link = _instances("fr3", 12, 200)
    o0, s0, _ = O.qpik_batch(om, O.default_params(0, exact=False), q, qd, xt, xdt, nthreads=4)
    o1, s1, _ = O.qpik_batch(om, O.default_params(0, exact=True), q, qd, xt, xdt, nthreads=4)
    both = (s0 == 1) & (s1 == 1)
    err = np.abs(o0 - o1).max(axis=0)[both]
    assert np.median(err) > 1e-4          # the band is real ...
    assert np.percentile(err, 99) < 2.0   # ... and bounded


def test_primal_infeasible_detected():
    # x in R^2, 1 <= x0 + x1 and x0 + x1 <= 0  -> infeasible
    P = np.eye(2)
    qv = np.zeros(2)
    A = np.array([[1.0, 1.0], [1.0, 1.0]])
    l = np.array([1.0, -1e30])
    u = np.array([1e30, 0.0])
    st, x, y, it, pol = O.solve_qp(P, qv, A, l, u, O.default_params(1, exact=True).solver)
    assert st == O.PRIMAL_INFEASIBLE


def test_simple_qp_exact():
    P = np.array([[4.0, 1.0], [1.0, 2.0]])
    qv = np.array([1.0, 1.0])
    A = np.array([[1.0, 1.0], [1.0, 0.0], [0.0, 1.0]])
    l = np.array([1.0, 0.0, 0.0])
    u = np.array([1.0, 0.7, 0.7])
    st, x, y, it, pol = O.solve_qp(P, qv, A, l, u, O.default_params(1, exact=True).solver)
    assert st == O.SOLVED
    np.testing.assert_allclose(x, [0.3, 0.7], atol=1e-9)    # OSQP README example


def test_polish_cap_changes_iterations_not_outputs():
    """The manipulator polish KKT cap of 16 (the kernel's register EQP, copied
    into the oracle) is a cost rule, not a numerical one: with the cap removed
    (polish_cap = 0, the LDS LDL^T for every size) the certified optimum is the
    same within 1e-6 on every instance, statuses identical, and the cap can
    only add ADMM iterations (a too-large KKT skips that polish attempt)."""
    pm, om, q, qd, xt, xdt, link = _instances("fr3", 13, 300)
    par = O.default_params(0, exact=True)
    assert par.solver.polish_cap == 16
    o16, s16, it16 = O.qpik_batch(om, par, q, qd, xt, xdt, nthreads=4)
    par.solver.polish_cap = 0
    o0, s0, it0 = O.qpik_batch(om, par, q, qd, xt, xdt, nthreads=4)
    np.testing.assert_array_equal(s16, s0)
    assert np.abs(o16 - o0).max() <= 1e-6
    assert np.all(it16 >= it0)

"""Oracle pins for the dynamics restatement.

Pinocchio is absent, so crba / computeGeneralizedGravity / nonLinearEffects
(robot_data.cpp:111-113) are pinned by: a textbook closed form (planar 2R),
two independent formulations agreeing (COM-Jacobian kinetic energy vs
Newton-Euler), gravity as the gradient of the potential, the Coriolis vector
from Christoffel symbols of finite-differenced M, and the passivity identity
qd^T (Mdot - 2C) qd = 0.  PinvCOD is pinned against numpy's SVD pseudo-inverse
on full-rank and rank-deficient inputs."""
import numpy as np
import pytest

import oracle as O
import pyref as R
from pyref_model import load_urdf
from _dyn_models import two_link, two_link_closed_form, rank_deficient

ROBOTS = ["fr3", "ur5e", "husky_fr3", "xls_fr3"]


def _rand_state(pm, rng):
    n = pm.nv
    lo, hi = np.array(pm.lower), np.array(pm.upper)
    q = np.where(hi > lo, rng.uniform(lo, hi), rng.uniform(-2, 2, n))
    return q, rng.uniform(-1.5, 1.5, n), rng.uniform(-2, 2, n)


def potential(pm, q):
    oMi = R.fk(pm, q)
    V = 0.0
    for j, (m, com, _) in enumerate(R.body_inertias(pm)):
        if j:
            V -= m * R.GRAVITY @ (oMi[j][:3, :3] @ com + oMi[j][:3, 3])
    return V


def test_two_link_closed_form(tmp_path):
    pm = load_urdf(two_link(str(tmp_path)))
    rng = np.random.default_rng(0)
    for _ in range(20):
        q, qd = rng.uniform(-3, 3, 2), rng.uniform(-2, 2, 2)
        M, g, c = two_link_closed_form(q, qd)
        d = R.dynamics(pm, q, qd)
        np.testing.assert_allclose(d["M"], M, atol=1e-13)
        np.testing.assert_allclose(d["g"], g, atol=1e-12)
        np.testing.assert_allclose(d["c"], c, atol=1e-12)
        np.testing.assert_allclose(d["Minv"] @ M, np.eye(2), atol=1e-11)


@pytest.mark.parametrize("robot", ROBOTS)
def test_newton_euler_matches_kinetic_energy_form(robot):
    pm, _, _ = O.load(robot)
    rng = np.random.default_rng(1)
    for _ in range(10):
        q, qd, qdd = _rand_state(pm, rng)
        M = R.mass_matrix(pm, q)
        np.testing.assert_allclose(M, M.T, atol=1e-14)
        assert np.linalg.eigvalsh(M).min() > 0
        tau = R.rnea(pm, q, qd, qdd)
        np.testing.assert_allclose(tau - R.rnea(pm, q, qd, 0 * qdd), M @ qdd, atol=1e-11 * max(1, np.abs(M).max()))


@pytest.mark.parametrize("robot", ROBOTS)
def test_gravity_is_potential_gradient(robot):
    pm, _, _ = O.load(robot)
    rng = np.random.default_rng(2)
    h = 1e-6
    for _ in range(5):
        q, _, _ = _rand_state(pm, rng)
        g = R.rnea(pm, q, 0 * q, 0 * q)
        fd = np.array([(potential(pm, q + h * e) - potential(pm, q - h * e)) / (2 * h) for e in np.eye(pm.nv)])
        np.testing.assert_allclose(g, fd, atol=1e-6)


@pytest.mark.parametrize("robot", ROBOTS)
def test_coriolis_from_christoffel_symbols(robot):
    pm, _, _ = O.load(robot)
    rng = np.random.default_rng(3)
    n, h = pm.nv, 1e-6
    q, qd, _ = _rand_state(pm, rng)
    dM = [(R.mass_matrix(pm, q + h * e) - R.mass_matrix(pm, q - h * e)) / (2 * h) for e in np.eye(n)]
    # c_i = sum_jk (dM_ij/dq_k - 1/2 dM_jk/dq_i) qd_j qd_k
    c = np.array([sum(dM[k][i, j] * qd[j] * qd[k] - 0.5 * dM[i][j, k] * qd[j] * qd[k]
                      for j in range(n) for k in range(n)) for i in range(n)])
    d = R.dynamics(pm, q, qd)
    np.testing.assert_allclose(d["c"], c, atol=1e-6 * max(1, np.abs(c).max()))
    # passivity: qd^T Mdot qd = 2 qd^T c
    Mdot = sum(dM[k] * qd[k] for k in range(n))
    assert abs(qd @ Mdot @ qd - 2 * qd @ d["c"]) < 1e-6 * max(1, abs(qd @ Mdot @ qd))


def test_pinv_cod_full_and_deficient_rank():
    rng = np.random.default_rng(4)
    for n in (3, 7, 12):
        A = rng.standard_normal((n, n))
        A = A @ A.T + 0.1 * np.eye(n)
        np.testing.assert_allclose(R.pinv_cod(A), np.linalg.inv(A), rtol=1e-9, atol=1e-12)
        U = rng.standard_normal((n, n - 2))
        A = U @ U.T                                  # rank n - 2
        np.testing.assert_allclose(R.pinv_cod(A), np.linalg.pinv(A, rcond=1e-10, hermitian=True), atol=1e-9)


def test_rank_deficient_mass_matrix(tmp_path):
    pm = load_urdf(rank_deficient(str(tmp_path)))
    q = np.array([0.3, -0.7, 1.1])
    d = R.dynamics(pm, q, np.array([0.5, -0.2, 0.9]))
    assert np.allclose(d["M"][2], 0) and np.allclose(d["M"][:, 2], 0)
    np.testing.assert_allclose(d["Minv"], np.linalg.pinv(d["M"]), atol=1e-10)
    assert abs(d["Minv"][2]).max() == 0


@pytest.mark.parametrize("robot", ["husky_fr3", "xls_fr3"])
def test_actuated_dynamics_projection(robot):
    pm, _, spec = O.load(robot)
    rng = np.random.default_rng(5)
    q, qd, _ = _rand_state(pm, rng)
    S = R.selection_matrix(pm.nv, spec["n_arm"], spec["n_wheel"], spec["joint_index"], spec["actuator_index"],
                           spec["J_mobile"](), q[spec["joint_index"][0] + 2])
    d, da = R.dynamics(pm, q, qd), R.dynamics_actuated(pm, q, qd, S)
    eta = rng.standard_normal(S.shape[1])
    # kinetic energy of the actuated velocities is the full-model kinetic energy of S eta
    assert abs(eta @ da["M"] @ eta - (S @ eta) @ d["M"] @ (S @ eta)) < 1e-10
    np.testing.assert_allclose(da["Minv"] @ da["M"], np.eye(S.shape[1]), atol=1e-7)

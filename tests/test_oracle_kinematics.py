"""Oracle pins (CPU): analytic known answers and finite-difference identities
for the restated Pinocchio conventions.  Parity with
Pinocchio/hpp-fcl themselves is unpinned (absent from the container); these
are the independent anchors."""
import numpy as np
import pytest

import oracle as O
import pyref as R

FR3_HOME = np.array([0, 0, 0, -np.pi / 2, 0, np.pi / 2, np.pi / 4])


@pytest.fixture(scope="module")
def fr3():
    return O.load("fr3")


def test_fr3_model_counts(fr3):
    pm, om, _ = fr3
    assert pm.nv == 7 and len(pm.geoms) == 35
    assert len(pm.pairs) == 180            # 533 candidate pairs minus 353 SRDF-disabled
    types = sorted((pm.geoms[a]["type"], pm.geoms[b]["type"]) for a, b in pm.pairs)
    assert types.count((0, 0)) == 48       # sphere-sphere


def test_fr3_fk_known_answers(fr3):
    pm, om, _ = fr3
    pose, _ = O.fk_pose(om, np.zeros(7))
    np.testing.assert_allclose(pose[9:], [0.088, 0.0, 0.926], atol=1e-12)
    np.testing.assert_allclose(pose[:9].reshape(3, 3), np.diag([1, -1, -1]), atol=1e-12)
    pose, _ = O.fk_pose(om, FR3_HOME)
    np.testing.assert_allclose(pose[9:], [0.5545, 0.0, 0.6245], atol=1e-12)


def test_c_oracle_matches_numpy_restatement(fr3):
    pm, om, _ = fr3
    rng = np.random.default_rng(0)
    for _ in range(40):
        q = rng.uniform(pm.lower + 0.05, pm.upper - 0.05)
        pose, J = O.fk_pose(om, q)
        oMi = R.fk(pm, q)
        T = R.frame_pose(pm, oMi, "fr3_link8")
        np.testing.assert_allclose(pose[:9], T[:3, :3].reshape(-1), atol=1e-13)
        np.testing.assert_allclose(J, R.frame_jacobian(pm, oMi, "fr3_link8"), atol=1e-13)
        m1, g1 = O.manipulability(om, q)
        m2, g2 = R.manipulability(pm, q, "fr3_link8")
        assert abs(m1 - m2) < 1e-12
        np.testing.assert_allclose(g1, g2, atol=1e-10)


def test_jacobian_and_djdq_finite_differences(fr3):
    pm, om, _ = fr3
    q = np.array([0.3, -0.4, 0.2, -1.9, 0.5, 1.6, 0.1])
    oMi = R.fk(pm, q)
    J = R.frame_jacobian(pm, oMi, "fr3_link8")
    dJ = R.frame_jacobian_dq(pm, oMi, "fr3_link8")
    h = 1e-6
    for k in range(7):
        e = np.zeros(7)
        e[k] = h
        Tp = R.frame_pose(pm, R.fk(pm, q + e), "fr3_link8")
        Tm = R.frame_pose(pm, R.fk(pm, q - e), "fr3_link8")
        np.testing.assert_allclose((Tp[:3, 3] - Tm[:3, 3]) / (2 * h), J[:3, k], atol=1e-8)
        Jp = R.frame_jacobian(pm, R.fk(pm, q + e), "fr3_link8")
        Jm = R.frame_jacobian(pm, R.fk(pm, q - e), "fr3_link8")
        np.testing.assert_allclose((Jp - Jm) / (2 * h), dJ[k], atol=1e-8)


def test_manipulability_gradient_fd(fr3):
    pm, om, _ = fr3
    q = np.array([0.1, 0.3, -0.2, -2.0, 0.4, 1.2, 0.3])
    m, g = O.manipulability(om, q)
    h = 1e-6
    fd = [(O.manipulability(om, q + h * np.eye(7)[k])[0] - O.manipulability(om, q - h * np.eye(7)[k])[0]) / (2 * h)
          for k in range(7)]
    np.testing.assert_allclose(g, fd, atol=1e-8)


def test_min_distance_gradient_fd(fr3):
    pm, om, _ = fr3
    rng = np.random.default_rng(5)
    checked = 0
    for _ in range(30):
        q = rng.uniform(pm.lower + 0.05, pm.upper - 0.05)
        d, g, pair = O.min_distance(om, q)
        h = 1e-7
        fwd = np.array([(O.min_distance(om, q + h * np.eye(7)[k])[0] - d) / h for k in range(7)])
        bwd = np.array([(d - O.min_distance(om, q - h * np.eye(7)[k])[0]) / h for k in range(7)])
        if np.max(np.abs(fwd - bwd)) > 1e-4:
            continue  # non-smooth point (argmin switch / non-unique witness)
        np.testing.assert_allclose(g, 0.5 * (fwd + bwd), atol=2e-5)
        checked += 1
    assert checked >= 20


def test_pinv_cod_rank_deficient():
    # JJ^T of a rank-5 Jacobian: COD pseudo-inverse = Moore-Penrose on the range
    rng = np.random.default_rng(1)
    J = rng.normal(size=(6, 5)) @ rng.normal(size=(5, 7))
    A = J @ J.T
    X = R.pinv_cod(A)
    np.testing.assert_allclose(X, np.linalg.pinv(A, rcond=1e-10), atol=1e-8)

"""ORACLE / TEST INFRASTRUCTURE ONLY — never imported by the product path.

Independent numpy restatement of the reference QP-IK hot path, used to
(1) cross-check the C restatement in ``oracle/drc_oracle.c`` and
(2) generate the committed golden fixtures under ``tests/golden``.

Each function cites the reference code it restates.  Pinocchio / hpp-fcl /
OSQP are absent from the container, so their published
mathematical definitions are restated; parity at those three boundaries is
**unpinned** and is anchored instead on analytic known answers, finite
differences, brute-force distance checks and KKT optimality certificates
(tests/test_oracle_*.py).
"""
import numpy as np

from pyref_model import REVOLUTE, PRISMATIC, SPHERE, CYLINDER, BOX, load_urdf  # noqa: F401

OSQP_INFTY = 1e30


# ----------------------------------------------------------------------------
# Kinematics  (robot_data.cpp:101-107, :392-402; Pinocchio LOCAL_WORLD_ALIGNED)
# ----------------------------------------------------------------------------
def axis_rot(axis, q):
    x, y, z = axis
    c, s = np.cos(q), np.sin(q)
    C = 1 - c
    return np.array([[c + x * x * C, x * y * C - z * s, x * z * C + y * s],
                     [y * x * C + z * s, c + y * y * C, y * z * C - x * s],
                     [z * x * C - y * s, z * y * C + x * s, c + z * z * C]])


def fk(m, q):
    """oMi for every joint (4x4), Pinocchio forwardKinematics."""
    oMi = [np.eye(4)]
    for j in range(1, m.nv + 1):
        T = oMi[m.jparent[j]] @ m.jplacement[j]
        M = np.eye(4)
        if m.jtype[j] == REVOLUTE:
            M[:3, :3] = axis_rot(m.jaxis[j], q[j - 1])
        else:
            M[:3, 3] = m.jaxis[j] * q[j - 1]
        oMi.append(T @ M)
    return oMi


def frame_pose(m, oMi, link):
    jid, place = m.frames[link]
    return oMi[jid] @ place


def joint_axes(m, oMi):
    z = [None] + [oMi[j][:3, :3] @ m.jaxis[j] for j in range(1, m.nv + 1)]
    p = [None] + [oMi[j][:3, 3] for j in range(1, m.nv + 1)]
    return z, p


def point_jacobian(m, oMi, jid, point):
    """6 x nv LWA Jacobian of a point rigidly attached to joint jid."""
    J = np.zeros((6, m.nv))
    z, p = joint_axes(m, oMi)
    for k in m.ancestors(jid):
        if m.jtype[k] == REVOLUTE:
            J[:3, k - 1] = np.cross(z[k], point - p[k])
            J[3:, k - 1] = z[k]
        else:
            J[:3, k - 1] = z[k]
    return J


def frame_jacobian(m, oMi, link):
    jid, _ = m.frames[link]
    return point_jacobian(m, oMi, jid, frame_pose(m, oMi, link)[:3, 3])


def frame_jacobian_dq(m, oMi, link):
    """dJ/dq_k (k = 0..nv-1) of the LWA frame Jacobian: the exact derivative
    that ``getFrameJacobianTimeVariation`` returns for qdot = e_k
    (robot_data.cpp:544-553).  Returns array [nv, 6, nv]."""
    jid, _ = m.frames[link]
    pe = frame_pose(m, oMi, link)[:3, 3]
    z, p = joint_axes(m, oMi)
    anc = m.ancestors(jid)
    ancset = {a: m.ancestors(a) for a in anc}
    nv = m.nv
    dJ = np.zeros((nv, 6, nv))

    def dz(i, k):   # d z_i / d q_k
        if k in ancset[i] and k != i and m.jtype[k] == REVOLUTE:
            return np.cross(z[k], z[i])
        return np.zeros(3)

    def dpoint(pt, k, chain):   # d pt / d q_k, pt attached after joints in chain
        if k not in chain:
            return np.zeros(3)
        return np.cross(z[k], pt - p[k]) if m.jtype[k] == REVOLUTE else z[k].copy()

    for k in anc:
        dpe = dpoint(pe, k, anc)
        for i in anc:
            chain_i = [a for a in ancset[i] if a != i]   # joints moving p_i
            dzi = dz(i, k)
            if m.jtype[i] == REVOLUTE:
                dpi = dpoint(p[i], k, chain_i)
                dJ[k - 1, :3, i - 1] = np.cross(dzi, pe - p[i]) + np.cross(z[i], dpe - dpi)
                dJ[k - 1, 3:, i - 1] = dzi
            else:
                dJ[k - 1, :3, i - 1] = dzi
    return dJ


def pinv_cod(A, thr=1e-6):
    """DyrosMath::PinvCOD (math_type_define.h:563-570): Eigen's
    CompleteOrthogonalDecomposition with setThreshold(1e-6).  The rank is the
    number of column-pivoted QR pivots with |R_ii| > thr*|R_00|; the result is
    the Moore-Penrose inverse of the QR-truncated matrix Q_r [R11 R12] P^T
    (what cod.pseudoInverse() returns; unique, so independent of the Z chosen)."""
    A = np.asarray(A, float)
    import scipy.linalg as sla
    if A.size == 0:
        return np.zeros(A.T.shape)
    Q, R, P = sla.qr(A, pivoting=True, mode="economic")
    d = np.abs(np.diag(R))
    if d[0] == 0:
        return np.zeros(A.T.shape)
    r = int(np.sum(d > thr * d[0]))
    W = R[:r, :]                                  # [R11 R12], full row rank
    Wp = W.T @ np.linalg.inv(W @ W.T)             # pinv of W
    X = np.zeros((A.shape[1], A.shape[0]))
    X[P, :] = Wp @ Q[:, :r].T
    return X


def manipulability(m, q, link, arm_cols=None):
    """RobotData::getManipulability(true,false) robot_data.cpp:519-553 (and the
    MoMa arm-block variant mobile_manipulator/robot_data.cpp:439-475)."""
    oMi = fk(m, q)
    J = frame_jacobian(m, oMi, link)
    dJ = frame_jacobian_dq(m, oMi, link)
    cols = np.arange(m.nv) if arm_cols is None else np.asarray(arm_cols)
    Jr = J[:, cols]
    JJt = Jr @ Jr.T
    man = np.sqrt(max(np.linalg.det(JJt), 0.0))
    Ainv = pinv_cod(JJt)
    grad = np.array([man * np.trace(dJ[k][:, cols] @ Jr.T @ Ainv) for k in cols])
    return man, grad


# ----------------------------------------------------------------------------
# Narrow phase  (hpp-fcl distance semantics through pinocchio::computeDistances)
# ----------------------------------------------------------------------------
def geom_poses(m, oMi):
    return [oMi[g["parent_joint"]] @ g["placement"] for g in m.geoms]


def support(g, T, d):
    """World support point of a geometry core (sphere core = its centre)."""
    R, c = T[:3, :3], T[:3, 3]
    if g["type"] == SPHERE:
        return c.copy()
    dl = R.T @ d
    if g["type"] == CYLINDER:
        r, h = g["params"][0], g["params"][1]
        rho = np.hypot(dl[0], dl[1])
        loc = np.zeros(3)
        if rho > 0:
            loc[0], loc[1] = r * dl[0] / rho, r * dl[1] / rho
        loc[2] = h if dl[2] > 0 else -h
    else:
        hx = g["params"]
        loc = np.array([hx[0] if dl[0] > 0 else -hx[0], hx[1] if dl[1] > 0 else -hx[1], hx[2] if dl[2] > 0 else -hx[2]])
    return c + R @ loc


def _closest_simplex(W):
    """Closest point to the origin on conv(W) (|W| = 1..4) with barycentric
    weights; returns (v, keep_indices, lambdas).  Exhaustive sub-simplex
    search (small, exact; the C/HIP restatements use the same rule)."""
    import itertools
    n = len(W)
    best = None
    for k in range(n, 0, -1):
        for sub in itertools.combinations(range(n), k):
            P = np.array([W[i] for i in sub])
            if k == 1:
                lam = np.array([1.0])
            else:
                # minimise |sum lam_i P_i|^2 s.t. sum lam = 1 (affine hull)
                D = P[1:] - P[0]
                G = D @ D.T
                try:
                    mu = np.linalg.solve(G, -D @ P[0])
                except np.linalg.LinAlgError:
                    continue
                lam = np.concatenate([[1 - mu.sum()], mu])
                if np.any(lam < -1e-14):
                    continue
            v = lam @ P
            dv = v @ v
            if best is None or dv < best[0] - 1e-18:
                best = (dv, v, list(sub), lam)
    return best[1], best[2], best[3]


def gjk_distance(gA, TA, gB, TB, tol=1e-12, max_iter=128):
    """GJK on the cores (sphere radius handled as a margin by the caller).
    Returns (dist, pA, pB, intersecting)."""
    v = TA[:3, 3] - TB[:3, 3]
    if v @ v < 1e-24:
        v = np.array([1.0, 0, 0])
    W, A_, B_ = [], [], []
    lam = None
    for it in range(max_iter):
        a = support(gA, TA, -v)
        b = support(gB, TB, v)
        w = a - b
        vv = v @ v
        if W and vv - v @ w <= tol * np.sqrt(vv):
            break
        if any(np.allclose(w, x, atol=0, rtol=0) for x in W):
            break
        W.append(w); A_.append(a); B_.append(b)
        v, keep, lam = _closest_simplex(W)
        W = [W[i] for i in keep]; A_ = [A_[i] for i in keep]; B_ = [B_[i] for i in keep]
        if len(W) == 4 or v @ v < 1e-24:
            return 0.0, None, None, True
    pA = sum(l * a for l, a in zip(lam, A_))
    pB = sum(l * b for l, b in zip(lam, B_))
    return float(np.linalg.norm(pA - pB)), pA, pB, False


def point_cylinder(c, T, r, h):
    """Signed distance and closest surface point of a solid cylinder."""
    R, cc = T[:3, :3], T[:3, 3]
    loc = R.T @ (c - cc)
    rho = np.hypot(loc[0], loc[1])
    inside = rho <= r and abs(loc[2]) <= h
    if not inside:
        q = loc.copy()
        if rho > r:
            q[0], q[1] = loc[0] * r / rho, loc[1] * r / rho
        q[2] = min(max(loc[2], -h), h)
        qw = cc + R @ q
        return np.linalg.norm(c - qw), qw
    dside, dtop, dbot = r - rho, h - loc[2], h + loc[2]
    q = loc.copy()
    if dside <= dtop and dside <= dbot:
        if rho > 0:
            q[0], q[1] = loc[0] * r / rho, loc[1] * r / rho
        else:
            q[0], q[1] = r, 0.0
        dd = dside
    elif dtop <= dbot:
        q[2] = h; dd = dtop
    else:
        q[2] = -h; dd = dbot
    return -dd, cc + R @ q


def point_box(c, T, hx):
    R, cc = T[:3, :3], T[:3, 3]
    loc = R.T @ (c - cc)
    inside = np.all(np.abs(loc) <= hx)
    if not inside:
        q = np.clip(loc, -hx, hx)
        qw = cc + R @ q
        return np.linalg.norm(c - qw), qw
    gaps = hx - np.abs(loc)
    a = int(np.argmin(gaps))
    q = loc.copy()
    q[a] = hx[a] if loc[a] >= 0 else -hx[a]
    return -gaps[a], cc + R @ q


def pair_distance(gA, TA, gB, TB):
    """Signed distance + witness points (pA on A, pB on B) with the hpp-fcl
    convention pB - pA = d * n, n the A->B separating direction."""
    tA, tB = gA["type"], gB["type"]
    if tA == SPHERE and tB == SPHERE:
        cA, cB = TA[:3, 3], TB[:3, 3]
        rA, rB = gA["params"][0], gB["params"][0]
        v = cB - cA
        L = np.linalg.norm(v)
        n = v / L if L > 0 else np.array([1.0, 0, 0])
        return L - rA - rB, cA + rA * n, cB - rB * n
    if tA == SPHERE or tB == SPHERE:
        flip = tB == SPHERE
        gs, Ts, go, To = (gB, TB, gA, TA) if flip else (gA, TA, gB, TB)
        c, rs = Ts[:3, 3], gs["params"][0]
        if go["type"] == CYLINDER:
            sd, q = point_cylinder(c, To, go["params"][0], go["params"][1])
        else:
            sd, q = point_box(c, To, go["params"])
        u = q - c
        L = np.linalg.norm(u)
        n = u / L if L > 0 else np.array([1.0, 0, 0])
        if sd < 0:
            n = -n           # centre inside: separating direction points out
        d = sd - rs
        ps = c + rs * n      # on the sphere
        if flip:             # A = other, B = sphere: n_AB = -n
            return d, q, ps
        return d, ps, q
    dist, pA, pB, inter = gjk_distance(gA, TA, gB, TB)
    if inter:
        raise PenetrationError()
    return dist, pA, pB


class PenetrationError(Exception):
    pass


def min_distance(m, q):
    """RobotData::getMinDistance(true,false,false) robot_data.cpp:424-494."""
    oMi = fk(m, q)
    Tg = geom_poses(m, oMi)
    best, bi, bw = np.inf, -1, None
    for idx, (a, b) in enumerate(m.pairs):
        d, pA, pB = pair_distance(m.geoms[a], Tg[a], m.geoms[b], Tg[b])
        if d < best:
            best, bi, bw = d, idx, (pA, pB)
    a, b = m.pairs[bi]
    pA, pB = bw
    jA, jB = m.geoms[a]["parent_joint"], m.geoms[b]["parent_joint"]
    n = pB - pA
    n = n / np.linalg.norm(n)
    JA = point_jacobian(m, oMi, jA, pA)[:3] if jA > 0 else np.zeros((3, m.nv))
    JB = point_jacobian(m, oMi, jB, pB)[:3] if jB > 0 else np.zeros((3, m.nv))
    grad = n @ (JB - JA)
    if best < 0:
        grad = -grad
    return best, grad, bi


# ----------------------------------------------------------------------------
# Task-space helpers  (include/math_type_define.h)
# ----------------------------------------------------------------------------
def get_phi(Rc, Rd):
    """DyrosMath::getPhi (math_type_define.h:283-298)."""
    s = np.zeros(3)
    for i in range(3):
        s += np.cross(Rc[:, i], Rd[:, i])
    return -0.5 * s


def task_space_error(x_target, xdot_target, x, xdot):
    """DyrosMath::getTaskSpaceError (math_type_define.h:633-645)."""
    e = np.zeros(6)
    e[:3] = x_target[:3, 3] - x[:3, 3]
    e[3:] = get_phi(x_target[:3, :3], x[:3, :3])
    return e, xdot_target - xdot


def cubic(t, t0, tf, x0, xf, xd0, xdf):
    """DyrosMath::cubic (math_type_define.h:62-102)."""
    if t < t0:
        return x0
    if t > tf:
        return xf
    e, T = t - t0, tf - t0
    dx = xf - x0
    return (x0 + xd0 * e + (3 * dx / T ** 2 - 2 * xd0 / T - xdf / T) * e * e
            + (-2 * dx / T ** 3 + (xd0 + xdf) / T ** 2) * e ** 3)


def cubic_dot(t, t0, tf, x0, xf, xd0, xdf):
    """DyrosMath::cubicDot (math_type_define.h:104-143)."""
    if t < t0:
        return xd0
    if t > tf:
        return xdf
    e, T = t - t0, tf - t0
    dx = xf - x0
    return (xd0 + 2 * (3 * dx / T ** 2 - 2 * xd0 / T - xdf / T) * e
            + 3 * (-2 * dx / T ** 3 + (xd0 + xdf) / T ** 2) * e * e)


def so3_log(R):
    """Principal matrix logarithm of a rotation (Eigen MatrixBase::log on a
    rotation matrix), returned as the axis-angle vector."""
    c = (np.trace(R) - 1) / 2
    c = min(1.0, max(-1.0, c))
    th = np.arccos(c)
    w = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]])
    if th < 1e-8:
        return 0.5 * w
    if np.pi - th < 1e-6:
        # near pi: axis from the symmetric part
        B = (R + np.eye(3)) / 2
        k = int(np.argmax(np.diag(B)))
        a = B[:, k] / np.sqrt(B[k, k])
        if a @ w < 0:
            a = -a
        return th * a
    return th / (2 * np.sin(th)) * w


def so3_exp(w):
    th = np.linalg.norm(w)
    K = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])
    if th < 1e-12:
        return np.eye(3) + K
    return np.eye(3) + np.sin(th) / th * K + (1 - np.cos(th)) / th ** 2 * K @ K


def task_space_cubic(x_target, xdot_target, x_init, xdot_init, t, t0, T):
    """DyrosMath::getTaskSpaceCubic (math_type_define.h:647-687) with
    rotationCubic (:235-255) and rotationCubicDot (:257-281)."""
    tf = t0 + T
    xd = np.eye(4)
    xdd = np.zeros(6)
    for i in range(3):
        xd[i, 3] = cubic(t, t0, tf, x_init[i, 3], x_target[i, 3], xdot_init[i], xdot_target[i])
        xdd[i] = cubic_dot(t, t0, tf, x_init[i, 3], x_target[i, 3], xdot_init[i], xdot_target[i])
    R0, Rf = x_init[:3, :3], x_target[:3, :3]
    if t >= tf:
        xd[:3, :3] = Rf
    elif t < t0:
        xd[:3, :3] = R0
    else:
        tau = cubic(t, t0, tf, 0, 1, 0, 0)
        xd[:3, :3] = R0 @ so3_exp(so3_log(R0.T @ Rf) * tau)
    r = so3_log(R0.T @ Rf)
    rd = np.array([cubic_dot(t, t0, tf, 0, r[i], 0, 0) for i in range(3)])
    rd = R0 @ rd
    tau = (t - t0) / (tf - t0)
    if tau < 0:
        rd = np.zeros(3)      # w_0 = 0 at the call site
    if tau > 1:
        rd = np.zeros(3)
    xdd[3:] = rd
    return xd, xdd


# ----------------------------------------------------------------------------
# Dynamics  (robot_data.cpp:109-124: crba, computeGeneralizedGravity,
#            nonLinearEffects, PinvCOD; MoMa robot_data.cpp:126-144)
# Two formulations that share nothing but the model, so each pins the other:
#   * mass_matrix: kinetic-energy definition, sum over bodies of the COM
#     Jacobian quadratic forms (what CRBA computes).
#   * rnea: Luh-Walker-Paul Newton-Euler in the world frame about each body's
#     COM (what nonLinearEffects / computeGeneralizedGravity compute with
#     qdd = 0 / qd = qdd = 0).
# ----------------------------------------------------------------------------
GRAVITY = np.array([0.0, 0.0, -9.81])   # pinocchio::Model::gravity981 default


def body_inertias(m):
    """Per joint: merged (mass, com, I about com) in the joint frame —
    Pinocchio's appendBodyToJoint for links behind fixed joints."""
    out = [(0.0, np.zeros(3), np.zeros((3, 3)))]
    for j in range(1, m.nv + 1):
        parts = m.inertia[j]
        mass = sum(p[0] for p in parts)
        if mass <= 0:
            out.append((0.0, np.zeros(3), sum((p[2] for p in parts), np.zeros((3, 3)))))
            continue
        com = sum(p[0] * p[1] for p in parts) / mass
        I = np.zeros((3, 3))
        for mk, ck, Ik in parts:
            d = ck - com
            I += Ik + mk * (d @ d * np.eye(3) - np.outer(d, d))
        out.append((mass, com, I))
    return out


def mass_matrix(m, q):
    """M(q) = sum_k m_k Jv_k^T Jv_k + Jw_k^T I_k Jw_k (full symmetric M of
    crba + selfadjointView<Upper>, robot_data.cpp:111,116)."""
    oMi = fk(m, q)
    M = np.zeros((m.nv, m.nv))
    for j, (mass, com, I) in enumerate(body_inertias(m)):
        if j == 0:
            continue
        R, p = oMi[j][:3, :3], oMi[j][:3, 3]
        J = point_jacobian(m, oMi, j, R @ com + p)
        Jv, Jw = J[:3], J[3:]
        M += mass * Jv.T @ Jv + Jw.T @ (R @ I @ R.T) @ Jw
    return M


def rnea(m, q, qd, qdd, gravity=GRAVITY):
    """Inverse dynamics tau = M qdd + C(q,qd) qd + g(q)."""
    n = m.nv
    oMi = fk(m, q)
    bi = body_inertias(m)
    w = [np.zeros(3)] * (n + 1)
    wd = [np.zeros(3)] * (n + 1)
    a = [-np.asarray(gravity, float)] + [None] * n      # origin acceleration of each joint frame
    F, N, c = [None] * (n + 1), [None] * (n + 1), [None] * (n + 1)
    for j in range(1, n + 1):
        pj = m.jparent[j]
        z = oMi[j][:3, :3] @ m.jaxis[j]
        r = oMi[j][:3, 3] - oMi[pj][:3, 3]
        aj = a[pj] + np.cross(wd[pj], r) + np.cross(w[pj], np.cross(w[pj], r))
        if m.jtype[j] == REVOLUTE:
            w[j] = w[pj] + z * qd[j - 1]
            wd[j] = wd[pj] + z * qdd[j - 1] + np.cross(w[pj], z) * qd[j - 1]
        else:
            w[j], wd[j] = w[pj], wd[pj]
            aj = aj + z * qdd[j - 1] + 2.0 * np.cross(w[pj], z) * qd[j - 1]
        a[j] = aj
        mass, com, I = bi[j]
        R = oMi[j][:3, :3]
        c[j] = R @ com + oMi[j][:3, 3]
        rc = c[j] - oMi[j][:3, 3]
        ac = aj + np.cross(wd[j], rc) + np.cross(w[j], np.cross(w[j], rc))
        Iw = R @ I @ R.T
        F[j] = mass * ac
        N[j] = Iw @ wd[j] + np.cross(w[j], Iw @ w[j])
    f = [np.zeros(3) for _ in range(n + 1)]
    nm = [np.zeros(3) for _ in range(n + 1)]     # moment about the joint-frame origin
    tau = np.zeros(n)
    for j in range(n, 0, -1):
        pj_ = oMi[j][:3, 3]
        f[j] = f[j] + F[j]
        nm[j] = nm[j] + N[j] + np.cross(c[j] - pj_, F[j])
        z = oMi[j][:3, :3] @ m.jaxis[j]
        tau[j - 1] = z @ nm[j] if m.jtype[j] == REVOLUTE else z @ f[j]
        pp = m.jparent[j]
        if pp > 0:
            f[pp] = f[pp] + f[j]
            nm[pp] = nm[pp] + nm[j] + np.cross(pj_ - oMi[pp][:3, 3], f[j])
    return tau


def dynamics(m, q, qd):
    """RobotData::updateDynamics (robot_data.cpp:109-124): M, M+, g, nle, c."""
    M = mass_matrix(m, q)
    g = rnea(m, q, np.zeros(m.nv), np.zeros(m.nv))
    nle = rnea(m, q, qd, np.zeros(m.nv))
    return dict(M=M, Minv=pinv_cod(M), g=g, nle=nle, c=nle - g)


def selection_matrix(nv, n_arm, n_wheel, joint_index, actuator_index, J_mobile, yaw):
    """MobileManipulator S (D x A): identity on the arm and wheel blocks
    (robot_data.cpp:22-25), Rz(yaw) J_mobile on the virtual block (:115-120)."""
    vs, ms, ws = joint_index
    am, aw = actuator_index
    S = np.zeros((nv, n_arm + n_wheel))
    S[ms:ms + n_arm, am:am + n_arm] = np.eye(n_arm)
    S[ws:ws + n_wheel, aw:aw + n_wheel] = np.eye(n_wheel)
    c, s = np.cos(yaw), np.sin(yaw)
    S[vs:vs + 3, aw:aw + n_wheel] = np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]]) @ J_mobile
    return S


def dynamics_actuated(m, q, qd, S):
    """MobileManipulator::RobotData::updateDynamics (robot_data.cpp:136-142)."""
    d = dynamics(m, q, qd)
    Ma = S.T @ d["M"] @ S
    return dict(M=Ma, Minv=pinv_cod(Ma), g=S.T @ d["g"], nle=S.T @ d["nle"], c=S.T @ d["c"])


# ----------------------------------------------------------------------------
# QP assembly  (QP_base.h:65-93,202-227; manipulator/QP_IK.cpp:7-131;
#               mobile_manipulator/QP_IK.cpp:7-128)
# ----------------------------------------------------------------------------
ALPHA = 50.0


def build_qp_manipulator(m, q, xdot_des, link, man=None, dist=None):
    n = m.nv
    oMi = fk(m, q)
    J = frame_jacobian(m, oMi, link)
    if man is None:
        man = manipulability(m, q, link)
    if dist is None:
        dist = min_distance(m, q)[:2]
    mval, mgrad = man
    dval, dgrad = dist
    nx = 3 * n + 2
    nineq = 2 * n + 2
    P = np.zeros((nx, nx))
    qv = np.zeros(nx)
    P[:n, :n] = 2.0 * J.T @ J + np.eye(n)
    qv[:n] = -2.0 * J.T @ xdot_des
    qv[n:] = 1000.0
    lb = np.concatenate([-m.vel, np.zeros(2 * n + 2)])
    ub = np.concatenate([m.vel, np.full(2 * n + 2, OSQP_INFTY)])
    G = np.zeros((nineq, nx))
    lg = np.zeros(nineq)
    for i in range(n):
        G[i, i] = 1.0; G[i, n + i] = 1.0
        lg[i] = -ALPHA * (q[i] - m.lower[i])
        G[n + i, i] = -1.0; G[n + i, 2 * n + i] = 1.0
        lg[n + i] = -ALPHA * (m.upper[i] - q[i])
    G[2 * n, :n] = mgrad; G[2 * n, 3 * n] = 1.0
    lg[2 * n] = -ALPHA * (mval - 0.01)
    G[2 * n + 1, :n] = dgrad; G[2 * n + 1, 3 * n + 1] = 1.0
    lg[2 * n + 1] = -ALPHA * (dval - 0.05)
    A = np.vstack([np.eye(nx), G])
    l = np.concatenate([lb, lg])
    u = np.concatenate([ub, np.full(nineq, OSQP_INFTY)])
    return P, qv, A, l, u


def build_qp_moma(m, q, S, xdot_des, link, mani_start_j, mani_start_a, n_arm, man=None, dist=None):
    """mobile_manipulator/QP_IK.cpp:59-128.  S: D x A selection matrix."""
    oMi = fk(m, q)
    J = frame_jacobian(m, oMi, link)
    Jt = J @ S
    na = S.shape[1]
    arm_cols = np.arange(mani_start_j, mani_start_j + n_arm)
    if man is None:
        man = manipulability(m, q, link, arm_cols)
    if dist is None:
        d, g, _ = min_distance(m, q)
        dist = (d, g[arm_cols])
    mval, mgrad = man
    dval, dgrad = dist
    P = 2.0 * Jt.T @ Jt + 0.01 * np.eye(na)
    qv = -2.0 * Jt.T @ xdot_des
    nineq = 2 * n_arm + 2
    G = np.zeros((nineq, na))
    lg = np.zeros(nineq)
    qa = q[arm_cols]
    lo, hi = m.lower[arm_cols], m.upper[arm_cols]
    for i in range(n_arm):
        G[i, mani_start_a + i] = 1.0
        lg[i] = -ALPHA * (qa[i] - lo[i])
        G[n_arm + i, mani_start_a + i] = -1.0
        lg[n_arm + i] = -ALPHA * (hi[i] - qa[i])
    G[2 * n_arm, mani_start_a:mani_start_a + n_arm] = mgrad
    lg[2 * n_arm] = -ALPHA * (mval - 0.01)
    G[2 * n_arm + 1, mani_start_a:mani_start_a + n_arm] = dgrad
    lg[2 * n_arm + 1] = -ALPHA * (dval - 0.05)
    A = np.vstack([np.eye(na), G])
    l = np.concatenate([np.full(na, -OSQP_INFTY), lg])
    u = np.full(na + nineq, OSQP_INFTY)
    return P, qv, A, l, u


def pose_from12(v12):
    """[R col-major (9) | p (3)] (the C-ABI pose layout) -> 4 x 4."""
    T = np.eye(4)
    T[:3, :3] = np.asarray(v12[:9]).reshape(3, 3).T
    T[:3, 3] = v12[9:]
    return T


def moma_step_qp(m, q, S, x_target12, xdot_target, link, mani_start_j, mani_start_a, n_arm, dist, kp=400.0):
    """MobileManipulator::RobotController::QPIKStep's QP for one robot
    (mobile_manipulator/robot_controller.cpp:170-180: xdot_des = Kp e +
    xdot_target, Kp = 400 (:15), no Kv term) over build_qp_moma, with the
    arm-block manipulability computed here and the distance stage (d,
    grad d[arm]) supplied.  Returns (P, q, A, l, u, xdot_des, (m, grad m))."""
    arm = np.arange(mani_start_j, mani_start_j + n_arm)
    x = frame_pose(m, fk(m, q), link)
    e, _ = task_space_error(pose_from12(x_target12), xdot_target, x, np.zeros(6))
    xdd = kp * e + xdot_target
    man = manipulability(m, q, link, arm)
    P, qv, A, l, u = build_qp_moma(m, q, S, xdd, link, mani_start_j, mani_start_a, n_arm, man=man, dist=dist)
    return P, qv, A, l, u, xdd, man


def build_qp_qpid(m, q, qd, Jt, xdd, jdot_v, M, g, man, dist, arm, arm_col, slacks):
    """QPID's QP (manipulator/QP_ID.cpp:85-192 with slacks; MoMa QP_ID.cpp:
    66-184 without).  Jt: 6 x na task Jacobian over the QP's task variables,
    jdot_v: its time variation times the actuated velocity, man/dist:
    (value, grad[arm], graddot . qdot_arm), arm: joint ids (0-based) of the
    arm, arm_col: QP column of arm joint 0."""
    na = Jt.shape[1]
    n = len(arm)
    nx = 2 * na + (4 * n + 2 if slacks else 0)
    P = np.zeros((nx, nx))
    qv = np.zeros(nx)
    P[:na, :na] = 2.0 * Jt.T @ Jt
    qv[:na] = -2.0 * Jt.T @ (xdd - jdot_v)
    if slacks:
        qv[2 * na:] = 1000.0
    nineq = 4 * n + 2
    G = np.zeros((nineq, nx))
    lg = np.zeros(nineq)
    qa, qda = q[arm], qd[arm]
    lo, hi, vm = m.lower[arm], m.upper[arm], m.vel[arm]
    a = ALPHA
    for i in range(n):
        c = arm_col + i
        G[i, c] = 1.0; lg[i] = -2 * a * qda[i] - a * a * (qa[i] - lo[i])
        G[n + i, c] = -1.0; lg[n + i] = 2 * a * qda[i] - a * a * (hi[i] - qa[i])
        G[2 * n + i, c] = 1.0; lg[2 * n + i] = -a * (qda[i] + vm[i])
        G[3 * n + i, c] = -1.0; lg[3 * n + i] = -a * (vm[i] - qda[i])
        if slacks:
            for k in range(4):
                G[k * n + i, 2 * na + k * n + i] = 1.0
    mval, mgrad, mgd = man
    dval, dgrad, dgd = dist
    G[4 * n, arm_col:arm_col + n] = mgrad
    lg[4 * n] = -mgd - 2 * a * mgrad @ qda - a * a * (mval - 0.01)
    G[4 * n + 1, arm_col:arm_col + n] = dgrad
    lg[4 * n + 1] = -dgd - 2 * a * dgrad @ qda - a * a * (dval - 0.05)
    if slacks:
        G[4 * n, 2 * na + 4 * n] = 1.0
        G[4 * n + 1, 2 * na + 4 * n + 1] = 1.0
    Ge = np.zeros((na, nx))
    Ge[:, :na] = M
    Ge[:, na:2 * na] = -np.eye(na)
    rows = [G, Ge]
    l = [lg, -g]
    u = [np.full(nineq, OSQP_INFTY), -g]
    if slacks:
        lb = np.concatenate([np.full(2 * na, -OSQP_INFTY), np.zeros(nx - 2 * na)])
        rows.insert(0, np.eye(nx)); l.insert(0, lb); u.insert(0, np.full(nx, OSQP_INFTY))
    return P, qv, np.vstack(rows), np.concatenate(l), np.concatenate(u)


# ----------------------------------------------------------------------------
# Exact QP solution (independent of the ADMM restatement): primal-dual
# interior point + active-set refinement + KKT certificate.
# ----------------------------------------------------------------------------
def _ineq_form(A, l, u):
    rows, d, sgn = [], [], []
    for i in range(A.shape[0]):
        if l[i] > -1e20:
            rows.append(A[i]); d.append(l[i]); sgn.append((i, -1))
        if u[i] < 1e20:
            rows.append(-A[i]); d.append(-u[i]); sgn.append((i, +1))
    return np.array(rows), np.array(d), sgn


def feasible(A, l, u):
    from scipy.optimize import linprog
    n = A.shape[1]
    fin_l, fin_u = l > -1e20, u < 1e20
    A_ub = np.vstack([-A[fin_l], A[fin_u]])
    b_ub = np.concatenate([-l[fin_l], u[fin_u]])
    r = linprog(np.zeros(n), A_ub=A_ub, b_ub=b_ub, bounds=[(None, None)] * n, method="highs")
    return r.status == 0


def solve_qp_exact(P, qv, A, l, u, iters=80):
    """Returns (x, y, status) with OSQP sign convention for y (y>0 on an
    active upper bound, y<0 on an active lower bound). status 1 = solved,
    3 = primal infeasible, 0 = no finite iterate (never happens on the test
    instances; callers treat it as a failure of the certificate)."""
    if not feasible(A, l, u):
        return None, None, 3
    C, d, sgn = _ineq_form(A, l, u)
    # equilibrate: unit-norm constraint rows, cost scaled to O(1)
    rn = np.linalg.norm(C, axis=1)
    rn[rn == 0] = 1.0
    C, d = C / rn[:, None], d / rn
    cs = max(1.0, np.max(np.abs(qv)), np.max(np.abs(P)))
    P, qv = P / cs, qv / cs
    n, mc = P.shape[0], C.shape[0]
    x = np.zeros(n)
    s = np.maximum(C @ x - d, 1.0)
    lam = np.ones(mc)
    # the iterate with the smallest merit max(|rd|, |rp|, mu) is kept: once mu
    # reaches ~1e-14 the Newton matrix is numerically singular (P has a null
    # space on QPID's qdd block) and further steps can diverge to inf/NaN
    best, best_merit = (x.copy(), s.copy(), lam.copy()), np.inf
    for it in range(iters):
        rd = P @ x + qv - C.T @ lam
        rp = C @ x - d - s
        mu = s @ lam / mc
        merit = max(np.max(np.abs(rd)), np.max(np.abs(rp)), mu)
        if not np.isfinite(merit):
            break
        if merit < best_merit:
            best, best_merit = (x.copy(), s.copy(), lam.copy()), merit
        if np.max(np.abs(rd)) < 1e-11 and np.max(np.abs(rp)) < 1e-11 and mu < 1e-14:
            break
        if mu < 1e-16 and merit > 1e3 * best_merit:
            break                      # diverging after convergence: keep the best iterate

        def newton(rs):
            # P dx - C^T dlam = -rd ; C dx - ds = -rp ; lam ds + s dlam = -rs
            W = lam / s
            H = P + C.T @ (W[:, None] * C)
            dx = np.linalg.solve(H, -rd - C.T @ ((rs + lam * rp) / s))
            ds = C @ dx + rp
            dl = (-rs - lam * ds) / s
            return dx, ds, dl

        rs = s * lam
        dx, ds, dl = newton(rs)

        def step(v, dv):
            neg = dv < 0
            return min(1.0, np.min(-v[neg] / dv[neg])) if np.any(neg) else 1.0

        a_aff = min(step(s, ds), step(lam, dl))
        mu_aff = (s + a_aff * ds) @ (lam + a_aff * dl) / mc
        sigma = (mu_aff / mu) ** 3
        rs = s * lam + ds * dl - sigma * mu
        dx, ds, dl = newton(rs)
        if not (np.all(np.isfinite(dx)) and np.all(np.isfinite(ds)) and np.all(np.isfinite(dl))):
            break
        a = 0.995 * min(step(s, ds), step(lam, dl))
        x += a * dx; s += a * ds; lam += a * dl
    x, s, lam = best
    if not np.isfinite(best_merit):
        return None, None, 0           # the interior point never produced a finite iterate
    # active-set refinement: equality-constrained solve on the active rows
    act = [k for k in range(mc) if lam[k] > s[k]]
    Ca, da = C[act], d[act]
    K = np.block([[P, -Ca.T], [Ca, np.zeros((len(act), len(act)))]])
    rhs = np.concatenate([-qv, da])
    sol = np.linalg.lstsq(K, rhs, rcond=None)[0]
    xr, lr = sol[:n], sol[n:]
    ok = (np.all(C @ xr - d >= -1e-9) and np.all(lr >= -1e-9)
          and np.max(np.abs(P @ xr + qv - Ca.T @ lr)) < 1e-9)
    if ok:
        x = xr
        lam = np.zeros(mc); lam[act] = lr
    y = np.zeros(A.shape[0])
    lam = lam / rn * cs
    for k, (i, sg) in enumerate(sgn):
        y[i] += sg * lam[k]
    if not (np.all(np.isfinite(x)) and np.all(np.isfinite(y))):
        return None, None, 0           # never report a non-finite point as solved
    return x, y, 1


def kkt_residuals(P, qv, A, l, u, x, y):
    """OSQP optimality conditions: stationarity, primal feasibility,
    complementarity (y_i>0 only at u_i, y_i<0 only at l_i)."""
    Ax = A @ x
    stat = np.max(np.abs(P @ x + qv + A.T @ y))
    prim = np.max(np.maximum(0, np.maximum(l - Ax, Ax - u)))
    comp = 0.0
    for i in range(A.shape[0]):
        if y[i] > 0:
            comp = max(comp, y[i] * abs(u[i] - Ax[i]) if u[i] < 1e20 else abs(y[i]))
        elif y[i] < 0:
            comp = max(comp, -y[i] * abs(Ax[i] - l[i]) if l[i] > -1e20 else abs(y[i]))
    return stat, prim, comp


def _support_md(gA, TA, gB, TB, d):
    a = support(gA, TA, d)
    b = support(gB, TB, -d)
    return (a - b, a, b)


def gjk_simplex(gA, TA, gB, TB, tol=1e-12, max_iter=128):
    """GJK returning the final simplex as (w, a, b) triples (w = a - b) and
    whether the origin is enclosed."""
    v = TA[:3, 3] - TB[:3, 3]
    if v @ v < 1e-24:
        v = np.array([1.0, 0, 0])
    S = []
    for it in range(max_iter):
        w = _support_md(gA, TA, gB, TB, -v)
        vv = v @ v
        if S and vv - v @ w[0] <= tol * np.sqrt(vv):
            return S, False, v
        if any(np.array_equal(w[0], x[0]) for x in S):
            return S, False, v
        S.append(w)
        v, keep, lam = _closest_simplex([x[0] for x in S])
        S = [S[i] for i in keep]
        if len(S) == 4 or v @ v < 1e-24:
            return S, True, v
    return S, False, v


def epa_penetration(gA, TA, gB, TB, tol=1e-12, max_iter=256):
    """Expanding-polytope penetration depth (hpp-fcl GJK+EPA semantics):
    returns d = -depth and witness points with pB - pA = d * n."""
    S, inter, _ = gjk_simplex(gA, TA, gB, TB)
    assert inter
    V = list(S)
    # complete a degenerate final simplex to a tetrahedron
    for d in ([1, 0, 0], [0, 1, 0], [0, 0, 1], [-1, 0, 0], [0, -1, 0], [0, 0, -1]):
        if len(V) >= 4:
            break
        w = _support_md(gA, TA, gB, TB, np.array(d, float))
        if all(np.linalg.norm(w[0] - x[0]) > 1e-12 for x in V):
            V.append(w)
    P = [x[0] for x in V]
    faces = []
    for f, o in (((0, 1, 2), 3), ((0, 3, 1), 2), ((0, 2, 3), 1), ((1, 3, 2), 0)):
        a, b, c = P[f[0]], P[f[1]], P[f[2]]
        nrm = np.cross(b - a, c - a)
        faces.append(f if nrm @ (P[o] - a) <= 0 else (f[0], f[2], f[1]))

    def fdat(f):
        a, b, c = P[f[0]], P[f[1]], P[f[2]]
        nrm = np.cross(b - a, c - a)
        L = np.linalg.norm(nrm)
        if L <= 1e-300:
            return np.zeros(3), np.inf
        nrm = nrm / L
        return nrm, nrm @ a

    for it in range(max_iter):
        fd = [fdat(f) for f in faces]
        k = int(np.argmin([x[1] for x in fd]))
        nrm, dist = fd[k]
        w = _support_md(gA, TA, gB, TB, nrm)
        if nrm @ w[0] - dist <= tol:
            break
        if any(np.max(np.abs(w[0] - x)) <= 1e-14 for x in P):
            break   # support point already a vertex: cannot expand (flat features)
        V.append(w); P.append(w[0])
        vi = len(P) - 1
        edges = []
        keep = []
        for f, (fn, fdist) in zip(faces, fd):
            if fn @ w[0] - fdist > 1e-12:
                for e in ((f[0], f[1]), (f[1], f[2]), (f[2], f[0])):
                    r = (e[1], e[0])
                    if r in edges:
                        edges.remove(r)
                    else:
                        edges.append(e)
            else:
                keep.append(f)
        faces = keep + [(e[0], e[1], vi) for e in edges]
    f = faces[k]
    a, b, c = P[f[0]], P[f[1]], P[f[2]]
    p = nrm * dist
    v0, v1, v2 = b - a, c - a, p - a
    d00, d01, d11, d20, d21 = v0 @ v0, v0 @ v1, v1 @ v1, v2 @ v0, v2 @ v1
    den = d00 * d11 - d01 * d01
    l1 = (d11 * d20 - d01 * d21) / den
    l2 = (d00 * d21 - d01 * d20) / den
    lam = np.array([1 - l1 - l2, l1, l2])
    pA = sum(l * V[i][1] for l, i in zip(lam, f))
    pB = sum(l * V[i][2] for l, i in zip(lam, f))
    return -dist, pA, pB, it

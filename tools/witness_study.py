"""Witness refinement study (CPU, diagnostic): for the argmin pair of the
oracle's min distance on a workload, compare the GJK/EPA witness points with
the critical point of |pA - pB|^2 on the identified surface features (Newton),
and measure how the raw and refined witnesses move under a 1e-13 perturbation
of q (the rounding-level path difference between two implementations).

    python tools/witness_study.py --robot ur5e --seed 1 --batch 512
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import oracle as O  # noqa: E402

SPHERE, CYL, BOX = 0, 1, 2


def shape_T(om, q, g):
    Tj = O.joint_placement(om, q, om.gparent[g])
    P = np.eye(4)
    gp = np.array(om.gplace[g][:])
    P[:3, :3] = gp[:9].reshape(3, 3)
    P[:3, 3] = gp[9:]
    return Tj @ P


# feature kinds: ('side',), ('cap', s), ('rim', s); box: ('box', fixed) with fixed = {axis: sign}
def classify(typ, prm, x, tau):
    if typ == CYL:
        r, h = prm[0], prm[1]
        rho, z = np.hypot(x[0], x[1]), x[2]
        s = 1.0 if z > 0 else -1.0
        if abs(z) > h - tau and rho > r - tau:
            return ("rim", s)
        if abs(z) > h - tau:
            return ("cap", s)
        return ("side",)
    fixed = {}
    for i in range(3):
        if abs(x[i]) > prm[i] - tau:
            fixed[i] = 1.0 if x[i] > 0 else -1.0
    if not fixed:
        i = int(np.argmax(np.abs(x) / np.array(prm[:3])))
        fixed[i] = 1.0 if x[i] > 0 else -1.0
    return ("box", fixed)


def param0(feat, prm, x):
    """initial feature parameters from a local point"""
    k = feat[0]
    if k == "side":
        return np.array([np.arctan2(x[1], x[0]), x[2]])
    if k == "rim":
        return np.array([np.arctan2(x[1], x[0])])
    if k == "cap":
        return np.array([x[0], x[1]])
    free = [i for i in range(3) if i not in feat[1]]
    return np.array([x[i] for i in free])


def point(feat, prm, u):
    """local point, its first derivatives (m x 3) and second derivatives (m x m x 3)"""
    k = feat[0]
    if k in ("side", "rim"):
        r, h = prm[0], prm[1]
        th = u[0]
        c, s = np.cos(th), np.sin(th)
        z = u[1] if k == "side" else feat[1] * h
        x = np.array([r * c, r * s, z])
        d1 = [np.array([-r * s, r * c, 0.0])]
        m = 2 if k == "side" else 1
        if k == "side":
            d1.append(np.array([0.0, 0.0, 1.0]))
        d2 = np.zeros((m, m, 3))
        d2[0, 0] = np.array([-r * c, -r * s, 0.0])
        return x, np.array(d1), d2
    if k == "cap":
        x = np.array([u[0], u[1], feat[1] * prm[1]])
        return x, np.array([[1.0, 0, 0], [0, 1.0, 0]]), np.zeros((2, 2, 3))
    fixed = feat[1]
    free = [i for i in range(3) if i not in fixed]
    x = np.zeros(3)
    for i, s in fixed.items():
        x[i] = s * prm[i]
    d1 = []
    for j, i in enumerate(free):
        x[i] = u[j]
        e = np.zeros(3)
        e[i] = 1
        d1.append(e)
    return x, np.array(d1).reshape(len(free), 3), np.zeros((len(free), len(free), 3))


def newton(TA, fA, prmA, uA, TB, fB, prmB, uB, iters=30):
    RA, RB = TA[:3, :3], TB[:3, :3]
    mA = len(uA)
    for it in range(iters):
        xA, dA, ddA = point(fA, prmA, uA)
        xB, dB, ddB = point(fB, prmB, uB)
        D = (RA @ xA + TA[:3, 3]) - (RB @ xB + TB[:3, 3])
        J = np.vstack([(RA @ dA.T).T, -(RB @ dB.T).T]) if (len(uA) + len(uB)) else np.zeros((0, 3))
        g = J @ D
        m = len(g)
        if m == 0:
            return uA, uB, True
        H = J @ J.T
        for i in range(mA):
            for j in range(mA):
                H[i, j] += D @ (RA @ ddA[i, j])
        for i in range(len(uB)):
            for j in range(len(uB)):
                H[mA + i, mA + j] -= D @ (RB @ ddB[i, j])
        try:
            if np.linalg.cond(H) > 1e12:
                return uA, uB, False
            step = -np.linalg.solve(H, g)
        except np.linalg.LinAlgError:
            return uA, uB, False
        uA = uA + step[:mA]
        uB = uB + step[mA:]
        if np.max(np.abs(step)) < 1e-15:
            break
    return uA, uB, True


def refine(om, q, pair, d, pA, pB, tau=1e-4):
    ga, gb = om.pair_a[pair], om.pair_b[pair]
    ta, tb = om.gtype[ga], om.gtype[gb]
    if ta == SPHERE or tb == SPHERE:
        return None
    TA, TB = shape_T(om, q, ga), shape_T(om, q, gb)
    prmA, prmB = list(om.gparam[ga][:]), list(om.gparam[gb][:])
    xA = TA[:3, :3].T @ (pA - TA[:3, 3])
    xB = TB[:3, :3].T @ (pB - TB[:3, 3])
    fA, fB = classify(ta, prmA, xA, tau), classify(tb, prmB, xB, tau)
    uA, uB, ok = newton(TA, fA, prmA, param0(fA, prmA, xA), TB, fB, prmB, param0(fB, prmB, xB))
    if not ok:
        return ("degenerate", fA, fB)
    XA = TA[:3, :3] @ point(fA, prmA, uA)[0] + TA[:3, 3]
    XB = TB[:3, :3] @ point(fB, prmB, uB)[0] + TB[:3, 3]
    L = np.linalg.norm(XB - XA)
    dn = L if d > 0 else -L
    return ("ok", fA, fB, XA, XB, dn)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--robot", default="ur5e")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--batch", type=int, default=512)
    a = ap.parse_args()
    from dyros_robot_controller_amd import workload
    pm, om, spec = O.load(a.robot)
    nv = om.nv
    lo, hi, v = (np.array(x[:nv]) for x in (om.lower, om.upper, om.vel))
    q, qd = workload.joint_states(lo, hi, v, a.seed, a.batch)

    def ev(qs):
        m = np.array([O.manipulability(om, qs[:, b])[0] for b in range(qs.shape[1])])
        dd = np.array([O.min_distance(om, qs[:, b])[0] for b in range(qs.shape[1])])
        return m, dd
    workload.apply_stress(q, lo, hi, list(range(nv)), a.seed, 0, ev)
    stats = {}
    for b in range(a.batch):
        d, _, pair = O.min_distance(om, q[:, b])
        d0, pA, pB = O.pair_distance(om, q[:, b], pair)
        r = refine(om, q[:, b], pair, d0, pA, pB)
        if r is None:
            continue
        key = (om.gtype[om.pair_a[pair]], om.gtype[om.pair_b[pair]], "pen" if d0 < 0 else "sep")
        st = stats.setdefault(key, {"n": 0, "deg": 0, "wit": [], "dd": [], "raw_pert": [], "ref_pert": [],
                                    "feat": {}})
        st["n"] += 1
        if r[0] != "ok":
            st["deg"] += 1
            continue
        _, fA, fB, XA, XB, dn = r
        fk = (fA[0], fB[0])
        st["feat"][fk] = st["feat"].get(fk, 0) + 1
        st["wit"].append(max(np.abs(XA - pA).max(), np.abs(XB - pB).max()))
        st["dd"].append(abs(dn - d0))
        # rounding-level perturbation of the configuration
        qp = q[:, b] + 1e-13 * np.sin(np.arange(nv) + 1.0)
        d1, pA1, pB1 = O.pair_distance(om, qp, pair)
        r1 = refine(om, qp, pair, d1, pA1, pB1)
        st["raw_pert"].append(max(np.abs(pA1 - pA).max(), np.abs(pB1 - pB).max()))
        if r1 and r1[0] == "ok":
            st["ref_pert"].append(max(np.abs(r1[3] - XA).max(), np.abs(r1[4] - XB).max()))
    for k, st in sorted(stats.items()):
        f = lambda xs: "%.2e/%.2e" % (np.median(xs), np.max(xs)) if xs else "-"
        print(k, "n", st["n"], "degenerate", st["deg"], "feat", st["feat"], "|raw-ref| med/max", f(st["wit"]),
              "|dd|", f(st["dd"]), "perturbed raw", f(st["raw_pert"]), "perturbed refined", f(st["ref_pert"]))


if __name__ == "__main__":
    main()

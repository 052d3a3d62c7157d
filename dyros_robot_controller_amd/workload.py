"""Synthetic control-cycle batches (SURVEY.md §8d "Synthetic inputs").

Counter-based ``splitmix64(seed, instance, field)`` so every instance is
reproducible on any host and independent of the batch size.  Targets are
built from the pose the *product kernel* computes (stage outputs), so the
generator needs no CPU kinematics.
"""
import numpy as np

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x):
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & M64
    z = x
    z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & M64
    z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & M64
    return z ^ (z >> np.uint64(31))


def uniform(seed, field, B, offset=0):
    """U[0,1) doubles for instances offset..offset+B-1 of one field."""
    with np.errstate(over="ignore"):
        inst = np.arange(offset, offset + B, dtype=np.uint64)
        key = _splitmix64(np.uint64(seed) * np.uint64(0x100000001B3) + np.uint64(field))
        x = _splitmix64(inst ^ key)
    return (x >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def normal(seed, field, B, offset=0):
    u1 = np.maximum(uniform(seed, 2 * field + 1000, B, offset), 1e-300)
    u2 = uniform(seed, 2 * field + 1001, B, offset)
    return np.sqrt(-2 * np.log(u1)) * np.cos(2 * np.pi * u2)


def joint_states(lower, upper, vel, seed, B, offset=0, margin=0.05):
    """q ~ U(q_min + margin, q_max - margin), qdot ~ U(-0.5, 0.5) * v_max ([n][B])."""
    n = len(lower)
    q = np.stack([lower[i] + margin + (upper[i] - lower[i] - 2 * margin) * uniform(seed, i, B, offset) for i in range(n)])
    qd = np.stack([(uniform(seed, 100 + i, B, offset) - 0.5) * vel[i] for i in range(n)])
    return q, qd


def mobile_states(lower, upper, vel, joint_index, n_arm, n_wheel, seed, B, offset=0):
    """Whole-body states: x,y ~ U(-5,5), yaw ~ U(-pi,pi), wheels ~ U(-pi,pi),
    arm within limits; qdot virtual U(-.5,.5), wheels U(-2,2), arm U(-.5,.5)v."""
    vs, ms, ws = joint_index
    n = len(lower)
    q = np.zeros((n, B))
    qd = np.zeros((n, B))
    q[vs] = -5 + 10 * uniform(seed, 0, B, offset)
    q[vs + 1] = -5 + 10 * uniform(seed, 1, B, offset)
    q[vs + 2] = np.pi * (2 * uniform(seed, 2, B, offset) - 1)
    for i in range(3):
        qd[vs + i] = uniform(seed, 200 + i, B, offset) - 0.5
    for w in range(n_wheel):
        q[ws + w] = np.pi * (2 * uniform(seed, 10 + w, B, offset) - 1)
        qd[ws + w] = 4 * uniform(seed, 210 + w, B, offset) - 2
    for i in range(n_arm):
        j = ms + i
        q[j] = lower[j] + 0.05 + (upper[j] - lower[j] - 0.1) * uniform(seed, 20 + i, B, offset)
        qd[j] = (uniform(seed, 220 + i, B, offset) - 0.5) * vel[j]
    return q, qd


# -- stress tiers (SURVEY.md §8d "Stress tiers, 10% each") ---------------------
# Instance b belongs to one tier, drawn from its own counter stream, so the tier
# of an instance does not depend on the batch size or on the shard it lands in.
TIER_NOMINAL, TIER_JOINT_LIMIT, TIER_SINGULAR, TIER_COLLISION = 0, 1, 2, 3
STRESS_MARGIN = 0.05      # tier 1: within 0.05 rad of a joint limit
STRESS_MAN = 0.03         # tier 2: manipulability below 0.03 (near-singular)
STRESS_DIST = 0.06        # tier 3: min self-distance below 0.06 m (CBF row live)


def tiers(seed, B, offset=0, frac=0.1):
    u = uniform(seed, 900, B, offset)
    t = np.zeros(B, np.int32)
    t[u < frac] = TIER_JOINT_LIMIT
    t[(u >= frac) & (u < 2 * frac)] = TIER_SINGULAR
    t[(u >= 2 * frac) & (u < 3 * frac)] = TIER_COLLISION
    return t


def _candidate_block(lower, upper, rows, seed, rnd, B, offset):
    """Round `rnd` of the rejection sampler: fresh in-limit joint values for
    the given rows (joint indices), from streams keyed by (seed, round, row)."""
    out = {}
    for k, j in enumerate(rows):
        u = uniform(seed, 4000 + 64 * rnd + k, B, offset)
        out[j] = lower[j] + STRESS_MARGIN + (upper[j] - lower[j] - 2 * STRESS_MARGIN) * u
    return out


def apply_stress(q, lower, upper, rows, seed, offset, evaluate, max_rounds=48):
    """Turns 30 % of a batch of states into the three stress tiers, in place.

    q: [nv][B] joint positions (full vectors); rows: the arm joint indices the
    tiers act on (manipulator: all joints; mobile manipulator: the arm block).
    evaluate(q_subset [nv][k]) -> (manipulability [k], min distance [k]) is the
    caller's stage evaluator (the device's stage kernel in bench.py; the oracle
    in CPU tests).  Tier 1 moves one arm joint to within STRESS_MARGIN of a limit
    (inside it).  Tiers 2/3 redraw the arm joints round by round until m <
    STRESS_MAN / d < STRESS_DIST; an instance that no round satisfies keeps its
    last draw (counted in the returned stats).  Returns (tier [B], stats)."""
    nv, B = q.shape
    tier = tiers(seed, B, offset)
    # tier 1: joint j = floor(u n), lower or upper side, depth U(0, margin)
    ua, ub, uc = (uniform(seed, 950 + i, B, offset) for i in range(3))
    jsel = np.minimum((ua * len(rows)).astype(int), len(rows) - 1)
    for b in np.nonzero(tier == TIER_JOINT_LIMIT)[0]:
        j = rows[jsel[b]]
        q[j, b] = lower[j] + STRESS_MARGIN * uc[b] if ub[b] < 0.5 else upper[j] - STRESS_MARGIN * uc[b]
    stats = {"joint_limit": int(np.sum(tier == TIER_JOINT_LIMIT))}
    for t, key in ((TIER_SINGULAR, "singular"), (TIER_COLLISION, "collision")):
        todo = np.nonzero(tier == t)[0]
        hit = 0
        for rnd in range(max_rounds):
            if todo.size == 0:
                break
            cand = _candidate_block(lower, upper, rows, seed + 7919 * t, rnd, B, offset)
            for j in rows:
                q[j, todo] = cand[j][todo]
            m, d = evaluate(np.ascontiguousarray(q[:, todo]))
            ok = (np.asarray(m) < STRESS_MAN) if t == TIER_SINGULAR else (np.asarray(d) < STRESS_DIST)
            hit += int(ok.sum())
            todo = todo[~ok]
        stats[key] = hit
        stats[key + "_unmet"] = int(todo.size)
    return tier, stats


def device_evaluator(model, link_name, device):
    """apply_stress evaluator backed by the product's stage kernel
    (drc_qpik_stages_batch): manipulability of ``link_name`` and min self-distance."""
    from . import _batch, _capi
    from .manipulator import QPIKParamsBuilder
    p = QPIKParamsBuilder(model, exact=True).params(link_name, _capi.MODE_QPIK)

    def evaluate(qs):
        k = qs.shape[1]
        z = _batch.as_device(np.zeros_like(qs), device)
        st = _batch.stages_batch(model, p, _batch.as_device(qs, device), z, None,
                                 _batch.as_device(np.zeros((6, k)), device))
        return st["man"][0].cpu().numpy(), st["dist"][0].cpu().numpy()
    return evaluate


def so3_exp_batch(w):
    """w [3][B] -> R [B][3][3]"""
    th = np.sqrt(np.sum(w * w, axis=0))
    B = w.shape[1]
    K = np.zeros((B, 3, 3))
    K[:, 0, 1], K[:, 0, 2] = -w[2], w[1]
    K[:, 1, 0], K[:, 1, 2] = w[2], -w[0]
    K[:, 2, 0], K[:, 2, 1] = -w[1], w[0]
    a = np.where(th > 1e-12, np.sin(th) / np.maximum(th, 1e-300), 1.0)
    b = np.where(th > 1e-12, (1 - np.cos(th)) / np.maximum(th, 1e-300) ** 2, 0.5)
    return np.eye(3)[None] + a[:, None, None] * K + b[:, None, None] * (K @ K)


def perturb_targets(pose12, seed, B, offset=0, sigma_p=0.02, sigma_r=0.05, sigma_v=0.05):
    """x_target = FK(q) (+) (N(0, sigma_p) m, exp(N(0, sigma_r) rad));
    xdot_target ~ N(0, sigma_v).  pose12: [12][B] (R col-major, p)."""
    R = pose12[:9].T.reshape(B, 3, 3).transpose(0, 2, 1)       # col-major -> [B][r][c]
    w = np.stack([sigma_r * normal(seed, 300 + i, B, offset) for i in range(3)])
    Rt = so3_exp_batch(w) @ R
    xt = np.zeros((12, B))
    xt[:9] = Rt.transpose(0, 2, 1).reshape(B, 9).T
    xt[9:] = pose12[9:] + np.stack([sigma_p * normal(seed, 310 + i, B, offset) for i in range(3)])
    xdt = np.stack([sigma_v * normal(seed, 320 + i, B, offset) for i in range(6)])
    return xt, xdt

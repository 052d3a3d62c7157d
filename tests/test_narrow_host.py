"""Device narrow-phase code (csrc/qpik_device.hpp: closed forms, GJK,
adjacency EPA) compiled for the host and checked against the oracle's
shape_distance on random shape pairs, about half of them penetrating.

Runs on the CPU: hipcc compiles the DRC_HD functions as plain host code."""
import os
import shutil
import subprocess

import numpy as np
import pytest

import oracle as O
import pyref as R

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    if not shutil.which(HIPCC) and not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    exe = str(tmp_path_factory.mktemp("nh") / "narrow_host")
    subprocess.check_call([HIPCC, "-O2", "-std=c++17", "--offload-arch=gfx950", "--cuda-host-only",
                           os.path.join(ROOT, "tools", "narrow_host_test.hip"), "-o", exe])
    return exe


def random_pairs(n, seed):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        ta, tb = rng.choice([0, 1, 2], size=2, p=[0.15, 0.5, 0.35])
        Ts = []
        for _k in range(2):
            T = np.zeros(12)
            T[:9] = R.so3_exp(rng.normal(size=3) * 2).reshape(9)
            T[9:] = rng.normal(size=3) * 0.08
            Ts.append(T)
        prm = []
        for t in (ta, tb):
            if t == 0:
                prm.append(np.array([rng.uniform(0.02, 0.08), 0, 0]))
            elif t == 1:
                prm.append(np.array([rng.uniform(0.03, 0.08), rng.uniform(0.02, 0.15), 0]))
            else:
                prm.append(rng.uniform(0.02, 0.1, size=3))
        out.append((int(ta), Ts[0], prm[0], int(tb), Ts[1], prm[1]))
    return out


def run_harness(exe, pairs):
    lines = []
    for ta, TA, pa, tb, TB, pb in pairs:
        lines.append(" ".join([str(ta)] + ["%.17g" % v for v in np.concatenate([TA, pa])] +
                              [str(tb)] + ["%.17g" % v for v in np.concatenate([TB, pb])]))
    res = subprocess.run([exe], input="\n".join(lines) + "\n", capture_output=True, text=True, check=True)
    return np.array([[float(x) for x in ln.split()] for ln in res.stdout.strip().splitlines()])


def oracle_dist(pairs, raw=True):
    """The oracle's narrow phase: raw GJK / EPA (raw=True) or with the witness
    refinement (D17)."""
    import ctypes as C
    out = []
    for ta, TA, pa, tb, TB, pb in pairs:
        d = C.c_double()
        how = C.c_int()
        pA, pB = np.zeros(3), np.zeros(3)
        if raw:
            O.lib().oracle_shape_distance_raw(ta, O._ptr(TA), O._ptr(pa), tb, O._ptr(TB), O._ptr(pb),
                                              C.byref(d), O._ptr(pA), O._ptr(pB), C.byref(how))
        else:
            O.lib().oracle_shape_distance(ta, O._ptr(TA), O._ptr(pa), tb, O._ptr(TB), O._ptr(pb),
                                          C.byref(d), O._ptr(pA), O._ptr(pB))
        out.append(np.concatenate([[d.value], pA, pB]))
    return np.array(out)


def test_device_narrow_phase_matches_oracle(harness):
    pairs = random_pairs(4000, 7)
    dev = run_harness(harness, pairs)
    ref = oracle_dist(pairs)
    pen = ref[:, 0] < 0
    assert 0.2 < pen.mean() < 0.8  # both GJK and EPA exercised
    err = np.abs(dev[:, 0] - ref[:, 0])
    # raw estimates (before the D17 refinement, test below): separated, GJK
    # stops at a 1e-6 support gap on both sides (hpp-fcl's gjk_tolerance), so
    # a rounding difference that moves the stop by one iteration shows up to
    # that gap; penetrating, identical EPA decisions agree to 1e-9 unless
    # rounding changes a step, and both sides stop within the EPA tolerance
    # (1e-6, hpp-fcl's default) of the depth
    assert err[~pen].max() <= 2e-6, err[~pen].max()
    assert np.mean(err[~pen] <= 1e-9) >= 0.97
    assert err[pen].max() <= 2e-6, err[pen].max()
    assert np.mean(err[pen] <= 1e-9) >= 0.97
    # raw witnesses: flat-flat contacts admit a face of witnesses, so compare
    # the separation vector pB - pA (unique).  GJK's 1e-6 gap leaves the
    # direction accurate to ~sqrt(gap * d); EPA's 1e-6 gap likewise -- the
    # footprint the D17 refinement removes (test_witness_refinement_matches_oracle)
    sep = dev[:, 4:7] - dev[:, 1:4]
    sep_ref = ref[:, 4:7] - ref[:, 1:4]
    serr = np.abs(sep - sep_ref).max(axis=1)
    # per pair: two GJK stops within the gap eps = 1e-6 of the distance d
    # leave the separation vector (length d) within ~d * sqrt(2 eps / d) =
    # sqrt(2 eps d) of the exact one on each side; the bound takes twice
    # that sum (derived, not fitted: the largest observed ratio is below 1)
    dsep = np.abs(ref[~pen, 0])
    bound = 2 * 2 * np.sqrt(2e-6 * np.maximum(dsep, 1e-12)) + 1e-9
    assert np.all(serr[~pen] <= bound), np.max(serr[~pen] / bound)
    assert np.median(serr[~pen]) <= 1e-12
    assert serr[pen].max() <= 1e-3, serr[pen].max()
    assert np.quantile(serr[pen], 0.9) <= 1e-7


def test_broad_phase_bound_and_gjk_cut(harness):
    """pair_lower_bound (swept core raised to the separating-axis value) never
    exceeds the signed distance, separated or penetrating, and is usually
    much tighter than the core bound; GJK's early exit, asked to stop once the
    pair is known to be farther than a cut just above its distance, never
    fires (its lower bound v.w/|v| never passes the true distance), so a
    pair that can still win is always computed in full."""
    pairs = [p for p in random_pairs(4000, 11) if p[0] != 0 and p[3] != 0]
    dev = run_harness(harness, pairs)
    d, lb, pruned = dev[:, 0], dev[:, 7], dev[:, 8]
    assert np.all(lb <= d + 1e-12), (lb - d).max()
    assert np.mean(d - lb < 0.25 * np.abs(d) + 1e-3) > 0.3  # informative, not just -inf
    assert not pruned.any(), np.nonzero(pruned)


def test_witness_refinement_matches_oracle(harness):
    """D17: the device refine_witness and the oracle's land on the same
    critical point from their own GJK / EPA estimates -- distance and
    separation vector to rounding, where the raw estimates differ by up to
    ~1e-5 -- and they accept / reject the same pairs."""
    pairs = random_pairs(4000, 17)
    dev = run_harness(harness, pairs)
    ref = oracle_dist(pairs, raw=False)
    raw = oracle_dist(pairs, raw=True)
    acc_dev = dev[:, 16] == 1
    acc_ref = np.any(ref[:, 1:] != raw[:, 1:], axis=1) | (ref[:, 0] != raw[:, 0])
    assert acc_dev.sum() > 1000
    # the oracle may return a refined point bit-identical to its estimate (box vertices)
    assert np.all(acc_ref <= acc_dev)
    d_err = np.abs(dev[acc_dev, 9] - ref[acc_dev, 0])
    assert d_err.max() <= 1e-12, d_err.max()
    sep = dev[acc_dev, 13:16] - dev[acc_dev, 10:13]
    sep_ref = ref[acc_dev, 4:7] - ref[acc_dev, 1:4]
    assert np.abs(sep - sep_ref).max() <= 1e-12, np.abs(sep - sep_ref).max()
    w_err = np.maximum(np.abs(dev[acc_dev, 10:13] - ref[acc_dev, 1:4]).max(1),
                       np.abs(dev[acc_dev, 13:16] - ref[acc_dev, 4:7]).max(1))
    assert np.quantile(w_err, 0.99) <= 1e-12, np.quantile(w_err, 0.99)
    # rejected on the device -> the oracle kept its estimate as well
    rej = ~acc_dev & (dev[:, 0] == dev[:, 9])
    assert np.all(~acc_ref[rej])

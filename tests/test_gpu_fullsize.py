"""Every BASELINE.json configuration's own bench path at its own batch size
(bench.py's workload: SURVEY §8d with the three stress tiers, seed 12345), so
the code the bench times -- four concurrent sub-batches, the XCD-aware
instance order for sub-batches of >= 16 Ki, the compile-time QP shapes
Dims<23,16,7> / <20,14,6> / <9,16,9> / <11,16,11>, the fused kernel at
B <= 16 384 (FR3 B = 4 096 and Husky-FR3's bench batch) -- is the code the
oracle checks:

  config                                   robot        B        offset
  FR3 QPIKStep (the metric)                fr3          65 536   0
  FR3 batch 4 096 (config 2, fused kernel) fr3           4 096   0
  UR5e (config 3)                          ur5e         65 536   0
  Husky-FR3 whole body (config 4)          husky_fr3    16 384   0
  XLS-FR3 8-GPU shard (config 5), rank 3   xls_fr3      65 536   3 x 65 536
  XLS-FR3 --global-batch 65536 on 1 GPU    xls_fr3      65 536   0
  Caster-FR3                               caster_fr3   65 536   0

Properties checked on every instance:
  * sub-batch invariance: the call split into 1, 3 or 4 (the default) concurrent
    sub-batches (drc_set_concurrency) returns bit-identical q-dot, status and
    iterations;
    at B = 4 096 and Husky-FR3's 16 384 the fused kernel against the
    two-kernel pipeline (drc_set_fusion), bit for bit;
  * feasibility: every output finite; non-solved instances exactly zero
    (QP_IK.cpp:56-61); manipulators: |q-dot| <= the velocity limit (the QP's
    bound rows, QP_IK.cpp:89-97) within 1e-6; whole-body QPs (no bounds, no
    slacks, mobile_manipulator/QP_IK.cpp:75-128): the arm's joint-limit CBF
    rows -alpha (q - q_min) <= q-dot_arm <= alpha (q_max - q) within 1e-6 on
    every solved instance, and statuses only Solved / PrimalInfeasible;
and on a spread sample of ~1 000 instances that includes every sub-batch
boundary, the parity contract of test_gpu_parity.py against the oracle
(assert_qpik_parity).
"""
import ctypes as C

import numpy as np
import pytest

from _common import (LINK, assert_qpik_parity, make_manipulator, make_moma, moma_step_inputs, step_inputs)
from dyros_robot_controller_amd import _capi, manipulator, mobile_manipulator

pytestmark = pytest.mark.gpu

SEED = 12345  # bench.py's workload seed
EXPECTED_OFF = 0  # end-to-end instances beyond 1e-4 on the sample
ALPHA = 50.0  # QP_IK.cpp:101 (MoMa :87)
CONFIGS = [("fr3", 65536, 0), ("fr3", 4096, 0), ("ur5e", 65536, 0), ("husky_fr3", 16384, 0),
           ("xls_fr3", 65536, 3 * 65536), ("xls_fr3", 65536, 0), ("caster_fr3", 65536, 0)]
IDS = ["%s-B%d-off%d" % c for c in CONFIGS]
_cache = {}


def _run(cfg, cuda):
    if cfg in _cache:
        return _cache[cfg]
    _cache.clear()   # one configuration's device buffers at a time
    import torch
    robot, B, offset = cfg
    moma = robot in ("husky_fr3", "xls_fr3", "caster_fr3")
    rd = make_moma(robot, cuda) if moma else make_manipulator(robot, cuda)
    ctrl = (mobile_manipulator if moma else manipulator).RobotController(0.001, rd, solver_mode="exact")
    q, qd, xt, xdt = (moma_step_inputs if moma else step_inputs)(rd, robot, SEED, B, cuda, offset=offset, stress=True)
    args = [torch.as_tensor(a, device=cuda) for a in (q, qd, xt, xdt)]
    h = rd.model.handle
    runs = {}
    # (label, concurrency, fusion): the bench's default call last
    variants = [("one", 1, 1), ("three", 3, 1), ("four", 4, 1)] if B > 16384 else [("pipeline", 4, 0), ("fused", 4, 1)]
    for label, chunks, fused in variants:
        _capi.check(_capi.lib().drc_set_concurrency(h, chunks))
        _capi.check(_capi.lib().drc_set_fusion(h, C.c_int(fused)))
        iters = torch.zeros(B, dtype=torch.int32, device=cuda)
        out, status = ctrl.QPIK_step_batch(*args, LINK[robot], iters=iters)
        torch.cuda.synchronize()
        runs[label] = (out.cpu().numpy(), status.cpu().numpy(), iters.cpu().numpy())
    _capi.check(_capi.lib().drc_set_concurrency(h, 4))
    _capi.check(_capi.lib().drc_set_fusion(h, C.c_int(1)))
    res = (rd, moma, (q, qd, xt, xdt), runs, variants[-1][0])
    _cache[cfg] = res
    return res


@pytest.mark.parametrize("cfg", CONFIGS, ids=IDS)
def test_fullsize_invariance(cuda, cfg):
    _, _, _, runs, _ = _run(cfg, cuda)
    a, *rest = list(runs.values())
    for b in rest:
        for x, y in zip(a, b):
            assert np.array_equal(x, y), np.count_nonzero(np.any(np.atleast_2d(x != y), axis=0))


@pytest.mark.parametrize("cfg", CONFIGS, ids=IDS)
def test_fullsize_feasible(cuda, cfg):
    rd, moma, (q, qd, xt, xdt), runs, default = _run(cfg, cuda)
    out, status, iters = runs[default]
    assert np.all(np.isfinite(out))
    solved = status == _capi.STATUS_SOLVED
    assert np.all(out[:, ~solved] == 0.0)
    assert iters[solved].max() <= 4000
    if not moma:
        _, vmax = rd.getJointVelocityLimit()
        assert solved.mean() >= 0.99
        viol = np.abs(out[:, solved]) - np.asarray(vmax)[:, None]
        assert viol.max() <= 1e-6, viol.max()
        return
    assert set(np.unique(status)) <= {_capi.STATUS_SOLVED, _capi.STATUS_PRIMAL_INFEASIBLE}
    assert solved.mean() >= 0.97
    ji, ai = rd.get_joint_index(), rd.get_actuator_index()
    n = rd.get_manipulator_dof()
    lo, hi = rd.get_joint_position_limit()
    qa = q[ji.mani_start:ji.mani_start + n]
    lo_a, hi_a = np.asarray(lo)[ji.mani_start:ji.mani_start + n, None], np.asarray(hi)[ji.mani_start:ji.mani_start + n, None]
    va = out[ai.mani_start:ai.mani_start + n]
    lower = -ALPHA * (qa - lo_a)
    upper = ALPHA * (hi_a - qa)
    viol = np.maximum(lower - va, va - upper)[:, solved]
    assert viol.max() <= 1e-6, viol.max()


@pytest.mark.parametrize("cfg", CONFIGS, ids=IDS)
def test_fullsize_sample_matches_oracle(cuda, cfg):
    rd, moma, (q, qd, xt, xdt), runs, default = _run(cfg, cuda)
    out, status, _ = runs[default]
    B = q.shape[1]
    # every sub-batch boundary of the 3- and 4-way splits (api.cpp: [B c / S, B (c + 1) / S))
    cuts = sorted({B * c // S for S in (3, 4) for c in range(1, S)})
    edges = [0, 1, B - 2, B - 1] + [e for c in cuts for e in (c - 1, c)]
    idx = np.unique(np.concatenate([np.linspace(0, B - 1, 1000).astype(int), edges]))
    sub = lambda a: np.ascontiguousarray(a[:, idx])
    assert_qpik_parity(cfg[0], rd.model, sub(q), sub(qd), sub(xt), sub(xdt), sub(out), status[idx], EXPECTED_OFF)

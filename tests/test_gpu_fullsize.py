"""Full-size checks at BASELINE.json's configuration (FR3 QPIKStep, 65 536
instances per GPU, the bench workload's seed), through properties that do not
need the oracle on every instance:

  * sub-batch invariance: the call split into 1 or 3 concurrent sub-batches
    (drc_set_concurrency) returns bit-identical q-dot, status and iterations
    (instances are independent; the split only changes placement);
  * feasibility on every instance: |q-dot| <= the velocity limit (the QP's
    bound rows) within 1e-6 rad/s: polished instances hold them to rounding,
    the few ADMM-fallback instances (eps_fallback 1e-7, scaled) to ~1e-8
    (measured max 9.9e-9);
  * parity on a spread sample (sub-batch boundaries included) against the
    oracle, under the contract of test_gpu_parity.py (assert_qpik_parity).
The workload is the bench's: SURVEY §8d's stress tiers included.
"""
import numpy as np
import pytest

from _common import LINK, assert_qpik_parity, make_manipulator, step_inputs
from dyros_robot_controller_amd import _capi, manipulator

pytestmark = pytest.mark.gpu

B = 65536
SEED = 12345  # bench.py's workload seed
EXPECTED_OFF = 0  # measured end-to-end count beyond 1e-4 on the sample


@pytest.fixture(scope="module")
def fullsize(cuda):
    import torch
    rd = make_manipulator("fr3", cuda)
    ctrl = manipulator.RobotController(0.001, rd, solver_mode="exact")
    q, qd, xt, xdt = step_inputs(rd, "fr3", SEED, B, cuda, stress=True)
    args = [torch.as_tensor(a, device=cuda) for a in (q, qd, xt, xdt)]
    runs = {}
    for chunks in (1, 3):
        _capi.check(_capi.lib().drc_set_concurrency(rd.model.handle, chunks))
        iters = torch.zeros(B, dtype=torch.int32, device=cuda)
        out, status = ctrl.QPIK_step_batch(*args, LINK["fr3"], iters=iters)
        runs[chunks] = (out.cpu().numpy(), status.cpu().numpy(), iters.cpu().numpy())
    _capi.check(_capi.lib().drc_set_concurrency(rd.model.handle, 3))
    return rd, (q, qd, xt, xdt), runs


def test_fullsize_subbatch_invariance(fullsize):
    _, _, runs = fullsize
    for a, b in zip(runs[1], runs[3]):
        assert np.array_equal(a, b)


def test_fullsize_feasible(fullsize):
    rd, _, runs = fullsize
    out, status, iters = runs[3]
    _, vmax = rd.getJointVelocityLimit()
    solved = status == _capi.STATUS_SOLVED
    assert solved.mean() >= 0.99
    viol = np.abs(out[:, solved]) - np.asarray(vmax)[:, None]
    print("max bound violation %.3g, instances above 1e-9: %d" % (viol.max(), int(np.sum(viol.max(axis=0) > 1e-9))))
    assert viol.max() <= 1e-6
    assert np.all(np.isfinite(out))
    assert iters[solved].max() <= 4000


def test_fullsize_sample_matches_oracle(fullsize):
    _, (q, qd, xt, xdt), runs = fullsize
    out, status, _ = runs[3]
    third = B // 3
    idx = np.unique(np.concatenate([np.linspace(0, B - 1, 1024).astype(int),
                                    [third - 1, third, 2 * third - 1, 2 * third, B - 2, B - 1]]))
    sub = lambda a: np.ascontiguousarray(a[:, idx])
    rd = fullsize[0]
    assert_qpik_parity("fr3", rd.model, sub(q), sub(qd), sub(xt), sub(xdt), sub(out), status[idx], EXPECTED_OFF)

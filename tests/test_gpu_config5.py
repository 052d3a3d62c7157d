"""BASELINE config 5 end to end on the one GPU: XLS-FR3 whole-body QPIKStep,
global batch 524 288 split over 8 ranks (dist.shard_global: rank r owns
instances [r x 65 536, (r + 1) x 65 536)), bench.py's workload (seed 12345,
the three stress tiers).  The 8-GPU run itself is the driver's; here every
one of the eight shards goes through the HIP path as that rank would run it
(its own inputs generated at its own offset), and then the whole global batch
in ONE call (world size 1, strong scaling), so that:

  * every shard passes the feasibility checks of test_gpu_fullsize.py on all
    of its 65 536 instances, and the parity contract (assert_qpik_parity) on a
    sample of each shard that includes its first and last instances;
  * the per-rank inputs equal the matching slice of the global batch (the
    workload is counter based: an instance does not depend on its shard);
  * the one-call global solve returns, bit for bit, the concatenation of the
    eight shard solves (q-dot*, status, ADMM iterations), so the whole-job
    statistics bench.py reduces from the ranks (bench.whole_job: sums of
    non-solved instances and tier counts, max of iteration p99 / max) are
    those of the global batch.

Reference path: src/mobile_manipulator/QP_IK.cpp:43-128 (the whole-body QP).
"""
import numpy as np
import pytest

from _common import LINK, assert_qpik_parity, make_moma, moma_step_inputs
from dyros_robot_controller_amd import _capi, mobile_manipulator

pytestmark = pytest.mark.gpu

ROBOT, GLOBAL, RANKS, SEED = "xls_fr3", 524288, 8, 12345
ALPHA = 50.0          # mobile_manipulator/QP_IK.cpp:87
SAMPLE = 192          # oracle instances per shard


def _solve(ctrl, args, cuda):
    import torch
    B = args[0].shape[1]
    iters = torch.zeros(B, dtype=torch.int32, device=cuda)
    out, status = ctrl.QPIK_step_batch(*[torch.as_tensor(a, device=cuda) for a in args], LINK[ROBOT], iters=iters)
    torch.cuda.synchronize()
    return out.cpu().numpy(), status.cpu().numpy(), iters.cpu().numpy()


def _feasible(rd, q, out, status, iters):
    assert np.all(np.isfinite(out))
    solved = status == _capi.STATUS_SOLVED
    assert np.all(out[:, ~solved] == 0.0)                       # QP_IK.cpp:43-57: zeros on failure
    assert set(np.unique(status)) <= {_capi.STATUS_SOLVED, _capi.STATUS_PRIMAL_INFEASIBLE}
    assert solved.mean() >= 0.97
    assert iters[solved].max() <= 4000
    ji, ai = rd.get_joint_index(), rd.get_actuator_index()
    n = rd.get_manipulator_dof()
    lo, hi = rd.get_joint_position_limit()
    qa = q[ji.mani_start:ji.mani_start + n]
    lo_a = np.asarray(lo)[ji.mani_start:ji.mani_start + n, None]
    hi_a = np.asarray(hi)[ji.mani_start:ji.mani_start + n, None]
    va = out[ai.mani_start:ai.mani_start + n]
    viol = np.maximum(-ALPHA * (qa - lo_a) - va, va - ALPHA * (hi_a - qa))[:, solved]
    assert viol.max() <= 1e-6, viol.max()


def _rank_row(r, status, iters):
    """bench.py's per-rank row layout (rank, device, bus, wall, iters p99, iters max, non-solved, instances)."""
    it = iters.astype(np.float64)
    return [r, 0, 0, 0.0, float(np.percentile(it, 99)), int(it.max()), int((status != 1).sum()), len(status)]


def test_config5_all_shards_and_global_call(cuda):
    import bench
    rd = make_moma(ROBOT, cuda)
    ctrl = mobile_manipulator.RobotController(0.001, rd, solver_mode="exact")
    Bs = GLOBAL // RANKS
    shards_in, shards_out, rows = [], [], []
    for r in range(RANKS):
        args = moma_step_inputs(rd, ROBOT, SEED, Bs, cuda, offset=r * Bs, stress=True)
        out, status, iters = _solve(ctrl, args, cuda)
        _feasible(rd, args[0], out, status, iters)
        idx = np.unique(np.concatenate([np.linspace(0, Bs - 1, SAMPLE).astype(int), [0, 1, Bs - 2, Bs - 1]]))
        sub = lambda a: np.ascontiguousarray(a[:, idx])
        assert_qpik_parity(ROBOT, rd.model, *[sub(a) for a in args], sub(out), status[idx], 0)
        shards_in.append(args)
        shards_out.append((out, status, iters))
        rows.append(_rank_row(r, status, iters))
    # the global batch in one call: the shard inputs are its slices
    g_in = moma_step_inputs(rd, ROBOT, SEED, GLOBAL, cuda, offset=0, stress=True)
    for f in range(4):
        np.testing.assert_array_equal(g_in[f], np.concatenate([s[f] for s in shards_in], axis=1))
    out, status, iters = _solve(ctrl, g_in, cuda)
    np.testing.assert_array_equal(out, np.concatenate([s[0] for s in shards_out], axis=1))
    np.testing.assert_array_equal(status, np.concatenate([s[1] for s in shards_out]))
    np.testing.assert_array_equal(iters, np.concatenate([s[2] for s in shards_out]))
    # whole-job statistics: the ranks' reduction equals the global batch's own
    whole = bench.whole_job(np.array(rows, dtype=np.float64), [], "none")
    assert whole["admm_iters_p99_max"][1] == int(iters.max())
    assert sum(r[6] for r in rows) == int((status != 1).sum())
    assert sum(r[7] for r in rows) == GLOBAL

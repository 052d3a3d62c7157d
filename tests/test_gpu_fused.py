"""The fused task + QP kernel (fused_kernel.hip, the default for the compiled
QP shapes and B <= 16 384) against the two-kernel pipeline
(drc_set_fusion(model, 0)): the same device functions on the same
task-record values, built with -ffp-contract=on (build.sh) so that every
multiply-add rounds the same in both kernels.  The contract is bit-identical
q-dot*, status and ADMM iteration counts -- for QPIK, QPIKStep and QPIKCubic,
stress-tier inputs, several batch sizes (one wave, partial and full grids).
An instance's result therefore depends neither on the batch size nor on the
fusion threshold (tests/test_gpu_dist.py crosses it)."""
import ctypes as C

import numpy as np
import pytest

from _common import LINK, make_moma, moma_step_inputs, step_inputs, make_manipulator
from dyros_robot_controller_amd import _capi, manipulator, mobile_manipulator

pytestmark = pytest.mark.gpu


def _run(ctrl, rd, fused, mode, q, qd, xt, xdt, robot):
    import torch
    _capi.check(_capi.lib().drc_set_fusion(rd.model.handle, C.c_int(fused)))
    B = q.shape[1]
    it = torch.zeros(B, dtype=torch.int32, device=torch.device("cuda", 0))
    if mode == "step":
        out, st = ctrl.QPIK_step_batch(q, qd, xt, xdt, LINK[robot], iters=it)
    elif mode == "qpik":
        out, st = ctrl.QPIK_batch(q, qd, xdt, LINK[robot])
    else:
        xi = xt.copy()
        xi[9:] -= 0.01
        out, st = ctrl.QPIK_cubic_batch(q, qd, xt, xdt, xi, np.zeros_like(xdt), 0.4, 0.0, 1.0, LINK[robot])
    torch.cuda.synchronize()
    return out.cpu().numpy(), st.cpu().numpy(), it.cpu().numpy()


@pytest.mark.parametrize("robot", ["fr3", "ur5e", "husky_fr3", "xls_fr3"])
@pytest.mark.parametrize("B", [1, 300, 5000])
def test_fused_matches_two_kernel_pipeline(cuda, robot, B):
    moma = robot in ("husky_fr3", "xls_fr3")
    rd = make_moma(robot, cuda) if moma else make_manipulator(robot, cuda)
    ctrl = (mobile_manipulator if moma else manipulator).RobotController(0.001, rd, solver_mode="exact")
    q, qd, xt, xdt = (moma_step_inputs if moma else step_inputs)(rd, robot, 77, B, cuda, stress=True)
    for mode in ("step", "qpik", "cubic") if B == 300 else ("step",):
        (o1, s1, i1), (o0, s0, i0) = (_run(ctrl, rd, f, mode, q, qd, xt, xdt, robot) for f in (1, 0))
        np.testing.assert_array_equal(s1, s0)
        np.testing.assert_array_equal(o1, o0)
        np.testing.assert_array_equal(i1, i0)
    _capi.check(_capi.lib().drc_set_fusion(rd.model.handle, C.c_int(1)))

"""Scheduling order of small calls (order_kernel.hip): the penetration-prone
instances are handed out first.  Instances are independent, so the order may
move only when each instance starts, never what it returns: the automatic
order (calls of up to DRC_ORDER_MAX instances), the identity order and a
reversed order (drc_debug_instance_order, which replaces the automatic one)
give bit-identical q-dot*, statuses and ADMM iteration counts -- fused
(B <= 16 384) and two-kernel pipeline (several sub-batches, each ordered
within its own range)."""
import ctypes as C

import numpy as np
import pytest

from _common import LINK, make_manipulator, make_moma, moma_step_inputs, step_inputs
from dyros_robot_controller_amd import _capi, manipulator, mobile_manipulator

pytestmark = pytest.mark.gpu


def _solve(ctrl, robot, args, cuda):
    import torch
    B = args[0].shape[1]
    it = torch.zeros(B, dtype=torch.int32, device=cuda)
    out, st = ctrl.QPIK_step_batch(*args, LINK[robot], iters=it)
    torch.cuda.synchronize()
    return out.cpu().numpy(), st.cpu().numpy(), it.cpu().numpy()


def _set_order(rd, order):
    lib = _capi.lib()
    if order is None:
        _capi.check(lib.drc_debug_instance_order(rd.model.handle, None, C.c_int64(0)))
    else:
        o = np.ascontiguousarray(order, np.int32)
        _capi.check(lib.drc_debug_instance_order(rd.model.handle, o.ctypes.data_as(C.POINTER(C.c_int32)),
                                                 C.c_int64(len(o))))


# fused: fr3 4 096, ur5e 3 000, fr3 12 000 and husky_fr3 16 384 (its ranges of
# three are still a permutation of the one fused range); fr3 20 000: the
# pipeline's three sub-batches, each ordered within its own range
@pytest.mark.parametrize("robot,B,subs", [("fr3", 4096, 1), ("ur5e", 3000, 1), ("fr3", 12000, 1),
                                          ("husky_fr3", 16384, 3), ("fr3", 20000, 3)])
def test_order_does_not_change_results(cuda, robot, B, subs):
    moma = robot in ("husky_fr3", "xls_fr3", "caster_fr3")
    rd = make_moma(robot, cuda) if moma else make_manipulator(robot, cuda)
    ctrl = (mobile_manipulator if moma else manipulator).RobotController(0.001, rd, solver_mode="exact")
    args = (moma_step_inputs if moma else step_inputs)(rd, robot, 31, B, cuda, stress=True)
    auto = _solve(ctrl, robot, args, cuda)
    cuts = [B * c // subs for c in range(subs + 1)]
    ident = np.arange(B)
    rev = np.concatenate([np.arange(cuts[c + 1] - 1, cuts[c] - 1, -1) for c in range(subs)])
    try:
        for order in (ident, rev):
            _set_order(rd, order)
            got = _solve(ctrl, robot, args, cuda)
            for a, b in zip(auto, got):
                np.testing.assert_array_equal(a, b)
    finally:
        _set_order(rd, None)


def test_order_rejects_non_permutation(cuda):
    rd = make_manipulator("fr3", cuda)
    lib = _capi.lib()
    o = np.array([0, 1, 1, 3], np.int32)
    rc = lib.drc_debug_instance_order(rd.model.handle, o.ctypes.data_as(C.POINTER(C.c_int32)), C.c_int64(4))
    assert rc == _capi.DRC_ERR_INVALID_ARGUMENT

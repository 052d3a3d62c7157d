"""Fused kernel vs two-kernel pipeline, bit for bit (dev tool): for each
robot, batch size and mode, the number of instances whose q-dot*, status or
ADMM iteration count differ between drc_set_fusion(1) and (0).  Run with
DRC_AMD_LIB to compare library builds (e.g. -ffp-contract variants).
    python tools/fused_bits.py [robot ...]"""
import ctypes as C
import sys

sys.path.insert(0, "tests"); sys.path.insert(0, "oracle"); sys.path.insert(0, ".")
import numpy as np
import torch

from _common import LINK, make_manipulator, make_moma, moma_step_inputs, step_inputs
from dyros_robot_controller_amd import _capi, manipulator, mobile_manipulator

dev = torch.device("cuda", 0)
robots = sys.argv[1:] or ["fr3", "ur5e", "husky_fr3", "xls_fr3"]
for robot in robots:
    moma = robot in ("husky_fr3", "xls_fr3", "caster_fr3")
    rd = make_moma(robot, dev) if moma else make_manipulator(robot, dev)
    ctrl = (mobile_manipulator if moma else manipulator).RobotController(0.001, rd, solver_mode="exact")
    for B in (300, 5000):
        q, qd, xt, xdt = (moma_step_inputs if moma else step_inputs)(rd, robot, 77, B, dev, stress=True)
        for mode in ("step", "qpik", "cubic"):
            res = []
            for fused in (1, 0):
                _capi.check(_capi.lib().drc_set_fusion(rd.model.handle, C.c_int(fused)))
                it = torch.zeros(B, dtype=torch.int32, device=dev)
                if mode == "step":
                    out, st = ctrl.QPIK_step_batch(q, qd, xt, xdt, LINK[robot], iters=it)
                elif mode == "qpik":
                    out, st = ctrl.QPIK_batch(q, qd, xdt, LINK[robot])
                else:
                    xi = xt.copy()
                    xi[9:] -= 0.01
                    out, st = ctrl.QPIK_cubic_batch(q, qd, xt, xdt, xi, np.zeros_like(xdt), 0.4, 0.0, 1.0,
                                                    LINK[robot])
                torch.cuda.synchronize()
                res.append((out.cpu().numpy(), st.cpu().numpy(), it.cpu().numpy()))
            (o1, s1, i1), (o0, s0, i0) = res
            diff = np.any(o1 != o0, axis=0) | (s1 != s0) | (i1 != i0)
            print(robot, B, mode, "instances differing: %d / %d, max |dq| %.3g, iters differ %d" % (
                int(diff.sum()), B, float(np.abs(o1 - o0).max()), int((i1 != i0).sum())), flush=True)
    _capi.check(_capi.lib().drc_set_fusion(rd.model.handle, C.c_int(1)))

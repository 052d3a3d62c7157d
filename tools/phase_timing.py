"""Diagnostic: per-phase cycle shares from the DRC_PHASE_TIMING build."""
import os, sys, ctypes as C
os.environ["DRC_AMD_LIB"] = "libdrc_amd_timing.so"
sys.path.insert(0, "tests"); sys.path.insert(0, "oracle"); sys.path.insert(0, ".")
import numpy as np, torch
from _common import make_manipulator, step_inputs
from dyros_robot_controller_amd import manipulator, _capi
dev = torch.device("cuda", 0)
robot = sys.argv[1] if len(sys.argv) > 1 else "fr3"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
rd = make_manipulator(robot, dev)
q, qd, xt, xdt = step_inputs(rd, robot, 7, B, dev)
ctrl = manipulator.RobotController(0.001, rd)
link = "fr3_link8" if robot == "fr3" else "tool0"
args = [torch.as_tensor(a, device=dev) for a in (q, qd, xt, xdt)]
ctrl.QPIK_step_batch(*args, link); torch.cuda.synchronize()
buf = (C.c_ulonglong * 32)()
_capi.lib().drc_debug_phase_cycles(buf, 1)
ctrl.QPIK_step_batch(*args, link); torch.cuda.synchronize()
_capi.lib().drc_debug_phase_cycles(buf, 0)
v = np.array(buf[:], dtype=np.float64)
names_t = ["fk+geoms", "J+taskvel", "manip", "broad+sphere", "gjk cand", "epa", "argmin+witness", "grad"]
names_q = ["load+assemble", "scaling", "-", "rho+factor+admm+checks", "-", "output"]
tt, tq = v[:8], v[16:22]
print("task kernel cycles/instance: %.0f" % (tt.sum() / B))
for n, x in zip(names_t, tt): print("  %-16s %6.1f%%  %8.0f cyc/inst" % (n, 100 * x / tt.sum(), x / B))
print("qp kernel cycles/instance: %.0f" % (tq.sum() / B))
for n, x in zip(names_q, tq): print("  %-16s %6.1f%%  %8.0f cyc/inst" % (n, 100 * x / tq.sum(), x / B))

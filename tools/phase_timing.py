"""Diagnostic: per-phase cycle shares from the DRC_PHASE_TIMING build."""
import os, sys, ctypes as C
os.environ["DRC_AMD_LIB"] = os.environ.get("DRC_TIMING_LIB", "libdrc_amd_timing.so")
SOLVER = os.environ.get("DRC_SOLVER", "exact")   # osqp_default: the reference-settings mode
sys.path.insert(0, "tests"); sys.path.insert(0, "oracle"); sys.path.insert(0, ".")
import numpy as np, torch
import bench
from dyros_robot_controller_amd import BUNDLED, make_robot, manipulator, mobile_manipulator, _capi
dev = torch.device("cuda", 0)
robot = sys.argv[1] if len(sys.argv) > 1 else "fr3"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
spec = BUNDLED[robot]
rd = make_robot(robot, dev)
mod = manipulator if spec["kind"] == "manipulator" else mobile_manipulator
ctrl = mod.RobotController(0.001, rd, solver_mode=SOLVER)
_, args, _ = bench.make_inputs(rd, robot, B, 12345, 0, dev)   # bench.py's workload (stress tiers)
_capi.lib().drc_set_concurrency(rd.model.handle, 1)  # one sub-batch: per-instance cycles without overlap
link = spec["link"]
ctrl.QPIK_step_batch(*args, link); torch.cuda.synchronize()
buf = (C.c_ulonglong * 64)()
_capi.lib().drc_debug_phase_cycles(buf, 1)
ctrl.QPIK_step_batch(*args, link); torch.cuda.synchronize()
_capi.lib().drc_debug_phase_cycles(buf, 0)
v = np.array(buf[:], dtype=np.float64)
names_t = ["fk+geoms", "J+taskvel", "manip", "broad+sphere", "gjk cand", "epa", "argmin+witness", "grad"]
names_q = ["load+assemble", "scaling", "-", "rho+factor+admm+checks", "-", "output"]
tt, tq = v[:8], v[16:22]
ta = v[24:28]
print("task kernel cycles/instance: %.0f" % (tt.sum() / B))
for n, x in zip(names_t, tt): print("  %-16s %6.1f%%  %8.0f cyc/inst" % (n, 100 * x / tt.sum(), x / B))
print("qp kernel cycles/instance: %.0f" % (tq.sum() / B))
for n, x in zip(names_q, tq): print("  %-16s %6.1f%%  %8.0f cyc/inst" % (n, 100 * x / tq.sum(), x / B))
names_a = ["set_rho+factor", "prep+load regs", "admm iterations (+publish)", "admm_check (residuals/polish/refactor)"]
print("inside rho+factor+admm+checks:")
for n, x in zip(names_a, ta): print("  %-40s %8.0f cyc/inst" % (n, x / B))
print("task stragglers: max instance %.0f cycles, %d instances > 400k cycles (%.1f%% of task cycles)" % (v[30], v[31], 100 * v[29] / max(tt.sum(), 1)))
print("straggler phase split: " + ", ".join("%s %.0f%%" % (n, 100 * x / max(v[8:16].sum(), 1)) for n, x in zip(names_t, v[8:16])))
print("EPA (all instances): %d calls, %d steps, max %d steps in one call" % (v[22], v[23], v[28]))
print("EPA step split: scan+support+tests %.0f, grow %.0f cycles/step" % (v[18] / max(v[23], 1), v[20] / max(v[23], 1)))
print("EPA grow split (cycles/step): visibility+component %.0f, horizon+cycle check %.0f, order+planes %.0f, writes %.0f"
      % tuple(v[k] / max(v[23], 1) for k in (59, 61, 62, 63)))
print("EPA seed polytope (GJK rerun + tetrahedron, lane-serial): %.0f cycles/call" % (v[60] / max(v[22], 1)))
print("admm_check: residuals %.0f cyc/inst (%d calls), polish %.0f cyc/inst (%d attempts, %d accepted), refactor after polish %.0f cyc/inst" % (v[32] / B, v[33], v[35] / B, v[36], v[37], v[38] / B))
print("eqp: %d calls, %.0f cycles/call, mean KKT size %.1f; polish residuals %.0f cycles/call" % (v[41], v[40] / max(v[41], 1), v[42] / max(v[41], 1), v[43] / max(v[41], 1)))
print("qp record load (inside load+assemble): %.0f cyc/inst" % (v[44] / B))
print("polish steps: infeasible->add/drop %d, wrong dual sign->drop %d, ratio-test blocks %d, KKT residual failures %d" % (v[45], v[46], v[47], v[48]))
print("Ruiz passes: %.2f per instance" % (v[49] / B))
sub = [("jacobi guess", 50), ("drop rule", 51), ("eqp setup (K0, rhs)", 52), ("eqp Gauss-Jordan", 53),
       ("eqp solve + refinement", 54), ("eqp x, y, stationarity", 55), ("ratio test", 56), ("candidate z", 57),
       ("polish residuals", 43), ("certify + add/drop", 58)]
print("polish sub-phases (cycles/instance): " + ", ".join("%s %.0f" % (n, v[k] / B) for n, k in sub))

"""Diagnostic: per-phase cycles of the lane-per-instance task stage and the
hard-list census (DRC_PHASE_TIMING build, slots 48..60)."""
import ctypes as C
import os
import sys
os.environ["DRC_AMD_LIB"] = "libdrc_amd_timing.so"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from _common import LINK, make_manipulator, step_inputs  # noqa: E402
from dyros_robot_controller_amd import _batch, _capi, manipulator  # noqa: E402

dev = torch.device("cuda", 0)
robot = sys.argv[1] if len(sys.argv) > 1 else "fr3"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
stress = len(sys.argv) <= 3 or sys.argv[3] != "nominal"
rd = make_manipulator(robot, dev)
q, qd, xt, xdt = step_inputs(rd, robot, 12345, B, dev, stress=stress)
args = [_batch.as_device(a, dev) for a in (q, qd, xt, xdt)]
_capi.lib().drc_set_concurrency(rd.model.handle, 1)
p = manipulator.QPIKParamsBuilder(rd.model, exact=True).params(LINK[robot], _capi.MODE_QPIK_STEP)
_batch.stages_batch(rd.model, p, *args)
torch.cuda.synchronize()
buf = (C.c_ulonglong * 64)()
_capi.lib().drc_debug_phase_cycles(buf, 1)
_batch.stages_batch(rd.model, p, *args)
torch.cuda.synchronize()
_capi.lib().drc_debug_phase_cycles(buf, 0)
v = np.array(buf[:], dtype=np.float64)
waves = (B + 63) // 64
names = ["FK+frame", "pass1 closed+bounds", "pass2 GJK", "axes+grad+J+xdd", "manip", "outputs"]
tot = v[48:54].sum()
print("lane stage: %d waves, %.0f cycles/wave (sum of phases), %.0f per instance" % (waves, tot / waves, tot / B))
for i, n in enumerate(names):
    print("  %-22s %6.1f%%  %9.0f cyc/wave" % (n, 100 * v[48 + i] / max(tot, 1), v[48 + i] / waves))
print("instances %d: hard (candidates) %d, hard (EPA) %d, manip fallback %d, GJK calls %d" %
      (v[58], v[56], v[57], v[59], v[60]))

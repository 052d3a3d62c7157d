"""Diagnostic: one FR3 QPIKStep batch with the lane task stage on and off
(for rocprofv3 --kernel-trace --stats), plus the hard-list size."""
import os
import sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
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
for lane in (1, 0, 1):
    _capi.check(_capi.lib().drc_debug_lane_stage(rd.model.handle, lane))
    for _ in range(3):
        _batch.qpik_batch(rd.model, p, *args)
    torch.cuda.synchronize()
print("done")

"""Diagnostic: exact-mode QPIK time and result at several ADMM check
intervals (the polish is attempted at every check; results are the
certified optimum either way)."""
import json
import os
import sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
from _common import LINK, make_manipulator, step_inputs  # noqa: E402
from dyros_robot_controller_amd import _batch, _capi, manipulator  # noqa: E402

dev = torch.device("cuda", 0)
robot = sys.argv[1] if len(sys.argv) > 1 else "fr3"
B = 65536
rd = make_manipulator(robot, dev)
q, qd, xt, xdt = step_inputs(rd, robot, 12345, B, dev, stress=True)
args = [_batch.as_device(a, dev) for a in (q, qd, xt, xdt)]
st = torch.cuda.current_stream(dev)
res, ref = {}, None
for chk in (25, 20, 15, 10, 5):
    p = manipulator.QPIKParamsBuilder(rd.model, exact=True).params(LINK[robot], _capi.MODE_QPIK_STEP)
    p.solver.check_termination = chk
    p.solver.adaptive_rho_interval = chk
    it = torch.zeros(B, dtype=torch.int32, device=dev)
    call = lambda: _batch.qpik_batch(rd.model, p, *args, iters=it)
    out, status = call()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(5):
        out, status = call()
    e1.record(st)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    if ref is None:
        ref = o
    res[chk] = dict(ms=e0.elapsed_time(e1) / 5, iters=float(it.float().mean()),
                    non_solved=int((status != 1).sum().item()), max_dq_vs_25=float(abs(o - ref).max()))
print(json.dumps(res, indent=1))

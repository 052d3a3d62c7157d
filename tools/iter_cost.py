"""Diagnostic: cost of one ADMM iteration and of the polish in the QPIK QP
kernel, from call times at forced iteration counts (one sub-batch).

eps = 1e-14 keeps OSQP from converging, so every instance runs exactly
max_iter iterations; the slope over max_iter is the per-iteration cost.
Printed as ns per call and as shader cycles per instance-iteration at the
kernel's wave slots (256 CUs x 4 SIMDs x 2 waves, 2.4 GHz)."""
import sys
import json
import torch
sys.path[:0] = [".", "tests", "oracle"]
from _common import make_manipulator, step_inputs  # noqa: E402
from dyros_robot_controller_amd import _batch, _capi, manipulator  # noqa: E402

dev = torch.device("cuda", 0)
robot, B = "fr3", 65536
rd = make_manipulator(robot, dev)
q, qd, xt, xdt = step_inputs(rd, robot, 12345, B, dev)
args = [_batch.as_device(a, dev) for a in (q, qd, xt, xdt)]
_capi.lib().drc_set_concurrency(rd.model.handle, 1)
st = torch.cuda.current_stream(dev)


def timed(exact, max_iter, eps, adaptive, steps=5):
    pb = manipulator.QPIKParamsBuilder(rd.model, exact=exact)
    p = pb.params("fr3_link8", _capi.MODE_QPIK_STEP)
    p.solver.max_iter = max_iter
    p.solver.eps_abs = p.solver.eps_rel = eps
    p.solver.adaptive_rho = adaptive
    it = torch.zeros(B, dtype=torch.int32, device=dev)
    call = lambda: _batch.qpik_batch(rd.model, p, *args, iters=it)
    call()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(steps):
        call()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps, float(it.float().mean())


slots = 256 * 4 * 2
res = {}
for ad in (0, 1):
    (t1, i1), (t2, i2) = timed(False, 50, 1e-14, ad), timed(False, 450, 1e-14, ad)
    cyc = (t2 - t1) * 1e-3 * 2.4e9 * slots / (B * (i2 - i1))
    res["adaptive%d" % ad] = dict(ms50=t1, ms450=t2, iters=(i1, i2), cycles_per_inst_iter=cyc)
# exact default vs osqp settings with the same iteration cap
te, ie = timed(True, 4000, 1e-3, 1)
to, io = timed(False, 4000, 1e-3, 1)
res["exact_default"] = dict(ms=te, iters=ie)
res["osqp_default"] = dict(ms=to, iters=io)
print(json.dumps(res, indent=1))

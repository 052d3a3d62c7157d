"""Diagnostic: QPIK call time at forced ADMM iteration counts (one sub-batch,
no polish, eps = 1e-14 so every instance runs exactly max_iter iterations),
next to the default exact-mode call.  Differences between rows give the
cost of the first iterations, of later ones, and of the setup outside the
ADMM loop, in shader cycles per instance at the kernel's wave slots."""
import ctypes as C
import json
import sys

import torch

sys.path[:0] = [".", "tests", "oracle"]
from _common import make_manipulator, step_inputs  # noqa: E402
from dyros_robot_controller_amd import _batch, _capi, manipulator  # noqa: E402

dev = torch.device("cuda", 0)
robot = sys.argv[1] if len(sys.argv) > 1 else "fr3"
B = 65536
rd = make_manipulator(robot, dev)
link = "fr3_link8" if robot == "fr3" else "tool0"
q, qd, xt, xdt = step_inputs(rd, robot, 12345, B, dev, stress=True)
args = [_batch.as_device(a, dev) for a in (q, qd, xt, xdt)]
_capi.lib().drc_set_concurrency(rd.model.handle, 1)
st = torch.cuda.current_stream(dev)
slots = 256 * 4 * 2


def timed(exact, max_iter, eps, adaptive=0, check=25, steps=5):
    pb = manipulator.QPIKParamsBuilder(rd.model, exact=exact)
    p = pb.params(link, _capi.MODE_QPIK_STEP)
    p.solver.max_iter = max_iter
    p.solver.eps_abs = p.solver.eps_rel = eps
    p.solver.adaptive_rho = adaptive
    p.solver.check_termination = check
    it = torch.zeros(B, dtype=torch.int32, device=dev)
    call = lambda: _batch.qpik_batch(rd.model, p, *args, iters=it)
    call()
    torch.cuda.synchronize()
    lib, h = _capi.lib(), rd.model.handle
    _capi.check(lib.drc_debug_kernel_timing(h, 1))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(steps):
        call()
    e1.record(st)
    torch.cuda.synchronize()
    tw, tk, tq, nc = C.c_double(), C.c_double(), C.c_double(), C.c_int()
    _capi.check(lib.drc_debug_kernel_times(h, C.byref(tw), C.byref(tk), C.byref(tq), C.byref(nc)))
    _capi.check(lib.drc_debug_kernel_timing(h, 0))
    ms = e0.elapsed_time(e1) / steps
    cyc = lambda t: t * 1e-3 * 2.4e9 * slots / B
    return dict(ms=ms, iters=float(it.float().mean()), task_ms=tk.value / nc.value, qp_ms=tq.value / nc.value,
                qp_cyc_per_inst=cyc(tq.value / nc.value), task_cyc_per_inst=cyc(tk.value / nc.value))


res = {}
for n in (1, 2, 25, 50, 100):
    res["iters%d" % n] = timed(False, n, 1e-14, check=25)
res["iters100_check0"] = timed(False, 100, 1e-14, check=0)
res["exact_default"] = timed(True, 4000, 1e-3, adaptive=1)
_capi.check(_capi.lib().drc_debug_lane_stage(rd.model.handle, 0))
res["exact_default_wave_task"] = timed(True, 4000, 1e-3, adaptive=1)
_capi.check(_capi.lib().drc_debug_lane_stage(rd.model.handle, 1))
print(json.dumps(res, indent=1))

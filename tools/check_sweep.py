"""Diagnostic: exact-mode QPIK call time vs the termination-check interval
(check_termination; the adaptive-rho interval follows it or stays at 25) or
the Ruiz iteration count (argv[2] == "scaling").
The certified optimum does not depend on it; the ADMM iterations before the
first polish attempt and the failed attempts do."""
import sys
import json
import torch
sys.path[:0] = [".", "tests", "oracle"]
from _common import make_manipulator, step_inputs  # noqa: E402
from dyros_robot_controller_amd import _batch, _capi, manipulator  # noqa: E402

dev = torch.device("cuda", 0)
robot = sys.argv[1] if len(sys.argv) > 1 else "fr3"
link = {"fr3": "fr3_link8", "ur5e": "tool0"}[robot]
B = 65536
rd = make_manipulator(robot, dev)
q, qd, xt, xdt = step_inputs(rd, robot, 12345, B, dev, stress=True)   # bench.py's workload
args = [_batch.as_device(a, dev) for a in (q, qd, xt, xdt)]
st = torch.cuda.current_stream(dev)
ref = None
knobs = sys.argv[2] if len(sys.argv) > 2 else "check"
grid = {"check": [(25, 25, 10), (15, 25, 10), (10, 25, 10), (8, 25, 10), (5, 25, 10), (3, 25, 10), (1, 25, 10)],
        "long": [(25, 25, 10), (50, 25, 10), (75, 25, 10), (50, 50, 10), (100, 100, 10)],
        "scaling": [(25, 25, 10), (25, 25, 5), (25, 25, 3), (25, 25, 1), (25, 25, 0)]}[knobs]
for ct, ar, sc in grid:
    p = manipulator.QPIKParamsBuilder(rd.model, exact=True).params(link, _capi.MODE_QPIK_STEP)
    p.solver.check_termination = ct
    p.solver.adaptive_rho_interval = ar
    p.solver.scaling = sc
    it = torch.zeros(B, dtype=torch.int32, device=dev)
    call = lambda: _batch.qpik_batch(rd.model, p, *args, iters=it)
    out, status = call()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(10):
        call()
    e1.record(st)
    torch.cuda.synchronize()
    o = out.cpu()
    if ref is None:
        ref = o
    print(json.dumps(dict(check=ct, adapt=ar, scaling=sc, ms=e0.elapsed_time(e1) / 10, iters_mean=float(it.float().mean()),
                          iters_max=int(it.max()), solved=float((status == 1).float().mean()),
                          maxdiff_vs_25=float((o - ref).abs().max()))), flush=True)

"""Diagnostic: one instance of the QPIK(xdot) parity batch where the device
and the oracle (fed the device's distance stage) disagree on the status
(dev tool).  usage: python tools/debug_status.py robot seed B b"""
import sys
sys.path[:0] = ["tests", "oracle", "."]
import numpy as np
import torch
import oracle as O
import pyref as R
from _common import LINK, make_manipulator, oracle_params, stage_pose, step_inputs
from dyros_robot_controller_amd import manipulator, workload

robot, seed, B, b = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
dev = torch.device("cuda", 0)
rd = make_manipulator(robot, dev)
q, qd, _, _ = step_inputs(rd, robot, seed, B, dev, stress=True)
xdot = np.stack([0.2 * workload.normal(seed, 600 + i, B) for i in range(6)])
ctrl = manipulator.RobotController(0.001, rd, solver_mode="exact")
iters = torch.zeros(B, dtype=torch.int32, device=dev)
out, status = ctrl._run(0, LINK[robot], q, qd, None, xdot, iters=iters)
out, status, iters = out.cpu().numpy(), status.cpu().numpy(), iters.cpu().numpy()
st = stage_pose(rd.model, dev, q, qd, LINK[robot])
par, om = oracle_params(robot, True, 0)
pm = O.load(robot)[0]
np.set_printoptions(precision=10, linewidth=180)
print("gpu status", status[b], "iters", iters[b], "out", out[:, b])
d, dg, pair = O.min_distance(om, q[:, b])
print("dist gpu", st["dist"][0, b], "orc", d, "grad diff", np.abs(st["dist"][1:, b] - dg).max())
for tag, din in (("dev-dist", st["dist"][:, b:b + 1]), ("own-dist", None)):
    if din is None:
        o, s, it = O.qpik_batch(om, par, q[:, b:b + 1], qd[:, b:b + 1], None, xdot[:, b:b + 1])
    else:
        o, s, it = O.qpik_batch_dist(om, par, q[:, b:b + 1], qd[:, b:b + 1], None, xdot[:, b:b + 1], din)
    print(tag, "oracle status", s[0], "iters", it[0], "out", o[:, 0], "|d|", np.abs(o[:, 0] - out[:, b]).max())
m, mg = st["man"][0, b], st["man"][1:, b]
P, qv, A, l, u = R.build_qp_manipulator(pm, q[:, b], xdot[:, b], LINK[robot], man=(m, mg),
                                        dist=(st["dist"][0, b], st["dist"][1:, b]))
x, y, s = R.solve_qp_exact(P, qv, A, l, u)
print("ipm status", s, "x", x[:pm.nv], "|gpu - ipm|", np.abs(x[:pm.nv] - out[:, b]).max())
print("P cond", np.linalg.cond(P))
np.savez("gpurun_out/inst_%s_%d_%d.npz" % (robot, seed, b), q=q[:, b], qd=qd[:, b], xdot=xdot[:, b],
         dist=st["dist"][:, b], out=out[:, b])

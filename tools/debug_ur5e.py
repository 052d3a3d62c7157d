import sys
sys.path.insert(0, "tests"); sys.path.insert(0, "oracle"); sys.path.insert(0, ".")
import numpy as np, torch, oracle as O
from _common import make_manipulator, step_inputs, stage_pose, LINK, oracle_batch
from dyros_robot_controller_amd import manipulator
dev = torch.device("cuda", 0)
rd = make_manipulator("ur5e", dev)
B = 512
q, qd, xt, xdt = step_inputs(rd, "ur5e", 2, B, dev)
st = stage_pose(rd.model, dev, q, qd, "tool0")
pm, om, spec = O.load("ur5e")
ctrl = manipulator.RobotController(0.001, rd)
out, status = ctrl.QPIK_step_batch(q, qd, xt, xdt, "tool0")
out = out.cpu().numpy()
ref, rst, _, _ = oracle_batch("ur5e", q, qd, xt, xdt, exact=True)
err = np.abs(out - ref).max(axis=0)
for b in np.argsort(-err)[:3]:
    d, dg, pair = O.min_distance(om, q[:, b])
    m, mg = O.manipulability(om, q[:, b])
    print(b, "err", err[b], "gpu pair", st["pair"][b], "dist", st["dist"][0, b], "oracle pair", pair, d)
    print("   gpu grad", st["dist"][1:, b], "\n   orc grad", dg)
    print("   man", st["man"][0, b], m, "xdd", st["xdot_des"][:, b])
    print("   gpu out", out[:, b], "\n   orc out", ref[:, b])
    sto, o1, dgn = O.qpik_one(om, O.default_params(0, True), q[:, b], qd[:, b], xt[:, b], xdt[:, b])
    print("   oracle diag xdd", np.array(dgn.xdot_des), "iters", dgn.iters, "pol", dgn.polished)

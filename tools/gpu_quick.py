"""Quick GPU probe: one FR3 batch, timing + oracle comparison (dev tool)."""
import sys, time
sys.path.insert(0, "tests"); sys.path.insert(0, "oracle"); sys.path.insert(0, ".")
import numpy as np, torch
from _common import make_manipulator, step_inputs, oracle_batch, stage_pose
from dyros_robot_controller_amd import manipulator
dev = torch.device("cuda", 0)
robot = sys.argv[1] if len(sys.argv) > 1 else "fr3"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
rd = make_manipulator(robot, dev)
print("model", rd.model.dof, rd.model.n_geoms, rd.model.n_pairs, flush=True)
q, qd, xt, xdt = step_inputs(rd, robot, 7, B, dev)
print("inputs ok", flush=True)
ctrl = manipulator.RobotController(0.001, rd, solver_mode="exact")
link = "fr3_link8" if robot == "fr3" else "tool0"
dq, dqd, dxt, dxdt = [torch.as_tensor(a, device=dev) for a in (q, qd, xt, xdt)]
iters = torch.zeros(B, dtype=torch.int32, device=dev)
out, st = ctrl.QPIK_step_batch(dq, dqd, dxt, dxdt, link, iters=iters)
torch.cuda.synchronize()
t = time.time()
for _ in range(int(sys.argv[3]) if len(sys.argv) > 3 else 3):
    out, st = ctrl.QPIK_step_batch(dq, dqd, dxt, dxdt, link, iters=iters)
torch.cuda.synchronize()
dt = (time.time() - t) / 3
print("B=%d  %.3f ms  %.3e solves/s" % (B, dt * 1e3, B / dt), flush=True)
out, st, it = out.cpu().numpy(), st.cpu().numpy(), iters.cpu().numpy()
print("status", np.unique(st, return_counts=True), "iters mean", it.mean(), "max", it.max())
n = min(B, 1024)
ref, rst, rit, _ = oracle_batch(robot, q[:, :n], qd[:, :n], xt[:, :n], xdt[:, :n], exact=True)
err = np.abs(out[:, :n] - ref).max(axis=0)
print("max err vs oracle", err.max(), "p99", np.percentile(err, 99), "status agree", np.mean(st[:n] == rst), "iters agree", np.mean(it[:n] == rit))

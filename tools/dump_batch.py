"""Dev tool: runs bench.py's workload for one robot through the product path
once and saves inputs, q̇*, status and ADMM iterations per instance to
gpurun_out/dump_<robot>_<B>.npz (for oracle comparison on the CPU).
usage: python tools/dump_batch.py robot B"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import bench
from dyros_robot_controller_amd import BUNDLED, make_robot, manipulator, mobile_manipulator

robot, B = sys.argv[1], int(sys.argv[2])
dev = torch.device("cuda", 0)
spec = BUNDLED[robot]
rd = make_robot(robot, dev)
mod = manipulator if spec["kind"] == "manipulator" else mobile_manipulator
ctrl = mod.RobotController(0.001, rd, solver_mode="exact")
(q, qd, xt, xdt), (dq, dqd, dxt, dxdt), tiers = bench.make_inputs(rd, robot, B, 12345, 0, dev)
iters = torch.zeros(B, dtype=torch.int32, device=dev)
out, status = ctrl.QPIK_step_batch(dq, dqd, dxt, dxdt, spec["link"], iters=iters)
torch.cuda.synchronize()
out = out if isinstance(out, torch.Tensor) else torch.cat([o for o in out], 0)
os.makedirs("gpurun_out", exist_ok=True)
st, it = status.cpu().numpy(), iters.cpu().numpy()
np.savez_compressed("gpurun_out/dump_%s_%d.npz" % (robot, B), q=q, qd=qd, xt=xt, xdt=xdt, out=out.cpu().numpy(),
                    status=st, iters=it)
print(robot, B, "statuses", np.unique(st, return_counts=True), "iters p99", np.percentile(it, 99), "max", it.max(),
      ">=500:", int((it >= 500).sum()))

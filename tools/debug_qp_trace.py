"""Diagnostic: run one dumped instance (tools/debug_status.py's npz) through
a DRC_QP_DEBUG build of the product library (DRC_AMD_LIB=libdrc_amd_dbg.so),
which prints the ADMM residuals at every termination check (dev tool)."""
import sys
sys.path[:0] = ["tests", "oracle", "."]
import numpy as np
import torch
from _common import LINK, make_manipulator
from dyros_robot_controller_amd import manipulator
robot, path, mode = sys.argv[1], sys.argv[2], int(sys.argv[3])
d = np.load(path)
dev = torch.device("cuda", 0)
rd = make_manipulator(robot, dev)
ctrl = manipulator.RobotController(0.001, rd, solver_mode="exact")
iters = torch.zeros(1, dtype=torch.int32, device=dev)
out, st = ctrl._run(mode, LINK[robot], d["q"][:, None], d["qd"][:, None], None, d["xdot"][:, None], iters=iters)
torch.cuda.synchronize()
print("status", st.cpu().numpy(), "iters", iters.cpu().numpy(), "out", out.cpu().numpy()[:, 0])

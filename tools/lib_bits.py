"""Two library builds, bit for bit (dev tool): runs bench.py's workload
(stress tiers, seed 12345) through the library DRC_AMD_LIB names and saves
q-dot*, status and ADMM iterations per robot; with --compare, reports how
many instances differ from a previous dump.
    DRC_AMD_LIB=<lib> [DRC_SOLVER=osqp_default] python tools/lib_bits.py <tag> [robot ...]
    python tools/lib_bits.py --compare <tagA> <tagB> [robot ...]"""
import os
import sys

sys.path.insert(0, "tests"); sys.path.insert(0, "oracle"); sys.path.insert(0, ".")
import numpy as np

OUT = os.environ.get("DRC_BITS_DIR", "gpurun_out")
ROBOTS = ["fr3", "ur5e", "husky_fr3", "xls_fr3", "caster_fr3"]
BATCH = {"husky_fr3": 16384}


def dump(tag, robots):
    import torch
    from _common import LINK, make_manipulator, make_moma, moma_step_inputs, step_inputs
    from dyros_robot_controller_amd import manipulator, mobile_manipulator
    dev = torch.device("cuda", 0)
    for robot in robots:
        moma = robot in ("husky_fr3", "xls_fr3", "caster_fr3")
        rd = make_moma(robot, dev) if moma else make_manipulator(robot, dev)
        ctrl = (mobile_manipulator if moma else manipulator).RobotController(0.001, rd, solver_mode=os.environ.get("DRC_SOLVER", "exact"))
        B = BATCH.get(robot, 65536)
        q, qd, xt, xdt = (moma_step_inputs if moma else step_inputs)(rd, robot, 12345, B, dev, stress=True)
        args = [torch.as_tensor(a, device=dev) for a in (q, qd, xt, xdt)]
        it = torch.zeros(B, dtype=torch.int32, device=dev)
        out, st = ctrl.QPIK_step_batch(*args, LINK[robot], iters=it)
        torch.cuda.synchronize()
        np.savez(os.path.join(OUT, "bits_%s_%s.npz" % (tag, robot)), out=out.cpu().numpy(), st=st.cpu().numpy(),
                 it=it.cpu().numpy())
        print(tag, robot, "saved", flush=True)


def compare(a, b, robots):
    for robot in robots:
        A = np.load(os.path.join(OUT, "bits_%s_%s.npz" % (a, robot)))
        Bz = np.load(os.path.join(OUT, "bits_%s_%s.npz" % (b, robot)))
        diff = np.any(A["out"] != Bz["out"], axis=0) | (A["st"] != Bz["st"]) | (A["it"] != Bz["it"])
        print(robot, "instances differing: %d / %d, max |dq| %.3g, status differ %d, iters differ %d" % (
            int(diff.sum()), diff.size, float(np.abs(A["out"] - Bz["out"]).max()), int((A["st"] != Bz["st"]).sum()),
            int((A["it"] != Bz["it"]).sum())), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        compare(sys.argv[2], sys.argv[3], sys.argv[4:] or ROBOTS)
    else:
        dump(sys.argv[1], sys.argv[2:] or ROBOTS)

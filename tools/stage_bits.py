"""How close are the device stage outputs to the oracle's, bit for bit?
(diagnostic; test infrastructure).  Prints, per robot, the fraction of
instances whose pose / Jacobian / manipulability / distance / gradient are
bit-identical to the oracle's and the max abs difference of each."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]


def main():
    import torch
    import oracle as O
    from _common import LINK, make_manipulator, make_moma, moma_step_inputs, stage_pose, step_inputs
    dev = torch.device("cuda", 0)
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    for robot in ("fr3", "ur5e", "husky_fr3", "xls_fr3"):
        moma = robot in ("husky_fr3", "xls_fr3")
        rd = make_moma(robot, dev) if moma else make_manipulator(robot, dev)
        q, qd, xt, xdt = (moma_step_inputs if moma else step_inputs)(rd, robot, 1, B, dev)
        st = stage_pose(rd.model, dev, q, qd, LINK[robot])
        pm, om, spec = O.load(robot)
        n = om.nv
        diff = {k: [] for k in ("pose", "jac", "m", "mg", "d", "dg")}
        for b in range(B):
            pose, J = O.fk_pose(om, q[:, b])
            Rcm = np.concatenate([pose[:9].reshape(3, 3).T.reshape(-1), pose[9:]])
            m, mg = O.manipulability(om, q[:, b])
            d, dg, pair = O.min_distance(om, q[:, b])
            diff["pose"].append(np.max(np.abs(st["pose"][:, b] - Rcm)))
            diff["jac"].append(np.max(np.abs(st["jac"][:, b].reshape(6, n) - J)))
            diff["m"].append(abs(st["man"][0, b] - m))
            diff["mg"].append(np.max(np.abs(st["man"][1:, b] - mg)))
            diff["d"].append(abs(st["dist"][0, b] - d))
            diff["dg"].append(np.max(np.abs(st["dist"][1:, b] - dg)))
        out = {"robot": robot, "B": B}
        for k, v in diff.items():
            v = np.array(v)
            out[k] = {"bit_equal": float(np.mean(v == 0)), "max": float(v.max()), "p99": float(np.percentile(v, 99))}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

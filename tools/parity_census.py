"""GPU-vs-oracle parity census (diagnostic; test infrastructure).

For each robot and seed: runs QPIKStep in exact mode on the device and in the
oracle, and writes, for every instance outside the north_star bound (1e-4 on
qdot* or on the task-space residual J (qdot_gpu - qdot_oracle)), the stage
data differences that explain it.  Output: JSON on stdout.

    python tools/parity_census.py [--batch 2048] [--seeds 1,2,3]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]


def main():
    import torch
    import oracle as O
    from _common import (LINK, make_manipulator, make_moma, moma_step_inputs, nonsmooth_min_distance, oracle_batch,
                         qp_from_stages, stage_step, step_inputs)
    from dyros_robot_controller_amd import manipulator, mobile_manipulator as MM

    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--seeds", default="1,2,3")
    ap.add_argument("--robots", default="fr3,ur5e,husky_fr3,xls_fr3")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    res = []
    for robot in a.robots.split(","):
        moma = robot in ("husky_fr3", "xls_fr3")
        rd = make_moma(robot, dev) if moma else make_manipulator(robot, dev)
        ctrl = (MM if moma else manipulator).RobotController(0.001, rd, solver_mode="exact")
        pm, om, spec = O.load(robot)
        for seed in [int(s) for s in a.seeds.split(",")]:
            B = a.batch
            q, qd, xt, xdt = (moma_step_inputs if moma else step_inputs)(rd, robot, seed, B, dev)
            out, status = ctrl.QPIK_step_batch(q, qd, xt, xdt, LINK[robot])
            out, status = out.cpu().numpy(), status.cpu().numpy()
            ref, rstat, _, _ = oracle_batch(robot, q, qd, xt, xdt, exact=True, nthreads=16)
            st = stage_step(rd.model, dev, q, qd, xt, xdt, LINK[robot])
            err = np.abs(out - ref).max(axis=0)
            rec = {"robot": robot, "seed": seed, "B": B, "status_mismatch": int(np.sum(status != rstat)),
                   "median_err": float(np.median(err)), "off": []}
            for b in range(B):
                _, J = O.fk_pose(om, q[:, b])
                if moma:
                    tr = float("nan")
                else:
                    tr = float(np.max(np.abs(J @ (out[:, b] - ref[:, b]))))
                if err[b] <= 1e-4 and not (tr > 1e-4):
                    continue
                d, dg, pair = O.min_distance(om, q[:, b])
                m, mg = O.manipulability(om, q[:, b])
                e = {"b": b, "err": float(err[b]), "task_res": tr, "status": int(status[b]), "ostatus": int(rstat[b]),
                     "d_gpu": float(st["dist"][0, b]), "d_orc": d, "pair_gpu": int(st["pair"][b]), "pair_orc": pair,
                     "dgrad_diff": float(np.max(np.abs(st["dist"][1:, b] - dg))),
                     "m_gpu": float(st["man"][0, b]), "m_orc": m,
                     "mgrad_diff": float(np.max(np.abs(st["man"][1:, b] - mg))),
                     "nonsmooth": bool(nonsmooth_min_distance(om, q[:, b]))}
                if not moma:
                    x = qp_from_stages(pm, q, st, b, LINK[robot])
                    e["own_stage_opt_err"] = float(np.max(np.abs(out[:, b] - x))) if x is not None else None
                rec["off"].append(e)
            rec["n_off"] = len(rec["off"])
            res.append(rec)
            print(json.dumps({k: v for k, v in rec.items() if k != "off"}), file=sys.stderr, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()

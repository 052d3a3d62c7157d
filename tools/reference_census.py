"""Reference-settings census (diagnostic; test infrastructure): the device's
osqp_default mode (OSQP eps 1e-3, no polish) against the oracle's, per robot
and case, without asserting.  Each instance is classed as

  agree     same status, |q-dot*| within 1e-7 (same ADMM trajectory);
  adjacent  the two sides stopped one termination check apart;
  diverged  anything else (the trajectories separated before either stopped);

and every solved answer is placed against the exact optimum (the oracle's
exact mode): the OSQP band |q-dot - q-dot_exact| of the oracle's own answers
is the yardstick for the device's.  JSON on stdout.

    python tools/reference_census.py [--robots fr3,ur5e] [--batch 1024]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]


def classify(robot, args, out, status, iters, check=25):
    import oracle as O
    from _common import oracle_params
    par, om = oracle_params(robot, exact=False)
    pex, _ = oracle_params(robot, exact=True)
    ref, rstat, riters = O.qpik_batch(om, par, *args, nthreads=16)
    ex, xstat, _ = O.qpik_batch(om, pex, *args, nthreads=16)
    dq = np.abs(out - ref).max(axis=0)
    agree = (status == rstat) & (dq <= 1e-7)
    adjacent = ~agree & (np.abs(iters - riters) == check)
    diverged = ~agree & ~adjacent
    both = (status == 1) & (rstat == 1) & (xstat == 1)
    band_o = np.abs(ref - ex).max(axis=0)
    band_g = np.abs(out - ex).max(axis=0)
    rows = [{"b": int(b), "iters": [int(iters[b]), int(riters[b])], "status": [int(status[b]), int(rstat[b])],
             "dq": float(dq[b]), "gpu_vs_exact": float(band_g[b]), "oracle_vs_exact": float(band_o[b])}
            for b in np.nonzero(diverged)[0]]
    return {"B": int(len(status)), "agree": int(agree.sum()), "adjacent": int(adjacent.sum()),
            "diverged": int(diverged.sum()), "status_mismatch": int((status != rstat).sum()),
            "nonsolved_gpu": int((status != 1).sum()), "nonsolved_oracle": int((rstat != 1).sum()),
            "band_oracle_max": float(band_o[both].max()) if both.any() else None,
            "band_gpu_max": float(band_g[both].max()) if both.any() else None,
            "band_oracle_p99": float(np.percentile(band_o[both], 99)) if both.any() else None,
            "band_gpu_p99": float(np.percentile(band_g[both], 99)) if both.any() else None,
            "iters_max": [int(iters.max()), int(riters.max())], "diverged_rows": rows[:20]}


def main():
    import torch
    from _common import LINK, make_manipulator, make_moma, moma_step_inputs, step_inputs
    from dyros_robot_controller_amd import manipulator, mobile_manipulator
    ap = argparse.ArgumentParser()
    ap.add_argument("--robots", default="fr3,ur5e,husky_fr3,xls_fr3,caster_fr3")
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--seed", type=int, default=4)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    res = []
    for robot in a.robots.split(","):
        moma = robot in ("husky_fr3", "xls_fr3", "caster_fr3")
        rd = make_moma(robot, dev) if moma else make_manipulator(robot, dev)
        ctrl = (mobile_manipulator if moma else manipulator).RobotController(0.001, rd, solver_mode="osqp_default")
        for stress in (False, True):
            args = (moma_step_inputs if moma else step_inputs)(rd, robot, a.seed, a.batch, dev, stress=stress)
            it = torch.zeros(a.batch, dtype=torch.int32, device=dev)
            o, st = ctrl.QPIK_step_batch(*[torch.as_tensor(x, device=dev) for x in args], LINK[robot], iters=it)
            torch.cuda.synchronize()
            r = classify(robot, args, o.cpu().numpy(), st.cpu().numpy(), it.cpu().numpy())
            r.update(robot=robot, stress=stress)
            res.append(r)
            print(json.dumps({k: v for k, v in r.items() if k != "diverged_rows"}), flush=True)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "reference_census.json"), "w"), indent=1)


if __name__ == "__main__":
    main()

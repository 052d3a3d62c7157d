"""One rank of tests/test_gpu_dist.py (started by dist.spawn_ranks): solve this
rank's contiguous shard with the product kernels (drc_qpik_batch), all-gather
the shards, reduce the counters through the device path, and on rank 0 check
the gathered batch against a single-process run over the whole range."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]


def main(outdir, robot, per_rank, strong):
    import numpy as np
    import torch
    from dyros_robot_controller_amd import dist as ddist, make_robot, manipulator, mobile_manipulator, BUNDLED
    from _common import LINK, moma_step_inputs, step_inputs

    rank, world, local = ddist.env_rank()
    dev = torch.device("cuda", 0)          # every rank shares the one GPU of the box
    torch.cuda.set_device(dev)
    d = ddist.init(os.environ.get("DRC_DIST_BACKEND", "gloo"))
    G = per_rank * world
    off, cnt = ddist.shard_global(rank, world, G) if strong else ddist.shard(rank, per_rank)
    counts = [ddist.shard_global(k, world, G)[1] if strong else per_rank for k in range(world)]
    rd = make_robot(robot, dev)
    manip = BUNDLED[robot]["kind"] == "manipulator"
    mod = manipulator if manip else mobile_manipulator
    ctrl = mod.RobotController(0.001, rd, solver_mode="exact")
    gen = step_inputs if manip else moma_step_inputs

    def solve(B, offset):
        q, qd, xt, xdt = gen(rd, robot, 2024, B, dev, offset=offset, stress=True)
        it = torch.zeros(B, dtype=torch.int32, device=dev)
        out, status = ctrl.QPIK_step_batch(q, qd, xt, xdt, LINK[robot], iters=it)
        torch.cuda.synchronize()
        return q, out, status, it

    q, out, status, it = solve(cnt, off)
    block = torch.cat([out, status.double().unsqueeze(0), it.double().unsqueeze(0)], 0)  # [A + 2][cnt] on device
    full = ddist.gather_outputs(block, counts, world)
    qfull = ddist.gather_outputs(torch.as_tensor(q, device=dev), counts, world)
    wall, n_bad, it_mean = ddist.reduce_stats(1.0 + rank, float((status != 1).sum().item()),
                                              float(it.double().mean().item()), world, dev)
    if rank == 0:
        q1, out1, st1, it1 = solve(G, 0)
        ref = torch.cat([out1, st1.double().unsqueeze(0), it1.double().unsqueeze(0)], 0)
        res = {"device": str(full.device), "inputs_equal": bool(np.array_equal(qfull.cpu().numpy(), q1)),
               "bitwise_equal": bool(torch.equal(full, ref)),
               "max_abs": float((full - ref).abs().max().item()),
               "wall_max": wall, "n_bad": n_bad, "n_bad_single": float((st1 != 1).sum().item()),
               "it_mean": it_mean, "it_mean_single": float(it1.double().mean().item()), "G": G}
        with open(os.path.join(outdir, "dist_result.json"), "w") as fh:
            json.dump(res, fh)
    d.barrier()
    d.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4] == "strong")

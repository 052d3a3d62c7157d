"""One rank of tests/test_gpu_rccl.py: an RCCL ("nccl") process group on
cuda:LOCAL_RANK and the bench's collectives (dist.reduce_stats, gather_stats,
gather_outputs) on device tensors; writes the results as JSON."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as tdist  # noqa: E402

from dyros_robot_controller_amd import dist as ddist  # noqa: E402

out_dir = sys.argv[1]
rank, world, local = ddist.env_rank()
dev = torch.device("cuda", local)
torch.cuda.set_device(dev)
ddist.init("nccl", dev)
wall, n_bad, it_mean = ddist.reduce_stats(0.5 + rank, 3.0 + rank, 8.0 + rank, world, dev)
rows = ddist.gather_stats([rank, 1.5, 2.5], world, dev)
loc = torch.arange(6, dtype=torch.float64, device=dev).reshape(2, 3) + 100 * rank
full = ddist.gather_outputs(loc, [3] * world, world)
try:
    ver = ".".join(str(v) for v in torch.cuda.nccl.version())
except Exception:  # (a build without the version query)
    ver = None
res = {"backend": tdist.get_backend(), "world": tdist.get_world_size(), "wall": wall, "n_bad": n_bad,
       "it_mean": it_mean, "rows": rows.tolist(), "full": full.cpu().tolist(), "device": str(full.device),
       "rccl_version": ver}
tdist.barrier()
tdist.destroy_process_group()
if rank == 0:
    with open(os.path.join(out_dir, "rccl_result.json"), "w") as fh:
        json.dump(res, fh)

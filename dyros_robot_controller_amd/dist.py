"""Multi-GPU plumbing for the batched QP-IK.

Instances are independent, so the batch shards across ranks as contiguous
instance ranges with no data-path collective: one process per GPU, rank r
owns instances [r * B, (r + 1) * B) of the global batch (weak scaling, B per
rank).  The only collectives are the benchmark's barrier and the reduction
of its timing / status counters (max of the timed region, sums of counts).
torch.distributed is the transport: "nccl" (RCCL over xGMI) on the GPUs,
"gloo" for the CPU tests.
"""
import os


def env_rank():
    """(rank, world_size, local_rank) from the torchrun environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend, device=None):
    """Initialise the process group from the environment (127.0.0.1 rendezvous)."""
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if device is not None:
        dist.init_process_group(backend, device_id=device)
    else:
        dist.init_process_group(backend)
    return dist


def shard(rank, per_rank):
    """Global instance offset and count of ``rank`` (contiguous ranges)."""
    return rank * per_rank, per_rank


def shard_global(rank, world, global_batch):
    """Strong scaling: ``rank``'s contiguous range [r G / W, (r + 1) G / W) of a
    fixed global batch G (SURVEY §8e partitioning).  Returns (offset, count)."""
    lo = rank * global_batch // world
    hi = (rank + 1) * global_batch // world
    return lo, hi - lo


def gather_outputs(local, counts, world):
    """Optional epilogue: all-gather every rank's [F][B_r] output
    block into one [F][sum B_r] tensor on each rank (instance order = rank
    order).  Blocks are padded to the largest shard for the collective."""
    import torch
    if world == 1:
        return local
    import torch.distributed as dist
    F, Bmax = local.shape[0], max(counts)
    pad = torch.zeros((F, Bmax), dtype=local.dtype, device=local.device)
    pad[:, :local.shape[1]] = local
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad)
    return torch.cat([p[:, :c] for p, c in zip(parts, counts)], dim=1)


def reduce_stats(wall_s, n_bad, iters_mean, world, device="cpu"):
    """Whole-job timing and counters: max wall time over ranks (the job ends
    with the slowest rank), sum of non-solved instances, mean of the per-rank
    mean ADMM iterations.  Returns plain floats."""
    import torch
    t = torch.tensor([float(wall_s), float(n_bad), float(iters_mean)], dtype=torch.float64, device=device)
    if world > 1:
        import torch.distributed as dist
        mx = t[:1].clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = t[1:].clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        return mx.item(), sm[0].item(), sm[1].item() / world
    return t[0].item(), t[1].item(), t[2].item()

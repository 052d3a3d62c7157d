"""Multi-GPU plumbing for the batched QP-IK.

Instances are independent, so the batch shards across ranks as contiguous
instance ranges with no data-path collective: one process per GPU, rank r
owns instances [r * B, (r + 1) * B) of the global batch (weak scaling, B per
rank).  The only collectives are the benchmark's barrier and the reduction
of its timing / status counters (max of the timed region, sums of counts).
torch.distributed is the transport: "nccl" (RCCL over xGMI) on the GPUs,
"gloo" for the CPU tests.  ``bench.py --gpus N`` run without torchrun starts
its N ranks itself (``launch_if_needed``).
"""
import os
import socket
import subprocess
import sys
import time


def free_port():
    """An unused TCP port on 127.0.0.1 for the rendezvous."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n, argv, extra_env=None, poll_s=0.2, timeout_s=None):
    """Launch ``n`` ranks of ``argv`` (one process per GPU, as torchrun would:
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set)
    and wait for them.  The caller must not have touched the GPU: the ranks are
    fresh child processes (fork + exec of a new interpreter), never an exec of
    the caller.  When one rank fails, the others are terminated (by their own
    PIDs) so none is left waiting in a collective; so are all of them when
    ``timeout_s`` elapses (return value 124, as timeout(1)) or when the parent
    is interrupted (the children never outlive this call).  The rendezvous
    port is chosen free just before the launch; should another process take
    it in between, the ranks fail to bind and the call returns their error.
    Returns the first non-zero exit status, or 0."""
    port = free_port()
    procs = []
    rc = 0
    t_end = None if timeout_s is None else time.monotonic() + timeout_s
    try:
        for r in range(n):
            env = dict(os.environ)
            env.update(extra_env or {})
            env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            procs.append(subprocess.Popen(argv, env=env))
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for o in live:
                        o.terminate()
            if live and t_end is not None and time.monotonic() > t_end:
                rc = rc or 124
                for o in live:
                    o.kill()
                break
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    return rc


def launch_if_needed(n_gpus, script, args):
    """bench.py's launcher: when ``--gpus N`` > 1 and no torchrun environment is
    present, run N ranks of ``script`` with the same arguments and return their
    exit status; None when this process is already a rank (or N = 1).  Raises
    when the torchrun world size contradicts ``--gpus``."""
    world = os.environ.get("WORLD_SIZE")
    if world is not None:
        if int(world) != n_gpus:
            raise SystemExit("bench: --gpus %d but WORLD_SIZE=%s" % (n_gpus, world))
        return None
    if n_gpus <= 1:
        return None
    return spawn_ranks(n_gpus, [sys.executable, "-u", script] + list(args))


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


def _group(world):
    """True when the collectives run: several ranks, or a process group that
    exists (a one-rank RCCL group runs the same code path: tests/test_gpu_rccl.py)."""
    if world > 1:
        return True
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


def gather_outputs(local, counts, world):
    """Optional epilogue: all-gather every rank's [F][B_r] output
    block into one [F][sum B_r] tensor on each rank (instance order = rank
    order).  Blocks are padded to the largest shard for the collective."""
    import torch
    if not _group(world):
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
    if _group(world):
        import torch.distributed as dist
        mx = t[:1].clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = t[1:].clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        return mx.item(), sm[0].item(), sm[1].item() / world
    return t[0].item(), t[1].item(), t[2].item()


def gather_stats(values, world, device="cpu"):
    """Every rank's vector of floats (same length on every rank), gathered:
    a [world][k] numpy array in rank order on every rank (one all-gather of
    world x k doubles; the bench's per-rank device ids, iteration
    percentiles and tier counts)."""
    import numpy as np
    import torch
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    if not _group(world):
        return t.cpu().numpy()[None, :]
    import torch.distributed as dist
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return np.stack([p.cpu().numpy() for p in parts])

"""bench.py's N-rank launch (VERDICT r02 "do this" #1) on the CPU:
``python bench.py --gpus N`` without a torchrun environment starts N ranks
itself (dist.launch_if_needed -> dist.spawn_ranks), each rank initialises the
process group (gloo here), takes its contiguous shard and joins the same
max / sum reduction the GPU bench uses.  ``--dry-run`` stops before any GPU
work, so the launcher, the rendezvous, the sharding and the reduction are
what is tested."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, drop=("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")):
    env = {k: v for k, v in os.environ.items() if k not in drop}
    env["DRC_DIST_BACKEND"] = "gloo"
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=240)
    return p


def _line(p):
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout        # rank 0 alone prints
    return json.loads(lines[0])


def test_gpus_2_launches_two_ranks_weak():
    d = _line(_run(["--gpus", "2", "--dry-run"]))
    assert d["n_gpus"] == 2 and d["ranks_reporting"] == 2
    assert d["instances"] == 2 * 65536                # weak: 65 536 per rank
    assert d["max_wall"] == 0.002                     # max over ranks of 0.001 * (rank + 1)
    assert d["mean_offset"] == 65536 / 2              # rank offsets 0 and 65 536


def test_gpus_3_strong_scaling_global_batch():
    d = _line(_run(["--gpus", "3", "--robot", "xls_fr3", "--global-batch", "23", "--dry-run"]))
    assert d["n_gpus"] == 3 and d["instances"] == 23  # [0, 7) [7, 15) [15, 23)
    assert abs(d["mean_offset"] - (0 + 7 + 15) / 3) < 1e-12


def test_single_gpu_runs_in_process():
    d = _line(_run(["--dry-run"]))
    assert d["n_gpus"] == 1 and d["instances"] == 65536


def test_world_size_must_match_gpus():
    p = _run(["--gpus", "2", "--dry-run"], env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"}, drop=())
    assert p.returncode != 0 and "WORLD_SIZE" in p.stderr

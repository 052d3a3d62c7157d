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
    # whole-job fields (bench.whole_job): iteration p99 / max are maxima over
    # ranks, tier counts sums, one row per rank, and the transport
    assert d["admm_iters_p99_max"] == [2.0, 20]
    assert d["stress_tiers"] == {"collision": 1, "singular": 2}
    assert [r["rank"] for r in d["ranks"]] == [0, 1] and [r["instances"] for r in d["ranks"]] == [65536, 65536]
    assert [r["non_solved"] for r in d["ranks"]] == [0, 1] and d["backend"] == "gloo"


def test_gpus_3_strong_scaling_global_batch():
    d = _line(_run(["--gpus", "3", "--robot", "xls_fr3", "--global-batch", "23", "--dry-run"]))
    assert d["n_gpus"] == 3 and d["instances"] == 23  # [0, 7) [7, 15) [15, 23)
    assert abs(d["mean_offset"] - (0 + 7 + 15) / 3) < 1e-12
    assert d["admm_iters_p99_max"] == [3.0, 30] and d["stress_tiers"] == {"collision": 3, "singular": 6}
    assert [r["instances"] for r in d["ranks"]] == [7, 8, 8]


def test_single_gpu_runs_in_process():
    d = _line(_run(["--dry-run"]))
    assert d["n_gpus"] == 1 and d["instances"] == 65536
    assert "ranks" not in d and d["admm_iters_p99_max"] == [1.0, 10]


def test_world_size_must_match_gpus():
    p = _run(["--gpus", "2", "--dry-run"], env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"}, drop=())
    assert p.returncode != 0 and "WORLD_SIZE" in p.stderr


def test_algorithmic_flop_count():
    """bench.py's roofline FLOPs come from the counting build of the oracle
    (pruned narrow phase): positive, reproducible, and the pruned search does
    less work than the all-pairs loop on the same sample."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import bench
    import oracle as O
    from dyros_robot_controller_amd import workload
    pm, om, spec = O.load("fr3")
    q, qd = workload.joint_states(pm.lower, pm.upper, pm.vel, 3, 64)
    xt = np.stack([O.fk_pose(om, q[:, b])[0] for b in range(64)], 1)
    xt[9:] += 0.01
    xdt = np.zeros((6, 64))
    a = bench.algorithmic_flops("fr3", "exact", q, qd, xt, xdt, n=16)
    b = bench.algorithmic_flops("fr3", "exact", q, qd, xt, xdt, n=16)
    assert a == b and a["flops_per_solve"] > 1e4
    par = O.default_params(spec["kind"], exact=True)
    idx = np.unique(np.linspace(0, 63, 16).astype(np.int64))
    with O.counting_build():
        O.flop_counts(reset=True)
        O.qpik_batch(om, par, *[np.ascontiguousarray(v[:, idx]) for v in (q, qd, xt, xdt)])
        full, _ = O.flop_counts(reset=True)
    assert a["flops_per_solve"] < full / len(idx)
    # the nonzero-operand count excludes the dense restatement's structural zeros
    assert a["flops_per_solve"] < 0.5 * a["dense_flops_per_solve"]


def test_valu_issue_roof():
    """roofline.valu_issue_roof: SIMDs x clock over the counted issue cycles,
    scaled by the job's GPUs, and absent without a count."""
    import bench
    r = bench.valu_issue_roof({"valu_issue_cycles_per_solve": 41084.0, "valu_insts_per_solve": 15194.0}, 22.32e6)
    assert abs(r["solves_per_s"] - 1024 * 2.4e9 / 41084.0) < 1.0
    assert abs(r["frac"] - 22.32e6 / r["solves_per_s"]) < 1e-12
    r8 = bench.valu_issue_roof({"valu_issue_cycles_per_solve": 41084.0}, 8 * 22.32e6, 8)
    assert abs(r8["frac"] - r["frac"]) < 1e-12
    assert bench.valu_issue_roof({}, 1.0) is None

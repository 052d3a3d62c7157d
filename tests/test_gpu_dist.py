"""The multi-rank path on the product kernels: two ranks on the
box's one GPU (gloo transport: RCCL needs one GPU per rank), each solving its
contiguous shard with drc_qpik_batch.  The gathered batch must equal a
single-process run over the whole range bit for bit (instances are
independent and their inputs are keyed by the instance, not the shard), and
reduce_stats must reduce device tensors: max of the per-rank walls, sum of
non-solved counts, mean of the per-rank mean iterations."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.parametrize("robot,per_rank,mode", [("fr3", 384, "weak"), ("xls_fr3", 257, "strong"),
                                                 ("fr3", 8500, "weak")])
def test_two_ranks_match_single_process(tmp_path, robot, per_rank, mode):
    """(fr3, 8500): each rank's shard runs the fused kernel (FR3: B <= 16 384),
    the single-process run of the whole 17 000 the sub-batch pipeline; the
    bit-identity contract holds across that threshold."""
    sys.path.insert(0, ROOT)
    from dyros_robot_controller_amd import dist as ddist
    rc = ddist.spawn_ranks(2, [sys.executable, "-u", os.path.join(ROOT, "tests", "_dist_gpu_worker.py"),
                               str(tmp_path), robot, str(per_rank), mode],
                           extra_env={"DRC_DIST_BACKEND": "gloo"}, timeout_s=100)
    assert rc == 0
    with open(tmp_path / "dist_result.json") as fh:
        r = json.load(fh)
    assert r["device"].startswith("cuda")
    assert r["inputs_equal"]
    assert r["bitwise_equal"], r["max_abs"]
    assert r["wall_max"] == 2.0
    assert r["n_bad"] == r["n_bad_single"]
    # per-rank means averaged: equal shards (weak) give the global mean exactly
    if mode == "weak":
        assert abs(r["it_mean"] - r["it_mean_single"]) < 1e-9

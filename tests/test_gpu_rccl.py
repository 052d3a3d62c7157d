"""RCCL on the MI355X: the bench's multi-GPU collectives (dist.reduce_stats,
gather_stats, gather_outputs) through a one-rank "nccl" (= RCCL)
process group on device tensors -- the code path every rank of the driver's
8-GPU run takes (the boxes here hold one GPU, and RCCL, like NCCL, admits one
rank per device, so two ranks cannot share it; tests/test_gpu_dist.py runs
two ranks on one GPU over gloo).  Checks that the group initialises with the
device id, that the reductions and all-gathers return the single rank's
values on the device, and that the process group tears down cleanly."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_rccl_one_rank_collectives(tmp_path):
    sys.path.insert(0, ROOT)
    from dyros_robot_controller_amd import dist as ddist
    rc = ddist.spawn_ranks(1, [sys.executable, "-u", os.path.join(ROOT, "tests", "_rccl_worker.py"), str(tmp_path)],
                           timeout_s=120)
    assert rc == 0
    with open(tmp_path / "rccl_result.json") as fh:
        r = json.load(fh)
    assert r["backend"] == "nccl" and r["world"] == 1
    assert r["wall"] == 0.5 and r["n_bad"] == 3.0 and r["it_mean"] == 8.0
    assert r["rows"] == [[0.0, 1.5, 2.5]]
    assert r["full"] == [[0.0, 1.0, 2.0], [3.0, 4.0, 5.0]]
    assert r["device"].startswith("cuda")

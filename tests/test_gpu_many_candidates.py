"""A model whose GJK candidate list is longer than the EPA seed stash's offset
(ADVICE r05, medium): the task kernel compacts the candidate pairs into an
LDS int list, and the candidate GJKs stash the simplices of the first
intersecting pairs for EPA (qpik_device.hpp epa_stash) while later
candidates are still being read from that list.  With the list laid over the
polytope's vertex slots, a list longer than 336 entries was overwritten by
the stash; api.cpp now places it in the face planes, which EPA writes only
after the last candidate is consumed (static_asserts there).

The model: a 6-joint chain whose links carry 6 boxes each around the chain's
axis (36 boxes, 540 pairs with different parent joints, no SRDF).  Boxes
have no closed form, so every pair is a GJK candidate (the broad phase's
upper bound stays +inf): 540 > 336 candidates per instance, many of them
intersecting.  The device's min self-distance must match the oracle's on
every instance (GJK / EPA tolerances of tests/test_gpu_parity.py)."""
import os

import numpy as np
import pytest

import oracle as O
from dyros_robot_controller_amd import _batch, _capi, manipulator

pytestmark = pytest.mark.gpu


def tangle_urdf(path, n_joints=6, boxes=6, seed=5):
    rng = np.random.default_rng(seed)
    out = ['<?xml version="1.0"?>', '<robot name="tangle">', '  <link name="base"/>']
    parent = "base"
    for j in range(1, n_joints + 1):
        link = "link%d" % j
        out.append('  <link name="%s">' % link)
        out.append('    <inertial><origin xyz="0 0 0.05"/><mass value="1.0"/>'
                   '<inertia ixx="0.01" iyy="0.01" izz="0.01" ixy="0" ixz="0" iyz="0"/></inertial>')
        for _ in range(boxes):
            c = rng.uniform(-0.06, 0.06, 3)
            r = rng.uniform(-np.pi, np.pi, 3)
            h = rng.uniform(0.02, 0.05, 3)
            out.append('    <collision><origin xyz="%.6f %.6f %.6f" rpy="%.6f %.6f %.6f"/>'
                       '<geometry><box size="%.6f %.6f %.6f"/></geometry></collision>' % (*c, *r, *(2 * h)))
        out.append('  </link>')
        axis = ["0 0 1", "0 1 0", "1 0 0"][j % 3]
        out.append('  <joint name="joint%d" type="revolute"><parent link="%s"/><child link="%s"/>'
                   '<origin xyz="0 0 0.03" rpy="0 0 0"/><axis xyz="%s"/>'
                   '<limit lower="-2.5" upper="2.5" velocity="2.0" effort="50"/></joint>' % (j, parent, link, axis))
        parent = link
    out.append('</robot>')
    with open(path, "w") as fh:
        fh.write("\n".join(out) + "\n")


def test_candidate_list_longer_than_stash_offset(cuda, tmp_path):
    urdf = str(tmp_path / "tangle.urdf")
    tangle_urdf(urdf)
    rd = manipulator.RobotData(urdf, "", device=cuda)
    assert rd.model.n_geoms == 36 and rd.model.n_pairs == 540
    pm, om, _ = O.load_paths(urdf, None, dict(ee="link6", kind=0))
    assert om.npairs == 540 and all(g["type"] == 2 for g in pm.geoms)   # boxes only: no closed form
    B = 64
    rng = np.random.default_rng(11)
    q = rng.uniform(-2.4, 2.4, (6, B))
    qd = np.zeros((6, B))
    pb = manipulator.QPIKParamsBuilder(rd.model, exact=True)
    p = pb.params("link6", _capi.MODE_QPIK)
    st = _batch.stages_batch(rd.model, p, _batch.as_device(q, cuda), _batch.as_device(qd, cuda), None,
                             _batch.as_device(np.zeros((6, B)), cuda))
    dist = st["dist"].cpu().numpy()
    pen = 0
    for b in range(B):
        d, g, _ = O.min_distance(om, q[:, b])
        pen += d < 0
        assert abs(dist[0, b] - d) <= (2e-6 if d < 0 else 1e-9), (b, dist[0, b], d)
    assert pen >= B // 2, pen          # the stash is written: intersecting candidates on most instances

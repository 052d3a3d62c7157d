"""Pins the one artefact the reference holds for the hot path: its FR3 model
(/root/reference/examples/robots/fr3/fr3.{urdf,srdf}).  The bundled fixture
(dyros_robot_controller_amd/robots/fr3, re-serialised by tools/gen_robots.py)
must describe the same robot: joint tree, placements, axes, limits,
inertias, the 35 collision primitives and the 180 active pairs that
Manipulator::RobotData builds (src/manipulator/robot_data.cpp:21-62).  Both
files go through the same parser (oracle/pyref_model.py).  Skipped where the
reference tree is absent (the GPU box)."""
import os

import numpy as np
import pytest

import pyref_model
from dyros_robot_controller_amd import robot_path

REF = "/root/reference/examples/robots/fr3"


@pytest.mark.skipif(not os.path.exists(os.path.join(REF, "fr3.urdf")), reason="reference tree absent")
def test_bundled_fr3_equals_reference_model():
    ref = pyref_model.load_urdf(os.path.join(REF, "fr3.urdf"), os.path.join(REF, "fr3.srdf"))
    ours = pyref_model.load_urdf(robot_path("fr3"), robot_path("fr3", "srdf"))
    assert ours.nv == ref.nv == 7
    assert ours.jname == ref.jname and ours.jtype == ref.jtype and ours.jparent == ref.jparent
    for a, b in zip(ours.jplacement, ref.jplacement):
        np.testing.assert_allclose(a, b, atol=1e-12)
    for a, b in zip(ours.jaxis, ref.jaxis):
        np.testing.assert_allclose(a, b, atol=1e-12)
    for f in ("lower", "upper", "vel", "effort"):
        np.testing.assert_allclose(getattr(ours, f), getattr(ref, f), atol=1e-12)
    assert len(ours.inertia) == len(ref.inertia)
    for a, b in zip(ours.inertia, ref.inertia):
        assert len(a) == len(b)
        for (ma, ca, Ia), (mb, cb, Ib) in zip(a, b):   # (mass, com, inertia about com) per body
            assert abs(ma - mb) <= 1e-12
            np.testing.assert_allclose(ca, cb, atol=1e-12)
            np.testing.assert_allclose(Ia, Ib, atol=1e-12)
    assert len(ours.geoms) == len(ref.geoms) == 35
    for g, h in zip(ours.geoms, ref.geoms):
        assert (g["parent_joint"], g["type"]) == (h["parent_joint"], h["type"])
        np.testing.assert_allclose(g["placement"], h["placement"], atol=1e-12)
        np.testing.assert_allclose(g["params"], h["params"], atol=1e-12)
    assert len(ours.pairs) == len(ref.pairs) == 180
    assert ours.pairs == ref.pairs
    assert set(ours.frames) >= {"fr3_link8"}
    np.testing.assert_allclose(ours.frames["fr3_link8"][1], ref.frames["fr3_link8"][1], atol=1e-12)
    assert ours.frames["fr3_link8"][0] == ref.frames["fr3_link8"][0]

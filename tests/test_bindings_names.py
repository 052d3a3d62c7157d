"""The pybind11 module dyros_robot_controller_cpp_wrapper registers every class
and method name of the reference's Boost.Python module (src/bindings.cpp:219-447;
tests/golden/bindings_names.json, written by tools/gen_binding_names.py), and the
reference's own drc/ Python package imports and runs on top of it unchanged
(drc/__init__.py -> drc.mobile / drc.manipulator / drc.mobile_manipulator, which
subclass the module's classes).  The mobile-base classes are host arithmetic,
so they run here without a GPU; the model classes need one (tests -m gpu)."""
import importlib
import json
import os
import sys

import numpy as np
import pytest

import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_DRC = "/root/reference"
GOLDEN = os.path.join(ROOT, "tests", "golden", "bindings_names.json")


@pytest.fixture(scope="module")
def wrapper():
    sys.path.insert(0, os.path.join(ROOT, "dyros_robot_controller_amd", "python"))
    return importlib.import_module("dyros_robot_controller_cpp_wrapper")


def test_every_reference_name_is_registered(wrapper):
    names = json.load(open(GOLDEN))
    missing = [(c, n) for c, ms in names.items() for n in [None] + ms
               if not hasattr(wrapper, c) or (n and not hasattr(getattr(wrapper, c), n))]
    assert not missing, missing
    for v in ("Differential", "Mecanum", "Caster"):
        assert int(getattr(wrapper, v)) == int(getattr(wrapper.DriveType, v))
    # bases<ManipulatorRobotData, MobileRobotData> (bindings.cpp:334)
    assert issubclass(wrapper.MobileManipulatorRobotData, wrapper.ManipulatorRobotData)
    assert issubclass(wrapper.MobileManipulatorRobotData, wrapper.MobileRobotData)


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "..", "reference", "src", "bindings.cpp"))
                    and not os.path.exists("/root/reference/src/bindings.cpp"), reason="reference tree absent")
def test_golden_names_match_reference_source():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import gen_binding_names
    assert gen_binding_names.parse("/root/reference/src/bindings.cpp") == json.load(open(GOLDEN))


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF_DRC, "drc")), reason="reference drc package absent")
def test_reference_drc_package_runs_on_this_module(wrapper):
    sys.path.insert(0, REF_DRC)
    try:
        import drc
        import drc.mobile
    finally:
        sys.path.remove(REF_DRC)
    assert issubclass(drc.mobile.RobotData, wrapper.MobileRobotData)
    assert issubclass(drc.manipulator.RobotData, wrapper.ManipulatorRobotData)
    assert issubclass(drc.mobile_manipulator.RobotData, wrapper.MobileManipulatorRobotData)
    assert issubclass(drc.mobile_manipulator.RobotController, wrapper.MobileManipulatorRobotController)
    # caster base through the reference's own Python classes
    c = O.CASTER_FR3
    kp = drc.KinematicParam(drc.DriveType.Caster, c["radius"], base2wheel_positions=[np.array(p) for p in c["positions"]],
                            wheel_offset=c["offset"])
    rd = drc.mobile.RobotData(kp)
    assert rd.get_wheel_num() == 4
    wp = np.array([0.3, 1.1, -0.7, 0.2])
    np.testing.assert_allclose(rd.compute_fk_jacobian(wp), O.ROBOTS["caster_fr3"]["J_mobile"](wp), atol=1e-12)
    wv = np.array([0.5, -1.0, 0.25, 2.0])
    assert rd.update_state(wp, wv)
    np.testing.assert_allclose(rd.get_base_vel(), O.ROBOTS["caster_fr3"]["J_mobile"](wp) @ wv, atol=1e-12)
    ctrl = drc.mobile.RobotController(0.001, rd)
    J = ctrl.compute_IK_jacobian()
    assert J.shape == (4, 3)
    np.testing.assert_allclose(ctrl.compute_wheel_vel(np.array([0.1, 0.2, 0.3])), J @ [0.1, 0.2, 0.3], atol=1e-12)
    # VelocityCommand saturates |v| at max_lin_speed (2.0) and |w| at max_ang_speed
    v = ctrl.velocity_command(np.array([3.0, 4.0, -5.0]))
    np.testing.assert_allclose(v, J @ [1.2, 1.6, -2.0], atol=1e-12)
    # mecanum: the FK Jacobian is PinvCOD of the IK map
    mk = drc.KinematicParam(drc.DriveType.Mecanum, 0.12, roller_angles=[-np.pi / 4, np.pi / 4, np.pi / 4, -np.pi / 4],
                            base2wheel_positions=[np.array([0.2225, 0.2045]), np.array([0.2225, -0.2045]),
                                                  np.array([-0.2225, 0.2045]), np.array([-0.2225, -0.2045])],
                            base2wheel_angles=[0, 0, 0, 0])
    mr = drc.mobile.RobotData(mk)
    np.testing.assert_allclose(mr.compute_fk_jacobian(np.zeros(4)), O.ROBOTS["xls_fr3"]["J_mobile"](), atol=1e-12)

"""C++ facade (include/drc_amd.hpp) and the pybind11 module with the
reference's module/class names (dyros_robot_controller_cpp_wrapper,
src/bindings.cpp:219-447).

CPU part: the module imports and exposes the reference's names; a C++
program using the facade compiles against the headers and links the HIP
library.  GPU part: the module's single-instance QPIKStep and its batched
form agree with the oracle, and calling it the way the reference's drc/
Python layer does (subclassing the classes) works."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PYDIR = os.path.join(ROOT, "dyros_robot_controller_amd", "python")

REFERENCE_NAMES = ["DriveType", "KinematicParam", "JointIndex", "ActuatorIndex", "MinDistResult",
                   "ManipulabilityResult", "ManipulatorRobotData", "ManipulatorRobotController",
                   "MobileManipulatorRobotData", "MobileManipulatorRobotController"]
METHODS = {
    "ManipulatorRobotData": ["getVerbose", "updateState", "getDof", "computePose", "computeJacobian", "getPose",
                             "getJacobian", "getVelocity", "getManipulability", "getMinDistance",
                             "getJointPositionLimit", "getJointVelocityLimit"],
    "ManipulatorRobotController": ["setTaskGain", "setTaskKpGain", "setTaskKvGain", "QPIK", "QPIKStep", "QPIKCubic",
                                   "QPIKBatch", "QPIKStepBatch", "QPIKCubicBatch", "QPID", "QPIDStep", "QPIDCubic",
                                   "QPIDBatch", "QPIDStepBatch", "QPIDCubicBatch", "CLIKStep", "CLIKCubic",
                                   "OSF", "OSFStep", "OSFCubic"],
    "MobileManipulatorRobotData": ["getVerbose", "updateState", "getDof", "getActuatorDof", "getManipulatorDof",
                                   "getMobileDof", "getJointIndex", "getActuatorIndex", "getMobileFKJacobian",
                                   "getMinDistance"],
    "MobileManipulatorRobotController": ["setTaskGain", "QPIK", "QPIKStep", "QPIKCubic", "QPIKStepBatch",
                                         "QPID", "QPIDStep", "QPIDCubic", "QPIDStepBatch"],
}


def _module():
    if PYDIR not in sys.path:
        sys.path.insert(0, PYDIR)
    import dyros_robot_controller_cpp_wrapper as drc
    return drc


def test_module_exposes_reference_names():
    drc = _module()
    for n in REFERENCE_NAMES:
        assert hasattr(drc, n), n
    for cls, ms in METHODS.items():
        for m in ms:
            assert hasattr(getattr(drc, cls), m), (cls, m)
    assert int(drc.DriveType.Differential) == 0 and int(drc.DriveType.Mecanum) == 1
    p = drc.KinematicParam()
    p.type = drc.DriveType.Mecanum
    p.base2wheel_positions = [[0.2, 0.1], [0.2, -0.1]]
    assert p.base2wheel_positions[1] == [0.2, -0.1]


def test_cpp_facade_compiles_and_links(tmp_path):
    src = tmp_path / "use_facade.cpp"
    src.write_text('''
#include "drc_amd.hpp"
#include <memory>
int main(int argc, char** argv) {
  if (argc < 3) return 0;  // link check only without a GPU
  auto rd = std::make_shared<drc_amd::Manipulator::RobotData>(argv[1], argv[2]);
  drc_amd::Manipulator::RobotController rc(0.001, rd);
  rd->updateState(drc_amd::Vec(rd->getDof(), 0.1), drc_amd::Vec(rd->getDof(), 0.0));
  drc_amd::Pose x = rd->getPose("fr3_link8");
  x[12] += 0.01;
  drc_amd::Vec qd = rc.QPIKStep(x, drc_amd::Vec(6, 0.0), "fr3_link8");
  return qd.size() == static_cast<size_t>(rd->getDof()) ? 0 : 1;
}
''')
    exe = tmp_path / "use_facade"
    lib = os.path.join(ROOT, "dyros_robot_controller_amd")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-I" + os.path.join(ROOT, "include"), str(src), "-o", str(exe),
                           "-L" + lib, "-ldrc_amd", "-Wl,-rpath," + lib])
    subprocess.check_call([str(exe)])


EIGEN_CALL_SITE = r'''
// Reference-style call site (examples/C++/src/fr3_controller.cpp:15-134):
// namespace drc, Eigen types, shared_ptr construction, the same calls.
#include "drc_amd_eigen.hpp"
#include <cmath>
#include <cstdio>
#include <memory>
int main(int argc, char** argv) {
  if (argc < 3) return 0;  // link check only without a GPU
  auto robot_data_ = std::make_shared<drc::Manipulator::RobotData>(argv[1], argv[2]);
  auto robot_controller_ = std::make_shared<drc::Manipulator::RobotController>(0.001, robot_data_);
  const int dof_ = robot_data_->getDof();
  Eigen::VectorXd q_ = Eigen::VectorXd::Constant(dof_, 0.1), qdot_ = Eigen::VectorXd::Zero(dof_);
  robot_data_->updateState(q_, qdot_);
  Eigen::Affine3d x_ = robot_data_->getPose("fr3_link8");
  Eigen::VectorXd xdot_ = robot_data_->getVelocity("fr3_link8");
  Eigen::Affine3d target_x = x_;
  target_x.matrix()(0, 3) += 0.02;
  Eigen::VectorXd qdot_desired_ = robot_controller_->QPIKCubic(target_x, Eigen::VectorXd::Zero(6), x_, xdot_,
                                                               0.5, 0.0, 1.0, "fr3_link8");
  Eigen::VectorXd tau_desired_ = robot_controller_->moveJointTorqueStep(q_, qdot_desired_);
  Eigen::MatrixXd J = robot_data_->getJacobian("fr3_link8");
  // the Eigen layer returns what the std:: facade returns
  drc_amd::Pose xt = drc::eigen_detail::pose(target_x);
  drc_amd::Vec ref = robot_controller_->impl().QPIKCubic(xt, drc_amd::Vec(6, 0.0), drc::eigen_detail::pose(x_),
                                                         drc::eigen_detail::vec(xdot_), 0.5, 0.0, 1.0, "fr3_link8");
  double err = 0;
  for (int i = 0; i < dof_; ++i) err = std::fmax(err, std::fabs(qdot_desired_(i) - ref[i]));
  // the QP layer driven directly (manipulator/QP_IK.h:31-38, QP_base.h:19-43):
  // the same optimum as the controller's QPIK, stage times filled
  drc::Manipulator::QPIK qp(robot_data_);
  Eigen::VectorXd xd = Eigen::VectorXd::Zero(6);
  xd(0) = 0.05;
  qp.setDesiredTaskVel(xd, "fr3_link8");
  Eigen::VectorXd qd_qp;
  drc::QP::TimeDuration ts;
  const bool ok = qp.getOptJointVel(qd_qp, ts);
  Eigen::VectorXd qd_rc = robot_controller_->QPIK(xd, "fr3_link8");
  double err2 = 0;
  for (int i = 0; i < dof_; ++i) err2 = std::fmax(err2, std::fabs(qd_qp(i) - qd_rc(i)));
  const bool times = ts.set_ineq > 0 && ts.set_constraint > 0 && ts.set_solver > 0 && ts.solve_qp > 0 &&
                     std::fabs(ts.set_qp - ts.set_ineq - ts.set_constraint) < 1e-15 && ts.set_ineq < 0.1;
  std::printf("%d %d %ld %ld %.3e %d %.3e %.2e %.2e %.2e %.2e\n", (int)qdot_desired_.size(), (int)tau_desired_.size(),
              (long)J.rows(), (long)J.cols(), err, (int)ok, err2, ts.set_ineq, ts.set_constraint, ts.set_solver,
              ts.solve_qp);
  return (qdot_desired_.size() == dof_ && tau_desired_.size() == dof_ && J.rows() == 6 && J.cols() == dof_ &&
          err == 0.0 && ok && err2 == 0.0 && times) ? 0 : 1;
}
'''


def _build_eigen_call_site(tmp_path):
    src = tmp_path / "eigen_call_site.cpp"
    src.write_text(EIGEN_CALL_SITE)
    exe = tmp_path / "eigen_call_site"
    lib = os.path.join(ROOT, "dyros_robot_controller_amd")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-I" + os.path.join(ROOT, "include"),
                           "-I" + os.path.join(ROOT, "tests", "mock_eigen"), str(src), "-o", str(exe),
                           "-L" + lib, "-ldrc_amd", "-Wl,-rpath," + lib])
    return exe


def test_eigen_layer_compiles_reference_call_site(tmp_path):
    """include/drc_amd_eigen.hpp keeps the reference's namespace and Eigen
    signatures (Weak #11): a call site shaped like fr3_controller.cpp
    compiles and links (against a test stand-in for Eigen's types)."""
    exe = _build_eigen_call_site(tmp_path)
    subprocess.check_call([str(exe)])


@pytest.mark.gpu
def test_eigen_layer_runs(cuda, tmp_path):
    from dyros_robot_controller_amd import robot_path
    exe = _build_eigen_call_site(tmp_path)
    r = subprocess.run([str(exe), robot_path("fr3"), robot_path("fr3", "srdf")], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
def test_module_qpik_step_matches_oracle(cuda):
    import oracle as O
    from _common import LINK, oracle_batch, step_inputs, make_manipulator
    drc = _module()
    from dyros_robot_controller_amd import robot_path
    rd = drc.ManipulatorRobotData(robot_path("fr3"), robot_path("fr3", "srdf"), "")
    rc = drc.ManipulatorRobotController(0.001, rd)
    B = 64
    q, qd, xt, xdt = step_inputs(make_manipulator("fr3", cuda), "fr3", 4, B, cuda)
    out, status = rc.QPIKStepBatch(q, qd, xt, xdt, "fr3_link8")
    ref, rstat, _, _ = oracle_batch("fr3", q, qd, xt, xdt, exact=True)
    assert np.array_equal(status, rstat)
    assert np.median(np.abs(out - ref).max(axis=0)) <= 1e-9
    # single instance through the reference signatures (4x4 numpy pose)
    from dyros_robot_controller_amd.manipulator import pose_from12
    for b in range(4):
        assert rd.updateState(q[:, b], qd[:, b])
        v = rc.QPIKStep(pose_from12(xt[:, b]), xdt[:, b], "fr3_link8")
        np.testing.assert_allclose(v, out[:, b], atol=1e-12)
    T = rd.getPose("fr3_link8")
    pose, _ = O.fk_pose(O.load("fr3")[1], q[:, 3])
    np.testing.assert_allclose(T[:3, :3], pose[:9].reshape(3, 3), atol=1e-12)
    md = rd.getMinDistance(True, False)
    d, dg, _ = O.min_distance(O.load("fr3")[1], q[:, 3])
    assert abs(md.distance - d) <= 1e-9


@pytest.mark.gpu
def test_reference_style_subclassing(cuda):
    """The reference's drc/manipulator/robot_data.py subclasses
    ManipulatorRobotData and calls super().__init__(urdf, srdf, packages)."""
    drc = _module()
    from dyros_robot_controller_amd import robot_path

    class RobotData(drc.ManipulatorRobotData):
        def __init__(self, urdf_path, srdf_path="", packages_path=""):
            super().__init__(urdf_path, srdf_path, packages_path)

        def get_dof(self):
            return super().getDof()

    class RobotController(drc.ManipulatorRobotController):
        def __init__(self, dt, robot_data):
            self._robot_data = robot_data
            super().__init__(dt, robot_data)

        def QPIK(self, xdot_target, link_name):
            return super().QPIK(xdot_target, link_name)

    rd = RobotData(robot_path("fr3"), robot_path("fr3", "srdf"))
    rc = RobotController(0.001, rd)
    assert rd.get_dof() == 7
    rd.updateState(np.zeros(7) + 0.1, np.zeros(7))
    assert rc.QPIK(np.zeros(6), "fr3_link8").shape == (7,)


@pytest.mark.gpu
def test_module_qpid_step_and_graddot(cuda):
    """QPIDStep (single instance and batch) through the pybind11 module, and
    getManipulability / getMinDistance with grad_dot and
    getJacobianTimeVariation, against the oracle."""
    import oracle as O
    from _common import step_inputs, make_manipulator
    from dyros_robot_controller_amd import robot_path
    from dyros_robot_controller_amd.manipulator import pose_from12
    drc = _module()
    rd = drc.ManipulatorRobotData(robot_path("fr3"), robot_path("fr3", "srdf"))
    rc = drc.ManipulatorRobotController(0.001, rd)
    q, qd, xt, xdt = step_inputs(make_manipulator("fr3", cuda), "fr3", 41, 8, cuda)
    qdd, tau, status = rc.QPIDStepBatch(q, qd, xt, xdt, "fr3_link8")
    pm, om, spec = O.load("fr3")
    par = O.default_qpid_params(0, exact=True)
    for b in range(8):
        M, g, gf = O.qpid_dynamics(pm, om, spec, q[:, b], qd[:, b])
        st, rq, rt, dg = O.qpid_one(om, par, q[:, b], qd[:, b], M, g, gf, xt[:, b], xdt[:, b])
        assert status[b] == st
        np.testing.assert_allclose(tau[:, b], rt, rtol=1e-5, atol=1e-6)
        assert rd.updateState(q[:, b], qd[:, b])
        np.testing.assert_allclose(rc.QPIDStep(pose_from12(xt[:, b]), xdt[:, b], "fr3_link8"), rt, rtol=1e-5, atol=1e-6)
        Jd, mgd, dgd = O.qpid_stages(om, q[:, b], qd[:, b])
        np.testing.assert_allclose(rd.getJacobianTimeVariation("fr3_link8"), Jd, atol=1e-10)
        mr = rd.getManipulability(True, True, "fr3_link8")
        np.testing.assert_allclose(mr.grad_dot, mgd, rtol=1e-7, atol=1e-8)
        dr = rd.getMinDistance(True, True, False)
        np.testing.assert_allclose(dr.grad_dot, dgd, atol=1e-5)


@pytest.mark.gpu
def test_module_clik_osf(cuda):
    import oracle as O
    import pyref as R
    from _common import step_inputs, make_manipulator
    from dyros_robot_controller_amd import robot_path
    from dyros_robot_controller_amd.manipulator import pose_from12
    drc = _module()
    rd = drc.ManipulatorRobotData(robot_path("fr3"), robot_path("fr3", "srdf"))
    rc = drc.ManipulatorRobotController(0.001, rd)
    q, qd, xt, xdt = step_inputs(make_manipulator("fr3", cuda), "fr3", 42, 4, cuda)
    pm, om, spec = O.load("fr3")
    par = O.default_params(0)
    for b in range(4):
        assert rd.updateState(q[:, b], qd[:, b])
        T = pose_from12(xt[:, b])
        par.mode = 1
        np.testing.assert_allclose(rc.CLIKStep(T, xdt[:, b], "fr3_link8"),
                                   O.clik_one(om, par, q[:, b], qd[:, b], xt[:, b], xdt[:, b]), rtol=1e-8, atol=1e-8)
        nu = np.linspace(-1, 1, 7)
        np.testing.assert_allclose(rc.CLIKStep(T, xdt[:, b], nu, "fr3_link8"),
                                   O.clik_one(om, par, q[:, b], qd[:, b], xt[:, b], xdt[:, b], null_qdot=nu),
                                   rtol=1e-8, atol=1e-8)
        d = R.dynamics(pm, q[:, b], qd[:, b])
        np.testing.assert_allclose(rc.OSFStep(T, xdt[:, b], nu, "fr3_link8"),
                                   O.osf_one(om, par, q[:, b], qd[:, b], d["Minv"], d["g"], xt[:, b], xdt[:, b],
                                             null_torque=nu), rtol=1e-6, atol=1e-6)


@pytest.mark.gpu
def test_module_dynamics_and_task_getters(cuda):
    """The getters/compute* the reference's drc layer calls, through the
    module, against the numpy restatement (robot_data.h:70-198)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    import pyref as R
    drc = _module()
    robot = "fr3"
    pm, om, spec = O.load(robot)
    rd = drc.ManipulatorRobotData(os.path.join(ROOT, "dyros_robot_controller_amd", "robots", "fr3", "fr3.urdf"),
                                  os.path.join(ROOT, "dyros_robot_controller_amd", "robots", "fr3", "fr3.srdf"), "")
    rng = np.random.default_rng(4)
    lo, hi = np.array(pm.lower), np.array(pm.upper)
    q, qd = rng.uniform(lo + 0.1, hi - 0.1), rng.uniform(-0.5, 0.5, 7)
    assert rd.updateState(q, qd)
    dyn = R.dynamics(pm, q, qd)
    np.testing.assert_allclose(rd.getMassMatrix(), dyn["M"], atol=1e-10)
    np.testing.assert_allclose(rd.computeMassMatrix(q), dyn["M"], atol=1e-10)
    np.testing.assert_allclose(rd.getGravity(), dyn["g"], atol=1e-10)
    np.testing.assert_allclose(rd.getNonlinearEffects(), dyn["nle"], atol=1e-10)
    np.testing.assert_allclose(rd.getCoriolis(), dyn["nle"] - dyn["g"], atol=1e-10)
    np.testing.assert_allclose(rd.getMassMatrixInv() @ rd.getMassMatrix(), np.eye(7), atol=1e-8)
    J = rd.getJacobian("fr3_link8")
    np.testing.assert_allclose(rd.computeVelocity(q, qd, "fr3_link8"), J @ qd, atol=1e-12)
    d, dg, _ = O.min_distance(om, q)
    r = rd.computeMinDistance(q, qd, True, False)
    assert abs(r.distance - d) <= 1e-9
    m, mg = O.manipulability(om, q)
    r = rd.computeManipulability(q, qd, True, False, "fr3_link8")
    assert abs(r.manipulability - m) <= 1e-10
    ctrl = drc.ManipulatorRobotController(0.001, rd)
    qdd = rng.normal(size=7)
    np.testing.assert_allclose(ctrl.moveJointTorqueStep(qdd), dyn["M"] @ qdd + dyn["g"], atol=1e-9)
    qt, qdt = q + 0.01, qd * 0.5
    np.testing.assert_allclose(ctrl.moveJointTorqueStep(qt, qdt),
                               dyn["M"] @ (400 * (qt - q) + 40 * (qdt - qd)) + dyn["g"], atol=1e-8)
    # cubic helpers at the ends of the profile
    np.testing.assert_allclose(ctrl.moveJointPositionCubic(qt, qdt, q, qd, 2.0, 0.0, 1.0), qt)
    np.testing.assert_allclose(ctrl.moveJointVelocityCubic(qt, qdt, q, qd, -1.0, 0.0, 1.0), qd)


@pytest.mark.gpu
def test_module_moma_getters(cuda):
    """MobileManipulatorRobotData's actuated quantities (robot_data.cpp:107-144,
    367-415) through the module: S, J S, S^T M S, base FK, caster base."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    import pyref as R
    drc = _module()
    robot = "caster_fr3"
    pm, om, spec = O.load(robot)
    c = O.CASTER_FR3
    kp = drc.KinematicParam()
    kp.type = drc.DriveType.Caster
    kp.wheel_radius, kp.wheel_offset = c["radius"], c["offset"]
    kp.base2wheel_positions = [list(p) for p in c["positions"]]
    ji, ai = drc.JointIndex(), drc.ActuatorIndex()
    ji.virtual_start, ji.mani_start, ji.mobi_start = spec["joint_index"]
    ai.mani_start, ai.mobi_start = spec["actuator_index"]
    base = os.path.join(ROOT, "dyros_robot_controller_amd", "robots", robot)
    rd = drc.MobileManipulatorRobotData(kp, ji, ai, os.path.join(base, robot + ".urdf"),
                                        os.path.join(base, robot + ".srdf"), "")
    rng = np.random.default_rng(9)
    qv, qm = np.array([0.3, -0.2, 0.7]), rng.uniform(-np.pi, np.pi, 4)
    lo, hi = np.array(pm.lower)[3:10], np.array(pm.upper)[3:10]
    qa = rng.uniform(lo + 0.1, hi - 0.1)
    dv, dm, da = rng.normal(size=3) * 0.1, rng.normal(size=4), rng.normal(size=7) * 0.2
    assert rd.updateState(qv, qm, qa, dv, dm, da)
    q = np.concatenate([qv, qa, qm])
    qdot = np.concatenate([dv, da, dm])
    Jm = spec["J_mobile"](qm)
    np.testing.assert_allclose(rd.getMobileFKJacobian(), Jm, atol=1e-12)
    np.testing.assert_allclose(rd.getMobileBaseVel(), Jm @ dm, atol=1e-12)
    S = R.selection_matrix(om.nv, 7, 4, spec["joint_index"], spec["actuator_index"], Jm, qv[2])
    np.testing.assert_allclose(rd.getSelectionMatrix(), S, atol=1e-12)
    np.testing.assert_allclose(rd.getJacobianActuated("fr3_link8"), rd.getJacobian("fr3_link8") @ S, atol=1e-12)
    dyn = R.dynamics(pm, q, qdot)
    np.testing.assert_allclose(rd.getMassMatrix(), dyn["M"], atol=1e-9)
    np.testing.assert_allclose(rd.getMassMatrixActuated(), S.T @ dyn["M"] @ S, atol=1e-9)
    np.testing.assert_allclose(rd.getGravityActuated(), S.T @ dyn["g"], atol=1e-9)
    np.testing.assert_allclose(rd.computeMassMatrixActuated(qv, qm, qa), S.T @ dyn["M"] @ S, atol=1e-9)
    np.testing.assert_allclose(rd.getManiJointPosition(), qa)
    np.testing.assert_allclose(rd.getJointPositionActuated(), np.concatenate([qa, qm]))
    ctrl = drc.MobileManipulatorRobotController(0.001, rd)
    qdd = rng.normal(size=7)
    np.testing.assert_allclose(ctrl.moveManipulatorJointTorqueStep(qdd),
                               dyn["M"][3:10, 3:10] @ qdd + dyn["g"][3:10], atol=1e-9)

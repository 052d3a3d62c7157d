// pybind11 module with the reference's Python module and class names for
// the QP-IK path (reference: src/bindings.cpp:219-447, Boost.Python +
// eigenpy).  It wraps the C++ facade include/drc_amd.hpp, which
// calls the HIP library through the C-ABI.  numpy float64 arrays stand in
// for Eigen types: VectorXd -> 1-D, MatrixXd -> 2-D, Affine3d -> 4x4.
//
// The reference's drc/ Python package subclasses these classes
// (drc/manipulator/robot_data.py, drc/mobile/robot_data.py, ...), so every
// class and method name of bindings.cpp:219-447 is registered here
// (tests/test_bindings_names.py checks the list).  Besides the reference
// methods, each controller has QPIKBatch / QPIKStepBatch / QPIKCubicBatch and
// QPIDBatch / QPIDStepBatch / QPIDCubicBatch over [field][B] numpy arrays.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "drc_amd.hpp"

namespace py = pybind11;
using namespace drc_amd;
using Arr = py::array_t<double, py::array::c_style | py::array::forcecast>;
using MN_RD = drc_amd::Manipulator::RobotData;
using MN_RC = drc_amd::Manipulator::RobotController;
using MM_RD = drc_amd::MobileManipulator::RobotData;
using MM_RC = drc_amd::MobileManipulator::RobotController;
using MO_RD = drc_amd::Mobile::RobotData;
using MO_RC = drc_amd::Mobile::RobotController;

namespace {

Vec to_vec(const Arr& a) { return Vec(a.data(), a.data() + a.size()); }
py::array_t<double> to_arr(const Vec& v) {
  py::array_t<double> a(static_cast<py::ssize_t>(v.size()));
  std::copy(v.begin(), v.end(), a.mutable_data());
  return a;
}
py::array_t<double> to_mat(const Vec& v, py::ssize_t rows, py::ssize_t cols) {
  py::array_t<double> a({rows, cols});
  std::copy(v.begin(), v.end(), a.mutable_data());
  return a;
}
Pose to_pose(const Arr& a) {
  if (a.ndim() != 2 || a.shape(0) != 4 || a.shape(1) != 4) throw std::invalid_argument("pose must be a 4x4 array");
  Pose T;
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 4; ++c) T[c * 4 + r] = a.at(r, c);
  return T;
}
py::array_t<double> from_pose(const Pose& T) {
  py::array_t<double> a({4, 4});
  auto m = a.mutable_unchecked<2>();
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 4; ++c) m(r, c) = T[c * 4 + r];
  return a;
}

// Python-side KinematicParam (reference fields, type_define.h:58-72)
struct PyKinematicParam {
  int type = DRC_DRIVE_DIFFERENTIAL;
  double wheel_radius = 0, max_lin_speed = 2, max_ang_speed = 2, max_lin_acc = 2, max_ang_acc = 2;
  double base_width = 0, wheel_offset = 0;
  std::vector<double> roller_angles, base2wheel_angles;
  std::vector<std::vector<double>> base2wheel_positions;
  drc_kinematic_param c() const {
    drc_kinematic_param p{};
    p.type = type;
    p.wheel_radius = wheel_radius;
    p.max_lin_speed = max_lin_speed;
    p.max_ang_speed = max_ang_speed;
    p.max_lin_acc = max_lin_acc;
    p.max_ang_acc = max_ang_acc;
    p.base_width = base_width;
    p.wheel_offset = wheel_offset;
    const size_t n = type == DRC_DRIVE_DIFFERENTIAL ? 2 : base2wheel_positions.size();
    if ((type == DRC_DRIVE_CASTER ? 2 * n : n) > DRC_MAX_WHEELS) throw std::invalid_argument("too many wheels");
    p.n_wheels = static_cast<int>(n);
    for (size_t i = 0; i < n && type != DRC_DRIVE_DIFFERENTIAL; ++i) {
      p.roller_angles[i] = i < roller_angles.size() ? roller_angles[i] : 0.0;
      p.base2wheel_angles[i] = i < base2wheel_angles.size() ? base2wheel_angles[i] : 0.0;
      p.base2wheel_positions[i][0] = base2wheel_positions[i].at(0);
      p.base2wheel_positions[i][1] = base2wheel_positions[i].at(1);
    }
    return p;
  }
  static PyKinematicParam from_c(const drc_kinematic_param& p) {
    PyKinematicParam k;
    k.type = p.type;
    k.wheel_radius = p.wheel_radius;
    k.max_lin_speed = p.max_lin_speed;
    k.max_ang_speed = p.max_ang_speed;
    k.max_lin_acc = p.max_lin_acc;
    k.max_ang_acc = p.max_ang_acc;
    k.base_width = p.base_width;
    k.wheel_offset = p.wheel_offset;
    for (int i = 0; i < p.n_wheels && p.type != DRC_DRIVE_DIFFERENTIAL; ++i) {
      k.roller_angles.push_back(p.roller_angles[i]);
      k.base2wheel_angles.push_back(p.base2wheel_angles[i]);
      k.base2wheel_positions.push_back({p.base2wheel_positions[i][0], p.base2wheel_positions[i][1]});
    }
    return k;
  }
};

// [field][B] numpy batch call -> (out [A][B], status [B])
py::tuple batch(const ControllerBase& self, int A, int mode, const Arr& q, const Arr& qdot, const Arr* xt,
                const Arr& xdt, const Arr* xi, const Arr* xdi, double t, double t0, double T,
                const std::string& link) {
  if (q.ndim() != 2) throw std::invalid_argument("q must be [dof][B]");
  const int64_t B = q.shape(1);
  py::array_t<double> out({static_cast<py::ssize_t>(A), static_cast<py::ssize_t>(B)});
  py::array_t<int32_t> status(static_cast<py::ssize_t>(B));
  {
    py::gil_scoped_release nogil;
    self.QPIKBatch(mode, B, q.data(), qdot.data(), xt ? xt->data() : nullptr, xdt.data(), xi ? xi->data() : nullptr,
                   xdi ? xdi->data() : nullptr, t, t0, T, link, out.mutable_data(), status.mutable_data(), false);
  }
  return py::make_tuple(out, status);
}

// [field][B] numpy QPID batch -> (qddot [A][B], tau [A][B], status [B])
py::tuple batch_id(const ControllerBase& self, int A, int mode, const Arr& q, const Arr& qdot, const Arr* xt,
                   const Arr& xdt, const Arr* xi, const Arr* xdi, double t, double t0, double T,
                   const std::string& link) {
  if (q.ndim() != 2) throw std::invalid_argument("q must be [dof][B]");
  const int64_t B = q.shape(1);
  py::array_t<double> qdd({static_cast<py::ssize_t>(A), static_cast<py::ssize_t>(B)});
  py::array_t<double> tau({static_cast<py::ssize_t>(A), static_cast<py::ssize_t>(B)});
  py::array_t<int32_t> status(static_cast<py::ssize_t>(B));
  {
    py::gil_scoped_release nogil;
    self.QPIDBatch(mode, B, q.data(), qdot.data(), xt ? xt->data() : nullptr, xdt.data(), xi ? xi->data() : nullptr,
                   xdi ? xdi->data() : nullptr, t, t0, T, link, qdd.mutable_data(), tau.mutable_data(),
                   status.mutable_data(), false);
  }
  return py::make_tuple(qdd, tau, status);
}

template <class RC, class RD>
void add_controller_common(py::class_<RC>& c) {
  c.def("QPIDBatch", [](const RC& s, const Arr& q, const Arr& qd, const Arr& xdd, const std::string& l) {
     return batch_id(s, s.actuatedDof(), DRC_MODE_QPID, q, qd, nullptr, xdd, nullptr, nullptr, 0, 0, 1, l);
   })
      .def("QPIDStepBatch", [](const RC& s, const Arr& q, const Arr& qd, const Arr& xt, const Arr& xdt,
                               const std::string& l) {
        return batch_id(s, s.actuatedDof(), DRC_MODE_QPID_STEP, q, qd, &xt, xdt, nullptr, nullptr, 0, 0, 1, l);
      })
      .def("QPIDCubicBatch", [](const RC& s, const Arr& q, const Arr& qd, const Arr& xt, const Arr& xdt,
                                const Arr& xi, const Arr& xdi, double t, double t0, double T, const std::string& l) {
        return batch_id(s, s.actuatedDof(), DRC_MODE_QPID_CUBIC, q, qd, &xt, xdt, &xi, &xdi, t, t0, T, l);
      });
  c.def("setTaskGain", [](RC& s, const Arr& kp, const Arr& kv) { s.setTaskGain(to_vec(kp), to_vec(kv)); })
      .def("setTaskKpGain", [](RC& s, const Arr& kp) { s.setTaskKpGain(to_vec(kp)); })
      .def("setTaskKvGain", [](RC& s, const Arr& kv) { s.setTaskKvGain(to_vec(kv)); })
      .def("setExact", &RC::setExact, "certified optimum (True, default) or the reference OSQP settings");
}

}  // namespace

PYBIND11_MODULE(dyros_robot_controller_cpp_wrapper, m) {
  m.doc() = "MI355X-native QP-IK path of dyros_robot_controller (HIP, gfx950) with the reference names";

  py::register_exception<drc_amd::Error>(m, "DrcError", PyExc_RuntimeError);

  {  // DriveType (bindings.cpp:235-238) as an IntEnum
    py::module_ enum_mod = py::module_::import("enum");
    py::dict members;
    members["Differential"] = static_cast<int>(DRC_DRIVE_DIFFERENTIAL);
    members["Mecanum"] = static_cast<int>(DRC_DRIVE_MECANUM);
    members["Caster"] = static_cast<int>(DRC_DRIVE_CASTER);
    m.attr("DriveType") = enum_mod.attr("IntEnum")("DriveType", members);
    for (const char* v : {"Differential", "Mecanum", "Caster"})  // bp::enum_::export_values (bindings.cpp:239)
      m.attr(v) = m.attr("DriveType").attr(v);
  }

  py::class_<PyKinematicParam>(m, "KinematicParam")
      .def(py::init<>())
      .def_property("type", [](const PyKinematicParam& p) { return p.type; },
                    [](PyKinematicParam& p, py::object t) { p.type = py::int_(t); })
      .def_readwrite("wheel_radius", &PyKinematicParam::wheel_radius)
      .def_readwrite("max_lin_speed", &PyKinematicParam::max_lin_speed)
      .def_readwrite("max_ang_speed", &PyKinematicParam::max_ang_speed)
      .def_readwrite("max_lin_acc", &PyKinematicParam::max_lin_acc)
      .def_readwrite("max_ang_acc", &PyKinematicParam::max_ang_acc)
      .def_readwrite("base_width", &PyKinematicParam::base_width)
      .def_readwrite("roller_angles", &PyKinematicParam::roller_angles)
      .def_readwrite("base2wheel_positions", &PyKinematicParam::base2wheel_positions)
      .def_readwrite("base2wheel_angles", &PyKinematicParam::base2wheel_angles)
      .def_readwrite("wheel_offset", &PyKinematicParam::wheel_offset);

  py::class_<drc_joint_index>(m, "JointIndex")
      .def(py::init<>())
      .def_readwrite("virtual_start", &drc_joint_index::virtual_start)
      .def_readwrite("mani_start", &drc_joint_index::mani_start)
      .def_readwrite("mobi_start", &drc_joint_index::mobi_start);
  py::class_<drc_actuator_index>(m, "ActuatorIndex")
      .def(py::init<>())
      .def_readwrite("mani_start", &drc_actuator_index::mani_start)
      .def_readwrite("mobi_start", &drc_actuator_index::mobi_start);

  py::class_<MinDistResult>(m, "MinDistResult")
      .def(py::init<>())
      .def_readwrite("distance", &MinDistResult::distance)
      .def_property("grad", [](const MinDistResult& r) { return to_arr(r.grad); },
                    [](MinDistResult& r, const Arr& a) { r.grad = to_vec(a); })
      .def_property("grad_dot", [](const MinDistResult& r) { return to_arr(r.grad_dot); },
                    [](MinDistResult& r, const Arr& a) { r.grad_dot = to_vec(a); })
      .def("setZero", &MinDistResult::setZero);
  py::class_<ManipulabilityResult>(m, "ManipulabilityResult")
      .def(py::init<>())
      .def_readwrite("manipulability", &ManipulabilityResult::manipulability)
      .def_property("grad", [](const ManipulabilityResult& r) { return to_arr(r.grad); },
                    [](ManipulabilityResult& r, const Arr& a) { r.grad = to_vec(a); })
      .def_property("grad_dot", [](const ManipulabilityResult& r) { return to_arr(r.grad_dot); },
                    [](ManipulabilityResult& r, const Arr& a) { r.grad_dot = to_vec(a); })
      .def("setZero", &ManipulabilityResult::setZero);

  // ---- MobileRobotData / MobileRobotController (bindings.cpp:280-291, 382-385) ----
  py::class_<MO_RD, std::shared_ptr<MO_RD>>(m, "MobileRobotData")
      .def(py::init([](const PyKinematicParam& p) { return std::make_shared<MO_RD>(p.c()); }), py::arg("param"))
      .def("getVerbose", &MO_RD::getVerbose)
      .def("updateState", [](MO_RD& s, const Arr& wp, const Arr& wv) { return s.updateState(to_vec(wp), to_vec(wv)); })
      .def("computeBaseVel", [](const MO_RD& s, const Arr& wp, const Arr& wv) {
        return to_arr(s.computeBaseVel(to_vec(wp), to_vec(wv)));
      })
      .def("computeFKJacobian", [](const MO_RD& s, const Arr& wp) {
        return to_mat(s.computeFKJacobian(to_vec(wp)), 3, s.getWheelNum());
      })
      .def("getWheelNum", &MO_RD::getWheelNum)
      .def("getKineParam", [](const MO_RD& s) { return PyKinematicParam::from_c(s.getKineParam()); })
      .def("getWheelPosition", [](const MO_RD& s) { return to_arr(s.getWheelPosition()); })
      .def("getWheelVelocity", [](const MO_RD& s) { return to_arr(s.getWheelVelocity()); })
      .def("getBaseVel", [](const MO_RD& s) { return to_arr(s.getBaseVel()); })
      .def("getFKJacobian", [](const MO_RD& s) { return to_mat(s.getFKJacobian(), 3, s.getWheelNum()); });
  py::class_<MO_RC>(m, "MobileRobotController")
      .def(py::init<double, std::shared_ptr<MO_RD>>(), py::keep_alive<1, 3>())
      .def("computeWheelVel", [](const MO_RC& s, const Arr& v) { return to_arr(s.computeWheelVel(to_vec(v))); })
      .def("computeIKJacobian", [](const MO_RC& s) {
        Vec J = s.computeIKJacobian();
        return to_mat(J, static_cast<py::ssize_t>(J.size() / 3), 3);
      })
      .def("VelocityCommand", [](const MO_RC& s, const Arr& v) { return to_arr(s.VelocityCommand(to_vec(v))); });

  // ---- ManipulatorRobotData (bindings.cpp:293-321) ---------------------------
  py::class_<MN_RD, std::shared_ptr<MN_RD>>(m, "ManipulatorRobotData")
      .def(py::init<const std::string&, const std::string&, const std::string&>(), py::arg("urdf_path"),
           py::arg("srdf_path") = "", py::arg("packages_path") = "")
      .def("getVerbose", [](const MN_RD& s) {
        return "dof " + std::to_string(s.getDof()) + " (MI355X HIP QP-IK model)";
      })
      .def("updateState", [](MN_RD& s, const Arr& q, const Arr& qd) { return s.updateState(to_vec(q), to_vec(qd)); })
      .def("computeMassMatrix", [](const MN_RD& s, const Arr& q) {
        return to_mat(s.computeMassMatrix(to_vec(q)), s.getDof(), s.getDof());
      })
      .def("computeGravity", [](const MN_RD& s, const Arr& q) { return to_arr(s.computeGravity(to_vec(q))); })
      .def("computeCoriolis", [](const MN_RD& s, const Arr& q, const Arr& qd) {
        return to_arr(s.computeCoriolis(to_vec(q), to_vec(qd)));
      })
      .def("computeNonlinearEffects", [](const MN_RD& s, const Arr& q, const Arr& qd) {
        return to_arr(s.computeNonlinearEffects(to_vec(q), to_vec(qd)));
      })
      .def("computePose", [](const MN_RD& s, const Arr& q, const std::string& l) { return from_pose(s.computePose(to_vec(q), l)); })
      .def("computeJacobian", [](const MN_RD& s, const Arr& q, const std::string& l) {
        return to_mat(s.computeJacobian(to_vec(q), l), 6, s.getDof());
      })
      .def("computeJacobianTimeVariation", [](const MN_RD& s, const Arr& q, const Arr& qd, const std::string& l) {
        return to_mat(s.computeJacobianTimeVariation(to_vec(q), to_vec(qd), l), 6, s.getDof());
      })
      .def("computeVelocity", [](const MN_RD& s, const Arr& q, const Arr& qd, const std::string& l) {
        return to_arr(s.computeVelocity(to_vec(q), to_vec(qd), l));
      })
      .def("computeMinDistance", [](const MN_RD& s, const Arr& q, const Arr& qd, bool wg, bool wgd, bool verbose) {
        return s.computeMinDistance(to_vec(q), to_vec(qd), wg, wgd, verbose);
      }, py::arg("q"), py::arg("qdot"), py::arg("with_grad"), py::arg("with_graddot"), py::arg("verbose") = false)
      .def("computeManipulability", [](const MN_RD& s, const Arr& q, const Arr& qd, bool wg, bool wgd,
                                       const std::string& l) {
        return s.computeManipulability(to_vec(q), to_vec(qd), wg, wgd, l);
      })
      .def("getDof", &MN_RD::getDof)
      .def("getJointPosition", [](const MN_RD& s) { return to_arr(s.getJointPosition()); })
      .def("getJointVelocity", [](const MN_RD& s) { return to_arr(s.getJointVelocity()); })
      .def("getJointPositionLimit", [](const MN_RD& s) {
        auto l = s.getJointPositionLimit();
        return py::make_tuple(to_arr(l.first), to_arr(l.second));
      })
      .def("getJointVelocityLimit", [](const MN_RD& s) {
        auto l = s.getJointVelocityLimit();
        return py::make_tuple(to_arr(l.first), to_arr(l.second));
      })
      .def("getMassMatrix", [](const MN_RD& s) { return to_mat(s.getMassMatrix(), s.getDof(), s.getDof()); })
      .def("getMassMatrixInv", [](const MN_RD& s) { return to_mat(s.getMassMatrixInv(), s.getDof(), s.getDof()); })
      .def("getCoriolis", [](const MN_RD& s) { return to_arr(s.getCoriolis()); })
      .def("getGravity", [](const MN_RD& s) { return to_arr(s.getGravity()); })
      .def("getNonlinearEffects", [](const MN_RD& s) { return to_arr(s.getNonlinearEffects()); })
      .def("getPose", [](const MN_RD& s, const std::string& l) { return from_pose(s.getPose(l)); })
      .def("getJacobian", [](const MN_RD& s, const std::string& l) { return to_mat(s.getJacobian(l), 6, s.getDof()); })
      .def("getJacobianTimeVariation", [](const MN_RD& s, const std::string& l) {
        return to_mat(s.getJacobianTimeVariation(l), 6, s.getDof());
      })
      .def("getVelocity", [](const MN_RD& s, const std::string& l) { return to_arr(s.getVelocity(l)); })
      .def("getMinDistance", &MN_RD::getMinDistance, py::arg("with_grad"), py::arg("with_graddot"),
           py::arg("verbose") = false)
      .def("getManipulability", &MN_RD::getManipulability);

  // ---- ManipulatorRobotController (bindings.cpp:398-426) --------------------
  py::class_<MN_RC> mnrc(m, "ManipulatorRobotController");
  mnrc.def(py::init<double, std::shared_ptr<MN_RD>>(), py::keep_alive<1, 3>())
      .def("setJointGain", [](MN_RC& s, const Arr& kp, const Arr& kv) { s.setJointGain(to_vec(kp), to_vec(kv)); })
      .def("setJointKpGain", [](MN_RC& s, const Arr& kp) { s.setJointKpGain(to_vec(kp)); })
      .def("setJointKvGain", [](MN_RC& s, const Arr& kv) { s.setJointKvGain(to_vec(kv)); })
      .def("moveJointPositionCubic", [](const MN_RC& s, const Arr& qt, const Arr& qdt, const Arr& qi, const Arr& qdi,
                                        double t, double t0, double T) {
        return to_arr(s.moveJointPositionCubic(to_vec(qt), to_vec(qdt), to_vec(qi), to_vec(qdi), t, t0, T));
      })
      .def("moveJointVelocityCubic", [](const MN_RC& s, const Arr& qt, const Arr& qdt, const Arr& qi, const Arr& qdi,
                                        double t, double t0, double T) {
        return to_arr(s.moveJointVelocityCubic(to_vec(qt), to_vec(qdt), to_vec(qi), to_vec(qdi), t, t0, T));
      })
      .def("moveJointTorqueStep", [](const MN_RC& s, const Arr& qdd) { return to_arr(s.moveJointTorqueStep(to_vec(qdd))); })
      .def("moveJointTorqueStep", [](const MN_RC& s, const Arr& qt, const Arr& qdt) {
        return to_arr(s.moveJointTorqueStep(to_vec(qt), to_vec(qdt)));
      })
      .def("moveJointTorqueCubic", [](const MN_RC& s, const Arr& qt, const Arr& qdt, const Arr& qi, const Arr& qdi,
                                      double t, double t0, double T) {
        return to_arr(s.moveJointTorqueCubic(to_vec(qt), to_vec(qdt), to_vec(qi), to_vec(qdi), t, t0, T));
      })
      .def("QPIK", [](const MN_RC& s, const Arr& xd, const std::string& l) { return to_arr(s.QPIK(to_vec(xd), l)); })
      .def("QPIKStep", [](const MN_RC& s, const Arr& x, const Arr& xd, const std::string& l) {
        return to_arr(s.QPIKStep(to_pose(x), to_vec(xd), l));
      })
      .def("QPIKCubic", [](const MN_RC& s, const Arr& xt, const Arr& xdt, const Arr& xi, const Arr& xdi, double t,
                           double t0, double T, const std::string& l) {
        return to_arr(s.QPIKCubic(to_pose(xt), to_vec(xdt), to_pose(xi), to_vec(xdi), t, t0, T, l));
      })
      .def("QPIKBatch", [](const MN_RC& s, const Arr& q, const Arr& qd, const Arr& xdt, const std::string& l) {
        return batch(s, s.actuatedDof(), DRC_MODE_QPIK, q, qd, nullptr, xdt, nullptr, nullptr, 0, 0, 1, l);
      })
      .def("QPIKStepBatch", [](const MN_RC& s, const Arr& q, const Arr& qd, const Arr& xt, const Arr& xdt,
                               const std::string& l) {
        return batch(s, s.actuatedDof(), DRC_MODE_QPIK_STEP, q, qd, &xt, xdt, nullptr, nullptr, 0, 0, 1, l);
      })
      .def("QPIKCubicBatch", [](const MN_RC& s, const Arr& q, const Arr& qd, const Arr& xt, const Arr& xdt,
                                const Arr& xi, const Arr& xdi, double t, double t0, double T, const std::string& l) {
        return batch(s, s.actuatedDof(), DRC_MODE_QPIK_CUBIC, q, qd, &xt, xdt, &xi, &xdi, t, t0, T, l);
      })
      .def("QPID", [](const MN_RC& s, const Arr& xdd, const std::string& l) { return to_arr(s.QPID(to_vec(xdd), l)); })
      .def("QPIDStep", [](const MN_RC& s, const Arr& x, const Arr& xd, const std::string& l) {
        return to_arr(s.QPIDStep(to_pose(x), to_vec(xd), l));
      })
      .def("QPIDCubic", [](const MN_RC& s, const Arr& xt, const Arr& xdt, const Arr& xi, const Arr& xdi, double t,
                           double t0, double T, const std::string& l) {
        return to_arr(s.QPIDCubic(to_pose(xt), to_vec(xdt), to_pose(xi), to_vec(xdi), t, t0, T, l));
      })
      // CLIK / OSF with the reference's overloads (bindings.cpp:398-426)
      .def("CLIKStep", [](const MN_RC& s, const Arr& x, const Arr& xd, const std::string& l) {
        return to_arr(s.CLIKStep(to_pose(x), to_vec(xd), l));
      })
      .def("CLIKStep", [](const MN_RC& s, const Arr& x, const Arr& xd, const Arr& nu, const std::string& l) {
        return to_arr(s.CLIKStep(to_pose(x), to_vec(xd), to_vec(nu), l));
      })
      .def("CLIKCubic", [](const MN_RC& s, const Arr& xt, const Arr& xdt, const Arr& xi, const Arr& xdi, double t,
                           double t0, double T, const std::string& l) {
        return to_arr(s.CLIKCubic(to_pose(xt), to_vec(xdt), to_pose(xi), to_vec(xdi), t, t0, T, l));
      })
      .def("CLIKCubic", [](const MN_RC& s, const Arr& xt, const Arr& xdt, const Arr& xi, const Arr& xdi, double t,
                           double t0, double T, const Arr& nu, const std::string& l) {
        return to_arr(s.CLIKCubic(to_pose(xt), to_vec(xdt), to_pose(xi), to_vec(xdi), t, t0, T, to_vec(nu), l));
      })
      .def("OSF", [](const MN_RC& s, const Arr& xdd, const std::string& l) { return to_arr(s.OSF(to_vec(xdd), l)); })
      .def("OSF", [](const MN_RC& s, const Arr& xdd, const Arr& nu, const std::string& l) {
        return to_arr(s.OSF(to_vec(xdd), to_vec(nu), l));
      })
      .def("OSFStep", [](const MN_RC& s, const Arr& x, const Arr& xd, const std::string& l) {
        return to_arr(s.OSFStep(to_pose(x), to_vec(xd), l));
      })
      .def("OSFStep", [](const MN_RC& s, const Arr& x, const Arr& xd, const Arr& nu, const std::string& l) {
        return to_arr(s.OSFStep(to_pose(x), to_vec(xd), to_vec(nu), l));
      })
      .def("OSFCubic", [](const MN_RC& s, const Arr& xt, const Arr& xdt, const Arr& xi, const Arr& xdi, double t,
                          double t0, double T, const std::string& l) {
        return to_arr(s.OSFCubic(to_pose(xt), to_vec(xdt), to_pose(xi), to_vec(xdi), t, t0, T, l));
      })
      .def("OSFCubic", [](const MN_RC& s, const Arr& xt, const Arr& xdt, const Arr& xi, const Arr& xdi, double t,
                          double t0, double T, const Arr& nu, const std::string& l) {
        return to_arr(s.OSFCubic(to_pose(xt), to_vec(xdt), to_pose(xi), to_vec(xdi), t, t0, T, to_vec(nu), l));
      });
  add_controller_common<MN_RC, MN_RD>(mnrc);

  // ---- MobileManipulatorRobotData (bindings.cpp:334-380) --------------------
  // bases<ManipulatorRobotData, MobileRobotData> as the reference; the whole-
  // body overloads take the (virtual, mobile, mani) blocks
  using V3 = const Arr&;
  auto jv = [](const MM_RD& s, V3 a, V3 b, V3 c) { return s.jointVector(to_vec(a), to_vec(b), to_vec(c)); };
  py::class_<MM_RD, MN_RD, MO_RD, std::shared_ptr<MM_RD>>(m, "MobileManipulatorRobotData")
      .def(py::init([](const PyKinematicParam& p, const drc_joint_index& j, const drc_actuator_index& a,
                       const std::string& urdf, const std::string& srdf, const std::string& pkg) {
             return std::make_shared<MM_RD>(p.c(), j, a, urdf, srdf, pkg);
           }),
           py::arg("param"), py::arg("joint_idx"), py::arg("actuator_idx"), py::arg("urdf_path"),
           py::arg("srdf_path") = "", py::arg("packages_path") = "")
      .def("getVerbose", [](const MM_RD& s) {
        return "dof " + std::to_string(s.getDof()) + " (MI355X HIP whole-body QP-IK model); base: " + s.MO_RD::getVerbose();
      })
      .def("updateState", [](MM_RD& s, V3 qv, V3 qm, V3 qa, V3 dv, V3 dm, V3 da) {
        return s.updateState(to_vec(qv), to_vec(qm), to_vec(qa), to_vec(dv), to_vec(dm), to_vec(da));
      })
      .def("computeMassMatrix", [jv](const MM_RD& s, V3 qv, V3 qm, V3 qa) {
        return to_mat(s.computeMassMatrix(jv(s, qv, qm, qa)), s.getDof(), s.getDof());
      })
      .def("computeGravity", [jv](const MM_RD& s, V3 qv, V3 qm, V3 qa) { return to_arr(s.computeGravity(jv(s, qv, qm, qa))); })
      .def("computeCoriolis", [jv](const MM_RD& s, V3 qv, V3 qm, V3 qa, V3 dv, V3 dm, V3 da) {
        return to_arr(s.computeCoriolis(jv(s, qv, qm, qa), jv(s, dv, dm, da)));
      })
      .def("computeNonlinearEffects", [jv](const MM_RD& s, V3 qv, V3 qm, V3 qa, V3 dv, V3 dm, V3 da) {
        return to_arr(s.computeNonlinearEffects(jv(s, qv, qm, qa), jv(s, dv, dm, da)));
      })
      .def("computeMassMatrixActuated", [](const MM_RD& s, V3 qv, V3 qm, V3 qa) {
        return to_mat(s.computeMassMatrixActuated(to_vec(qv), to_vec(qm), to_vec(qa)), s.getActuatorDof(),
                      s.getActuatorDof());
      })
      .def("computeGravityActuated", [](const MM_RD& s, V3 qv, V3 qm, V3 qa) {
        return to_arr(s.computeGravityActuated(to_vec(qv), to_vec(qm), to_vec(qa)));
      })
      .def("computeCoriolisActuated", [](const MM_RD& s, V3 qv, V3 qm, V3 qa, V3 dm, V3 da) {
        return to_arr(s.computeCoriolisActuated(to_vec(qv), to_vec(qm), to_vec(qa), to_vec(dm), to_vec(da)));
      })
      .def("computeNonlinearEffectsActuated", [](const MM_RD& s, V3 qv, V3 qm, V3 qa, V3 dm, V3 da) {
        return to_arr(s.computeNonlinearEffectsActuated(to_vec(qv), to_vec(qm), to_vec(qa), to_vec(dm), to_vec(da)));
      })
      .def("computePose", [jv](const MM_RD& s, V3 qv, V3 qm, V3 qa, const std::string& l) {
        return from_pose(s.computePose(jv(s, qv, qm, qa), l));
      })
      .def("computeJacobian", [jv](const MM_RD& s, V3 qv, V3 qm, V3 qa, const std::string& l) {
        return to_mat(s.computeJacobian(jv(s, qv, qm, qa), l), 6, s.getDof());
      })
      .def("computeJacobianTimeVariation", [jv](const MM_RD& s, V3 qv, V3 qm, V3 qa, V3 dv, V3 dm, V3 da,
                                                const std::string& l) {
        return to_mat(s.computeJacobianTimeVariation(jv(s, qv, qm, qa), jv(s, dv, dm, da), l), 6, s.getDof());
      })
      .def("computeVelocity", [jv](const MM_RD& s, V3 qv, V3 qm, V3 qa, V3 dv, V3 dm, V3 da, const std::string& l) {
        return to_arr(s.computeVelocity(jv(s, qv, qm, qa), jv(s, dv, dm, da), l));
      })
      .def("computeMinDistance", [jv](const MM_RD& s, V3 qv, V3 qm, V3 qa, V3 dv, V3 dm, V3 da, bool wg, bool wgd,
                                      bool verbose) {
        return s.computeMinDistance(jv(s, qv, qm, qa), jv(s, dv, dm, da), wg, wgd, verbose);
      })
      .def("computeSelectionMatrix", [](const MM_RD& s, V3 qv, V3 qm) {
        return to_mat(s.computeSelectionMatrix(to_vec(qv), to_vec(qm)), s.getDof(), s.getActuatorDof());
      })
      .def("computeJacobianActuated", [](const MM_RD& s, V3 qv, V3 qm, V3 qa, const std::string& l) {
        return to_mat(s.computeJacobianActuated(to_vec(qv), to_vec(qm), to_vec(qa), l), 6, s.getActuatorDof());
      })
      .def("computeJacobianTimeVariationActuated", [](const MM_RD& s, V3 qv, V3 qm, V3 qa, V3 dv, V3 dm, V3 da,
                                                      const std::string& l) {
        return to_mat(s.computeJacobianTimeVariationActuated(to_vec(qv), to_vec(qm), to_vec(qa), to_vec(dv),
                                                             to_vec(dm), to_vec(da), l),
                      6, s.getActuatorDof());
      })
      .def("computeManipulability", [](const MM_RD& s, V3 qa, V3 da, bool wg, bool wgd, const std::string& l) {
        return s.computeManipulability(to_vec(qa), to_vec(da), wg, wgd, l);
      })
      .def("computeMobileFKJacobian", [](const MM_RD& s, V3 qm) {
        return to_mat(s.computeMobileFKJacobian(to_vec(qm)), 3, s.getMobileDof());
      })
      .def("computeMobileBaseVel", [](const MM_RD& s, V3 qm, V3 dm) {
        return to_arr(s.computeMobileBaseVel(to_vec(qm), to_vec(dm)));
      })
      .def("getActuatordDof", &MM_RD::getActuatordDof)
      .def("getActuatorDof", &MM_RD::getActuatordDof)
      .def("getManipulatorDof", &MM_RD::getManipulatorDof)
      .def("getMobileDof", &MM_RD::getMobileDof)
      .def("getJointIndex", &MM_RD::getJointIndex)
      .def("getActuatorIndex", &MM_RD::getActuatorIndex)
      .def("getMobileJointPosition", [](const MM_RD& s) { return to_arr(s.getMobileJointPosition()); })
      .def("getVirtualJointPosition", [](const MM_RD& s) { return to_arr(s.getVirtualJointPosition()); })
      .def("getManiJointPosition", [](const MM_RD& s) { return to_arr(s.getManiJointPosition()); })
      .def("getJointVelocityActuated", [](const MM_RD& s) { return to_arr(s.getJointVelocityActuated()); })
      .def("getMobileJointVelocity", [](const MM_RD& s) { return to_arr(s.getMobileJointVelocity()); })
      .def("getVirtualJointVelocity", [](const MM_RD& s) { return to_arr(s.getVirtualJointVelocity()); })
      .def("getManiJointVelocity", [](const MM_RD& s) { return to_arr(s.getManiJointVelocity()); })
      .def("getJointPositionActuated", [](const MM_RD& s) { return to_arr(s.getJointPositionActuated()); })
      .def("getMassMatrixActuated", [](const MM_RD& s) {
        return to_mat(s.getMassMatrixActuated(), s.getActuatorDof(), s.getActuatorDof());
      })
      .def("getMassMatrixActuatedInv", [](const MM_RD& s) {
        return to_mat(s.getMassMatrixActuatedInv(), s.getActuatorDof(), s.getActuatorDof());
      })
      .def("getGravityActuated", [](const MM_RD& s) { return to_arr(s.getGravityActuated()); })
      .def("getCoriolisActuated", [](const MM_RD& s) { return to_arr(s.getCoriolisActuated()); })
      .def("getNonlinearEffectsActuated", [](const MM_RD& s) { return to_arr(s.getNonlinearEffectsActuated()); })
      .def("getJacobianActuated", [](const MM_RD& s, const std::string& l) {
        return to_mat(s.getJacobianActuated(l), 6, s.getActuatorDof());
      })
      .def("getJacobianActuatedTimeVariation", [](const MM_RD& s, const std::string& l) {
        return to_mat(s.getJacobianActuatedTimeVariation(l), 6, s.getActuatorDof());
      })
      .def("getSelectionMatrix", [](const MM_RD& s) { return to_mat(s.getSelectionMatrix(), s.getDof(), s.getActuatorDof()); })
      .def("getManipulability", &MM_RD::getManipulability)
      .def("getMobileFKJacobian", [](const MM_RD& s) { return to_mat(s.getMobileFKJacobian(), 3, s.getMobileDof()); })
      .def("getMobileBaseVel", [](const MM_RD& s) { return to_arr(s.getMobileBaseVel()); });

  // ---- MobileManipulatorRobotController (bindings.cpp:430-446) --------------
  py::class_<MM_RC> mmrc(m, "MobileManipulatorRobotController");
  mmrc.def(py::init<double, std::shared_ptr<MM_RD>>(), py::keep_alive<1, 3>())
      .def("setManipulatorJointGain", [](MM_RC& s, V3 kp, V3 kv) { s.setManipulatorJointGain(to_vec(kp), to_vec(kv)); })
      .def("setManipulatorJointKpGain", [](MM_RC& s, V3 kp) { s.setManipulatorJointKpGain(to_vec(kp)); })
      .def("setManipulatorJointKvGain", [](MM_RC& s, V3 kv) { s.setManipulatorJointKvGain(to_vec(kv)); })
      .def("moveManipulatorJointPositionCubic", [](const MM_RC& s, V3 qt, V3 qdt, V3 qi, V3 qdi, double t, double t0,
                                                   double T) {
        return to_arr(s.moveManipulatorJointPositionCubic(to_vec(qt), to_vec(qdt), to_vec(qi), to_vec(qdi), t, t0, T));
      })
      .def("moveManipulatorJointTorqueStep", [](const MM_RC& s, V3 qdd) {
        return to_arr(s.moveManipulatorJointTorqueStep(to_vec(qdd)));
      })
      .def("moveManipulatorJointTorqueStep", [](const MM_RC& s, V3 qt, V3 qdt) {
        return to_arr(s.moveManipulatorJointTorqueStep(to_vec(qt), to_vec(qdt)));
      })
      .def("moveManipulatorJointTorqueCubic", [](const MM_RC& s, V3 qt, V3 qdt, V3 qi, V3 qdi, double t, double t0,
                                                 double T) {
        return to_arr(s.moveManipulatorJointTorqueCubic(to_vec(qt), to_vec(qdt), to_vec(qi), to_vec(qdi), t, t0, T));
      })
      .def("QPIK", [](const MM_RC& s, const Arr& xd, const std::string& l) {
        Vec vm, va;
        s.QPIK(to_vec(xd), l, vm, va);
        return py::make_tuple(to_arr(vm), to_arr(va));
      })
      .def("QPIKStep", [](const MM_RC& s, const Arr& x, const Arr& xd, const std::string& l) {
        Vec vm, va;
        s.QPIKStep(to_pose(x), to_vec(xd), l, vm, va);
        return py::make_tuple(to_arr(vm), to_arr(va));
      })
      .def("QPIKCubic", [](const MM_RC& s, const Arr& xt, const Arr& xdt, const Arr& xi, const Arr& xdi, double t,
                           double t0, double T, const std::string& l) {
        Vec vm, va;
        s.QPIKCubic(to_pose(xt), to_vec(xdt), to_pose(xi), to_vec(xdi), t, t0, T, l, vm, va);
        return py::make_tuple(to_arr(vm), to_arr(va));
      })
      .def("QPIKBatch", [](const MM_RC& s, const Arr& q, const Arr& qd, const Arr& xdt, const std::string& l) {
        return batch(s, s.actuatedDof(), DRC_MODE_QPIK, q, qd, nullptr, xdt, nullptr, nullptr, 0, 0, 1, l);
      })
      .def("QPIKStepBatch", [](const MM_RC& s, const Arr& q, const Arr& qd, const Arr& xt, const Arr& xdt,
                               const std::string& l) {
        return batch(s, s.actuatedDof(), DRC_MODE_QPIK_STEP, q, qd, &xt, xdt, nullptr, nullptr, 0, 0, 1, l);
      })
      .def("QPIKCubicBatch", [](const MM_RC& s, const Arr& q, const Arr& qd, const Arr& xt, const Arr& xdt,
                                const Arr& xi, const Arr& xdi, double t, double t0, double T, const std::string& l) {
        return batch(s, s.actuatedDof(), DRC_MODE_QPIK_CUBIC, q, qd, &xt, xdt, &xi, &xdi, t, t0, T, l);
      })
      .def("QPID", [](const MM_RC& s, const Arr& xdd, const std::string& l) {
        Vec am, ta;
        s.QPID(to_vec(xdd), l, am, ta);
        return py::make_tuple(to_arr(am), to_arr(ta));
      })
      .def("QPIDStep", [](const MM_RC& s, const Arr& x, const Arr& xd, const std::string& l) {
        Vec am, ta;
        s.QPIDStep(to_pose(x), to_vec(xd), l, am, ta);
        return py::make_tuple(to_arr(am), to_arr(ta));
      })
      .def("QPIDCubic", [](const MM_RC& s, const Arr& xt, const Arr& xdt, const Arr& xi, const Arr& xdi, double t,
                           double t0, double T, const std::string& l) {
        Vec am, ta;
        s.QPIDCubic(to_pose(xt), to_vec(xdt), to_pose(xi), to_vec(xdi), t, t0, T, l, am, ta);
        return py::make_tuple(to_arr(am), to_arr(ta));
      });
  add_controller_common<MM_RC, MM_RD>(mmrc);
}

// pybind11 module with the reference's Python module and class names for
// the QP-IK path (reference: src/bindings.cpp:219-447, Boost.Python +
// eigenpy).  It wraps the C++ facade include/drc_amd.hpp, which
// calls the HIP library through the C-ABI.  numpy float64 arrays stand in
// for Eigen types: VectorXd -> 1-D, MatrixXd -> 2-D, Affine3d -> 4x4.
//
// The reference's drc/ Python package subclasses these classes
// (drc/manipulator/robot_data.py, robot_controller.py, ...).  Besides the
// reference methods, each controller has QPIKBatch / QPIKStepBatch /
// QPIKCubicBatch and QPIDBatch / QPIDStepBatch / QPIDCubicBatch over
// [field][B] numpy arrays.
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
    if (n > DRC_MAX_WHEELS) throw std::invalid_argument("too many wheels");
    p.n_wheels = static_cast<int>(n);
    for (size_t i = 0; i < n && type != DRC_DRIVE_DIFFERENTIAL; ++i) {
      p.roller_angles[i] = i < roller_angles.size() ? roller_angles[i] : 0.0;
      p.base2wheel_angles[i] = i < base2wheel_angles.size() ? base2wheel_angles[i] : 0.0;
      p.base2wheel_positions[i][0] = base2wheel_positions[i].at(0);
      p.base2wheel_positions[i][1] = base2wheel_positions[i].at(1);
    }
    return p;
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

  // ---- ManipulatorRobotData (bindings.cpp:293-333) ----------------------------
  py::class_<MN_RD, std::shared_ptr<MN_RD>>(m, "ManipulatorRobotData")
      .def(py::init<const std::string&, const std::string&, const std::string&>(), py::arg("urdf_path"),
           py::arg("srdf_path") = "", py::arg("packages_path") = "")
      .def("getVerbose", [](const MN_RD& s) {
        return "dof " + std::to_string(s.getDof()) + " (MI355X HIP QP-IK model)";
      })
      .def("updateState", [](MN_RD& s, const Arr& q, const Arr& qd) { return s.updateState(to_vec(q), to_vec(qd)); })
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
      .def("computePose", [](const MN_RD& s, const Arr& q, const std::string& l) { return from_pose(s.computePose(to_vec(q), l)); })
      .def("computeJacobian", [](const MN_RD& s, const Arr& q, const std::string& l) {
        return to_mat(s.computeJacobian(to_vec(q), l), 6, s.getDof());
      })
      .def("getPose", [](const MN_RD& s, const std::string& l) { return from_pose(s.getPose(l)); })
      .def("getJacobian", [](const MN_RD& s, const std::string& l) { return to_mat(s.getJacobian(l), 6, s.getDof()); })
      .def("getVelocity", [](const MN_RD& s, const std::string& l) { return to_arr(s.getVelocity(l)); })
      .def("getManipulability", &MN_RD::getManipulability)
      .def("getMinDistance", &MN_RD::getMinDistance, py::arg("with_grad"), py::arg("with_graddot"),
           py::arg("verbose") = false)
      .def("getJacobianTimeVariation", [](const MN_RD& s, const std::string& l) {
        return to_mat(s.getJacobianTimeVariation(l), 6, s.getDof());
      })
      .def("computeJacobianTimeVariation", [](const MN_RD& s, const Arr& q, const Arr& qd, const std::string& l) {
        return to_mat(s.computeJacobianTimeVariation(to_vec(q), to_vec(qd), l), 6, s.getDof());
      });

  // ---- ManipulatorRobotController (bindings.cpp:398-426) --------------------
  py::class_<MN_RC> mnrc(m, "ManipulatorRobotController");
  mnrc.def(py::init<double, std::shared_ptr<MN_RD>>(), py::keep_alive<1, 3>())
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
  py::class_<MM_RD, std::shared_ptr<MM_RD>>(m, "MobileManipulatorRobotData")
      .def(py::init([](const PyKinematicParam& p, const drc_joint_index& j, const drc_actuator_index& a,
                       const std::string& urdf, const std::string& srdf, const std::string& pkg) {
             return std::make_shared<MM_RD>(p.c(), j, a, urdf, srdf, pkg);
           }),
           py::arg("param"), py::arg("joint_idx"), py::arg("actuator_idx"), py::arg("urdf_path"),
           py::arg("srdf_path") = "", py::arg("packages_path") = "")
      .def("getVerbose", [](const MM_RD& s) {
        return "dof " + std::to_string(s.getDof()) + " (MI355X HIP whole-body QP-IK model)";
      })
      .def("updateState", [](MM_RD& s, const Arr& qv, const Arr& qm, const Arr& qa, const Arr& dv, const Arr& dm,
                             const Arr& da) {
        return s.updateState(to_vec(qv), to_vec(qm), to_vec(qa), to_vec(dv), to_vec(dm), to_vec(da));
      })
      .def("getDof", &MM_RD::getDof)
      .def("getActuatorDof", &MM_RD::getActuatorDof)
      .def("getManipulatorDof", &MM_RD::getManipulatorDof)
      .def("getMobileDof", &MM_RD::getMobileDof)
      .def("getJointIndex", &MM_RD::getJointIndex)
      .def("getActuatorIndex", &MM_RD::getActuatorIndex)
      .def("getJointPosition", [](const MM_RD& s) { return to_arr(s.getJointPosition()); })
      .def("getJointVelocity", [](const MM_RD& s) { return to_arr(s.getJointVelocity()); })
      .def("getMobileFKJacobian", [](const MM_RD& s) { return to_mat(s.getMobileFKJacobian(), 3, s.getMobileDof()); })
      .def("getPose", [](const MM_RD& s, const std::string& l) { return from_pose(s.getPose(l)); })
      .def("getJacobian", [](const MM_RD& s, const std::string& l) { return to_mat(s.getJacobian(l), 6, s.getDof()); })
      .def("getMinDistance", &MM_RD::getMinDistance, py::arg("with_grad"), py::arg("with_graddot"),
           py::arg("verbose") = false)
      .def("getManipulability", &MM_RD::getManipulability)
      .def("getJacobianTimeVariation", [](const MM_RD& s, const std::string& l) {
        return to_mat(s.getJacobianTimeVariation(l), 6, s.getDof());
      });

  // ---- MobileManipulatorRobotController (bindings.cpp:430-444) --------------
  py::class_<MM_RC> mmrc(m, "MobileManipulatorRobotController");
  mmrc.def(py::init<double, std::shared_ptr<MM_RD>>(), py::keep_alive<1, 3>())
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

// drc_amd.hpp — C++ façade over the C-ABI (include/drc_amd.h) with the
// reference's class and method names for the QP-IK path.
//
//   reference (include/dyros_robot_controller/...)        here (namespace drc_amd)
//   Manipulator::RobotData(urdf, srdf, packages)           Manipulator::RobotData(urdf, srdf, packages, device)
//     updateState(q, qdot)            robot_data.h:59        updateState
//     getPose / getJacobian / getVelocity (:110-116)         same (HIP kernel stage outputs)
//     getManipulability(true,false,l) / getMinDistance       same
//   Manipulator::RobotController(dt, shared_ptr<RobotData>)  same
//     setTaskGain / setTaskKpGain / setTaskKvGain            same
//     QPIK / QPIKStep / QPIKCubic  (robot_controller.h:295-321)  same (B = 1 on the GPU)
//   MobileManipulator::RobotData(KinematicParam, JointIndex, ActuatorIndex, urdf, srdf, packages)
//     updateState(q_virtual, q_mobile, q_mani, qdot_*)      same
//   MobileManipulator::RobotController::QPIK*(..., qdot_mobile, qdot_mani)  same
//   (none)                                                   QPIK*Batch over [field][B] host or device arrays
//
// Eigen is not required: vectors are std::vector<double>, poses are 4x4
// column-major (Eigen::Affine3d::matrix() memory order) in std::array<double,16>.
// Any type with data()/size() (Eigen::VectorXd) converts through vec().
// Reference error behaviour: a failed QP prints
// "QP IK failed to compute optimal joint velocity." and returns zeros
// (robot_controller.cpp:283-287); bad gain sizes throw std::runtime_error
// (:23-26); an unknown link throws drc_amd::Error (reference: stderr).
#ifndef DRC_AMD_HPP
#define DRC_AMD_HPP

#include <array>
#include <cstdint>
#include <iostream>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "drc_amd.h"

namespace drc_amd {

using Vec = std::vector<double>;
using Pose = std::array<double, 16>;  // 4x4 column-major

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};
inline void check(int rc) {
  if (rc != DRC_OK) throw Error(rc, std::string(drc_error_string(rc)) + ": " + drc_last_error());
}
template <class V>
inline Vec vec(const V& v) {
  return Vec(v.data(), v.data() + v.size());
}
// 4x4 column-major <-> [R col-major (9), p (3)]
inline std::array<double, 12> pose12(const Pose& T) {
  return {T[0], T[1], T[2], T[4], T[5], T[6], T[8], T[9], T[10], T[12], T[13], T[14]};
}
inline Pose pose44(const double* v) {
  return {v[0], v[1], v[2], 0, v[3], v[4], v[5], 0, v[6], v[7], v[8], 0, v[9], v[10], v[11], 1};
}

struct MinDistResult {  // type_define.h:140-150
  double distance = 0;
  Vec grad, grad_dot;
  void setZero() {
    distance = 0;
    std::fill(grad.begin(), grad.end(), 0.0);
    std::fill(grad_dot.begin(), grad_dot.end(), 0.0);
  }
};
struct ManipulabilityResult {  // type_define.h:152-162
  double manipulability = 0;
  Vec grad, grad_dot;
  void setZero() {
    manipulability = 0;
    std::fill(grad.begin(), grad.end(), 0.0);
    std::fill(grad_dot.begin(), grad_dot.end(), 0.0);
  }
};

// Owns a drc_model* and the host copy of the robot state.
class ModelBase {
 public:
  ModelBase(const ModelBase&) = delete;
  ModelBase& operator=(const ModelBase&) = delete;
  virtual ~ModelBase() { drc_model_destroy(model_); }
  drc_model* handle() const { return model_; }
  int getDof() const { return dof_; }
  int getActuatorDof() const { return act_; }
  std::pair<Vec, Vec> getJointPositionLimit() const { return {lims_[0], lims_[1]}; }
  std::pair<Vec, Vec> getJointVelocityLimit() const { return {lims_[2], lims_[3]}; }
  const Vec& getJointPosition() const { return q_; }
  const Vec& getJointVelocity() const { return qdot_; }
  int frameId(const std::string& link) const {
    int fid = -1;
    check(drc_model_find_frame(model_, link.c_str(), &fid));
    return fid;
  }
  drc_qpik_params defaultParams(bool exact) const {
    drc_qpik_params p;
    check(drc_default_qpik_params(model_, exact ? 1 : 0, &p));
    return p;
  }

  // stage outputs at (q, qdot); link == "" selects no task frame
  struct Stages {
    std::array<double, 12> pose;
    Vec jac, man, dist;
    int pair = -1;
  };
  Stages stages(const Vec& q, const Vec& qdot, const std::string& link) const {
    drc_qpik_params p = defaultParams(true);
    p.mode = DRC_MODE_QPIK;
    p.frame_id = link.empty() ? -1 : frameId(link);
    Stages s;
    s.jac.resize(6 * dof_);
    s.man.resize(1 + mani_);
    s.dist.resize(1 + dof_);
    Vec xdd(6), zero6(6, 0.0);
    int32_t pair = -1;
    check(drc_qpik_stages_host(model_, &p, 1, q.data(), qdot.data(), nullptr, zero6.data(), nullptr, nullptr,
                               s.pose.data(), s.jac.data(), s.man.data(), s.dist.data(), &pair, xdd.data()));
    s.pair = pair;
    return s;
  }
  // QPID stage outputs at (q, qdot): frame Jacobian time variation (6 x dof,
  // row-major) and the grad_dot vectors of getManipulability / getMinDistance
  struct QpidStages {
    Vec jdot, man_graddot, dist_graddot;
  };
  QpidStages qpidStages(const Vec& q, const Vec& qdot, const std::string& link) const {
    drc_qpik_params p;
    check(drc_default_qpid_params(model_, 1, &p));
    p.mode = DRC_MODE_QPID;
    p.frame_id = link.empty() ? -1 : frameId(link);
    QpidStages s;
    s.jdot.resize(6 * dof_);
    Vec gdv(mani_ + dof_), zero6(6, 0.0);
    check(drc_qpid_stages_host(model_, &p, 1, q.data(), qdot.data(), nullptr, zero6.data(), nullptr, nullptr,
                               nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, s.jdot.data(), nullptr,
                               gdv.data()));
    s.man_graddot.assign(gdv.begin(), gdv.begin() + mani_);
    s.dist_graddot.assign(gdv.begin() + mani_, gdv.end());
    return s;
  }

 protected:
  ModelBase() = default;
  void init(drc_model* m) {
    model_ = m;
    int ng = 0, np = 0;
    check(drc_model_info(model_, &dof_, &act_, &mani_, &mobi_, &ng, &np));
    for (auto& v : lims_) v.assign(dof_, 0.0);
    check(drc_model_limits(model_, lims_[0].data(), lims_[1].data(), lims_[2].data(), lims_[3].data()));
    q_.assign(dof_, 0.0);
    qdot_.assign(dof_, 0.0);
  }
  drc_model* model_ = nullptr;
  int dof_ = 0, act_ = 0, mani_ = 0, mobi_ = 0;
  std::array<Vec, 4> lims_;
  Vec q_, qdot_;
};

namespace Manipulator {

class RobotData : public ModelBase {
 public:
  RobotData(const std::string& urdf, const std::string& srdf = "", const std::string& packages = "",
            int device = 0) {
    drc_model* m = nullptr;
    check(drc_model_create_manipulator(urdf.c_str(), srdf.c_str(), packages.c_str(), device, &m));
    init(m);
  }
  bool updateState(const Vec& q, const Vec& qdot) {
    if (static_cast<int>(q.size()) != dof_ || static_cast<int>(qdot.size()) != dof_) return false;
    q_ = q;
    qdot_ = qdot;
    return true;
  }
  Pose computePose(const Vec& q, const std::string& link) const {
    return pose44(stages(q, Vec(dof_, 0.0), link).pose.data());
  }
  Vec computeJacobian(const Vec& q, const std::string& link) const {  // 6 x dof, row-major
    return stages(q, Vec(dof_, 0.0), link).jac;
  }
  Pose getPose(const std::string& link) const { return pose44(stages(q_, qdot_, link).pose.data()); }
  Vec getJacobian(const std::string& link) const { return stages(q_, qdot_, link).jac; }
  Vec getVelocity(const std::string& link) const {  // J qdot (robot_data.cpp:419-422)
    Vec J = getJacobian(link), v(6, 0.0);
    for (int r = 0; r < 6; ++r)
      for (int c = 0; c < dof_; ++c) v[r] += J[r * dof_ + c] * qdot_[c];
    return v;
  }
  ManipulabilityResult getManipulability(bool with_grad, bool with_graddot, const std::string& link) const {
    Stages s = stages(q_, qdot_, link);
    ManipulabilityResult r;
    r.manipulability = s.man[0];
    r.grad = (with_grad || with_graddot) ? Vec(s.man.begin() + 1, s.man.end()) : Vec(mani_, 0.0);
    r.grad_dot = with_graddot ? qpidStages(q_, qdot_, link).man_graddot : Vec(mani_, 0.0);
    return r;
  }
  MinDistResult getMinDistance(bool with_grad, bool with_graddot, bool verbose = false) const {
    Stages s = stages(q_, qdot_, "");
    MinDistResult r;
    r.distance = s.dist[0];
    r.grad = (with_grad || with_graddot) ? Vec(s.dist.begin() + 1, s.dist.end()) : Vec(dof_, 0.0);
    r.grad_dot = with_graddot ? qpidStages(q_, qdot_, "").dist_graddot : Vec(dof_, 0.0);
    if (verbose) std::cout << "min distance " << r.distance << " (pair " << s.pair << ")\n";
    return r;
  }
  // getJacobianTimeVariation / computeJacobianTimeVariation (robot_data.cpp:404-417), 6 x dof row-major
  Vec getJacobianTimeVariation(const std::string& link) const { return qpidStages(q_, qdot_, link).jdot; }
  Vec computeJacobianTimeVariation(const Vec& q, const Vec& qdot, const std::string& link) const {
    return qpidStages(q, qdot, link).jdot;
  }
};

}  // namespace Manipulator

// Shared by both controllers: gains, solver mode, batched entries.
class ControllerBase {
 public:
  // task gains are shared by QPIK and QPID, as the reference's Kp_task_ / Kv_task_
  // (a MoMa QPIKStep has no Kv term: its parameters keep kv = 0)
  void setTaskGain(const Vec& Kp, const Vec& Kv) {
    if (Kp.size() != 6 || Kv.size() != 6) throw std::runtime_error("Kp and Kv must be of size 6.");
    setTaskKpGain(Kp);
    setTaskKvGain(Kv);
  }
  void setTaskKpGain(const Vec& Kp) {
    if (Kp.size() != 6) throw std::runtime_error("Kp must be of size 6.");
    for (int i = 0; i < 6; ++i) params_.kp[i] = id_params_.kp[i] = Kp[i];
  }
  void setTaskKvGain(const Vec& Kv) {
    if (Kv.size() != 6) throw std::runtime_error("Kv must be of size 6.");
    for (int i = 0; i < 6; ++i) {
      id_params_.kv[i] = Kv[i];
      if (params_.feedforward == 0) params_.kv[i] = Kv[i];
    }
  }
  // "exact" (certified optimum, default) or reference OSQP settings
  void setExact(bool exact) {
    drc_qpik_params d = model_->defaultParams(exact);
    params_.solver = d.solver;
    check(drc_default_qpid_params(model_->handle(), exact ? 1 : 0, &d));
    id_params_.solver = d.solver;
  }
  const drc_qpik_params& params() const { return params_; }
  int actuatedDof() const { return model_->getActuatorDof(); }

  // Batched QPIK* over [field][B] arrays.  Host arrays: synchronous.
  // Device arrays: asynchronous on `stream` (a hipStream_t).
  void QPIKBatch(int mode, int64_t B, const double* q, const double* qdot, const double* x_target,
                 const double* xdot_target, const double* x_init, const double* xdot_init, double t, double t0,
                 double duration, const std::string& link, double* eta_out, int32_t* status, bool device,
                 void* stream = nullptr, int32_t* iters = nullptr) const {
    drc_qpik_params p = params_;
    p.mode = mode;
    p.frame_id = model_->frameId(link);
    p.t = t;
    p.t0 = t0;
    p.duration = duration;
    if (device)
      check(drc_qpik_batch(model_->handle(), &p, B, q, qdot, x_target, xdot_target, x_init, xdot_init, eta_out,
                           status, iters, stream));
    else
      check(drc_qpik_host(model_->handle(), &p, B, q, qdot, x_target, xdot_target, x_init, xdot_init, eta_out,
                          status, iters));
  }
  // Batched QPID* (drc_qpid_batch): qddot / eta_dot and torques [A][B].
  void QPIDBatch(int mode, int64_t B, const double* q, const double* qdot, const double* x_target,
                 const double* xdot_target, const double* x_init, const double* xdot_init, double t, double t0,
                 double duration, const std::string& link, double* qddot_out, double* tau_out, int32_t* status,
                 bool device, void* stream = nullptr, int32_t* iters = nullptr) const {
    drc_qpik_params p = id_params_;
    p.mode = mode;
    p.frame_id = model_->frameId(link);
    p.t = t;
    p.t0 = t0;
    p.duration = duration;
    if (device)
      check(drc_qpid_batch(model_->handle(), &p, B, q, qdot, x_target, xdot_target, x_init, xdot_init, qddot_out,
                           tau_out, status, iters, stream));
    else
      check(drc_qpid_host(model_->handle(), &p, B, q, qdot, x_target, xdot_target, x_init, xdot_init, qddot_out,
                          tau_out, status, iters));
  }

 protected:
  ControllerBase(double dt, const ModelBase* model) : dt_(dt), model_(model) {
    params_ = model_->defaultParams(true);
    check(drc_default_qpid_params(model_->handle(), 1, &id_params_));
  }
  // one QPID instance at the model's stored state; tau = gravity on failure
  // (the kernel writes it), stderr message as the reference
  void solveOneID(int mode, const Pose* xt, const Vec* xdt, const Pose* xi, const Vec* xdi, double t, double t0,
                  double T, const std::string& link, Vec& qdd, Vec& tau) const {
    const int A = model_->getActuatorDof();
    std::array<double, 12> xt12{}, xi12{};
    if (xt) xt12 = pose12(*xt);
    if (xi) xi12 = pose12(*xi);
    qdd.assign(A, 0.0);
    tau.assign(A, 0.0);
    int32_t status = 0;
    QPIDBatch(mode, 1, model_->getJointPosition().data(), model_->getJointVelocity().data(),
              xt ? xt12.data() : nullptr, xdt->data(), xi ? xi12.data() : nullptr, xdi ? xdi->data() : nullptr, t, t0,
              T, link, qdd.data(), tau.data(), &status, false);
    if (status != DRC_STATUS_SOLVED) std::cerr << "QP ID failed to compute optimal joint torque." << std::endl;
  }
  // one instance at the model's stored state; zeros + stderr on failure
  Vec solveOne(int mode, const Pose* xt, const Vec* xdt, const Pose* xi, const Vec* xdi, double t, double t0,
               double T, const std::string& link) const {
    const int A = model_->getActuatorDof();
    std::array<double, 12> xt12{}, xi12{};
    if (xt) xt12 = pose12(*xt);
    if (xi) xi12 = pose12(*xi);
    Vec eta(A, 0.0);
    int32_t status = 0;
    QPIKBatch(mode, 1, model_->getJointPosition().data(), model_->getJointVelocity().data(),
              xt ? xt12.data() : nullptr, xdt->data(), xi ? xi12.data() : nullptr, xdi ? xdi->data() : nullptr, t,
              t0, T, link, eta.data(), &status, false);
    if (status != DRC_STATUS_SOLVED) {
      std::cerr << "QP IK failed to compute optimal joint velocity." << std::endl;
      eta.assign(A, 0.0);
    }
    return eta;
  }
  static void check6(const Vec& v) {
    if (v.size() != 6) throw std::runtime_error("task vectors must be of size 6.");
  }
  double dt_;
  const ModelBase* model_;
  drc_qpik_params params_, id_params_;
};

namespace Manipulator {

class RobotController : public ControllerBase {
 public:
  RobotController(double dt, std::shared_ptr<RobotData> robot_data)
      : ControllerBase(dt, robot_data.get()), robot_data_(std::move(robot_data)) {}
  Vec QPIK(const Vec& xdot_target, const std::string& link) const {
    check6(xdot_target);
    return solveOne(DRC_MODE_QPIK, nullptr, &xdot_target, nullptr, nullptr, 0, 0, 1, link);
  }
  Vec QPIKStep(const Pose& x_target, const Vec& xdot_target, const std::string& link) const {
    check6(xdot_target);
    return solveOne(DRC_MODE_QPIK_STEP, &x_target, &xdot_target, nullptr, nullptr, 0, 0, 1, link);
  }
  Vec QPIKCubic(const Pose& x_target, const Vec& xdot_target, const Pose& x_init, const Vec& xdot_init,
                double current_time, double init_time, double duration, const std::string& link) const {
    check6(xdot_target);
    check6(xdot_init);
    return solveOne(DRC_MODE_QPIK_CUBIC, &x_target, &xdot_target, &x_init, &xdot_init, current_time, init_time,
                    duration, link);
  }
  // QPID / QPIDStep / QPIDCubic (robot_controller.cpp:319-361): joint torques
  Vec QPID(const Vec& xddot_target, const std::string& link) const {
    check6(xddot_target);
    Vec qdd, tau;
    solveOneID(DRC_MODE_QPID, nullptr, &xddot_target, nullptr, nullptr, 0, 0, 1, link, qdd, tau);
    return tau;
  }
  Vec QPIDStep(const Pose& x_target, const Vec& xdot_target, const std::string& link) const {
    check6(xdot_target);
    Vec qdd, tau;
    solveOneID(DRC_MODE_QPID_STEP, &x_target, &xdot_target, nullptr, nullptr, 0, 0, 1, link, qdd, tau);
    return tau;
  }
  Vec QPIDCubic(const Pose& x_target, const Vec& xdot_target, const Pose& x_init, const Vec& xdot_init,
                double current_time, double init_time, double duration, const std::string& link) const {
    check6(xdot_target);
    check6(xdot_init);
    Vec qdd, tau;
    solveOneID(DRC_MODE_QPID_CUBIC, &x_target, &xdot_target, &x_init, &xdot_init, current_time, init_time, duration,
               link, qdd, tau);
    return tau;
  }
  // CLIKStep / CLIKCubic (robot_controller.cpp:156-214): joint velocities
  Vec CLIKStep(const Pose& x_target, const Vec& xdot_target, const Vec& null_qdot, const std::string& link) const {
    return closedForm(1, DRC_MODE_QPIK_STEP, &x_target, xdot_target, nullptr, nullptr, 0, 0, 1, &null_qdot, link);
  }
  Vec CLIKStep(const Pose& x_target, const Vec& xdot_target, const std::string& link) const {
    return closedForm(1, DRC_MODE_QPIK_STEP, &x_target, xdot_target, nullptr, nullptr, 0, 0, 1, nullptr, link);
  }
  Vec CLIKCubic(const Pose& x_target, const Vec& xdot_target, const Pose& x_init, const Vec& xdot_init,
                double current_time, double init_time, double duration, const Vec& null_qdot,
                const std::string& link) const {
    return closedForm(1, DRC_MODE_QPIK_CUBIC, &x_target, xdot_target, &x_init, &xdot_init, current_time, init_time,
                      duration, &null_qdot, link);
  }
  Vec CLIKCubic(const Pose& x_target, const Vec& xdot_target, const Pose& x_init, const Vec& xdot_init,
                double current_time, double init_time, double duration, const std::string& link) const {
    return closedForm(1, DRC_MODE_QPIK_CUBIC, &x_target, xdot_target, &x_init, &xdot_init, current_time, init_time,
                      duration, nullptr, link);
  }
  // OSF / OSFStep / OSFCubic (robot_controller.cpp:216-275): joint torques
  Vec OSF(const Vec& xddot_target, const Vec& null_torque, const std::string& link) const {
    return closedForm(2, DRC_MODE_QPIK, nullptr, xddot_target, nullptr, nullptr, 0, 0, 1, &null_torque, link);
  }
  Vec OSF(const Vec& xddot_target, const std::string& link) const {
    return closedForm(2, DRC_MODE_QPIK, nullptr, xddot_target, nullptr, nullptr, 0, 0, 1, nullptr, link);
  }
  Vec OSFStep(const Pose& x_target, const Vec& xdot_target, const Vec& null_torque, const std::string& link) const {
    return closedForm(2, DRC_MODE_QPIK_STEP, &x_target, xdot_target, nullptr, nullptr, 0, 0, 1, &null_torque, link);
  }
  Vec OSFStep(const Pose& x_target, const Vec& xdot_target, const std::string& link) const {
    return closedForm(2, DRC_MODE_QPIK_STEP, &x_target, xdot_target, nullptr, nullptr, 0, 0, 1, nullptr, link);
  }
  Vec OSFCubic(const Pose& x_target, const Vec& xdot_target, const Pose& x_init, const Vec& xdot_init,
               double current_time, double init_time, double duration, const Vec& null_torque,
               const std::string& link) const {
    return closedForm(2, DRC_MODE_QPIK_CUBIC, &x_target, xdot_target, &x_init, &xdot_init, current_time, init_time,
                      duration, &null_torque, link);
  }
  Vec OSFCubic(const Pose& x_target, const Vec& xdot_target, const Pose& x_init, const Vec& xdot_init,
               double current_time, double init_time, double duration, const std::string& link) const {
    return closedForm(2, DRC_MODE_QPIK_CUBIC, &x_target, xdot_target, &x_init, &xdot_init, current_time, init_time,
                      duration, nullptr, link);
  }

 private:
  Vec closedForm(int kind, int mode, const Pose* xt, const Vec& xdt, const Pose* xi, const Vec* xdi, double t,
                 double t0, double T, const Vec* nullv, const std::string& link) const {
    check6(xdt);
    if (xdi) check6(*xdi);
    const int n = robot_data_->getDof();
    if (nullv && static_cast<int>(nullv->size()) != n) throw std::runtime_error("null vector must be of size dof_.");
    drc_qpik_params p = id_params_;  // Kp_task_ / Kv_task_
    p.mode = mode;
    p.frame_id = robot_data_->frameId(link);
    p.t = t;
    p.t0 = t0;
    p.duration = T;
    std::array<double, 12> xt12{}, xi12{};
    if (xt) xt12 = pose12(*xt);
    if (xi) xi12 = pose12(*xi);
    Vec out(n, 0.0);
    check(drc_closed_form_host(robot_data_->handle(), &p, kind, 1, robot_data_->getJointPosition().data(),
                               robot_data_->getJointVelocity().data(), xt ? xt12.data() : nullptr, xdt.data(),
                               xi ? xi12.data() : nullptr, xdi ? xdi->data() : nullptr,
                               nullv ? nullv->data() : nullptr, out.data()));
    return out;
  }
  std::shared_ptr<RobotData> robot_data_;
};

}  // namespace Manipulator

namespace MobileManipulator {

using KinematicParam = drc_kinematic_param;
using JointIndex = drc_joint_index;
using ActuatorIndex = drc_actuator_index;

class RobotData : public ModelBase {
 public:
  RobotData(const KinematicParam& param, const JointIndex& joint_idx, const ActuatorIndex& actuator_idx,
            const std::string& urdf, const std::string& srdf = "", const std::string& packages = "", int device = 0)
      : jidx_(joint_idx), aidx_(actuator_idx) {
    drc_model* m = nullptr;
    check(drc_model_create_mobile_manipulator(&param, &joint_idx, &actuator_idx, urdf.c_str(), srdf.c_str(),
                                              packages.c_str(), device, &m));
    init(m);
  }
  // getJointVector (mobile_manipulator/robot_data.cpp:418-427)
  Vec jointVector(const Vec& v_virtual, const Vec& v_mobile, const Vec& v_mani) const {
    Vec v(dof_, 0.0);
    for (size_t i = 0; i < v_virtual.size(); ++i) v[jidx_.virtual_start + i] = v_virtual[i];
    for (size_t i = 0; i < v_mobile.size(); ++i) v[jidx_.mobi_start + i] = v_mobile[i];
    for (size_t i = 0; i < v_mani.size(); ++i) v[jidx_.mani_start + i] = v_mani[i];
    return v;
  }
  bool updateState(const Vec& q_virtual, const Vec& q_mobile, const Vec& q_mani, const Vec& qdot_virtual,
                   const Vec& qdot_mobile, const Vec& qdot_mani) {
    if (q_virtual.size() != 3 || static_cast<int>(q_mobile.size()) != mobi_ ||
        static_cast<int>(q_mani.size()) != mani_)
      return false;
    q_ = jointVector(q_virtual, q_mobile, q_mani);
    qdot_ = jointVector(qdot_virtual, qdot_mobile, qdot_mani);
    return true;
  }
  int getManipulatorDof() const { return mani_; }
  int getMobileDof() const { return mobi_; }
  const JointIndex& getJointIndex() const { return jidx_; }
  const ActuatorIndex& getActuatorIndex() const { return aidx_; }
  Vec getMobileFKJacobian() const {  // 3 x W row-major
    Vec J(3 * mobi_);
    check(drc_model_mobile_fk_jacobian(model_, J.data()));
    return J;
  }
  Pose getPose(const std::string& link) const { return pose44(stages(q_, qdot_, link).pose.data()); }
  Vec getJacobian(const std::string& link) const { return stages(q_, qdot_, link).jac; }
  MinDistResult getMinDistance(bool with_grad, bool with_graddot, bool verbose = false) const {
    Stages s = stages(q_, qdot_, "");
    MinDistResult r;
    r.distance = s.dist[0];
    r.grad = (with_grad || with_graddot) ? Vec(s.dist.begin() + 1, s.dist.end()) : Vec(dof_, 0.0);
    r.grad_dot = with_graddot ? qpidStages(q_, qdot_, "").dist_graddot : Vec(dof_, 0.0);
    if (verbose) std::cout << "min distance " << r.distance << " (pair " << s.pair << ")\n";
    return r;
  }
  // arm-block manipulability (robot_data.cpp:439-496)
  ManipulabilityResult getManipulability(bool with_grad, bool with_graddot, const std::string& link) const {
    Stages s = stages(q_, qdot_, link);
    ManipulabilityResult r;
    r.manipulability = s.man[0];
    r.grad = (with_grad || with_graddot) ? Vec(s.man.begin() + 1, s.man.end()) : Vec(mani_, 0.0);
    r.grad_dot = with_graddot ? qpidStages(q_, qdot_, link).man_graddot : Vec(mani_, 0.0);
    return r;
  }
  Vec getJacobianTimeVariation(const std::string& link) const { return qpidStages(q_, qdot_, link).jdot; }

 private:
  JointIndex jidx_;
  ActuatorIndex aidx_;
};

class RobotController : public ControllerBase {
 public:
  RobotController(double dt, std::shared_ptr<RobotData> robot_data)
      : ControllerBase(dt, robot_data.get()), robot_data_(std::move(robot_data)) {}
  // (qdot_mobile, qdot_mani) split by ActuatorIndex (robot_controller.cpp:182-196)
  void QPIK(const Vec& xdot_target, const std::string& link, Vec& qdot_mobile, Vec& qdot_mani) const {
    check6(xdot_target);
    split(solveOne(DRC_MODE_QPIK, nullptr, &xdot_target, nullptr, nullptr, 0, 0, 1, link), qdot_mobile, qdot_mani);
  }
  void QPIKStep(const Pose& x_target, const Vec& xdot_target, const std::string& link, Vec& qdot_mobile,
                Vec& qdot_mani) const {
    check6(xdot_target);
    split(solveOne(DRC_MODE_QPIK_STEP, &x_target, &xdot_target, nullptr, nullptr, 0, 0, 1, link), qdot_mobile,
          qdot_mani);
  }
  void QPIKCubic(const Pose& x_target, const Vec& xdot_target, const Pose& x_init, const Vec& xdot_init,
                 double current_time, double init_time, double duration, const std::string& link, Vec& qdot_mobile,
                 Vec& qdot_mani) const {
    check6(xdot_target);
    check6(xdot_init);
    split(solveOne(DRC_MODE_QPIK_CUBIC, &x_target, &xdot_target, &x_init, &xdot_init, current_time, init_time,
                   duration, link),
          qdot_mobile, qdot_mani);
  }
  // QPID / QPIDStep / QPIDCubic (robot_controller.cpp:199-250): (qddot_mobile, torque_arm)
  void QPID(const Vec& xddot_target, const std::string& link, Vec& qddot_mobile, Vec& torque_mani) const {
    check6(xddot_target);
    Vec qdd, tau;
    solveOneID(DRC_MODE_QPID, nullptr, &xddot_target, nullptr, nullptr, 0, 0, 1, link, qdd, tau);
    splitID(qdd, tau, qddot_mobile, torque_mani);
  }
  void QPIDStep(const Pose& x_target, const Vec& xdot_target, const std::string& link, Vec& qddot_mobile,
                Vec& torque_mani) const {
    check6(xdot_target);
    Vec qdd, tau;
    solveOneID(DRC_MODE_QPID_STEP, &x_target, &xdot_target, nullptr, nullptr, 0, 0, 1, link, qdd, tau);
    splitID(qdd, tau, qddot_mobile, torque_mani);
  }
  void QPIDCubic(const Pose& x_target, const Vec& xdot_target, const Pose& x_init, const Vec& xdot_init,
                 double current_time, double init_time, double duration, const std::string& link, Vec& qddot_mobile,
                 Vec& torque_mani) const {
    check6(xdot_target);
    check6(xdot_init);
    Vec qdd, tau;
    solveOneID(DRC_MODE_QPID_CUBIC, &x_target, &xdot_target, &x_init, &xdot_init, current_time, init_time, duration,
               link, qdd, tau);
    splitID(qdd, tau, qddot_mobile, torque_mani);
  }

 private:
  void splitID(const Vec& qdd, const Vec& tau, Vec& qddot_mobile, Vec& torque_mani) const {
    const ActuatorIndex& a = robot_data_->getActuatorIndex();
    const int W = robot_data_->getMobileDof(), n = robot_data_->getManipulatorDof();
    qddot_mobile.assign(qdd.begin() + a.mobi_start, qdd.begin() + a.mobi_start + W);
    torque_mani.assign(tau.begin() + a.mani_start, tau.begin() + a.mani_start + n);
  }
  void split(const Vec& eta, Vec& qdot_mobile, Vec& qdot_mani) const {
    const ActuatorIndex& a = robot_data_->getActuatorIndex();
    const int W = robot_data_->getMobileDof(), n = robot_data_->getManipulatorDof();
    qdot_mobile.assign(eta.begin() + a.mobi_start, eta.begin() + a.mobi_start + W);
    qdot_mani.assign(eta.begin() + a.mani_start, eta.begin() + a.mani_start + n);
  }
  std::shared_ptr<RobotData> robot_data_;
};

}  // namespace MobileManipulator
}  // namespace drc_amd

#endif  // DRC_AMD_HPP

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

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <iostream>
#include <map>
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

namespace QP {
// QP::TimeDuration (include/dyros_robot_controller/QP_base.h:19-43), seconds;
// filled by the QP objects below from the kernels' stage stamps
// (drc_qpik_host_timed, include/drc_amd.h)
struct TimeDuration {
  double set_qp = 0, set_cost = 0, set_bound = 0, set_ineq = 0, set_eq = 0, set_constraint = 0, set_solver = 0,
         solve_qp = 0;
  void setZero() { *this = TimeDuration(); }
};
}  // namespace QP

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
  // joint-space dynamics at (q, qdot) (drc_dynamics_host): M, M^-1 row-major
  // n x n, g, nle, c [n]; actuated: the S^T (.) S projections of a mobile
  // manipulator (n = actuated dof)
  struct Dyn {
    Vec M, Minv, g, nle, c;
  };
  Dyn dynamics(const Vec& q, const Vec& qdot, bool actuated = false) const {
    const int n = actuated ? act_ : dof_;
    Dyn d;
    d.M.assign(n * n, 0.0);
    d.Minv.assign(n * n, 0.0);
    d.g.assign(n, 0.0);
    d.nle.assign(n, 0.0);
    d.c.assign(n, 0.0);
    check(drc_dynamics_host(model_, actuated ? 1 : 0, 1, q.data(), qdot.data(), d.M.data(), d.Minv.data(),
                            d.g.data(), d.nle.data(), d.c.data()));
    return d;
  }
  // The control cycle's getters at the stored state: the frame's pose, J and
  // J qdot (getPose / getJacobian / getVelocity, robot_data.cpp:378-422) and,
  // on the first call after updateState, updateDynamics' M, M^-1, g, nle, c
  // (:109-124) -- one drc_state_host round trip per (state, link); the
  // cycle's further getters and moveJointTorqueStep read the cache.
  struct Kin {
    std::array<double, 12> pose;
    Vec jac, xdot;
  };
  const Kin& stateKinematics(const std::string& link) const {
    auto it = kin_.find(link);
    if (it != kin_.end()) return it->second;
    const int fid = frameId(link);
    Kin k;
    k.jac.assign(6 * dof_, 0.0);
    k.xdot.assign(6, 0.0);
    const bool dyn = !dyn_ok_;
    if (dyn) {
      dyn_.M.assign(dof_ * dof_, 0.0);
      dyn_.Minv.assign(dof_ * dof_, 0.0);
      dyn_.g.assign(dof_, 0.0);
      dyn_.nle.assign(dof_, 0.0);
      dyn_.c.assign(dof_, 0.0);
    }
    check(drc_state_host(model_, fid, 1, q_.data(), qdot_.data(), k.pose.data(), k.jac.data(), k.xdot.data(),
                         dyn ? dyn_.M.data() : nullptr, dyn ? dyn_.Minv.data() : nullptr, dyn ? dyn_.g.data() : nullptr,
                         dyn ? dyn_.nle.data() : nullptr, dyn ? dyn_.c.data() : nullptr));
    if (dyn) dyn_ok_ = true;
    return kin_.emplace(link, std::move(k)).first->second;
  }
  // updateDynamics' cached quantities at the stored state (robot_data.cpp:109-124)
  const Dyn& stateDynamics(bool actuated = false) const {
    Dyn& d = actuated ? dyn_act_ : dyn_;
    bool& ok = actuated ? dyn_act_ok_ : dyn_ok_;
    if (!ok) {
      d = dynamics(q_, qdot_, actuated);
      ok = true;
    }
    return d;
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
  void setState(const Vec& q, const Vec& qdot) {
    q_ = q;
    qdot_ = qdot;
    dyn_ok_ = dyn_act_ok_ = false;
    kin_.clear();
  }
  drc_model* model_ = nullptr;
  int dof_ = 0, act_ = 0, mani_ = 0, mobi_ = 0;
  std::array<Vec, 4> lims_;
  Vec q_, qdot_;
  mutable Dyn dyn_, dyn_act_;
  mutable bool dyn_ok_ = false, dyn_act_ok_ = false;
  mutable std::map<std::string, Kin> kin_;  // stateKinematics per link, cleared by updateState
};

inline MinDistResult minDist(const Vec& dist, const Vec& graddot, bool with_grad, bool with_graddot) {
  MinDistResult r;
  const size_t n = dist.size() - 1;
  r.distance = dist[0];
  r.grad = (with_grad || with_graddot) ? Vec(dist.begin() + 1, dist.end()) : Vec(n, 0.0);
  r.grad_dot = with_graddot ? graddot : Vec(n, 0.0);
  return r;
}
inline ManipulabilityResult manip(const Vec& man, const Vec& graddot, bool with_grad, bool with_graddot) {
  ManipulabilityResult r;
  const size_t n = man.size() - 1;
  r.manipulability = man[0];
  r.grad = (with_grad || with_graddot) ? Vec(man.begin() + 1, man.end()) : Vec(n, 0.0);
  r.grad_dot = with_graddot ? graddot : Vec(n, 0.0);
  return r;
}
inline Vec matvec(const Vec& A, const Vec& x, int rows) {  // A rows x x.size(), row-major
  const int cols = static_cast<int>(x.size());
  Vec y(rows, 0.0);
  for (int r = 0; r < rows; ++r)
    for (int c = 0; c < cols; ++c) y[r] += A[r * cols + c] * x[c];
  return y;
}
// DyrosMath::cubicVector / cubicDotVector (math_type_define.h:62-143,179-229)
inline Vec cubicVector(double t, double t0, double tf, const Vec& x0, const Vec& xf, const Vec& xd0, const Vec& xdf,
                       bool dot) {
  Vec out(x0.size());
  for (size_t i = 0; i < x0.size(); ++i) {
    if (t < t0) {
      out[i] = dot ? xd0[i] : x0[i];
      continue;
    }
    if (t > tf) {
      out[i] = dot ? xdf[i] : xf[i];
      continue;
    }
    const double e = t - t0, T = tf - t0, T2 = T * T, T3 = T2 * T, dx = xf[i] - x0[i];
    const double a2 = 3 * dx / T2 - 2 * xd0[i] / T - xdf[i] / T, a3 = -2 * dx / T3 + (xd0[i] + xdf[i]) / T2;
    out[i] = dot ? xd0[i] + 2 * a2 * e + 3 * a3 * e * e : x0[i] + xd0[i] * e + a2 * e * e + a3 * e * e * e;
  }
  return out;
}

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
    setState(q, qdot);
    return true;
  }
  // getters of updateDynamics' quantities (robot_data.h:176-198), n x n row-major
  Vec getMassMatrix() const { return stateDynamics().M; }
  Vec getMassMatrixInv() const { return stateDynamics().Minv; }
  Vec getGravity() const { return stateDynamics().g; }
  Vec getCoriolis() const { return stateDynamics().c; }
  Vec getNonlinearEffects() const { return stateDynamics().nle; }
  // stateless variants (robot_data.h:70-144)
  Vec computeMassMatrix(const Vec& q) const { return dynamics(q, Vec(dof_, 0.0)).M; }
  Vec computeGravity(const Vec& q) const { return dynamics(q, Vec(dof_, 0.0)).g; }
  Vec computeCoriolis(const Vec& q, const Vec& qdot) const { return dynamics(q, qdot).c; }
  Vec computeNonlinearEffects(const Vec& q, const Vec& qdot) const { return dynamics(q, qdot).nle; }
  Vec computeVelocity(const Vec& q, const Vec& qdot, const std::string& link) const {
    return matvec(computeJacobian(q, link), qdot, 6);
  }
  MinDistResult computeMinDistance(const Vec& q, const Vec& qdot, bool with_grad, bool with_graddot,
                                   bool verbose = false) const {
    Stages s = stages(q, qdot, "");
    MinDistResult r = minDist(s.dist, with_graddot ? qpidStages(q, qdot, "").dist_graddot : Vec(), with_grad,
                              with_graddot);
    if (verbose) std::cout << "min distance " << r.distance << " (pair " << s.pair << ")\n";
    return r;
  }
  ManipulabilityResult computeManipulability(const Vec& q, const Vec& qdot, bool with_grad, bool with_graddot,
                                             const std::string& link) const {
    Stages s = stages(q, qdot, link);
    return manip(s.man, with_graddot ? qpidStages(q, qdot, link).man_graddot : Vec(), with_grad, with_graddot);
  }
  Pose computePose(const Vec& q, const std::string& link) const {
    return pose44(stages(q, Vec(dof_, 0.0), link).pose.data());
  }
  Vec computeJacobian(const Vec& q, const std::string& link) const {  // 6 x dof, row-major
    return stages(q, Vec(dof_, 0.0), link).jac;
  }
  // the cycle's getters: one round trip per state and link (stateKinematics)
  Pose getPose(const std::string& link) const { return pose44(stateKinematics(link).pose.data()); }
  Vec getJacobian(const std::string& link) const { return stateKinematics(link).jac; }
  Vec getVelocity(const std::string& link) const {  // J qdot (robot_data.cpp:419-422)
    return stateKinematics(link).xdot;
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

 protected:
  RobotData() = default;  // MobileManipulator::RobotData adopts its own model
};

}  // namespace Manipulator

namespace Mobile {

using KinematicParam = drc_kinematic_param;

// Mobile::RobotData (include/dyros_robot_controller/mobile/robot_data.h,
// src/mobile/robot_data.cpp): wheel state, FK Jacobian, base twist.  Host
// arithmetic (a 3 x W matrix per call) through the C-ABI.
class RobotData {
 public:
  explicit RobotData(const KinematicParam& param) : param_(param) {
    Vec J(3 * DRC_MAX_WHEELS), w0(DRC_MAX_WHEELS, 0.0);
    check(drc_mobile_fk_jacobian(&param_, w0.data(), J.data(), &wheel_num_));
    wheel_pos_.assign(wheel_num_, 0.0);
    wheel_vel_.assign(wheel_num_, 0.0);
    J_mobile_.assign(J.begin(), J.begin() + 3 * wheel_num_);
    base_vel_.assign(3, 0.0);
  }
  virtual ~RobotData() = default;
  std::string getVerbose() const {
    static const char* names[3] = {"Differential", "Mecanum", "Caster"};
    return std::string("type ") + (param_.type >= 0 && param_.type < 3 ? names[param_.type] : "Unknown") +
           ", wheel_num " + std::to_string(wheel_num_) + ", wheel_radius " + std::to_string(param_.wheel_radius);
  }
  bool updateState(const Vec& wheel_pos, const Vec& wheel_vel) {
    if (static_cast<int>(wheel_pos.size()) != wheel_num_ || static_cast<int>(wheel_vel.size()) != wheel_num_)
      return false;
    wheel_pos_ = wheel_pos;
    wheel_vel_ = wheel_vel;
    J_mobile_ = computeFKJacobian(wheel_pos);
    base_vel_ = matvec(J_mobile_, wheel_vel_, 3);
    return true;
  }
  Vec computeBaseVel(const Vec& wheel_pos, const Vec& wheel_vel) const {
    return matvec(computeFKJacobian(wheel_pos), wheel_vel, 3);
  }
  Vec computeFKJacobian(const Vec& wheel_pos) const {  // 3 x W row-major
    if (static_cast<int>(wheel_pos.size()) != wheel_num_) throw std::runtime_error("wheel_pos must be of size wheel_num.");
    Vec J(3 * DRC_MAX_WHEELS);
    int W = 0;
    check(drc_mobile_fk_jacobian(&param_, wheel_pos.data(), J.data(), &W));
    return Vec(J.begin(), J.begin() + 3 * W);
  }
  int getWheelNum() const { return wheel_num_; }
  const KinematicParam& getKineParam() const { return param_; }
  const Vec& getWheelPosition() const { return wheel_pos_; }
  const Vec& getWheelVelocity() const { return wheel_vel_; }
  const Vec& getBaseVel() const { return base_vel_; }
  const Vec& getFKJacobian() const { return J_mobile_; }

 protected:
  KinematicParam param_;
  int wheel_num_ = 0;
  Vec wheel_pos_, wheel_vel_, J_mobile_, base_vel_;
};

// Mobile::RobotController (src/mobile/robot_controller.cpp): wheel IK and
// base-velocity saturation.
class RobotController {
 public:
  RobotController(double dt, std::shared_ptr<RobotData> robot_data) : dt_(dt), robot_data_(std::move(robot_data)) {}
  Vec computeIKJacobian() const {  // W x 3 row-major (:55-125)
    const Vec& wp = robot_data_->getWheelPosition();
    Vec J(DRC_MAX_WHEELS * 3);
    int W = 0;
    check(drc_mobile_ik_jacobian(&robot_data_->getKineParam(), wp.data(), J.data(), &W));
    return Vec(J.begin(), J.begin() + 3 * W);
  }
  Vec computeWheelVel(const Vec& base_vel) const {  // (:48-52)
    if (base_vel.size() != 3) throw std::runtime_error("base_vel must be of size 3.");
    return matvec(computeIKJacobian(), base_vel, robot_data_->getWheelNum());
  }
  // VelocityCommand (:18-46): speed and yaw-rate saturation, then wheel IK
  Vec VelocityCommand(const Vec& desired_base_vel) const {
    if (desired_base_vel.size() != 3) throw std::runtime_error("desired_base_vel must be of size 3.");
    const KinematicParam& p = robot_data_->getKineParam();
    double vx = desired_base_vel[0], vy = desired_base_vel[1];
    double speed = std::sqrt(vx * vx + vy * vy), dx = 0, dy = 0;
    if (std::fabs(speed) >= 1e-4) {
      dx = vx / speed;
      dy = vy / speed;
    }
    speed = std::min(std::max(speed, -p.max_lin_speed), p.max_lin_speed);
    const double w = std::min(std::max(desired_base_vel[2], -p.max_ang_speed), p.max_ang_speed);
    return computeWheelVel({dx * speed, dy * speed, w});
  }

 private:
  double dt_;
  std::shared_ptr<RobotData> robot_data_;
};

}  // namespace Mobile

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
      : ControllerBase(dt, robot_data.get()), robot_data_(std::move(robot_data)),
        Kp_joint_(robot_data_->getDof(), 400.0), Kv_joint_(robot_data_->getDof(), 40.0) {}
  // joint-space gains and helpers (robot_controller.cpp:21-155)
  void setJointGain(const Vec& Kp, const Vec& Kv) {
    if (Kp.size() != Kp_joint_.size() || Kv.size() != Kv_joint_.size())
      throw std::runtime_error("Kp and Kv must be of size dof_.");
    Kp_joint_ = Kp;
    Kv_joint_ = Kv;
  }
  void setJointKpGain(const Vec& Kp) {
    if (Kp.size() != Kp_joint_.size()) throw std::runtime_error("Kp must be of size dof_.");
    Kp_joint_ = Kp;
  }
  void setJointKvGain(const Vec& Kv) {
    if (Kv.size() != Kv_joint_.size()) throw std::runtime_error("Kv must be of size dof_.");
    Kv_joint_ = Kv;
  }
  Vec moveJointPositionCubic(const Vec& q_target, const Vec& qdot_target, const Vec& q_init, const Vec& qdot_init,
                             double current_time, double init_time, double duration) const {
    return cubicVector(current_time, init_time, init_time + duration, q_init, q_target, qdot_init, qdot_target, false);
  }
  Vec moveJointVelocityCubic(const Vec& q_target, const Vec& qdot_target, const Vec& q_init, const Vec& qdot_init,
                             double current_time, double init_time, double duration) const {
    return cubicVector(current_time, init_time, init_time + duration, q_init, q_target, qdot_init, qdot_target, true);
  }
  // M qddot + g with the cached M, g of the stored state (robot_controller.cpp:115-118)
  Vec moveJointTorqueStep(const Vec& qddot_target) const {
    const int n = robot_data_->getDof();
    Vec tau = matvec(robot_data_->getMassMatrix(), qddot_target, n), g = robot_data_->getGravity();
    for (int i = 0; i < n; ++i) tau[i] += g[i];
    return tau;
  }
  Vec moveJointTorqueStep(const Vec& q_target, const Vec& qdot_target) const {  // (:120-125)
    const Vec &q = robot_data_->getJointPosition(), &qd = robot_data_->getJointVelocity();
    Vec qdd(q.size());
    for (size_t i = 0; i < q.size(); ++i)
      qdd[i] = Kp_joint_[i] * (q_target[i] - q[i]) + Kv_joint_[i] * (qdot_target[i] - qd[i]);
    return moveJointTorqueStep(qdd);
  }
  Vec moveJointTorqueCubic(const Vec& q_target, const Vec& qdot_target, const Vec& q_init, const Vec& qdot_init,
                           double current_time, double init_time, double duration) const {
    return moveJointTorqueStep(
        moveJointPositionCubic(q_target, qdot_target, q_init, qdot_init, current_time, init_time, duration),
        moveJointVelocityCubic(q_target, qdot_target, q_init, qdot_init, current_time, init_time, duration));
  }
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
  Vec Kp_joint_, Kv_joint_;
};

}  // namespace Manipulator

namespace MobileManipulator {

using KinematicParam = drc_kinematic_param;
using JointIndex = drc_joint_index;
using ActuatorIndex = drc_actuator_index;

// MobileManipulator::RobotData (mobile_manipulator/robot_data.h:42): a
// Manipulator::RobotData over the whole-body model and a Mobile::RobotData of
// the base, as the reference's multiple inheritance.
class RobotData : public Manipulator::RobotData, public Mobile::RobotData {
 public:
  RobotData(const KinematicParam& param, const JointIndex& joint_idx, const ActuatorIndex& actuator_idx,
            const std::string& urdf, const std::string& srdf = "", const std::string& packages = "", int device = 0)
      : Mobile::RobotData(param), jidx_(joint_idx), aidx_(actuator_idx) {
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
  // getActuatorVector (:429-437)
  Vec actuatorVector(const Vec& v_mobile, const Vec& v_mani) const {
    Vec v(act_, 0.0);
    for (size_t i = 0; i < v_mobile.size(); ++i) v[aidx_.mobi_start + i] = v_mobile[i];
    for (size_t i = 0; i < v_mani.size(); ++i) v[aidx_.mani_start + i] = v_mani[i];
    return v;
  }
  bool updateState(const Vec& q_virtual, const Vec& q_mobile, const Vec& q_mani, const Vec& qdot_virtual,
                   const Vec& qdot_mobile, const Vec& qdot_mani) {
    if (q_virtual.size() != 3 || static_cast<int>(q_mobile.size()) != mobi_ ||
        static_cast<int>(q_mani.size()) != mani_)
      return false;
    setState(jointVector(q_virtual, q_mobile, q_mani), jointVector(qdot_virtual, qdot_mobile, qdot_mani));
    Mobile::RobotData::updateState(q_mobile, qdot_mobile);
    return true;
  }
  int getManipulatorDof() const { return mani_; }
  int getMobileDof() const { return mobi_; }
  int getActuatordDof() const { return act_; }  // (sic) mobile_manipulator/robot_data.h:359
  const JointIndex& getJointIndex() const { return jidx_; }
  const ActuatorIndex& getActuatorIndex() const { return aidx_; }
  Vec block(const Vec& v, int start, int n) const { return Vec(v.begin() + start, v.begin() + start + n); }
  Vec getVirtualJointPosition() const { return block(q_, jidx_.virtual_start, 3); }
  Vec getMobileJointPosition() const { return block(q_, jidx_.mobi_start, mobi_); }
  Vec getManiJointPosition() const { return block(q_, jidx_.mani_start, mani_); }
  Vec getVirtualJointVelocity() const { return block(qdot_, jidx_.virtual_start, 3); }
  Vec getMobileJointVelocity() const { return block(qdot_, jidx_.mobi_start, mobi_); }
  Vec getManiJointVelocity() const { return block(qdot_, jidx_.mani_start, mani_); }
  Vec getJointPositionActuated() const { return actuatorVector(getMobileJointPosition(), getManiJointPosition()); }
  Vec getJointVelocityActuated() const { return actuatorVector(getMobileJointVelocity(), getManiJointVelocity()); }
  // mobile base (:344-357): J_mobile at the wheel positions and the base twist
  Vec computeMobileFKJacobian(const Vec& q_mobile) const { return computeFKJacobian(q_mobile); }
  Vec computeMobileBaseVel(const Vec& q_mobile, const Vec& qdot_mobile) const {
    return computeBaseVel(q_mobile, qdot_mobile);
  }
  Vec getMobileFKJacobian() const { return computeFKJacobian(getMobileJointPosition()); }
  Vec getMobileBaseVel() const { return computeBaseVel(getMobileJointPosition(), getMobileJointVelocity()); }
  // selection matrix S (dof x A, row-major; :22-25,115-120,367-387)
  Vec computeSelectionMatrix(const Vec& q_virtual, const Vec& q_mobile) const {
    Vec S(dof_ * act_, 0.0), Jm = computeFKJacobian(q_mobile);
    for (int i = 0; i < mani_; ++i) S[(jidx_.mani_start + i) * act_ + aidx_.mani_start + i] = 1;
    for (int i = 0; i < mobi_; ++i) S[(jidx_.mobi_start + i) * act_ + aidx_.mobi_start + i] = 1;
    const double cy = std::cos(q_virtual.at(2)), sy = std::sin(q_virtual.at(2));
    const double Rz[3][3] = {{cy, -sy, 0}, {sy, cy, 0}, {0, 0, 1}};
    for (int r = 0; r < 3; ++r)
      for (int w = 0; w < mobi_; ++w) {
        double t = 0;
        for (int k = 0; k < 3; ++k) t += Rz[r][k] * Jm[k * mobi_ + w];
        S[(jidx_.virtual_start + r) * act_ + aidx_.mobi_start + w] = t;
      }
    return S;
  }
  Vec getSelectionMatrix() const { return computeSelectionMatrix(getVirtualJointPosition(), getMobileJointPosition()); }
  // J S (6 x A row-major; :389-415, Sdot neglected as the reference)
  Vec times(const Vec& J, const Vec& S) const {
    Vec out(6 * act_, 0.0);
    for (int r = 0; r < 6; ++r)
      for (int k = 0; k < dof_; ++k)
        for (int a = 0; a < act_; ++a) out[r * act_ + a] += J[r * dof_ + k] * S[k * act_ + a];
    return out;
  }
  Vec computeJacobianActuated(const Vec& q_virtual, const Vec& q_mobile, const Vec& q_mani,
                              const std::string& link) const {
    return times(computeJacobian(jointVector(q_virtual, q_mobile, q_mani), link),
                 computeSelectionMatrix(q_virtual, q_mobile));
  }
  Vec computeJacobianTimeVariationActuated(const Vec& q_virtual, const Vec& q_mobile, const Vec& q_mani,
                                           const Vec& qdot_virtual, const Vec& qdot_mobile, const Vec& qdot_mani,
                                           const std::string& link) const {
    return times(computeJacobianTimeVariation(jointVector(q_virtual, q_mobile, q_mani),
                                              jointVector(qdot_virtual, qdot_mobile, qdot_mani), link),
                 computeSelectionMatrix(q_virtual, q_mobile));
  }
  Vec getJacobianActuated(const std::string& link) const { return times(getJacobian(link), getSelectionMatrix()); }
  Vec getJacobianActuatedTimeVariation(const std::string& link) const {
    return times(getJacobianTimeVariation(link), getSelectionMatrix());
  }
  // actuated dynamics (:126-144 cached, :187-227 stateless); M n x n row-major
  Vec getMassMatrixActuated() const { return stateDynamics(true).M; }
  Vec getMassMatrixActuatedInv() const { return stateDynamics(true).Minv; }
  Vec getGravityActuated() const { return stateDynamics(true).g; }
  Vec getCoriolisActuated() const { return stateDynamics(true).c; }
  Vec getNonlinearEffectsActuated() const { return stateDynamics(true).nle; }
  // the actuated velocities (qdot_mobile, qdot_mani) map to joints by S (virtual rows = Rz J_mobile)
  Vec actuatedJointVelocity(const Vec& q_virtual, const Vec& q_mobile, const Vec& qdot_mobile,
                            const Vec& qdot_mani) const {
    return matvec(computeSelectionMatrix(q_virtual, q_mobile), actuatorVector(qdot_mobile, qdot_mani), dof_);
  }
  Vec computeMassMatrixActuated(const Vec& q_virtual, const Vec& q_mobile, const Vec& q_mani) const {
    return dynamics(jointVector(q_virtual, q_mobile, q_mani), Vec(dof_, 0.0), true).M;
  }
  Vec computeGravityActuated(const Vec& q_virtual, const Vec& q_mobile, const Vec& q_mani) const {
    return dynamics(jointVector(q_virtual, q_mobile, q_mani), Vec(dof_, 0.0), true).g;
  }
  Vec computeCoriolisActuated(const Vec& q_virtual, const Vec& q_mobile, const Vec& q_mani, const Vec& qdot_mobile,
                              const Vec& qdot_mani) const {
    return dynamics(jointVector(q_virtual, q_mobile, q_mani),
                    actuatedJointVelocity(q_virtual, q_mobile, qdot_mobile, qdot_mani), true).c;
  }
  Vec computeNonlinearEffectsActuated(const Vec& q_virtual, const Vec& q_mobile, const Vec& q_mani,
                                      const Vec& qdot_mobile, const Vec& qdot_mani) const {
    return dynamics(jointVector(q_virtual, q_mobile, q_mani),
                    actuatedJointVelocity(q_virtual, q_mobile, qdot_mobile, qdot_mani), true).nle;
  }
  // whole-body task space with the joint blocks (:229-286)
  ManipulabilityResult computeManipulability(const Vec& q_mani, const Vec& qdot_mani, bool with_grad,
                                             bool with_graddot, const std::string& link) const {
    return Manipulator::RobotData::computeManipulability(jointVector(Vec(3, 0.0), Vec(mobi_, 0.0), q_mani),
                                                         jointVector(Vec(3, 0.0), Vec(mobi_, 0.0), qdot_mani),
                                                         with_grad, with_graddot, link);
  }

 private:
  JointIndex jidx_;
  ActuatorIndex aidx_;
};

class RobotController : public ControllerBase {
 public:
  RobotController(double dt, std::shared_ptr<RobotData> robot_data)
      : ControllerBase(dt, static_cast<const Manipulator::RobotData*>(robot_data.get())),
        robot_data_(std::move(robot_data)), Kp_mani_joint_(robot_data_->getManipulatorDof(), 400.0),
        Kv_mani_joint_(robot_data_->getManipulatorDof(), 40.0) {}
  // arm joint-space gains and helpers (mobile_manipulator/robot_controller.cpp:24-145)
  void setManipulatorJointGain(const Vec& Kp, const Vec& Kv) {
    if (Kp.size() != Kp_mani_joint_.size() || Kv.size() != Kv_mani_joint_.size())
      throw std::runtime_error("Kp and Kv must be of size mani_dof_.");
    Kp_mani_joint_ = Kp;
    Kv_mani_joint_ = Kv;
  }
  void setManipulatorJointKpGain(const Vec& Kp) {
    if (Kp.size() != Kp_mani_joint_.size()) throw std::runtime_error("Kp must be of size mani_dof_.");
    Kp_mani_joint_ = Kp;
  }
  void setManipulatorJointKvGain(const Vec& Kv) {
    if (Kv.size() != Kv_mani_joint_.size()) throw std::runtime_error("Kv must be of size mani_dof_.");
    Kv_mani_joint_ = Kv;
  }
  Vec moveManipulatorJointPositionCubic(const Vec& q_target, const Vec& qdot_target, const Vec& q_init,
                                        const Vec& qdot_init, double current_time, double init_time,
                                        double duration) const {
    return cubicVector(current_time, init_time, init_time + duration, q_init, q_target, qdot_init, qdot_target, false);
  }
  // arm block of M qddot + g at the stored state (:96-104)
  Vec moveManipulatorJointTorqueStep(const Vec& qddot_mani_target) const {
    const int n = robot_data_->getManipulatorDof(), D = robot_data_->getDof();
    const int s0 = robot_data_->getJointIndex().mani_start;
    const Vec &M = robot_data_->getMassMatrix(), &g = robot_data_->getGravity();
    Vec tau(n, 0.0);
    for (int i = 0; i < n; ++i) {
      tau[i] = g[s0 + i];
      for (int j = 0; j < n; ++j) tau[i] += M[(s0 + i) * D + s0 + j] * qddot_mani_target[j];
    }
    return tau;
  }
  Vec moveManipulatorJointTorqueStep(const Vec& q_mani_target, const Vec& qdot_mani_target) const {  // (:106-114)
    const Vec q = robot_data_->getManiJointPosition(), qd = robot_data_->getManiJointVelocity();
    Vec qdd(q.size());
    for (size_t i = 0; i < q.size(); ++i)
      qdd[i] = Kp_mani_joint_[i] * (q_mani_target[i] - q[i]) + Kv_mani_joint_[i] * (qdot_mani_target[i] - qd[i]);
    return moveManipulatorJointTorqueStep(qdd);
  }
  Vec moveManipulatorJointTorqueCubic(const Vec& q_target, const Vec& qdot_target, const Vec& q_init,
                                      const Vec& qdot_init, double current_time, double init_time,
                                      double duration) const {
    const double tf = init_time + duration;
    return moveManipulatorJointTorqueStep(
        cubicVector(current_time, init_time, tf, q_init, q_target, qdot_init, qdot_target, false),
        cubicVector(current_time, init_time, tf, q_init, q_target, qdot_init, qdot_target, true));
  }
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
  Vec Kp_mani_joint_, Kv_mani_joint_;
};

}  // namespace MobileManipulator

// ---- the QP layer (include/dyros_robot_controller/{manipulator,mobile_manipulator}/QP_{IK,ID}.h)
// QP objects over the robot data's stored state, for callers that drive the
// QP directly instead of through the controller.  The velocity QP solves
// through drc_qpik_host_timed (the same kernels as the controllers' QPIK) and
// fills QP::TimeDuration from the kernels' stage stamps.
namespace detail {
// QPIK::setDesiredTaskVel / getOptJointVel (QP_IK.cpp:47-67; MoMa QP_IK.cpp:37-57)
class QPIKObject {
 public:
  void setDesiredTaskVel(const Vec& xdot_desired, const std::string& link_name) {
    if (xdot_desired.size() != 6) throw std::runtime_error("xdot_desired must be of size 6.");
    xdot_desired_ = xdot_desired;
    link_name_ = link_name;
  }
  // false (opt_qdot zero, time_status zero) unless the QP is Solved
  bool getOptJointVel(Vec& opt_qdot, QP::TimeDuration& time_status) const {
    const int A = model_->getActuatorDof();
    opt_qdot.assign(A, 0.0);
    if (xdot_desired_.size() != 6) throw std::runtime_error("setDesiredTaskVel has not been called.");
    drc_qpik_params p = params_;
    p.mode = DRC_MODE_QPIK;  // the QP's task velocity is xdot_desired itself
    p.frame_id = model_->frameId(link_name_);
    drc_time_duration t;
    int32_t status = 0, iters = 0;
    check(drc_qpik_host_timed(model_->handle(), &p, 1, model_->getJointPosition().data(),
                              model_->getJointVelocity().data(), nullptr, xdot_desired_.data(), nullptr, nullptr,
                              opt_qdot.data(), &status, &iters, &t));
    iters_ = iters;
    status_ = status;
    if (status != DRC_STATUS_SOLVED) {
      opt_qdot.assign(A, 0.0);
      time_status.setZero();
      return false;
    }
    time_status.set_qp = t.set_qp;
    time_status.set_cost = t.set_cost;
    time_status.set_bound = t.set_bound;
    time_status.set_ineq = t.set_ineq;
    time_status.set_eq = t.set_eq;
    time_status.set_constraint = t.set_constraint;
    time_status.set_solver = t.set_solver;
    time_status.solve_qp = t.solve_qp;
    return true;
  }
  // extensions: solver settings ("exact" certified optimum by default, or the
  // reference's OSQP settings) and the last solve's status / ADMM iterations
  void setExact(bool exact) { params_.solver = model_->defaultParams(exact).solver; }
  int lastStatus() const { return status_; }
  int lastIterations() const { return iters_; }

 protected:
  explicit QPIKObject(const ModelBase* model) : model_(model), params_(model->defaultParams(true)) {}
  const ModelBase* model_;
  drc_qpik_params params_;
  Vec xdot_desired_;
  std::string link_name_;
  mutable int status_ = 0, iters_ = 0;
};
// QPID::setDesiredTaskAcc / getOptJoint (QP_ID.cpp:66-90; MoMa QP_ID.cpp:49-73)
class QPIDObject {
 public:
  void setDesiredTaskAcc(const Vec& xddot_desired, const std::string& link_name) {
    if (xddot_desired.size() != 6) throw std::runtime_error("xddot_desired must be of size 6.");
    xddot_desired_ = xddot_desired;
    link_name_ = link_name;
  }
  // false (both outputs zero, time_status zero) unless the QP is Solved;
  // time_status.set_solver holds the call's wall time (the QPID kernels carry
  // no stage stamps)
  bool getOptJoint(Vec& opt_qddot, Vec& opt_torque, QP::TimeDuration& time_status) const {
    const int A = model_->getActuatorDof();
    opt_qddot.assign(A, 0.0);
    opt_torque.assign(A, 0.0);
    if (xddot_desired_.size() != 6) throw std::runtime_error("setDesiredTaskAcc has not been called.");
    drc_qpik_params p = params_;
    p.mode = DRC_MODE_QPID;
    p.frame_id = model_->frameId(link_name_);
    int32_t status = 0, iters = 0;
    const auto t0 = std::chrono::steady_clock::now();
    check(drc_qpid_host(model_->handle(), &p, 1, model_->getJointPosition().data(), model_->getJointVelocity().data(),
                        nullptr, xddot_desired_.data(), nullptr, nullptr, opt_qddot.data(), opt_torque.data(), &status,
                        &iters));
    const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    status_ = status;
    time_status.setZero();
    if (status != DRC_STATUS_SOLVED) {  // the kernel's failure output is the controller's (tau = g): zero here
      opt_qddot.assign(A, 0.0);
      opt_torque.assign(A, 0.0);
      return false;
    }
    time_status.set_solver = wall;
    return true;
  }
  void setExact(bool exact) {
    drc_qpik_params d;
    check(drc_default_qpid_params(model_->handle(), exact ? 1 : 0, &d));
    params_.solver = d.solver;
  }
  int lastStatus() const { return status_; }

 protected:
  explicit QPIDObject(const ModelBase* model) : model_(model) {
    check(drc_default_qpid_params(model_->handle(), 1, &params_));
  }
  const ModelBase* model_;
  drc_qpik_params params_;
  Vec xddot_desired_;
  std::string link_name_;
  mutable int status_ = 0;
};
}  // namespace detail

namespace Manipulator {
// Manipulator::QPIK (manipulator/QP_IK.h:16-100): x = [qdot | slacks]; the
// optimal joint velocity (dof)
class QPIK : public detail::QPIKObject {
 public:
  explicit QPIK(std::shared_ptr<RobotData> robot_data)
      : detail::QPIKObject(robot_data.get()), robot_data_(std::move(robot_data)) {}

 private:
  std::shared_ptr<RobotData> robot_data_;
};
// Manipulator::QPID (manipulator/QP_ID.h): optimal qddot and torque (dof each)
class QPID : public detail::QPIDObject {
 public:
  explicit QPID(std::shared_ptr<RobotData> robot_data)
      : detail::QPIDObject(robot_data.get()), robot_data_(std::move(robot_data)) {}

 private:
  std::shared_ptr<RobotData> robot_data_;
};
}  // namespace Manipulator

namespace MobileManipulator {
// MobileManipulator::QPIK (mobile_manipulator/QP_IK.h:16-93): x = eta, the
// actuated velocities in ActuatorIndex order
class QPIK : public detail::QPIKObject {
 public:
  explicit QPIK(std::shared_ptr<RobotData> robot_data)
      : detail::QPIKObject(static_cast<const Manipulator::RobotData*>(robot_data.get())),
        robot_data_(std::move(robot_data)) {}

 private:
  std::shared_ptr<RobotData> robot_data_;
};
// MobileManipulator::QPID (mobile_manipulator/QP_ID.h): eta_dot and the
// actuated torques
class QPID : public detail::QPIDObject {
 public:
  explicit QPID(std::shared_ptr<RobotData> robot_data)
      : detail::QPIDObject(static_cast<const Manipulator::RobotData*>(robot_data.get())),
        robot_data_(std::move(robot_data)) {}

 private:
  std::shared_ptr<RobotData> robot_data_;
};
}  // namespace MobileManipulator
}  // namespace drc_amd

#endif  // DRC_AMD_HPP

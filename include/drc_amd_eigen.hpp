// drc_amd_eigen.hpp — source-compatible layer for the reference's C++ call
// sites: namespace drc with Eigen-typed signatures, over the std:: façade in
// drc_amd.hpp (and so over the C-ABI / HIP kernels).
//
//   reference header (include/dyros_robot_controller/...)      here
//   manipulator/robot_data.h:59    bool updateState(VectorXd, VectorXd)         same
//                           :178   MatrixXd getMassMatrix()                     same
//                           :193   VectorXd getGravity()                        same
//                           :206   Affine3d getPose(link)                       same
//                           :212   MatrixXd getJacobian(link)                   same
//                           :224   VectorXd getVelocity(link)                   same
//   manipulator/robot_controller.h:27   RobotController(dt, shared_ptr<RobotData>)  same
//                           :108-130    moveJointTorqueStep / joint cubics       same
//                           :295-321    VectorXd QPIK / QPIKStep / QPIKCubic      same
//                           QPID / QPIDStep / QPIDCubic                           same
//   mobile_manipulator/robot_data.h:26,77     ctor, updateState(6 x VectorXd)     same
//   mobile_manipulator/robot_controller.h:30,130-173
//                           void QPIK*(..., VectorXd& qdot_mobile, VectorXd& qdot_mani)  same
//   QP_base.h:19-43        QP::TimeDuration                                    same
//   manipulator/QP_IK.h:25-38, mobile_manipulator/QP_IK.h:25-38
//                           QPIK(shared_ptr<RobotData>), setDesiredTaskVel, getOptJointVel  same
//   manipulator/QP_ID.h:25-39, mobile_manipulator/QP_ID.h:25-39
//                           QPID(shared_ptr<RobotData>), setDesiredTaskAcc, getOptJoint     same
//
// A reference example such as examples/C++/src/fr3_controller.cpp switches by
// including this header instead of the reference's and linking libdrc_amd.so;
// the calls above keep their shape.  Needs Eigen (VectorXd, MatrixXd,
// Affine3d: data(), size(), matrix()); nothing else of Eigen is used.
#ifndef DRC_AMD_EIGEN_HPP
#define DRC_AMD_EIGEN_HPP

#include <Eigen/Dense>

#include <algorithm>
#include <memory>
#include <string>
#include <utility>

#include "drc_amd.hpp"

namespace drc {

using Eigen::Affine3d;
using Eigen::MatrixXd;
using Eigen::VectorXd;

namespace eigen_detail {
inline drc_amd::Vec vec(const VectorXd& v) { return drc_amd::Vec(v.data(), v.data() + v.size()); }
inline VectorXd evec(const drc_amd::Vec& v) {
  VectorXd r(static_cast<Eigen::Index>(v.size()));
  std::copy(v.begin(), v.end(), r.data());
  return r;
}
inline drc_amd::Pose pose(const Affine3d& T) {  // Affine3d::matrix() is 4x4 column-major
  drc_amd::Pose p;
  std::copy(T.matrix().data(), T.matrix().data() + 16, p.begin());
  return p;
}
inline Affine3d affine(const drc_amd::Pose& p) {
  Affine3d T;
  std::copy(p.begin(), p.end(), T.matrix().data());
  return T;
}
inline MatrixXd rowmajor(const drc_amd::Vec& v, int rows, int cols) {
  MatrixXd M(rows, cols);
  for (int r = 0; r < rows; ++r)
    for (int c = 0; c < cols; ++c) M(r, c) = v[static_cast<size_t>(r) * cols + c];
  return M;
}
}  // namespace eigen_detail

namespace QP {
using TimeDuration = drc_amd::QP::TimeDuration;
}

namespace Manipulator {

class RobotData {
 public:
  RobotData(const std::string& urdf_path, const std::string& srdf_path = "", const std::string& packages_path = "")
      : impl_(std::make_shared<drc_amd::Manipulator::RobotData>(urdf_path, srdf_path, packages_path)) {}
  virtual ~RobotData() = default;
  virtual bool updateState(const VectorXd& q, const VectorXd& qdot) {
    return impl_->updateState(eigen_detail::vec(q), eigen_detail::vec(qdot));
  }
  int getDof() const { return impl_->getDof(); }
  VectorXd getJointPosition() const { return eigen_detail::evec(impl_->getJointPosition()); }
  VectorXd getJointVelocity() const { return eigen_detail::evec(impl_->getJointVelocity()); }
  std::pair<VectorXd, VectorXd> getJointPositionLimit() const {
    auto l = impl_->getJointPositionLimit();
    return {eigen_detail::evec(l.first), eigen_detail::evec(l.second)};
  }
  std::pair<VectorXd, VectorXd> getJointVelocityLimit() const {
    auto l = impl_->getJointVelocityLimit();
    return {eigen_detail::evec(l.first), eigen_detail::evec(l.second)};
  }
  virtual MatrixXd getMassMatrix() const { return eigen_detail::rowmajor(impl_->getMassMatrix(), getDof(), getDof()); }
  virtual MatrixXd getMassMatrixInv() const {
    return eigen_detail::rowmajor(impl_->getMassMatrixInv(), getDof(), getDof());
  }
  virtual VectorXd getGravity() const { return eigen_detail::evec(impl_->getGravity()); }
  virtual VectorXd getCoriolis() const { return eigen_detail::evec(impl_->getCoriolis()); }
  virtual VectorXd getNonlinearEffects() const { return eigen_detail::evec(impl_->getNonlinearEffects()); }
  virtual Affine3d getPose(const std::string& link_name) const { return eigen_detail::affine(impl_->getPose(link_name)); }
  virtual MatrixXd getJacobian(const std::string& link_name) {
    return eigen_detail::rowmajor(impl_->getJacobian(link_name), 6, getDof());
  }
  virtual VectorXd getVelocity(const std::string& link_name) {
    return eigen_detail::evec(impl_->getVelocity(link_name));
  }
  // the std:: façade object (batched entry points, stage outputs)
  const std::shared_ptr<drc_amd::Manipulator::RobotData>& impl() const { return impl_; }

 protected:
  RobotData() = default;
  std::shared_ptr<drc_amd::Manipulator::RobotData> impl_;
};

class RobotController {
 public:
  RobotController(const double& dt, std::shared_ptr<RobotData> robot_data)
      : robot_data_(std::move(robot_data)), impl_(dt, robot_data_->impl()) {}
  virtual ~RobotController() = default;
  virtual void setJointGain(const VectorXd& Kp, const VectorXd& Kv) {
    impl_.setJointGain(eigen_detail::vec(Kp), eigen_detail::vec(Kv));
  }
  virtual void setTaskGain(const VectorXd& Kp, const VectorXd& Kv) {
    impl_.setTaskGain(eigen_detail::vec(Kp), eigen_detail::vec(Kv));
  }
  virtual void setTaskKpGain(const VectorXd& Kp) { impl_.setTaskKpGain(eigen_detail::vec(Kp)); }
  virtual void setTaskKvGain(const VectorXd& Kv) { impl_.setTaskKvGain(eigen_detail::vec(Kv)); }
  virtual VectorXd moveJointPositionCubic(const VectorXd& q_target, const VectorXd& qdot_target,
                                          const VectorXd& q_init, const VectorXd& qdot_init,
                                          const double& current_time, const double& init_time,
                                          const double& duration) {
    return eigen_detail::evec(impl_.moveJointPositionCubic(eigen_detail::vec(q_target), eigen_detail::vec(qdot_target),
                                                           eigen_detail::vec(q_init), eigen_detail::vec(qdot_init),
                                                           current_time, init_time, duration));
  }
  virtual VectorXd moveJointVelocityCubic(const VectorXd& q_target, const VectorXd& qdot_target,
                                          const VectorXd& q_init, const VectorXd& qdot_init,
                                          const double& current_time, const double& init_time,
                                          const double& duration) {
    return eigen_detail::evec(impl_.moveJointVelocityCubic(eigen_detail::vec(q_target), eigen_detail::vec(qdot_target),
                                                           eigen_detail::vec(q_init), eigen_detail::vec(qdot_init),
                                                           current_time, init_time, duration));
  }
  virtual VectorXd moveJointTorqueStep(const VectorXd& qddot_target) {
    return eigen_detail::evec(impl_.moveJointTorqueStep(eigen_detail::vec(qddot_target)));
  }
  virtual VectorXd moveJointTorqueStep(const VectorXd& q_target, const VectorXd& qdot_target) {
    return eigen_detail::evec(impl_.moveJointTorqueStep(eigen_detail::vec(q_target), eigen_detail::vec(qdot_target)));
  }
  virtual VectorXd QPIK(const VectorXd& xdot_target, const std::string& link_name) {
    return eigen_detail::evec(impl_.QPIK(eigen_detail::vec(xdot_target), link_name));
  }
  virtual VectorXd QPIKStep(const Affine3d& x_target, const VectorXd& xdot_target, const std::string& link_name) {
    return eigen_detail::evec(impl_.QPIKStep(eigen_detail::pose(x_target), eigen_detail::vec(xdot_target), link_name));
  }
  virtual VectorXd QPIKCubic(const Affine3d& x_target, const VectorXd& xdot_target, const Affine3d& x_init,
                             const VectorXd& xdot_init, const double& current_time, const double& init_time,
                             const double& duration, const std::string& link_name) {
    return eigen_detail::evec(impl_.QPIKCubic(eigen_detail::pose(x_target), eigen_detail::vec(xdot_target),
                                              eigen_detail::pose(x_init), eigen_detail::vec(xdot_init), current_time,
                                              init_time, duration, link_name));
  }
  virtual VectorXd QPID(const VectorXd& xddot_target, const std::string& link_name) {
    return eigen_detail::evec(impl_.QPID(eigen_detail::vec(xddot_target), link_name));
  }
  virtual VectorXd QPIDStep(const Affine3d& x_target, const VectorXd& xdot_target, const std::string& link_name) {
    return eigen_detail::evec(impl_.QPIDStep(eigen_detail::pose(x_target), eigen_detail::vec(xdot_target), link_name));
  }
  virtual VectorXd QPIDCubic(const Affine3d& x_target, const VectorXd& xdot_target, const Affine3d& x_init,
                             const VectorXd& xdot_init, const double& current_time, const double& init_time,
                             const double& duration, const std::string& link_name) {
    return eigen_detail::evec(impl_.QPIDCubic(eigen_detail::pose(x_target), eigen_detail::vec(xdot_target),
                                              eigen_detail::pose(x_init), eigen_detail::vec(xdot_init), current_time,
                                              init_time, duration, link_name));
  }
  drc_amd::Manipulator::RobotController& impl() { return impl_; }

 protected:
  std::shared_ptr<RobotData> robot_data_;
  drc_amd::Manipulator::RobotController impl_;
};

// QPIK / QPID objects (manipulator/QP_IK.h:16-100, QP_ID.h)
class QPIK {
 public:
  explicit QPIK(std::shared_ptr<RobotData> robot_data) : robot_data_(std::move(robot_data)), impl_(robot_data_->impl()) {}
  void setDesiredTaskVel(const VectorXd& xdot_desired, const std::string& link_name) {
    impl_.setDesiredTaskVel(eigen_detail::vec(xdot_desired), link_name);
  }
  bool getOptJointVel(VectorXd& opt_qdot, QP::TimeDuration& time_status) {
    drc_amd::Vec v;
    const bool ok = impl_.getOptJointVel(v, time_status);
    opt_qdot = eigen_detail::evec(v);
    return ok;
  }
  drc_amd::Manipulator::QPIK& impl() { return impl_; }

 private:
  std::shared_ptr<RobotData> robot_data_;
  drc_amd::Manipulator::QPIK impl_;
};
class QPID {
 public:
  explicit QPID(std::shared_ptr<RobotData> robot_data) : robot_data_(std::move(robot_data)), impl_(robot_data_->impl()) {}
  void setDesiredTaskAcc(const VectorXd& xddot_desired, const std::string& link_name) {
    impl_.setDesiredTaskAcc(eigen_detail::vec(xddot_desired), link_name);
  }
  bool getOptJoint(VectorXd& opt_qddot, VectorXd& opt_torque, QP::TimeDuration& time_status) {
    drc_amd::Vec a, t;
    const bool ok = impl_.getOptJoint(a, t, time_status);
    opt_qddot = eigen_detail::evec(a);
    opt_torque = eigen_detail::evec(t);
    return ok;
  }

 private:
  std::shared_ptr<RobotData> robot_data_;
  drc_amd::Manipulator::QPID impl_;
};

}  // namespace Manipulator

namespace Mobile {
using KinematicParam = drc_amd::Mobile::KinematicParam;
}

namespace MobileManipulator {

using JointIndex = drc_amd::MobileManipulator::JointIndex;
using ActuatorIndex = drc_amd::MobileManipulator::ActuatorIndex;

class RobotData : public Manipulator::RobotData {
 public:
  RobotData(const Mobile::KinematicParam& mobile_param, const JointIndex& joint_idx,
            const ActuatorIndex& actuator_idx, const std::string& urdf_path, const std::string& srdf_path = "",
            const std::string& packages_path = "")
      : mm_(std::make_shared<drc_amd::MobileManipulator::RobotData>(mobile_param, joint_idx, actuator_idx, urdf_path,
                                                                   srdf_path, packages_path)) {
    impl_ = mm_;
  }
  using Manipulator::RobotData::updateState;
  bool updateState(const VectorXd& q_virtual, const VectorXd& q_mobile, const VectorXd& q_mani,
                   const VectorXd& qdot_virtual, const VectorXd& qdot_mobile, const VectorXd& qdot_mani) {
    return mm_->updateState(eigen_detail::vec(q_virtual), eigen_detail::vec(q_mobile), eigen_detail::vec(q_mani),
                            eigen_detail::vec(qdot_virtual), eigen_detail::vec(qdot_mobile),
                            eigen_detail::vec(qdot_mani));
  }
  int getActuatordDof() const { return mm_->getActuatordDof(); }  // (sic) robot_data.h:359
  int getManipulatorDof() const { return mm_->getManipulatorDof(); }
  int getMobileDof() const { return mm_->getMobileDof(); }
  const std::shared_ptr<drc_amd::MobileManipulator::RobotData>& mm() const { return mm_; }

 private:
  std::shared_ptr<drc_amd::MobileManipulator::RobotData> mm_;
};

class RobotController {
 public:
  RobotController(const double& dt, std::shared_ptr<RobotData> robot_data)
      : robot_data_(std::move(robot_data)), impl_(dt, robot_data_->mm()) {}
  virtual ~RobotController() = default;
  virtual void setTaskGain(const VectorXd& Kp, const VectorXd& Kv) {
    impl_.setTaskGain(eigen_detail::vec(Kp), eigen_detail::vec(Kv));
  }
  virtual void QPIK(const VectorXd& xdot_target, const std::string& link_name, VectorXd& opt_qdot_mobile,
                    VectorXd& opt_qdot_manipulator) {
    drc_amd::Vec m, a;
    impl_.QPIK(eigen_detail::vec(xdot_target), link_name, m, a);
    opt_qdot_mobile = eigen_detail::evec(m);
    opt_qdot_manipulator = eigen_detail::evec(a);
  }
  virtual void QPIKStep(const Affine3d& x_target, const VectorXd& xdot_target, const std::string& link_name,
                        VectorXd& opt_qdot_mobile, VectorXd& opt_qdot_manipulator) {
    drc_amd::Vec m, a;
    impl_.QPIKStep(eigen_detail::pose(x_target), eigen_detail::vec(xdot_target), link_name, m, a);
    opt_qdot_mobile = eigen_detail::evec(m);
    opt_qdot_manipulator = eigen_detail::evec(a);
  }
  virtual void QPIKCubic(const Affine3d& x_target, const VectorXd& xdot_target, const Affine3d& x_init,
                         const VectorXd& xdot_init, const double& current_time, const double& init_time,
                         const double& duration, const std::string& link_name, VectorXd& opt_qdot_mobile,
                         VectorXd& opt_qdot_manipulator) {
    drc_amd::Vec m, a;
    impl_.QPIKCubic(eigen_detail::pose(x_target), eigen_detail::vec(xdot_target), eigen_detail::pose(x_init),
                    eigen_detail::vec(xdot_init), current_time, init_time, duration, link_name, m, a);
    opt_qdot_mobile = eigen_detail::evec(m);
    opt_qdot_manipulator = eigen_detail::evec(a);
  }
  drc_amd::MobileManipulator::RobotController& impl() { return impl_; }

 protected:
  std::shared_ptr<RobotData> robot_data_;
  drc_amd::MobileManipulator::RobotController impl_;
};

// QPIK / QPID objects (mobile_manipulator/QP_IK.h:16-93, QP_ID.h): eta in ActuatorIndex order
class QPIK {
 public:
  explicit QPIK(std::shared_ptr<RobotData> robot_data) : robot_data_(std::move(robot_data)), impl_(robot_data_->mm()) {}
  void setDesiredTaskVel(const VectorXd& xdot_desired, const std::string& link_name) {
    impl_.setDesiredTaskVel(eigen_detail::vec(xdot_desired), link_name);
  }
  bool getOptJointVel(VectorXd& opt_qdot, QP::TimeDuration& time_status) {
    drc_amd::Vec v;
    const bool ok = impl_.getOptJointVel(v, time_status);
    opt_qdot = eigen_detail::evec(v);
    return ok;
  }

 private:
  std::shared_ptr<RobotData> robot_data_;
  drc_amd::MobileManipulator::QPIK impl_;
};
class QPID {
 public:
  explicit QPID(std::shared_ptr<RobotData> robot_data) : robot_data_(std::move(robot_data)), impl_(robot_data_->mm()) {}
  void setDesiredTaskAcc(const VectorXd& xddot_desired, const std::string& link_name) {
    impl_.setDesiredTaskAcc(eigen_detail::vec(xddot_desired), link_name);
  }
  bool getOptJoint(VectorXd& opt_etadot, VectorXd& opt_torque, QP::TimeDuration& time_status) {
    drc_amd::Vec a, t;
    const bool ok = impl_.getOptJoint(a, t, time_status);
    opt_etadot = eigen_detail::evec(a);
    opt_torque = eigen_detail::evec(t);
    return ok;
  }

 private:
  std::shared_ptr<RobotData> robot_data_;
  drc_amd::MobileManipulator::QPID impl_;
};

}  // namespace MobileManipulator
}  // namespace drc

#endif  // DRC_AMD_EIGEN_HPP

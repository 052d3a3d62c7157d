"""``drc.mobile_manipulator`` mirror: RobotData + RobotController (QPIK).

Mirrors the reference's Python interface for the whole-body QP-IK path
(drc/mobile_manipulator/robot_data.py:16-44, robot_controller.py:188-249;
src/mobile_manipulator/robot_data.cpp:7-144,407-496; QP_IK.cpp:7-128;
robot_controller.cpp:147-197) and the types of drc/type_define.py:6-91.

=====================================================  ==========================================
reference                                              here
=====================================================  ==========================================
``KinematicParam / JointIndex / ActuatorIndex``        same classes (``DriveType`` enum)
``RobotData(param, joint_idx, actuator_idx, urdf,      same (+ ``device``)
srdf, packages)``
``update_state(q_virtual, q_mobile, q_mani, qdot_*)``  same
``get_dof / get_actuator_dof / get_manipulator_dof /   same
get_mobile_dof / get_joint_index / ...``
``get_mobile_FK_jacobian``                             same (model build, HIP library)
``RobotController(dt, robot_data)``                    same
``QPIK / QPIK_step / QPIK_cubic -> (qdot_mobile,       same
qdot_mani)``
(none)                                                 ``QPIK_batch`` / ``QPIK_step_batch`` /
                                                       ``QPIK_cubic_batch`` over [field][B]
                                                       device tensors -> (eta [A][B], status)
=====================================================  ==========================================

Every result comes from ``libdrc_amd.so``; the single-instance calls are
B = 1 launches of the batched kernel.
"""
import sys
from enum import IntEnum

import numpy as np

from . import _batch, _capi
from ._capi import C
from .manipulator import QPIKParamsBuilder, _ModelHandle, _default_device, pose_to12


class DriveType(IntEnum):
    """drc/type_define.py:6-9."""
    Differential = _capi.DRIVE_DIFFERENTIAL
    Mecanum = _capi.DRIVE_MECANUM
    Caster = _capi.DRIVE_CASTER


class KinematicParam:
    """drc/type_define.py:11-54 (include/dyros_robot_controller/type_define.h:58-120)."""

    def __init__(self, type, wheel_radius, max_lin_speed=2.0, max_ang_speed=2.0, max_lin_acc=2.0,
                 max_ang_acc=2.0, base_width=None, roller_angles=None, base2wheel_positions=None,
                 base2wheel_angles=None, wheel_offset=None):
        self.type = DriveType(type)
        self.wheel_radius = float(wheel_radius)
        self.max_lin_speed, self.max_ang_speed = float(max_lin_speed), float(max_ang_speed)
        self.max_lin_acc, self.max_ang_acc = float(max_lin_acc), float(max_ang_acc)
        self.base_width = base_width
        self.roller_angles = roller_angles
        self.base2wheel_positions = base2wheel_positions
        self.base2wheel_angles = base2wheel_angles
        self.wheel_offset = wheel_offset
        if self.type == DriveType.Differential and base_width is None:
            raise ValueError("Differential drive requires base_width")
        if self.type == DriveType.Mecanum and (roller_angles is None or base2wheel_positions is None
                                               or base2wheel_angles is None):
            raise ValueError("Mecanum drive requires roller_angles, base2wheel_positions, base2wheel_angles")
        if self.type == DriveType.Caster and (base2wheel_positions is None or not wheel_offset):
            raise ValueError("Caster drive requires base2wheel_positions and a nonzero wheel_offset")

    def c_struct(self):
        p = _capi.KinematicParam()
        p.type = int(self.type)
        p.wheel_radius = self.wheel_radius
        p.max_lin_speed, p.max_ang_speed = self.max_lin_speed, self.max_ang_speed
        p.max_lin_acc, p.max_ang_acc = self.max_lin_acc, self.max_ang_acc
        p.base_width = float(self.base_width) if self.base_width is not None else 0.0
        n = 2
        if self.type == DriveType.Mecanum:
            n = len(self.roller_angles)
            if n > _capi.MAX_WHEELS:
                raise ValueError("at most %d wheels" % _capi.MAX_WHEELS)
            for i in range(n):
                p.roller_angles[i] = float(self.roller_angles[i])
                p.base2wheel_positions[i][0] = float(self.base2wheel_positions[i][0])
                p.base2wheel_positions[i][1] = float(self.base2wheel_positions[i][1])
                p.base2wheel_angles[i] = float(self.base2wheel_angles[i])
        if self.type == DriveType.Caster:   # n_wheels counts casters (2 joints each, robot_data.cpp:27-30)
            n = len(self.base2wheel_positions)
            if 2 * n > _capi.MAX_WHEELS:
                raise ValueError("at most %d casters" % (_capi.MAX_WHEELS // 2))
            for i in range(n):
                p.base2wheel_positions[i][0] = float(self.base2wheel_positions[i][0])
                p.base2wheel_positions[i][1] = float(self.base2wheel_positions[i][1])
        p.n_wheels = n
        p.wheel_offset = float(self.wheel_offset) if self.wheel_offset is not None else 0.0
        return p


class JointIndex:
    """drc/type_define.py:56-74."""

    def __init__(self, virtual_start, mani_start, mobi_start):
        self.virtual_start, self.mani_start, self.mobi_start = int(virtual_start), int(mani_start), int(mobi_start)

    def c_struct(self):
        j = _capi.JointIndex()
        j.virtual_start, j.mani_start, j.mobi_start = self.virtual_start, self.mani_start, self.mobi_start
        return j


class ActuatorIndex:
    """drc/type_define.py:76-91."""

    def __init__(self, mani_start, mobi_start):
        self.mani_start, self.mobi_start = int(mani_start), int(mobi_start)

    def c_struct(self):
        a = _capi.ActuatorIndex()
        a.mani_start, a.mobi_start = self.mani_start, self.mobi_start
        return a


class RobotData:
    """MobileManipulator::RobotData (mobile_manipulator/robot_data.h:55)."""

    def __init__(self, mobile_param, joint_idx, actuator_idx, urdf_path, srdf_path="", packages_path="",
                 device=None):
        import torch
        self.device = torch.device(device) if device is not None else _default_device()
        self._param, self._jidx, self._aidx = mobile_param, joint_idx, actuator_idx
        kp, ji, ai = mobile_param.c_struct(), joint_idx.c_struct(), actuator_idx.c_struct()
        h = C.c_void_p()
        _capi.check(_capi.lib().drc_model_create_mobile_manipulator(
            C.byref(kp), C.byref(ji), C.byref(ai), urdf_path.encode(), (srdf_path or "").encode(),
            (packages_path or "").encode(), C.c_int(self.device.index or 0), C.byref(h)))
        self.model = _ModelHandle(h, self.device)
        n = self.model.dof
        self._lims = [np.zeros(n) for _ in range(4)]
        _capi.check(_capi.lib().drc_model_limits(h, *(a.ctypes.data_as(C.POINTER(C.c_double)) for a in self._lims)))
        self._kp_c = kp
        self.q_ = np.zeros(n)
        self.qdot_ = np.zeros(n)
        self._dyn_cache = {}

    # -- sizes and indices -----------------------------------------------------
    def get_dof(self):
        return self.model.dof

    def get_actuator_dof(self):
        return self.model.actuated_dof

    def get_manipulator_dof(self):
        return self.model.mani_dof

    def get_mobile_dof(self):
        return self.model.mobi_dof

    def get_joint_index(self):
        return self._jidx

    def get_actuator_index(self):
        return self._aidx

    def compute_mobile_FK_jacobian(self, q_mobile):
        """Mobile::RobotData::computeFKJacobian(q_mobile) (mobile/robot_data.cpp:123-204):
        constant for differential / mecanum bases, steer-angle dependent for casters."""
        W = self.model.mobi_dof
        J = np.zeros(3 * W)
        qm = np.ascontiguousarray(np.asarray(q_mobile, float).reshape(-1))
        if qm.size != W:
            raise ValueError("q_mobile must have %d entries" % W)
        nw = C.c_int()
        dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))
        _capi.check(_capi.lib().drc_mobile_fk_jacobian(C.byref(self._kp_c), dp(qm), dp(J), C.byref(nw)))
        return J.reshape(3, W)

    def get_mobile_FK_jacobian(self):
        ji = self.get_joint_index()
        return self.compute_mobile_FK_jacobian(self.q_[ji.mobi_start:ji.mobi_start + self.model.mobi_dof])

    def get_joint_position_limit(self):
        return self._lims[0].copy(), self._lims[1].copy()

    def get_joint_velocity_limit(self):
        return self._lims[2].copy(), self._lims[3].copy()

    # -- state -----------------------------------------------------------------
    def joint_vector(self, q_virtual, q_mobile, q_mani):
        """getJointVector (robot_data.cpp:418-427): place the blocks by JointIndex."""
        q = np.zeros(self.get_dof())
        ji = self._jidx
        q[ji.virtual_start:ji.virtual_start + 3] = np.asarray(q_virtual, float).reshape(-1)
        q[ji.mobi_start:ji.mobi_start + self.get_mobile_dof()] = np.asarray(q_mobile, float).reshape(-1)
        q[ji.mani_start:ji.mani_start + self.get_manipulator_dof()] = np.asarray(q_mani, float).reshape(-1)
        return q

    def update_state(self, q_virtual, q_mobile, q_mani, qdot_virtual, qdot_mobile, qdot_mani):
        self.q_ = self.joint_vector(q_virtual, q_mobile, q_mani)
        self.qdot_ = self.joint_vector(qdot_virtual, qdot_mobile, qdot_mani)
        self._dyn_cache = {}
        return True

    updateState = update_state

    def get_joint_position(self):
        return self.q_.copy()

    def get_joint_velocity(self):
        return self.qdot_.copy()

    # -- task-space values through the kernel's stage outputs ----------------
    def _stages(self, link_name):
        pb = QPIKParamsBuilder(self.model, exact=True)
        p = pb.params(link_name, mode=_capi.MODE_QPIK) if link_name else pb.params_no_frame(_capi.MODE_QPIK)
        dev = self.device
        st = _batch.stages_batch(self.model, p, _batch.as_device(self.q_.reshape(-1, 1), dev),
                                 _batch.as_device(self.qdot_.reshape(-1, 1), dev), None,
                                 _batch.as_device(np.zeros((6, 1)), dev))
        return {k: v.cpu().numpy() for k, v in st.items()}

    def get_pose(self, link_name):
        from .manipulator import pose_from12
        return pose_from12(self._stages(link_name)["pose"][:, 0])

    def get_jacobian(self, link_name):
        return self._stages(link_name)["jac"][:, 0].reshape(6, self.get_dof())

    def _qpid_stages(self, link_name):
        pb = QPIKParamsBuilder(self.model, exact=True, qpid=True)
        p = pb.params(link_name, mode=_capi.MODE_QPID) if link_name else pb.params_no_frame(_capi.MODE_QPID)
        dev = self.device
        st = _batch.qpid_stages_batch(self.model, p, _batch.as_device(self.q_.reshape(-1, 1), dev),
                                      _batch.as_device(self.qdot_.reshape(-1, 1), dev), None,
                                      _batch.as_device(np.zeros((6, 1)), dev))
        return {k: v.cpu().numpy()[..., 0] for k, v in st.items()}

    def get_manipulability(self, with_grad, with_graddot, link_name):
        """Arm-block manipulability (robot_data.cpp:439-496)."""
        from .manipulator import ManipulabilityResult
        n = self.get_manipulator_dof()
        if with_graddot:
            st = self._qpid_stages(link_name)
            r = ManipulabilityResult(st["man"][0], st["man"][1:])
            r.grad_dot = st["man_graddot"].copy()
            return r
        m = self._stages(link_name)["man"][:, 0]
        return ManipulabilityResult(m[0], m[1:] if with_grad else np.zeros(n))

    def get_min_distance(self, with_grad, with_graddot, verbose=False):
        from .manipulator import MinDistResult
        if with_graddot:
            st = self._qpid_stages(None)
            r = MinDistResult(st["dist"][0], st["dist"][1:])
            r.grad_dot = st["dist_graddot"].copy()
            return r
        d = self._stages(None)["dist"][:, 0]
        return MinDistResult(d[0], d[1:] if with_grad else np.zeros(self.get_dof()))

    def get_selection_matrix(self):
        """S (dof x A): identity on the arm and wheel blocks, Rz(yaw) J_mobile
        on the virtual block (robot_data.cpp:22-25,115-120)."""
        ji, ai = self.get_joint_index(), self.get_actuator_index()
        n, W = self.get_manipulator_dof(), self.get_mobile_dof()
        S = np.zeros((self.get_dof(), n + W))
        S[ji.mani_start:ji.mani_start + n, ai.mani_start:ai.mani_start + n] = np.eye(n)
        S[ji.mobi_start:ji.mobi_start + W, ai.mobi_start:ai.mobi_start + W] = np.eye(W)
        c, s_ = np.cos(self.q_[ji.virtual_start + 2]), np.sin(self.q_[ji.virtual_start + 2])
        S[ji.virtual_start:ji.virtual_start + 3, ai.mobi_start:ai.mobi_start + W] = (
            np.array([[c, -s_, 0], [s_, c, 0], [0, 0, 1]]) @ self.get_mobile_FK_jacobian())
        return S

    def get_jacobian_time_variation(self, link_name):
        """LOCAL_WORLD_ALIGNED dJ/dt at the full (q, qdot) (robot_data.cpp:404-417)."""
        return self._qpid_stages(link_name)["jdot"].reshape(6, self.get_dof())

    def get_jacobian_actuated(self, link_name):
        """J S (robot_data.cpp:407-410)."""
        return self.get_jacobian(link_name) @ self.get_selection_matrix()

    def get_jacobian_actuated_time_variation(self, link_name):
        """Jdot S, Sdot neglected (robot_data.cpp:412-415)."""
        return self.get_jacobian_time_variation(link_name) @ self.get_selection_matrix()

    # -- dynamics (robot_data.cpp:126-144; getters robot_data.h:425-445) --------
    def _dynamics(self, q, qdot, actuated):
        dq = _batch.as_device(np.asarray(q, float).reshape(-1, 1), self.device)
        dqd = _batch.as_device(np.asarray(qdot, float).reshape(-1, 1), self.device)
        d = _batch.dynamics_batch(self.model, dq, dqd, actuated=actuated)
        return {k: v.cpu().numpy()[..., 0] for k, v in d.items()}

    def _cached(self, actuated):
        if actuated not in self._dyn_cache:
            self._dyn_cache[actuated] = self._dynamics(self.q_, self.qdot_, actuated)
        return self._dyn_cache[actuated]

    def get_mass_matrix(self):
        return self._cached(False)["M"].copy()

    def get_mass_matrix_inv(self):
        return self._cached(False)["Minv"].copy()

    def get_gravity(self):
        return self._cached(False)["g"].copy()

    def get_coriolis(self):
        return self._cached(False)["c"].copy()

    def get_nonlinear_effects(self):
        return self._cached(False)["nle"].copy()

    def get_mass_matrix_actuated(self):
        return self._cached(True)["M"].copy()

    def get_mass_matrix_actuated_inv(self):
        return self._cached(True)["Minv"].copy()

    def get_gravity_actuated(self):
        return self._cached(True)["g"].copy()

    def get_coriolis_actuated(self):
        return self._cached(True)["c"].copy()

    def get_nonlinear_effects_actuated(self):
        return self._cached(True)["nle"].copy()

    def _blocks(self, q_virtual, q_mobile, q_mani, qdot_virtual=None, qdot_mobile=None, qdot_mani=None):
        q = self.joint_vector(q_virtual, q_mobile, q_mani)
        qd = (np.zeros_like(q) if qdot_virtual is None
              else self.joint_vector(qdot_virtual, qdot_mobile, qdot_mani))
        return q, qd

    def compute_mass_matrix(self, q_virtual, q_mobile, q_mani):
        return self._dynamics(*self._blocks(q_virtual, q_mobile, q_mani), False)["M"]

    def compute_gravity(self, q_virtual, q_mobile, q_mani):
        return self._dynamics(*self._blocks(q_virtual, q_mobile, q_mani), False)["g"]

    def compute_coriolis(self, q_virtual, q_mobile, q_mani, qdot_virtual, qdot_mobile, qdot_mani):
        return self._dynamics(*self._blocks(q_virtual, q_mobile, q_mani, qdot_virtual, qdot_mobile, qdot_mani),
                              False)["c"]

    def compute_nonlinear_effects(self, q_virtual, q_mobile, q_mani, qdot_virtual, qdot_mobile, qdot_mani):
        return self._dynamics(*self._blocks(q_virtual, q_mobile, q_mani, qdot_virtual, qdot_mobile, qdot_mani),
                              False)["nle"]

    def compute_mass_matrix_actuated(self, q_virtual, q_mobile, q_mani):
        return self._dynamics(*self._blocks(q_virtual, q_mobile, q_mani), True)["M"]

    def compute_gravity_actuated(self, q_virtual, q_mobile, q_mani):
        return self._dynamics(*self._blocks(q_virtual, q_mobile, q_mani), True)["g"]

    def compute_coriolis_actuated(self, q_virtual, q_mobile, q_mani, qdot_virtual, qdot_mobile, qdot_mani):
        return self._dynamics(*self._blocks(q_virtual, q_mobile, q_mani, qdot_virtual, qdot_mobile, qdot_mani),
                              True)["c"]

    def compute_nonlinear_effects_actuated(self, q_virtual, q_mobile, q_mani, qdot_virtual, qdot_mobile,
                                           qdot_mani):
        return self._dynamics(*self._blocks(q_virtual, q_mobile, q_mani, qdot_virtual, qdot_mobile, qdot_mani),
                              True)["nle"]

    def dynamics_batch(self, q, qdot=None, actuated=False, fields=_batch.DYN_FIELDS):
        """Batched updateDynamics on device tensors [dof][B] (full joint vectors)."""
        return _batch.dynamics_batch(self.model, _batch.as_device(q, self.device),
                                     _batch.as_device(qdot, self.device), actuated=actuated, fields=fields)


class RobotController:
    """MobileManipulator::RobotController QPIK entries
    (src/mobile_manipulator/robot_controller.cpp:7-22,147-197): xdot_des =
    Kp (x) e + xdot_target with Kp = 400 (no Kv term), eta split by
    ActuatorIndex into (qdot_mobile, qdot_mani); zeros on failure."""

    def __init__(self, dt, robot_data, solver_mode="exact"):
        if not isinstance(robot_data, RobotData):
            raise TypeError("robot_data must be a mobile_manipulator.RobotData")
        self.dt_ = float(dt)
        self.robot_data_ = robot_data
        self.Kp_task_ = np.full(6, 400.0)         # robot_controller.cpp:15-16
        self.Kv_task_ = np.full(6, 40.0)          # used by QPID only (QPIKStep has no Kv term, :177)
        n = robot_data.get_manipulator_dof()
        self.Kp_mani_joint_ = np.full(n, 400.0)   # mobile_manipulator/robot_controller.cpp:17-18
        self.Kv_mani_joint_ = np.full(n, 40.0)
        self.set_solver_mode(solver_mode)

    def set_solver_mode(self, mode):
        if mode not in ("exact", "osqp_default"):
            raise ValueError("solver_mode must be 'exact' or 'osqp_default'")
        self.solver_mode = mode
        self._pb = QPIKParamsBuilder(self.robot_data_.model, exact=(mode == "exact"))
        self._pbd = QPIKParamsBuilder(self.robot_data_.model, exact=(mode == "exact"), qpid=True)

    def set_task_gain(self, kp, kv):
        kp, kv = np.asarray(kp, float).reshape(-1), np.asarray(kv, float).reshape(-1)
        if kp.size != 6 or kv.size != 6:
            raise RuntimeError("Kp and Kv must be of size 6.")
        self.Kp_task_, self.Kv_task_ = kp, kv

    def set_task_kp_gain(self, kp):
        kp = np.asarray(kp, float).reshape(-1)
        if kp.size != 6:
            raise RuntimeError("Kp must be of size 6.")
        self.Kp_task_ = kp

    def set_task_kv_gain(self, kv):
        kv = np.asarray(kv, float).reshape(-1)
        if kv.size != 6:
            raise RuntimeError("Kv must be of size 6.")
        self.Kv_task_ = kv

    setTaskGain, setTaskKpGain, setTaskKvGain = set_task_gain, set_task_kp_gain, set_task_kv_gain

    def _mani_vec(self, v, what):
        v = np.asarray(v, float).reshape(-1)
        if v.size != self.robot_data_.get_manipulator_dof():
            raise RuntimeError("%s must be of size mani_dof_." % what)
        return v

    def set_manipulator_joint_gain(self, kp, kv):
        self.Kp_mani_joint_, self.Kv_mani_joint_ = self._mani_vec(kp, "Kp"), self._mani_vec(kv, "Kv")

    def set_manipulator_joint_kp_gain(self, kp):
        self.Kp_mani_joint_ = self._mani_vec(kp, "Kp")

    def set_manipulator_joint_kv_gain(self, kv):
        self.Kv_mani_joint_ = self._mani_vec(kv, "Kv")

    setManipulatorJointGain = set_manipulator_joint_gain
    setManipulatorJointKpGain, setManipulatorJointKvGain = set_manipulator_joint_kp_gain, set_manipulator_joint_kv_gain

    # -- arm joint torque step (mobile_manipulator/robot_controller.cpp:103-118) --
    def move_manipulator_joint_torque_step_batch(self, q, qdot, q_mani_target=None, qdot_mani_target=None,
                                                 qddot_mani_target=None, dt=None):
        """tau_mani [n_arm][B] from full states q, qdot [dof][B]."""
        dev = self.robot_data_.device
        a = lambda t: _batch.as_device(t, dev)
        return _batch.joint_torque_step_batch(self.robot_data_.model, a(q), a(qdot), a(q_mani_target),
                                              a(qdot_mani_target), a(qddot_mani_target),
                                              self.dt_ if dt is None else dt, self.Kp_mani_joint_, self.Kv_mani_joint_)

    def moveManipulatorJointTorqueStep(self, *args):
        rd = self.robot_data_
        q, qd = rd.q_.reshape(-1, 1), rd.qdot_.reshape(-1, 1)
        col = lambda v: np.asarray(v, float).reshape(-1, 1)
        if len(args) == 1:
            tau = self.move_manipulator_joint_torque_step_batch(q, qd, qddot_mani_target=col(args[0]))
        else:
            tau = self.move_manipulator_joint_torque_step_batch(q, qd, col(args[0]), col(args[1]))
        return tau.cpu().numpy()[:, 0]

    def move_manipulator_joint_torque_step(self, q_mani_target=None, qdot_mani_target=None, qddot_mani_target=None):
        if qddot_mani_target is not None:
            return self.moveManipulatorJointTorqueStep(qddot_mani_target)
        if q_mani_target is not None and qdot_mani_target is not None:
            return self.moveManipulatorJointTorqueStep(q_mani_target, qdot_mani_target)
        return None

    # -- batched entries (device tensors, [field][B]; q is the full joint vector)
    def _run(self, mode, link_name, q, qdot, x_target, xdot_target, x_init=None, xdot_init=None,
             t=0.0, t0=0.0, duration=1.0, iters=None):
        p = self._pb.params(link_name, mode, self.Kp_task_, np.zeros(6), t, t0, duration)   # no Kv in QPIKStep
        dev = self.robot_data_.device
        return _batch.qpik_batch(self.robot_data_.model, p, _batch.as_device(q, dev), _batch.as_device(qdot, dev),
                                 _batch.as_device(x_target, dev), _batch.as_device(xdot_target, dev),
                                 _batch.as_device(x_init, dev), _batch.as_device(xdot_init, dev), iters=iters)

    def QPIK_batch(self, q, qdot, xdot_target, link_name):
        return self._run(_capi.MODE_QPIK, link_name, q, qdot, None, xdot_target)

    def QPIK_step_batch(self, q, qdot, x_target, xdot_target, link_name, iters=None):
        return self._run(_capi.MODE_QPIK_STEP, link_name, q, qdot, x_target, xdot_target, iters=iters)

    def QPIK_cubic_batch(self, q, qdot, x_target, xdot_target, x_init, xdot_init, current_time, init_time,
                         duration, link_name):
        return self._run(_capi.MODE_QPIK_CUBIC, link_name, q, qdot, x_target, xdot_target, x_init, xdot_init,
                         current_time, init_time, duration)

    def split_actuated(self, eta):
        """eta [A] -> (qdot_mobile [W], qdot_mani [n]) by ActuatorIndex."""
        a = self.robot_data_.get_actuator_index()
        W, n = self.robot_data_.get_mobile_dof(), self.robot_data_.get_manipulator_dof()
        return eta[a.mobi_start:a.mobi_start + W].copy(), eta[a.mani_start:a.mani_start + n].copy()

    # -- single-instance entries (reference signatures; B = 1 launches) -------
    def _one(self, out_status):
        out, status = out_status
        eta, st = out.cpu().numpy()[:, 0], int(status.cpu().numpy()[0])
        if st != _capi.STATUS_SOLVED:
            print("QP IK failed to compute optimal joint velocity.", file=sys.stderr)
            eta = np.zeros(self.robot_data_.get_actuator_dof())
        return self.split_actuated(eta)

    def _state(self):
        rd = self.robot_data_
        return rd.q_.reshape(-1, 1), rd.qdot_.reshape(-1, 1)

    def QPIK(self, xdot_target, link_name):
        q, qd = self._state()
        return self._one(self.QPIK_batch(q, qd, np.asarray(xdot_target, float).reshape(6, 1), link_name))

    def QPIK_step(self, x_target, xdot_target, link_name):
        q, qd = self._state()
        return self._one(self.QPIK_step_batch(q, qd, pose_to12(x_target).reshape(12, 1),
                                              np.asarray(xdot_target, float).reshape(6, 1), link_name))

    def QPIK_cubic(self, x_target, xdot_target, x_init, xdot_init, current_time, init_time, duration, link_name):
        q, qd = self._state()
        return self._one(self.QPIK_cubic_batch(
            q, qd, pose_to12(x_target).reshape(12, 1), np.asarray(xdot_target, float).reshape(6, 1),
            pose_to12(x_init).reshape(12, 1), np.asarray(xdot_init, float).reshape(6, 1),
            current_time, init_time, duration, link_name))

    QPIKStep, QPIKCubic = QPIK_step, QPIK_cubic

    # -- QPID / QPIDStep / QPIDCubic (robot_controller.cpp:199-250)
    def _run_id(self, mode, link_name, q, qdot, x_target, xdot_target, x_init=None, xdot_init=None,
                t=0.0, t0=0.0, duration=1.0, iters=None):
        p = self._pbd.params(link_name, mode, self.Kp_task_, self.Kv_task_, t, t0, duration)
        a = lambda v: _batch.as_device(v, self.robot_data_.device)
        return _batch.qpid_batch(self.robot_data_.model, p, a(q), a(qdot), a(x_target), a(xdot_target), a(x_init),
                                 a(xdot_init), iters=iters)

    def QPID_batch(self, q, qdot, xddot_target, link_name):
        """(eta_dot [A][B], tau [A][B], status [B]) in ActuatorIndex order."""
        return self._run_id(_capi.MODE_QPID, link_name, q, qdot, None, xddot_target)

    def QPID_step_batch(self, q, qdot, x_target, xdot_target, link_name, iters=None):
        return self._run_id(_capi.MODE_QPID_STEP, link_name, q, qdot, x_target, xdot_target, iters=iters)

    def QPID_cubic_batch(self, q, qdot, x_target, xdot_target, x_init, xdot_init, current_time, init_time,
                         duration, link_name):
        return self._run_id(_capi.MODE_QPID_CUBIC, link_name, q, qdot, x_target, xdot_target, x_init, xdot_init,
                            current_time, init_time, duration)

    def _one_id(self, res):
        """-> (qddot_mobile [W], torque_manipulator [n]) (robot_controller.cpp:215-218)."""
        qdd, tau, status = res
        if int(status.cpu().numpy()[0]) != _capi.STATUS_SOLVED:
            print("QP ID failed to compute optimal joint torque.", file=sys.stderr)
        qdd, tau = qdd.cpu().numpy()[:, 0], tau.cpu().numpy()[:, 0]
        a = self.robot_data_.get_actuator_index()
        W, n = self.robot_data_.get_mobile_dof(), self.robot_data_.get_manipulator_dof()
        return qdd[a.mobi_start:a.mobi_start + W].copy(), tau[a.mani_start:a.mani_start + n].copy()

    def QPID(self, xddot_target, link_name):
        q, qd = self._state()
        return self._one_id(self.QPID_batch(q, qd, np.asarray(xddot_target, float).reshape(6, 1), link_name))

    def QPID_step(self, x_target, xdot_target, link_name):
        q, qd = self._state()
        return self._one_id(self.QPID_step_batch(q, qd, pose_to12(x_target).reshape(12, 1),
                                                 np.asarray(xdot_target, float).reshape(6, 1), link_name))

    def QPID_cubic(self, x_target, xdot_target, x_init, xdot_init, current_time, init_time, duration, link_name):
        q, qd = self._state()
        return self._one_id(self.QPID_cubic_batch(
            q, qd, pose_to12(x_target).reshape(12, 1), np.asarray(xdot_target, float).reshape(6, 1),
            pose_to12(x_init).reshape(12, 1), np.asarray(xdot_init, float).reshape(6, 1),
            current_time, init_time, duration, link_name))

    QPIDStep, QPIDCubic = QPID_step, QPID_cubic

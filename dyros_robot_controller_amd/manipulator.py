"""``drc.manipulator`` mirror: RobotData + RobotController (QPIK entries).

Mirrors the reference's Python/C++ interface for the hot path
(src/bindings.cpp:293-321,398-426; drc/manipulator/*.py):

=====================================  =========================================
reference                              here
=====================================  =========================================
``RobotData(urdf, srdf, packages)``    ``RobotData(urdf, srdf, packages, device)``
``updateState(q, qdot)``               ``updateState`` / ``update_state``
``getPose/getJacobian/getVelocity``    same names (computed by the HIP kernel)
``getManipulability(true,false,l)``    ``getManipulability``
``getMinDistance(true,false,false)``   ``getMinDistance``
``RobotController(dt, robot_data)``    same
``QPIK/QPIKStep/QPIKCubic``            same names + snake_case aliases
(none: one robot per call)             ``QPIK_batch`` / ``QPIK_step_batch`` /
                                       ``QPIK_cubic_batch`` over [field][B]
                                       device tensors
=====================================  =========================================

Every result comes from ``libdrc_amd.so``; single-instance calls are B=1
launches of the same kernel (there is no CPU path).
"""
import sys

import numpy as np

from . import _batch, _capi
from ._capi import C


def pose_to12(T):
    """4x4 homogeneous (Eigen::Affine3d::matrix()) -> [R col-major(9), p(3)]."""
    T = np.asarray(T, dtype=np.float64)
    return np.concatenate([T[:3, :3].T.reshape(-1), T[:3, 3]])


def pose_from12(v):
    v = np.asarray(v, dtype=np.float64)
    T = np.eye(4)
    T[:3, :3] = v[:9].reshape(3, 3).T
    T[:3, 3] = v[9:12]
    return T


def _default_device():
    import torch
    return torch.device("cuda", torch.cuda.current_device())


class _ModelHandle:
    """Owns a ``drc_model*`` (device copy of the robot model)."""

    def __init__(self, handle, device):
        self.handle = handle
        self.device = device
        dof, act, mani, mobi, ng, npair = (C.c_int() for _ in range(6))
        _capi.check(_capi.lib().drc_model_info(handle, *(C.byref(v) for v in (dof, act, mani, mobi, ng, npair))))
        self.dof, self.actuated_dof, self.mani_dof, self.mobi_dof = dof.value, act.value, mani.value, mobi.value
        self.n_geoms, self.n_pairs = ng.value, npair.value

    def frame_id(self, link_name):
        fid = C.c_int()
        _capi.check(_capi.lib().drc_model_find_frame(self.handle, link_name.encode(), C.byref(fid)))
        return fid.value

    def close(self):
        if self.handle:
            _capi.lib().drc_model_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class RobotData:
    """Manipulator::RobotData (include/dyros_robot_controller/manipulator/robot_data.h:49)."""

    def __init__(self, urdf_path, srdf_path="", packages_path="", device=None):
        import torch
        self.device = torch.device(device) if device is not None else _default_device()
        h = C.c_void_p()
        _capi.check(_capi.lib().drc_model_create_manipulator(
            urdf_path.encode(), (srdf_path or "").encode(), (packages_path or "").encode(),
            C.c_int(self.device.index or 0), C.byref(h)))
        self.model = _ModelHandle(h, self.device)
        n = self.model.dof
        self._lims = [np.zeros(n) for _ in range(4)]
        _capi.check(_capi.lib().drc_model_limits(h, *(a.ctypes.data_as(C.POINTER(C.c_double)) for a in self._lims)))
        self.q_ = np.zeros(n)
        self.qdot_ = np.zeros(n)
        self._dyn_cache = None

    # -- state ---------------------------------------------------------------
    def updateState(self, q, qdot):
        q, qdot = np.asarray(q, float).reshape(-1), np.asarray(qdot, float).reshape(-1)
        if q.size != self.getDof() or qdot.size != self.getDof():
            raise ValueError("q and qdot must have size dof")
        self.q_, self.qdot_ = q.copy(), qdot.copy()
        self._dyn_cache = None
        return True

    update_state = updateState

    def getDof(self):
        return self.model.dof

    get_dof = getDof

    def getJointPosition(self):
        return self.q_.copy()

    def getJointVelocity(self):
        return self.qdot_.copy()

    def getJointPositionLimit(self):
        return self._lims[0].copy(), self._lims[1].copy()

    def getJointVelocityLimit(self):
        return self._lims[2].copy(), self._lims[3].copy()

    # -- task-space getters through the kernel's stage outputs ---------------
    def _stages(self, q, qdot, link_name):
        pb = QPIKParamsBuilder(self.model, exact=True)
        p = pb.params(link_name, mode=_capi.MODE_QPIK) if link_name else pb.params_no_frame(_capi.MODE_QPIK)
        dq = _batch.as_device(np.asarray(q, float).reshape(-1, 1), self.device)
        dqd = _batch.as_device(np.asarray(qdot, float).reshape(-1, 1), self.device)
        z6 = _batch.as_device(np.zeros((6, 1)), self.device)
        st = _batch.stages_batch(self.model, p, dq, dqd, None, z6)
        return {k: v.cpu().numpy()[..., 0] for k, v in st.items()}

    def computePose(self, q, link_name):
        return pose_from12(self._stages(q, np.zeros_like(q), link_name)["pose"])

    def computeJacobian(self, q, link_name):
        return self._stages(q, np.zeros_like(q), link_name)["jac"].reshape(6, self.getDof())

    def computeVelocity(self, q, qdot, link_name):
        return self.computeJacobian(q, link_name) @ np.asarray(qdot, float)

    def getPose(self, link_name):
        """Pose at the current q (the reference returns the frame
        cached by the last getFrameJacobian; we return FK(q))."""
        return self.computePose(self.q_, link_name)

    def getJacobian(self, link_name):
        return self.computeJacobian(self.q_, link_name)

    def getVelocity(self, link_name):
        return self.getJacobian(link_name) @ self.qdot_

    def _qpid_stages(self, q, qdot, link_name):
        """QPID stage outputs (Jdot, grad_dot vectors) at (q, qdot) for one robot."""
        pb = QPIKParamsBuilder(self.model, exact=True, qpid=True)
        p = pb.params(link_name, mode=_capi.MODE_QPID) if link_name else pb.params_no_frame(_capi.MODE_QPID)
        dq = _batch.as_device(np.asarray(q, float).reshape(-1, 1), self.device)
        dqd = _batch.as_device(np.asarray(qdot, float).reshape(-1, 1), self.device)
        z6 = _batch.as_device(np.zeros((6, 1)), self.device)
        st = _batch.qpid_stages_batch(self.model, p, dq, dqd, None, z6)
        return {k: v.cpu().numpy()[..., 0] for k, v in st.items()}

    def getManipulability(self, with_grad=True, with_graddot=False, link_name=None):
        """robot_data.cpp:519-573 (grad_dot: :555-569, through the QPID stage)."""
        if with_graddot:
            st = self._qpid_stages(self.q_, self.qdot_, link_name)
            r = ManipulabilityResult(st["man"][0], st["man"][1:])
            r.grad_dot = st["man_graddot"].copy()
            return r
        st = self._stages(self.q_, self.qdot_, link_name)
        return ManipulabilityResult(st["man"][0], st["man"][1:] if with_grad else np.zeros(self.getDof()))

    def getMinDistance(self, with_grad=True, with_graddot=False, verbose=False):
        """robot_data.cpp:424-517 (grad_dot: :496-512, through the QPID stage)."""
        if with_graddot:
            st = self._qpid_stages(self.q_, self.qdot_, None)
            r = MinDistResult(st["dist"][0], st["dist"][1:])
            r.grad_dot = st["dist_graddot"].copy()
        else:
            st = self._stages(self.q_, self.qdot_, None)  # no task frame needed
            r = MinDistResult(st["dist"][0], st["dist"][1:] if with_grad else np.zeros(self.getDof()))
        if verbose:
            print("[RobotDataBase] closest pair %d | distance = %g [m]" % (int(st["pair"]), r.distance))
        return r

    def computeJacobianTimeVariation(self, q, qdot, link_name):
        """LOCAL_WORLD_ALIGNED dJ/dt (robot_data.cpp:404-417)."""
        return self._qpid_stages(q, qdot, link_name)["jdot"].reshape(6, self.getDof())

    def getJacobianTimeVariation(self, link_name):
        return self.computeJacobianTimeVariation(self.q_, self.qdot_, link_name)

    get_jacobian_time_variation, compute_jacobian_time_variation = getJacobianTimeVariation, computeJacobianTimeVariation
    get_pose, get_jacobian, get_velocity = getPose, getJacobian, getVelocity
    get_manipulability, get_min_distance = getManipulability, getMinDistance
    compute_pose, compute_jacobian, compute_velocity = computePose, computeJacobian, computeVelocity

    # -- joint-space dynamics (robot_data.cpp:109-124; getters robot_data.h:176-198) ----
    def _dynamics(self, q, qdot, actuated=False):
        dq = _batch.as_device(np.asarray(q, float).reshape(-1, 1), self.device)
        dqd = _batch.as_device(np.asarray(qdot, float).reshape(-1, 1), self.device)
        d = _batch.dynamics_batch(self.model, dq, dqd, actuated=actuated)
        return {k: v.cpu().numpy()[..., 0] for k, v in d.items()}

    def _cached_dynamics(self):
        if self._dyn_cache is None:
            self._dyn_cache = self._dynamics(self.q_, self.qdot_)
        return self._dyn_cache

    def getMassMatrix(self):
        return self._cached_dynamics()["M"].copy()

    def getMassMatrixInv(self):
        return self._cached_dynamics()["Minv"].copy()

    def getGravity(self):
        return self._cached_dynamics()["g"].copy()

    def getCoriolis(self):
        return self._cached_dynamics()["c"].copy()

    def getNonlinearEffects(self):
        return self._cached_dynamics()["nle"].copy()

    def computeMassMatrix(self, q):
        return self._dynamics(q, np.zeros_like(np.asarray(q, float)))["M"]

    def computeGravity(self, q):
        return self._dynamics(q, np.zeros_like(np.asarray(q, float)))["g"]

    def computeCoriolis(self, q, qdot):
        return self._dynamics(q, qdot)["c"]

    def computeNonlinearEffects(self, q, qdot):
        return self._dynamics(q, qdot)["nle"]

    def dynamics_batch(self, q, qdot=None, fields=_batch.DYN_FIELDS):
        """Batched updateDynamics on device tensors [dof][B]; see _batch.dynamics_batch."""
        return _batch.dynamics_batch(self.model, _batch.as_device(q, self.device),
                                     _batch.as_device(qdot, self.device), fields=fields)

    get_mass_matrix, get_mass_matrix_inv, get_gravity = getMassMatrix, getMassMatrixInv, getGravity
    get_coriolis, get_nonlinear_effects = getCoriolis, getNonlinearEffects
    compute_mass_matrix, compute_gravity = computeMassMatrix, computeGravity
    compute_coriolis, compute_nonlinear_effects = computeCoriolis, computeNonlinearEffects


class ManipulabilityResult:
    """type_define.h:116-132"""

    def __init__(self, manipulability, grad):
        self.manipulability = float(manipulability)
        self.grad = np.asarray(grad, float)
        self.grad_dot = np.zeros_like(self.grad)


class MinDistResult:
    """type_define.h:88-104"""

    def __init__(self, distance, grad):
        self.distance = float(distance)
        self.grad = np.asarray(grad, float)
        self.grad_dot = np.zeros_like(self.grad)


class QPIKParamsBuilder:
    """Fills ``drc_qpik_params`` from the reference defaults of the model kind
    (``qpid``: the QPID defaults, drc_default_qpid_params)."""

    def __init__(self, model, exact=True, qpid=False):
        self.model = model
        self.base = _capi.QPIKParams()
        fn = _capi.lib().drc_default_qpid_params if qpid else _capi.lib().drc_default_qpik_params
        _capi.check(fn(model.handle, C.c_int(1 if exact else 0), C.byref(self.base)))

    def params_no_frame(self, mode):
        """Stage-only parameters without a task frame (frame_id = -1)."""
        p = _capi.QPIKParams()
        C.pointer(p)[0] = self.base
        p.frame_id = -1
        p.mode = mode
        return p

    def params(self, link_name, mode, kp=None, kv=None, t=0.0, t0=0.0, duration=1.0):
        p = _capi.QPIKParams()
        C.pointer(p)[0] = self.base
        p.frame_id = self.model.frame_id(link_name)
        p.mode = mode
        if kp is not None:
            for i in range(6):
                p.kp[i] = float(kp[i])
        if kv is not None:
            for i in range(6):
                p.kv[i] = float(kv[i])
        p.t, p.t0, p.duration = float(t), float(t0), float(duration)
        return p


class RobotController:
    """Manipulator::RobotController QPIK entries
    (src/manipulator/robot_controller.cpp:7-19,277-317).

    ``solver_mode``: "exact" (default) returns the certified QP optimum
    (parity contract); "osqp_default" runs the reference's OSQP
    settings (eps 1e-3, no polish) — the same algorithm, reference accuracy.
    """

    def __init__(self, dt, robot_data, solver_mode="exact"):
        self.dt_ = dt
        self.robot_data_ = robot_data
        self.dof_ = robot_data.getDof()
        self.Kp_task_ = np.full(6, 100.0)
        self.Kv_task_ = np.full(6, 20.0)
        self.Kp_joint_ = np.full(self.dof_, 400.0)    # robot_controller.cpp:14-15
        self.Kv_joint_ = np.full(self.dof_, 40.0)
        self.set_solver_mode(solver_mode)

    def set_solver_mode(self, mode):
        if mode not in ("exact", "osqp_default"):
            raise ValueError("solver_mode must be 'exact' or 'osqp_default'")
        self.solver_mode = mode
        self._pb = QPIKParamsBuilder(self.robot_data_.model, exact=(mode == "exact"))
        self._pbd = QPIKParamsBuilder(self.robot_data_.model, exact=(mode == "exact"), qpid=True)

    def setTaskGain(self, Kp, Kv):
        Kp, Kv = np.asarray(Kp, float).reshape(-1), np.asarray(Kv, float).reshape(-1)
        if Kp.size != 6 or Kv.size != 6:
            raise RuntimeError("Kp and Kv must be of size 6.")
        self.Kp_task_, self.Kv_task_ = Kp, Kv

    def setTaskKpGain(self, Kp):
        Kp = np.asarray(Kp, float).reshape(-1)
        if Kp.size != 6:
            raise RuntimeError("Kp must be of size 6.")
        self.Kp_task_ = Kp

    def setTaskKvGain(self, Kv):
        Kv = np.asarray(Kv, float).reshape(-1)
        if Kv.size != 6:
            raise RuntimeError("Kv must be of size 6.")
        self.Kv_task_ = Kv

    set_task_gain, set_task_kp_gain, set_task_kv_gain = setTaskGain, setTaskKpGain, setTaskKvGain

    def setJointGain(self, Kp, Kv):
        Kp, Kv = np.asarray(Kp, float).reshape(-1), np.asarray(Kv, float).reshape(-1)
        if Kp.size != self.dof_ or Kv.size != self.dof_:
            raise RuntimeError("Kp and Kv must be of size dof_.")
        self.Kp_joint_, self.Kv_joint_ = Kp, Kv

    def setJointKpGain(self, Kp):
        Kp = np.asarray(Kp, float).reshape(-1)
        if Kp.size != self.dof_:
            raise RuntimeError("Kp must be of size dof_.")
        self.Kp_joint_ = Kp

    def setJointKvGain(self, Kv):
        Kv = np.asarray(Kv, float).reshape(-1)
        if Kv.size != self.dof_:
            raise RuntimeError("Kv must be of size dof_.")
        self.Kv_joint_ = Kv

    set_joint_gain, set_joint_kp_gain, set_joint_kv_gain = setJointGain, setJointKpGain, setJointKvGain

    # -- joint torque step (robot_controller.cpp:115-125) -----------------------
    def moveJointTorqueStep_batch(self, q, qdot, q_target=None, qdot_target=None, qddot_target=None, dt=None):
        """tau [dof][B]; q_target None -> q + dt * qdot_target (fr3_controller.cpp:133)."""
        dev = self.robot_data_.device
        a = lambda t: _batch.as_device(t, dev)
        return _batch.joint_torque_step_batch(self.robot_data_.model, a(q), a(qdot), a(q_target), a(qdot_target),
                                              a(qddot_target), self.dt_ if dt is None else dt,
                                              self.Kp_joint_, self.Kv_joint_)

    def moveJointTorqueStep(self, *args):
        """moveJointTorqueStep(qddot_target) or moveJointTorqueStep(q_target, qdot_target)."""
        q, qd = self._state()
        col = lambda v: np.asarray(v, float).reshape(-1, 1)
        if len(args) == 1:
            tau = self.moveJointTorqueStep_batch(q, qd, qddot_target=col(args[0]))
        else:
            tau = self.moveJointTorqueStep_batch(q, qd, q_target=col(args[0]), qdot_target=col(args[1]))
        return tau.cpu().numpy()[:, 0]

    def move_joint_torque_step(self, q_target=None, qdot_target=None, qddot_target=None):
        if qddot_target is not None:
            return self.moveJointTorqueStep(qddot_target)
        if q_target is not None and qdot_target is not None:
            return self.moveJointTorqueStep(q_target, qdot_target)
        return None

    # -- batched entries (device tensors, [field][B]) --------------------------
    def _run(self, mode, link_name, q, qdot, x_target, xdot_target, x_init=None, xdot_init=None,
             t=0.0, t0=0.0, duration=1.0, iters=None):
        p = self._pb.params(link_name, mode, self.Kp_task_, self.Kv_task_, t, t0, duration)
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

    # -- single-instance entries (reference signatures; B = 1 launches) -------
    def _one(self, out_status):
        out, status = out_status
        out, st = out.cpu().numpy()[:, 0], int(status.cpu().numpy()[0])
        if st != _capi.STATUS_SOLVED:
            print("QP IK failed to compute optimal joint velocity.", file=sys.stderr)
            out = np.zeros(self.dof_)
        return out

    def _state(self):
        rd = self.robot_data_
        return rd.q_.reshape(-1, 1), rd.qdot_.reshape(-1, 1)

    def QPIK(self, xdot_target, link_name):
        q, qd = self._state()
        return self._one(self.QPIK_batch(q, qd, np.asarray(xdot_target, float).reshape(6, 1), link_name))

    def QPIKStep(self, x_target, xdot_target, link_name):
        q, qd = self._state()
        return self._one(self.QPIK_step_batch(q, qd, pose_to12(x_target).reshape(12, 1),
                                              np.asarray(xdot_target, float).reshape(6, 1), link_name))

    def QPIKCubic(self, x_target, xdot_target, x_init, xdot_init, current_time, init_time, duration, link_name):
        q, qd = self._state()
        return self._one(self.QPIK_cubic_batch(
            q, qd, pose_to12(x_target).reshape(12, 1), np.asarray(xdot_target, float).reshape(6, 1),
            pose_to12(x_init).reshape(12, 1), np.asarray(xdot_init, float).reshape(6, 1),
            current_time, init_time, duration, link_name))

    QPIK_step, QPIK_cubic = QPIKStep, QPIKCubic

    # -- QPID / QPIDStep / QPIDCubic (robot_controller.cpp:319-361)
    def _run_id(self, mode, link_name, q, qdot, x_target, xdot_target, x_init=None, xdot_init=None,
                t=0.0, t0=0.0, duration=1.0, iters=None):
        p = self._pbd.params(link_name, mode, self.Kp_task_, self.Kv_task_, t, t0, duration)
        a = lambda v: _batch.as_device(v, self.robot_data_.device)
        return _batch.qpid_batch(self.robot_data_.model, p, a(q), a(qdot), a(x_target), a(xdot_target), a(x_init),
                                 a(xdot_init), iters=iters)

    def QPID_batch(self, q, qdot, xddot_target, link_name):
        """(qddot, tau, status) for B robots; tau = gravity where not solved."""
        return self._run_id(_capi.MODE_QPID, link_name, q, qdot, None, xddot_target)

    def QPID_step_batch(self, q, qdot, x_target, xdot_target, link_name, iters=None):
        return self._run_id(_capi.MODE_QPID_STEP, link_name, q, qdot, x_target, xdot_target, iters=iters)

    def QPID_cubic_batch(self, q, qdot, x_target, xdot_target, x_init, xdot_init, current_time, init_time,
                         duration, link_name):
        return self._run_id(_capi.MODE_QPID_CUBIC, link_name, q, qdot, x_target, xdot_target, x_init, xdot_init,
                            current_time, init_time, duration)

    def _one_id(self, res):
        qdd, tau, status = res
        if int(status.cpu().numpy()[0]) != _capi.STATUS_SOLVED:
            print("QP ID failed to compute optimal joint torque.", file=sys.stderr)
        return tau.cpu().numpy()[:, 0]   # already the gravity torque on failure (:333-336)

    def QPID(self, xddot_target, link_name):
        q, qd = self._state()
        return self._one_id(self.QPID_batch(q, qd, np.asarray(xddot_target, float).reshape(6, 1), link_name))

    def QPIDStep(self, x_target, xdot_target, link_name):
        q, qd = self._state()
        return self._one_id(self.QPID_step_batch(q, qd, pose_to12(x_target).reshape(12, 1),
                                                 np.asarray(xdot_target, float).reshape(6, 1), link_name))

    def QPIDCubic(self, x_target, xdot_target, x_init, xdot_init, current_time, init_time, duration, link_name):
        q, qd = self._state()
        return self._one_id(self.QPID_cubic_batch(
            q, qd, pose_to12(x_target).reshape(12, 1), np.asarray(xdot_target, float).reshape(6, 1),
            pose_to12(x_init).reshape(12, 1), np.asarray(xdot_init, float).reshape(6, 1),
            current_time, init_time, duration, link_name))

    QPID_step, QPID_cubic = QPIDStep, QPIDCubic

    # -- closed-form controllers (robot_controller.cpp:156-275) --
    def _run_cf(self, kind, mode, link_name, q, qdot, x_target, xdot_target, x_init=None, xdot_init=None,
                t=0.0, t0=0.0, duration=1.0, null=None):
        p = self._pb.params(link_name, mode, self.Kp_task_, self.Kv_task_, t, t0, duration)
        a = lambda v: _batch.as_device(v, self.robot_data_.device)
        return _batch.closed_form_batch(self.robot_data_.model, p, kind, a(q), a(qdot), a(x_target), a(xdot_target),
                                        a(x_init), a(xdot_init), a(null))

    def CLIK_step_batch(self, q, qdot, x_target, xdot_target, link_name, null_qdot=None):
        return self._run_cf("clik", _capi.MODE_QPIK_STEP, link_name, q, qdot, x_target, xdot_target, null=null_qdot)

    def CLIK_cubic_batch(self, q, qdot, x_target, xdot_target, x_init, xdot_init, current_time, init_time, duration,
                         link_name, null_qdot=None):
        return self._run_cf("clik", _capi.MODE_QPIK_CUBIC, link_name, q, qdot, x_target, xdot_target, x_init,
                            xdot_init, current_time, init_time, duration, null=null_qdot)

    def OSF_batch(self, q, qdot, xddot_target, link_name, null_torque=None):
        return self._run_cf("osf", _capi.MODE_QPIK, link_name, q, qdot, None, xddot_target, null=null_torque)

    def OSF_step_batch(self, q, qdot, x_target, xdot_target, link_name, null_torque=None):
        return self._run_cf("osf", _capi.MODE_QPIK_STEP, link_name, q, qdot, x_target, xdot_target, null=null_torque)

    def OSF_cubic_batch(self, q, qdot, x_target, xdot_target, x_init, xdot_init, current_time, init_time, duration,
                        link_name, null_torque=None):
        return self._run_cf("osf", _capi.MODE_QPIK_CUBIC, link_name, q, qdot, x_target, xdot_target, x_init,
                            xdot_init, current_time, init_time, duration, null=null_torque)

    @staticmethod
    def _split_null(args, n_fixed):
        """Reference overloads: (..., null_vec, link_name) or (..., link_name)."""
        if len(args) == n_fixed + 2:
            return args[:n_fixed], np.asarray(args[n_fixed], float).reshape(-1, 1), args[n_fixed + 1]
        return args[:n_fixed], None, args[n_fixed]

    def CLIKStep(self, *args):
        """CLIKStep(x_target, xdot_target[, null_qdot], link_name) -> qdot."""
        (x_t, xd_t), nu, link = self._split_null(args, 2)
        q, qd = self._state()
        return self.CLIK_step_batch(q, qd, pose_to12(x_t).reshape(12, 1), np.asarray(xd_t, float).reshape(6, 1), link,
                                    nu).cpu().numpy()[:, 0]

    def CLIKCubic(self, *args):
        """CLIKCubic(x_target, xdot_target, x_init, xdot_init, t, t0, T[, null_qdot], link_name)."""
        (x_t, xd_t, x_i, xd_i, t, t0, T), nu, link = self._split_null(args, 7)
        q, qd = self._state()
        return self.CLIK_cubic_batch(q, qd, pose_to12(x_t).reshape(12, 1), np.asarray(xd_t, float).reshape(6, 1),
                                     pose_to12(x_i).reshape(12, 1), np.asarray(xd_i, float).reshape(6, 1), t, t0, T,
                                     link, nu).cpu().numpy()[:, 0]

    def OSF(self, *args):
        """OSF(xddot_target[, null_torque], link_name) -> tau."""
        (xdd,), nu, link = self._split_null(args, 1)
        q, qd = self._state()
        return self.OSF_batch(q, qd, np.asarray(xdd, float).reshape(6, 1), link, nu).cpu().numpy()[:, 0]

    def OSFStep(self, *args):
        """OSFStep(x_target, xdot_target[, null_torque], link_name) -> tau."""
        (x_t, xd_t), nu, link = self._split_null(args, 2)
        q, qd = self._state()
        return self.OSF_step_batch(q, qd, pose_to12(x_t).reshape(12, 1), np.asarray(xd_t, float).reshape(6, 1), link,
                                   nu).cpu().numpy()[:, 0]

    def OSFCubic(self, *args):
        """OSFCubic(x_target, xdot_target, x_init, xdot_init, t, t0, T[, null_torque], link_name)."""
        (x_t, xd_t, x_i, xd_i, t, t0, T), nu, link = self._split_null(args, 7)
        q, qd = self._state()
        return self.OSF_cubic_batch(q, qd, pose_to12(x_t).reshape(12, 1), np.asarray(xd_t, float).reshape(6, 1),
                                    pose_to12(x_i).reshape(12, 1), np.asarray(xd_i, float).reshape(6, 1), t, t0, T,
                                    link, nu).cpu().numpy()[:, 0]

    CLIK_step, CLIK_cubic, OSF_step, OSF_cubic = CLIKStep, CLIKCubic, OSFStep, OSFCubic

"""Shared helpers for the parity tests (test infrastructure)."""
import numpy as np

import oracle as O
import pyref as R
from dyros_robot_controller_amd import manipulator, mobile_manipulator, robot_path, workload, _batch, _capi

LINK = {"fr3": "fr3_link8", "ur5e": "tool0", "husky_fr3": "fr3_link8", "xls_fr3": "fr3_link8"}


def make_manipulator(robot, device):
    rd = manipulator.RobotData(robot_path(robot), robot_path(robot, "srdf"), device=device)
    return rd


def stage_pose(model, device, q, qd, link):
    pb = manipulator.QPIKParamsBuilder(model, exact=True)
    p = pb.params(link, _capi.MODE_QPIK)
    B = q.shape[1]
    st = _batch.stages_batch(model, p, _batch.as_device(q, device), _batch.as_device(qd, device), None,
                             _batch.as_device(np.zeros((6, B)), device))
    return {k: v.cpu().numpy() for k, v in st.items()}


def stage_step(model, device, q, qd, xt, xdt, link):
    """Stage outputs of the QPIKStep pipeline (same params as the solve)."""
    pb = manipulator.QPIKParamsBuilder(model, exact=True)
    p = pb.params(link, _capi.MODE_QPIK_STEP)
    st = _batch.stages_batch(model, p, _batch.as_device(q, device), _batch.as_device(qd, device),
                             _batch.as_device(xt, device), _batch.as_device(xdt, device))
    return {k: v.cpu().numpy() for k, v in st.items()}


def qp_from_stages(pm, q, st, b, link):
    """Exact optimum (numpy IPM, oracle/pyref.py) of the manipulator QP built
    from one instance's device stage data (QP_IK.cpp:59-128)."""
    man = (st["man"][0, b], st["man"][1:, b])
    dist = (st["dist"][0, b], st["dist"][1:, b])
    P, qv, A, l, u = R.build_qp_manipulator(pm, q[:, b], st["xdot_des"][:, b], link, man=man, dist=dist)
    x, _, status = R.solve_qp_exact(P, qv, A, l, u)
    return x[:pm.nv] if x is not None else None


def step_inputs(rd, robot, seed, B, device, offset=0):
    lo, hi = rd.getJointPositionLimit()
    _, vmax = rd.getJointVelocityLimit()
    q, qd = workload.joint_states(lo, hi, vmax, seed, B, offset)
    st = stage_pose(rd.model, device, q, qd, LINK[robot])
    xt, xdt = workload.perturb_targets(st["pose"], seed, B, offset)
    return q, qd, xt, xdt


def oracle_batch(robot, q, qd, xt, xdt, exact=True, xi=None, xdi=None, mode=1, t=0.0, t0=0.0, T=1.0, nthreads=8):
    pm, om, spec = O.load(robot)
    par = O.default_params(spec["kind"], exact=exact)
    par.mode = mode
    par.t, par.t0, par.duration = t, t0, T
    out, status, iters = O.qpik_batch(om, par, q, qd, xt, xdt, xi, xdi, nthreads=nthreads)
    return out, status, iters, om


def task_residual(J, dq):
    return np.max(np.abs(J @ dq))


def nonsmooth_min_distance(om, q, h=1e-7, tol=1e-3):
    """True where the oracle's min self-distance is not differentiable at q
    (one-sided derivatives differ): argmin switches between pairs, or the
    witness points are not unique (parallel flat/cylindrical features, e.g.
    UR5e's three parallel joint axes).  The reference's gradient
    (robot_data.cpp:476-494) is ill-defined there — SURVEY H2."""
    d0 = O.min_distance(om, q)[0]
    for k in range(len(q)):
        e = np.zeros(len(q))
        e[k] = h
        fwd = (O.min_distance(om, q + e)[0] - d0) / h
        bwd = (d0 - O.min_distance(om, q - e)[0]) / h
        if abs(fwd - bwd) > tol:
            return True
    return False


# -- mobile manipulators (fixture robots, N5) -------------
def moma_kinematic_param(robot):
    MM = mobile_manipulator
    if robot == "husky_fr3":
        return MM.KinematicParam(MM.DriveType.Differential, 0.165, base_width=0.555)
    return MM.KinematicParam(MM.DriveType.Mecanum, 0.120, roller_angles=[-np.pi / 4, np.pi / 4, np.pi / 4, -np.pi / 4],
                             base2wheel_positions=[(0.2225, 0.2045), (0.2225, -0.2045), (-0.2225, 0.2045),
                                                   (-0.2225, -0.2045)],
                             base2wheel_angles=[0, 0, 0, 0])


def make_moma(robot, device):
    MM = mobile_manipulator
    spec = O.ROBOTS[robot]
    vs, ms, ws = spec["joint_index"]
    am, aw = spec["actuator_index"]
    return MM.RobotData(moma_kinematic_param(robot), MM.JointIndex(vs, ms, ws), MM.ActuatorIndex(am, aw),
                        robot_path(robot), robot_path(robot, "srdf"), device=device)


def moma_step_inputs(rd, robot, seed, B, device, offset=0):
    lo, hi = rd.get_joint_position_limit()
    _, vmax = rd.get_joint_velocity_limit()
    ji = rd.get_joint_index()
    q, qd = workload.mobile_states(lo, hi, vmax, (ji.virtual_start, ji.mani_start, ji.mobi_start),
                                   rd.get_manipulator_dof(), rd.get_mobile_dof(), seed, B, offset)
    st = stage_pose(rd.model, device, q, qd, LINK[robot])
    xt, xdt = workload.perturb_targets(st["pose"], seed, B, offset)
    return q, qd, xt, xdt

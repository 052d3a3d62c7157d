"""Batched device-side entry: torch tensors in HBM -> C-ABI -> HIP kernel.

torch is used as plumbing only (device allocations and the current HIP
stream); the arithmetic happens in ``libdrc_amd.so``.
"""
import ctypes as C

import numpy as np

from . import _capi

_FIELD_SHAPES = {"q": "dof", "qdot": "dof", "x_target": 12, "xdot_target": 6, "x_init": 12, "xdot_init": 6}


def _torch():
    import torch
    return torch


def as_device(a, device):
    """float64, contiguous, on ``device`` (a torch.device)."""
    torch = _torch()
    if a is None:
        return None
    if not isinstance(a, torch.Tensor):
        a = torch.as_tensor(np.asarray(a, dtype=np.float64))
    return a.to(device=device, dtype=torch.float64).contiguous()


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def check_shapes(dof, B, **fields):
    for k, v in fields.items():
        if v is None:
            continue
        rows = dof if _FIELD_SHAPES[k] == "dof" else _FIELD_SHAPES[k]
        if tuple(v.shape) != (rows, B):
            raise ValueError("%s must be [%d][B=%d] (field-major SoA), got %s" % (k, rows, B, tuple(v.shape)))


def qpik_batch(model, params, q, qdot, x_target=None, xdot_target=None, x_init=None, xdot_init=None,
               out=None, status=None, iters=None, stream=None):
    """Launch ``drc_qpik_batch`` on device tensors laid out [field][B]."""
    torch = _torch()
    dev = q.device
    B = q.shape[1]
    check_shapes(model.dof, B, q=q, qdot=qdot, x_target=x_target, xdot_target=xdot_target,
                 x_init=x_init, xdot_init=xdot_init)
    if out is None:
        out = torch.empty((model.actuated_dof, B), dtype=torch.float64, device=dev)
    if status is None:
        status = torch.empty(B, dtype=torch.int32, device=dev)
    if stream is None:
        stream = torch.cuda.current_stream(dev).cuda_stream
    _capi.check(_capi.lib().drc_qpik_batch(
        model.handle, C.byref(params), C.c_int64(B), _ptr(q), _ptr(qdot), _ptr(x_target), _ptr(xdot_target),
        _ptr(x_init), _ptr(xdot_init), _ptr(out), _ptr(status), _ptr(iters), C.c_void_p(stream)))
    return out, status


def qpid_batch(model, params, q, qdot, x_target=None, xdot_target=None, x_init=None, xdot_init=None,
               qddot=None, tau=None, status=None, iters=None, stream=None):
    """Launch ``drc_qpid_batch``: returns (qddot [na][B],
    tau [na][B], status [B]) device tensors."""
    torch = _torch()
    dev = q.device
    B = q.shape[1]
    check_shapes(model.dof, B, q=q, qdot=qdot, x_target=x_target, xdot_target=xdot_target,
                 x_init=x_init, xdot_init=xdot_init)
    na = model.actuated_dof
    if qddot is None:
        qddot = torch.empty((na, B), dtype=torch.float64, device=dev)
    if tau is None:
        tau = torch.empty((na, B), dtype=torch.float64, device=dev)
    if status is None:
        status = torch.empty(B, dtype=torch.int32, device=dev)
    if stream is None:
        stream = torch.cuda.current_stream(dev).cuda_stream
    _capi.check(_capi.lib().drc_qpid_batch(
        model.handle, C.byref(params), C.c_int64(B), _ptr(q), _ptr(qdot), _ptr(x_target), _ptr(xdot_target),
        _ptr(x_init), _ptr(xdot_init), _ptr(qddot), _ptr(tau), _ptr(status), _ptr(iters), C.c_void_p(stream)))
    return qddot, tau, status


def qpid_stages_batch(model, params, q, qdot, x_target=None, xdot_target=None, x_init=None, xdot_init=None):
    """QPID stage outputs: the QPIK stage fields plus jdot [6*nv][B] and
    qpid_terms [8][B] = (Jdot v, man grad_dot . qdot_arm, dist grad_dot . qdot_arm)."""
    torch = _torch()
    dev = q.device
    B = q.shape[1]
    nv = model.dof
    f = lambda r: torch.zeros((r, B), dtype=torch.float64, device=dev)
    pose, jac, man, dist, xdd, jdot, terms = f(12), f(6 * nv), f(1 + model.mani_dof), f(1 + nv), f(6), f(6 * nv), f(8)
    gdv = f(model.mani_dof + nv)
    pair = torch.zeros(B, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    _capi.check(_capi.lib().drc_qpid_stages_batch(
        model.handle, C.byref(params), C.c_int64(B), _ptr(q), _ptr(qdot), _ptr(x_target), _ptr(xdot_target),
        _ptr(x_init), _ptr(xdot_init), _ptr(pose), _ptr(jac), _ptr(man), _ptr(dist), _ptr(pair), _ptr(xdd),
        _ptr(jdot), _ptr(terms), _ptr(gdv), C.c_void_p(stream)))
    return dict(pose=pose, jac=jac, man=man, dist=dist, pair=pair, xddot_des=xdd, jdot=jdot, qpid_terms=terms,
                man_graddot=gdv[:model.mani_dof], dist_graddot=gdv[model.mani_dof:])


def stages_batch(model, params, q, qdot, x_target=None, xdot_target=None, x_init=None, xdot_init=None):
    """Stage outputs (pose, J, manipulability, min distance, task velocity)."""
    torch = _torch()
    dev = q.device
    B = q.shape[1]
    nv = model.dof
    mani = model.mani_dof
    f = lambda r: torch.zeros((r, B), dtype=torch.float64, device=dev)
    pose, jac, man, dist, xdd = f(12), f(6 * nv), f(1 + mani), f(1 + nv), f(6)
    pair = torch.zeros(B, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    _capi.check(_capi.lib().drc_qpik_stages_batch(
        model.handle, C.byref(params), C.c_int64(B), _ptr(q), _ptr(qdot), _ptr(x_target), _ptr(xdot_target),
        _ptr(x_init), _ptr(xdot_init), _ptr(pose), _ptr(jac), _ptr(man), _ptr(dist), _ptr(pair), _ptr(xdd),
        C.c_void_p(stream)))
    return dict(pose=pose, jac=jac, man=man, dist=dist, pair=pair, xdot_des=xdd)


DYN_FIELDS = ("M", "Minv", "g", "nle", "c")


def dynamics_batch(model, q, qdot=None, actuated=False, fields=DYN_FIELDS, stream=None):
    """Launch ``drc_dynamics_batch`` on device tensors
    [dof][B]; returns {name: tensor} with M, Minv as [n][n][B] and the vectors
    as [n][B] (n = actuated dof when ``actuated``)."""
    torch = _torch()
    dev = q.device
    B = q.shape[1]
    check_shapes(model.dof, B, q=q, qdot=qdot)
    n = model.actuated_dof if actuated else model.dof
    out = {}
    for k in fields:
        rows = n * n if k in ("M", "Minv") else n
        out[k] = torch.empty((rows, B), dtype=torch.float64, device=dev)
    if stream is None:
        stream = torch.cuda.current_stream(dev).cuda_stream
    _capi.check(_capi.lib().drc_dynamics_batch(
        model.handle, C.c_int(1 if actuated else 0), C.c_int64(B), _ptr(q), _ptr(qdot),
        _ptr(out.get("M")), _ptr(out.get("Minv")), _ptr(out.get("g")), _ptr(out.get("nle")), _ptr(out.get("c")),
        C.c_void_p(stream)))
    for k in ("M", "Minv"):
        if k in out:
            out[k] = out[k].view(n, n, B)
    return out


def dynamics_host(model, q, qdot=None, actuated=False):
    """``drc_dynamics_host`` on numpy arrays [dof][B] (synchronous)."""
    q = np.ascontiguousarray(q, dtype=np.float64)
    B = q.shape[1]
    qd = None if qdot is None else np.ascontiguousarray(qdot, dtype=np.float64)
    n = model.actuated_dof if actuated else model.dof
    M, Mi = np.zeros((n, n, B)), np.zeros((n, n, B))
    g = np.zeros((n, B))
    nle = np.zeros((n, B)) if qd is not None else None
    c = np.zeros((n, B)) if qd is not None else None
    dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double)) if a is not None else None
    _capi.check(_capi.lib().drc_dynamics_host(model.handle, C.c_int(1 if actuated else 0), C.c_int64(B), dp(q),
                                              dp(qd), dp(M), dp(Mi), dp(g), dp(nle), dp(c)))
    return dict(M=M, Minv=Mi, g=g, nle=nle, c=c)


def joint_torque_step_batch(model, q, qdot=None, q_target=None, qdot_target=None, qddot_target=None, dt=0.0,
                            kp=None, kv=None, stream=None):
    """``drc_joint_torque_step_batch`` on device tensors: tau [nb][B] for the
    controlled block (all joints, or the arm of a mobile manipulator)."""
    torch = _torch()
    dev = q.device
    B = q.shape[1]
    check_shapes(model.dof, B, q=q, qdot=qdot)
    nb = model.mani_dof
    for name, t in (("q_target", q_target), ("qdot_target", qdot_target), ("qddot_target", qddot_target)):
        if t is not None and tuple(t.shape) != (nb, B):
            raise ValueError("%s must be [%d][B=%d], got %s" % (name, nb, B, tuple(t.shape)))
    tau = torch.empty((nb, B), dtype=torch.float64, device=dev)
    gain = lambda g: None if g is None else np.ascontiguousarray(np.broadcast_to(np.asarray(g, float), (nb,)))
    kp, kv = gain(kp), gain(kv)
    dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double)) if a is not None else None
    if stream is None:
        stream = torch.cuda.current_stream(dev).cuda_stream
    _capi.check(_capi.lib().drc_joint_torque_step_batch(
        model.handle, C.c_int64(B), _ptr(q), _ptr(qdot), _ptr(q_target), _ptr(qdot_target), _ptr(qddot_target),
        C.c_double(dt), dp(kp), dp(kv), _ptr(tau), C.c_void_p(stream)))
    return tau


def closed_form_batch(model, params, kind, q, qdot, x_target=None, xdot_target=None, x_init=None, xdot_init=None,
                      null=None, out=None, stream=None):
    """``drc_clik_batch`` (kind "clik") / ``drc_osf_batch`` (kind "osf") on
    device tensors [field][B]; returns qdot / tau [dof][B]."""
    torch = _torch()
    dev = q.device
    B = q.shape[1]
    check_shapes(model.dof, B, q=q, qdot=qdot, x_target=x_target, xdot_target=xdot_target,
                 x_init=x_init, xdot_init=xdot_init)
    if null is not None and tuple(null.shape) != (model.dof, B):
        raise ValueError("null vector must be [%d][B=%d]" % (model.dof, B))
    if out is None:
        out = torch.empty((model.dof, B), dtype=torch.float64, device=dev)
    if stream is None:
        stream = torch.cuda.current_stream(dev).cuda_stream
    fn = _capi.lib().drc_clik_batch if kind == "clik" else _capi.lib().drc_osf_batch
    _capi.check(fn(model.handle, C.byref(params), C.c_int64(B), _ptr(q), _ptr(qdot), _ptr(x_target),
                   _ptr(xdot_target), _ptr(x_init), _ptr(xdot_init), _ptr(null), _ptr(out), C.c_void_p(stream)))
    return out

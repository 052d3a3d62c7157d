"""ctypes binding of the C-ABI declared in ``include/drc_amd.h``.

The product path: every call here ends in ``libdrc_amd.so`` (hand-written
HIP for gfx950).  There is no CPU fallback — if the shared library is
missing or fails to load, importing this module raises.
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# DRC_AMD_LIB selects a diagnostic build (e.g. libdrc_amd_timing.so); default is the product library
LIB_PATH = os.path.join(HERE, os.environ.get("DRC_AMD_LIB", "libdrc_amd.so"))

# return codes
DRC_OK = 0
DRC_ERR_INVALID_ARGUMENT = 1
DRC_ERR_FILE = 2
DRC_ERR_PARSE = 3
DRC_ERR_UNSUPPORTED = 4
DRC_ERR_UNKNOWN_LINK = 5
DRC_ERR_HIP = 6
DRC_ERR_SIZE_MISMATCH = 7
# per-instance status (OSQP values)
STATUS_SOLVED = 1
STATUS_MAX_ITER = -2
STATUS_PRIMAL_INFEASIBLE = -3
STATUS_NONFINITE = -10
# modes
MODE_QPIK, MODE_QPIK_STEP, MODE_QPIK_CUBIC = 0, 1, 2
MODE_QPID, MODE_QPID_STEP, MODE_QPID_CUBIC = 0, 1, 2
# drive types
DRIVE_DIFFERENTIAL, DRIVE_MECANUM, DRIVE_CASTER = 0, 1, 2
MAX_WHEELS = 8

# every symbol include/drc_amd.h and include/drc_amd_debug.h declare (checked by tests/test_capi.py)
EXPORTED_SYMBOLS = (
    "drc_model_create_manipulator", "drc_model_create_mobile_manipulator", "drc_model_destroy",
    "drc_model_info", "drc_model_limits", "drc_model_find_frame", "drc_model_mobile_fk_jacobian",
    "drc_mobile_fk_jacobian", "drc_mobile_ik_jacobian",
    "drc_default_qpik_params", "drc_qpik_batch", "drc_qpik_stages_batch", "drc_debug_kernel_timing", "drc_debug_lds_plan",
    "drc_debug_host_timeline", "drc_debug_waves", "drc_debug_qpik_stamps",
    "drc_debug_kernel_times", "drc_debug_instance_order", "drc_set_concurrency", "drc_set_fusion", "drc_model_release_stream", "drc_debug_lane_stage", "drc_qpik_host", "drc_qpik_stages_host",
    "drc_dynamics_batch", "drc_dynamics_host", "drc_joint_torque_step_batch", "drc_joint_torque_step_host",
    "drc_default_qpid_params", "drc_qpid_batch", "drc_qpid_stages_batch", "drc_qpid_host",
    "drc_qpid_stages_host", "drc_clik_batch", "drc_osf_batch", "drc_closed_form_host",
    "drc_error_string", "drc_last_error", "drc_build_id", "drc_qpik_host_timed", "drc_kinematics_batch",
    "drc_state_host",
)


class TimeDuration(C.Structure):
    """drc_time_duration = QP::TimeDuration (QP_base.h:19-43), seconds."""
    _fields_ = [(n, C.c_double) for n in ("set_qp", "set_cost", "set_bound", "set_ineq", "set_eq", "set_constraint",
                                          "set_solver", "solve_qp")]


class SolverSettings(C.Structure):
    _fields_ = [
        ("rho", C.c_double), ("sigma", C.c_double), ("alpha", C.c_double),
        ("eps_abs", C.c_double), ("eps_rel", C.c_double), ("eps_prim_inf", C.c_double),
        ("max_iter", C.c_int), ("check_termination", C.c_int), ("scaling", C.c_int),
        ("adaptive_rho", C.c_int), ("adaptive_rho_interval", C.c_int),
        ("adaptive_rho_tolerance", C.c_double),
        ("polish", C.c_int), ("polish_refine_iter", C.c_int), ("delta", C.c_double),
        ("exact", C.c_int), ("eps_exact", C.c_double), ("eps_fallback", C.c_double),
    ]


class QPIKParams(C.Structure):
    _fields_ = [
        ("kp", C.c_double * 6), ("kv", C.c_double * 6), ("feedforward", C.c_double),
        ("alpha_cbf", C.c_double), ("w_reg", C.c_double), ("slack_w", C.c_double),
        ("man_min", C.c_double), ("dist_min", C.c_double),
        ("mode", C.c_int), ("frame_id", C.c_int),
        ("t", C.c_double), ("t0", C.c_double), ("duration", C.c_double),
        ("solver", SolverSettings),
    ]


class KinematicParam(C.Structure):
    _fields_ = [
        ("type", C.c_int), ("wheel_radius", C.c_double),
        ("max_lin_speed", C.c_double), ("max_ang_speed", C.c_double),
        ("max_lin_acc", C.c_double), ("max_ang_acc", C.c_double),
        ("base_width", C.c_double), ("n_wheels", C.c_int),
        ("roller_angles", C.c_double * MAX_WHEELS),
        ("base2wheel_positions", (C.c_double * 2) * MAX_WHEELS),
        ("base2wheel_angles", C.c_double * MAX_WHEELS),
        ("wheel_offset", C.c_double),
    ]


class JointIndex(C.Structure):
    _fields_ = [("virtual_start", C.c_int), ("mani_start", C.c_int), ("mobi_start", C.c_int)]


class ActuatorIndex(C.Structure):
    _fields_ = [("mani_start", C.c_int), ("mobi_start", C.c_int)]


class DrcError(RuntimeError):
    def __init__(self, code, detail):
        super().__init__("%s (code %d): %s" % (_lib.drc_error_string(code).decode(), code, detail))
        self.code = code


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError("libdrc_amd.so is not built (%s): run __graft_entry__.build() — "
                          "there is no CPU fallback for the QP-IK hot path" % LIB_PATH)
    # torch ships the HIP runtime under the same soname; import it first so the
    # library binds to the runtime that owns torch's device allocations.
    try:
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch is plumbing only
        pass
    lib = C.CDLL(LIB_PATH)
    vp, dp, ip = C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_int)
    lib.drc_error_string.restype = C.c_char_p
    lib.drc_error_string.argtypes = [C.c_int]
    lib.drc_last_error.restype = C.c_char_p
    lib.drc_last_error.argtypes = []
    lib.drc_build_id.restype = C.c_char_p
    lib.drc_build_id.argtypes = []
    lib.drc_model_create_manipulator.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_int, C.POINTER(vp)]
    lib.drc_model_create_mobile_manipulator.argtypes = [
        C.POINTER(KinematicParam), C.POINTER(JointIndex), C.POINTER(ActuatorIndex),
        C.c_char_p, C.c_char_p, C.c_char_p, C.c_int, C.POINTER(vp)]
    lib.drc_model_destroy.argtypes = [vp]
    lib.drc_model_destroy.restype = None
    lib.drc_model_info.argtypes = [vp, ip, ip, ip, ip, ip, ip]
    lib.drc_model_limits.argtypes = [vp, dp, dp, dp, dp]
    lib.drc_model_find_frame.argtypes = [vp, C.c_char_p, ip]
    lib.drc_model_mobile_fk_jacobian.argtypes = [vp, dp]
    lib.drc_mobile_fk_jacobian.argtypes = [C.POINTER(KinematicParam), dp, dp, ip]
    lib.drc_mobile_ik_jacobian.argtypes = [C.POINTER(KinematicParam), dp, dp, ip]
    lib.drc_default_qpik_params.argtypes = [vp, C.c_int, C.POINTER(QPIKParams)]
    lib.drc_qpik_batch.argtypes = [vp, C.POINTER(QPIKParams), C.c_int64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    lib.drc_qpik_stages_batch.argtypes = [vp, C.POINTER(QPIKParams), C.c_int64, vp, vp, vp, vp, vp, vp,
                                          vp, vp, vp, vp, vp, vp, vp]
    lib.drc_debug_kernel_timing.argtypes = [vp, C.c_int]
    # diagnostics added in r05: bound only when present, so A/B runs can load
    # an older build (tests/test_capi_symbols.py checks the product exports them)
    if hasattr(lib, "drc_debug_waves"):
        lib.drc_debug_waves.argtypes = [vp, C.c_void_p, ip, ip]
    if hasattr(lib, "drc_debug_host_timeline"):
        lib.drc_debug_host_timeline.argtypes = [vp, C.c_int, C.POINTER(C.c_int64), C.c_int64, C.POINTER(C.c_int64)]
    if hasattr(lib, "drc_debug_qpik_stamps"):
        lib.drc_debug_qpik_stamps.argtypes = [vp, C.POINTER(QPIKParams), C.c_int64, dp, dp, dp, dp, dp, dp, dp, ip,
                                              ip, C.POINTER(C.c_uint64)]
    if hasattr(lib, "drc_debug_lds_plan"):  # diagnostic; absent from older A/B builds (tools/ab_bench.sh)
        lib.drc_debug_lds_plan.argtypes = [vp, C.POINTER(QPIKParams), C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]
    lib.drc_debug_kernel_times.argtypes = [vp, dp, dp, dp, ip]
    lib.drc_debug_lane_stage.argtypes = [vp, C.c_int]
    lib.drc_set_concurrency.argtypes = [vp, C.c_int]
    lib.drc_model_release_stream.argtypes = [vp, vp]
    lib.drc_set_fusion.argtypes = [vp, C.c_int]
    lib.drc_qpik_host.argtypes = [vp, C.POINTER(QPIKParams), C.c_int64, dp, dp, dp, dp, dp, dp, dp, ip, ip]
    lib.drc_qpik_stages_host.argtypes = [vp, C.POINTER(QPIKParams), C.c_int64, dp, dp, dp, dp, dp, dp,
                                         dp, dp, dp, dp, ip, dp]
    lib.drc_dynamics_batch.argtypes = [vp, C.c_int, C.c_int64, vp, vp, vp, vp, vp, vp, vp, vp]
    lib.drc_dynamics_host.argtypes = [vp, C.c_int, C.c_int64, dp, dp, dp, dp, dp, dp, dp]
    lib.drc_qpik_host_timed.argtypes = [vp, C.POINTER(QPIKParams), C.c_int64, dp, dp, dp, dp, dp, dp, dp, ip, ip,
                                        C.POINTER(TimeDuration)]
    lib.drc_kinematics_batch.argtypes = [vp, C.c_int, C.c_int64, vp, vp, vp, vp, vp, vp]
    lib.drc_state_host.argtypes = [vp, C.c_int, C.c_int64, dp, dp, dp, dp, dp, dp, dp, dp, dp, dp]
    lib.drc_joint_torque_step_batch.argtypes = [vp, C.c_int64, vp, vp, vp, vp, vp, C.c_double, dp, dp, vp, vp]
    lib.drc_joint_torque_step_host.argtypes = [vp, C.c_int64, dp, dp, dp, dp, dp, C.c_double, dp, dp, dp]
    lib.drc_default_qpid_params.argtypes = [vp, C.c_int, C.POINTER(QPIKParams)]
    lib.drc_qpid_batch.argtypes = [vp, C.POINTER(QPIKParams), C.c_int64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    lib.drc_qpid_stages_batch.argtypes = [vp, C.POINTER(QPIKParams), C.c_int64, vp, vp, vp, vp, vp, vp,
                                          vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    lib.drc_qpid_stages_host.argtypes = [vp, C.POINTER(QPIKParams), C.c_int64, dp, dp, dp, dp, dp, dp,
                                         dp, dp, dp, dp, ip, dp, dp, dp, dp]
    lib.drc_qpid_host.argtypes = [vp, C.POINTER(QPIKParams), C.c_int64, dp, dp, dp, dp, dp, dp, dp, dp, ip, ip]
    lib.drc_clik_batch.argtypes = [vp, C.POINTER(QPIKParams), C.c_int64, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    lib.drc_osf_batch.argtypes = [vp, C.POINTER(QPIKParams), C.c_int64, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    lib.drc_closed_form_host.argtypes = [vp, C.POINTER(QPIKParams), C.c_int, C.c_int64, dp, dp, dp, dp, dp, dp, dp, dp]
    for name in EXPORTED_SYMBOLS:
        if name in ("drc_debug_lds_plan", "drc_debug_waves", "drc_debug_host_timeline",
                    "drc_debug_qpik_stamps", "drc_debug_instance_order") and not hasattr(lib, name):
            continue  # diagnostics an older A/B build may lack
        if name not in ("drc_model_destroy", "drc_error_string", "drc_last_error", "drc_build_id"):
            getattr(lib, name).restype = C.c_int
    return lib


_lib = _load()


def lib():
    return _lib


def check(rc):
    if rc != DRC_OK:
        raise DrcError(rc, _lib.drc_last_error().decode())
    return rc


def build_id():
    """drc_build_id(): hash of the loaded library's sources and flags (build.sh)."""
    return lib().drc_build_id().decode()

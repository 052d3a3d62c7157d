"""The C-ABI library loads (no GPU needed) and exports every function that
include/drc_amd.h (the drop-in boundary) and include/drc_amd_debug.h (the
diagnostic entries) declare; the Python ctypes layer mirrors the structs."""
import ctypes
import os
import re

from dyros_robot_controller_amd import _capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header="drc_amd.h"):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(drc_[a-z0-9_]+)\s*\(", src)))


def test_header_symbols_exported():
    lib = ctypes.CDLL(_capi.LIB_PATH)
    names = _declared()
    debug = _declared("drc_amd_debug.h")
    assert len(names) >= 12
    assert debug and all(n.startswith("drc_debug_") for n in debug)
    assert not any(n.startswith("drc_debug_") for n in names)   # diagnostics stay out of the boundary
    for n in names + debug:
        assert hasattr(lib, n), n
    assert set(names) | set(debug) == set(_capi.EXPORTED_SYMBOLS)


def test_error_strings():
    assert _capi.lib().drc_error_string(_capi.DRC_ERR_UNKNOWN_LINK) == b"link name not found in URDF"


def test_struct_layouts_match_header(tmp_path):
    """Compile the header with gcc and compare sizeof/offsetof with ctypes."""
    import subprocess
    src = tmp_path / "sz.c"
    src.write_text("""#include <stdio.h>
#include <stddef.h>
#include "drc_amd.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(drc_solver_settings), sizeof(drc_qpik_params),
         sizeof(drc_kinematic_param), sizeof(drc_joint_index), sizeof(drc_actuator_index),
         offsetof(drc_qpik_params, solver), offsetof(drc_qpik_params, frame_id),
         offsetof(drc_kinematic_param, wheel_offset));
  return 0;
}
""")
    exe = tmp_path / "sz"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    got = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    C = ctypes
    want = [C.sizeof(_capi.SolverSettings), C.sizeof(_capi.QPIKParams), C.sizeof(_capi.KinematicParam),
            C.sizeof(_capi.JointIndex), C.sizeof(_capi.ActuatorIndex), _capi.QPIKParams.solver.offset,
            _capi.QPIKParams.frame_id.offset, _capi.KinematicParam.wheel_offset.offset]
    assert got == want

"""GJK tolerance census on the CPU (diagnostic; test infrastructure): the
oracle's exact-mode QPIKStep over a device dump of the bench inputs
(tools/dump_batch.py) at several GJK stop tolerances, with the GJK iteration
count (oracle_gjk_study) and how far q-dot moves from the 1e-9 run.

    python tools/gjk_tol_census.py <robot> [dump.npz]
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]


def main():
    import oracle as O
    robot = sys.argv[1] if len(sys.argv) > 1 else "ur5e"
    path = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", "dump_%s_16384.npz" % robot)
    d = np.load(path)
    _, om, spec = O.load(robot)
    par = O.default_params(spec["kind"], exact=True)
    L = O.lib()
    L.oracle_gjk_study.argtypes = [C.c_double, C.POINTER(C.c_longlong), C.c_int]
    ins = [np.ascontiguousarray(d[x]) for x in ("q", "qd", "xt", "xdt")]
    ref = None
    for tol in (1e-9, 1e-7, 1e-6):
        it = C.c_longlong()
        L.oracle_gjk_study(tol, None, 1)
        out, st, its = O.qpik_batch(om, par, *ins, nthreads=8)
        L.oracle_gjk_study(0.0, C.byref(it), 0)
        ref = out if ref is None else ref
        dq = np.abs(out - ref).max(axis=0)
        print(robot, tol, "gjk iterations", it.value, "instances |dq|>1e-9:", int((dq > 1e-9).sum()),
              "max |dq| %.3g" % float(dq.max()), flush=True)
    L.oracle_gjk_study(1e-6, None, 0)   # back to the product tolerance


if __name__ == "__main__":
    main()

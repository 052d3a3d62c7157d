"""Dev tool: QPID GPU-vs-oracle error distribution (exact mode)."""
import sys
sys.path[:0] = ["tests", "oracle", "."]
import numpy as np
import torch
from test_gpu_qpid import _inputs, _oracle, _task_matrix
from _common import LINK
import oracle as O

cuda = torch.device("cuda", 0)
for robot in sys.argv[1:] or ["fr3", "ur5e", "husky_fr3", "xls_fr3"]:
    rd, ctrl, q, qd, xt, xdt = _inputs(robot, cuda, 32, 192)
    qdd, tau, status = [v.cpu().numpy() for v in ctrl.QPID_step_batch(q, qd, xt, xdt, LINK[robot])]
    rq, rt, rs, diags, om, spec, _ = _oracle(robot, q, qd, xt, xdt)
    ok = (rs == O.SOLVED) & (status == rs)
    scale = np.maximum(1.0, np.maximum(np.abs(rq).max(axis=0), np.abs(rt).max(axis=0)))
    err = np.maximum(np.abs(qdd - rq).max(axis=0), np.abs(tau - rt).max(axis=0))
    rel = err / scale
    terr = []
    for b in np.nonzero(ok)[0]:
        Jt = _task_matrix(om, spec, q[:, b], diags[b])
        tr = Jt @ rq[:, b]
        terr.append(np.abs(Jt @ qdd[:, b] - tr).max() / (1 + np.abs(tr).max()))
    terr = np.array(terr)
    pct = lambda a: " ".join("%.1e" % np.percentile(a, p) for p in (50, 90, 99, 100))
    print(robot, "status agree %.3f solved %d/%d" % (np.mean(status == rs), ok.sum(), len(rs)))
    print("  abs err p50/90/99/max", pct(err[ok]))
    print("  rel err p50/90/99/max", pct(rel[ok]))
    print("  task-acc rel p50/90/99/max", pct(terr))
    it = np.array([d.iters for d in diags]); pol = np.array([d.polished for d in diags])
    print("  oracle iters mean %.1f polished %.3f" % (it[ok].mean(), pol[ok].mean()))
    sys.stdout.flush()

# outlier detail (argv: ur5e)
from dyros_robot_controller_amd import _batch, _capi
from _common import nonsmooth_min_distance
robot = "ur5e"
rd, ctrl, q, qd, xt, xdt = _inputs(robot, cuda, 32, 192)
qdd, tau, status = [v.cpu().numpy() for v in ctrl.QPID_step_batch(q, qd, xt, xdt, LINK[robot])]
rq, rt, rs, diags, om, spec, _ = _oracle(robot, q, qd, xt, xdt)
p = ctrl._pbd.params(LINK[robot], _capi.MODE_QPID_STEP, ctrl.Kp_task_, ctrl.Kv_task_)
a = lambda v: _batch.as_device(v, cuda)
st = _batch.qpid_stages_batch(rd.model, p, a(q), a(qd), a(xt), a(xdt))
st = {k: v.cpu().numpy() for k, v in st.items()}
for b in range(192):
    Jt = _task_matrix(om, spec, q[:, b], diags[b])
    tr = Jt @ rq[:, b]
    e = np.abs(Jt @ qdd[:, b] - tr).max() / (1 + np.abs(tr).max())
    if e > 1e-6:
        dg = diags[b]
        gd = np.max(np.abs(st["dist"][1:, b] - np.array(dg.dist_grad[:om.nv])))
        print("b %d tacc %.1e d %.4f gpu d %.4f pair %d/%d graddiff %.1e gd %.3e/%.3e man %.3e/%.3e mgd %.3e/%.3e ns %s" % (
            b, e, dg.dist, st["dist"][0, b], dg.pair, st["pair"][b], gd, dg.dist_gd, st["qpid_terms"][7, b],
            dg.man, st["man"][0, b], dg.man_gd, st["qpid_terms"][6, b], nonsmooth_min_distance(om, q[:, b])))

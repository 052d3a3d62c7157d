"""Boundary contract (include/drc_amd.h): one model driven from two HIP
streams at once, and from two host threads on one stream, returns exactly
what single-stream calls return (per-stream scratch: task records, work-queue
counters and fork/join lanes are not shared)."""
import threading

import numpy as np
import pytest

from _common import LINK, make_manipulator, step_inputs
from dyros_robot_controller_amd import _batch, manipulator

pytestmark = pytest.mark.gpu


def test_two_streams_one_model(cuda):
    import torch
    rd = make_manipulator("fr3", cuda)
    ctrl = manipulator.RobotController(0.001, rd, solver_mode="exact")
    B = 32768   # two concurrent sub-batches per call, each >= 16 Ki instances
    ins = [[torch.as_tensor(a, device=cuda) for a in step_inputs(rd, "fr3", s, B, cuda)] for s in (3, 4)]
    ref = [ctrl.QPIK_step_batch(*x, LINK["fr3"]) for x in ins]
    torch.cuda.synchronize()
    ref = [(o.cpu().numpy(), s.cpu().numpy()) for o, s in ref]
    p = ctrl._pb.params(LINK["fr3"], 1, ctrl.Kp_task_, ctrl.Kv_task_)
    streams = [torch.cuda.Stream(cuda) for _ in range(2)]
    for rep in range(3):
        outs = []
        for x, st in zip(ins, streams):   # enqueue both before either finishes
            outs.append(_batch.qpik_batch(rd.model, p, *x, stream=st.cuda_stream))
        torch.cuda.synchronize()
        for (o, s), (ro, rs) in zip(outs, ref):
            np.testing.assert_array_equal(o.cpu().numpy(), ro)
            np.testing.assert_array_equal(s.cpu().numpy(), rs)


def test_two_host_threads_one_stream(cuda):
    import torch
    rd = make_manipulator("ur5e", cuda)
    ctrl = manipulator.RobotController(0.001, rd, solver_mode="exact")
    B = 20000
    ins = [[torch.as_tensor(a, device=cuda) for a in step_inputs(rd, "ur5e", s, B, cuda)] for s in (5, 6)]
    ref = [ctrl.QPIK_step_batch(*x, LINK["ur5e"]) for x in ins]
    torch.cuda.synchronize()
    ref = [(o.cpu().numpy(), s.cpu().numpy()) for o, s in ref]
    p = ctrl._pb.params(LINK["ur5e"], 1, ctrl.Kp_task_, ctrl.Kv_task_)
    stream = torch.cuda.current_stream(cuda).cuda_stream
    res = [None, None]

    def run(i):
        for _ in range(4):
            res[i] = _batch.qpik_batch(rd.model, p, *ins[i], stream=stream)
    th = [threading.Thread(target=run, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    torch.cuda.synchronize()
    for (o, s), (ro, rs) in zip(res, ref):
        np.testing.assert_array_equal(o.cpu().numpy(), ro)
        np.testing.assert_array_equal(s.cpu().numpy(), rs)

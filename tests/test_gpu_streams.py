"""Boundary contract (include/drc_amd.h): one model driven from two HIP
streams at once, and from two host threads on one stream, returns exactly
what single-stream calls return (per-stream scratch: task records and
work-queue counters are not shared; the internal fork/join streams are the
model's, shared by every caller stream)."""
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


def test_many_streams_bounded_scratch(cuda):
    """A caller cycling through streams: the model keeps at most 8
    per-stream contexts, so device memory stays flat past the eighth stream,
    every call still returns the single-stream result, and
    drc_model_release_stream frees a context at once."""
    import ctypes as C
    import torch
    from dyros_robot_controller_amd import _capi
    rd = make_manipulator("fr3", cuda)
    ctrl = manipulator.RobotController(0.001, rd, solver_mode="exact")
    B = 16384                                   # task-record pool ~10.5 MB per context
    x = [torch.as_tensor(a, device=cuda) for a in step_inputs(rd, "fr3", 9, B, cuda)]
    ro, rs = [t.cpu().numpy() for t in ctrl.QPIK_step_batch(*x, LINK["fr3"])]
    p = ctrl._pb.params(LINK["fr3"], 1, ctrl.Kp_task_, ctrl.Kv_task_)
    out = torch.empty((7, B), dtype=torch.float64, device=cuda)
    st = torch.empty(B, dtype=torch.int32, device=cuda)
    torch.cuda.synchronize()

    def used():
        torch.cuda.synchronize()
        free, total = torch.cuda.mem_get_info(cuda)
        return total - free

    streams, mem = [], []
    for k in range(24):
        s = torch.cuda.Stream(cuda)
        streams.append(s)
        _batch.qpik_batch(rd.model, p, *x, out=out, status=st, stream=s.cuda_stream)
        s.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy(), ro)
        np.testing.assert_array_equal(st.cpu().numpy(), rs)
        mem.append(used())
    # 16 more streams past the 8-context cap: only the HIP stream objects
    # themselves (~1 MB each) may add, not 16 more ~10.5 MB pools
    grown = mem[-1] - mem[7]
    assert grown < 48 * 2 ** 20, (grown, mem)
    before = used()
    for s in streams:
        _capi.check(_capi.lib().drc_model_release_stream(rd.model.handle, C.c_void_p(s.cuda_stream)))
    freed = before - used()
    assert freed >= 6 * 10 * 2 ** 20, (freed, before)   # the 8 live pools (~10.5 MB each) went back

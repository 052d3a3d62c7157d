// Fused task + QP kernel of QPIK / QPIKStep / QPIKCubic for the compiled QP
// shapes (FR3, UR5e, Husky-FR3, XLS-FR3): each wave takes an instance from
// the per-XCD work queue, runs the task stage (task_stage.hpp) and then the
// QP (qp_solver.hpp) on it, and only then takes the next one.  The task
// record never leaves the CU: it is written to and read from an LDS slot past
// both stages' LDS plans (the plans overlay each other; the task data are dead
// once the record is written).  Against the two-kernel pipeline this removes
// the record's HBM round trip and the kernel boundary: a call's makespan is
// the slowest wave's sum over its instances of (task + QP) instead of the
// slowest task plus the slowest QP, which is what bounds small batches.
// Same device functions on the same record values as the two-kernel
// pipeline; the contract with it (tests/test_gpu_fused.py) is in
// drc_set_fusion's comment (include/drc_amd.h).
#include "task_stage.hpp"
#include "qp_solver.hpp"
#include "launch.hpp"

namespace drc_amd {

// Occupancy target of the fused kernel (waves per SIMD)
#ifndef DRC_FUSED_WAVES
#define DRC_FUSED_WAVES 2
#endif
template <class QD>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(DRC_FUSED_WAVES, 8)))
fused_kernel(const DevModel* __restrict__ M0, const KParams kt, const KParams kq, const IO io) {
  extern __shared__ __attribute__((aligned(16))) double S[];
  PH_KSCOPE();
  __shared__ KParams kpl;  // LDS copy of the QP parameters for the out-of-line ADMM blocks
  {
    static_assert(sizeof(KParams) % 8 == 0, "KParams copied as 8-byte words");
    const uint64_t* src = reinterpret_cast<const uint64_t*>(&kq);
    uint64_t* dst = reinterpret_cast<uint64_t*>(&kpl);
    for (int e = lane_id(); e < static_cast<int>(sizeof(KParams) / 8); e += 64) dst[e] = src[e];
    wsync();
  }
  static_assert(QD::gs == 64, "the fused kernel runs one instance per wave");
  const int64_t B = io.B;
  IO iol = io;  // the record lives in LDS: one slot, reused by every instance of the wave
  iol.rec = S + fused_rec_offset(kt, kq);  // (kernel_common.hpp: past the QP plan, in the task plan's dead overlay)
  iol.rec_stride = 0;
  const InstSeq seq(B, kq.xcd_map, io.queue);
  for (int64_t j = seq.first(); j < seq.n; j = seq.next(j)) {
    const int64_t jj = seq.at(j);
    if (jj >= B) continue;
    const int64_t b = io.ordered(jj);
    stage_stamp(io, ST_TASK0, io.b0 + b);
    stage_where(io, ST_WTASK, io.b0 + b);
    task_instance<0>(M0, kt, iol, S, b);
    wsync();
    stage_stamp(io, ST_TASK1, io.b0 + b);
    qp_instance<QD>(M0, kq, kpl, iol, S, b);
  }
}

int launch_fused_kernel(unsigned grid, size_t lds, hipStream_t st, const DevModel* m, const KParams& kt,
                        const KParams& kq, const IO& io) {
  const dim3 g(grid), blk(64);
  if (kq.nx == 23 && kq.ng == 16 && kq.np == 7)  // FR3
    hipLaunchKernelGGL((fused_kernel<Dims<23, 16, 7, true, true, 64>>), g, blk, lds, st, m, kt, kq, io);
  else if (kq.nx == 20 && kq.ng == 14 && kq.np == 6)  // UR5e
    hipLaunchKernelGGL((fused_kernel<Dims<20, 14, 6, true, true, 64>>), g, blk, lds, st, m, kt, kq, io);
  else if (kq.nx == 9 && kq.ng == 16 && kq.np == 9)  // Husky-FR3
    hipLaunchKernelGGL((fused_kernel<Dims<9, 16, 9, true, true, 64>>), g, blk, lds, st, m, kt, kq, io);
  else if (kq.nx == 11 && kq.ng == 16 && kq.np == 11)  // XLS-FR3
    hipLaunchKernelGGL((fused_kernel<Dims<11, 16, 11, true, true, 64>>), g, blk, lds, st, m, kt, kq, io);
  else
    return hipErrorInvalidValue;  // not a compiled shape: the two-kernel pipeline runs it
  return hipGetLastError();
}

#ifdef DRC_PHASE_TIMING
DRC_PHASE_EXPORT(phase_cycles_fused)
#endif

}  // namespace drc_amd

// QP stage of the QP-IK hot path: one wavefront
// per instance assembles the QP of QP_IK.cpp:69-131 (MoMa QP_IK.cpp:59-128)
// from the task record and solves it with the OSQP ADMM of qp_solver.hpp.
// Compile-time shapes for the bundled robots (register Schur ADMM), a
// runtime-sized instantiation for anything else.
#include "kernel_common.hpp"
#include "launch.hpp"
#include "qp_solver.hpp"

namespace drc_amd {


// QP kernel: assembles and solves the QP of each instance from the task
// record written by task_kernel.
// Occupancy target (waves per SIMD): 3 (168 VGPRs) since the ADMM loop keeps
// one register set per lane role (core / auxiliary variable) and fits without
// spills in its iterations; the spills at this budget (a 320-336 B per-lane
// scratch frame for the compiled shapes) sit in the per-instance prologue and
// in the termination check with the certified polish (admm_check, every 8 /
// 2 ADMM iterations in exact mode, OSQP's 25 in reference mode; DESIGN.md
// "Traffic")
#ifndef DRC_QP_WAVES
#define DRC_QP_WAVES 3
#endif
template <class QD>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(DRC_QP_WAVES, 8)))
qp_kernel(const DevModel* __restrict__ M0, const KParams kp, const IO io) {
  extern __shared__ __attribute__((aligned(16))) double S[];
  PH_KSCOPE();
  // LDS copy of the parameters for the out-of-line (rare) ADMM blocks: a
  // reference to the kernel argument itself would be copied to scratch
  __shared__ KParams kpl;
  {
    static_assert(sizeof(KParams) % 8 == 0, "KParams copied as 8-byte words");
    const uint64_t* src = reinterpret_cast<const uint64_t*>(&kp);
    uint64_t* dst = reinterpret_cast<uint64_t*>(&kpl);
    for (int e = lane_id(); e < static_cast<int>(sizeof(KParams) / 8); e += 64) dst[e] = src[e];
    wsync();
  }
  // QD::gs = 32: two instances per wave, each lane group on its own LDS
  // plan (the launch allocates one per group) and its own instance sequence
  using GL = Grp<QD::gs>;
  double* const Sg = S + (GL::upper() ? kp.lds_doubles : 0);
  const int64_t B = io.B;
  // hard_mode 1: the lane stage's hard list (grid stride); 2: every instance
  // except the flagged ones (their records are still being written)
  const bool hl = io.hard_mode == 1;
  const InstSeqG<QD::gs> seq(hl ? int64_t(*io.hard_n) : B, hl ? 0 : kp.xcd_map, hl ? nullptr : io.queue);
  for (int64_t j = seq.first(); j < seq.n; j = seq.next(j)) {
    const int64_t b = hl ? int64_t(io.hard_list[j]) : seq.at(j);
    if (b >= B) continue;
    if (io.hard_mode == 2 && io.hard_flag[b]) continue;
    qp_instance<QD>(M0, kp, kpl, io, Sg, b);
  }
}


bool qp_compiled(int nx, int ng, int np) {
  return (nx == 23 && ng == 16 && np == 7) || (nx == 20 && ng == 14 && np == 6) || (nx == 9 && ng == 16 && np == 9) ||
         (nx == 11 && ng == 16 && np == 11);
}

int qp_waves_per_simd() { return DRC_QP_WAVES; }

int launch_qp_kernel(unsigned grid, size_t lds, hipStream_t st, const DevModel* m, const KParams& kp, const IO& io) {
  const dim3 g(grid), blk(64);
  const size_t lg = lds * (64 / kQpGroup);  // one LDS plan per lane group
  if (kp.nx == 23 && kp.ng == 16 && kp.np == 7)  // FR3
    hipLaunchKernelGGL((qp_kernel<Dims<23, 16, 7, true, true, kQpGroup>>), g, blk, lg, st, m, kp, io);
  else if (kp.nx == 20 && kp.ng == 14 && kp.np == 6)  // UR5e
    hipLaunchKernelGGL((qp_kernel<Dims<20, 14, 6, true, true, kQpGroup>>), g, blk, lg, st, m, kp, io);
  else if (kp.nx == 9 && kp.ng == 16 && kp.np == 9)  // Husky-FR3
    hipLaunchKernelGGL((qp_kernel<Dims<9, 16, 9, true, true, kQpGroup>>), g, blk, lg, st, m, kp, io);
  else if (kp.nx == 11 && kp.ng == 16 && kp.np == 11)  // XLS-FR3
    hipLaunchKernelGGL((qp_kernel<Dims<11, 16, 11, true, true, kQpGroup>>), g, blk, lg, st, m, kp, io);
  else  // any other model: runtime-sized shapes
    hipLaunchKernelGGL((qp_kernel<Dims<0, 0, 0>>), g, blk, lds, st, m, kp, io);
  return hipGetLastError();
}

#ifdef DRC_PHASE_TIMING
DRC_PHASE_EXPORT(phase_cycles_qp)
#endif

}  // namespace drc_amd

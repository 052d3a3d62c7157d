// Host-side launchers of the kernel translation units (task_kernel.hip,
// qp_kernel.hip, qpid_kernel.hip), called by the C-ABI in api.cpp.  Each
// returns the hipError_t of its launch (0 = hipSuccess).
#pragma once

#include <hip/hip_runtime.h>

#include "kernel_common.hpp"

namespace drc_amd {

// task_kernel<problem>: 0 QPIK stage, 1 QPID stage, 2 closed-form CLIK / OSF
int launch_task_kernel(int problem, unsigned grid, size_t lds, hipStream_t st, const DevModel* m, const KParams& kp,
                       const IO& io);
// register-budget waves per SIMD of the task build launch_task_kernel picks
// for a plan of `lds` bytes per wave, and of the QP kernel
int task_waves_per_simd(int problem, size_t lds);
int qp_waves_per_simd();
// lane-per-instance task stage (nv = 6 or 7)
int launch_lane_task_kernel(int nv, unsigned grid, hipStream_t st, const DevModel* m, const KParams& kp,
                            const IO& io);
// QPIK shapes with a compile-time qp_kernel instantiation (register Schur ADMM)
bool qp_compiled(int nx, int ng, int np);
// qp_kernel for kp's shape; lds = one lane group's plan
int launch_qp_kernel(unsigned grid, size_t lds, hipStream_t st, const DevModel* m, const KParams& kp, const IO& io);
int launch_qpid_kernel(unsigned grid, size_t lds, hipStream_t st, const DevModel* m, const KParams& kp, const IO& io);
// fused task + QP kernel (compiled QPIK shapes; hipErrorInvalidValue otherwise);
// lds = both plans' maximum plus the record slot
int launch_fused_kernel(unsigned grid, size_t lds, hipStream_t st, const DevModel* m, const KParams& kt,
                        const KParams& kq, const IO& io);

// queue order of one sub-batch (order_kernel.hip): penetration-prone
// instances first (*hot_n zeroed; hot_list [B], hot_flag [B] scratch), then the
// others in index order, into order[b0 .. b0 + B)
int launch_order_kernel(int64_t B, hipStream_t st, const DevModel* m, const IO& io, int* hot_n, int32_t* hot_list,
                        uint8_t* hot_flag, int32_t* order);

#ifdef DRC_PHASE_TIMING
// diagnostic build: add each unit's phase slots to out[64]
int phase_cycles_task(unsigned long long* out, int reset);
int phase_cycles_qp(unsigned long long* out, int reset);
int phase_cycles_qpid(unsigned long long* out, int reset);
int phase_cycles_fused(unsigned long long* out, int reset);
#endif

}  // namespace drc_amd

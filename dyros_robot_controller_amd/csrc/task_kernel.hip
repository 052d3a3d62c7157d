// Task-space stage of the QP-IK hot path: one wavefront per robot instance
// (task_kernel), and the lane-per-instance variant (lane_task.hpp).
//   FK / LWA frame Jacobian        robot_data.cpp:101-107,392-402
//   task error (+ cubic profile)   math_type_define.h:633-687, robot_controller.cpp:292-317
//   manipulability + gradient      robot_data.cpp:519-553 (MoMa :439-475)
//   min self-distance + gradient   robot_data.cpp:424-494 (hpp-fcl GJK/EPA semantics)
//   QPID stage data, CLIK / OSF    robot_data.cpp:109,476-512, robot_controller.cpp:150-260
// The stage writes one task record per instance that qp_kernel / qpid_kernel
// read (or the stage outputs of drc_qpik_stages_batch).
#include "task_stage.hpp"
#include "launch.hpp"

#include <cstdlib>

namespace drc_amd {

// Occupancy target of the task kernel (waves per SIMD): the lane-serial
// narrow phase and task-velocity code would otherwise take all 512 registers.
#ifndef DRC_TASK_WAVES
#define DRC_TASK_WAVES 2
#endif
// PROBLEM 0: QPIK stage data; 1: also the QPID extras (a separate
// instantiation, so the QPIK kernel carries no call frame for them); 2: CLIK / OSF
// WAVES: the register budget's occupancy target; the QPIK stage also has a
// three-wave build (168 VGPRs, more spills) for models whose LDS plan lets a
// CU hold more than the 8 waves the two-wave build can (FR3, UR5e); where the
// plan allows only 8 it loses 1.6-3 % to the spills (profiles/r04j_ab_lds.jsonl)
template <int PROBLEM, int WAVES = DRC_TASK_WAVES>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WAVES, 8)))
task_kernel(const DevModel* __restrict__ M0, const KParams kp, const IO io) {
  extern __shared__ __attribute__((aligned(16))) double S[];
  PH_KSCOPE();
  const int64_t B = io.B;
  // hard mode: the instances the lane-per-instance stage left (grid stride)
  const bool hard_mode = io.hard_mode != 0;
  const InstSeq seq(hard_mode ? int64_t(*io.hard_n) : B, hard_mode ? 0 : kp.xcd_map, hard_mode ? nullptr : io.queue);
  for (int64_t j = seq.first(); j < seq.n; j = seq.next(j)) {
    const int64_t jj = hard_mode ? int64_t(io.hard_list[j]) : seq.at(j);
    if (jj >= B) continue;
    const int64_t b = hard_mode ? jj : io.ordered(jj);
    if (PROBLEM == 0) stage_stamp(io, ST_TASK0, io.b0 + b);
    if (PROBLEM == 0) stage_where(io, ST_WTASK, io.b0 + b);
    task_instance<PROBLEM>(M0, kp, io, S, b);
    if (PROBLEM == 0) stage_stamp(io, ST_TASK1, io.b0 + b);
  }
}


#include "lane_task.hpp"  // lane-per-instance stage (inside namespace drc_amd)

int task_waves_per_simd(int problem, size_t lds) {
  // the two-wave build holds 8 waves per CU; the three-wave build pays where the
  // plan lets a CU hold 9 or more (<= 160 KB / 9: FR3 17.1 KB +0.9 %, UR5e 14.0 KB
  // +11 % with the narrowed plan, profiles/r04l_envab_w3.jsonl, r04k_ab_w3_ldsnarrow.jsonl)
  // (DRC_TASK_W3=0 / 1 forces the choice: A/B experiments)
  static const int w3_env = [] {
    const char* e = std::getenv("DRC_TASK_W3");
    return e ? std::atoi(e) : -1;
  }();
  const bool w3 = w3_env >= 0 ? w3_env != 0 : lds * 9 <= 160 * 1024;
  return problem == 0 && w3 ? 3 : DRC_TASK_WAVES;
}

int launch_task_kernel(int problem, unsigned grid, size_t lds, hipStream_t st, const DevModel* m, const KParams& kp,
                       const IO& io) {
  const bool w3 = task_waves_per_simd(problem, lds) == 3 && DRC_TASK_WAVES != 3;
  if (problem == 0 && w3)
    hipLaunchKernelGGL((task_kernel<0, 3>), dim3(grid), dim3(64), lds, st, m, kp, io);
  else if (problem == 0)
    hipLaunchKernelGGL(task_kernel<0>, dim3(grid), dim3(64), lds, st, m, kp, io);
  else if (problem == 1)
    hipLaunchKernelGGL(task_kernel<1>, dim3(grid), dim3(64), lds, st, m, kp, io);
  else
    hipLaunchKernelGGL(task_kernel<2>, dim3(grid), dim3(64), lds, st, m, kp, io);
  return hipGetLastError();
}

int launch_lane_task_kernel(int nv, unsigned grid, hipStream_t st, const DevModel* m, const KParams& kp,
                            const IO& io) {
  if (nv == 7)
    hipLaunchKernelGGL(lane_task_kernel<7>, dim3(grid), dim3(64), 0, st, m, kp, io);
  else
    hipLaunchKernelGGL(lane_task_kernel<6>, dim3(grid), dim3(64), 0, st, m, kp, io);
  return hipGetLastError();
}

#ifdef DRC_PHASE_TIMING
DRC_PHASE_EXPORT(phase_cycles_task)
#endif

}  // namespace drc_amd

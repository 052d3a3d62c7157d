// Batched joint-space dynamics launcher (dynamics.hip); see include/drc_amd.h
// drc_dynamics_batch for the contract.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "model.hpp"

namespace drc_amd {

// LDS bytes per 256-thread block (16 robots) for an n-joint model with na
// actuated dof; act selects the actuated (S^T M S) outputs.
int dyn_lds_bytes(int n, int na, bool act, bool fallback);

// list: device int32 buffer of 1 + B entries (fallback queue) when Minv != nullptr.
// Returns 0 on success, 1 for a bad size, 2 for a HIP launch error.
int launch_dynamics(const DevModel* d_model, const DevModel& host, bool act, int64_t B, const double* q,
                    const double* qd, double* M, double* Minv, double* g, double* nle, double* c, int* list,
                    hipStream_t st);

// Joint torque step for the controlled block (all joints of a manipulator, the
// arm of a mobile manipulator): tau = M_b acc + g_b with acc = qddot_target or
// kp (q_target - q_b) + kv (qdot_target - qdot_b); q_target == nullptr means
// q_b + dt qdot_target.  kp, kv: host arrays of the block size.
int launch_torque_step(const DevModel* d_model, const DevModel& host, int64_t B, const double* q, const double* qd,
                       const double* q_target, const double* qdot_target, const double* qddot_target, double dt,
                       const double* kp, const double* kv, double* tau, hipStream_t st);

}  // namespace drc_amd

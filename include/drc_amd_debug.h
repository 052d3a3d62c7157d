/*
 * drc_amd_debug.h -- diagnostic entries of libdrc_amd.so (no reference
 * counterpart).  Not part of the drop-in boundary (drc_amd.h): they serve the
 * benchmark (bench.py), the profiling tools (tools/) and the parity tests,
 * and expose kernel timing, per-instance stage stamps, LDS / occupancy plans
 * and the lane-per-instance task-stage switch.
 */
#ifndef DRC_AMD_DEBUG_H
#define DRC_AMD_DEBUG_H

#include "drc_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Diagnostics (no reference counterpart): when enabled, drc_qpik_batch
 * records HIP events on its stream around the task and QP kernels;
 * drc_debug_kernel_times waits for them and returns the summed durations
 * (ms) and the number of timed calls since the last query. */
int drc_debug_kernel_timing(drc_model* model, int enable);
/* Host-side timeline of the synchronous entries (drc_qpik_host and the other
 * *_host calls): while enabled, each call appends five steady-clock ns stamps
 * -- entry, inputs packed into the pinned buffer, copy in + launches + copy
 * back enqueued, completion seen, exit.  Returns up to `cap` rows of the calls
 * since the last query in out[5 * cap] (n = rows recorded), clears them and
 * sets the enable state.  Diagnostic (bench.py latency_b1); no reference
 * counterpart. */
int drc_debug_host_timeline(drc_model* model, int enable, int64_t* out, int64_t cap, int64_t* n);
/* Per-wave LDS of this model's kernels (bytes): task kernel, QP kernel and the
 * fused kernel (0 for QPID), problem 0 = QPIK, 1 = QPID.  Diagnostic (DESIGN.md
 * "Occupancy"); no reference counterpart. */
int drc_debug_lds_plan(drc_model* model, const drc_qpik_params* params, int problem, int* task_bytes, int* qp_bytes,
                       int* fused_bytes);
/* wall_ms: summed caller-stream time of the timed calls (fork to join; a call
 * of one sub-batch: its first kernel's start to its last kernel's end);
 * task_ms / qp_ms: summed durations of the task / QP kernels of every
 * sub-batch (they overlap in time when a call runs several sub-batches). */
int drc_debug_kernel_times(drc_model* model, double* wall_ms, double* task_ms, double* qp_ms, int* calls);
/* Register-budget occupancy (waves per SIMD) of the QPIK task-kernel build a
 * call with these params launches (two- or three-wave build, chosen from its
 * LDS plan) and of the QP kernel.  Diagnostic (bench.py latency roof). */
int drc_debug_waves(drc_model* model, const drc_qpik_params* params, int* task_waves, int* qp_waves);

/* drc_qpik_host that also returns the kernels' per-instance stage stamps,
 * stamps[8][B]: s_memrealtime ticks (100 MHz) at task start / end, QP start /
 * assembled / solved / stored, then where the task and the QP stage ran
 * (workgroup << 32 | CU id (XCC, SE, CU) << 2 | SIMD).  Diagnostic (the
 * small-batch makespan study, tools/stamp_study.py); no reference counterpart. */
int drc_debug_qpik_stamps(drc_model* model, const drc_qpik_params* params, int64_t B, const double* q,
                          const double* qdot, const double* x_target, const double* xdot_target,
                          const double* x_init, const double* xdot_init, double* qdot_out, int32_t* status,
                          int32_t* iters, uint64_t* stamps);

/* Task stage of drc_qpik_batch / drc_qpik_stages_batch.  0: the
 * wave-per-instance kernel on every instance (default).  1: the lane-per-instance stage
 * for the compiled joint counts (6, 7); the instances it hands back (EPA, COD
 * pseudo-inverse, many GJK candidates) run the wave-per-instance kernel on a
 * side stream while the QP of the others runs, then their QP.  2: as 1, but
 * the hand-backs run before one QP pass.  3: the lane stage for
 * drc_qpik_stages_batch only.  Default 0.  Results agree to rounding (GJK
 * witness points to their ~1e-6 convergence tolerance); used by the parity
 * tests and benchmarks. */
int drc_debug_lane_stage(drc_model* model, int enable);

/* Scheduling order of the instances for calls of exactly n instances
 * (drc_qpik_batch and the host forms; the task / fused kernels take the
 * instance at queue position j of a sub-batch [b0, b1) as order[b0 + j], so
 * `order` must map each sub-batch range onto itself -- any permutation when the
 * call runs as one sub-batch).  Host array, copied; NULL or n <= 0 clears it.
 * Results do not depend on it (instances are independent); it moves only when
 * each instance starts.  Diagnostic (the small-batch scheduling study,
 * tools/stamp_study.py --order); no reference counterpart. */
int drc_debug_instance_order(drc_model* model, const int32_t* order, int64_t n);

#ifdef __cplusplus
}
#endif
#endif /* DRC_AMD_DEBUG_H */

// Diagnostic phase instrumentation (tools/phase_timing.py, the
// libdrc_amd_timing.so build of tools/build_variants.sh).  With
// -DDRC_PHASE_TIMING the kernels accumulate s_memtime cycle stamps per phase
// into a 64-slot device array of their translation unit (drc_debug_phase_cycles
// sums the units); without it every macro below expands to nothing, so the
// product kernels carry no instrumentation.
#pragma once

#ifdef DRC_PHASE_TIMING
namespace drc_amd {
static __device__ unsigned long long g_phase_cycles[64];
// per-wave accumulators in LDS (lane 0 adds; the kernel adds them to the
// device array once, at its end): a global atomic per phase and call from
// every wave queued at the L2 and inflated the very cycles being measured
static __shared__ unsigned long long g_ph_lds[64];
}
#define PH_KINIT()                         \
  do {                                     \
    g_ph_lds[__lane_id()] = 0ull;          \
    __builtin_amdgcn_wave_barrier();       \
  } while (0)
#define PH_KFLUSH()                                                   \
  do {                                                                \
    __builtin_amdgcn_wave_barrier();                                  \
    const unsigned long long v_ = g_ph_lds[__lane_id()];              \
    if (v_) atomicAdd(&g_phase_cycles[__lane_id()], v_);              \
  } while (0)
// PH_KSCOPE(): zero the wave's slots at kernel entry, add them to the device
// array at kernel exit
namespace drc_amd {
struct PhKernelScope {
  __device__ PhKernelScope() { PH_KINIT(); }
  __device__ ~PhKernelScope() { PH_KFLUSH(); }
};
}
#define PH_KSCOPE() drc_amd::PhKernelScope ph_kscope_
// whole statements that exist only in the timing build
#define PH_ONLY(...) __VA_ARGS__
// a named stamp, and its elapsed cycles added to a slot by lane 0
#define PH_STAMP(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define PH_ADD(slot, val)                                                                        \
  do {                                                                                           \
    if (__lane_id() == 0) g_ph_lds[(slot)] += (unsigned long long)(val);                        \
  } while (0)
#define PH_SINCE(slot, v) PH_ADD(slot, __builtin_amdgcn_s_memtime() - (v))
// a private accumulator and an addition of the cycles since a stamp
#define PH_ACC(v) unsigned long long v = 0
#define PH_ACC_SINCE(acc, v) ((acc) += __builtin_amdgcn_s_memtime() - (v))
// per-kernel phase accumulators: PH(k) closes phase k, PH_FLUSH adds the
// 16 accumulators to slots base .. base + 15
#define PH_DECL unsigned long long ph_prev = __builtin_amdgcn_s_memtime(), ph_acc[16] = {0};
#define PH(k)                                              \
  do {                                                     \
    unsigned long long t_ = __builtin_amdgcn_s_memtime();  \
    ph_acc[k] += t_ - ph_prev;                             \
    ph_prev = t_;                                          \
  } while (0)
#define PH_FLUSH(base)                                                                     \
  do {                                                                                     \
    if (__lane_id() == 0)                                                                  \
      for (int k_ = 0; k_ < 16; ++k_) g_ph_lds[(base) + k_] += ph_acc[k_];                 \
  } while (0)
// direct accumulation (functions without the kernel's stamp locals)
#define PHG_DECL unsigned long long phg_t = __builtin_amdgcn_s_memtime();
#define PHG(slot)                                                                 \
  do {                                                                            \
    unsigned long long t_ = __builtin_amdgcn_s_memtime();                         \
    if (__lane_id() == 0) g_ph_lds[(slot)] += t_ - phg_t;                        \
    phg_t = t_;                                                                   \
  } while (0)
#define PHG_RESET() \
  do {              \
    phg_t = __builtin_amdgcn_s_memtime(); \
  } while (0)
// ADMM termination checks (admm_check): stamp, elapsed, count
#define CK_T0() unsigned long long ck_t = __builtin_amdgcn_s_memtime()
#define CK_T(slot)                                                      \
  do {                                                                  \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();         \
    if (__lane_id() == 0) g_ph_lds[(slot)] += t_ - ck_t;                \
    ck_t = t_;                                                          \
  } while (0)
#define CK_N(slot) PH_ADD(slot, 1)
// host: add this unit's slots to out[64] (and zero them when reset)
#define DRC_PHASE_EXPORT(fn)                                                                       \
  int fn(unsigned long long* out, int reset) {                                                     \
    unsigned long long v[64];                                                                      \
    if (hipMemcpyFromSymbol(v, HIP_SYMBOL(g_phase_cycles), sizeof(v)) != hipSuccess) return 1;     \
    for (int i = 0; i < 64; ++i) out[i] += v[i];                                                   \
    if (reset) {                                                                                   \
      for (int i = 0; i < 64; ++i) v[i] = 0;                                                       \
      if (hipMemcpyToSymbol(HIP_SYMBOL(g_phase_cycles), v, sizeof(v)) != hipSuccess) return 1;     \
    }                                                                                              \
    return 0;                                                                                      \
  }
#else
#define PH_ONLY(...)
#define PH_KINIT() do {} while (0)
#define PH_KFLUSH() do {} while (0)
#define PH_KSCOPE() do {} while (0)
#define PH_STAMP(v) do {} while (0)
#define PH_ADD(slot, val) do {} while (0)
#define PH_SINCE(slot, v) do {} while (0)
#define PH_ACC(v) do {} while (0)
#define PH_ACC_SINCE(acc, v) do {} while (0)
#define PH_DECL
#define PH(k) do {} while (0)
#define PH_FLUSH(base) do {} while (0)
#define PHG_DECL
#define PHG(slot) do {} while (0)
#define PHG_RESET() do {} while (0)
#define CK_T0() do {} while (0)
#define CK_T(slot) do {} while (0)
#define CK_N(slot) do {} while (0)
#endif

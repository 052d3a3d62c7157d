// Device-side building blocks of the QP-IK kernel (gfx950, wave64).
//
// One 64-lane wavefront owns one robot instance; the workgroup is exactly
// one wave, so __syncthreads() is a wave-local LDS fence.  Lanes take the
// natural parallel axis of each phase: joints (FK / Jacobian columns),
// (k, c) pairs (dJ/dq for the manipulability gradient), collision pairs
// (narrow phase), QP variables / constraint rows (ADMM, polish).
#pragma once
#include <utility>

#include <hip/hip_runtime.h>

#include <cstdint>

#include "model.hpp"

namespace drc_amd {

#define DRC_HD __host__ __device__

constexpr double kInf = 1e30;  // OSQP_INFTY (QP_base.h:82-91)
constexpr double kMinScaling = 1e-4, kMaxScaling = 1e4;
constexpr double kRhoMin = 1e-6, kRhoMax = 1e6, kRhoTol = 1e-4, kRhoEqRatio = 1e3;
constexpr double kDivTol = 1e-30;

// ------------------------------------------------------------ wave helpers
// opaque per call: lane-derived values (offsets, masks, per-lane pointers) are
// recomputed where used instead of being hoisted out of the persistent
// instance loops and spilled to scratch
__device__ __forceinline__ int lane_id() {
  int l = threadIdx.x & 63;
  asm volatile("" : "+v"(l));
  return l;
}
// Lane exchange point of the one-wave workgroups (task / QP / fused / QPID
// kernels), whose lanes talk through LDS only.  A wavefront-scope release /
// acquire fence pair around the wave barrier: the compiler's memory model then
// emits whatever waits one lane's store -> another lane's load needs for the
// address space each access compiles to (ds_* or, through a generic pointer,
// flat_*), instead of this code relying on the issue order of LDS instructions.
// No vmcnt / lgkmcnt drain of unrelated accesses and no s_barrier
// (__syncthreads waited for every outstanding global and scratch access at each
// exchange).  -DDRC_BLOCK_SYNC restores __syncthreads.
#if defined(DRC_WSYNC_ASM)  // A/B variant: the r04 compiler-barrier form
__device__ __forceinline__ void wsync() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}
#elif !defined(DRC_BLOCK_SYNC)
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
#else
__device__ __forceinline__ void wsync() { __syncthreads(); }
#endif

// Wave reductions: DPP within each row of 16 lanes (quad swaps, half-row
// and row mirrors: every lane of a row ends with the row's value), then the
// four row values through v_readlane.  No LDS crossbar (ds_bpermute) round
// trips; called with the whole wave active.
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(v, v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = dpp_i<CTRL>(static_cast<int>(b)), hi = dpp_i<CTRL>(static_cast<int>(b >> 32));
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double rd_lane(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane(static_cast<int>(b), lane);
  const int hi = __builtin_amdgcn_readlane(static_cast<int>(b >> 32), lane);
  return __hiloint2double(hi, lo);
}
constexpr int kDppQuad1032 = 0xB1, kDppQuad2301 = 0x4E, kDppHalfMirror = 0x141, kDppMirror = 0x140;
__device__ __forceinline__ double wave_max(double v) {
  v = fmax(v, dpp_d<kDppQuad1032>(v));
  v = fmax(v, dpp_d<kDppQuad2301>(v));
  v = fmax(v, dpp_d<kDppHalfMirror>(v));
  v = fmax(v, dpp_d<kDppMirror>(v));
  return fmax(fmax(rd_lane(v, 0), rd_lane(v, 16)), fmax(rd_lane(v, 32), rd_lane(v, 48)));
}
__device__ __forceinline__ double wave_sum(double v) {
  v += dpp_d<kDppQuad1032>(v);
  v += dpp_d<kDppQuad2301>(v);
  v += dpp_d<kDppHalfMirror>(v);
  v += dpp_d<kDppMirror>(v);
  return (rd_lane(v, 0) + rd_lane(v, 16)) + (rd_lane(v, 32) + rd_lane(v, 48));
}
__device__ __forceinline__ int wave_min_int(int v) {
  v = min(v, dpp_i<kDppQuad1032>(v));
  v = min(v, dpp_i<kDppQuad2301>(v));
  v = min(v, dpp_i<kDppHalfMirror>(v));
  v = min(v, dpp_i<kDppMirror>(v));
  return min(min(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
             min(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}
// argmin with ties broken toward the smaller index (reference: first strict
// minimum in pair order, robot_data.cpp:434-442); the (value, index) order
// is total, so the result does not depend on the reduction tree
__device__ __forceinline__ void argmin_step(double& v, int& idx, double ov, int oi) {
  if (ov < v || (ov == v && oi < idx)) {
    v = ov;
    idx = oi;
  }
}
template <int CTRL>
__device__ __forceinline__ void argmin_dpp(double& v, int& idx) {
  const double ov = dpp_d<CTRL>(v);
  const int oi = dpp_i<CTRL>(idx);
  argmin_step(v, idx, ov, oi);
}
__device__ __forceinline__ void wave_argmin(double& v, int& idx) {
  argmin_dpp<kDppQuad1032>(v, idx);
  argmin_dpp<kDppQuad2301>(v, idx);
  argmin_dpp<kDppHalfMirror>(v, idx);
  argmin_dpp<kDppMirror>(v, idx);
  double bv = rd_lane(v, 0);
  int bi = __builtin_amdgcn_readlane(idx, 0);
#pragma unroll
  for (int r = 16; r < 64; r += 16) {
    const double ov = rd_lane(v, r);
    const int oi = __builtin_amdgcn_readlane(idx, r);
    argmin_step(bv, bi, ov, oi);
  }
  v = bv;
  idx = bi;
}

// Lane groups: the QPIK QP kernel packs two instances per wave (32 lanes
// each, GS = 32); GS = 64 is the whole wave (the helpers above).  Reductions
// stay inside a group: DPP steps never leave a row of 16 lanes, and the
// row values of the caller's group are combined through v_readlane (which
// reads the other group's lanes too, whatever their exec state; only the own
// group's are used).  bcast takes a lane index uniform across the wave.
template <int GS>
struct Grp {
  static_assert(GS == 64 || GS == 32, "lane groups of 32 or 64");
  static constexpr int size = GS;
  static __device__ __forceinline__ int lane() {  // opaque per call, as lane_id()
    int l = threadIdx.x & (GS - 1);
    asm volatile("" : "+v"(l));
    return l;
  }
  static __device__ __forceinline__ bool upper() { return GS == 32 && (threadIdx.x & 32); }
  static __device__ __forceinline__ unsigned long long ballot(bool p) {
    const unsigned long long m = __ballot(p);
    if constexpr (GS == 64) return m;
    else return upper() ? (m >> 32) : (m & 0xffffffffull);
  }
  static __device__ __forceinline__ bool all(bool p) {
    if constexpr (GS == 64) return __all(p);
    else return ballot(!p) == 0;
  }
  static __device__ __forceinline__ bool any(bool p) {
    if constexpr (GS == 64) return __any(p);
    else return ballot(p) != 0;
  }
  static __device__ __forceinline__ double bcast(double v, int k) {
    if constexpr (GS == 64) return rd_lane(v, k);
    else {  // lane k of the own group through the LDS crossbar (no LDS memory)
      const int addr = static_cast<int>(((threadIdx.x & 32) + k) << 2);
      const long long b = __double_as_longlong(v);
      const int lo = __builtin_amdgcn_ds_bpermute(addr, static_cast<int>(b));
      const int hi = __builtin_amdgcn_ds_bpermute(addr, static_cast<int>(b >> 32));
      return __hiloint2double(hi, lo);
    }
  }
  // lane K of the own group, K a compile-time constant.  GS = 32: DPP
  // row_newbcast puts lane K % 16 of every 16-lane row in the whole row, and
  // v_permlane16_swap of that value with itself yields, in every row of a row
  // pair, the even row's value (first result) and the odd row's (second):
  // four VALU ops per double, no LDS crossbar round trip
  template <int K>
  static __device__ __forceinline__ double bcastc(double v) {
    if constexpr (GS == 64) {
      return rd_lane(v, K);
    } else {
      static_assert(K >= 0 && K < 32, "lane within the group");
      const long long b = __double_as_longlong(v);
      const int lo = __builtin_amdgcn_update_dpp(0, static_cast<int>(b), 0x150 + (K & 15), 0xF, 0xF, false);
      const int hi = __builtin_amdgcn_update_dpp(0, static_cast<int>(b >> 32), 0x150 + (K & 15), 0xF, 0xF, false);
      const auto pl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
      const auto ph = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
      return K < 16 ? __hiloint2double(ph[0], pl[0]) : __hiloint2double(ph[1], pl[1]);
    }
  }
  template <class T>
  static __device__ __forceinline__ T shfl(T v, int k) { return __shfl(v, k, GS); }
  static __device__ __forceinline__ double max(double v) {
    if constexpr (GS == 64) return wave_max(v);
    else {
      v = fmax(v, dpp_d<kDppQuad1032>(v));
      v = fmax(v, dpp_d<kDppQuad2301>(v));
      v = fmax(v, dpp_d<kDppHalfMirror>(v));
      v = fmax(v, dpp_d<kDppMirror>(v));
      const double a = fmax(rd_lane(v, 0), rd_lane(v, 16)), b = fmax(rd_lane(v, 32), rd_lane(v, 48));
      return upper() ? b : a;
    }
  }
  static __device__ __forceinline__ double sum(double v) {
    if constexpr (GS == 64) return wave_sum(v);
    else {
      v += dpp_d<kDppQuad1032>(v);
      v += dpp_d<kDppQuad2301>(v);
      v += dpp_d<kDppHalfMirror>(v);
      v += dpp_d<kDppMirror>(v);
      const double a = rd_lane(v, 0) + rd_lane(v, 16), b = rd_lane(v, 32) + rd_lane(v, 48);
      return upper() ? b : a;
    }
  }
  static __device__ __forceinline__ void argmin(double& v, int& idx) {
    if constexpr (GS == 64) {
      wave_argmin(v, idx);
    } else {
      argmin_dpp<kDppQuad1032>(v, idx);
      argmin_dpp<kDppQuad2301>(v, idx);
      argmin_dpp<kDppHalfMirror>(v, idx);
      argmin_dpp<kDppMirror>(v, idx);
      const int r0 = upper() ? 32 : 0;  // lane index from a VGPR: read both groups' rows, select
      double av = rd_lane(v, 0), bv = rd_lane(v, 32);
      int ai = __builtin_amdgcn_readlane(idx, 0), bi = __builtin_amdgcn_readlane(idx, 32);
      argmin_step(av, ai, rd_lane(v, 16), __builtin_amdgcn_readlane(idx, 16));
      argmin_step(bv, bi, rd_lane(v, 48), __builtin_amdgcn_readlane(idx, 48));
      v = r0 ? bv : av;
      idx = r0 ? bi : ai;
    }
  }
  static __device__ __forceinline__ void argmax(double& v, int& idx) {
    double nv = -v;
    argmin(nv, idx);
    v = -nv;
  }
};

// compile-time loop: f(std::integral_constant<int, I>) for I = 0 .. N-1
template <class F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// ------------------------------------------------------------ 3-vectors
struct V3 {
  double x, y, z;
};
DRC_HD __forceinline__ V3 v3(double x, double y, double z) { return V3{x, y, z}; }
DRC_HD __forceinline__ V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
DRC_HD __forceinline__ V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
DRC_HD __forceinline__ V3 operator*(double s, V3 a) { return v3(s * a.x, s * a.y, s * a.z); }
DRC_HD __forceinline__ double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
DRC_HD __forceinline__ V3 cross(V3 a, V3 b) {
  return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
DRC_HD __forceinline__ V3 ld3(const double* p) { return v3(p[0], p[1], p[2]); }
DRC_HD __forceinline__ void st3(double* p, V3 v) {
  p[0] = v.x;
  p[1] = v.y;
  p[2] = v.z;
}
// T = [R row-major | p]
template <class PT>
DRC_HD __forceinline__ V3 rot(PT T, V3 v) {
  return v3(T[0] * v.x + T[1] * v.y + T[2] * v.z, T[3] * v.x + T[4] * v.y + T[5] * v.z,
            T[6] * v.x + T[7] * v.y + T[8] * v.z);
}
template <class PT>
DRC_HD __forceinline__ V3 rotT(PT T, V3 v) {
  return v3(T[0] * v.x + T[3] * v.y + T[6] * v.z, T[1] * v.x + T[4] * v.y + T[7] * v.z,
            T[2] * v.x + T[5] * v.y + T[8] * v.z);
}
template <class PT>
DRC_HD __forceinline__ V3 xform(PT T, V3 v) { return rot(T, v) + v3(T[9], T[10], T[11]); }
// c = a * b (12-vector transforms)
DRC_HD __forceinline__ void tmul(const double* a, const double* b, double* c) {
  double r[12];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int j = 0; j < 3; ++j) r[3 * i + j] = a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j] + a[3 * i + 2] * b[6 + j];
    r[9 + i] = a[3 * i] * b[9] + a[3 * i + 1] * b[10] + a[3 * i + 2] * b[11] + a[9 + i];
  }
#pragma unroll
  for (int i = 0; i < 12; ++i) c[i] = r[i];
}

// ------------------------------------------------------------ narrow phase
// A primitive and its pose.  The pose pointer's type is a parameter: the
// wave task stage's poses live in LDS and its shapes carry an LDS-typed
// pointer (ShapeL), so every support evaluation of GJK / EPA / the witness
// refinement reads them with ds_read; a generic pointer (Shape: host code,
// the lane stage's private poses, the tests) would make each of those reads
// a flat access
template <class PT>
struct ShapeT {
  int type;
  PT T;              // pose (3x3 row-major rotation, then the origin)
  double p0, p1, p2; // parameters
};
using Shape = ShapeT<const double*>;
#ifdef __HIP_DEVICE_COMPILE__
typedef __attribute__((address_space(3))) const double lds_pose;
#else
typedef const double lds_pose;
#endif
using ShapeL = ShapeT<lds_pose*>;

template <class SH>
DRC_HD __forceinline__ V3 support(const SH& s, V3 d) {
  if (s.type == kSphere) return v3(s.T[9], s.T[10], s.T[11]);
  V3 dl = rotT(s.T, d), loc;
  if (s.type == kCylinder) {
    const double rho = sqrt(dl.x * dl.x + dl.y * dl.y), f = rho > 0 ? s.p0 / rho : 0.0;
    loc.x = f * dl.x;
    loc.y = f * dl.y;
    loc.z = dl.z > 0 ? s.p1 : -s.p1;
  } else {
    loc.x = dl.x > 0 ? s.p0 : -s.p0;
    loc.y = dl.y > 0 ? s.p1 : -s.p1;
    loc.z = dl.z > 0 ? s.p2 : -s.p2;
  }
  return xform(s.T, loc);
}

struct SV {
  V3 w, a, b;
};
template <class SH>
DRC_HD __forceinline__ SV sup_md(const SH& A, const SH& B, V3 d) {
  SV o;
  o.a = support(A, d);
  o.b = support(B, -1.0 * d);
  o.w = o.a - o.b;
  return o;
}

// GJK simplex vertex: support point w = a - b of the Minkowski difference and
// the matching support point a on A (b = a - w).
struct SV2 {
  V3 w, a;
};

// Closest point of conv(S[0..N)) to the origin: exhaustive sub-simplex
// search, same visiting order (masks from 2^N-1 down to 1) and tolerances as
// oracle/drc_oracle.c:closest_simplex.  The mask loop is expanded at compile
// time (template recursion), so the simplex is only ever indexed with
// constants and stays in registers.
constexpr int cs_popc(int m) { return m == 0 ? 0 : (m & 1) + cs_popc(m >> 1); }
constexpr int cs_bit(int m, int k) {  // index of the k-th set bit of m
  return (m & 1) ? (k == 0 ? 0 : 1 + cs_bit(m >> 1, k - 1)) : 1 + cs_bit(m >> 1, k);
}
struct CsBest {
  double best, l[4];
  int mask;
  V3 v;
};
template <int MASK>
DRC_HD __forceinline__ void cs_try(const SV2 (&S)[4], CsBest& B) {
  constexpr int k = cs_popc(MASK);
  constexpr int i0 = cs_bit(MASK, 0), i1 = k > 1 ? cs_bit(MASK, 1) : 0, i2 = k > 2 ? cs_bit(MASK, 2) : 0,
                i3 = k > 3 ? cs_bit(MASK, 3) : 0;
  double l0 = 1, l1 = 0, l2 = 0, l3 = 0;
  const V3 w0 = S[i0].w;
  if (k == 2) {
    const V3 D0 = S[i1].w - w0;
    const double G0 = dot(D0, D0), r0 = -dot(D0, w0);
    if (!(G0 > 0)) return;
    l1 = r0 / G0;
    l0 = 1 - l1;
    if (l0 < -1e-14 || l1 < -1e-14) return;
  } else if (k == 3) {
    const V3 D0 = S[i1].w - w0, D1 = S[i2].w - w0;
    const double G0 = dot(D0, D0), G1 = dot(D0, D1), G3 = dot(D1, D0), G4 = dot(D1, D1);
    const double r0 = -dot(D0, w0), r1 = -dot(D1, w0);
    const double det = G0 * G4 - G1 * G3;
    if (fabs(det) < 1e-300) return;
    const double id = 1.0 / det;
    l1 = (r0 * G4 - G1 * r1) * id;
    l2 = (G0 * r1 - r0 * G3) * id;
    l0 = 1 - (l1 + l2);
    if (l0 < -1e-14 || l1 < -1e-14 || l2 < -1e-14) return;
  } else if (k == 4) {
    const V3 D0 = S[i1].w - w0, D1 = S[i2].w - w0, D2 = S[i3].w - w0;
    const double a = dot(D0, D0), b = dot(D0, D1), c = dot(D0, D2), dd = dot(D1, D0), e = dot(D1, D1),
                 f = dot(D1, D2), g = dot(D2, D0), h = dot(D2, D1), ii = dot(D2, D2);
    const double r0 = -dot(D0, w0), r1 = -dot(D1, w0), r2 = -dot(D2, w0);
    const double det = a * (e * ii - f * h) - b * (dd * ii - f * g) + c * (dd * h - e * g);
    if (fabs(det) < 1e-300) return;
    const double id = 1.0 / det;
    l1 = (r0 * (e * ii - f * h) - b * (r1 * ii - f * r2) + c * (r1 * h - e * r2)) * id;
    l2 = (a * (r1 * ii - f * r2) - r0 * (dd * ii - f * g) + c * (dd * r2 - r1 * g)) * id;
    l3 = (a * (e * r2 - r1 * h) - b * (dd * r2 - r1 * g) + r0 * (dd * h - e * g)) * id;
    l0 = 1 - ((l1 + l2) + l3);
    if (l0 < -1e-14 || l1 < -1e-14 || l2 < -1e-14 || l3 < -1e-14) return;
  }
  V3 p = l0 * w0;
  if (k > 1) p = p + l1 * S[i1].w;
  if (k > 2) p = p + l2 * S[i2].w;
  if (k > 3) p = p + l3 * S[i3].w;
  const double dv = dot(p, p);
  // a tetrahedron spans R^3, so its candidate must be the origin itself; a
  // nonzero p means a flat, ill-conditioned tetrahedron (oracle: same test)
  if (k == 4 && dv > 1e-20) return;
  if (B.mask == 0 || dv < B.best - 1e-18) {
    B.best = dv;
    B.mask = MASK;
    B.v = p;
    B.l[0] = l0;
    B.l[1] = l1;
    B.l[2] = l2;
    B.l[3] = l3;
  }
}
// masks MASK, MASK-1, ..., LO
template <int MASK, int LO, bool DONE = (MASK < LO)>
struct CsLoop {
  DRC_HD static __forceinline__ void run(const SV2 (&S)[4], CsBest& B) {
    cs_try<MASK>(S, B);
    CsLoop<MASK - 1, LO>::run(S, B);
  }
};
template <int MASK, int LO>
struct CsLoop<MASK, LO, true> {
  DRC_HD static __forceinline__ void run(const SV2 (&)[4], CsBest&) {}
};
template <int N>
DRC_HD __forceinline__ int closest_n(SV2 (&S)[4], V3* v, double (&lam)[4]) {
  CsBest B;
  B.best = 0;
  B.mask = 0;
  B.v = v3(0, 0, 0);
  B.l[0] = B.l[1] = B.l[2] = B.l[3] = 0;
  // The newest vertex is S[N-1] and the masks holding it come first in the
  // descending order.  GJK appends a support point only when it improves on
  // |v| by the gap tolerance, so the closest point then involves it and the
  // masks without it (sub-simplices of the previous simplex, no closer than
  // |v|) are searched only when none with it is valid (oracle: same rule).
  CsLoop<(1 << N) - 1, 1 << (N - 1)>::run(S, B);
  if (N > 1 && B.mask == 0) CsLoop<(1 << (N - 1)) - 1, 1>::run(S, B);
  const int bmask = B.mask;
  *v = B.v;
  const double b0 = B.l[0], b1 = B.l[1], b2 = B.l[2], b3 = B.l[3];
  // compact kept vertices to the front with selects only
  SV2 T[4] = {S[0], S[0], S[0], S[0]};
  int k = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const bool keep = (bmask >> i) & 1;
#pragma unroll
    for (int t = 0; t <= i; ++t) {
      const bool here = keep && k == t;
      T[t].w = v3(here ? S[i].w.x : T[t].w.x, here ? S[i].w.y : T[t].w.y, here ? S[i].w.z : T[t].w.z);
      T[t].a = v3(here ? S[i].a.x : T[t].a.x, here ? S[i].a.y : T[t].a.y, here ? S[i].a.z : T[t].a.z);
    }
    k += keep;
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) S[t] = T[t];
  lam[0] = b0;
  lam[1] = b1;
  lam[2] = b2;
  lam[3] = b3;
  return k;
}

// closest_n for a per-lane simplex size n (lane-per-instance GJK, where
// lanes of one wave hold simplices of different sizes): one descending pass
// over all 15 masks, each taken only where it exists for this lane's n, with
// the same two phases (masks holding the newest vertex, then the rest if none
// of those was valid) -- per lane bit-identical to closest_n<n>, at the cost
// of closest_n<4> instead of the sum over the sizes present in the wave.
template <int MASK>
struct CsAny {
  DRC_HD static __forceinline__ void run(const SV2 (&S)[4], int n, CsBest& B, bool& allow2) {
    if (MASK + 1 == (1 << (n - 1))) allow2 = B.mask == 0;  // entering phase 2
    if (MASK < (1 << n) && (MASK >= (1 << (n - 1)) || allow2)) cs_try<MASK>(S, B);
    CsAny<MASK - 1>::run(S, n, B, allow2);
  }
};
template <>
struct CsAny<0> {
  DRC_HD static __forceinline__ void run(const SV2 (&)[4], int, CsBest&, bool&) {}
};
DRC_HD __forceinline__ int closest_any(SV2 (&S)[4], int n, V3* v, double (&lam)[4]) {
  CsBest B;
  B.best = 0;
  B.mask = 0;
  B.v = v3(0, 0, 0);
  B.l[0] = B.l[1] = B.l[2] = B.l[3] = 0;
  bool allow2 = false;
  CsAny<15>::run(S, n, B, allow2);
  const int bmask = B.mask;
  *v = B.v;
  SV2 T[4] = {S[0], S[0], S[0], S[0]};
  int k = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const bool keep = (bmask >> i) & 1;
#pragma unroll
    for (int t = 0; t <= i; ++t) {
      const bool here = keep && k == t;
      T[t].w = v3(here ? S[i].w.x : T[t].w.x, here ? S[i].w.y : T[t].w.y, here ? S[i].w.z : T[t].w.z);
      T[t].a = v3(here ? S[i].a.x : T[t].a.x, here ? S[i].a.y : T[t].a.y, here ? S[i].a.z : T[t].a.z);
    }
    k += keep;
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) S[t] = T[t];
  lam[0] = B.l[0];
  lam[1] = B.l[1];
  lam[2] = B.l[2];
  lam[3] = B.l[3];
  return k;
}

// Support-gap stop tolerances (metres; oracle: GJK_TOL / EPA_TOL).  The
// winning pair's witnesses are refined to the exact critical point afterwards
// (refine_witness, D17), so GJK / EPA only decide the argmin and the basin:
// both stop at hpp-fcl's GJKSolver defaults (gjk_tolerance, epa_tolerance)
constexpr double kGjkTol = 1e-6, kEpaTol = 1e-6;

// GJK on the cores (same iteration, tolerances and duplicate test as
// oracle/drc_oracle.c:gjk).  The simplex stays in registers.  ANY: the
// closest-point step for per-lane simplex sizes (closest_any).
struct GjkState {
  SV2 S[4];
  double lam[4];
  V3 v;
  int n, intersect, pruned;
};
// cut: the caller only needs the distance if it is <= cut.  Every support
// point gives the lower bound v.w / |v| of the (signed) distance; once it
// exceeds cut the pair cannot matter and the run stops with pruned = 1.
template <bool ANY = false, class SH = Shape>
DRC_HD __forceinline__ void gjk_run(const SH& A, const SH& B, GjkState& g, double cut = 1e300) {
  SV2(&S)[4] = g.S;
#pragma unroll
  for (int i = 0; i < 4; ++i) S[i].w = S[i].a = v3(0, 0, 0);
  g.lam[0] = 1;
  g.lam[1] = g.lam[2] = g.lam[3] = 0;
  V3 v = v3(A.T[9] - B.T[9], A.T[10] - B.T[10], A.T[11] - B.T[11]);
  if (dot(v, v) < 1e-24) v = v3(1, 0, 0);
  int n = 0;
  g.intersect = 0;
  g.pruned = 0;
  for (int it = 0; it < 128; ++it) {
    const SV w = sup_md(A, B, -1.0 * v);
    const double vv = dot(v, v), vw = dot(v, w.w), sv = sqrt(vv);
    if (vw > cut * sv) {
      g.pruned = 1;
      break;
    }
    if (n > 0 && vv - vw <= kGjkTol * sv) break;
    bool dup = false;
#pragma unroll
    for (int i = 0; i < 4; ++i) dup |= i < n && S[i].w.x == w.w.x && S[i].w.y == w.w.y && S[i].w.z == w.w.z;
    // a repeated support point before the gap test passed: the simplex
    // stalled numerically; v.w <= 0 means the difference reaches past the
    // origin (overlap), as in oracle/drc_oracle.c:gjk
    if (dup) {
      g.intersect = dot(v, w.w) <= 0;
      break;
    }
    SV2 nw;
    nw.w = w.w;
    nw.a = w.a;
    // append with selects (a dynamic S[n] store would force S into scratch)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool here = i == n;
      S[i].w = v3(here ? nw.w.x : S[i].w.x, here ? nw.w.y : S[i].w.y, here ? nw.w.z : S[i].w.z);
      S[i].a = v3(here ? nw.a.x : S[i].a.x, here ? nw.a.y : S[i].a.y, here ? nw.a.z : S[i].a.z);
    }
    ++n;
#ifdef DRC_NARROW_DEBUG
    printf("gjk it %d add w %.17g %.17g %.17g (n=%d) vv %.6g vw %.6g\n", it, w.w.x, w.w.y, w.w.z, n, vv, dot(v, w.w));
#endif
    if constexpr (ANY) {
      n = closest_any(S, n, &v, g.lam);
    } else {
      if (n == 1) n = closest_n<1>(S, &v, g.lam);
      else if (n == 2) n = closest_n<2>(S, &v, g.lam);
      else if (n == 3) n = closest_n<3>(S, &v, g.lam);
      else n = closest_n<4>(S, &v, g.lam);
    }
#ifdef DRC_NARROW_DEBUG
    printf("   -> n %d v %.6g %.6g %.6g |v| %.6g\n", n, v.x, v.y, v.z, sqrt(dot(v, v)));
#endif
    if (n == 4 || dot(v, v) < 1e-24) {
      g.intersect = 1;
      break;
    }
  }
  g.n = n;
  g.v = v;
}
// EPA seed stash (epa_stash, below): the task stage's GJK of a pair that
// turns out to intersect leaves its final simplex for EPA, which would
// otherwise rerun the same GJK on one lane
struct EpaPoly;
DRC_HD void epa_stash(EpaPoly* E, const GjkState& g, int pair);
// separation distance and witnesses (valid when !intersect)
struct GjkDist {
  int intersect, pruned;
  double dist;
  V3 pA, pB;
};
template <class SH>
DRC_HD inline __noinline__ GjkDist gjk(const SH A, const SH B, double cut = 1e300, EpaPoly* stash = nullptr,
                                       int pair = 0) {
  GjkState g;
  gjk_run(A, B, g, cut);
  if (stash && g.intersect) epa_stash(stash, g, pair);
  GjkDist o;
  o.intersect = g.intersect;
  o.pruned = g.pruned;
  // witnesses: sum_i lam_i a_i and sum_i lam_i b_i (oracle accumulation order)
  V3 pA = v3(0, 0, 0), pB = v3(0, 0, 0);
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (i < g.n) {
      pA = pA + g.lam[i] * g.S[i].a;
      pB = pB + g.lam[i] * (g.S[i].a - g.S[i].w);
    }
  o.pA = pA;
  o.pB = pB;
  o.dist = sqrt(dot(g.v, g.v));
  return o;
}

// Expanding polytope (EPA) with face adjacency (Bullet/libccd style).  The
// polytope lives in LDS.  One expansion step from the closest face `best` by
// the support point w (oracle/drc_oracle.c:epa_grow_canon, same decisions):
//  - the removed region C is the connected component of `best` among the
//    alive faces that see w (what btGjkEpa2's recursive flood fill kills);
//  - its horizon (edges of C faces whose neighbour is outside C) must be one
//    simple cycle of >= 3 edges; the new faces (start, end, w) take slots in
//    cycle order from the edge of smallest key 3 face + edge: free list first
//    (last freed first), then fresh slots;
//  - every new face must be non-degenerate, keep the origin inside and not
//    undercut `best` (EPA's lower bound never decreases);
//  - C is freed in ascending slot order, `best` last.
// A failed step leaves the polytope unchanged and EPA stops.  The task kernel
// runs a step on the whole wave (epa_grow_wave: component by ballots, horizon
// compaction, cycle order by pointer jumping, one new face per lane);
// epa_grow_canon is the lane-serial form (host harness, single-lane use).
// caps: hpp-fcl's GJKSolver defaults (epa_max_vertex_num 64,
// epa_max_face_num 128, epa_max_iterations 255), mirrored by the oracle
constexpr int kEpaMaxV = 64, kEpaMaxF = 128;
static_assert(kEpaMaxF == 128, "face bit masks are two 64-bit words");
static_assert(kEpaMaxF <= 256 && kEpaMaxV <= 127, "EpaPoly's 8-bit face and horizon fields");
struct EpaPoly {
  double vw[kEpaMaxV][3], va[kEpaMaxV][3];
  double fn[kEpaMaxF][3], fd[kEpaMaxF];
  double out[6];
  // narrow index types (faces < 128, edges < 3, horizon positions < 64): the
  // polytope is most of the task kernel's per-wave LDS
  int16_t adj[kEpaMaxF][3];  // neighbour across edge e: face | (its edge << 8)
  int16_t hl[kEpaMaxV];      // a step's horizon edges: face | (edge << 8)
  int8_t vout[kEpaMaxV], vin[kEpaMaxV];  // horizon edge leaving / entering each vertex (-1: none)
  int16_t fv[kEpaMaxF][3];
  int16_t freel[kEpaMaxF];  // recycled slots, last freed first
  int8_t alive[kEpaMaxF];
  int nv, nf, fail, stop, nfree;
};
DRC_HD __forceinline__ V3 epa_vw(const EpaPoly* E, int i) { return v3(E->vw[i][0], E->vw[i][1], E->vw[i][2]); }
DRC_HD __forceinline__ V3 epa_va(const EpaPoly* E, int i) { return v3(E->va[i][0], E->va[i][1], E->va[i][2]); }
DRC_HD __forceinline__ void epa_addv(EpaPoly* E, V3 w, V3 a) {
  st3(E->vw[E->nv], w);
  st3(E->va[E->nv], a);
  E->nv++;
}
// Seed stash: kEpaStash simplices of intersecting pairs in the vertex slots
// kEpaStashV0.. (only a polytope grown past kEpaStashV0 vertices reaches
// them), their pair and size in out[] (written only by epa_finish).  The
// slot comes from an LDS counter in E->nv, zeroed before the candidate GJKs.
// The GJK of a pair that intersects never took its cut exit, so its final
// simplex is exactly the one epa_init's rerun would build (same iterations).
constexpr int kEpaStash = 2, kEpaStashV0 = kEpaMaxV - 4 * kEpaStash;
DRC_HD __forceinline__ void epa_stash(EpaPoly* E, const GjkState& g, int pair) {
  const int k = __atomic_fetch_add(&E->nv, 1, __ATOMIC_RELAXED);
  if (k >= kEpaStash) return;
  for (int i = 0; i < 4; ++i)
    if (i < g.n) {
      st3(E->vw[kEpaStashV0 + 4 * k + i], g.S[i].w);
      st3(E->va[kEpaStashV0 + 4 * k + i], g.S[i].a);
    }
  E->out[2 * k] = pair;
  E->out[2 * k + 1] = g.n;
}
// "face f sees w": the oracle's visibility test (not (n.w - d < -1e-12))
DRC_HD __forceinline__ bool epa_sees(const EpaPoly* E, int f, V3 w) {
  return !(dot(ld3(E->fn[f]), w) - E->fd[f] < -1e-12);
}
// normal and offset of the face (a, b, c); false if degenerate, seeing the
// origin from outside or closer than fdmin (oracle epa_newface / epa_grow_canon)
DRC_HD __forceinline__ bool epa_face_plane(const EpaPoly* E, int a, int b, int c, double fdmin, V3* n, double* fd) {
  const V3 va_ = epa_vw(E, a);
  V3 nn = cross(epa_vw(E, b) - va_, epa_vw(E, c) - va_);
  const double L = sqrt(dot(nn, nn));
  if (!(L > 1e-300)) return false;
  nn = v3(nn.x / L, nn.y / L, nn.z / L);  // same rounding as the oracle
  *n = nn;
  *fd = dot(nn, va_);
  return !(*fd < -1e-12 || *fd < fdmin - 1e-12);
}
// initial tetrahedron face (lane-serial)
DRC_HD __forceinline__ int epa_newface(EpaPoly* E, int a, int b, int c) {
  int f;
  if (E->nfree > 0) {
    f = E->freel[--E->nfree];
  } else if (E->nf < kEpaMaxF) {
    f = E->nf++;
  } else {
    E->fail = 1;
    return -1;
  }
  E->fv[f][0] = a;
  E->fv[f][1] = b;
  E->fv[f][2] = c;
  V3 n;
  double fd;
  const bool ok = epa_face_plane(E, a, b, c, -1e300, &n, &fd);
  st3(E->fn[f], n);
  E->fd[f] = fd;
  E->alive[f] = ok;
  if (!ok) E->fail = 1;
  return ok ? f : -1;
}
DRC_HD __forceinline__ void epa_bind(EpaPoly* E, int f0, int e0, int f1, int e1) {
  E->adj[f0][e0] = f1 | (e1 << 8);
  E->adj[f1][e1] = f0 | (e0 << 8);
}
// rerun GJK and build the initial tetrahedron from its final simplex
// (lane-serial)
// (epa_seed: the vertices E->vw / va [0, nv) are GJK's simplex)
template <class SH>
DRC_HD __forceinline__ void epa_seed(const SH A, const SH B, EpaPoly* E);
template <class SH>
DRC_HD __forceinline__ void epa_init(const SH A, const SH B, EpaPoly* E) {
  GjkState g;
  gjk_run(A, B, g);
  E->nv = 0;
  for (int i = 0; i < 4; ++i)
    if (i < g.n) epa_addv(E, g.S[i].w, g.S[i].a);
  epa_seed(A, B, E);
}
// the same from stash slot k (epa_stash)
template <class SH>
DRC_HD __forceinline__ void epa_init_stash(const SH A, const SH B, EpaPoly* E, int k, int n) {
  for (int i = 0; i < 4; ++i)
    if (i < n) {
      st3(E->vw[i], epa_vw(E, kEpaStashV0 + 4 * k + i));
      st3(E->va[i], epa_va(E, kEpaStashV0 + 4 * k + i));
    }
  E->nv = n;
  epa_seed(A, B, E);
}
template <class SH>
DRC_HD __forceinline__ void epa_seed(const SH A, const SH B, EpaPoly* E) {
  E->nf = 0;
  E->fail = 0;
  E->nfree = 0;
  for (int di = 0; di < 6 && E->nv < 4; ++di) {
    const double sgn = di < 3 ? 1.0 : -1.0;
    const int ax = di % 3;
    const SV w = sup_md(A, B, v3(ax == 0 ? sgn : 0.0, ax == 1 ? sgn : 0.0, ax == 2 ? sgn : 0.0));
    bool ok = true;
    for (int i = 0; i < E->nv; ++i) {
      const V3 d = w.w - epa_vw(E, i);
      ok &= sqrt(dot(d, d)) > 1e-12;
    }
    if (ok) epa_addv(E, w.w, w.a);
  }
  {  // orient the tetrahedron so that face (0,1,2) looks away from vertex 3
    const V3 nn = cross(epa_vw(E, 1) - epa_vw(E, 0), epa_vw(E, 2) - epa_vw(E, 0));
    if (dot(nn, epa_vw(E, 3) - epa_vw(E, 0)) > 0) {
      for (int c = 0; c < 3; ++c) {
        double t = E->vw[0][c];
        E->vw[0][c] = E->vw[1][c];
        E->vw[1][c] = t;
        t = E->va[0][c];
        E->va[0][c] = E->va[1][c];
        E->va[1][c] = t;
      }
    }
  }
  const int t0 = epa_newface(E, 0, 1, 2), t1 = epa_newface(E, 1, 0, 3), t2 = epa_newface(E, 2, 1, 3),
            t3 = epa_newface(E, 0, 2, 3);
  if (!E->fail) {
    epa_bind(E, t0, 0, t1, 0);
    epa_bind(E, t0, 1, t2, 0);
    epa_bind(E, t0, 2, t3, 0);
    epa_bind(E, t1, 1, t3, 2);
    epa_bind(E, t1, 2, t2, 1);
    epa_bind(E, t2, 2, t3, 1);
  }
  E->stop = E->fail;
}
// stop tests of one expansion step from face `best`, given the support point
// w in direction n_best: support gap below tolerance or vertex cap reached.
// The duplicate-vertex test is separate so a wave can spread it over lanes.
DRC_HD __forceinline__ bool epa_gap_stop(const EpaPoly* E, int best, const SV& w) {
  return dot(ld3(E->fn[best]), w.w) - E->fd[best] <= kEpaTol || E->nv >= kEpaMaxV;
}
DRC_HD __forceinline__ bool epa_is_dup(const EpaPoly* E, int i, const SV& w) {
  const V3 d = w.w - epa_vw(E, i);
  return fabs(d.x) <= 1e-14 && fabs(d.y) <= 1e-14 && fabs(d.z) <= 1e-14;
}
DRC_HD __forceinline__ int epa_next_edge(int e) { return e == 2 ? 0 : e + 1; }
// lane-serial step (see the header comment); sets E->stop on failure
DRC_HD inline void epa_grow_canon(EpaPoly* E, const SV w, int best) {
  bool inC[kEpaMaxF];
  int hf[kEpaMaxV], he[kEpaMaxV], ord[kEpaMaxV], slot[kEpaMaxV];
  const int wi = E->nv, nf = E->nf;
  st3(E->vw[wi], w.w);
  st3(E->va[wi], w.a);
  for (int f = 0; f < nf; ++f) inC[f] = f == best;
  for (bool grown = true; grown;) {
    grown = false;
    for (int f = 0; f < nf; ++f) {
      if (inC[f] || !E->alive[f] || !epa_sees(E, f, w.w)) continue;
      for (int e = 0; e < 3; ++e)
        if (inC[E->adj[f][e] & 0xff]) {
          inC[f] = true;
          grown = true;
          break;
        }
    }
  }
  for (int v = 0; v < kEpaMaxV; ++v) E->vout[v] = E->vin[v] = -1;
  int H = 0;
  bool ok = true;
  for (int c = 0; c < nf && ok; ++c) {
    if (!inC[c]) continue;
    for (int e = 0; e < 3 && ok; ++e) {
      if (inC[E->adj[c][e] & 0xff]) continue;
      const int a = E->fv[c][e], b = E->fv[c][epa_next_edge(e)];
      if (H >= kEpaMaxV || E->vout[a] >= 0 || E->vin[b] >= 0) {
        ok = false;
        break;
      }
      E->vout[a] = H;
      E->vin[b] = H;
      hf[H] = c;
      he[H] = e;
      ++H;
    }
  }
  ok = ok && H >= 3;
  int cur = 0;
  for (int k = 0; k < H && ok; ++k) {
    if (cur < 0 || (k > 0 && cur == 0)) ok = false;
    else {
      ord[k] = cur;
      cur = E->vout[E->fv[hf[cur]][epa_next_edge(he[cur])]];
    }
  }
  ok = ok && cur == 0 && H <= E->nfree + (kEpaMaxF - nf);
  const double fdmin = E->fd[best];
  for (int k = 0; k < H && ok; ++k) {
    const int h = ord[k], c = hf[h], e = he[h];
    V3 n;
    double fd;
    ok = epa_face_plane(E, E->fv[c][e], E->fv[c][epa_next_edge(e)], wi, fdmin, &n, &fd);
    slot[k] = k < E->nfree ? E->freel[E->nfree - 1 - k] : nf + (k - E->nfree);
  }
  if (!ok) {
    E->stop = 1;
    return;
  }
  for (int k = 0; k < H; ++k) {
    const int f = slot[k], h = ord[k], c = hf[h], e = he[h];
    const int a = E->fv[c][e], b = E->fv[c][epa_next_edge(e)];
    V3 n;
    double fd;
    epa_face_plane(E, a, b, wi, fdmin, &n, &fd);
    st3(E->fn[f], n);
    E->fd[f] = fd;
    E->fv[f][0] = a;
    E->fv[f][1] = b;
    E->fv[f][2] = wi;
    const int g = E->adj[c][e];
    E->adj[f][0] = g;
    E->adj[g & 0xff][g >> 8] = f;
    E->adj[f][1] = slot[(k + 1) % H] | (2 << 8);
    E->adj[f][2] = slot[(k + H - 1) % H] | (1 << 8);
  }
  const int nfree0 = E->nfree > H ? E->nfree - H : 0;
  if (H > E->nfree) E->nf = nf + (H - E->nfree);
  E->nfree = nfree0;
  for (int c = 0; c < nf; ++c)
    if (inC[c] && c != best) {
      E->alive[c] = 0;
      E->freel[E->nfree++] = c;
    }
  E->alive[best] = 0;
  E->freel[E->nfree++] = best;
  for (int k = 0; k < H; ++k) E->alive[slot[k]] = 1;
  E->nv = wi + 1;
}
// witness points on the closest face (lane-serial); returns -depth
DRC_HD __forceinline__ double epa_finish(EpaPoly* E, int best) {
  const double bd = E->fd[best];
  const V3 bn = ld3(E->fn[best]);
  const int i0 = E->fv[best][0], i1 = E->fv[best][1], i2 = E->fv[best][2];
  const V3 aw = epa_vw(E, i0), bw = epa_vw(E, i1), cw = epa_vw(E, i2);
  const V3 p = bd * bn, v0 = bw - aw, v1 = cw - aw, v2 = p - aw;
  const double d00 = dot(v0, v0), d01 = dot(v0, v1), d11 = dot(v1, v1), d20 = dot(v2, v0), d21 = dot(v2, v1);
  const double den = d00 * d11 - d01 * d01;
  const double l1 = (d11 * d20 - d01 * d21) / den, l2 = (d00 * d21 - d01 * d20) / den, l0 = 1 - l1 - l2;
  const V3 aa = epa_va(E, i0), ba = epa_va(E, i1), ca = epa_va(E, i2);
  st3(E->out, l0 * aa + l1 * ba + l2 * ca);
  st3(E->out + 3, l0 * (aa - aw) + l1 * (ba - bw) + l2 * (ca - cw));
  return -bd;
}
// A lane's two faces (l, l + 64) as the step's closest-face scan loads them:
// alive, offset, normal, adjacency.  epa_run_wave loads them before the scan's
// reduction and the support point, so the growth's visibility pass starts from
// registers instead of a second round of LDS reads.
struct EpaFaces {
  bool h0, h1, al0, al1;
  double fd0, fd1;
  V3 fn0, fn1;
  int n0[3], n1[3];
};
__device__ __forceinline__ void epa_load_faces(const EpaPoly* E, int nf, int l, EpaFaces& F) {
  const int f0 = l, f1 = l + 64;
  F.h0 = f0 < nf;
  F.h1 = f1 < nf;
  F.al0 = F.h0 && E->alive[f0];
  F.al1 = F.h1 && E->alive[f1];
  F.fd0 = F.h0 ? E->fd[f0] : 0.0;
  F.fd1 = F.h1 ? E->fd[f1] : 0.0;
  F.fn0 = F.h0 ? ld3(E->fn[f0]) : v3(0, 0, 0);
  F.fn1 = F.h1 ? ld3(E->fn[f1]) : v3(0, 0, 0);
#pragma unroll
  for (int e = 0; e < 3; ++e) {
    F.n0[e] = F.h0 ? E->adj[f0][e] : 0;
    F.n1[e] = F.h1 ? E->adj[f1][e] : 0;
  }
}
// Wave form of epa_grow_canon (the task kernel; every lane calls it with the
// same w and best).  Lane l owns faces l and l + 64 and, after compaction,
// horizon edge l.  Same slots, adjacency, face data, free list and decisions.
__device__ __forceinline__ void epa_grow_wave(EpaPoly* E, const SV& w, int best, const EpaFaces& F,
                                              unsigned long long* gt = nullptr) {
  const int l = threadIdx.x & 63;
  // (timing builds: gt[0..3] += cycles in visibility + component, horizon +
  // cycle check, cycle order + new planes, writes)
  unsigned long long tg = gt ? __builtin_amdgcn_s_memtime() : 0;
  auto lap = [&](int k) {
    if (gt) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      gt[k] += t - tg;
      tg = t;
    }
  };
  const int nf = E->nf, wi = E->nv, nfree = E->nfree;
  if (l == 0) {
    st3(E->vw[wi], w.w);
    st3(E->va[wi], w.a);
  }
  E->vout[l] = -1;
  E->vin[l] = -1;
  const int f0 = l, f1 = l + 64;
  // "face f sees w" (epa_sees) on the registers of the scan
  const bool s0 = F.al0 && !(dot(F.fn0, w.w) - F.fd0 < -1e-12);
  const bool s1 = F.al1 && !(dot(F.fn1, w.w) - F.fd1 < -1e-12);
  const int *n0 = F.n0, *n1 = F.n1;
  auto in = [](uint64_t lo, uint64_t hi, int f) -> bool {
    return f < 64 ? (lo >> f) & 1ull : (hi >> (f - 64)) & 1ull;
  };
  uint64_t clo = best < 64 ? 1ull << best : 0ull, chi = best < 64 ? 0ull : 1ull << (best - 64);
  for (;;) {  // component of best among the visible faces, one ring per round
    const bool j0 = s0 && !in(clo, chi, f0) &&
                    (in(clo, chi, n0[0] & 0xff) || in(clo, chi, n0[1] & 0xff) || in(clo, chi, n0[2] & 0xff));
    const bool j1 = s1 && !in(clo, chi, f1) &&
                    (in(clo, chi, n1[0] & 0xff) || in(clo, chi, n1[1] & 0xff) || in(clo, chi, n1[2] & 0xff));
    const uint64_t nlo = clo | __ballot(j0), nhi = chi | __ballot(j1);
    if (nlo == clo && nhi == chi) break;
    clo = nlo;
    chi = nhi;
  }
  lap(0);
  // horizon edges (c, e), compacted in (edge slot j, lane) order
  const bool c0 = in(clo, chi, f0), c1 = in(clo, chi, f1);
  bool hz[6];
#pragma unroll
  for (int e = 0; e < 3; ++e) {
    hz[e] = c0 && !in(clo, chi, n0[e] & 0xff);
    hz[3 + e] = c1 && !in(clo, chi, n1[e] & 0xff);
  }
  const uint64_t below = (1ull << l) - 1;
  int H = 0;
  int pos[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const uint64_t m = __ballot(hz[j]);
    pos[j] = H + __popcll(m & below);
    H += __popcll(m);
  }
  wsync();  // vout / vin cleared, vertex wi stored
  bool bad = H < 3 || H > kEpaMaxV || H > nfree + (kEpaMaxF - nf);
  if (!bad) {
#pragma unroll
    for (int j = 0; j < 6; ++j)
      if (hz[j]) {
        const int c = j < 3 ? f0 : f1, e = j % 3;
        E->hl[pos[j]] = c | (e << 8);
        E->vout[E->fv[c][e]] = pos[j];
        E->vin[E->fv[c][epa_next_edge(e)]] = pos[j];
      }
  }
  wsync();
  const bool own = l < H && !bad;
  int hc = 0, he_ = 0, a = 0, b = 0, nx = 0, pv = 0;
  if (own) {
    const int hv = E->hl[l];
    hc = hv & 0xff;
    he_ = hv >> 8;
    a = E->fv[hc][he_];
    b = E->fv[hc][epa_next_edge(he_)];
    nx = E->vout[b];
    pv = E->vin[a];
    // a vertex starting or ending two edges (the other write won), or an end
    // with no continuation: not one simple cycle
    bad = E->vout[a] != l || E->vin[b] != l || nx < 0 || pv < 0;
  }
  // the new face's plane (independent of the cycle order below, so its FP64
  // chain issues before the cross-lane steps; used only when nothing is bad)
  V3 nn = v3(0, 0, 0);
  double fd = 0;
  bool pbad = false;
  if (own) pbad = !epa_face_plane(E, a, b, wi, E->fd[best], &nn, &fd);
  bad = __any(bad);
  lap(1);
  // cycle position relative to the edge of smallest key 3 face + edge (unique
  // per edge, < 2^9): one integer minimum of key << 6 | lane
  const int s = wave_min_int(own ? ((3 * hc + he_) << 6) | l : 0x7fffffff) & 63;
  int d = (own && l != s) ? 1 : 0, p = own ? (l == s ? s : nx) : l;
  // ceil(log2 H) rounds reach s from every edge of a cycle of H edges (a
  // pointer at s stays there with d += 0, so more rounds change nothing); the
  // pair (d, p) travels in one word: one crossbar shuffle per round
  const int rounds = H > 1 ? 32 - __builtin_clz(H - 1) : 0;
  for (int r = 0; r < rounds; ++r) {
    const int dp = __shfl(d * 64 + p, p, 64);
    d += dp >> 6;
    p = dp & 63;
  }
  bad = __any(bad || (own && p != s));
  int slot = 0;
  bool gbad = bad;
  if (own && !bad) {
    const int k = d == 0 ? 0 : H - d;
    slot = k < nfree ? E->freel[nfree - 1 - k] : nf + (k - nfree);
    gbad = pbad;
  }
  if (__any(gbad)) {
    if (l == 0) E->stop = 1;
    wsync();
    return;
  }
  lap(2);
  const int snx = __shfl(slot, nx, 64), spv = __shfl(slot, pv, 64);
  const int g = own ? E->adj[hc][he_] : 0;
  // C's faces, ascending, then best: positions in the new free list
  const uint64_t rlo = clo & ~(best < 64 ? 1ull << best : 0ull), rhi = chi & ~(best < 64 ? 0ull : 1ull << (best - 64));
  const int nC = __popcll(rlo) + __popcll(rhi), nfree0 = nfree > H ? nfree - H : 0;
  wsync();  // every free-list read (slots) before the free list is rewritten
  if (own) {
    st3(E->fn[slot], nn);
    E->fd[slot] = fd;
    E->fv[slot][0] = a;
    E->fv[slot][1] = b;
    E->fv[slot][2] = wi;
    E->adj[slot][0] = g;
    E->adj[g & 0xff][g >> 8] = slot;
    E->adj[slot][1] = snx | (2 << 8);
    E->adj[slot][2] = spv | (1 << 8);
    E->alive[slot] = 1;
  }
  if (in(rlo, rhi, f0)) {
    E->alive[f0] = 0;
    E->freel[nfree0 + __popcll(rlo & below)] = f0;
  }
  if (in(rlo, rhi, f1)) {
    E->alive[f1] = 0;
    E->freel[nfree0 + __popcll(rlo) + __popcll(rhi & below)] = f1;
  }
  if (l == 0) {
    E->alive[best] = 0;
    E->freel[nfree0 + nC] = best;
    E->nfree = nfree0 + nC + 1;
    if (H > nfree) E->nf = nf + (H - nfree);
    E->nv = wi + 1;
  }
  wsync();
  lap(3);
}
// EPA on the whole wave for one penetrating pair: lane ln seeds the polytope
// from GJK's simplex; per step the wave takes the closest alive face, the
// support point and the stop tests, then grows (epa_grow_wave).  Returns the
// signed distance (-depth) on every lane; lane ln leaves the witnesses in
// E->out.  Same steps and result as epa_serial.  st (timing builds): steps,
// cycles in face scan, support + tests, growth.
template <class SH>
__device__ __forceinline__ double epa_run_wave(const SH& A, const SH& B, EpaPoly* E, int ln, int sk = -1,
                                               int sn = 0, unsigned long long* st = nullptr) {
  const int l = threadIdx.x & 63;
  const unsigned long long ti = st ? __builtin_amdgcn_s_memtime() : 0;
  if (l == ln) {  // seed from the stashed simplex (sk >= 0) or rerun GJK
    if (sk >= 0) epa_init_stash(A, B, E, sk, sn);
    else epa_init(A, B, E);
  }
  wsync();
  if (st) st[8] += __builtin_amdgcn_s_memtime() - ti;  // (timing builds: the seed polytope)
  double dres = 0;
  for (int it = 0; it <= 255; ++it) {
    unsigned long long t0 = 0, t1 = 0;
    if (st) {
      st[0] = it;
      t0 = __builtin_amdgcn_s_memtime();
    }
    bool stop = E->stop || it == 255;
    double fdm = 1e300;
    int fb = 0x7fffffff;
    EpaFaces F;
    epa_load_faces(E, E->nf, l, F);  // (faces l, l + 64: nf <= 128)
    if (F.al0 && F.fd0 < fdm) {
      fdm = F.fd0;
      fb = l;
    }
    if (F.al1 && F.fd1 < fdm) {
      fdm = F.fd1;
      fb = l + 64;
    }
    wave_argmin(fdm, fb);
    if (fb == 0x7fffffff) {  // no alive face (failed seed): the oracle takes face 0
      fb = 0;
      stop = true;
    }
    if (st) {
      t1 = __builtin_amdgcn_s_memtime();
      st[1] += t1 - t0;
    }
    SV w;
    if (!stop) {  // support, gap and duplicate tests on the whole wave
      w = sup_md(A, B, ld3(E->fn[fb]));
      stop = epa_gap_stop(E, fb, w);
      if (!stop) {
        bool dup = false;
        for (int i = l; i < E->nv; i += 64) dup |= epa_is_dup(E, i, w);
        stop = __any(dup);
      }
    }
    if (stop) {
      if (l == ln) dres = epa_finish(E, fb);
      break;
    }
    if (st) t0 = __builtin_amdgcn_s_memtime(), st[2] += t0 - t1;
    epa_grow_wave(E, w, fb, F, st ? st + 4 : nullptr);
    if (st) st[3] += __builtin_amdgcn_s_memtime() - t0;
  }
  return __shfl(dres, ln, 64);
}
// one expansion step (lane-serial form, host harness)
template <class SH>
DRC_HD inline void epa_step(const SH& A, const SH& B, EpaPoly* E, int best) {
  const SV w = sup_md(A, B, ld3(E->fn[best]));
  bool stop = epa_gap_stop(E, best, w);
  for (int i = 0; !stop && i < E->nv; ++i) stop = epa_is_dup(E, i, w);
  if (stop) {
    E->stop = 1;
    return;
  }
  epa_grow_canon(E, w, best);
}
// closest alive face by a serial scan (host / oracle-style reference)
DRC_HD inline int epa_best_serial(const EpaPoly* E) {
  int best = -1;
  double bd = 1e300;
  for (int f = 0; f < E->nf; ++f)
    if (E->alive[f] && E->fd[f] < bd) {
      bd = E->fd[f];
      best = f;
    }
  return best;
}
// lane-serial driver (host harness and single-lane use)
template <class SH>
DRC_HD inline double epa_serial(const SH& A, const SH& B, EpaPoly* E) {
  epa_init(A, B, E);
  for (int it = 0; it < 255 && !E->stop; ++it) epa_step(A, B, E, epa_best_serial(E));
  const int bb = epa_best_serial(E);
  return epa_finish(E, bb < 0 ? 0 : bb);
}

// signed distance + closest surface point of a solid cylinder / box
template <class SH>
DRC_HD __forceinline__ double point_cylinder(V3 c, const SH& s, V3* qw) {
  V3 loc = rotT(s.T, c - v3(s.T[9], s.T[10], s.T[11])), q = loc;
  double r = s.p0, h = s.p1, rho = sqrt(loc.x * loc.x + loc.y * loc.y), sd;
  if (!(rho <= r && fabs(loc.z) <= h)) {
    if (rho > r) {
      q.x = loc.x * r / rho;
      q.y = loc.y * r / rho;
    }
    q.z = loc.z < -h ? -h : (loc.z > h ? h : loc.z);
    V3 dq = loc - q;
    sd = sqrt(dot(dq, dq));
  } else {
    double dside = r - rho, dtop = h - loc.z, dbot = h + loc.z;
    if (dside <= dtop && dside <= dbot) {
      if (rho > 0) {
        q.x = loc.x * r / rho;
        q.y = loc.y * r / rho;
      } else {
        q.x = r;
        q.y = 0;
      }
      sd = -dside;
    } else if (dtop <= dbot) {
      q.z = h;
      sd = -dtop;
    } else {
      q.z = -h;
      sd = -dbot;
    }
  }
  *qw = xform(s.T, q);
  return sd;
}
template <class SH>
DRC_HD __forceinline__ double point_box(V3 c, const SH& s, V3* qw) {
  V3 loc = rotT(s.T, c - v3(s.T[9], s.T[10], s.T[11])), q = loc;
  double hx[3] = {s.p0, s.p1, s.p2}, l[3] = {loc.x, loc.y, loc.z}, qq[3] = {loc.x, loc.y, loc.z}, sd;
  bool inside = fabs(l[0]) <= hx[0] && fabs(l[1]) <= hx[1] && fabs(l[2]) <= hx[2];
  if (!inside) {
    for (int i = 0; i < 3; ++i) qq[i] = l[i] < -hx[i] ? -hx[i] : (l[i] > hx[i] ? hx[i] : l[i]);
    V3 dq = v3(l[0] - qq[0], l[1] - qq[1], l[2] - qq[2]);
    sd = sqrt(dot(dq, dq));
  } else {
    int a = 0;
    double g = hx[0] - fabs(l[0]);
    for (int i = 1; i < 3; ++i) {
      double gi = hx[i] - fabs(l[i]);
      if (gi < g) {
        g = gi;
        a = i;
      }
    }
    qq[a] = l[a] >= 0 ? hx[a] : -hx[a];
    sd = -g;
  }
  q = v3(qq[0], qq[1], qq[2]);
  *qw = xform(s.T, q);
  return sd;
}

// Closed-form pairs (sphere-X).  Returns the hpp-fcl convention
// pB - pA = d * n with n the A->B direction.
template <class SH>
DRC_HD __forceinline__ double sphere_pair(const SH& A, const SH& B, V3* pA, V3* pB) {
  if (A.type == kSphere && B.type == kSphere) {
    V3 cA = v3(A.T[9], A.T[10], A.T[11]), cB = v3(B.T[9], B.T[10], B.T[11]);
    V3 v = cB - cA;
    double L = sqrt(dot(v, v));
    V3 n = L > 0 ? (1.0 / L) * v : v3(1, 0, 0);
    *pA = cA + A.p0 * n;
    *pB = cB - B.p0 * n;
    return L - A.p0 - B.p0;
  }
  bool flip = B.type == kSphere;
  const SH& s = flip ? B : A;
  const SH& o = flip ? A : B;
  V3 c = v3(s.T[9], s.T[10], s.T[11]), q;
  double sd = o.type == kCylinder ? point_cylinder(c, o, &q) : point_box(c, o, &q);
  V3 u = q - c;
  double L = sqrt(dot(u, u));
  V3 n = L > 0 ? (1.0 / L) * u : v3(1, 0, 0);
  if (sd < 0) n = -1.0 * n;
  V3 ps = c + s.p0 * n;
  if (flip) {
    *pA = q;
    *pB = ps;
  } else {
    *pA = ps;
    *pB = q;
  }
  return sd - s.p0;
}

// ------------------------------------------------------------ witness refinement
// DESIGN.md D17 (oracle twin: refine_witness in oracle/drc_oracle.c, same
// features, rules and tolerances).  The GJK / EPA witnesses of the winning
// pair converge only to ~sqrt(gap) / the EPA vertex cap, so implementations
// whose iterations differ by rounding disagree by up to ~1e-5 there, and the
// distance gradient n^T (J_B(pB) - J_A(pA)), n = (pB - pA)/|pB - pA|, with
// them.  The exact witnesses are a critical point of |X_A(u_A) - X_B(u_B)|^2
// over the surface features the estimates lie on -- cylinder side (theta, z),
// cap (x, y), rim (theta); box face / edge / vertex (the free coordinates) --
// which Newton reaches quadratically from either implementation's estimate.
// Accepted when the point lies inside its features, n* = (pB - pA)/sd is in
// A's normal cone and -n* in B's, and sd moves by <= 1e-6; otherwise the
// estimates stay (parallel flat features: witnesses not unique).
// Device form: register-only and compact (the task kernel calls it once per
// instance on one lane, so its code size matters more than its FLOPs).  One
// 4-unknown Newton system for every feature pair (absent parameters get
// identity rows), and the angle of a side / rim point is kept as its unit
// radial vector (c, s) moved by the retraction normalize(r + delta t / r): no
// transcendental calls.  The oracle's form (angles, variable-size system)
// converges to the same critical point.
enum : int { kFtSide = 0, kFtCap = 1, kFtRim = 2, kFtBox = 3 };
struct Feat {
  int kind;
  double s;
  int fx, fy, fz;  // box: 0 free, +-1 the face sign of that axis
  DRC_HD __forceinline__ int fix(int i) const { return i == 0 ? fx : (i == 1 ? fy : fz); }
  DRC_HD __forceinline__ void set_fix(int i, int v) {
    if (i == 0) fx = v;
    else if (i == 1) fy = v;
    else fz = v;
  }
  DRC_HD __forceinline__ int nparam() const {
    return kind == kFtRim ? 1 : (kind == kFtBox ? (fx == 0) + (fy == 0) + (fz == 0) : 2);
  }
};
// feature parameters: side (c, s, z), rim (c, s), cap (x, y), box (first, second free coordinate)
struct FParam {
  double a, b, c;
};
constexpr double kRwTau = 1e-4, kRwPivot = 1e-9, kRwStep = 1e-12, kRwCone = 1e-9, kRwDMove = 1e-5;

DRC_HD __forceinline__ double v3c(V3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }
DRC_HD __forceinline__ V3 v3e(int i) { return v3(i == 0, i == 1, i == 2); }
template <class SH>
DRC_HD __forceinline__ double shp(const SH& s, int i) { return i == 0 ? s.p0 : (i == 1 ? s.p1 : s.p2); }

template <class SH>
DRC_HD inline void rw_classify(const SH& s, V3 x, Feat* f) {
  f->fx = f->fy = f->fz = 0;
  f->s = x.z > 0 ? 1.0 : -1.0;
  if (s.type == kCylinder) {
    const double r = s.p0, h = s.p1, rho = sqrt(x.x * x.x + x.y * x.y);
    if (fabs(x.z) > h - kRwTau && rho > r - kRwTau) f->kind = kFtRim;
    else if (fabs(x.z) > h - kRwTau) f->kind = kFtCap;
    else f->kind = kFtSide;
    return;
  }
  f->kind = kFtBox;
  int any = 0, im = 0;
  double best = -1;
  for (int i = 0; i < 3; ++i) {
    const double xi = v3c(x, i), hi = shp(s, i);
    const int fi = fabs(xi) > hi - kRwTau ? (xi > 0 ? 1 : -1) : 0;
    f->set_fix(i, fi);
    any |= fi != 0;
    const double t = fabs(xi) / hi;
    if (t > best) {
      best = t;
      im = i;
    }
  }
  if (!any) f->set_fix(im, v3c(x, im) > 0 ? 1 : -1);
}
// parameters of feature f at the local point x
DRC_HD inline FParam rw_params(const Feat& f, V3 x) {
  FParam u{0, 0, 0};
  if (f.kind == kFtSide || f.kind == kFtRim) {
    const double rho = sqrt(x.x * x.x + x.y * x.y);
    u.a = rho > 0 ? x.x / rho : 1.0;
    u.b = rho > 0 ? x.y / rho : 0.0;
    u.c = x.z;
  } else if (f.kind == kFtCap) {
    u.a = x.x;
    u.b = x.y;
  } else {
    int k = 0;
    for (int i = 0; i < 3; ++i)
      if (!f.fix(i)) {
        if (k == 0) u.a = v3c(x, i);
        else u.b = v3c(x, i);
        ++k;
      }
  }
  return u;
}
// world point, unit-speed tangents t0, t1 (zero where the feature has fewer
// parameters) and the curvature vector c0 of the first (angle: arc length)
template <class SH>
DRC_HD inline V3 rw_eval(const SH& s, const Feat& f, const FParam& u, V3* t0, V3* t1, V3* c0) {
  V3 x, a = v3(0, 0, 0), b = v3(0, 0, 0), c = v3(0, 0, 0);
  if (f.kind == kFtSide || f.kind == kFtRim) {
    const double r = s.p0;
    x = v3(r * u.a, r * u.b, f.kind == kFtSide ? u.c : f.s * s.p1);
    a = v3(-u.b, u.a, 0);
    c = v3(-u.a / r, -u.b / r, 0);
    if (f.kind == kFtSide) b = v3(0, 0, 1);
  } else if (f.kind == kFtCap) {
    x = v3(u.a, u.b, f.s * s.p1);
    a = v3(1, 0, 0);
    b = v3(0, 1, 0);
  } else {
    double xl[3];
    int k = 0;
    for (int i = 0; i < 3; ++i) {
      const int fi = f.fix(i);
      xl[i] = fi ? fi * shp(s, i) : (k == 0 ? u.a : u.b);
      if (!fi) {
        if (k == 0) a = v3e(i);
        else b = v3e(i);
        ++k;
      }
    }
    x = v3(xl[0], xl[1], xl[2]);
  }
  *t0 = rot(s.T, a);
  *t1 = rot(s.T, b);
  *c0 = rot(s.T, c);
  return xform(s.T, x);
}
template <class SH>
DRC_HD __forceinline__ void rw_step(const SH& s, const Feat& f, FParam* u, double d0, double d1) {
  if (f.kind == kFtSide || f.kind == kFtRim) {  // rotate the radial vector by the arc d0 (retraction)
    const double w = d0 / s.p0, ca = u->a - w * u->b, sa = u->b + w * u->a, n = 1.0 / sqrt(ca * ca + sa * sa);
    u->a = ca * n;
    u->b = sa * n;
    if (f.kind == kFtSide) u->c += d1;
  } else {
    u->a += d0;
    u->b += d1;
  }
}
// Newton on grad |X_A - X_B|^2 = 0 (unknowns A0 A1 B0 B1; absent ones get
// identity rows); false when degenerate or not converged.
template <class SH>
DRC_HD inline bool rw_newton(const SH& A, const Feat& fA, FParam* uA, const SH& B, const Feat& fB, FParam* uB,
                             V3* XA, V3* XB) {
  const int mA = fA.nparam(), mB = fB.nparam();
  const bool act[4] = {mA > 0, mA > 1, mB > 0, mB > 1};
#pragma unroll 1
  for (int it = 0; it < 20; ++it) {
    V3 tA0, tA1, cA, tB0, tB1, cB;
    *XA = rw_eval(A, fA, *uA, &tA0, &tA1, &cA);
    *XB = rw_eval(B, fB, *uB, &tB0, &tB1, &cB);
    if (mA + mB == 0) return true;
    const V3 D = *XA - *XB;
    const V3 J[4] = {tA0, tA1, -1.0 * tB0, -1.0 * tB1};
    double H[4][5];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) H[i][j] = act[i] && act[j] ? dot(J[i], J[j]) : (i == j ? 1.0 : 0.0);
      H[i][4] = act[i] ? -dot(J[i], D) : 0.0;
    }
    if (act[0]) H[0][0] += dot(D, cA);  // angle curvature (first parameter only)
    if (act[2]) H[2][2] -= dot(D, cB);
#pragma unroll
    for (int c = 0; c < 4; ++c) {  // Gaussian elimination, partial pivoting (swaps by selects)
      double pv = fabs(H[c][c]);
      int p = c;
#pragma unroll
      for (int r = c + 1; r < 4; ++r)
        if (fabs(H[r][c]) > pv) {
          pv = fabs(H[r][c]);
          p = r;
        }
      if (!(pv > kRwPivot)) return false;
#pragma unroll
      for (int r = c + 1; r < 4; ++r)
        if (r == p)
#pragma unroll
          for (int j = 0; j < 5; ++j) {
            const double t = H[c][j];
            H[c][j] = H[r][j];
            H[r][j] = t;
          }
      const double ip = 1.0 / H[c][c];
#pragma unroll
      for (int r = c + 1; r < 4; ++r) {
        const double g = H[r][c] * ip;
#pragma unroll
        for (int j = c; j < 5; ++j) H[r][j] -= g * H[c][j];
      }
    }
    double du[4], mx = 0;
#pragma unroll
    for (int r = 3; r >= 0; --r) {
      double t = H[r][4];
#pragma unroll
      for (int j = r + 1; j < 4; ++j) t -= H[r][j] * du[j];
      du[r] = t / H[r][r];
      mx = fmax(mx, fabs(du[r]));
    }
    rw_step(A, fA, uA, du[0], du[1]);
    rw_step(B, fB, uB, du[2], du[3]);
    if (mx <= kRwStep) {
      *XA = rw_eval(A, fA, *uA, &tA0, &tA1, &cA);
      *XB = rw_eval(B, fB, *uB, &tB0, &tB1, &cB);
      return true;
    }
  }
  return false;
}
// outside the feature's domain: move to the bounding feature (true)
template <class SH>
DRC_HD inline bool rw_domain(const SH& s, Feat* f, const FParam& u) {
  if (f->kind == kFtSide && fabs(u.c) > s.p1) {
    f->kind = kFtRim;
    f->s = u.c > 0 ? 1 : -1;
    return true;
  }
  if (f->kind == kFtCap && u.a * u.a + u.b * u.b > s.p0 * s.p0) {
    f->kind = kFtRim;
    return true;
  }
  if (f->kind == kFtBox) {
    int k = 0;
    for (int i = 0; i < 3; ++i) {
      if (f->fix(i)) continue;
      const double ui = k == 0 ? u.a : u.b;
      if (fabs(ui) > shp(s, i)) {
        f->set_fix(i, ui > 0 ? 1 : -1);
        return true;
      }
      ++k;
    }
  }
  return false;
}
// the outward normal nrm in the normal cone of f at u: -1 impossible, 1
// feature moves to a neighbour, 0 holds
template <class SH>
DRC_HD inline int rw_cone(const SH& s, Feat* f, const FParam& u, V3 nrm) {
  const V3 ax = v3(s.T[2], s.T[5], s.T[8]);
  if (f->kind == kFtBox) {
    const int nfix = (f->fx != 0) + (f->fy != 0) + (f->fz != 0);
    for (int i = 0; i < 3; ++i) {
      const int fi = f->fix(i);
      if (!fi) continue;
      const V3 e = v3(s.T[i], s.T[3 + i], s.T[6 + i]);
      if (fi * dot(nrm, e) < -kRwCone) {
        if (nfix == 1) return -1;  // no face left
        f->set_fix(i, 0);
        return 1;
      }
    }
    return 0;
  }
  if (f->kind == kFtCap) return f->s * dot(nrm, ax) > 0 ? 0 : -1;
  const V3 rad = rot(s.T, v3(u.a, u.b, 0));
  const double a = dot(nrm, rad), b = f->s * dot(nrm, ax);
  if (f->kind == kFtSide) return a > 0 ? 0 : -1;
  if (a < -kRwCone) {
    f->kind = kFtCap;
    return 1;
  }
  if (b < -kRwCone) {
    f->kind = kFtSide;
    return 1;
  }
  return 0;
}
// sharpens (d, pA, pB) in place; false: the estimates stay
template <class SH>
DRC_HD inline __noinline__ bool refine_witness(const SH A, const SH B, double* d, V3* pA, V3* pB) {
  Feat fA, fB;
  const V3 cA = v3(A.T[9], A.T[10], A.T[11]), cB = v3(B.T[9], B.T[10], B.T[11]);
  const V3 xA = rotT(A.T, *pA - cA), xB = rotT(B.T, *pB - cB);
  rw_classify(A, xA, &fA);
  rw_classify(B, xB, &fB);
  FParam uA = rw_params(fA, xA), uB = rw_params(fB, xB);
  const double sgn = *d < 0 ? -1.0 : 1.0;
#pragma unroll 1
  for (int round = 0; round < 4; ++round) {
    V3 XA, XB;
    if (!rw_newton(A, fA, &uA, B, fB, &uB, &XA, &XB)) return false;
    int ca = rw_domain(A, &fA, uA), cb = rw_domain(B, &fB, uB);
    if (!ca && !cb) {
      const V3 D = XB - XA;
      const double L = sqrt(dot(D, D));
      if (!(L > 1e-12)) return false;
      const double sd = sgn * L;
      const V3 n = v3(D.x / sd, D.y / sd, D.z / sd), nb = v3(-n.x, -n.y, -n.z);
      ca = rw_cone(A, &fA, uA, n);
      cb = rw_cone(B, &fB, uB, nb);
      if (ca < 0 || cb < 0) return false;
      if (!ca && !cb) {
        if (!(fabs(sd - *d) <= kRwDMove)) return false;
        *d = sd;
        *pA = XA;
        *pB = XB;
        return true;
      }
    }
    uA = rw_params(fA, rotT(A.T, XA - cA));
    uB = rw_params(fB, rotT(B.T, XB - cB));
  }
  return false;
}

// Lower bound on the distance of two geometries via their swept cores:
// cylinder -> axis segment (radius r), box -> centre point (bounding radius),
// sphere -> centre.  Exact closed form for segment/segment.
template <class SH>
DRC_HD __forceinline__ void core_segment(const SH& s, double bound, V3* a, V3* b, double* rad) {
  V3 c = v3(s.T[9], s.T[10], s.T[11]);
  if (s.type == kCylinder) {
    V3 ax = v3(s.T[2], s.T[5], s.T[8]);
    *a = c - s.p1 * ax;
    *b = c + s.p1 * ax;
  } else {
    *a = c;
    *b = c;
  }
  *rad = bound;
}
// Cylinder/cylinder distance in closed form when the closest points of the
// two axis segments are interior to both: the connecting line is then normal
// to both axes, meets both lateral surfaces, and the swept-core (capsule)
// bound is attained -- the exact distance GJK converges to.  Separated,
// non-parallel pairs only; every other cylinder pair goes to GJK/EPA.
// Oracle twin: cyl_cyl_side in oracle/drc_oracle.c (same operation order).
template <class SH>
DRC_HD __forceinline__ bool cyl_cyl_side(const SH& A, const SH& B, double* d, V3* pA, V3* pB) {
  const V3 ua = v3(A.T[2], A.T[5], A.T[8]), ub = v3(B.T[2], B.T[5], B.T[8]);
  const V3 p1 = v3(A.T[9], A.T[10], A.T[11]) - A.p1 * ua, p2 = v3(B.T[9], B.T[10], B.T[11]) - B.p1 * ub;
  const V3 d1 = (2.0 * A.p1) * ua, d2 = (2.0 * B.p1) * ub, r = p1 - p2;
  const double a = dot(d1, d1), e = dot(d2, d2), b = dot(d1, d2), c = dot(d1, r), f = dot(d2, r);
  const double den = a * e - b * b;
  if (!(den > 1e-12 * a * e)) return false;
  const double s = (b * f - c * e) / den, t = (a * f - b * c) / den;
  if (!(s > 0.0 && s < 1.0 && t > 0.0 && t < 1.0)) return false;
  const V3 c1 = p1 + s * d1, c2 = p2 + t * d2;
  V3 n = c2 - c1;
  const double L = sqrt(dot(n, n)), dd = L - A.p0 - B.p0;
  if (!(dd > 0.0)) return false;
  n = (1.0 / L) * n;
  *pA = c1 + A.p0 * n;
  *pB = c2 - B.p0 * n;
  *d = dd;
  return true;
}
DRC_HD __forceinline__ double seg_seg_dist(V3 p1, V3 q1, V3 p2, V3 q2, V3* c1o = nullptr, V3* c2o = nullptr) {
  V3 d1 = q1 - p1, d2 = q2 - p2, r = p1 - p2;
  double a = dot(d1, d1), e = dot(d2, d2), f = dot(d2, r), s, t;
  if (a <= 1e-30 && e <= 1e-30) {  // two points (box / box cores): the closest points are the points
    if (c1o) {
      *c1o = p1;
      *c2o = p2;
    }
    return sqrt(dot(r, r));
  }
  if (a <= 1e-30) {
    s = 0;
    t = fmin(fmax(f / e, 0.0), 1.0);
  } else {
    double c = dot(d1, r);
    if (e <= 1e-30) {
      t = 0;
      s = fmin(fmax(-c / a, 0.0), 1.0);
    } else {
      double b = dot(d1, d2), den = a * e - b * b;
      s = den > 0 ? fmin(fmax((b * f - c * e) / den, 0.0), 1.0) : 0.0;
      t = (b * s + f) / e;
      if (t < 0) {
        t = 0;
        s = fmin(fmax(-c / a, 0.0), 1.0);
      } else if (t > 1) {
        t = 1;
        s = fmin(fmax((b - c) / a, 0.0), 1.0);
      }
    }
  }
  V3 c1 = p1 + s * d1, c2 = p2 + t * d2, dd = c1 - c2;
  if (c1o) {
    *c1o = c1;
    *c2o = c2;
  }
  return sqrt(dot(dd, dd));
}

// Lower bound on the (signed) distance of two geometries: the swept-core
// (capsule / bounding sphere) distance, raised to the separating-axis value
// along the core closest-point direction n,  min_B n.x - max_A n.x  (the
// geometry lies inside its core's swept volume, so this is never below the
// core bound).
template <class SH>
DRC_HD __forceinline__ double pair_lower_bound(const SH& A, const SH& B, double boundA, double boundB) {
  V3 a0, a1, b0, b1, c1, c2;
  double ra, rb;
  core_segment(A, boundA, &a0, &a1, &ra);
  core_segment(B, boundB, &b0, &b1, &rb);
  const double L = seg_seg_dist(a0, a1, b0, b1, &c1, &c2), pd = L - ra - rb;
  if (!(L > 1e-12)) return pd;
  const V3 n = (1.0 / L) * (c2 - c1);
  const double sat = dot(n, support(B, -1.0 * n)) - dot(n, support(A, n));
  return fmax(pd, sat);
}

}  // namespace drc_amd

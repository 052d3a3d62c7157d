// Scheduling order of a small call's instances: penetration-prone instances
// first.  A small QPIK call's makespan is its tail -- a few instances whose
// narrow phase runs EPA (tens of serial growth steps, 5-10x a typical
// instance) and that a wave happened to take as its second or third instance
// (DESIGN.md "Small batches").  This kernel predicts those instances cheaply
// and writes a queue order that hands them out first; the task / fused kernels
// then take the instance at queue position j as order[b0 + j] (IO::ordered).
// Results do not depend on the order (instances are independent): it moves
// only when each instance starts.
//
// Predictor: some pair that GJK / EPA would run (no sphere; a cylinder pair
// only where the side-to-side closed form does not apply) has a negative
// swept-core lower bound, the broad phase's pair_lower_bound (qpik_device.hpp)
// -- a superset of the instances with an intersecting GJK candidate
// (recall 1 in tools/epa_hint_study.py; FR3 bench workload: 6 % flagged).
// One lane per instance; the joint frames of the 64 lanes in LDS, [frame
// element][lane] (conflict-free); model indices are wave-uniform scalar loads.
#include "kernel_common.hpp"
#include "launch.hpp"

namespace drc_amd {

__global__ void __launch_bounds__(64) order_kernel(const DevModel* __restrict__ M, const IO io, int* __restrict__ cnt,
                                                   int32_t* __restrict__ order) {
  extern __shared__ __attribute__((aligned(16))) double S[];
  const int l = lane_id();
  const int64_t b = int64_t(blockIdx.x) * 64 + l;
  const bool live = b < io.B;
  const int64_t gb = io.b0 + (live ? b : 0), LD = io.ld;
  const int nv = M->nv;
  auto TT = [&](int j, int e) -> double& { return S[(j * 12 + e) * 64 + l]; };
#pragma unroll
  for (int e = 0; e < 12; ++e) TT(0, e) = (e == 0 || e == 4 || e == 8) ? 1.0 : 0.0;
  for (int j = 1; j <= nv; ++j) {
    const double qq = io.q[(j - 1) * LD + gb];
    const double* ax = M->axis[j];
    double Mj[12];
    if (M->jtype[j] == kRevolute) {
      const double c = cos(qq), s = sin(qq), C = 1 - c, x = ax[0], y = ax[1], z = ax[2];
      Mj[0] = c + x * x * C; Mj[1] = x * y * C - z * s; Mj[2] = x * z * C + y * s;
      Mj[3] = y * x * C + z * s; Mj[4] = c + y * y * C; Mj[5] = y * z * C - x * s;
      Mj[6] = z * x * C - y * s; Mj[7] = z * y * C + x * s; Mj[8] = c + z * z * C;
      Mj[9] = Mj[10] = Mj[11] = 0;
    } else {
      Mj[0] = Mj[4] = Mj[8] = 1;
      Mj[1] = Mj[2] = Mj[3] = Mj[5] = Mj[6] = Mj[7] = 0;
      Mj[9] = ax[0] * qq; Mj[10] = ax[1] * qq; Mj[11] = ax[2] * qq;
    }
    double Lj[12], Tp[12], Tj[12];
    tmul(M->jplace[j], Mj, Lj);
    const int p = M->parent[j];
#pragma unroll
    for (int e = 0; e < 12; ++e) Tp[e] = TT(p, e);
    tmul(Tp, Lj, Tj);
#pragma unroll
    for (int e = 0; e < 12; ++e) TT(j, e) = Tj[e];
  }
  bool flag = false;
  for (int s = 0; s < M->ncand_slots; ++s) {
    const int p = M->cand_pair[s], ga = M->pair_a[p], gb_ = M->pair_b[p];
    double TA[12], TB[12], Tp[12];
#pragma unroll
    for (int e = 0; e < 12; ++e) Tp[e] = TT(M->gparent[ga], e);
    tmul(Tp, M->gplace[ga], TA);
#pragma unroll
    for (int e = 0; e < 12; ++e) Tp[e] = TT(M->gparent[gb_], e);
    tmul(Tp, M->gplace[gb_], TB);
    const Shape A{M->gtype[ga], TA, M->gparam[ga][0], M->gparam[ga][1], M->gparam[ga][2]};
    const Shape Bs{M->gtype[gb_], TB, M->gparam[gb_][0], M->gparam[gb_][1], M->gparam[gb_][2]};
    // bounding spheres apart: the pair cannot touch (cheap reject)
    const double ra = A.type == kCylinder ? sqrt(A.p0 * A.p0 + A.p1 * A.p1) : M->gbound[ga];
    const double rb = Bs.type == kCylinder ? sqrt(Bs.p0 * Bs.p0 + Bs.p1 * Bs.p1) : M->gbound[gb_];
    const V3 dc = v3(TA[9] - TB[9], TA[10] - TB[10], TA[11] - TB[11]);
    if (dot(dc, dc) > (ra + rb) * (ra + rb)) continue;
    double d;
    V3 pA, pB;
    if (A.type == kCylinder && Bs.type == kCylinder && cyl_cyl_side(A, Bs, &d, &pA, &pB)) continue;  // closed form
    if (pair_lower_bound(A, Bs, M->gbound[ga], M->gbound[gb_]) < 0.0) flag = true;
  }
  // flagged instances from the front, the others from the back
  const unsigned long long mf = __ballot(live && flag), mu = __ballot(live && !flag);
  int bf = 0, bu = 0;
  if (l == 0) {
    bf = atomicAdd(cnt, __popcll(mf));
    bu = atomicAdd(cnt + 1, __popcll(mu));
  }
  bf = __builtin_amdgcn_readfirstlane(bf);
  bu = __builtin_amdgcn_readfirstlane(bu);
  const unsigned long long below = (1ull << l) - 1;
  if (live) {
    const int64_t pos = flag ? int64_t(bf + __popcll(mf & below)) : io.B - 1 - (bu + __popcll(mu & below));
    order[io.b0 + pos] = static_cast<int32_t>(io.b0 + b);
  }
}

int launch_order_kernel(int64_t B, hipStream_t st, const DevModel* m, int nv, const IO& io, int* cnt, int32_t* order) {
  const size_t lds = static_cast<size_t>(nv + 1) * 12 * 64 * sizeof(double);
  hipLaunchKernelGGL(order_kernel, dim3(static_cast<unsigned>((B + 63) / 64)), dim3(64), lds, st, m, io, cnt, order);
  return hipGetLastError();
}

}  // namespace drc_amd

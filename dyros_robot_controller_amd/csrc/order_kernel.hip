// Scheduling order of a small call's instances: penetration-prone instances
// first.  A small QPIK call's makespan is its tail -- a few instances whose
// narrow phase runs EPA (tens of serial growth steps, 5-10x a typical
// instance) and that a wave happened to take as its second or third instance
// (DESIGN.md "Small batches").  This kernel predicts those instances cheaply
// and writes a queue order that hands them out first, then every other
// instance in index order; the task / fused kernels take queue position j as
// order[b0 + j] (IO::ordered).
// Results do not depend on the order (instances are independent): it moves
// only when each instance starts.
//
// Predictor: some pair that GJK / EPA would run (no sphere; a cylinder pair
// only where the side-to-side closed form does not apply) has a negative
// swept-core lower bound, the broad phase's pair_lower_bound (qpik_device.hpp)
// -- a superset of the instances with an intersecting GJK candidate
// (recall 1 in tools/epa_hint_study.py; FR3 bench workload: 6 % flagged).
#include "kernel_common.hpp"
#include "launch.hpp"

namespace drc_amd {

// One wave per instance: lanes 1..nv form the joints' local transforms, then
// each lane j composes its joint's world frame along its ancestor chain
// (M->anc: the ancestors of j, in index order, are a path from the root, each
// the parent of the next), then one lane per candidate pair (cand_pair slots)
// evaluates the bound.  (A first version with one lane per instance held 64
// instances' frames per wave and ran 64 waves at B = 4 096: 75 us against the
// 80 us the order saves, profiles/r06g_kt_order_b4096.csv.)
__global__ void __launch_bounds__(64) order_kernel(const DevModel* __restrict__ M, const IO io, int* __restrict__ hot_n,
                                                   int32_t* __restrict__ hot_list, uint8_t* __restrict__ hot_flag) {
  __shared__ double Lq[kMaxJoints + 1][12], Tw[kMaxJoints + 1][12];
  const int l = lane_id();
  const int64_t b = blockIdx.x;
  const int64_t gb = io.b0 + b, LD = io.ld;
  const int nv = M->nv;
  if (l >= 1 && l <= nv) {  // local transform of joint l: jplace * motion(q_l)
    const int j = l;
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
    double Lj[12];
    tmul(M->jplace[j], Mj, Lj);
#pragma unroll
    for (int e = 0; e < 12; ++e) Lq[j][e] = Lj[e];
  }
  wsync();
  if (l <= nv) {  // world frame of joint l (0: the world)
    double T[12];
#pragma unroll
    for (int e = 0; e < 12; ++e) T[e] = (e == 0 || e == 4 || e == 8) ? 1.0 : 0.0;
    const uint32_t anc = l > 0 ? M->anc[l] : 0u;
    for (int k = 1; k <= l; ++k)
      if (anc & (1u << (k - 1))) tmul(T, Lq[k], T);
#pragma unroll
    for (int e = 0; e < 12; ++e) Tw[l][e] = T[e];
  }
  wsync();
  bool flag = false;
  for (int s = l; s < M->ncand_slots; s += 64) {
    const int p = M->cand_pair[s], ga = M->pair_a[p], gb_ = M->pair_b[p];
    double TA[12], TB[12];
    tmul(Tw[M->gparent[ga]], M->gplace[ga], TA);
    tmul(Tw[M->gparent[gb_]], M->gplace[gb_], TB);
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
  // a hot instance goes on the hot list (one atomic per hot instance: a few
  // per cent of them; an atomic per instance on one address serialised 4 096
  // of them at the L2, 53 us at B = 4 096, profiles/r06h_kt_order_b4096.csv)
  const bool hot = __ballot(flag) != 0;
  if (l == 0) {
    hot_flag[b] = hot ? 1 : 0;
    if (hot) hot_list[atomicAdd(hot_n, 1)] = static_cast<int32_t>(b);
  }
}

// The queue order from the flags: the hot list first, then every other
// instance in index order (one workgroup: a block-wide exclusive scan of the
// cold flags, in LDS).  Writes order[b0 .. b0 + B) with instance indices
// b0 + b (IO::ordered).
__global__ void __launch_bounds__(1024) order_scan_kernel(int64_t B, int64_t b0, const int* __restrict__ hot_n,
                                                          const int32_t* __restrict__ hot_list,
                                                          const uint8_t* __restrict__ hot_flag,
                                                          int32_t* __restrict__ order) {
  __shared__ int part[1024];
  const int t = threadIdx.x;
  const int64_t per = (B + 1023) / 1024, lo = t * per, hi = lo + per < B ? lo + per : B;
  int cold = 0;
  for (int64_t i = lo; i < hi; ++i) cold += hot_flag[i] ? 0 : 1;
  part[t] = cold;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {  // inclusive scan (Hillis-Steele)
    const int v = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  const int nh = *hot_n;
  int64_t pos = nh + (part[t] - cold);
  for (int64_t i = lo; i < hi; ++i)
    if (!hot_flag[i]) order[b0 + pos++] = static_cast<int32_t>(b0 + i);
  for (int64_t k = t; k < nh; k += 1024) order[b0 + k] = static_cast<int32_t>(b0 + hot_list[k]);
}

int launch_order_kernel(int64_t B, hipStream_t st, const DevModel* m, const IO& io, int* hot_n, int32_t* hot_list,
                        uint8_t* hot_flag, int32_t* order) {
  hipLaunchKernelGGL(order_kernel, dim3(static_cast<unsigned>(B)), dim3(64), 0, st, m, io, hot_n, hot_list, hot_flag);
  if (hipError_t e = hipGetLastError()) return e;
  hipLaunchKernelGGL(order_scan_kernel, dim3(1), dim3(1024), 0, st, B, io.b0, hot_n, hot_list, hot_flag, order);
  return hipGetLastError();
}

}  // namespace drc_amd

// Batched joint-space dynamics on gfx950.
//
// Restates, for B robots per launch:
//   Manipulator::RobotData::updateDynamics   src/manipulator/robot_data.cpp:109-124
//     pinocchio::crba (+ selfadjointView<Upper>), computeGeneralizedGravity,
//     nonLinearEffects, M_inv = DyrosMath::PinvCOD(M), c = nle - g
//   MobileManipulator::RobotData::updateDynamics   src/mobile_manipulator/robot_data.cpp:126-144
//     M~ = S^T M S, M~+ = PinvCOD(M~), g~ = S^T g, nle~ = S^T nle, c~ = S^T (nle - g)
//     with S from robot_data.cpp:22-25,115-120.
//
// Execution model: one 16-lane DPP row per robot, lane j <-> joint j+1, 16
// robots per 256-thread block.  Everything runs in FP64 with spatial algebra in
// the world frame (moments about a per-robot reference point, see dyn_origin):
//   FK (each lane walks its ancestor chain through LDS-staged local transforms)
//   -> body spatial inertia, joint motion axis S_j
//   -> velocity-product accelerations and body forces (RNEA with qdd = 0)
//   -> subtree sums: composite inertia (CRBA) and joint-force sums (nle)
//   -> M column j in registers -> symmetric sweep inversion in registers with
//      DPP row_newbcast broadcasts (no LDS traffic in the inverse).
// PinvCOD's rank decision (column-pivoted QR, |R_ii| > 1e-6 max|R_ii|,
// math_type_define.h:563-570) is certified full rank from
// sigma_min >= 1/||M^-1||_F and |R_00| = max column norm; an instance without the
// certificate is queued and re-solved by a serial COD pseudo-inverse (rare).
// I/O is field-major [field][B]; outputs are staged in LDS and stored as
// 16-instance (128-B) runs.
#include <hip/hip_runtime.h>

#include "dynamics.hpp"
#include "mobile_fk.hpp"
#include "model.hpp"
#include "pinv_cod.hpp"
#include "qpik_device.hpp"

namespace drc_amd {
namespace {

constexpr int kDI = 16;          // robots per block
constexpr int kDT = 16 * kDI;    // threads per block
constexpr double kCodThreshold = 1e-6;   // COD_THRESHOLD (math_type_define.h:7)
constexpr double kCertMargin = 1.0001;

template <int K>
__device__ __forceinline__ double row_bcast(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x150 + K, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x150 + K, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
// k must fold to a constant after unrolling (it selects the DPP control)
__device__ __forceinline__ double row_bcast_k(double v, int k) {
  switch (k) {
    case 0: return row_bcast<0>(v);
    case 1: return row_bcast<1>(v);
    case 2: return row_bcast<2>(v);
    case 3: return row_bcast<3>(v);
    case 4: return row_bcast<4>(v);
    case 5: return row_bcast<5>(v);
    case 6: return row_bcast<6>(v);
    case 7: return row_bcast<7>(v);
    case 8: return row_bcast<8>(v);
    case 9: return row_bcast<9>(v);
    case 10: return row_bcast<10>(v);
    case 11: return row_bcast<11>(v);
    case 12: return row_bcast<12>(v);
    case 13: return row_bcast<13>(v);
    case 14: return row_bcast<14>(v);
    default: return row_bcast<15>(v);
  }
}
__device__ __forceinline__ double row_sum(double v) {
#pragma unroll
  for (int s = 1; s < 16; s <<= 1) v += __shfl_xor(v, s, 16);
  return v;
}
__device__ __forceinline__ double row_max(double v) {
#pragma unroll
  for (int s = 1; s < 16; s <<= 1) v = fmax(v, __shfl_xor(v, s, 16));
  return v;
}

// spatial vectors: motion (w, v) / force (n, f), moments about the reference point
struct Sp {
  V3 a, b;
};
__device__ __forceinline__ Sp sp_ld(const double* p) { return Sp{ld3(p), ld3(p + 3)}; }
__device__ __forceinline__ void sp_st(double* p, const Sp& s) {
  st3(p, s.a);
  st3(p + 3, s.b);
}
__device__ __forceinline__ double sp_dot(const Sp& m, const Sp& f) { return dot(m.a, f.a) + dot(m.b, f.b); }
// motion x motion
__device__ __forceinline__ Sp crm(const Sp& x, const Sp& y) {
  return Sp{cross(x.a, y.a), cross(x.a, y.b) + cross(x.b, y.a)};
}
// motion x* force
__device__ __forceinline__ Sp crf(const Sp& x, const Sp& f) {
  return Sp{cross(x.a, f.a) + cross(x.b, f.b), cross(x.a, f.b)};
}
// rigid-body inertia about the reference point: mass m, first moment h = m c,
// rotational inertia Io (xx yy zz xy xz yz) about the point
struct SpI {
  double m;
  V3 h;
  double I[6];
};
__device__ __forceinline__ V3 sym_mul(const double* I, V3 w) {
  return v3(I[0] * w.x + I[3] * w.y + I[4] * w.z, I[3] * w.x + I[1] * w.y + I[5] * w.z,
            I[4] * w.x + I[5] * w.y + I[2] * w.z);
}
__device__ __forceinline__ Sp inertia_mul(const SpI& I, const Sp& m) {
  return Sp{sym_mul(I.I, m.a) + cross(I.h, m.b), I.m * m.b - cross(I.h, m.a)};
}

// LDS layout (doubles), sized from the model at launch
struct DynLayout {
  int n, na, no;      // joints, actuated dof, output dim
  int q, qd, vec, veca, U;
  int L, P, body, S, f, F;   // phase A (U region)
  int M, Ma, X;              // phase B (U region)
  int W, wlen;               // fallback workspace
  int total;
};
__host__ __device__ inline DynLayout dyn_layout(int n, int na, bool act, bool fallback) {
  DynLayout d{};
  d.n = n;
  d.na = na;
  d.no = act ? na : n;
  int o = 0;
  d.q = o; o += n * kDI;
  d.qd = o; o += n * kDI;
  d.vec = o; o += 3 * n * kDI;
  d.veca = o; o += act ? 3 * na * kDI : 0;
  d.U = o;
  // phase A: [inst][joint][k]
  int a = o;
  d.L = a;                       // local transforms (12), dead after FK; shares with f, F
  d.f = a; d.F = a + 6 * n * kDI;
  a += 12 * n * kDI;
  d.P = a; a += 3 * n * kDI;
  d.body = a; a += 10 * n * kDI;
  d.S = a; a += 6 * n * kDI;
  // phase B: [field][inst]
  int b = o;
  d.M = b; b += n * n * kDI;
  d.Ma = b; b += act ? na * na * kDI : 0;
  d.X = b; b += d.no * d.no * kDI;
  o = a > b ? a : b;
  d.wlen = 3 * d.no * d.no + 3 * d.no;
  d.W = o; o += fallback ? d.wlen * kDI : 0;
  d.total = o;
  return d;
}

struct DynIO {
  int64_t B;
  const double* q;
  const double* qd;
  double *M, *Minv, *g, *nle, *c;
  int* list;      // fallback queue (count at list[0], entries from list[1])
  // joint torque step (kTorque): controlled block [bs, bs + bn) of the joints
  const double *qt, *qdt, *qddt;
  double dt;
  int bs, bn;
  double kp[kMaxJoints], kv[kMaxJoints];
  double* tau;
};

enum DynMode { kDyn = 0, kDynActuated = 1, kTorque = 2 };

template <int MODE, bool FALLBACK>
__global__ void __launch_bounds__(kDT) __attribute__((amdgpu_waves_per_eu(4, 8))) dyn_kernel(const DevModel* __restrict__ M0, const DynIO io) {
  constexpr bool ACT = MODE == kDynActuated, TQ = MODE == kTorque;
  extern __shared__ double lds[];
  const int tid = threadIdx.x, g = tid >> 4, j = tid & 15, J = j + 1;
  const int n = M0->nv;
  const int na = ACT ? M0->n_arm + M0->n_wheel : n;
  const DynLayout L = dyn_layout(n, na, ACT, FALLBACK);
  const int no = L.no;
  const int64_t B = io.B;
  int64_t b;  // this row's instance (-1: none)
  if (FALLBACK) {
    const int cnt = io.list[0];
    const int64_t k = static_cast<int64_t>(blockIdx.x) * kDI + g;
    if (static_cast<int64_t>(blockIdx.x) * kDI >= cnt) return;  // whole block idle (uniform)
    b = k < cnt ? io.list[1 + k] : -1;
  } else {
    b = static_cast<int64_t>(blockIdx.x) * kDI + g;
    if (b >= B) b = -1;
  }
  double* sq = lds + L.q;
  double* sqd = lds + L.qd;
  // ---- inputs: q, qd [D][B] -> LDS [D][kDI] --------------------------------
  if (FALLBACK) {
    for (int f = j; f < n; f += 16) {
      sq[f * kDI + g] = b >= 0 ? io.q[f * B + b] : 0.0;
      sqd[f * kDI + g] = (b >= 0 && io.qd) ? io.qd[f * B + b] : 0.0;
    }
  } else {
    const int64_t b0 = static_cast<int64_t>(blockIdx.x) * kDI;
    for (int idx = tid; idx < n * kDI; idx += kDT) {
      const int f = idx >> 4, t = idx & 15;
      const bool in = b0 + t < B;
      sq[idx] = in ? io.q[f * B + b0 + t] : 0.0;
      sqd[idx] = (in && io.qd) ? io.qd[f * B + b0 + t] : 0.0;
    }
  }
  double* svec = lds + L.vec;
  if (TQ) {
    __syncthreads();  // q, qd staged by other lanes
    // joint-space acceleration command of the controlled block -> svec row n + j
    // (moveJointTorqueStep robot_controller.cpp:115-125; MoMa arm block
    // mobile_manipulator/robot_controller.cpp:103-118)
    if (j < io.bn) {
      const int jj = io.bs + j;
      double acc = 0;
      if (b >= 0) {
        if (io.qddt) {
          acc = io.qddt[j * B + b];
        } else {
          const double qv = sq[jj * kDI + g], qdv = sqd[jj * kDI + g], qdt = io.qdt[j * B + b];
          const double qt = io.qt ? io.qt[j * B + b] : qv + io.dt * qdt;   // fr3_controller.cpp:133
          acc = io.kp[j] * (qt - qv) + io.kv[j] * (qdt - qdv);
        }
      }
      svec[(n + j) * kDI + g] = acc;
    }
  }
  __syncthreads();
  const bool on = j < n;
  const uint32_t ancJ = on ? M0->anc[J] : 0u;
  // ---- local joint transforms L_J = jplace_J * X_J(q_J) -> LDS --------------
  double* sL = lds + L.L + (g * n) * 12;
  if (on) {
    const double qq = sq[j * kDI + g];
    const double* ax = M0->axis[J];
    double Xj[12];
    if (M0->jtype[J] == kRevolute) {
      const double c = cos(qq), s = sin(qq), C = 1 - c, x = ax[0], y = ax[1], z = ax[2];
      Xj[0] = c + x * x * C; Xj[1] = x * y * C - z * s; Xj[2] = x * z * C + y * s;
      Xj[3] = y * x * C + z * s; Xj[4] = c + y * y * C; Xj[5] = y * z * C - x * s;
      Xj[6] = z * x * C - y * s; Xj[7] = z * y * C + x * s; Xj[8] = c + z * z * C;
      Xj[9] = Xj[10] = Xj[11] = 0;
    } else {
      Xj[0] = Xj[4] = Xj[8] = 1;
      Xj[1] = Xj[2] = Xj[3] = Xj[5] = Xj[6] = Xj[7] = 0;
      Xj[9] = ax[0] * qq; Xj[10] = ax[1] * qq; Xj[11] = ax[2] * qq;
    }
    double Lj[12];
    tmul(M0->jplace[J], Xj, Lj);
#pragma unroll
    for (int i = 0; i < 12; ++i) sL[j * 12 + i] = Lj[i];
  }
  __syncthreads();
  // ---- FK: oMi_J = prod over the ancestor chain (root first) ------------------
  double T[12] = {1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0};
  for (int k = 1; k <= n; ++k) {
    if ((ancJ >> (k - 1)) & 1u) {
      double Lk[12];
#pragma unroll
      for (int i = 0; i < 12; ++i) Lk[i] = sL[(k - 1) * 12 + i];
      tmul(T, Lk, T);
    }
  }
  double* sP = lds + L.P + (g * n) * 3;
  if (on) st3(sP + 3 * j, v3(T[9], T[10], T[11]));
  __syncthreads();  // sL dead from here (f, F reuse it)
  const int ref = M0->dyn_origin;
  const V3 o = ref > 0 ? ld3(sP + 3 * (ref - 1)) : v3(0, 0, 0);
  const V3 p = v3(T[9], T[10], T[11]) - o;
  // ---- body inertia about the reference point, joint motion axis -----------
  const double* bi = M0->inertia[on ? J : 0];
  SpI I;
  {
    const double m = bi[0];
    const V3 cw = rot(T, v3(bi[1], bi[2], bi[3])) + p;
    // Iw = R Ic R^T
    const double Ic[9] = {bi[4], bi[7], bi[8], bi[7], bi[5], bi[9], bi[8], bi[9], bi[6]};
    double RI[9];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) RI[3 * r + c] = T[3 * r] * Ic[c] + T[3 * r + 1] * Ic[3 + c] + T[3 * r + 2] * Ic[6 + c];
    double Iw[9];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) Iw[3 * r + c] = RI[3 * r] * T[3 * c] + RI[3 * r + 1] * T[3 * c + 1] + RI[3 * r + 2] * T[3 * c + 2];
    const double cc = dot(cw, cw);
    I.m = m;
    I.h = m * cw;
    I.I[0] = Iw[0] + m * (cc - cw.x * cw.x);
    I.I[1] = Iw[4] + m * (cc - cw.y * cw.y);
    I.I[2] = Iw[8] + m * (cc - cw.z * cw.z);
    I.I[3] = Iw[1] - m * cw.x * cw.y;
    I.I[4] = Iw[2] - m * cw.x * cw.z;
    I.I[5] = Iw[5] - m * cw.y * cw.z;
  }
  const V3 z = rot(T, ld3(M0->axis[on ? J : 1]));
  const bool rev = M0->jtype[on ? J : 1] == kRevolute;
  const Sp SJ = rev ? Sp{z, cross(p, z)} : Sp{v3(0, 0, 0), z};
  double* sB = lds + L.body + (g * n) * 10;
  double* sS = lds + L.S + (g * n) * 6;
  if (on) {
    sB[10 * j] = I.m;
    st3(sB + 10 * j + 1, I.h);
#pragma unroll
    for (int i = 0; i < 6; ++i) sB[10 * j + 4 + i] = I.I[i];
    sp_st(sS + 6 * j, SJ);
  }
  __syncthreads();
  // ---- RNEA, qdd = 0: body velocity V, bias acceleration A (gravity as a
  //      base acceleration), body force f = I A + V x* I V -------------------
  const V3 ag = v3(0, 0, 9.81);  // -pinocchio::Model::gravity981
  double* sf = lds + L.f + (g * n) * 6;
  double* sF = lds + L.F + (g * n) * 6;
  if (!TQ) {
    Sp V{v3(0, 0, 0), v3(0, 0, 0)}, A{v3(0, 0, 0), ag};
    for (int k = 1; k <= n; ++k) {
      if ((ancJ >> (k - 1)) & 1u) {
        const Sp Sk = sp_ld(sS + 6 * (k - 1));
        const double w = sqd[(k - 1) * kDI + g];
        const Sp vk{w * Sk.a, w * Sk.b};
        const Sp x = crm(V, vk);
        A = Sp{A.a + x.a, A.b + x.b};
        V = Sp{V.a + vk.a, V.b + vk.b};
      }
    }
    const Sp IA = inertia_mul(I, A), IV = inertia_mul(I, V), x = crf(V, IV);
    if (on) sp_st(sf + 6 * j, Sp{IA.a + x.a, IA.b + x.b});
  }
  __syncthreads();
  // ---- subtree sums: composite inertia Ic_J, joint force; g, nle, c --------
  SpI Ic{0, v3(0, 0, 0), {0, 0, 0, 0, 0, 0}};
  Sp Fs{v3(0, 0, 0), v3(0, 0, 0)};
  for (int k = 1; k <= n; ++k) {
    if (on && ((M0->anc[k] >> j) & 1u)) {
      const double* bk = sB + 10 * (k - 1);
      Ic.m += bk[0];
      Ic.h = Ic.h + ld3(bk + 1);
#pragma unroll
      for (int i = 0; i < 6; ++i) Ic.I[i] += bk[4 + i];
      if (!TQ) {
        const Sp fk = sp_ld(sf + 6 * (k - 1));
        Fs = Sp{Fs.a + fk.a, Fs.b + fk.b};
      }
    }
  }
  const double nleJ = sp_dot(SJ, Fs);
  const double gJ = sp_dot(SJ, Sp{cross(Ic.h, ag), Ic.m * ag});
  const Sp FJ = inertia_mul(Ic, SJ);
  __syncthreads();  // every lane is done reading sf before sF (aliased region) is written
  if (on) {
    sp_st(sF + 6 * j, FJ);
    if (!TQ) {
      svec[(0 * n + j) * kDI + g] = gJ;
      svec[(1 * n + j) * kDI + g] = nleJ;
      svec[(2 * n + j) * kDI + g] = nleJ - gJ;
    }
  }
  __syncthreads();
  // ---- M column J: M_IJ = S_I . (Ic_J S_J) for I ancestor-or-self of J,
  //      S_J . (Ic_I S_I) for J an ancestor of I --------------------------------
  double a[kMaxJoints];
#pragma unroll
  for (int i = 0; i < kMaxJoints; ++i) {
    a[i] = 0;
    if (i < n && on) {
      if ((ancJ >> i) & 1u)
        a[i] = sp_dot(sp_ld(sS + 6 * i), FJ);
      else if ((M0->anc[i + 1] >> j) & 1u)
        a[i] = sp_dot(SJ, sp_ld(sF + 6 * i));
    }
  }
  if (TQ) {
    // tau_J = sum_I M_JI acc_I + g_J over the block (M symmetric: column J = row J)
    const int s0 = io.bs, bn = io.bn;
    if (on && j >= s0 && j < s0 + bn) {
      double t = gJ;
#pragma unroll
      for (int i = 0; i < kMaxJoints; ++i)
        if (i >= s0 && i < s0 + bn) t = fma(a[i], svec[(n + i - s0) * kDI + g], t);
      svec[(2 * n + j - s0) * kDI + g] = t;
    }
    __syncthreads();
    const int64_t b0 = static_cast<int64_t>(blockIdx.x) * kDI;
    for (int idx = tid; idx < bn * kDI; idx += kDT) {
      const int f = idx >> 4, t = idx & 15;
      if (b0 + t < B) io.tau[f * B + b0 + t] = svec[2 * n * kDI + idx];
    }
    return;
  }
  __syncthreads();  // phase A dead: phase B overwrites the union
  double* sM = lds + L.M;
#pragma unroll
  for (int i = 0; i < kMaxJoints; ++i)
    if (i < n && on) sM[(i * n + j) * kDI + g] = a[i];
  if (ACT) {
    // S (D x A): arm block identity, wheel block identity, virtual block Rz(yaw) J_mobile
    __syncthreads();
    const int vs = M0->virtual_start, ms = M0->mani_start, ws = M0->mobi_start;
    const int am = M0->act_mani_start, aw = M0->act_mobi_start, W = M0->n_wheel, nar = M0->n_arm;
    const double yaw = sq[(vs + 2) * kDI + g], cy = cos(yaw), sy = sin(yaw);
    // J_mobile at this robot's wheel positions (caster: steer dependent)
    double jm[3][kMaxWheels];
    {
      double wp[kMaxWheels];
#pragma unroll
      for (int w = 0; w < kMaxWheels; ++w) wp[w] = w < W ? sq[(ws + w) * kDI + g] : 0.0;
      mobile_fk(M0, wp, jm);
    }
    // lane's actuated column: rows/weights of S e_j (<= 4 nonzeros)
    int rr[4] = {0, 0, 0, 0};
    double rw[4] = {0, 0, 0, 0};
    if (j < na) {
      if (j >= am && j < am + nar) {
        rr[0] = ms + (j - am);
        rw[0] = 1;
      } else if (j >= aw && j < aw + W) {
        const int w = j - aw;
        double j0 = 0, j1 = 0, j2 = 0;
#pragma unroll
        for (int k = 0; k < kMaxWheels; ++k)
          if (k == w) j0 = jm[0][k], j1 = jm[1][k], j2 = jm[2][k];
        rr[0] = ws + w; rw[0] = 1;
        rr[1] = vs;     rw[1] = cy * j0 - sy * j1;
        rr[2] = vs + 1; rw[2] = sy * j0 + cy * j1;
        rr[3] = vs + 2; rw[3] = j2;
      }
    }
    // t = M S e_j (D) -> reuse the lane's a[]; then M~ column = S^T t
    double t[kMaxJoints];
#pragma unroll
    for (int i = 0; i < kMaxJoints; ++i) {
      t[i] = 0;
      if (i < n && j < na)
#pragma unroll
        for (int e = 0; e < 4; ++e) t[i] += rw[e] * sM[(i * n + rr[e]) * kDI + g];
    }
    // vectors: S^T v for g, nle, c
    double* sveca = lds + L.veca;
    if (j < na)
      for (int v = 0; v < 3; ++v) {
        double s = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) s += rw[e] * svec[(v * n + rr[e]) * kDI + g];
        sveca[(v * na + j) * kDI + g] = s;
      }
    // (S^T t)_b for every actuated row b: row b of S^T is column b of S
    double* sMa = lds + L.Ma;
    for (int bb = 0; bb < na; ++bb) {
      double s = 0;
      if (bb >= am && bb < am + nar) {
        const int r0 = ms + (bb - am);
#pragma unroll
        for (int i = 0; i < kMaxJoints; ++i) s += i == r0 ? t[i] : 0.0;
      } else {
        const int w = bb - aw;
        double j0 = 0, j1 = 0, j2 = 0;
#pragma unroll
        for (int k = 0; k < kMaxWheels; ++k)
          if (k == w) j0 = jm[0][k], j1 = jm[1][k], j2 = jm[2][k];
        const double w0 = cy * j0 - sy * j1, w1 = sy * j0 + cy * j1;
#pragma unroll
        for (int i = 0; i < kMaxJoints; ++i)
          s += i == ws + w ? t[i] : (i == vs ? w0 * t[i] : (i == vs + 1 ? w1 * t[i] : (i == vs + 2 ? j2 * t[i] : 0.0)));
      }
      if (j < na) sMa[(bb * na + j) * kDI + g] = s;
    }
    __syncthreads();
    // M~ is symmetric: the lane's column j is row j
#pragma unroll
    for (int i = 0; i < kMaxJoints; ++i) a[i] = (i < na && j < na) ? sMa[(i * na + j) * kDI + g] : 0.0;
  }
  // ---- inverse: symmetric sweep on the register-resident columns -----------
  double cn2 = 0;
#pragma unroll
  for (int i = 0; i < kMaxJoints; ++i) cn2 += a[i] * a[i];
  const double maxcol = sqrt(row_max(cn2));
  bool pd = true;
#pragma unroll
  for (int k = 0; k < kMaxJoints; ++k) {
    if (k < no) {
      double ck[kMaxJoints];
#pragma unroll
      for (int i = 0; i < kMaxJoints; ++i) ck[i] = row_bcast_k(a[i], k);
      const double d = ck[k];
      pd = pd && d > 0;
      const double inv = 1.0 / d;
      const double tk = a[k] * inv;
      const bool piv = j == k;
#pragma unroll
      for (int i = 0; i < kMaxJoints; ++i)
        if (i != k) a[i] = piv ? ck[i] * inv : fma(-ck[i], tk, a[i]);
      a[k] = piv ? -inv : tk;
    }
  }
  double xf2 = 0;
#pragma unroll
  for (int i = 0; i < kMaxJoints; ++i) {
    a[i] = -a[i];
    if (j < no) xf2 += a[i] * a[i];
  }
  xf2 = row_sum(xf2);
  // full rank certified: |R_ii| >= sigma_min >= 1/||M^-1||_F, |R_00| <= max column norm
  const bool cert = pd && maxcol > 0 && 1.0 / (sqrt(xf2) * maxcol) > kCodThreshold * kCertMargin;
  double* sX = lds + L.X;
#pragma unroll
  for (int i = 0; i < kMaxJoints; ++i)
    if (i < no && j < no) sX[(i * no + j) * kDI + g] = a[i];
  if (FALLBACK) {
    __syncthreads();
    if (j == 0 && b >= 0)
      pinv_cod_serial(lds + (ACT ? L.Ma : L.M) + g, no, kDI, sX + g, lds + L.W + g * L.wlen);
    __syncthreads();
    if (b >= 0 && io.Minv)
      for (int f = j; f < no * no; f += 16) io.Minv[f * B + b] = sX[f * kDI + g];
    return;
  }
  if (io.Minv && j == 0 && b >= 0 && !cert) {
    const int slot = atomicAdd(io.list, 1);
    io.list[1 + slot] = static_cast<int>(b);
  }
  __syncthreads();
  // ---- outputs: LDS [field][kDI] -> 16-instance runs ---------------------------
  const int64_t b0 = static_cast<int64_t>(blockIdx.x) * kDI;
  auto store = [&](double* out, const double* src, int F) {
    if (!out) return;
    for (int idx = tid; idx < F * kDI; idx += kDT) {
      const int f = idx >> 4, t = idx & 15;
      if (b0 + t < B) out[f * B + b0 + t] = src[idx];
    }
  };
  const double* vsrc = lds + (ACT ? L.veca : L.vec);
  store(io.M, lds + (ACT ? L.Ma : L.M), no * no);
  store(io.Minv, sX, no * no);
  store(io.g, vsrc, no);
  store(io.nle, vsrc + no * kDI, no);
  store(io.c, vsrc + 2 * no * kDI, no);
}

template <int MODE, bool FB>
int launch_one(const DevModel* d_model, const DynLayout& L, int64_t blocks, const DynIO& io, hipStream_t st) {
  const size_t lds = static_cast<size_t>(L.total) * sizeof(double);
  if (lds > 65536 &&
      hipFuncSetAttribute(reinterpret_cast<const void*>(&dyn_kernel<MODE, FB>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)) != hipSuccess)
    return 2;
  hipLaunchKernelGGL((dyn_kernel<MODE, FB>), dim3(static_cast<unsigned>(blocks)), dim3(kDT), lds, st, d_model, io);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

template <int MODE>
int launch_pair(const DevModel* d_model, int n, int na, int64_t B, const DynIO& io, hipStream_t st) {
  const int64_t blocks = (B + kDI - 1) / kDI;
  if (blocks > 0x7fffffff) return 1;
  if (io.Minv && hipMemsetAsync(io.list, 0, sizeof(int), st) != hipSuccess) return 2;
  constexpr bool ACT = MODE == kDynActuated;
  if (int rc = launch_one<MODE, false>(d_model, dyn_layout(n, na, ACT, false), blocks, io, st)) return rc;
  // re-solve the uncertified instances (queued by the first kernel); blocks
  // past the queue length exit at once
  if (io.Minv)
    if (int rc = launch_one<MODE, true>(d_model, dyn_layout(n, na, ACT, true), blocks, io, st)) return rc;
  return 0;
}

}  // namespace

int dyn_lds_bytes(int n, int na, bool act, bool fallback) {
  return dyn_layout(n, na, act, fallback).total * static_cast<int>(sizeof(double));
}

int launch_dynamics(const DevModel* d_model, const DevModel& host, bool act, int64_t B, const double* q,
                    const double* qd, double* M, double* Minv, double* g, double* nle, double* c, int* list,
                    hipStream_t st) {
  DynIO io{};
  io.B = B; io.q = q; io.qd = qd;
  io.M = M; io.Minv = Minv; io.g = g; io.nle = nle; io.c = c; io.list = list;
  const int n = host.nv, na = act ? host.n_arm + host.n_wheel : host.nv;
  return act ? launch_pair<kDynActuated>(d_model, n, na, B, io, st) : launch_pair<kDyn>(d_model, n, na, B, io, st);
}

int launch_torque_step(const DevModel* d_model, const DevModel& host, int64_t B, const double* q, const double* qd,
                       const double* q_target, const double* qdot_target, const double* qddot_target, double dt,
                       const double* kp, const double* kv, double* tau, hipStream_t st) {
  DynIO io{};
  io.B = B; io.q = q; io.qd = qd;
  io.qt = q_target; io.qdt = qdot_target; io.qddt = qddot_target; io.dt = dt;
  io.bs = host.kind == 1 ? host.mani_start : 0;
  io.bn = host.kind == 1 ? host.n_arm : host.nv;
  for (int i = 0; i < kMaxJoints; ++i) {
    io.kp[i] = i < io.bn ? kp[i] : 0.0;
    io.kv[i] = i < io.bn ? kv[i] : 0.0;
  }
  io.tau = tau;
  const int64_t blocks = (B + kDI - 1) / kDI;
  if (blocks > 0x7fffffff) return 1;
  return launch_one<kTorque, false>(d_model, dyn_layout(host.nv, host.nv, false, false), blocks, io, st);
}

}  // namespace drc_amd

// Device-side definitions shared by the kernel translation units (task,
// QP, QPID) and the host API: kernel parameters, the per-launch IO block,
// instance sequencing, compile-time QP shapes and small serial helpers.
// MI355X-native batched QP-IK: one wavefront per robot instance.
//
// Hot path of the reference (SURVEY.md §3 call stacks A and C), fused into a
// single kernel per control cycle:
//   FK / LWA frame Jacobian        robot_data.cpp:101-107,392-402
//   task error (+ cubic profile)   math_type_define.h:633-687, robot_controller.cpp:292-317
//   manipulability + gradient      robot_data.cpp:519-553 (MoMa :439-475)
//   min self-distance + gradient   robot_data.cpp:424-494 (hpp-fcl GJK/EPA semantics)
//   QP assembly                    QP_IK.cpp:69-131 (MoMa QP_IK.cpp:59-128), QP_base.h:202-227
//   QP solve                       QP_base.h:100-180 -> OSQP ADMM (+ polish) restated
//   zero-on-failure                QP_IK.cpp:53-67
//
// HBM layout: every batched array is field-major [F][B] so each field is a
// contiguous, coalesced stream over the batch.  Model constants (~12 KB)
// stay in L2/scalar cache; per-instance working state lives in LDS.
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../../include/drc_amd.h"
#include "mobile_fk.hpp"
#include "model.hpp"
#include "pinv_cod.hpp"
#include "qpik_device.hpp"
#include "instrument.hpp"

namespace drc_amd {

// Kernel parameters, passed by value.  LDS offsets (in doubles) are laid out
// by the host from the model dimensions (see plan_layout()).
struct KParams {
  double kp[6], kv[6], ff, alpha_cbf, w_reg, slack_w, man_min, dist_min;
  double t, t0, duration;
  double frame_place[12];
  int frame_joint, mode, stages;
  int nv, nx, ng, np, na, m, narm, c0;
  int xcd_map;                         // XCD-aware instance order (grid % 8 == 0)
  int rJac, rMan, rDist, rXdd, rQ, rLen;  // per-instance task record (doubles)
  int problem;                         // 0 QPIK, 1 QPID (torque-level QP)
  int rQd, rBias, rMgd, rDgd;          // QPID extras of the task record
  int nbuf;                            // polish work-vector stride (>= ncap)
  int ncap;                            // largest polish KKT the LDS plan holds (nx + ng, or 48 for QPID)
  drc_solver_settings s;
  // persistent QP region
  int oP, oG, oQ, oAB, oL, oU, oD, oE, oRho, oX, oZ, oY, oDY, oXT, oZT, oT1, oT2, oRed, oSc;
  int oDi, oEi;  // D^-1 and E^-1 beside the scaling (OSQP scaling.c keeps Dinv / Einv)
  int oBc;  // max(32, nx + ng) doubles: vectors broadcast through LDS (ADMM passes, polish KKT sweeps)
  // union region (kinematics | K^-1 | polish)
  int oU0;
  int oHi;  // whole-body polish: cached rows of (P + delta I)^-1 (persistent, nx * nx), -1 if unused
  int kT, kZ, kTe, kJ, kTg, kq, kqd, kA6, kAi, kW, kPart, kPd, kPf, kCand, kxdd, kmg, kdg, kJt, kSv, kScr, kEpa;
  int kJd, kDa, kVf, kX6, kBias, kMq, kGq;  // QPID: Jdot, arm-only Jdot, S eta, 6x6 scratch, bias | M, g
  int kGdv;                                 // QPID stage: grad_dot vectors
  int cf;                                   // closed-form controller: 1 CLIK, 2 OSF (task_kernel<2>)
  int kCf;                                  // its LDS work area
  int lds_doubles;
};


// diagnostic phase stamps: instrument.hpp (compile to nothing unless -DDRC_PHASE_TIMING)

// scalar slots in the oSc region
enum { SC_C = 0, SC_RHO, SC_MAN, SC_DIST, SC_PAIR, SC_PRI, SC_DUA, SC_EPSP, SC_EPSD, SC_PRIS, SC_DUAS,
       SC_NAX, SC_NZ, SC_NPX, SC_NATY, SC_NQ, SC_NF, SC_NR, SC_WIN, SC_PFAIL, SC_HIV, SC_HOW, SC_CINV, SC_COUNT };
// Parity mode tries the certified polish at every termination check, but only
// until this many attempts failed on a not-yet-converged iterate; after that
// only at convergence (bounds the cost of slow or non-converging instances —
// the oracle makes the same decisions, oracle/drc_oracle.c:POLISH_MAX_EARLY)
constexpr int kPolishMaxEarly = 4;
// ... and at convergence (eps_abs / eps_rel met) until this many attempts in
// total failed; after that only the tight ADMM fallback (eps_fallback) ends it
constexpr int kPolishMaxTotal = 12;

// ------------------------------------------------------------------------
// small serial helpers (lane 0)
// ------------------------------------------------------------------------
// Serial 6x6 kernels run by one lane; every work array lives in LDS
// (ws, 160 doubles) so nothing is a dynamically indexed private array.
__device__ double det_lu6(const double* A, double* M) {
  for (int i = 0; i < 36; ++i) M[i] = A[i];
  double det = 1;
  for (int c = 0; c < 6; ++c) {
    int p = c;
    for (int r = c + 1; r < 6; ++r)
      if (fabs(M[r * 6 + c]) > fabs(M[p * 6 + c])) p = r;
    if (M[p * 6 + c] == 0) return 0;
    if (p != c) {
      for (int j = 0; j < 6; ++j) {
        double t = M[c * 6 + j];
        M[c * 6 + j] = M[p * 6 + j];
        M[p * 6 + j] = t;
      }
      det = -det;
    }
    det *= M[c * 6 + c];
    for (int r = c + 1; r < 6; ++r) {
      double f = M[r * 6 + c] / M[c * 6 + c];
      for (int j = c; j < 6; ++j) M[r * 6 + j] -= f * M[c * 6 + j];
    }
  }
  return det;
}

// column-pivoted Householder QR rank with |R_ii| > 1e-6 max|R_ii| (Eigen COD)
__device__ int rank_cpqr6(const double* A, double* ws) {
  double *M = ws, *cn = ws + 36, *piv = ws + 42, *v = ws + 48;
  double maxpiv = 0;
  for (int i = 0; i < 36; ++i) M[i] = A[i];
  for (int k = 0; k < 6; ++k) {
    for (int j = k; j < 6; ++j) {
      double s = 0;
      for (int i = k; i < 6; ++i) s += M[i * 6 + j] * M[i * 6 + j];
      cn[j] = s;
    }
    int p = k;
    for (int j = k + 1; j < 6; ++j)
      if (cn[j] > cn[p]) p = j;
    if (p != k)
      for (int i = 0; i < 6; ++i) {
        double t = M[i * 6 + k];
        M[i * 6 + k] = M[i * 6 + p];
        M[i * 6 + p] = t;
      }
    double nrm = sqrt(cn[p]);
    piv[k] = nrm;
    maxpiv = fmax(maxpiv, nrm);
    if (nrm == 0) {
      for (int r = k + 1; r < 6; ++r) piv[r] = 0;
      break;
    }
    double alpha = M[k * 6 + k] > 0 ? -nrm : nrm, vn = 0;
    for (int i = k; i < 6; ++i) v[i] = M[i * 6 + k];
    v[k] -= alpha;
    for (int i = k; i < 6; ++i) vn += v[i] * v[i];
    if (vn > 0)
      for (int j = k; j < 6; ++j) {
        double s = 0;
        for (int i = k; i < 6; ++i) s += v[i] * M[i * 6 + j];
        s = 2 * s / vn;
        for (int i = k; i < 6; ++i) M[i * 6 + j] -= s * v[i];
      }
  }
  int r = 0;
  for (int k = 0; k < 6; ++k) r += piv[k] > 1e-6 * maxpiv;
  return r;
}

// DyrosMath::PinvCOD of the symmetric PSD 6x6 JJ^T (math_type_define.h:563)
__device__ void pinv_cod6(const double* A, double* X, double* ws) {
  int r = rank_cpqr6(A, ws);
  double* L = ws;  // rank work is dead now
  double* e = ws + 36;
  bool ok = r == 6;
  if (ok) {
    for (int i = 0; i < 36; ++i) L[i] = A[i];
    for (int j = 0; j < 6 && ok; ++j) {
      double s = L[j * 6 + j];
      for (int k = 0; k < j; ++k) s -= L[j * 6 + k] * L[j * 6 + k];
      if (!(s > 0)) {
        ok = false;
        break;
      }
      double d = sqrt(s);
      L[j * 6 + j] = d;
      for (int i = j + 1; i < 6; ++i) {
        double t = L[i * 6 + j];
        for (int k = 0; k < j; ++k) t -= L[i * 6 + k] * L[j * 6 + k];
        L[i * 6 + j] = t / d;
      }
    }
  }
  if (ok) {
    for (int c = 0; c < 6; ++c) {
      for (int i = 0; i < 6; ++i) e[i] = i == c ? 1.0 : 0.0;
      for (int i = 0; i < 6; ++i) {
        double t = e[i];
        for (int k = 0; k < i; ++k) t -= L[i * 6 + k] * e[k];
        e[i] = t / L[i * 6 + i];
      }
      for (int i = 5; i >= 0; --i) {
        double t = e[i];
        for (int k = i + 1; k < 6; ++k) t -= L[k * 6 + i] * e[k];
        e[i] = t / L[i * 6 + i];
      }
      for (int i = 0; i < 6; ++i) X[i * 6 + c] = e[i];
    }
    return;
  }
  // rank-deficient (or not numerically PD): Eigen's COD pseudo-inverse
  pinv_cod_serial(A, 6, 1, X, ws);
}

__device__ double cubic(double t, double t0, double tf, double x0, double xf, double xd0, double xdf) {
  if (t < t0) return x0;
  if (t > tf) return xf;
  double e = t - t0, T = tf - t0, T2 = T * T, T3 = T2 * T, dx = xf - x0;
  return x0 + xd0 * e + (3 * dx / T2 - 2 * xd0 / T - xdf / T) * e * e + (-2 * dx / T3 + (xd0 + xdf) / T2) * e * e * e;
}
__device__ double cubic_dot(double t, double t0, double tf, double x0, double xf, double xd0, double xdf) {
  if (t < t0) return xd0;
  if (t > tf) return xdf;
  double e = t - t0, T = tf - t0, T2 = T * T, T3 = T2 * T, dx = xf - x0;
  return xd0 + 2 * (3 * dx / T2 - 2 * xd0 / T - xdf / T) * e + 3 * (-2 * dx / T3 + (xd0 + xdf) / T2) * e * e;
}
// principal log of a rotation matrix (row-major) as an axis-angle vector
__device__ V3 so3_log(const double* R) {
  double c = (R[0] + R[4] + R[8] - 1) / 2;
  c = c > 1 ? 1 : (c < -1 ? -1 : c);
  double th = acos(c);
  V3 v = v3(R[7] - R[5], R[2] - R[6], R[3] - R[1]);
  if (th < 1e-8) return 0.5 * v;
  if (M_PI - th < 1e-6) {
    double B[9];
    for (int i = 0; i < 9; ++i) B[i] = R[i] / 2;
    B[0] += 0.5;
    B[4] += 0.5;
    B[8] += 0.5;
    int k = 0;
    if (B[4] > B[k * 4]) k = 1;
    if (B[8] > B[k * 4]) k = 2;
    double s = sqrt(B[k * 4]);
    V3 a = v3(B[k] / s, B[3 + k] / s, B[6 + k] / s);
    if (dot(a, v) < 0) a = -1.0 * a;
    return th * a;
  }
  return (th / (2 * sin(th))) * v;
}
__device__ void so3_exp(V3 w, double* R) {
  double th = sqrt(dot(w, w));
  double K[9] = {0, -w.z, w.y, w.z, 0, -w.x, -w.y, w.x, 0}, K2[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) K2[3 * i + j] = K[3 * i] * K[j] + K[3 * i + 1] * K[3 + j] + K[3 * i + 2] * K[6 + j];
  double a = th < 1e-12 ? 1 : sin(th) / th, b = th < 1e-12 ? 0 : (1 - cos(th)) / (th * th);
  for (int i = 0; i < 9; ++i) R[i] = (i % 4 == 0 ? 1 : 0) + a * K[i] + b * K2[i];
}

// Compile-time QP dimensions (nx variables, ng general rows, np = leading
// block of P).  Dims<0,0,0> is the runtime-sized fallback; the named robots
// get fully unrolled inner products (LDS loads issued ahead of the FMAs).
// QP shape: compile-time sizes (0 = runtime, from KParams).  reg: the
// register-resident Ruiz / K^-1 / ADMM path (QPIK shapes); otherwise the LDS
// path, whose loops still unroll when the sizes are compile-time.
// schur: the register ADMM solves K x~ = rhs through the Schur complement of
// K's auxiliary block (every variable past np — slacks — sits in exactly one G
// row, so that block is diagonal): S = K_cc - K_ca D^-1 K_ac is np x np.
// gs: lanes per instance (64, or 32 = two instances per wave; the QPIK
// shapes whose n + NG Schur lanes and polish rows fit in 32).
template <int NX, int NG, int NP, bool REG = (NX > 0), bool SCHUR = false, int GS = 64>
struct Dims {
  static constexpr int nx = NX, ng = NG, np = NP;
  static constexpr bool reg = REG;
  static constexpr bool schur = SCHUR;
  static constexpr int gs = GS;
};
#define DNX (QD::nx ? QD::nx : kp.nx)
#define DNG (QD::ng ? QD::ng : kp.ng)
#define DNP (QD::np ? QD::np : kp.np)
#define DM (DNX + DNG)


// ------------------------------------------------------------------------
// the fused per-instance solve
// ------------------------------------------------------------------------
// Instance order.  With xcd_map, the instances of each 128-B line of a
// [field][B] row (16 doubles) are handled by workgroups of one XCD (blocks
// are dealt to the 8 XCDs round-robin), so a line is fetched once per L2 and
// stores to it merge there before write-back; otherwise plain grid-stride.
// Placement only affects speed, never which instances run.
//
// Work queue (queue != nullptr): the waves of residue class x = blockIdx & 7
// take the positions of sequence x from an atomic counter (queue[x], zeroed
// before the launch) instead of a fixed stride, so a straggler instance
// (thousands of ADMM iterations, a deep EPA) holds up only its own wave and
// never the instances that would have followed it.  Every wave leaves once
// its counter passes the sequence end; all 8 classes have waves (grid >= 8).
struct InstSeq {
  int64_t j0, step, n;
  int xcd, map;
  int* queue;
  __device__ __forceinline__ InstSeq(int64_t B, int map_, int* queue_ = nullptr) {
    map = map_;
    queue = queue_;
    xcd = blockIdx.x & 7;
    j0 = map ? (blockIdx.x >> 3) : blockIdx.x;
    step = map ? (gridDim.x >> 3) : gridDim.x;
    n = map ? ((B + 127) >> 7) << 4 : B;
  }
  __device__ __forceinline__ int64_t fetch() const {
    int v = 0;
    if (lane_id() == 0) v = atomicAdd(queue + (map ? xcd : 0), 1);
    return __builtin_amdgcn_readfirstlane(v);
  }
  __device__ __forceinline__ int64_t first() const { return queue ? fetch() : j0; }
  __device__ __forceinline__ int64_t next(int64_t j) const { return queue ? fetch() : j + step; }
  __device__ __forceinline__ int64_t at(int64_t j) const {
    return map ? ((((j >> 4) << 3) + xcd) << 4) + (j & 15) : j;
  }
};

// InstSeq for lane groups: each group of GS lanes is its own consumer (its
// leader lane takes the queue position; with a fixed stride the groups of a
// wave interleave).
template <int GS>
struct InstSeqG {
  int64_t j0, step, n;
  int xcd, map;
  int* queue;
  __device__ __forceinline__ InstSeqG(int64_t B, int map_, int* queue_ = nullptr) {
    constexpr int G = 64 / GS;
    const int g = GS == 64 ? 0 : ((threadIdx.x >> 5) & 1);
    map = map_;
    queue = queue_;
    xcd = blockIdx.x & 7;
    j0 = (map ? (blockIdx.x >> 3) : blockIdx.x) * G + g;
    step = (map ? (gridDim.x >> 3) : gridDim.x) * G;
    n = map ? ((B + 127) >> 7) << 4 : B;
  }
  __device__ __forceinline__ int64_t fetch() const {
    int v = 0;
    if (Grp<GS>::lane() == 0) v = atomicAdd(queue + (map ? xcd : 0), 1);
    if constexpr (GS == 64) return __builtin_amdgcn_readfirstlane(v);
    else return Grp<GS>::shfl(v, 0);
  }
  __device__ __forceinline__ int64_t first() const { return queue ? fetch() : j0; }
  __device__ __forceinline__ int64_t next(int64_t j) const { return queue ? fetch() : j + step; }
  __device__ __forceinline__ int64_t at(int64_t j) const {
    return map ? ((((j >> 4) << 3) + xcd) << 4) + (j & 15) : j;
  }
};

// The model pointer, opaque to the optimizer (re-derived per instance so that
// model-constant loads are not hoisted out of the persistent instance loops
// into spilled registers, D19) but still known to point to constant memory:
// the opaque copy is taken in the constant address space and only then cast
// back, so uniform model reads stay scalar loads (s_load) instead of turning
// into per-lane flat loads.
// LDS (address space 3) views: an opaque copy of an LDS address must keep its
// address space, or every access through it becomes a flat access (vector
// memory path and its waits) instead of a ds_read / ds_write
// The fused kernel's LDS: the task plan (kt) and the QP plan (kq) overlay each
// other from offset 0, and the task record sits where neither stage touches it
// while the other reads it: in the task plan's overlay region (kEpa: EPA
// polytope, GJK candidates, manipulability scratch -- dead once the record is
// written, task_stage.hpp "task data out") when that region lies past the QP
// plan and holds the record, else past both plans.  Whole-body plans then need
// no extra space for the record: 8 instead of 7 fused waves per CU (r06).
// Offsets in doubles; same function on the host (launch size) and the device.
__host__ __device__ __forceinline__ int fused_rec_offset(const KParams& kt, const KParams& kq) {
  const int rec = (kt.rLen + 1) & ~1;
  const int plans = kt.lds_doubles > kq.lds_doubles ? kt.lds_doubles : kq.lds_doubles;
  const int inside = kt.kEpa > kq.lds_doubles ? kt.kEpa : kq.lds_doubles;
  return kt.kEpa > 0 && inside + rec <= kt.lds_doubles ? inside : plans;
}
__host__ __device__ __forceinline__ int fused_lds_doubles(const KParams& kt, const KParams& kq) {
  const int plans = kt.lds_doubles > kq.lds_doubles ? kt.lds_doubles : kq.lds_doubles;
  const int end = fused_rec_offset(kt, kq) + ((kt.rLen + 1) & ~1);
  return end > plans ? end : plans;
}

typedef __attribute__((address_space(3))) double lds_double;
typedef __attribute__((address_space(3))) const double lds_cdouble;
typedef __attribute__((address_space(3))) const int lds_cint;
typedef __attribute__((address_space(3))) const KParams lds_ckparams;
typedef __attribute__((address_space(4))) const DevModel const_devmodel;
// opaque copy of a wave-uniform LDS address, held in an SGPR (readfirstlane
// first: inside an out-of-line function the argument arrives in a VGPR)
template <class T>
__device__ __forceinline__ T* opaque_lds(T* p) {
  uint32_t v = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(reinterpret_cast<uintptr_t>(p)));
  asm volatile("" : "+s"(v));
  return reinterpret_cast<T*>(static_cast<uintptr_t>(v));
}
__device__ __forceinline__ const DevModel* opaque_model(const DevModel* M0) {
  const_devmodel* Mc = (const_devmodel*)M0;
  asm volatile("" : "+s"(Mc));
  return (const DevModel*)Mc;
}

struct IO {
  int64_t B;       // instances of this launch
  int64_t b0, ld;  // global offset of instance 0, row stride of the [field][B] arrays
  const double *q, *qdot, *xt, *xdt, *xi, *xdi;
  double* out;
  int32_t *status, *iters;
  double *st_pose, *st_jac, *st_man, *st_dist, *st_xdd;
  int32_t* st_pair;
  double* rec;  // product path: per-instance task record [B][rec_stride] (coalesced)
  int64_t rec_stride;
  // QPID: dynamics of the equality rows ([na*na][B], [na][B]; MoMa also the
  // joint-order gravity [nv][B]), torque output, and the QPID stage outputs
  const double *dM, *dG, *dGf;
  double* out2;
  double *st_jdot, *st_qpid;  // [6*nv][B] Jdot; [8][B] bias(6), man_gd, dist_gd
  double* st_gdv;             // [narm + nv][B] grad_dot vectors (manipulability | min distance)
  const double* cf_null;      // closed-form: null_qdot / null_torque [nv][B] (may be NULL)
  int* queue;                 // per-launch work-queue counters (8, zeroed), or NULL: fixed stride
  // lane-per-instance task stage (lane_task.hpp): instances it leaves to the
  // wave-per-instance task_kernel; hard_mode makes task_kernel run that list
  int* hard_list;
  int* hard_n;
  uint8_t* hard_flag;  // [B] 1 = instance on the hard list (QP pass over the others skips it)
  int hard_mode;       // task_kernel / qp_kernel: 1 = run the hard list; qp_kernel: 2 = skip flagged
  // per-instance stage stamps [kStamps][B] (s_memrealtime, 100 MHz), or NULL:
  // task start / end, QP start / assembled / solved / stored
  // (drc_qpik_host_timed -> QP::TimeDuration, include/drc_amd.h)
  uint64_t* stamps;
  // scheduling order of the instances (task / fused kernels), or NULL: the
  // instance at queue position j of this launch is order[b0 + j] - b0 (a
  // permutation of [b0, b0 + B)); results do not depend on it
  const int32_t* order = nullptr;
  __device__ __forceinline__ int64_t ordered(int64_t j) const { return order ? int64_t(order[b0 + j]) - b0 : j; }
};
// six clock stamps, then where the task and the QP stage ran (stage_where)
constexpr int kTimeStamps = 6, kStamps = 8;
enum { ST_TASK0 = 0, ST_TASK1 = 1, ST_QP0 = 2, ST_ASM = 3, ST_SOLVED = 4, ST_OUT = 5, ST_WTASK = 6, ST_WQP = 7 };
// Stage stamp k of instance gb (wave-uniform branch; no stamp executes in a
// call without io.stamps).  The wait keeps the clock read from returning out
// of order with the LDS reads that follow (cdna_hip_programming.md).
// Written by the leader of the instance's lane group (every instance of a
// two-instance QP wave gets its stamps); the host clears the region before the
// launch and skips instances whose stamps are missing or out of order.
template <int GS = 64>
__device__ __forceinline__ void stage_stamp(const IO& io, int k, int64_t gb) {
  if (io.stamps) {
    const uint64_t t = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    if ((__lane_id() & (GS - 1)) == 0) io.stamps[k * io.ld + gb] = t;
  }
}
// Where the stage of instance gb runs: workgroup index << 32 | __smid() (XCC,
// SE, CU) << 2 | SIMD (HW_ID bits 5:4) -- drc_debug_qpik_stamps, the
// small-batch makespan study (tools/stamp_study.py)
template <int GS = 64>
__device__ __forceinline__ void stage_where(const IO& io, int k, int64_t gb) {
  if (io.stamps) {
    const uint64_t w = (static_cast<uint64_t>(blockIdx.x) << 32) | (static_cast<uint64_t>(__smid()) << 2) |
                       static_cast<uint64_t>(__builtin_amdgcn_s_getreg(GETREG_IMMED(1, 4, 4)));
    if ((__lane_id() & (GS - 1)) == 0) io.stamps[k * io.ld + gb] = w;
  }
}

// J_mobile of this instance (row stride kMaxWheels) staged in LDS (kSv): the
// model table for the configuration-independent drives; a caster base's
// depends on the steer angles q[mobi_start + 2i] and is evaluated by lane 0.
// Wave-uniform call (contains a wave barrier).
template <int GS = 64>
__device__ __forceinline__ const double (*mobile_jac(const DevModel* M, const KParams& kp, double* S,
                                                     const double* q))[kMaxWheels] {
  double(*Jm)[kMaxWheels] = reinterpret_cast<double(*)[kMaxWheels]>(S + kp.kSv);
  const int l = Grp<GS>::lane();
  if (M->drive == kDriveCaster) {
    if (l == 0) mobile_fk(M, q + M->mobi_start, Jm);
  } else if (l < 3 * kMaxWheels) {
    Jm[l / kMaxWheels][l % kMaxWheels] = M->J_mobile[l / kMaxWheels][l % kMaxWheels];
  }
  wsync();
  return Jm;
}

// v of lane `lane`, broadcast to the wave (two v_readlane, no LDS)
__device__ __forceinline__ double bcast(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane(static_cast<int>(b), lane);
  const int hi = __builtin_amdgcn_readlane(static_cast<int>(b >> 32), lane);
  return __hiloint2double(hi, lo);
}

// Wave forms of det_lu6 and pinv_cod6 (the ill-conditioned JJ^T path of
// every near-singular instance, formerly ~0.6 M cycles on one lane): the same
// operation sequences with the 6 rows / columns in registers of lanes 0..5,
// pivots and broadcasts by v_readlane, the six triangular solves one per lane.
// Bit-identical to the serial forms (tests/test_gpu_parity.py near-singular
// tier).  Call with the whole wave; results are wave-uniform.
__device__ __forceinline__ double det_lu6_wave(const double* A) {
  const int l = lane_id(), lr = l < 6 ? l : 0;
  double r[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) r[j] = A[lr * 6 + j];
  double det = 1;
#pragma unroll
  for (int c = 0; c < 6; ++c) {
    double col[6];
#pragma unroll
    for (int i = c; i < 6; ++i) col[i] = bcast(r[c], i);
    int p = c;  // first row of maximal |M[r][c]| (serial scan)
#pragma unroll
    for (int i = c + 1; i < 6; ++i)
      if (fabs(col[i]) > fabs(col[p])) p = i;
    p = __builtin_amdgcn_readfirstlane(p);
    double pv = col[c];
#pragma unroll
    for (int i = c + 1; i < 6; ++i) pv = p == i ? col[i] : pv;
    if (pv == 0) return 0;
    if (p != c) {
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        const double rc = bcast(r[j], c), rp = bcast(r[j], p);
        r[j] = l == c ? rp : (l == p ? rc : r[j]);
      }
      det = -det;
    }
    det *= pv;
    double pr[6];
#pragma unroll
    for (int j = c; j < 6; ++j) pr[j] = bcast(r[j], c);
    if (l > c && l < 6) {
      const double f = r[c] / pr[c];
#pragma unroll
      for (int j = c; j < 6; ++j) r[j] -= f * pr[j];
    }
  }
  return det;
}
// rank_cpqr6 with column j in lane j
__device__ __forceinline__ int rank_cpqr6_wave(const double* A) {
  const int l = lane_id(), lc = l < 6 ? l : 0;
  double m[6], piv[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) m[i] = A[i * 6 + lc];
  double maxpiv = 0;
  bool done = false;
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    if (done) {
      piv[k] = 0;
      continue;
    }
    double cn = 0;
#pragma unroll
    for (int i = k; i < 6; ++i) cn += m[i] * m[i];
    double cv[6];
#pragma unroll
    for (int j = k; j < 6; ++j) cv[j] = bcast(cn, j);
    int p = k;
#pragma unroll
    for (int j = k + 1; j < 6; ++j)
      if (cv[j] > cv[p]) p = j;
    p = __builtin_amdgcn_readfirstlane(p);
    double cp = cv[k];
#pragma unroll
    for (int j = k + 1; j < 6; ++j) cp = p == j ? cv[j] : cp;
    if (p != k)
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const double mk = bcast(m[i], k), mp = bcast(m[i], p);
        m[i] = l == k ? mp : (l == p ? mk : m[i]);
      }
    const double nrm = sqrt(cp);
    piv[k] = nrm;
    maxpiv = fmax(maxpiv, nrm);
    if (nrm == 0) {
      done = true;
      continue;
    }
    double v[6];
#pragma unroll
    for (int i = k; i < 6; ++i) v[i] = bcast(m[i], k);
    const double alpha = v[k] > 0 ? -nrm : nrm;
    v[k] -= alpha;
    double vn = 0;
#pragma unroll
    for (int i = k; i < 6; ++i) vn += v[i] * v[i];
    if (vn > 0 && l >= k && l < 6) {
      double sm = 0;
#pragma unroll
      for (int i = k; i < 6; ++i) sm += v[i] * m[i];
      sm = 2 * sm / vn;
#pragma unroll
      for (int i = k; i < 6; ++i) m[i] -= sm * v[i];
    }
  }
  int r = 0;
#pragma unroll
  for (int k = 0; k < 6; ++k) r += piv[k] > 1e-6 * maxpiv;
  return r;
}
// pinv_cod6: rank, Cholesky (row i in lane i), the six column solves one per
// lane against L in LDS (ws[0..35]); rank-deficient / not-PD -> the serial
// COD on lane 0
__device__ __forceinline__ void pinv_cod6_wave(const double* A, double* X, double* ws) {
  const int l = lane_id(), lr = l < 6 ? l : 0;
  bool ok = rank_cpqr6_wave(A) == 6;
  if (ok) {
    double Lr[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) Lr[j] = A[lr * 6 + j];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      double rj[6];
#pragma unroll
      for (int k = 0; k <= j; ++k) rj[k] = bcast(Lr[k], j);
      double sv = rj[j];
#pragma unroll
      for (int k = 0; k < j; ++k) sv -= rj[k] * rj[k];
      if (!(sv > 0)) {
        ok = false;
        break;
      }
      const double d = sqrt(sv);
      if (l == j) Lr[j] = d;
      if (l > j && l < 6) {
        double t = Lr[j];
#pragma unroll
        for (int k = 0; k < j; ++k) t -= Lr[k] * rj[k];
        Lr[j] = t / d;
      }
    }
    if (ok) {
      if (l < 6)
#pragma unroll
        for (int j = 0; j < 6; ++j) ws[l * 6 + j] = Lr[j];
      wsync();
      if (l < 6) {
        const double* L = ws;
        double e[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) e[i] = i == l ? 1.0 : 0.0;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          double t = e[i];
#pragma unroll
          for (int k = 0; k < i; ++k) t -= L[i * 6 + k] * e[k];
          e[i] = t / L[i * 6 + i];
        }
#pragma unroll
        for (int i = 5; i >= 0; --i) {
          double t = e[i];
#pragma unroll
          for (int k = i + 1; k < 6; ++k) t -= L[k * 6 + i] * e[k];
          e[i] = t / L[i * 6 + i];
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) X[i * 6 + l] = e[i];
      }
      wsync();
      return;
    }
  }
  if (l == 0) pinv_cod_serial(A, 6, 1, X, ws);
  wsync();
}


// Register EQP of the polish (eqp_regs): reduced KKTs of up to this many rows
// are solved lane-per-row in registers; the LDS plan sizes follow it.
constexpr int kEqpRegCap = 16;

// Lanes per QP instance (qp_kernel): 64, or 32 = two instances per wave
// (Grp<32>; DESIGN.md: measured slower on FR3, so 64 is the default).
#ifndef DRC_QP_GROUP
#define DRC_QP_GROUP 64
#endif
constexpr int kQpGroup = DRC_QP_GROUP;

}  // namespace drc_amd

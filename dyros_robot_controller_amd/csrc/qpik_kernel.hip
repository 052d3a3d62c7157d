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
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/drc_amd.h"
#include "dynamics.hpp"
#include "mobile_fk.hpp"
#include "model.hpp"
#include "pinv_cod.hpp"
#include "qpik_device.hpp"

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


// ---- diagnostic phase stamps (built only with -DDRC_PHASE_TIMING) ---------
#ifdef DRC_PHASE_TIMING
__device__ unsigned long long g_phase_cycles[64];
#define PH_DECL unsigned long long ph_prev = __builtin_amdgcn_s_memtime(), ph_acc[16] = {0};
#define PH(k)                                              \
  do {                                                     \
    unsigned long long t_ = __builtin_amdgcn_s_memtime();  \
    ph_acc[k] += t_ - ph_prev;                             \
    ph_prev = t_;                                          \
  } while (0)
#define PH_FLUSH(base)                                                            \
  do {                                                                            \
    if (lane_id() == 0)                                                           \
      for (int k_ = 0; k_ < 16; ++k_) atomicAdd(&g_phase_cycles[(base) + k_], ph_acc[k_]); \
  } while (0)
// direct accumulation (functions without the kernel's stamp locals)
#define PHG_DECL unsigned long long phg_t = __builtin_amdgcn_s_memtime();
#define PHG(slot)                                                                  \
  do {                                                                             \
    unsigned long long t_ = __builtin_amdgcn_s_memtime();                          \
    if (lane_id() == 0) atomicAdd(&g_phase_cycles[(slot)], t_ - phg_t);             \
    phg_t = t_;                                                                    \
  } while (0)
#define PHG_RESET() do { phg_t = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define PH_DECL
#define PH(k) do {} while (0)
#define PH_FLUSH(base) do {} while (0)
#define PHG_DECL
#define PHG(slot) do {} while (0)
#define PHG_RESET() do {} while (0)
#endif

// scalar slots in the oSc region
enum { SC_C = 0, SC_RHO, SC_MAN, SC_DIST, SC_PAIR, SC_PRI, SC_DUA, SC_EPSP, SC_EPSD, SC_PRIS, SC_DUAS,
       SC_NAX, SC_NZ, SC_NPX, SC_NATY, SC_NQ, SC_NF, SC_NR, SC_WIN, SC_PFAIL, SC_HIV, SC_COUNT };
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
// OSQP residuals (lane-parallel): fills SC_* slots.  x, z, y in LDS (scaled)
// ------------------------------------------------------------------------
template <class QD, bool UNSCALED = true>
__device__ __forceinline__ void residuals(const KParams& kp, double* S, const double* x, const double* z, const double* y,
                          double eps_abs, double eps_rel) {
  using GL = Grp<QD::gs>;
  // UNSCALED = false (the polish's certification) skips the unscaled norms
  // that only adaptive rho reads (SC_PRIS .. SC_NQ keep the ADMM values)
  const int l = GL::lane(), nx = DNX, ng = DNG, np = DNP;
  const double *P = S + kp.oP, *G = S + kp.oG, *q = S + kp.oQ, *ab = S + kp.oAB, *D = S + kp.oD, *E = S + kp.oE;
  double pr = 0, prs = 0, nAx = 0, nz = 0, nAxs = 0, nzs = 0;
  double dr = 0, drs = 0, nPx = 0, nAty = 0, nq = 0, nPxs = 0, nAtys = 0, nqs = 0;
  if (l < nx) {  // bound row l and variable l
    const int lx = l < nx ? l : 0;
    double ax = ab[lx] * x[lx], r = ax - z[lx];
    prs = fabs(r);
    pr = fabs(r / E[lx]);
    nAx = fabs(ax / E[lx]);
    nz = fabs(z[lx] / E[lx]);
    nAxs = fabs(ax);
    nzs = fabs(z[lx]);
    double px = 0;
    if (l < np) {
      const int lp = l < np ? l : 0;
#pragma unroll
      for (int c = 0; c < np; ++c) px += P[lp * np + c] * x[c];
    }
    double aty = ab[lx] * y[lx];
#pragma unroll
    for (int i = 0; i < ng; ++i) aty += G[i * nx + lx] * y[nx + i];
    double rr = px + q[lx] + aty;
    drs = fabs(rr);
    dr = fabs(rr / D[lx]);
    nPx = fabs(px / D[lx]);
    nAty = fabs(aty / D[lx]);
    nq = fabs(q[lx] / D[lx]);
    nPxs = fabs(px);
    nAtys = fabs(aty);
    nqs = fabs(q[lx]);
  }
  if (l < ng) {
    const int lg = l < ng ? l : 0;
    double ax = 0;
#pragma unroll
    for (int j = 0; j < nx; ++j) ax += G[lg * nx + j] * x[j];
    int row = nx + lg;
    double r = ax - z[row];
    prs = fmax(prs, fabs(r));
    pr = fmax(pr, fabs(r / E[row]));
    nAx = fmax(nAx, fabs(ax / E[row]));
    nz = fmax(nz, fabs(z[row] / E[row]));
    nAxs = fmax(nAxs, fabs(ax));
    nzs = fmax(nzs, fabs(z[row]));
  }
  pr = GL::max(pr);
  nAx = GL::max(nAx);
  nz = GL::max(nz);
  dr = GL::max(dr);
  nPx = GL::max(nPx);
  nAty = GL::max(nAty);
  nq = GL::max(nq);
  if constexpr (UNSCALED) {
    prs = GL::max(prs);
    nAxs = GL::max(nAxs);
    nzs = GL::max(nzs);
    drs = GL::max(drs);
    nPxs = GL::max(nPxs);
    nAtys = GL::max(nAtys);
    nqs = GL::max(nqs);
  }
  double c = S[kp.oSc + SC_C];
  if (l == 0) {
    double* sc = S + kp.oSc;
    sc[SC_PRI] = pr;
    sc[SC_DUA] = dr / c;
    if constexpr (UNSCALED) {
      sc[SC_PRIS] = prs;
      sc[SC_DUAS] = drs;
      sc[SC_NAX] = nAxs;
      sc[SC_NZ] = nzs;
      sc[SC_NPX] = nPxs;
      sc[SC_NATY] = nAtys;
      sc[SC_NQ] = nqs;
    }
    sc[SC_EPSP] = eps_abs + eps_rel * fmax(nAx, nz);
    sc[SC_EPSD] = eps_abs + eps_rel * fmax(fmax(nPx, nAty), nq) / c;
  }
  wsync();
}

// K = P + sigma I + A^T diag(rho) A, inverted in place (Gauss-Jordan, SPD)
template <class QD>
__device__ __forceinline__ void factor_kinv(const KParams& kp, double* S) {
  using GL = Grp<QD::gs>;
  const int l = GL::lane(), nx = DNX, ng = DNG, np = DNP;
  const double *P = S + kp.oP, *G = S + kp.oG, *ab = S + kp.oAB, *rho = S + kp.oRho;
  double* K = S + kp.oU0;
  if (l < nx) {
    for (int c = 0; c < nx; ++c) {
      double s = (l < np && c < np) ? P[l * np + c] : 0.0;
      if (c == l) s += kp.s.sigma + ab[l] * ab[l] * rho[l];
      for (int i = 0; i < ng; ++i) s += G[i * nx + l] * rho[nx + i] * G[i * nx + c];
      K[l * nx + c] = s;
    }
  }
  wsync();
  for (int k = 0; k < nx; ++k) {
    if (l == k) {
      double p = 1.0 / K[k * nx + k];
      K[k * nx + k] = 1.0;
      for (int j = 0; j < nx; ++j) K[k * nx + j] *= p;
    }
    wsync();
    if (l < nx && l != k) {
      double f = K[l * nx + k];
      K[l * nx + k] = 0.0;
      for (int j = 0; j < nx; ++j) K[l * nx + j] -= f * K[k * nx + j];
    }
    wsync();
  }
}

// Register form for compile-time shapes: lane l assembles row l of K and the
// Gauss-Jordan sweep runs on registers, the pivot row moving by v_readlane.
// Same operation sequence as factor_kinv's LDS sweep (bit-identical).
__device__ __forceinline__ double bcast(double v, int lane);
template <class QD>
__device__ __noinline__ void factor_kinv_regs(const KParams& kp, double* S) {
  using GL = Grp<QD::gs>;
  constexpr int NX = QD::nx, NG = QD::ng, NP = QD::np;
  const int l = GL::lane();
  const double *P = S + kp.oP, *G = S + kp.oG, *ab = S + kp.oAB, *rho = S + kp.oRho;
  double* K = S + kp.oU0;
  if (l < NX) {  // row l of K = P + sigma I + A^T diag(rho) A (LDS, as factor_kinv)
    for (int c = 0; c < NX; ++c) {
      double s = (l < NP && c < NP) ? P[l * NP + c] : 0.0;
      if (c == l) s += kp.s.sigma + ab[l] * ab[l] * rho[l];
      for (int i = 0; i < NG; ++i) s += G[i * NX + l] * rho[NX + i] * G[i * NX + c];
      K[l * NX + c] = s;
    }
  }
  wsync();
  const int lr = l < NX ? l : 0;
  double Kr[NX];
#pragma unroll
  for (int c = 0; c < NX; ++c) Kr[c] = K[lr * NX + c];
#pragma unroll
  for (int k = 0; k < NX; ++k) {
    if (l == k) {
      const double p = 1.0 / Kr[k];
      Kr[k] = 1.0;
#pragma unroll
      for (int j = 0; j < NX; ++j) Kr[j] *= p;
    }
    const double f = Kr[k];
    if (l != k) Kr[k] = 0.0;
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      const double rkj = GL::bcast(Kr[j], k);
      if (l != k) Kr[j] -= f * rkj;
    }
  }
  if (l < NX) {
#pragma unroll
    for (int c = 0; c < NX; ++c) K[l * NX + c] = Kr[c];
  }
  wsync();
}

// ------------------------------------------------------------------------
// Schur-complement factorisation (QD::schur).  Variables j >= np ("aux":
// slacks) appear in the cost only linearly and each sits in exactly one G row
// a(r) (QP_IK.cpp:99-131), so with rows r = 0..ng-1, bound rows b:
//   K_cc = P + sigma I + diag(rho_b ab^2) + sum_r rho_r G_rc G_rc^T
//   K_aa = diag(d_a),  d_a = sigma + rho_b(a) ab_a^2 + rho_r g_r^2   (g_r = G[r][a(r)])
//   S    = K_cc - K_ca K_aa^-1 K_ac = P + sigma I + diag(rho_b ab^2) + sum_r w_r G_rc G_rc^T,
//   w_r  = rho_r - (rho_r g_r)^2 / d_a.
// LDS union layout: S^-1 (np x np) | G_c S^-1 (ng x np) | 1/d | coef = rho_r g_r / d | w | aux (int).
// Same linear solve as K^-1 (different rounding).
// ------------------------------------------------------------------------
template <class QD>
__device__ __noinline__ void schur_setup(const KParams& kp, double* S) {
  using GL = Grp<QD::gs>;
  constexpr int NX = QD::nx, NG = QD::ng, NP = QD::np;
  const int l = GL::lane();
  const double *P = S + kp.oP, *G = S + kp.oG, *ab = S + kp.oAB, *rho = S + kp.oRho;
  double* Si = S + kp.oU0;             // NP x NP
  double* GS = Si + NP * NP;           // NG x NP
  double* dv = GS + NG * NP;           // NG
  double* cf = dv + NG;                // NG
  double* wt = cf + NG;                // NG (row weights w_r)
  int* aux = reinterpret_cast<int*>(wt + NG);  // NG
  const double sig = kp.s.sigma;
  if (l < NG) {
    int a = -1;
    for (int j = NP; j < NX; ++j)
      if (G[l * NX + j] != 0.0) a = j;
    const double rr = rho[NX + l];
    double d = 1.0, w = rr, c = 0.0;
    if (a >= 0) {
      const double g = G[l * NX + a];
      d = sig + rho[a] * ab[a] * ab[a] + rr * g * g;
      c = rr * g / d;
      w = rr - rr * g * c;
    }
    aux[l] = a;
    dv[l] = 1.0 / d;  // the ADMM loop multiplies by 1 / d_a
    cf[l] = c;
    wt[l] = w;
  }
  wsync();
  for (int e = l; e < NP * NP; e += GL::size) {  // entry (i, c) of S, one per lane
    const int i = e / NP, c = e % NP;
    double sv = P[i * NP + c];
    if (c == i) sv += sig + rho[i] * ab[i] * ab[i];
#pragma unroll
    for (int r = 0; r < NG; ++r) sv += wt[r] * G[r * NX + i] * G[r * NX + c];
    Si[e] = sv;
  }
  wsync();
  // Gauss-Jordan in registers, lane l holding row l (S is SPD)
  const int lr = l < NP ? l : 0;
  double Sr[NP];
#pragma unroll
  for (int c = 0; c < NP; ++c) Sr[c] = Si[lr * NP + c];
  static_for<NP>([&](auto K) {
    constexpr int k = decltype(K)::value;
    if (l == k) {
      const double pv = 1.0 / Sr[k];
      Sr[k] = 1.0;
#pragma unroll
      for (int j = 0; j < NP; ++j) Sr[j] *= pv;
    }
    const double f = Sr[k];
    if (l != k) Sr[k] = 0.0;
    static_for<NP>([&](auto J) {
      constexpr int j = decltype(J)::value;
      const double rkj = GL::template bcastc<k>(Sr[j]);
      if (l != k) Sr[j] -= f * rkj;
    });
  });
  if (l < NP) {
#pragma unroll
    for (int c = 0; c < NP; ++c) Si[l * NP + c] = Sr[c];
  }
  wsync();
  for (int e = l; e < NG * NP; e += GL::size) {  // G_c S^-1
    const int r = e / NP, c = e % NP;
    double sv = 0;
#pragma unroll
    for (int k = 0; k < NP; ++k) sv += G[r * NX + k] * Si[k * NP + c];
    GS[e] = sv;
  }
  wsync();
}

template <class QD>
__device__ __forceinline__ void factor_any(const KParams& kp, double* S) {
  if constexpr (QD::schur) schur_setup<QD>(kp, S);
  else if constexpr (QD::reg) factor_kinv_regs<QD>(kp, S);
  else factor_kinv<QD>(kp, S);
}

template <class QD>
__device__ __forceinline__ void set_rho(const KParams& kp, double* S, double rho) {
  using GL = Grp<QD::gs>;
  const int l = GL::lane(), nx = DNX, ng = DNG;
  const double *lo = S + kp.oL, *up = S + kp.oU;
  double* rv = S + kp.oRho;
  for (int row = l; row < nx + ng; row += GL::size) {
    double a = lo[row], b = up[row];
    bool loose = a < -kInf * kMinScaling && b > kInf * kMinScaling;
    bool eq = !loose && b - a < kRhoTol;
    rv[row] = loose ? kRhoMin : (eq ? kRhoEqRatio * rho : rho);
  }
  if (l == 0) S[kp.oSc + SC_RHO] = rho;
  wsync();
}

// Primal infeasibility certificate (OSQP / Banjac et al.) on the last dy
template <class QD>
__device__ __forceinline__ bool primal_infeasible(const KParams& kp, double* S, double eps) {
  using GL = Grp<QD::gs>;
  const int l = GL::lane(), nx = DNX, ng = DNG;
  const double *lo = S + kp.oL, *up = S + kp.oU, *E = S + kp.oE, *dyv = S + kp.oDY, *G = S + kp.oG,
               *ab = S + kp.oAB, *D = S + kp.oD;
  double* dy = S + kp.oT1;
  double nrm = 0, lhs = 0;
  for (int row = l; row < nx + ng; row += GL::size) {
    double d = dyv[row], a = lo[row], b = up[row];
    bool lb_inf = a < -kInf * kMinScaling, ub_inf = b > kInf * kMinScaling;
    if (lb_inf && ub_inf) d = 0;
    else if (ub_inf) d = fmin(d, 0.0);
    else if (lb_inf) d = fmax(d, 0.0);
    dy[row] = d;
    nrm = fmax(nrm, fabs(E[row] * d));
    lhs += d > 0 ? b * d : (d < 0 ? a * d : 0.0);
  }
  nrm = GL::max(nrm);
  lhs = GL::sum(lhs);
  wsync();
  if (nrm <= kDivTol || !(lhs < -eps * nrm)) return false;
  double viol = 0;
  if (l < nx) {
    double s = ab[l] * dy[l];
    for (int i = 0; i < ng; ++i) s += G[i * nx + l] * dy[nx + i];
    viol = fabs(s / D[l]);
  }
  viol = GL::max(viol);
  return viol < eps * nrm;
}

// ------------------------------------------------------------------------
// Register-resident ADMM (compile-time QP shapes).  Per iteration
//   rhs = sigma x - q + A^T (rho z - y),  x~ = K^-1 rhs,  G x~ = (G K^-1) rhs,
// so two broadcast passes (the G-row duals, then rhs) give x~ and the G-row
// values together.  Lane l keeps column l of G and rows l of K^-1 and
// G K^-1 in VGPRs; the vectors move by v_readlane (no LDS traffic inside
// the iteration).  Same algebra as the LDS path, different summation order.
// ------------------------------------------------------------------------
__device__ __forceinline__ double bcast(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane(static_cast<int>(b), lane);
  const int hi = __builtin_amdgcn_readlane(static_cast<int>(b >> 32), lane);
  return __hiloint2double(hi, lo);
}

// G K^-1 (NG x NX) into LDS after K^-1 (once per factorisation; out of line
// so the ADMM loop's register file stays free)
template <class QD>
__device__ __noinline__ void prep_admm_mats(const KParams& kp, double* S) {
  using GL = Grp<QD::gs>;
  if constexpr (QD::schur) return;  // schur_setup already formed G_c S^-1
  constexpr int NX = QD::nx, NG = QD::ng;
  const int l = GL::lane();
  const double* K = S + kp.oU0;
  double* GK = S + kp.oU0 + NX * NX;
  const double* G = S + kp.oG;
  for (int e = l; e < NG * NX; e += GL::size) {
    const int i = e / NX, c = e % NX;
    double s = 0;
    for (int k = 0; k < NX; ++k) s += G[i * NX + k] * K[k * NX + c];
    GK[e] = s;
  }
  wsync();
}

// lane l: column l of G (rhs), row l of K^-1 (x~), row l of G K^-1 (G x~)
template <class QD>
__device__ __forceinline__ void load_admm_regs(const KParams& kp, const double* S, double (&Gc)[QD::ng],
                                               double (&Kr)[QD::nx], double (&GKr)[QD::nx]) {
  using GL = Grp<QD::gs>;
  constexpr int NX = QD::nx, NG = QD::ng;
  const int l = GL::lane();
  const double* K = S + kp.oU0;
  const double* GK = S + kp.oU0 + NX * NX;
  const double* G = S + kp.oG;
  const int lb = l < NX ? l : 0, lg = l < NG ? l : 0;
#pragma unroll
  for (int i = 0; i < NG; ++i) Gc[i] = G[i * NX + lb];
#pragma unroll
  for (int c = 0; c < NX; ++c) Kr[c] = K[lb * NX + c];
#pragma unroll
  for (int c = 0; c < NX; ++c) GKr[c] = GK[lg * NX + c];
}

// Termination / polish / adaptive-rho block of the register ADMM, out of
// line (runs every check_termination iterations).  Works on the published
// LDS iterate.  Returns 0 = continue, 1 = continue after reloading the
// registers (K^-1 or rho changed, or the iterate was touched), 2 = stop.
#ifdef DRC_PHASE_TIMING
#define CK_T0() unsigned long long ck_t = __builtin_amdgcn_s_memtime()
#define CK_T(slot)                                                              \
  do {                                                                          \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();                 \
    if (lane_id() == 0) atomicAdd(&g_phase_cycles[(slot)], t_ - ck_t);          \
    ck_t = t_;                                                                  \
  } while (0)
#define CK_N(slot) do { if (lane_id() == 0) atomicAdd(&g_phase_cycles[(slot)], 1ull); } while (0)
#else
#define CK_T0() do {} while (0)
#define CK_T(slot) do {} while (0)
#define CK_N(slot) do {} while (0)
#endif
template <class QD>
__device__ __noinline__ int admm_check(const KParams& kp, double* S, int it, int check, int adapt, int* status) {
  using GL = Grp<QD::gs>;
  double *x = S + kp.oX, *z = S + kp.oZ, *y = S + kp.oY, *sc = S + kp.oSc;
  int reload = 0;
  CK_T0();
  // parity mode: a certified polish is exact whatever the ADMM residual, so
  // the first kPolishMaxEarly checks try it before anything else (converged
  // or not, the oracle makes exactly one polish attempt at such a check).  The
  // polish reads only the iterate, so the ADMM residuals -- which decide
  // convergence, the fallback and adaptive rho -- are formed only when it
  // fails (the usual case solves here and never needs them)
  bool early_failed = false;
  if (check && kp.s.exact && sc[SC_PFAIL] < kPolishMaxEarly) {
    CK_T(34);
    const bool ok_ = polish<QD>(kp, S, true);
    CK_T(35);
    CK_N(36);
    if (ok_) {
      CK_N(37);
      *status = DRC_STATUS_SOLVED;
      return 2;
    }
    if (GL::lane() == 0) sc[SC_PFAIL] += 1.0;
    factor_any<QD>(kp, S);
    CK_T(38);  // polish used the union region
    early_failed = true;
    reload = 1;
  }
  residuals<QD>(kp, S, x, z, y, kp.s.eps_abs, kp.s.eps_rel);
  CK_T(32);
  CK_N(33);
  if (check) {
    const bool conv = sc[SC_PRI] < sc[SC_EPSP] && sc[SC_DUA] < sc[SC_EPSD];
#ifdef DRC_QP_DEBUG
    if (GL::lane() == 0 && it <= 200)
      printf("it %d rho %.4g pri %.3e/%.3e dua %.3e/%.3e x3 %.6f\n", it, sc[SC_RHO], sc[SC_PRI], sc[SC_EPSP],
             sc[SC_DUA], sc[SC_EPSD], x[3] * S[kp.oD + 3]);
#endif
    if (conv) {
      if (!kp.s.exact) {
        *status = DRC_STATUS_SOLVED;
        return 2;
      }
      if (!early_failed && sc[SC_PFAIL] < kPolishMaxTotal) {
        CK_T(34);
        const bool ok_ = polish<QD>(kp, S, true);
        CK_T(35);
        CK_N(36);
        if (ok_) {
          CK_N(37);
          *status = DRC_STATUS_SOLVED;
          return 2;
        }
        if (GL::lane() == 0) sc[SC_PFAIL] += 1.0;
        factor_any<QD>(kp, S);
        CK_T(38);
      }
      residuals<QD>(kp, S, x, z, y, kp.s.eps_fallback, kp.s.eps_fallback);
      if (sc[SC_PRI] < sc[SC_EPSP] && sc[SC_DUA] < sc[SC_EPSD]) {
        *status = DRC_STATUS_SOLVED;
        return 2;
      }
      reload = 1;
    } else if (primal_infeasible<QD>(kp, S, kp.s.eps_prim_inf)) {
      *status = DRC_STATUS_PRIMAL_INFEASIBLE;
      return 2;
    }
  }
  if (adapt) {
    const double pr = sc[SC_PRIS] / (fmax(sc[SC_NAX], sc[SC_NZ]) + kDivTol);
    const double dr = sc[SC_DUAS] / (fmax(fmax(sc[SC_NQ], sc[SC_NATY]), sc[SC_NPX]) + kDivTol);
    const double rho = sc[SC_RHO];
    double rn = rho * sqrt(pr / (dr + kDivTol));
    rn = fmin(fmax(rn, kRhoMin), kRhoMax);
    if (rn > rho * kp.s.adaptive_rho_tolerance || rn < rho / kp.s.adaptive_rho_tolerance) {
      set_rho<QD>(kp, S, rn);
      factor_any<QD>(kp, S);
      CK_T(38);
      reload = 1;
    }
  }
  if (reload) prep_admm_mats<QD>(kp, S);
  return reload;
}

// argmax with ties toward the smaller index (row order of the oracle scans)
__device__ __forceinline__ void wave_argmax(double& v, int& idx) {
  double nv = -v;
  wave_argmin(nv, idx);
  v = -nv;
}

__device__ __forceinline__ int pk(int i, int j) { return i * (i + 1) / 2 + j; }
// solve (L D L^T) b = b in place: L packed unit-lower, D in dg
__device__ __forceinline__ void ldl_solve(const double* L, const double* dg, int N, double* b) {
  const int l = lane_id();
  for (int j = 0; j < N; ++j) {  // L y = b (column oriented)
    const double bj = b[j];
    for (int i = l; i < N; i += 64)
      if (i > j) b[i] -= L[pk(i, j)] * bj;
    wsync();
  }
  for (int i = l; i < N; i += 64) b[i] /= dg[i];
  wsync();
  for (int j = N - 1; j >= 0; --j) {  // L^T x = y
    const double bj = b[j];
    for (int i = l; i < N; i += 64)
      if (i < j) b[i] -= L[pk(j, i)] * bj;
    wsync();
  }
}

// Register form of eqp for compile-time shapes and small reduced KKTs
// (N <= kEqpRegCap, the common case: most q-dot are at their bounds or the
// active set is small).  Lane i holds row i of the unregularised KKT (K0) and
// of the inverse of the regularised one, formed by a Gauss-Jordan sweep with
// the pivot row moving by v_readlane (no pivoting: the regularised KKT is
// quasi-definite, so the natural order has nonzero pivots, as the LDL^T).
// Solve and iterative refinement against K0 are N broadcasts each.  Same
// system, assembly, refinement count and outputs as eqp's LDS LDL^T; only
// the rounding of the factorisation differs.
constexpr int kEqpRegCap = 16;
template <class QD>
__device__ __forceinline__ bool eqp_regs(const KParams& kp, double* S, int actb, int actg, double* xx, double* yy,
                                         unsigned long long freeMask, unsigned long long rowMask, int nF, int nR) {
  using GL = Grp<QD::gs>;
  constexpr int NX = QD::nx, NG = QD::ng, NP = QD::np, M = NX + NG, NK = kEqpRegCap;
  const int l = GL::lane(), N = nF + nR;
  const double *P = S + kp.oP, *G = S + kp.oG, *q = S + kp.oQ, *ab = S + kp.oAB, *lo = S + kp.oL,
               *up = S + kp.oU;
  int* Fidx = reinterpret_cast<int*>(S + kp.oU0);  // 64 ints
  int* Ridx = Fidx + 64;                           // 64 ints
  const unsigned long long below = (1ull << l) - 1;
  if (l < NX && actb == 0) Fidx[__popcll(freeMask & below)] = l;
  if (l < NG && actg != 0) Ridx[__popcll(rowMask & below)] = l;
  if (l < NX) xx[l] = actb == 0 ? 0.0 : (actb < 0 ? lo[l] : up[l]) / ab[l];
  wsync();
  // right-hand sides by their owners: variable l (free) and G row l (active)
  // (free variables hold xx = 0 here, so the sums run over the fixed part;
  // unconditional and unrolled, the LDS loads issue back to back)
  double rF = 0.0, rG = 0.0;
  if (l < NX && actb == 0) {
    double r = -q[l];
    if (l < NP) {
      const int lp = l < NP ? l : 0;
#pragma unroll
      for (int c = 0; c < NP; ++c) r -= P[lp * NP + c] * xx[c];
    }
    rF = r;
  }
  if (l < NG && actg != 0) {
    const int lg = l < NG ? l : 0;
    double r = actg < 0 ? lo[NX + lg] : up[NX + lg];
#pragma unroll
    for (int c = 0; c < NX; ++c) r -= G[lg * NX + c] * xx[c];
    rG = r;
  }
  const bool hf = l < nF, hr = l >= nF && l < N;
  const int fi = hf ? Fidx[l] : 0, gi = hr ? Ridx[l - nF] : 0;
  const double rF_ = GL::shfl(rF, fi), rG_ = GL::shfl(rG, gi);
  const double rhs = hf ? rF_ : (hr ? rG_ : 0.0);
  // row l of K0: columns j < nF are the free variables, j >= nF the active rows
  double K0[NK], Ki[NK];
  {
    unsigned long long fm = freeMask, rm = rowMask;
#pragma unroll
    for (int j = 0; j < NK; ++j) {
      double v = 0.0;
      if (j < nF) {
        const int fj = __builtin_ctzll(fm);
        fm &= fm - 1;
        if (hf) v = (fi < NP && fj < NP) ? P[fi * NP + fj] : 0.0;
        else if (hr) v = G[gi * NX + fj];
      } else if (j < N) {
        const int gj = __builtin_ctzll(rm);
        rm &= rm - 1;
        if (hf) v = G[gj * NX + fi];
      }
      K0[j] = v;
      Ki[j] = v + (j == l ? (hf ? kp.s.delta : (hr ? -kp.s.delta : 0.0)) : 0.0);
    }
  }
  // Gauss-Jordan inverse of the regularised KKT
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    if (k >= N) break;
    const double piv = GL::bcast(Ki[k], k);
    if (piv == 0.0) return false;  // uniform
    if (l == k) {
      const double p = 1.0 / Ki[k];
      Ki[k] = 1.0;
#pragma unroll
      for (int j = 0; j < NK; ++j) Ki[j] *= p;
    }
    const double f = Ki[k];
    if (l != k) Ki[k] = 0.0;
#pragma unroll
    for (int j = 0; j < NK; ++j) {
      if (j >= N) break;
      const double rkj = GL::bcast(Ki[j], k);
      if (l != k) Ki[j] -= f * rkj;
    }
  }
  auto apply = [&](const double (&A)[NK], double v) {  // row l of A times the vector held by lanes 0..N-1
    double s0 = 0, s1 = 0;
#pragma unroll
    for (int j = 0; j < NK; ++j) {
      if (j >= N) break;
      const double vj = GL::bcast(v, j);
      if (j & 1) s1 += A[j] * vj;
      else s0 += A[j] * vj;
    }
    return s0 + s1;
  };
  double sol = apply(Ki, rhs);
  for (int it = 0; it < kp.s.polish_refine_iter; ++it) {
    const double res = rhs - apply(K0, sol);
    sol += apply(Ki, res);
  }
  if (hf) xx[fi] = sol;
  for (int row = l; row < M; row += GL::size) yy[row] = 0.0;
  wsync();
  if (hr) yy[NX + gi] = sol;
  wsync();
  if (l < NX && actb != 0) {  // bound multipliers from stationarity
    const int lx = l < NX ? l : 0;
    double g = q[lx];
    if (l < NP) {
      const int lp = l < NP ? l : 0;
#pragma unroll
      for (int c = 0; c < NP; ++c) g += P[lp * NP + c] * xx[c];
    }
#pragma unroll
    for (int i = 0; i < NG; ++i) g += G[i * NX + lx] * yy[NX + i];
    yy[lx] = -g / ab[lx];
  }
  wsync();
  return true;
}

// Range-space form of eqp for the whole-body QPs (no variable bounds, so
// every variable is free and the reduced KKT is [H, G_R^T; G_R, -dI] with
// H = P + dI fixed for the instance).  Its inverse applied to (r_x, r_l):
//   t = H^-1 r_x,  (G_R H^-1 G_R^T + dI) lam = G_R t - r_l,  x = t - H^-1 G_R^T lam
// so a polish attempt factors only the nR x nR Schur matrix of the active rows
// (mean 1.3 on XLS-FR3) instead of the (nx + nR)-row KKT (nx = 11).  H^-1
// (register Gauss-Jordan, lane per row) is formed on the first attempt and
// kept in LDS (oHi).  Lanes: l < NX hold x / row l of H^-1 / (H^-1 g_a)_l;
// lane NX + a holds active row a: lam_a, g_a and row a of the Schur inverse.
// Same system, refinement count and outputs as eqp's LDL^T (the oracle's
// qp_eqp); only the rounding of the factorisation differs.
template <class QD>
__device__ __forceinline__ bool eqp_range(const KParams& kp, double* S, int actg, double* xx, double* yy,
                                          unsigned long long rowMask, int nR) {
  constexpr int NX = QD::nx, NG = QD::ng, M = NX + NG, NK = kEqpRegCap;
  static_assert(NX + NK <= 64 && QD::gs == 64, "x lanes and active-row lanes in one wave");
  const int l = lane_id();
  const double *P = S + kp.oP, *G = S + kp.oG, *q = S + kp.oQ, *lo = S + kp.oL, *up = S + kp.oU;
  double* Hi = S + kp.oHi;
  double* sc = S + kp.oSc;
  int* Ridx = reinterpret_cast<int*>(S + kp.oU0) + 64;
  double* Vb = S + kp.oU0 + 256;  // [nR][NX]: H^-1 g_a
  const double dl = kp.s.delta;
  const bool hx = l < NX, hl = l >= NX && l < NX + nR;
  const int lx = hx ? l : 0, a = hl ? l - NX : 0;
  if (sc[SC_HIV] == 0.0) {  // uniform
    double h[NX];
#pragma unroll
    for (int j = 0; j < NX; ++j) h[j] = P[lx * NX + j] + (j == lx ? dl : 0.0);
#pragma unroll
    for (int k = 0; k < NX; ++k) {
      const double piv = rd_lane(h[k], k);
      if (piv == 0.0) return false;  // uniform
      if (l == k) {
        const double p = 1.0 / h[k];
        h[k] = 1.0;
#pragma unroll
        for (int j = 0; j < NX; ++j) h[j] *= p;
      }
      const double f = h[k];
      if (l != k) h[k] = 0.0;
#pragma unroll
      for (int j = 0; j < NX; ++j) {
        const double hkj = rd_lane(h[j], k);
        if (l != k) h[j] -= f * hkj;
      }
    }
    if (hx)
#pragma unroll
      for (int j = 0; j < NX; ++j) Hi[l * NX + j] = h[j];
    wsync();
    if (l == 0) sc[SC_HIV] = 1.0;
  }
  if (l < NG && actg != 0) Ridx[__popcll(rowMask & ((1ull << l) - 1))] = l;
  // right-hand side of active row a, formed by its owner lane (the G row)
  double rG = 0.0;
  if (l < NG && actg != 0) rG = actg < 0 ? lo[NX + l] : up[NX + l];
  wsync();
  const int gi = hl ? Ridx[a] : 0;
  const double rl = __shfl(rG, gi, 64);
  const double rx = hx ? -q[lx] : 0.0;
  // A1: row l of H^-1 (x lanes) or g_a (row lanes); A2: (H^-1 g_b)_l (x lanes)
  // or row a of the Schur inverse (row lanes)
  double A1[NX], A2[NK];
#pragma unroll
  for (int j = 0; j < NX; ++j) A1[j] = hl ? G[gi * NX + j] : Hi[lx * NX + j];
  if (hx) {
#pragma unroll
    for (int b = 0; b < NK; ++b) {
      if (b >= nR) break;
      const int gb = Ridx[b];
      double s = 0.0;
#pragma unroll
      for (int j = 0; j < NX; ++j) s += A1[j] * G[gb * NX + j];
      A2[b] = s;
      Vb[b * NX + l] = s;
    }
  }
  wsync();
  if (hl) {  // row a of G_R H^-1 G_R^T + dI
#pragma unroll
    for (int b = 0; b < NK; ++b) {
      if (b >= nR) break;
      double s = 0.0;
#pragma unroll
      for (int j = 0; j < NX; ++j) s += A1[j] * Vb[b * NX + j];
      A2[b] = s + (b == a ? dl : 0.0);
    }
  }
  // Gauss-Jordan inverse of the Schur matrix on lanes NX .. NX + nR - 1
  // (symmetric positive definite: nonzero pivots in natural order)
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    if (k >= nR) break;
    const double piv = rd_lane(A2[k], NX + k);
    if (piv == 0.0) return false;  // uniform
    if (l == NX + k) {
      const double p = 1.0 / A2[k];
      A2[k] = 1.0;
#pragma unroll
      for (int j = 0; j < NK; ++j) A2[j] *= p;
    }
    const double f = A2[k];
    if (hl && l != NX + k) A2[k] = 0.0;
#pragma unroll
    for (int j = 0; j < NK; ++j) {
      if (j >= nR) break;
      const double rkj = rd_lane(A2[j], NX + k);
      if (hl && l != NX + k) A2[j] -= f * rkj;
    }
  }
  // K^-1 (vx on x lanes, vl on row lanes) -> (x on x lanes, lam on row lanes)
  auto solve = [&](double vx, double vl, double& ox, double& ol) {
    double t0 = 0, t1 = 0;
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      const double v = rd_lane(vx, j);
      if (j & 1) t1 += A1[j] * v;
      else t0 += A1[j] * v;
    }
    const double t = t0 + t1;  // x lanes: (H^-1 vx)_l
    double s0 = 0, s1 = 0;
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      const double v = rd_lane(t, j);
      if (j & 1) s1 += A1[j] * v;
      else s0 += A1[j] * v;
    }
    const double sr = s0 + s1 - vl;  // row lanes: (G_R t - vl)_a
    double lam = 0;
#pragma unroll
    for (int b = 0; b < NK; ++b) {
      if (b >= nR) break;
      lam += A2[b] * rd_lane(sr, NX + b);
    }
    double xc = t;
#pragma unroll
    for (int b = 0; b < NK; ++b) {
      if (b >= nR) break;
      xc -= A2[b] * rd_lane(lam, NX + b);
    }
    ox = xc;
    ol = lam;
  };
  double sx, sl;
  solve(rx, rl, sx, sl);
  for (int it = 0; it < kp.s.polish_refine_iter; ++it) {
    // residual against the unregularised KKT [P, G_R^T; G_R, 0]
    double px = 0, gl = 0;
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      const double xj = rd_lane(sx, j);
      px += P[lx * NX + j] * xj;
      gl += A1[j] * xj;  // row lanes: g_a . x
    }
#pragma unroll
    for (int b = 0; b < NK; ++b) {
      if (b >= nR) break;
      px += G[Ridx[b] * NX + lx] * rd_lane(sl, NX + b);
    }
    double dx, dlam;
    solve(rx - px, rl - gl, dx, dlam);
    sx += dx;
    sl += dlam;
  }
  if (hx) xx[l] = sx;
  for (int row = l; row < M; row += 64) yy[row] = 0.0;
  wsync();
  if (hl) yy[NX + gi] = sl;
  wsync();
  return true;
}

// Equality-constrained QP on the flagged rows (OSQP polish's reduced KKT):
// bound-active variables are fixed at their bound (eliminated exactly), the
// active G rows enter [P_FF + dI, G_RF^T; G_RF, -dI] solved by a packed
// left-looking LDL^T with iterative refinement against the unregularised
// system.  Writes the full primal xx[nx] and dual yy[m] (scaled space).
// Flags: actb (bound row l) / actg (G row l) held by lane l.
template <class QD>
__device__ __forceinline__ bool eqp(const KParams& kp, double* S, int actb, int actg, double* xx, double* yy) {
  using GL = Grp<QD::gs>;
  const int l = GL::lane(), nx = DNX, ng = DNG, np = DNP, m = DM;
  const double *P = S + kp.oP, *G = S + kp.oG, *q = S + kp.oQ, *ab = S + kp.oAB, *lo = S + kp.oL,
               *up = S + kp.oU;
  unsigned long long freeMask = GL::ballot(l < nx && actb == 0);
  unsigned long long rowMask = GL::ballot(l < ng && actg != 0);
  const int nF = __popcll(freeMask), nR = __popcll(rowMask), N = nF + nR;
  if (N > kp.ncap) return false;  // uniform: this polish attempt fails, ADMM continues
#ifdef DRC_PHASE_TIMING
  const unsigned long long eq_t0 = __builtin_amdgcn_s_memtime();
  if (l == 0) {
    atomicAdd(&g_phase_cycles[41], 1ull);
    atomicAdd(&g_phase_cycles[42], (unsigned long long)N);
  }
#endif
  if constexpr (QD::gs < 64) {  // two instances per wave: register EQP only (ncap <= kEqpRegCap)
    if (N > kEqpRegCap) return false;
  }
  if constexpr (QD::nx > 0 && QD::nx == QD::np && QD::gs == 64) {  // whole-body shapes: range-space form
    if (kp.oHi >= 0 && nF == QD::nx && nR <= kEqpRegCap) {
      const bool ok_ = eqp_range<QD>(kp, S, actg, xx, yy, rowMask, nR);
#ifdef DRC_PHASE_TIMING
      if (l == 0) atomicAdd(&g_phase_cycles[40], __builtin_amdgcn_s_memtime() - eq_t0);
#endif
      return ok_;
    }
    if (kp.oHi >= 0) return false;  // no LDS LDL^T region in this plan (never reached: no variable bounds)
  }
  if constexpr (QD::nx > 0) {
    if (N <= kEqpRegCap) {
      const bool ok_ = eqp_regs<QD>(kp, S, actb, actg, xx, yy, freeMask, rowMask, nF, nR);
#ifdef DRC_PHASE_TIMING
      if (l == 0) atomicAdd(&g_phase_cycles[40], __builtin_amdgcn_s_memtime() - eq_t0);
#endif
      return ok_;
    }
  }
  double* U = S + kp.oU0;
  int* Fidx = reinterpret_cast<int*>(U);  // 64 ints
  int* Ridx = Fidx + 64;                   // 64 ints
  const int nb = kp.nbuf;                   // >= N
  double* rhs = U + 64 + 64 + 128;         // [N]  (xx, yy live at U+64 / U+128)
  double* sol = rhs + nb;
  double* res = sol + nb;
  double* vv = res + nb;
  double* dg = vv + nb;
  double* L = dg + nb;  // packed lower triangle N(N+1)/2
  if (l < nx && actb == 0) Fidx[__popcll(freeMask & ((1ull << l) - 1))] = l;
  if (l < ng && actg != 0) Ridx[__popcll(rowMask & ((1ull << l) - 1))] = l;
  if (l < nx) xx[l] = actb == 0 ? 0.0 : (actb < 0 ? lo[l] : up[l]) / ab[l];
  wsync();
  const double dl = kp.s.delta;
  for (int i = l; i < N; i += GL::size) {  // K (packed rows i >= j) and rhs; lane i owns row i
    if (i < nF) {
      int fi = Fidx[i];
      for (int j = 0; j <= i; ++j) {
        int fj = Fidx[j];
        double v = (fi < np && fj < np) ? P[fi * np + fj] : 0.0;
        L[pk(i, j)] = v + (i == j ? dl : 0.0);
      }
      double r = -q[fi];
      if (fi < np)
        for (int c = 0; c < np; ++c)
          if (xx[c] != 0.0) r -= P[fi * np + c] * xx[c];
      rhs[i] = r;
    } else {
      int gi = Ridx[i - nF], row = nx + gi;
      for (int j = 0; j < nF; ++j) L[pk(i, j)] = G[gi * nx + Fidx[j]];
      for (int j = nF; j <= i; ++j) L[pk(i, j)] = (i == j) ? -dl : 0.0;
      // the lane owning G row gi knows its side; read it back through the flags
      double r = 0;
      (void)row;
      rhs[i] = r;
    }
  }
  // rhs of the active G rows: b = l or u of that row, minus the fixed part
  if (l < ng && actg != 0) {
    const int i = nF + __popcll(rowMask & ((1ull << l) - 1)), row = nx + l;
    double r = actg < 0 ? lo[row] : up[row];
    for (int c = 0; c < nx; ++c)
      if (xx[c] != 0.0) r -= G[l * nx + c] * xx[c];
    rhs[i] = r;
  }
  wsync();
  for (int j = 0; j < N; ++j) {  // left-looking LDL^T, in place
    for (int k = l; k < j; k += GL::size) vv[k] = L[pk(j, k)] * dg[k];
    wsync();
    double part = 0;
    for (int k = l; k < j; k += GL::size) part += L[pk(j, k)] * vv[k];
    double dj = L[pk(j, j)] - GL::sum(part);
    if (dj == 0.0) return false;  // uniform
    for (int i = l; i < N; i += GL::size)
      if (i > j) {
        double t = L[pk(i, j)];
        for (int k = 0; k < j; ++k) t -= L[pk(i, k)] * vv[k];
        L[pk(i, j)] = t / dj;
      }
    if (l == 0) dg[j] = dj;
    wsync();
  }
  for (int i = l; i < N; i += GL::size) sol[i] = rhs[i];
  wsync();
  ldl_solve(L, dg, N, sol);
  for (int it = 0; it < kp.s.polish_refine_iter; ++it) {
    for (int i = l; i < N; i += GL::size) {
      double r = rhs[i];
      if (i < nF) {
        int fi = Fidx[i];
        if (fi < np)
          for (int j = 0; j < nF; ++j) {
            int fj = Fidx[j];
            if (fj < np) r -= P[fi * np + fj] * sol[j];
          }
        for (int k = 0; k < nR; ++k) r -= G[Ridx[k] * nx + fi] * sol[nF + k];
      } else {
        int gi = Ridx[i - nF];
        for (int j = 0; j < nF; ++j) r -= G[gi * nx + Fidx[j]] * sol[j];
      }
      res[i] = r;
    }
    wsync();
    ldl_solve(L, dg, N, res);
    for (int i = l; i < N; i += GL::size) sol[i] += res[i];
    wsync();
  }
  for (int i = l; i < nF; i += GL::size) xx[Fidx[i]] = sol[i];
  for (int row = l; row < m; row += GL::size) yy[row] = 0.0;
  wsync();
  for (int k = l; k < nR; k += GL::size) yy[nx + Ridx[k]] = sol[nF + k];
  wsync();
  if (l < nx && actb != 0) {  // bound multipliers from stationarity
    double g = q[l];
    if (l < np)
      for (int c = 0; c < np; ++c) g += P[l * np + c] * xx[c];
    for (int i = 0; i < ng; ++i) g += G[i * nx + l] * yy[nx + i];
    yy[l] = -g / ab[l];
  }
  wsync();
#ifdef DRC_PHASE_TIMING
  if (l == 0) atomicAdd(&g_phase_cycles[40], __builtin_amdgcn_s_memtime() - eq_t0);
#endif
  return true;
}

// OSQP polish (polish.c) restated.  strict == 0: OSQP's single attempt and
// acceptance rule.  strict != 0 (parity mode): accept only a KKT-certified
// point (residuals at eps_exact, dual signs matching the active bounds); on a
// wrong ADMM active-set guess continue with a primal active-set method
// (Nocedal & Wright Alg. 16.3) from the first feasible polished point.  Same
// decisions, in the same row order, as oracle/drc_oracle.c:qp_polish.
constexpr int kPolishFeasAttempts = 4, kPolishAsIters = 24;
template <class QD>
__device__ __forceinline__ bool polish(const KParams& kp, double* S, bool strict) {
  using GL = Grp<QD::gs>;
  const int l = GL::lane(), nx = DNX, ng = DNG, np = DNP, m = DM;
  const double *G = S + kp.oG, *ab = S + kp.oAB, *lo = S + kp.oL, *up = S + kp.oU, *E = S + kp.oE;
  double *x = S + kp.oX, *z = S + kp.oZ, *y = S + kp.oY;
  (void)np;
  int actb = 0, actg = 0;
  if (l < nx) actb = (z[l] - lo[l] < -y[l]) ? -1 : ((up[l] - z[l] < y[l]) ? 1 : 0);
  if (l < ng) {
    int r = nx + l;
    actg = (z[r] - lo[r] < -y[r]) ? -1 : ((up[r] - z[r] < y[r]) ? 1 : 0);
  }
  double* U = S + kp.oU0;
  double* xx = U + 64;       // [nx]
  double* yy = U + 128;      // [m] (<= 128)
  double* zz = S + kp.oT2;   // z candidate
  double* xc = S + kp.oXT;   // feasible iterate of the active-set phase
  double* sc = S + kp.oSc;
  const double pr0 = sc[SC_PRI], dr0 = sc[SC_DUA];
  bool have_feas = false;
  const int iters = strict ? kPolishFeasAttempts + kPolishAsIters : 1;
  for (int it = 0; it < iters; ++it) {
    {
      // a working-set G row with no weight on the free variables depends on
      // the fixed bounds alone and makes the reduced KKT singular (its
      // solution then hangs on rounding noise, e.g. the structurally-zero
      // manipulability gradient of the first/last joint).  When the fixed
      // values already satisfy it strictly it is not active: drop it (the
      // oracle's qp_polish applies the same rule)
      const unsigned long long fixed = GL::ballot(l < nx && actb != 0), atup = GL::ballot(l < nx && actb > 0);
      if (l < ng && actg != 0) {
        const int lg = l < ng ? l : 0, row = nx + lg;
        double sf = 0, sa = 0, act = 0;
#pragma unroll
        for (int j = 0; j < nx; ++j) {
          const double g = G[lg * nx + j];
          sa = fmax(sa, fabs(g));
          if (!((fixed >> j) & 1ull)) sf = fmax(sf, fabs(g));
          else act += g * (((atup >> j) & 1ull) ? up[j] : lo[j]) / ab[j];
        }
        const double b = actg < 0 ? lo[row] : up[row], slack = actg < 0 ? act - b : b - act;
        if (sf <= 1e-12 * sa && slack > 1e-12 * (fabs(act) + fabs(b))) actg = 0;
      }
    }
    if (!eqp<QD>(kp, S, actb, actg, xx, yy)) break;
    if (have_feas) {
      double stepmax = 0, xnorm = 0;
      if (l < nx) {
        stepmax = fabs(xx[l] - xc[l]);
        xnorm = fabs(xc[l]);
      }
      stepmax = GL::max(stepmax);
      xnorm = GL::max(xnorm);
      if (stepmax > 1e-12 * (1 + xnorm)) {
        // ratio test along p = xx - xc over the inactive rows
        double amin = 1.0;
        int blk = 0x7fffffff, side = 0;
        if (l < nx && actb == 0) {
          double axc = ab[l] * xc[l], ap = ab[l] * (xx[l] - xc[l]), a = 2.0;
          int sd = 0;
          if (ap < 0 && lo[l] > -kInf * kMinScaling) { a = (lo[l] - axc) / ap; sd = -1; }
          else if (ap > 0 && up[l] < kInf * kMinScaling) { a = (up[l] - axc) / ap; sd = 1; }
          if (a < amin) { amin = a; blk = l; side = sd; }
        }
        if (l < ng && actg == 0) {
          const int lg = l < ng ? l : 0, row = nx + lg;
          double axc = 0, ap = 0, a = 2.0;
#pragma unroll
          for (int j = 0; j < nx; ++j) {
            axc += G[lg * nx + j] * xc[j];
            ap += G[lg * nx + j] * (xx[j] - xc[j]);
          }
          int sd = 0;
          if (ap < 0 && lo[row] > -kInf * kMinScaling) { a = (lo[row] - axc) / ap; sd = -1; }
          else if (ap > 0 && up[row] < kInf * kMinScaling) { a = (up[row] - axc) / ap; sd = 1; }
          if (a < amin) { amin = a; blk = row; side = sd; }
        }
        int enc = blk == 0x7fffffff ? blk : blk * 4 + (side + 1);
        GL::argmin(amin, enc);
        const double alpha = amin < 0 ? 0.0 : amin;
        wsync();
        if (l < nx) xc[l] += alpha * (xx[l] - xc[l]);
        wsync();
        if (enc != 0x7fffffff && amin < 1.0) {
          CK_N(47);
          const int row = enc >> 2, sd = (enc & 3) - 1;
          if (row < nx) { if (l == row) actb = sd; }
          else if (l == row - nx) actg = sd;
          continue;
        }
      }
    }
    // candidate point: z = clamp(A x), residuals, certification
    double axb = 0, axg = 0;
    if (l < nx) {
      axb = ab[l] * xx[l];
      zz[l] = fmin(fmax(axb, lo[l]), up[l]);
    }
    if (l < ng) {
      const int lg = l < ng ? l : 0;
#pragma unroll
      for (int j = 0; j < nx; ++j) axg += G[lg * nx + j] * xx[j];
      zz[nx + lg] = fmin(fmax(axg, lo[nx + lg]), up[nx + lg]);
    }
    wsync();
#ifdef DRC_PHASE_TIMING
    const unsigned long long rs_t0 = __builtin_amdgcn_s_memtime();
#endif
    residuals<QD, false>(kp, S, xx, zz, yy, kp.s.eps_exact, kp.s.eps_exact);
#ifdef DRC_PHASE_TIMING
    if (l == 0) atomicAdd(&g_phase_cycles[43], __builtin_amdgcn_s_memtime() - rs_t0);
#endif
    const double pr1 = sc[SC_PRI], dr1 = sc[SC_DUA], epsp = sc[SC_EPSP], epsd = sc[SC_EPSD], c = sc[SC_C];
    bool ok = (pr1 < pr0 && dr1 < dr0) || (pr1 < pr0 && dr0 < 1e-10) || (dr1 < dr0 && pr0 < 1e-10);
    double wv = 0;
    int worst = 0x7fffffff;
    bool feasible = pr1 <= epsp;
    if (strict) {
      ok = feasible && dr1 <= epsd;
      if (l < nx && actb != 0 && lo[l] != up[l]) {
        double yi = E[l] * yy[l] / c, viol = actb < 0 ? yi - epsd : -yi - epsd;
        if (viol > wv) { wv = viol; worst = l; }
      }
      if (l < ng && actg != 0 && lo[nx + l] != up[nx + l]) {
        double yi = E[nx + l] * yy[nx + l] / c, viol = actg < 0 ? yi - epsd : -yi - epsd;
        if (viol > wv) { wv = viol; worst = nx + l; }
      }
      GL::argmax(wv, worst);
      if (worst != 0x7fffffff) ok = false;
#ifdef DRC_QP_DEBUG
      {
        const unsigned long long fb = GL::ballot(l < nx && actb != 0), fg = GL::ballot(l < ng && actg != 0);
        if (l == 0)
          printf("polish it %d feas %d pri %.2e dua %.2e worst %d (%.2e) havefeas %d bmask %llx gmask %llx\n", it,
                 (int)feasible, pr1, dr1, worst, wv, (int)have_feas, fb, fg);
      }
#endif
      if (!ok && feasible && !have_feas) {
        if (l < nx) xc[l] = xx[l];
        have_feas = true;
      }
    }
    if (ok) {
      if (l < nx) x[l] = xx[l];
      for (int row = l; row < m; row += GL::size) {
        y[row] = yy[row];
        z[row] = zz[row];
      }
      wsync();
      return true;
    }
    if (!strict) break;
    if (have_feas) {
      if (worst == 0x7fffffff) {
        CK_N(48);
        break;  // KKT residual failure, not an active-set issue
      }
      CK_N(46);
      if (worst < nx) { if (l == worst) actb = 0; }
      else if (l == worst - nx) actg = 0;
      if (l < nx) xc[l] = xx[l];
      wsync();
    } else {
      if (it >= kPolishFeasAttempts - 1) break;
      // not yet feasible: add every violated inactive row at its violated
      // side (QPIK: the ADMM guess typically misses a couple), or only the
      // most violated one (QPID); the oracle makes the same choice
      // (polish_add_all)
      int sb = 0, sg = 0, add = 0x7fffffff;
      double av = 0;
      if (l < nx && actb == 0) {
        const double vlo = (lo[l] - axb) / E[l] - epsp, vhi = (axb - up[l]) / E[l] - epsp;
        if (vlo > 0 || vhi > 0) sb = vhi > vlo ? 1 : -1;
        if (vlo > av) { av = vlo; add = l * 4 + 0; }
        if (vhi > av) { av = vhi; add = l * 4 + 2; }
      }
      if (l < ng && actg == 0) {
        const int row = nx + l;
        const double vlo = (lo[row] - axg) / E[row] - epsp, vhi = (axg - up[row]) / E[row] - epsp;
        if (vlo > 0 || vhi > 0) sg = vhi > vlo ? 1 : -1;
        if (vlo > av) { av = vlo; add = row * 4 + 0; }
        if (vhi > av) { av = vhi; add = row * 4 + 2; }
      }
      CK_N(45);
      if (!GL::any(sb != 0 || sg != 0)) {
        if (worst == 0x7fffffff) break;
        if (worst < nx) { if (l == worst) actb = 0; }
        else if (l == worst - nx) actg = 0;
      } else if (kp.problem == 0) {
        if (sb) actb = sb;
        if (sg) actg = sg;
      } else {
        GL::argmax(av, add);
        const int row = add >> 2, sd = (add & 3) - 1;
        if (row < nx) { if (l == row) actb = sd; }
        else if (l == row - nx) actg = sd;
      }
    }
  }
  if (l == 0) {  // restore the ADMM residuals for the caller
    sc[SC_PRI] = pr0;
    sc[SC_DUA] = dr0;
  }
  wsync();
  return false;
}

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
};

// ------------------------------------------------------------------------
// QPID stage data.  Pinocchio's LOCAL_WORLD_ALIGNED
// Jacobian time variation is d/dt of the LWA Jacobian (robot_data.cpp:109,
// 414, 476-477).  Column c of the Jacobian of a point p carried by a body,
// differentiated with the joint velocities restricted to `mask`:
//   revolute c:  [zd x (p - o_c) + z_c x (pdot - od_c); zd],  zd = w_par(c) x z_c
//   prismatic c: [zd; 0]
// with w_par(c) the angular velocity of c's parent body and od_c the velocity
// of c's origin.  One lane per column, O(nv) per lane.
// ------------------------------------------------------------------------
__device__ __forceinline__ void col_dot(const DevModel* M, const double* T, const double* Zw, const double* qd, int nv,
                                        int c, V3 p, V3 pdot, uint32_t mask, V3* lin, V3* ang) {
  const V3 oc = v3(T[12 * c + 9], T[12 * c + 10], T[12 * c + 11]), zc = ld3(Zw + 3 * c);
  V3 w = v3(0, 0, 0), od = v3(0, 0, 0);
  const uint32_t ac = M->anc[c] & mask;
  for (int a = 1; a <= nv; ++a) {
    if (!(ac & (1u << (a - 1)))) continue;
    const V3 za = ld3(Zw + 3 * a);
    if (M->jtype[a] == kRevolute) {
      if (a != c) w = w + qd[a - 1] * za;
      od = od + qd[a - 1] * cross(za, oc - v3(T[12 * a + 9], T[12 * a + 10], T[12 * a + 11]));
    } else {
      od = od + qd[a - 1] * za;
    }
  }
  const V3 zd = cross(w, zc);
  if (M->jtype[c] == kRevolute) {
    *lin = cross(zd, p - oc) + cross(zc, pdot - od);
    *ang = zd;
  } else {
    *lin = zd;
    *ang = v3(0, 0, 0);
  }
}

// velocity and angular velocity of the body of joint X (point p on it)
__device__ __forceinline__ void body_velocity(const DevModel* M, const double* T, const double* Zw, const double* qd,
                                              int nv, int X, V3 p, V3* v, V3* w) {
  *v = v3(0, 0, 0);
  *w = v3(0, 0, 0);
  if (X <= 0) return;
  const uint32_t ax = M->anc[X];
  for (int a = 1; a <= nv; ++a) {
    if (!(ax & (1u << (a - 1)))) continue;
    const V3 za = ld3(Zw + 3 * a);
    if (M->jtype[a] == kRevolute) {
      *w = *w + qd[a - 1] * za;
      *v = *v + qd[a - 1] * cross(za, p - v3(T[12 * a + 9], T[12 * a + 10], T[12 * a + 11]));
    } else {
      *v = *v + qd[a - 1] * za;
    }
  }
}

// Fills kBias = [Jdot v (6), man_gd, dist_gd] and kJd (6 x nv frame Jdot):
//   v = qdot (manipulator) or S eta (MoMa, getJacobianActuatedTimeVariation *
//       eta, mobile_manipulator/robot_data.cpp:412-415, Sdot neglected);
//   man_gd  = getManipulability(true,true).grad_dot . qdot_arm, contracted:
//       sum_i qdot_i dJ_i = Da (arm-only Jdot), so with W = Ja^T Ai
//       man_gd = mdot tr(Da W) + m [tr(Da Jda^T Ai) - 2 tr((Da W)(Jda W))],
//       mdot = m tr(Jda W)           (robot_data.cpp:555-569, MoMa :477-492);
//   dist_gd = getMinDistance(..,true,..).grad_dot . qdot_arm
//       = sum_{c in arm} qdot_c n.(JB_dot - JA_dot)[:, c]   (robot_data.cpp:496-512).
// full: also the reference's grad_dot VECTORS (stage outputs) into kGdv =
//   [getManipulability grad_dot (narm) | getMinDistance grad_dot (nv)].
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

__device__ __noinline__ void qpid_task_extras(const DevModel* M, const KParams& kp, double* S, double bestd,
                                              int besti, bool full) {
  const int l = lane_id(), nv = kp.nv, narm = kp.narm, c0 = kp.c0;
  const double *T = S + kp.kT, *Zw = S + kp.kZ, *J = S + kp.kJ, *qd = S + kp.kqd, *Te = S + kp.kTe,
               *red = S + kp.oRed, *W = S + kp.kW, *Ai = S + kp.kAi, *qv = S + kp.kq;
  double *Jd = S + kp.kJd, *Da = S + kp.kDa, *vf = S + kp.kVf, *X = S + kp.kX6, *out = S + kp.kBias;
  const uint32_t all = 0xffffffffu, arm = ((1u << narm) - 1) << c0;
  const uint32_t anc_e = M->anc[kp.frame_joint];
  const V3 pe = v3(Te[9], Te[10], Te[11]);
  V3 ve = v3(0, 0, 0), va = v3(0, 0, 0);  // frame-point velocity: full / arm joints only
  for (int c = 0; c < nv; ++c) {
    const V3 jc = v3(J[c], J[nv + c], J[2 * nv + c]);
    ve = ve + qd[c] * jc;
    if (arm & (1u << c)) va = va + qd[c] * jc;
  }
  double dsum = 0;
  const double(*Jm)[kMaxWheels] = mobile_jac(M, kp, S, qv);  // read for mobile manipulators only
  if (l < nv) {
    const int j = l + 1;
    V3 lin = v3(0, 0, 0), ang = v3(0, 0, 0), lina = v3(0, 0, 0), anga = v3(0, 0, 0);
    if (anc_e & (1u << l)) {
      col_dot(M, T, Zw, qd, nv, j, pe, ve, all, &lin, &ang);
      if (arm & (1u << l)) col_dot(M, T, Zw, qd, nv, j, pe, va, arm, &lina, &anga);
    }
    Jd[0 * nv + l] = lin.x; Jd[1 * nv + l] = lin.y; Jd[2 * nv + l] = lin.z;
    Jd[3 * nv + l] = ang.x; Jd[4 * nv + l] = ang.y; Jd[5 * nv + l] = ang.z;
    if (arm & (1u << l)) {
      const int c = l - c0;
      Da[0 * narm + c] = lina.x; Da[1 * narm + c] = lina.y; Da[2 * narm + c] = lina.z;
      Da[3 * narm + c] = anga.x; Da[4 * narm + c] = anga.y; Da[5 * narm + c] = anga.z;
    }
    // actuated velocity mapped to the joints: S eta (MoMa robot_data.cpp:115-120)
    double v = qd[l];
    if (M->kind == 1 && l >= M->virtual_start && l < M->virtual_start + 3) {
      const int r = l - M->virtual_start;
      const double yaw = qv[M->virtual_start + 2], cy = cos(yaw), sy = sin(yaw);
      v = 0;
      for (int w = 0; w < M->n_wheel; ++w) {
        const double j0 = Jm[0][w], j1 = Jm[1][w], j2 = Jm[2][w];
        const double sw = r == 0 ? cy * j0 - sy * j1 : (r == 1 ? sy * j0 + cy * j1 : j2);
        v += sw * qd[M->mobi_start + w];
      }
    }
    vf[l] = v;
    // self-collision grad_dot of this column (robot_data.cpp:496-512)
    double gcol = 0;
    if (besti < M->npairs && (full || (arm & (1u << l)))) {
      const V3 pA = ld3(red), pB = ld3(red + 3);
      V3 n = pB - pA;
      n = (1.0 / sqrt(dot(n, n))) * n;
      V3 jdx[2];
      for (int s_ = 0; s_ < 2; ++s_) {
        const int jX = M->gparent[s_ == 0 ? M->pair_a[besti] : M->pair_b[besti]];
        jdx[s_] = v3(0, 0, 0);
        if (jX <= 0 || !(M->anc[jX] & (1u << l))) continue;
        const V3 oX = v3(T[12 * jX + 9], T[12 * jX + 10], T[12 * jX + 11]);
        const V3 pX = s_ == 0 ? pA : pB, zj = ld3(Zw + 3 * j);
        V3 cl, ca;  // column of the joint Jacobian of jX at oX
        if (M->jtype[j] == kRevolute) {
          cl = cross(zj, oX - v3(T[12 * j + 9], T[12 * j + 10], T[12 * j + 11]));
          ca = zj;
        } else {
          cl = zj;
          ca = v3(0, 0, 0);
        }
        V3 vX, wX, ld, ad;
        body_velocity(M, T, Zw, qd, nv, jX, oX, &vX, &wX);
        col_dot(M, T, Zw, qd, nv, j, oX, vX, all, &ld, &ad);
        const V3 r = pX - oX, rd = cross(wX, r);
        jdx[s_] = ld - (cross(rd, ca) + cross(r, ad));
      }
      gcol = dot(n, jdx[1] - jdx[0]);
      if (arm & (1u << l)) dsum = qd[l] * gcol;
    }
    if (full) S[kp.kGdv + narm + l] = gcol;
  }
  const double dist_gd = wave_sum(dsum);
  (void)bestd;
  wsync();
  // 6x6 products for the manipulability term (lanes (a, b))
  double t1 = 0, t2 = 0, t3 = 0;
  if (l < 36) {
    const int a = l / 6, b = l % 6;
    double x1 = 0, x2 = 0, x3 = 0;
    for (int c = 0; c < narm; ++c) {
      const double dac = Da[a * narm + c], jac = Jd[a * nv + c0 + c];
      x1 += dac * W[c * 6 + b];
      x2 += jac * W[c * 6 + b];
      x3 += dac * Jd[b * nv + c0 + c];
    }
    X[l] = x1;
    X[36 + l] = x2;
    if (a == b) {
      t1 = x2;
      t2 = x1;
    }
    t3 = x3 * Ai[b * 6 + a];
  }
  wsync();
  double t4 = 0;
  if (l < 36) t4 = X[l] * X[36 + (l % 6) * 6 + l / 6];
  t1 = wave_sum(t1);
  t2 = wave_sum(t2);
  t3 = wave_sum(t3);
  t4 = wave_sum(t4);
  const double m = S[kp.oSc + SC_MAN], mdot = m * t1;
  if (l < 6) {
    double s = 0;
    for (int c = 0; c < nv; ++c) s += Jd[l * nv + c] * vf[c];
    out[l] = s;
  }
  if (l == 0) {
    out[6] = mdot * t2 + m * (t3 - 2.0 * t4);
    out[7] = dist_gd;
  }
  if (full) {
    // grad_dot_k = mdot tr(dJ_k Ja^T Ai) + m tr(dJ_k (Jda^T Ai + Ja^T Ai_dot)),
    // Ja^T Ai_dot = -2 W (Jda W) = -2 W X2; lane per (k, c) builds dJ_k[:, c]
    // (the manipulability gradient's closed form) and dots it with the rows.
    double* Y = X + 72;  // narm x 6: Jda^T Ai - 2 W X2
    for (int e = l; e < narm * 6; e += 64) {
      const int c = e / 6, a = e % 6;
      double y = 0;
      for (int b_ = 0; b_ < 6; ++b_) y += Jd[b_ * nv + c0 + c] * Ai[b_ * 6 + a] - 2.0 * W[c * 6 + b_] * X[36 + b_ * 6 + a];
      Y[e] = y;
    }
    wsync();
    double* part = X + 72 + 6 * narm;  // narm x narm x 2
    for (int e = l; e < narm * narm; e += 64) {
      const int kk = e / narm, c = e % narm, jk = c0 + kk + 1, ji = c0 + c + 1;
      double p1 = 0, p2 = 0;
      if ((anc_e & (1u << (jk - 1))) && (anc_e & (1u << (ji - 1)))) {
        const V3 zk = ld3(Zw + 3 * jk), zi = ld3(Zw + 3 * ji);
        const V3 pk_ = v3(T[12 * jk + 9], T[12 * jk + 10], T[12 * jk + 11]);
        const V3 pi_ = v3(T[12 * ji + 9], T[12 * ji + 10], T[12 * ji + 11]);
        const bool krev = M->jtype[jk] == kRevolute;
        const V3 dpe = krev ? cross(zk, pe - pk_) : zk;
        const bool moves_i = jk != ji && (M->anc[ji] & (1u << (jk - 1)));
        const V3 dzi = (moves_i && krev) ? cross(zk, zi) : v3(0, 0, 0);
        const V3 dpi = moves_i ? (krev ? cross(zk, pi_ - pk_) : zk) : v3(0, 0, 0);
        V3 lin, ang;
        if (M->jtype[ji] == kRevolute) {
          lin = cross(dzi, pe - pi_) + cross(zi, dpe - dpi);
          ang = dzi;
        } else {
          lin = dzi;
          ang = v3(0, 0, 0);
        }
        const double *w = W + c * 6, *y = Y + c * 6;
        p1 = lin.x * w[0] + lin.y * w[1] + lin.z * w[2] + ang.x * w[3] + ang.y * w[4] + ang.z * w[5];
        p2 = lin.x * y[0] + lin.y * y[1] + lin.z * y[2] + ang.x * y[3] + ang.y * y[4] + ang.z * y[5];
      }
      part[2 * e] = p1;
      part[2 * e + 1] = p2;
    }
    wsync();
    if (l < narm) {
      double s1 = 0, s2 = 0;
      for (int c = 0; c < narm; ++c) {
        s1 += part[2 * (l * narm + c)];
        s2 += part[2 * (l * narm + c) + 1];
      }
      S[kp.kGdv + l] = mdot * s1 + m * s2;
    }
  }
  wsync();
}

// ------------------------------------------------------------------------
// Closed-form controllers, Manipulator::RobotController
// (robot_controller.cpp:156-275), on the task stage's J and task vector
// (xdd: CLIK Kp e + xdot_target; OSF Kp e + Kv edot, or xddot_target):
//   CLIK: qdot = J^+ xdd + (I - J^+ J) nu,              J^+ = PinvCOD(J)
//   OSF:  Lambda = PinvCOD(J M^-1 J^T), tau = J^T Lambda xdd + (I - J^T Lambda J M^-1) nu + g
// Small dense products are lane-parallel; a 6x6 SPD inverse goes through six
// lane-parallel Jordan exchanges when the Frobenius condition estimate
// certifies that PinvCOD keeps every mode (< 1e5), otherwise one lane runs the
// serial COD (PinvCOD's rank cut).
// ------------------------------------------------------------------------
__device__ __forceinline__ bool inv6_certified(const double* A, double* Ai) {
  const int l = lane_id(), ii = l / 6, jj = l % 6;
  if (l < 36) Ai[l] = A[l];
  wsync();
  double piv_min = 1e300;
  for (int k = 0; k < 6; ++k) {
    const double akk = Ai[k * 6 + k];
    double nv_ = 0;
    if (l < 36) {
      const double aij = Ai[l], aik = Ai[ii * 6 + k], akj = Ai[k * 6 + jj];
      if (ii == k && jj == k) nv_ = 1.0 / akk;
      else if (ii == k) nv_ = akj / akk;
      else if (jj == k) nv_ = -aik / akk;
      else nv_ = aij - aik * akj / akk;
    }
    piv_min = fmin(piv_min, akk);
    wsync();
    if (l < 36) Ai[l] = nv_;
    wsync();
  }
  const double fa = wave_sum(l < 36 ? A[l] * A[l] : 0.0), fi = wave_sum(l < 36 ? Ai[l] * Ai[l] : 0.0);
  return piv_min > 0 && fa * fi < 1e10;
}

__device__ __noinline__ void closed_form_stage(const DevModel* M, const KParams& kp, double* S, const IO& io,
                                               int64_t gb, int64_t LD) {
  const int l = lane_id(), nv = kp.nv;
  const double *J = S + kp.kJ, *xdd = S + kp.kxdd;
  double* A6 = S + kp.kA6;
  double* Ai = S + kp.kAi;
  double* W = S + kp.kCf;           // 6 x nv: J^+ ^T (CLIK) / J M^-1 (OSF)
  double* W2 = W + 6 * nv;          // 6 x nv: Lambda J M^-1 (OSF)
  double* Mi = W2 + 6 * nv;         // nv x nv
  double* nu = Mi + nv * nv;        // nv
  double* gv = nu + nv;             // nv
  double* vec = gv + 2 * nv;        // 48: task vectors
  double* ws = vec + 48;            // serial COD work
  if (l < nv) {
    nu[l] = io.cf_null ? io.cf_null[(int64_t)l * LD + gb] : 0.0;
    if (kp.cf == 2) gv[l] = io.dG[(int64_t)l * LD + gb];
  }
  if (kp.cf == 2)
    for (int e = l; e < nv * nv; e += 64) Mi[e] = io.dM[(int64_t)e * LD + gb];
  wsync();
  double out = 0;
  if (kp.cf == 1) {  // CLIK (robot_controller.cpp:156-172)
    if (l < 36) {
      const int a = l / 6, b = l % 6;
      double s = 0;
      for (int c = 0; c < nv; ++c) s += J[a * nv + c] * J[b * nv + c];
      A6[l] = s;
    }
    wsync();
    if (inv6_certified(A6, Ai)) {  // J^+ = J^T (J J^T)^-1, stored transposed: W[i][c] = J^+[c][i]
      for (int e = l; e < 6 * nv; e += 64) {
        const int i = e / nv, c = e % nv;
        double s = 0;
        for (int r = 0; r < 6; ++r) s += J[r * nv + c] * Ai[r * 6 + i];
        W[e] = s;
      }
    } else if (l == 0) {
      double* X = ws + 6 * nv + 36 + 6 * nv + 18 + 2 * nv;  // nv x 6 after the COD work
      pinv_cod_rect(J, 6, nv, X, ws);
      for (int c = 0; c < nv; ++c)
        for (int i = 0; i < 6; ++i) W[i * nv + c] = X[c * 6 + i];
    }
    wsync();
    if (l < 6) {
      double s = 0;
      for (int c = 0; c < nv; ++c) s += J[l * nv + c] * nu[c];
      vec[l] = xdd[l] - s;  // xdd - J nu
    }
    wsync();
    if (l < nv) {
      double s = nu[l];
      for (int i = 0; i < 6; ++i) s += W[i * nv + l] * vec[i];
      out = s;
    }
  } else {  // OSF (robot_controller.cpp:216-230)
    for (int e = l; e < 6 * nv; e += 64) {
      const int i = e / nv, c = e % nv;
      double s = 0;
      for (int a = 0; a < nv; ++a) s += J[i * nv + a] * Mi[a * nv + c];
      W[e] = s;
    }
    wsync();
    if (l < 36) {
      const int a = l / 6, b = l % 6;
      double s = 0;
      for (int c = 0; c < nv; ++c) s += W[a * nv + c] * J[b * nv + c];
      A6[l] = s;
    }
    wsync();
    if (!inv6_certified(A6, Ai)) {
      if (l == 0) pinv_cod6(A6, Ai, ws);
      wsync();
    }
    for (int e = l; e < 6 * nv; e += 64) {
      const int i = e / nv, c = e % nv;
      double s = 0;
      for (int j = 0; j < 6; ++j) s += Ai[i * 6 + j] * W[j * nv + c];
      W2[e] = s;
    }
    if (l < 6) {
      double s = 0;
      for (int j = 0; j < 6; ++j) s += Ai[l * 6 + j] * xdd[j];
      vec[l] = s;  // F = Lambda xdd
    }
    wsync();
    if (l < 6) {
      double s = 0;
      for (int c = 0; c < nv; ++c) s += W2[l * nv + c] * nu[c];
      vec[6 + l] = vec[l] - s;  // F - J_T_pinv nu
    }
    wsync();
    if (l < nv) {
      double s = gv[l] + nu[l];
      for (int i = 0; i < 6; ++i) s += J[i * nv + l] * vec[6 + i];
      out = s;
    }
  }
  if (l < nv) io.out[(int64_t)l * LD + gb] = out;
  wsync();
}

// Occupancy target of the task kernel (waves per SIMD): the lane-serial
// narrow phase and task-velocity code would otherwise take all 512 registers.
#ifndef DRC_TASK_WAVES
#define DRC_TASK_WAVES 2
#endif
// PROBLEM 0: QPIK stage data; 1: also the QPID extras (a separate
// instantiation, so the QPIK kernel carries no call frame for them)
template <int PROBLEM>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(DRC_TASK_WAVES, 8))) task_kernel(const DevModel* __restrict__ M0, const KParams kp, const IO io) {
  extern __shared__ __attribute__((aligned(16))) double S[];
  const int l = lane_id();
  const int nv = kp.nv;
  const int64_t B = io.B;
  EpaPoly* ews = reinterpret_cast<EpaPoly*>(S + kp.kEpa);  // LDS-resident polytope
  PH_DECL
  // hard mode: the instances the lane-per-instance stage left (grid stride)
  const bool hard_mode = io.hard_mode != 0;
  const InstSeq seq(hard_mode ? int64_t(*io.hard_n) : B, hard_mode ? 0 : kp.xcd_map, hard_mode ? nullptr : io.queue);
  for (int64_t j = seq.first(); j < seq.n; j = seq.next(j)) {
    const int64_t b = hard_mode ? int64_t(io.hard_list[j]) : seq.at(j);
    if (b >= B) continue;
    const int64_t gb = io.b0 + b, LD = io.ld;  // position in the caller's [field][B] arrays
#ifdef DRC_PHASE_TIMING
    const unsigned long long inst_t0 = __builtin_amdgcn_s_memtime();
    unsigned long long ph_snap[8];
    for (int k_ = 0; k_ < 8; ++k_) ph_snap[k_] = ph_acc[k_];
    unsigned long long epa_calls = 0, epa_steps = 0, epa_maxsteps = 0, epa_t[3] = {0, 0, 0};
#endif
    // re-derive the model pointer each instance: keeps LICM from hoisting
    // model-constant loads out of the instance loop into spilled registers
    const DevModel* M = M0;
    asm volatile("" : "+s"(M));
    // ---------------- state in ----------------
    double* qv = S + kp.kq;
    double* qd = S + kp.kqd;
    if (l < nv) {
      qv[l] = io.q[l * LD + gb];
      qd[l] = io.qdot[l * LD + gb];
    }
    // task targets, one value per lane (lanes 0-11 x_target, 12-17 xdot_target,
    // 18-29 x_init, 30-35 xdot_init): issued here so their latency overlaps the
    // FK; the task-velocity stage reads them by v_readlane
    double tgt = 0.0;
    if (l < 12) {
      if (kp.mode != DRC_MODE_QPIK) tgt = io.xt[l * LD + gb];
    } else if (l < 18) {
      tgt = io.xdt[(l - 12) * LD + gb];
    } else if (l < 36 && kp.mode == DRC_MODE_QPIK_CUBIC) {
      tgt = l < 30 ? io.xi[(l - 18) * LD + gb] : io.xdi[(l - 30) * LD + gb];
    }
    wsync();
    // ---------------- FK: local joint transforms, then the chain ------------
    double* T = S + kp.kT;  // (nv+1) x 12
    double* Zw = S + kp.kZ;  // (nv+1) x 3
    if (l < 12) T[l] = (l == 0 || l == 4 || l == 8) ? 1.0 : 0.0;
    double* loc = S + kp.kTg;  // scratch: local transforms nv x 12 (before geometry poses)
    if (l >= 1 && l <= nv) {
      const int j = l;
      double Mj[12];
      const double* ax = M->axis[j];
      const double qq = qv[j - 1];
      if (M->jtype[j] == kRevolute) {
        double c = cos(qq), s = sin(qq), C = 1 - c, x = ax[0], y = ax[1], z = ax[2];
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
      for (int i = 0; i < 12; ++i) loc[(j - 1) * 12 + i] = Lj[i];
    }
    wsync();
    for (int j = 1; j <= nv; ++j) {  // oMi[j] = oMi[parent] * local[j]; 12 lanes
      const double* a = T + M->parent[j] * 12;
      const double* bb = loc + (j - 1) * 12;
      double v = 0;
      if (l < 9) {
        int r = l / 3, c = l % 3;
        v = a[3 * r] * bb[c] + a[3 * r + 1] * bb[3 + c] + a[3 * r + 2] * bb[6 + c];
      } else if (l < 12) {
        int r = l - 9;
        v = a[3 * r] * bb[9] + a[3 * r + 1] * bb[10] + a[3 * r + 2] * bb[11] + a[9 + r];
      }
      wsync();
      if (l < 12) T[j * 12 + l] = v;
      wsync();
    }
    double* Te = S + kp.kTe;
    if (l >= 1 && l <= nv) st3(Zw + 3 * l, rot(T + 12 * l, ld3(M->axis[l])));
    if (l == 0) tmul(T + 12 * kp.frame_joint, kp.frame_place, Te);
    wsync();
    // geometry poses
    double* Tg = S + kp.kTg;
    for (int g = l; g < M->ngeom; g += 64) {
      double out[12];
      tmul(T + 12 * M->gparent[g], M->gplace[g], out);
      for (int i = 0; i < 12; ++i) Tg[g * 12 + i] = out[i];
    }
    PH(0);
    // ---------------- frame Jacobian (LWA), 6 x nv row-major -------------
    double* J = S + kp.kJ;
    const V3 pe = v3(Te[9], Te[10], Te[11]);
    const uint32_t anc_e = M->anc[kp.frame_joint];
    if (l < nv) {
      const int j = l + 1;
      V3 lin = v3(0, 0, 0), ang = v3(0, 0, 0);
      if (anc_e & (1u << l)) {
        V3 z = ld3(Zw + 3 * j);
        if (M->jtype[j] == kRevolute) {
          lin = cross(z, pe - v3(T[12 * j + 9], T[12 * j + 10], T[12 * j + 11]));
          ang = z;
        } else {
          lin = z;
        }
      }
      J[0 * nv + l] = lin.x; J[1 * nv + l] = lin.y; J[2 * nv + l] = lin.z;
      J[3 * nv + l] = ang.x; J[4 * nv + l] = ang.y; J[5 * nv + l] = ang.z;
    }
    wsync();
    // ---------------- task velocity ---------------------------------------
    double* xdd = S + kp.kxdd;
    // getVelocity = J qdot (robot_data.cpp:419-422), row r on lane r
    double jq = 0.0;
    if (l < 6)
      for (int c = 0; c < nv; ++c) jq += J[l * nv + c] * qd[c];
    if (l == 0) {
      if (kp.mode == DRC_MODE_QPIK) {
        for (int i = 0; i < 6; ++i) xdd[i] = rd_lane(tgt, 12 + i);
      } else {
        double xt[12], xdt[6];
        for (int i = 0; i < 12; ++i) xt[i] = rd_lane(tgt, i);
        for (int i = 0; i < 6; ++i) xdt[i] = rd_lane(tgt, 12 + i);
        if (kp.mode == DRC_MODE_QPIK_CUBIC) {  // getTaskSpaceCubic (math_type_define.h:647)
          double xi[12], xdi[6], Rt[9], Ri[9];
          for (int i = 0; i < 12; ++i) xi[i] = rd_lane(tgt, 18 + i);
          for (int i = 0; i < 6; ++i) xdi[i] = rd_lane(tgt, 30 + i);
          for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) {
              Rt[3 * r + c] = xt[3 * c + r];
              Ri[3 * r + c] = xi[3 * c + r];
            }
          const double t = kp.t, t0 = kp.t0, tf = kp.t0 + kp.duration;
          double pd[3], vd[3];
          for (int i = 0; i < 3; ++i) {
            pd[i] = cubic(t, t0, tf, xi[9 + i], xt[9 + i], xdi[i], xdt[i]);
            vd[i] = cubic_dot(t, t0, tf, xi[9 + i], xt[9 + i], xdi[i], xdt[i]);
          }
          double RiT_Rt[9], Rd[9];
          for (int a = 0; a < 3; ++a)
            for (int c = 0; c < 3; ++c)
              RiT_Rt[3 * a + c] = Ri[a] * Rt[c] + Ri[3 + a] * Rt[3 + c] + Ri[6 + a] * Rt[6 + c];
          V3 r = so3_log(RiT_Rt);
          if (t >= tf) {
            for (int i = 0; i < 9; ++i) Rd[i] = Rt[i];
          } else if (t < t0) {
            for (int i = 0; i < 9; ++i) Rd[i] = Ri[i];
          } else {
            double E3[9];
            so3_exp(cubic(t, t0, tf, 0, 1, 0, 0) * r, E3);
            for (int a = 0; a < 3; ++a)
              for (int c = 0; c < 3; ++c)
                Rd[3 * a + c] = Ri[3 * a] * E3[c] + Ri[3 * a + 1] * E3[3 + c] + Ri[3 * a + 2] * E3[6 + c];
          }
          V3 rd = v3(cubic_dot(t, t0, tf, 0, r.x, 0, 0), cubic_dot(t, t0, tf, 0, r.y, 0, 0),
                     cubic_dot(t, t0, tf, 0, r.z, 0, 0));
          rd = v3(Ri[0] * rd.x + Ri[1] * rd.y + Ri[2] * rd.z, Ri[3] * rd.x + Ri[4] * rd.y + Ri[5] * rd.z,
                  Ri[6] * rd.x + Ri[7] * rd.y + Ri[8] * rd.z);
          double tau = (t - t0) / (tf - t0);
          if (tau < 0 || tau > 1) rd = v3(0, 0, 0);
          for (int r0 = 0; r0 < 3; ++r0)
            for (int c = 0; c < 3; ++c) xt[3 * c + r0] = Rd[3 * r0 + c];
          for (int i = 0; i < 3; ++i) {
            xt[9 + i] = pd[i];
            xdt[i] = vd[i];
          }
          xdt[3] = rd.x; xdt[4] = rd.y; xdt[5] = rd.z;
        }
        // getTaskSpaceError (math_type_define.h:633) with getPhi (:283)
        double e[6], xdot[6];
        for (int i = 0; i < 3; ++i) e[i] = xt[9 + i] - Te[9 + i];
        V3 phi = v3(0, 0, 0);
        for (int i = 0; i < 3; ++i)
          phi = phi + cross(v3(xt[3 * i], xt[3 * i + 1], xt[3 * i + 2]), v3(Te[i], Te[3 + i], Te[6 + i]));
        e[3] = -0.5 * phi.x; e[4] = -0.5 * phi.y; e[5] = -0.5 * phi.z;
        for (int r = 0; r < 6; ++r) xdot[r] = rd_lane(jq, r);
        for (int i = 0; i < 6; ++i)
          xdd[i] = kp.kp[i] * e[i] + kp.kv[i] * (xdt[i] - xdot[i]) + kp.ff * xdt[i];
      }
    }
    PH(1);
    if constexpr (PROBLEM == 2) {  // closed-form controllers: no CBF stages
      closed_form_stage(M, kp, S, io, gb, LD);
      continue;
    }
    // ---------------- manipulability (arm columns c0..c0+narm) -------------
    const int narm = kp.narm, c0 = kp.c0;
    double* A6 = S + kp.kA6;
    double* Ai = S + kp.kAi;
    if (l < 36) {
      int a = l / 6, bb = l % 6;
      double s = 0;
      for (int c = 0; c < narm; ++c) s += J[a * nv + c0 + c] * J[bb * nv + c0 + c];
      A6[l] = s;
    }
    wsync();
    {
      // JJ^T (SPD) inverted by six lane-parallel Jordan exchanges (36 lanes),
      // det = product of the pivots.  Ill-conditioned JJ^T (Frobenius
      // condition estimate >= 1e5) takes the serial COD path (rank by pivoted
      // QR, Moore-Penrose on the kept modes), matching DyrosMath::PinvCOD's
      // threshold semantics (math_type_define.h:563).
      // lane i < 6 holds row i in registers; the pivot row moves by
      // v_readlane (same element formulas as the LDS form it replaced)
      double piv_min = 1e300, det = 1;
      const int lr = l < 6 ? l : 0;
      double r6[6];
#pragma unroll
      for (int j = 0; j < 6; ++j) r6[j] = A6[lr * 6 + j];
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const double akk = bcast(r6[k], k), aik = r6[k], ia = 1.0 / akk;  // one FP64 divide per pivot
        double pk6[6];
#pragma unroll
        for (int j = 0; j < 6; ++j) pk6[j] = bcast(r6[j], k);
#pragma unroll
        for (int j = 0; j < 6; ++j) {
          double v;
          if (l == k && j == k) v = ia;
          else if (l == k) v = pk6[j] * ia;
          else if (j == k) v = -aik * ia;
          else v = r6[j] - aik * (pk6[j] * ia);
          r6[j] = v;
        }
        piv_min = fmin(piv_min, akk);
        det *= akk;
      }
      if (l < 6)
#pragma unroll
        for (int j = 0; j < 6; ++j) Ai[l * 6 + j] = r6[j];
      wsync();
      // kappa_2 <= |A|_F |A^-1|_F; below 1e5 the pivoted QR of PinvCOD keeps
      // every mode (|R_55|/|R_00| >= 1/kappa_2 > COD_THRESHOLD 1e-6)
      const double fa = wave_sum(l < 36 ? A6[l] * A6[l] : 0.0), fi = wave_sum(l < 36 ? Ai[l] * Ai[l] : 0.0);
      if (!(piv_min > 0) || !(fa * fi < 1e10)) {  // uniform
        if (l == 0) {
          double* ws = S + kp.kScr;
          S[kp.oSc + SC_MAN] = sqrt(det_lu6(A6, ws));
          pinv_cod6(A6, Ai, ws);
        }
      } else if (l == 0) {
        S[kp.oSc + SC_MAN] = sqrt(det);
      }
      wsync();
    }
    double* W = S + kp.kW;  // narm x 6 = Jr^T Ai
    for (int e = l; e < narm * 6; e += 64) {
      int c = e / 6, a = e % 6;
      double s = 0;
      for (int i = 0; i < 6; ++i) s += J[i * nv + c0 + c] * Ai[i * 6 + a];
      W[e] = s;
    }
    wsync();
    double* part = S + kp.kPart;
    for (int e = l; e < narm * narm; e += 64) {
      const int kk = e / narm, c = e % narm;
      const int jk = c0 + kk + 1, ji = c0 + c + 1;  // joint ids of q_k and column i
      double acc = 0;
      if ((anc_e & (1u << (jk - 1))) && (anc_e & (1u << (ji - 1)))) {
        V3 zk = ld3(Zw + 3 * jk), zi = ld3(Zw + 3 * ji);
        V3 pk_ = v3(T[12 * jk + 9], T[12 * jk + 10], T[12 * jk + 11]);
        V3 pi_ = v3(T[12 * ji + 9], T[12 * ji + 10], T[12 * ji + 11]);
        const bool krev = M->jtype[jk] == kRevolute;
        V3 dpe = krev ? cross(zk, pe - pk_) : zk;
        const bool moves_i = jk != ji && (M->anc[ji] & (1u << (jk - 1)));
        V3 dzi = (moves_i && krev) ? cross(zk, zi) : v3(0, 0, 0);
        V3 dpi = moves_i ? (krev ? cross(zk, pi_ - pk_) : zk) : v3(0, 0, 0);
        V3 lin, ang;
        if (M->jtype[ji] == kRevolute) {
          lin = cross(dzi, pe - pi_) + cross(zi, dpe - dpi);
          ang = dzi;
        } else {
          lin = dzi;
          ang = v3(0, 0, 0);
        }
        const double* w = W + c * 6;
        acc = lin.x * w[0] + lin.y * w[1] + lin.z * w[2] + ang.x * w[3] + ang.y * w[4] + ang.z * w[5];
      }
      part[e] = acc;
    }
    wsync();
    double* mg = S + kp.kmg;
    if (l < narm) {
      double s = 0;
      for (int c = 0; c < narm; ++c) s += part[l * narm + c];
      mg[l] = S[kp.oSc + SC_MAN] * s;
    }
    PH(2);
    // ---------------- self-collision distance (broad + narrow phase) -------
    // Each lane owns pairs p = l, l+64, ... and keeps its running minimum with
    // witness points in registers (ties -> lowest pair index, the oracle's
    // first-strict-min rule), so the winner's witnesses never get recomputed.
    double* pd = S + kp.kPd;
    double* pf = S + kp.kPf;
    double bestd = 1.7976931348623157e308;
    int besti = 0x7fffffff;
    V3 bpA = v3(0, 0, 0), bpB = v3(0, 0, 0);
    double ub = 1e300;
    // slots in type-class order (model.cpp pair_order): each round of 64 lanes
    // runs one or two pair types instead of all of them
    for (int sl = l; sl < M->npairs; sl += 64) {
      const int p = M->pair_order[sl], ga = M->slot_a[sl], gb = M->slot_b[sl];
      Shape A{M->gtype[ga], Tg + 12 * ga, M->gparam[ga][0], M->gparam[ga][1], M->gparam[ga][2]};
      Shape Bs{M->gtype[gb], Tg + 12 * gb, M->gparam[gb][0], M->gparam[gb][1], M->gparam[gb][2]};
      V3 pA, pB;
      double d;
      const bool closed = (A.type == kSphere || Bs.type == kSphere)
                              ? (d = sphere_pair(A, Bs, &pA, &pB), true)
                              : (A.type == kCylinder && Bs.type == kCylinder && cyl_cyl_side(A, Bs, &d, &pA, &pB));
      if (closed) {
        pf[p] = 1.0;
        ub = fmin(ub, d);
        if (d < bestd || (d == bestd && p < besti)) {  // ties -> lowest pair index
          bestd = d;
          besti = p;
          bpA = pA;
          bpB = pB;
        }
      } else {  // swept-core / separating-axis lower bound
        pd[p] = pair_lower_bound(A, Bs, M->gbound[ga], M->gbound[gb]);
        pf[p] = 0.0;
      }
    }
    ub = -wave_max(-ub);
    PH(3);
    // exact GJK only where the swept-core bound can still win.  The candidates
    // are compacted into a list first, so a wave runs them in ceil(n / 64)
    // rounds instead of one round per 64 pair slots.
    {
      int* cand = reinterpret_cast<int*>(S + kp.kCand);
      int ncand = 0;
      for (int p0 = 0; p0 < M->npairs; p0 += 64) {
        const int p = p0 + l;
        const bool c = p < M->npairs && pf[p] == 0.0 && pd[p] - 1e-9 <= ub;
        const unsigned long long m = __ballot(c);
        if (c) cand[ncand + __popcll(m & ((1ull << l) - 1))] = p;
        ncand += __popcll(m);
      }
      wsync();
      for (int c = l; c < ncand; c += 64) {
        const int p = cand[c];
        const int ga = M->pair_a[p], gb = M->pair_b[p];
        Shape A{M->gtype[ga], Tg + 12 * ga, M->gparam[ga][0], M->gparam[ga][1], M->gparam[ga][2]};
        Shape Bs{M->gtype[gb], Tg + 12 * gb, M->gparam[gb][0], M->gparam[gb][1], M->gparam[gb][2]};
        // early exit once GJK's lower bound shows the pair cannot reach ub
        const GjkDist g = gjk(A, Bs, ub + 1e-9);
        if (g.pruned) {
          pf[p] = 1.0;
        } else if (g.intersect) {
          pf[p] = 2.0;  // penetrating: EPA below
        } else {
          pf[p] = 1.0;
          if (g.dist < bestd || (g.dist == bestd && p < besti)) {
            bestd = g.dist;
            besti = p;
            bpA = g.pA;
            bpB = g.pB;
          }
        }
      }
    }
    wsync();
    PH(4);
    // EPA, best-first with bounds: the lower bound pd[p] <= d(p) also
    // caps the penetration depth, so pairs are expanded in increasing pd and
    // the search stops once no remaining pair can undercut the running
    // minimum (same argmin and tie rule as computing every pair).  The owning
    // lane expands the polytope, the whole wave scans for the closest face.
    {
      double gbd = bestd;
      int gbi = besti;
      wave_argmin(gbd, gbi);
      for (;;) {
        double cpd = 1.7976931348623157e308;
        int cp = 0x7fffffff;
        for (int p = l; p < M->npairs; p += 64)
          if (pf[p] == 2.0 && pd[p] < cpd) {
            cpd = pd[p];
            cp = p;
          }
        wave_argmin(cpd, cp);
        if (cp == 0x7fffffff || cpd > gbd || (cpd == gbd && cp > gbi)) break;
        const int p = cp, ln = p & 63, ga = M->pair_a[p], gb = M->pair_b[p];
        const Shape A{M->gtype[ga], Tg + 12 * ga, M->gparam[ga][0], M->gparam[ga][1], M->gparam[ga][2]};
        const Shape Bs{M->gtype[gb], Tg + 12 * gb, M->gparam[gb][0], M->gparam[gb][1], M->gparam[gb][2]};
        if (l == ln) epa_init(A, Bs, ews);
        wsync();
        double dres = 0;
#ifdef DRC_PHASE_TIMING
        epa_calls++;
#endif
        for (int it = 0; it <= 255; ++it) {
#ifdef DRC_PHASE_TIMING
          epa_steps++;
          if ((unsigned long long)it > epa_maxsteps) epa_maxsteps = it;
#endif
#ifdef DRC_PHASE_TIMING
          unsigned long long te0 = __builtin_amdgcn_s_memtime();
#endif
          bool stop = ews->stop || it == 255;
          double fdm = 1e300;
          int fb = 0x7fffffff;
          for (int f = l; f < ews->nf; f += 64)
            if (ews->alive[f] && ews->fd[f] < fdm) {
              fdm = ews->fd[f];
              fb = f;
            }
          wave_argmin(fdm, fb);
          if (fb == 0x7fffffff) {  // no alive face (failed seed): oracle takes face 0
            fb = 0;
            stop = true;
          }
#ifdef DRC_PHASE_TIMING
          unsigned long long te1 = __builtin_amdgcn_s_memtime();
          epa_t[0] += te1 - te0;
#endif
          SV w;
          if (!stop) {  // support, gap and duplicate tests on the whole wave
            w = sup_md(A, Bs, ld3(ews->fn[fb]));
            stop = epa_gap_stop(ews, fb, w);
            if (!stop) {
              bool dup = false;
              for (int i = l; i < ews->nv; i += 64) dup |= epa_is_dup(ews, i, w);
              stop = __any(dup);
            }
          }
          if (stop) {
            if (l == ln) {
              const double d = epa_finish(ews, fb);
              dres = d;
              if (d < bestd || (d == bestd && p < besti)) {
                bestd = d;
                besti = p;
                bpA = ld3(ews->out);
                bpB = ld3(ews->out + 3);
              }
            }
            break;
          }
#ifdef DRC_PHASE_TIMING
          unsigned long long te2 = __builtin_amdgcn_s_memtime();
          epa_t[1] += te2 - te1;
#endif
          FaceMask vis;  // visibility of every face for w, one bit per face
          vis.lo = __ballot(l < ews->nf && epa_sees(ews, l, w.w));
          vis.hi = __ballot(l + 64 < ews->nf && epa_sees(ews, l + 64, w.w));
          // horizon walk on one lane (slots, adjacency), the new faces'
          // normals and validity tests one per lane, then commit / roll back
          if (l == ln) epa_grow_walk(ews, w, fb, vis);
          wsync();
          {
            const double fdmin = ews->fd[fb];
            bool gfail = false;
            for (int i = l; i < ews->nnew; i += 64) gfail |= !epa_face_geometry(ews, ews->newl[i], fdmin);
            gfail = __any(gfail);
            wsync();
            if (l == ln) epa_grow_finish(ews, fb, gfail);
          }
          wsync();
#ifdef DRC_PHASE_TIMING
          epa_t[2] += __builtin_amdgcn_s_memtime() - te2;
#endif
        }
        const double dall = __shfl(dres, ln, 64);
        if (dall < gbd || (dall == gbd && p < gbi)) {
          gbd = dall;
          gbi = p;
        }
        if (l == ln) pf[p] = 1.0;
        wsync();
      }
    }
    PH(5);
    const double myd = bestd;
    const int myi = besti;
    wave_argmin(bestd, besti);
    double* dgv = S + kp.kdg;
    double* red = S + kp.oRed;
    if (myi == besti && myi < M->npairs) {  // the winning lane publishes its witnesses
      st3(red, bpA);
      st3(red + 3, bpB);
    }
    if (l == 0) {
      S[kp.oSc + SC_DIST] = bestd;
      S[kp.oSc + SC_PAIR] = besti;
    }
    (void)myd;
    wsync();
    PH(6);
    if (l < nv) {  // grad d = n^T (J_B(pB) - J_A(pA)), sign flipped when penetrating
      double g = 0;
      if (besti < M->npairs) {
        const int jA = M->gparent[M->pair_a[besti]], jB = M->gparent[M->pair_b[besti]];
        V3 pA = ld3(red), pB = ld3(red + 3), n = pB - pA;
        n = (1.0 / sqrt(dot(n, n))) * n;
        const int j = l + 1;
        V3 z = ld3(Zw + 3 * j), pj = v3(T[12 * j + 9], T[12 * j + 10], T[12 * j + 11]);
        const bool rev = M->jtype[j] == kRevolute;
        V3 cA = v3(0, 0, 0), cB = v3(0, 0, 0);
        if (jA > 0 && (M->anc[jA] & (1u << l))) cA = rev ? cross(z, pA - pj) : z;
        if (jB > 0 && (M->anc[jB] & (1u << l))) cB = rev ? cross(z, pB - pj) : z;
        g = dot(n, cB - cA);
        if (bestd < 0) g = -g;
      }
      dgv[l] = g;
    }
    wsync();
    if constexpr (PROBLEM == 1) qpid_task_extras(M, kp, S, bestd, besti, io.st_gdv != nullptr);
    PH(7);
#ifdef DRC_PHASE_TIMING
    if (l == 0) {  // straggler census: max instance cycles, count above 2M
      const unsigned long long dt = __builtin_amdgcn_s_memtime() - inst_t0;
      atomicMax(&g_phase_cycles[30], dt);
      if (dt > 2000000ull) atomicAdd(&g_phase_cycles[31], 1ull);
      if (dt > 2000000ull) atomicAdd(&g_phase_cycles[29], dt);
      if (dt > 2000000ull) {
        for (int k_ = 0; k_ < 8; ++k_) atomicAdd(&g_phase_cycles[8 + k_], ph_acc[k_] - ph_snap[k_]);
        atomicAdd(&g_phase_cycles[22], epa_calls);
        atomicAdd(&g_phase_cycles[23], epa_steps);
        atomicMax(&g_phase_cycles[28], epa_maxsteps);
        atomicAdd(&g_phase_cycles[18], epa_t[0] + epa_t[1]);  // (qp kernel leaves 18, 20 free)
        atomicAdd(&g_phase_cycles[20], epa_t[2]);
      }
    }
#endif
    // ---------------- task data out -----------------------------------------
    if (io.rec) {  // product path: one coalesced record per instance
      double* rec = io.rec + b * io.rec_stride;
      for (int e = l; e < kp.rLen; e += 64) {
        double v;
        if (e < kp.rMan) v = J[e];
        else if (e == kp.rMan) v = S[kp.oSc + SC_MAN];
        else if (e < kp.rDist) v = mg[e - kp.rMan - 1];
        else if (e == kp.rDist) v = bestd;
        else if (e < kp.rXdd) v = dgv[e - kp.rDist - 1];
        else if (e < kp.rQ) v = xdd[e - kp.rXdd];
        else if (PROBLEM == 0 || e < kp.rQd) v = qv[e - kp.rQ];
        else if (e < kp.rBias) v = qd[e - kp.rQd];
        else v = S[kp.kBias + e - kp.rBias];  // QPID: Jdot v (6), man_gd, dist_gd
        rec[e] = v;
      }
    } else {  // stage outputs, [field][B]
      if (io.st_pose && l < 12) {
        // R row-major -> column-major storage, then p
        double v = l < 9 ? Te[(l % 3) * 3 + l / 3] : Te[l];
        io.st_pose[l * LD + gb] = v;
      }
      if (io.st_jac)
        for (int e = l; e < 6 * nv; e += 64) io.st_jac[(int64_t)e * LD + gb] = J[e];
      if (io.st_man) {
        if (l == 0) io.st_man[gb] = S[kp.oSc + SC_MAN];
        if (l < narm) io.st_man[(int64_t)(1 + l) * LD + gb] = mg[l];
      }
      if (io.st_dist) {
        if (l == 0) io.st_dist[gb] = bestd;
        if (l < nv) io.st_dist[(int64_t)(1 + l) * LD + gb] = dgv[l];
      }
      if (io.st_pair && l == 0) io.st_pair[gb] = besti < M->npairs ? besti : -1;
      if (io.st_xdd && l < 6) io.st_xdd[l * LD + gb] = xdd[l];
      if constexpr (PROBLEM == 1) {
        if (io.st_jdot)
          for (int e = l; e < 6 * nv; e += 64) io.st_jdot[(int64_t)e * LD + gb] = S[kp.kJd + e];
        if (io.st_qpid && l < 8) io.st_qpid[l * LD + gb] = S[kp.kBias + l];
        if (io.st_gdv)
          for (int e = l; e < narm + nv; e += 64) io.st_gdv[(int64_t)e * LD + gb] = S[kp.kGdv + e];
      }
    }
    wsync();
  }
  PH_FLUSH(0);
}

#include "lane_task.hpp"

// ---- QP kernel phases ------------------------------------------------------
template <class QD>
__device__ __forceinline__ void qp_assemble(const DevModel* M, const KParams& kp, double* S, const IO& io, int64_t b) {
  using GL = Grp<QD::gs>;
  const int l = GL::lane();
  const int nv = kp.nv, narm = kp.narm;
  double* qv = S + kp.kq;
  double* J = S + kp.kJ;
  double* xdd = S + kp.kxdd;
  double* mg = S + kp.kmg;
  double* dgv = S + kp.kdg;
#ifdef DRC_PHASE_TIMING
  const unsigned long long as_t0 = __builtin_amdgcn_s_memtime();
#endif
  {  // task record written by task_kernel (one coalesced read)
    const double* rec = io.rec + b * io.rec_stride;
    for (int e = l; e < kp.rLen; e += GL::size) {
      const double v = rec[e];
      if (e < kp.rMan) J[e] = v;
      else if (e == kp.rMan) S[kp.oSc + SC_MAN] = v;
      else if (e < kp.rDist) mg[e - kp.rMan - 1] = v;
      else if (e == kp.rDist) S[kp.oSc + SC_DIST] = v;
      else if (e < kp.rXdd) dgv[e - kp.rDist - 1] = v;
      else if (e < kp.rQ) xdd[e - kp.rXdd] = v;
      else qv[e - kp.rQ] = v;
    }
  }
  wsync();
#ifdef DRC_PHASE_TIMING
  if (GL::lane() == 0) atomicAdd(&g_phase_cycles[44], __builtin_amdgcn_s_memtime() - as_t0);
#endif
  const double bestd = S[kp.oSc + SC_DIST];
  // ---------------- QP assembly (QP_IK.cpp:69-131 / MoMa :59-128) --------
  const int nx = DNX, ng = DNG, np = DNP, m = DM;
  double *P = S + kp.oP, *G = S + kp.oG, *qq = S + kp.oQ, *ab = S + kp.oAB, *lo = S + kp.oL, *up = S + kp.oU;
  const double alpha = kp.alpha_cbf, man = S[kp.oSc + SC_MAN];
  double* Jt = S + kp.kJt;  // task Jacobian over the QP's task variables: 6 x np
  if (M->kind == 0) {
    for (int e = l; e < 6 * np; e += GL::size) Jt[e] = J[(e / np) * nv + e % np];
  } else {
    // J~ = J S  (mobile_manipulator/robot_data.cpp:407-410); S virtual block = Rz(yaw) J_mobile
    const double yaw = qv[M->virtual_start + 2], cy = cos(yaw), sy = sin(yaw);
    const double(*Jm)[kMaxWheels] = mobile_jac<QD::gs>(M, kp, S, qv);
    for (int e = l; e < 6 * np; e += GL::size) {
      const int r = e / np, a = e % np;
      double v = 0;
      const int am = a - M->act_mani_start, aw = a - M->act_mobi_start;
      if (am >= 0 && am < M->n_arm) {
        v = J[r * nv + M->mani_start + am];
      } else if (aw >= 0 && aw < M->n_wheel) {
        const double s0 = cy * Jm[0][aw] - sy * Jm[1][aw];
        const double s1 = sy * Jm[0][aw] + cy * Jm[1][aw];
        const double s2 = Jm[2][aw];
        const int vs = M->virtual_start;
        v = J[r * nv + M->mobi_start + aw] + J[r * nv + vs] * s0 + J[r * nv + vs + 1] * s1 + J[r * nv + vs + 2] * s2;
      }
      Jt[e] = v;
    }
  }
  wsync();
  for (int e = l; e < np * np; e += GL::size) {
    const int i = e / np, j = e % np;
    double s = 0;
    for (int r = 0; r < 6; ++r) s += Jt[r * np + i] * Jt[r * np + j];
    P[e] = 2.0 * s + (i == j ? kp.w_reg : 0.0);
  }
  for (int e = l; e < ng * nx; e += GL::size) G[e] = 0.0;
  if (l < nx) {
    double qi;
    if (l < np) {
      double s = 0;
      for (int r = 0; r < 6; ++r) s += Jt[r * np + l] * xdd[r];
      qi = -2.0 * s;
    } else {
      qi = kp.slack_w;
    }
    qq[l] = qi;
    ab[l] = 1.0;
    if (M->kind == 0) {
      lo[l] = l < nv ? -M->vel[l] : 0.0;
      up[l] = l < nv ? M->vel[l] : kInf;
    } else {  // setBoundConstraint is a no-op for MoMa (QP_IK.cpp:75-83)
      lo[l] = -kInf;
      up[l] = kInf;
    }
  }
  wsync();
  if (l < ng) {
    const int n = narm, row = nx + l;
    double lval = 0;
    const int vo = M->kind == 0 ? 0 : M->act_mani_start;  // task-variable offset of the arm
    const int qo = M->kind == 0 ? 0 : M->mani_start;      // joint offset of the arm
    if (l < n) {
      G[l * nx + vo + l] = 1.0;
      if (M->kind == 0) G[l * nx + n + l] = 1.0;
      lval = -alpha * (qv[qo + l] - M->lower[qo + l]);
    } else if (l < 2 * n) {
      const int i = l - n;
      G[l * nx + vo + i] = -1.0;
      if (M->kind == 0) G[l * nx + 2 * n + i] = 1.0;
      lval = -alpha * (M->upper[qo + i] - qv[qo + i]);
    } else if (l == 2 * n) {
      for (int c = 0; c < n; ++c) G[l * nx + vo + c] = mg[c];
      if (M->kind == 0) G[l * nx + 3 * n] = 1.0;
      lval = -alpha * (man - kp.man_min);
    } else {
      for (int c = 0; c < n; ++c) G[l * nx + vo + c] = dgv[qo + c];
      if (M->kind == 0) G[l * nx + 3 * n + 1] = 1.0;
      lval = -alpha * (bestd - kp.dist_min);
    }
    lo[row] = lval;
    up[row] = kInf;
  }
  wsync();
}

// Whole-body QP infeasibility certificate (exact mode, D15).  The MoMa QP has
// no slacks and no variable bounds (mobile_manipulator/QP_IK.cpp:75-128); its
// rows are the arm's CBF box blo <= qdot_arm <= bhi and the two gradient rows
// g_m . qdot_arm >= r_m, g_d . qdot_arm >= r_d.  By Farkas, it is infeasible
// iff some mu in [0, 1] has phi(mu) = max over the box of
// (mu g_m + (1 - mu) g_d) . v - (mu r_m + (1 - mu) r_d) < 0; phi is convex
// and piecewise linear, so its minimum sits at mu = 0, 1 or a root of a
// component of mu g_m + (1 - mu) g_d.  Lane c evaluates candidate c on the
// unscaled rows (before Ruiz); certified when some phi < -1e-6 (1 + scale),
// a margin no point the certified polish accepts (residual ~1e-9) can
// cross.  Same candidates, order of sums and margin as the oracle's
// moma_lp_infeasible.
template <class QD>
__device__ __forceinline__ bool moma_lp_infeasible(const DevModel* M, const KParams& kp, const double* S) {
  using GL = Grp<QD::gs>;
  const int l = GL::lane();
  const int nx = DNX, n = kp.narm, vo = M->act_mani_start;
  const double *G = S + kp.oG, *lo = S + kp.oL + nx;
  const double *gm = G + (2 * n) * nx + vo, *gd = G + (2 * n + 1) * nx + vo;
  const double rm = lo[2 * n], rd = lo[2 * n + 1];
  double mu = -1.0;
  if (l == 0) mu = 1.0;
  else if (l == 1) mu = 0.0;
  else if (l < n + 2) {
    const int i = l - 2;
    const double den = gm[i] - gd[i];
    if (den != 0.0) {
      const double t = -gd[i] / den;
      if (t > 0.0 && t < 1.0) mu = t;
    }
  }
  double scale = fabs(rm) + fabs(rd), phi = -(mu * rm + (1.0 - mu) * rd);
  for (int i = 0; i < n; ++i) {
    const double blo = lo[i], bhi = -lo[n + i], g = mu * gm[i] + (1.0 - mu) * gd[i];
    phi += fmax(g * blo, g * bhi);
    scale += (fabs(gm[i]) + fabs(gd[i])) * fmax(fabs(blo), fabs(bhi));
  }
  return GL::any(mu >= 0.0 && phi < -1e-6 * (1.0 + scale));
}

// finiteness check + Ruiz equilibration (OSQP scaling.c); returns
// DRC_STATUS_NONFINITE or DRC_STATUS_MAX_ITER (= not yet solved)
template <class QD>
__device__ __forceinline__ int qp_scale(const KParams& kp, double* S) {
  using GL = Grp<QD::gs>;
  const int l = GL::lane();
  const int nx = DNX, ng = DNG, np = DNP, m = DM;
  double *P = S + kp.oP, *G = S + kp.oG, *qq = S + kp.oQ, *ab = S + kp.oAB, *lo = S + kp.oL, *up = S + kp.oU;
  int status = DRC_STATUS_MAX_ITER;
  {
    bool finite = true;
    for (int e = l; e < np * np; e += GL::size) finite &= isfinite(P[e]);
    for (int e = l; e < ng * nx; e += GL::size) finite &= isfinite(G[e]);
    if (l < nx) finite &= isfinite(qq[l]);
    for (int row = l; row < m; row += GL::size) finite &= !isnan(lo[row]) && !isnan(up[row]);
    if (!GL::all(finite)) status = DRC_STATUS_NONFINITE;
  }
  double *D = S + kp.oD, *E = S + kp.oE, *x = S + kp.oX, *z = S + kp.oZ, *y = S + kp.oY, *dy = S + kp.oDY;
  double* sc = S + kp.oSc;
  if (status != DRC_STATUS_NONFINITE) {
    if (l < nx) D[l] = 1.0;
    for (int row = l; row < m; row += GL::size) E[row] = 1.0;
    if (l == 0) sc[SC_C] = 1.0;
    double* Dt = S + kp.oT1;
    double* Et = S + kp.oT2;
    wsync();
    for (int it = 0; it < kp.s.scaling; ++it) {
      if (l < nx) {
        double s = fabs(ab[l]);
        if (l < np)
          for (int i = 0; i < np; ++i) s = fmax(s, fabs(P[i * np + l]));
        for (int i = 0; i < ng; ++i) s = fmax(s, fabs(G[i * nx + l]));
        s = s < kMinScaling ? 1.0 : (s > kMaxScaling ? kMaxScaling : s);
        Dt[l] = 1.0 / sqrt(s);
        double eb = fabs(ab[l]);
        eb = eb < kMinScaling ? 1.0 : (eb > kMaxScaling ? kMaxScaling : eb);
        Et[l] = 1.0 / sqrt(eb);
      }
      if (l < ng) {
        double s = 0;
        for (int j = 0; j < nx; ++j) s = fmax(s, fabs(G[l * nx + j]));
        s = s < kMinScaling ? 1.0 : (s > kMaxScaling ? kMaxScaling : s);
        Et[nx + l] = 1.0 / sqrt(s);
      }
      wsync();
      if (l < np)
        for (int c = 0; c < np; ++c) P[l * np + c] *= Dt[l] * Dt[c];
      if (l < ng)
        for (int j = 0; j < nx; ++j) G[l * nx + j] *= Et[nx + l] * Dt[j];
      if (l < nx) {
        ab[l] *= Et[l] * Dt[l];
        qq[l] *= Dt[l];
        D[l] *= Dt[l];
        E[l] *= Et[l];
      }
      if (l < ng) E[nx + l] *= Et[nx + l];
      wsync();
      // cost scaling: mean column norm of P vs |q|_inf
      double cn = 0, qn = 0;
      if (l < nx) {
        if (l < np)
          for (int i = 0; i < np; ++i) cn = fmax(cn, fabs(P[i * np + l]));
        qn = fabs(qq[l]);
      }
      cn = GL::sum(cn) / nx;
      qn = GL::max(qn);
      qn = qn < kMinScaling ? 1.0 : (qn > kMaxScaling ? kMaxScaling : qn);
      double ct = fmax(cn, qn);
      ct = ct < kMinScaling ? 1.0 : (ct > kMaxScaling ? kMaxScaling : ct);
      ct = 1.0 / ct;
      if (l < np)
        for (int c = 0; c < np; ++c) P[l * np + c] *= ct;
      if (l < nx) qq[l] *= ct;
      if (l == 0) sc[SC_C] *= ct;
      // fixed point (as qp_scale_regs and the oracle)
      const bool ones = (l >= nx || (Dt[l] == 1.0 && Et[l] == 1.0)) && (l >= ng || Et[nx + l] == 1.0);
      wsync();
      if (ct == 1.0 && GL::all(ones)) break;
    }
    for (int row = l; row < m; row += GL::size) {
      lo[row] = fmax(lo[row], -kInf) * E[row];
      up[row] = fmin(up[row], kInf) * E[row];
    }
    wsync();
    }
  return status;
}

// Register form of qp_scale for compile-time shapes: lane l holds row l of P
// (= column l: P is symmetric bit for bit), column l and row l of G; the
// Ruiz factors move by v_readlane.  Same operations in the same order as
// qp_scale (bit-identical results); P, G, q, D, E written back at the end.
template <class QD>
__device__ __noinline__ int qp_scale_regs(const KParams& kp, double* S) {
  using GL = Grp<QD::gs>;
  constexpr int NX = QD::nx, NG = QD::ng, NP = QD::np, M = NX + NG;
  const int l = GL::lane();
  double *P = S + kp.oP, *G = S + kp.oG, *qq = S + kp.oQ, *ab = S + kp.oAB, *lo = S + kp.oL, *up = S + kp.oU;
  double *D = S + kp.oD, *E = S + kp.oE, *sc = S + kp.oSc;
  {
    bool finite = true;
    for (int e = l; e < NP * NP; e += GL::size) finite &= isfinite(P[e]);
    for (int e = l; e < NG * NX; e += GL::size) finite &= isfinite(G[e]);
    if (l < NX) finite &= isfinite(qq[l]);
    for (int row = l; row < M; row += GL::size) finite &= !isnan(lo[row]) && !isnan(up[row]);
    if (!GL::all(finite)) return DRC_STATUS_NONFINITE;
  }
  const bool hx = l < NX, hg = l < NG, hp = l < NP;
  const int lx = hx ? l : 0, lg = hg ? l : 0, lp = hp ? l : 0;
  double Prow[NP], Gcol[NG], Grow[NX];
#pragma unroll
  for (int c = 0; c < NP; ++c) Prow[c] = P[lp * NP + c];
#pragma unroll
  for (int i = 0; i < NG; ++i) Gcol[i] = G[i * NX + lx];
#pragma unroll
  for (int j = 0; j < NX; ++j) Grow[j] = G[lg * NX + j];
  double abl = ab[lx], ql = qq[lx], Dl = 1.0, El = 1.0, EGl = 1.0, cs = 1.0;
  auto clampf = [](double v) { return v < kMinScaling ? 1.0 : (v > kMaxScaling ? kMaxScaling : v); };
  for (int it = 0; it < kp.s.scaling; ++it) {
    double s = fabs(abl);
    if (hp)
#pragma unroll
      for (int i = 0; i < NP; ++i) s = fmax(s, fabs(Prow[i]));
#pragma unroll
    for (int i = 0; i < NG; ++i) s = fmax(s, fabs(Gcol[i]));
    const double Dt = 1.0 / sqrt(clampf(s));
    const double Et = 1.0 / sqrt(clampf(fabs(abl)));
    double sg = 0;
#pragma unroll
    for (int j = 0; j < NX; ++j) sg = fmax(sg, fabs(Grow[j]));
    const double EtG = 1.0 / sqrt(clampf(sg));
    double DtA[NX], EtGA[NG];
    static_for<NX>([&](auto C) { DtA[decltype(C)::value] = GL::template bcastc<decltype(C)::value>(Dt); });
    static_for<NG>([&](auto I) { EtGA[decltype(I)::value] = GL::template bcastc<decltype(I)::value>(EtG); });
    if (hp)
#pragma unroll
      for (int c = 0; c < NP; ++c) Prow[c] *= Dt * DtA[c];
    if (hx)
#pragma unroll
      for (int i = 0; i < NG; ++i) Gcol[i] *= EtGA[i] * Dt;
    if (hg)
#pragma unroll
      for (int j = 0; j < NX; ++j) Grow[j] *= EtG * DtA[j];
    if (hx) {
      abl *= Et * Dt;
      ql *= Dt;
      Dl *= Dt;
      El *= Et;
    }
    if (hg) EGl *= EtG;
    // cost scaling: mean column norm of P vs |q|_inf
    double cn = 0, qn = 0;
    if (hp)
#pragma unroll
      for (int i = 0; i < NP; ++i) cn = fmax(cn, fabs(Prow[i]));
    if (hx) qn = fabs(ql);
    cn = GL::sum(cn) / NX;
    qn = GL::max(qn);
    qn = clampf(qn);
    double ct = clampf(fmax(cn, qn));
    ct = 1.0 / ct;
    if (hp)
#pragma unroll
      for (int c = 0; c < NP; ++c) Prow[c] *= ct;
    if (hx) ql *= ct;
    cs *= ct;
    // fixed point: every factor of this pass was exactly 1, so the remaining
    // passes would repeat it bit for bit (oracle: same exit)
    if (ct == 1.0 && GL::all((!hx || (Dt == 1.0 && Et == 1.0)) && (!hg || EtG == 1.0))) break;
  }
  if (hp)
#pragma unroll
    for (int c = 0; c < NP; ++c) P[l * NP + c] = Prow[c];
  if (hg)
#pragma unroll
    for (int j = 0; j < NX; ++j) G[l * NX + j] = Grow[j];
  if (hx) {
    ab[l] = abl;
    qq[l] = ql;
    D[l] = Dl;
    E[l] = El;
  }
  if (hg) E[NX + l] = EGl;
  if (l == 0) sc[SC_C] = cs;
  wsync();
  for (int row = l; row < M; row += GL::size) {
    lo[row] = fmax(lo[row], -kInf) * E[row];
    up[row] = fmin(up[row], kInf) * E[row];
  }
  wsync();
  return DRC_STATUS_MAX_ITER;
}

// rho, K^-1 and the ADMM iterations (+ polish); returns the status
template <class QD>
__device__ __forceinline__ int qp_admm(const KParams& kp, const KParams& kpl, double* S, int* iters_out) {
  using GL = Grp<QD::gs>;
  const int l = GL::lane();
  const int nx = DNX, ng = DNG, m = DM;
  double *G = S + kp.oG, *qq = S + kp.oQ, *ab = S + kp.oAB, *lo = S + kp.oL, *up = S + kp.oU;
  double *x = S + kp.oX, *z = S + kp.oZ, *y = S + kp.oY, *dy = S + kp.oDY;
  double* sc = S + kp.oSc;
  int status = DRC_STATUS_MAX_ITER;
  (void)G;
  PHG_DECL
  if (l == 0) {
    sc[SC_PFAIL] = 0.0;
    sc[SC_HIV] = 0.0;  // the polish's cached (P + delta I)^-1 is formed on first use
  }
  set_rho<QD>(kp, S, kp.s.rho);
  factor_any<QD>(kpl, S);
  PHG(24);
  if (l < nx) x[l] = 0.0;
  for (int row = l; row < m; row += GL::size) z[row] = y[row] = 0.0;
  wsync();
  // ---------------- OSQP: ADMM ----------------------------------------
  const double* K = S + kp.oU0;
  const double* rv = S + kp.oRho;
  double* w = S + kp.oT1;
  double* xt = S + kp.oXT;
  const double sig = kp.s.sigma, al = kp.s.alpha;
  int it;
  if constexpr (QD::schur) {
    // Lane roles: l < NP core variable l (and its bound row); NP + r < NP + NG:
    // G row r together with its auxiliary variable a(r) and that variable's
    // bound row.  R[] holds, on core lanes, row l of S^-1 then column l of
    // G_c; on row lanes, row r of G_c S^-1.  Per iteration:
    //   rows: t_a = r_a / d_a, u_r = w_r - rho_r g_r t_a       (w = rho z - y)
    //   core: r'_c = sigma x_c - q_c + ab_c w_b + sum_r G_rc u_r   (NG broadcasts)
    //   core: x~_c = S^-1 r';  rows: v_r = G_r,c x~_c = (G_c S^-1)_r r'   (NP broadcasts)
    //   rows: x~_a = t_a - coef_r v_r,  (G x~)_r = v_r + g_r x~_a
    constexpr int NX = QD::nx, NG = QD::ng, NP = QD::np;
    static_assert(NP + NG <= QD::gs, "one lane per core variable and per G row");
    const double* Si = S + kp.oU0;
    const double* GS = Si + NP * NP;
    const double* dv = GS + NG * NP;
    const double* cf = dv + NG;
    const int* aux = reinterpret_cast<const int*>(cf + 2 * NG);
    const double* G = S + kp.oG;
    double R[NP + NG];
    const bool hc = l < NP, hr = l >= NP && l < NP + NG;
    const int rr_ = hr ? l - NP : 0, lc_ = hc ? l : 0;
    auto load_regs = [&]() {
      if (hc) {
#pragma unroll
        for (int c = 0; c < NP; ++c) R[c] = Si[lc_ * NP + c];
#pragma unroll
        for (int i = 0; i < NG; ++i) R[NP + i] = G[i * NX + lc_];
      } else {
#pragma unroll
        for (int c = 0; c < NP; ++c) R[c] = GS[rr_ * NP + c];
#pragma unroll
        for (int i = 0; i < NG; ++i) R[NP + i] = 0.0;
      }
    };
    load_regs();
    PHG(25);
#ifdef DRC_PHASE_TIMING
    unsigned long long tchk = 0;
#endif
    const int a_ = hr ? aux[rr_] : -1;           // auxiliary variable of row r (or -1)
    const bool ha = a_ >= 0;
    const int ia = ha ? a_ : 0, ig = NX + rr_;   // its bound row, the G row
    // core lane: its bound row; row lane: the G row and the aux bound row
    const double ab_c = ab[lc_], q_c = qq[lc_], lo_c = lo[lc_], up_c = up[lc_];
    const double g_r = ha ? G[rr_ * NX + ia] : 0.0, ab_a = ab[ia], q_a = qq[ia];
    const double lo_a = lo[ia], up_a = up[ia], lo_g = lo[ig], up_g = up[ig];
    double d_r = dv[rr_], c_r = cf[rr_];
    double rc = rv[lc_], ra = rv[ia], rg = rv[ig];
    double irc = 1.0 / rc, ira = 1.0 / ra, irg = 1.0 / rg;  // y / rho as a product in the loop
    double xc = 0, zc = 0, yc = 0, dyc = 0, xa = 0, za = 0, ya = 0, dya = 0, zg = 0, yg = 0, dyg = 0;
    for (it = 1; it <= kp.s.max_iter; ++it) {
      double u = 0, ta = 0, loc = 0;
      if (hr) {
        const double wg = rg * zg - yg;
        if (ha) {
          const double r_a = sig * xa - q_a + ab_a * (ra * za - ya) + g_r * wg;
          ta = r_a * d_r;  // d_r holds 1 / d_a
          u = wg - rg * g_r * ta;
        } else {
          u = wg;
        }
      }
      if (hc) loc = sig * xc - q_c + ab_c * (rc * zc - yc);
      double r0 = 0, r1 = 0;
      static_for<NG>([&](auto I) {
        constexpr int i = decltype(I)::value;
        const double ui = GL::template bcastc<NP + i>(u);
        if constexpr (i & 1) r1 += R[NP + i] * ui;
        else r0 += R[NP + i] * ui;
      });
      const double rp = loc + (r0 + r1);
      double s0 = 0, s1 = 0;
      static_for<NP>([&](auto C) {
        constexpr int c = decltype(C)::value;
        const double rpc = GL::template bcastc<c>(rp);
        if constexpr (c & 1) s1 += R[c] * rpc;
        else s0 += R[c] * rpc;
      });
      const double sv = s0 + s1;  // core: x~_c; row: v_r = G_r,c x~_c
      if (hc) {
        const double zr = al * ab_c * sv + (1 - al) * zc;
        double zn = zr + yc * irc;
        zn = fmin(fmax(zn, lo_c), up_c);
        dyc = rc * (zr - zn);
        yc += dyc;
        zc = zn;
        xc = al * sv + (1 - al) * xc;
      }
      if (hr) {
        const double xta = ha ? ta - c_r * sv : 0.0;
        {  // G row
          const double zr = al * (sv + g_r * xta) + (1 - al) * zg;
          double zn = zr + yg * irg;
          zn = fmin(fmax(zn, lo_g), up_g);
          dyg = rg * (zr - zn);
          yg += dyg;
          zg = zn;
        }
        if (ha) {  // bound row of the aux variable
          const double zr = al * ab_a * xta + (1 - al) * za;
          double zn = zr + ya * ira;
          zn = fmin(fmax(zn, lo_a), up_a);
          dya = ra * (zr - zn);
          ya += dya;
          za = zn;
          xa = al * xta + (1 - al) * xa;
        }
      }
      const bool check = kp.s.check_termination > 0 && it % kp.s.check_termination == 0;
      const bool adapt = kp.s.adaptive_rho && kp.s.adaptive_rho_interval > 0 && it % kp.s.adaptive_rho_interval == 0;
      if (!(check || adapt) && it < kp.s.max_iter) continue;
      // publish the iterate for the (LDS) residual / polish / rho code
      if (hc) {
        x[l] = xc;
        z[l] = zc;
        y[l] = yc;
        dy[l] = dyc;
      }
      if (hr) {
        z[ig] = zg;
        y[ig] = yg;
        dy[ig] = dyg;
        if (ha) {
          x[ia] = xa;
          z[ia] = za;
          y[ia] = ya;
          dy[ia] = dya;
        }
      }
      wsync();
      if (!(check || adapt)) continue;  // last iteration: published for the output
#ifdef DRC_PHASE_TIMING
      const unsigned long long tc0 = __builtin_amdgcn_s_memtime();
#endif
      const int act = admm_check<QD>(kpl, S, it, check, adapt, &status);
#ifdef DRC_PHASE_TIMING
      tchk += __builtin_amdgcn_s_memtime() - tc0;
#endif
      if (act == 2) break;
      load_regs();  // S^-1 / rho may have changed, the iterate may be polished
      d_r = dv[rr_];
      c_r = cf[rr_];
      rc = rv[lc_];
      ra = rv[ia];
      rg = rv[ig];
      irc = 1.0 / rc;
      ira = 1.0 / ra;
      irg = 1.0 / rg;
      xc = x[lc_];
      zc = z[lc_];
      yc = y[lc_];
      xa = x[ia];
      za = z[ia];
      ya = y[ia];
      zg = z[ig];
      yg = y[ig];
    }
#ifdef DRC_PHASE_TIMING
    PHG(26);
    if (l == 0) {
      atomicAdd(&g_phase_cycles[27], tchk);
      atomicAdd(&g_phase_cycles[26], 0ull - tchk);
    }
#endif
  } else if constexpr (QD::reg) {
    constexpr int NX = QD::nx, NG = QD::ng;
    double Gc[NG], Kr[NX], GKr[NX];
    prep_admm_mats<QD>(kpl, S);
    load_admm_regs<QD>(kp, S, Gc, Kr, GKr);
    PHG(25);
#ifdef DRC_PHASE_TIMING
    unsigned long long tchk = 0;
#endif
    const bool hb = l < NX, hg = l < NG;
    const int lb_ = hb ? l : 0, lg_ = hg ? NX + l : 0;
    const double ab_l = ab[lb_], q_l = qq[lb_], lo_b = lo[lb_], up_b = up[lb_], lo_g = lo[lg_], up_g = up[lg_];
    double rb = rv[lb_], rg = rv[lg_];
    double xl = 0, zb = 0, yb = 0, zg = 0, yg = 0, dyb = 0, dyg = 0;
    for (it = 1; it <= kp.s.max_iter; ++it) {
      const double wg = hg ? rg * zg - yg : 0.0;
      double r0 = hb ? sig * xl - q_l + ab_l * (rb * zb - yb) : 0.0, r1 = 0;
#pragma unroll
      for (int i = 0; i < NG; ++i) {
        const double wi = GL::bcast(wg, i);
        if (i & 1) r1 += Gc[i] * wi;
        else r0 += Gc[i] * wi;
      }
      const double rhs = hb ? r0 + r1 : 0.0;
      double x0 = 0, x1 = 0, a0 = 0, a1 = 0;
#pragma unroll
      for (int c = 0; c < NX; ++c) {
        const double rc = GL::bcast(rhs, c);
        if (c & 1) {
          x1 += Kr[c] * rc;
          a1 += GKr[c] * rc;
        } else {
          x0 += Kr[c] * rc;
          a0 += GKr[c] * rc;
        }
      }
      const double xtil = x0 + x1, ag = a0 + a1;
      if (hb) {  // z~ = A x~ ; relaxation ; projection ; dual update
        const double zr = al * ab_l * xtil + (1 - al) * zb;
        double zn = zr + yb / rb;
        zn = fmin(fmax(zn, lo_b), up_b);
        dyb = rb * (zr - zn);
        yb += dyb;
        zb = zn;
        xl = al * xtil + (1 - al) * xl;
      }
      if (hg) {
        const double zr = al * ag + (1 - al) * zg;
        double zn = zr + yg / rg;
        zn = fmin(fmax(zn, lo_g), up_g);
        dyg = rg * (zr - zn);
        yg += dyg;
        zg = zn;
      }
      const bool check = kp.s.check_termination > 0 && it % kp.s.check_termination == 0;
      const bool adapt = kp.s.adaptive_rho && kp.s.adaptive_rho_interval > 0 && it % kp.s.adaptive_rho_interval == 0;
      if (!(check || adapt) && it < kp.s.max_iter) continue;
      // publish the iterate for the (LDS) residual / polish / rho code
      if (hb) {
        x[l] = xl;
        z[l] = zb;
        y[l] = yb;
        dy[l] = dyb;
      }
      if (hg) {
        z[NX + l] = zg;
        y[NX + l] = yg;
        dy[NX + l] = dyg;
      }
      wsync();
      if (!(check || adapt)) continue;  // last iteration: published for the output
#ifdef DRC_PHASE_TIMING
      const unsigned long long tc0 = __builtin_amdgcn_s_memtime();
#endif
      const int act = admm_check<QD>(kpl, S, it, check, adapt, &status);
#ifdef DRC_PHASE_TIMING
      tchk += __builtin_amdgcn_s_memtime() - tc0;
#endif
      if (act == 2) break;
      // Always re-read the register state from LDS (published above, or
      // updated by the check): nothing large stays live across the call, so
      // the out-of-line block costs no spill traffic.
      load_admm_regs<QD>(kp, S, Gc, Kr, GKr);
      rb = rv[lb_];
      rg = rv[lg_];
      xl = x[lb_];
      zb = z[lb_];
      yb = y[lb_];
      zg = z[lg_];
      yg = y[lg_];
    }
#ifdef DRC_PHASE_TIMING
    PHG(26);
    if (l == 0) {
      atomicAdd(&g_phase_cycles[27], tchk);
      atomicAdd(&g_phase_cycles[26], 0ull - tchk);
    }
#endif
  } else {
    for (it = 1; it <= kp.s.max_iter; ++it) {
      for (int row = l; row < m; row += GL::size) w[row] = rv[row] * z[row] - y[row];
      wsync();
      if (l < nx) {
        double r0 = sig * x[l] - qq[l] + ab[l] * w[l], r1 = 0.0;
  #pragma unroll
        for (int i = 0; i < ng; i += 2) {
          r0 += G[i * nx + l] * w[nx + i];
          if (i + 1 < ng) r1 += G[(i + 1) * nx + l] * w[nx + i + 1];
        }
        xt[l] = r0 + r1;
      }
      wsync();
      double xtil = 0;
      if (l < nx) {
        double a0 = 0, a1 = 0;
  #pragma unroll
        for (int c = 0; c < nx; c += 2) {
          a0 += K[l * nx + c] * xt[c];
          if (c + 1 < nx) a1 += K[l * nx + c + 1] * xt[c + 1];
        }
        xtil = a0 + a1;
      }
      wsync();
      if (l < nx) xt[l] = xtil;
      wsync();
      // z~ = A x~ ; relaxation ; projection ; dual update
      if (l < nx) {
        const double zr = al * ab[l] * xtil + (1 - al) * z[l];
        double zn = zr + y[l] / rv[l];
        zn = fmin(fmax(zn, lo[l]), up[l]);
        const double d = rv[l] * (zr - zn);
        dy[l] = d;
        y[l] += d;
        z[l] = zn;
        x[l] = al * xtil + (1 - al) * x[l];
      }
      if (l < ng) {
        const int row = nx + l;
        double a0 = 0, a1 = 0;
  #pragma unroll
        for (int j = 0; j < nx; j += 2) {
          a0 += G[l * nx + j] * xt[j];
          if (j + 1 < nx) a1 += G[l * nx + j + 1] * xt[j + 1];
        }
        const double a = a0 + a1;
        const double zr = al * a + (1 - al) * z[row];
        double zn = zr + y[row] / rv[row];
        zn = fmin(fmax(zn, lo[row]), up[row]);
        const double d = rv[row] * (zr - zn);
        dy[row] = d;
        y[row] += d;
        z[row] = zn;
      }
      wsync();
      const bool check = kp.s.check_termination > 0 && it % kp.s.check_termination == 0;
      const bool adapt = kp.s.adaptive_rho && kp.s.adaptive_rho_interval > 0 && it % kp.s.adaptive_rho_interval == 0;
      if (check || adapt) residuals<QD>(kp, S, x, z, y, kp.s.eps_abs, kp.s.eps_rel);
      if (check) {
        const bool conv = sc[SC_PRI] < sc[SC_EPSP] && sc[SC_DUA] < sc[SC_EPSD];
        // parity mode: a certified polish is exact whatever the ADMM
        // residual, so also try it every 4th check (slow-ADMM vertices)
        if (kp.s.exact && !conv && sc[SC_PFAIL] < kPolishMaxEarly) {
          if (polish<QD>(kp, S, true)) {
            status = DRC_STATUS_SOLVED;
            break;
          }
          if (l == 0) sc[SC_PFAIL] += 1.0;
          factor_kinv<QD>(kp, S);  // polish used the union region
          residuals<QD>(kp, S, x, z, y, kp.s.eps_abs, kp.s.eps_rel);
        }
        if (conv) {
          if (!kp.s.exact) {
            status = DRC_STATUS_SOLVED;
            break;
          }
          if (sc[SC_PFAIL] < kPolishMaxTotal) {
            if (polish<QD>(kp, S, true)) {
              status = DRC_STATUS_SOLVED;
              break;
            }
            if (l == 0) sc[SC_PFAIL] += 1.0;
            factor_kinv<QD>(kp, S);  // polish used the union region
          }
          residuals<QD>(kp, S, x, z, y, kp.s.eps_fallback, kp.s.eps_fallback);
          if (sc[SC_PRI] < sc[SC_EPSP] && sc[SC_DUA] < sc[SC_EPSD]) {
            status = DRC_STATUS_SOLVED;
            break;
          }
        } else if (primal_infeasible<QD>(kp, S, kp.s.eps_prim_inf)) {
          status = DRC_STATUS_PRIMAL_INFEASIBLE;
          break;
        }
      }
      if (adapt) {
        const double pr = sc[SC_PRIS] / (fmax(sc[SC_NAX], sc[SC_NZ]) + kDivTol);
        const double dr = sc[SC_DUAS] / (fmax(fmax(sc[SC_NQ], sc[SC_NATY]), sc[SC_NPX]) + kDivTol);
        const double rho = sc[SC_RHO];
        double rn = rho * sqrt(pr / (dr + kDivTol));
        rn = fmin(fmax(rn, kRhoMin), kRhoMax);
        if (rn > rho * kp.s.adaptive_rho_tolerance || rn < rho / kp.s.adaptive_rho_tolerance) {
          set_rho<QD>(kp, S, rn);
          factor_kinv<QD>(kp, S);
        }
      }
    }
  }
  *iters_out = it > kp.s.max_iter ? kp.s.max_iter : it;
  if (status == DRC_STATUS_SOLVED && kp.s.polish && !kp.s.exact) polish<QD>(kp, S, false);
  return status;
}

// QP kernel: assembles and solves the QP of each instance from the task
// record written by task_kernel.
#ifndef DRC_QP_WAVES
#define DRC_QP_WAVES 2
#endif
template <class QD>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(DRC_QP_WAVES, 8)))
qp_kernel(const DevModel* __restrict__ M0, const KParams kp, const IO io) {
  extern __shared__ __attribute__((aligned(16))) double S[];
  // LDS copy of the parameters for the out-of-line (rare) ADMM blocks: a
  // reference to the kernel argument itself would be copied to scratch
  __shared__ KParams kpl;
  {
    static_assert(sizeof(KParams) % 8 == 0, "KParams copied as 8-byte words");
    const uint64_t* src = reinterpret_cast<const uint64_t*>(&kp);
    uint64_t* dst = reinterpret_cast<uint64_t*>(&kpl);
    for (int e = lane_id(); e < static_cast<int>(sizeof(KParams) / 8); e += 64) dst[e] = src[e];
    wsync();
  }
  // QD::gs = 32: two instances per wave, each lane group on its own LDS
  // plan (the launch allocates one per group) and its own instance sequence
  using GL = Grp<QD::gs>;
  const int l = GL::lane();
  double* const Sg = S + (GL::upper() ? kp.lds_doubles : 0);
  const int64_t B = io.B;
  PH_DECL
  // hard_mode 1: the lane stage's hard list (grid stride); 2: every instance
  // except the flagged ones (their records are still being written)
  const bool hl = io.hard_mode == 1;
  const InstSeqG<QD::gs> seq(hl ? int64_t(*io.hard_n) : B, hl ? 0 : kp.xcd_map, hl ? nullptr : io.queue);
  for (int64_t j = seq.first(); j < seq.n; j = seq.next(j)) {
    const int64_t b = hl ? int64_t(io.hard_list[j]) : seq.at(j);
    if (b >= B) continue;
    if (io.hard_mode == 2 && io.hard_flag[b]) continue;
    const int64_t gb = io.b0 + b, LD = io.ld;  // position in the caller's [field][B] arrays
    const DevModel* M = M0;
    asm volatile("" : "+s"(M));
    double* S = Sg;
    qp_assemble<QD>(M, kp, S, io, b);
    PH(0);
    const bool lp_inf = M->kind == 1 && kp.s.exact && moma_lp_infeasible<QD>(M, kp, S);
    int status, iters = 0;
    if constexpr (QD::reg) status = qp_scale_regs<QD>(kpl, S);
    else status = qp_scale<QD>(kp, S);
    PH(1);
    if (status != DRC_STATUS_NONFINITE) {
      if (lp_inf) status = DRC_STATUS_PRIMAL_INFEASIBLE;
      else status = qp_admm<QD>(kp, kpl, S, &iters);
    }
    PH(3);
    // ---------------- outputs (zero on failure, QP_IK.cpp:56-61) ------------
    const double *D = S + kp.oD, *x = S + kp.oX;
    if (l < kp.na) io.out[(int64_t)l * LD + gb] = status == DRC_STATUS_SOLVED ? D[l] * x[l] : 0.0;
    if (l == 0) {
      io.status[gb] = status;
      if (io.iters) io.iters[gb] = iters;
    }
    wsync();
    PH(5);
  }
  PH_FLUSH(16);
}

// ------------------------------------------------------------------------
// QPID: the torque-level QP.
//   manipulator  (src/manipulator/QP_ID.cpp:7-193):
//     x = [qdd(n) | tau(n) | s_qmin | s_qmax | s_qdmin | s_qdmax (n each) | s_sing | s_col]
//     P[qdd,qdd] = 2 J^T J, q[qdd] = -2 J^T (xdd - Jdot qdot), q[slacks] = 1000
//     bounds: slacks >= 0, the rest free
//   mobile manipulator (src/mobile_manipulator/QP_ID.cpp:7-184):
//     x = [eta_dot(A) | tau(A)], P = 2 J~^T J~, q = -2 J~^T (xdd - J~dot eta), no bound rows
//   rows (arm joints i, alpha = 50):
//     qdd_i (+s) >= -2a qdot_i - a^2 (q_i - q_min)     -qdd_i (+s) >= 2a qdot_i - a^2 (q_max - q_i)
//     qdd_i (+s) >= -a (qdot_i - qdot_min)             -qdd_i (+s) >= -a (qdot_max - qdot_i)
//     grad_m . qdd (+s) >= -gd_m - 2a grad_m . qdot - a^2 (m - 0.01)
//     grad_d . qdd (+s) >= -gd_d - 2a grad_d . qdot - a^2 (d - 0.05)
//     [M -I] [qdd; tau] = -g                           (equality rows)
// Runs the generic (runtime-sized, LDS) OSQP path: nx = 6n+2 / 2A, ng = 4n+2+A.
// ------------------------------------------------------------------------
__device__ __forceinline__ void qpid_assemble(const DevModel* M, const KParams& kp, double* S, const IO& io,
                                              int64_t b) {
  const int l = lane_id();
  const int nv = kp.nv, narm = kp.narm, na = kp.na;
  const int64_t gb = io.b0 + b, LD = io.ld;
  double *qv = S + kp.kq, *qdl = S + kp.kqd, *J = S + kp.kJ, *xdd = S + kp.kxdd, *mg = S + kp.kmg, *dgv = S + kp.kdg,
         *bias = S + kp.kBias, *Mq = S + kp.kMq, *Gq = S + kp.kGq;
  {
    const double* rec = io.rec + b * io.rec_stride;
    for (int e = l; e < kp.rLen; e += 64) {
      const double v = rec[e];
      if (e < kp.rMan) J[e] = v;
      else if (e == kp.rMan) S[kp.oSc + SC_MAN] = v;
      else if (e < kp.rDist) mg[e - kp.rMan - 1] = v;
      else if (e == kp.rDist) S[kp.oSc + SC_DIST] = v;
      else if (e < kp.rXdd) dgv[e - kp.rDist - 1] = v;
      else if (e < kp.rQ) xdd[e - kp.rXdd] = v;
      else if (e < kp.rQd) qv[e - kp.rQ] = v;
      else if (e < kp.rBias) qdl[e - kp.rQd] = v;
      else bias[e - kp.rBias] = v;
    }
    for (int e = l; e < na * na; e += 64) Mq[e] = io.dM[(int64_t)e * LD + gb];
    if (l < na) Gq[l] = io.dG[(int64_t)l * LD + gb];
  }
  wsync();
  const int nx = kp.nx, ng = kp.ng, np = kp.np;
  double *P = S + kp.oP, *G = S + kp.oG, *qq = S + kp.oQ, *ab = S + kp.oAB, *lo = S + kp.oL, *up = S + kp.oU;
  const double a = kp.alpha_cbf, man = S[kp.oSc + SC_MAN], dist = S[kp.oSc + SC_DIST];
  double* Jt = S + kp.kJt;  // 6 x na
  if (M->kind == 0) {
    for (int e = l; e < 6 * np; e += 64) Jt[e] = J[(e / np) * nv + e % np];
  } else {  // J~ = J S (robot_data.cpp:407-410)
    const double yaw = qv[M->virtual_start + 2], cy = cos(yaw), sy = sin(yaw);
    const double(*Jm)[kMaxWheels] = mobile_jac(M, kp, S, qv);
    for (int e = l; e < 6 * np; e += 64) {
      const int r = e / np, c = e % np;
      double v = 0;
      const int am = c - M->act_mani_start, aw = c - M->act_mobi_start;
      if (am >= 0 && am < M->n_arm) {
        v = J[r * nv + M->mani_start + am];
      } else if (aw >= 0 && aw < M->n_wheel) {
        const double s0 = cy * Jm[0][aw] - sy * Jm[1][aw];
        const double s1 = sy * Jm[0][aw] + cy * Jm[1][aw];
        const double s2 = Jm[2][aw];
        const int vs = M->virtual_start;
        v = J[r * nv + M->mobi_start + aw] + J[r * nv + vs] * s0 + J[r * nv + vs + 1] * s1 + J[r * nv + vs + 2] * s2;
      }
      Jt[e] = v;
    }
  }
  wsync();
  for (int e = l; e < np * np; e += 64) {
    const int i = e / np, j = e % np;
    double s = 0;
    for (int r = 0; r < 6; ++r) s += Jt[r * np + i] * Jt[r * np + j];
    P[e] = 2.0 * s + (i == j ? kp.w_reg : 0.0);
  }
  for (int e = l; e < ng * nx; e += 64) G[e] = 0.0;
  const bool slacks = M->kind == 0;
  if (l < nx) {
    double qi = 0;
    if (l < np) {
      double s = 0;
      for (int r = 0; r < 6; ++r) s += Jt[r * np + l] * (xdd[r] - bias[r]);
      qi = -2.0 * s;
    } else if (l >= 2 * na) {
      qi = kp.slack_w;
    }
    qq[l] = qi;
    ab[l] = slacks ? 1.0 : 0.0;  // MoMa: nbc = 0 -> zero rows, equivalent to no bound rows
    lo[l] = (slacks && l >= 2 * na) ? 0.0 : -kInf;
    up[l] = kInf;
  }
  wsync();
  if (l < ng) {
    const int n = narm, row = nx + l;
    const int vo = M->kind == 0 ? 0 : M->act_mani_start;  // QP column of arm joint 0
    const int qo = M->kind == 0 ? 0 : M->mani_start;      // joint index of arm joint 0
    double* Gr = G + l * nx;
    double lval, uval = kInf;
    if (l < 4 * n) {
      const int k = l / n, i = l % n, jq = qo + i;
      const double qi = qv[jq], qdi = qdl[jq];
      Gr[vo + i] = (k & 1) ? -1.0 : 1.0;
      if (slacks) Gr[2 * na + k * n + i] = 1.0;
      if (k == 0) lval = -2 * a * qdi - a * a * (qi - M->lower[jq]);
      else if (k == 1) lval = 2 * a * qdi - a * a * (M->upper[jq] - qi);
      else if (k == 2) lval = -a * (qdi + M->vel[jq]);
      else lval = -a * (M->vel[jq] - qdi);
    } else if (l == 4 * n) {
      double gq = 0;
      for (int c = 0; c < n; ++c) {
        Gr[vo + c] = mg[c];
        gq += mg[c] * qdl[qo + c];
      }
      if (slacks) Gr[2 * na + 4 * n] = 1.0;
      lval = -bias[6] - 2 * a * gq - a * a * (man - kp.man_min);
    } else if (l == 4 * n + 1) {
      double gq = 0;
      for (int c = 0; c < n; ++c) {
        Gr[vo + c] = dgv[qo + c];
        gq += dgv[qo + c] * qdl[qo + c];
      }
      if (slacks) Gr[2 * na + 4 * n + 1] = 1.0;
      lval = -bias[7] - 2 * a * gq - a * a * (dist - kp.dist_min);
    } else {  // [M -I][qdd; tau] = -g (QP_ID.cpp:176-192)
      const int i = l - (4 * n + 2);
      for (int c = 0; c < na; ++c) Gr[c] = Mq[i * na + c];
      Gr[na + i] = -1.0;
      lval = uval = -Gq[i];
    }
    lo[row] = lval;
    up[row] = uval;
  }
  wsync();
}

// QD: Dims<nx, ng, np, false> for the bundled robots' QPID shapes (loops
// unroll, loads pipeline), Dims<0, 0, 0> otherwise.
template <class QD>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 8)))
qpid_kernel(const DevModel* __restrict__ M0, const KParams kp, const IO io) {
  extern __shared__ __attribute__((aligned(16))) double S[];
  __shared__ KParams kpl;
  const int l = lane_id();
  {
    const uint64_t* src = reinterpret_cast<const uint64_t*>(&kp);
    uint64_t* dst = reinterpret_cast<uint64_t*>(&kpl);
    for (int e = l; e < static_cast<int>(sizeof(KParams) / 8); e += 64) dst[e] = src[e];
    wsync();
  }
  const int64_t B = io.B;
  const InstSeq seq(B, kp.xcd_map, io.queue);
  for (int64_t j = seq.first(); j < seq.n; j = seq.next(j)) {
    const int64_t b = seq.at(j);
    if (b >= B) continue;
    const int64_t gb = io.b0 + b, LD = io.ld;
    const DevModel* M = M0;
    asm volatile("" : "+s"(M));
    qpid_assemble(M, kp, S, io, b);
    int status, iters = 0;
    status = qp_scale<QD>(kp, S);
    if (status != DRC_STATUS_NONFINITE) status = qp_admm<QD>(kp, kpl, S, &iters);
    // outputs: QP_ID.cpp:74-83 getOptJoint; failure -> qdd = 0, tau = gravity
    // (robot_controller.cpp:333-336; MoMa :208-213 slices the joint-order
    // gravity at actuator offsets — restated as written)
    const double *D = S + kp.oD, *x = S + kp.oX;
    const int na = kp.na;
    const bool ok = status == DRC_STATUS_SOLVED;
    if (l < na) {
      io.out[(int64_t)l * LD + gb] = ok ? D[l] * x[l] : 0.0;
      const double gfail = M->kind == 0 ? io.dG[(int64_t)l * LD + gb] : io.dGf[(int64_t)l * LD + gb];
      io.out2[(int64_t)l * LD + gb] = ok ? D[na + l] * x[na + l] : gfail;
    }
    if (l == 0) {
      io.status[gb] = status;
      if (io.iters) io.iters[gb] = iters;
    }
    wsync();
  }
}

}  // namespace drc_amd

// ==========================================================================
// host side: the C-ABI (include/drc_amd.h)
// ==========================================================================
namespace drc_amd {

// Per-stream scratch of a model: the task-record pool, the work-queue
// counters and the fork/join lanes.  Calls on one stream are ordered by that
// stream, so they may share it; calls on two streams get disjoint contexts
// (the C-ABI's "reentrant per stream", include/drc_amd.h).
struct StreamCtx {
  hipStream_t stream = nullptr;
  void* pool = nullptr;  // task records / QPID dynamics / OSF M^-1, g
  int64_t pool_bytes = 0;
  // work-queue counters: [slot][kernel (task, QP)][8 XCD classes]; slots
  // 0..15 the QPIK sub-batches, 16 QPID, 17 the closed-form controllers
  static constexpr int kSlotInts = 32;  // task queue 8, QP queue 8, lane-stage hard count 1
  static constexpr int kQueueSlotQpid = 16, kQueueSlotCf = 17, kQueueInts = 18 * kSlotInts;
  int* d_queue = nullptr;
  std::vector<hipStream_t> lanes;  // concurrent sub-batches (drc_set_concurrency)
  std::vector<hipEvent_t> joins;
  // per sub-batch: the lane stage's hard instances run their task kernel on a
  // side stream while the QP of the other instances runs
  std::vector<hipStream_t> sides;
  std::vector<hipEvent_t> side_fork, side_join;
  hipEvent_t fork = nullptr;
  int* dyn_list = nullptr;  // instances whose M_inv needs the serial COD
  int64_t dyn_list_cap = 0;
};

struct drc_model_impl {
  HostModel hm;
  DevModel* d_model = nullptr;
  int device = 0;
  drc_kinematic_param kparam{};
  drc_joint_index jidx{};
  drc_actuator_index aidx{};
  std::vector<std::unique_ptr<StreamCtx>> ctxs;  // one per caller stream seen
  int timing = 0;  // drc_debug_kernel_timing: HIP events around each launch
  int lane_stage = 0;  // drc_debug_lane_stage: 0 off, 1 lane stage + side-stream hard path, 2 + serial hard path, 3 auto
  // timed calls: {caller-stream start, caller-stream end, per chunk: task start, task end, qp end}
  std::vector<std::vector<hipEvent_t>> events;
  // concurrent sub-batches: the batch is cut into `chunks` contiguous ranges
  // run on internal streams forked from / joined to the caller's stream, so
  // one range's task kernel overlaps another's QP kernel and the straggler
  // tails of the kernels interleave.  3 measured best on MI355X (FR3, B = 65 536:
  // 1 / 2 / 3 / 4 chunks = 7.3 / 8.5 / 8.9 / 7.3 M solves/s; 3 lanes plus the
  // caller's stream fit the 4 hardware queues a process gets by default)
  int chunks = 3;
  // host-buffer entry points: device staging + an internal stream
  std::mutex host_mu;
  void* stage = nullptr;
  int64_t stage_bytes = 0;
  hipStream_t hstream = nullptr;
  std::mutex mu;         // the context list, timing events, concurrency
  std::mutex launch_mu;  // one call's launch sequence is enqueued as a unit, so
                         // two host threads sharing a stream cannot interleave
                         // their kernels on its scratch
};

static thread_local std::string g_last_error;
static int set_err(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}
#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) return set_err(DRC_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

// The scratch context of `st` (created on first use; caller holds m->mu).
static int stream_ctx(drc_model_impl* m, hipStream_t st, StreamCtx** out) {
  for (auto& c : m->ctxs)
    if (c->stream == st) {
      *out = c.get();
      return DRC_OK;
    }
  std::unique_ptr<StreamCtx> c(new StreamCtx());
  c->stream = st;
  HIP_TRY(hipMalloc(&c->d_queue, StreamCtx::kQueueInts * sizeof(int)));
  *out = c.get();
  m->ctxs.push_back(std::move(c));
  return DRC_OK;
}
static int ensure_pool(StreamCtx* c, int64_t bytes) {
  if (c->pool_bytes >= bytes) return DRC_OK;
  if (c->pool) HIP_TRY(hipFree(c->pool));  // synchronises: no launch still reads it
  c->pool = nullptr;
  c->pool_bytes = 0;
  HIP_TRY(hipMalloc(&c->pool, bytes));
  c->pool_bytes = bytes;
  return DRC_OK;
}
static void free_ctx(StreamCtx* c) {
  for (hipStream_t ls : c->lanes) (void)hipStreamSynchronize(ls);
  if (c->d_queue) (void)hipFree(c->d_queue);
  if (c->pool) (void)hipFree(c->pool);
  if (c->dyn_list) (void)hipFree(c->dyn_list);
  for (hipStream_t ls : c->sides) (void)hipStreamSynchronize(ls);
  for (hipStream_t ls : c->lanes) (void)hipStreamDestroy(ls);
  for (hipEvent_t e : c->joins) (void)hipEventDestroy(e);
  for (hipStream_t ls : c->sides) (void)hipStreamDestroy(ls);
  for (hipEvent_t e : c->side_fork) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->side_join) (void)hipEventDestroy(e);
  if (c->fork) (void)hipEventDestroy(c->fork);
}

// DyrosMath::PinvCOD on a small dense matrix (host, model build only):
// Moore-Penrose inverse via the normal equations' symmetric eigen-system,
// rank cut at 1e-6 relative (math_type_define.h:7,563-570).
static void pinv_small(const double* A, int r, int c, double* X /* c x r */) {
  // X = (A^T A)^+ A^T with (A^T A) symmetric c x c (c <= 3 here)
  double N[9] = {0}, V[9], w[3];
  for (int i = 0; i < c; ++i)
    for (int j = 0; j < c; ++j)
      for (int k = 0; k < r; ++k) N[i * c + j] += A[k * c + i] * A[k * c + j];
  for (int i = 0; i < c * c; ++i) V[i] = (i % (c + 1) == 0) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0;
    for (int i = 0; i < c; ++i)
      for (int j = i + 1; j < c; ++j) off += N[i * c + j] * N[i * c + j];
    if (off < 1e-300) break;
    for (int p = 0; p < c; ++p)
      for (int q = p + 1; q < c; ++q) {
        if (std::fabs(N[p * c + q]) < 1e-300) continue;
        double th = (N[q * c + q] - N[p * c + p]) / (2 * N[p * c + q]);
        double t = (th >= 0 ? 1 : -1) / (std::fabs(th) + std::sqrt(th * th + 1));
        double cs = 1 / std::sqrt(t * t + 1), sn = t * cs;
        for (int k = 0; k < c; ++k) {
          double a = N[k * c + p], b = N[k * c + q];
          N[k * c + p] = cs * a - sn * b;
          N[k * c + q] = sn * a + cs * b;
        }
        for (int k = 0; k < c; ++k) {
          double a = N[p * c + k], b = N[q * c + k];
          N[p * c + k] = cs * a - sn * b;
          N[q * c + k] = sn * a + cs * b;
        }
        for (int k = 0; k < c; ++k) {
          double a = V[k * c + p], b = V[k * c + q];
          V[k * c + p] = cs * a - sn * b;
          V[k * c + q] = sn * a + cs * b;
        }
      }
  }
  double wmax = 0;
  for (int i = 0; i < c; ++i) {
    w[i] = N[i * c + i];
    wmax = std::fmax(wmax, std::fabs(w[i]));
  }
  double Ni[9] = {0};
  for (int e = 0; e < c; ++e) {
    if (std::sqrt(std::fabs(w[e])) <= 1e-6 * std::sqrt(wmax)) continue;
    for (int i = 0; i < c; ++i)
      for (int j = 0; j < c; ++j) Ni[i * c + j] += V[i * c + e] * V[j * c + e] / w[e];
  }
  for (int i = 0; i < c; ++i)
    for (int k = 0; k < r; ++k) {
      double s = 0;
      for (int j = 0; j < c; ++j) s += Ni[i * c + j] * A[k * c + j];
      X[i * r + k] = s;
    }
}

// Mobile::RobotData::computeFKJacobian (src/mobile/robot_data.cpp:123-204) at
// the wheel positions `wheel_pos` (used by the caster drive only; may be NULL
// for the configuration-independent drives, then zero steer angles).
static int mobile_fk_jacobian(const drc_kinematic_param& p, int* W, double out[3][kMaxWheels],
                              const double* wheel_pos = nullptr) {
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < kMaxWheels; ++c) out[r][c] = 0;
  if (p.type == DRC_DRIVE_DIFFERENTIAL) {
    *W = 2;
    out[0][0] = p.wheel_radius / 2.;
    out[0][1] = p.wheel_radius / 2.;
    out[2][0] = -p.wheel_radius / p.base_width;
    out[2][1] = p.wheel_radius / p.base_width;
    return DRC_OK;
  }
  if (p.type == DRC_DRIVE_MECANUM) {
    const int n = p.n_wheels;
    if (n < 1 || n > kMaxWheels) return set_err(DRC_ERR_INVALID_ARGUMENT, "mecanum wheel count out of range");
    double Jinv[kMaxWheels * 3], X[3 * kMaxWheels];
    for (int i = 0; i < n; ++i) {
      const double r = p.wheel_radius, g = p.roller_angles[i], px = p.base2wheel_positions[i][0],
                   py = p.base2wheel_positions[i][1], pt = p.base2wheel_angles[i];
      // (1/r) [1 tan g] [[cos pt, sin pt], [-sin pt, cos pt]] [[1 0 -py], [0 1 px]]
      const double a0 = std::cos(pt) - std::tan(g) * std::sin(pt), a1 = std::sin(pt) + std::tan(g) * std::cos(pt);
      Jinv[i * 3 + 0] = a0 / r;
      Jinv[i * 3 + 1] = a1 / r;
      Jinv[i * 3 + 2] = (-a0 * py + a1 * px) / r;
    }
    pinv_small(Jinv, n, 3, X);
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < n; ++c) out[r][c] = X[r * n + c];
    *W = n;
    return DRC_OK;
  }
  if (p.type == DRC_DRIVE_CASTER) {  // CasterFKJacobian (:179-204): W = 2 x casters
    const int C = p.n_wheels;
    if (C < 1 || 2 * C > kMaxWheels) return set_err(DRC_ERR_INVALID_ARGUMENT, "caster count out of range");
    double zero[kMaxWheels] = {0};
    caster_fk_jacobian(C, p.wheel_radius, p.wheel_offset, p.base2wheel_positions, wheel_pos ? wheel_pos : zero, out);
    *W = 2 * C;
    return DRC_OK;
  }
  return set_err(DRC_ERR_INVALID_ARGUMENT, "unknown drive type");
}

// Mobile::RobotController::computeIKJacobian (src/mobile/robot_controller.cpp:55-125):
// wheel velocities = J_ik (W x 3, row-major) * base twist.
static int mobile_ik_jacobian(const drc_kinematic_param& p, const double* wheel_pos, double* J, int* W) {
  const double r = p.wheel_radius;
  if (p.type == DRC_DRIVE_DIFFERENTIAL) {  // DifferentialIKJacobian (:76-84)
    *W = 2;
    const double e[6] = {1 / r, 0, -p.base_width / (2 * r), 1 / r, 0, p.base_width / (2 * r)};
    for (int i = 0; i < 6; ++i) J[i] = e[i];
    return DRC_OK;
  }
  if (p.type == DRC_DRIVE_MECANUM) {  // MecanumIKJacobian (:86-107)
    const int n = p.n_wheels;
    if (n < 1 || n > kMaxWheels) return set_err(DRC_ERR_INVALID_ARGUMENT, "mecanum wheel count out of range");
    for (int i = 0; i < n; ++i) {
      const double g = p.roller_angles[i], px = p.base2wheel_positions[i][0], py = p.base2wheel_positions[i][1],
                   pt = p.base2wheel_angles[i];
      const double a0 = std::cos(pt) - std::tan(g) * std::sin(pt), a1 = std::sin(pt) + std::tan(g) * std::cos(pt);
      J[i * 3 + 0] = a0 / r;
      J[i * 3 + 1] = a1 / r;
      J[i * 3 + 2] = (-a0 * py + a1 * px) / r;
    }
    *W = n;
    return DRC_OK;
  }
  if (p.type == DRC_DRIVE_CASTER) {  // CasterIKJacobian (:109-125), steer angle = wheel_pos(2i)
    const int C = p.n_wheels;
    if (C < 1 || 2 * C > kMaxWheels) return set_err(DRC_ERR_INVALID_ARGUMENT, "caster count out of range");
    const double b = p.wheel_offset;
    for (int i = 0; i < C; ++i) {
      const double phi = wheel_pos ? wheel_pos[2 * i] : 0.0, sp = std::sin(phi), cp = std::cos(phi);
      const double px = p.base2wheel_positions[i][0], py = p.base2wheel_positions[i][1];
      double* r0 = J + (2 * i) * 3;
      double* r1 = J + (2 * i + 1) * 3;
      r0[0] = -sp / b;
      r0[1] = cp / b;
      r0[2] = (px * cp + py * sp) / b - 1;
      r1[0] = cp / r;
      r1[1] = sp / r;
      r1[2] = (px * sp - py * cp) / r;
    }
    *W = 2 * C;
    return DRC_OK;
  }
  return set_err(DRC_ERR_INVALID_ARGUMENT, "unknown drive type");
}

static int upload(drc_model_impl* m) {
  HIP_TRY(hipSetDevice(m->device));
  HIP_TRY(hipMalloc(&m->d_model, sizeof(DevModel)));
  HIP_TRY(hipMemcpy(m->d_model, &m->hm.dev, sizeof(DevModel), hipMemcpyHostToDevice));
  return DRC_OK;
}

// LDS plan: persistent QP region + a union of (kinematics | K^-1 | polish)
// lanes per instance of the compiled QPIK QP shapes.  32 packs two instances
// per wave (Grp<32>: group reductions, DPP / ds_bpermute broadcasts,
// per-group instance sequence and LDS plan; parity tests green) but measured
// slower on FR3: 13.7 M solves/s at two waves per SIMD, 13.4 M at one,
// against 15.9 M for 64
#ifndef DRC_QP_GROUP
#define DRC_QP_GROUP 64
#endif
constexpr int kQpGroup = DRC_QP_GROUP;

// QPIK QP shapes with a compile-time qp_kernel instantiation (register ADMM
// on the Schur complement); launch() dispatches on the same list
static bool qp_compiled(int nx, int ng, int np) {
  return (nx == 23 && ng == 16 && np == 7) || (nx == 20 && ng == 14 && np == 6) || (nx == 9 && ng == 16 && np == 9) ||
         (nx == 11 && ng == 16 && np == 11);
}

static int plan_layout(const DevModel& M, KParams* k, bool task_only) {
  int off = 0;
  auto take = [&](int n) {
    int o = off;
    off += (n + 1) & ~1;  // keep 16-byte alignment
    return o;
  };
  const int nx = k->nx, ng = k->ng, np = k->np, m = k->m, nv = M.nv;
  if (task_only) {  // task_kernel: scalars + kinematics only
    k->oRed = take(64);
    k->oSc = take(32);
  } else {
  k->oP = take(np * np);
  k->oG = take(ng * nx);
  k->oQ = take(nx);
  k->oAB = take(nx);
  k->oL = take(m);
  k->oU = take(m);
  k->oD = take(nx);
  k->oE = take(m);
  k->oRho = take(m);
  k->oX = take(nx);
  k->oZ = take(m);
  k->oY = take(m);
  k->oDY = take(m);
  k->oXT = take(nx);
  k->oZT = take(m);
  k->oT1 = take(m > nx ? m : nx);
  k->oT2 = take(m > nx ? m : nx);
  k->oRed = take(64);
  k->oSc = take(32);
  }
  k->oHi = -1;
  if (!task_only && k->problem == 0 && M.kind == 1 && qp_compiled(nx, ng, np)) k->oHi = take(nx * nx);
  k->oU0 = off;
  if (!task_only && k->problem == 0) {
    // QPIK QP kernel: the union holds only what it uses -- the task record
    // view (q, J, xdd, grad m, grad d, the mobile Jacobian, the task
    // Jacobian), the factor (Schur blocks for the compiled shapes, K^-1
    // otherwise) and the polish (index lists, x / y candidates; the LDS
    // EQP only where a KKT can exceed the register EQP's kEqpRegCap).
    // FR3: ~10 KB per wave instead of ~20.
    int u = k->oU0;
    auto takeu = [&](int n) {
      int o = u;
      u += (n + 1) & ~1;
      return o;
    };
    k->kq = takeu(nv);
    k->kJ = takeu(6 * nv);
    k->kxdd = takeu(6);
    k->kmg = takeu(k->narm);
    k->kdg = takeu(nv);
    k->kSv = takeu(3 * kMaxWheels);
    k->kJt = takeu(6 * np);
    const int kin_end = u;
    const int fac_end = k->oU0 + (qp_compiled(nx, ng, np) ? np * np + ng * np + 4 * ng : nx * nx + nx * ng);
    // manipulator QPs: the register EQP's size; a larger reduced KKT fails
    // that polish attempt and ADMM continues (the oracle applies the same
    // cap).  Whole-body QPs have no variable bounds, so every variable is free
    // in the reduced KKT (N = nx + active rows): capped at 16 their polish
    // fails whenever 6 (XLS-FR3) / 8 (Husky-FR3) rows are active and the
    // instance runs to the tight ADMM fallback (up to ~3 000 iterations);
    // they get the LDS EQP for N > 16
    const int N = M.kind == 1 ? nx + ng : (nx + ng < kEqpRegCap ? nx + ng : kEqpRegCap);
    k->ncap = N;
    k->nbuf = (N + 7) & ~7;
    const int reg_pol = k->oU0 + 128 + m;  // Fidx/Ridx | xx | yy
    // (compiled whole-body shapes solve every polish KKT in range-space form,
    // eqp_range: its H^-1 g_a buffer instead of the LDS LDL^T's)
    const int lds_pol = k->oHi >= 0 ? k->oU0 + 256 + kEqpRegCap * nx
                        : (qp_compiled(nx, ng, np) && N <= kEqpRegCap) ? 0
                        : k->oU0 + 64 + 64 + 128 + k->nbuf * 5 + N * (N + 1) / 2;
    int end = kin_end;
    end = end > fac_end ? end : fac_end;
    end = end > reg_pol ? end : reg_pol;
    end = end > lds_pol ? end : lds_pol;
    k->lds_doubles = (end + 1) & ~1;  // 16-byte aligned: the second lane group's plan follows
    if (end * 8 > 160 * 1024) return set_err(DRC_ERR_UNSUPPORTED, "model too large for the per-wave LDS plan");
    return DRC_OK;
  }
  // kinematics view of the union
  int u = k->oU0;
  auto takeu = [&](int n) {
    int o = u;
    u += (n + 1) & ~1;
    return o;
  };
  k->kT = takeu((nv + 1) * 12);
  k->kZ = takeu((nv + 1) * 3);
  k->kTe = takeu(12);
  k->kJ = takeu(6 * nv);
  const int ng_ = M.ngeom > nv ? M.ngeom : nv;
  k->kTg = takeu(ng_ * 12);
  k->kq = takeu(nv);
  k->kqd = takeu(nv);
  k->kPd = takeu(M.npairs);
  k->kPf = takeu(M.npairs);
  k->kxdd = takeu(6);
  k->kmg = takeu(k->narm);
  k->kdg = takeu(nv);
  k->kSv = takeu(3 * kMaxWheels);
  const bool epa = task_only && !k->cf;
  // QPID's task extras read Ai and W after the collision stage
  if (!epa || k->problem == 1) {
    k->kAi = takeu(36);
    k->kW = takeu(k->narm * 6);
  }
  if (k->problem == 1) {  // QPID stage data (task kernel) and dynamics (QP kernel)
    k->kJd = takeu(6 * nv);
    k->kDa = takeu(6 * k->narm);
    k->kVf = takeu(nv);
    k->kX6 = takeu(72 + 6 * k->narm + 2 * k->narm * k->narm);
    k->kGdv = takeu(k->narm + nv);
    k->kBias = takeu(8);
    k->kMq = takeu(k->na * k->na);
    k->kGq = takeu(k->na);
  }
  if (k->cf) {  // W, W2 (6 x nv), M^-1, nu, g, task vectors, then the serial COD work (+ its nv x 6 result)
    const int ws = 6 * nv + 36 + 6 * nv + 18 + 2 * nv + 6 * nv;
    k->kCf = takeu(2 * 6 * nv + nv * nv + 3 * nv + 48 + (ws > 160 ? ws : 160));
  }
  // Regions dead once the collision stage starts (manipulability work, the
  // QP kernel's task Jacobian), then the EPA polytope laid over them: they
  // share LDS, which keeps the QPIK task kernel within 20 KB per wave
  // (8 waves per CU).  The GJK candidate list lives in the polytope's space
  // too (it is consumed before EPA starts).
  const int scr0 = u;
  if (epa && k->problem != 1) {
    k->kAi = takeu(36);
    k->kW = takeu(k->narm * 6);
  }
  k->kA6 = takeu(36);
  k->kPart = takeu(k->narm * k->narm);
  k->kJt = takeu(6 * np);
  k->kScr = takeu(160);  // serial 6x6 COD work (pinv_cod_serial: 3n^2 + 3n)
  if (epa) {
    k->kEpa = scr0;
    const int ep = scr0 + ((static_cast<int>((sizeof(EpaPoly) + 7) / 8) + 1) & ~1);
    u = u > ep ? u : ep;
    k->kCand = scr0;  // int list of the GJK candidates
    const int ce = scr0 + (M.npairs + 1) / 2;
    u = u > ce ? u : ce;
  } else {
    k->kEpa = 0;
    k->kCand = takeu((M.npairs + 1) / 2);
  }
  int kin_end = u;
  // K^-1, and G K^-1 for the register ADMM (QPIK shapes); QPID runs the LDS path (K^-1 only)
  int kinv_end = k->oU0 + nx * nx + (k->problem == 1 ? 0 : nx * ng);
  // polish KKT: free variables + active G rows.  QPID's (<= 81) is capped at 48 —
  // typically 7 qdd + 7 tau + 7 equality rows + the few active CBF rows and free
  // slacks — which halves the per-wave LDS; a larger guess fails that polish try
  const int N = k->problem == 1 ? 48 : nx + ng;
  k->ncap = N;
  k->nbuf = N > 64 ? 128 : 64;
  int pol_end = k->oU0 + 64 + 64 + 128 + k->nbuf * 5 + N * (N + 1) / 2;
  int end = kin_end;
  if (!task_only) {
    end = end > kinv_end ? end : kinv_end;
    end = end > pol_end ? end : pol_end;
  }
  k->lds_doubles = end;
  if (end * 8 > 160 * 1024) return set_err(DRC_ERR_UNSUPPORTED, "model too large for the per-wave LDS plan");
  return DRC_OK;
}

static int make_kparams(const drc_model_impl* mm, const drc_qpik_params* p, int stages, KParams* k,
                        int problem = 0, int cf = 0) {
  const DevModel& M = mm->hm.dev;
  std::memset(k, 0, sizeof(*k));
  k->problem = problem;
  k->cf = cf;
  for (int i = 0; i < 6; ++i) {
    k->kp[i] = p->kp[i];
    k->kv[i] = p->kv[i];
  }
  k->ff = p->feedforward;
  k->alpha_cbf = p->alpha_cbf;
  k->w_reg = p->w_reg;
  k->slack_w = p->slack_w;
  k->man_min = p->man_min;
  k->dist_min = p->dist_min;
  k->t = p->t;
  k->t0 = p->t0;
  k->duration = p->duration;
  if (stages && p->frame_id == -1) {  // stage outputs without a task frame: last joint
    k->frame_joint = M.nv;
    static const double eye[12] = {1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0};
    std::memcpy(k->frame_place, eye, sizeof(k->frame_place));
  } else {
    if (p->frame_id < 0 || p->frame_id >= M.nframes)
      return set_err(DRC_ERR_UNKNOWN_LINK, "params.frame_id does not name a link of the model");
    if (M.frame_joint[p->frame_id] == 0)
      return set_err(DRC_ERR_UNKNOWN_LINK, "task frame is attached to the universe (no joint moves it)");
    k->frame_joint = M.frame_joint[p->frame_id];
    std::memcpy(k->frame_place, M.frame_place[p->frame_id], sizeof(k->frame_place));
  }
  if (p->mode < DRC_MODE_QPIK || p->mode > DRC_MODE_QPIK_CUBIC) return set_err(DRC_ERR_INVALID_ARGUMENT, "bad mode");
  k->mode = p->mode;
  k->stages = stages;
  k->s = p->solver;
  k->nv = M.nv;
  if (M.kind == 0) {
    k->narm = M.nv;
    k->c0 = 0;
    k->np = M.nv;
    k->nx = 3 * M.nv + 2;  // QP_IK.cpp:24-28
    k->na = M.nv;
  } else {
    k->narm = M.n_arm;
    k->c0 = M.mani_start;
    k->np = M.n_arm + M.n_wheel;
    k->nx = k->np;  // MoMa QP_IK.cpp:20
    k->na = k->np;
  }
  k->ng = 2 * k->narm + 2;
  if (problem == 1) {  // QPID: QP_ID.cpp:11-63 / MoMa QP_ID.cpp:11-33
    k->nx = M.kind == 0 ? 6 * M.nv + 2 : 2 * k->na;
    k->ng = 4 * k->narm + 2 + k->na;
  }
  k->m = k->nx + k->ng;
  k->rJac = 0;
  k->rMan = 6 * M.nv;
  k->rDist = k->rMan + 1 + k->narm;
  k->rXdd = k->rDist + 1 + M.nv;
  k->rQ = k->rXdd + 6;
  k->rQd = k->rQ + M.nv;
  k->rBias = k->rQd + M.nv;
  k->rMgd = k->rBias + 6;
  k->rDgd = k->rMgd + 1;
  k->rLen = problem == 1 ? k->rDgd + 1 : k->rQd;
  k->xcd_map = 0;
  if (k->nx > 64 || k->ng > 64 || k->narm > 8 || k->m > 128)
    return set_err(DRC_ERR_UNSUPPORTED, "QP larger than one wavefront's row mapping");
  if (k->s.max_iter < 1 || k->s.check_termination < 0) return set_err(DRC_ERR_INVALID_ARGUMENT, "bad solver settings");
  return plan_layout(M, k, stages != 0);
}

static int launch(const drc_model_impl* cm, const drc_qpik_params* params, int stages, int64_t B, const double* q,
                  const double* qdot, const double* xt, const double* xdt, const double* xi, const double* xdi,
                  double* out, int32_t* status, int32_t* iters, double* pose, double* jac, double* man,
                  double* dist, int32_t* pair, double* xdd, void* stream) {
  drc_model_impl* m = const_cast<drc_model_impl*>(cm);
  if (!m || !params) return set_err(DRC_ERR_INVALID_ARGUMENT, "null model/params");
  std::lock_guard<std::mutex> launch_lock(m->launch_mu);
  if (B < 0) return set_err(DRC_ERR_INVALID_ARGUMENT, "negative batch");
  if (B == 0) return DRC_OK;
  if (B > 0x7ffffff0) return set_err(DRC_ERR_INVALID_ARGUMENT, "batch too large");  // 32-bit work-queue counters
  if (!q || !qdot || !xdt) return set_err(DRC_ERR_INVALID_ARGUMENT, "q, qdot and xdot_target are required");
  if (params->mode != DRC_MODE_QPIK && !xt) return set_err(DRC_ERR_INVALID_ARGUMENT, "x_target required for QPIKStep/QPIKCubic");
  if (params->mode == DRC_MODE_QPIK_CUBIC && (!xi || !xdi))
    return set_err(DRC_ERR_INVALID_ARGUMENT, "x_init/xdot_init required for QPIKCubic");
  if (!stages && (!out || !status)) return set_err(DRC_ERR_INVALID_ARGUMENT, "qdot_out and status are required");
  KParams kt, kq;
  int rc = make_kparams(m, params, 1, &kt);
  if (rc) return rc;
  if (!stages) {
    rc = make_kparams(m, params, 0, &kq);
    if (rc) return rc;
  }
  HIP_TRY(hipSetDevice(m->device));
  // product path: per-instance task records (rLen doubles padded to whole
  // 128-B lines) in a model-owned pool; the stage API writes [field][B]
  const int64_t stride = (kt.rLen + 15) & ~int64_t(15);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  double* rec = nullptr;
  int* hard = nullptr;           // lane-stage hard list, B ints
  uint8_t* hard_flag = nullptr;  // and its per-instance flags
  StreamCtx* cx = nullptr;
  // lane-per-instance task stage (lane_task.hpp) for the compiled joint counts
  const DevModel& dm = m->hm.dev;
  // (3, auto: stage-only calls, where nothing overlaps the task stage.  The
  // default is 0: a full QPIK call is faster with the wave-per-instance
  // kernel, which shares the CUs with the QP kernels of the other sub-batches
  // (DESIGN.md), and stage and QPIK calls then see the same GJK witnesses)
  const int ls = m->lane_stage;
  const bool lane = (ls == 1 || ls == 2 || (ls == 3 && stages)) && (dm.nv == 6 || dm.nv == 7) &&
                    dm.ncand_slots <= kMaxCandSlots;
  {
    std::lock_guard<std::mutex> g(m->mu);
    if (int r = stream_ctx(m, st, &cx)) return r;
    if (!stages || lane) {
      const int64_t rec_bytes = stages ? 0 : stride * B * 8;
      if (int r = ensure_pool(cx, rec_bytes + B * 4 + B)) return r;
      if (!stages) rec = reinterpret_cast<double*>(cx->pool);
      hard = reinterpret_cast<int*>(static_cast<char*>(cx->pool) + rec_bytes);
      hard_flag = reinterpret_cast<uint8_t*>(static_cast<char*>(cx->pool) + rec_bytes + B * 4);
    }
  }
  // sub-batches of >= 4 Ki instances (a chunk of >= 16 Ki keeps the XCD-aware
  // order; smaller ones run grid-stride order): with one sub-batch the QP
  // kernel waits for the whole task kernel, with several they overlap
  // (Husky-FR3's 16 Ki batch)
  static const int64_t min_sub = getenv("DRC_MIN_SUBBATCH") ? atoll(getenv("DRC_MIN_SUBBATCH")) : 4096;
  int S = 1;
  if (!stages)
    for (int c = m->chunks; c > 1; --c)
      if (B / c >= min_sub) {
        S = c;
        break;
      }
  const bool timed = m->timing && !stages;
  std::vector<hipEvent_t> tev;
  auto mkev = [&](hipEvent_t* e) -> int {
    HIP_TRY(hipEventCreate(e));
    tev.push_back(*e);
    return DRC_OK;
  };
  {
    std::lock_guard<std::mutex> g(m->mu);
    while (static_cast<int>(cx->lanes.size()) < S) {
      hipStream_t ls;
      hipEvent_t je;
      HIP_TRY(hipStreamCreateWithFlags(&ls, hipStreamNonBlocking));
      HIP_TRY(hipEventCreateWithFlags(&je, hipEventDisableTiming));
      cx->lanes.push_back(ls);
      cx->joins.push_back(je);
    }
    while (lane && !stages && ls == 1 && static_cast<int>(cx->sides.size()) < S) {
      hipStream_t ss;
      hipEvent_t f, j;
      HIP_TRY(hipStreamCreateWithFlags(&ss, hipStreamNonBlocking));
      HIP_TRY(hipEventCreateWithFlags(&f, hipEventDisableTiming));
      HIP_TRY(hipEventCreateWithFlags(&j, hipEventDisableTiming));
      cx->sides.push_back(ss);
      cx->side_fork.push_back(f);
      cx->side_join.push_back(j);
    }
    if (!cx->fork) HIP_TRY(hipEventCreateWithFlags(&cx->fork, hipEventDisableTiming));
  }
  hipEvent_t e_start = nullptr, e_end = nullptr;
  if (timed) {
    if (int r = mkev(&e_start)) return r;
    if (int r = mkev(&e_end)) return r;
    HIP_TRY(hipEventRecord(e_start, st));
  }
  if (S > 1) HIP_TRY(hipEventRecord(cx->fork, st));
  for (int c = 0; c < S; ++c) {
    const int64_t b0 = B * c / S, b1 = B * (c + 1) / S, Bc = b1 - b0;
    hipStream_t cs = S > 1 ? cx->lanes[c] : st;
    if (S > 1) HIP_TRY(hipStreamWaitEvent(cs, cx->fork, 0));
    KParams kt_c = kt, kq_c = kq;
    kt_c.xcd_map = kq_c.xcd_map = Bc >= 16384 ? 1 : 0;
    // persistent grids (work queues hand out the instances): 2048 waves per
    // kernel and sub-batch keep every SIMD fed while each wave's prologue
    // (kernel-argument spills, written once per wave) stays a small share of
    // the HBM writes -- measured sweep in DESIGN.md; DRC_GRID_TASK / _QP
    // override for such experiments
    static const int64_t cap_t = getenv("DRC_GRID_TASK") ? atoll(getenv("DRC_GRID_TASK")) : 2048;
    static const int64_t cap_q = getenv("DRC_GRID_QP") ? atoll(getenv("DRC_GRID_QP")) : 2048;
    const int64_t gq = Bc < cap_q ? Bc : cap_q, gt = Bc < cap_t ? Bc : cap_t;
    IO io{Bc, b0, B, q, qdot, xt, xdt, xi, xdi, out, status, iters, pose, jac, man, dist, xdd, pair,
          rec ? rec + b0 * stride : nullptr, stride};
    int* qc = cx->d_queue + c * StreamCtx::kSlotInts;  // c < 16 (drc_set_concurrency)
    HIP_TRY(hipMemsetAsync(qc, 0, 17 * sizeof(int), cs));
    io.queue = qc;
    hipEvent_t e0 = nullptr, e1 = nullptr, e2 = nullptr;
    if (timed) {
      if (int r = mkev(&e0)) return r;
      if (int r = mkev(&e1)) return r;
      if (int r = mkev(&e2)) return r;
      HIP_TRY(hipEventRecord(e0, cs));
    }
    const size_t lds_t = static_cast<size_t>(kt_c.lds_doubles) * sizeof(double);
    const size_t lds_q = stages ? 0 : static_cast<size_t>(kq_c.lds_doubles) * sizeof(double);
    auto launch_task = [&](hipStream_t sm) -> int {
      hipLaunchKernelGGL(task_kernel<0>, dim3(static_cast<unsigned>(gt)), dim3(64), lds_t, sm, m->d_model, kt_c, io);
      HIP_TRY(hipGetLastError());
      return DRC_OK;
    };
    auto launch_qp = [&]() -> int {
      io.queue = qc + 8;
      const dim3 g(static_cast<unsigned>(gq)), blk(64);
      // compile-time QP shapes of the bundled robots; anything else runs the
      // runtime-sized instantiation
      // (two instances per wave: one LDS plan per lane group)
      if (kq_c.nx == 23 && kq_c.ng == 16 && kq_c.np == 7)
        hipLaunchKernelGGL((qp_kernel<Dims<23, 16, 7, true, true, kQpGroup>>), g, blk, lds_q * (64 / kQpGroup), cs,
                           m->d_model, kq_c, io);  // FR3
      else if (kq_c.nx == 20 && kq_c.ng == 14 && kq_c.np == 6)
        hipLaunchKernelGGL((qp_kernel<Dims<20, 14, 6, true, true, kQpGroup>>), g, blk, lds_q * (64 / kQpGroup), cs,
                           m->d_model, kq_c, io);  // UR5e
      else if (kq_c.nx == 9 && kq_c.ng == 16 && kq_c.np == 9)
        hipLaunchKernelGGL((qp_kernel<Dims<9, 16, 9, true, true, kQpGroup>>), g, blk, lds_q * (64 / kQpGroup), cs,
                           m->d_model, kq_c, io);  // Husky-FR3
      else if (kq_c.nx == 11 && kq_c.ng == 16 && kq_c.np == 11)
        hipLaunchKernelGGL((qp_kernel<Dims<11, 16, 11, true, true, kQpGroup>>), g, blk, lds_q * (64 / kQpGroup), cs,
                           m->d_model, kq_c, io);  // XLS-FR3
      else
        hipLaunchKernelGGL((qp_kernel<Dims<0, 0, 0>>), g, blk, lds_q, cs, m->d_model, kq_c, io);
      HIP_TRY(hipGetLastError());
      return DRC_OK;
    };
    if (!lane) {  // wave-per-instance task kernel on every instance, then the QP
      if (int r = launch_task(cs)) return r;
      if (timed) HIP_TRY(hipEventRecord(e1, cs));
      if (!stages)
        if (int r = launch_qp()) return r;
    } else {
      // lane stage for every instance; the wave-per-instance task kernel only
      // for the instances it hands back (hard list)
      io.hard_list = hard + b0;
      io.hard_n = qc + 16;
      io.hard_flag = stages ? nullptr : hard_flag + b0;
      const dim3 gl(static_cast<unsigned>((Bc + 63) / 64)), bl(64);
      if (dm.nv == 7)
        hipLaunchKernelGGL(lane_task_kernel<7>, gl, bl, 0, cs, m->d_model, kt_c, io);
      else
        hipLaunchKernelGGL(lane_task_kernel<6>, gl, bl, 0, cs, m->d_model, kt_c, io);
      HIP_TRY(hipGetLastError());
      if (timed) HIP_TRY(hipEventRecord(e1, cs));
      io.hard_mode = 1;
      if (stages || ls != 1) {  // hard task kernel, then one QP pass over every instance
        if (int r = launch_task(cs)) return r;
        io.hard_mode = 0;
        if (!stages)
          if (int r = launch_qp()) return r;
      } else {
        // hard task kernel on the side stream, overlapped with the QP of the
        // other instances; then the QP of the hard ones
        hipStream_t ss = cx->sides[c];
        HIP_TRY(hipEventRecord(cx->side_fork[c], cs));
        HIP_TRY(hipStreamWaitEvent(ss, cx->side_fork[c], 0));
        if (int r = launch_task(ss)) return r;
        HIP_TRY(hipEventRecord(cx->side_join[c], ss));
        io.hard_mode = 2;
        if (int r = launch_qp()) return r;
        HIP_TRY(hipStreamWaitEvent(cs, cx->side_join[c], 0));
        io.hard_mode = 1;
        if (int r = launch_qp()) return r;
      }
      io.hard_mode = 0;
    }
    if (timed) HIP_TRY(hipEventRecord(e2, cs));
    if (S > 1) HIP_TRY(hipEventRecord(cx->joins[c], cs));
  }
  if (S > 1)
    for (int c = 0; c < S; ++c) HIP_TRY(hipStreamWaitEvent(st, cx->joins[c], 0));
  if (timed) {
    HIP_TRY(hipEventRecord(e_end, st));
    std::lock_guard<std::mutex> g(m->mu);
    m->events.push_back(tev);
  }
  return DRC_OK;
}

// QPID pipeline for one call: dynamics launch(es) -> task kernel (QPID stage
// data into the records) -> QPID kernel; or, with stages, the task kernel
// writing the stage outputs.  Model-owned scratch holds the records and the
// dynamics ([na*na][B] M, [na][B] g, MoMa also [nv][B] joint-order g).
static int launch_qpid(const drc_model_impl* cm, const drc_qpik_params* params, int stages, int64_t B,
                       const double* q, const double* qdot, const double* xt, const double* xdt, const double* xi,
                       const double* xdi, double* qdd, double* tau, int32_t* status, int32_t* iters, double* pose,
                       double* jac, double* man, double* dist, int32_t* pair, double* xdd, double* jdot,
                       double* qpid_st, double* gdv, void* stream) {
  drc_model_impl* m = const_cast<drc_model_impl*>(cm);
  if (!m || !params) return set_err(DRC_ERR_INVALID_ARGUMENT, "null model/params");
  std::lock_guard<std::mutex> launch_lock(m->launch_mu);
  if (B < 0) return set_err(DRC_ERR_INVALID_ARGUMENT, "negative batch");
  if (B == 0) return DRC_OK;
  if (B > 0x7ffffff0) return set_err(DRC_ERR_INVALID_ARGUMENT, "batch too large");
  if (!q || !qdot || !xdt) return set_err(DRC_ERR_INVALID_ARGUMENT, "q, qdot and xdot_target are required");
  if (params->mode != DRC_MODE_QPIK && !xt) return set_err(DRC_ERR_INVALID_ARGUMENT, "x_target required for QPIDStep/QPIDCubic");
  if (params->mode == DRC_MODE_QPIK_CUBIC && (!xi || !xdi))
    return set_err(DRC_ERR_INVALID_ARGUMENT, "x_init/xdot_init required for QPIDCubic");
  if (!stages && (!qdd || !tau || !status)) return set_err(DRC_ERR_INVALID_ARGUMENT, "qddot_out, tau_out and status are required");
  KParams kt, kq;
  int rc = make_kparams(m, params, 1, &kt, 1);
  if (rc) return rc;
  if (!stages) {
    rc = make_kparams(m, params, 0, &kq, 1);
    if (rc) return rc;
  }
  const DevModel& d = m->hm.dev;
  HIP_TRY(hipSetDevice(m->device));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t stride = (kt.rLen + 15) & ~int64_t(15);
  const int na = kt.na, nv = d.nv;
  const int64_t dyn_words = stages ? 0 : (int64_t(na) * na + na + (d.kind == 1 ? nv : 0)) * B;
  double *rec = nullptr, *dM = nullptr, *dG = nullptr, *dGf = nullptr;
  StreamCtx* cx = nullptr;
  {
    std::lock_guard<std::mutex> g(m->mu);
    if (int r = stream_ctx(m, st, &cx)) return r;
    if (!stages)
      if (int r = ensure_pool(cx, (stride * B + dyn_words) * 8)) return r;
  }
  if (!stages) {
    rec = reinterpret_cast<double*>(cx->pool);
    dM = rec + stride * B;
    dG = dM + int64_t(na) * na * B;
    dGf = d.kind == 1 ? dG + int64_t(na) * B : nullptr;
    // getMassMatrix / getGravity (or the *Actuated getters) the equality rows use
    rc = launch_dynamics(m->d_model, d, d.kind == 1, B, q, qdot, dM, nullptr, dG, nullptr, nullptr, nullptr, st);
    if (!rc && d.kind == 1) rc = launch_dynamics(m->d_model, d, false, B, q, qdot, nullptr, nullptr, dGf, nullptr, nullptr, nullptr, st);
    if (rc) return set_err(DRC_ERR_HIP, std::string("dynamics launch: ") + hipGetErrorString(hipGetLastError()));
  }
  const int64_t grid = B < 8192 ? B : 8192;
  KParams kt_c = kt, kq_c = kq;
  kt_c.xcd_map = kq_c.xcd_map = B >= 16384 ? 1 : 0;
  IO io{B, 0, B, q, qdot, xt, xdt, xi, xdi, qdd, status, iters, pose, jac, man, dist, xdd, pair, rec, stride};
  io.dM = dM;
  io.dG = dG;
  io.dGf = dGf;
  io.out2 = tau;
  io.st_jdot = jdot;
  io.st_qpid = qpid_st;
  io.st_gdv = gdv;
  int* qc = cx->d_queue + StreamCtx::kQueueSlotQpid * StreamCtx::kSlotInts;
  HIP_TRY(hipMemsetAsync(qc, 0, 16 * sizeof(int), st));
  io.queue = qc;
  hipLaunchKernelGGL(task_kernel<1>, dim3(static_cast<unsigned>(grid)), dim3(64),
                     static_cast<size_t>(kt_c.lds_doubles) * sizeof(double), st, m->d_model, kt_c, io);
  HIP_TRY(hipGetLastError());
  if (!stages) {
    io.queue = qc + 8;
    const dim3 g(static_cast<unsigned>(grid)), blk(64);
    const size_t lds = static_cast<size_t>(kq_c.lds_doubles) * sizeof(double);
    if (kq_c.nx == 44 && kq_c.ng == 37 && kq_c.np == 7)  // FR3
      hipLaunchKernelGGL((qpid_kernel<Dims<44, 37, 7, false, true>>), g, blk, lds, st, m->d_model, kq_c, io);
    else if (kq_c.nx == 38 && kq_c.ng == 32 && kq_c.np == 6)  // UR5e
      hipLaunchKernelGGL((qpid_kernel<Dims<38, 32, 6, false, true>>), g, blk, lds, st, m->d_model, kq_c, io);
    else if (kq_c.nx == 18 && kq_c.ng == 39 && kq_c.np == 9)  // Husky-FR3
      hipLaunchKernelGGL((qpid_kernel<Dims<18, 39, 9, false, true>>), g, blk, lds, st, m->d_model, kq_c, io);
    else if (kq_c.nx == 22 && kq_c.ng == 41 && kq_c.np == 11)  // XLS-FR3
      hipLaunchKernelGGL((qpid_kernel<Dims<22, 41, 11, false, true>>), g, blk, lds, st, m->d_model, kq_c, io);
    else
      hipLaunchKernelGGL((qpid_kernel<Dims<0, 0, 0>>), g, blk, lds, st, m->d_model, kq_c, io);
    HIP_TRY(hipGetLastError());
  }
  return DRC_OK;
}

// Closed-form controllers: [dynamics (OSF: M^-1, g)] -> task_kernel<2>.
static int launch_closed_form(const drc_model_impl* cm, const drc_qpik_params* params, int cf, int64_t B,
                              const double* q, const double* qdot, const double* xt, const double* xdt,
                              const double* xi, const double* xdi, const double* nullv, double* out, void* stream) {
  drc_model_impl* m = const_cast<drc_model_impl*>(cm);
  if (!m || !params) return set_err(DRC_ERR_INVALID_ARGUMENT, "null model/params");
  std::lock_guard<std::mutex> launch_lock(m->launch_mu);
  if (m->hm.dev.kind != 0) return set_err(DRC_ERR_INVALID_ARGUMENT, "CLIK / OSF are Manipulator::RobotController entries");
  if (B < 0) return set_err(DRC_ERR_INVALID_ARGUMENT, "negative batch");
  if (B == 0) return DRC_OK;
  if (B > 0x7ffffff0) return set_err(DRC_ERR_INVALID_ARGUMENT, "batch too large");
  if (!q || !qdot || !xdt || !out) return set_err(DRC_ERR_INVALID_ARGUMENT, "q, qdot, xdot_target and out are required");
  if (cf == 1 && params->mode == DRC_MODE_QPIK) return set_err(DRC_ERR_INVALID_ARGUMENT, "CLIK has Step and Cubic forms only");
  if (params->mode != DRC_MODE_QPIK && !xt) return set_err(DRC_ERR_INVALID_ARGUMENT, "x_target required");
  if (params->mode == DRC_MODE_QPIK_CUBIC && (!xi || !xdi)) return set_err(DRC_ERR_INVALID_ARGUMENT, "x_init/xdot_init required");
  drc_qpik_params pp = *params;
  for (int i = 0; i < 6; ++i) pp.kv[i] = cf == 1 ? 0.0 : params->kv[i];  // CLIK: Kp e + xdot_target (:168)
  pp.feedforward = cf == 1 ? 1.0 : 0.0;                                 // OSF: Kp e + Kv edot (:243)
  KParams kt;
  int rc = make_kparams(m, &pp, 1, &kt, 2, cf);
  if (rc) return rc;
  const DevModel& d = m->hm.dev;
  HIP_TRY(hipSetDevice(m->device));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  double *dMi = nullptr, *dG = nullptr;
  StreamCtx* cx = nullptr;
  {
    std::lock_guard<std::mutex> g(m->mu);
    if (int r = stream_ctx(m, st, &cx)) return r;
    if (cf == 2) {
      if (int r = ensure_pool(cx, (int64_t(d.nv) * d.nv + d.nv) * B * 8)) return r;
      if (cx->dyn_list_cap < B + 1) {
        if (cx->dyn_list) HIP_TRY(hipFree(cx->dyn_list));
        cx->dyn_list = nullptr;
        cx->dyn_list_cap = 0;
        HIP_TRY(hipMalloc(&cx->dyn_list, (B + 1) * sizeof(int)));
        cx->dyn_list_cap = B + 1;
      }
    }
  }
  if (cf == 2) {  // getMassMatrixInv (PinvCOD(M)) and getGravity (robot_data.cpp:111-118)
    dMi = reinterpret_cast<double*>(cx->pool);
    dG = dMi + int64_t(d.nv) * d.nv * B;
    rc = launch_dynamics(m->d_model, d, false, B, q, qdot, nullptr, dMi, dG, nullptr, nullptr, cx->dyn_list, st);
    if (rc) return set_err(DRC_ERR_HIP, std::string("dynamics launch: ") + hipGetErrorString(hipGetLastError()));
  }
  const int64_t grid = B < 8192 ? B : 8192;
  kt.xcd_map = B >= 16384 ? 1 : 0;
  IO io{B, 0, B, q, qdot, xt, xdt, xi, xdi, out, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
        nullptr, nullptr, 0};
  io.dM = dMi;
  io.dG = dG;
  io.cf_null = nullv;
  io.queue = cx->d_queue + StreamCtx::kQueueSlotCf * StreamCtx::kSlotInts;
  HIP_TRY(hipMemsetAsync(io.queue, 0, 8 * sizeof(int), st));
  hipLaunchKernelGGL(task_kernel<2>, dim3(static_cast<unsigned>(grid)), dim3(64),
                     static_cast<size_t>(kt.lds_doubles) * sizeof(double), st, m->d_model, kt, io);
  HIP_TRY(hipGetLastError());
  return DRC_OK;
}

}  // namespace drc_amd

using drc_amd::drc_model_impl;
struct drc_model : drc_model_impl {};

extern "C" {

const char* drc_error_string(int code) {
  switch (code) {
    case DRC_OK: return "ok";
    case DRC_ERR_INVALID_ARGUMENT: return "invalid argument";
    case DRC_ERR_FILE: return "file does not exist";
    case DRC_ERR_PARSE: return "parse error";
    case DRC_ERR_UNSUPPORTED: return "unsupported model";
    case DRC_ERR_UNKNOWN_LINK: return "link name not found in URDF";
    case DRC_ERR_HIP: return "HIP runtime error";
    case DRC_ERR_SIZE_MISMATCH: return "size mismatch";
    default: return "unknown error";
  }
}
const char* drc_last_error(void) { return drc_amd::g_last_error.c_str(); }

int drc_debug_kernel_timing(drc_model* m, int enable) {
  if (!m) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null model");
  m->timing = enable != 0;
  return DRC_OK;
}

int drc_debug_kernel_times(drc_model* m, double* wall_ms, double* task_ms, double* qp_ms, int* calls) {
  if (!m || !wall_ms || !task_ms || !qp_ms || !calls) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null argument");
  std::lock_guard<std::mutex> g(m->mu);
  double tw = 0, t0 = 0, t1 = 0;
  for (auto& ev : m->events) {  // {start, end, [task start, task end, qp end] per chunk}
    float a = 0;
    if (hipEventSynchronize(ev[1]) != hipSuccess) return drc_amd::set_err(DRC_ERR_HIP, "hipEventSynchronize");
    if (hipEventElapsedTime(&a, ev[0], ev[1]) != hipSuccess) return drc_amd::set_err(DRC_ERR_HIP, "hipEventElapsedTime");
    tw += a;
    for (size_t c = 2; c + 2 < ev.size(); c += 3) {
      float x = 0, y = 0;
      if (hipEventElapsedTime(&x, ev[c], ev[c + 1]) != hipSuccess ||
          hipEventElapsedTime(&y, ev[c + 1], ev[c + 2]) != hipSuccess)
        return drc_amd::set_err(DRC_ERR_HIP, "hipEventElapsedTime");
      t0 += x;
      t1 += y;
    }
  }
  *calls = static_cast<int>(m->events.size());
  for (auto& ev : m->events)
    for (hipEvent_t e : ev) (void)hipEventDestroy(e);
  m->events.clear();
  *wall_ms = tw;
  *task_ms = t0;
  *qp_ms = t1;
  return DRC_OK;
}

int drc_set_concurrency(drc_model* m, int chunks) {
  if (!m || chunks < 1 || chunks > 16) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "chunks must be 1..16");
  std::lock_guard<std::mutex> g(m->mu);
  m->chunks = chunks;
  return DRC_OK;
}

int drc_debug_lane_stage(drc_model* m, int enable) {
  if (!m) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null model");
  std::lock_guard<std::mutex> g(m->launch_mu);
  m->lane_stage = enable < 0 ? 0 : (enable > 3 ? 3 : enable);
  return DRC_OK;
}

#ifdef DRC_PHASE_TIMING
// diagnostic build only: accumulated per-phase s_memtime cycles (32 slots)
int drc_debug_phase_cycles(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(drc_amd::g_phase_cycles), sizeof(unsigned long long) * 64) != hipSuccess)
    return DRC_ERR_HIP;
  if (reset) {
    unsigned long long z[64] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(drc_amd::g_phase_cycles), z, sizeof(z)) != hipSuccess) return DRC_ERR_HIP;
  }
  return DRC_OK;
}
#endif

int drc_model_create_manipulator(const char* urdf, const char* srdf, const char* packages, int device,
                                 drc_model** out) {
  (void)packages;  // collision meshes are not supported: primitives only
  if (!urdf || !out) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null argument");
  auto* m = new drc_model();
  std::string err;
  int rc = drc_amd::build_model_from_urdf(urdf, srdf ? srdf : "", &m->hm, &err);
  if (rc) {
    delete m;
    return drc_amd::set_err(rc, err);
  }
  m->hm.dev.kind = 0;
  m->device = device;
  rc = drc_amd::upload(m);
  if (rc) {
    delete m;
    return rc;
  }
  *out = m;
  return DRC_OK;
}

int drc_model_create_mobile_manipulator(const drc_kinematic_param* param, const drc_joint_index* ji,
                                        const drc_actuator_index* ai, const char* urdf, const char* srdf,
                                        const char* packages, int device, drc_model** out) {
  (void)packages;
  if (!param || !ji || !ai || !urdf || !out) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null argument");
  auto* m = new drc_model();
  std::string err;
  int rc = drc_amd::build_model_from_urdf(urdf, srdf ? srdf : "", &m->hm, &err);
  if (rc) {
    delete m;
    return drc_amd::set_err(rc, err);
  }
  drc_amd::DevModel& d = m->hm.dev;
  int W = 0;
  rc = drc_amd::mobile_fk_jacobian(*param, &W, d.J_mobile);
  if (rc) {
    delete m;
    return rc;
  }
  d.drive = param->type;
  d.wheel_radius = param->wheel_radius;
  d.wheel_offset = param->wheel_offset;
  for (int i = 0; i < drc_amd::kMaxWheels / 2; ++i)
    for (int k = 0; k < 2; ++k) d.caster_pos[i][k] = param->base2wheel_positions[i][k];
  if (param->type == DRC_DRIVE_CASTER && !(param->wheel_offset != 0)) {
    delete m;
    return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "caster drive needs a nonzero wheel_offset");
  }
  // MobileManipulator::RobotData ctor (mobile_manipulator/robot_data.cpp:18-25)
  const int virtual_dof = 3;
  d.kind = 1;
  d.n_wheel = W;
  d.n_arm = d.nv - (virtual_dof + W);  // every joint 1-DoF, no extra joints
  d.virtual_start = ji->virtual_start;
  d.mani_start = ji->mani_start;
  d.mobi_start = ji->mobi_start;
  d.act_mani_start = ai->mani_start;
  d.act_mobi_start = ai->mobi_start;
  d.dyn_origin = ji->virtual_start + 3;  // the base (yaw joint) origin: keeps spatial moments small
  if (d.n_arm < 1 || d.n_arm > 8 || ji->virtual_start + 3 > d.nv || ji->mani_start + d.n_arm > d.nv ||
      ji->mobi_start + W > d.nv || ai->mani_start + d.n_arm > d.n_arm + W || ai->mobi_start + W > d.n_arm + W) {
    delete m;
    return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "JointIndex/ActuatorIndex inconsistent with the URDF dof");
  }
  m->kparam = *param;
  m->jidx = *ji;
  m->aidx = *ai;
  m->device = device;
  rc = drc_amd::upload(m);
  if (rc) {
    delete m;
    return rc;
  }
  *out = m;
  return DRC_OK;
}

void drc_model_destroy(drc_model* m) {
  if (!m) return;
  (void)hipSetDevice(m->device);
  for (auto& c : m->ctxs) drc_amd::free_ctx(c.get());
  if (m->d_model) (void)hipFree(m->d_model);
  if (m->hstream) (void)hipStreamSynchronize(m->hstream), (void)hipStreamDestroy(m->hstream);
  if (m->stage) (void)hipFree(m->stage);
  for (auto& ev : m->events)
    for (hipEvent_t e : ev) (void)hipEventDestroy(e);
  delete m;
}

int drc_model_info(const drc_model* m, int* dof, int* act, int* mani, int* mobi, int* ngeom, int* npairs) {
  if (!m) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null model");
  const drc_amd::DevModel& d = m->hm.dev;
  if (dof) *dof = d.nv;
  if (act) *act = d.kind == 1 ? d.n_arm + d.n_wheel : d.nv;
  if (mani) *mani = d.kind == 1 ? d.n_arm : d.nv;
  if (mobi) *mobi = d.kind == 1 ? d.n_wheel : 0;
  if (ngeom) *ngeom = d.ngeom;
  if (npairs) *npairs = d.npairs;
  return DRC_OK;
}

int drc_model_limits(const drc_model* m, double* q_lb, double* q_ub, double* qd_lb, double* qd_ub) {
  if (!m) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null model");
  const drc_amd::DevModel& d = m->hm.dev;
  for (int i = 0; i < d.nv; ++i) {
    if (q_lb) q_lb[i] = d.lower[i];
    if (q_ub) q_ub[i] = d.upper[i];
    if (qd_lb) qd_lb[i] = -d.vel[i];
    if (qd_ub) qd_ub[i] = d.vel[i];
  }
  return DRC_OK;
}

int drc_model_find_frame(const drc_model* m, const char* name, int* id) {
  if (!m || !name || !id) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null argument");
  const auto& names = m->hm.frame_names;
  for (size_t i = 0; i < names.size(); ++i)
    if (names[i] == name) {
      *id = static_cast<int>(i);
      return DRC_OK;
    }
  *id = -1;
  return drc_amd::set_err(DRC_ERR_UNKNOWN_LINK, std::string("Link name ") + name + " not found in URDF.");
}

int drc_model_mobile_fk_jacobian(const drc_model* m, double* J) {
  if (!m || !J) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null argument");
  const drc_amd::DevModel& d = m->hm.dev;
  if (d.kind != 1) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "not a mobile manipulator");
  if (d.drive == drc_amd::kDriveCaster)
    return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT,
                            "caster drive: J_mobile depends on the steer angles (drc_mobile_fk_jacobian)");
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < d.n_wheel; ++c) J[r * d.n_wheel + c] = d.J_mobile[r][c];
  return DRC_OK;
}

int drc_mobile_fk_jacobian(const drc_kinematic_param* p, const double* wheel_pos, double* J, int* n_wheels) {
  if (!p || !J || !n_wheels) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null argument");
  if (p->type == DRC_DRIVE_CASTER && !wheel_pos)
    return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "caster drive: wheel positions required");
  double Jm[3][drc_amd::kMaxWheels];
  int W = 0;
  if (int rc = drc_amd::mobile_fk_jacobian(*p, &W, Jm, wheel_pos)) return rc;
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < W; ++c) J[r * W + c] = Jm[r][c];
  *n_wheels = W;
  return DRC_OK;
}

int drc_mobile_ik_jacobian(const drc_kinematic_param* p, const double* wheel_pos, double* J, int* n_wheels) {
  if (!p || !J || !n_wheels) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null argument");
  if (p->type == DRC_DRIVE_CASTER && !wheel_pos)
    return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "caster drive: wheel positions required");
  return drc_amd::mobile_ik_jacobian(*p, wheel_pos, J, n_wheels);
}

int drc_default_qpik_params(const drc_model* m, int exact, drc_qpik_params* p) {
  if (!m || !p) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null argument");
  std::memset(p, 0, sizeof(*p));
  const bool moma = m->hm.dev.kind == 1;
  for (int i = 0; i < 6; ++i) {
    p->kp[i] = moma ? 400 : 100;  // robot_controller.cpp:12 ; MoMa :15
    p->kv[i] = moma ? 0 : 20;     // MoMa QPIKStep: Kp*e + xdot_target (:177)
  }
  p->feedforward = moma ? 1.0 : 0.0;
  p->alpha_cbf = 50;
  p->w_reg = moma ? 0.01 : 1.0;
  p->slack_w = 1000;
  p->man_min = 0.01;
  p->dist_min = 0.05;
  p->mode = DRC_MODE_QPIK_STEP;
  p->frame_id = -1;
  drc_solver_settings& s = p->solver;
  s.rho = 0.1;
  s.sigma = 1e-6;
  s.alpha = 1.6;
  s.eps_abs = 1e-3;
  s.eps_rel = 1e-3;
  s.eps_prim_inf = 1e-4;
  s.max_iter = 4000;
  s.check_termination = 25;
  s.scaling = 10;
  s.adaptive_rho = 1;
  s.adaptive_rho_interval = 25;
  s.adaptive_rho_tolerance = 5;
  s.polish = exact ? 1 : 0;
  s.polish_refine_iter = 3;
  s.delta = 1e-6;
  s.exact = exact ? 1 : 0;
  s.eps_exact = 1e-9;
  s.eps_fallback = 1e-7;
  return DRC_OK;
}

int drc_qpik_batch(const drc_model* m, const drc_qpik_params* p, int64_t B, const double* q, const double* qdot,
                   const double* xt, const double* xdt, const double* xi, const double* xdi, double* out,
                   int32_t* status, int32_t* iters, void* stream) {
  return drc_amd::launch(m, p, 0, B, q, qdot, xt, xdt, xi, xdi, out, status, iters, nullptr, nullptr, nullptr,
                         nullptr, nullptr, nullptr, stream);
}

int drc_qpik_stages_batch(const drc_model* m, const drc_qpik_params* p, int64_t B, const double* q,
                          const double* qdot, const double* xt, const double* xdt, const double* xi,
                          const double* xdi, double* pose, double* jac, double* man, double* dist, int32_t* pair,
                          double* xdd, void* stream) {
  return drc_amd::launch(m, p, 1, B, q, qdot, xt, xdt, xi, xdi, nullptr, nullptr, nullptr, pose, jac, man, dist,
                         pair, xdd, stream);
}


// ---- QPID -------------------------------------------------
int drc_default_qpid_params(const drc_model* m, int exact, drc_qpik_params* p) {
  int rc = drc_default_qpik_params(m, exact, p);
  if (rc) return rc;
  const bool moma = m->hm.dev.kind == 1;
  for (int i = 0; i < 6; ++i) {
    p->kp[i] = moma ? 400 : 100;  // robot_controller.cpp:12-13; MoMa :15-16
    p->kv[i] = moma ? 40 : 20;    // QPIDStep: Kp e + Kv (xdot_target - xdot) (:347; MoMa :230)
  }
  p->feedforward = 0;
  p->w_reg = 0;  // QP_ID.cpp:102: the regulariser is commented out
  // P is singular on null(J); OSQP's polish delta 1e-6 cannot certify at
  // eps_exact there, so parity mode regularises the polish with 1e-10
  if (exact) p->solver.delta = 1e-10;
  return DRC_OK;
}

int drc_qpid_batch(const drc_model* m, const drc_qpik_params* p, int64_t B, const double* q, const double* qdot,
                   const double* xt, const double* xdt, const double* xi, const double* xdi, double* qddot_out,
                   double* tau_out, int32_t* status, int32_t* iters, void* stream) {
  return drc_amd::launch_qpid(m, p, 0, B, q, qdot, xt, xdt, xi, xdi, qddot_out, tau_out, status, iters, nullptr,
                              nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, stream);
}

int drc_qpid_stages_batch(const drc_model* m, const drc_qpik_params* p, int64_t B, const double* q,
                          const double* qdot, const double* xt, const double* xdt, const double* xi,
                          const double* xdi, double* pose, double* jac, double* man, double* dist, int32_t* pair,
                          double* xddot_des, double* jdot, double* qpid_terms, double* graddot, void* stream) {
  return drc_amd::launch_qpid(m, p, 1, B, q, qdot, xt, xdt, xi, xdi, nullptr, nullptr, nullptr, nullptr, pose, jac,
                              man, dist, pair, xddot_des, jdot, qpid_terms, graddot, stream);
}

int drc_qpid_stages_host(drc_model* m, const drc_qpik_params* p, int64_t B, const double* q, const double* qdot,
                         const double* xt, const double* xdt, const double* xi, const double* xdi, double* pose,
                         double* jac, double* man, double* dist, int32_t* pair, double* xddot_des, double* jdot,
                         double* qpid_terms, double* graddot) {
  using drc_amd::set_err;
  if (!m || !p) return set_err(DRC_ERR_INVALID_ARGUMENT, "null model/params");
  if (B <= 0) return B == 0 ? DRC_OK : set_err(DRC_ERR_INVALID_ARGUMENT, "negative batch");
  const drc_amd::DevModel& d = m->hm.dev;
  const int64_t n = d.nv, na = d.kind == 1 ? d.n_arm : n;
  std::lock_guard<std::mutex> lk(m->host_mu);
  HIP_TRY(hipSetDevice(m->device));
  const double* src[6] = {q, qdot, xt, xdt, xi, xdi};
  const int64_t rin[6] = {n, n, 12, 6, 12, 6};
  double* outs[8] = {pose, jac, man, dist, xddot_des, jdot, qpid_terms, graddot};
  const int64_t rout[8] = {12, 6 * n, 1 + na, 1 + n, 6, 6 * n, 8, na + n};
  int64_t words = (B + 1) / 2;
  for (int i = 0; i < 6; ++i) words += src[i] ? rin[i] * B : 0;
  for (int i = 0; i < 8; ++i) words += outs[i] ? rout[i] * B : 0;
  if (m->stage_bytes < words * 8) {
    if (m->stage) (void)hipFree(m->stage);
    m->stage = nullptr;
    m->stage_bytes = 0;
    HIP_TRY(hipMalloc(&m->stage, words * 8));
    m->stage_bytes = words * 8;
  }
  if (!m->hstream) HIP_TRY(hipStreamCreateWithFlags(&m->hstream, hipStreamNonBlocking));
  double* dp = reinterpret_cast<double*>(m->stage);
  const double* din[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  for (int i = 0; i < 6; ++i)
    if (src[i]) {
      HIP_TRY(hipMemcpyAsync(dp, src[i], rin[i] * B * 8, hipMemcpyHostToDevice, m->hstream));
      din[i] = dp;
      dp += rin[i] * B;
    }
  double* dout[8] = {nullptr};
  for (int i = 0; i < 8; ++i)
    if (outs[i]) {
      dout[i] = dp;
      dp += rout[i] * B;
    }
  int32_t* dpair = pair ? reinterpret_cast<int32_t*>(dp) : nullptr;
  int rc = drc_qpid_stages_batch(m, p, B, din[0], din[1], din[2], din[3], din[4], din[5], dout[0], dout[1], dout[2],
                                 dout[3], dpair, dout[4], dout[5], dout[6], dout[7], m->hstream);
  if (rc) return rc;
  for (int i = 0; i < 8; ++i)
    if (outs[i]) HIP_TRY(hipMemcpyAsync(outs[i], dout[i], rout[i] * B * 8, hipMemcpyDeviceToHost, m->hstream));
  if (pair) HIP_TRY(hipMemcpyAsync(pair, dpair, B * 4, hipMemcpyDeviceToHost, m->hstream));
  HIP_TRY(hipStreamSynchronize(m->hstream));
  return DRC_OK;
}

// ---- host-buffer entry points (synchronous; staged through device memory) --
namespace {
struct HostIO {
  const double* src[6];  // q, qdot, xt, xdt, xi, xdi
  int64_t rows[6];
};
}  // namespace

static int host_call(drc_model* m, const drc_qpik_params* p, int stages, int64_t B, const HostIO& in,
                     double** outs, const int64_t* out_rows, int nouts, int32_t** iouts, int niouts) {
  if (!m || !p) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null model/params");
  if (B <= 0) return B == 0 ? DRC_OK : drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "negative batch");
  std::lock_guard<std::mutex> g(m->host_mu);
  if (hipSetDevice(m->device) != hipSuccess) return drc_amd::set_err(DRC_ERR_HIP, "hipSetDevice");
  int64_t words = 0;
  for (int i = 0; i < 6; ++i) words += in.src[i] ? in.rows[i] * B : 0;
  for (int i = 0; i < nouts; ++i) words += outs[i] ? out_rows[i] * B : 0;
  words += niouts * ((B + 1) / 2);
  const int64_t bytes = words * 8;
  if (m->stage_bytes < bytes) {
    if (m->stage) (void)hipFree(m->stage);
    m->stage = nullptr;
    m->stage_bytes = 0;
    if (hipMalloc(&m->stage, bytes) != hipSuccess) return drc_amd::set_err(DRC_ERR_HIP, "hipMalloc (staging)");
    m->stage_bytes = bytes;
  }
  if (!m->hstream && hipStreamCreateWithFlags(&m->hstream, hipStreamNonBlocking) != hipSuccess)
    return drc_amd::set_err(DRC_ERR_HIP, "hipStreamCreate");
  double* d = reinterpret_cast<double*>(m->stage);
  const double* din[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  for (int i = 0; i < 6; ++i)
    if (in.src[i]) {
      if (hipMemcpyAsync(d, in.src[i], in.rows[i] * B * 8, hipMemcpyHostToDevice, m->hstream) != hipSuccess)
        return drc_amd::set_err(DRC_ERR_HIP, "hipMemcpyAsync H2D");
      din[i] = d;
      d += in.rows[i] * B;
    }
  double* dout[8] = {nullptr};
  for (int i = 0; i < nouts; ++i)
    if (outs[i]) {
      dout[i] = d;
      d += out_rows[i] * B;
    }
  int32_t* diout[2] = {nullptr, nullptr};
  for (int i = 0; i < niouts; ++i)
    if (iouts[i]) {
      diout[i] = reinterpret_cast<int32_t*>(d);
      d += (B + 1) / 2;
    }
  int rc;
  if (!stages)
    rc = drc_amd::launch(m, p, 0, B, din[0], din[1], din[2], din[3], din[4], din[5], dout[0], diout[0], diout[1],
                         nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, m->hstream);
  else
    rc = drc_amd::launch(m, p, 1, B, din[0], din[1], din[2], din[3], din[4], din[5], nullptr, nullptr, nullptr,
                         dout[0], dout[1], dout[2], dout[3], diout[0], dout[4], m->hstream);
  if (rc) return rc;
  for (int i = 0; i < nouts; ++i)
    if (outs[i] && hipMemcpyAsync(outs[i], dout[i], out_rows[i] * B * 8, hipMemcpyDeviceToHost, m->hstream) != hipSuccess)
      return drc_amd::set_err(DRC_ERR_HIP, "hipMemcpyAsync D2H");
  for (int i = 0; i < niouts; ++i)
    if (iouts[i] && hipMemcpyAsync(iouts[i], diout[i], B * 4, hipMemcpyDeviceToHost, m->hstream) != hipSuccess)
      return drc_amd::set_err(DRC_ERR_HIP, "hipMemcpyAsync D2H");
  if (hipStreamSynchronize(m->hstream) != hipSuccess) return drc_amd::set_err(DRC_ERR_HIP, "hipStreamSynchronize");
  return DRC_OK;
}

int drc_qpik_host(drc_model* m, const drc_qpik_params* p, int64_t B, const double* q, const double* qdot,
                  const double* xt, const double* xdt, const double* xi, const double* xdi, double* out,
                  int32_t* status, int32_t* iters) {
  if (!m) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null model");
  if (!out || !status) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "qdot_out and status are required");
  const int64_t n = m->hm.dev.nv, a = m->hm.dev.kind == 1 ? m->hm.dev.n_arm + m->hm.dev.n_wheel : n;
  HostIO in{{q, qdot, xt, xdt, xi, xdi}, {n, n, 12, 6, 12, 6}};
  double* outs[1] = {out};
  const int64_t rows[1] = {a};
  int32_t* iouts[2] = {status, iters};
  return host_call(m, p, 0, B, in, outs, rows, 1, iouts, 2);
}

int drc_qpik_stages_host(drc_model* m, const drc_qpik_params* p, int64_t B, const double* q, const double* qdot,
                         const double* xt, const double* xdt, const double* xi, const double* xdi, double* pose,
                         double* jac, double* man, double* dist, int32_t* pair, double* xdd) {
  if (!m) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null model");
  const int64_t n = m->hm.dev.nv, na = m->hm.dev.kind == 1 ? m->hm.dev.n_arm : n;
  HostIO in{{q, qdot, xt, xdt, xi, xdi}, {n, n, 12, 6, 12, 6}};
  double* outs[5] = {pose, jac, man, dist, xdd};
  const int64_t rows[5] = {12, 6 * n, 1 + na, 1 + n, 6};
  int32_t* iouts[1] = {pair};
  return host_call(m, p, 1, B, in, outs, rows, 5, iouts, 1);
}


// ---- closed-form controllers ------------------------------
int drc_clik_batch(const drc_model* m, const drc_qpik_params* p, int64_t B, const double* q, const double* qdot,
                   const double* xt, const double* xdt, const double* xi, const double* xdi, const double* null_qdot,
                   double* qdot_out, void* stream) {
  return drc_amd::launch_closed_form(m, p, 1, B, q, qdot, xt, xdt, xi, xdi, null_qdot, qdot_out, stream);
}

int drc_osf_batch(const drc_model* m, const drc_qpik_params* p, int64_t B, const double* q, const double* qdot,
                  const double* xt, const double* xdt, const double* xi, const double* xdi, const double* null_torque,
                  double* tau_out, void* stream) {
  return drc_amd::launch_closed_form(m, p, 2, B, q, qdot, xt, xdt, xi, xdi, null_torque, tau_out, stream);
}

int drc_closed_form_host(drc_model* m, const drc_qpik_params* p, int kind, int64_t B, const double* q,
                         const double* qdot, const double* xt, const double* xdt, const double* xi, const double* xdi,
                         const double* nullv, double* out) {
  using drc_amd::set_err;
  if (!m || !p) return set_err(DRC_ERR_INVALID_ARGUMENT, "null model/params");
  if (kind != 1 && kind != 2) return set_err(DRC_ERR_INVALID_ARGUMENT, "kind must be 1 (CLIK) or 2 (OSF)");
  if (B <= 0) return B == 0 ? DRC_OK : set_err(DRC_ERR_INVALID_ARGUMENT, "negative batch");
  if (!out) return set_err(DRC_ERR_INVALID_ARGUMENT, "out is required");
  const int64_t n = m->hm.dev.nv;
  std::lock_guard<std::mutex> lk(m->host_mu);
  HIP_TRY(hipSetDevice(m->device));
  const double* src[7] = {q, qdot, xt, xdt, xi, xdi, nullv};
  const int64_t rows[7] = {n, n, 12, 6, 12, 6, n};
  int64_t words = n * B;
  for (int i = 0; i < 7; ++i) words += src[i] ? rows[i] * B : 0;
  if (m->stage_bytes < words * 8) {
    if (m->stage) (void)hipFree(m->stage);
    m->stage = nullptr;
    m->stage_bytes = 0;
    HIP_TRY(hipMalloc(&m->stage, words * 8));
    m->stage_bytes = words * 8;
  }
  if (!m->hstream) HIP_TRY(hipStreamCreateWithFlags(&m->hstream, hipStreamNonBlocking));
  double* dp = reinterpret_cast<double*>(m->stage);
  const double* din[7] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  for (int i = 0; i < 7; ++i)
    if (src[i]) {
      HIP_TRY(hipMemcpyAsync(dp, src[i], rows[i] * B * 8, hipMemcpyHostToDevice, m->hstream));
      din[i] = dp;
      dp += rows[i] * B;
    }
  int rc = drc_amd::launch_closed_form(m, p, kind, B, din[0], din[1], din[2], din[3], din[4], din[5], din[6], dp,
                                       m->hstream);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(out, dp, n * B * 8, hipMemcpyDeviceToHost, m->hstream));
  HIP_TRY(hipStreamSynchronize(m->hstream));
  return DRC_OK;
}

int drc_qpid_host(drc_model* m, const drc_qpik_params* p, int64_t B, const double* q, const double* qdot,
                  const double* xt, const double* xdt, const double* xi, const double* xdi, double* qdd, double* tau,
                  int32_t* status, int32_t* iters) {
  using drc_amd::set_err;
  if (!m || !p) return set_err(DRC_ERR_INVALID_ARGUMENT, "null model/params");
  if (B <= 0) return B == 0 ? DRC_OK : set_err(DRC_ERR_INVALID_ARGUMENT, "negative batch");
  if (!qdd || !tau || !status) return set_err(DRC_ERR_INVALID_ARGUMENT, "qddot_out, tau_out and status are required");
  const drc_amd::DevModel& d = m->hm.dev;
  const int64_t n = d.nv, na = d.kind == 1 ? d.n_arm + d.n_wheel : n;
  std::lock_guard<std::mutex> lk(m->host_mu);
  HIP_TRY(hipSetDevice(m->device));
  const double* src[6] = {q, qdot, xt, xdt, xi, xdi};
  const int64_t rows[6] = {n, n, 12, 6, 12, 6};
  int64_t words = 2 * na * B + B;  // outputs + status/iters
  for (int i = 0; i < 6; ++i) words += src[i] ? rows[i] * B : 0;
  if (m->stage_bytes < words * 8) {
    if (m->stage) (void)hipFree(m->stage);
    m->stage = nullptr;
    m->stage_bytes = 0;
    HIP_TRY(hipMalloc(&m->stage, words * 8));
    m->stage_bytes = words * 8;
  }
  if (!m->hstream) HIP_TRY(hipStreamCreateWithFlags(&m->hstream, hipStreamNonBlocking));
  double* dp = reinterpret_cast<double*>(m->stage);
  const double* din[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  for (int i = 0; i < 6; ++i)
    if (src[i]) {
      HIP_TRY(hipMemcpyAsync(dp, src[i], rows[i] * B * 8, hipMemcpyHostToDevice, m->hstream));
      din[i] = dp;
      dp += rows[i] * B;
    }
  double* dqdd = dp;
  double* dtau = dp + na * B;
  int32_t* dst = reinterpret_cast<int32_t*>(dp + 2 * na * B);
  int32_t* dit = iters ? dst + B : nullptr;
  int rc = drc_qpid_batch(m, p, B, din[0], din[1], din[2], din[3], din[4], din[5], dqdd, dtau, dst, dit, m->hstream);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(qdd, dqdd, na * B * 8, hipMemcpyDeviceToHost, m->hstream));
  HIP_TRY(hipMemcpyAsync(tau, dtau, na * B * 8, hipMemcpyDeviceToHost, m->hstream));
  HIP_TRY(hipMemcpyAsync(status, dst, B * 4, hipMemcpyDeviceToHost, m->hstream));
  if (iters) HIP_TRY(hipMemcpyAsync(iters, dit, B * 4, hipMemcpyDeviceToHost, m->hstream));
  HIP_TRY(hipStreamSynchronize(m->hstream));
  return DRC_OK;
}

// ---- joint-space dynamics ------------------------------
int drc_dynamics_batch(drc_model* m, int actuated, int64_t B, const double* q, const double* qdot, double* M,
                       double* M_inv, double* g, double* nle, double* c, void* stream) {
  using drc_amd::set_err;
  if (!m) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null model");
  if (B < 0) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "negative batch");
  if (B == 0) return DRC_OK;
  if (!q) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "q is required");
  if ((nle || c) && !qdot) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "qdot is required for nle / c");
  if (actuated && m->hm.dev.kind != 1)
    return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "actuated dynamics need a mobile-manipulator model");
  if (B > 0x7ffffff0) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "batch too large");
  HIP_TRY(hipSetDevice(m->device));
  std::lock_guard<std::mutex> launch_lock(m->launch_mu);
  int* list = nullptr;
  if (M_inv) {
    std::lock_guard<std::mutex> lk(m->mu);
    drc_amd::StreamCtx* cx = nullptr;
    if (int r = drc_amd::stream_ctx(m, reinterpret_cast<hipStream_t>(stream), &cx)) return r;
    if (cx->dyn_list_cap < B + 1) {
      if (cx->dyn_list) HIP_TRY(hipFree(cx->dyn_list));
      cx->dyn_list = nullptr;
      cx->dyn_list_cap = 0;
      HIP_TRY(hipMalloc(&cx->dyn_list, (B + 1) * sizeof(int)));
      cx->dyn_list_cap = B + 1;
    }
    list = cx->dyn_list;
  }
  const int rc = drc_amd::launch_dynamics(m->d_model, m->hm.dev, actuated != 0, B, q, qdot, M, M_inv, g, nle, c,
                                          list, reinterpret_cast<hipStream_t>(stream));
  if (rc == 1) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "batch too large");
  if (rc) return drc_amd::set_err(DRC_ERR_HIP, std::string("dynamics launch: ") + hipGetErrorString(hipGetLastError()));
  return DRC_OK;
}

int drc_dynamics_host(drc_model* m, int actuated, int64_t B, const double* q, const double* qdot, double* M,
                      double* M_inv, double* g, double* nle, double* c) {
  using drc_amd::set_err;
  if (!m) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "null model");
  if (B <= 0) return B == 0 ? DRC_OK : drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "negative batch");
  if (!q) return drc_amd::set_err(DRC_ERR_INVALID_ARGUMENT, "q is required");
  const drc_amd::DevModel& d = m->hm.dev;
  const int64_t n = d.nv, no = actuated ? d.n_arm + d.n_wheel : n;
  std::lock_guard<std::mutex> lk(m->host_mu);
  HIP_TRY(hipSetDevice(m->device));
  double* outs[5] = {M, M_inv, g, nle, c};
  const int64_t rows[5] = {no * no, no * no, no, no, no};
  int64_t words = (qdot ? 2 : 1) * n * B;
  for (int i = 0; i < 5; ++i) words += outs[i] ? rows[i] * B : 0;
  if (m->stage_bytes < words * 8) {
    if (m->stage) (void)hipFree(m->stage);
    m->stage = nullptr;
    m->stage_bytes = 0;
    HIP_TRY(hipMalloc(&m->stage, words * 8));
    m->stage_bytes = words * 8;
  }
  if (!m->hstream) HIP_TRY(hipStreamCreateWithFlags(&m->hstream, hipStreamNonBlocking));
  double* dp = reinterpret_cast<double*>(m->stage);
  double* dq = dp;
  dp += n * B;
  HIP_TRY(hipMemcpyAsync(dq, q, n * B * 8, hipMemcpyHostToDevice, m->hstream));
  double* dqd = nullptr;
  if (qdot) {
    dqd = dp;
    dp += n * B;
    HIP_TRY(hipMemcpyAsync(dqd, qdot, n * B * 8, hipMemcpyHostToDevice, m->hstream));
  }
  double* dout[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  for (int i = 0; i < 5; ++i)
    if (outs[i]) {
      dout[i] = dp;
      dp += rows[i] * B;
    }
  int rc = drc_dynamics_batch(m, actuated, B, dq, dqd, dout[0], dout[1], dout[2], dout[3], dout[4], m->hstream);
  if (rc) return rc;
  for (int i = 0; i < 5; ++i)
    if (outs[i]) HIP_TRY(hipMemcpyAsync(outs[i], dout[i], rows[i] * B * 8, hipMemcpyDeviceToHost, m->hstream));
  HIP_TRY(hipStreamSynchronize(m->hstream));
  return DRC_OK;
}

// ---- joint torque step ---------------------------------
int drc_joint_torque_step_batch(drc_model* m, int64_t B, const double* q, const double* qdot, const double* q_target,
                                const double* qdot_target, const double* qddot_target, double dt, const double* kp,
                                const double* kv, double* tau, void* stream) {
  using drc_amd::set_err;
  if (!m) return set_err(DRC_ERR_INVALID_ARGUMENT, "null model");
  if (B < 0) return set_err(DRC_ERR_INVALID_ARGUMENT, "negative batch");
  if (B == 0) return DRC_OK;
  if (!q || !tau) return set_err(DRC_ERR_INVALID_ARGUMENT, "q and tau are required");
  if (!qddot_target && (!qdot || !qdot_target))
    return set_err(DRC_ERR_INVALID_ARGUMENT, "qdot and qdot_target are required without qddot_target");
  const drc_amd::DevModel& d = m->hm.dev;
  const int nb = d.kind == 1 ? d.n_arm : d.nv;
  double kpv[drc_amd::kMaxJoints], kvv[drc_amd::kMaxJoints];
  for (int i = 0; i < nb; ++i) {  // robot_controller.cpp:14-15 (MoMa :17-18): 400 / 40
    kpv[i] = kp ? kp[i] : 400.0;
    kvv[i] = kv ? kv[i] : 40.0;
  }
  HIP_TRY(hipSetDevice(m->device));
  const int rc = drc_amd::launch_torque_step(m->d_model, d, B, q, qdot, q_target, qdot_target, qddot_target, dt, kpv,
                                             kvv, tau, reinterpret_cast<hipStream_t>(stream));
  if (rc == 1) return set_err(DRC_ERR_INVALID_ARGUMENT, "batch too large");
  if (rc) return set_err(DRC_ERR_HIP, std::string("torque step launch: ") + hipGetErrorString(hipGetLastError()));
  return DRC_OK;
}

int drc_joint_torque_step_host(drc_model* m, int64_t B, const double* q, const double* qdot, const double* q_target,
                               const double* qdot_target, const double* qddot_target, double dt, const double* kp,
                               const double* kv, double* tau) {
  using drc_amd::set_err;
  if (!m) return set_err(DRC_ERR_INVALID_ARGUMENT, "null model");
  if (B <= 0) return B == 0 ? DRC_OK : set_err(DRC_ERR_INVALID_ARGUMENT, "negative batch");
  if (!q || !tau) return set_err(DRC_ERR_INVALID_ARGUMENT, "q and tau are required");
  const drc_amd::DevModel& d = m->hm.dev;
  const int64_t n = d.nv, nb = d.kind == 1 ? d.n_arm : d.nv;
  std::lock_guard<std::mutex> lk(m->host_mu);
  HIP_TRY(hipSetDevice(m->device));
  const double* src[5] = {q, qdot, q_target, qdot_target, qddot_target};
  const int64_t rows[5] = {n, n, nb, nb, nb};
  int64_t words = nb * B;
  for (int i = 0; i < 5; ++i) words += src[i] ? rows[i] * B : 0;
  if (m->stage_bytes < words * 8) {
    if (m->stage) (void)hipFree(m->stage);
    m->stage = nullptr;
    m->stage_bytes = 0;
    HIP_TRY(hipMalloc(&m->stage, words * 8));
    m->stage_bytes = words * 8;
  }
  if (!m->hstream) HIP_TRY(hipStreamCreateWithFlags(&m->hstream, hipStreamNonBlocking));
  double* dp = reinterpret_cast<double*>(m->stage);
  const double* din[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  for (int i = 0; i < 5; ++i)
    if (src[i]) {
      HIP_TRY(hipMemcpyAsync(dp, src[i], rows[i] * B * 8, hipMemcpyHostToDevice, m->hstream));
      din[i] = dp;
      dp += rows[i] * B;
    }
  int rc = drc_joint_torque_step_batch(m, B, din[0], din[1], din[2], din[3], din[4], dt, kp, kv, dp, m->hstream);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(tau, dp, nb * B * 8, hipMemcpyDeviceToHost, m->hstream));
  HIP_TRY(hipStreamSynchronize(m->hstream));
  return DRC_OK;
}

}  // extern "C"

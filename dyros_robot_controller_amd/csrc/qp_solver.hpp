// OSQP ADMM restated for one wavefront per instance:
// residuals, K factorisations (LDS and register forms, the Schur complement of
// the slack block), adaptive rho, the certified polish (register / range-space
// / LDS EQPs), primal infeasibility, and the QP kernel's phases (assembly,
// Ruiz scaling, the ADMM loop).  Included by qp_kernel.hip and qpid_kernel.hip.
#pragma once

#include "kernel_common.hpp"

namespace drc_amd {

// ------------------------------------------------------------------------
// OSQP residuals (lane-parallel): fills SC_* slots.  x, z, y in LDS (scaled)
// ------------------------------------------------------------------------
// PRE: the caller already holds this lane's A x entry (bound row: ab x, G row:
// G x, formed by the same expressions in the same order -- the polish's
// candidate), so the products are not formed twice
template <class QD, bool UNSCALED = true, bool PRE = false>
__device__ __forceinline__ void residuals(const KParams& kp, double* S, const double* x, const double* z, const double* y,
                          double eps_abs, double eps_rel, double axb_pre = 0.0, double axg_pre = 0.0) {
  using GL = Grp<QD::gs>;
  // UNSCALED = false (the polish's certification) skips the unscaled norms
  // that only adaptive rho reads (SC_PRIS .. SC_NQ keep the ADMM values)
  const int l = GL::lane(), nx = DNX, ng = DNG, np = DNP;
  const double *P = S + kp.oP, *G = S + kp.oG, *q = S + kp.oQ, *ab = S + kp.oAB, *Di = S + kp.oDi, *Ei = S + kp.oEi;
  double pr = 0, prs = 0, nAx = 0, nz = 0, nAxs = 0, nzs = 0;
  double dr = 0, drs = 0, nPx = 0, nAty = 0, nq = 0, nPxs = 0, nAtys = 0, nqs = 0;
  if (l < nx) {  // bound row l and variable l
    const int lx = l < nx ? l : 0;
    double ax = PRE ? axb_pre : ab[lx] * x[lx], r = ax - z[lx];
    prs = fabs(r);
    pr = fabs(r * Ei[lx]);
    nAx = fabs(ax * Ei[lx]);
    nz = fabs(z[lx] * Ei[lx]);
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
    dr = fabs(rr * Di[lx]);
    nPx = fabs(px * Di[lx]);
    nAty = fabs(aty * Di[lx]);
    nq = fabs(q[lx] * Di[lx]);
    nPxs = fabs(px);
    nAtys = fabs(aty);
    nqs = fabs(q[lx]);
  }
  if (l < ng) {
    const int lg = l < ng ? l : 0;
    double ax = 0;
    if constexpr (PRE) {
      ax = axg_pre;
    } else {
#pragma unroll
      for (int j = 0; j < nx; ++j) ax += G[lg * nx + j] * x[j];
    }
    int row = nx + lg;
    double r = ax - z[row];
    prs = fmax(prs, fabs(r));
    pr = fmax(pr, fabs(r * Ei[row]));
    nAx = fmax(nAx, fabs(ax * Ei[row]));
    nz = fmax(nz, fabs(z[row] * Ei[row]));
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
  const double ci = S[kp.oSc + SC_CINV];
  if (l == 0) {
    double* sc = S + kp.oSc;
    sc[SC_PRI] = pr;
    sc[SC_DUA] = dr * ci;
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
    sc[SC_EPSD] = eps_abs + eps_rel * fmax(fmax(nPx, nAty), nq) * ci;
  }
  wsync();
}

// OSQP keeps D^-1, E^-1 and c^-1 beside the Ruiz scaling (scaling.c) and its
// residuals and tolerances multiply by them (vec_scaled_norm_inf): one division
// per entry once per instance, none per residual evaluation.  The oracle's
// qp_scale / qp_residuals do the same.
template <class QD>
__device__ __forceinline__ void scaling_inverses(const KParams& kp, double* S) {
  using GL = Grp<QD::gs>;
  const int l = GL::lane(), nx = DNX, m = DM;
  const double *D = S + kp.oD, *E = S + kp.oE;
  double *Di = S + kp.oDi, *Ei = S + kp.oEi;
  for (int i = l; i < nx; i += GL::size) Di[i] = 1.0 / D[i];
  for (int i = l; i < m; i += GL::size) Ei[i] = 1.0 / E[i];
  if (l == 0) S[kp.oSc + SC_CINV] = 1.0 / S[kp.oSc + SC_C];
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
  // the pivot row reaches the lanes through LDS on 64-lane waves (the pivot
  // lane writes it, every lane reads the same addresses: no VALU broadcasts)
  lds_double* bc = (lds_double*)(S + kp.oBc);
  constexpr bool kLds = QD::gs == 64;
  static_for<NP>([&](auto K) {
    constexpr int k = decltype(K)::value;
    if (l == k) {
      const double pv = 1.0 / Sr[k];
      Sr[k] = 1.0;
#pragma unroll
      for (int j = 0; j < NP; ++j) Sr[j] *= pv;
      if constexpr (kLds) {
#pragma unroll
        for (int j = 0; j < NP; ++j) bc[j] = Sr[j];
      }
    }
    if constexpr (kLds) asm volatile("" ::: "memory");
    const double f = Sr[k];
    if (l != k) Sr[k] = 0.0;
    static_for<NP>([&](auto J) {
      constexpr int j = decltype(J)::value;
      double rkj;
      if constexpr (kLds) rkj = bc[j];
      else rkj = GL::template bcastc<k>(Sr[j]);
      if (l != k) Sr[j] -= f * rkj;
    });
    if constexpr (kLds) asm volatile("" ::: "memory");
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
    viol = fabs(s * S[kp.oDi + l]);
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
#ifndef DRC_POLISH_ATTR
#define DRC_POLISH_ATTR __forceinline__
#endif
template <class QD>
__device__ DRC_POLISH_ATTR bool polish(const KParams& kp, double* S, bool strict);

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
  bool early_failed = false, conv = false;
  // One polish call site (inlined once): round 0 is the early polish (exact
  // mode, fewer than kPolishMaxEarly failed attempts), round 1 forms the ADMM
  // residuals and, at convergence, polishes when round 0 did not try
  for (int round = 0; round < 2; ++round) {
    bool try_polish;
    if (round == 0) {
      try_polish = check && kp.s.exact && sc[SC_PFAIL] < kPolishMaxEarly;
    } else {
      residuals<QD>(kp, S, x, z, y, kp.s.eps_abs, kp.s.eps_rel);
      CK_T(32);
      CK_N(33);
      if (!check) break;
      conv = sc[SC_PRI] < sc[SC_EPSP] && sc[SC_DUA] < sc[SC_EPSD];
#ifdef DRC_QP_DEBUG
      if (GL::lane() == 0 && it <= 200)
        printf("it %d rho %.4g pri %.3e/%.3e dua %.3e/%.3e x3 %.6f\n", it, sc[SC_RHO], sc[SC_PRI], sc[SC_EPSP],
               sc[SC_DUA], sc[SC_EPSD], x[3] * S[kp.oD + 3]);
#endif
      if (!conv) break;
      if (!kp.s.exact) {
        *status = DRC_STATUS_SOLVED;
        return 2;
      }
      try_polish = !early_failed && sc[SC_PFAIL] < kPolishMaxTotal;
    }
    if (try_polish) {
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
      if (round == 0) {
        early_failed = true;
        reload = 1;
      }
    }
  }
  if (check) {
    if (conv) {
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
  PH_STAMP(er_t0);
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
    // (QPIK with slacks: the q-dot columns and the row's own slack column,
    // as polish's G-row products)
    const bool slk = kp.problem == 0 && NP < NX;
#pragma unroll
    for (int c = 0; c < NX; ++c) {
      if (c >= NP && slk) break;
      r -= G[lg * NX + c] * xx[c];
    }
    if (slk) r -= G[lg * NX + NP + lg] * xx[NP + lg];
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
    // (entries j >= N are never read: every loop below stops at N)
#pragma unroll
    for (int j = 0; j < NK; ++j) {
      if (j >= N) break;
      double v = 0.0;
      if (j < nF) {
        const int fj = __builtin_ctzll(fm);
        fm &= fm - 1;
        if (hf) v = (fi < NP && fj < NP) ? P[fi * NP + fj] : 0.0;
        else if (hr) v = G[gi * NX + fj];
      } else {
        const int gj = __builtin_ctzll(rm);
        rm &= rm - 1;
        if (hf) v = G[gj * NX + fi];
      }
      K0[j] = v;
      Ki[j] = v + (j == l ? (hf ? kp.s.delta : (hr ? -kp.s.delta : 0.0)) : 0.0);
    }
  }
  PH_SINCE(52, er_t0);
  PH_STAMP(er_t1);
  // Gauss-Jordan inverse of the regularised KKT.  The pivot row and the
  // vectors of the products below reach every lane through LDS (the pivot
  // lane / the owners write, every lane reads the same addresses): no VALU
  // broadcast instructions, same values, same products (64-lane waves; a
  // lane group of 32 keeps the register broadcasts)
  lds_double* bc = (lds_double*)(S + kp.oBc);
  constexpr bool kLds = QD::gs == 64;
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    if (k >= N) break;
    const double piv = GL::bcast(Ki[k], k);
    if (piv == 0.0) return false;  // uniform
    if (l == k) {
      const double p = 1.0 / Ki[k];
      Ki[k] = 1.0;
#pragma unroll
      for (int j = 0; j < NK; ++j) {
        if (j >= N) break;
        Ki[j] *= p;
      }
      if constexpr (kLds) {
#pragma unroll
        for (int j = 0; j < NK; ++j) {
          if (j >= N) break;
          bc[j] = Ki[j];
        }
      }
    }
    if constexpr (kLds) asm volatile("" ::: "memory");
    const double f = Ki[k];
    if (l != k) Ki[k] = 0.0;
#pragma unroll
    for (int j = 0; j < NK; ++j) {
      if (j >= N) break;
      double rkj;
      if constexpr (kLds) rkj = bc[j];
      else rkj = GL::bcast(Ki[j], k);
      if (l != k) Ki[j] -= f * rkj;
    }
    if constexpr (kLds) asm volatile("" ::: "memory");
  }
  auto apply = [&](const double (&A)[NK], double v) {  // row l of A times the vector held by lanes 0..N-1
    if constexpr (kLds) {
      if (l < N) bc[l] = v;
      asm volatile("" ::: "memory");
    }
    double s0 = 0, s1 = 0;
#pragma unroll
    for (int j = 0; j < NK; ++j) {
      if (j >= N) break;
      double vj;
      if constexpr (kLds) vj = bc[j];
      else vj = GL::bcast(v, j);
      if (j & 1) s1 += A[j] * vj;
      else s0 += A[j] * vj;
    }
    if constexpr (kLds) asm volatile("" ::: "memory");
    return s0 + s1;
  };
  PH_SINCE(53, er_t1);
  PH_STAMP(er_t2);
  double sol = apply(Ki, rhs);
  for (int it = 0; it < kp.s.polish_refine_iter; ++it) {
    const double res = rhs - apply(K0, sol);
    sol += apply(Ki, res);
  }
  PH_SINCE(54, er_t2);
  PH_STAMP(er_t3);
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
  PH_SINCE(55, er_t3);
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
  PH_STAMP(eq_t0);
  PH_ADD(41, 1);
  PH_ADD(42, N);
  if constexpr (QD::gs < 64) {  // two instances per wave: register EQP only (ncap <= kEqpRegCap)
    if (N > kEqpRegCap) return false;
  }
  if constexpr (QD::nx > 0 && QD::nx == QD::np && QD::gs == 64) {  // whole-body shapes: range-space form
    if (kp.oHi >= 0 && nF == QD::nx && nR <= kEqpRegCap) {
      const bool ok_ = eqp_range<QD>(kp, S, actg, xx, yy, rowMask, nR);
      PH_SINCE(40, eq_t0);
      return ok_;
    }
    if (kp.oHi >= 0) return false;  // no LDS LDL^T region in this plan (never reached: no variable bounds)
  }
  if constexpr (QD::nx > 0) {
    if (N <= kEqpRegCap) {
      const bool ok_ = eqp_regs<QD>(kp, S, actb, actg, xx, yy, freeMask, rowMask, nF, nR);
      PH_SINCE(40, eq_t0);
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
  PH_SINCE(40, eq_t0);
  return true;
}

// OSQP polish (polish.c) restated.  strict == 0: OSQP's single attempt and
// acceptance rule.  strict != 0 (parity mode): accept only a KKT-certified
// point (residuals at eps_exact, dual signs matching the active bounds); on a
// wrong ADMM active-set guess continue with a primal active-set method
// (Nocedal & Wright Alg. 16.3) from the first feasible polished point.  Same
// decisions, in the same row order, as oracle/drc_oracle.c:qp_polish.
constexpr int kPolishFeasAttempts = 6, kPolishAsIters = 24, kPolishJacobiSweeps = 3;
constexpr double kPolishSlackTol = 0.3;
template <class QD>
__device__ DRC_POLISH_ATTR bool polish(const KParams& kp, double* S, bool strict) {
  using GL = Grp<QD::gs>;
  const int l = GL::lane(), nx = DNX, ng = DNG, np = DNP, m = DM;
  const double *G = S + kp.oG, *ab = S + kp.oAB, *lo = S + kp.oL, *up = S + kp.oU, *E = S + kp.oE;
  double *x = S + kp.oX, *z = S + kp.oZ, *y = S + kp.oY;
  int ob = 0, og = 0;  // OSQP's guess
  if (l < nx) ob = (z[l] - lo[l] < -y[l]) ? -1 : ((up[l] - z[l] < y[l]) ? 1 : 0);
  if (l < ng) {
    int r = nx + l;
    og = (z[r] - lo[r] < -y[r]) ? -1 : ((up[r] - z[r] < y[r]) ? 1 : 0);
  }
  int actb = ob, actg = og;
  // QPIK parity mode: the bound rows of the q-dot (the variables with cost
  // curvature, P_ll > 0) take the sides at which kPolishJacobiSweeps projected
  // Jacobi sweeps on their box -- the G-row duals of the ADMM iterate held
  // fixed -- clamp them.  At the first check the ADMM iterate has usually not
  // reached the velocity bounds the optimum saturates: OSQP's rule above then
  // misses about two rows per FR3 instance (12 % right first time, 2.7 EQP
  // solves per polish); with this guess 77 % and 1.55, with the slack rule
  // below 81 % and 1.45 (tools/polish_census.py).  Same rules and summation
  // order as oracle/drc_oracle.c:polish_guess_jacobi / polish_guess_slack.
  PH_STAMP(pj_t0);
  if (strict && kp.problem == 0 && np < nx) {
    const double *P = S + kp.oP, *qv = S + kp.oQ;
    lds_double* bc = (lds_double*)(S + kp.oBc);
    const int lp = l < np ? l : 0, lx = l < nx ? l : 0;
    // one pass over this lane's G column: the q-dot lanes' Jacobi constant
    // c = q_l + sum_i g_il y_i (two partial sums) and the slack lanes' single
    // row (gv, yr, cnt; used below)
    double c0 = qv[lx], c1 = 0.0, gv = 0.0, yr = 0.0;
    int cnt = 0;
#pragma unroll
    for (int i = 0; i < ng; ++i) {
      const double g = G[i * nx + lx], yi = y[nx + i];
      if (i & 1) c1 += g * yi;
      else c0 += g * yi;
      if (g != 0.0) {
        gv = g;
        yr = yi;
        ++cnt;
      }
    }
    const double c = c0 + c1;
    double xv = x[lp];
    const double ipll = 1.0 / P[lp * np + lp], a = ab[lp], bl = lo[lp], bu = up[lp], xl = bl / a, xu = bu / a;
    int side = 0;
    for (int sw = 0; sw < kPolishJacobiSweeps; ++sw) {
      lds_double* xb = bc + (sw & 1) * np;  // alternate halves: no exchange point between the reads and the next writes
      if (l < np) xb[l] = xv;
      wsync();
      double g = c;
#pragma unroll
      for (int k = 0; k < np; ++k) g += P[lp * np + k] * xb[k];
      const double v = xv - g * ipll, av = a * v;
      side = av <= bl ? -1 : (av >= bu ? 1 : 0);
      xv = side < 0 ? xl : (side > 0 ? xu : v);
    }
    wsync();
    if (l < np) actb = side;
    // slack lanes (no curvature, a linear cost, in exactly one G row r): the
    // bound stays active only while its multiplier from stationarity with the
    // ADMM dual of row r, -(q_l + g_rl y_r) / ab_l, is below
    // -kPolishSlackTol |q_l| / ab_l (oracle: polish_guess_slack)
    if (l >= np && l < nx) {
      const double ql = qv[lx], a = ab[lx];
      if (cnt == 1 && ql != 0.0) {
        const double yb = -(ql + gv * yr) / a;
        actb = yb < -kPolishSlackTol * fabs(ql) / a ? -1 : 0;
      }
    }
  }
  PH_SINCE(50, pj_t0);
  // when the polish from this guess fails and it differs from OSQP's, the
  // same polish runs once more from OSQP's guess (oracle: qp_polish): a guess
  // whose ADMM duals settle slowly can fail at every check, and a UR5e bench
  // instance then ran 1 400 ADMM iterations instead of one extra attempt
  // (QPIK: the retry also differs in the infeasible phase's drop rule, below,
  // so it runs whenever the first pass fails)
  const bool alt = strict && (kp.problem == 0 || GL::any(actb != ob || actg != og));
  double* U = S + kp.oU0;
  double* xx = U + 64;       // [nx]
  double* yy = U + 128;      // [m] (<= 128)
  double* zz = S + kp.oT2;   // z candidate
  double* xc = S + kp.oXT;   // feasible iterate of the active-set phase
  double* sc = S + kp.oSc;
  const double pr0 = sc[SC_PRI], dr0 = sc[SC_DUA];
  const int iters = strict ? kPolishFeasAttempts + kPolishAsIters : 1;
  // QPIK with slacks: G row r is nonzero only in the q-dot columns and its own
  // slack column np + r (qp_assemble), so the G-row products below take those
  // np + 1 terms, in the same order (the skipped terms are exact zeros)
  const bool slk = kp.problem == 0 && np < nx;
  for (int pass = 0; pass < 2; ++pass) {
  if (pass == 1) {
    if (!alt) break;
    actb = ob;
    actg = og;
  }
  bool have_feas = false;
  for (int it = 0; it < iters; ++it) {
    PH_STAMP(pd_t0);
    {
      // a working-set G row with no weight on the free variables depends on
      // the fixed bounds alone and makes the reduced KKT singular (its
      // solution then hangs on rounding noise, e.g. the structurally-zero
      // manipulability gradient of the first/last joint).  When the fixed
      // values already satisfy it strictly it is not active: drop it (the
      // oracle's qp_polish applies the same rule)
      // (the fixed values b_j / ab_j, one division per variable lane, go to xx
      // -- where the EQP puts them too -- instead of a division per term)
      const unsigned long long fixed = GL::ballot(l < nx && actb != 0);
      if (l < nx) xx[l] = actb == 0 ? 0.0 : (actb < 0 ? lo[l] : up[l]) / ab[l];
      wsync();
      if (l < ng && actg != 0) {
        const int lg = l < ng ? l : 0, row = nx + lg;
        double sf = 0, sa = 0, act = 0;
#pragma unroll
        for (int j = 0; j < nx; ++j) {
          if (j >= np && slk) break;  // (the slack column below)
          const double g = G[lg * nx + j];
          sa = fmax(sa, fabs(g));
          if (!((fixed >> j) & 1ull)) sf = fmax(sf, fabs(g));
          else act += g * xx[j];
        }
        if (slk) {
          const int j = np + lg;
          const double g = G[lg * nx + j];
          sa = fmax(sa, fabs(g));
          if (!((fixed >> j) & 1ull)) sf = fmax(sf, fabs(g));
          else act += g * xx[j];
        }
        const double b = actg < 0 ? lo[row] : up[row], slack = actg < 0 ? act - b : b - act;
        if (sf <= 1e-12 * sa && slack > 1e-12 * (fabs(act) + fabs(b))) actg = 0;
      }
    }
    PH_SINCE(51, pd_t0);
    if (!eqp<QD>(kp, S, actb, actg, xx, yy)) break;
    PH_STAMP(pr_t0);
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
            if (j >= np && slk) break;
            axc += G[lg * nx + j] * xc[j];
            ap += G[lg * nx + j] * (xx[j] - xc[j]);
          }
          if (slk) {
            const int j = np + lg;
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
          PH_SINCE(56, pr_t0);
          continue;
        }
      }
    }
    PH_SINCE(56, pr_t0);
    PH_STAMP(pc_t0);
    // candidate point: z = clamp(A x), residuals, certification
    double axb = 0, axg = 0;
    if (l < nx) {
      axb = ab[l] * xx[l];
      zz[l] = fmin(fmax(axb, lo[l]), up[l]);
    }
    if (l < ng) {
      const int lg = l < ng ? l : 0;
#pragma unroll
      for (int j = 0; j < nx; ++j) {
        if (j >= np && slk) break;
        axg += G[lg * nx + j] * xx[j];
      }
      if (slk) axg += G[lg * nx + np + lg] * xx[np + lg];
      zz[nx + lg] = fmin(fmax(axg, lo[nx + lg]), up[nx + lg]);
    }
    wsync();
    PH_SINCE(57, pc_t0);
    PH_STAMP(rs_t0);
    residuals<QD, false, true>(kp, S, xx, zz, yy, kp.s.eps_exact, kp.s.eps_exact, axb, axg);
    PH_SINCE(43, rs_t0);
    PH_STAMP(pk_t0);
    const double pr1 = sc[SC_PRI], dr1 = sc[SC_DUA], epsp = sc[SC_EPSP], epsd = sc[SC_EPSD], ci = sc[SC_CINV];
    const double* Ei = S + kp.oEi;
    bool ok = (pr1 < pr0 && dr1 < dr0) || (pr1 < pr0 && dr0 < 1e-10) || (dr1 < dr0 && pr0 < 1e-10);
    double wv = 0;
    int worst = 0x7fffffff;
    bool feasible = pr1 <= epsp;
    if (strict) {
      ok = feasible && dr1 <= epsd;
      if (l < nx && actb != 0 && lo[l] != up[l]) {
        double yi = E[l] * yy[l] * ci, viol = actb < 0 ? yi - epsd : -yi - epsd;
        if (viol > wv) { wv = viol; worst = l; }
      }
      if (l < ng && actg != 0 && lo[nx + l] != up[nx + l]) {
        double yi = E[nx + l] * yy[nx + l] * ci, viol = actg < 0 ? yi - epsd : -yi - epsd;
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
      PH_SINCE(58, pk_t0);
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
        const double vlo = (lo[l] - axb) * Ei[l] - epsp, vhi = (axb - up[l]) * Ei[l] - epsp;
        if (vlo > 0 || vhi > 0) sb = vhi > vlo ? 1 : -1;
        if (vlo > av) { av = vlo; add = l * 4 + 0; }
        if (vhi > av) { av = vhi; add = l * 4 + 2; }
      }
      if (l < ng && actg == 0) {
        const int row = nx + l;
        const double vlo = (lo[row] - axg) * Ei[row] - epsp, vhi = (axg - up[row]) * Ei[row] - epsp;
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
        // ... and, in the first pass, the active row with the worst
        // wrong-signed multiplier leaves in the same step (a wrong row of the
        // first guess otherwise stays until the set is feasible; FR3
        // stragglers never got there and ran 60 ADMM iterations).  The retry
        // pass adds only: an infeasible EQP's multipliers can also point at a
        // right row (oracle: qp_polish_from).  It is an active row, so never
        // one just added
        if (sb) actb = sb;
        if (sg) actg = sg;
        if (pass == 0 && worst != 0x7fffffff) {
          if (worst < nx) { if (l == worst) actb = 0; }
          else if (l == worst - nx) actg = 0;
        }
      } else {
        GL::argmax(av, add);
        const int row = add >> 2, sd = (add & 3) - 1;
        if (row < nx) { if (l == row) actb = sd; }
        else if (l == row - nx) actg = sd;
      }
    }
    PH_SINCE(58, pk_t0);
  }
  }  // pass
  if (l == 0) {  // restore the ADMM residuals for the caller
    sc[SC_PRI] = pr0;
    sc[SC_DUA] = dr0;
  }
  wsync();
  return false;
}


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
  PH_STAMP(as_t0);
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
  PH_SINCE(44, as_t0);
  const double bestd = S[kp.oSc + SC_DIST];
  // ---------------- QP assembly (QP_IK.cpp:69-131 / MoMa :59-128) --------
  const int nx = DNX, ng = DNG, np = DNP, m = DM;
  (void)m;
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
  (void)x, (void)z, (void)y, (void)dy;  // the runtime-sized (LDS) path only
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

// max |a_i| as a balanced tree: fmax of non-NaN values is exact and
// order-free, so this is bit for bit the serial chain's result at a depth of
// log2 N instead of N dependent fmax (the Ruiz passes' critical path)
template <int N>
__device__ __forceinline__ double absmax_tree(const double (&a)[N]) {
  double t[N];
#pragma unroll
  for (int i = 0; i < N; ++i) t[i] = fabs(a[i]);
#pragma unroll
  for (int w = 1; w < N; w *= 2)
#pragma unroll
    for (int i = 0; i + w < N; i += 2 * w) t[i] = fmax(t[i], t[i + w]);
  return t[0];
}

// Register form of qp_scale for compile-time shapes: lane l holds row l of P
// (= column l: P is symmetric bit for bit), column l and row l of G; the
// Ruiz factors move by v_readlane.  Same operations in the same order as
// qp_scale (bit-identical results); P, G, q, D, E written back at the end.
template <class QD>
__device__ __forceinline__ int qp_scale_regs(const KParams& kp, double* S) {
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
    PH_ADD(49, 1);  // Ruiz passes
    // (the inputs are finite -- checked above -- so every fmax below is exact)
    const double sgc = absmax_tree(Gcol);
    const double s = fmax(fabs(abl), hp ? fmax(absmax_tree(Prow), sgc) : sgc);
    const double Dt = 1.0 / sqrt(clampf(s));
    const double Et = 1.0 / sqrt(clampf(fabs(abl)));
    const double sg = absmax_tree(Grow);
    const double EtG = 1.0 / sqrt(clampf(sg));
    // every factor of this pass exactly 1 (the fixed-point pass, usually the
    // second): the products below would multiply by 1.0, an identity, so
    // they are skipped -- bit for bit the same matrices, without the pass's
    // 23 broadcasts
    const bool unit = GL::all((!hx || (Dt == 1.0 && Et == 1.0)) && (!hg || EtG == 1.0));
    if (!unit) {
      // the broadcast factors are used as they arrive (not gathered into
      // per-lane arrays: 39 doubles more would not fit the QP kernel's 168-VGPR
      // budget and spilled); same products in the same order
      // (64-lane waves: the factors reach the lanes through LDS -- each lane
      // writes its own, every lane reads them all -- instead of NX + NG VALU
      // broadcasts)
      constexpr bool kLds = QD::gs == 64;
      lds_double* wb = (lds_double*)(S + kp.oBc);  // NX + NG doubles (plan_layout)
      if constexpr (kLds) {
        if (hx) wb[l] = Dt;
        if (hg) wb[NX + l] = EtG;
        asm volatile("" ::: "memory");
      }
      static_for<NX>([&](auto C) {
        constexpr int c = decltype(C)::value;
        double dc;
        if constexpr (kLds) dc = wb[c];
        else dc = GL::template bcastc<c>(Dt);
        if constexpr (c < NP) {
          if (hp) Prow[c] *= Dt * dc;
        }
        if (hg) Grow[c] *= EtG * dc;
      });
      static_for<NG>([&](auto I) {
        constexpr int i = decltype(I)::value;
        double ei;
        if constexpr (kLds) ei = wb[NX + i];
        else ei = GL::template bcastc<i>(EtG);
        if (hx) Gcol[i] *= ei * Dt;
      });
      if constexpr (kLds) asm volatile("" ::: "memory");
      if (hx) {
        abl *= Et * Dt;
        ql *= Dt;
        Dl *= Dt;
        El *= Et;
      }
      if (hg) EGl *= EtG;
    }
    // cost scaling: mean column norm of P vs |q|_inf
    double cn = 0, qn = 0;
    if (hp) cn = absmax_tree(Prow);
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
    if (ct == 1.0 && unit) break;
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

// Ruiz passes with one role per lane (64-lane waves, NX + NG <= 64): lane c < NX
// holds column c of [P; G] (P's part only for c < NP), lane NX + r holds row r
// of G, so a lane forms one absolute maximum, one factor F (D~ on column lanes,
// E~ on row lanes) and one set of products instead of all three.  Same
// operands, same products in the same order as qp_scale_regs (bit-identical);
// the column copy of G is dropped at the end, as there.
template <class QD>
__device__ __forceinline__ int qp_scale_roles(const KParams& kp, double* S) {
  using GL = Grp<64>;
  constexpr int NX = QD::nx, NG = QD::ng, NP = QD::np, M = NX + NG;
  constexpr int KV = NP + NG > NX ? NP + NG : NX;
  static_assert(M <= 64, "one lane per column and per G row");
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
  const bool col = l < NX, row = l >= NX && l < M, hp = l < NP;
  const int lc = col ? l : 0, lp = hp ? l : 0, r = row ? l - NX : 0;
  double V[KV];
#pragma unroll
  for (int k = 0; k < KV; ++k) {
    double vc = 0.0, vr = 0.0;
    if (k < NP) vc = hp ? P[lp * NP + k] : 0.0;
    else if (k - NP < NG) vc = G[(k - NP) * NX + lc];
    if (k < NX) vr = G[r * NX + k];
    V[k] = col ? vc : (row ? vr : 0.0);
  }
  double abl = ab[lc], ql = qq[lc], Dl = 1.0, El = 1.0, EGl = 1.0, cs = 1.0;
  auto clampf = [](double v) { return v < kMinScaling ? 1.0 : (v > kMaxScaling ? kMaxScaling : v); };
  lds_double* wb = (lds_double*)(S + kp.oBc);  // NX + NG doubles (plan_layout)
  for (int it = 0; it < kp.s.scaling; ++it) {
    PH_ADD(49, 1);  // Ruiz passes
    const double mx = absmax_tree(V);
    const double F = 1.0 / sqrt(clampf(col ? fmax(fabs(abl), mx) : mx));  // D~ (column) / E~ (row)
    const double Et = 1.0 / sqrt(clampf(fabs(abl)));                       // bound-row E~ (column lanes)
    const bool unit = GL::all((!col || (F == 1.0 && Et == 1.0)) && (!row || F == 1.0));
    if (!unit) {
      if (l < M) wb[l] = F;  // wb[c] = D~_c, wb[NX + r] = E~_r
      asm volatile("" ::: "memory");
      static_for<KV>([&](auto K) {
        constexpr int k = decltype(K)::value;
        if constexpr (k < NP) {  // column: P entry (D~_l D~_k); row: G entry (E~_r D~_k)
          V[k] *= F * wb[k];
        } else {
          double m = 1.0;
          if constexpr (k - NP < NG) m = wb[NX + k - NP] * F;  // column: G entry (E~_i D~_l)
          if constexpr (k < NX) {
            const double mr = F * wb[k];  // row: G entry (E~_r D~_k)
            m = col ? m : mr;
          }
          V[k] *= m;
        }
      });
      asm volatile("" ::: "memory");
      if (col) {
        abl *= Et * F;
        ql *= F;
        Dl *= F;
        El *= Et;
      }
      if (row) EGl *= F;
    }
    // cost scaling: mean column norm of P vs |q|_inf
    double cn = 0, qn = 0;
    if (hp) {
      double t[NP];
#pragma unroll
      for (int c = 0; c < NP; ++c) t[c] = V[c];
      cn = absmax_tree(t);
    }
    if (col) qn = fabs(ql);
    cn = GL::sum(cn) / NX;
    qn = GL::max(qn);
    qn = clampf(qn);
    double ct = clampf(fmax(cn, qn));
    ct = 1.0 / ct;
    if (hp)
#pragma unroll
      for (int c = 0; c < NP; ++c) V[c] *= ct;
    if (col) ql *= ct;
    cs *= ct;
    if (ct == 1.0 && unit) break;
  }
  if (hp)
#pragma unroll
    for (int c = 0; c < NP; ++c) P[l * NP + c] = V[c];
  if (row)
#pragma unroll
    for (int j = 0; j < NX; ++j) G[r * NX + j] = V[j];
  if (col) {
    ab[l] = abl;
    qq[l] = ql;
    D[l] = Dl;
    E[l] = El;
  }
  if (row) E[NX + r] = EGl;
  if (l == 0) sc[SC_C] = cs;
  wsync();
  for (int rw = l; rw < M; rw += GL::size) {
    lo[rw] = fmax(lo[rw], -kInf) * E[rw];
    up[rw] = fmin(up[rw], kInf) * E[rw];
  }
  wsync();
  return DRC_STATUS_MAX_ITER;
}

// Addresses and lane-role indices of the Schur ADMM loop, derived from an
// opaque copy of the parameter pointer and lane index: built once for the
// loop's setup and again where the (every check_termination iterations)
// publish and reload need them, so none of it stays live through the
// iterations, where at the QP kernel's 168-VGPR budget it was spilled before
// the loop and reloaded at every check (D20)
// SchurLanes' opaque copies keep the LDS address space (lds_double, kernel_common.hpp)
template <class QD>
struct SchurLanes {
  static constexpr int NX = QD::nx, NG = QD::ng, NP = QD::np;
  lds_double *qq, *ab, *lo, *up, *x, *z, *y, *dy;
  lds_cdouble *rv, *Si, *GS, *dv, *cf, *G;
  int l, rr, lc, ia, ig, iv;
  bool hc, hr, ha, hv;
  __device__ __forceinline__ SchurLanes(const KParams& kpl, double* S0) {
    // kpl and S0 point into this wave's LDS (the kernel's __shared__ copy and plan)
    lds_ckparams* kq = opaque_lds((lds_ckparams*)&kpl);
    lds_double* S = opaque_lds((lds_double*)S0);
    lds_ckparams& kp = *kq;
    l = Grp<QD::gs>::lane();
    qq = S + kp.oQ; ab = S + kp.oAB; lo = S + kp.oL; up = S + kp.oU;
    x = S + kp.oX; z = S + kp.oZ; y = S + kp.oY; dy = S + kp.oDY;
    rv = S + kp.oRho;
    Si = S + kp.oU0;
    GS = Si + NP * NP;
    dv = GS + NG * NP;
    cf = dv + NG;
    G = S + kp.oG;
    lds_cint* aux = (lds_cint*)(cf + 2 * NG);
    hc = l < NP;
    hr = l >= NP && l < NP + NG;
    rr = hr ? l - NP : 0;
    lc = hc ? l : 0;
    const int a_ = hr ? aux[rr] : -1;  // auxiliary variable of row r (or -1)
    ha = a_ >= 0;
    ia = ha ? a_ : 0;
    ig = NX + rr;  // the G row
    hv = hc || ha;
    iv = hc ? lc : ia;
  }
  // lane l: row l of S^-1 then column l of G_c (core lanes); row r of G_c S^-1 (row lanes)
  __device__ __forceinline__ void load(double (&R)[NP + NG]) const {
    if (hc) {
#pragma unroll
      for (int c = 0; c < NP; ++c) R[c] = Si[lc * NP + c];
#pragma unroll
      for (int i = 0; i < NG; ++i) R[NP + i] = G[i * NX + lc];
    } else {
#pragma unroll
      for (int c = 0; c < NP; ++c) R[c] = GS[rr * NP + c];
#pragma unroll
      for (int i = 0; i < NG; ++i) R[NP + i] = 0.0;
    }
  }
};

// The Schur-complement register ADMM iterations (QD::schur shapes): `steps`
// iterations from the iterate published in LDS, which they publish again.
// The caller (qp_admm) runs the iterations between two checks / adaptive-rho
// steps per call and calls admm_check in between, so no call sits inside the
// iteration loop: with admm_check called from inside it (r03-r06k), the
// loop's scalar state (counters, lane masks) lived across that call in VGPR
// lanes, a v_readlane / v_writelane per value and iteration (about 40 of an
// FR3 iteration's 170 instructions; now about 100, none of them spills).
// Reads its parameters from the LDS copy kpl.
// Lane roles: l < NP core variable l (and its bound row); NP + r < NP + NG:
// G row r together with its auxiliary variable a(r) and that variable's
// bound row.  R[] holds, on core lanes, row l of S^-1 then column l of
// G_c; on row lanes, row r of G_c S^-1.  Per iteration:
//   rows: t_a = r_a / d_a, u_r = w_r - rho_r g_r t_a       (w = rho z - y)
//   core: r'_c = sigma x_c - q_c + ab_c w_b + sum_r G_rc u_r   (NG broadcasts)
//   core: x~_c = S^-1 r';  rows: v_r = G_r,c x~_c = (G_c S^-1)_r r'   (NP broadcasts)
//   rows: x~_a = t_a - coef_r v_r,  (G x~)_r = v_r + g_r x~_a
template <class QD>
__device__ __forceinline__ void admm_iters_schur(const KParams& kpl, double* S, int steps) {
  using GL = Grp<QD::gs>;
  const KParams& kp = kpl;
  const double sig = kp.s.sigma, al = kp.s.alpha;
  PHG_DECL
  constexpr int NX = QD::nx, NG = QD::ng, NP = QD::np;
  (void)NX;
  static_assert(NP + NG <= QD::gs, "one lane per core variable and per G row");
  double R[NP + NG];
  // The lane's variable v (with its bound row): the core variable on a core
  // lane, the auxiliary variable on a row lane that has one.  A lane is never
  // both, so the two share one register set (same update formulas; fewer
  // registers live across the loop and one code path instead of two)
  bool hc, hr, ha, hv;
  double ab_v, q_v, lo_v, up_v, g_r, lo_g, up_g, d_r, c_r, r_v, rg;
  double xv, zv, yv, dyv = 0, zg, yg, dyg = 0;
#ifndef DRC_ADMM_READLANE_BCAST
  int rr_l = 0, lc_l = 0;
#endif
  {  // S^-1 / rho and the iterate as the setup or the last check left them
    const SchurLanes<QD> L(kpl, S);
    L.load(R);
    hc = L.hc; hr = L.hr; ha = L.ha; hv = L.hv;
    ab_v = L.ab[L.iv]; q_v = L.qq[L.iv]; lo_v = L.lo[L.iv]; up_v = L.up[L.iv];
    g_r = ha ? L.G[L.rr * NX + L.ia] : 0.0;
    lo_g = L.lo[L.ig]; up_g = L.up[L.ig];
    d_r = L.dv[L.rr]; c_r = L.cf[L.rr];
    r_v = L.rv[L.iv]; rg = L.rv[L.ig];
    xv = L.x[L.iv]; zv = L.z[L.iv]; yv = L.y[L.iv];
    zg = L.z[L.ig]; yg = L.y[L.ig];
#ifndef DRC_ADMM_READLANE_BCAST
    rr_l = L.rr;
    lc_l = L.lc;
#endif
  }
  PHG(25);
  const double ir_v = 1.0 / r_v, irg = 1.0 / rg;  // y / rho as a product in the loop
#ifndef DRC_ADMM_READLANE_BCAST
  // (formed once: the compiler barriers below would re-read kpl.oBc per iteration)
  lds_double* const wb = (lds_double*)(S + kpl.oBc);
#endif
  const int n = __builtin_amdgcn_readfirstlane(steps);  // wave-uniform trip count
  for (int k = 0; k < n; ++k) {
      // core: r'_c's own term; aux: r_a before the G row's share
      const double tv = hv ? sig * xv - q_v + ab_v * (r_v * zv - yv) : 0.0;
      double u = 0, ta = 0;
      if (hr) {
        const double wg = rg * zg - yg;
        if (ha) {
          const double r_a = tv + g_r * wg;
          ta = r_a * d_r;  // d_r holds 1 / d_a
          u = wg - rg * g_r * ta;
        } else {
          u = wg;
        }
      }
      const double loc = hc ? tv : 0.0;
      double r0 = 0, r1 = 0;
#ifndef DRC_ADMM_READLANE_BCAST  // the two passes' vectors broadcast through LDS (r04: +1-3 %)
      if (hr) wb[rr_l] = u;
      asm volatile("" ::: "memory");
      static_for<NG>([&](auto I) {
        constexpr int i = decltype(I)::value;
        const double ui = wb[i];
        if constexpr (i & 1) r1 += R[NP + i] * ui;
        else r0 += R[NP + i] * ui;
      });
      const double rp = loc + (r0 + r1);
      if (hc) wb[NG + lc_l] = rp;
      asm volatile("" ::: "memory");
      double s0 = 0, s1 = 0;
      static_for<NP>([&](auto C) {
        constexpr int c = decltype(C)::value;
        const double rpc = wb[NG + c];
        if constexpr (c & 1) s1 += R[c] * rpc;
        else s0 += R[c] * rpc;
      });
#else
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
#endif
      const double sv = s0 + s1;  // core: x~_c; row: v_r = G_r,c x~_c
      const double xta = ha ? ta - c_r * sv : 0.0;  // aux: x~_a
      if (hv) {  // the variable's bound row: z~ = ab x~, relaxation, projection, dual update
        const double xin = hc ? sv : xta;
        const double zr = al * ab_v * xin + (1 - al) * zv;
        double zn = zr + yv * ir_v;
        zn = fmin(fmax(zn, lo_v), up_v);
        dyv = r_v * (zr - zn);
        yv += dyv;
        zv = zn;
        xv = al * xin + (1 - al) * xv;
      }
      if (hr) {  // G row
        const double zr = al * (sv + g_r * xta) + (1 - al) * zg;
        double zn = zr + yg * irg;
        zn = fmin(fmax(zn, lo_g), up_g);
        dyg = rg * (zr - zn);
        yg += dyg;
        zg = zn;
      }
  }
  {  // publish the iterate for the (LDS) residual / polish / rho code
    const SchurLanes<QD> L(kpl, S);
    if (hv) {
      L.x[L.iv] = xv;
      L.z[L.iv] = zv;
      L.y[L.iv] = yv;
      L.dy[L.iv] = dyv;
    }
    if (hr) {
      L.z[L.ig] = zg;
      L.y[L.ig] = yg;
      L.dy[L.ig] = dyg;
    }
  }
  wsync();
  PHG(26);
}

// The same iterations out of line (the reference-settings mode: about 120
// iterations in five calls per instance ran faster in a leaf function of their
// own than inlined into the QP kernel, exact mode's single call of 8
// iterations slower -- profiles/r06l_ab_admm_iters_*.jsonl, r06m_ab_*)
template <class QD>
__device__ __noinline__ void admm_iters_schur_call(const KParams& kpl, double* S, int steps) {
  admm_iters_schur<QD>(kpl, S, steps);
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
    // the iterations between two checks / adaptive-rho steps (or the last)
    // per call; wave-uniform control in SGPRs (the LDS parameter copy reads
    // into VGPRs, and admm_check's verdict is uniform by construction)
    const int max_iter = __builtin_amdgcn_readfirstlane(kp.s.max_iter);
    const int check_every = __builtin_amdgcn_readfirstlane(kp.s.check_termination);
    const int adapt_every = __builtin_amdgcn_readfirstlane(
        kp.s.adaptive_rho && kp.s.adaptive_rho_interval > 0 ? kp.s.adaptive_rho_interval : 0);
    constexpr int kNever = 0x7fffffff;
    int to_check = check_every > 0 ? check_every : kNever, to_adapt = adapt_every > 0 ? adapt_every : kNever;
    bool stopped = false;
    it = 0;
    while (it < max_iter) {
      const int steps = min(min(to_check, to_adapt), max_iter - it);
      if (kp.s.exact) admm_iters_schur<QD>(kpl, S, steps);
      else admm_iters_schur_call<QD>(kpl, S, steps);
      it += steps;
      to_check -= steps;
      to_adapt -= steps;
      const bool check = to_check == 0, adapt = to_adapt == 0;
      if (check) to_check = check_every;
      if (adapt) to_adapt = adapt_every;
      if (!(check || adapt)) continue;  // last iteration: published for the output
      PH_STAMP(tc0);
      const int act = __builtin_amdgcn_readfirstlane(admm_check<QD>(kpl, S, it, check, adapt, &status));
      PH_ONLY(const unsigned long long dchk = __builtin_amdgcn_s_memtime() - tc0; PH_ADD(27, dchk));
      if (act == 2) {
        stopped = true;
        break;
      }
    }
    if (!stopped) it = (max_iter > 0 ? max_iter : 0) + 1;  // as a counted loop 1..max_iter leaves it
  } else if constexpr (QD::reg) {
    constexpr int NX = QD::nx, NG = QD::ng;
    double Gc[NG], Kr[NX], GKr[NX];
    prep_admm_mats<QD>(kpl, S);
    load_admm_regs<QD>(kp, S, Gc, Kr, GKr);
    PHG(25);
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
      PH_STAMP(tc0);
      const int act = admm_check<QD>(kpl, S, it, check, adapt, &status);
      PH_ONLY(const unsigned long long dchk = __builtin_amdgcn_s_memtime() - tc0; PH_ADD(27, dchk); PH_ADD(26, 0ull - dchk));  // checks out of the loop's slot
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
    PHG(26);
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

// One instance b of the QP stage on this lane group (S: its LDS plan kp; kpl:
// an LDS copy of kp for the out-of-line ADMM blocks): assembly from the task
// record, Ruiz scaling, ADMM + certified polish, outputs (zero on failure,
// QP_IK.cpp:56-61).  Used by qp_kernel and the fused task + QP kernel.
template <class QD>
__device__ __forceinline__ void qp_instance(const DevModel* __restrict__ M0, const KParams& kp, const KParams& kpl,
                                            const IO& io, double* S, int64_t b) {
  using GL = Grp<QD::gs>;
  const int l = GL::lane();
  PH_DECL
  const int64_t gb = io.b0 + b, LD = io.ld;  // position in the caller's [field][B] arrays
  const DevModel* M = opaque_model(M0);
  stage_stamp<QD::gs>(io, ST_QP0, gb);
  stage_where<QD::gs>(io, ST_WQP, gb);
  qp_assemble<QD>(M, kp, S, io, b);
  stage_stamp<QD::gs>(io, ST_ASM, gb);
  PH(0);
  const bool lp_inf = M->kind == 1 && kp.s.exact && moma_lp_infeasible<QD>(M, kp, S);
  int status, iters = 0;
  if constexpr (QD::reg && QD::gs == 64 && QD::nx + QD::ng <= 64) status = qp_scale_roles<QD>(kpl, S);
  else if constexpr (QD::reg) status = qp_scale_regs<QD>(kpl, S);
  else status = qp_scale<QD>(kp, S);
  scaling_inverses<QD>(kp, S);
  PH(1);
  if (status != DRC_STATUS_NONFINITE) {
    if (lp_inf) status = DRC_STATUS_PRIMAL_INFEASIBLE;
    else status = qp_admm<QD>(kp, kpl, S, &iters);
  }
  PH(3);
  stage_stamp<QD::gs>(io, ST_SOLVED, gb);
  // ---------------- outputs (zero on failure, QP_IK.cpp:56-61) ------------
  const double *D = S + kp.oD, *x = S + kp.oX;
  if (l < kp.na) io.out[(int64_t)l * LD + gb] = status == DRC_STATUS_SOLVED ? D[l] * x[l] : 0.0;
  if (l == 0) {
    io.status[gb] = status;
    if (io.iters) io.iters[gb] = iters;
  }
  wsync();
  stage_stamp<QD::gs>(io, ST_OUT, gb);
  PH(5);
  PH_FLUSH(16);
}

}  // namespace drc_amd

// Torque-level QP of QPID / QPIDStep / QPIDCubic (SURVEY §8f row 2;
// QP_ID.cpp:11-131, MoMa QP_ID.cpp:11-33): assembly from the task record and
// the dynamics launch's M, g, then the same OSQP ADMM (qp_solver.hpp) on the
// Schur complement of the torque / slack block.
#include "kernel_common.hpp"
#include "launch.hpp"
#include "qp_solver.hpp"

namespace drc_amd {

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
#ifndef DRC_QPID_WAVES
#define DRC_QPID_WAVES 1
#endif
template <class QD>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(DRC_QPID_WAVES, 8)))
qpid_kernel(const DevModel* __restrict__ M0, const KParams kp, const IO io) {
  extern __shared__ __attribute__((aligned(16))) double S[];
  PH_KSCOPE();
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
    const DevModel* M = opaque_model(M0);
    qpid_assemble(M, kp, S, io, b);
    int status, iters = 0;
    status = qp_scale<QD>(kp, S);
    scaling_inverses<QD>(kp, S);
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

int launch_qpid_kernel(unsigned grid, size_t lds, hipStream_t st, const DevModel* m, const KParams& kp, const IO& io) {
  const dim3 g(grid), blk(64);
  if (kp.nx == 44 && kp.ng == 37 && kp.np == 7)  // FR3
    hipLaunchKernelGGL((qpid_kernel<Dims<44, 37, 7, false, true>>), g, blk, lds, st, m, kp, io);
  else if (kp.nx == 38 && kp.ng == 32 && kp.np == 6)  // UR5e
    hipLaunchKernelGGL((qpid_kernel<Dims<38, 32, 6, false, true>>), g, blk, lds, st, m, kp, io);
  else if (kp.nx == 18 && kp.ng == 39 && kp.np == 9)  // Husky-FR3
    hipLaunchKernelGGL((qpid_kernel<Dims<18, 39, 9, false, true>>), g, blk, lds, st, m, kp, io);
  else if (kp.nx == 22 && kp.ng == 41 && kp.np == 11)  // XLS-FR3
    hipLaunchKernelGGL((qpid_kernel<Dims<22, 41, 11, false, true>>), g, blk, lds, st, m, kp, io);
  else
    hipLaunchKernelGGL((qpid_kernel<Dims<0, 0, 0>>), g, blk, lds, st, m, kp, io);
  return hipGetLastError();
}

#ifdef DRC_PHASE_TIMING
DRC_PHASE_EXPORT(phase_cycles_qpid)
#endif

}  // namespace drc_amd

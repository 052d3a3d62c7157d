// Task stage of one instance (one wavefront): FK, frame Jacobian, task
// velocity, manipulability + gradient, self-collision distance + gradient
// (and the QPID / closed-form extras), ending in the task record or the
// stage outputs.  Used by task_kernel (task_kernel.hip) and the fused
// task + QP kernel (fused_kernel.hip).
//   FK / LWA frame Jacobian        robot_data.cpp:101-107,392-402
//   task error (+ cubic profile)   math_type_define.h:633-687, robot_controller.cpp:292-317
//   manipulability + gradient      robot_data.cpp:519-553 (MoMa :439-475)
//   min self-distance + gradient   robot_data.cpp:424-494 (hpp-fcl GJK/EPA semantics)
//   QPID stage data, CLIK / OSF    robot_data.cpp:109,476-512, robot_controller.cpp:150-260
#pragma once

#include "kernel_common.hpp"

namespace drc_amd {

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
    if (!inv6_certified(A6, Ai)) pinv_cod6_wave(A6, Ai, ws);
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

// One instance b of the task stage on this wave (S: the wave's LDS plan kp).
// PROBLEM 0: QPIK stage data; 1: also the QPID extras; 2: closed-form CLIK / OSF.
template <int PROBLEM>
__device__ __forceinline__ void task_instance(const DevModel* __restrict__ M0, const KParams& kp, const IO& io, double* S,
                                              int64_t b) {
  const int l = lane_id();
  const int nv = kp.nv;
  EpaPoly* ews = reinterpret_cast<EpaPoly*>(S + kp.kEpa);  // LDS-resident polytope
  PH_DECL
  const int64_t gb = io.b0 + b, LD = io.ld;  // position in the caller's [field][B] arrays
  PH_ONLY(const unsigned long long inst_t0 = __builtin_amdgcn_s_memtime(); unsigned long long ph_snap[8];
          for (int k_ = 0; k_ < 8; ++k_) ph_snap[k_] = ph_acc[k_];
          unsigned long long epa_calls = 0, epa_steps = 0, epa_maxsteps = 0, epa_t[8] = {0, 0, 0, 0, 0, 0, 0, 0};)
  // re-derive the model pointer each instance: keeps LICM from hoisting
  // model-constant loads out of the instance loop into spilled registers
  const DevModel* M = opaque_model(M0);
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
  if (PROBLEM == 2 && kp.cf == 3) {
    // kinematics only (drc_kinematics_batch): no task targets
  } else if (l < 12) {
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
    if (kp.cf == 3) {  // kinematics only: getPose / getJacobian / getVelocity (robot_data.cpp:378-422)
      if (io.st_pose && l < 12) io.st_pose[l * LD + gb] = l < 9 ? Te[(l % 3) * 3 + l / 3] : Te[l];
      if (io.st_jac)
        for (int e = l; e < 6 * nv; e += 64) io.st_jac[(int64_t)e * LD + gb] = J[e];
      if (io.st_xdd && l < 6) io.st_xdd[l * LD + gb] = jq;  // J qdot, row r on lane r
      wsync();
      return;
    }
    closed_form_stage(M, kp, S, io, gb, LD);
    PH_FLUSH(0);
    return;
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
      const double dt = det_lu6_wave(A6);
      pinv_cod6_wave(A6, Ai, S + kp.kScr);
      if (l == 0) S[kp.oSc + SC_MAN] = sqrt(dt);
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
  int8_t* pf = reinterpret_cast<int8_t*>(S + kp.kPf);  // 0 open, 1 done, 2 penetrating (EPA)
  double bestd = 1.7976931348623157e308;
  int besti = 0x7fffffff;
  int bhow = 0;  // how the running best was found: 0 closed form, 1 GJK, 2 EPA
  V3 bpA = v3(0, 0, 0), bpB = v3(0, 0, 0);
  double ub = 1e300;
  // slots in type-class order (model.cpp pair_order): each round of 64 lanes
  // runs one or two pair types instead of all of them
  for (int sl = l; sl < M->npairs; sl += 64) {
    const int p = M->pair_order[sl], ga = M->slot_a[sl], gb = M->slot_b[sl];
    ShapeL A{M->gtype[ga], (lds_pose*)(Tg + 12 * ga), M->gparam[ga][0], M->gparam[ga][1], M->gparam[ga][2]};
    ShapeL Bs{M->gtype[gb], (lds_pose*)(Tg + 12 * gb), M->gparam[gb][0], M->gparam[gb][1], M->gparam[gb][2]};
    V3 pA, pB;
    double d;
    const bool closed = (A.type == kSphere || Bs.type == kSphere)
                            ? (d = sphere_pair(A, Bs, &pA, &pB), true)
                            : (A.type == kCylinder && Bs.type == kCylinder && cyl_cyl_side(A, Bs, &d, &pA, &pB));
    if (closed) {
      pf[p] = 1;
      ub = fmin(ub, d);
      if (d < bestd || (d == bestd && p < besti)) {  // ties -> lowest pair index
        bestd = d;
        besti = p;
        bhow = 0;
        bpA = pA;
        bpB = pB;
      }
    } else {  // swept-core / separating-axis lower bound
      pd[p] = pair_lower_bound(A, Bs, M->gbound[ga], M->gbound[gb]);
      pf[p] = 0;
    }
  }
  ub = -wave_max(-ub);
  PH(3);
  // exact GJK only where the swept-core bound can still win.  The candidates
  // are compacted into a list first, so a wave runs them in ceil(n / 64)
  // rounds instead of one round per 64 pair slots.
  bool pen = false;  // some candidate intersects: the EPA search below has work
  {
    int* cand = reinterpret_cast<int*>(S + kp.kCand);
    int ncand = 0;
    for (int p0 = 0; p0 < M->npairs; p0 += 64) {
      const int p = p0 + l;
      const bool c = p < M->npairs && pf[p] == 0 && pd[p] - 1e-9 <= ub;
      const unsigned long long m = __ballot(c);
      if (c) cand[ncand + __popcll(m & ((1ull << l) - 1))] = p;
      ncand += __popcll(m);
    }
    if (l == 0) ews->nv = 0;  // EPA seed stash counter (epa_stash)
    wsync();
    for (int c = l; c < ncand; c += 64) {
      const int p = cand[c];
      const int ga = M->pair_a[p], gb = M->pair_b[p];
      ShapeL A{M->gtype[ga], (lds_pose*)(Tg + 12 * ga), M->gparam[ga][0], M->gparam[ga][1], M->gparam[ga][2]};
      ShapeL Bs{M->gtype[gb], (lds_pose*)(Tg + 12 * gb), M->gparam[gb][0], M->gparam[gb][1], M->gparam[gb][2]};
      // early exit once GJK's lower bound shows the pair cannot reach ub
      const GjkDist g = gjk(A, Bs, ub + 1e-9, ews, p);
      if (g.pruned) {
        pf[p] = 1;
      } else if (g.intersect) {
        pf[p] = 2;  // penetrating: EPA below
        pen = true;
      } else {
        pf[p] = 1;
        if (g.dist < bestd || (g.dist == bestd && p < besti)) {
          bestd = g.dist;
          besti = p;
          bhow = 1;
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
  // (Only pairs whose GJK intersected are searched: none, no search.)
  if (__any(pen)) {
#ifdef DRC_EPA_PRIO  // A/B variant: an EPA wave takes issue priority on its SIMD
    __builtin_amdgcn_s_setprio(DRC_EPA_PRIO);
#endif
    double gbd = bestd;
    int gbi = besti;
    wave_argmin(gbd, gbi);
    // stashed GJK simplices of intersecting pairs (epa_stash): pair and size
    // per slot, valid until a polytope grows into the stash's vertex slots
    const int nst = ews->nv < kEpaStash ? ews->nv : kEpaStash;
    int sp0 = nst > 0 ? static_cast<int>(ews->out[0]) : -1, sp1 = nst > 1 ? static_cast<int>(ews->out[2]) : -1;
    const int sn0 = nst > 0 ? static_cast<int>(ews->out[1]) : 0, sn1 = nst > 1 ? static_cast<int>(ews->out[3]) : 0;
    wsync();  // stash metadata read before the first EPA overwrites out[]
    for (;;) {
      double cpd = 1.7976931348623157e308;
      int cp = 0x7fffffff;
      for (int p = l; p < M->npairs; p += 64)
        if (pf[p] == 2 && pd[p] < cpd) {
          cpd = pd[p];
          cp = p;
        }
      wave_argmin(cpd, cp);
      if (cp == 0x7fffffff || cpd > gbd || (cpd == gbd && cp > gbi)) break;
      const int p = cp, ln = p & 63, ga = M->pair_a[p], gb = M->pair_b[p];
      const ShapeL A{M->gtype[ga], (lds_pose*)(Tg + 12 * ga), M->gparam[ga][0], M->gparam[ga][1], M->gparam[ga][2]};
      const ShapeL Bs{M->gtype[gb], (lds_pose*)(Tg + 12 * gb), M->gparam[gb][0], M->gparam[gb][1], M->gparam[gb][2]};
      PH_ONLY(epa_calls++; unsigned long long est[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};)
      const int sk = p == sp0 ? 0 : (p == sp1 ? 1 : -1);
      const double dall = epa_run_wave(A, Bs, ews, ln, sk, sk == 0 ? sn0 : sn1 PH_ONLY(, est));
      if (ews->nv > kEpaStashV0) sp0 = sp1 = -1;  // grown into the stash slots
      PH_ONLY(epa_steps += est[0]; if (est[0] > epa_maxsteps) epa_maxsteps = est[0];
              epa_t[0] += est[1]; epa_t[1] += est[2]; epa_t[2] += est[3];
              for (int k_ = 0; k_ < 5; ++k_) epa_t[3 + k_] += est[4 + k_];)
      if (l == ln && (dall < bestd || (dall == bestd && p < besti))) {
        bestd = dall;
        besti = p;
        bhow = 2;
        bpA = ld3(ews->out);
        bpB = ld3(ews->out + 3);
      }
      if (dall < gbd || (dall == gbd && p < gbi)) {
        gbd = dall;
        gbi = p;
      }
      if (l == ln) pf[p] = 1;
      wsync();
    }
#ifdef DRC_EPA_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
  }
  PH(5);
  const double myd = bestd;
  const int myi = besti;
  wave_argmin(bestd, besti);
  double* dgv = S + kp.kdg;
  double* red = S + kp.oRed;
  // The winning pair's GJK / EPA witnesses are refined to the exact critical
  // point (D17).  The QPIK stage does it after the task data are written,
  // where little is live across the call (in place, the call's register
  // saves and frame slowed every instance: measured); QPID's extras read
  // the witnesses, so QPID refines here.
  auto refine_winner = [&]() {
    const int ga = M->pair_a[besti], gb = M->pair_b[besti];
    const ShapeL A{M->gtype[ga], (lds_pose*)(Tg + 12 * ga), M->gparam[ga][0], M->gparam[ga][1], M->gparam[ga][2]};
    const ShapeL Bs{M->gtype[gb], (lds_pose*)(Tg + 12 * gb), M->gparam[gb][0], M->gparam[gb][1], M->gparam[gb][2]};
    double dref = S[kp.oSc + SC_DIST];
    V3 rA = ld3(red), rB = ld3(red + 3);
#ifdef DRC_NO_REFINE  // diagnostic build: the raw GJK / EPA witnesses
    if (false && refine_witness(A, Bs, &dref, &rA, &rB)) {
#else
    if (refine_witness(A, Bs, &dref, &rA, &rB)) {
#endif
      st3(red, rA);
      st3(red + 3, rB);
      S[kp.oSc + SC_DIST] = dref;
    }
  };
  // grad d = n^T (J_B(pB) - J_A(pA)) for joint l + 1, sign flipped when penetrating
  auto dist_grad = [&](double dd) {
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
      if (dd < 0) g = -g;
    }
    return g;
  };
  if (myi == besti && myi < M->npairs) {  // the winning lane publishes its witnesses
    st3(red, bpA);
    st3(red + 3, bpB);
    S[kp.oSc + SC_DIST] = myd;
    S[kp.oSc + SC_HOW] = bhow;
  }
  if (l == 0) {
    if (besti >= M->npairs) {
      S[kp.oSc + SC_DIST] = bestd;
      S[kp.oSc + SC_HOW] = 0;
    }
    S[kp.oSc + SC_PAIR] = besti;
  }
  wsync();
  if constexpr (PROBLEM == 1) {
    if (l == 0 && S[kp.oSc + SC_HOW] != 0) refine_winner();
    wsync();
  }
  bestd = S[kp.oSc + SC_DIST];
  PH(6);
  if (l < nv) dgv[l] = dist_grad(bestd);
  wsync();
  if constexpr (PROBLEM == 1) qpid_task_extras(M, kp, S, bestd, besti, io.st_gdv != nullptr);
  PH(7);
  PH_ONLY(if (l == 0) {  // straggler census: max instance cycles, count above 400 k (~7x FR3's mean)
    const unsigned long long dt = __builtin_amdgcn_s_memtime() - inst_t0;
    atomicMax(&g_phase_cycles[30], dt);
    if (dt > 400000ull) {
      atomicAdd(&g_phase_cycles[31], 1ull);
      atomicAdd(&g_phase_cycles[29], dt);
      for (int k_ = 0; k_ < 8; ++k_) atomicAdd(&g_phase_cycles[8 + k_], ph_acc[k_] - ph_snap[k_]);
    }
    if (epa_calls) {  // EPA census over every instance
      atomicAdd(&g_phase_cycles[22], epa_calls);
      atomicAdd(&g_phase_cycles[23], epa_steps);
      atomicMax(&g_phase_cycles[28], epa_maxsteps);
      atomicAdd(&g_phase_cycles[18], epa_t[0] + epa_t[1]);  // (qp kernel leaves 18, 20 free)
      atomicAdd(&g_phase_cycles[20], epa_t[2]);
      // growth split (slots no other stage of a QPIK call writes)
      atomicAdd(&g_phase_cycles[59], epa_t[3]);
      atomicAdd(&g_phase_cycles[61], epa_t[4]);
      atomicAdd(&g_phase_cycles[62], epa_t[5]);
      atomicAdd(&g_phase_cycles[63], epa_t[6]);
      atomicAdd(&g_phase_cycles[60], epa_t[7]);  // seed polytope (slot 60: the lane stage's, not run here)
    }
  })
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
  if constexpr (PROBLEM == 0) {  // late refinement of the winner (D17): patch d and grad d
    if (S[kp.oSc + SC_HOW] != 0) {
      if (l == 0) refine_winner();
      wsync();
      const double dd = S[kp.oSc + SC_DIST];
      const double g = l < nv ? dist_grad(dd) : 0.0;
      if (io.rec) {
        double* rec = io.rec + b * io.rec_stride;
        if (l == 0) rec[kp.rDist] = dd;
        if (l < nv) rec[kp.rDist + 1 + l] = g;
      } else if (io.st_dist) {
        if (l == 0) io.st_dist[gb] = dd;
        if (l < nv) io.st_dist[(int64_t)(1 + l) * LD + gb] = g;
      }
      wsync();
    }
  }
  PH_FLUSH(0);
}

}  // namespace drc_amd

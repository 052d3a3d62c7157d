// Lane-per-instance task stage of QPIK (included by task_kernel.hip).
//
// The wave-per-instance task_kernel spends most of its time in phases that
// use a handful of lanes (the FK chain, the 6x6 manipulability algebra, one
// GJK per instance) and waits on LDS round trips between them.  Here one
// lane owns one instance end to end: the robot's joint chain, geometry list
// and pair list are identical for every lane, so control flow is uniform
// (model indices are scalar loads), the joint frames stay in registers
// (compile-time joint count NV), and 64 instances advance per instruction.
// Only GJK iteration counts diverge; its candidates are drained per lane.
//
// Same formulas and decisions as task_kernel (and so as the oracle):
//   FK / frame pose / LWA Jacobian   robot_data.cpp:101-107,392-402
//   task velocity                    robot_controller.cpp:277-317, math_type_define.h:633-687
//   manipulability + gradient        robot_data.cpp:519-553
//   min self-distance + gradient     robot_data.cpp:424-494
// Instances that need the serial fallbacks (EPA on a penetrating GJK pair,
// more than kLaneMaxCand GJK candidates, the COD pseudo-inverse of an
// ill-conditioned JJ^T) are appended to a hard list (and flagged) that the
// wave-per-instance task_kernel then processes; their records are written
// only there, and the QP of the other instances need not wait for them.
// (inside namespace drc_amd: included after task_kernel)

constexpr int kLaneCandWords = kMaxCandSlots / 64;  // candidate bit words per lane
constexpr int kLaneMaxCand = 8;                     // GJK calls per instance before it goes to the hard list

#ifdef DRC_PHASE_TIMING
// per-wave phase stamps of the lane stage (slots 48..53) and counters (56..61)
#define LPH_DECL unsigned long long lph_t = __builtin_amdgcn_s_memtime();
#define LPH(slot)                                                                   \
  do {                                                                              \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();                     \
    if (l == __ffsll(__ballot(1)) - 1) atomicAdd(&g_phase_cycles[(slot)], t_ - lph_t); \
    lph_t = t_;                                                                     \
  } while (0)
#define LCNT(slot, cond)                                                                       \
  do {                                                                                         \
    const unsigned long long m_ = __ballot(cond);                                              \
    if (l == __ffsll(__ballot(1)) - 1) atomicAdd(&g_phase_cycles[(slot)], (unsigned long long)__popcll(m_)); \
  } while (0)
#else
#define LPH_DECL
#define LPH(slot) do {} while (0)
#define LCNT(slot, cond) do {} while (0)
#endif

// (frame j of the chain; 0 = world) -> 12 doubles, j uniform or per lane
template <int NV>
__device__ __forceinline__ void lane_frame(const double (&T)[NV][12], int j, double* out) {
#pragma unroll
  for (int i = 0; i < 12; ++i) out[i] = (i == 0 || i == 4 || i == 8) ? 1.0 : 0.0;
#pragma unroll
  for (int k = 0; k < NV; ++k)
    if (j == k + 1) {
#pragma unroll
      for (int i = 0; i < 12; ++i) out[i] = T[k][i];
    }
}

// world pose of geometry g (full transform; a sphere needs only its centre,
// which is the same translation row of tmul)
template <int NV>
__device__ __forceinline__ void lane_geom(const DevModel* M, const double (&T)[NV][12], int g, bool full,
                                          double* out) {
  double Tp[12];
  lane_frame<NV>(T, M->gparent[g], Tp);
  const double* b = M->gplace[g];
  if (full) {
    tmul(Tp, b, out);
  } else {
#pragma unroll
    for (int i = 0; i < 9; ++i) out[i] = 0.0;
#pragma unroll
    for (int i = 0; i < 3; ++i) out[9 + i] = Tp[3 * i] * b[9] + Tp[3 * i + 1] * b[10] + Tp[3 * i + 2] * b[11] + Tp[9 + i];
  }
}

template <int NV>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1)))
lane_task_kernel(const DevModel* __restrict__ M, const KParams kp, const IO io) {
  const int l = lane_id();
  const int64_t b = int64_t(blockIdx.x) * 64 + l;
  if (b >= io.B) return;
  const int64_t gb = io.b0 + b, LD = io.ld;
  LPH_DECL
  // ---------------- state in ----------------
  double qv[NV], qd[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    qv[k] = io.q[k * LD + gb];
    qd[k] = io.qdot[k * LD + gb];
  }
  // ---------------- FK ----------------------
  double T[NV][12];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int j = k + 1;
    double Mj[12];
    const double* ax = M->axis[j];
    const double qq = qv[k];
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
    double Lj[12], Tp[12];
    tmul(M->jplace[j], Mj, Lj);
    lane_frame<NV>(T, M->parent[j], Tp);
    tmul(Tp, Lj, T[k]);
  }
  double Te[12];
  {
    double Tf[12];
    lane_frame<NV>(T, kp.frame_joint, Tf);
    tmul(Tf, kp.frame_place, Te);
  }
  const V3 pe = v3(Te[9], Te[10], Te[11]);
  const uint32_t anc_e = M->anc[kp.frame_joint];
  LPH(48);
  // ---------------- self-collision distance --------------------------------
  // pass 1: closed forms (sphere pairs, side-to-side cylinders) with the
  // running minimum, and lower bounds for the rest (swept core raised to the
  // separating-axis value, pair_lower_bound).  Candidate pairs (bound can
  // still reach the closed-form minimum) are remembered as bits of their
  // position in the pair list, re-tested against the final minimum in pass 2
  // (bound - 1e-9 <= ub).  A pair whose bound exceeds the minimum cannot be
  // the argmin, so pruning it leaves the result of computing every pair.
  double bestd = 1.7976931348623157e308, ub = 1e300;
  int besti = 0x7fffffff;
  bool bgjk = false;  // the running best came from GJK (refined below, D17)
  V3 bpA = v3(0, 0, 0), bpB = v3(0, 0, 0);
  uint64_t cmask[kLaneCandWords];
#pragma unroll
  for (int w = 0; w < kLaneCandWords; ++w) cmask[w] = 0;
  bool hard = false;
  for (int p = 0; p < M->npairs; ++p) {
    const int ga = M->pair_a[p], gb_ = M->pair_b[p];
    const int ta = M->gtype[ga], tb = M->gtype[gb_];
    double TA[12], TB[12];
    lane_geom<NV>(M, T, ga, ta != kSphere, TA);
    lane_geom<NV>(M, T, gb_, tb != kSphere, TB);
    const Shape A{ta, TA, M->gparam[ga][0], M->gparam[ga][1], M->gparam[ga][2]};
    const Shape Bs{tb, TB, M->gparam[gb_][0], M->gparam[gb_][1], M->gparam[gb_][2]};
    V3 pA, pB;
    double d;
    const bool closed = (ta == kSphere || tb == kSphere)
                            ? (d = sphere_pair(A, Bs, &pA, &pB), true)
                            : (ta == kCylinder && tb == kCylinder && cyl_cyl_side(A, Bs, &d, &pA, &pB));
    if (closed) {
      ub = fmin(ub, d);
      if (d < bestd) {
        bestd = d;
        besti = p;
        bgjk = false;
        bpA = pA;
        bpB = pB;
      }
    } else {
      const double pd = pair_lower_bound(A, Bs, M->gbound[ga], M->gbound[gb_]);
      if (pd - 1e-9 <= ub) {
        const int slot = M->cand_slot[p];  // position among the non-closed-type pairs
#pragma unroll
        for (int w = 0; w < kLaneCandWords; ++w)
          if ((slot >> 6) == w) cmask[w] |= 1ull << (slot & 63);
      }
    }
  }
  LPH(49);
  // pass 2: GJK on each lane's own candidates, lowest pair first
  int ncand = 0;
  bool why_int = false;
#pragma unroll
  for (int w = 0; w < kLaneCandWords; ++w) {
    for (;;) {
      if (cmask[w] == 0) break;
      const int bit = __builtin_ctzll(cmask[w]);
      cmask[w] &= cmask[w] - 1;
      const int p = M->cand_pair[w * 64 + bit];
      const int ga = M->pair_a[p], gb_ = M->pair_b[p];
      const int ta = M->gtype[ga], tb = M->gtype[gb_];
      double TA[12], TB[12];
      lane_geom<NV>(M, T, ga, true, TA);
      lane_geom<NV>(M, T, gb_, true, TB);
      const Shape A{ta, TA, M->gparam[ga][0], M->gparam[ga][1], M->gparam[ga][2]};
      const Shape Bs{tb, TB, M->gparam[gb_][0], M->gparam[gb_][1], M->gparam[gb_][2]};
      const double pd = pair_lower_bound(A, Bs, M->gbound[ga], M->gbound[gb_]);
      if (!(pd - 1e-9 <= ub)) continue;
      if (++ncand > kLaneMaxCand) {
        hard = true;
        break;
      }
      // the pair matters only if it can reach the closed-form minimum (or
      // the best GJK result so far, which is never above it)
      GjkState g;
      gjk_run<true>(A, Bs, g, fmin(ub, bestd) + 1e-9);
      if (g.pruned) continue;
      if (g.intersect) {  // penetrating: EPA runs in the wave-per-instance kernel
        hard = true;
        why_int = true;
        break;
      }
      V3 gA = v3(0, 0, 0), gB = v3(0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (i < g.n) {
          gA = gA + g.lam[i] * g.S[i].a;
          gB = gB + g.lam[i] * (g.S[i].a - g.S[i].w);
        }
      const double gd = sqrt(dot(g.v, g.v));
      if (gd < bestd || (gd == bestd && p < besti)) {
        bestd = gd;
        besti = p;
        bgjk = true;
        bpA = gA;
        bpB = gB;
      }
    }
  }
  LPH(50);
  LCNT(56, hard && !why_int);
  LCNT(57, why_int);
  (void)why_int;  // counted in the timing build only
  LCNT(58, true);
#ifdef DRC_PHASE_TIMING
  atomicAdd(&g_phase_cycles[60], (unsigned long long)ncand);
#endif
  if (hard) {  // the wave-per-instance kernel recomputes this instance
    const int k = atomicAdd(io.hard_n, 1);
    io.hard_list[k] = static_cast<int>(b);
    if (io.hard_flag) io.hard_flag[b] = 1;
    return;
  }
  if (bgjk) {  // the winner's GJK witnesses sharpened to the exact critical point (D17)
    const int ga = M->pair_a[besti], gb_ = M->pair_b[besti];
    double TA[12], TB[12];
    lane_geom<NV>(M, T, ga, true, TA);
    lane_geom<NV>(M, T, gb_, true, TB);
    const Shape A{M->gtype[ga], TA, M->gparam[ga][0], M->gparam[ga][1], M->gparam[ga][2]};
    const Shape Bs{M->gtype[gb_], TB, M->gparam[gb_][0], M->gparam[gb_][1], M->gparam[gb_][2]};
    refine_witness(A, Bs, &bestd, &bpA, &bpB);
  }
  // ---------------- joint axes, Jacobian, distance gradient ----------------
  V3 z[NV], pj[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    z[k] = rot(T[k], ld3(M->axis[k + 1]));
    pj[k] = v3(T[k][9], T[k][10], T[k][11]);
  }
  const int nv = NV;
  double dgv[NV];
  {
    V3 n = v3(0, 0, 0);
    int jA = 0, jB = 0;
    uint32_t aA = 0, aB = 0;
    if (besti < M->npairs) {
      jA = M->gparent[M->pair_a[besti]];
      jB = M->gparent[M->pair_b[besti]];
      aA = jA > 0 ? M->anc[jA] : 0u;
      aB = jB > 0 ? M->anc[jB] : 0u;
      n = bpB - bpA;
      n = (1.0 / sqrt(dot(n, n))) * n;
    }
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      double g = 0;
      if (besti < M->npairs) {
        const bool rev = M->jtype[k + 1] == kRevolute;
        V3 cA = v3(0, 0, 0), cB = v3(0, 0, 0);
        if (aA & (1u << k)) cA = rev ? cross(z[k], bpA - pj[k]) : z[k];
        if (aB & (1u << k)) cB = rev ? cross(z[k], bpB - pj[k]) : z[k];
        g = dot(n, cB - cA);
        if (bestd < 0) g = -g;
      }
      dgv[k] = g;
    }
  }
  double J[6][NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    V3 lin = v3(0, 0, 0), ang = v3(0, 0, 0);
    if (anc_e & (1u << k)) {
      if (M->jtype[k + 1] == kRevolute) {
        lin = cross(z[k], pe - pj[k]);
        ang = z[k];
      } else {
        lin = z[k];
      }
    }
    J[0][k] = lin.x; J[1][k] = lin.y; J[2][k] = lin.z;
    J[3][k] = ang.x; J[4][k] = ang.y; J[5][k] = ang.z;
  }
  // ---------------- task velocity (task_kernel's lane-0 block) -------------
  double xdd[6];
  if (kp.mode == DRC_MODE_QPIK) {
#pragma unroll
    for (int i = 0; i < 6; ++i) xdd[i] = io.xdt[i * LD + gb];
  } else {
    double xt[12], xdt[6];
#pragma unroll
    for (int i = 0; i < 12; ++i) xt[i] = io.xt[i * LD + gb];
#pragma unroll
    for (int i = 0; i < 6; ++i) xdt[i] = io.xdt[i * LD + gb];
    if (kp.mode == DRC_MODE_QPIK_CUBIC) {  // getTaskSpaceCubic (math_type_define.h:647)
      double xi[12], xdi[6], Rt[9], Ri[9];
#pragma unroll
      for (int i = 0; i < 12; ++i) xi[i] = io.xi[i * LD + gb];
#pragma unroll
      for (int i = 0; i < 6; ++i) xdi[i] = io.xdi[i * LD + gb];
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          Rt[3 * r + c] = xt[3 * c + r];
          Ri[3 * r + c] = xi[3 * c + r];
        }
      const double t = kp.t, t0 = kp.t0, tf = kp.t0 + kp.duration;
      double pdv[3], vd[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        pdv[i] = cubic(t, t0, tf, xi[9 + i], xt[9 + i], xdi[i], xdt[i]);
        vd[i] = cubic_dot(t, t0, tf, xi[9 + i], xt[9 + i], xdi[i], xdt[i]);
      }
      double RiT_Rt[9], Rd[9];
#pragma unroll
      for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int c = 0; c < 3; ++c)
          RiT_Rt[3 * a + c] = Ri[a] * Rt[c] + Ri[3 + a] * Rt[3 + c] + Ri[6 + a] * Rt[6 + c];
      const V3 r = so3_log(RiT_Rt);
      if (t >= tf) {
#pragma unroll
        for (int i = 0; i < 9; ++i) Rd[i] = Rt[i];
      } else if (t < t0) {
#pragma unroll
        for (int i = 0; i < 9; ++i) Rd[i] = Ri[i];
      } else {
        double E3[9];
        so3_exp(cubic(t, t0, tf, 0, 1, 0, 0) * r, E3);
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
          for (int c = 0; c < 3; ++c)
            Rd[3 * a + c] = Ri[3 * a] * E3[c] + Ri[3 * a + 1] * E3[3 + c] + Ri[3 * a + 2] * E3[6 + c];
      }
      V3 rd = v3(cubic_dot(t, t0, tf, 0, r.x, 0, 0), cubic_dot(t, t0, tf, 0, r.y, 0, 0),
                 cubic_dot(t, t0, tf, 0, r.z, 0, 0));
      rd = v3(Ri[0] * rd.x + Ri[1] * rd.y + Ri[2] * rd.z, Ri[3] * rd.x + Ri[4] * rd.y + Ri[5] * rd.z,
              Ri[6] * rd.x + Ri[7] * rd.y + Ri[8] * rd.z);
      const double tau = (t - t0) / (tf - t0);
      if (tau < 0 || tau > 1) rd = v3(0, 0, 0);
#pragma unroll
      for (int r0 = 0; r0 < 3; ++r0)
#pragma unroll
        for (int c = 0; c < 3; ++c) xt[3 * c + r0] = Rd[3 * r0 + c];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        xt[9 + i] = pdv[i];
        xdt[i] = vd[i];
      }
      xdt[3] = rd.x; xdt[4] = rd.y; xdt[5] = rd.z;
    }
    double e[6], xdot[6];
#pragma unroll
    for (int i = 0; i < 3; ++i) e[i] = xt[9 + i] - Te[9 + i];
    V3 phi = v3(0, 0, 0);
#pragma unroll
    for (int i = 0; i < 3; ++i)
      phi = phi + cross(v3(xt[3 * i], xt[3 * i + 1], xt[3 * i + 2]), v3(Te[i], Te[3 + i], Te[6 + i]));
    e[3] = -0.5 * phi.x; e[4] = -0.5 * phi.y; e[5] = -0.5 * phi.z;
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      double s = 0;
#pragma unroll
      for (int c = 0; c < NV; ++c) s += J[r][c] * qd[c];
      xdot[r] = s;
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) xdd[i] = kp.kp[i] * e[i] + kp.kv[i] * (xdt[i] - xdot[i]) + kp.ff * xdt[i];
  }
  LPH(51);
  // ---------------- manipulability (arm columns c0 .. c0+narm) -------------
  // JJ^T by Jordan exchanges without pivoting (SPD), det = product of the
  // pivots; the ill-conditioned case takes the serial COD path on private
  // arrays (same functions and threshold as task_kernel).
  const int narm = kp.narm, c0 = kp.c0;
  double A6[36], Ai[36];
#pragma unroll
  for (int a = 0; a < 6; ++a)
#pragma unroll
    for (int bb = 0; bb < 6; ++bb) {
      double s = 0;
#pragma unroll
      for (int c = 0; c < NV; ++c)
        if (c >= c0 && c < c0 + narm) s += J[a][c] * J[bb][c];
      A6[a * 6 + bb] = s;
    }
  double man;
  {
    double piv_min = 1e300, det = 1;
#pragma unroll
    for (int i = 0; i < 36; ++i) Ai[i] = A6[i];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const double akk = Ai[k * 6 + k];
      double nw[36];
#pragma unroll
      for (int ii = 0; ii < 6; ++ii)
#pragma unroll
        for (int jj = 0; jj < 6; ++jj) {
          const double aij = Ai[ii * 6 + jj], aik = Ai[ii * 6 + k], akj = Ai[k * 6 + jj];
          double v;
          if (ii == k && jj == k) v = 1.0 / akk;
          else if (ii == k) v = akj / akk;
          else if (jj == k) v = -aik / akk;
          else v = aij - aik * akj / akk;
          nw[ii * 6 + jj] = v;
        }
      piv_min = fmin(piv_min, akk);
      det *= akk;
#pragma unroll
      for (int i = 0; i < 36; ++i) Ai[i] = nw[i];
    }
    double fa = 0, fi = 0;
#pragma unroll
    for (int i = 0; i < 36; ++i) {
      fa += A6[i] * A6[i];
      fi += Ai[i] * Ai[i];
    }
    LCNT(59, !(piv_min > 0) || !(fa * fi < 1e10));
    if (!(piv_min > 0) || !(fa * fi < 1e10)) {  // serial COD path: wave-per-instance kernel
      const int k = atomicAdd(io.hard_n, 1);
      io.hard_list[k] = static_cast<int>(b);
      if (io.hard_flag) io.hard_flag[b] = 1;
      return;
    } else {
      man = sqrt(det);
    }
  }
  // W = Jr^T Ai (narm x 6); part(k, i) = d(J_i)/dq_k . W_i; mg_k = m sum_i part
  double W[NV][6];
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    double Jc[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      Jc[i] = 0;
#pragma unroll
      for (int u = 0; u < NV; ++u)
        if (u == c0 + c) Jc[i] = J[i][u];
    }
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      double t = 0;
#pragma unroll
      for (int i = 0; i < 6; ++i) t += Jc[i] * Ai[i * 6 + a];
      W[c][a] = t;
    }
  }
  double mg[NV];
#pragma unroll
  for (int kk = 0; kk < NV; ++kk) {
    double s = 0;
    if (kk < narm) {
      const int jk = c0 + kk + 1;
      V3 zk = v3(0, 0, 0), pk_ = v3(0, 0, 0);
#pragma unroll
      for (int u = 0; u < NV; ++u)
        if (u + 1 == jk) {
          zk = z[u];
          pk_ = pj[u];
        }
      const bool krev = M->jtype[jk] == kRevolute;
      const V3 dpe = krev ? cross(zk, pe - pk_) : zk;
#pragma unroll
      for (int c = 0; c < NV; ++c) {
        if (c >= narm) continue;
        const int ji = c0 + c + 1;
        double acc = 0;
        if ((anc_e & (1u << (jk - 1))) && (anc_e & (1u << (ji - 1)))) {
          V3 zi = v3(0, 0, 0), pi_ = v3(0, 0, 0);
#pragma unroll
          for (int u = 0; u < NV; ++u)
            if (u + 1 == ji) {
              zi = z[u];
              pi_ = pj[u];
            }
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
          const double* w = W[c];
          acc = lin.x * w[0] + lin.y * w[1] + lin.z * w[2] + ang.x * w[3] + ang.y * w[4] + ang.z * w[5];
        }
        s += acc;
      }
      s = man * s;
    }
    mg[kk] = s;
  }
  LPH(52);
  if (io.hard_flag) io.hard_flag[b] = 0;
  // ---------------- outputs --------------------------------------------------
  if (io.rec) {
    double* rec = io.rec + b * io.rec_stride;
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
      for (int c = 0; c < NV; ++c) rec[r * nv + c] = J[r][c];
    rec[kp.rMan] = man;
#pragma unroll
    for (int k = 0; k < NV; ++k)
      if (k < narm) rec[kp.rMan + 1 + k] = mg[k];
    rec[kp.rDist] = bestd;
#pragma unroll
    for (int k = 0; k < NV; ++k) rec[kp.rDist + 1 + k] = dgv[k];
#pragma unroll
    for (int i = 0; i < 6; ++i) rec[kp.rXdd + i] = xdd[i];
#pragma unroll
    for (int k = 0; k < NV; ++k) rec[kp.rQ + k] = qv[k];
  } else {
    if (io.st_pose)
#pragma unroll
      for (int i = 0; i < 12; ++i) io.st_pose[i * LD + gb] = i < 9 ? Te[(i % 3) * 3 + i / 3] : Te[i];
    if (io.st_jac)
#pragma unroll
      for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int c = 0; c < NV; ++c) io.st_jac[int64_t(r * nv + c) * LD + gb] = J[r][c];
    if (io.st_man) {
      io.st_man[gb] = man;
#pragma unroll
      for (int k = 0; k < NV; ++k)
        if (k < narm) io.st_man[int64_t(1 + k) * LD + gb] = mg[k];
    }
    if (io.st_dist) {
      io.st_dist[gb] = bestd;
#pragma unroll
      for (int k = 0; k < NV; ++k) io.st_dist[int64_t(1 + k) * LD + gb] = dgv[k];
    }
    if (io.st_pair) io.st_pair[gb] = besti < M->npairs ? besti : -1;
    if (io.st_xdd)
#pragma unroll
      for (int i = 0; i < 6; ++i) io.st_xdd[i * LD + gb] = xdd[i];
  }
}


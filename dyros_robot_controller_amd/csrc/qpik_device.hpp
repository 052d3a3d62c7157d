// Device-side building blocks of the QP-IK kernel (gfx950, wave64).
//
// One 64-lane wavefront owns one robot instance; the workgroup is exactly
// one wave, so __syncthreads() is a wave-local LDS fence.  Lanes take the
// natural parallel axis of each phase: joints (FK / Jacobian columns),
// (k, c) pairs (dJ/dq for the manipulability gradient), collision pairs
// (narrow phase), QP variables / constraint rows (ADMM, polish).
#pragma once

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
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ void wsync() { __syncthreads(); }

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// argmin with ties broken toward the smaller index (reference: first strict
// minimum in pair order, robot_data.cpp:434-442)
__device__ __forceinline__ void wave_argmin(double& v, int& idx) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    double ov = __shfl_xor(v, o, 64);
    int oi = __shfl_xor(idx, o, 64);
    if (ov < v || (ov == v && oi < idx)) {
      v = ov;
      idx = oi;
    }
  }
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
DRC_HD __forceinline__ V3 rot(const double* T, V3 v) {
  return v3(T[0] * v.x + T[1] * v.y + T[2] * v.z, T[3] * v.x + T[4] * v.y + T[5] * v.z,
            T[6] * v.x + T[7] * v.y + T[8] * v.z);
}
DRC_HD __forceinline__ V3 rotT(const double* T, V3 v) {
  return v3(T[0] * v.x + T[3] * v.y + T[6] * v.z, T[1] * v.x + T[4] * v.y + T[7] * v.z,
            T[2] * v.x + T[5] * v.y + T[8] * v.z);
}
DRC_HD __forceinline__ V3 xform(const double* T, V3 v) { return rot(T, v) + v3(T[9], T[10], T[11]); }
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
struct Shape {
  int type;
  const double* T;   // pose in LDS
  double p0, p1, p2; // parameters
};

DRC_HD __forceinline__ V3 support(const Shape& s, V3 d) {
  if (s.type == kSphere) return v3(s.T[9], s.T[10], s.T[11]);
  V3 dl = rotT(s.T, d), loc;
  if (s.type == kCylinder) {
    double rho = sqrt(dl.x * dl.x + dl.y * dl.y);
    loc.x = rho > 0 ? s.p0 * dl.x / rho : 0.0;
    loc.y = rho > 0 ? s.p0 * dl.y / rho : 0.0;
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
DRC_HD __forceinline__ SV sup_md(const Shape& A, const Shape& B, V3 d) {
  SV o;
  o.a = support(A, d);
  o.b = support(B, -1.0 * d);
  o.w = o.a - o.b;
  return o;
}

// Simplex storage in registers; pick() selects by runtime index with
// conditional moves so no private array is ever dynamically indexed.
struct Simplex {
  V3 w0, w1, w2, w3;   // support points of the Minkowski difference A - B
  V3 a0, a1, a2, a3;   // matching support points on A (B = a - w)
};
DRC_HD __forceinline__ V3 pick(V3 s0, V3 s1, V3 s2, V3 s3, int i) {
  return i == 0 ? s0 : (i == 1 ? s1 : (i == 2 ? s2 : s3));
}
DRC_HD __forceinline__ V3 simplex_w(const Simplex& S, int i) { return pick(S.w0, S.w1, S.w2, S.w3, i); }
DRC_HD __forceinline__ V3 simplex_a(const Simplex& S, int i) { return pick(S.a0, S.a1, S.a2, S.a3, i); }
DRC_HD __forceinline__ void simplex_set(Simplex& S, int i, V3 w, V3 a) {
  if (i == 0) { S.w0 = w; S.a0 = a; }
  else if (i == 1) { S.w1 = w; S.a1 = a; }
  else if (i == 2) { S.w2 = w; S.a2 = a; }
  else { S.w3 = w; S.a3 = a; }
}

// Closest point of conv(S[0..n)) to the origin: exhaustive sub-simplex
// search, same visiting order (masks from 2^n-1 down to 1) and tolerances as
// oracle/drc_oracle.c.  Compacts the kept vertices to the front.
DRC_HD __forceinline__ int closest_simplex(Simplex& S, int n, V3* v, double* l0o, double* l1o, double* l2o,
                                               double* l3o) {
  double best = 0.0, b0 = 0, b1 = 0, b2 = 0, b3 = 0;
  int bmask = 0;
  for (int mask = (1 << n) - 1; mask > 0; --mask) {
    int k = __builtin_popcount(mask);
    int i0 = __builtin_ffs(mask) - 1;
    int r1 = mask & (mask - 1), i1 = __builtin_ffs(r1) - 1;
    int r2 = r1 & (r1 - 1), i2 = __builtin_ffs(r2) - 1;
    int r3 = r2 & (r2 - 1), i3 = __builtin_ffs(r3) - 1;
    const V3 w0 = simplex_w(S, i0);
    double l0 = 1, l1 = 0, l2 = 0, l3 = 0;
    bool valid = true;
    if (k > 1) {
      V3 D0 = simplex_w(S, i1) - w0;
      V3 D1 = k > 2 ? simplex_w(S, i2) - w0 : v3(0, 0, 0);
      V3 D2 = k > 3 ? simplex_w(S, i3) - w0 : v3(0, 0, 0);
      double mu0 = 0, mu1 = 0, mu2 = 0;
      if (k == 2) {
        double G0 = dot(D0, D0), r0 = -dot(D0, w0);
        valid = G0 > 0;
        mu0 = valid ? r0 / G0 : 0;
      } else if (k == 3) {
        double G0 = dot(D0, D0), G1 = dot(D0, D1), G3 = dot(D1, D0), G4 = dot(D1, D1);
        double r0 = -dot(D0, w0), r1 = -dot(D1, w0);
        double det = G0 * G4 - G1 * G3;
        valid = fabs(det) >= 1e-300;
        mu0 = valid ? (r0 * G4 - G1 * r1) / det : 0;
        mu1 = valid ? (G0 * r1 - r0 * G3) / det : 0;
      } else {
        double a = dot(D0, D0), b = dot(D0, D1), c = dot(D0, D2), dd = dot(D1, D0), e = dot(D1, D1),
               f = dot(D1, D2), g = dot(D2, D0), h = dot(D2, D1), ii = dot(D2, D2);
        double r0 = -dot(D0, w0), r1 = -dot(D1, w0), r2 = -dot(D2, w0);
        double det = a * (e * ii - f * h) - b * (dd * ii - f * g) + c * (dd * h - e * g);
        valid = fabs(det) >= 1e-300;
        if (valid) {
          mu0 = (r0 * (e * ii - f * h) - b * (r1 * ii - f * r2) + c * (r1 * h - e * r2)) / det;
          mu1 = (a * (r1 * ii - f * r2) - r0 * (dd * ii - f * g) + c * (dd * r2 - r1 * g)) / det;
          mu2 = (a * (e * r2 - r1 * h) - b * (dd * r2 - r1 * g) + r0 * (dd * h - e * g)) / det;
        }
      }
      l0 = 1 - (mu0 + mu1 + mu2);
      l1 = mu0;
      l2 = mu1;
      l3 = mu2;
      valid = valid && !(l0 < -1e-14) && !(l1 < -1e-14) && !(k > 2 && l2 < -1e-14) && !(k > 3 && l3 < -1e-14);
    }
    if (valid) {
      V3 p = l0 * w0;
      if (k > 1) p = p + l1 * simplex_w(S, i1);
      if (k > 2) p = p + l2 * simplex_w(S, i2);
      if (k > 3) p = p + l3 * simplex_w(S, i3);
      double dv = dot(p, p);
      if (bmask == 0 || dv < best - 1e-18) {
        best = dv;
        bmask = mask;
        *v = p;
        b0 = l0; b1 = l1; b2 = l2; b3 = l3;
      }
    }
  }
  Simplex T = S;
  int k = 0;
  for (int i = 0; i < n; ++i)
    if (bmask & (1 << i)) simplex_set(T, k++, simplex_w(S, i), simplex_a(S, i));
  S = T;
  *l0o = b0; *l1o = b1; *l2o = b2; *l3o = b3;
  return k;
}

// GJK on the cores (all state register-resident inside this function).
// Returns {intersect, dist, pA, pB}; on intersection the final simplex is
// written to ws->V[0..ns) for EPA and ns is returned.
struct GjkOut {
  int intersect, ns;
  double dist;
  V3 pA, pB;
};
struct EpaWs;
DRC_HD __forceinline__ void epa_seed(EpaWs* ws, int i, V3 w, V3 a);
DRC_HD __noinline__ GjkOut gjk(const Shape A, const Shape B, EpaWs* ws) {
  Simplex S;
  S.w0 = S.w1 = S.w2 = S.w3 = v3(0, 0, 0);
  S.a0 = S.a1 = S.a2 = S.a3 = v3(0, 0, 0);
  V3 v = v3(A.T[9] - B.T[9], A.T[10] - B.T[10], A.T[11] - B.T[11]);
  if (dot(v, v) < 1e-24) v = v3(1, 0, 0);
  int n = 0;
  double l0 = 1, l1 = 0, l2 = 0, l3 = 0;
  GjkOut o;
  o.intersect = 0;
  for (int it = 0; it < 128; ++it) {
    SV w = sup_md(A, B, -1.0 * v);
    double vv = dot(v, v);
    if (n > 0 && vv - dot(v, w.w) <= 1e-12 * sqrt(vv)) break;
    bool dup = false;
    for (int i = 0; i < n; ++i) {
      V3 si = simplex_w(S, i);
      dup |= (si.x == w.w.x && si.y == w.w.y && si.z == w.w.z);
    }
    if (dup) break;
    simplex_set(S, n, w.w, w.a);
    ++n;
    n = closest_simplex(S, n, &v, &l0, &l1, &l2, &l3);
    if (n == 4 || dot(v, v) < 1e-24) {
      o.intersect = 1;
      break;
    }
  }
  o.ns = n;
  if (o.intersect) {
    if (ws)
      for (int i = 0; i < n; ++i) epa_seed(ws, i, simplex_w(S, i), simplex_a(S, i));
    o.dist = 0;
    o.pA = o.pB = v3(0, 0, 0);
    return o;
  }
  // witnesses: sum_i lam_i a_i and sum_i lam_i b_i (oracle accumulation order)
  V3 pA = v3(0, 0, 0), pB = v3(0, 0, 0);
  for (int i = 0; i < n; ++i) {
    const double li = i == 0 ? l0 : (i == 1 ? l1 : (i == 2 ? l2 : l3));
    const V3 ai = simplex_a(S, i), bi = ai - simplex_w(S, i);
    pA = pA + li * ai;
    pB = pB + li * bi;
  }
  o.pA = pA;
  o.pB = pB;
  o.dist = sqrt(dot(v, v));
  return o;
}

// Expanding polytope (EPA) with face adjacency (Bullet/libccd style): the
// visible region is flood-filled from the closest face across shared edges
// (explicit DFS stack, same visiting order as the recursive oracle), so the
// horizon is a single loop and the polytope stays a closed 2-manifold even
// when flat features (cylinder caps, box faces) make the support mapping
// degenerate.  Lane-serial, polytope in a per-wave global workspace (rare
// path: penetrating candidate pairs only).
constexpr int kEpaMaxV = 256, kEpaMaxF = 512;
struct EpaWs {
  SV V[kEpaMaxV];
  int fv[kEpaMaxF][3], ff[kEpaMaxF][3], fe[kEpaMaxF][3];
  int fpass[kEpaMaxF], alive[kEpaMaxF];
  int stk_f[kEpaMaxF], stk_e[kEpaMaxF], stk_s[kEpaMaxF];
  double fn[kEpaMaxF][3], fd[kEpaMaxF];
  double out[6];
  int nv, nf, pass, hcf, hff, hnf, fail;
};
DRC_HD __forceinline__ void epa_seed(EpaWs* ws, int i, V3 w, V3 a) {
  ws->V[i].w = w;
  ws->V[i].a = a;
  ws->V[i].b = a - w;
}
DRC_HD __forceinline__ int epa_newface(EpaWs* E, int a, int b, int c) {
  if (E->nf >= kEpaMaxF) {
    E->fail = 1;
    return -1;
  }
  const int f = E->nf++;
  E->fv[f][0] = a;
  E->fv[f][1] = b;
  E->fv[f][2] = c;
  E->alive[f] = 1;
  E->fpass[f] = 0;
  V3 nn = cross(E->V[b].w - E->V[a].w, E->V[c].w - E->V[a].w);
  const double L = sqrt(dot(nn, nn));
  if (!(L > 1e-300)) {
    E->fail = 1;
    E->alive[f] = 0;
    return -1;
  }
  nn = (1.0 / L) * nn;
  E->fn[f][0] = nn.x;
  E->fn[f][1] = nn.y;
  E->fn[f][2] = nn.z;
  E->fd[f] = dot(nn, E->V[a].w);
  return f;
}
DRC_HD __forceinline__ void epa_bind(EpaWs* E, int f0, int e0, int f1, int e1) {
  E->ff[f0][e0] = f1;
  E->fe[f0][e0] = e1;
  E->ff[f1][e1] = f0;
  E->fe[f1][e1] = e0;
}
// iterative form of btGjkEpa2::expand over the three edges of `best`
DRC_HD __forceinline__ bool epa_expand_all(EpaWs* E, int w, int best) {
  const V3 ww = E->V[w].w;
  for (int j = 0; j < 3; ++j) {
    int sp = 0;
    E->stk_f[0] = E->ff[best][j];
    E->stk_e[0] = E->fe[best][j];
    E->stk_s[0] = 0;
    sp = 1;
    while (sp > 0) {
      const int f = E->stk_f[sp - 1], e = E->stk_e[sp - 1], st = E->stk_s[sp - 1];
      if (st == 0) {
        if (E->fpass[f] == E->pass) {
          --sp;
          continue;
        }
        const int e1 = e == 2 ? 0 : e + 1;
        const V3 n = v3(E->fn[f][0], E->fn[f][1], E->fn[f][2]);
        if (dot(n, ww) - E->fd[f] < -1e-12) {
          const int nf = epa_newface(E, E->fv[f][e1], E->fv[f][e], w);
          if (nf < 0) return false;
          epa_bind(E, nf, 0, f, e);
          if (E->hcf >= 0) epa_bind(E, E->hcf, 1, nf, 2);
          else E->hff = nf;
          E->hcf = nf;
          ++E->hnf;
          --sp;
          continue;
        }
        E->fpass[f] = E->pass;
        E->stk_s[sp - 1] = 1;
        if (sp >= kEpaMaxF) return false;
        E->stk_f[sp] = E->ff[f][e1];
        E->stk_e[sp] = E->fe[f][e1];
        E->stk_s[sp] = 0;
        ++sp;
      } else if (st == 1) {
        const int e2 = e == 0 ? 2 : e - 1;
        E->stk_s[sp - 1] = 2;
        if (sp >= kEpaMaxF) return false;
        E->stk_f[sp] = E->ff[f][e2];
        E->stk_e[sp] = E->fe[f][e2];
        E->stk_s[sp] = 0;
        ++sp;
      } else {
        E->alive[f] = 0;
        --sp;
      }
    }
  }
  return true;
}

// The GJK simplex arrives in ws->V[0..ns) (epa_seed) so no private array
// crosses the call; witness points come back in ws->out.
DRC_HD __noinline__ double epa(const Shape A, const Shape B, int ns, EpaWs* E) {
  E->nv = ns;
  E->nf = 0;
  E->pass = 0;
  E->fail = 0;
  for (int di = 0; di < 6 && E->nv < 4; ++di) {
    const double sgn = di < 3 ? 1.0 : -1.0;
    const int ax = di % 3;
    SV w = sup_md(A, B, v3(ax == 0 ? sgn : 0.0, ax == 1 ? sgn : 0.0, ax == 2 ? sgn : 0.0));
    bool ok = true;
    for (int i = 0; i < E->nv; ++i) {
      V3 d = w.w - E->V[i].w;
      ok &= sqrt(dot(d, d)) > 1e-12;
    }
    if (ok) E->V[E->nv++] = w;
  }
  {  // orient the tetrahedron so that face (0,1,2) looks away from vertex 3
    V3 nn = cross(E->V[1].w - E->V[0].w, E->V[2].w - E->V[0].w);
    if (dot(nn, E->V[3].w - E->V[0].w) > 0) {
      SV t = E->V[0];
      E->V[0] = E->V[1];
      E->V[1] = t;
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
    for (int it = 0; it < 255; ++it) {
      int best = -1;
      double bd = 1e300;
      for (int f = 0; f < E->nf; ++f)
        if (E->alive[f] && E->fd[f] < bd) {
          bd = E->fd[f];
          best = f;
        }
      const V3 bn = v3(E->fn[best][0], E->fn[best][1], E->fn[best][2]);
      SV w = sup_md(A, B, bn);
      if (dot(bn, w.w) - E->fd[best] <= 1e-12 || E->nv >= kEpaMaxV) break;
      bool dupv = false;
      for (int i = 0; i < E->nv; ++i) {
        V3 d = w.w - E->V[i].w;
        dupv |= fabs(d.x) <= 1e-14 && fabs(d.y) <= 1e-14 && fabs(d.z) <= 1e-14;
      }
      if (dupv) break;
      const int wi = E->nv;
      E->V[E->nv++] = w;
      E->pass++;
      E->hcf = -1;
      E->hff = -1;
      E->hnf = 0;
      E->fpass[best] = E->pass;
      const bool valid = epa_expand_all(E, wi, best);
      if (!valid || E->hnf < 3 || E->fail) {
        E->nv--;
        break;
      }
      epa_bind(E, E->hcf, 1, E->hff, 2);
      E->alive[best] = 0;
    }
  }
  double bd = 1e300;
  int best = 0;
  for (int f = 0; f < E->nf; ++f)
    if (E->alive[f] && E->fd[f] < bd) {
      bd = E->fd[f];
      best = f;
    }
  const V3 bn = v3(E->fn[best][0], E->fn[best][1], E->fn[best][2]);
  const SV &a = E->V[E->fv[best][0]], &b = E->V[E->fv[best][1]], &c = E->V[E->fv[best][2]];
  V3 p = bd * bn, v0 = b.w - a.w, v1 = c.w - a.w, v2 = p - a.w;
  double d00 = dot(v0, v0), d01 = dot(v0, v1), d11 = dot(v1, v1), d20 = dot(v2, v0), d21 = dot(v2, v1);
  double den = d00 * d11 - d01 * d01;
  double l1 = (d11 * d20 - d01 * d21) / den, l2 = (d00 * d21 - d01 * d20) / den, l0 = 1 - l1 - l2;
  st3(E->out, l0 * a.a + l1 * b.a + l2 * c.a);
  st3(E->out + 3, l0 * a.b + l1 * b.b + l2 * c.b);
  return -bd;
}

// signed distance + closest surface point of a solid cylinder / box
DRC_HD __forceinline__ double point_cylinder(V3 c, const Shape& s, V3* qw) {
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
DRC_HD __forceinline__ double point_box(V3 c, const Shape& s, V3* qw) {
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
DRC_HD __forceinline__ double sphere_pair(const Shape& A, const Shape& B, V3* pA, V3* pB) {
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
  const Shape& s = flip ? B : A;
  const Shape& o = flip ? A : B;
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

// Lower bound on the distance of two geometries via their swept cores:
// cylinder -> axis segment (radius r), box -> centre point (bounding radius),
// sphere -> centre.  Exact closed form for segment/segment.
DRC_HD __forceinline__ void core_segment(const Shape& s, double bound, V3* a, V3* b, double* rad) {
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
DRC_HD __forceinline__ double seg_seg_dist(V3 p1, V3 q1, V3 p2, V3 q2) {
  V3 d1 = q1 - p1, d2 = q2 - p2, r = p1 - p2;
  double a = dot(d1, d1), e = dot(d2, d2), f = dot(d2, r), s, t;
  if (a <= 1e-30 && e <= 1e-30) {
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
  return sqrt(dot(dd, dd));
}

}  // namespace drc_amd

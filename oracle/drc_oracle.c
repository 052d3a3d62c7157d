/*
 * ORACLE / TEST INFRASTRUCTURE ONLY — see drc_oracle.h for what is restated
 * and where.  Scalar, straightforward C: it is the checker and the CPU
 * baseline, never the thing measured on the GPU.
 */
#include "drc_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>

#define INFTY 1e30               /* OSQP_INFTY                               */
#define MIN_SCALING 1e-4
#define MAX_SCALING 1e4
#define RHO_MIN 1e-6
#define RHO_MAX 1e6
#define RHO_TOL 1e-4
#define RHO_EQ_OVER_RHO_INEQ 1e3
#define DIVISION_TOL 1e-30

/* ------------------------------------------------------------------------ */
/* small dense helpers                                                      */
/* ------------------------------------------------------------------------ */
static inline double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static inline void cross3(const double* a, const double* b, double* c) {
    double x = a[1] * b[2] - a[2] * b[1], y = a[2] * b[0] - a[0] * b[2], z = a[0] * b[1] - a[1] * b[0];
    c[0] = x; c[1] = y; c[2] = z;
}
static inline void sub3(const double* a, const double* b, double* c) { c[0] = a[0] - b[0]; c[1] = a[1] - b[1]; c[2] = a[2] - b[2]; }
static inline double norm3(const double* a) { return sqrt(dot3(a, a)); }
/* R (row-major) * v */
static inline void matvec3(const double* R, const double* v, double* o) {
    double x = R[0] * v[0] + R[1] * v[1] + R[2] * v[2];
    double y = R[3] * v[0] + R[4] * v[1] + R[5] * v[2];
    double z = R[6] * v[0] + R[7] * v[1] + R[8] * v[2];
    o[0] = x; o[1] = y; o[2] = z;
}
static inline void matTvec3(const double* R, const double* v, double* o) {
    double x = R[0] * v[0] + R[3] * v[1] + R[6] * v[2];
    double y = R[1] * v[0] + R[4] * v[1] + R[7] * v[2];
    double z = R[2] * v[0] + R[5] * v[1] + R[8] * v[2];
    o[0] = x; o[1] = y; o[2] = z;
}
static inline void matmul3(const double* A, const double* B, double* C) {
    double T[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) T[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
    memcpy(C, T, sizeof(T));
}
/* compose 12-vector transforms: out = a * b */
static void tcompose(const double* a, const double* b, double* out) {
    double R[9], p[3];
    matmul3(a, b, R);
    matvec3(a, b + 9, p);
    p[0] += a[9]; p[1] += a[10]; p[2] += a[11];
    memcpy(out, R, sizeof(R));
    memcpy(out + 9, p, sizeof(p));
}
static void axis_rot(const double* ax, double q, double* R) {
    double x = ax[0], y = ax[1], z = ax[2], c = cos(q), s = sin(q), C = 1 - c;
    R[0] = c + x * x * C;     R[1] = x * y * C - z * s; R[2] = x * z * C + y * s;
    R[3] = y * x * C + z * s; R[4] = c + y * y * C;     R[5] = y * z * C - x * s;
    R[6] = z * x * C - y * s; R[7] = z * y * C + x * s; R[8] = c + z * z * C;
}

/* ------------------------------------------------------------------------ */
/* kinematics  (robot_data.cpp:101-107 computeJointJacobians; :392-402)     */
/* ------------------------------------------------------------------------ */
typedef struct Kin {
    double T[ORC_MAXJ + 1][12]; /* oMi */
    double z[ORC_MAXJ + 1][3];  /* joint axis (world) */
    double pe[3];               /* task frame origin */
    double Te[12];
} Kin;

static void kin_fk(const OracleModel* m, const double* q, Kin* k) {
    static const double I12[12] = {1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0};
    memcpy(k->T[0], I12, sizeof(I12));
    for (int j = 1; j <= m->nv; ++j) {
        double base[12], M[12];
        tcompose(k->T[m->parent[j]], m->jplace[j], base);
        memcpy(M, I12, sizeof(I12));
        if (m->jtype[j] == 0) axis_rot(m->axis[j], q[j - 1], M);
        else { M[9] = m->axis[j][0] * q[j - 1]; M[10] = m->axis[j][1] * q[j - 1]; M[11] = m->axis[j][2] * q[j - 1]; }
        tcompose(base, M, k->T[j]);
        matvec3(k->T[j], m->axis[j], k->z[j]);
    }
    tcompose(k->T[m->ee_joint], m->ee_place, k->Te);
    memcpy(k->pe, k->Te + 9, 3 * sizeof(double));
}

static int is_ancestor(const OracleModel* m, int k, int j) { /* k supports j (k<=j on the path) */
    while (j > 0) { if (j == k) return 1; j = m->parent[j]; }
    return 0;
}

/* 6 x nv LWA Jacobian of a point attached to joint jid (row-major) */
static void point_jacobian(const OracleModel* m, const Kin* k, int jid, const double* pt, double* J) {
    int nv = m->nv;
    memset(J, 0, 6 * nv * sizeof(double));
    for (int a = jid; a > 0; a = m->parent[a]) {
        double c[3];
        if (m->jtype[a] == 0) {
            double r[3];
            sub3(pt, k->T[a] + 9, r);
            cross3(k->z[a], r, c);
            for (int i = 0; i < 3; ++i) { J[i * nv + a - 1] = c[i]; J[(3 + i) * nv + a - 1] = k->z[a][i]; }
        } else {
            for (int i = 0; i < 3; ++i) J[i * nv + a - 1] = k->z[a][i];
        }
    }
}

/* dJ/dq_kk of the task-frame LWA Jacobian: dJ[kk][6][nv] (getFrameJacobian-
 * TimeVariation with qdot = e_k, robot_data.cpp:544-553) */
static void frame_jacobian_dq(const OracleModel* m, const Kin* k, double* dJ /* nv*6*nv */) {
    int nv = m->nv, je = m->ee_joint;
    memset(dJ, 0, (size_t)nv * 6 * nv * sizeof(double));
    for (int kk = je; kk > 0; kk = m->parent[kk]) {
        double dpe[3] = {0, 0, 0};
        if (m->jtype[kk] == 0) { double r[3]; sub3(k->pe, k->T[kk] + 9, r); cross3(k->z[kk], r, dpe); }
        else memcpy(dpe, k->z[kk], sizeof(dpe));
        double* D = dJ + (size_t)(kk - 1) * 6 * nv;
        for (int i = je; i > 0; i = m->parent[i]) {
            double dzi[3] = {0, 0, 0}, dpi[3] = {0, 0, 0};
            int kk_moves_i = (kk != i) && is_ancestor(m, kk, i);
            if (kk_moves_i && m->jtype[kk] == 0) cross3(k->z[kk], k->z[i], dzi);
            if (kk_moves_i) {
                if (m->jtype[kk] == 0) { double r[3]; sub3(k->T[i] + 9, k->T[kk] + 9, r); cross3(k->z[kk], r, dpi); }
                else memcpy(dpi, k->z[kk], sizeof(dpi));
            }
            if (m->jtype[i] == 0) {
                double r[3], a[3], b[3], dd[3];
                sub3(k->pe, k->T[i] + 9, r);
                cross3(dzi, r, a);
                sub3(dpe, dpi, dd);
                cross3(k->z[i], dd, b);
                for (int c = 0; c < 3; ++c) { D[c * nv + i - 1] = a[c] + b[c]; D[(3 + c) * nv + i - 1] = dzi[c]; }
            } else {
                for (int c = 0; c < 3; ++c) D[c * nv + i - 1] = dzi[c];
            }
        }
    }
}

/* ------------------------------------------------------------------------ */
/* dense linear algebra                                                     */
/* ------------------------------------------------------------------------ */
/* LU determinant with partial pivoting (Eigen MatrixBase::determinant) */
static double det_lu(const double* A, int n) {
    double M[64];
    memcpy(M, A, n * n * sizeof(double));
    double det = 1;
    for (int c = 0; c < n; ++c) {
        int p = c;
        for (int r = c + 1; r < n; ++r) if (fabs(M[r * n + c]) > fabs(M[p * n + c])) p = r;
        if (M[p * n + c] == 0) return 0;
        if (p != c) { for (int j = 0; j < n; ++j) { double t = M[c * n + j]; M[c * n + j] = M[p * n + j]; M[p * n + j] = t; } det = -det; }
        det *= M[c * n + c];
        for (int r = c + 1; r < n; ++r) {
            double f = M[r * n + c] / M[c * n + c];
            for (int j = c; j < n; ++j) M[r * n + j] -= f * M[c * n + j];
        }
    }
    return det;
}

/* rank by column-pivoted Householder QR, |R_ii| > thr * max|R_ii| (Eigen COD) */
static int rank_cpqr(const double* A, int n, double thr) {
    double M[64], cn[8];
    memcpy(M, A, n * n * sizeof(double));
    double maxpiv = 0, piv[8];
    for (int k = 0; k < n; ++k) {
        for (int j = k; j < n; ++j) { double s = 0; for (int i = k; i < n; ++i) s += M[i * n + j] * M[i * n + j]; cn[j] = s; }
        int p = k;
        for (int j = k + 1; j < n; ++j) if (cn[j] > cn[p]) p = j;
        if (p != k) for (int i = 0; i < n; ++i) { double t = M[i * n + k]; M[i * n + k] = M[i * n + p]; M[i * n + p] = t; }
        double nrm = sqrt(cn[p]);
        piv[k] = nrm;
        if (nrm > maxpiv) maxpiv = nrm;
        if (nrm == 0) { for (int r = k + 1; r < n; ++r) piv[r] = 0; break; }
        double alpha = M[k * n + k] > 0 ? -nrm : nrm;
        double v[8];
        for (int i = k; i < n; ++i) v[i] = M[i * n + k];
        v[k] -= alpha;
        double vn = 0; for (int i = k; i < n; ++i) vn += v[i] * v[i];
        if (vn > 0)
            for (int j = k; j < n; ++j) {
                double s = 0; for (int i = k; i < n; ++i) s += v[i] * M[i * n + j];
                s = 2 * s / vn;
                for (int i = k; i < n; ++i) M[i * n + j] -= s * v[i];
            }
    }
    int r = 0;
    for (int k = 0; k < n; ++k) if (piv[k] > thr * maxpiv) ++r;
    return r;
}

/* Moore-Penrose inverse of the QR-truncated matrix Q_r [R11 R12] P^T: what
   Eigen's CompleteOrthogonalDecomposition::pseudoInverse() returns with the
   rank cut |R_ii| > thr * max|R_ii| (math_type_define.h:563-570).
   A is m x n (row-major), X = P W^T (W W^T)^-1 Q_r^T (n x m) with W = R[:r, :].
   m, n <= 16. */
static void pinv_qr_trunc_mn(const double* A, int m, int n, double thr, double* X) {
    double R[256], G[256], Y[256], beta[16], v0[16], cn[16];
    int perm[16];
    const int kmax = m < n ? m : n;
    memcpy(R, A, (size_t)m * n * sizeof(double));
    for (int j = 0; j < n; ++j) perm[j] = j;
    double maxpiv = 0;
    for (int k = 0; k < kmax; ++k) {
        int p = k;
        for (int j = k; j < n; ++j) {
            double s = 0;
            for (int i = k; i < m; ++i) s += R[i * n + j] * R[i * n + j];
            cn[j] = s;
            if (s > cn[p]) p = j;
        }
        if (p != k) {
            for (int i = 0; i < m; ++i) { double t = R[i * n + k]; R[i * n + k] = R[i * n + p]; R[i * n + p] = t; }
            int t = perm[k]; perm[k] = perm[p]; perm[p] = t;
            double c = cn[k]; cn[k] = cn[p]; cn[p] = c;
        }
        double nrm = sqrt(cn[k]);
        beta[k] = 0; v0[k] = 0;
        if (nrm > 0) {
            double x0 = R[k * n + k], alpha = x0 > 0 ? -nrm : nrm, w0 = x0 - alpha, vn = w0 * w0;
            for (int i = k + 1; i < m; ++i) vn += R[i * n + k] * R[i * n + k];
            double bt = vn > 0 ? 2.0 / vn : 0.0;
            for (int j = k + 1; j < n; ++j) {
                double s = w0 * R[k * n + j];
                for (int i = k + 1; i < m; ++i) s += R[i * n + k] * R[i * n + j];
                s *= bt;
                R[k * n + j] -= s * w0;
                for (int i = k + 1; i < m; ++i) R[i * n + j] -= s * R[i * n + k];
            }
            R[k * n + k] = alpha;
            beta[k] = bt; v0[k] = w0;
        }
        if (fabs(R[k * n + k]) > maxpiv) maxpiv = fabs(R[k * n + k]);
    }
    int r = 0;
    for (int k = 0; k < kmax; ++k) if (fabs(R[k * n + k]) > thr * maxpiv) ++r;
    memset(X, 0, (size_t)n * m * sizeof(double));
    if (r == 0) return;
    for (int i = 0; i < r; ++i)
        for (int j = 0; j <= i; ++j) {
            double s = 0;
            for (int k = i; k < n; ++k) s += R[i * n + k] * R[j * n + k];
            G[i * r + j] = s;
        }
    for (int j = 0; j < r; ++j) {
        double s = G[j * r + j];
        for (int k = 0; k < j; ++k) s -= G[j * r + k] * G[j * r + k];
        double d = sqrt(s > 1e-300 ? s : 1e-300);
        G[j * r + j] = d;
        for (int i = j + 1; i < r; ++i) {
            double t = G[i * r + j];
            for (int k = 0; k < j; ++k) t -= G[i * r + k] * G[j * r + k];
            G[i * r + j] = t / d;
        }
    }
    /* Y = W^T (W W^T)^-1, row c of Y: solve (G G^T) y = W[:, c] */
    for (int c = 0; c < n; ++c) {
        double* y = Y + c * r;
        for (int i = 0; i < r; ++i) y[i] = c >= i ? R[i * n + c] : 0.0;
        for (int i = 0; i < r; ++i) { double t = y[i]; for (int k = 0; k < i; ++k) t -= G[i * r + k] * y[k]; y[i] = t / G[i * r + i]; }
        for (int i = r - 1; i >= 0; --i) { double t = y[i]; for (int k = i + 1; k < r; ++k) t -= G[k * r + i] * y[k]; y[i] = t / G[i * r + i]; }
    }
    /* X[perm[c]][col] = Y[c] . (Q^T e_col)[:r] */
    for (int col = 0; col < m; ++col) {
        double u[16];
        for (int i = 0; i < m; ++i) u[i] = i == col ? 1.0 : 0.0;
        for (int k = 0; k < kmax; ++k) {
            if (beta[k] == 0) continue;
            double s = v0[k] * u[k];
            for (int i = k + 1; i < m; ++i) s += R[i * n + k] * u[i];
            s *= beta[k];
            u[k] -= s * v0[k];
            for (int i = k + 1; i < m; ++i) u[i] -= s * R[i * n + k];
        }
        for (int c = 0; c < n; ++c) {
            double s = 0;
            for (int i = 0; i < r; ++i) s += Y[c * r + i] * u[i];
            X[perm[c] * m + col] = s;
        }
    }
}
static void pinv_qr_trunc(const double* A, int n, double thr, double* X) { pinv_qr_trunc_mn(A, n, n, thr, X); }

/* Cholesky LL^T in place (lower), returns 0 on failure */
static int chol(double* A, int n) {
    for (int j = 0; j < n; ++j) {
        double s = A[j * n + j];
        for (int k = 0; k < j; ++k) s -= A[j * n + k] * A[j * n + k];
        if (!(s > 0)) return 0;
        double d = sqrt(s);
        A[j * n + j] = d;
        for (int i = j + 1; i < n; ++i) {
            double t = A[i * n + j];
            for (int k = 0; k < j; ++k) t -= A[i * n + k] * A[j * n + k];
            A[i * n + j] = t / d;
        }
    }
    return 1;
}
static void chol_solve(const double* L, int n, double* b) {
    for (int i = 0; i < n; ++i) { double t = b[i]; for (int k = 0; k < i; ++k) t -= L[i * n + k] * b[k]; b[i] = t / L[i * n + i]; }
    for (int i = n - 1; i >= 0; --i) { double t = b[i]; for (int k = i + 1; k < n; ++k) t -= L[k * n + i] * b[k]; b[i] = t / L[i * n + i]; }
}

/* DyrosMath::PinvCOD for a symmetric PSD matrix (math_type_define.h:563) */
static void pinv_cod_sym(const double* A, int n, double* X) {
    int r = rank_cpqr(A, n, 1e-6);
    if (r == n) {
        double L[64];
        memcpy(L, A, n * n * sizeof(double));
        if (chol(L, n)) {
            for (int c = 0; c < n; ++c) {
                double e[8] = {0};
                e[c] = 1;
                chol_solve(L, n, e);
                for (int i = 0; i < n; ++i) X[i * n + c] = e[i];
            }
            return;
        }
    }
    pinv_qr_trunc(A, n, 1e-6, X);
}

/* Mobile::RobotData::computeFKJacobian (src/mobile/robot_data.cpp:123-204):
 * the constant table for differential / mecanum; CasterFKJacobian (:179-204)
 * at the steer angles q[mobi_start + 2i]:
 *   J = PinvCOD(Jp~^T Jp~) Jp~^T Jq^-1                                       */
static void mobile_fk_jac(const OracleModel* m, const double* q, double J[3][8]) {
    if (m->drive != 2) { memcpy(J, m->J_mobile, sizeof(double) * 24); return; }
    int W = m->n_wheel, C = W / 2;
    double Jp[16 * 3], Jq[16 * 16], N[9], Ni[9];
    memset(Jp, 0, sizeof(Jp));
    memset(Jq, 0, sizeof(Jq));
    double r = m->wheel_radius, b = m->wheel_offset;
    for (int i = 0; i < C; ++i) {
        double phi = q[m->mobi_start + 2 * i], px = m->caster_pos[i][0], py = m->caster_pos[i][1];
        double* r0 = Jp + (2 * i) * 3;
        double* r1 = Jp + (2 * i + 1) * 3;
        r0[0] = 1; r0[1] = 0; r0[2] = -(py + b * sin(phi));
        r1[0] = 0; r1[1] = 1; r1[2] = px + b * cos(phi);
        Jq[(2 * i) * W + 2 * i] = b * sin(phi);     Jq[(2 * i) * W + 2 * i + 1] = r * cos(phi);
        Jq[(2 * i + 1) * W + 2 * i] = -b * cos(phi); Jq[(2 * i + 1) * W + 2 * i + 1] = r * sin(phi);
    }
    for (int a = 0; a < 3; ++a)
        for (int c = 0; c < 3; ++c) { double t = 0; for (int k = 0; k < W; ++k) t += Jp[k * 3 + a] * Jp[k * 3 + c]; N[a * 3 + c] = t; }
    pinv_cod_sym(N, 3, Ni);
    for (int a = 0; a < 3; ++a)
        for (int w = 0; w < 8; ++w) {
            double t = 0;
            if (w < W)
                for (int k = 0; k < W; ++k) {
                    double pk = 0;   /* (Ni Jp~^T)[a][k] */
                    for (int c = 0; c < 3; ++c) pk += Ni[a * 3 + c] * Jp[k * 3 + c];
                    t += pk * Jq[k * W + w];
                }
            J[a][w] = t;
        }
}

/* ------------------------------------------------------------------------ */
/* manipulability  (robot_data.cpp:519-553; MoMa :439-475)                  */
/* ------------------------------------------------------------------------ */
static void manip(const OracleModel* m, const Kin* k, const double* J, int c0, int nc, double* man, double* grad) {
    int nv = m->nv;
    double Jr[6 * ORC_MAXJ], A[36], Ai[36], W[ORC_MAXJ * 6];
    double* dJ = (double*)malloc((size_t)nv * 6 * nv * sizeof(double));
    for (int i = 0; i < 6; ++i) for (int c = 0; c < nc; ++c) Jr[i * nc + c] = J[i * nv + c0 + c];
    for (int i = 0; i < 6; ++i) for (int j = 0; j < 6; ++j) { double s = 0; for (int c = 0; c < nc; ++c) s += Jr[i * nc + c] * Jr[j * nc + c]; A[i * 6 + j] = s; }
    double det = det_lu(A, 6);
    *man = sqrt(det);
    pinv_cod_sym(A, 6, Ai);
    /* W = Jr^T Ai  (nc x 6) */
    for (int c = 0; c < nc; ++c) for (int j = 0; j < 6; ++j) { double s = 0; for (int i = 0; i < 6; ++i) s += Jr[i * nc + c] * Ai[i * 6 + j]; W[c * 6 + j] = s; }
    frame_jacobian_dq(m, k, dJ);
    for (int kk = 0; kk < nc; ++kk) {
        const double* D = dJ + (size_t)(c0 + kk) * 6 * nv;
        double tr = 0;
        for (int a = 0; a < 6; ++a) for (int c = 0; c < nc; ++c) tr += D[a * nv + c0 + c] * W[c * 6 + a];
        grad[kk] = *man * tr;
    }
    free(dJ);
}

/* ------------------------------------------------------------------------ */
/* narrow phase (hpp-fcl semantics, restated)                               */
/* ------------------------------------------------------------------------ */
typedef struct Shape { int type; double T[12]; double prm[3]; } Shape;

static void support(const Shape* s, const double* d, double* out) {
    if (s->type == 0) { memcpy(out, s->T + 9, 3 * sizeof(double)); return; }
    double dl[3], loc[3];
    matTvec3(s->T, d, dl);
    if (s->type == 1) {
        double r = s->prm[0], h = s->prm[1], rho = sqrt(dl[0] * dl[0] + dl[1] * dl[1]);
        double f = rho > 0 ? r / rho : 0;  /* one division (kernel: same) */
        loc[0] = f * dl[0];
        loc[1] = f * dl[1];
        loc[2] = dl[2] > 0 ? h : -h;
    } else {
        for (int i = 0; i < 3; ++i) loc[i] = dl[i] > 0 ? s->prm[i] : -s->prm[i];
    }
    matvec3(s->T, loc, out);
    out[0] += s->T[9]; out[1] += s->T[10]; out[2] += s->T[11];
}

typedef struct SV { double w[3], a[3], b[3]; } SV;

static void sup_md(const Shape* A, const Shape* B, const double* d, SV* o) {
    double nd[3] = {-d[0], -d[1], -d[2]};
    support(A, d, o->a);
    support(B, nd, o->b);
    sub3(o->a, o->b, o->w);
}

/* closest point of conv(W) to the origin by exhaustive sub-simplex search */
static int closest_simplex(SV* S, int n, double* v, double* lam_out) {
    double best = INFINITY, bl[4] = {0};
    int bmask = 0;
    /* masks holding the newest vertex S[n-1] come first; the others (the
     * previous simplex's faces, no closer than |v|: GJK appends a support
     * point only when it improves by the gap tolerance) are searched only
     * when none of the first group is valid */
    for (int mask = (1 << n) - 1; mask > 0; --mask) {
        if (mask == (1 << (n - 1)) - 1 && bmask != 0) break;
        int idx[4], k = 0;
        for (int i = 0; i < n; ++i) if (mask & (1 << i)) idx[k++] = i;
        double lam[4];
        if (k == 1) lam[0] = 1;
        else {
            double D[3][3], G[9], r[3];
            for (int i = 1; i < k; ++i) sub3(S[idx[i]].w, S[idx[0]].w, D[i - 1]);
            int d = k - 1;
            for (int i = 0; i < d; ++i) { for (int j = 0; j < d; ++j) G[i * 3 + j] = dot3(D[i], D[j]); r[i] = -dot3(D[i], S[idx[0]].w); }
            double mu[3];
            if (d == 1) { if (G[0] <= 0) continue; mu[0] = r[0] / G[0]; }
            else if (d == 2) {
                double det = G[0] * G[4] - G[1] * G[3];
                if (fabs(det) < 1e-300) continue;
                double id = 1.0 / det;
                mu[0] = (r[0] * G[4] - G[1] * r[1]) * id;
                mu[1] = (G[0] * r[1] - r[0] * G[3]) * id;
            } else {
                double a = G[0], b = G[1], c = G[2], dd = G[3], e = G[4], f = G[5], g = G[6], h = G[7], ii = G[8];
                double det = a * (e * ii - f * h) - b * (dd * ii - f * g) + c * (dd * h - e * g);
                if (fabs(det) < 1e-300) continue;
                double id = 1.0 / det;
                mu[0] = (r[0] * (e * ii - f * h) - b * (r[1] * ii - f * r[2]) + c * (r[1] * h - e * r[2])) * id;
                mu[1] = (a * (r[1] * ii - f * r[2]) - r[0] * (dd * ii - f * g) + c * (dd * r[2] - r[1] * g)) * id;
                mu[2] = (a * (e * r[2] - r[1] * h) - b * (dd * r[2] - r[1] * g) + r[0] * (dd * h - e * g)) * id;
            }
            double s = 0;
            for (int i = 0; i < d; ++i) s += mu[i];
            lam[0] = 1 - s;
            for (int i = 0; i < d; ++i) lam[i + 1] = mu[i];
            int bad = 0;
            for (int i = 0; i < k; ++i) if (lam[i] < -1e-14) bad = 1;
            if (bad) continue;
        }
        double p[3] = {0, 0, 0};
        for (int i = 0; i < k; ++i) for (int c = 0; c < 3; ++c) p[c] += lam[i] * S[idx[i]].w[c];
        double dv = dot3(p, p);
        /* a tetrahedron spans R^3, so its candidate must be the origin itself;
         * a nonzero p means a flat, ill-conditioned tetrahedron: reject it */
        if (k == 4 && dv > 1e-20) continue;
        if (bmask == 0 || dv < best - 1e-18) {
            best = dv; bmask = mask;
            memcpy(v, p, sizeof(p));
            for (int i = 0; i < k; ++i) bl[i] = lam[i];
        }
    }
    /* compact */
    SV T[4];
    int k = 0;
    for (int i = 0; i < n; ++i) if (bmask & (1 << i)) T[k++] = S[i];
    for (int i = 0; i < k; ++i) { S[i] = T[i]; lam_out[i] = bl[i]; }
    return k;
}

/* Stop tolerances (support gaps, metres).  The winning pair's witnesses are
 * refined to the exact critical point afterwards (refine_witness, D17), so
 * GJK / EPA only have to decide the argmin and land in the right basin: both
 * stop at hpp-fcl's defaults, GJKSolver gjk_tolerance and epa_tolerance 1e-6
 * (pairs whose distances lie closer than that are a tie at the reference's
 * own tolerance).  r05: GJK from 1e-9 to 1e-6 took 37 % of the GJK
 * iterations off the UR5e / FR3 bench workloads and moved no q-dot by more
 * than 7e-12 (16 384 device-dump instances each; the D17 refinement absorbs
 * the looser estimates).  Kernel twins: kGjkTol / kEpaTol in qpik_device.hpp. */
#define GJK_TOL g_gjk_tol
#define EPA_TOL 1e-6
/* study switch (tolerance census) and a GJK iteration counter,
 * counted only while a study has it on (reset = 1 zeroes and enables it,
 * reset = 0 reads and disables it): a shared atomic in the GJK loop would
 * serialise the multi-threaded CPU baseline */
static double g_gjk_tol = 1e-6;
static long long g_gjk_it;
static int g_diag_on;
void oracle_gjk_study(double tol, long long* iters, int reset) {
    if (tol > 0) g_gjk_tol = tol;
    if (iters) *iters = __atomic_load_n(&g_gjk_it, __ATOMIC_RELAXED);
    if (reset) __atomic_store_n(&g_gjk_it, 0, __ATOMIC_RELAXED);
    g_diag_on = reset != 0;
}
#define GJK_COUNT() do { if (g_diag_on) __atomic_fetch_add(&g_gjk_it, 1, __ATOMIC_RELAXED); } while (0)

/* GJK on the cores.  Returns 1 when the origin is enclosed (penetration). */
static int gjk(const Shape* A, const Shape* B, SV* S, int* ns, double* lam, double* v) {
    sub3(A->T + 9, B->T + 9, v);
    if (dot3(v, v) < 1e-24) { v[0] = 1; v[1] = 0; v[2] = 0; }
    int n = 0;
    for (int it = 0; it < 128; ++it) {
        double nv[3] = {-v[0], -v[1], -v[2]};
        SV w;
        sup_md(A, B, nv, &w);
        GJK_COUNT();
        double vv = dot3(v, v);
        if (n > 0 && vv - dot3(v, w.w) <= GJK_TOL * sqrt(vv)) break;
        int dup = 0;
        for (int i = 0; i < n; ++i) if (S[i].w[0] == w.w[0] && S[i].w[1] == w.w[1] && S[i].w[2] == w.w[2]) dup = 1;
        /* a repeated support point before the gap test passed: the simplex
         * stalled numerically.  The support in -v then tells the side: v.w <= 0
         * means the Minkowski difference reaches past the origin (overlap). */
        if (dup) { if (dot3(v, w.w) <= 0) { *ns = n; return 1; } break; }
        S[n++] = w;
        n = closest_simplex(S, n, v, lam);
        if (n == 4 || dot3(v, v) < 1e-24) { *ns = n; return 1; }
    }
    *ns = n;
    return 0;
}

/* hpp-fcl GJKSolver defaults (epa_max_vertex_num, epa_max_face_num) */
#define EPA_MAXV 64
#define EPA_MAXF 128
/* Expanding polytope with face adjacency (Bullet/libccd style): the visible
 * region is flood-filled from the closest face across shared edges, so the
 * horizon is always a single loop and the polytope stays a valid closed
 * 2-manifold even when flat features (cylinder caps, box faces) make the
 * support mapping degenerate.  Same decisions as the device version. */
typedef struct Epa {
    SV V[EPA_MAXV];
    int nv, nf, pass;
    int fv[EPA_MAXF][3], ff[EPA_MAXF][3], fe[EPA_MAXF][3], alive[EPA_MAXF];
    double fn[EPA_MAXF][3], fd[EPA_MAXF];
    int freel[EPA_MAXF];  /* recycled slots, last freed first */
    int fail, nfree;
} Epa;

static int epa_newface(Epa* E, int a, int b, int c) {
    int f;
    if (E->nfree > 0) f = E->freel[--E->nfree];
    else if (E->nf < EPA_MAXF) f = E->nf++;
    else { E->fail = 1; return -1; }
    E->fv[f][0] = a; E->fv[f][1] = b; E->fv[f][2] = c;
    E->alive[f] = 1;
    double e1[3], e2[3], nn[3];
    sub3(E->V[b].w, E->V[a].w, e1);
    sub3(E->V[c].w, E->V[a].w, e2);
    cross3(e1, e2, nn);
    double L = norm3(nn);
    if (!(L > 1e-300)) { E->fail = 1; E->alive[f] = 0; return -1; }
    for (int k = 0; k < 3; ++k) E->fn[f][k] = nn[k] / L;
    E->fd[f] = dot3(E->fn[f], E->V[a].w);
    /* the origin must stay inside (Bullet's EPA_INSIDE_EPS test): a face
     * that sees it from outside means the hull went non-convex numerically */
    if (E->fd[f] < -1e-12) { E->fail = 1; E->alive[f] = 0; return -1; }
    return f;
}
static void epa_bind(Epa* E, int f0, int e0, int f1, int e1) {
    E->ff[f0][e0] = f1; E->fe[f0][e0] = e1;
    E->ff[f1][e1] = f0; E->fe[f1][e1] = e0;
}
/* One expansion step from face `best` by the new vertex wi (btGjkEpa2::expand's
 * result, in the order the task kernel's wave form produces it -- kernel twin:
 * epa_grow_canon / the wave form in task_stage.hpp):
 *  - the removed region C is the connected component of `best` among the
 *    alive faces that see w (exactly the faces the recursive flood fill from
 *    `best` visits and kills);
 *  - the horizon is every edge (c, e) of a face c in C whose neighbour is not
 *    in C; it must be a single simple cycle (each vertex starts and ends at
 *    most one edge, one cycle through all of them) of >= 3 edges;
 *  - the new faces (start, end, w) of the horizon edges take slots in cycle
 *    order from the edge of smallest key 3c + e: the free list first (last
 *    freed first), then fresh slots;
 *  - every new face passes epa_newface's tests (non-degenerate, origin
 *    inside, no closer than `best`);
 *  - the faces of C are freed in ascending slot order, `best` last.
 * Any failure leaves the polytope as it was.  Returns 1 when committed. */
static int epa_grow_canon(Epa* E, int wi, int best) {
    static __thread int inC[EPA_MAXF], hc[EPA_MAXV], he[EPA_MAXV], outv[EPA_MAXV], inv[EPA_MAXV], ord[EPA_MAXV];
    static __thread int slot[EPA_MAXV];
    const double* w = E->V[wi].w;
    for (int f = 0; f < E->nf; ++f) inC[f] = 0;
    inC[best] = 1;
    for (int grown = 1; grown;) {  /* component of best among visible faces */
        grown = 0;
        for (int f = 0; f < E->nf; ++f) {
            if (inC[f] || !E->alive[f] || dot3(E->fn[f], w) - E->fd[f] < -1e-12) continue;
            for (int e = 0; e < 3; ++e)
                if (inC[E->ff[f][e]]) { inC[f] = 1; grown = 1; break; }
        }
    }
    int H = 0;
    for (int v = 0; v < EPA_MAXV; ++v) { outv[v] = -1; inv[v] = -1; }
    for (int c = 0; c < E->nf; ++c) {
        if (!inC[c]) continue;
        for (int e = 0; e < 3; ++e) {
            if (inC[E->ff[c][e]]) continue;
            if (H >= EPA_MAXV) return 0;
            const int a = E->fv[c][e], b = E->fv[c][e == 2 ? 0 : e + 1];
            if (outv[a] >= 0 || inv[b] >= 0) return 0;  /* not a simple cycle */
            outv[a] = H; inv[b] = H;
            hc[H] = c; he[H] = e; ++H;
        }
    }
    if (H < 3) return 0;
    /* cycle order from edge 0 (smallest key: c ascending, then e) */
    int cur = 0;
    for (int k = 0; k < H; ++k) {
        if (cur < 0 || (k > 0 && cur == 0)) return 0;
        ord[k] = cur;
        cur = outv[E->fv[hc[cur]][he[cur] == 2 ? 0 : he[cur] + 1]];
    }
    if (cur != 0) return 0;
    if (H > E->nfree + (EPA_MAXF - E->nf)) return 0;
    const double fdmin = E->fd[best];
    for (int k = 0; k < H; ++k) {
        const int f = k < E->nfree ? E->freel[E->nfree - 1 - k] : E->nf + (k - E->nfree);
        const int h = ord[k], c = hc[h], e = he[h];
        const int a = E->fv[c][e], b = E->fv[c][e == 2 ? 0 : e + 1];
        double e1[3], e2[3], nn[3], fn[3];
        sub3(E->V[b].w, E->V[a].w, e1);
        sub3(w, E->V[a].w, e2);
        cross3(e1, e2, nn);
        const double L = norm3(nn);
        if (!(L > 1e-300)) return 0;
        for (int i = 0; i < 3; ++i) fn[i] = nn[i] / L;
        const double fd = dot3(fn, E->V[a].w);
        if (fd < -1e-12 || fd < fdmin - 1e-12) return 0;
        slot[k] = f;
    }
    /* commit */
    for (int k = 0; k < H; ++k) {
        const int f = slot[k], h = ord[k], c = hc[h], e = he[h];
        const int a = E->fv[c][e], b = E->fv[c][e == 2 ? 0 : e + 1];
        double e1[3], e2[3], nn[3];
        sub3(E->V[b].w, E->V[a].w, e1);
        sub3(w, E->V[a].w, e2);
        cross3(e1, e2, nn);
        const double L = norm3(nn);
        for (int i = 0; i < 3; ++i) E->fn[f][i] = nn[i] / L;
        E->fd[f] = dot3(E->fn[f], E->V[a].w);
        E->fv[f][0] = a; E->fv[f][1] = b; E->fv[f][2] = wi;
        /* edge 0 faces the outer neighbour, edge 1 the next new face, edge 2 the previous */
        const int g = E->ff[c][e], ge = E->fe[c][e];
        E->ff[f][0] = g; E->fe[f][0] = ge;
        E->ff[g][ge] = f; E->fe[g][ge] = 0;
        E->ff[f][1] = slot[(k + 1) % H]; E->fe[f][1] = 2;
        E->ff[f][2] = slot[(k + H - 1) % H]; E->fe[f][2] = 1;
    }
    const int nf0 = E->nf, nfree0 = E->nfree > H ? E->nfree - H : 0;
    if (H > E->nfree) E->nf += H - E->nfree;
    E->nfree = nfree0;
    for (int c = 0; c < nf0; ++c)
        if (inC[c] && c != best) { E->alive[c] = 0; E->freel[E->nfree++] = c; }
    E->alive[best] = 0;
    E->freel[E->nfree++] = best;
    for (int k = 0; k < H; ++k) E->alive[slot[k]] = 1;
    return 1;
}

/* EPA census (diagnostic, tools/polish_census.py --epa): calls, growth steps,
 * calls and steps of pairs that did not end up as the argmin */
static long long g_ec[8];
static int g_ec_on;  /* on between oracle_epa_census(.., 1) and (.., 0): no shared atomics otherwise */
static __thread int g_epa_steps;
void oracle_epa_census(long long* out, int reset) {
    if (out) for (int i = 0; i < 8; ++i) out[i] = __atomic_load_n(&g_ec[i], __ATOMIC_RELAXED);
    if (reset) for (int i = 0; i < 8; ++i) __atomic_store_n(&g_ec[i], 0, __ATOMIC_RELAXED);
    g_ec_on = reset != 0;
}
/* EPA step histogram (diagnostic): [0..7] calls by steps 0-7, 8-15, 16-23,
 * 24-31, 32-39, 40-47, 48-59, 60+; [8..11] how they ended: support gap,
 * vertex cap, duplicate support point, rolled-back growth */
static long long g_eh[12];
static int g_eh_on;  /* on between oracle_epa_hist(.., 1) and oracle_epa_hist(.., 0) */
void oracle_epa_hist(long long* out, int reset) {
    if (out) for (int i = 0; i < 12; ++i) out[i] = __atomic_load_n(&g_eh[i], __ATOMIC_RELAXED);
    if (reset) for (int i = 0; i < 12; ++i) __atomic_store_n(&g_eh[i], 0, __ATOMIC_RELAXED);
    g_eh_on = reset != 0;
}
static void epa_hist_add(int steps, int why) {
    if (!g_eh_on) return;
    const int b = steps < 48 ? steps / 8 : (steps < 60 ? 6 : 7);
    __atomic_fetch_add(&g_eh[b], 1, __ATOMIC_RELAXED);
    __atomic_fetch_add(&g_eh[8 + why], 1, __ATOMIC_RELAXED);
}
static double epa(const Shape* A, const Shape* B, SV* S, int ns, double* pA, double* pB) {
    static const double dirs[6][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {-1, 0, 0}, {0, -1, 0}, {0, 0, -1}};
    static __thread Epa E;
    E.nv = ns; E.nf = 0; E.fail = 0; E.nfree = 0;
    for (int i = 0; i < ns; ++i) E.V[i] = S[i];
    for (int di = 0; di < 6 && E.nv < 4; ++di) {
        SV w;
        sup_md(A, B, dirs[di], &w);
        int ok = 1;
        for (int i = 0; i < E.nv; ++i) { double d[3]; sub3(w.w, E.V[i].w, d); if (norm3(d) <= 1e-12) ok = 0; }
        if (ok) E.V[E.nv++] = w;
    }
    /* orient the tetrahedron so that face (0,1,2) looks away from vertex 3 */
    {
        double e1[3], e2[3], nn[3], o[3];
        sub3(E.V[1].w, E.V[0].w, e1);
        sub3(E.V[2].w, E.V[0].w, e2);
        cross3(e1, e2, nn);
        sub3(E.V[3].w, E.V[0].w, o);
        if (dot3(nn, o) > 0) { SV t = E.V[0]; E.V[0] = E.V[1]; E.V[1] = t; }
    }
    int t0 = epa_newface(&E, 0, 1, 2), t1 = epa_newface(&E, 1, 0, 3), t2 = epa_newface(&E, 2, 1, 3),
        t3 = epa_newface(&E, 0, 2, 3);
    int best = 0;
    if (!E.fail) {
        epa_bind(&E, t0, 0, t1, 0); epa_bind(&E, t0, 1, t2, 0); epa_bind(&E, t0, 2, t3, 0);
        epa_bind(&E, t1, 1, t3, 2); epa_bind(&E, t1, 2, t2, 1); epa_bind(&E, t2, 2, t3, 1);
        int nst = 0, why = 0;
        for (int it = 0; it < 255; ++it) {
            best = -1;
            double bd = INFINITY;
            for (int f = 0; f < E.nf; ++f)
                if (E.alive[f] && E.fd[f] < bd) { bd = E.fd[f]; best = f; }
            SV w;
            sup_md(A, B, E.fn[best], &w);
            if (dot3(E.fn[best], w.w) - E.fd[best] <= EPA_TOL || E.nv >= EPA_MAXV) {
                why = E.nv >= EPA_MAXV && dot3(E.fn[best], w.w) - E.fd[best] > EPA_TOL;
                break;
            }
            int dupv = 0;
            for (int i = 0; i < E.nv; ++i) {
                double d[3];
                sub3(w.w, E.V[i].w, d);
                if (fabs(d[0]) <= 1e-14 && fabs(d[1]) <= 1e-14 && fabs(d[2]) <= 1e-14) dupv = 1;
            }
            if (dupv) { why = 2; break; }
            int wi = E.nv;
            E.V[E.nv++] = w;
            ++g_epa_steps;
            ++nst;
            if (!epa_grow_canon(&E, wi, best)) {  /* rolled back: the last closed polytope */
                E.nv--;
                why = 3;
                break;
            }
        }
        epa_hist_add(nst, why);
    }
    double bd = INFINITY;
    best = 0;
    for (int f = 0; f < E.nf; ++f)
        if (E.alive[f] && E.fd[f] < bd) { bd = E.fd[f]; best = f; }
    const double *a = E.V[E.fv[best][0]].w, *b = E.V[E.fv[best][1]].w, *c = E.V[E.fv[best][2]].w;
    double p[3] = {E.fn[best][0] * bd, E.fn[best][1] * bd, E.fn[best][2] * bd};
    double v0[3], v1[3], v2[3];
    sub3(b, a, v0); sub3(c, a, v1); sub3(p, a, v2);
    double d00 = dot3(v0, v0), d01 = dot3(v0, v1), d11 = dot3(v1, v1), d20 = dot3(v2, v0), d21 = dot3(v2, v1);
    double den = d00 * d11 - d01 * d01;
    double l1 = (d11 * d20 - d01 * d21) / den, l2 = (d00 * d21 - d01 * d20) / den, l0 = 1 - l1 - l2;
    for (int k = 0; k < 3; ++k) {
        pA[k] = l0 * E.V[E.fv[best][0]].a[k] + l1 * E.V[E.fv[best][1]].a[k] + l2 * E.V[E.fv[best][2]].a[k];
        pB[k] = l0 * E.V[E.fv[best][0]].b[k] + l1 * E.V[E.fv[best][1]].b[k] + l2 * E.V[E.fv[best][2]].b[k];
    }
    return -bd;
}

/* signed distance and closest surface point of a solid cylinder / box */
static double point_cylinder(const double* c, const Shape* s, double* qw) {
    double d[3], loc[3], q[3];
    sub3(c, s->T + 9, d);
    matTvec3(s->T, d, loc);
    double r = s->prm[0], h = s->prm[1], rho = sqrt(loc[0] * loc[0] + loc[1] * loc[1]), sd;
    memcpy(q, loc, sizeof(q));
    if (!(rho <= r && fabs(loc[2]) <= h)) {
        if (rho > r) { q[0] = loc[0] * r / rho; q[1] = loc[1] * r / rho; }
        q[2] = loc[2] < -h ? -h : (loc[2] > h ? h : loc[2]);
        double dq[3] = {loc[0] - q[0], loc[1] - q[1], loc[2] - q[2]};
        sd = norm3(dq);
    } else {
        double dside = r - rho, dtop = h - loc[2], dbot = h + loc[2];
        if (dside <= dtop && dside <= dbot) {
            if (rho > 0) { q[0] = loc[0] * r / rho; q[1] = loc[1] * r / rho; } else { q[0] = r; q[1] = 0; }
            sd = -dside;
        } else if (dtop <= dbot) { q[2] = h; sd = -dtop; }
        else { q[2] = -h; sd = -dbot; }
    }
    matvec3(s->T, q, qw);
    qw[0] += s->T[9]; qw[1] += s->T[10]; qw[2] += s->T[11];
    return sd;
}
static double point_box(const double* c, const Shape* s, double* qw) {
    double d[3], loc[3], q[3], sd;
    sub3(c, s->T + 9, d);
    matTvec3(s->T, d, loc);
    int inside = 1;
    for (int i = 0; i < 3; ++i) if (fabs(loc[i]) > s->prm[i]) inside = 0;
    memcpy(q, loc, sizeof(q));
    if (!inside) {
        for (int i = 0; i < 3; ++i) q[i] = loc[i] < -s->prm[i] ? -s->prm[i] : (loc[i] > s->prm[i] ? s->prm[i] : loc[i]);
        double dq[3] = {loc[0] - q[0], loc[1] - q[1], loc[2] - q[2]};
        sd = norm3(dq);
    } else {
        int a = 0;
        double g = s->prm[0] - fabs(loc[0]);
        for (int i = 1; i < 3; ++i) { double gi = s->prm[i] - fabs(loc[i]); if (gi < g) { g = gi; a = i; } }
        q[a] = loc[a] >= 0 ? s->prm[a] : -s->prm[a];
        sd = -g;
    }
    matvec3(s->T, q, qw);
    qw[0] += s->T[9]; qw[1] += s->T[10]; qw[2] += s->T[11];
    return sd;
}

/* Cylinder/cylinder side-to-side closed form: when the closest
 * points of the two axis segments are interior to both, the connecting line
 * is normal to both axes and the capsule bound is attained -- the exact
 * distance hpp-fcl's GJK (robot_data.cpp:424-494 -> fcl::distance) converges
 * to within its tolerance.  Separated, non-parallel pairs only; kernel twin:
 * cyl_cyl_side in qpik_device.hpp. */
static int cyl_cyl_side(const Shape* A, const Shape* B, double* d, double* pA, double* pB) {
    const double ua[3] = {A->T[2], A->T[5], A->T[8]}, ub[3] = {B->T[2], B->T[5], B->T[8]};
    double p1[3], p2[3], d1[3], d2[3], r[3];
    for (int i = 0; i < 3; ++i) {
        p1[i] = A->T[9 + i] - A->prm[1] * ua[i];
        p2[i] = B->T[9 + i] - B->prm[1] * ub[i];
        d1[i] = (2.0 * A->prm[1]) * ua[i];
        d2[i] = (2.0 * B->prm[1]) * ub[i];
        r[i] = p1[i] - p2[i];
    }
    const double a = dot3(d1, d1), e = dot3(d2, d2), b = dot3(d1, d2), c = dot3(d1, r), f = dot3(d2, r);
    const double den = a * e - b * b;
    if (!(den > 1e-12 * a * e)) return 0;
    const double s = (b * f - c * e) / den, t = (a * f - b * c) / den;
    if (!(s > 0.0 && s < 1.0 && t > 0.0 && t < 1.0)) return 0;
    double c1[3], c2[3], n[3];
    for (int i = 0; i < 3; ++i) { c1[i] = p1[i] + s * d1[i]; c2[i] = p2[i] + t * d2[i]; n[i] = c2[i] - c1[i]; }
    const double L = norm3(n), dd = L - A->prm[0] - B->prm[0];
    if (!(dd > 0.0)) return 0;
    for (int i = 0; i < 3; ++i) {
        n[i] = (1.0 / L) * n[i];
        pA[i] = c1[i] + A->prm[0] * n[i];
        pB[i] = c2[i] - B->prm[0] * n[i];
    }
    *d = dd;
    return 1;
}

/* ------------------------------------------------------------------------
 * Witness refinement.  GJK's witness points converge only to
 * ~sqrt(gap) and EPA's to its vertex cap, so two implementations whose
 * iterations differ by rounding return witnesses up to ~1e-5 apart, and the
 * gradient n^T (J_B(pB) - J_A(pA)) with n = (pB - pA)/|pB - pA|
 * (robot_data.cpp:476-494) inherits the difference.  The exact witnesses are
 * a critical point of |X_A(u_A) - X_B(u_B)|^2 over the surface features the
 * approximate witnesses lie on -- cylinder side (theta, z), cap (x, y), rim
 * (theta); box face / edge / vertex (the free coordinates) -- and Newton
 * converges to it quadratically from the GJK / EPA estimate (the same point
 * from any nearby start).  Accepted only when the solution lies inside its
 * features, n* = (pB - pA) / sd lies in A's normal cone and -n* in B's, and
 * sd moves by at most 1e-6; otherwise the GJK / EPA witnesses stay (parallel
 * flat features: the witnesses are not unique).  Kernel twin: refine_witness
 * in qpik_device.hpp (same features, rules and tolerances).
 * ------------------------------------------------------------------------ */
enum { FT_SIDE = 0, FT_CAP = 1, FT_RIM = 2, FT_BOX = 3 };
typedef struct Feat { int kind; double s; int fix[3]; } Feat;  /* box: fix[i] = 0 free, +-1 face sign */

#define RW_TAU 1e-4       /* feature classification tolerance on the GJK / EPA witness  */
#define RW_PIVOT 1e-9     /* smallest Newton pivot (unit-speed parameters): else degenerate */
#define RW_STEP 1e-12     /* Newton stops after a step this small                        */
#define RW_CONE 1e-9      /* normal-cone slack                                           */
#define RW_DMOVE 1e-5     /* largest accepted change of the signed distance (EPA gap 1e-6) */

static void rw_classify(const Shape* s, const double* x, Feat* f) {
    if (s->type == 1) {
        const double r = s->prm[0], h = s->prm[1], rho = sqrt(x[0] * x[0] + x[1] * x[1]);
        f->s = x[2] > 0 ? 1.0 : -1.0;
        if (fabs(x[2]) > h - RW_TAU && rho > r - RW_TAU) f->kind = FT_RIM;
        else if (fabs(x[2]) > h - RW_TAU) f->kind = FT_CAP;
        else f->kind = FT_SIDE;
        return;
    }
    f->kind = FT_BOX;
    int any = 0, im = 0;
    double best = -1;
    for (int i = 0; i < 3; ++i) {
        f->fix[i] = fabs(x[i]) > s->prm[i] - RW_TAU ? (x[i] > 0 ? 1 : -1) : 0;
        any |= f->fix[i] != 0;
        const double t = fabs(x[i]) / s->prm[i];
        if (t > best) { best = t; im = i; }
    }
    if (!any) f->fix[im] = x[im] > 0 ? 1 : -1;
}
/* parameters of feature f at the local point x */
static int rw_params(const Shape* s, const Feat* f, const double* x, double* u) {
    switch (f->kind) {
    case FT_SIDE: u[0] = atan2(x[1], x[0]); u[1] = x[2]; return 2;
    case FT_RIM: u[0] = atan2(x[1], x[0]); return 1;
    case FT_CAP: u[0] = x[0]; u[1] = x[1]; return 2;
    default: {
        int k = 0;
        for (int i = 0; i < 3; ++i) if (!f->fix[i]) u[k++] = x[i];
        (void)s;
        return k;
    }
    }
}
/* world point, unit-speed tangents t[k] and curvature vectors c[k] (theta:
 * arc-length derivatives; all other parameters are linear) */
static void rw_eval(const Shape* s, const Feat* f, const double* u, double* X, double t[2][3], double c[2][3]) {
    double x[3], tl[2][3] = {{0, 0, 0}, {0, 0, 0}}, cl[2][3] = {{0, 0, 0}, {0, 0, 0}};
    int k = 0;
    if (f->kind == FT_SIDE || f->kind == FT_RIM) {
        const double r = s->prm[0], cs = cos(u[0]), sn = sin(u[0]);
        x[0] = r * cs; x[1] = r * sn; x[2] = f->kind == FT_SIDE ? u[1] : f->s * s->prm[1];
        tl[0][0] = -sn; tl[0][1] = cs;
        cl[0][0] = -cs / r; cl[0][1] = -sn / r;
        if (f->kind == FT_SIDE) tl[1][2] = 1;
        k = f->kind == FT_SIDE ? 2 : 1;
    } else if (f->kind == FT_CAP) {
        x[0] = u[0]; x[1] = u[1]; x[2] = f->s * s->prm[1];
        tl[0][0] = 1; tl[1][1] = 1;
        k = 2;
    } else {
        for (int i = 0; i < 3; ++i) {
            if (f->fix[i]) { x[i] = f->fix[i] * s->prm[i]; continue; }
            x[i] = u[k];
            tl[k][i] = 1;
            ++k;
        }
    }
    matvec3(s->T, x, X);
    X[0] += s->T[9]; X[1] += s->T[10]; X[2] += s->T[11];
    for (int j = 0; j < k; ++j) { matvec3(s->T, tl[j], t[j]); matvec3(s->T, cl[j], c[j]); }
}
/* theta parameters move by the arc-length step / r */
static void rw_step(const Shape* s, const Feat* f, double* u, const double* du) {
    if (f->kind == FT_SIDE || f->kind == FT_RIM) {
        u[0] += du[0] / s->prm[0];
        if (f->kind == FT_SIDE) u[1] += du[1];
    } else {
        const int k = f->kind == FT_CAP ? 2 : (!f->fix[0]) + (!f->fix[1]) + (!f->fix[2]);
        for (int j = 0; j < k; ++j) u[j] += du[j];
    }
}
/* Newton on grad |X_A - X_B|^2 = 0.  Returns 1 converged, 0 degenerate / not converged. */
static int rw_newton(const Shape* A, const Feat* fA, double* uA, int mA, const Shape* B, const Feat* fB, double* uB,
                     int mB, double* XA, double* XB) {
    const int m = mA + mB;
    for (int it = 0; it < 20; ++it) {
        double tA[2][3], cA[2][3], tB[2][3], cB[2][3], D[3], J[4][3], H[4][5];
        rw_eval(A, fA, uA, XA, tA, cA);
        rw_eval(B, fB, uB, XB, tB, cB);
        sub3(XA, XB, D);
        if (m == 0) return 1;
        for (int i = 0; i < mA; ++i) memcpy(J[i], tA[i], sizeof(J[i]));
        for (int i = 0; i < mB; ++i) for (int c = 0; c < 3; ++c) J[mA + i][c] = -tB[i][c];
        for (int i = 0; i < m; ++i) {
            for (int j = 0; j < m; ++j) H[i][j] = dot3(J[i], J[j]);
            H[i][m] = -dot3(J[i], D);
        }
        H[0][0] += mA > 0 ? dot3(D, cA[0]) : -dot3(D, cB[0]);   /* theta curvature terms (index 0 only) */
        if (mA > 0 && mB > 0) H[mA][mA] -= dot3(D, cB[0]);
        /* Gaussian elimination, partial pivoting */
        for (int c = 0; c < m; ++c) {
            int p = c;
            for (int r = c + 1; r < m; ++r) if (fabs(H[r][c]) > fabs(H[p][c])) p = r;
            if (!(fabs(H[p][c]) > RW_PIVOT)) return 0;
            if (p != c) for (int j = 0; j <= m; ++j) { const double t = H[c][j]; H[c][j] = H[p][j]; H[p][j] = t; }
            for (int r = c + 1; r < m; ++r) {
                const double g = H[r][c] / H[c][c];
                for (int j = c; j <= m; ++j) H[r][j] -= g * H[c][j];
            }
        }
        double du[4], mx = 0;
        for (int r = m - 1; r >= 0; --r) {
            double t = H[r][m];
            for (int j = r + 1; j < m; ++j) t -= H[r][j] * du[j];
            du[r] = t / H[r][r];
            mx = fmax(mx, fabs(du[r]));
        }
        rw_step(A, fA, uA, du);
        rw_step(B, fB, uB, du + mA);
        if (mx <= RW_STEP) {
            rw_eval(A, fA, uA, XA, tA, cA);
            rw_eval(B, fB, uB, XB, tB, cB);
            return 1;
        }
    }
    return 0;
}
/* Outside the feature's domain: move to the bounding feature (returns 1). */
static int rw_domain(const Shape* s, Feat* f, const double* u) {
    if (f->kind == FT_SIDE && fabs(u[1]) > s->prm[1]) { f->kind = FT_RIM; f->s = u[1] > 0 ? 1 : -1; return 1; }
    if (f->kind == FT_CAP && u[0] * u[0] + u[1] * u[1] > s->prm[0] * s->prm[0]) { f->kind = FT_RIM; return 1; }
    if (f->kind == FT_BOX) {
        int k = 0;
        for (int i = 0; i < 3; ++i) {
            if (f->fix[i]) continue;
            if (fabs(u[k]) > s->prm[i]) { f->fix[i] = u[k] > 0 ? 1 : -1; return 1; }
            ++k;
        }
    }
    return 0;
}
/* The outward normal nrm must lie in the normal cone of feature f at u.
 * Returns -1 when it cannot (refinement fails), 1 when the feature moves to a
 * neighbour (rim -> cap / side, box face -> edge ...), 0 when it holds. */
static int rw_cone(const Shape* s, Feat* f, const double* u, const double* nrm) {
    const double ax[3] = {s->T[2], s->T[5], s->T[8]};
    if (f->kind == FT_BOX) {
        for (int i = 0; i < 3; ++i) {
            if (!f->fix[i]) continue;
            const double e[3] = {s->T[i], s->T[3 + i], s->T[6 + i]};
            if (f->fix[i] * dot3(nrm, e) < -RW_CONE) {
                if ((f->fix[0] != 0) + (f->fix[1] != 0) + (f->fix[2] != 0) == 1) return -1;  /* no face left */
                f->fix[i] = 0;
                return 1;
            }
        }
        return 0;
    }
    if (f->kind == FT_CAP) return f->s * dot3(nrm, ax) > 0 ? 0 : -1;
    const double rl[3] = {cos(u[0]), sin(u[0]), 0};
    double rad[3];
    matvec3(s->T, rl, rad);
    const double a = dot3(nrm, rad), b = f->s * dot3(nrm, ax);
    if (f->kind == FT_SIDE) return a > 0 ? 0 : -1;
    if (a < -RW_CONE) { f->kind = FT_CAP; return 1; }
    if (b < -RW_CONE) { f->kind = FT_SIDE; return 1; }
    return 0;
}
/* feature parameters at the world point X */
static int rw_reparam(const Shape* s, const Feat* f, const double* X, double* u) {
    double t[3], x[3];
    sub3(X, s->T + 9, t);
    matTvec3(s->T, t, x);
    return rw_params(s, f, x, u);
}
static int refine_witness(const Shape* A, const Shape* B, double* d, double* pA, double* pB) {
    Feat fA, fB;
    double xA[3], xB[3], t[3], uA[2], uB[2];
    sub3(pA, A->T + 9, t); matTvec3(A->T, t, xA);
    sub3(pB, B->T + 9, t); matTvec3(B->T, t, xB);
    rw_classify(A, xA, &fA);
    rw_classify(B, xB, &fB);
    int mA = rw_params(A, &fA, xA, uA), mB = rw_params(B, &fB, xB, uB);
    const double sgn = *d < 0 ? -1.0 : 1.0;
    for (int round = 0; round < 4; ++round) {
        double XA[3], XB[3], D[3], n[3], nb[3];
        if (!rw_newton(A, &fA, uA, mA, B, &fB, uB, mB, XA, XB)) return 0;
        int ca = rw_domain(A, &fA, uA), cb = rw_domain(B, &fB, uB);
        if (!ca && !cb) {
            sub3(XB, XA, D);
            const double L = norm3(D);
            if (!(L > 1e-12)) return 0;
            const double sd = sgn * L;
            for (int c = 0; c < 3; ++c) { n[c] = D[c] / sd; nb[c] = -n[c]; }
            ca = rw_cone(A, &fA, uA, n);
            cb = rw_cone(B, &fB, uB, nb);
            if (ca < 0 || cb < 0) return 0;
            if (!ca && !cb) {
                if (!(fabs(sd - *d) <= RW_DMOVE)) return 0;
                *d = sd;
                memcpy(pA, XA, sizeof(XA));
                memcpy(pB, XB, sizeof(XB));
                return 1;
            }
        }
        mA = rw_reparam(A, &fA, XA, uA);
        mB = rw_reparam(B, &fB, XB, uB);
    }
    return 0;
}

/* signed distance and witnesses of one pair; *how: 0 closed form (sphere
 * pairs, cylinder sides), 1 GJK, 2 EPA -- the latter two are what
 * refine_witness sharpens */
static double shape_distance(const Shape* A, const Shape* B, double* pA, double* pB, int* how) {
    *how = 0;
    if (A->type == 0 && B->type == 0) {
        double v[3];
        sub3(B->T + 9, A->T + 9, v);
        double L = norm3(v), n[3] = {1, 0, 0};
        if (L > 0) { n[0] = v[0] / L; n[1] = v[1] / L; n[2] = v[2] / L; }
        for (int i = 0; i < 3; ++i) { pA[i] = A->T[9 + i] + A->prm[0] * n[i]; pB[i] = B->T[9 + i] - B->prm[0] * n[i]; }
        return L - A->prm[0] - B->prm[0];
    }
    if (A->type == 0 || B->type == 0) {
        int flip = B->type == 0;
        const Shape *s = flip ? B : A, *o = flip ? A : B;
        const double* c = s->T + 9;
        double q[3], sd = o->type == 1 ? point_cylinder(c, o, q) : point_box(c, o, q);
        double u[3];
        sub3(q, c, u);
        double L = norm3(u), n[3] = {1, 0, 0};
        if (L > 0) { n[0] = u[0] / L; n[1] = u[1] / L; n[2] = u[2] / L; }
        if (sd < 0) { n[0] = -n[0]; n[1] = -n[1]; n[2] = -n[2]; }
        double ps[3] = {c[0] + s->prm[0] * n[0], c[1] + s->prm[0] * n[1], c[2] + s->prm[0] * n[2]};
        if (flip) { memcpy(pA, q, sizeof(q)); memcpy(pB, ps, sizeof(ps)); }
        else { memcpy(pA, ps, sizeof(ps)); memcpy(pB, q, sizeof(q)); }
        return sd - s->prm[0];
    }
    double dside;
    if (A->type == 1 && B->type == 1 && cyl_cyl_side(A, B, &dside, pA, pB)) return dside;
    SV S[4];
    int ns;
    double lam[4], v[3];
    if (gjk(A, B, S, &ns, lam, v)) { *how = 2; return epa(A, B, S, ns, pA, pB); }
    *how = 1;
    for (int c = 0; c < 3; ++c) {
        pA[c] = 0; pB[c] = 0;
        for (int i = 0; i < ns; ++i) { pA[c] += lam[i] * S[i].a[c]; pB[c] += lam[i] * S[i].b[c]; }
    }
    double d[3];
    sub3(pA, pB, d);
    return norm3(d);
}

static void make_shape(const OracleModel* m, const Kin* k, int g, Shape* s) {
    s->type = m->gtype[g];
    tcompose(k->T[m->gparent[g]], m->gplace[g], s->T);
    memcpy(s->prm, m->gparam[g], sizeof(s->prm));
}

/* RobotData::getMinDistance(true,false,false)  robot_data.cpp:424-494 */
static void min_distance_w(const OracleModel* m, const Kin* k, double* dist, double* grad, int* pair_out,
                           double* wA, double* wB);
static void min_distance(const OracleModel* m, const Kin* k, double* dist, double* grad, int* pair_out) {
    double wA[3], wB[3];
    min_distance_w(m, k, dist, grad, pair_out, wA, wB);
}
/* ---- the kernel's pruned narrow phase (FLOP count; same argmin) ---------- */
/* Segment / segment closest points (the kernel's seg_seg_dist). */
static double seg_seg(const double* p1, const double* q1, const double* p2, const double* q2, double* c1, double* c2) {
    double d1[3], d2[3], r[3];
    sub3(q1, p1, d1); sub3(q2, p2, d2); sub3(p1, p2, r);
    const double a = dot3(d1, d1), e = dot3(d2, d2), f = dot3(d2, r);
    double s, t;
    if (a <= 1e-30 && e <= 1e-30) { s = 0; t = 0; }
    else if (a <= 1e-30) { s = 0; t = fmin(fmax(f / e, 0.0), 1.0); }
    else {
        const double c = dot3(d1, r);
        if (e <= 1e-30) { t = 0; s = fmin(fmax(-c / a, 0.0), 1.0); }
        else {
            const double b = dot3(d1, d2), den = a * e - b * b;
            s = den > 0 ? fmin(fmax((b * f - c * e) / den, 0.0), 1.0) : 0.0;
            t = (b * s + f) / e;
            if (t < 0) { t = 0; s = fmin(fmax(-c / a, 0.0), 1.0); }
            else if (t > 1) { t = 1; s = fmin(fmax((b - c) / a, 0.0), 1.0); }
        }
    }
    double dd[3];
    for (int i = 0; i < 3; ++i) { c1[i] = p1[i] + s * d1[i]; c2[i] = p2[i] + t * d2[i]; dd[i] = c1[i] - c2[i]; }
    return norm3(dd);
}
/* Swept-core lower bound of the signed distance raised to the separating-axis
 * value along the cores' closest-point direction (kernel: pair_lower_bound). */
static double pair_lower_bound(const Shape* A, const Shape* B) {
    double a0[3], a1[3], b0[3], b1[3], c1[3], c2[3];
    const Shape* S2[2] = {A, B};
    double* ends[2][2] = {{a0, a1}, {b0, b1}};
    double rad[2];
    for (int k = 0; k < 2; ++k) {
        const Shape* s = S2[k];
        for (int i = 0; i < 3; ++i) { ends[k][0][i] = s->T[9 + i]; ends[k][1][i] = s->T[9 + i]; }
        if (s->type == 1) {
            const double ax[3] = {s->T[2], s->T[5], s->T[8]};
            for (int i = 0; i < 3; ++i) { ends[k][0][i] -= s->prm[1] * ax[i]; ends[k][1][i] += s->prm[1] * ax[i]; }
            rad[k] = s->prm[0];
        } else if (s->type == 2) {
            rad[k] = sqrt(s->prm[0] * s->prm[0] + s->prm[1] * s->prm[1] + s->prm[2] * s->prm[2]);
        } else {
            rad[k] = s->prm[0];
        }
    }
    const double L = seg_seg(a0, a1, b0, b1, c1, c2), pd = L - rad[0] - rad[1];
    if (!(L > 1e-12)) return pd;
    double n[3], mn[3], sa[3], sb[3];
    for (int i = 0; i < 3; ++i) { n[i] = (c2[i] - c1[i]) / L; mn[i] = -n[i]; }
    support(A, n, sa);
    support(B, mn, sb);
    return fmax(pd, dot3(n, sb) - dot3(n, sa));
}
/* GJK that stops once its lower bound v.w/|v| exceeds `cut` (the kernel's
 * early exit): returns 0 separated, 1 penetrating, 2 pruned. */
static int gjk_cut(const Shape* A, const Shape* B, SV* S, int* ns, double* lam, double* v, double cut) {
    sub3(A->T + 9, B->T + 9, v);
    if (dot3(v, v) < 1e-24) { v[0] = 1; v[1] = 0; v[2] = 0; }
    int n = 0;
    for (int it = 0; it < 128; ++it) {
        double nv[3] = {-v[0], -v[1], -v[2]};
        SV w;
        sup_md(A, B, nv, &w);
        GJK_COUNT();
        const double vv = dot3(v, v), vw = dot3(v, w.w), sv = sqrt(vv);
        if (vw > cut * sv) { *ns = n; return 2; }
        if (n > 0 && vv - vw <= GJK_TOL * sv) break;
        int dup = 0;
        for (int i = 0; i < n; ++i) if (S[i].w[0] == w.w[0] && S[i].w[1] == w.w[1] && S[i].w[2] == w.w[2]) dup = 1;
        if (dup) { if (vw <= 0) { *ns = n; return 1; } break; }
        S[n++] = w;
        n = closest_simplex(S, n, v, lam);
        if (n == 4 || dot3(v, v) < 1e-24) { *ns = n; return 1; }
    }
    *ns = n;
    return 0;
}
/* getMinDistance's argmin by the kernel's algorithm (task_stage.hpp): closed
 * forms for every pair they cover, the lower bound for the rest, GJK (with
 * the early exit) only where the bound can still reach the closed-form
 * minimum, EPA best-first in increasing bound order while a bound can still
 * undercut the running minimum.  Pruning only drops pairs that provably cannot
 * be the argmin, so the result is min_distance_w's (tests/test_oracle_distance.py). */
static void min_distance_pruned(const OracleModel* m, const Kin* k, double* dist, double* grad, int* pair_out,
                                double* wA, double* wB) {
    Shape sh[ORC_MAXG];
    for (int g = 0; g < m->ngeom; ++g) make_shape(m, k, g, &sh[g]);
    static __thread double pd[ORC_MAXP];
    static __thread int st[ORC_MAXP];  /* 0 done, 1 candidate, 2 penetrating */
    double best = 1.7976931348623157e308, bpA[3] = {0}, bpB[3] = {0}, ub = 1e300;
    int bi = -1, bhow = 0;
    for (int p = 0; p < m->npairs; ++p) {
        const Shape *A = &sh[m->pair_a[p]], *B = &sh[m->pair_b[p]];
        double pA[3], pB[3], d;
        int closed = 0;
        if (A->type == 0 || B->type == 0) { int how; d = shape_distance(A, B, pA, pB, &how); closed = 1; }
        else if (A->type == 1 && B->type == 1 && cyl_cyl_side(A, B, &d, pA, pB)) closed = 1;
        st[p] = 0;
        if (closed) {
            ub = fmin(ub, d);
            if (d < best || (d == best && p < bi)) { best = d; bi = p; bhow = 0; memcpy(bpA, pA, sizeof(pA)); memcpy(bpB, pB, sizeof(pB)); }
        } else {
            pd[p] = pair_lower_bound(A, B);
            st[p] = 1;
        }
    }
    for (int p = 0; p < m->npairs; ++p) {
        if (st[p] != 1) continue;
        st[p] = 0;
        if (!(pd[p] - 1e-9 <= ub)) continue;
        SV S[4];
        int ns;
        double lam[4], v[3];
        const int r = gjk_cut(&sh[m->pair_a[p]], &sh[m->pair_b[p]], S, &ns, lam, v, ub + 1e-9);
        if (r == 2) continue;
        if (r == 1) { st[p] = 2; continue; }
        double pA[3] = {0, 0, 0}, pB[3] = {0, 0, 0}, dd[3];
        for (int c = 0; c < 3; ++c) for (int i = 0; i < ns; ++i) { pA[c] += lam[i] * S[i].a[c]; pB[c] += lam[i] * S[i].b[c]; }
        sub3(pA, pB, dd);
        const double d = norm3(dd);
        if (d < best || (d == best && p < bi)) { best = d; bi = p; bhow = 1; memcpy(bpA, pA, sizeof(pA)); memcpy(bpB, pB, sizeof(pB)); }
    }
    int ep_calls = 0, ep_steps = 0, ep_win_steps = 0;
    for (;;) {  /* EPA best-first */
        int cp = -1;
        for (int p = 0; p < m->npairs; ++p)
            if (st[p] == 2 && (cp < 0 || pd[p] < pd[cp])) cp = p;
        if (cp < 0 || pd[cp] > best || (pd[cp] == best && cp > bi)) break;
        st[cp] = 0;
        const Shape *A = &sh[m->pair_a[cp]], *B = &sh[m->pair_b[cp]];
        SV S[4];
        int ns;
        double lam[4], v[3], pA[3], pB[3];
        gjk(A, B, S, &ns, lam, v);
        g_epa_steps = 0;
        const double d = epa(A, B, S, ns, pA, pB);
        ++ep_calls; ep_steps += g_epa_steps;
        if (d < best || (d == best && cp < bi)) { best = d; bi = cp; bhow = 2; memcpy(bpA, pA, sizeof(pA)); memcpy(bpB, pB, sizeof(pB)); ep_win_steps = g_epa_steps; }
    }
    if (ep_calls && g_ec_on) {
        __atomic_fetch_add(&g_ec[0], ep_calls, __ATOMIC_RELAXED);
        __atomic_fetch_add(&g_ec[1], ep_steps, __ATOMIC_RELAXED);
        __atomic_fetch_add(&g_ec[2], bhow == 2 ? ep_calls - 1 : ep_calls, __ATOMIC_RELAXED);
        __atomic_fetch_add(&g_ec[3], ep_steps - (bhow == 2 ? ep_win_steps : 0), __ATOMIC_RELAXED);
        __atomic_fetch_add(&g_ec[4], 1, __ATOMIC_RELAXED);
    }
    if (bi >= 0 && bhow) refine_witness(&sh[m->pair_a[bi]], &sh[m->pair_b[bi]], &best, bpA, bpB);
    *dist = best;
    *pair_out = bi;
    memcpy(wA, bpA, sizeof(bpA));
    memcpy(wB, bpB, sizeof(bpB));
    const int nv = m->nv;
    memset(grad, 0, nv * sizeof(double));
    if (bi < 0) return;
    int jA = m->gparent[m->pair_a[bi]], jB = m->gparent[m->pair_b[bi]];
    double n[3];
    sub3(bpB, bpA, n);
    const double L = norm3(n);
    n[0] /= L; n[1] /= L; n[2] /= L;
    double JA[6 * ORC_MAXJ], JB[6 * ORC_MAXJ];
    point_jacobian(m, k, jA, bpA, JA);
    point_jacobian(m, k, jB, bpB, JB);
    for (int c = 0; c < nv; ++c) {
        double s2 = 0;
        for (int i = 0; i < 3; ++i) s2 += n[i] * (JB[i * nv + c] - JA[i * nv + c]);
        grad[c] = best < 0 ? -s2 : s2;
    }
}
/* 1: min_distance_w (all pairs, the reference's computeDistances loop) is
 * replaced by the pruned search above in every oracle entry point (tests and
 * the FLOP count set it; the default is the reference's all-pairs loop) */
static int g_pruned_narrow_phase = 0;
void oracle_set_pruned_narrow_phase(int on) { g_pruned_narrow_phase = on; }

static void min_distance_w(const OracleModel* m, const Kin* k, double* dist, double* grad, int* pair_out,
                           double* wA, double* wB) {
    if (g_pruned_narrow_phase) { min_distance_pruned(m, k, dist, grad, pair_out, wA, wB); return; }
    Shape sh[ORC_MAXG];
    for (int g = 0; g < m->ngeom; ++g) make_shape(m, k, g, &sh[g]);
    double best = 1.7976931348623157e308, bpA[3] = {0}, bpB[3] = {0};
    int bi = -1, bhow = 0;
    for (int p = 0; p < m->npairs; ++p) {
        double pA[3], pB[3];
        int how;
        double d = shape_distance(&sh[m->pair_a[p]], &sh[m->pair_b[p]], pA, pB, &how);
        if (d < best) { best = d; bi = p; bhow = how; memcpy(bpA, pA, sizeof(pA)); memcpy(bpB, pB, sizeof(pB)); }
    }
    /* the winner's GJK / EPA witnesses sharpened to the exact critical point (D17) */
    if (bi >= 0 && bhow) refine_witness(&sh[m->pair_a[bi]], &sh[m->pair_b[bi]], &best, bpA, bpB);
    *dist = best;
    *pair_out = bi;
    memcpy(wA, bpA, sizeof(bpA));
    memcpy(wB, bpB, sizeof(bpB));
    int nv = m->nv;
    memset(grad, 0, nv * sizeof(double));
    if (bi < 0) return;  /* reference indexes pair -1; we return zero gradient */
    int jA = m->gparent[m->pair_a[bi]], jB = m->gparent[m->pair_b[bi]];
    double n[3];
    sub3(bpB, bpA, n);
    double L = norm3(n);
    n[0] /= L; n[1] /= L; n[2] /= L;
    double JA[6 * ORC_MAXJ], JB[6 * ORC_MAXJ];
    point_jacobian(m, k, jA, bpA, JA);
    point_jacobian(m, k, jB, bpB, JB);
    for (int c = 0; c < nv; ++c) {
        double s = 0;
        for (int i = 0; i < 3; ++i) s += n[i] * (JB[i * nv + c] - JA[i * nv + c]);
        grad[c] = best < 0 ? -s : s;
    }
}

/* ------------------------------------------------------------------------ */
/* Jacobian time variation and the grad_dot terms of QPID                   */
/* ------------------------------------------------------------------------ */
#define ORC_ALL_JOINTS 0xffffffffu
/* velocity of a point p rigidly attached to the body of joint X, from the
 * joints a on its support path whose bit (a-1) is set in mask */
static void point_velocity(const OracleModel* m, const Kin* k, int X, const double* p, const double* qd,
                           uint32_t mask, double* v) {
    v[0] = v[1] = v[2] = 0;
    for (int a = X; a > 0; a = m->parent[a]) {
        if (!(mask & (1u << (a - 1)))) continue;
        double c[3];
        if (m->jtype[a] == 0) { double r[3]; sub3(p, k->T[a] + 9, r); cross3(k->z[a], r, c); }
        else memcpy(c, k->z[a], sizeof(c));
        for (int i = 0; i < 3; ++i) v[i] += qd[a - 1] * c[i];
    }
}

/* d/dt of the 6 x nv LWA Jacobian of a point p attached to joint X
 * (pinocchio computeJointJacobiansTimeVariation + get{Joint,Frame}Jacobian-
 * TimeVariation(LOCAL_WORLD_ALIGNED), robot_data.cpp:109,414,476-477) with the
 * joint velocities restricted to `mask`.  Column c (revolute):
 * [zdot_c x (p - o_c) + z_c x (pdot - odot_c); zdot_c], zdot_c = w_parent(c) x z_c;
 * (prismatic): [zdot_c; 0]. */
static void point_jacobian_dot(const OracleModel* m, const Kin* k, int X, const double* p, const double* qd,
                               uint32_t mask, double* Jd) {
    int nv = m->nv;
    memset(Jd, 0, 6 * nv * sizeof(double));
    double pdot[3];
    point_velocity(m, k, X, p, qd, mask, pdot);
    for (int c = X; c > 0; c = m->parent[c]) {
        double w[3] = {0, 0, 0};
        for (int a = m->parent[c]; a > 0; a = m->parent[a])
            if (m->jtype[a] == 0 && (mask & (1u << (a - 1))))
                for (int i = 0; i < 3; ++i) w[i] += qd[a - 1] * k->z[a][i];
        double zd[3];
        cross3(w, k->z[c], zd);
        if (m->jtype[c] == 0) {
            double od[3], r[3], t1[3], dv[3], t2[3];
            point_velocity(m, k, c, k->T[c] + 9, qd, mask, od);
            sub3(p, k->T[c] + 9, r);
            cross3(zd, r, t1);
            sub3(pdot, od, dv);
            cross3(k->z[c], dv, t2);
            for (int i = 0; i < 3; ++i) { Jd[i * nv + c - 1] = t1[i] + t2[i]; Jd[(3 + i) * nv + c - 1] = zd[i]; }
        } else {
            for (int i = 0; i < 3; ++i) Jd[i * nv + c - 1] = zd[i];
        }
    }
}

/* getManipulability(true, true, link) grad_dot, literally
 * (robot_data.cpp:555-569; MoMa :477-492 on the arm block c0..c0+nc):
 *   mani_dot = m tr(Jd J^T Ai), Ai_dot = -Ai (2 Jd J^T) Ai,
 *   grad_dot_i = mani_dot tr(dJ_i J^T Ai) + m tr(dJ_i Jd^T Ai + dJ_i J^T Ai_dot)
 * with dJ_i = the frame Jacobian time variation at qdot = e_(c0+i). */
static void manip_graddot(const OracleModel* m, const Kin* k, const double* J, int c0, int nc, const double* qd,
                          double man, double* gd) {
    int nv = m->nv;
    double Jr[6 * ORC_MAXJ], Jdf[6 * ORC_MAXJ], Jd[6 * ORC_MAXJ], A[36], Ai[36], JJd[36], T1[36], Aid[36];
    for (int i = 0; i < 6; ++i) for (int c = 0; c < nc; ++c) Jr[i * nc + c] = J[i * nv + c0 + c];
    for (int i = 0; i < 6; ++i) for (int j = 0; j < 6; ++j) { double s = 0; for (int c = 0; c < nc; ++c) s += Jr[i * nc + c] * Jr[j * nc + c]; A[i * 6 + j] = s; }
    pinv_cod_sym(A, 6, Ai);
    point_jacobian_dot(m, k, m->ee_joint, k->pe, qd, ORC_ALL_JOINTS, Jdf);
    for (int i = 0; i < 6; ++i) for (int c = 0; c < nc; ++c) Jd[i * nc + c] = Jdf[i * nv + c0 + c];
    /* JJt_dot = 2 Jd J^T (robot_data.cpp:562, as written: not symmetrised) */
    for (int i = 0; i < 6; ++i) for (int j = 0; j < 6; ++j) { double s = 0; for (int c = 0; c < nc; ++c) s += Jd[i * nc + c] * Jr[j * nc + c]; JJd[i * 6 + j] = 2 * s; }
    for (int i = 0; i < 6; ++i) for (int j = 0; j < 6; ++j) { double s = 0; for (int a = 0; a < 6; ++a) s += Ai[i * 6 + a] * JJd[a * 6 + j]; T1[i * 6 + j] = s; }
    for (int i = 0; i < 6; ++i) for (int j = 0; j < 6; ++j) { double s = 0; for (int a = 0; a < 6; ++a) s += T1[i * 6 + a] * Ai[a * 6 + j]; Aid[i * 6 + j] = -s; }
    /* tr(X Y^T Z) = sum_{a,c,b} X[a][c] Y[b][c] Z[b][a] */
    #define TR3(X, Y, Z) ({ double t_ = 0; for (int a_ = 0; a_ < 6; ++a_) for (int b_ = 0; b_ < 6; ++b_) { double u_ = 0; \
        for (int c_ = 0; c_ < nc; ++c_) { u_ += (X)[a_ * nc + c_] * (Y)[b_ * nc + c_]; } t_ += u_ * (Z)[b_ * 6 + a_]; } t_; })
    double mani_dot = man * TR3(Jd, Jr, Ai);
    double* dJ = (double*)malloc((size_t)nv * 6 * nv * sizeof(double));
    frame_jacobian_dq(m, k, dJ);
    for (int i = 0; i < nc; ++i) {
        const double* D = dJ + (size_t)(c0 + i) * 6 * nv;
        double Db[6 * ORC_MAXJ];
        for (int a = 0; a < 6; ++a) for (int c = 0; c < nc; ++c) Db[a * nc + c] = D[a * nv + c0 + c];
        gd[i] = mani_dot * TR3(Db, Jr, Ai) + man * (TR3(Db, Jd, Ai) + TR3(Db, Jr, Aid));
    }
    #undef TR3
    free(dJ);
}

/* getMinDistance(.., with_graddot = true, ..) grad_dot, literally
 * (robot_data.cpp:496-512): JX_dot = J_jX_dot.top - (skew(rX_dot) J_jX.bottom
 * + skew(rX) J_jX_dot.bottom), rX_dot = JX qdot - J_jX.top qdot;
 * grad_dot = n^T (JB_dot - JA_dot) (n_dot neglected; no sign flip). */
static void mindist_graddot(const OracleModel* m, const Kin* k, int pair, const double* pA, const double* pB,
                            const double* qd, double* gd) {
    int nv = m->nv;
    memset(gd, 0, nv * sizeof(double));
    if (pair < 0) return;
    double n[3];
    sub3(pB, pA, n);
    double L = norm3(n);
    n[0] /= L; n[1] /= L; n[2] /= L;
    double JXd[2][3 * ORC_MAXJ];
    for (int s = 0; s < 2; ++s) {
        int jX = m->gparent[s == 0 ? m->pair_a[pair] : m->pair_b[pair]];
        const double* pX = s == 0 ? pA : pB;
        const double* oX = k->T[jX] + 9;
        double Jj[6 * ORC_MAXJ], Jjd[6 * ORC_MAXJ], r[3], vt[3] = {0, 0, 0}, pd[3] = {0, 0, 0}, rd[3];
        point_jacobian(m, k, jX, oX, Jj);
        point_jacobian_dot(m, k, jX, oX, qd, ORC_ALL_JOINTS, Jjd);
        sub3(pX, oX, r);
        for (int c = 0; c < nv; ++c) {
            double top[3] = {Jj[0 * nv + c], Jj[1 * nv + c], Jj[2 * nv + c]}, bot[3] = {Jj[3 * nv + c], Jj[4 * nv + c], Jj[5 * nv + c]}, rb[3];
            cross3(r, bot, rb);
            for (int i = 0; i < 3; ++i) { pd[i] += (top[i] - rb[i]) * qd[c]; vt[i] += top[i] * qd[c]; }
        }
        sub3(pd, vt, rd);
        for (int c = 0; c < nv; ++c) {
            double bot[3] = {Jj[3 * nv + c], Jj[4 * nv + c], Jj[5 * nv + c]}, botd[3] = {Jjd[3 * nv + c], Jjd[4 * nv + c], Jjd[5 * nv + c]};
            double t1[3], t2[3];
            cross3(rd, bot, t1);
            cross3(r, botd, t2);
            for (int i = 0; i < 3; ++i) JXd[s][i * nv + c] = Jjd[i * nv + c] - (t1[i] + t2[i]);
        }
    }
    for (int c = 0; c < nv; ++c) {
        double t = 0;
        for (int i = 0; i < 3; ++i) t += n[i] * (JXd[1][i * nv + c] - JXd[0][i * nv + c]);
        gd[c] = t;
    }
}

/* ------------------------------------------------------------------------ */
/* task-space helpers  (math_type_define.h)                                 */
/* ------------------------------------------------------------------------ */
static double cubic(double t, double t0, double tf, double x0, double xf, double xd0, double xdf) {
    if (t < t0) return x0;
    if (t > tf) return xf;
    double e = t - t0, T = tf - t0, T2 = T * T, T3 = T2 * T, dx = xf - x0;
    return x0 + xd0 * e + (3 * dx / T2 - 2 * xd0 / T - xdf / T) * e * e + (-2 * dx / T3 + (xd0 + xdf) / T2) * e * e * e;
}
static double cubic_dot(double t, double t0, double tf, double x0, double xf, double xd0, double xdf) {
    if (t < t0) return xd0;
    if (t > tf) return xdf;
    double e = t - t0, T = tf - t0, T2 = T * T, T3 = T2 * T, dx = xf - x0;
    return xd0 + 2 * (3 * dx / T2 - 2 * xd0 / T - xdf / T) * e + 3 * (-2 * dx / T3 + (xd0 + xdf) / T2) * e * e;
}
/* principal log of a rotation (row-major) as axis-angle vector */
static void so3_log(const double* R, double* w) {
    double c = (R[0] + R[4] + R[8] - 1) / 2;
    c = c > 1 ? 1 : (c < -1 ? -1 : c);
    double th = acos(c);
    double v[3] = {R[7] - R[5], R[2] - R[6], R[3] - R[1]};
    if (th < 1e-8) { w[0] = 0.5 * v[0]; w[1] = 0.5 * v[1]; w[2] = 0.5 * v[2]; return; }
    if (M_PI - th < 1e-6) {
        double B[9];
        for (int i = 0; i < 9; ++i) B[i] = R[i] / 2;
        B[0] += 0.5; B[4] += 0.5; B[8] += 0.5;
        int kk = 0;
        if (B[4] > B[kk * 4]) kk = 1;
        if (B[8] > B[kk * 4]) kk = 2;
        double s = sqrt(B[kk * 4]);
        double a[3] = {B[0 * 3 + kk] / s, B[1 * 3 + kk] / s, B[2 * 3 + kk] / s};
        if (dot3(a, v) < 0) { a[0] = -a[0]; a[1] = -a[1]; a[2] = -a[2]; }
        w[0] = th * a[0]; w[1] = th * a[1]; w[2] = th * a[2];
        return;
    }
    double f = th / (2 * sin(th));
    w[0] = f * v[0]; w[1] = f * v[1]; w[2] = f * v[2];
}
static void so3_exp(const double* w, double* R) {
    double th = norm3(w);
    double K[9] = {0, -w[2], w[1], w[2], 0, -w[0], -w[1], w[0], 0}, K2[9];
    matmul3(K, K, K2);
    double a = th < 1e-12 ? 1 : sin(th) / th, b = th < 1e-12 ? 0 : (1 - cos(th)) / (th * th);
    for (int i = 0; i < 9; ++i) R[i] = (i % 4 == 0 ? 1 : 0) + a * K[i] + b * K2[i];
}
/* 12-vector pose (R col-major 9, p 3) -> R row-major, p */
static void pose_unpack(const double* x, double* R, double* p) {
    for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) R[3 * r + c] = x[3 * c + r];
    p[0] = x[9]; p[1] = x[10]; p[2] = x[11];
}
/* DyrosMath::getTaskSpaceCubic (math_type_define.h:647-687) */
static void task_space_cubic(const double* xt, const double* xdt, const double* xi, const double* xdi,
                             double t, double t0, double T, double* xd_out, double* xdd_out) {
    double Rt[9], pt[3], Ri[9], pi_[3];
    pose_unpack(xt, Rt, pt);
    pose_unpack(xi, Ri, pi_);
    double tf = t0 + T, Rd[9], pd[3];
    for (int i = 0; i < 3; ++i) {
        pd[i] = cubic(t, t0, tf, pi_[i], pt[i], xdi[i], xdt[i]);
        xdd_out[i] = cubic_dot(t, t0, tf, pi_[i], pt[i], xdi[i], xdt[i]);
    }
    double RiT[9], M[9], r[3];
    for (int a = 0; a < 3; ++a) for (int b = 0; b < 3; ++b) RiT[3 * a + b] = Ri[3 * b + a];
    matmul3(RiT, Rt, M);
    so3_log(M, r);
    if (t >= tf) memcpy(Rd, Rt, sizeof(Rd));
    else if (t < t0) memcpy(Rd, Ri, sizeof(Rd));
    else {
        double tau = cubic(t, t0, tf, 0, 1, 0, 0), wr[3] = {r[0] * tau, r[1] * tau, r[2] * tau}, E[9];
        so3_exp(wr, E);
        matmul3(Ri, E, Rd);
    }
    double rd[3];
    for (int i = 0; i < 3; ++i) rd[i] = cubic_dot(t, t0, tf, 0, r[i], 0, 0);
    double tau = (t - t0) / (tf - t0), o[3];
    matvec3(Ri, rd, o);
    if (tau < 0 || tau > 1) { o[0] = o[1] = o[2] = 0; }
    xdd_out[3] = o[0]; xdd_out[4] = o[1]; xdd_out[5] = o[2];
    for (int rr = 0; rr < 3; ++rr) for (int c = 0; c < 3; ++c) xd_out[3 * c + rr] = Rd[3 * rr + c];
    xd_out[9] = pd[0]; xd_out[10] = pd[1]; xd_out[11] = pd[2];
}

/* ------------------------------------------------------------------------ */
/* OSQP ADMM restatement (QP_base.h:100-180 -> OSQP)                        */
/* ------------------------------------------------------------------------ */
static double vnorm_inf(const double* v, int n) { double r = 0; for (int i = 0; i < n; ++i) if (fabs(v[i]) > r) r = fabs(v[i]); return r; }
static void limit_scaling(double* v, int n) {
    for (int i = 0; i < n; ++i) { if (v[i] < MIN_SCALING) v[i] = 1.0; else if (v[i] > MAX_SCALING) v[i] = MAX_SCALING; }
}

/* residuals and tolerances of one iterate (scaled problem) */
typedef struct Res {
    double pri_res, dua_res, pri_res_s, dua_res_s;
    double nAx_s, nz_s, nPx_s, nAty_s, nq_s;
    double eps_pri, eps_dua;
} Res;

typedef struct QPW {
    int n, m;
    double P[ORC_MAXX * ORC_MAXX], q[ORC_MAXX], A[ORC_MAXC * ORC_MAXX], l[ORC_MAXC], u[ORC_MAXC];
    double D[ORC_MAXX], E[ORC_MAXC], c;
    double Dinv[ORC_MAXX], Einv[ORC_MAXC], cinv;  /* OSQP scaling.c keeps them; residuals multiply */
    double rho_vec[ORC_MAXC], rho;
    int ctype[ORC_MAXC];  /* -1 loose, 0 ineq, 1 eq */
    double L[ORC_MAXX * ORC_MAXX];
    double x[ORC_MAXX], z[ORC_MAXC], y[ORC_MAXC], dy[ORC_MAXC];
    Res r;
} QPW;

static void qp_factor(QPW* w, double sigma) {
    int n = w->n, m = w->m;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            double s = w->P[i * n + j] + (i == j ? sigma : 0);
            for (int k = 0; k < m; ++k) s += w->A[k * n + i] * w->rho_vec[k] * w->A[k * n + j];
            w->L[i * n + j] = s;
        }
    chol(w->L, n);
}

static void set_rho_vec(QPW* w) {
    for (int i = 0; i < w->m; ++i)
        w->rho_vec[i] = w->ctype[i] < 0 ? RHO_MIN : (w->ctype[i] > 0 ? RHO_EQ_OVER_RHO_INEQ * w->rho : w->rho);
}

static void qp_scale(QPW* w, int iters) {
    int n = w->n, m = w->m;
    for (int i = 0; i < n; ++i) w->D[i] = 1;
    for (int i = 0; i < m; ++i) w->E[i] = 1;
    w->c = 1;
    for (int it = 0; it < iters; ++it) {
        double Dt[ORC_MAXX], Et[ORC_MAXC];
        for (int j = 0; j < n; ++j) {
            double s = 0;
            for (int i = 0; i < n; ++i) s = fmax(s, fabs(w->P[i * n + j]));
            for (int i = 0; i < m; ++i) s = fmax(s, fabs(w->A[i * n + j]));
            Dt[j] = s;
        }
        for (int i = 0; i < m; ++i) { double s = 0; for (int j = 0; j < n; ++j) s = fmax(s, fabs(w->A[i * n + j])); Et[i] = s; }
        limit_scaling(Dt, n);
        limit_scaling(Et, m);
        for (int j = 0; j < n; ++j) Dt[j] = 1.0 / sqrt(Dt[j]);
        for (int i = 0; i < m; ++i) Et[i] = 1.0 / sqrt(Et[i]);
        for (int i = 0; i < n; ++i) for (int j = 0; j < n; ++j) w->P[i * n + j] *= Dt[i] * Dt[j];
        for (int i = 0; i < m; ++i) for (int j = 0; j < n; ++j) w->A[i * n + j] *= Et[i] * Dt[j];
        for (int j = 0; j < n; ++j) { w->q[j] *= Dt[j]; w->D[j] *= Dt[j]; }
        for (int i = 0; i < m; ++i) w->E[i] *= Et[i];
        /* cost scaling */
        double cm = 0;
        for (int j = 0; j < n; ++j) { double s = 0; for (int i = 0; i < n; ++i) s = fmax(s, fabs(w->P[i * n + j])); cm += s; }
        cm /= n;
        double nq = vnorm_inf(w->q, n);
        limit_scaling(&nq, 1);
        double ct = fmax(cm, nq);
        limit_scaling(&ct, 1);
        ct = 1.0 / ct;
        for (int i = 0; i < n * n; ++i) w->P[i] *= ct;
        for (int j = 0; j < n; ++j) w->q[j] *= ct;
        w->c *= ct;
        /* fixed point: every factor of this pass was exactly 1, so the
         * remaining passes would repeat it bit for bit (kernel: same exit) */
        int ones = ct == 1.0;
        for (int j = 0; j < n && ones; ++j) ones = Dt[j] == 1.0;
        for (int i = 0; i < m && ones; ++i) ones = Et[i] == 1.0;
        if (ones) break;
    }
    for (int i = 0; i < m; ++i) {
        w->l[i] *= w->E[i];
        w->u[i] *= w->E[i];
    }
    for (int j = 0; j < n; ++j) w->Dinv[j] = 1.0 / w->D[j];
    for (int i = 0; i < m; ++i) w->Einv[i] = 1.0 / w->E[i];
    w->cinv = 1.0 / w->c;
}

/* residuals at the current iterate (scaled and unscaled) */
static void qp_residuals(const QPW* w, Res* o, const double* x, const double* z, const double* y, double eps_abs, double eps_rel) {
    int n = w->n, m = w->m;
    double Ax[ORC_MAXC], Px[ORC_MAXX], Aty[ORC_MAXX];
    for (int i = 0; i < m; ++i) { double s = 0; for (int j = 0; j < n; ++j) s += w->A[i * n + j] * x[j]; Ax[i] = s; }
    for (int i = 0; i < n; ++i) { double s = 0, t = 0; for (int j = 0; j < n; ++j) s += w->P[i * n + j] * x[j]; for (int k = 0; k < m; ++k) t += w->A[k * n + i] * y[k]; Px[i] = s; Aty[i] = t; }
    double pr = 0, prs = 0, nAx = 0, nz = 0, nAxs = 0, nzs = 0;
    for (int i = 0; i < m; ++i) {
        double r = Ax[i] - z[i];
        prs = fmax(prs, fabs(r));
        pr = fmax(pr, fabs(r * w->Einv[i]));
        nAx = fmax(nAx, fabs(Ax[i] * w->Einv[i]));
        nz = fmax(nz, fabs(z[i] * w->Einv[i]));
        nAxs = fmax(nAxs, fabs(Ax[i]));
        nzs = fmax(nzs, fabs(z[i]));
    }
    double dr = 0, drs = 0, nPx = 0, nAty = 0, nq = 0, nPxs = 0, nAtys = 0, nqs = 0;
    for (int i = 0; i < n; ++i) {
        double r = Px[i] + w->q[i] + Aty[i];
        drs = fmax(drs, fabs(r));
        dr = fmax(dr, fabs(r * w->Dinv[i]));
        nPx = fmax(nPx, fabs(Px[i] * w->Dinv[i]));
        nAty = fmax(nAty, fabs(Aty[i] * w->Dinv[i]));
        nq = fmax(nq, fabs(w->q[i] * w->Dinv[i]));
        nPxs = fmax(nPxs, fabs(Px[i]));
        nAtys = fmax(nAtys, fabs(Aty[i]));
        nqs = fmax(nqs, fabs(w->q[i]));
    }
    o->pri_res = pr;
    o->dua_res = dr * w->cinv;
    o->pri_res_s = prs;
    o->dua_res_s = drs;
    o->nAx_s = nAxs; o->nz_s = nzs; o->nPx_s = nPxs; o->nAty_s = nAtys; o->nq_s = nqs;
    o->eps_pri = eps_abs + eps_rel * fmax(nAx, nz);
    o->eps_dua = eps_abs + eps_rel * fmax(fmax(nPx, nAty), nq) * w->cinv;
}

static int qp_primal_infeasible(QPW* w, double eps) {
    int n = w->n, m = w->m;
    double dy[ORC_MAXC], nrm = 0;
    for (int i = 0; i < m; ++i) {
        double d = w->dy[i];
        if (w->ctype[i] < 0) d = 0;
        else if (w->u[i] > INFTY * MIN_SCALING) d = d < 0 ? d : 0;
        else if (w->l[i] < -INFTY * MIN_SCALING) d = d > 0 ? d : 0;
        dy[i] = d;
        nrm = fmax(nrm, fabs(w->E[i] * d));
    }
    if (nrm <= DIVISION_TOL) return 0;
    double lhs = 0;
    for (int i = 0; i < m; ++i) {
        if (dy[i] > 0) lhs += w->u[i] * dy[i];
        else if (dy[i] < 0) lhs += w->l[i] * dy[i];
    }
    if (!(lhs < -eps * nrm)) return 0;
    for (int j = 0; j < n; ++j) {
        double s = 0;
        for (int i = 0; i < m; ++i) s += w->A[i * n + j] * dy[i];
        if (fabs(s * w->Dinv[j]) >= eps * nrm) return 0;
    }
    return 1;
}

/* LDL^T of a quasi-definite dense matrix (no pivoting) */
static int ldlt(double* K, int N, double* Dg) {
    for (int j = 0; j < N; ++j) {
        double d = K[j * N + j];
        for (int k = 0; k < j; ++k) d -= K[j * N + k] * K[j * N + k] * Dg[k];
        if (d == 0) return 0;
        Dg[j] = d;
        for (int i = j + 1; i < N; ++i) {
            double t = K[i * N + j];
            for (int k = 0; k < j; ++k) t -= K[i * N + k] * K[j * N + k] * Dg[k];
            K[i * N + j] = t / d;
        }
    }
    return 1;
}
static void ldlt_solve(const double* L, const double* Dg, int N, double* b) {
    for (int i = 0; i < N; ++i) { double t = b[i]; for (int k = 0; k < i; ++k) t -= L[i * N + k] * b[k]; b[i] = t; }
    for (int i = 0; i < N; ++i) b[i] /= Dg[i];
    for (int i = N - 1; i >= 0; --i) { double t = b[i]; for (int k = i + 1; k < N; ++k) t -= L[k * N + i] * b[k]; b[i] = t; }
}

/* Equality-constrained QP on the rows flagged active (flag -1: A_i x = l_i,
 * +1: A_i x = u_i): OSQP polish's reduced KKT [P+dI, A_r^T; A_r, -dI] with
 * iterative refinement against the unregularised system (polish.c). */
static int qp_eqp(const QPW* w, const OracleSettings* s, const int* flag, double* xp, double* yp) {
    int n = w->n, m = w->m;
    static __thread double K[(ORC_MAXX + ORC_MAXC) * (ORC_MAXX + ORC_MAXC)], K0[(ORC_MAXX + ORC_MAXC) * (ORC_MAXX + ORC_MAXC)];
    int act[ORC_MAXC], nact = 0;
    double b[ORC_MAXC];
    for (int i = 0; i < m; ++i)
        if (flag[i]) { act[nact] = i; b[nact++] = flag[i] < 0 ? w->l[i] : w->u[i]; }
    if (s->polish_cap > 0) {  /* the kernel's size: free variables + active G rows (rows n.. of A = [I; G]) */
        int nfix = 0;
        for (int i = 0; i < n; ++i) nfix += flag[i] != 0;
        if (n - nfix + (nact - nfix) > s->polish_cap) return 0;
    }
    int N = n + nact;
    double Dg[ORC_MAXX + ORC_MAXC], rhs[ORC_MAXX + ORC_MAXC], sol[ORC_MAXX + ORC_MAXC], r[ORC_MAXX + ORC_MAXC];
    for (int i = 0; i < N * N; ++i) K0[i] = 0;
    for (int i = 0; i < n; ++i) for (int j = 0; j < n; ++j) K0[i * N + j] = w->P[i * n + j];
    for (int a = 0; a < nact; ++a)
        for (int j = 0; j < n; ++j) { K0[(n + a) * N + j] = w->A[act[a] * n + j]; K0[j * N + n + a] = w->A[act[a] * n + j]; }
    memcpy(K, K0, N * N * sizeof(double));
    for (int i = 0; i < n; ++i) K[i * N + i] += s->delta;
    for (int a = 0; a < nact; ++a) K[(n + a) * N + n + a] -= s->delta;
    if (!ldlt(K, N, Dg)) return 0;
    for (int i = 0; i < n; ++i) rhs[i] = -w->q[i];
    for (int a = 0; a < nact; ++a) rhs[n + a] = b[a];
    memcpy(sol, rhs, N * sizeof(double));
    ldlt_solve(K, Dg, N, sol);
    for (int it = 0; it < s->polish_refine_iter; ++it) {
        for (int i = 0; i < N; ++i) { double t = rhs[i]; for (int j = 0; j < N; ++j) t -= K0[i * N + j] * sol[j]; r[i] = t; }
        ldlt_solve(K, Dg, N, r);
        for (int i = 0; i < N; ++i) sol[i] += r[i];
    }
    for (int i = 0; i < n; ++i) xp[i] = sol[i];
    for (int i = 0; i < m; ++i) yp[i] = 0;
    for (int a = 0; a < nact; ++a) yp[act[a]] = sol[n + a];
    return 1;
}

/* OSQP polish (polish.c) restated; on success writes x, z, y (scaled).
 * strict == 0: OSQP's single attempt with its acceptance rule.
 * strict != 0 (parity mode): the polished point must be KKT-certified
 * (residuals at eps_exact, dual signs matching the active bounds).  When the
 * ADMM active-set guess is wrong, continue with a primal active-set method
 * (Nocedal & Wright Alg. 16.3) from the first feasible polished point:
 * drop the worst wrong-sign multiplier, step to the equality-QP minimiser
 * with a ratio test, add the blocking row.  Exact on termination. */
/* parity mode polishes at every check, but a not-yet-converged iterate gets at
 * most POLISH_MAX_EARLY failed attempts; later only at convergence (same
 * decisions as the kernel's kPolishMaxEarly) */
#define POLISH_MAX_EARLY 4
#define POLISH_MAX_TOTAL 12   /* then at convergence only the tight ADMM fallback */
#define POLISH_FEAS_ATTEMPTS 6
#define POLISH_AS_ITERS 24

/* a working-set row with no weight on the free variables depends on the
 * fixed bounds alone and makes the reduced KKT singular; when the fixed
 * values already satisfy it strictly it is not active: drop it (the
 * kernel's polish applies the same rule) */
static void polish_drop_fixed_rows(const QPW* w, int* flag) {
    int n = w->n, m = w->m;
    for (int i = n; i < m; ++i) {
        if (!flag[i]) continue;
        double sf = 0, sa = 0, act = 0;
        for (int j = 0; j < n; ++j) {
            double g = w->A[i * n + j];
            sa = fmax(sa, fabs(g));
            if (!flag[j]) sf = fmax(sf, fabs(g));
            else act += g * ((flag[j] > 0 ? w->u[j] : w->l[j]) / w->A[j * n + j]);  /* kernel: the fixed value b_j / ab_j */
        }
        double b = flag[i] < 0 ? w->l[i] : w->u[i], slack = flag[i] < 0 ? act - b : b - act;
        if (sf <= 1e-12 * sa && slack > 1e-12 * (fabs(act) + fabs(b))) flag[i] = 0;
    }
}

/* ---- polish census (diagnostic, tools/polish_census.py) ------------------
 * Counts the certified polish's steps and scores alternative first guesses of
 * the active set against the one each successful polish certifies.  Off by
 * default; no decision of the solver depends on it. */
#define PC_RULES 16
enum { PC_CALLS, PC_OK, PC_EQP, PC_ADD, PC_DROP, PC_RATIO, PC_OK1, PC_RETRY, PC_HIST0 = 8, PC_MATCH0 = PC_HIST0 + 8,
       PC_FN0 = PC_MATCH0 + PC_RULES, PC_FP0 = PC_FN0 + PC_RULES, PC_N = PC_FP0 + PC_RULES };
static long long g_pc[PC_N];
static long long g_pc_row[3][ORC_MAXC];  /* rule 0: false neg / false pos / final active, per row */
void oracle_polish_census_rows(long long* out, int reset) {
    if (out) memcpy(out, g_pc_row, sizeof(g_pc_row));
    if (reset) memset(g_pc_row, 0, sizeof(g_pc_row));
}
static int g_pc_on = 0, g_pc_guess = -1;
void oracle_polish_guess(int rule) { g_pc_guess = rule; }
/* study switches of the infeasible phase (tools/polish_census.py --feas-drop / --feas-att):
 * mode 0 no drop, 1 drop the worst wrong-signed row in both passes, 4 only in the
 * retry pass, 5 only in the first pass (the product rule); attempts before the
 * phase gives up (POLISH_FEAS_ATTEMPTS) */
static int g_feas_drop = 5, g_feas_att = POLISH_FEAS_ATTEMPTS;
void oracle_polish_feas(int mode, int attempts) { g_feas_drop = mode; g_feas_att = attempts; }
static double g_pc_tol[PC_RULES];
void oracle_polish_census(int on, const double* tol, long long* out, int reset) {
    if (out) for (int i = 0; i < PC_N; ++i) out[i] = __atomic_load_n(&g_pc[i], __ATOMIC_RELAXED);
    if (reset) for (int i = 0; i < PC_N; ++i) __atomic_store_n(&g_pc[i], 0, __ATOMIC_RELAXED);
    if (tol) memcpy(g_pc_tol, tol, sizeof(g_pc_tol));
    g_pc_on = on;
}
static void pc_add(int k, long long v) { __atomic_fetch_add(&g_pc[k], v, __ATOMIC_RELAXED); }
/* candidate first guesses from the ADMM iterate (scaled problem) */
static void pc_guess(const QPW* w, int rule, int* f) {
    int n = w->n, m = w->m;
    double t = g_pc_tol[rule];
    double gr[ORC_MAXX];  /* Lagrangian gradient without the bound multipliers */
    for (int j = 0; j < n; ++j) {
        double s = w->q[j];
        for (int k = 0; k < n; ++k) s += w->P[j * n + k] * w->x[k];
        for (int i = n; i < m; ++i) s += w->A[i * n + j] * w->y[i];
        gr[j] = s;
    }
    /* projected Gauss-Seidel (11-13: 1, 2, 4 sweeps) / Jacobi (14: 3 sweeps,
     * step t) on the bound rows of variables with P_ii > 0, G-row duals fixed */
    double xgs[ORC_MAXX];
    memcpy(xgs, w->x, n * sizeof(double));
    if (rule >= 11) {
        int sweeps = rule == 11 ? 1 : rule == 12 ? 2 : rule == 13 ? 4 : 3;
        for (int sw = 0; sw < sweeps; ++sw) {
            double xo[ORC_MAXX];
            memcpy(xo, xgs, n * sizeof(double));
            for (int j = 0; j < n; ++j) {
                if (!(w->P[j * n + j] > 0)) continue;
                double s = w->q[j];
                const double* xs = rule == 14 ? xo : xgs;
                for (int k = 0; k < n; ++k) s += w->P[j * n + k] * xs[k];
                for (int i = n; i < m; ++i) s += w->A[i * n + j] * w->y[i];
                double a = w->A[j * n + j], v = xs[j] - (rule == 14 ? t : 1.0) * s / w->P[j * n + j];
                v = fmin(fmax(v, w->l[j] / a), w->u[j] / a);
                xgs[j] = v;
            }
        }
    }
    for (int i = 0; i < m; ++i) {
        double ax = 0;
        for (int j = 0; j < n; ++j) ax += w->A[i * n + j] * w->x[j];
        const double l = w->l[i], u = w->u[i], z = w->z[i], y = w->y[i];
        int g = 0;
        switch (rule) {
        case 0: g = (z - l < -y) ? -1 : ((u - z < y) ? 1 : 0); break;                  /* OSQP */
        case 1: g = (ax - l < -y) ? -1 : ((u - ax < y) ? 1 : 0); break;                /* OSQP on A x */
        case 2: g = (y < -t) ? -1 : (y > t ? 1 : 0); break;                            /* dual sign */
        case 3: g = (ax - l < t) ? -1 : (u - ax < t ? 1 : 0); break;                   /* primal near */
        case 4: g = (z - l < -y || ax - l < -t) ? -1 : ((u - z < y || u - ax < -t) ? 1 : 0); break; /* OSQP + violated */
        case 5: g = (z - l < -y + t) ? -1 : ((u - z < y + t) ? 1 : 0); break;          /* OSQP, widened */
        case 6: g = (ax - l < -y + t) ? -1 : ((u - ax < y + t) ? 1 : 0); break;
        case 7: g = ((ax - l < t && y < 0) || ax - l < -t) ? -1 : (((u - ax < t && y > 0) || u - ax < -t) ? 1 : 0); break;
        case 11: case 12: case 13: case 14:
            if (i < n && w->P[i * n + i] > 0) {
                const double a = w->A[i * n + i];
                g = (a * xgs[i] <= l) ? -1 : (a * xgs[i] >= u ? 1 : 0);
            } else g = (z - l < -y) ? -1 : ((u - z < y) ? 1 : 0);
            break;
        case 8: case 9: case 10:
            if (i < n && w->P[i * n + i] > 0) {
                const double a = w->A[i * n + i], xt = w->x[i] - t * gr[i] / w->P[i * n + i];
                g = (a * xt <= l) ? -1 : (a * xt >= u ? 1 : 0);
                if (rule == 9 && !g) g = (z - l < -y) ? -1 : ((u - z < y) ? 1 : 0);
            } else g = (z - l < -y) ? -1 : ((u - z < y) ? 1 : 0);
            break;
        default: g = 0;
        }
        if (l < -INFTY * MIN_SCALING && g < 0) g = 0;
        if (u > INFTY * MIN_SCALING && g > 0) g = 0;
        f[i] = g;
    }
    polish_drop_fixed_rows(w, f);
}

/* First active-set guess of the parity-mode polish (QPIK, polish_guess = 1):
 * the bound rows of the variables with cost curvature (P_jj > 0: the q-dot)
 * take the sides at which POLISH_JACOBI_SWEEPS projected Jacobi sweeps on
 * their box, with the G-row duals of the ADMM iterate held fixed, clamp
 * them; every other row keeps OSQP's rule.  At the first check the ADMM
 * iterate has usually not reached the velocity bounds the optimum saturates,
 * so OSQP's rule misses about two rows per FR3 instance (12 % right first
 * time, 2.7 EQP solves per polish); this guess 77 %, 1.55
 * (tools/polish_census.py).  Only the path to the certified optimum changes,
 * not the optimum.  Same rule and summation order as the kernel's polish(). */
#define POLISH_JACOBI_SWEEPS 3
static void polish_guess_jacobi(const QPW* w, int* flag) {
    int n = w->n, m = w->m;
    double c[ORC_MAXX], xv[ORC_MAXX], xo[ORC_MAXX];
    int side[ORC_MAXX];
    for (int j = 0; j < n; ++j) {  /* two partial sums over the G rows, as the kernel */
        double s0 = w->q[j], s1 = 0;
        for (int i = n; i < m; ++i) {
            if ((i - n) & 1) s1 += w->A[i * n + j] * w->y[i];
            else s0 += w->A[i * n + j] * w->y[i];
        }
        c[j] = s0 + s1;
        xv[j] = w->x[j];
        side[j] = 0;
    }
    for (int sw = 0; sw < POLISH_JACOBI_SWEEPS; ++sw) {
        memcpy(xo, xv, n * sizeof(double));
        for (int j = 0; j < n; ++j) {
            const double pjj = w->P[j * n + j];
            if (!(pjj > 0)) continue;
            double g = c[j];
            for (int k = 0; k < n; ++k) g += w->P[j * n + k] * xo[k];
            const double ipjj = 1.0 / pjj, a = w->A[j * n + j], v = xo[j] - g * ipjj, av = a * v;
            side[j] = av <= w->l[j] ? -1 : (av >= w->u[j] ? 1 : 0);
            xv[j] = side[j] < 0 ? w->l[j] / a : (side[j] > 0 ? w->u[j] / a : v);
        }
    }
    for (int j = 0; j < n; ++j)
        if (w->P[j * n + j] > 0) flag[j] = side[j];
}

/* census rule 15 (experiment): a slack-like variable (no curvature, in one G
 * row) keeps its bound active iff its bound multiplier from stationarity with
 * the ADMM G-row dual, -(q_j + g_rj y_r) / ab_j, is below -t |q_j| / ab_j */
static void pc_guess_slacks(const QPW* w, int* flag, double t) {
    int n = w->n, m = w->m;
    for (int j = 0; j < n; ++j) {
        if (w->P[j * n + j] != 0 || w->q[j] == 0) continue;
        int r = -1, cnt = 0;
        for (int i = n; i < m; ++i) if (w->A[i * n + j] != 0) { r = i; ++cnt; }
        if (cnt != 1) continue;
        const double ab = w->A[j * n + j], yb = -(w->q[j] + w->A[r * n + j] * w->y[r]) / ab;
        flag[j] = yb < -t * fabs(w->q[j]) / ab ? -1 : 0;
    }
}

/* census rule 16 (experiment): projected Jacobi on the EFFECTIVE box of each
 * curvature variable -- its bound row intersected with the G rows that bound
 * it alone (one nonzero among the curvature columns: the joint-limit CBF rows,
 * slack at 0) -- and the guess marks whichever constraint binds */
static void pc_guess_effbox(const QPW* w, int* flag) {
    int n = w->n, m = w->m;
    double c[ORC_MAXX], xv[ORC_MAXX], xo[ORC_MAXX], elo[ORC_MAXX], ehi[ORC_MAXX];
    int blo[ORC_MAXX], bhi[ORC_MAXX], side[ORC_MAXX], boxrow[ORC_MAXC];
    for (int i = n; i < m; ++i) {
        int cnt = 0, jj = -1;
        for (int j = 0; j < n; ++j) if (w->P[j * n + j] > 0 && w->A[i * n + j] != 0) { ++cnt; jj = j; }
        boxrow[i] = cnt == 1 ? jj : -1;
    }
    for (int j = 0; j < n; ++j) {
        double sm = w->q[j];
        for (int i = n; i < m; ++i) sm += w->A[i * n + j] * w->y[i];
        c[j] = sm; xv[j] = w->x[j]; side[j] = 0;
        const double a = w->A[j * n + j];
        elo[j] = w->l[j] / a; ehi[j] = w->u[j] / a; blo[j] = j; bhi[j] = j;
    }
    for (int i = n; i < m; ++i) {
        const int j = boxrow[i];
        if (j < 0) continue;
        const double g = w->A[i * n + j];
        if (w->l[i] > -INFTY * MIN_SCALING) {
            const double v = w->l[i] / g;
            if (g > 0 && v > elo[j]) { elo[j] = v; blo[j] = i; }
            if (g < 0 && v < ehi[j]) { ehi[j] = v; bhi[j] = i; }
        }
        if (w->u[i] < INFTY * MIN_SCALING) {
            const double v = w->u[i] / g;
            if (g > 0 && v < ehi[j]) { ehi[j] = v; bhi[j] = i; }
            if (g < 0 && v > elo[j]) { elo[j] = v; blo[j] = i; }
        }
    }
    for (int sw = 0; sw < POLISH_JACOBI_SWEEPS; ++sw) {
        memcpy(xo, xv, n * sizeof(double));
        for (int j = 0; j < n; ++j) {
            const double pjj = w->P[j * n + j];
            if (!(pjj > 0)) continue;
            double g = c[j];
            for (int k = 0; k < n; ++k) g += w->P[j * n + k] * xo[k];
            const double v = xo[j] - g / pjj;
            side[j] = v <= elo[j] ? -1 : (v >= ehi[j] ? 1 : 0);
            xv[j] = side[j] < 0 ? elo[j] : (side[j] > 0 ? ehi[j] : v);
        }
    }
    for (int i = n; i < m; ++i) if (boxrow[i] >= 0) flag[i] = 0;
    for (int j = 0; j < n; ++j) {
        if (!(w->P[j * n + j] > 0)) continue;
        flag[j] = 0;
        if (!side[j]) continue;
        const int r = side[j] < 0 ? blo[j] : bhi[j];
        if (r == j) { flag[j] = side[j]; continue; }
        const double g = w->A[r * n + j];
        /* row r binds at its l (g > 0 bounds from below, g < 0 from above) or u */
        const int at_l = (side[j] < 0) == (g > 0);
        flag[r] = at_l ? -1 : 1;
    }
}

/* polish_guess = 2 adds this to polish_guess_jacobi: a slack variable (no
 * cost curvature, a nonzero linear cost, in exactly one G row r) keeps its
 * bound active only while its bound multiplier from stationarity with the
 * ADMM dual of row r, y_b = -(q_j + g_rj y_r) / ab_j, is below
 * -POLISH_SLACK_TOL |q_j| / ab_j; a row dual that has grown to a large share
 * of the slack's cost marks a row the optimum pays to violate (slack free).
 * FR3 bench workload: 1.55 -> 1.45 EQP solves per polish
 * (tools/polish_census.py).  Kernel: polish() in qp_solver.hpp. */
#define POLISH_SLACK_TOL 0.3
static void polish_guess_slack(const QPW* w, int* flag) {
    int n = w->n, m = w->m;
    for (int j = 0; j < n; ++j) {
        if (w->P[j * n + j] != 0 || w->q[j] == 0) continue;
        int r = -1, cnt = 0;
        for (int i = n; i < m; ++i)
            if (w->A[i * n + j] != 0) { r = i; ++cnt; }
        if (cnt != 1) continue;
        const double ab = w->A[j * n + j], yb = -(w->q[j] + w->A[r * n + j] * w->y[r]) / ab;
        flag[j] = yb < -POLISH_SLACK_TOL * fabs(w->q[j]) / ab ? -1 : 0;
    }
}

static __thread int pcg[PC_RULES][ORC_MAXC];
/* the polish from one first guess of the active set (flag, modified) */
static int qp_polish_from(QPW* w, const OracleSettings* s, int strict, int* flag, double pr0, double dr0,
                          int census, int drop) {
    int n = w->n, m = w->m;
    Res tmp;
    double xp[ORC_MAXX], yp[ORC_MAXC], zp[ORC_MAXC], ax[ORC_MAXC], xc[ORC_MAXX];
    int have_feasible = 0, neqp = 0;
    for (int it = 0; it < (strict ? g_feas_att + POLISH_AS_ITERS : 1); ++it) {
        polish_drop_fixed_rows(w, flag);
        ++neqp;
        if (census) pc_add(PC_EQP, 1);
        if (!qp_eqp(w, s, flag, xp, yp)) return 0;
        double stepmax = 0, xnorm = 0;
        if (have_feasible) {
            for (int j = 0; j < n; ++j) { stepmax = fmax(stepmax, fabs(xp[j] - xc[j])); xnorm = fmax(xnorm, fabs(xc[j])); }
        }
        if (have_feasible && stepmax > 1e-12 * (1 + xnorm)) {
            /* ratio test along p = xp - xc over the inactive rows */
            double amin = 1.0;
            int blk = -1, side = 0;
            for (int i = 0; i < m; ++i) {
                if (flag[i]) continue;
                double axc = 0, ap = 0;
                for (int j = 0; j < n; ++j) { axc += w->A[i * n + j] * xc[j]; ap += w->A[i * n + j] * (xp[j] - xc[j]); }
                double a = 2.0;
                int sd = 0;
                if (ap < 0 && w->l[i] > -INFTY * MIN_SCALING) { a = (w->l[i] - axc) / ap; sd = -1; }
                else if (ap > 0 && w->u[i] < INFTY * MIN_SCALING) { a = (w->u[i] - axc) / ap; sd = 1; }
                if (a < amin) { amin = a; blk = i; side = sd; }
            }
            double alpha = amin < 0 ? 0 : amin;
            for (int j = 0; j < n; ++j) xc[j] += alpha * (xp[j] - xc[j]);
            if (blk >= 0) { flag[blk] = side; if (census) pc_add(PC_RATIO, 1); continue; }
            /* full step: xc is the EQP minimiser, fall through to the checks */
        }
        for (int i = 0; i < m; ++i) {
            double t = 0;
            for (int j = 0; j < n; ++j) t += w->A[i * n + j] * xp[j];
            ax[i] = t;
            zp[i] = t < w->l[i] ? w->l[i] : (t > w->u[i] ? w->u[i] : t);
        }
        qp_residuals(w, &tmp, xp, zp, yp, s->eps_exact, s->eps_exact);
        int ok = (tmp.pri_res < pr0 && tmp.dua_res < dr0) || (tmp.pri_res < pr0 && dr0 < 1e-10) || (tmp.dua_res < dr0 && pr0 < 1e-10);
        int worst = -1;
        double wv = 0;
        if (strict) {
            int feasible = tmp.pri_res <= tmp.eps_pri;
            ok = feasible && tmp.dua_res <= tmp.eps_dua;
            for (int i = 0; i < m; ++i) {
                if (!flag[i] || w->l[i] == w->u[i]) continue;
                double yi = w->E[i] * yp[i] * w->cinv;
                double viol = flag[i] < 0 ? yi - tmp.eps_dua : -yi - tmp.eps_dua;
                if (viol > wv) { wv = viol; worst = i; }
            }
            if (worst >= 0) ok = 0;
            if (getenv("ORC_DEBUG")) {
                fprintf(stderr, "polish it %d feas %d pri %.2e dua %.2e worst %d (%.2e) havefeas %d flags", it, feasible,
                        tmp.pri_res, tmp.dua_res, worst, wv, have_feasible);
                for (int i = 0; i < m; ++i) if (flag[i]) fprintf(stderr, " %d%c", i, flag[i] < 0 ? 'l' : 'u');
                fprintf(stderr, "\n");
            }
            if (!ok && feasible && !have_feasible) { memcpy(xc, xp, n * sizeof(double)); have_feasible = 1; }
        }
        if (ok) {
            memcpy(w->x, xp, n * sizeof(double));
            memcpy(w->y, yp, m * sizeof(double));
            memcpy(w->z, zp, m * sizeof(double));
            w->r.pri_res = tmp.pri_res;
            w->r.dua_res = tmp.dua_res;
            if (census) {
                pc_add(PC_OK, 1);
                if (neqp == 1) pc_add(PC_OK1, 1);
                pc_add(PC_HIST0 + (neqp < 8 ? neqp - 1 : 7), 1);
                for (int r = 0; r < PC_RULES; ++r) {
                    int fn = 0, fp = 0;
                    for (int i = 0; i < m; ++i) {
                        if (flag[i] && pcg[r][i] != flag[i]) ++fn;
                        else if (!flag[i] && pcg[r][i]) ++fp;
                    }
                    if (!fn && !fp) pc_add(PC_MATCH0 + r, 1);
                    if (r == 0)
                        for (int i = 0; i < m; ++i) {
                            if (flag[i] && pcg[r][i] != flag[i]) __atomic_fetch_add(&g_pc_row[0][i], 1, __ATOMIC_RELAXED);
                            else if (!flag[i] && pcg[r][i]) __atomic_fetch_add(&g_pc_row[1][i], 1, __ATOMIC_RELAXED);
                            if (flag[i]) __atomic_fetch_add(&g_pc_row[2][i], 1, __ATOMIC_RELAXED);
                        }
                    pc_add(PC_FN0 + r, fn);
                    pc_add(PC_FP0 + r, fp);
                }
            }
            return 1;
        }
        if (!strict) return 0;
        if (have_feasible) {
            if (worst < 0) return 0;   /* KKT residual failure, not an active-set issue */
            flag[worst] = 0;
            if (census) pc_add(PC_DROP, 1);
            memcpy(xc, xp, n * sizeof(double));
        } else {
            if (census) pc_add(PC_ADD, 1);
            if (it >= g_feas_att - 1) return 0;
            /* not yet feasible: add every violated inactive row at its
             * violated side (QPIK: the ADMM guess typically misses a
             * couple), or only the most violated one (QPID) */
            int add[ORC_MAXC], nadd = 0, best = -1, bf = 0;
            double av = 0;
            for (int i = 0; i < m; ++i) {
                add[i] = 0;
                if (flag[i]) continue;
                double lo = (w->l[i] - ax[i]) * w->Einv[i] - tmp.eps_pri, hi = (ax[i] - w->u[i]) * w->Einv[i] - tmp.eps_pri;
                if (lo > 0 || hi > 0) { add[i] = hi > lo ? 1 : -1; ++nadd; }
                if (lo > av) { av = lo; best = i; bf = -1; }
                if (hi > av) { av = hi; best = i; bf = 1; }
            }
            if (nadd == 0) {
                if (worst < 0) return 0;
                flag[worst] = 0;
            } else if (s->polish_add_all) {
                /* ... and, in the first pass, the active row whose multiplier
                 * has the worst wrong sign leaves in the same step: otherwise
                 * a wrong row of the first guess stays until the set is
                 * feasible, and on some instances never gets there (FR3 bench
                 * stragglers: three failed polishes, 60 ADMM iterations;
                 * tools/straggler_study.py).  The multipliers of an
                 * infeasible EQP can also point at a right row (a Husky-FR3
                 * instance then cycled to 300 iterations), so the retry pass
                 * from OSQP's guess adds only.  Dropping every wrong-signed
                 * row measured worse (more EQPs); census in DESIGN.md. */
                for (int i = 0; i < m; ++i) if (add[i]) flag[i] = add[i];
                if (drop && worst >= 0) flag[worst] = 0;
            } else {
                flag[best] = bf;
            }
        }
    }
    return 0;
}

/* Parity mode: the polish from the QPIK guess (polish_guess >= 1); when that
 * fails and differs from OSQP's own guess, once more from OSQP's guess, so a
 * guess that keeps failing at every check (the ADMM duals it reads settle
 * slowly on some instances: a UR5e bench instance ran 1 400 ADMM iterations
 * without this) costs one extra attempt instead of the ADMM tail. */
static int qp_polish(QPW* w, const OracleSettings* s, int strict) {
    int m = w->m;
    int osqp[ORC_MAXC], flag[ORC_MAXC];  /* -1 lower-active, +1 upper-active, 0 inactive */
    for (int i = 0; i < m; ++i)
        osqp[i] = (w->z[i] - w->l[i] < -w->y[i]) ? -1 : ((w->u[i] - w->z[i] < w->y[i]) ? 1 : 0);
    memcpy(flag, osqp, m * sizeof(int));
    if (strict && s->polish_guess >= 1) polish_guess_jacobi(w, flag);
    if (strict && s->polish_guess >= 2) polish_guess_slack(w, flag);
    if (g_pc_guess >= 0 && g_pc_guess < 15 && strict) pc_guess(w, g_pc_guess, flag);
    if (g_pc_guess == 15 && strict) pc_guess_slacks(w, flag, g_pc_tol[15]);
    if (g_pc_guess == 16 && strict) pc_guess_effbox(w, flag);
    if (g_pc_guess == 17 && strict) { pc_guess_effbox(w, flag); pc_guess_slacks(w, flag, g_pc_tol[15]); }
    const int differs = memcmp(flag, osqp, m * sizeof(int)) != 0;
    const double pr0 = w->r.pri_res, dr0 = w->r.dua_res;
    const int census = g_pc_on && strict;
    if (census) {
        pc_add(PC_CALLS, 1);
        for (int r = 0; r < PC_RULES; ++r) pc_guess(w, r, pcg[r]);
    }
    const int d0 = g_feas_drop == 1 || g_feas_drop == 5, d1 = g_feas_drop == 1 || g_feas_drop == 4;
    if (qp_polish_from(w, s, strict, flag, pr0, dr0, census, d0)) return 1;
    /* (QPIK: the retry runs whenever the first pass fails -- it also differs
     * in the drop rule; QPID only from a different guess) */
    if (!strict || (!differs && !(s->polish_add_all && d0 != d1))) return 0;
    if (census) pc_add(PC_RETRY, 1);
    return qp_polish_from(w, s, strict, osqp, pr0, dr0, census, d1);
}

/* the last termination check's max(pri_res / eps_pri, dua_res / eps_dua) of
 * this thread's last oracle_solve_qp (OracleDiag.res_ratio) */
static __thread double g_res_ratio;
int oracle_solve_qp(int n, int m, const double* P, const double* qv, const double* A,
                    const double* l, const double* u, const OracleSettings* s,
                    double* x, double* y, int* iters, int* polished) {
    static __thread QPW w;
    w.n = n; w.m = m;
    for (int i = 0; i < n * n; ++i) if (!isfinite(P[i])) return ORC_NONFINITE;
    for (int i = 0; i < n; ++i) if (!isfinite(qv[i])) return ORC_NONFINITE;
    for (int i = 0; i < m * n; ++i) if (!isfinite(A[i])) return ORC_NONFINITE;
    for (int i = 0; i < m; ++i) if (isnan(l[i]) || isnan(u[i])) return ORC_NONFINITE;
    memcpy(w.P, P, n * n * sizeof(double));
    memcpy(w.q, qv, n * sizeof(double));
    memcpy(w.A, A, m * n * sizeof(double));
    for (int i = 0; i < m; ++i) { w.l[i] = fmax(l[i], -INFTY); w.u[i] = fmin(u[i], INFTY); }
    qp_scale(&w, s->scaling);
    for (int i = 0; i < m; ++i) {
        if (w.l[i] < -INFTY * MIN_SCALING && w.u[i] > INFTY * MIN_SCALING) w.ctype[i] = -1;
        else if (w.u[i] - w.l[i] < RHO_TOL) w.ctype[i] = 1;
        else w.ctype[i] = 0;
    }
    w.rho = s->rho;
    set_rho_vec(&w);
    qp_factor(&w, s->sigma);
    memset(w.x, 0, sizeof(w.x));
    memset(w.z, 0, sizeof(w.z));
    memset(w.y, 0, sizeof(w.y));
    int status = ORC_MAX_ITER, it, pol = 0, pfail = 0;
    g_res_ratio = NAN;
    double alpha = s->alpha;
    for (it = 1; it <= s->max_iter; ++it) {
        double xt[ORC_MAXX], zt[ORC_MAXC], rhs[ORC_MAXX];
        for (int j = 0; j < n; ++j) {
            double t = s->sigma * w.x[j] - w.q[j];
            for (int i = 0; i < m; ++i) t += w.A[i * n + j] * (w.rho_vec[i] * w.z[i] - w.y[i]);
            rhs[j] = t;
        }
        memcpy(xt, rhs, n * sizeof(double));
        chol_solve(w.L, n, xt);
        for (int i = 0; i < m; ++i) { double t = 0; for (int j = 0; j < n; ++j) t += w.A[i * n + j] * xt[j]; zt[i] = t; }
        for (int j = 0; j < n; ++j) w.x[j] = alpha * xt[j] + (1 - alpha) * w.x[j];
        for (int i = 0; i < m; ++i) {
            double zr = alpha * zt[i] + (1 - alpha) * w.z[i];
            double zn = zr + w.y[i] / w.rho_vec[i];
            zn = zn < w.l[i] ? w.l[i] : (zn > w.u[i] ? w.u[i] : zn);
            w.dy[i] = w.rho_vec[i] * (zr - zn);
            w.y[i] += w.dy[i];
            w.z[i] = zn;
        }
        int check = s->check_termination > 0 && it % s->check_termination == 0;
        int adapt = s->adaptive_rho && s->adaptive_rho_interval > 0 && it % s->adaptive_rho_interval == 0;
        if (check || adapt) qp_residuals(&w, &w.r, w.x, w.z, w.y, s->eps_abs, s->eps_rel);
        if (check) g_res_ratio = fmax(w.r.pri_res / w.r.eps_pri, w.r.dua_res / w.r.eps_dua);
        if (s->stop_at > 0 && it == s->stop_at) { status = ORC_SOLVED; break; }
        if (check && s->stop_at <= 0) {
            int conv = w.r.pri_res < w.r.eps_pri && w.r.dua_res < w.r.eps_dua;
            if (getenv("ORC_DEBUG") && it <= 200)
                fprintf(stderr, "it %d rho %.4g pri %.3e/%.3e dua %.3e/%.3e x3 %.6f\n", it, w.rho, w.r.pri_res, w.r.eps_pri,
                        w.r.dua_res, w.r.eps_dua, w.x[3] * w.D[3]);
            /* parity mode: a certified polish is exact whatever the ADMM
             * residual, so try it at every check (the active set settles
             * long before OSQP's eps_rel termination) */
            if (s->exact && !conv && pfail < POLISH_MAX_EARLY) {
                if (qp_polish(&w, s, 1)) { status = ORC_SOLVED; pol = 1; break; }
                ++pfail;
            }
            if (conv) {
                if (!s->exact) { status = ORC_SOLVED; break; }
                if (pfail < POLISH_MAX_TOTAL) {
                    if (qp_polish(&w, s, 1)) { status = ORC_SOLVED; pol = 1; break; }
                    ++pfail;
                }
                /* tight ADMM-only fallback */
                Res t2;
                qp_residuals(&w, &t2, w.x, w.z, w.y, s->eps_fallback, s->eps_fallback);
                if (t2.pri_res < t2.eps_pri && t2.dua_res < t2.eps_dua) { status = ORC_SOLVED; break; }
            } else if (qp_primal_infeasible(&w, s->eps_prim_inf)) {
                status = ORC_PRIMAL_INFEASIBLE;
                break;
            }
        }
        if (adapt) {
            double pr = w.r.pri_res_s / (fmax(w.r.nAx_s, w.r.nz_s) + DIVISION_TOL);
            double dr = w.r.dua_res_s / (fmax(fmax(w.r.nq_s, w.r.nAty_s), w.r.nPx_s) + DIVISION_TOL);
            double rn = w.rho * sqrt(pr / (dr + DIVISION_TOL));
            rn = fmin(fmax(rn, RHO_MIN), RHO_MAX);
            if (rn > w.rho * s->adaptive_rho_tolerance || rn < w.rho / s->adaptive_rho_tolerance) {
                w.rho = rn;
                set_rho_vec(&w);
                qp_factor(&w, s->sigma);
            }
        }
    }
    if (status == ORC_SOLVED && s->polish && !s->exact && !pol) pol = qp_polish(&w, s, 0);
    *iters = it > s->max_iter ? s->max_iter : it;
    *polished = pol;
    for (int j = 0; j < n; ++j) x[j] = w.D[j] * w.x[j];
    for (int i = 0; i < m; ++i) y[i] = w.E[i] * w.y[i] / w.c;
    return status;
}

/* ------------------------------------------------------------------------ */
/* controller entry: QPIK / QPIKStep / QPIKCubic                            */
/* ------------------------------------------------------------------------ */
void oracle_default_params(int kind, OracleParams* p, int exact) {
    memset(p, 0, sizeof(*p));
    for (int i = 0; i < 6; ++i) {
        p->kp[i] = kind == 0 ? 100 : 400;   /* robot_controller.cpp:12 / MoMa :15 */
        p->kv[i] = kind == 0 ? 20 : 0;      /* MoMa QPIKStep has no Kv term (:177) */
    }
    p->alpha_cbf = 50;
    p->w_reg = kind == 0 ? 1.0 : 0.01;
    p->slack_w = 1000;
    p->man_min = 0.01;
    p->dist_min = 0.05;
    p->mode = 1;
    OracleSettings* s = &p->solver;
    s->rho = 0.1; s->sigma = 1e-6; s->alpha = 1.6;
    s->eps_abs = 1e-3; s->eps_rel = 1e-3; s->eps_prim_inf = 1e-4;
    s->max_iter = 4000; s->check_termination = 25; s->scaling = 10;
    s->adaptive_rho = 1; s->adaptive_rho_interval = 25; s->adaptive_rho_tolerance = 5;
    s->polish = exact ? 1 : 0; s->polish_refine_iter = 3; s->delta = 1e-6;
    s->exact = exact; s->eps_exact = 1e-9; s->eps_fallback = 1e-7;
    /* the kernel's QPIK polish KKT cap (kEqpRegCap, its register EQP): a
     * larger reduced KKT fails that polish attempt and ADMM continues.  The
     * whole-body QP (no variable bounds) is uncapped, as the kernel's LDS EQP
     * takes N > 16 there (D16) */
    s->polish_cap = kind == 0 ? 16 : 0;
    s->polish_add_all = 1;
    s->polish_guess = exact ? 2 : 0;
    /* parity mode: the first polish at iteration 8 (manipulators) / 2 (whole-body)
     * (kernel: drc_default_qpik_params) */
    if (exact) s->check_termination = kind == 0 ? 8 : 2;
    /* parity mode: one (manipulators) / two (whole-body) Ruiz passes
     * (kernel: drc_default_qpik_params) */
    if (exact) s->scaling = kind == 0 ? 1 : 2;
}

/* Farkas certificate for the whole-body QP (mobile_manipulator/QP_IK.cpp:
 * 75-128: no slacks, no variable bounds).  Rows: the arm's CBF box
 * blo_i = lg[i] <= v_i <= bhi_i = -lg[n+i], and gm.v >= lg[2n], gd.v >= lg[2n+1].
 * Infeasible iff min over mu in [0,1] of phi(mu) = sum_i max(g_i blo_i,
 * g_i bhi_i) - (mu rm + (1-mu) rd) < 0 with g = mu gm + (1-mu) gd; phi is
 * convex piecewise linear, minimised at mu = 1, 0 or a root of some g_i.
 * Certified only below -1e-6 (1 + scale) (a point the exact-mode polish
 * accepts has residuals ~1e-9).  Test infrastructure restating the kernel's
 * moma_lp_infeasible: same candidates, summation order and margin. */
static int moma_lp_infeasible(int n, const double* gm, const double* gd, const double* lg) {
    const double rm = lg[2 * n], rd = lg[2 * n + 1];
    for (int c = 0; c < n + 2; ++c) {
        double mu = -1.0;
        if (c == 0) mu = 1.0;
        else if (c == 1) mu = 0.0;
        else {
            int i = c - 2;
            double den = gm[i] - gd[i];
            if (den != 0.0) {
                double t = -gd[i] / den;
                if (t > 0.0 && t < 1.0) mu = t;
            }
        }
        if (!(mu >= 0.0)) continue;
        double scale = fabs(rm) + fabs(rd), phi = -(mu * rm + (1.0 - mu) * rd);
        for (int i = 0; i < n; ++i) {
            double blo = lg[i], bhi = -lg[n + i], g = mu * gm[i] + (1.0 - mu) * gd[i];
            phi += fmax(g * blo, g * bhi);
            scale += (fabs(gm[i]) + fabs(gd[i])) * fmax(fabs(blo), fabs(bhi));
        }
        if (phi < -1e-6 * (1.0 + scale)) return 1;
    }
    return 0;
}

/* dist_in (optional): the distance stage (d, grad[nv]) supplied by the caller
 * instead of computed — parity tests feed the device's narrow-phase result so
 * the QP assembly and solve are compared on identical distance data */
static int qpik_one_impl(const OracleModel* m, const OracleParams* p, const double* q, const double* qdot,
                         const double* x_target, const double* xdot_target, const double* x_init,
                         const double* xdot_init, const double* dist_in, const double* man_in, double* out,
                         OracleDiag* diag) {
    int nv = m->nv;
    Kin k;
    kin_fk(m, q, &k);
    double J[6 * ORC_MAXJ];
    point_jacobian(m, &k, m->ee_joint, k.pe, J);
    int moma = m->kind == 1;
    int na = moma ? m->n_wheel + m->n_arm : nv;
    /* selection matrix (MoMa robot_data.cpp:24-25,115-120) */
    double S[ORC_MAXJ * ORC_MAXJ];
    if (moma) {
        memset(S, 0, sizeof(double) * nv * na);
        for (int i = 0; i < m->n_arm; ++i) S[(m->mani_start + i) * na + m->act_mani_start + i] = 1;
        for (int i = 0; i < m->n_wheel; ++i) S[(m->mobi_start + i) * na + m->act_mobi_start + i] = 1;
        double yaw = q[m->virtual_start + 2], cy = cos(yaw), sy = sin(yaw);
        double Rz[9] = {cy, -sy, 0, sy, cy, 0, 0, 0, 1}, Jmob[3][8];
        mobile_fk_jac(m, q, Jmob);
        for (int r = 0; r < 3; ++r)
            for (int wcol = 0; wcol < m->n_wheel; ++wcol) {
                double s = 0;
                for (int c = 0; c < 3; ++c) s += Rz[3 * r + c] * Jmob[c][wcol];
                S[(m->virtual_start + r) * na + m->act_mobi_start + wcol] = s;
            }
    }
    /* task error and desired task velocity */
    double xdot_des[6];
    if (p->mode == 0) memcpy(xdot_des, xdot_target, sizeof(xdot_des));
    else {
        double xt[12], xdt[6];
        if (p->mode == 2) task_space_cubic(x_target, xdot_target, x_init, xdot_init, p->t, p->t0, p->duration, xt, xdt);
        else { memcpy(xt, x_target, sizeof(xt)); memcpy(xdt, xdot_target, sizeof(xdt)); }
        double Rt[9], pt[3];
        pose_unpack(xt, Rt, pt);
        double xd[6];  /* getVelocity = J qdot (robot_data.cpp:419-422) */
        for (int i = 0; i < 6; ++i) { double s = 0; for (int c = 0; c < nv; ++c) s += J[i * nv + c] * qdot[c]; xd[i] = s; }
        double e[6];
        for (int i = 0; i < 3; ++i) e[i] = pt[i] - k.pe[i];
        /* getPhi(R_target, R) = -1/2 sum_i Rt[:,i] x R[:,i] */
        double phi[3] = {0, 0, 0};
        for (int i = 0; i < 3; ++i) {
            double a[3] = {Rt[i], Rt[3 + i], Rt[6 + i]}, b[3] = {k.Te[i], k.Te[3 + i], k.Te[6 + i]}, c[3];
            cross3(a, b, c);
            phi[0] += c[0]; phi[1] += c[1]; phi[2] += c[2];
        }
        for (int i = 0; i < 3; ++i) e[3 + i] = -0.5 * phi[i];
        for (int i = 0; i < 6; ++i)
            xdot_des[i] = moma ? p->kp[i] * e[i] + xdt[i] : p->kp[i] * e[i] + p->kv[i] * (xdt[i] - xd[i]);
    }
    /* manipulability + min distance */
    double man, mgrad[ORC_MAXJ], dist, dgrad[ORC_MAXJ];
    int pair;
    int c0 = moma ? m->mani_start : 0, narm = moma ? m->n_arm : nv;
    if (man_in) { man = man_in[0]; memcpy(mgrad, man_in + 1, narm * sizeof(double)); }
    else manip(m, &k, J, c0, narm, &man, mgrad);
    if (dist_in) { dist = dist_in[0]; memcpy(dgrad, dist_in + 1, nv * sizeof(double)); pair = -1; }
    else min_distance(m, &k, &dist, dgrad, &pair);
    /* QP assembly */
    static __thread double P[ORC_MAXX * ORC_MAXX], A[ORC_MAXC * ORC_MAXX];
    double qv[ORC_MAXX], l[ORC_MAXC], u[ORC_MAXC];
    int nx, nc;
    double a = p->alpha_cbf;
    if (!moma) {
        int n = nv;
        nx = 3 * n + 2;
        int ng = 2 * n + 2;
        nc = nx + ng;
        memset(P, 0, sizeof(double) * nx * nx);
        memset(A, 0, sizeof(double) * nc * nx);
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j) {
                double s = 0;
                for (int r = 0; r < 6; ++r) s += J[r * nv + i] * J[r * nv + j];
                P[i * nx + j] = 2 * s + (i == j ? p->w_reg : 0);
            }
        for (int i = 0; i < n; ++i) { double s = 0; for (int r = 0; r < 6; ++r) s += J[r * nv + i] * xdot_des[r]; qv[i] = -2 * s; }
        for (int i = n; i < nx; ++i) qv[i] = p->slack_w;
        for (int i = 0; i < nx; ++i) A[i * nx + i] = 1;
        for (int i = 0; i < n; ++i) { l[i] = -m->vel[i]; u[i] = m->vel[i]; }
        for (int i = n; i < nx; ++i) { l[i] = 0; u[i] = INFTY; }
        double* G = A + nx * nx;
        double* lg = l + nx;
        for (int i = 0; i < n; ++i) {
            G[i * nx + i] = 1; G[i * nx + n + i] = 1; lg[i] = -a * (q[i] - m->lower[i]);
            G[(n + i) * nx + i] = -1; G[(n + i) * nx + 2 * n + i] = 1; lg[n + i] = -a * (m->upper[i] - q[i]);
        }
        for (int c = 0; c < n; ++c) { G[(2 * n) * nx + c] = mgrad[c]; G[(2 * n + 1) * nx + c] = dgrad[c]; }
        G[(2 * n) * nx + 3 * n] = 1; G[(2 * n + 1) * nx + 3 * n + 1] = 1;
        lg[2 * n] = -a * (man - p->man_min);
        lg[2 * n + 1] = -a * (dist - p->dist_min);
        for (int i = nx; i < nc; ++i) u[i] = INFTY;
    } else {
        int n = m->n_arm;
        nx = na;
        int ng = 2 * n + 2;
        nc = nx + ng;
        double Jt[6 * ORC_MAXJ];
        for (int r = 0; r < 6; ++r)
            for (int c = 0; c < na; ++c) { double s = 0; for (int j = 0; j < nv; ++j) s += J[r * nv + j] * S[j * na + c]; Jt[r * na + c] = s; }
        memset(A, 0, sizeof(double) * nc * nx);
        for (int i = 0; i < na; ++i)
            for (int j = 0; j < na; ++j) {
                double s = 0;
                for (int r = 0; r < 6; ++r) s += Jt[r * na + i] * Jt[r * na + j];
                P[i * nx + j] = 2 * s + (i == j ? p->w_reg : 0);
            }
        for (int i = 0; i < na; ++i) { double s = 0; for (int r = 0; r < 6; ++r) s += Jt[r * na + i] * xdot_des[r]; qv[i] = -2 * s; }
        for (int i = 0; i < nx; ++i) { A[i * nx + i] = 1; l[i] = -INFTY; u[i] = INFTY; }
        double* G = A + nx * nx;
        double* lg = l + nx;
        int as = m->act_mani_start, js = m->mani_start;
        for (int i = 0; i < n; ++i) {
            G[i * nx + as + i] = 1; lg[i] = -a * (q[js + i] - m->lower[js + i]);
            G[(n + i) * nx + as + i] = -1; lg[n + i] = -a * (m->upper[js + i] - q[js + i]);
        }
        for (int c = 0; c < n; ++c) { G[(2 * n) * nx + as + c] = mgrad[c]; G[(2 * n + 1) * nx + as + c] = dgrad[js + c]; }
        lg[2 * n] = -a * (man - p->man_min);
        lg[2 * n + 1] = -a * (dist - p->dist_min);
        for (int i = nx; i < nc; ++i) u[i] = INFTY;
    }
    double x[ORC_MAXX], y[ORC_MAXC];
    int iters = 0, pol = 0;
    int st;
    /* exact mode, whole-body QP: an LP-certified infeasible instance returns
     * PrimalInfeasible without the ADMM (the kernel's moma_lp_infeasible, D15);
     * non-finite data keeps OSQP's check (the certificate never fires on it) */
    if (moma && p->solver.exact &&
        moma_lp_infeasible(m->n_arm, A + (nx + 2 * m->n_arm) * nx + m->act_mani_start,
                           A + (nx + 2 * m->n_arm + 1) * nx + m->act_mani_start, l + nx))
        st = ORC_PRIMAL_INFEASIBLE;
    else
        st = oracle_solve_qp(nx, nc, P, qv, A, l, u, &p->solver, x, y, &iters, &pol);
    /* QP_IK.cpp:53-67 / MoMa :43-57: zero on any non-Solved status */
    for (int i = 0; i < na; ++i) out[i] = st == ORC_SOLVED ? x[i] : 0.0;
    if (diag) {
        for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) diag->pose[3 * r + c] = k.Te[3 * r + c];
        memcpy(diag->pose + 9, k.pe, 3 * sizeof(double));
        memcpy(diag->J, J, 6 * nv * sizeof(double));
        memcpy(diag->xdot_des, xdot_des, sizeof(xdot_des));
        diag->man = man;
        memcpy(diag->man_grad, mgrad, narm * sizeof(double));
        diag->dist = dist;
        memcpy(diag->dist_grad, dgrad, nv * sizeof(double));
        diag->pair = pair;
        diag->iters = iters;
        diag->polished = pol;
        diag->res_ratio = g_res_ratio;
    }
    return st;
}

int oracle_qpik_one(const OracleModel* m, const OracleParams* p, const double* q, const double* qdot,
                    const double* x_target, const double* xdot_target, const double* x_init,
                    const double* xdot_init, double* out, OracleDiag* diag) {
    return qpik_one_impl(m, p, q, qdot, x_target, xdot_target, x_init, xdot_init, NULL, NULL, out, diag);
}

/* ------------------------------------------------------------------------ */
/* controller entry: QPID / QPIDStep / QPIDCubic                            */
/* ------------------------------------------------------------------------ */
void oracle_default_qpid_params(int kind, OracleParams* p, int exact) {
    oracle_default_params(kind, p, exact);
    for (int i = 0; i < 6; ++i) {
        p->kp[i] = kind == 0 ? 100 : 400;   /* robot_controller.cpp:12-13 / MoMa :15-16 */
        p->kv[i] = kind == 0 ? 20 : 40;     /* MoMa QPIDStep uses Kv (:230)            */
    }
    p->w_reg = 0;                           /* QP_ID.cpp:102 regulariser commented out */
    /* P = 2 J^T J is singular on null(J) (no regulariser) and the cost
     * scaling (slack weight 1000) leaves eigenvalues of the scaled reduced KKT
     * near OSQP's delta = 1e-6, where 3 refinement steps cannot certify at
     * eps_exact: parity mode regularises the polish with delta = 1e-10 */
    if (exact) p->solver.delta = 1e-10;
    p->solver.polish_cap = 48;              /* the kernel's QPID polish KKT (ncap)     */
    p->solver.polish_add_all = 0;           /* one row per step (kernel: problem 1)    */
    p->solver.polish_guess = 0;             /* OSQP's first guess (kernel: problem 1)  */
    p->solver.polish_refine_iter = 3;       /* OSQP's refinement count (kernel: QPID)  */
    p->solver.check_termination = 25;       /* OSQP's check interval (kernel: QPID)    */
    p->solver.scaling = 10;                 /* OSQP's Ruiz passes (kernel: QPID)       */
}

/* Manipulator::QPID (src/manipulator/QP_ID.cpp:7-193) and MobileManipulator::
 * QPID (src/mobile_manipulator/QP_ID.cpp:7-184) through the controllers'
 * QPID / QPIDStep / QPIDCubic (robot_controller.cpp:319-361; MoMa :199-250).
 * M, g: the (actuated, for MoMa) mass matrix and gravity the QP's equality
 * rows use (getMassMatrix / getGravity, or the *Actuated getters), row-major
 * na x na and na; g_full: the full joint-order gravity (MoMa failure path,
 * robot_controller.cpp:211,218 — the reference slices the joint-order vector
 * at actuator offsets; restated as written).  Outputs qdd[na], tau[na]:
 * non-Solved -> qdd = 0, tau = g (manipulator :335) / g_full[0..na) (MoMa). */
int oracle_qpid_one(const OracleModel* m, const OracleParams* p, const double* q, const double* qdot,
                    const double* x_target, const double* xdot_target, const double* x_init,
                    const double* xdot_init, const double* Mq, const double* gq, const double* g_full,
                    double* qdd, double* tau, OracleDiag* diag) {
    int nv = m->nv;
    Kin k;
    kin_fk(m, q, &k);
    double J[6 * ORC_MAXJ];
    point_jacobian(m, &k, m->ee_joint, k.pe, J);
    int moma = m->kind == 1;
    int na = moma ? m->n_wheel + m->n_arm : nv;
    double S[ORC_MAXJ * ORC_MAXJ];
    double eta[ORC_MAXJ], v[ORC_MAXJ];   /* eta = qdot_actuated, v = S eta */
    if (moma) {
        memset(S, 0, sizeof(double) * nv * na);
        for (int i = 0; i < m->n_arm; ++i) S[(m->mani_start + i) * na + m->act_mani_start + i] = 1;
        for (int i = 0; i < m->n_wheel; ++i) S[(m->mobi_start + i) * na + m->act_mobi_start + i] = 1;
        double yaw = q[m->virtual_start + 2], cy = cos(yaw), sy = sin(yaw);
        double Rz[9] = {cy, -sy, 0, sy, cy, 0, 0, 0, 1}, Jmob[3][8];
        mobile_fk_jac(m, q, Jmob);
        for (int r = 0; r < 3; ++r)
            for (int wc = 0; wc < m->n_wheel; ++wc) {
                double t = 0;
                for (int c = 0; c < 3; ++c) t += Rz[3 * r + c] * Jmob[c][wc];
                S[(m->virtual_start + r) * na + m->act_mobi_start + wc] = t;
            }
        for (int i = 0; i < m->n_arm; ++i) eta[m->act_mani_start + i] = qdot[m->mani_start + i];
        for (int i = 0; i < m->n_wheel; ++i) eta[m->act_mobi_start + i] = qdot[m->mobi_start + i];
        for (int j = 0; j < nv; ++j) { double t = 0; for (int a = 0; a < na; ++a) t += S[j * na + a] * eta[a]; v[j] = t; }
    } else {
        memcpy(v, qdot, nv * sizeof(double));
    }
    /* desired task acceleration */
    double xdd[6];
    if (p->mode == 0) memcpy(xdd, xdot_target, sizeof(xdd));   /* QPID(xddot_target) */
    else {
        double xt[12], xdt[6];
        if (p->mode == 2) task_space_cubic(x_target, xdot_target, x_init, xdot_init, p->t, p->t0, p->duration, xt, xdt);
        else { memcpy(xt, x_target, sizeof(xt)); memcpy(xdt, xdot_target, sizeof(xdt)); }
        double Rt[9], pt[3], xd[6], e[6], phi[3] = {0, 0, 0};
        pose_unpack(xt, Rt, pt);
        for (int i = 0; i < 6; ++i) { double t = 0; for (int c = 0; c < nv; ++c) t += J[i * nv + c] * qdot[c]; xd[i] = t; }
        for (int i = 0; i < 3; ++i) e[i] = pt[i] - k.pe[i];
        for (int i = 0; i < 3; ++i) {
            double a[3] = {Rt[i], Rt[3 + i], Rt[6 + i]}, b[3] = {k.Te[i], k.Te[3 + i], k.Te[6 + i]}, c[3];
            cross3(a, b, c);
            phi[0] += c[0]; phi[1] += c[1]; phi[2] += c[2];
        }
        for (int i = 0; i < 3; ++i) e[3 + i] = -0.5 * phi[i];
        /* QPIDStep: Kp e + Kv (xdot_target - xdot) (robot_controller.cpp:347; MoMa :230) */
        for (int i = 0; i < 6; ++i) xdd[i] = p->kp[i] * e[i] + p->kv[i] * (xdt[i] - xd[i]);
    }
    /* Jdot (frame, full qdot) and its product with S eta / qdot */
    double Jd[6 * ORC_MAXJ], bias[6];
    point_jacobian_dot(m, &k, m->ee_joint, k.pe, qdot, ORC_ALL_JOINTS, Jd);
    for (int i = 0; i < 6; ++i) { double t = 0; for (int c = 0; c < nv; ++c) t += Jd[i * nv + c] * v[c]; bias[i] = t; }
    /* manipulability (+grad, grad_dot) and min distance (+grad, grad_dot) */
    int c0 = moma ? m->mani_start : 0, n = moma ? m->n_arm : nv;
    double man, mgrad[ORC_MAXJ], mgd[ORC_MAXJ], dist, dgrad[ORC_MAXJ], dgd[ORC_MAXJ], wA[3], wB[3];
    int pair;
    manip(m, &k, J, c0, n, &man, mgrad);
    manip_graddot(m, &k, J, c0, n, qdot, man, mgd);
    min_distance_w(m, &k, &dist, dgrad, &pair, wA, wB);
    mindist_graddot(m, &k, pair, wA, wB, qdot, dgd);
    const double* qa = q + c0;      /* arm joint positions / velocities */
    const double* qda = qdot + c0;
    double man_gd = 0, dist_gd = 0, mg_qd = 0, dg_qd = 0;
    for (int i = 0; i < n; ++i) {
        man_gd += mgd[i] * qda[i];
        dist_gd += dgd[c0 + i] * qda[i];
        mg_qd += mgrad[i] * qda[i];
        dg_qd += dgrad[c0 + i] * qda[i];
    }
    /* task Jacobian over the QP's task variables */
    double Jt[6 * ORC_MAXJ];
    if (moma) {
        for (int r = 0; r < 6; ++r)
            for (int c = 0; c < na; ++c) { double t = 0; for (int j = 0; j < nv; ++j) t += J[r * nv + j] * S[j * na + c]; Jt[r * na + c] = t; }
    } else {
        memcpy(Jt, J, 6 * nv * sizeof(double));
    }
    /* QP assembly */
    static __thread double P[ORC_MAXX * ORC_MAXX], A[ORC_MAXC * ORC_MAXX];
    double qv[ORC_MAXX], l[ORC_MAXC], u[ORC_MAXC];
    const double a = p->alpha_cbf;
    const int nb = moma ? 0 : 1;                    /* bound rows present (nbc = nx or 0) */
    const int nx = moma ? 2 * na : 6 * n + 2;       /* QP_ID.cpp:48-56 / MoMa :22 */
    const int nineq = 4 * n + 2, neq = na, nc = nb * nx + nineq + neq;
    const int as = moma ? m->act_mani_start : 0;    /* QP column of arm joint 0 */
    memset(P, 0, sizeof(double) * nx * nx);
    memset(A, 0, sizeof(double) * nc * nx);
    for (int i = 0; i < nx; ++i) qv[i] = 0;
    for (int i = 0; i < na; ++i)
        for (int j = 0; j < na; ++j) {
            double t = 0;
            for (int r = 0; r < 6; ++r) t += Jt[r * na + i] * Jt[r * na + j];
            P[i * nx + j] = 2 * t + (i == j ? p->w_reg : 0);
        }
    for (int i = 0; i < na; ++i) { double t = 0; for (int r = 0; r < 6; ++r) t += Jt[r * na + i] * (xdd[r] - bias[r]); qv[i] = -2 * t; }
    int row = 0;
    if (nb) {   /* setBoundConstraint (QP_ID.cpp:112-120): slacks >= 0, the rest free */
        for (int i = 0; i < nx; ++i) { A[i * nx + i] = 1; l[i] = i < 2 * n ? -INFTY : 0; u[i] = INFTY; }
        for (int i = 2 * n; i < nx; ++i) qv[i] = p->slack_w;
        row = nx;
    }
    double* G = A + row * nx;
    double* lg = l + row;
    double* ug = u + row;
    for (int i = 0; i < nineq; ++i) ug[i] = INFTY;
    for (int i = 0; i < n; ++i) {
        const int j = c0 + i;
        G[i * nx + as + i] = 1;               lg[i] = -2 * a * qda[i] - a * a * (qa[i] - m->lower[j]);
        G[(n + i) * nx + as + i] = -1;        lg[n + i] = 2 * a * qda[i] - a * a * (m->upper[j] - qa[i]);
        G[(2 * n + i) * nx + as + i] = 1;     lg[2 * n + i] = -a * (qda[i] + m->vel[j]);
        G[(3 * n + i) * nx + as + i] = -1;    lg[3 * n + i] = -a * (m->vel[j] - qda[i]);
        if (!moma) {
            G[i * nx + 2 * n + i] = 1; G[(n + i) * nx + 3 * n + i] = 1;
            G[(2 * n + i) * nx + 4 * n + i] = 1; G[(3 * n + i) * nx + 5 * n + i] = 1;
        }
    }
    for (int c = 0; c < n; ++c) { G[(4 * n) * nx + as + c] = mgrad[c]; G[(4 * n + 1) * nx + as + c] = dgrad[c0 + c]; }
    if (!moma) { G[(4 * n) * nx + 6 * n] = 1; G[(4 * n + 1) * nx + 6 * n + 1] = 1; }
    lg[4 * n] = -man_gd - 2 * a * mg_qd - a * a * (man - p->man_min);
    lg[4 * n + 1] = -dist_gd - 2 * a * dg_qd - a * a * (dist - p->dist_min);
    /* setEqConstraint: [M -I][qdd; tau] = -g (QP_ID.cpp:176-192) */
    double* Ge = G + nineq * nx;
    for (int i = 0; i < na; ++i) {
        for (int j = 0; j < na; ++j) Ge[i * nx + j] = Mq[i * na + j];
        Ge[i * nx + na + i] = -1;
        lg[nineq + i] = ug[nineq + i] = -gq[i];
    }
    double x[ORC_MAXX], y[ORC_MAXC];
    int iters = 0, pol = 0;
    int st = oracle_solve_qp(nx, nc, P, qv, A, l, u, &p->solver, x, y, &iters, &pol);
    for (int i = 0; i < na; ++i) {
        qdd[i] = st == ORC_SOLVED ? x[i] : 0.0;
        tau[i] = st == ORC_SOLVED ? x[na + i] : (moma ? g_full[i] : gq[i]);
    }
    if (diag) {
        for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) diag->pose[3 * r + c] = k.Te[3 * r + c];
        memcpy(diag->pose + 9, k.pe, 3 * sizeof(double));
        memcpy(diag->J, J, 6 * nv * sizeof(double));
        memcpy(diag->xdot_des, xdd, sizeof(xdd));
        diag->man = man;
        memcpy(diag->man_grad, mgrad, n * sizeof(double));
        diag->dist = dist;
        memcpy(diag->dist_grad, dgrad, nv * sizeof(double));
        diag->pair = pair;
        diag->iters = iters;
        diag->polished = pol;
        diag->res_ratio = g_res_ratio;
        memcpy(diag->jdot_v, bias, sizeof(bias));
        memcpy(diag->man_graddot, mgd, n * sizeof(double));
        memcpy(diag->dist_graddot, dgd, nv * sizeof(double));
        diag->man_gd = man_gd;
        diag->dist_gd = dist_gd;
        memcpy(diag->Jdot, Jd, 6 * nv * sizeof(double));
    }
    return st;
}

/* ------------------------------------------------------------------------ */
/* closed-form controllers: CLIK and OSF                 */
/* robot_controller.cpp:156-275                                             */
/* ------------------------------------------------------------------------ */
/* getTaskSpaceError(x_t, xd_t, getPose, getVelocity) after the optional
 * getTaskSpaceCubic (mode 2): e (6) and edot = xdot_target - J qdot (6) */
static void task_error(const OracleModel* m, const Kin* k, const double* J, const OracleParams* p,
                       const double* qdot, const double* x_target, const double* xdot_target,
                       const double* x_init, const double* xdot_init, double* e, double* edot, double* xdt_out) {
    int nv = m->nv;
    double xt[12], xdt[6];
    if (p->mode == 2) task_space_cubic(x_target, xdot_target, x_init, xdot_init, p->t, p->t0, p->duration, xt, xdt);
    else { memcpy(xt, x_target, sizeof(xt)); memcpy(xdt, xdot_target, sizeof(xdt)); }
    double Rt[9], pt[3], phi[3] = {0, 0, 0};
    pose_unpack(xt, Rt, pt);
    for (int i = 0; i < 3; ++i) e[i] = pt[i] - k->pe[i];
    for (int i = 0; i < 3; ++i) {
        double a[3] = {Rt[i], Rt[3 + i], Rt[6 + i]}, b[3] = {k->Te[i], k->Te[3 + i], k->Te[6 + i]}, c[3];
        cross3(a, b, c);
        phi[0] += c[0]; phi[1] += c[1]; phi[2] += c[2];
    }
    for (int i = 0; i < 3; ++i) e[3 + i] = -0.5 * phi[i];
    for (int i = 0; i < 6; ++i) {
        double t = 0;
        for (int c = 0; c < nv; ++c) t += J[i * nv + c] * qdot[c];
        edot[i] = xdt[i] - t;
        xdt_out[i] = xdt[i];
    }
}

/* CLIKStep / CLIKCubic (robot_controller.cpp:156-214), mode 1 / 2:
 * qdot = J^+ (Kp e + xdot_target) + (I - J^+ J) null_qdot, J^+ = PinvCOD(J). */
void oracle_clik_one(const OracleModel* m, const OracleParams* p, const double* q, const double* qdot,
                     const double* x_target, const double* xdot_target, const double* x_init,
                     const double* xdot_init, const double* null_qdot, double* out) {
    int nv = m->nv;
    Kin k;
    kin_fk(m, q, &k);
    double J[6 * ORC_MAXJ], Jp[6 * ORC_MAXJ], e[6], ed[6], xdt[6], v[6], Jn[6];
    point_jacobian(m, &k, m->ee_joint, k.pe, J);
    task_error(m, &k, J, p, qdot, x_target, xdot_target, x_init, xdot_init, e, ed, xdt);
    pinv_qr_trunc_mn(J, 6, nv, 1e-6, Jp);                     /* nv x 6 */
    for (int i = 0; i < 6; ++i) {
        v[i] = p->kp[i] * e[i] + xdt[i];
        double t = 0;
        for (int c = 0; c < nv; ++c) t += J[i * nv + c] * (null_qdot ? null_qdot[c] : 0.0);
        Jn[i] = t;
    }
    for (int c = 0; c < nv; ++c) {
        double t = 0, nt = 0;
        for (int i = 0; i < 6; ++i) { t += Jp[c * 6 + i] * v[i]; nt += Jp[c * 6 + i] * Jn[i]; }
        out[c] = t + (null_qdot ? null_qdot[c] : 0.0) - nt;
    }
}

/* OSF / OSFStep / OSFCubic (robot_controller.cpp:216-275), mode 0 / 1 / 2:
 * Lambda = PinvCOD(J M^-1 J^T), tau = J^T Lambda xdd + (I - J^T Lambda J M^-1) null_torque + g
 * with xdd = xddot_target (mode 0, passed in xdot_target) or Kp e + Kv edot.
 * Minv (n x n, = getMassMatrixInv) and g from the caller. */
void oracle_osf_one(const OracleModel* m, const OracleParams* p, const double* q, const double* qdot,
                    const double* x_target, const double* xdot_target, const double* x_init,
                    const double* xdot_init, const double* Minv, const double* g, const double* null_torque,
                    double* out) {
    int nv = m->nv;
    Kin k;
    kin_fk(m, q, &k);
    double J[6 * ORC_MAXJ], JMi[6 * ORC_MAXJ], L[36], Lam[36], JTp[6 * ORC_MAXJ], xdd[6], F[6], w[6];
    point_jacobian(m, &k, m->ee_joint, k.pe, J);
    if (p->mode == 0) memcpy(xdd, xdot_target, sizeof(xdd));
    else {
        double e[6], ed[6], xdt[6];
        task_error(m, &k, J, p, qdot, x_target, xdot_target, x_init, xdot_init, e, ed, xdt);
        for (int i = 0; i < 6; ++i) xdd[i] = p->kp[i] * e[i] + p->kv[i] * ed[i];
    }
    for (int i = 0; i < 6; ++i)
        for (int c = 0; c < nv; ++c) { double t = 0; for (int a = 0; a < nv; ++a) t += J[i * nv + a] * Minv[a * nv + c]; JMi[i * nv + c] = t; }
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) { double t = 0; for (int c = 0; c < nv; ++c) t += JMi[i * nv + c] * J[j * nv + c]; L[i * 6 + j] = t; }
    pinv_cod_sym(L, 6, Lam);
    for (int i = 0; i < 6; ++i) {
        double t = 0;
        for (int j = 0; j < 6; ++j) t += Lam[i * 6 + j] * xdd[j];
        F[i] = t;
        for (int c = 0; c < nv; ++c) { double s2 = 0; for (int j = 0; j < 6; ++j) s2 += Lam[i * 6 + j] * JMi[j * nv + c]; JTp[i * nv + c] = s2; }
    }
    for (int i = 0; i < 6; ++i) { double t = 0; for (int c = 0; c < nv; ++c) t += JTp[i * nv + c] * (null_torque ? null_torque[c] : 0.0); w[i] = t; }
    for (int c = 0; c < nv; ++c) {
        double t = g[c] + (null_torque ? null_torque[c] : 0.0);
        for (int i = 0; i < 6; ++i) t += J[i * nv + c] * (F[i] - w[i]);
        out[c] = t;
    }
}

/* stage helper: frame Jacobian time variation (getJacobianTimeVariation,
 * robot_data.cpp:404-417) and the QPID grad_dot vectors at (q, qdot) */
void oracle_qpid_stages(const OracleModel* m, const double* q, const double* qdot, double* Jdot,
                        double* man_graddot, double* dist_graddot) {
    Kin k;
    kin_fk(m, q, &k);
    double J[6 * ORC_MAXJ], man, mg[ORC_MAXJ], dist, dg[ORC_MAXJ], wA[3], wB[3];
    int pair, c0 = m->kind == 1 ? m->mani_start : 0, n = m->kind == 1 ? m->n_arm : m->nv;
    point_jacobian(m, &k, m->ee_joint, k.pe, J);
    point_jacobian_dot(m, &k, m->ee_joint, k.pe, qdot, ORC_ALL_JOINTS, Jdot);
    manip(m, &k, J, c0, n, &man, mg);
    manip_graddot(m, &k, J, c0, n, qdot, man, man_graddot);
    min_distance_w(m, &k, &dist, dg, &pair, wA, wB);
    mindist_graddot(m, &k, pair, wA, wB, qdot, dist_graddot);
}

/* joint-frame Jacobian time variation of joint jid at a world point p moving
 * rigidly with that joint's body (for finite-difference tests) */
void oracle_point_jacobian_dot(const OracleModel* m, const double* q, const double* qdot, int jid,
                               const double* p, double* J, double* Jdot) {
    Kin k;
    kin_fk(m, q, &k);
    if (J) point_jacobian(m, &k, jid, p, J);
    if (Jdot) point_jacobian_dot(m, &k, jid, p, qdot, ORC_ALL_JOINTS, Jdot);
}

/* joint placement (oMi, R row-major + p) for the tests */
void oracle_joint_placement(const OracleModel* m, const double* q, int jid, double* T12) {
    Kin k;
    kin_fk(m, q, &k);
    memcpy(T12, k.T[jid], 12 * sizeof(double));
}

/* ------------------------------------------------------------------------ */
/* batched SoA driver with a thread pool                                    */
/* ------------------------------------------------------------------------ */
typedef struct Job {
    const OracleModel* m; const OracleParams* p; int64_t B, lo, hi;
    const double *q, *qdot, *xt, *xdt, *xi, *xdi, *dist_in, *man_in;
    double* out; int32_t* status; int32_t* iters; int64_t fails;
} Job;

static void* worker(void* arg) {
    Job* j = (Job*)arg;
    const OracleModel* m = j->m;
    int nv = m->nv, na = m->kind == 1 ? m->n_wheel + m->n_arm : nv;
    for (int64_t b = j->lo; b < j->hi; ++b) {
        double q[ORC_MAXJ], qd[ORC_MAXJ], xt[12], xdt[6], xi[12], xdi[6], out[ORC_MAXJ];
        for (int i = 0; i < nv; ++i) { q[i] = j->q[i * j->B + b]; qd[i] = j->qdot[i * j->B + b]; }
        for (int i = 0; i < 12; ++i) xt[i] = j->xt ? j->xt[i * j->B + b] : 0;
        for (int i = 0; i < 6; ++i) xdt[i] = j->xdt[i * j->B + b];
        for (int i = 0; i < 12; ++i) xi[i] = j->xi ? j->xi[i * j->B + b] : 0;
        for (int i = 0; i < 6; ++i) xdi[i] = j->xdi ? j->xdi[i * j->B + b] : 0;
        double din[1 + ORC_MAXJ], mi[1 + ORC_MAXJ];
        int narm = m->kind == 1 ? m->n_arm : nv;
        if (j->dist_in) for (int i = 0; i <= nv; ++i) din[i] = j->dist_in[i * j->B + b];
        if (j->man_in) for (int i = 0; i <= narm; ++i) mi[i] = j->man_in[i * j->B + b];
        OracleDiag dg;
        int st = qpik_one_impl(m, j->p, q, qd, xt, xdt, xi, xdi, j->dist_in ? din : NULL, j->man_in ? mi : NULL, out,
                               &dg);
        for (int i = 0; i < na; ++i) j->out[i * j->B + b] = out[i];
        if (j->status) j->status[b] = st;
        if (j->iters) j->iters[b] = dg.iters;
        if (st != ORC_SOLVED) j->fails++;
    }
    return NULL;
}

static int64_t qpik_batch_impl(const OracleModel* m, const OracleParams* p, int64_t B, const double* q,
                          const double* qdot, const double* x_target, const double* xdot_target,
                          const double* x_init, const double* xdot_init, double* out, int32_t* status,
                          int32_t* iters, int nthreads, const double* dist_in,
                               const double* man_in) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    Job jobs[256];
    pthread_t th[256];
    int64_t per = (B + nthreads - 1) / nthreads;
    for (int t = 0; t < nthreads; ++t) {
        Job* j = &jobs[t];
        j->m = m; j->p = p; j->B = B; j->lo = t * per; j->hi = (t + 1) * per < B ? (t + 1) * per : B;
        if (j->lo > B) j->lo = B;
        j->q = q; j->qdot = qdot; j->xt = x_target; j->xdt = xdot_target; j->xi = x_init; j->xdi = xdot_init; j->dist_in = dist_in; j->man_in = man_in;
        j->out = out; j->status = status; j->iters = iters; j->fails = 0;
        pthread_create(&th[t], NULL, worker, j);
    }
    int64_t fails = 0;
    for (int t = 0; t < nthreads; ++t) { pthread_join(th[t], NULL); fails += jobs[t].fails; }
    return fails;
}

int64_t oracle_qpik_batch(const OracleModel* m, const OracleParams* p, int64_t B, const double* q,
                          const double* qdot, const double* x_target, const double* xdot_target,
                          const double* x_init, const double* xdot_init, double* out, int32_t* status,
                          int32_t* iters, int nthreads) {
    return qpik_batch_impl(m, p, B, q, qdot, x_target, xdot_target, x_init, xdot_init, out, status, iters,
                           nthreads, NULL, NULL);
}

/* as oracle_qpik_batch with stage data given: dist_in [1+nv][B] = (d, grad),
 * man_in [1+narm][B] = (m, grad) (either may be NULL: computed) */
int64_t oracle_qpik_batch_dist(const OracleModel* m, const OracleParams* p, int64_t B, const double* q,
                               const double* qdot, const double* x_target, const double* xdot_target,
                               const double* x_init, const double* xdot_init, const double* dist_in,
                               const double* man_in, double* out, int32_t* status, int32_t* iters, int nthreads) {
    return qpik_batch_impl(m, p, B, q, qdot, x_target, xdot_target, x_init, xdot_init, out, status, iters,
                           nthreads, dist_in, man_in);
}

/* ------------------------------------------------------------------------ */
/* stage helpers for tests                                                  */
/* ------------------------------------------------------------------------ */
void oracle_fk_pose(const OracleModel* m, const double* q, double* pose12, double* J) {
    Kin k;
    kin_fk(m, q, &k);
    memcpy(pose12, k.Te, 12 * sizeof(double));
    if (J) point_jacobian(m, &k, m->ee_joint, k.pe, J);
}
void oracle_mobile_fk_jacobian(const OracleModel* m, const double* q, double* J) {
    double Jm[3][8];
    mobile_fk_jac(m, q, Jm);
    for (int r = 0; r < 3; ++r) for (int c = 0; c < m->n_wheel; ++c) J[r * m->n_wheel + c] = Jm[r][c];
}
void oracle_min_distance(const OracleModel* m, const double* q, double* dist, double* grad, int* pair) {
    Kin k;
    kin_fk(m, q, &k);
    min_distance(m, &k, dist, grad, pair);
}
void oracle_pair_distance(const OracleModel* m, const double* q, int pair, double* d, double* pA, double* pB) {
    Kin k;
    kin_fk(m, q, &k);
    Shape a, b;
    make_shape(m, &k, m->pair_a[pair], &a);
    make_shape(m, &k, m->pair_b[pair], &b);
    int how;
    *d = shape_distance(&a, &b, pA, pB, &how);
    if (how) refine_witness(&a, &b, d, pA, pB);
}
/* narrow phase on two free shapes (T: R row-major then p), for checking the
 * device narrow-phase code in isolation */
void oracle_shape_distance(int ta, const double* TA, const double* prmA, int tb, const double* TB,
                           const double* prmB, double* d, double* pA, double* pB) {
    Shape a, b;
    a.type = ta; b.type = tb;
    memcpy(a.T, TA, sizeof(a.T)); memcpy(b.T, TB, sizeof(b.T));
    memcpy(a.prm, prmA, sizeof(a.prm)); memcpy(b.prm, prmB, sizeof(b.prm));
    int how;
    *d = shape_distance(&a, &b, pA, pB, &how);
    if (how) refine_witness(&a, &b, d, pA, pB);
}
/* the pair's raw GJK / EPA result, without the witness refinement (tests) */
void oracle_pair_distance_raw(const OracleModel* m, const double* q, int pair, double* d, double* pA, double* pB,
                              int* how) {
    Kin k;
    kin_fk(m, q, &k);
    Shape a, b;
    make_shape(m, &k, m->pair_a[pair], &a);
    make_shape(m, &k, m->pair_b[pair], &b);
    *d = shape_distance(&a, &b, pA, pB, how);
}
/* the raw GJK / EPA result without the witness refinement (tests) */
void oracle_shape_distance_raw(int ta, const double* TA, const double* prmA, int tb, const double* TB,
                               const double* prmB, double* d, double* pA, double* pB, int* how) {
    Shape a, b;
    a.type = ta; b.type = tb;
    memcpy(a.T, TA, sizeof(a.T)); memcpy(b.T, TB, sizeof(b.T));
    memcpy(a.prm, prmA, sizeof(a.prm)); memcpy(b.prm, prmB, sizeof(b.prm));
    *d = shape_distance(&a, &b, pA, pB, how);
}
void oracle_manipulability(const OracleModel* m, const double* q, double* man, double* grad) {
    Kin k;
    kin_fk(m, q, &k);
    double J[6 * ORC_MAXJ];
    point_jacobian(m, &k, m->ee_joint, k.pe, J);
    int c0 = m->kind == 1 ? m->mani_start : 0, nc = m->kind == 1 ? m->n_arm : m->nv;
    manip(m, &k, J, c0, nc, man, grad);
}

/* DyrosMath::PinvCOD of an m x n matrix (tests) */
void oracle_pinv_cod(const double* A, int m, int n, double* X) { pinv_qr_trunc_mn(A, m, n, 1e-6, X); }

/* Diagnostic (the small-batch scheduling study, tools/epa_hint_study.py): per
 * instance, whether the pruned narrow phase runs EPA (some GJK candidate
 * intersects: *truth) and the cheap predictors a scheduling pass could
 * evaluate first -- *lb: some non-closed-form pair's pair_lower_bound < 0;
 * *core: some non-closed-form pair's swept-core bound (segment distance minus
 * the radii, before the separating-axis raise) < 0. */
void oracle_epa_predict(const OracleModel* m, const double* q, int* truth, int* lb, int* core) {
    Kin k;
    kin_fk(m, q, &k);
    Shape sh[ORC_MAXG];
    for (int g = 0; g < m->ngeom; ++g) make_shape(m, &k, g, &sh[g]);
    double ub = 1e300;
    *truth = *lb = *core = 0;
    for (int p = 0; p < m->npairs; ++p) {
        const Shape *A = &sh[m->pair_a[p]], *B = &sh[m->pair_b[p]];
        double pA[3], pB[3], d;
        if (A->type == 0 || B->type == 0) { int how; d = shape_distance(A, B, pA, pB, &how); ub = fmin(ub, d); }
        else if (A->type == 1 && B->type == 1 && cyl_cyl_side(A, B, &d, pA, pB)) ub = fmin(ub, d);
    }
    for (int p = 0; p < m->npairs; ++p) {
        const Shape *A = &sh[m->pair_a[p]], *B = &sh[m->pair_b[p]];
        double pA[3], pB[3], d;
        if (A->type == 0 || B->type == 0) continue;
        if (A->type == 1 && B->type == 1 && cyl_cyl_side(A, B, &d, pA, pB)) continue;
        const double pd = pair_lower_bound(A, B);
        if (pd < 0) *lb = 1;
        {
            double a0[3], a1[3], b0[3], b1[3], c1[3], c2[3], rad[2];
            const Shape* S2[2] = {A, B};
            double* ends[2][2] = {{a0, a1}, {b0, b1}};
            for (int kk = 0; kk < 2; ++kk) {
                const Shape* s = S2[kk];
                for (int i = 0; i < 3; ++i) { ends[kk][0][i] = s->T[9 + i]; ends[kk][1][i] = s->T[9 + i]; }
                if (s->type == 1) {
                    const double ax[3] = {s->T[2], s->T[5], s->T[8]};
                    for (int i = 0; i < 3; ++i) { ends[kk][0][i] -= s->prm[1] * ax[i]; ends[kk][1][i] += s->prm[1] * ax[i]; }
                    rad[kk] = s->prm[0];
                } else if (s->type == 2) {
                    rad[kk] = sqrt(s->prm[0] * s->prm[0] + s->prm[1] * s->prm[1] + s->prm[2] * s->prm[2]);
                } else {
                    rad[kk] = s->prm[0];
                }
            }
            if (seg_seg(a0, a1, b0, b1, c1, c2) - rad[0] - rad[1] < 0) *core = 1;
        }
        if (!(pd - 1e-9 <= ub)) continue;
        SV S[4];
        int ns;
        double lam[4], v[3];
        if (gjk_cut(A, B, S, &ns, lam, v, ub + 1e-9) == 1) *truth = 1;
    }
}

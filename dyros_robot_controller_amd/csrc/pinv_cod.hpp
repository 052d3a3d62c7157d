// DyrosMath::PinvCOD (math_type_define.h:563-570) as a serial device routine,
// shared by the manipulability stage (6x6 JJ^T, task_kernel.hip) and the
// dynamics kernel (M, S^T M S; dynamics.hip) for the rare inputs whose full rank
// the fast paths cannot certify.
#pragma once

#include <hip/hip_runtime.h>

#include "model.hpp"

namespace drc_amd {

constexpr double kPinvCodThreshold = 1e-6;  // COD_THRESHOLD (math_type_define.h:7)

// Serial DyrosMath::PinvCOD of a symmetric no x no matrix A (element (i,j) at
// A[(i*n+j)*st]; X likewise; w: 3n^2+3n doubles): column-pivoted Householder QR, rank |R_ii| > 1e-6 max|R_ii|,
// X = P W^T (W W^T)^-1 Q_r^T with W = R[:r, :] — the Moore-Penrose inverse of the
// QR-truncated matrix, which is what Eigen's cod.pseudoInverse() returns.
__device__ inline void pinv_cod_serial(const double* A, int n, int st, double* X, double* w) {
  double* R = w;                 // n x n, Householder vectors below the diagonal
  double* G = w + n * n;         // r x r, then its Cholesky factor
  double* Y = w + 2 * n * n;     // n x r
  double* beta = w + 3 * n * n;  // n
  double* cn = beta + n;         // n
  double* perm = cn + n;         // n
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) R[i * n + j] = A[(i * n + j) * st];
  for (int j = 0; j < n; ++j) perm[j] = j;
  double maxpiv = 0;
  for (int k = 0; k < n; ++k) {
    int p = k;
    for (int j = k; j < n; ++j) {
      double s = 0;
      for (int i = k; i < n; ++i) s += R[i * n + j] * R[i * n + j];
      cn[j] = s;
      if (s > cn[p]) p = j;
    }
    if (p != k) {
      for (int i = 0; i < n; ++i) {
        double t = R[i * n + k];
        R[i * n + k] = R[i * n + p];
        R[i * n + p] = t;
      }
      double t = perm[k];
      perm[k] = perm[p];
      perm[p] = t;
      t = cn[k];
      cn[k] = cn[p];
      cn[p] = t;
    }
    const double nrm = sqrt(cn[k]);
    beta[k] = 0;
    if (nrm > 0) {
      const double x0 = R[k * n + k], alpha = x0 > 0 ? -nrm : nrm;
      // v = x - alpha e1, stored with v0 implicit in R[k][k] slot afterwards
      const double v0 = x0 - alpha;
      double vn = v0 * v0;
      for (int i = k + 1; i < n; ++i) vn += R[i * n + k] * R[i * n + k];
      const double bt = vn > 0 ? 2.0 / vn : 0.0;
      for (int j = k + 1; j < n; ++j) {
        double s = v0 * R[k * n + j];
        for (int i = k + 1; i < n; ++i) s += R[i * n + k] * R[i * n + j];
        s *= bt;
        R[k * n + j] -= s * v0;
        for (int i = k + 1; i < n; ++i) R[i * n + j] -= s * R[i * n + k];
      }
      R[k * n + k] = alpha;   // v = (v0, R[k+1.., k]); v0 kept in cn[k] (no longer a pivot norm)
      beta[k] = bt;
      cn[k] = v0;  // v0 of reflector k
    } else {
      cn[k] = 0;
    }
    maxpiv = fmax(maxpiv, fabs(R[k * n + k]));
  }
  int r = 0;
  for (int k = 0; k < n; ++k) r += fabs(R[k * n + k]) > kPinvCodThreshold * maxpiv;
  for (int i = 0; i < n * n; ++i) X[i * st] = 0;
  if (r == 0) return;
  // G = W W^T (r x r), W[i][j] = R[i][j] for j >= i (upper part), 0 below
  for (int i = 0; i < r; ++i)
    for (int j = 0; j <= i; ++j) {
      double s = 0;
      for (int k = i; k < n; ++k) s += R[i * n + k] * R[j * n + k];  // j <= i so W[j][k] valid for k >= i
      G[i * r + j] = s;
    }
  for (int j = 0; j < r; ++j) {  // Cholesky (lower) in place
    double s = G[j * r + j];
    for (int k = 0; k < j; ++k) s -= G[j * r + k] * G[j * r + k];
    const double d = sqrt(fmax(s, 1e-300));
    G[j * r + j] = d;
    for (int i = j + 1; i < r; ++i) {
      double t = G[i * r + j];
      for (int k = 0; k < j; ++k) t -= G[i * r + k] * G[j * r + k];
      G[i * r + j] = t / d;
    }
  }
  // Y = W^T G^-1: row c of Y solves G y = W[:, c]
  for (int c = 0; c < n; ++c) {
    double* y = Y + c * r;
    for (int i = 0; i < r; ++i) y[i] = c >= i ? R[i * n + c] : 0.0;
    for (int i = 0; i < r; ++i) {
      double t = y[i];
      for (int k = 0; k < i; ++k) t -= G[i * r + k] * y[k];
      y[i] = t / G[i * r + i];
    }
    for (int i = r - 1; i >= 0; --i) {
      double t = y[i];
      for (int k = i + 1; k < r; ++k) t -= G[k * r + i] * y[k];
      y[i] = t / G[i * r + i];
    }
  }
  // X[perm[c]][col] = sum_i Y[c][i] (Q^T e_col)_i, Q^T e = H_{n-1} ... H_0 e
  for (int col = 0; col < n; ++col) {
    double u[kMaxJoints];
    for (int i = 0; i < n; ++i) u[i] = i == col ? 1.0 : 0.0;
    for (int k = 0; k < n; ++k) {
      if (beta[k] == 0) continue;
      double s = cn[k] * u[k];
      for (int i = k + 1; i < n; ++i) s += R[i * n + k] * u[i];
      s *= beta[k];
      u[k] -= s * cn[k];
      for (int i = k + 1; i < n; ++i) u[i] -= s * R[i * n + k];
    }
    for (int c = 0; c < n; ++c) {
      double s = 0;
      for (int i = 0; i < r; ++i) s += Y[c * r + i] * u[i];
      X[(static_cast<int>(perm[c]) * n + col) * st] = s;
    }
  }
}

// DyrosMath::PinvCOD of a rectangular m x n matrix A (row-major, m <= 6,
// n <= kMaxJoints) into X (n x m, row-major): column-pivoted Householder QR
// (k < min(m, n)), rank |R_ii| > 1e-6 max|R_ii|, X = P W^T (W W^T)^-1 Q_r^T.
// Serial (one lane); w: m*n + m*m + n*m + 3m + 2n doubles in LDS.
__device__ inline void pinv_cod_rect(const double* A, int m, int n, double* X, double* w) {
  double* R = w;               // m x n
  double* G = R + m * n;       // r x r (r <= m)
  double* Y = G + m * m;       // n x r
  double* beta = Y + n * m;    // m
  double* v0 = beta + m;       // m
  double* cn = v0 + m;         // n
  double* perm = cn + n;       // n
  const int kmax = m < n ? m : n;
  for (int i = 0; i < m * n; ++i) R[i] = A[i];
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
      for (int i = 0; i < m; ++i) {
        const double t = R[i * n + k];
        R[i * n + k] = R[i * n + p];
        R[i * n + p] = t;
      }
      double t = perm[k];
      perm[k] = perm[p];
      perm[p] = t;
      t = cn[k];
      cn[k] = cn[p];
      cn[p] = t;
    }
    const double nrm = sqrt(cn[k]);
    beta[k] = 0;
    v0[k] = 0;
    if (nrm > 0) {
      const double x0 = R[k * n + k], alpha = x0 > 0 ? -nrm : nrm, w0 = x0 - alpha;
      double vn = w0 * w0;
      for (int i = k + 1; i < m; ++i) vn += R[i * n + k] * R[i * n + k];
      const double bt = vn > 0 ? 2.0 / vn : 0.0;
      for (int j = k + 1; j < n; ++j) {
        double s = w0 * R[k * n + j];
        for (int i = k + 1; i < m; ++i) s += R[i * n + k] * R[i * n + j];
        s *= bt;
        R[k * n + j] -= s * w0;
        for (int i = k + 1; i < m; ++i) R[i * n + j] -= s * R[i * n + k];
      }
      R[k * n + k] = alpha;
      beta[k] = bt;
      v0[k] = w0;
    }
    maxpiv = fmax(maxpiv, fabs(R[k * n + k]));
  }
  int r = 0;
  for (int k = 0; k < kmax; ++k) r += fabs(R[k * n + k]) > kPinvCodThreshold * maxpiv;
  for (int i = 0; i < n * m; ++i) X[i] = 0;
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
    const double d = sqrt(fmax(s, 1e-300));
    G[j * r + j] = d;
    for (int i = j + 1; i < r; ++i) {
      double t = G[i * r + j];
      for (int k = 0; k < j; ++k) t -= G[i * r + k] * G[j * r + k];
      G[i * r + j] = t / d;
    }
  }
  for (int c = 0; c < n; ++c) {
    double* y = Y + c * r;
    for (int i = 0; i < r; ++i) y[i] = c >= i ? R[i * n + c] : 0.0;
    for (int i = 0; i < r; ++i) {
      double t = y[i];
      for (int k = 0; k < i; ++k) t -= G[i * r + k] * y[k];
      y[i] = t / G[i * r + i];
    }
    for (int i = r - 1; i >= 0; --i) {
      double t = y[i];
      for (int k = i + 1; k < r; ++k) t -= G[k * r + i] * y[k];
      y[i] = t / G[i * r + i];
    }
  }
  for (int col = 0; col < m; ++col) {
    double* u = beta + 2 * m + 2 * n;  // m scratch after perm
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
      X[static_cast<int>(perm[c]) * m + col] = s;
    }
  }
}

}  // namespace drc_amd

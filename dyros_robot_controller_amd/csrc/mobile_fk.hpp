// Mobile base FK Jacobian J_mobile (3 x W: base twist [vx, vy, wz] = J_mobile *
// wheel velocities) of Mobile::RobotData::computeFKJacobian
// (src/mobile/robot_data.cpp:123-204), host and device.  Differential and
// mecanum are configuration independent and live in the model table
// (DevModel::J_mobile, built once on the host); the caster drive depends on
// the steer angles and is evaluated per instance here.
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>

#include "model.hpp"

namespace drc_amd {

#define DRC_FK_HD __host__ __device__

// Moore-Penrose inverse of a symmetric 3x3 matrix by cyclic Jacobi: modes whose
// |eigenvalue| is at most 1e-6 of the largest are cut (DyrosMath::PinvCOD's
// relative threshold, math_type_define.h:7,563-570, for a symmetric PSD matrix).
DRC_FK_HD inline void pinv_sym3(const double* N, double* X) {
  double A[3][3], V[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) A[i][j] = N[3 * i + j];
  for (int sweep = 0; sweep < 16; ++sweep) {
    const double off = A[0][1] * A[0][1] + A[0][2] * A[0][2] + A[1][2] * A[1][2];
    const double dia = A[0][0] * A[0][0] + A[1][1] * A[1][1] + A[2][2] * A[2][2];
    if (!(off > 1e-32 * dia)) break;
    for (int pq = 0; pq < 3; ++pq) {
      const int p = pq == 2 ? 1 : 0, q = pq == 0 ? 1 : 2;
      if (A[p][q] == 0) continue;
      const double th = (A[q][q] - A[p][p]) / (2 * A[p][q]);
      const double t = (th >= 0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1));
      const double c = 1 / sqrt(t * t + 1), s = t * c;
      for (int k = 0; k < 3; ++k) {
        const double a = A[k][p], b = A[k][q];
        A[k][p] = c * a - s * b;
        A[k][q] = s * a + c * b;
      }
      for (int k = 0; k < 3; ++k) {
        const double a = A[p][k], b = A[q][k];
        A[p][k] = c * a - s * b;
        A[q][k] = s * a + c * b;
      }
      for (int k = 0; k < 3; ++k) {
        const double a = V[k][p], b = V[k][q];
        V[k][p] = c * a - s * b;
        V[k][q] = s * a + c * b;
      }
    }
  }
  double wmax = 0;
  for (int e = 0; e < 3; ++e) wmax = fmax(wmax, fabs(A[e][e]));
  for (int i = 0; i < 9; ++i) X[i] = 0;
  for (int e = 0; e < 3; ++e) {
    const double w = A[e][e];
    if (!(fabs(w) > 1e-6 * wmax)) continue;
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) X[3 * i + j] += V[i][e] * V[j][e] / w;
  }
}

// Mobile::RobotData::CasterFKJacobian (src/mobile/robot_data.cpp:179-204):
// C casters, wheel_pos[2i] = steer angle phi_i, wheel_pos[2i+1] = drive angle;
//   Jp~ (2C x 3): rows [1, 0, -(py + b sin phi)], [0, 1, px + b cos phi]
//   Jq^-1 (2C x 2C) block diag [[b sin phi, r cos phi], [-b cos phi, r sin phi]]
//   J_mobile = PinvCOD(Jp~^T Jp~) Jp~^T Jq^-1          (3 x 2C, row stride kMaxWheels)
DRC_FK_HD inline void caster_fk_jacobian(int C, double r, double b, const double (*pos)[2], const double* wheel_pos,
                                         double (*J)[kMaxWheels]) {
  double N[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, R[3][kMaxWheels];
  for (int i = 0; i < C; ++i) {
    const double phi = wheel_pos[2 * i], sp = sin(phi), cp = cos(phi);
    const double a = pos[i][1] + b * sp, c = pos[i][0] + b * cp;
    // Jp~^T Jp~ accumulated over the two rows of caster i
    N[0] += 1;
    N[4] += 1;
    N[2] -= a;
    N[5] += c;
    N[8] += a * a + c * c;
    // Jp~^T Jq^-1: columns 2i (b sin, -b cos) and 2i+1 (r cos, r sin)
    R[0][2 * i] = b * sp;
    R[1][2 * i] = -b * cp;
    R[2][2 * i] = -a * b * sp - c * b * cp;
    R[0][2 * i + 1] = r * cp;
    R[1][2 * i + 1] = r * sp;
    R[2][2 * i + 1] = -a * r * cp + c * r * sp;
  }
  N[6] = N[2];
  N[7] = N[5];
  double Ni[9];
  pinv_sym3(N, Ni);
  for (int k = 0; k < 3; ++k)
    for (int w = 0; w < kMaxWheels; ++w) {
      double s = 0;
      if (w < 2 * C)
        for (int m = 0; m < 3; ++m) s += Ni[3 * k + m] * R[m][w];
      J[k][w] = s;
    }
}

// J_mobile of a model at the wheel positions (any drive)
DRC_FK_HD inline void mobile_fk(const DevModel* M, const double* wheel_pos, double (*J)[kMaxWheels]) {
  if (M->drive == kDriveCaster) {
    caster_fk_jacobian(M->n_wheel / 2, M->wheel_radius, M->wheel_offset, M->caster_pos, wheel_pos, J);
    return;
  }
  for (int k = 0; k < 3; ++k)
    for (int w = 0; w < kMaxWheels; ++w) J[k][w] = M->J_mobile[k][w];
}

}  // namespace drc_amd

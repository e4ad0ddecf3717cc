// ba_geometry.hpp — host-side geometry of the optimizer shim (no Eigen).
//
// The reference converts between the float 4x4 poses of its model
// (Frame::getPose, camera -> world) and the double angle-axis camera blocks
// of the solver with Eigen and ceres/rotation.h (Optimizer.cpp:260-267,
// 296-299).  This header restates exactly those conversions on plain
// column-major arrays so the shim needs neither Eigen nor Ceres.
#pragma once

#include <cmath>
#include <limits>

namespace ba_amd {

struct Vec2f { float x = 0, y = 0; };
struct Vec3f { float v[3] = {0, 0, 0}; float operator[](int i) const { return v[i]; } };
struct Mat3f { float m[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}; };   // column-major (Eigen storage)
struct Mat4f { float m[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}; };  // column-major

inline Mat4f identity4() {
  Mat4f r;
  r.m[0] = r.m[5] = r.m[10] = r.m[15] = 1.0f;
  return r;
}

// ceres::AngleAxisToRotationMatrix (rotation.h), column-major R.
inline void angle_axis_to_rotation(const double* w, double* R) {
  const double theta2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  if (theta2 > std::numeric_limits<double>::epsilon()) {
    const double theta = std::sqrt(theta2);
    const double wx = w[0] / theta, wy = w[1] / theta, wz = w[2] / theta;
    const double c = std::cos(theta), s = std::sin(theta), c1 = 1.0 - c;
    R[0] = c + wx * wx * c1;      R[3] = wx * wy * c1 - wz * s;  R[6] = wy * s + wx * wz * c1;
    R[1] = wz * s + wx * wy * c1; R[4] = c + wy * wy * c1;       R[7] = -(wx * s) + wy * wz * c1;
    R[2] = -(wy * s) + wx * wz * c1; R[5] = wx * s + wy * wz * c1; R[8] = c + wz * wz * c1;
  } else {  // first-order expansion (Ceres)
    R[0] = 1.0;   R[3] = -w[2]; R[6] = w[1];
    R[1] = w[2];  R[4] = 1.0;   R[7] = -w[0];
    R[2] = -w[1]; R[5] = w[0];  R[8] = 1.0;
  }
}

// ceres::RotationMatrixToAngleAxis = RotationMatrixToQuaternion (Shepperd)
// + QuaternionToAngleAxis, column-major R.
inline void rotation_to_angle_axis(const double* R, double* w) {
  auto Rm = [&](int r, int c) { return R[c * 3 + r]; };
  double q[4];
  const double trace = Rm(0, 0) + Rm(1, 1) + Rm(2, 2);
  if (trace >= 0.0) {
    double t = std::sqrt(trace + 1.0);
    q[0] = 0.5 * t;
    t = 0.5 / t;
    q[1] = (Rm(2, 1) - Rm(1, 2)) * t;
    q[2] = (Rm(0, 2) - Rm(2, 0)) * t;
    q[3] = (Rm(1, 0) - Rm(0, 1)) * t;
  } else {
    int i = 0;
    if (Rm(1, 1) > Rm(0, 0)) i = 1;
    if (Rm(2, 2) > Rm(i, i)) i = 2;
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    double t = std::sqrt(Rm(i, i) - Rm(j, j) - Rm(k, k) + 1.0);
    q[i + 1] = 0.5 * t;
    t = 0.5 / t;
    q[0] = (Rm(k, j) - Rm(j, k)) * t;
    q[j + 1] = (Rm(j, i) + Rm(i, j)) * t;
    q[k + 1] = (Rm(k, i) + Rm(i, k)) * t;
  }
  const double sin_sq = q[1] * q[1] + q[2] * q[2] + q[3] * q[3];
  double kk = 2.0;
  if (sin_sq > 0.0) {
    const double sin_theta = std::sqrt(sin_sq), cos_theta = q[0];
    const double two_theta =
        2.0 * ((cos_theta < 0.0) ? std::atan2(-sin_theta, -cos_theta) : std::atan2(sin_theta, cos_theta));
    kk = two_theta / sin_theta;
  }
  w[0] = q[1] * kk; w[1] = q[2] * kk; w[2] = q[3] * kk;
}

// General 4x4 float inverse by cofactors (stands in for Eigen's
// Matrix4f::inverse(); its last-ulp rounding is not pinned to Eigen's).
inline Mat4f inverse4(const Mat4f& a) {
  const float* m = a.m;
  float inv[16];
  inv[0] = m[5] * m[10] * m[15] - m[5] * m[11] * m[14] - m[9] * m[6] * m[15] + m[9] * m[7] * m[14] +
           m[13] * m[6] * m[11] - m[13] * m[7] * m[10];
  inv[4] = -m[4] * m[10] * m[15] + m[4] * m[11] * m[14] + m[8] * m[6] * m[15] - m[8] * m[7] * m[14] -
           m[12] * m[6] * m[11] + m[12] * m[7] * m[10];
  inv[8] = m[4] * m[9] * m[15] - m[4] * m[11] * m[13] - m[8] * m[5] * m[15] + m[8] * m[7] * m[13] +
           m[12] * m[5] * m[11] - m[12] * m[7] * m[9];
  inv[12] = -m[4] * m[9] * m[14] + m[4] * m[10] * m[13] + m[8] * m[5] * m[14] - m[8] * m[6] * m[13] -
            m[12] * m[5] * m[10] + m[12] * m[6] * m[9];
  inv[1] = -m[1] * m[10] * m[15] + m[1] * m[11] * m[14] + m[9] * m[2] * m[15] - m[9] * m[3] * m[14] -
           m[13] * m[2] * m[11] + m[13] * m[3] * m[10];
  inv[5] = m[0] * m[10] * m[15] - m[0] * m[11] * m[14] - m[8] * m[2] * m[15] + m[8] * m[3] * m[14] +
           m[12] * m[2] * m[11] - m[12] * m[3] * m[10];
  inv[9] = -m[0] * m[9] * m[15] + m[0] * m[11] * m[13] + m[8] * m[1] * m[15] - m[8] * m[3] * m[13] -
           m[12] * m[1] * m[11] + m[12] * m[3] * m[9];
  inv[13] = m[0] * m[9] * m[14] - m[0] * m[10] * m[13] - m[8] * m[1] * m[14] + m[8] * m[2] * m[13] +
            m[12] * m[1] * m[10] - m[12] * m[2] * m[9];
  inv[2] = m[1] * m[6] * m[15] - m[1] * m[7] * m[14] - m[5] * m[2] * m[15] + m[5] * m[3] * m[14] +
           m[13] * m[2] * m[7] - m[13] * m[3] * m[6];
  inv[6] = -m[0] * m[6] * m[15] + m[0] * m[7] * m[14] + m[4] * m[2] * m[15] - m[4] * m[3] * m[14] -
           m[12] * m[2] * m[7] + m[12] * m[3] * m[6];
  inv[10] = m[0] * m[5] * m[15] - m[0] * m[7] * m[13] - m[4] * m[1] * m[15] + m[4] * m[3] * m[13] +
            m[12] * m[1] * m[7] - m[12] * m[3] * m[5];
  inv[14] = -m[0] * m[5] * m[14] + m[0] * m[6] * m[13] + m[4] * m[1] * m[14] - m[4] * m[2] * m[13] -
            m[12] * m[1] * m[6] + m[12] * m[2] * m[5];
  inv[3] = -m[1] * m[6] * m[11] + m[1] * m[7] * m[10] + m[5] * m[2] * m[11] - m[5] * m[3] * m[10] -
           m[9] * m[2] * m[7] + m[9] * m[3] * m[6];
  inv[7] = m[0] * m[6] * m[11] - m[0] * m[7] * m[10] - m[4] * m[2] * m[11] + m[4] * m[3] * m[10] +
           m[8] * m[2] * m[7] - m[8] * m[3] * m[6];
  inv[11] = -m[0] * m[5] * m[11] + m[0] * m[7] * m[9] + m[4] * m[1] * m[11] - m[4] * m[3] * m[9] -
            m[8] * m[1] * m[7] + m[8] * m[3] * m[5];
  inv[15] = m[0] * m[5] * m[10] - m[0] * m[6] * m[9] - m[4] * m[1] * m[10] + m[4] * m[2] * m[9] +
            m[8] * m[1] * m[6] - m[8] * m[2] * m[5];
  const float det = m[0] * inv[0] + m[1] * inv[4] + m[2] * inv[8] + m[3] * inv[12];
  const float idet = 1.0f / det;
  Mat4f r;
  for (int i = 0; i < 16; ++i) r.m[i] = inv[i] * idet;
  return r;
}

// optimizedExtr from a pose (Optimizer.cpp:294-299):
//   extr = pose.inverse();  w = RotationMatrixToAngleAxis(double(R));  t = double(extr t)
inline void camera_block_from_pose(const Mat4f& pose, double* cam6, Mat4f* extr_out = nullptr) {
  const Mat4f extr = inverse4(pose);
  double R[9];
  for (int c = 0; c < 3; ++c)
    for (int r = 0; r < 3; ++r) R[c * 3 + r] = static_cast<double>(extr.m[c * 4 + r]);
  rotation_to_angle_axis(R, cam6);
  for (int r = 0; r < 3; ++r) cam6[3 + r] = static_cast<double>(extr.m[12 + r]);
  if (extr_out) *extr_out = extr;
}

// Float write-back of a camera block (Optimizer.cpp:260-267):
//   newExtr = [float(R(w)) | float(t)];  pose = newExtr.inverse()
inline Mat4f pose_from_camera_block(const double* cam6) {
  double R[9];
  angle_axis_to_rotation(cam6, R);
  Mat4f e = identity4();
  for (int c = 0; c < 3; ++c)
    for (int r = 0; r < 3; ++r) e.m[c * 4 + r] = static_cast<float>(R[c * 3 + r]);
  for (int r = 0; r < 3; ++r) e.m[12 + r] = static_cast<float>(cam6[3 + r]);
  return inverse4(e);
}

}  // namespace ba_amd

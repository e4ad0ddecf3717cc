// ba_device.h — device math for the MI355X bundle-adjustment kernels.
//
// Camera model = the reference's AngleReprojectionError (Optimizer.h:54-76):
//   R = AngleAxisToRotationMatrix(w)   (ceres rotation.h, column-major)
//   p = R X + t ;  q = K p ;  r = (q0/q2 - u, q1/q2 - v)
// Fixed cameras follow PointOnlyReprojectionError (Optimizer.h:96-107):
//   p = hnormalized(E [X;1]) with the float 4x4 extrinsic E.
//
// The Jacobian is analytic but structured like Ceres' Jet evaluation: dR/dw
// is the forward derivative of the very same Rodrigues formula (including the
// first-order branch for theta^2 <= DBL_EPSILON), computed once per camera;
// the per-observation chain rule then matches autodiff term for term.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bahip {

// Camera record: 48 doubles per camera (384 B), shared by all observations of
// that camera.  Variable camera:
//   [0..8]  R (col-major)       [9..35] dR/dw_k (k-major, col-major each)
//   [36..38] t                  [39..47] K (col-major, double of float)
// Fixed camera: [0..15] E (col-major 4x4, double of float), [39..47] K.
// Linearisation table (written with the derivatives, [48..87]): K folded
// into the camera so the per-observation chain rule is 36 FMA shorter:
//   variable: [0..8] K R  [9..35] K dR/dw_k  [36..38] K t      (col-major)
//   fixed:    [0..11] K E(0:3, 0:4)  [12..15] E(3, 0:4)
// (re-association of the Jet products K (R X + t): differs by rounding only)
constexpr int kCamRec = 88;
constexpr int kRecR = 0, kRecdR = 9, kRecT = 36, kRecK = 39, kRecL = 48, kLin = 40;
constexpr int kLinKR = 0, kLinKdR = 9, kLinKt = 36, kLinKE = 0, kLinE3 = 12;

struct D3 {  // value + 3 partial derivatives (d/dw0, d/dw1, d/dw2)
  double a, d[3];
};
__host__ __device__ inline D3 mk(double a, double d0, double d1, double d2) { D3 r; r.a = a; r.d[0] = d0; r.d[1] = d1; r.d[2] = d2; return r; }
__host__ __device__ inline D3 operator+(D3 f, D3 g) { return mk(f.a + g.a, f.d[0] + g.d[0], f.d[1] + g.d[1], f.d[2] + g.d[2]); }
__host__ __device__ inline D3 operator-(D3 f, D3 g) { return mk(f.a - g.a, f.d[0] - g.d[0], f.d[1] - g.d[1], f.d[2] - g.d[2]); }
__host__ __device__ inline D3 operator-(D3 f) { return mk(-f.a, -f.d[0], -f.d[1], -f.d[2]); }
__host__ __device__ inline D3 operator*(D3 f, D3 g) {
  return mk(f.a * g.a, f.a * g.d[0] + f.d[0] * g.a, f.a * g.d[1] + f.d[1] * g.a, f.a * g.d[2] + f.d[2] * g.a);
}
__host__ __device__ inline D3 operator/(D3 f, D3 g) {
  const double gi = 1.0 / g.a, fg = f.a * gi;
  return mk(fg, (f.d[0] - fg * g.d[0]) * gi, (f.d[1] - fg * g.d[1]) * gi, (f.d[2] - fg * g.d[2]) * gi);
}
__host__ __device__ inline D3 rsub(double s, D3 f) { return mk(s - f.a, -f.d[0], -f.d[1], -f.d[2]); }
__host__ __device__ inline D3 dsqrt(D3 f) {
  const double t = sqrt(f.a), ti = 1.0 / (2.0 * t);
  return mk(t, f.d[0] * ti, f.d[1] * ti, f.d[2] * ti);
}
__host__ __device__ inline D3 dcos(D3 f) { const double s = -sin(f.a); return mk(cos(f.a), s * f.d[0], s * f.d[1], s * f.d[2]); }
__host__ __device__ inline D3 dsin(D3 f) { const double c = cos(f.a); return mk(sin(f.a), c * f.d[0], c * f.d[1], c * f.d[2]); }

// ceres::AngleAxisToRotationMatrix on duals; R column-major (R[c*3+r]).
__host__ __device__ __forceinline__ void angle_axis_to_R_d3(const double w[3], D3 R[9]) {
  const D3 a0 = mk(w[0], 1, 0, 0), a1 = mk(w[1], 0, 1, 0), a2 = mk(w[2], 0, 0, 1);
  const D3 theta2 = a0 * a0 + a1 * a1 + a2 * a2;
  if (theta2.a > 2.220446049250313080847e-16) {
    const D3 theta = dsqrt(theta2);
    const D3 wx = a0 / theta, wy = a1 / theta, wz = a2 / theta;
    const D3 c = dcos(theta), s = dsin(theta);
    const D3 oc = rsub(1.0, c);
    R[0] = c + wx * wx * oc;
    R[1] = wz * s + wx * wy * oc;
    R[2] = -(wy * s) + wx * wz * oc;
    R[3] = wx * wy * oc - wz * s;
    R[4] = c + wy * wy * oc;
    R[5] = wx * s + wy * wz * oc;
    R[6] = wy * s + wx * wz * oc;
    R[7] = -(wx * s) + wy * wz * oc;
    R[8] = c + wz * wz * oc;
  } else {
    R[0] = mk(1, 0, 0, 0); R[1] = a2;             R[2] = -a1;
    R[3] = -a2;            R[4] = mk(1, 0, 0, 0); R[5] = a0;
    R[6] = a1;             R[7] = -a0;            R[8] = mk(1, 0, 0, 0);
  }
}

// Value-only Rodrigues (same branches, same arithmetic order as the dual one).
__host__ __device__ inline void angle_axis_to_R(const double w[3], double R[9]) {
  const double theta2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  if (theta2 > 2.220446049250313080847e-16) {
    const double theta = sqrt(theta2);
    const double wx = w[0] / theta, wy = w[1] / theta, wz = w[2] / theta;
    const double c = cos(theta), s = sin(theta);
    const double oc = 1.0 - c;
    R[0] = c + wx * wx * oc;
    R[1] = wz * s + wx * wy * oc;
    R[2] = -(wy * s) + wx * wz * oc;
    R[3] = wx * wy * oc - wz * s;
    R[4] = c + wy * wy * oc;
    R[5] = wx * s + wy * wz * oc;
    R[6] = wy * s + wx * wz * oc;
    R[7] = -(wx * s) + wy * wz * oc;
    R[8] = c + wz * wz * oc;
  } else {
    R[0] = 1;     R[1] = w[2];  R[2] = -w[1];
    R[3] = -w[2]; R[4] = 1;     R[5] = w[0];
    R[6] = w[1];  R[7] = -w[0]; R[8] = 1;
  }
}

// ceres::HuberLoss(a) + Corrector: returns rho(s); *scale = sqrt(rho'(s)).
__host__ __device__ inline double huber(double s, double a, double b, double* scale) {
  if (a > 0.0 && s > b) {
    const double r = sqrt(s);
    double rho1 = a / r;
    rho1 = rho1 > 2.2250738585072014e-308 ? rho1 : 2.2250738585072014e-308;
    *scale = sqrt(rho1);
    return 2.0 * a * r - b;
  }
  *scale = 1.0;
  return s;
}


// The 16-value rank-2 PCG record of one observation (ITERATIVE_SCHUR, K
// without skew): W_o = c^T Z with c = Jc s_c (its scaled rotation columns
// [0..5], the four nonzero translation entries c0[3], c0[5], c1[4], c1[5]
// [6..9]) and Z = Jp s_p L_p^-T [10..15].  j: lin_obs's corrected row pair,
// sc: s_c, s: s_p, li: L_p^-1 (lower, row-major 00 10 11 20 21 22).
// The record's writer (k_obs_w_rc<.., PC>) and the J-free point pass
// (k_pcg_point_jf) form it here, and the point passes take their products
// through pc_v / pc_t, all without FMA contraction: each operation rounds on
// its own, so the value does not depend on the code around the call and
// both matvec forms are bitwise the same.
__device__ __forceinline__ void pc_record(const double* j, const double (&sc)[6], const double (&s)[3],
                                          const double (&li)[6], bool live, double (&wv)[16]) {
#pragma clang fp contract(off)
  const double jp0[3] = {j[12] * s[0], j[13] * s[1], j[14] * s[2]};
  const double jp1[3] = {j[15] * s[0], j[16] * s[1], j[17] * s[2]};
  const double z[6] = {jp0[0] * li[0], jp0[0] * li[1] + jp0[1] * li[2], jp0[0] * li[3] + jp0[1] * li[4] + jp0[2] * li[5],
                       jp1[0] * li[0], jp1[0] * li[1] + jp1[1] * li[2], jp1[0] * li[3] + jp1[1] * li[4] + jp1[2] * li[5]};
  for (int a = 0; a < 3; ++a) {
    wv[a] = live ? j[a] * sc[a] : 0.0;
    wv[3 + a] = live ? j[6 + a] * sc[a] : 0.0;
  }
  wv[6] = live ? j[3] * sc[3] : 0.0;
  wv[7] = live ? j[5] * sc[5] : 0.0;
  wv[8] = live ? j[10] * sc[4] : 0.0;
  wv[9] = live ? j[11] * sc[5] : 0.0;
  for (int k = 0; k < 6; ++k) wv[10 + k] = live ? z[k] : 0.0;
}
// v = Z^T (c x) of a record (zero unless on)
__device__ __forceinline__ void pc_v(const double (&wr)[16], const double (&x)[6], bool on, double (&v)[3]) {
#pragma clang fp contract(off)
  const double y0 = wr[0] * x[0] + wr[1] * x[1] + wr[2] * x[2] + wr[6] * x[3] + wr[7] * x[5];
  const double y1 = wr[3] * x[0] + wr[4] * x[1] + wr[5] * x[2] + wr[8] * x[4] + wr[9] * x[5];
  for (int k = 0; k < 3; ++k) v[k] = on ? wr[10 + k] * y0 + wr[13 + k] * y1 : 0.0;
}
// t = c^T (Z v) of a record
__device__ __forceinline__ void pc_t(const double (&wr)[16], const double (&vp)[3], double (&tv)[6]) {
#pragma clang fp contract(off)
  const double q0 = wr[10] * vp[0] + wr[11] * vp[1] + wr[12] * vp[2];
  const double q1 = wr[13] * vp[0] + wr[14] * vp[1] + wr[15] * vp[2];
  for (int a = 0; a < 3; ++a) tv[a] = wr[a] * q0 + wr[3 + a] * q1;
  tv[3] = wr[6] * q0;
  tv[4] = wr[8] * q1;
  tv[5] = wr[7] * q0 + wr[9] * q1;
}

}  // namespace bahip

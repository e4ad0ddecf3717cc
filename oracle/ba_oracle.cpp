// =============================================================================
//  ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, called by, or shipped
//  with the product (libba_hip.so).  Only tests/, __graft_entry__.smoke() and
//  bench.py's cpu_baseline leg may load it, and only as the checker / the
//  labelled "CPU restatement, not Ceres" baseline.
//
//  What it is: a plain C++17 CPU restatement of the reference's bundle-
//  adjustment hot path (MatteoWohlrapp/BundleAdjustment, ba_project/src/ba):
//
//    * the three cost functors the application uses, templated on a scalar
//      type exactly like the reference and differentiated by a forward-mode
//      Jet (the same mechanism as ceres::AutoDiffCostFunction):
//        AngleReprojectionError          Optimizer.h:49-88   (2 x [6,3])
//        PointOnlyReprojectionError      Optimizer.h:91-120  (2 x [3])
//        PoseOnlyAngleReprojectionError  Optimizer.h:156-194 (2 x [6])
//    * ceres::HuberLoss(sqrt(5.991)) + Ceres' Corrector
//        (Optimizer.cpp:312, 489, 645, 686)
//    * ceres AngleAxisToRotationMatrix / RotationMatrixToAngleAxis
//        (called Optimizer.h:61,167; Optimizer.cpp:264,298,450,464,592,631)
//    * Ceres' TrustRegionMinimizer + LevenbergMarquardtStrategy with the
//      options of BAOptimizer::configureSolver (Optimizer.cpp:80-90) and
//      Ceres defaults for everything else
//    * the DENSE_SCHUR linear solver (Optimizer.cpp:85): Schur elimination of
//      point (e-)blocks, dense Cholesky of the reduced camera system, back-
//      substitution.
//
//  Ceres itself is a third-party dependency that is NOT vendored in the
//  reference (CMakeLists.txt:22, version unpinned: libceres-dev from
//  ubuntu:latest = Ceres 2.0.0 / 2.2.0).  Its algorithm is restated here from
//  its published source/documentation (trust_region_minimizer.cc,
//  levenberg_marquardt_strategy.cc, trust_region_step_evaluator.cc,
//  corrector.cc, loss_function.cc, rotation.h, jet.h).
//
//  PARITY UNPINNED: the reference holds no golden vectors, fixtures or tests
//  for this path and cannot be built here (Ceres, Eigen,
//  OpenCV absent).  This restatement is cross-checked instead by known-answer
//  tests (rotation round trips, noise-free convergence to ground truth) and by
//  an independent torch-fp64 restatement of the functors (tests/golden/).
// =============================================================================
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace oracle {

// ----------------------------------------------------------------------------
// Forward-mode dual number with N derivative slots (ceres/jet.h semantics).
// ----------------------------------------------------------------------------
template <int N>
struct Jet {
  double a;
  double v[N];
  Jet() : a(0) { for (int i = 0; i < N; ++i) v[i] = 0; }
  explicit Jet(double x) : a(x) { for (int i = 0; i < N; ++i) v[i] = 0; }
  Jet(double x, int k) : a(x) { for (int i = 0; i < N; ++i) v[i] = 0; v[k] = 1.0; }
};
template <int N> inline Jet<N> operator+(const Jet<N>& f, const Jet<N>& g) { Jet<N> h(f.a + g.a); for (int i = 0; i < N; ++i) h.v[i] = f.v[i] + g.v[i]; return h; }
template <int N> inline Jet<N> operator-(const Jet<N>& f, const Jet<N>& g) { Jet<N> h(f.a - g.a); for (int i = 0; i < N; ++i) h.v[i] = f.v[i] - g.v[i]; return h; }
template <int N> inline Jet<N> operator-(const Jet<N>& f) { Jet<N> h(-f.a); for (int i = 0; i < N; ++i) h.v[i] = -f.v[i]; return h; }
template <int N> inline Jet<N> operator*(const Jet<N>& f, const Jet<N>& g) { Jet<N> h(f.a * g.a); for (int i = 0; i < N; ++i) h.v[i] = f.a * g.v[i] + f.v[i] * g.a; return h; }
template <int N> inline Jet<N> operator/(const Jet<N>& f, const Jet<N>& g) {
  // ceres: a/b, derivative (f.v - (f.a/g.a) g.v) / g.a
  const double ginv = 1.0 / g.a; const double fg = f.a * ginv;
  Jet<N> h(fg); for (int i = 0; i < N; ++i) h.v[i] = (f.v[i] - fg * g.v[i]) * ginv; return h;
}
template <int N> inline Jet<N> operator+(const Jet<N>& f, double s) { Jet<N> h = f; h.a += s; return h; }
template <int N> inline Jet<N> operator+(double s, const Jet<N>& f) { Jet<N> h = f; h.a += s; return h; }
template <int N> inline Jet<N> operator-(const Jet<N>& f, double s) { Jet<N> h = f; h.a -= s; return h; }
template <int N> inline Jet<N> operator-(double s, const Jet<N>& f) { Jet<N> h(s - f.a); for (int i = 0; i < N; ++i) h.v[i] = -f.v[i]; return h; }
template <int N> inline Jet<N> operator*(const Jet<N>& f, double s) { Jet<N> h(f.a * s); for (int i = 0; i < N; ++i) h.v[i] = f.v[i] * s; return h; }
template <int N> inline Jet<N> operator*(double s, const Jet<N>& f) { return f * s; }
template <int N> inline Jet<N> operator/(const Jet<N>& f, double s) { const double si = 1.0 / s; Jet<N> h(f.a * si); for (int i = 0; i < N; ++i) h.v[i] = f.v[i] * si; return h; }
template <int N> inline bool operator>(const Jet<N>& f, double s) { return f.a > s; }
template <int N> inline Jet<N> sqrt(const Jet<N>& f) { const double t = std::sqrt(f.a); const double ti = 1.0 / (2.0 * t); Jet<N> h(t); for (int i = 0; i < N; ++i) h.v[i] = f.v[i] * ti; return h; }
template <int N> inline Jet<N> cos(const Jet<N>& f) { Jet<N> h(std::cos(f.a)); const double d = -std::sin(f.a); for (int i = 0; i < N; ++i) h.v[i] = d * f.v[i]; return h; }
template <int N> inline Jet<N> sin(const Jet<N>& f) { Jet<N> h(std::sin(f.a)); const double d = std::cos(f.a); for (int i = 0; i < N; ++i) h.v[i] = d * f.v[i]; return h; }
using std::sqrt; using std::sin; using std::cos;

inline double scalar_of(double x) { return x; }
template <int N> inline double scalar_of(const Jet<N>& x) { return x.a; }

// ----------------------------------------------------------------------------
// ceres/rotation.h restated.  R is column-major (ceres ColumnMajorAdapter3x3),
// which is also how Eigen reads it at Optimizer.h:62 (Matrix<T,3,3>(rotMat)).
// ----------------------------------------------------------------------------
template <typename T>
void AngleAxisToRotationMatrix(const T* aa, T* R) {
  auto Rm = [&](int r, int c) -> T& { return R[c * 3 + r]; };
  const T theta2 = aa[0] * aa[0] + aa[1] * aa[1] + aa[2] * aa[2];
  if (scalar_of(theta2) > std::numeric_limits<double>::epsilon()) {
    const T theta = sqrt(theta2);
    const T wx = aa[0] / theta, wy = aa[1] / theta, wz = aa[2] / theta;
    const T c = cos(theta), s = sin(theta);
    const T one_c = 1.0 - c;
    Rm(0, 0) = c + wx * wx * one_c;
    Rm(1, 0) = wz * s + wx * wy * one_c;
    Rm(2, 0) = -(wy * s) + wx * wz * one_c;
    Rm(0, 1) = wx * wy * one_c - wz * s;
    Rm(1, 1) = c + wy * wy * one_c;
    Rm(2, 1) = wx * s + wy * wz * one_c;
    Rm(0, 2) = wy * s + wx * wz * one_c;
    Rm(1, 2) = -(wx * s) + wy * wz * one_c;
    Rm(2, 2) = c + wz * wz * one_c;
  } else {
    // first-order Taylor expansion near zero (ceres)
    Rm(0, 0) = T(1.0); Rm(1, 0) = aa[2];  Rm(2, 0) = -aa[1];
    Rm(0, 1) = -aa[2]; Rm(1, 1) = T(1.0); Rm(2, 1) = aa[0];
    Rm(0, 2) = aa[1];  Rm(1, 2) = -aa[0]; Rm(2, 2) = T(1.0);
  }
}

// RotationMatrixToAngleAxis = RotationMatrixToQuaternion (Shepperd) followed by
// QuaternionToAngleAxis (atan2 with the cos<0 flip).  R column-major.
void RotationMatrixToAngleAxis(const double* R, double* aa) {
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
  const double q1 = q[1], q2 = q[2], q3 = q[3];
  const double sin_sq = q1 * q1 + q2 * q2 + q3 * q3;
  if (sin_sq > 0.0) {
    const double sin_theta = std::sqrt(sin_sq);
    const double cos_theta = q[0];
    const double two_theta = 2.0 * ((cos_theta < 0.0) ? std::atan2(-sin_theta, -cos_theta)
                                                       : std::atan2(sin_theta, cos_theta));
    const double k = two_theta / sin_theta;
    aa[0] = q1 * k; aa[1] = q2 * k; aa[2] = q3 * k;
  } else {
    aa[0] = q1 * 2.0; aa[1] = q2 * 2.0; aa[2] = q3 * 2.0;
  }
}

// ----------------------------------------------------------------------------
// The three functors, restated from Optimizer.h.  K and the observation are
// float in the reference (Matrix3f / Vector2f) and promoted to T.
// K and extr are column-major (Eigen default storage).
// ----------------------------------------------------------------------------
template <typename T>
inline void project_K(const float* K, const T* p, T* res, float u, float v) {
  // (cameraIntrinsics.cast<T>() * p).hnormalized() - observed_pos.cast<T>()
  T q[3];
  for (int i = 0; i < 3; ++i)
    q[i] = p[0] * double(K[0 * 3 + i]) + p[1] * double(K[1 * 3 + i]) + p[2] * double(K[2 * 3 + i]);
  res[0] = q[0] / q[2] - double(u);
  res[1] = q[1] / q[2] - double(v);
}

// AngleReprojectionError::operator()  (Optimizer.h:54-76)
template <typename T>
void angle_reprojection(const T* cam, const T* pt, const float* K, float u, float v, T* res) {
  T R[9];
  AngleAxisToRotationMatrix(cam, R);
  T p[3];
  for (int i = 0; i < 3; ++i) p[i] = R[0 * 3 + i] * pt[0] + R[1 * 3 + i] * pt[1] + R[2 * 3 + i] * pt[2] + cam[3 + i];
  project_K(K, p, res, u, v);
}

// PointOnlyReprojectionError::operator()  (Optimizer.h:96-107)
template <typename T>
void point_only_reprojection(const T* pt, const float* extr, const float* K, float u, float v, T* res) {
  T ph[4];
  for (int i = 0; i < 4; ++i)
    ph[i] = pt[0] * double(extr[0 * 4 + i]) + pt[1] * double(extr[1 * 4 + i]) + pt[2] * double(extr[2 * 4 + i]) + double(extr[3 * 4 + i]);
  T p[3] = {ph[0] / ph[3], ph[1] / ph[3], ph[2] / ph[3]};
  project_K(K, p, res, u, v);
}

// PoseOnlyAngleReprojectionError::operator()  (Optimizer.h:163-182);  the point
// is a constant Vector4f (x,y,z,1).
template <typename T>
void pose_only_angle_reprojection(const T* cam, const double* X, const float* K, float u, float v, T* res) {
  T R[9];
  AngleAxisToRotationMatrix(cam, R);
  T p[3];
  for (int i = 0; i < 3; ++i) p[i] = R[0 * 3 + i] * X[0] + R[1 * 3 + i] * X[1] + R[2 * 3 + i] * X[2] + cam[3 + i];
  project_K(K, p, res, u, v);
}

// ----------------------------------------------------------------------------
// ceres::HuberLoss::Evaluate + Corrector (rho'' <= 0 branch: sqrt(rho') scaling)
// ----------------------------------------------------------------------------
struct Huber {
  double a, b;
  bool on;
  explicit Huber(double a_) : a(a_), b(a_ * a_), on(a_ > 0) {}
  // returns rho0, sets scale = sqrt(rho1)
  double eval(double s, double* scale) const {
    if (!on) { *scale = 1.0; return s; }
    if (s > b) {
      const double r = std::sqrt(s);
      const double rho1 = std::max(std::numeric_limits<double>::min(), a / r);
      *scale = std::sqrt(rho1);
      return 2.0 * a * r - b;
    }
    *scale = 1.0;
    return s;
  }
};

// ----------------------------------------------------------------------------
// Problem (same data meaning as the product ABI, restated independently).
// ----------------------------------------------------------------------------
enum RBType { RB_ANGLE = 0, RB_POINT_ONLY = 1, RB_POSE_ONLY = 2, RB_CONST = 3 };

struct Problem {
  int nc, np, no;
  double* cams;           // 6*nc, in/out
  const uint8_t* cam_fixed;
  const float* cam_extr;  // 16*nc col-major (fixed cameras)
  const float* K;         // 9*nc col-major
  double* pts;            // 3*np in/out
  const uint8_t* pt_fixed;
  const int32_t* obs_cam;
  const int32_t* obs_pt;
  const float* obs_uv;
  double huber_a;
  // derived
  std::vector<int> type;      // per obs
  std::vector<int> cam_col;   // per cam: column offset of its 6-block or -1
  std::vector<int> pt_col;    // per point: column offset or -1
  int ncols = 0;
  std::vector<int> var_cams, var_pts;   // active (in problem) blocks
};

static void build_structure(Problem& P) {
  P.type.resize(P.no);
  std::vector<char> cam_used(P.nc, 0), pt_used(P.np, 0);
  for (int o = 0; o < P.no; ++o) {
    const int c = P.obs_cam[o], p = P.obs_pt[o];
    const bool cf = P.cam_fixed && P.cam_fixed[c];
    const bool pf = P.pt_fixed && P.pt_fixed[p];
    int t = cf ? (pf ? RB_CONST : RB_POINT_ONLY) : (pf ? RB_POSE_ONLY : RB_ANGLE);
    P.type[o] = t;
    if (!cf) cam_used[c] = 1;
    if (!pf) pt_used[p] = 1;
  }
  P.cam_col.assign(P.nc, -1);
  P.pt_col.assign(P.np, -1);
  int col = 0;
  for (int c = 0; c < P.nc; ++c) if (cam_used[c]) { P.cam_col[c] = col; col += 6; P.var_cams.push_back(c); }
  for (int p = 0; p < P.np; ++p) if (pt_used[p]) { P.pt_col[p] = col; col += 3; P.var_pts.push_back(p); }
  P.ncols = col;
}

// x <-> problem parameters
static void gather_x(const Problem& P, std::vector<double>& x) {
  x.resize(P.ncols);
  for (int c : P.var_cams) for (int k = 0; k < 6; ++k) x[P.cam_col[c] + k] = P.cams[6 * c + k];
  for (int p : P.var_pts) for (int k = 0; k < 3; ++k) x[P.pt_col[p] + k] = P.pts[3 * p + k];
}
static void scatter_x(Problem& P, const std::vector<double>& x) {
  for (int c : P.var_cams) for (int k = 0; k < 6; ++k) P.cams[6 * c + k] = x[P.cam_col[c] + k];
  for (int p : P.var_pts) for (int k = 0; k < 3; ++k) P.pts[3 * p + k] = x[P.pt_col[p] + k];
}

// Per-obs linearisation: corrected residual r (2), corrected jacobian blocks
// Jc (2x6 row-major) and Jp (2x3 row-major); returns block cost 0.5*rho.
struct Lin { double r[2]; double Jc[12]; double Jp[6]; };

static inline const double* param_cam(const Problem& P, const std::vector<double>& x, int c) {
  return P.cam_col[c] >= 0 ? &x[P.cam_col[c]] : &P.cams[6 * c];
}
static inline const double* param_pt(const Problem& P, const std::vector<double>& x, int p) {
  return P.pt_col[p] >= 0 ? &x[P.pt_col[p]] : &P.pts[3 * p];
}

static double eval_obs(const Problem& P, const std::vector<double>& x, int o, Lin* L, bool* finite) {
  const int c = P.obs_cam[o], p = P.obs_pt[o];
  const float u = P.obs_uv[2 * o], v = P.obs_uv[2 * o + 1];
  const float* K = P.K + 9 * c;
  const double* cam = param_cam(P, x, c);
  const double* pt = param_pt(P, x, p);
  double r[2];
  double Jc[12] = {0}, Jp[6] = {0};
  // Cost-only evaluation: ceres calls the functor with T = double (no Jets),
  // so the divisions are true divisions rather than Jet reciprocal-multiply.
  const int kind = L ? P.type[o] : RB_CONST;
  switch (kind) {
    case RB_ANGLE: {
      Jet<9> jc[6], jp[3], res[2];
      for (int k = 0; k < 6; ++k) jc[k] = Jet<9>(cam[k], k);
      for (int k = 0; k < 3; ++k) jp[k] = Jet<9>(pt[k], 6 + k);
      angle_reprojection(jc, jp, K, u, v, res);
      for (int i = 0; i < 2; ++i) {
        r[i] = res[i].a;
        for (int k = 0; k < 6; ++k) Jc[i * 6 + k] = res[i].v[k];
        for (int k = 0; k < 3; ++k) Jp[i * 3 + k] = res[i].v[6 + k];
      }
      break;
    }
    case RB_POINT_ONLY: {
      Jet<3> jp[3], res[2];
      for (int k = 0; k < 3; ++k) jp[k] = Jet<3>(pt[k], k);
      point_only_reprojection(jp, P.cam_extr + 16 * c, K, u, v, res);
      for (int i = 0; i < 2; ++i) { r[i] = res[i].a; for (int k = 0; k < 3; ++k) Jp[i * 3 + k] = res[i].v[k]; }
      break;
    }
    case RB_POSE_ONLY: {
      Jet<6> jc[6], res[2];
      for (int k = 0; k < 6; ++k) jc[k] = Jet<6>(cam[k], k);
      pose_only_angle_reprojection(jc, pt, K, u, v, res);
      for (int i = 0; i < 2; ++i) { r[i] = res[i].a; for (int k = 0; k < 6; ++k) Jc[i * 6 + k] = res[i].v[k]; }
      break;
    }
    default: {  // constant block: value only
      if (P.cam_fixed && P.cam_fixed[c]) {
        double pr[3] = {pt[0], pt[1], pt[2]};
        point_only_reprojection(pr, P.cam_extr + 16 * c, K, u, v, r);
      } else {
        angle_reprojection(cam, pt, K, u, v, r);
      }
    }
  }
  const double sq = r[0] * r[0] + r[1] * r[1];
  *finite = std::isfinite(r[0]) && std::isfinite(r[1]);
  Huber h(P.huber_a);
  double scale;
  const double rho = h.eval(sq, &scale);
  if (L) {
    L->r[0] = r[0] * scale; L->r[1] = r[1] * scale;
    for (int k = 0; k < 12; ++k) L->Jc[k] = Jc[k] * scale;
    for (int k = 0; k < 6; ++k) L->Jp[k] = Jp[k] * scale;
    if (P.type[o] == RB_POINT_ONLY || P.type[o] == RB_CONST) for (int k = 0; k < 12; ++k) L->Jc[k] = 0;
    if (P.type[o] == RB_POSE_ONLY || P.type[o] == RB_CONST) for (int k = 0; k < 6; ++k) L->Jp[k] = 0;
  }
  return 0.5 * rho;
}

// cost only (ceres Evaluator with residuals = jacobians = nullptr)
static bool eval_cost(const Problem& P, const std::vector<double>& x, double* cost) {
  double total = 0.0;
  bool ok = true;
#pragma omp parallel for reduction(+ : total) reduction(&& : ok) schedule(static)
  for (int o = 0; o < P.no; ++o) {
    bool f;
    total += eval_obs(P, x, o, nullptr, &f);
    ok = ok && f;
  }
  *cost = total;
  return ok && std::isfinite(total);
}

static bool eval_lin(const Problem& P, const std::vector<double>& x, std::vector<Lin>& L, double* cost) {
  L.resize(P.no);
  double total = 0.0;
  bool ok = true;
#pragma omp parallel for reduction(+ : total) reduction(&& : ok) schedule(static)
  for (int o = 0; o < P.no; ++o) {
    bool f;
    total += eval_obs(P, x, o, &L[o], &f);
    bool jf = true;
    for (int k = 0; k < 12; ++k) jf = jf && std::isfinite(L[o].Jc[k]);
    for (int k = 0; k < 6; ++k) jf = jf && std::isfinite(L[o].Jp[k]);
    ok = ok && f && jf;
  }
  *cost = total;
  return ok && std::isfinite(total);
}

// gradient g = J^T r  and squared column norms of J (both unscaled)
static void gradient_colnorm(const Problem& P, const std::vector<Lin>& L, std::vector<double>& g,
                             std::vector<double>& cn) {
  g.assign(P.ncols, 0.0);
  cn.assign(P.ncols, 0.0);
  for (int o = 0; o < P.no; ++o) {
    const int c = P.obs_cam[o], p = P.obs_pt[o];
    const Lin& l = L[o];
    const int cc = (P.type[o] == RB_ANGLE || P.type[o] == RB_POSE_ONLY) ? P.cam_col[c] : -1;
    const int pc = (P.type[o] == RB_ANGLE || P.type[o] == RB_POINT_ONLY) ? P.pt_col[p] : -1;
    if (cc >= 0)
      for (int k = 0; k < 6; ++k) {
        g[cc + k] += l.Jc[k] * l.r[0] + l.Jc[6 + k] * l.r[1];
        cn[cc + k] += l.Jc[k] * l.Jc[k] + l.Jc[6 + k] * l.Jc[6 + k];
      }
    if (pc >= 0)
      for (int k = 0; k < 3; ++k) {
        g[pc + k] += l.Jp[k] * l.r[0] + l.Jp[3 + k] * l.r[1];
        cn[pc + k] += l.Jp[k] * l.Jp[k] + l.Jp[3 + k] * l.Jp[3 + k];
      }
  }
}

// ----------------------------------------------------------------------------
// Dense Cholesky (lower, row-major, in place).  Returns false on a
// non-positive / non-finite pivot (Eigen LLT info() != Success).
// ----------------------------------------------------------------------------
static bool cholesky(std::vector<double>& A, int n) {
  const int nb = 64;
  for (int k = 0; k < n; k += nb) {
    const int b = std::min(nb, n - k);
    // factor diagonal block
    for (int j = k; j < k + b; ++j) {
      double d = A[(size_t)j * n + j];
      for (int t = k; t < j; ++t) d -= A[(size_t)j * n + t] * A[(size_t)j * n + t];
      if (!(d > 0.0) || !std::isfinite(d)) return false;
      d = std::sqrt(d);
      A[(size_t)j * n + j] = d;
      for (int i = j + 1; i < k + b; ++i) {
        double s = A[(size_t)i * n + j];
        for (int t = k; t < j; ++t) s -= A[(size_t)i * n + t] * A[(size_t)j * n + t];
        A[(size_t)i * n + j] = s / d;
      }
    }
    // panel below
#pragma omp parallel for schedule(static)
    for (int i = k + b; i < n; ++i) {
      for (int j = k; j < k + b; ++j) {
        double s = A[(size_t)i * n + j];
        for (int t = k; t < j; ++t) s -= A[(size_t)i * n + t] * A[(size_t)j * n + t];
        A[(size_t)i * n + j] = s / A[(size_t)j * n + j];
      }
    }
    // trailing update (lower)
#pragma omp parallel for schedule(dynamic, 8)
    for (int i = k + b; i < n; ++i) {
      const double* ai = &A[(size_t)i * n + k];
      for (int j = k + b; j <= i; ++j) {
        const double* aj = &A[(size_t)j * n + k];
        double s = 0.0;
        for (int t = 0; t < b; ++t) s += ai[t] * aj[t];
        A[(size_t)i * n + j] -= s;
      }
    }
  }
  return true;
}
static void chol_solve(const std::vector<double>& L, int n, std::vector<double>& b) {
  for (int i = 0; i < n; ++i) {
    double s = b[i];
    for (int t = 0; t < i; ++t) s -= L[(size_t)i * n + t] * b[t];
    b[i] = s / L[(size_t)i * n + i];
  }
  for (int i = n - 1; i >= 0; --i) {
    double s = b[i];
    for (int t = i + 1; t < n; ++t) s -= L[(size_t)t * n + i] * b[t];
    b[i] = s / L[(size_t)i * n + i];
  }
}

// 3x3 SPD inverse through LLT (Eigen selfadjointView.llt().solve(I))
static bool inv3_spd(const double A[9], double Ai[9]) {
  double l00 = A[0];
  if (!(l00 > 0)) return false;
  l00 = std::sqrt(l00);
  const double l10 = A[3] / l00, l20 = A[6] / l00;
  double l11 = A[4] - l10 * l10;
  if (!(l11 > 0)) return false;
  l11 = std::sqrt(l11);
  const double l21 = (A[7] - l20 * l10) / l11;
  double l22 = A[8] - l20 * l20 - l21 * l21;
  if (!(l22 > 0)) return false;
  l22 = std::sqrt(l22);
  for (int col = 0; col < 3; ++col) {
    double e[3] = {0, 0, 0};
    e[col] = 1.0;
    double z0 = e[0] / l00, z1 = (e[1] - l10 * z0) / l11, z2 = (e[2] - l20 * z0 - l21 * z1) / l22;
    double y2 = z2 / l22, y1 = (z1 - l21 * y2) / l11, y0 = (z0 - l10 * y1 - l20 * y2) / l00;
    Ai[0 * 3 + col] = y0; Ai[1 * 3 + col] = y1; Ai[2 * 3 + col] = y2;
  }
  return true;
}

// ----------------------------------------------------------------------------
// DENSE_SCHUR restated: solve (Js^T Js + diag(D)^2) y = Js^T r  where Js is
// the column-scaled jacobian (Js = J diag(s)).  Points are the eliminated
// e-blocks, cameras the f-blocks.  Returns false on solver failure.
// ----------------------------------------------------------------------------
struct Schur {
  // per variable point: list of obs
  std::vector<std::vector<int>> pt_obs;
  std::vector<int> fidx;   // per cam: f-block index or -1
  int nf = 0;
};

// Reduced camera system (lower triangle of lhs, rhs) of the scaled, damped
// normal equations; the point blocks' inverses and gradients are returned
// for the back substitution.  add_cam_D = false leaves out the camera LM
// diagonal (a point shard's contribution in the distributed test: the
// system is a sum over point shards plus the camera diagonal once).
static bool assemble_schur(const Problem& P, const Schur& S, const std::vector<Lin>& L, const std::vector<double>& s,
                           const std::vector<double>& D, bool add_cam_D, std::vector<double>& lhs,
                           std::vector<double>& rhs, std::vector<double>& ete_inv, std::vector<double>& ge) {
  const int nf = S.nf, n = 6 * nf;
  lhs.assign((size_t)n * n, 0.0);
  rhs.assign(n, 0.0);
  auto scJc = [&](int o, double* Jc) {  // scaled camera jacobian 2x6
    const int cc = P.cam_col[P.obs_cam[o]];
    for (int i = 0; i < 2; ++i) for (int k = 0; k < 6; ++k) Jc[i * 6 + k] = L[o].Jc[i * 6 + k] * s[cc + k];
  };
  auto scJp = [&](int o, double* Jp) {
    const int pc = P.pt_col[P.obs_pt[o]];
    for (int i = 0; i < 2; ++i) for (int k = 0; k < 3; ++k) Jp[i * 3 + k] = L[o].Jp[i * 3 + k] * s[pc + k];
  };
  // F^T F + D_f^2 and F^T r over all residuals that touch a variable camera
  for (int o = 0; o < P.no; ++o) {
    const int t = P.type[o];
    if (t != RB_ANGLE && t != RB_POSE_ONLY) continue;
    const int f = S.fidx[P.obs_cam[o]];
    double Jc[12];
    scJc(o, Jc);
    for (int a = 0; a < 6; ++a) {
      rhs[6 * f + a] += Jc[a] * L[o].r[0] + Jc[6 + a] * L[o].r[1];
      for (int b = 0; b <= a; ++b)
        lhs[(size_t)(6 * f + a) * n + 6 * f + b] += Jc[a] * Jc[b] + Jc[6 + a] * Jc[6 + b];
    }
  }
  if (add_cam_D)
    for (int c : P.var_cams) {
      const int f = S.fidx[c], cc = P.cam_col[c];
      for (int a = 0; a < 6; ++a) lhs[(size_t)(6 * f + a) * n + 6 * f + a] += D[cc + a] * D[cc + a];
    }
  // eliminate points
  const int npv = (int)P.var_pts.size();
  ete_inv.assign((size_t)npv * 9, 0.0);
  ge.assign((size_t)npv * 3, 0.0);
  bool ok = true;
  int nthreads = 1;
#ifdef _OPENMP
  nthreads = omp_get_max_threads();
#endif
  // per-thread lhs accumulation, reduced in thread order
  const size_t lhs_bytes = (size_t)n * n * sizeof(double);
  int nacc = std::max(1, std::min(nthreads, (int)(2e9 / std::max<size_t>(lhs_bytes, 1))));
  std::vector<std::vector<double>> acc_l(nacc, std::vector<double>()), acc_r(nacc, std::vector<double>(n, 0.0));
  for (auto& a : acc_l) a.assign((size_t)n * n, 0.0);
#pragma omp parallel num_threads(nacc) reduction(&& : ok)
  {
    int tid = 0;
#ifdef _OPENMP
    tid = omp_get_thread_num();
#endif
    std::vector<double>& al = acc_l[tid];
    std::vector<double>& ar = acc_r[tid];
    std::vector<int> fl;
    std::vector<double> FtE;  // per distinct f-block in chunk: 6x3
#pragma omp for schedule(dynamic, 64)
    for (int ip = 0; ip < npv; ++ip) {
      const int p = P.var_pts[ip], pc = P.pt_col[p];
      double ete[9] = {0}, g[3] = {0};
      fl.clear();
      FtE.clear();
      for (int o : S.pt_obs[ip]) {
        double Jp[6];
        scJp(o, Jp);
        for (int a = 0; a < 3; ++a) {
          g[a] += Jp[a] * L[o].r[0] + Jp[3 + a] * L[o].r[1];
          for (int b = 0; b < 3; ++b) ete[a * 3 + b] += Jp[a] * Jp[b] + Jp[3 + a] * Jp[3 + b];
        }
        if (P.type[o] == RB_ANGLE) {
          const int f = S.fidx[P.obs_cam[o]];
          int slot = -1;
          for (size_t q = 0; q < fl.size(); ++q) if (fl[q] == f) slot = (int)q;
          if (slot < 0) { slot = (int)fl.size(); fl.push_back(f); FtE.resize(FtE.size() + 18, 0.0); }
          double Jc[12];
          scJc(o, Jc);
          double* B = &FtE[(size_t)slot * 18];
          for (int a = 0; a < 6; ++a) for (int b = 0; b < 3; ++b) B[a * 3 + b] += Jc[a] * Jp[b] + Jc[6 + a] * Jp[3 + b];
        }
      }
      for (int a = 0; a < 3; ++a) ete[a * 3 + a] += D[pc + a] * D[pc + a];
      double* inv = &ete_inv[(size_t)ip * 9];
      if (!inv3_spd(ete, inv)) { ok = false; continue; }
      for (int a = 0; a < 3; ++a) ge[(size_t)ip * 3 + a] = g[a];
      const int m = (int)fl.size();
      // tmp_q = FtE_q * inv  (6x3)
      std::vector<double> T((size_t)m * 18);
      for (int q = 0; q < m; ++q)
        for (int a = 0; a < 6; ++a)
          for (int b = 0; b < 3; ++b) {
            double v = 0;
            for (int t = 0; t < 3; ++t) v += FtE[(size_t)q * 18 + a * 3 + t] * inv[t * 3 + b];
            T[(size_t)q * 18 + a * 3 + b] = v;
          }
      for (int q = 0; q < m; ++q) {
        const int fq = fl[q];
        for (int a = 0; a < 6; ++a) {
          double v = 0;
          for (int t = 0; t < 3; ++t) v += T[(size_t)q * 18 + a * 3 + t] * g[t];
          ar[6 * fq + a] -= v;
        }
        for (int w = 0; w < m; ++w) {
          const int fw = fl[w];
          if (fw > fq) continue;  // lower triangle only: block (fq, fw) with fw <= fq
          for (int a = 0; a < 6; ++a)
            for (int b = 0; b < 6; ++b) {
              if (fw == fq && b > a) continue;
              double v = 0;
              for (int t = 0; t < 3; ++t) v += T[(size_t)q * 18 + a * 3 + t] * FtE[(size_t)w * 18 + b * 3 + t];
              al[(size_t)(6 * fq + a) * n + 6 * fw + b] -= v;
            }
        }
      }
    }
  }
  if (!ok) return false;
  for (int t = 0; t < nacc; ++t) {
    for (size_t i = 0; i < lhs.size(); ++i) lhs[i] += acc_l[t][i];
    for (int i = 0; i < n; ++i) rhs[i] += acc_r[t][i];
  }
  return true;
}

static bool dense_schur_solve(const Problem& P, const Schur& S, const std::vector<Lin>& L,
                              const std::vector<double>& s, const std::vector<double>& D,
                              std::vector<double>& y) {
  const int nf = S.nf, n = 6 * nf;
  y.assign(P.ncols, 0.0);
  std::vector<double> lhs, rhs, ete_inv, ge;
  if (!assemble_schur(P, S, L, s, D, true, lhs, rhs, ete_inv, ge)) return false;
  const int npv = (int)P.var_pts.size();
  const bool has_cam = nf > 0;
  auto scJc = [&](int o, double* Jc) {
    const int cc = P.cam_col[P.obs_cam[o]];
    for (int i = 0; i < 2; ++i) for (int k = 0; k < 6; ++k) Jc[i * 6 + k] = L[o].Jc[i * 6 + k] * s[cc + k];
  };
  auto scJp = [&](int o, double* Jp) {
    const int pc = P.pt_col[P.obs_pt[o]];
    for (int i = 0; i < 2; ++i) for (int k = 0; k < 3; ++k) Jp[i * 3 + k] = L[o].Jp[i * 3 + k] * s[pc + k];
  };
  std::vector<double> yf(rhs);
  if (has_cam) {
    if (!cholesky(lhs, n)) return false;
    chol_solve(lhs, n, yf);
  }
  for (int c : P.var_cams) for (int a = 0; a < 6; ++a) y[P.cam_col[c] + a] = yf[6 * S.fidx[c] + a];
  // back substitution  y_e = inv (g_e - sum_f (F^T E)^T y_f)
#pragma omp parallel for schedule(dynamic, 64)
  for (int ip = 0; ip < npv; ++ip) {
    const int p = P.var_pts[ip], pc = P.pt_col[p];
    double w[3] = {ge[(size_t)ip * 3], ge[(size_t)ip * 3 + 1], ge[(size_t)ip * 3 + 2]};
    for (int o : S.pt_obs[ip]) {
      if (P.type[o] != RB_ANGLE) continue;
      double Jp[6], Jc[12];
      scJp(o, Jp);
      scJc(o, Jc);
      const int f = S.fidx[P.obs_cam[o]];
      double z[2] = {0, 0};
      for (int k = 0; k < 6; ++k) { z[0] += Jc[k] * yf[6 * f + k]; z[1] += Jc[6 + k] * yf[6 * f + k]; }
      for (int a = 0; a < 3; ++a) w[a] -= Jp[a] * z[0] + Jp[3 + a] * z[1];
    }
    const double* inv = &ete_inv[(size_t)ip * 9];
    for (int a = 0; a < 3; ++a) y[pc + a] = inv[a * 3] * w[0] + inv[a * 3 + 1] * w[1] + inv[a * 3 + 2] * w[2];
  }
  for (double v : y) if (!std::isfinite(v)) return false;
  return true;
}

// ceres::Solver::Options fields used here (Ceres defaults: oracle_default_options)
struct Options {
  int max_num_iterations;
  int max_num_consecutive_invalid_steps;
  int jacobi_scaling;
  int linear_solver;                  // 0 DENSE_SCHUR, 1 ITERATIVE_SCHUR
  double function_tolerance, gradient_tolerance, parameter_tolerance;
  double initial_trust_region_radius, max_trust_region_radius, min_trust_region_radius;
  double min_relative_decrease, min_lm_diagonal, max_lm_diagonal;
  // ITERATIVE_SCHUR (ceres::Solver::Options defaults)
  int preconditioner_type;            // 0 JACOBI (ceres default), 1 SCHUR_JACOBI
  int max_linear_solver_iterations;   // 500
  int min_linear_solver_iterations;   // 0
  int precision;                      // 0 fp64; 1 MIXED_FP32: the Schur blocks W stored in float; 3: c, Z of W = c'Z in float (matvec)
                                      // (iterative_schur_solve_w below); 2 the W form in fp64 (test hook)
  double eta;                         // 1e-1 (LM forcing sequence -> CG q_tolerance)
};
enum { LS_DENSE_SCHUR = 0, LS_ITERATIVE_SCHUR = 1 };
enum { PC_JACOBI = 0, PC_SCHUR_JACOBI = 1 };

// ----------------------------------------------------------------------------
// ITERATIVE_SCHUR restated (Ceres 2.0/2.2: iterative_schur_complement_solver.cc,
// implicit_schur_complement.cc, conjugate_gradients_solver.cc,
// schur_jacobi_preconditioner.cc, block_random_access_diagonal_matrix.cc).
// Not used by the reference (configureSolver picks DENSE_SCHUR,
// Optimizer.cpp:85); it is the scalable linear solver SURVEY.md §8a-a7 / §8e
// name for C5, restated so the GPU's implicit-Schur PCG has a checker.
//
//   S x = D_f^2 x + F'(F x - E (E'E + D_e^2)^-1 E'F x)     (RightMultiply)
//   rhs = F'(b - E (E'E + D_e^2)^-1 E'b)                    (UpdateRhs)
//   CG on S x = rhs from x = 0 with Ceres' termination rules
//   (q_tolerance = eta, r_tolerance = -1: LevenbergMarquardtStrategy),
//   preconditioner JACOBI = blockdiag(F'F + D_f^2)^-1 or SCHUR_JACOBI =
//   blockdiag(S)^-1 (6x6 LLT solves against I);
//   back substitution y_e = (E'E + D_e^2)^-1 E'(b - F x).
// F holds the rows of residuals with a variable camera, E those with a
// variable point, b = the corrected residuals (Ceres solves J step = r and
// negates).  Returns false on LINEAR_SOLVER_FAILURE or a non-finite step.
// ----------------------------------------------------------------------------
static bool llt_inverse(const double* A, int n, double* Ai) {   // Eigen selfadjointView<Upper>().llt().solve(I)
  std::vector<double> Lm((size_t)n * n, 0.0);
  for (int j = 0; j < n; ++j) {
    double d = A[j * n + j];
    for (int t = 0; t < j; ++t) d -= Lm[j * n + t] * Lm[j * n + t];
    if (!(d > 0.0)) return false;
    d = std::sqrt(d);
    Lm[j * n + j] = d;
    for (int i = j + 1; i < n; ++i) {
      double v = A[i * n + j];
      for (int t = 0; t < j; ++t) v -= Lm[i * n + t] * Lm[j * n + t];
      Lm[i * n + j] = v / d;
    }
  }
  for (int col = 0; col < n; ++col) {
    std::vector<double> z(n, 0.0);
    for (int i = 0; i < n; ++i) {
      double v = i == col ? 1.0 : 0.0;
      for (int t = 0; t < i; ++t) v -= Lm[i * n + t] * z[t];
      z[i] = v / Lm[i * n + i];
    }
    for (int i = n - 1; i >= 0; --i) {
      double v = z[i];
      for (int t = i + 1; t < n; ++t) v -= Lm[t * n + i] * z[t];
      z[i] = v / Lm[i * n + i];
    }
    for (int i = 0; i < n; ++i) Ai[i * n + col] = z[i];
  }
  return true;
}

static inline bool zero_or_inf(double x) { return x == 0.0 || std::isinf(x); }   // ceres IsZeroOrInfinity

// ceres ConjugateGradientsSolver::Solve (x = 0 start, r_tolerance = -1,
// q_tolerance = eta, residual reset every 10 iterations) on S x = rhs with
// the block-diagonal preconditioner Minv (nf blocks 6x6).  Returns false on
// LINEAR_SOLVER_FAILURE (NO_CONVERGENCE keeps the iterate).
template <class SchurMul>
static bool pcg_solve(const std::vector<double>& rhs, SchurMul&& schur_mul, const std::vector<double>& Minv, int nf,
                      const Options& opt, std::vector<double>& x, int* cg_iterations) {
  const int n = 6 * nf;
  auto precond = [&](const std::vector<double>& r, std::vector<double>& z) {
    z.assign(n, 0.0);
    for (int f = 0; f < nf; ++f)
      for (int a = 0; a < 6; ++a) {
        double v = 0;
        for (int c = 0; c < 6; ++c) v += Minv[(size_t)f * 36 + a * 6 + c] * r[6 * f + c];
        z[6 * f + a] = v;
      }
  };
  auto dot = [](const std::vector<double>& u, const std::vector<double>& v) {
    double d = 0;
    for (size_t i = 0; i < u.size(); ++i) d += u[i] * v[i];
    return d;
  };
  x.assign(n, 0.0);
  bool failure = false;
  if (nf > 0) {
    const double norm_b = std::sqrt(dot(rhs, rhs));
    if (norm_b != 0.0) {
      const double r_tolerance = -1.0, q_tolerance = opt.eta;
      const double tol_r = r_tolerance * norm_b;
      std::vector<double> r = rhs, p(n), z, q, tmp;   // x = 0: r = b - A x = b
      double norm_r = std::sqrt(dot(r, r));
      if (!(opt.min_linear_solver_iterations == 0 && norm_r <= tol_r)) {
        double rho = 1.0;
        std::vector<double> bpr(n);
        for (int i = 0; i < n; ++i) bpr[i] = rhs[i] + r[i];
        double Q0 = -1.0 * dot(x, bpr);
        for (int it = 1;; ++it) {
          *cg_iterations = it;
          precond(r, z);
          const double last_rho = rho;
          rho = dot(r, z);
          if (zero_or_inf(rho)) { failure = true; break; }
          if (it == 1) p = z;
          else {
            const double beta = rho / last_rho;
            if (zero_or_inf(beta)) { failure = true; break; }
            for (int i = 0; i < n; ++i) p[i] = z[i] + beta * p[i];
          }
          schur_mul(p, q);
          const double pq = dot(p, q);
          if (pq <= 0 || std::isinf(pq)) break;   // LINEAR_SOLVER_NO_CONVERGENCE: x is still used
          const double alpha = rho / pq;
          if (std::isinf(alpha)) { failure = true; break; }
          for (int i = 0; i < n; ++i) x[i] = x[i] + alpha * p[i];
          if (it % 10 == 0) {   // residual_reset_period
            schur_mul(x, tmp);
            for (int i = 0; i < n; ++i) r[i] = rhs[i] - tmp[i];
          } else {
            for (int i = 0; i < n; ++i) r[i] = r[i] - alpha * q[i];
          }
          for (int i = 0; i < n; ++i) bpr[i] = rhs[i] + r[i];
          const double Q1 = -1.0 * dot(x, bpr);
          const double zeta = it * (Q1 - Q0) / Q1;
          if (zeta < q_tolerance && it >= opt.min_linear_solver_iterations) break;
          Q0 = Q1;
          norm_r = std::sqrt(dot(r, r));
          if (norm_r <= tol_r && it >= opt.min_linear_solver_iterations) break;
          if (it >= opt.max_linear_solver_iterations) break;
        }
      }
    }
  }
  return !failure;
}

static bool iterative_schur_solve(const Problem& P, const Schur& S, const std::vector<Lin>& L,
                                  const std::vector<double>& s, const std::vector<double>& D, const Options& opt,
                                  std::vector<double>& y, int* cg_iterations) {
  const int nf = S.nf, n = 6 * nf, npv = (int)P.var_pts.size();
  y.assign(P.ncols, 0.0);
  *cg_iterations = 0;
  auto scJc = [&](int o, double* Jc) {
    const int cc = P.cam_col[P.obs_cam[o]];
    for (int i = 0; i < 2; ++i) for (int k = 0; k < 6; ++k) Jc[i * 6 + k] = L[o].Jc[i * 6 + k] * s[cc + k];
  };
  auto scJp = [&](int o, double* Jp) {
    const int pc = P.pt_col[P.obs_pt[o]];
    for (int i = 0; i < 2; ++i) for (int k = 0; k < 3; ++k) Jp[i * 3 + k] = L[o].Jp[i * 3 + k] * s[pc + k];
  };
  auto has_f = [&](int o) { return P.type[o] == RB_ANGLE || P.type[o] == RB_POSE_ONLY; };
  auto has_e = [&](int o) { return P.type[o] == RB_ANGLE || P.type[o] == RB_POINT_ONLY; };
  std::vector<int> vp(P.np, -1);
  for (int i = 0; i < npv; ++i) vp[P.var_pts[i]] = i;
  // (E'E + D_e^2)^-1 per point (ImplicitSchurComplement::AddDiagonalAndInvert)
  std::vector<double> ete_inv((size_t)npv * 9);
  for (int ip = 0; ip < npv; ++ip) {
    const int pc = P.pt_col[P.var_pts[ip]];
    double ete[9] = {0};
    for (int o : S.pt_obs[ip]) {
      double Jp[6];
      scJp(o, Jp);
      for (int a = 0; a < 3; ++a) for (int b = 0; b < 3; ++b) ete[a * 3 + b] += Jp[a] * Jp[b] + Jp[3 + a] * Jp[3 + b];
    }
    for (int a = 0; a < 3; ++a) ete[a * 3 + a] += D[pc + a] * D[pc + a];
    if (!inv3_spd(ete, &ete_inv[(size_t)ip * 9])) return false;
  }
  // rows: 2 per observation
  auto F_mul = [&](const std::vector<double>& xf, std::vector<double>& rows) {   // rows += F xf
    for (int o = 0; o < P.no; ++o) {
      if (!has_f(o)) continue;
      double Jc[12];
      scJc(o, Jc);
      const double* xc = &xf[6 * S.fidx[P.obs_cam[o]]];
      for (int i = 0; i < 2; ++i) {
        double v = 0;
        for (int k = 0; k < 6; ++k) v += Jc[i * 6 + k] * xc[k];
        rows[2 * o + i] += v;
      }
    }
  };
  auto Ft_mul = [&](const std::vector<double>& rows, std::vector<double>& yf) {   // yf += F' rows
    for (int o = 0; o < P.no; ++o) {
      if (!has_f(o)) continue;
      double Jc[12];
      scJc(o, Jc);
      double* yc = &yf[6 * S.fidx[P.obs_cam[o]]];
      for (int k = 0; k < 6; ++k) yc[k] += Jc[k] * rows[2 * o] + Jc[6 + k] * rows[2 * o + 1];
    }
  };
  auto Et_mul = [&](const std::vector<double>& rows, std::vector<double>& ye) {   // ye += E' rows
    for (int o = 0; o < P.no; ++o) {
      if (!has_e(o)) continue;
      double Jp[6];
      scJp(o, Jp);
      double* yp = &ye[3 * vp[P.obs_pt[o]]];
      for (int k = 0; k < 3; ++k) yp[k] += Jp[k] * rows[2 * o] + Jp[3 + k] * rows[2 * o + 1];
    }
  };
  auto E_mul = [&](const std::vector<double>& xe, std::vector<double>& rows) {   // rows += E xe
    for (int o = 0; o < P.no; ++o) {
      if (!has_e(o)) continue;
      double Jp[6];
      scJp(o, Jp);
      const double* xp = &xe[3 * vp[P.obs_pt[o]]];
      for (int i = 0; i < 2; ++i) rows[2 * o + i] += Jp[i * 3] * xp[0] + Jp[i * 3 + 1] * xp[1] + Jp[i * 3 + 2] * xp[2];
    }
  };
  auto ete_mul = [&](const std::vector<double>& xe, std::vector<double>& ye, double sign) {
    for (int ip = 0; ip < npv; ++ip) {
      const double* m = &ete_inv[(size_t)ip * 9];
      for (int a = 0; a < 3; ++a)
        ye[3 * ip + a] += sign * (m[a * 3] * xe[3 * ip] + m[a * 3 + 1] * xe[3 * ip + 1] + m[a * 3 + 2] * xe[3 * ip + 2]);
    }
  };
  std::vector<double> b(2 * (size_t)P.no, 0.0);
  for (int o = 0; o < P.no; ++o) { b[2 * o] = L[o].r[0]; b[2 * o + 1] = L[o].r[1]; }
  const std::vector<double> zf(n, 0.0), ze(3 * (size_t)npv, 0.0), zr(2 * (size_t)P.no, 0.0);
  auto schur_mul = [&](const std::vector<double>& x, std::vector<double>& out) {   // ImplicitSchurComplement::RightMultiply
    std::vector<double> rows = zr, te = ze, te2 = ze;
    F_mul(x, rows);
    Et_mul(rows, te);
    ete_mul(te, te2, -1.0);
    E_mul(te2, rows);
    out.assign(n, 0.0);
    for (int c : P.var_cams) {
      const int f = S.fidx[c], cc = P.cam_col[c];
      for (int a = 0; a < 6; ++a) out[6 * f + a] = D[cc + a] * D[cc + a] * x[6 * f + a];
    }
    Ft_mul(rows, out);
  };
  // rhs (UpdateRhs)
  std::vector<double> rhs(n, 0.0);
  {
    std::vector<double> te = ze, y2 = ze, rows = zr;
    Et_mul(b, te);
    ete_mul(te, y2, 1.0);
    E_mul(y2, rows);
    for (size_t i = 0; i < rows.size(); ++i) rows[i] = b[i] - rows[i];
    Ft_mul(rows, rhs);
  }
  // preconditioner blocks
  std::vector<double> Minv((size_t)nf * 36, 0.0);
  {
    std::vector<double> blk((size_t)nf * 36, 0.0);
    for (int o = 0; o < P.no; ++o) {
      if (!has_f(o)) continue;
      double Jc[12];
      scJc(o, Jc);
      double* B = &blk[(size_t)S.fidx[P.obs_cam[o]] * 36];
      for (int a = 0; a < 6; ++a) for (int c = 0; c < 6; ++c) B[a * 6 + c] += Jc[a] * Jc[c] + Jc[6 + a] * Jc[6 + c];
    }
    for (int c : P.var_cams) {
      const int f = S.fidx[c], cc = P.cam_col[c];
      for (int a = 0; a < 6; ++a) blk[(size_t)f * 36 + a * 7] += D[cc + a] * D[cc + a];
    }
    if (opt.preconditioner_type == PC_SCHUR_JACOBI) {
      // - sum_p (F_pf'E_p) (E_p'E_p + D^2)^-1 (E_p'F_pf) on the diagonal blocks
      std::vector<int> fl;
      std::vector<double> FtE;
      for (int ip = 0; ip < npv; ++ip) {
        fl.clear();
        FtE.clear();
        for (int o : S.pt_obs[ip]) {
          if (P.type[o] != RB_ANGLE) continue;
          const int f = S.fidx[P.obs_cam[o]];
          int slot = -1;
          for (size_t q = 0; q < fl.size(); ++q) if (fl[q] == f) slot = (int)q;
          if (slot < 0) { slot = (int)fl.size(); fl.push_back(f); FtE.resize(FtE.size() + 18, 0.0); }
          double Jc[12], Jp[6];
          scJc(o, Jc);
          scJp(o, Jp);
          double* B = &FtE[(size_t)slot * 18];
          for (int a = 0; a < 6; ++a) for (int c = 0; c < 3; ++c) B[a * 3 + c] += Jc[a] * Jp[c] + Jc[6 + a] * Jp[3 + c];
        }
        const double* m = &ete_inv[(size_t)ip * 9];
        for (size_t q = 0; q < fl.size(); ++q) {
          const double* B = &FtE[q * 18];
          double T[18];
          for (int a = 0; a < 6; ++a)
            for (int c = 0; c < 3; ++c) T[a * 3 + c] = B[a * 3] * m[c] + B[a * 3 + 1] * m[3 + c] + B[a * 3 + 2] * m[6 + c];
          double* M = &blk[(size_t)fl[q] * 36];
          for (int a = 0; a < 6; ++a)
            for (int c = 0; c < 6; ++c) M[a * 6 + c] -= T[a * 3] * B[c * 3] + T[a * 3 + 1] * B[c * 3 + 1] + T[a * 3 + 2] * B[c * 3 + 2];
        }
      }
    }
    for (int f = 0; f < nf; ++f)
      if (!llt_inverse(&blk[(size_t)f * 36], 6, &Minv[(size_t)f * 36]))
        for (int k = 0; k < 36; ++k) Minv[(size_t)f * 36 + k] = std::numeric_limits<double>::quiet_NaN();
  }
  std::vector<double> x(n, 0.0);
  if (!pcg_solve(rhs, schur_mul, Minv, nf, opt, x, cg_iterations)) return false;
  // BackSubstitute
  {
    std::vector<double> rows = zr, te = ze, ye = ze;
    F_mul(x, rows);
    for (size_t i = 0; i < rows.size(); ++i) rows[i] = b[i] - rows[i];
    Et_mul(rows, te);
    ete_mul(te, ye, 1.0);
    for (int ip = 0; ip < npv; ++ip)
      for (int a = 0; a < 3; ++a) y[P.pt_col[P.var_pts[ip]] + a] = ye[3 * ip + a];
    for (int c : P.var_cams) for (int a = 0; a < 6; ++a) y[P.cam_col[c] + a] = x[6 * S.fidx[c] + a];
  }
  for (double v : y) if (!std::isfinite(v)) return false;
  return true;
}

// ----------------------------------------------------------------------------
// ITERATIVE_SCHUR with the per-observation Schur blocks stored in fp32
// (BA_MIXED_FP32 of include/ba_hip.h; SURVEY.md §8a-a7 / §8c: C5 "fp32
// mixed-precision Schur").  Restated from the definition, not from the
// device code: with L_p L_p^T = E_p'E_p + D_e^2 (lower Cholesky) and
//   W_o = F_o' E_o L_p^-T      (6x3, o = a residual with a variable camera
//                               and a variable point),
// the implicit reduced system of iterative_schur_solve is
//   S x = (F'F + D_f^2) x - sum_p W_p W_p' x,   rhs = F'b - sum_o W_o u_p,
//   u_p = L_p^-1 E_p' b,   back substitution y_e = L_p^-T (u_p - W_p' x),
// and MIXED_FP32 means every W_o entry is rounded to float once and used
// in that form in the matvec, the rhs and the SCHUR_JACOBI blocks; the back
// substitution uses the unrounded W_o (the device recomputes it from J in
// fp64: k_point_step_rc); all sums, the CG vectors and everything else stay
// fp64.
// precision 3 (MIXED_FP32 with the rank-2 records of the PCG point pass,
// include/ba_hip.h BA_MIXED_FP32): W_o = c_o' Z_o with c_o = F_o (scaled,
// 2x6) and Z_o = E_o L_p^-T (2x3); the matvec uses c_o and Z_o each rounded
// to float, associated as W_o' x = Z_o' (c_o x) and W_o v = c_o' (Z_o v);
// the rhs and the SCHUR_JACOBI blocks use the rounded W_o entries (mode 1).
// The CG (termination rules, preconditioner inversion) is the one above.
// ----------------------------------------------------------------------------
static bool iterative_schur_solve_w(const Problem& P, const Schur& S, const std::vector<Lin>& L,
                                    const std::vector<double>& s, const std::vector<double>& D, const Options& opt,
                                    std::vector<double>& y, int* cg_iterations) {
  const int nf = S.nf, n = 6 * nf, npv = (int)P.var_pts.size();
  y.assign(P.ncols, 0.0);
  *cg_iterations = 0;
  auto rnd = [&](double v) { return opt.precision == 1 || opt.precision == 3 ? (double)(float)v : v; };
  const bool rank2 = opt.precision == 3;
  auto scJc = [&](int o, double* Jc) {
    const int cc = P.cam_col[P.obs_cam[o]];
    for (int i = 0; i < 2; ++i) for (int k = 0; k < 6; ++k) Jc[i * 6 + k] = L[o].Jc[i * 6 + k] * s[cc + k];
  };
  auto scJp = [&](int o, double* Jp) {
    const int pc = P.pt_col[P.obs_pt[o]];
    for (int i = 0; i < 2; ++i) for (int k = 0; k < 3; ++k) Jp[i * 3 + k] = L[o].Jp[i * 3 + k] * s[pc + k];
  };
  auto has_f = [&](int o) { return P.type[o] == RB_ANGLE || P.type[o] == RB_POSE_ONLY; };
  // per variable point: L_p^-1 (lower, row-major 3x3) and u_p
  std::vector<double> Linv((size_t)npv * 9, 0.0), u((size_t)npv * 3, 0.0);
  std::vector<int> vp(P.np, -1);
  for (int i = 0; i < npv; ++i) vp[P.var_pts[i]] = i;
  for (int ip = 0; ip < npv; ++ip) {
    const int pc = P.pt_col[P.var_pts[ip]];
    double A[9] = {0}, g[3] = {0};
    for (int o : S.pt_obs[ip]) {
      double Jp[6];
      scJp(o, Jp);
      for (int a = 0; a < 3; ++a) {
        g[a] += Jp[a] * L[o].r[0] + Jp[3 + a] * L[o].r[1];
        for (int b = 0; b < 3; ++b) A[a * 3 + b] += Jp[a] * Jp[b] + Jp[3 + a] * Jp[3 + b];
      }
    }
    for (int a = 0; a < 3; ++a) A[a * 3 + a] += D[pc + a] * D[pc + a];
    if (!(A[0] > 0.0)) return false;
    const double l00 = std::sqrt(A[0]), l10 = A[3] / l00, l20 = A[6] / l00;
    const double d11 = A[4] - l10 * l10;
    if (!(d11 > 0.0)) return false;
    const double l11 = std::sqrt(d11), l21 = (A[7] - l20 * l10) / l11;
    const double d22 = A[8] - l20 * l20 - l21 * l21;
    if (!(d22 > 0.0)) return false;
    const double l22 = std::sqrt(d22);
    double* M = &Linv[(size_t)ip * 9];   // inverse of [[l00,0,0],[l10,l11,0],[l20,l21,l22]]
    M[0] = 1.0 / l00;
    M[4] = 1.0 / l11;
    M[8] = 1.0 / l22;
    M[3] = -l10 * M[0] / l11;
    M[7] = -l21 * M[4] / l22;
    M[6] = -(l20 * M[0] + l21 * M[3]) / l22;
    for (int a = 0; a < 3; ++a) u[(size_t)ip * 3 + a] = M[a * 3] * g[0] + M[a * 3 + 1] * g[1] + M[a * 3 + 2] * g[2];
  }
  // W_o (stored rounded) for residuals with a variable camera and point
  std::vector<double> W((size_t)P.no * 18, 0.0), W64((size_t)P.no * 18, 0.0);   // (W64: unrounded)
  // precision 3: the float-rounded factors c_o (2x6) and Z_o (2x3)
  std::vector<double> Cr(rank2 ? (size_t)P.no * 12 : 0, 0.0), Zr(rank2 ? (size_t)P.no * 6 : 0, 0.0);
  for (int o = 0; o < P.no; ++o) {
    if (P.type[o] != RB_ANGLE) continue;
    const int ip = vp[P.obs_pt[o]];
    double Jc[12], Jp[6];
    scJc(o, Jc);
    scJp(o, Jp);
    const double* M = &Linv[(size_t)ip * 9];
    if (rank2) {
      for (int k = 0; k < 12; ++k) Cr[(size_t)o * 12 + k] = (double)(float)Jc[k];
      for (int i = 0; i < 2; ++i)
        for (int k = 0; k < 3; ++k)   // (Jp_i L^-T)_k = sum_t Jp_it M[k][t]
          Zr[(size_t)o * 6 + i * 3 + k] =
              (double)(float)(Jp[i * 3] * M[k * 3] + Jp[i * 3 + 1] * M[k * 3 + 1] + Jp[i * 3 + 2] * M[k * 3 + 2]);
    }
    for (int a = 0; a < 6; ++a) {
      const double e[3] = {Jc[a] * Jp[0] + Jc[6 + a] * Jp[3], Jc[a] * Jp[1] + Jc[6 + a] * Jp[4],
                           Jc[a] * Jp[2] + Jc[6 + a] * Jp[5]};
      for (int k = 0; k < 3; ++k) {   // (e L^-T)_k = sum_t e_t M[k][t]
        const double wv = e[0] * M[k * 3] + e[1] * M[k * 3 + 1] + e[2] * M[k * 3 + 2];
        W64[(size_t)o * 18 + a * 3 + k] = wv;
        W[(size_t)o * 18 + a * 3 + k] = rnd(wv);
      }
    }
  }
  // A_f = F'F + D_f^2 per camera block, rhs
  std::vector<double> Af((size_t)nf * 36, 0.0), rhs(n, 0.0);
  for (int o = 0; o < P.no; ++o) {
    if (!has_f(o)) continue;
    double Jc[12];
    scJc(o, Jc);
    const int f = S.fidx[P.obs_cam[o]];
    double* B = &Af[(size_t)f * 36];
    for (int a = 0; a < 6; ++a) {
      rhs[6 * f + a] += Jc[a] * L[o].r[0] + Jc[6 + a] * L[o].r[1];
      for (int c = 0; c < 6; ++c) B[a * 6 + c] += Jc[a] * Jc[c] + Jc[6 + a] * Jc[6 + c];
    }
  }
  for (int c : P.var_cams) {
    const int f = S.fidx[c], cc = P.cam_col[c];
    for (int a = 0; a < 6; ++a) Af[(size_t)f * 36 + a * 7] += D[cc + a] * D[cc + a];
  }
  for (int o = 0; o < P.no; ++o) {
    if (P.type[o] != RB_ANGLE) continue;
    const int f = S.fidx[P.obs_cam[o]], ip = vp[P.obs_pt[o]];
    const double* w = &W[(size_t)o * 18];
    const double* up = &u[(size_t)ip * 3];
    for (int a = 0; a < 6; ++a) rhs[6 * f + a] -= w[a * 3] * up[0] + w[a * 3 + 1] * up[1] + w[a * 3 + 2] * up[2];
  }
  auto schur_mul = [&](const std::vector<double>& x, std::vector<double>& out) {
    std::vector<double> v((size_t)npv * 3, 0.0);
    for (int o = 0; o < P.no; ++o) {
      if (P.type[o] != RB_ANGLE) continue;
      const double* xc = &x[6 * S.fidx[P.obs_cam[o]]];
      double* vv = &v[(size_t)vp[P.obs_pt[o]] * 3];
      if (rank2) {   // Z' (c x)
        const double* c = &Cr[(size_t)o * 12];
        const double* z = &Zr[(size_t)o * 6];
        double y[2] = {0.0, 0.0};
        for (int i = 0; i < 2; ++i)
          for (int a = 0; a < 6; ++a) y[i] += c[i * 6 + a] * xc[a];
        for (int k = 0; k < 3; ++k) vv[k] += z[k] * y[0] + z[3 + k] * y[1];
        continue;
      }
      const double* w = &W[(size_t)o * 18];
      for (int k = 0; k < 3; ++k)
        for (int a = 0; a < 6; ++a) vv[k] += w[a * 3 + k] * xc[a];
    }
    out.assign(n, 0.0);
    for (int f = 0; f < nf; ++f)
      for (int a = 0; a < 6; ++a) {
        double t = 0.0;
        for (int c = 0; c < 6; ++c) t += Af[(size_t)f * 36 + a * 6 + c] * x[6 * f + c];
        out[6 * f + a] = t;
      }
    for (int o = 0; o < P.no; ++o) {
      if (P.type[o] != RB_ANGLE) continue;
      const double* vv = &v[(size_t)vp[P.obs_pt[o]] * 3];
      double* oc = &out[6 * S.fidx[P.obs_cam[o]]];
      if (rank2) {   // c' (Z v)
        const double* c = &Cr[(size_t)o * 12];
        const double* z = &Zr[(size_t)o * 6];
        const double q0 = z[0] * vv[0] + z[1] * vv[1] + z[2] * vv[2];
        const double q1 = z[3] * vv[0] + z[4] * vv[1] + z[5] * vv[2];
        for (int a = 0; a < 6; ++a) oc[a] -= c[a] * q0 + c[6 + a] * q1;
        continue;
      }
      const double* w = &W[(size_t)o * 18];
      for (int a = 0; a < 6; ++a) oc[a] -= w[a * 3] * vv[0] + w[a * 3 + 1] * vv[1] + w[a * 3 + 2] * vv[2];
    }
  };
  // preconditioner blocks: A_f (JACOBI) or A_f - sum_p B_pf B_pf' (SCHUR_JACOBI),
  // B_pf = sum of the W_o of point p seen by camera f
  std::vector<double> Minv((size_t)nf * 36, 0.0);
  {
    std::vector<double> blk(Af);
    if (opt.preconditioner_type == PC_SCHUR_JACOBI) {
      std::vector<int> fl;
      std::vector<double> Bs;
      for (int ip = 0; ip < npv; ++ip) {
        fl.clear();
        Bs.clear();
        for (int o : S.pt_obs[ip]) {
          if (P.type[o] != RB_ANGLE) continue;
          const int f = S.fidx[P.obs_cam[o]];
          int slot = -1;
          for (size_t q = 0; q < fl.size(); ++q) if (fl[q] == f) slot = (int)q;
          if (slot < 0) { slot = (int)fl.size(); fl.push_back(f); Bs.resize(Bs.size() + 18, 0.0); }
          for (int k = 0; k < 18; ++k) Bs[(size_t)slot * 18 + k] += W[(size_t)o * 18 + k];
        }
        for (size_t q = 0; q < fl.size(); ++q) {
          const double* B = &Bs[q * 18];
          double* M = &blk[(size_t)fl[q] * 36];
          for (int a = 0; a < 6; ++a)
            for (int c = 0; c < 6; ++c) M[a * 6 + c] -= B[a * 3] * B[c * 3] + B[a * 3 + 1] * B[c * 3 + 1] + B[a * 3 + 2] * B[c * 3 + 2];
        }
      }
    }
    for (int f = 0; f < nf; ++f)
      if (!llt_inverse(&blk[(size_t)f * 36], 6, &Minv[(size_t)f * 36]))
        for (int k = 0; k < 36; ++k) Minv[(size_t)f * 36 + k] = std::numeric_limits<double>::quiet_NaN();
  }
  std::vector<double> x(n, 0.0);
  if (!pcg_solve(rhs, schur_mul, Minv, nf, opt, x, cg_iterations)) return false;
  // back substitution (scaled space, the unrounded W), then the camera part
  for (int ip = 0; ip < npv; ++ip) {
    double w3[3] = {u[(size_t)ip * 3], u[(size_t)ip * 3 + 1], u[(size_t)ip * 3 + 2]};
    for (int o : S.pt_obs[ip]) {
      if (P.type[o] != RB_ANGLE) continue;
      const double* w = &W64[(size_t)o * 18];
      const double* xc = &x[6 * S.fidx[P.obs_cam[o]]];
      for (int k = 0; k < 3; ++k)
        for (int a = 0; a < 6; ++a) w3[k] -= w[a * 3 + k] * xc[a];
    }
    const double* M = &Linv[(size_t)ip * 9];
    const int pc = P.pt_col[P.var_pts[ip]];
    for (int a = 0; a < 3; ++a) y[pc + a] = M[a] * w3[0] + M[3 + a] * w3[1] + M[6 + a] * w3[2];   // L^-T w
  }
  for (int c : P.var_cams) for (int a = 0; a < 6; ++a) y[P.cam_col[c] + a] = x[6 * S.fidx[c] + a];
  for (double v : y) if (!std::isfinite(v)) return false;
  return true;
}

static bool linear_solve(const Problem& P, const Schur& S, const std::vector<Lin>& L, const std::vector<double>& s,
                         const std::vector<double>& D, const Options& opt, std::vector<double>& y, int* ls_iters) {
  *ls_iters = 1;
  if (opt.linear_solver == LS_ITERATIVE_SCHUR) {
    // precision 1: MIXED_FP32 (W in float); 2: the same W form in fp64 (test
    // hook: checks the W-form restatement against the F/E form above); 3:
    // MIXED_FP32 with the rank-2 records (c, Z in float) in the matvec
    if (opt.precision >= 1 && opt.precision <= 3) return iterative_schur_solve_w(P, S, L, s, D, opt, y, ls_iters);
    return iterative_schur_solve(P, S, L, s, D, opt, y, ls_iters);
  }
  return dense_schur_solve(P, S, L, s, D, y);
}

// ----------------------------------------------------------------------------
// Ceres TrustRegionMinimizer + LevenbergMarquardtStrategy restated.
// ----------------------------------------------------------------------------

enum { LOG_ITER = 0, LOG_COST, LOG_COST_CHANGE, LOG_GMAX, LOG_GNORM, LOG_STEP_NORM, LOG_REL_DEC,
       LOG_RADIUS, LOG_VALID, LOG_SUCCESS, LOG_MCC, LOG_LS_ITERS, LOG_WIDTH = 12 };
enum { TERM_CONVERGENCE = 0, TERM_NO_CONVERGENCE = 1, TERM_FAILURE = 2 };

struct Summary {
  double initial_cost, final_cost;
  int num_iterations, num_successful, num_unsuccessful, termination;
};

static double norm2(const std::vector<double>& v) { double s = 0; for (double a : v) s += a * a; return std::sqrt(s); }

static void prepare_schur(const Problem& P, Schur& S) {
  S.fidx.assign(P.nc, -1);
  S.nf = 0;
  for (int c : P.var_cams) S.fidx[c] = S.nf++;
  std::vector<int> vp(P.np, -1);
  for (size_t i = 0; i < P.var_pts.size(); ++i) vp[P.var_pts[i]] = (int)i;
  S.pt_obs.assign(P.var_pts.size(), {});
  for (int o = 0; o < P.no; ++o)
    if (P.type[o] == RB_ANGLE || P.type[o] == RB_POINT_ONLY) S.pt_obs[vp[P.obs_pt[o]]].push_back(o);
}

// model_cost_change = -(Js step)^T (r + Js step / 2), step = -y (scaled space)
static double model_cost_change(const Problem& P, const std::vector<Lin>& L, const std::vector<double>& scale,
                                const std::vector<double>& y) {
  double m = 0.0;
#pragma omp parallel for reduction(+ : m) schedule(static)
  for (int o = 0; o < P.no; ++o) {
    const int t = P.type[o];
    double js[2] = {0, 0};
    if (t == RB_ANGLE || t == RB_POSE_ONLY) {
      const int cc = P.cam_col[P.obs_cam[o]];
      for (int k = 0; k < 6; ++k) {
        const double st = -y[cc + k];
        js[0] += (L[o].Jc[k] * scale[cc + k]) * st;
        js[1] += (L[o].Jc[6 + k] * scale[cc + k]) * st;
      }
    }
    if (t == RB_ANGLE || t == RB_POINT_ONLY) {
      const int pc = P.pt_col[P.obs_pt[o]];
      for (int k = 0; k < 3; ++k) {
        const double st = -y[pc + k];
        js[0] += (L[o].Jp[k] * scale[pc + k]) * st;
        js[1] += (L[o].Jp[3 + k] * scale[pc + k]) * st;
      }
    }
    m += js[0] * (L[o].r[0] + js[0] / 2.0) + js[1] * (L[o].r[1] + js[1] / 2.0);
  }
  return -m;
}

// CPU baseline timing: the same per-iteration work as the GPU bench step
// (linearise + gradient/column norms + LM diagonal + DENSE_SCHUR solve +
// model cost change + candidate cost) at a fixed trust-region radius.
static double bench_iteration_seconds(Problem& P, int iters, double radius) {
  build_structure(P);
  Schur S;
  prepare_schur(P, S);
  const int n = P.ncols;
  std::vector<double> x, g, cn, scale(n, 1.0), D(n), y, cand(n);
  std::vector<Lin> L;
  gather_x(P, x);
  double cost;
  eval_lin(P, x, L, &cost);
  gradient_colnorm(P, L, g, cn);
  for (int i = 0; i < n; ++i) scale[i] = 1.0 / (1.0 + std::sqrt(cn[i]));
  const auto t0 = std::chrono::steady_clock::now();
  for (int it = 0; it < iters; ++it) {
    eval_lin(P, x, L, &cost);
    gradient_colnorm(P, L, g, cn);
    for (int i = 0; i < n; ++i) {
      const double d = std::min(std::max(cn[i] * scale[i] * scale[i], 1e-6), 1e32);
      D[i] = std::sqrt(d / radius);
    }
    dense_schur_solve(P, S, L, scale, D, y);
    volatile double mcc = model_cost_change(P, L, scale, y);
    (void)mcc;
    for (int i = 0; i < n; ++i) cand[i] = x[i] + (-y[i]) * scale[i];
    double cc;
    eval_cost(P, cand, &cc);
  }
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / iters;
}

static int minimize(Problem& P, const Options& opt, double* log, int max_log, Summary* sum) {
  build_structure(P);
  Schur S;
  prepare_schur(P, S);
  const int n = P.ncols;
  std::vector<double> x, cand, g, cn, scale(n, 1.0), diag(n, 0.0), D(n), y, delta(n);
  std::vector<Lin> L;
  gather_x(P, x);
  int nlog = 0;
  auto push_log = [&](const double* rec) {
    if (log && nlog < max_log) std::memcpy(log + (size_t)nlog * LOG_WIDTH, rec, sizeof(double) * LOG_WIDTH);
    ++nlog;
  };
  sum->num_successful = sum->num_unsuccessful = 0;
  double x_cost;
  if (n == 0) {  // nothing to optimise (ceres: no non-constant parameter blocks)
    eval_cost(P, x, &x_cost);
    sum->initial_cost = sum->final_cost = x_cost;
    sum->termination = TERM_CONVERGENCE;
    sum->num_iterations = 0;
    return 0;
  }
  double x_norm = norm2(x);
  double radius = opt.initial_trust_region_radius, decrease_factor = 2.0;
  bool reuse_diagonal = false;
  int consecutive_invalid = 0;

  // ---- EvaluateGradientAndJacobian
  auto evaluate_gj = [&](int iteration, double* gmax, double* gnorm) -> bool {
    if (!eval_lin(P, x, L, &x_cost)) return false;
    gradient_colnorm(P, L, g, cn);
    double gm = 0, gn = 0;
    for (int i = 0; i < n; ++i) {
      const double pg = x[i] + (-g[i]);  // Plus(x, -gradient)
      const double d = x[i] - pg;
      gm = std::max(gm, std::fabs(d));
      gn += d * d;
    }
    *gmax = gm; *gnorm = std::sqrt(gn);
    if (opt.jacobi_scaling) {
      if (iteration == 0)
        for (int i = 0; i < n; ++i) scale[i] = 1.0 / (1.0 + std::sqrt(cn[i]));
    }
    return true;
  };

  double rec[LOG_WIDTH];
  std::memset(rec, 0, sizeof rec);
  double gmax = 0, gnorm = 0;
  if (!evaluate_gj(0, &gmax, &gnorm)) {
    sum->termination = TERM_FAILURE;
    sum->initial_cost = sum->final_cost = x_cost;
    sum->num_iterations = 0;
    return 0;
  }
  sum->initial_cost = x_cost;
  double min_cost = x_cost;
  rec[LOG_ITER] = 0; rec[LOG_COST] = x_cost; rec[LOG_GMAX] = gmax; rec[LOG_GNORM] = gnorm;
  rec[LOG_RADIUS] = radius; rec[LOG_VALID] = 1; rec[LOG_SUCCESS] = 1;
  push_log(rec);
  int iteration = 0;
  int termination = TERM_NO_CONVERGENCE;
  bool last_success = true;
  // FinalizeIterationAndCheckIfMinimizerCanContinue for iteration 0
  auto can_continue = [&](double cur_gmax) -> bool {
    if (iteration >= opt.max_num_iterations) { termination = TERM_NO_CONVERGENCE; return false; }
    if (last_success && cur_gmax <= opt.gradient_tolerance) { termination = TERM_CONVERGENCE; return false; }
    if (radius <= opt.min_trust_region_radius) { termination = TERM_CONVERGENCE; return false; }
    return true;
  };
  double cur_gmax = gmax, cur_gnorm = gnorm;
  while (can_continue(cur_gmax)) {
    ++iteration;
    std::memset(rec, 0, sizeof rec);
    rec[LOG_ITER] = iteration;
    // ---- LevenbergMarquardtStrategy::ComputeStep
    if (!reuse_diagonal) {
      for (int i = 0; i < n; ++i) {
        const double sc = scale[i];
        diag[i] = std::min(std::max(cn[i] * sc * sc, opt.min_lm_diagonal), opt.max_lm_diagonal);
      }
    }
    for (int i = 0; i < n; ++i) D[i] = std::sqrt(diag[i] / radius);
    int ls_iters = 0;
    bool solved = linear_solve(P, S, L, scale, D, opt, y, &ls_iters);
    rec[LOG_LS_ITERS] = ls_iters;
    reuse_diagonal = true;
    bool valid = false;
    double mcc = 0.0;
    if (solved) {
      mcc = model_cost_change(P, L, scale, y);
      valid = mcc > 0.0;
      if (valid) for (int i = 0; i < n; ++i) delta[i] = (-y[i]) * scale[i];
    }
    rec[LOG_MCC] = mcc;
    if (!valid) {
      // HandleInvalidStep
      if (++consecutive_invalid >= opt.max_num_consecutive_invalid_steps) { termination = TERM_FAILURE; break; }
      radius = radius / decrease_factor; decrease_factor *= 2.0; reuse_diagonal = true;  // StepRejected(0)
      rec[LOG_COST] = x_cost; rec[LOG_GMAX] = cur_gmax; rec[LOG_GNORM] = cur_gnorm;
      rec[LOG_RADIUS] = radius; rec[LOG_VALID] = 0; rec[LOG_SUCCESS] = 0;
      last_success = false;
      sum->num_unsuccessful++;
      push_log(rec);
      continue;
    }
    consecutive_invalid = 0;
    // ComputeCandidatePointAndEvaluateCost
    cand.resize(n);
    for (int i = 0; i < n; ++i) cand[i] = x[i] + delta[i];
    double cand_cost;
    if (!eval_cost(P, cand, &cand_cost)) cand_cost = std::numeric_limits<double>::max();
    // ParameterToleranceReached
    double sn = 0;
    for (int i = 0; i < n; ++i) { const double d = x[i] - cand[i]; sn += d * d; }
    const double step_norm = std::sqrt(sn);
    rec[LOG_STEP_NORM] = step_norm;
    if (step_norm <= opt.parameter_tolerance * (x_norm + opt.parameter_tolerance)) {
      termination = TERM_CONVERGENCE; break;
    }
    // FunctionToleranceReached
    const double cost_change = x_cost - cand_cost;
    rec[LOG_COST_CHANGE] = cost_change;
    if (std::fabs(cost_change) <= opt.function_tolerance * x_cost) { termination = TERM_CONVERGENCE; break; }
    // IsStepSuccessful (monotonic TrustRegionStepEvaluator::StepQuality)
    const double rel = cand_cost >= std::numeric_limits<double>::max()
                           ? std::numeric_limits<double>::lowest()
                           : (x_cost - cand_cost) / mcc;
    rec[LOG_REL_DEC] = rel;
    if (rel > opt.min_relative_decrease) {
      // HandleSuccessfulStep
      x = cand;
      x_norm = norm2(x);
      if (!evaluate_gj(iteration, &cur_gmax, &cur_gnorm)) { termination = TERM_FAILURE; break; }
      radius = std::min(opt.max_trust_region_radius,
                        radius / std::max(1.0 / 3.0, 1.0 - std::pow(2.0 * rel - 1.0, 3)));
      decrease_factor = 2.0;
      reuse_diagonal = false;
      last_success = true;
      if (x_cost < min_cost) min_cost = x_cost;
      sum->num_successful++;
      rec[LOG_COST] = x_cost; rec[LOG_SUCCESS] = 1;
    } else {
      radius = radius / decrease_factor; decrease_factor *= 2.0; reuse_diagonal = true;
      last_success = false;
      sum->num_unsuccessful++;
      rec[LOG_COST] = cand_cost; rec[LOG_SUCCESS] = 0;
    }
    rec[LOG_GMAX] = cur_gmax; rec[LOG_GNORM] = cur_gnorm; rec[LOG_RADIUS] = radius; rec[LOG_VALID] = 1;
    push_log(rec);
  }
  scatter_x(P, x);
  sum->final_cost = x_cost;
  sum->termination = termination;
  sum->num_iterations = iteration;
  return nlog;
}

}  // namespace oracle

// ============================================================================
// C entry points for ctypes (tests / bench cpu_baseline only).
// ============================================================================
extern "C" {

typedef struct {
  int32_t n_cams, n_pts, n_obs, pad;
  double* cams;
  const uint8_t* cam_fixed;
  const float* cam_fixed_extr;
  const float* K;
  double* pts;
  const uint8_t* pt_fixed;
  const int32_t* obs_cam;
  const int32_t* obs_pt;
  const float* obs_uv;
  double huber_a;
} oracle_problem;

static oracle::Problem to_problem(const oracle_problem* p) {
  oracle::Problem P;
  P.nc = p->n_cams; P.np = p->n_pts; P.no = p->n_obs;
  P.cams = p->cams; P.cam_fixed = p->cam_fixed; P.cam_extr = p->cam_fixed_extr; P.K = p->K;
  P.pts = p->pts; P.pt_fixed = p->pt_fixed; P.obs_cam = p->obs_cam; P.obs_pt = p->obs_pt;
  P.obs_uv = p->obs_uv; P.huber_a = p->huber_a;
  return P;
}

void oracle_set_threads(int n) {
#ifdef _OPENMP
  if (n > 0) omp_set_num_threads(n);
#else
  (void)n;
#endif
}

// Levenberg-Marquardt + DENSE_SCHUR solve in place.  iter_log: [max_log][12].
// summary: [initial_cost, final_cost, num_iterations, num_successful,
//           num_unsuccessful, termination].  Returns number of log records.
int oracle_solve(const oracle_problem* prob, const oracle::Options* opt, double* iter_log, int max_log,
                 double* summary) {
  oracle::Problem P = to_problem(prob);
  oracle::Summary s{};
  int nlog = oracle::minimize(P, *opt, iter_log, max_log, &s);
  summary[0] = s.initial_cost; summary[1] = s.final_cost; summary[2] = s.num_iterations;
  summary[3] = s.num_successful; summary[4] = s.num_unsuccessful; summary[5] = s.termination;
  return nlog;
}

// Corrected residuals r[2N], jacobian J[N][2][9] (cam 6 | point 3, zeros for
// constant blocks) and total cost at the given parameters.
int oracle_linearize(const oracle_problem* prob, double* r, double* J, double* cost) {
  oracle::Problem P = to_problem(prob);
  oracle::build_structure(P);
  std::vector<double> x;
  oracle::gather_x(P, x);
  std::vector<oracle::Lin> L;
  bool ok = oracle::eval_lin(P, x, L, cost);
  for (int o = 0; o < P.no; ++o) {
    r[2 * o] = L[o].r[0]; r[2 * o + 1] = L[o].r[1];
    for (int i = 0; i < 2; ++i) {
      for (int k = 0; k < 6; ++k) J[(size_t)o * 18 + i * 9 + k] = L[o].Jc[i * 6 + k];
      for (int k = 0; k < 3; ++k) J[(size_t)o * 18 + i * 9 + 6 + k] = L[o].Jp[i * 3 + k];
    }
  }
  return ok ? 0 : 1;
}

// Raw (uncorrected) residuals of the functors.
void oracle_residuals(const oracle_problem* prob, double* r) {
  oracle::Problem P = to_problem(prob);
  oracle::build_structure(P);
  for (int o = 0; o < P.no; ++o) {
    const int c = P.obs_cam[o], p = P.obs_pt[o];
    const float u = P.obs_uv[2 * o], v = P.obs_uv[2 * o + 1];
    if (P.cam_fixed && P.cam_fixed[c]) {
      oracle::point_only_reprojection(P.pts + 3 * p, P.cam_extr + 16 * c, P.K + 9 * c, u, v, r + 2 * o);
    } else {
      oracle::angle_reprojection(P.cams + 6 * c, P.pts + 3 * p, P.K + 9 * c, u, v, r + 2 * o);
    }
  }
}

// Seconds per LM iteration (CPU baseline; same work as ba_bench_iterations).
double oracle_bench(const oracle_problem* prob, int iters, double radius) {
  oracle::Problem P = to_problem(prob);
  return oracle::bench_iteration_seconds(P, iters, radius);
}

int oracle_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

void oracle_angle_axis_to_R(const double* aa, double* R) { oracle::AngleAxisToRotationMatrix(aa, R); }
void oracle_R_to_angle_axis(const double* R, double* aa) { oracle::RotationMatrixToAngleAxis(R, aa); }

void oracle_angle_axis_to_R_jac(const double* aa, double* R, double* dR /*[3][9]*/) {
  oracle::Jet<3> a[3], Rj[9];
  for (int k = 0; k < 3; ++k) a[k] = oracle::Jet<3>(aa[k], k);
  oracle::AngleAxisToRotationMatrix(a, Rj);
  for (int i = 0; i < 9; ++i) { R[i] = Rj[i].a; for (int k = 0; k < 3; ++k) dR[k * 9 + i] = Rj[i].v[k]; }
}

// pruneCorrespondences restated (Optimizer.cpp:6-79), float arithmetic in the
// operation order documented for ba_prune in include/ba_hip.h (column-wise
// matrix-vector accumulation, sqrt((x*x + y*y) + z*z), no contraction: this
// file is built with -ffp-contract=off).  result: 0 inlier, 1 behind the
// camera (:36-41), 2 outside the depth range (:43-51), 3 chi test (:53-64).
void oracle_prune(int n_obs, const float* extr, const float* center, const float* K, const int32_t* obs_cam,
                  const float* X, const float* uv, const float* inv_sigma, const float* dist, uint8_t* result) {
  for (int o = 0; o < n_obs; ++o) {
    const int c = obs_cam[o];
    const float* e = extr + 16 * c;
    const float x0 = X[3 * o], x1 = X[3 * o + 1], x2 = X[3 * o + 2];
    float v[4];
    for (int i = 0; i < 4; ++i) v[i] = ((e[i] * x0 + e[4 + i] * x1) + e[8 + i] * x2) + e[12 + i];
    const float cam[3] = {v[0] / v[3], v[1] / v[3], v[2] / v[3]};
    if (cam[2] <= 0.0f) { result[o] = 1; continue; }
    const float* ctr = center + 3 * c;
    const float d0 = x0 - ctr[0], d1 = x1 - ctr[1], d2 = x2 - ctr[2];
    const float wd = std::sqrt((d0 * d0 + d1 * d1) + d2 * d2);
    if (wd > dist[2 * o + 1] || wd < dist[2 * o]) { result[o] = 2; continue; }
    const float* k = K + 9 * c;
    float q[3];
    for (int i = 0; i < 3; ++i) q[i] = (k[i] * cam[0] + k[3 + i] * cam[1]) + k[6 + i] * cam[2];
    const float e0 = q[0] / q[2] - uv[2 * o], e1 = q[1] / q[2] - uv[2 * o + 1];
    const float nrm = std::sqrt(e0 * e0 + e1 * e1);
    const float chi = nrm * inv_sigma[o];
    const float thresh = 5.991;
    result[o] = chi > thresh ? 3 : 0;
  }
}

// Column norms^2 of the (corrected) camera jacobian, [6*n_cams] (zero for
// constant / unobserved cameras).  Additive over point shards.
void oracle_camera_colnorm2(const oracle_problem* prob, double* out) {
  oracle::Problem P = to_problem(prob);
  oracle::build_structure(P);
  std::vector<double> x, g, cn;
  oracle::gather_x(P, x);
  std::vector<oracle::Lin> L;
  double cost;
  oracle::eval_lin(P, x, L, &cost);
  oracle::gradient_colnorm(P, L, g, cn);
  for (int c = 0; c < P.nc; ++c)
    for (int k = 0; k < 6; ++k) out[6 * c + k] = P.cam_col[c] >= 0 ? cn[P.cam_col[c] + k] : 0.0;
}

// Reduced camera system of one LM step at `radius` (Jacobi scaling and LM
// diagonal as at iteration 0).  cam_colnorm2 [6*n_cams]: the camera column
// norms to scale with (the global ones for a point shard; NULL = this
// problem's own).  add_cam_D: add the camera LM diagonal (once over shards).
// lhs: [n*n] row-major, lower triangle; rhs: [n].  Returns n = 6 x variable
// cameras, or -1 on failure.  The distributed test checks that the sum over
// point shards equals the unsharded system: the property the RCCL path uses.
int oracle_reduced_system(const oracle_problem* prob, const double* cam_colnorm2, double radius, int add_cam_D,
                          double* lhs_out, double* rhs_out) {
  oracle::Problem P = to_problem(prob);
  oracle::build_structure(P);
  std::vector<double> x, g, cn;
  oracle::gather_x(P, x);
  std::vector<oracle::Lin> L;
  double cost;
  if (!oracle::eval_lin(P, x, L, &cost)) return -1;
  oracle::gradient_colnorm(P, L, g, cn);
  if (cam_colnorm2)
    for (int c = 0; c < P.nc; ++c)
      if (P.cam_col[c] >= 0)
        for (int k = 0; k < 6; ++k) cn[P.cam_col[c] + k] = cam_colnorm2[6 * c + k];
  const int ncol = P.ncols;
  std::vector<double> s(ncol), D(ncol);
  for (int i = 0; i < ncol; ++i) {
    s[i] = 1.0 / (1.0 + std::sqrt(cn[i]));
    const double d = std::min(std::max(cn[i] * s[i] * s[i], 1e-6), 1e32);
    D[i] = std::sqrt(d / radius);
  }
  oracle::Schur S;
  oracle::prepare_schur(P, S);
  std::vector<double> lhs, rhs, ete_inv, ge;
  if (!oracle::assemble_schur(P, S, L, s, D, add_cam_D != 0, lhs, rhs, ete_inv, ge)) return -1;
  const int n = 6 * S.nf;
  std::copy(lhs.begin(), lhs.end(), lhs_out);
  std::copy(rhs.begin(), rhs.end(), rhs_out);
  return n;
}

void oracle_default_options(oracle::Options* o) {
  o->max_num_iterations = 50;
  o->max_num_consecutive_invalid_steps = 5;
  o->jacobi_scaling = 1;
  o->linear_solver = 0;
  o->preconditioner_type = 0;
  o->max_linear_solver_iterations = 500;
  o->min_linear_solver_iterations = 0;
  o->precision = 0;
  o->eta = 1e-1;
  o->function_tolerance = 1e-6;
  o->gradient_tolerance = 1e-10;
  o->parameter_tolerance = 1e-8;
  o->initial_trust_region_radius = 1e4;
  o->max_trust_region_radius = 1e16;
  o->min_trust_region_radius = 1e-32;
  o->min_relative_decrease = 1e-3;
  o->min_lm_diagonal = 1e-6;
  o->max_lm_diagonal = 1e32;
}

}  // extern "C"

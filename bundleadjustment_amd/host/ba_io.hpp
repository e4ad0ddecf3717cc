// ba_io.hpp — problem exchange in C++, byte-compatible
// with bundleadjustment_amd/io.py:
//   * BAS dump: the ba_problem arrays of include/ba_hip.h, little-endian
//     (magic "BASOA\0\0\1"; int32 C, P, N, flags; f64 huber_a; cams f64[6C],
//     K f32[9C], [cam_fixed u8[C], extr f32[16C]], pts f64[3P], [pt_fixed
//     u8[P]], obs_cam i32[N], obs_pt i32[N], obs_uv f32[2N]).  Lossless, so a
//     problem gathered by prepareConstraints (Optimizer.cpp:279-333) can be
//     replayed through ceres::Solve on a Ceres-equipped host and through
//     ba_solve here on the same inputs.
//   * BAL text reader: angle-axis + t carried over unchanged, K = diag(-f, -f, 1)
//     (BAL's p = -P / P_z; the reference's functor has no distortion, so
//     cameras with k1/k2 != 0 are refused unless ignore_distortion).
// Header-only, no dependency beyond the C++17 standard library.
#pragma once

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "ba_hip.h"

namespace ba_amd {

// Owning SoA problem; view() gives the ba_problem the C ABI takes.
struct ProblemData {
  int32_t n_cams = 0, n_pts = 0, n_obs = 0;
  double huber_a = 0.0;
  std::vector<double> cams, pts;
  std::vector<float> K, cam_fixed_extr, obs_uv;
  std::vector<uint8_t> cam_fixed, pt_fixed;      // empty = none fixed
  std::vector<int32_t> obs_cam, obs_pt;

  ba_problem view() const {
    ba_problem p{};
    p.n_cams = n_cams; p.n_pts = n_pts; p.n_obs = n_obs;
    p.cams = cams.data(); p.K = K.data(); p.pts = pts.data();
    p.cam_fixed = cam_fixed.empty() ? nullptr : cam_fixed.data();
    p.cam_fixed_extr = cam_fixed_extr.empty() ? nullptr : cam_fixed_extr.data();
    p.pt_fixed = pt_fixed.empty() ? nullptr : pt_fixed.data();
    p.obs_cam = obs_cam.data(); p.obs_pt = obs_pt.data(); p.obs_uv = obs_uv.data();
    p.huber_a = huber_a;
    return p;
  }
};

namespace detail {
inline const char kBasMagic[8] = {'B', 'A', 'S', 'O', 'A', '\0', '\0', '\1'};
static_assert(sizeof(float) == 4 && sizeof(double) == 8, "IEEE types");

template <class T>
void put(std::ofstream& f, const std::vector<T>& v) {
  f.write(reinterpret_cast<const char*>(v.data()), static_cast<std::streamsize>(v.size() * sizeof(T)));
}
template <class T>
void get(std::ifstream& f, std::vector<T>& v, size_t n, const std::string& path) {
  v.resize(n);
  f.read(reinterpret_cast<char*>(v.data()), static_cast<std::streamsize>(n * sizeof(T)));
  if (!f) throw std::runtime_error(path + ": truncated BAS dump");
}
inline void check_indices(const ProblemData& p, const std::string& where) {
  for (int32_t o = 0; o < p.n_obs; ++o)
    if (p.obs_cam[o] < 0 || p.obs_cam[o] >= p.n_cams || p.obs_pt[o] < 0 || p.obs_pt[o] >= p.n_pts)
      throw std::runtime_error(where + ": observation index out of range");
}
}  // namespace detail

inline void save_problem(const std::string& path, const ProblemData& p) {
  std::ofstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error(path + ": cannot open for writing");
  const int32_t flags = (p.cam_fixed.empty() ? 0 : 1) | (p.pt_fixed.empty() ? 0 : 2);
  const int32_t hdr[4] = {p.n_cams, p.n_pts, p.n_obs, flags};
  f.write(detail::kBasMagic, 8);
  f.write(reinterpret_cast<const char*>(hdr), sizeof(hdr));
  f.write(reinterpret_cast<const char*>(&p.huber_a), sizeof(double));
  detail::put(f, p.cams);
  detail::put(f, p.K);
  if (flags & 1) {
    detail::put(f, p.cam_fixed);
    std::vector<float> extr = p.cam_fixed_extr;
    extr.resize(static_cast<size_t>(16) * p.n_cams, 0.0f);
    detail::put(f, extr);
  }
  detail::put(f, p.pts);
  if (flags & 2) detail::put(f, p.pt_fixed);
  detail::put(f, p.obs_cam);
  detail::put(f, p.obs_pt);
  detail::put(f, p.obs_uv);
  if (!f) throw std::runtime_error(path + ": write failed");
}

inline ProblemData load_problem(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error(path + ": cannot open");
  char magic[8];
  int32_t hdr[4];
  ProblemData p;
  f.read(magic, 8);
  f.read(reinterpret_cast<char*>(hdr), sizeof(hdr));
  f.read(reinterpret_cast<char*>(&p.huber_a), sizeof(double));
  if (!f || std::memcmp(magic, detail::kBasMagic, 8) != 0) throw std::runtime_error(path + ": not a BAS dump");
  p.n_cams = hdr[0]; p.n_pts = hdr[1]; p.n_obs = hdr[2];
  if (p.n_cams < 0 || p.n_pts < 0 || p.n_obs < 0) throw std::runtime_error(path + ": negative sizes");
  const size_t C = p.n_cams, P = p.n_pts, N = p.n_obs;
  detail::get(f, p.cams, 6 * C, path);
  detail::get(f, p.K, 9 * C, path);
  if (hdr[3] & 1) {
    detail::get(f, p.cam_fixed, C, path);
    detail::get(f, p.cam_fixed_extr, 16 * C, path);
  }
  detail::get(f, p.pts, 3 * P, path);
  if (hdr[3] & 2) detail::get(f, p.pt_fixed, P, path);
  detail::get(f, p.obs_cam, N, path);
  detail::get(f, p.obs_pt, N, path);
  detail::get(f, p.obs_uv, 2 * N, path);
  if (f.peek() != std::char_traits<char>::eof()) throw std::runtime_error(path + ": trailing bytes");
  detail::check_indices(p, path);
  return p;
}

// BAL text (uncompressed).  Observations stay float (the reference keeps
// keypoints as cv::KeyPoint floats, Optimizer.h:54-76 takes Vector2f).
inline ProblemData read_bal(const std::string& path, double huber_a, bool ignore_distortion = false) {
  FILE* f = std::fopen(path.c_str(), "r");
  if (!f) throw std::runtime_error(path + ": cannot open");
  ProblemData p;
  p.huber_a = huber_a;
  auto fail = [&](const char* what) {
    std::fclose(f);
    throw std::runtime_error(path + ": " + what);
  };
  if (std::fscanf(f, "%d %d %d", &p.n_cams, &p.n_pts, &p.n_obs) != 3 || p.n_cams < 0 || p.n_pts < 0 || p.n_obs < 0)
    fail("bad BAL header");
  const size_t C = p.n_cams, P = p.n_pts, N = p.n_obs;
  p.obs_cam.resize(N); p.obs_pt.resize(N); p.obs_uv.resize(2 * N);
  for (size_t o = 0; o < N; ++o) {
    double u, v;
    if (std::fscanf(f, "%d %d %lf %lf", &p.obs_cam[o], &p.obs_pt[o], &u, &v) != 4) fail("truncated observations");
    p.obs_uv[2 * o] = static_cast<float>(u);
    p.obs_uv[2 * o + 1] = static_cast<float>(v);
  }
  p.cams.resize(6 * C);
  p.K.assign(9 * C, 0.0f);
  for (size_t c = 0; c < C; ++c) {
    double v[9];
    for (double& x : v)
      if (std::fscanf(f, "%lf", &x) != 1) fail("truncated cameras");
    if ((v[7] != 0.0 || v[8] != 0.0) && !ignore_distortion) fail("camera with radial distortion (model has none)");
    for (int k = 0; k < 6; ++k) p.cams[6 * c + k] = v[k];
    p.K[9 * c + 0] = static_cast<float>(-v[6]);
    p.K[9 * c + 4] = static_cast<float>(-v[6]);
    p.K[9 * c + 8] = 1.0f;
  }
  p.pts.resize(3 * P);
  for (double& x : p.pts)
    if (std::fscanf(f, "%lf", &x) != 1) fail("truncated points");
  std::fclose(f);
  detail::check_indices(p, path);
  return p;
}

}  // namespace ba_amd

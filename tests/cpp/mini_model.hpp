// mini_model.hpp — a minimal stand-in for the reference's model classes
// (ba_project/src/model: Frame, MapPoint, SceneMap) with the accessors the
// optimizer shim uses, plus a seeded synthetic scene.  Test code only.
#pragma once

#include <algorithm>
#include <cmath>
#include <map>
#include <memory>
#include <random>
#include <utility>
#include <vector>

#include "ba_geometry.hpp"

namespace mini {

using ba_amd::Mat3f;
using ba_amd::Mat4f;
using ba_amd::Vec2f;
using ba_amd::Vec3f;

struct MapPoint;

struct Frame {
  int id = 0;
  bool keyframe = true;
  Mat4f pose;                                   // camera -> world (Frame::getPose)
  Mat3f K;
  std::vector<Vec2f> kp;                        // keypoint positions
  std::vector<int> octave;
  std::vector<std::shared_ptr<MapPoint>> mps;   // per keypoint (may be null)
  std::vector<bool> outlier;
};

struct MapPoint {
  Vec3f X;
  float min_dist = 0, max_dist = 0;
  bool invalid = false;
  std::map<std::shared_ptr<Frame>, size_t> obs; // observing keyframes -> keypoint index
};

struct Scene {
  std::vector<std::shared_ptr<Frame>> frames;
  std::vector<std::shared_ptr<MapPoint>> points;
  int erase_calls = 0;
  Scene() = default;
  Scene(Scene&&) = default;
  Scene& operator=(Scene&&) = default;
  // frames and points own each other (Frame::mps <-> MapPoint::obs, as the
  // reference's model does): break the cycles so the scene is freed (the
  // ASan build's leak check, tests/cpp `make sanitize`)
  ~Scene() {
    for (auto& f : frames) if (f) f->mps.clear();
    for (auto& p : points) if (p) p->obs.clear();
  }
};

struct Model {
  using Map = Scene;
  using FramePtr = std::shared_ptr<Frame>;
  using PointPtr = std::shared_ptr<MapPoint>;
  static std::vector<FramePtr> key_frames(Map* m) { return m->frames; }
  static std::vector<PointPtr> map_points(Map* m) { return m->points; }
  static std::vector<PointPtr> frame_map_points(const FramePtr& f) { return f->mps; }
  static PointPtr frame_map_point(const FramePtr& f, int i) { return f->mps[i]; }
  static int keypoint_count(const FramePtr& f) { return static_cast<int>(f->kp.size()); }
  static Vec2f keypoint_pt(const FramePtr& f, int i) { return f->kp[i]; }
  static int keypoint_octave(const FramePtr& f, int i) { return f->octave[i]; }
  static bool is_outlier(const FramePtr& f, int i) { return f->outlier[i]; }
  static void set_outlier(const FramePtr& f, int i, bool o) { f->outlier[i] = o; }
  static int id(const FramePtr& f) { return f->id; }
  static bool is_key_frame(const FramePtr& f) { return f->keyframe; }
  static Mat4f pose(const FramePtr& f) { return f->pose; }
  static void set_pose(const FramePtr& f, const Mat4f& p) { f->pose = p; }
  static Mat3f intrinsics(const FramePtr& f) { return f->K; }
  static std::vector<FramePtr> best_covisibility_frames(const FramePtr& f, int n) {
    // frames sharing the most map points with f (ties by id), as Frame::getBestCovisibilityFrames
    std::map<Frame*, std::pair<int, FramePtr>> cnt;
    for (const auto& mp : f->mps)
      if (mp)
        for (const auto& ob : mp->obs)
          if (ob.first.get() != f.get()) { auto& e = cnt[ob.first.get()]; e.first++; e.second = ob.first; }
    std::vector<std::pair<int, FramePtr>> v;
    for (auto& e : cnt) v.push_back(e.second);
    std::sort(v.begin(), v.end(), [](const auto& a, const auto& b) {
      return a.first != b.first ? a.first > b.first : a.second->id < b.second->id;
    });
    std::vector<FramePtr> out;
    for (int i = 0; i < (int)v.size() && i < n; ++i) out.push_back(v[i].second);
    return out;
  }
  static Vec3f position(const PointPtr& p) { return p->X; }
  static void set_position(const PointPtr& p, const Vec3f& X) { p->X = X; }
  static Vec2f keypoint_of(const PointPtr& p, const FramePtr& f) { return f->kp[p->obs.at(f)]; }
  static float min_distance(const PointPtr& p) { return p->min_dist; }
  static float max_distance(const PointPtr& p) { return p->max_dist; }
  static bool is_invalid(const PointPtr& p) { return p->invalid; }
  static std::vector<std::pair<FramePtr, size_t>> observing_keyframes(const PointPtr& p) {
    return std::vector<std::pair<FramePtr, size_t>>(p->obs.begin(), p->obs.end());
  }
  static void erase_outliers(Map* m, int) { m->erase_calls++; }
};

// Seeded synthetic scene: n_frames keyframes on an arc looking at a cloud of
// n_points points; every point is seen by the frames where it projects into
// the 640x480 image; keypoints carry 0.7 px noise, 4 % gross outliers, random
// octaves; min/max distances as in MapPoint's constructor (MapPoint.cpp:15-22).
inline Scene make_scene(int n_frames, int n_points, unsigned seed) {
  std::mt19937 rng(seed);
  std::normal_distribution<double> N01(0.0, 1.0);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  Scene s;
  std::vector<Mat4f> truth;   // unperturbed poses: the keypoints are generated from these
  Mat3f K;
  K.m[0] = 525.0f; K.m[4] = 525.0f; K.m[6] = 319.5f; K.m[7] = 239.5f; K.m[8] = 1.0f;
  for (int f = 0; f < n_frames; ++f) {
    auto fr = std::make_shared<Frame>();
    fr->id = f;
    fr->K = K;
    // camera centre on an arc, looking at the origin (+z forward)
    const double a = -0.6 + 1.2 * f / std::max(1, n_frames - 1);
    const double C[3] = {4.0 * std::sin(a), 0.3 * std::sin(3.0 * a), -4.0 * std::cos(a)};
    double z[3] = {-C[0], -C[1], -C[2]};
    const double zn = std::sqrt(z[0] * z[0] + z[1] * z[1] + z[2] * z[2]);
    for (double& v : z) v /= zn;
    double x[3] = {z[2], 0.0, -z[0]};                       // up = y
    const double xn = std::sqrt(x[0] * x[0] + x[2] * x[2]);
    x[0] /= xn; x[2] /= xn;
    const double y[3] = {z[1] * x[2] - z[2] * x[1], z[2] * x[0] - z[0] * x[2], z[0] * x[1] - z[1] * x[0]};
    Mat4f P = ba_amd::identity4();                          // camera -> world: columns x, y, z, C
    for (int r = 0; r < 3; ++r) {
      P.m[0 + r] = (float)x[r]; P.m[4 + r] = (float)y[r]; P.m[8 + r] = (float)z[r]; P.m[12 + r] = (float)C[r];
    }
    truth.push_back(P);
    if (f > 0) {  // perturb the estimate (not keyframe 0: the world anchor)
      for (int r = 0; r < 3; ++r) P.m[12 + r] += (float)(0.03 * N01(rng));
    }
    fr->pose = P;
    s.frames.push_back(fr);
  }
  const float maxScale = std::pow(1.2f, 7);
  for (int p = 0; p < n_points; ++p) {
    double X[3];
    do { for (double& v : X) v = 2.0 * U(rng) - 1.0; } while (X[0] * X[0] + X[1] * X[1] + X[2] * X[2] > 1.0);
    auto mp = std::make_shared<MapPoint>();
    for (int r = 0; r < 3; ++r) mp->X.v[r] = (float)(1.5 * X[r] + 0.02 * N01(rng));
    int seen = 0;
    for (size_t fi = 0; fi < s.frames.size(); ++fi) {
      auto& fr = s.frames[fi];
      const Mat4f e = ba_amd::inverse4(truth[fi]);
      double pc[3];
      for (int r = 0; r < 3; ++r) pc[r] = e.m[r] * 1.5 * X[0] + e.m[4 + r] * 1.5 * X[1] + e.m[8 + r] * 1.5 * X[2] + e.m[12 + r];
      if (pc[2] <= 0.1) continue;
      const double u = 525.0 * pc[0] / pc[2] + 319.5, v = 525.0 * pc[1] / pc[2] + 239.5;
      if (u < 0 || u >= 640 || v < 0 || v >= 480) continue;
      const bool gross = U(rng) < 0.04;
      Vec2f kp;
      kp.x = (float)(gross ? 640.0 * U(rng) : u + 0.7 * N01(rng));
      kp.y = (float)(gross ? 480.0 * U(rng) : v + 0.7 * N01(rng));
      const int idx = (int)fr->kp.size();
      fr->kp.push_back(kp);
      fr->octave.push_back((int)(U(rng) * 4));
      fr->mps.push_back(mp);
      fr->outlier.push_back(false);
      mp->obs.emplace(fr, idx);
      if (seen == 0) {
        const double d0 = mp->X[0] - fr->pose.m[12], d1 = mp->X[1] - fr->pose.m[13], d2 = mp->X[2] - fr->pose.m[14];
        mp->max_dist = (float)std::sqrt(d0 * d0 + d1 * d1 + d2 * d2) * std::pow(1.2f, fr->octave.back()) * 1.5f;
        mp->min_dist = mp->max_dist / maxScale;
      }
      ++seen;
    }
    // unmatched keypoints (no map point) in every frame
    s.points.push_back(mp);
  }
  for (auto& fr : s.frames)
    for (int k = 0; k < 5; ++k) {
      fr->kp.push_back(Vec2f{(float)(640 * U(rng)), (float)(480 * U(rng))});
      fr->octave.push_back(0);
      fr->mps.push_back(nullptr);
      fr->outlier.push_back(false);
    }
  return s;
}

}  // namespace mini

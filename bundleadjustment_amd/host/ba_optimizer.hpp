// ba_optimizer.hpp — drop-in for the reference's optimizer classes
// (ba_project/src/ba/Optimizer.h:196-295) on top of libba_hip.so.
//
// Same class names, same public methods and the same outer-loop semantics as
// Optimizer.cpp; only the Ceres seam (Problem + AddResidualBlock + Solve,
// Optimizer.cpp:225-242 / 427-442 / 548-570) is replaced by the C ABI of
// include/ba_hip.h, and pruneCorrespondences (Optimizer.cpp:6-79) runs as a
// device kernel (ba_prune).
//
// The reference's model classes (Frame, MapPoint, SceneMap) need Eigen and
// OpenCV, so the shim reaches them through a Model adapter with static
// members (INTEGRATION.md shows the adapter for the reference's classes):
//
//   struct Model {
//     using Map = SceneMap; using FramePtr = std::shared_ptr<Frame>;
//     using PointPtr = std::shared_ptr<MapPoint>;
//     static std::vector<FramePtr> key_frames(Map*);                  // SceneMap::getKeyFrames
//     static std::vector<PointPtr> map_points(Map*);                  // SceneMap::getMapPoints
//     static std::vector<PointPtr> frame_map_points(const FramePtr&); // Frame::getMapPoints
//     static PointPtr frame_map_point(const FramePtr&, int i);        // Frame::getMapPoint
//     static int  keypoint_count(const FramePtr&);                    // Frame::getKeypointCount
//     static Vec2f keypoint_pt(const FramePtr&, int i);               // getKeypoint(i)->pt
//     static int  keypoint_octave(const FramePtr&, int i);            // getKeypoint(i)->octave
//     static bool is_outlier(const FramePtr&, int i);                 // Frame::isOutlier
//     static void set_outlier(const FramePtr&, int i, bool outlier);  // setOutlier / setInlier
//     static int  id(const FramePtr&);                                // Frame::getID
//     static bool is_key_frame(const FramePtr&);                      // Frame::isKeyFrame
//     static Mat4f pose(const FramePtr&);                             // Frame::getPose (camera->world)
//     static void set_pose(const FramePtr&, const Mat4f&);            // Frame::setPose
//     static Mat3f intrinsics(const FramePtr&);                       // Frame::getIntrinsics
//     static std::vector<FramePtr> best_covisibility_frames(const FramePtr&, int n);
//     static Vec3f position(const PointPtr&);                         // MapPoint::getPosition
//     static void set_position(const PointPtr&, const Vec3f&);        // MapPoint::setPosition
//     static Vec2f keypoint_of(const PointPtr&, const FramePtr&);     // getCorresponding2DKeyPointPosition
//     static float min_distance(const PointPtr&), max_distance(const PointPtr&);
//     static bool is_invalid(const PointPtr&);                        // MapPoint::isInvalid
//     static std::vector<std::pair<FramePtr, size_t>> observing_keyframes(const PointPtr&);
//     static void erase_outliers(Map*, int current_frame_id);         // SfMHelper::eraseOutlier
//   };
//
// Error behaviour: like the reference (which ignores the Ceres summary and
// never aborts), optimize calls do not throw on solver failure; a failed
// round leaves the model untouched and is reported by lastStatus() /
// lastError().
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

#include "ba_geometry.hpp"
#include "ba_hip.h"

namespace ba_amd {

// The product backend: one ba_ctx on one HIP device.
class HipBackend {
 public:
  explicit HipBackend(int device = 0) {
    const int st = ba_create(&ctx_, device);
    if (st != BA_OK) throw std::runtime_error("ba_create failed (status " + std::to_string(st) + ")");
  }
  ~HipBackend() { ba_destroy(ctx_); }
  HipBackend(const HipBackend&) = delete;
  HipBackend& operator=(const HipBackend&) = delete;

  int solve(const ba_problem& p, const ba_options& o, double* cams, double* pts, ba_summary* s) {
    if (pose_only(p)) return solve_pose(p, o, cams, pts, s);
    int st = ba_set_problem(ctx_, &p);
    if (st == BA_OK) st = ba_solve(ctx_, &o, s);
    if (st == BA_OK) st = ba_get_params(ctx_, cams, pts);
    return st;
  }
  int prune(const ba_prune_problem& p, uint8_t* result) { return ba_prune(ctx_, &p, result); }

  // The motion-only problem (one variable camera, every point constant:
  // MotionOnlyBAOptimizerAngles::prepareConstraints, Optimizer.cpp:459-498)
  // goes through the batched pose solver: the whole LM loop in one launch.
  static bool pose_only(const ba_problem& p) {
    if (p.n_cams != 1 || (p.cam_fixed && p.cam_fixed[0]) || !p.pt_fixed) return false;
    for (int32_t i = 0; i < p.n_pts; ++i)
      if (!p.pt_fixed[i]) return false;
    return true;
  }
  int solve_pose(const ba_problem& p, const ba_options& o, double* cams, double* pts, ba_summary* s) {
    const int32_t off[2] = {0, p.n_obs};
    std::vector<double> X(3 * static_cast<size_t>(p.n_obs));
    for (int32_t k = 0; k < p.n_obs; ++k)
      for (int i = 0; i < 3; ++i) X[3 * k + i] = p.pts[3 * static_cast<size_t>(p.obs_pt[k]) + i];
    ba_pose_batch b{};
    b.n_problems = 1;
    b.obs_offset = off;
    b.cams = p.cams;
    b.K = p.K;
    b.pts = X.data();
    b.obs_uv = p.obs_uv;
    b.huber_a = p.huber_a;
    const int st = ba_solve_pose_batch(ctx_, &b, &o, cams, s);
    if (st == BA_OK && pts && p.n_pts > 0) std::copy(p.pts, p.pts + 3 * static_cast<size_t>(p.n_pts), pts);
    return st;
  }
  std::string last_error() const { return ba_last_error(ctx_); }

 private:
  ba_ctx* ctx_ = nullptr;
};

// Host SoA of one ba_problem (the gather of prepareConstraints).
struct ProblemBuffers {
  std::vector<double> cams, pts;
  std::vector<uint8_t> cam_fixed, pt_fixed;
  std::vector<float> extr, K, uv;
  std::vector<int32_t> obs_cam, obs_pt;

  int add_camera(const double* cam6, bool fixed, const Mat4f& e, const Mat3f& k) {
    cams.insert(cams.end(), cam6, cam6 + 6);
    cam_fixed.push_back(fixed ? 1 : 0);
    extr.insert(extr.end(), e.m, e.m + 16);
    K.insert(K.end(), k.m, k.m + 9);
    return static_cast<int>(cam_fixed.size()) - 1;
  }
  int add_point(const Vec3f& X, bool fixed) {
    for (int i = 0; i < 3; ++i) pts.push_back(static_cast<double>(X[i]));
    pt_fixed.push_back(fixed ? 1 : 0);
    return static_cast<int>(pt_fixed.size()) - 1;
  }
  void add_obs(int c, int p, const Vec2f& kp) {
    obs_cam.push_back(c);
    obs_pt.push_back(p);
    uv.push_back(kp.x);
    uv.push_back(kp.y);
  }
  ba_problem view() const {
    ba_problem p{};
    p.n_cams = static_cast<int32_t>(cam_fixed.size());
    p.n_pts = static_cast<int32_t>(pt_fixed.size());
    p.n_obs = static_cast<int32_t>(obs_cam.size());
    p.cams = cams.data(); p.cam_fixed = cam_fixed.data(); p.cam_fixed_extr = extr.data(); p.K = K.data();
    p.pts = pts.data(); p.pt_fixed = pt_fixed.data();
    p.obs_cam = obs_cam.data(); p.obs_pt = obs_pt.data(); p.obs_uv = uv.data();
    p.huber_a = std::sqrt(5.991);   // HuberLoss(sqrt(5.991)), Optimizer.cpp:312
    return p;
  }
};

// BAOptimizer (Optimizer.h:196-222).
template <class Model, class Backend = HipBackend>
class BAOptimizer {
 public:
  using FramePtr = typename Model::FramePtr;
  using PointPtr = typename Model::PointPtr;

  explicit BAOptimizer(Backend& backend) : backend_(backend) {}

  void setNbOfIterations(unsigned nIterations) { m_nIterations = nIterations; }
  void setNbOfMaxItPerBA(unsigned nMaxItPerBA) { m_nMaxItPerBA = nMaxItPerBA; }

  int lastStatus() const { return status_; }
  const std::string& lastError() const { return error_; }
  const ba_summary& lastSummary() const { return summary_; }

 protected:
  unsigned m_nIterations = 3;      // Optimizer.h:201-202
  unsigned m_nMaxItPerBA = 200;
  Backend& backend_;
  int status_ = BA_OK;
  std::string error_;
  ba_summary summary_{};

  // configureSolver (Optimizer.cpp:80-90): LM, monotonic, DENSE_SCHUR,
  // max_num_iterations = m_nMaxItPerBA, everything else Ceres defaults.
  void configureSolver(ba_options& o) const {
    ba_default_options(&o);
    o.max_num_iterations = static_cast<int32_t>(m_nMaxItPerBA);
    o.linear_solver = BA_DENSE_SCHUR;
  }

  bool run_solver(ProblemBuffers& B) {
    ba_options o;
    configureSolver(o);
    const ba_problem p = B.view();
    status_ = backend_.solve(p, o, B.cams.data(), B.pts.data(), &summary_);
    if (status_ != BA_OK) error_ = backend_.last_error();
    return status_ == BA_OK;
  }

  // pruneCorrespondences (Optimizer.cpp:6-79) for several frames in one
  // device batch: per keypoint with a map point (and, unless considerOutlier,
  // not already an outlier) the float tests of the reference.
  void pruneCorrespondences(const std::vector<FramePtr>& frames, bool considerOutlier) {
    std::vector<float> extr, center, K, X, uv, inv_sigma, dist;
    std::vector<int32_t> cam;
    std::vector<std::pair<int, int>> who;   // (frame, keypoint)
    for (size_t f = 0; f < frames.size(); ++f) {
      const FramePtr& fr = frames[f];
      const Mat4f pose = Model::pose(fr);
      const Mat4f e = inverse4(pose);
      const Mat3f k = Model::intrinsics(fr);
      extr.insert(extr.end(), e.m, e.m + 16);
      for (int r = 0; r < 3; ++r) center.push_back(pose.m[12 + r]);   // getWorldPos = pose.block(0,3,3,1)
      K.insert(K.end(), k.m, k.m + 9);
      const int n = Model::keypoint_count(fr);
      for (int i = 0; i < n; ++i) {
        if (!(considerOutlier || !Model::is_outlier(fr, i))) continue;
        const PointPtr mp = Model::frame_map_point(fr, i);
        if (!mp) continue;
        const Vec3f P = Model::position(mp);
        const Vec2f kp = Model::keypoint_pt(fr, i);
        cam.push_back(static_cast<int32_t>(f));
        X.insert(X.end(), P.v, P.v + 3);
        uv.push_back(kp.x);
        uv.push_back(kp.y);
        inv_sigma.push_back(static_cast<float>(1.0 / std::pow(1.2, Model::keypoint_octave(fr, i))));
        dist.push_back(Model::min_distance(mp));
        dist.push_back(Model::max_distance(mp));
        who.emplace_back(static_cast<int>(f), i);
      }
    }
    if (who.empty()) return;
    ba_prune_problem pp{};
    pp.n_cams = static_cast<int32_t>(frames.size());
    pp.n_obs = static_cast<int32_t>(who.size());
    pp.extr = extr.data(); pp.cam_center = center.data(); pp.K = K.data(); pp.obs_cam = cam.data();
    pp.obs_X = X.data(); pp.obs_uv = uv.data(); pp.obs_inv_sigma = inv_sigma.data(); pp.obs_dist = dist.data();
    std::vector<uint8_t> res(who.size());
    const int st = backend_.prune(pp, res.data());
    if (st != BA_OK) { status_ = st; error_ = backend_.last_error(); return; }
    for (size_t k = 0; k < who.size(); ++k)
      Model::set_outlier(frames[who[k].first], who[k].second, res[k] != BA_INLIER);
  }

  void write_back_points(const std::vector<PointPtr>& points, const ProblemBuffers& B) {
    for (size_t i = 0; i < points.size(); ++i) {
      Vec3f v;
      for (int r = 0; r < 3; ++r) v.v[r] = static_cast<float>(B.pts[3 * i + r]);   // .cast<float>()
      Model::set_position(points[i], v);
    }
  }
};

// GlobalBAOptimizerAngles (Optimizer.h:243-254, Optimizer.cpp:216-333).
template <class Model, class Backend = HipBackend>
class GlobalBAOptimizerAngles : public BAOptimizer<Model, Backend> {
  using Base = BAOptimizer<Model, Backend>;

 public:
  using typename Base::FramePtr;
  using typename Base::PointPtr;
  using Base::Base;

  void optimizeCamerasAndMapPoints(typename Model::Map* optimizedMap, bool eraseOutliers, int currentFrameID) {
    const auto frames = Model::key_frames(optimizedMap);
    const auto points = Model::map_points(optimizedMap);
    for (unsigned it = 0; it < this->m_nIterations; ++it) {
      ProblemBuffers B;
      prepareConstraints(frames, points, B);
      if (!this->run_solver(B)) return;
      this->write_back_points(points, B);
      for (size_t i = 0; i < frames.size(); ++i) Model::set_pose(frames[i], pose_from_camera_block(&B.cams[6 * i]));
      this->pruneCorrespondences(frames, false);
    }
    if (eraseOutliers) Model::erase_outliers(optimizedMap, currentFrameID);
  }

 private:
  void prepareConstraints(const std::vector<FramePtr>& frames, const std::vector<PointPtr>& points,
                          ProblemBuffers& B) const {
    std::unordered_map<const void*, int> pidx;
    for (const auto& p : points) pidx.emplace(p.get(), B.add_point(Model::position(p), false));
    for (const auto& fr : frames) {
      double cam6[6];
      Mat4f extr;
      camera_block_from_pose(Model::pose(fr), cam6, &extr);
      // keyframe 0 is the world anchor: PointOnlyReprojectionError with its extr
      const int c = B.add_camera(cam6, Model::id(fr) == 0, extr, Model::intrinsics(fr));
      const auto vis = Model::frame_map_points(fr);
      for (size_t j = 0; j < vis.size(); ++j) {
        const PointPtr& mp = vis[j];
        if (!mp || Model::is_outlier(fr, static_cast<int>(j))) continue;
        const auto f = pidx.find(mp.get());
        if (f == pidx.end()) continue;   // the reference dereferences end() here (undefined)
        B.add_obs(c, f->second, Model::keypoint_of(mp, fr));
      }
    }
  }
};

// LocalBAOptimizerAngles (Optimizer.h:280-291, Optimizer.cpp:500-698).
template <class Model, class Backend = HipBackend>
class LocalBAOptimizerAngles : public BAOptimizer<Model, Backend> {
  using Base = BAOptimizer<Model, Backend>;

 public:
  using typename Base::FramePtr;
  using typename Base::PointPtr;
  using Base::Base;

  void optimizeCamerasAndMapPoints(typename Model::Map* optimizedMap, FramePtr currentFrame, bool eraseOutliers) {
    std::vector<FramePtr> localFrames = Model::best_covisibility_frames(currentFrame, 10);
    localFrames.push_back(currentFrame);
    std::vector<PointPtr> localPoints;
    std::unordered_set<const void*> inLocal;
    for (const auto& fr : localFrames) {
      const auto mps = Model::frame_map_points(fr);
      for (size_t j = 0; j < mps.size(); ++j) {
        const PointPtr& mp = mps[j];
        if (mp && !Model::is_outlier(fr, static_cast<int>(j)) && !Model::is_invalid(mp) && inLocal.insert(mp.get()).second)
          localPoints.push_back(mp);
      }
    }
    std::vector<FramePtr> fixedFrames;
    std::unordered_set<const void*> seen;
    for (const auto& fr : localFrames) seen.insert(fr.get());
    for (const auto& mp : localPoints)
      for (const auto& ob : Model::observing_keyframes(mp))
        if (!Model::is_outlier(ob.first, static_cast<int>(ob.second)) && Model::is_key_frame(ob.first) &&
            seen.insert(ob.first.get()).second)
          fixedFrames.push_back(ob.first);

    for (unsigned it = 0; it < this->m_nIterations; ++it) {
      ProblemBuffers B;
      prepareConstraints(localFrames, fixedFrames, localPoints, B);
      if (!this->run_solver(B)) return;
      this->write_back_points(localPoints, B);
      for (size_t i = 0; i < localFrames.size(); ++i)
        Model::set_pose(localFrames[i], pose_from_camera_block(&B.cams[6 * i]));
      this->pruneCorrespondences(localFrames, false);
      this->pruneCorrespondences(fixedFrames, false);
    }
    if (eraseOutliers) Model::erase_outliers(optimizedMap, Model::id(currentFrame));
  }

 private:
  void prepareConstraints(const std::vector<FramePtr>& localFrames, const std::vector<FramePtr>& fixedFrames,
                          const std::vector<PointPtr>& points, ProblemBuffers& B) const {
    std::unordered_map<const void*, int> pidx;
    for (const auto& p : points) pidx.emplace(p.get(), B.add_point(Model::position(p), false));
    for (const auto& fr : localFrames) {
      double cam6[6];
      Mat4f extr;
      camera_block_from_pose(Model::pose(fr), cam6, &extr);
      const int c = B.add_camera(cam6, Model::id(fr) == 0, extr, Model::intrinsics(fr));
      const auto vis = Model::frame_map_points(fr);
      for (size_t j = 0; j < vis.size(); ++j) {
        const PointPtr& mp = vis[j];
        if (!mp || Model::is_outlier(fr, static_cast<int>(j))) continue;
        const auto f = pidx.find(mp.get());
        if (f == pidx.end()) continue;   // invalid point: the reference dereferences end() (undefined)
        B.add_obs(c, f->second, Model::keypoint_of(mp, fr));
      }
    }
    // fixed frames: PointOnlyReprojectionError on local points only (:673-694)
    for (const auto& fr : fixedFrames) {
      double cam6[6];
      Mat4f extr;
      camera_block_from_pose(Model::pose(fr), cam6, &extr);
      const int c = B.add_camera(cam6, true, extr, Model::intrinsics(fr));
      const auto vis = Model::frame_map_points(fr);
      for (size_t j = 0; j < vis.size(); ++j) {
        const PointPtr& mp = vis[j];
        if (!mp || Model::is_outlier(fr, static_cast<int>(j))) continue;
        const auto f = pidx.find(mp.get());
        if (f == pidx.end()) continue;
        B.add_obs(c, f->second, Model::keypoint_of(mp, fr));
      }
    }
  }
};

// MotionOnlyBAOptimizerAngles (Optimizer.h:267-277, Optimizer.cpp:416-498):
// one camera, constant points (PoseOnlyAngleReprojectionError), Huber on.
template <class Model, class Backend = HipBackend>
class MotionOnlyBAOptimizerAngles : public BAOptimizer<Model, Backend> {
  using Base = BAOptimizer<Model, Backend>;

 public:
  using typename Base::FramePtr;
  using typename Base::PointPtr;
  using Base::Base;

  void optimizeCameraPose(FramePtr frame) {
    const auto points = Model::frame_map_points(frame);
    for (unsigned it = 0; it < this->m_nIterations; ++it) {
      ProblemBuffers B;
      double cam6[6];
      Mat4f extr;
      camera_block_from_pose(Model::pose(frame), cam6, &extr);
      B.add_camera(cam6, false, extr, Model::intrinsics(frame));
      for (size_t j = 0; j < points.size(); ++j) {
        const PointPtr& mp = points[j];
        if (!mp || Model::is_outlier(frame, static_cast<int>(j))) continue;
        const int p = B.add_point(Model::position(mp), true);
        B.add_obs(0, p, Model::keypoint_of(mp, frame));
      }
      if (!this->run_solver(B)) return;
      Model::set_pose(frame, pose_from_camera_block(B.cams.data()));
      this->pruneCorrespondences({frame}, true);   // default considerOutlier = true (Optimizer.h:219)
    }
  }
};

}  // namespace ba_amd

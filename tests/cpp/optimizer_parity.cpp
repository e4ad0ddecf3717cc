// optimizer_parity.cpp — drives the optimizer-class shim
// (bundleadjustment_amd/host/ba_optimizer.hpp) over a synthetic mini model
// with a chosen backend and prints the resulting model state as JSON:
//   hip     libba_hip.so (the product path; needs a GPU)
//   oracle  oracle/liboracle.so (CPU restatement; test infrastructure)
// Scenarios: global BA (2 outer rounds), local BA around the last keyframe,
// motion-only BA of the last frame.  Test code only.
#include <cstdio>
#include <cstring>
#include <string>

#include "ba_optimizer.hpp"
#include "mini_model.hpp"

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
int oracle_solve(const oracle_problem* prob, const void* opt, double* iter_log, int max_log, double* summary);
void oracle_prune(int n_obs, const float* extr, const float* center, const float* K, const int32_t* obs_cam,
                  const float* X, const float* uv, const float* inv_sigma, const float* dist, uint8_t* result);
}

struct OracleBackend {
  int solve(const ba_problem& p, const ba_options& o, double* cams, double* pts, ba_summary* s) {
    if (cams != p.cams) std::memcpy(cams, p.cams, sizeof(double) * 6 * p.n_cams);
    if (pts != p.pts) std::memcpy(pts, p.pts, sizeof(double) * 3 * p.n_pts);
    oracle_problem q{p.n_cams, p.n_pts, p.n_obs, 0, cams, p.cam_fixed, p.cam_fixed_extr, p.K,
                     pts, p.pt_fixed, p.obs_cam, p.obs_pt, p.obs_uv, p.huber_a};
    double sum[6];
    oracle_solve(&q, &o, nullptr, 0, sum);
    s->initial_cost = sum[0];
    s->final_cost = sum[1];
    s->num_iterations = (int)sum[2];
    s->termination_type = (int)sum[5];
    return BA_OK;
  }
  int prune(const ba_prune_problem& p, uint8_t* r) {
    oracle_prune(p.n_obs, p.extr, p.cam_center, p.K, p.obs_cam, p.obs_X, p.obs_uv, p.obs_inv_sigma, p.obs_dist, r);
    return BA_OK;
  }
  std::string last_error() const { return ""; }
};

static void dump(const char* name, const mini::Scene& s, const ba_summary& sum, int status, bool last) {
  std::printf("  \"%s\": {\"status\": %d, \"final_cost\": %.17g, \"iterations\": %d, \"erase_calls\": %d,\n", name,
              status, sum.final_cost, sum.num_iterations, s.erase_calls);
  std::printf("    \"poses\": [");
  for (size_t f = 0; f < s.frames.size(); ++f)
    for (int k = 0; k < 16; ++k)
      std::printf("%s%.9g", (f || k) ? ", " : "", s.frames[f]->pose.m[k]);
  std::printf("],\n    \"points\": [");
  for (size_t p = 0; p < s.points.size(); ++p)
    for (int k = 0; k < 3; ++k) std::printf("%s%.9g", (p || k) ? ", " : "", s.points[p]->X.v[k]);
  std::printf("],\n    \"outliers\": [");
  bool first = true;
  for (const auto& f : s.frames)
    for (bool o : f->outlier) { std::printf("%s%d", first ? "" : ", ", o ? 1 : 0); first = false; }
  std::printf("]}%s\n", last ? "" : ",");
}

template <class Backend>
static int run(Backend& be, unsigned seed) {
  using namespace ba_amd;
  std::printf("{\n");
  {
    mini::Scene s = mini::make_scene(8, 500, seed);
    GlobalBAOptimizerAngles<mini::Model, Backend> opt(be);
    opt.setNbOfIterations(2);
    opt.setNbOfMaxItPerBA(30);
    opt.optimizeCamerasAndMapPoints(&s, true, (int)s.frames.size() - 1);
    dump("global", s, opt.lastSummary(), opt.lastStatus(), false);
  }
  {
    mini::Scene s = mini::make_scene(14, 500, seed + 1);
    LocalBAOptimizerAngles<mini::Model, Backend> opt(be);
    opt.setNbOfIterations(2);
    opt.setNbOfMaxItPerBA(30);
    opt.optimizeCamerasAndMapPoints(&s, s.frames.back(), false);
    dump("local", s, opt.lastSummary(), opt.lastStatus(), false);
  }
  {
    mini::Scene s = mini::make_scene(4, 400, seed + 2);
    MotionOnlyBAOptimizerAngles<mini::Model, Backend> opt(be);
    opt.setNbOfIterations(4);      // SfMHelper::estimatePoseUsingBA: 4 x 20
    opt.setNbOfMaxItPerBA(20);
    opt.optimizeCameraPose(s.frames.back());
    dump("motion_only", s, opt.lastSummary(), opt.lastStatus(), true);
  }
  std::printf("}\n");
  return 0;
}

int main(int argc, char** argv) {
  const std::string which = argc > 1 ? argv[1] : "oracle";
  const unsigned seed = argc > 2 ? (unsigned)std::stoul(argv[2]) : 7u;
  if (which == "oracle") {
    OracleBackend be;
    return run(be, seed);
  }
#ifndef BA_NO_HIP_BACKEND   // the sanitizer build links the oracle only (make sanitize)
  if (which == "hip") {
    try {
      ba_amd::HipBackend be(0);
      return run(be, seed);
    } catch (const std::exception& e) {
      std::fprintf(stderr, "%s\n", e.what());
      return 2;
    }
  }
#endif
  std::fprintf(stderr, "usage: %s hip|oracle [seed]\n", argv[0]);
  return 1;
}

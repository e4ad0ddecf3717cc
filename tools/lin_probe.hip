// lin_probe.hip — diagnostic ablations of the linearisation kernel on a
// C3-shaped synthetic problem (200 cams, 100k points, 10 obs / point).
// timing the k_linearize_lds_t<threads, stage rows> variants (one block
// per CU) and the global-table kernel
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/lin_probe tools/lin_probe.hip
#include "../bundleadjustment_amd/csrc/ba_kernels.hip"

#include <cstdio>
#include <random>
#include <vector>

using namespace bahip;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)




namespace bahip {
// VAR 0: product body; 1: all lanes on camera 1 (broadcast table reads);
// 2: stage with b128 (row stride 22); 3: no stage (row-per-lane stores);
// 4: table reads + trivial arithmetic (sum of the row) + stage + stores
template <int VAR>
__global__ __launch_bounds__(512) void k_lin_var(DevProblem P, const double* __restrict__ rec,
                                                 const double* __restrict__ pts, double* __restrict__ JR,
                                                 double* __restrict__ part) {
  constexpr int LD = kStageLd;
  __shared__ double lds[2 * 16];
  __shared__ __attribute__((aligned(16))) double stage[8 * 64 * kStageLd];
  __shared__ __attribute__((aligned(16))) double tbl[kLinLdsCams * kTblRec];
  __shared__ float ktb[kLinLdsCams * 9];
  fill_lin_table<512>(P, rec, tbl, ktb);
  double acc[2] = {0.0, 0.0};
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double* st = stage + w * (64 * LD);
  const int step = gridDim.x * 8 * 64;
  for (int base = (blockIdx.x * 8 + w) * 64; base < P.no; base += step) {
    const int o = base + lane;
    double out[kJR];
    if (o < P.no) {
      int c = P.obs_cam[o];
      const int p = P.obs_pt[o];
      const float2 uv = P.uv[o];
      if (VAR == 1) c = 1;
      const CamLds cam{tbl + c * kTblRec, ktb + c * 9};
      if (VAR == 4) {
        double T[kLin];
        cam.load(T);
        double sum = pts[3 * p] + uv.x;
#pragma unroll
        for (int k = 0; k < kLin; ++k) sum += T[k];
#pragma unroll
        for (int k = 0; k < kJR; ++k) out[k] = sum + k;
      } else {
        bool fin;
        acc[0] += 0.5 * lin_obs(P, cam, cam.var(), P.pt_var[p] != 0, pts[3 * p], pts[3 * p + 1], pts[3 * p + 2], uv,
                                out, fin);
        acc[1] += fin ? 0.0 : 1.0;
      }
    }
    const int nrec = min(64, P.no - base);
    if (VAR == 3) {
      if (o < P.no) {
        double2* d = reinterpret_cast<double2*>(JR + (size_t)o * kJR);
#pragma unroll
        for (int k = 0; k < kJR / 2; ++k) d[k] = make_double2(out[2 * k], out[2 * k + 1]);
      }
      continue;
    }
    if (o < P.no) {
      double* row = st + lane * LD;
      if (VAR == 2) {
#pragma unroll
        for (int k = 0; k < kJR / 2; ++k) reinterpret_cast<double2*>(row)[k] = make_double2(out[2 * k], out[2 * k + 1]);
      } else {
#pragma unroll
        for (int k = 0; k < kJR; ++k) row[k] = out[k];
      }
    }
    wave_lds_sync();
    double2* dst = reinterpret_cast<double2*>(JR + (size_t)base * kJR);
#pragma unroll
    for (int it = 0; it < kJR / 2; ++it) {
      const int e = it * 64 + lane;
      const int r = e / (kJR / 2), f = 2 * (e - r * (kJR / 2));
      double2 v;
      if (VAR == 2) v = reinterpret_cast<const double2*>(st + r * LD)[f / 2];
      else v = make_double2(st[r * LD + f], st[r * LD + f + 1]);
      if (r < nrec) dst[e] = v;
    }
    wave_lds_sync();
  }
  double tot[2];
  block_sum<2>(acc, lds, tot);
  if (threadIdx.x == 0) { part[blockIdx.x] = tot[0]; part[kMaxBlocks + blockIdx.x] = tot[1]; }
}
}  // namespace bahip

template <class T>
static T* up(const std::vector<T>& h) {
  T* d = nullptr;
  if (hipMalloc(&d, h.size() * sizeof(T)) != hipSuccess) return nullptr;
  (void)hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice);
  return d;
}

int main() {
  const int nc = 200, np = 100000, k = 10, no = np * k;
  std::mt19937 rng(7);
  std::vector<int> oc(no), op(no), voff(np + 1), vc(nc), cov(nc);
  std::vector<float2> uv(no);
  std::vector<double> cams(6 * nc), pts(3 * np);
  std::vector<float> K(9 * nc), extr(16 * nc, 0.f);
  std::vector<uint8_t> cfix(nc, 0), pvar(np, 1);
  std::uniform_real_distribution<double> U(-1, 1);
  for (int c = 0; c < nc; ++c) {
    for (int a = 0; a < 3; ++a) cams[6 * c + a] = 0.3 * U(rng);
    for (int a = 3; a < 6; ++a) cams[6 * c + a] = U(rng);
    cams[6 * c + 5] += 5.0;
    const float Kc[9] = {525.f, 0.f, 0.f, 0.f, 525.f, 0.f, 319.5f, 239.5f, 1.f};
    for (int a = 0; a < 9; ++a) K[9 * c + a] = Kc[a];
    vc[c] = c;
  }
  cfix[0] = 1; vc[0] = -1;
  for (int a = 0; a < 4; ++a) extr[a * 5] = 1.f;
  extr[14] = 5.f;
  for (int p = 0; p < np; ++p) {
    for (int a = 0; a < 3; ++a) pts[3 * p + a] = U(rng);
    std::vector<int> cs;
    while ((int)cs.size() < k) {
      int c = rng() % nc;
      bool dup = false;
      for (int x : cs) dup |= x == c;
      if (!dup) cs.push_back(c);
    }
    std::sort(cs.begin(), cs.end());
    for (int j = 0; j < k; ++j) {
      oc[p * k + j] = cs[j]; op[p * k + j] = p;
      uv[p * k + j] = make_float2(300.f + 10.f * (float)U(rng), 200.f + 10.f * (float)U(rng));
    }
    voff[p + 1] = (p + 1) * k;
  }
  DevProblem P{};
  P.nc = nc; P.np = np; P.no = no; P.nvc = nc - 1; P.n = 6 * (nc - 1); P.ld = P.n;
  P.huber_a = std::sqrt(5.991); P.huber_b = 5.991;
  P.obs_cam = up(oc); P.obs_pt = up(op); P.uv = up(uv); P.pt_off = up(voff); P.vc = up(vc);
  P.cam_fixed = up(cfix); P.pt_var = up(pvar); P.K = up(K); P.extr = up(extr);
  double* d_cams = up(cams);
  double* d_pts = up(pts);
  double *rec, *JR, *part;
  CK(hipMalloc(&rec, sizeof(double) * kCamRec * nc));
  CK(hipMalloc(&JR, sizeof(double) * kJR * (size_t)no));
  CK(hipMalloc(&part, sizeof(double) * kNumSlots * kMaxBlocks));
  launch_cam_prep(P, d_cams, rec, true, 0);
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  const double bytes = 176.0 * no + 24.0 * np + 48.0 * nc;
  auto run = [&](const char* name, auto launch) {
    launch(); launch();
    CK(hipDeviceSynchronize());
    const int reps = 30;
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    printf("%-34s %8.2f us  %7.1f GB/s (algorithmic B_rj)\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
    return 0;
  };
  const int g = 256;
  run("k_linearize_lds_t<512,64>", [&] { hipLaunchKernelGGL((k_linearize_lds_t<512, 64>), dim3(g), dim3(512), 0, 0, P, rec, d_pts, JR, part); });
  run("k_linearize_lds_t<512,64> fill hook", [&] { hipLaunchKernelGGL((k_linearize_lds_t<512, 64, 0, true>), dim3(g), dim3(512), 0, 0, P, rec, d_pts, JR, part); });
  run("var0 product body (no prefetch)", [&] { hipLaunchKernelGGL(k_lin_var<0>, dim3(g), dim3(512), 0, 0, P, rec, d_pts, JR, part); });
  run("var1 one camera", [&] { hipLaunchKernelGGL(k_lin_var<1>, dim3(g), dim3(512), 0, 0, P, rec, d_pts, JR, part); });

  run("var3 no stage", [&] { hipLaunchKernelGGL(k_lin_var<3>, dim3(g), dim3(512), 0, 0, P, rec, d_pts, JR, part); });
  run("var4 table+stage+store, no arith", [&] { hipLaunchKernelGGL(k_lin_var<4>, dim3(g), dim3(512), 0, 0, P, rec, d_pts, JR, part); });
  run("product pipeline, no stores", [&] { hipLaunchKernelGGL((k_linearize_lds_t<512, 64, 1>), dim3(g), dim3(512), 0, 0, P, rec, d_pts, JR, part); });
  run("product pipeline, no arith", [&] { hipLaunchKernelGGL((k_linearize_lds_t<512, 64, 2>), dim3(g), dim3(512), 0, 0, P, rec, d_pts, JR, part); });
  run("product pipeline, fill only", [&] { hipLaunchKernelGGL((k_linearize_lds_t<512, 64, 3>), dim3(g), dim3(512), 0, 0, P, rec, d_pts, JR, part); });
  run("product pipeline, loads only", [&] { hipLaunchKernelGGL((k_linearize_lds_t<512, 64, 4>), dim3(g), dim3(512), 0, 0, P, rec, d_pts, JR, part); });
  run("arith only (5)", [&] { hipLaunchKernelGGL((k_linearize_lds_t<512, 64, 5>), dim3(g), dim3(512), 0, 0, P, rec, d_pts, JR, part); });
  run("arith only one camera (6)", [&] { hipLaunchKernelGGL((k_linearize_lds_t<512, 64, 6>), dim3(g), dim3(512), 0, 0, P, rec, d_pts, JR, part); });
  run("lazy <512,64>", [&] { hipLaunchKernelGGL((k_linearize_lds_t<512, 64, 0, true>), dim3(g), dim3(512), 0, 0, P, rec, d_pts, JR, part); });
  run("lazy <512,32>", [&] { hipLaunchKernelGGL((k_linearize_lds_t<512, 32, 0, true>), dim3(g), dim3(512), 0, 0, P, rec, d_pts, JR, part); });
  run("k_linearize_lds_t<512,32>", [&] { hipLaunchKernelGGL((k_linearize_lds_t<512, 32>), dim3(g), dim3(512), 0, 0, P, rec, d_pts, JR, part); });
  run("k_linearize_lds_t<768,32>", [&] { hipLaunchKernelGGL((k_linearize_lds_t<768, 32>), dim3(g), dim3(768), 0, 0, P, rec, d_pts, JR, part); });
  run("k_linearize_lds_t<1024,32>", [&] { hipLaunchKernelGGL((k_linearize_lds_t<1024, 32>), dim3(g), dim3(1024), 0, 0, P, rec, d_pts, JR, part); });
  CK(hipDeviceSynchronize());
  return 0;
}

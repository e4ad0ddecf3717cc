// overlap_probe.hip — can the persistent Cholesky (k_chol_persist) and the
// camera-pair Schur pass (k_schur_pairs_c) run side by side on one MI355X?
// Times each alone and both launched together on two streams (either order),
// on a C3-sized system: n = 1194 (199 cameras), 1M observations of 100k
// points, 10 cameras each (4.5M partner pairs, ~20k camera-pair blocks).
// Checks that the factor is bitwise the same with the pair pass beside it.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I bundleadjustment_amd/csrc -I include \
//         tools/overlap_probe.hip -o tools/overlap_probe && tools/overlap_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "ba_chol.hip"
#include "ba_chol_split.hip"
#include "ba_chol_persist.hip"
#include "ba_kernels.hip"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

using namespace bahip;

int main(int argc, char** argv) {
  const int nvc = 199, n = 6 * nvc, ld = n, nrows = n + 1;
  const int np = 100000, per = 10, no = np * per;
  std::mt19937_64 rng(11);
  std::normal_distribution<double> N01;
  // SPD system for the factor
  const int m = n + 16;
  std::vector<double> G((size_t)n * m);
  for (auto& v : G) v = N01(rng);
  std::vector<double> A((size_t)nrows * ld, 0.0);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j <= i; ++j) {
      double s = 0;
      for (int k = 0; k < m; ++k) s += G[(size_t)i * m + k] * G[(size_t)j * m + k];
      s /= m;
      if (i == j) s += 1.0;
      A[(size_t)i * ld + j] = s;
    }
  for (int j = 0; j < n; ++j) A[(size_t)n * ld + j] = N01(rng);
  // observations: point-major, 10 distinct cameras per point
  std::vector<int> ocam(no);
  {
    std::vector<int> cams(nvc);
    for (int v = 0; v < nvc; ++v) cams[v] = v;
    for (int p = 0; p < np; ++p) {
      for (int i = 0; i < per; ++i) std::swap(cams[i], cams[i + rng() % (nvc - i)]);
      std::vector<int> c(cams.begin(), cams.begin() + per);
      std::sort(c.begin(), c.end());
      for (int i = 0; i < per; ++i) ocam[(size_t)p * per + i] = c[i];
    }
  }
  // blocks (a > b) sorted by key, pairs in point order inside a block
  std::vector<std::vector<int2>> lists((size_t)nvc * nvc);
  for (int p = 0; p < np; ++p)
    for (int i = 0; i < per; ++i)
      for (int j = 0; j < per; ++j) {
        const int oa = p * per + i, ob = p * per + j;
        if (ocam[oa] > ocam[ob]) lists[(size_t)ocam[oa] * nvc + ocam[ob]].push_back(make_int2(oa, ob));
      }
  std::vector<int4> blocks;
  std::vector<int2> pairs;
  for (int a = 0; a < nvc; ++a)
    for (int b = 0; b < a; ++b) {
      const auto& L = lists[(size_t)a * nvc + b];
      if (L.empty()) continue;
      blocks.push_back(make_int4(a, b, (int)pairs.size(), (int)(pairs.size() + L.size())));
      pairs.insert(pairs.end(), L.begin(), L.end());
    }
  printf("blocks %zu  pairs %zu\n", blocks.size(), pairs.size());
  std::vector<double> Wc((size_t)no * kWcRec);
  for (auto& v : Wc) v = N01(rng) * 0.1;
  std::vector<float> K((size_t)9 * nvc, 0.5f);
  std::vector<int> cov(nvc);
  for (int v = 0; v < nvc; ++v) cov[v] = v;
  std::vector<double> sc((size_t)6 * nvc, 1.0);

  double *dA, *dA0, *dL, *dV, *dS, *dSc, *dWc, *dScale;
  int4* dBlocks;
  int2* dPairs;
  float* dK;
  int* dCov;
  unsigned* dflags;
  const int T = (n + CB - 1) / CB, TR = (n + 1 + CB - 1) / CB;
  CK(hipMalloc(&dA, sizeof(double) * A.size()));
  CK(hipMalloc(&dA0, sizeof(double) * A.size()));
  CK(hipMalloc(&dL, sizeof(double) * A.size()));
  CK(hipMalloc(&dV, sizeof(double) * (size_t)(T + 1) * CB * CB));
  CK(hipMalloc(&dS, sizeof(double) * 64));
  CK(hipMalloc(&dSc, sizeof(double) * (size_t)(n + 1) * ld));
  CK(hipMalloc(&dWc, sizeof(double) * Wc.size()));
  CK(hipMalloc(&dScale, sizeof(double) * sc.size()));
  CK(hipMalloc(&dBlocks, sizeof(int4) * blocks.size()));
  CK(hipMalloc(&dPairs, sizeof(int2) * pairs.size()));
  CK(hipMalloc(&dK, sizeof(float) * K.size()));
  CK(hipMalloc(&dCov, sizeof(int) * cov.size()));
  CK(hipMalloc(&dflags, sizeof(unsigned) * (T + TR * T)));
  CK(hipMemset(dflags, 0, sizeof(unsigned) * (T + TR * T)));
  CK(hipMemcpy(dA0, A.data(), sizeof(double) * A.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dWc, Wc.data(), sizeof(double) * Wc.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dScale, sc.data(), sizeof(double) * sc.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dBlocks, blocks.data(), sizeof(int4) * blocks.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dPairs, pairs.data(), sizeof(int2) * pairs.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dK, K.data(), sizeof(float) * K.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dCov, cov.data(), sizeof(int) * cov.size(), hipMemcpyHostToDevice));
  DevProblem P{};
  P.nvc = nvc;
  P.ld = ld;
  P.K = dK;
  P.cam_of_vc = dCov;
  int* dXoff;
  {
    std::vector<int> xoff(9);
    const int R = ((int)blocks.size() + 7) / 8;
    for (int x = 0; x <= 8; ++x) xoff[x] = std::min((int)blocks.size(), x * R);
    CK(hipMalloc(&dXoff, sizeof(int) * 9));
    CK(hipMemcpy(dXoff, xoff.data(), sizeof(int) * 9, hipMemcpyHostToDevice));
  }
  int grid = ((int)blocks.size() + 15) / 16;
  grid = std::min(grid, 2048);
  grid = (grid + 7) / 8 * 8;

  hipStream_t sA, sB, sC;
  CK(hipStreamCreateWithFlags(&sA, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sB, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sC, hipStreamNonBlocking));
  hipEvent_t a0, a1, b0, b1, c1, ez;
  CK(hipEventCreate(&c1));
  CK(hipEventCreate(&ez));
  CK(hipEventCreate(&a0));
  CK(hipEventCreate(&a1));
  CK(hipEventCreate(&b0));
  CK(hipEventCreate(&b1));
  unsigned epoch = 1;
  std::vector<double> Lref(A.size()), Lx(A.size());
  auto chol = [&](hipStream_t s) {
    hipMemcpyAsync(dA, dA0, sizeof(double) * A.size(), hipMemcpyDeviceToDevice, s);
    hipEventRecord(a0, s);
    launch_chol_persist(dA, dL, ld, n, dV, dS, dflags, epoch++, s);
    hipEventRecord(a1, s);
  };
  // split form: critical workgroup on sA, workers on sC
  auto chol2 = [&]() {
    hipMemcpyAsync(dA, dA0, sizeof(double) * A.size(), hipMemcpyDeviceToDevice, sA);
    hipEventRecord(ez, sA);
    hipStreamWaitEvent(sC, ez, 0);
    hipEventRecord(a0, sA);
    launch_chol_persist2(dA, dL, ld, n, dV, dS, dflags, epoch++, sA, sC);
    hipEventRecord(a1, sA);
    hipEventRecord(c1, sC);
  };
  auto pairs_k = [&](hipStream_t s) {
    hipEventRecord(b0, s);
    hipLaunchKernelGGL(k_schur_pairs_c<false>, dim3(grid), dim3(256), 0, s, P, dBlocks, dXoff, dPairs, dWc, dScale,
                       dSc, nullptr, nullptr);
    hipEventRecord(b1, s);
  };
  auto ms = [](hipEvent_t x, hipEvent_t y) { float t; hipEventElapsedTime(&t, x, y); return t * 1e3f; };
  const char* names[7] = {"chol alone", "pairs alone", "chol then pairs", "pairs then chol", "split alone",
                          "split then pairs", "split, pairs 1"};
  const int grid0 = grid;
  for (int mode = 0; mode < 7; ++mode) {
    grid = mode == 6 ? std::min(grid0, 512) : grid0;
    for (int rep = 0; rep < 4; ++rep) {
      CK(hipDeviceSynchronize());
      if (mode == 0) chol(sA);
      if (mode == 1) pairs_k(sB);
      if (mode == 2) { chol(sA); pairs_k(sB); }
      if (mode == 3) { pairs_k(sB); chol(sA); }
      if (mode == 4) chol2();
      if (mode >= 5) { chol2(); pairs_k(sB); }
      CK(hipDeviceSynchronize());
      if (rep == 0) continue;
      if (mode == 0) printf("%-16s chol %6.1f us\n", names[mode], ms(a0, a1));
      if (mode == 1) printf("%-16s pairs %6.1f us\n", names[mode], ms(b0, b1));
      if (mode == 4) printf("%-16s crit %6.1f us  workers end %6.1f us\n", names[mode], ms(a0, a1), ms(a0, c1));
      if (mode == 2 || mode == 3 || mode >= 5) {
        const float ta = ms(a0, a1), tb = ms(b0, b1), start = std::min(0.f, ms(a0, b0));
        float end = std::max(ms(a0, a1), ms(a0, b1));
        if (mode >= 5) end = std::max(end, ms(a0, c1));
        printf("%-16s chol %6.1f us  pairs %6.1f us  pairs start %+6.1f us after chol start  span %6.1f us\n",
               names[mode], ta, tb, ms(a0, b0), end - start);
      }
    }
    if (mode != 1) {
      std::vector<double> Sh(64);
      CK(hipMemcpy(Sh.data(), dS, sizeof(double) * 64, hipMemcpyDeviceToHost));
      CK(hipMemcpy(mode == 0 ? Lref.data() : Lx.data(), dL, sizeof(double) * A.size(), hipMemcpyDeviceToHost));
      size_t diff = 0;
      if (mode != 0)
        for (int i = 0; i <= n; ++i)
          for (int j = 0; j < n && j <= i; ++j)
            diff += std::memcmp(&Lx[(size_t)i * ld + j], &Lref[(size_t)i * ld + j], 8) != 0;
      printf("   chol_bad %g  L entries differing from chol-alone: %zu\n", Sh[SL_CHOL_BAD], diff);
      if (Sh[SL_CHOL_BAD] != 0.0 || diff) return 2;
    }
  }
  return 0;
}

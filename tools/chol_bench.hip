// chol_bench.hip — diagnostic harness for the reduced-camera Cholesky
// (bundleadjustment_amd/csrc/ba_chol.hip), built with in-kernel s_memtime
// stamps (-DBA_CHOL_STAMPS; they cost ~1.3k cycles per sub-panel sweep, so
// time with a build without them: tools/chol_bench_ns).  Factors a random SPD (n+1) x n trapezoid, times every block step
// with HIP events, prints the critical workgroup's phase cycles, solves and
// checks the solution against a CPU Cholesky.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DBA_CHOL_STAMPS -I bundleadjustment_amd/csrc \
//         tools/chol_bench.hip -o tools/chol_bench && tools/chol_bench 1194
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I bundleadjustment_amd/csrc tools/chol_bench.hip -o tools/chol_bench_ns
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <cstdio>
#include <algorithm>
#include <random>
#include <vector>

#include "ba_chol.hip"
#include "ba_chol_split.hip"
#ifndef CHOL_BENCH_NO_PERSIST   // (-DCHOL_BENCH_NO_PERSIST: a split-form-only build, e.g. with another LDS pad)
#include "ba_chol_persist.hip"
#else
namespace bahip {   // (referenced by ba_chol.hip's solver entry points, never called here)
void launch_chol_persist(double*, double*, int, int, double*, double*, unsigned*, unsigned, hipStream_t) { abort(); }
void launch_chol_persist_ov(const DevProblem&, const DevWork&, OvPlan&, double, int, hipStream_t, bool) { abort(); }
}  // namespace bahip
#endif

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

using namespace bahip;

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 1194;
  const int ld = n, nrows = n + 1;
  std::mt19937_64 rng(7);
  std::normal_distribution<double> N01;
  // S = G G^T / m + diag, lower part stored; rhs row random
  const int m = n + 16;
  std::vector<double> G((size_t)n * m);
  for (auto& v : G) v = N01(rng);
  std::vector<double> A((size_t)nrows * ld, 0.0), full((size_t)n * n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j <= i; ++j) {
      double s = 0;
      for (int k = 0; k < m; ++k) s += G[(size_t)i * m + k] * G[(size_t)j * m + k];
      s /= m;
      if (i == j) s += 1.0;
      A[(size_t)i * ld + j] = s;
      full[(size_t)i * n + j] = full[(size_t)j * n + i] = s;
    }
  std::vector<double> b(n);
  for (auto& v : b) v = N01(rng);
  for (int j = 0; j < n; ++j) A[(size_t)n * ld + j] = b[j];

  double *dA, *dL, *dV, *dS, *dy;
  const int T = (n + CB - 1) / CB;
  CK(hipMalloc(&dA, sizeof(double) * A.size()));
  CK(hipMalloc(&dL, sizeof(double) * A.size()));
  CK(hipMalloc(&dV, sizeof(double) * (size_t)(T + 1) * CB * CB));
  CK(hipMalloc(&dS, sizeof(double) * 64));
  CK(hipMalloc(&dy, sizeof(double) * n));
  double* dF;
  CK(hipMalloc(&dF, sizeof(double) * 2 * n));
  double* dU;   // the per-step form's update accumulator
  CK(hipMalloc(&dU, sizeof(double) * A.size()));
  // the split form's task table (null: the rank-64 form, BA_CHOL_RANK=0)
  int4* dtask = nullptr;
  std::vector<int4> tasks;
  std::vector<int> toff;
  if (T >= kCholSplitBlocks && chol_split_rank() > 0) {
    chol_split_tasks(n, tasks, toff);
    CK(hipMalloc(&dtask, sizeof(int4) * std::max<size_t>(tasks.size(), 1)));
    CK(hipMemcpy(dtask, tasks.data(), sizeof(int4) * tasks.size(), hipMemcpyHostToDevice));
    printf("task table: %zu tasks over %d steps (rank %d)\n", tasks.size(), T - 1, chol_split_rank());
  }
  // the fused form's V flags (epoch-tagged, one per block column)
  unsigned* dvf = nullptr;
  unsigned vepoch = 0;
  CK(hipMalloc(&dvf, sizeof(unsigned) * T));
  CK(hipMemset(dvf, 0, sizeof(unsigned) * T));
  unsigned* vf = dtask && chol_split_fused() ? dvf : nullptr;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 3; ++rep) {
    ++vepoch;   // (a fresh flag epoch per factorisation)
    CK(hipMemcpy(dA, A.data(), sizeof(double) * A.size(), hipMemcpyHostToDevice));
    CK(hipMemset(dS, 0, sizeof(double) * 64));
    double tot = 0;
    const bool verbose = rep == 2;
    for (int k = -1; k + 1 < T; ++k) {
      const int st = (k + 1) * CB;
      const int tr = (nrows - st + CB - 1) / CB, tc = (n - st + CB - 1) / CB;
      dim3 grid = k < 0 ? dim3(1, 1) : dim3(tc, tr);
      CK(hipEventRecord(e0));
      if (k >= 0 && T >= kCholSplitBlocks) {
        launch_chol_split_step(dA, dL, ld, n, k, grid.x, grid.y, dV, dS, dtask, toff.data(), vf, vepoch, 0);
      } else {
        hipLaunchKernelGGL(k_chol_step, grid, dim3(256), 0, 0, dA, dL, ld, n, k, dV, dS, dU);
      }
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      tot += ms;
#ifdef BA_CHOL_STAMPS
      unsigned long long st_h[64];
      CK(hipMemcpyFromSymbol(st_h, HIP_SYMBOL(g_stamps), sizeof(st_h)));
      if (verbose && (k < 2 || k == T / 2 || k + 2 == T))
        printf("step %3d grid %3dx%3d  %7.2f us | stage+gemm %6llu  init %6llu  factor %6llu  inverse %6llu  tail %6llu"
               "  write %6llu cycles\n",
               k, grid.x, grid.y, ms * 1e3, st_h[1] - st_h[0], st_h[2] - st_h[1], st_h[3] - st_h[2],
               st_h[4] - st_h[3], st_h[5] - st_h[4], st_h[6] - st_h[5]);
      if (verbose && k >= 0 && (k < 1 || k == T / 2))
        printf("    stage %llu  gemm1 %llu  store %llu  gemm2 %llu  rest %llu\n", st_h[20] - st_h[0], st_h[21] - st_h[20],
               st_h[22] - st_h[21], st_h[23] - st_h[22], st_h[1] - st_h[23]);
      if (verbose && k >= 0 && (k < 1 || k == T / 2))
        printf("    sub-panel 0: load %llu  columns %llu  scale+store %llu\n", st_h[30] - st_h[2], st_h[31] - st_h[30],
               st_h[10] - st_h[31]);
      if (verbose && (k < 1 || k == T / 2))
        printf("    inverse tail: diag16 (wave 0) %llu  wait for the sums %llu  fin + barrier %llu\n", st_h[40] - st_h[3],
               st_h[41] - st_h[40], st_h[4] - st_h[41]);
      if (verbose && (k < 1 || k == T / 2))
        printf("    sub-panels (sweep / update cycles): %llu/%llu %llu/%llu %llu/%llu %llu/%llu\n", st_h[10] - st_h[2],
               st_h[11] - st_h[10], st_h[12] - st_h[11], st_h[13] - st_h[12], st_h[14] - st_h[13], st_h[15] - st_h[14],
               st_h[16] - st_h[15], st_h[17] - st_h[16]);

#endif
    }
    CK(hipMemset(dF, 0, sizeof(double) * 2 * n));
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_back_flow, dim3(T), dim3(256), 0, 0, dA, dL, ld, n, dV, dy, dF, 1, dS);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float mb;
    CK(hipEventElapsedTime(&mb, e0, e1));
    if (verbose) printf("factor total %.1f us (%d steps), back-solve %.1f us\n", tot * 1e3, T, mb * 1e3);
  }
  if (T >= kCholSplitBlocks) {
    // the split form as the solver runs it: every step enqueued back to back
    for (int rep = 0; rep < 3; ++rep) {
    ++vepoch;   // (a fresh flag epoch per factorisation)
      CK(hipMemcpy(dA, A.data(), sizeof(double) * A.size(), hipMemcpyHostToDevice));
      CK(hipMemset(dS, 0, sizeof(double) * 64));
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(k_chol_step, dim3(1, 1), dim3(256), 0, 0, dA, dL, ld, n, -1, dV, dS, dU);
      for (int k = 0; k + 1 < T; ++k) {
        const int st = (k + 1) * CB;
        launch_chol_split_step(dA, dL, ld, n, k, (n - st + CB - 1) / CB, (nrows - st + CB - 1) / CB, dV, dS, dtask,
                               toff.data(), vf, vepoch, 0);
      }
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("factor streamed %.1f us (%s)\n", ms * 1e3,
             dtask ? (vf ? "scheduled tasks, fused panels" : "scheduled tasks") : "rank-64 form");
    }
    CK(hipMemset(dF, 0, sizeof(double) * 2 * n));
    hipLaunchKernelGGL(k_back_flow, dim3(T), dim3(256), 0, 0, dA, dL, ld, n, dV, dy, dF, 2, dS);
    CK(hipDeviceSynchronize());
  }
  if (T >= kCholSplitBlocks && dtask) {
    // the flow form: the whole factorisation as one dataflow launch; its
    // solution must equal the per-step forms' bit for bit
    std::vector<double> ys(n), yf(n);
    CK(hipMemcpy(ys.data(), dy, sizeof(double) * n, hipMemcpyDeviceToHost));
    std::vector<int4> flow;
    chol_flow_tasks(tasks, toff, flow);
    int4* dflow;
    unsigned* dtf;
    const int TRr = (nrows + CB - 1) / CB;
    CK(hipMalloc(&dflow, sizeof(int4) * flow.size()));
    CK(hipMemcpy(dflow, flow.data(), sizeof(int4) * flow.size(), hipMemcpyHostToDevice));
    CK(hipMalloc(&dtf, sizeof(unsigned) * (2 * TRr * T + 2)));
    CK(hipMemset(dtf, 0, sizeof(unsigned) * (2 * TRr * T + 2)));
    for (int rep = 0; rep < 3; ++rep) {
      ++vepoch;
      CK(hipMemcpy(dA, A.data(), sizeof(double) * A.size(), hipMemcpyHostToDevice));
      CK(hipMemset(dS, 0, sizeof(double) * 64));
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(k_chol_step, dim3(1, 1), dim3(256), 0, 0, dA, dL, ld, n, -1, dV, dS, dU);
      launch_chol_flow(dA, dL, ld, n, dV, dS, dflow, (int)flow.size(), dvf, dtf, dtf + (size_t)TRr * T, vepoch, 0);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      double sh[64];
      CK(hipMemcpy(sh, dS, sizeof(sh), hipMemcpyDeviceToHost));
      printf("factor flow %.1f us (one launch, %zu tasks)  spin %g bad %g\n", ms * 1e3, flow.size(), sh[SL_CHOL_SPIN],
             sh[SL_CHOL_BAD]);
    }
    CK(hipMemset(dF, 0, sizeof(double) * 2 * n));
    hipLaunchKernelGGL(k_back_flow, dim3(T), dim3(256), 0, 0, dA, dL, ld, n, dV, dy, dF, 3, dS);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(yf.data(), dy, sizeof(double) * n, hipMemcpyDeviceToHost));
    size_t diff = 0;
    for (int i = 0; i < n; ++i) diff += std::memcmp(&ys[i], &yf[i], 8) != 0;
    printf("flow vs per-step: y entries differing %zu\n", diff);
#ifdef BA_CHOL_FLOW_TRACE
    {
      // the last flow launch's task stamps + the list, for tools/flow_trace.py
      std::vector<unsigned long long> tr((size_t)(1 << 16) * 4);
      CK(hipMemcpyFromSymbol(tr.data(), HIP_SYMBOL(g_ftrace), sizeof(unsigned long long) * tr.size()));
      FILE* f = fopen(getenv("FLOW_TRACE_OUT") ? getenv("FLOW_TRACE_OUT") : "flow_trace.bin", "wb");
      std::vector<int4> lst(1, make_int4(1 << 21, 0, 0, 0));   // slot 0: the chain workgroup
      lst.insert(lst.end(), flow.begin(), flow.end());
      const unsigned nt = (unsigned)std::min<size_t>(lst.size(), 1 << 16);
      fwrite(&nt, 4, 1, f);
      fwrite(lst.data(), sizeof(int4), nt, f);
      fwrite(tr.data(), sizeof(unsigned long long) * 4, nt, f);
      std::vector<unsigned long long> ch(4096 * 6);
      CK(hipMemcpyFromSymbol(ch.data(), HIP_SYMBOL(g_fchain), sizeof(unsigned long long) * ch.size()));
      const unsigned nc = (unsigned)(T - 1);
      fwrite(&nc, 4, 1, f);
      fwrite(ch.data(), sizeof(unsigned long long) * 6, nc, f);
      fclose(f);
    }
#endif
    if (diff) return 5;
  }
  std::vector<double> y(n), Sh(64);
  CK(hipMemcpy(y.data(), dy, sizeof(double) * n, hipMemcpyDeviceToHost));
  // the persistent form (one launch, look-ahead): time it and check that it
  // reproduces the per-step factorisation bit for bit
#ifndef CHOL_BENCH_NO_PERSIST
  if (chol_persist_fits(0, n)) {
    unsigned* dflags;
    const int TR = (n + 1 + CB - 1) / CB;
    CK(hipMalloc(&dflags, sizeof(unsigned) * (T + TR * T)));
    CK(hipMemset(dflags, 0, sizeof(unsigned) * (T + TR * T)));
    std::vector<double> Lp(A.size()), Ls(A.size()), yp(n);
    CK(hipMemcpy(Ls.data(), dL, sizeof(double) * A.size(), hipMemcpyDeviceToHost));
    for (int rep = 0; rep < 5; ++rep) {
      CK(hipMemcpy(dA, A.data(), sizeof(double) * A.size(), hipMemcpyHostToDevice));
      CK(hipMemset(dS, 0, sizeof(double) * 64));
      CK(hipEventRecord(e0));
      launch_chol_persist(dA, dL, ld, n, dV, dS, dflags, 100 + rep, 0);
      CK(hipEventRecord(e1));
      hipLaunchKernelGGL(k_back_flow, dim3(T), dim3(256), 0, 0, dA, dL, ld, n, dV, dy, dF, 100 + rep, dS);
      CK(hipEventSynchronize(e1));
      float mp;
      CK(hipEventElapsedTime(&mp, e0, e1));
      CK(hipDeviceSynchronize());
      printf("persistent factor %.1f us (grid %d)\n", mp * 1e3, chol_persist_grid(n));
    }
#ifdef BA_CHOL_STAMPS
    {
      unsigned long long ps[64][8];
      CK(hipMemcpyFromSymbol(ps, HIP_SYMBOL(g_pstamps), sizeof(ps)));
      double avg[7] = {0, 0, 0, 0, 0, 0, 0};
      int cnt = 0;
      for (int c = 1; c < T && c < 64; ++c, ++cnt)
        for (int i = 0; i < 6; ++i) avg[i] += (double)(ps[c][i + 1] - ps[c][i]);
      const double tot = cnt ? (double)(ps[T - 1][6] - ps[1][0]) / cnt : 0.0;
      printf("persistent critical cycles per step (avg of %d): wait %.0f  fetch+V publish %.0f  P gemm+store %.0f"
             "  C col0 %.0f  factor %.0f  V clean+store %.0f  | step %.0f\n",
             cnt, avg[0] / cnt, avg[1] / cnt, avg[2] / cnt, avg[3] / cnt, avg[4] / cnt, avg[5] / cnt, tot);
      {
        // the next-panel tile's worker (J+1, J), its last update (k = J-1),
        // against the critical workgroup: cycles after V_{J-1}'s publish
        // stamp (ps[J-1][6]) and the hook's sub-panel 1 start of step J
        unsigned long long ws[64][6], pr[64][8];
        CK(hipMemcpyFromSymbol(ws, HIP_SYMBOL(g_wstamps), sizeof(ws)));
        CK(hipMemcpyFromSymbol(pr, HIP_SYMBOL(g_prt), sizeof(pr)));
        double av[5] = {0, 0, 0, 0, 0}, sp1 = 0, st = 0;
        int nn = 0;
        for (int J = 2; J + 1 < T && J < 64; ++J, ++nn) {
          for (int i = 0; i < 5; ++i) av[i] += 10.0 * (double)(long long)(ws[J][i] - pr[J - 1][6]);
          sp1 += 10.0 * (double)(long long)(pr[J][4] - pr[J - 1][6]);
          st += 10.0 * (double)(long long)(pr[J][5] - pr[J - 1][6]);
        }
        if (nn)
          printf("    panel-tile worker, last update, ns after V_{J-1}'s publish stamp (avg of %d): V seen %.0f  tiles in"
                 " LDS %.0f  strips %.0f  GEMM %.0f  published %.0f | critical: factor starts %.0f, ends %.0f\n",
                 nn, av[0] / nn, av[1] / nn, av[2] / nn, av[3] / nn, av[4] / nn, sp1 / nn, st / nn);
      }
      {
        unsigned long long es[64][2];
        CK(hipMemcpyFromSymbol(es, HIP_SYMBOL(g_estamps), sizeof(es)));
        double a0 = 0, a1 = 0, a2 = 0;
        int ne = 0;
        for (int c = 1; c + 2 < T && c < 63; ++c, ++ne) {
          a0 += (double)(es[c][0] - ps[c][5]);
          a1 += (double)(es[c][1] - es[c][0]);
          a2 += (double)(ps[c][6] - es[c][1]);
        }
        if (ne)
          printf("    V clean+store split (avg of %d): to end_step %.0f  V stores issued %.0f  diag fetch issue %.0f\n", ne,
                 a0 / ne, a1 / ne, a2 / ne);
      }
      int ph[4] = {0, 0, 0, 0};
      for (int c = 0; c + 1 < T && c < 64; ++c) ph[ps[c][7] & 3]++;
      printf("    next panel tile prefetched in sub-panel 1/2/3: %d/%d/%d, at the next step's start: %d\n", ph[1], ph[2],
             ph[3], ph[0]);
      unsigned long long st_h[64];
      CK(hipMemcpyFromSymbol(st_h, HIP_SYMBOL(g_stamps), sizeof(st_h)));
      printf("    persistent step %d: sub-panels (sweep / update) %llu/%llu %llu/%llu %llu/%llu %llu/%llu"
             "  inverse tail %llu/%llu/%llu\n", T / 2, st_h[10] - st_h[2], st_h[11] - st_h[10], st_h[12] - st_h[11],
             st_h[13] - st_h[12], st_h[14] - st_h[13], st_h[15] - st_h[14], st_h[16] - st_h[15], st_h[17] - st_h[16],
             st_h[40] - st_h[3], st_h[41] - st_h[40], st_h[4] - st_h[41]);
    }
#endif
    CK(hipMemcpy(Lp.data(), dL, sizeof(double) * A.size(), hipMemcpyDeviceToHost));
    CK(hipMemcpy(yp.data(), dy, sizeof(double) * n, hipMemcpyDeviceToHost));
    std::vector<double> Sp(64);
    CK(hipMemcpy(Sp.data(), dS, sizeof(double) * 64, hipMemcpyDeviceToHost));
    size_t ldiff = 0;
    for (int i = 0; i <= n; ++i)
      for (int j = 0; j < n && j <= i; ++j)
        if (i < n ? true : true) ldiff += std::memcmp(&Lp[(size_t)i * ld + j], &Ls[(size_t)i * ld + j], 8) != 0;
    size_t ydiff = 0;
    for (int i = 0; i < n; ++i) ydiff += std::memcmp(&yp[i], &y[i], 8) != 0;
    printf("persistent vs per-step: L entries differing %zu, y entries differing %zu, chol_bad=%g\n", ldiff, ydiff,
           Sp[SL_CHOL_BAD]);
    if (ydiff != 0 || Sp[SL_CHOL_BAD] != 0.0) return 4;
  } else {
    printf("persistent form: grid %d does not fit\n", chol_persist_grid(n));
  }
#endif
  CK(hipMemcpy(Sh.data(), dS, sizeof(double) * 64, hipMemcpyDeviceToHost));
  if (T >= 16 && getenv("CHOL_TASK_PROBE")) {
    // throughput of the split form's tile tasks alone (k_chol_upd with k = -2:
    // no critical workgroup): N distinct tiles, each A_IJ -= sum of R panels
    // (values: the factor above; A is overwritten, the checks are done)
    std::vector<int4> pt;
    for (int I = 8; I < T && (int)pt.size() < 4096; ++I)
      for (int J = 8; J <= I && (int)pt.size() < 4096; ++J) pt.push_back(make_int4(I, J, 0, 0));
    int4* dpt;
    CK(hipMalloc(&dpt, sizeof(int4) * pt.size()));
    for (int R : {1, 2, 4, 8})
      for (int N : {1, 64, 256, 512, 1024, 2048}) {
        if (N > (int)pt.size()) continue;
        for (auto& q : pt) { q.z = 0; q.w = R; }
        CK(hipMemcpy(dpt, pt.data(), sizeof(int4) * N, hipMemcpyHostToDevice));
        float best = 1e30f;
        for (int rep = 0; rep < 3; ++rep) {
          CK(hipEventRecord(e0));
          hipLaunchKernelGGL(k_chol_upd, dim3(1 + N), dim3(256), 0, 0, dA, dL, ld, n, -2, dV, dS, dpt, nullptr, 0u, 1u);
          CK(hipEventRecord(e1));
          CK(hipEventSynchronize(e1));
          float ms;
          CK(hipEventElapsedTime(&ms, e0, e1));
          best = std::min(best, ms);
        }
        const double fl = 2.0 * 64 * 64 * 64 * R * (double)N;
        printf("task probe: rank %d x64, %5d tiles: %8.1f us  %6.2f TF/s  %.2f us per tile-panel per CU\n", R, N,
               best * 1e3, fl / (best * 1e-3) / 1e12, best * 1e3 * std::min(N, 256) / ((double)N * R));
      }
  }
  // residual |S y - b| / |b|
  double rn = 0, bn = 0;
  for (int i = 0; i < n; ++i) {
    double s = 0;
    for (int j = 0; j < n; ++j) s += full[(size_t)i * n + j] * y[j];
    rn += (s - b[i]) * (s - b[i]);
    bn += b[i] * b[i];
  }
  printf("n=%d  relative residual %.3e  chol_bad=%g\n", n, std::sqrt(rn / bn), Sh[SL_CHOL_BAD]);
  return std::sqrt(rn / bn) < 1e-10 ? 0 : 3;
}

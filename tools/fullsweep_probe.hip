// fullsweep_probe.hip — the factor + inverse of one full 64 x 64 diagonal
// block of the dense Cholesky (ba_chol.h factor_invert_blk<1>) in isolation:
// one workgroup, s_memtime cycles over repeated factorisations, checked
// against a long-double CPU Cholesky.  Build it twice to compare the forms:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I bundleadjustment_amd/csrc tools/fullsweep_probe.hip \
//         -o tools/fullsweep_probe                         (the 64-column register sweep, default)
//   ... -DBA_CHOL_SWEEP64=0 -o tools/fullsweep_probe_sp    (four 16-column sub-panels)
// Cases: T = C final (the first block step), and T = A with the panel
// product Pc still to subtract (C = A - Pc Pc^T, every later step).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "ba_chol.h"

using namespace bahip;

__device__ __forceinline__ unsigned long long stamp() {
  unsigned long long t;
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

template <bool PC>
__global__ __launch_bounds__(256) void k_probe(const double* __restrict__ A, const double* __restrict__ Pg,
                                               double* __restrict__ out, unsigned long long* __restrict__ cyc,
                                               int reps) {
  __shared__ double T[CB][LDP];
  __shared__ double T0[CB][LDP];
  __shared__ double X[CB][LDP];
  __shared__ double Pc[CB][LDP];
  __shared__ CholLds W;
  const int tid = threadIdx.x;
  for (int e = tid; e < CB * CB; e += 256) T0[e / CB][e % CB] = (e % CB <= e / CB) ? A[e] : 0.0;
  __syncthreads();
  unsigned long long tot = 0, mn = ~0ull;
  for (int rep = 0; rep < reps; ++rep) {
    for (int e = tid; e < CB * CB; e += 256) {
      T[e / CB][e % CB] = T0[e / CB][e % CB];
      Pc[e / CB][e % CB] = Pg[e];
    }
    if (tid == 0) W.bad = 0;
    __syncthreads();
    if (PC) mfma_xxT_col0(Pc, T);   // column 0 of C = A - Pc Pc^T, as the callers do
    __syncthreads();
    const unsigned long long t0 = stamp();
    factor_invert_blk<1>(T, X, Pc, W, CB, CB, PC ? Pc : nullptr);
    const unsigned long long t1 = stamp();
    tot += t1 - t0;
    mn = t1 - t0 < mn ? t1 - t0 : mn;
    __syncthreads();
  }
  for (int e = tid; e < CB * CB; e += 256) out[e] = T[e / CB][e % CB];
  for (int e = tid; e < CB * CB; e += 256) out[4096 + e] = X[e / CB][e % CB];
  if (tid == 0) { cyc[0] = tot / reps; cyc[1] = mn; cyc[2] = W.bad; }
}

int main() {
  std::mt19937_64 rng(3);
  std::normal_distribution<double> N01;
  std::vector<double> G(64 * 80), A(64 * 64), Pm(64 * 64);
  for (auto& v : G) v = N01(rng);
  for (int i = 0; i < 64; ++i)
    for (int j = 0; j < 64; ++j) {
      double s = 0;
      for (int k = 0; k < 80; ++k) s += G[i * 80 + k] * G[j * 80 + k];
      A[i * 64 + j] = s / 80 + (i == j ? 1.0 : 0.0);
    }
  for (auto& v : Pm) v = 0.05 * N01(rng);
  double *dA, *dP, *dO;
  unsigned long long* dC;
  if (hipMalloc(&dA, 8 * 4096) != hipSuccess || hipMalloc(&dP, 8 * 4096) != hipSuccess ||
      hipMalloc(&dO, 16 * 4096) != hipSuccess || hipMalloc(&dC, 32) != hipSuccess)
    return 1;
  (void)hipMemcpy(dA, A.data(), 8 * 4096, hipMemcpyHostToDevice);
  (void)hipMemcpy(dP, Pm.data(), 8 * 4096, hipMemcpyHostToDevice);
  std::vector<double> o(2 * 4096);
  auto run = [&](auto kern, bool pc, const char* name) {
    // CPU: C = A - Pc Pc^T (pc), its Cholesky in long double
    std::vector<long double> C(64 * 64), Lc(64 * 64, 0.0L);
    for (int i = 0; i < 64; ++i)
      for (int j = 0; j < 64; ++j) {
        long double s = A[i * 64 + j];
        if (pc)
          for (int k = 0; k < 64; ++k) s -= (long double)Pm[i * 64 + k] * Pm[j * 64 + k];
        C[i * 64 + j] = s;
      }
    for (int j = 0; j < 64; ++j) {
      long double s = C[j * 64 + j];
      for (int k = 0; k < j; ++k) s -= Lc[j * 64 + k] * Lc[j * 64 + k];
      Lc[j * 64 + j] = sqrtl(s);
      for (int i = j + 1; i < 64; ++i) {
        long double t = C[i * 64 + j];
        for (int k = 0; k < j; ++k) t -= Lc[i * 64 + k] * Lc[j * 64 + k];
        Lc[i * 64 + j] = t / Lc[j * 64 + j];
      }
    }
    hipLaunchKernelGGL(kern, dim3(1), dim3(256), 0, 0, dA, dP, dO, dC, 64);
    if (hipDeviceSynchronize() != hipSuccess) { printf("%s: launch failed\n", name); return; }
    unsigned long long c[3];
    (void)hipMemcpy(c, dC, 24, hipMemcpyDeviceToHost);
    (void)hipMemcpy(o.data(), dO, 16 * 4096, hipMemcpyDeviceToHost);
    double el = 0, ei = 0;
    for (int i = 0; i < 64; ++i)
      for (int j = 0; j <= i; ++j) el = std::fmax(el, std::fabs((double)(o[i * 64 + j] - Lc[i * 64 + j])));
    for (int i = 0; i < 64; ++i)
      for (int j = 0; j <= i; ++j) {   // | X L - I |
        long double s = 0;
        for (int k = j; k <= i; ++k) s += (long double)o[4096 + i * 64 + k] * Lc[k * 64 + j];
        ei = std::fmax(ei, std::fabs((double)(s - (i == j ? 1.0L : 0.0L))));
      }
    printf("%-44s avg %7llu  min %7llu cycles  max|L - L_cpu| %.2e  max|XL - I| %.2e  bad %llu\n", name, c[0], c[1],
           el, ei, c[2]);
  };
  const char* form = BA_CHOL_SWEEP64 ? "register sweep" : "sub-panels";
  char n0[96], n1[96];
  snprintf(n0, sizeof n0, "%s, C final", form);
  snprintf(n1, sizeof n1, "%s, C = A - Pc Pc^T in the factor", form);
  run(k_probe<false>, false, n0);
  run(k_probe<true>, true, n1);
  return 0;
}

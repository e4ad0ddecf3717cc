// sweep_probe.hip — the Cholesky sub-panel sweep (ba_chol.h panel_sweep) in
// isolation: one workgroup, wave 0 sweeps the 64 x 16 sub-panel 0 of an SPD
// 64 x 64 block (row load, 8 pair steps, scaling + store), s_memtime cycles
// per sweep; waves 1..3 idle, or streaming MFMA operand reads from LDS
// (contention as in the product's first sub-panel).  Variants of the sweep's
// schedule are compared against the product code; every variant must leave
// the same L columns.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DBA_CHOL_STAMPS -I bundleadjustment_amd/csrc tools/sweep_probe.hip \
//         -o tools/sweep_probe   (BA_CHOL_STAMPS: the sweep's own column-loop stamps)
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "ba_chol.h"

using namespace bahip;

// V1: panel_sweep without the scheduling barriers (the compiler interleaves
// the remaining-column updates with the next pair's pivot chain)
__device__ __forceinline__ void panel_sweep_free(double (*T)[LDP], CholLds& W, int c0, int b, int m) {
  const int r = threadIdx.x & 63;
  double a[16];
  {
    const double2* src = reinterpret_cast<const double2*>(&T[r][c0]);
    double2 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = src[k];
#pragma unroll
    for (int cc = 0; cc < 16; ++cc) {
      const int t = c0 + cc;
      const double x = (cc & 1) ? v[cc >> 1].y : v[cc >> 1].x;
      a[cc] = (r >= c0 && r < m && t < b && (t <= r || r >= b)) ? x : 0.0;
    }
  }
  W.colp[0][r] = make_double2(a[0], a[1]);
  double2 q0 = W.colp[0][c0], q1 = W.colp[0][c0 + 1];
  double2 ct[16];
#pragma unroll
  for (int t = 2; t < 16; ++t) ct[t] = W.colp[0][c0 + t];
#pragma unroll
  for (int jj = 0; jj < 16; jj += 2) {
    const int j = c0 + jj;
    if (j + 1 >= b) break;
    const int buf = (jj >> 1) & 1;
    const double d0 = q0.x, e = q1.x, d1 = q1.y;
    const double rdet = recip(d0 * d1 - e * e);
    const double rd0 = recip(d0);
    const bool row = r > j + 1 && r < m;
    const double u0 = a[jj], u1 = a[jj + 1];
    const double f0 = row ? fma(u0, d1, -u1 * e) * rdet : 0.0;
    const double f1 = row ? fma(u1, d0, -u0 * e) * rdet : 0.0;
    if (jj + 2 < 16) {
      a[jj + 2] = fma(-f1, ct[jj + 2].y, fma(-f0, ct[jj + 2].x, a[jj + 2]));
      a[jj + 3] = fma(-f1, ct[jj + 3].y, fma(-f0, ct[jj + 3].x, a[jj + 3]));
      W.colp[buf ^ 1][r] = make_double2(a[jj + 2], a[jj + 3]);
      __builtin_amdgcn_wave_barrier();
      const double2 q0n = W.colp[buf ^ 1][c0 + jj + 2], q1n = W.colp[buf ^ 1][c0 + jj + 3];
      double2 ctn[16];
#pragma unroll
      for (int t = jj + 4; t < 16; ++t) ctn[t] = W.colp[buf ^ 1][c0 + t];
#pragma unroll
      for (int t = jj + 4; t < 16; ++t) a[t] = fma(-f1, ct[t].y, fma(-f0, ct[t].x, a[t]));
      q0 = q0n;
      q1 = q1n;
#pragma unroll
      for (int t = jj + 4; t < 16; ++t) ct[t] = ctn[t];
    }
    if (r > j && r < m) a[jj + 1] -= u0 * (e * rd0);
  }
  double d_own = 1.0;
#pragma unroll
  for (int cc = 0; cc < 16; ++cc)
    if (r == c0 + cc) d_own = a[cc];
  const bool own = r >= c0 && r < c0 + 16;
  if (own && r < b && !(d_own > 0.0 && isfinite(d_own))) W.bad = 1;
  const double rs_own = rsqrt_nr(d_own);
  if (own) W.rsv[r] = rs_own;
  __builtin_amdgcn_wave_barrier();
  double rs[16];
  {
    const double2* src = reinterpret_cast<const double2*>(&W.rsv[c0]);
#pragma unroll
    for (int k = 0; k < 8; ++k) { const double2 x = src[k]; rs[2 * k] = x.x; rs[2 * k + 1] = x.y; }
  }
  if (r >= c0 && r < m) {
    double2* dst = reinterpret_cast<double2*>(&T[r][c0]);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      double lv[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int cc = 2 * k + h, t = c0 + cc;
        lv[h] = (t < b && t <= r) ? a[cc] * rs[cc] : 0.0;
      }
      dst[k] = make_double2(lv[0], lv[1]);
    }
  }
}

// V2: the product sweep with c0 / b / m as run-time values (as in
// factor_invert_blk's sub-panel loop) instead of compile-time constants
template <int V, bool BUSY>
__global__ __launch_bounds__(256) void k_sweep(const double* __restrict__ A, double* __restrict__ out,
                                               unsigned long long* __restrict__ cyc, int reps, int rc0, int rb,
                                               int rm) {
  __shared__ double T[CB][LDP];
  __shared__ double T0[CB][LDP];
  __shared__ double M[CB][LDP];
  __shared__ CholLds W;
  const int tid = threadIdx.x, w = tid >> 6;
  for (int e = tid; e < CB * CB; e += 256) { T0[e / CB][e % CB] = A[e]; M[e / CB][e % CB] = A[e] * 1e-3; }
  __syncthreads();
  unsigned long long tot = 0, mn = ~0ull;
  d4 sink = {0, 0, 0, 0};
  for (int rep = 0; rep < reps; ++rep) {
    for (int e = tid; e < CB * CB; e += 256) T[e / CB][e % CB] = T0[e / CB][e % CB];
    __syncthreads();
    if (w == 0) {
      unsigned long long t0, t1;
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
      if (V == 0) panel_sweep(T, W, 0, CB, CB);
      else if (V == 1) panel_sweep_free(T, W, 0, CB, CB);
      else panel_sweep(T, W, rc0, rb, rm);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
      tot += t1 - t0;
      mn = t1 - t0 < mn ? t1 - t0 : mn;
    } else if (BUSY) {   // the product's mfma_xxT_rest-like LDS operand stream (6 tiles x 16 MFMAs)
      for (int h = 0; h < 2; ++h) sink += mfma_tile<64>(sink, M, 16 * w, 0, M, 16 * ((w + h) & 3), 0, 1.0);
    }
    __syncthreads();
  }
  for (int e = tid; e < CB * CB; e += 256) out[e] = T[e / CB][e % CB] + (w == 9 ? sink[0] : 0.0);
  if (tid == 0) { cyc[0] = tot / reps; cyc[1] = mn; }
}

int main() {
  std::mt19937_64 rng(3);
  std::normal_distribution<double> N01;
  std::vector<double> G(64 * 80), A(64 * 64);
  for (auto& v : G) v = N01(rng);
  for (int i = 0; i < 64; ++i)
    for (int j = 0; j < 64; ++j) {
      double s = 0;
      for (int k = 0; k < 80; ++k) s += G[i * 80 + k] * G[j * 80 + k];
      A[i * 64 + j] = s / 80 + (i == j ? 1.0 : 0.0);
    }
  double *dA, *dO;
  unsigned long long* dC;
  hipMalloc(&dA, 8 * 4096); hipMalloc(&dO, 8 * 4096); hipMalloc(&dC, 16);
  hipMemcpy(dA, A.data(), 8 * 4096, hipMemcpyHostToDevice);
  std::vector<double> ref(4096), o(4096);
  auto run = [&](auto kern, const char* name, bool check, int rc0 = 0) {
    hipLaunchKernelGGL(kern, dim3(1), dim3(256), 0, 0, dA, dO, dC, 64, rc0, 64, 64);
    hipDeviceSynchronize();
    unsigned long long c[2];
    hipMemcpy(c, dC, 16, hipMemcpyDeviceToHost);
    hipMemcpy(o.data(), dO, 8 * 4096, hipMemcpyDeviceToHost);
    if (!check) ref = o;
    size_t diff = 0;
    for (int i = 0; i < 64; ++i)
      for (int j = 0; j < 16; ++j) diff += check && std::memcmp(&o[i * 64 + j], &ref[i * 64 + j], 8) != 0;
    unsigned long long st[64];
    hipMemcpyFromSymbol(st, HIP_SYMBOL(g_stamps), sizeof(st));
    printf("%-34s avg %6llu  min %6llu cycles per 16-column sweep (columns %llu)  L entries differing from V0: %zu\n",
           name, c[0], c[1], st[31] - st[30], diff);
  };
  run(k_sweep<0, false>, "V0 product, other waves idle", false);
  run(k_sweep<0, true>, "V0 product, MFMA LDS stream", true);
  run(k_sweep<1, false>, "V1 no sched barriers, idle", true);
  run(k_sweep<1, true>, "V1 no sched barriers, MFMA stream", true);
  run(k_sweep<2, false>, "V2 run-time c0/b/m, idle", true);
  run(k_sweep<2, true>, "V2 run-time c0/b/m, MFMA stream", true);
  run(k_sweep<2, false>, "V2 run-time c0=32, idle", false, 32);
  return 0;
}

// fullsweep_probe.hip — the 64-column diagonal-block factor of the dense
// Cholesky (ba_chol.h) in isolation: one workgroup, s_memtime cycles.
//   V0  the product factor_invert_blk<1> (four 16-column sub-panel sweeps by
//       wave 0, MFMA trailing updates by all waves, the inverse pipelined)
//   V1  ONE 64-column register sweep by wave 0 (lane = row, the whole row in
//       registers, 2 x 2 pivot pairs, pivot columns broadcast through LDS),
//       the scaled L columns stored as each pair completes; no inverse
//   V2  V1 + the inverse X = L^-1 by waves 1..3 behind the sweep (progress
//       counter in LDS), last row block after the sweep
// Every variant is checked against a CPU Cholesky of the same block.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I bundleadjustment_amd/csrc tools/fullsweep_probe.hip \
//         -o tools/fullsweep_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <utility>
#include <vector>

#include "ba_chol.h"

using namespace bahip;

#ifndef FS_CHUNK
#define FS_CHUNK 8
#endif

__device__ __forceinline__ unsigned long long stamp() {
  unsigned long long t;
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

// the whole 64 x 64 lower block, one wave: lane r = row r.  The pair steps
// are instantiated per JJ (compile-time register indices throughout).
// Pair JJ (pivot columns JJ, JJ+1; f0, f1 of this lane formed in pair JJ-2):
//   A  the next pair's two columns (the chain), its pivot block by readlane,
//      those columns published to LDS, the next pair's chain operands read
//   B  the next pair's reciprocals and f0, f1 (off this pair's bulk)
//   C  the remaining columns, FS_CHUNK at a time, reads one chunk ahead
// with scheduling barriers between the chunks, so the reads in flight stay
// bounded (otherwise every read of the sweep is hoisted: 512 VGPRs + spills).
// reads stay in their chunk: a compiler memory fence (the selection DAG
// otherwise hoists every LDS read of the unrolled sweep) plus a scheduling
// barrier for the machine scheduler
__device__ __forceinline__ void fs_fence() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
struct FsState {
  double a[64];
  double2 c2, c3;      // this pair's chain operands: columns JJ+2, JJ+3 of the pivot rows
  double f0, f1;       // this lane's multipliers of this pair
  double d0, e, d1;    // this pair's pivot block
};
template <int JJ>
__device__ __forceinline__ void fs_pair(FsState& s, double (*T)[LDP], CholLds& W, double2 (*colp)[CB], int r,
                                        bool& bad, int* prog) {
  constexpr int buf = (JJ >> 1) & 1;
  constexpr int NB = (64 - (JJ + 4) + FS_CHUNK - 1) / FS_CHUNK;   // bulk chunks (0 on the last two pairs)
  const double f0 = s.f0, f1 = s.f1, u0 = s.a[JJ];
  const double d0j = s.d0, ej = s.e;
  double2 ct[2][FS_CHUNK];
  if constexpr (JJ + 2 < 64) {
    s.a[JJ + 2] = fma(-f1, s.c2.y, fma(-f0, s.c2.x, s.a[JJ + 2]));
    s.a[JJ + 3] = fma(-f1, s.c3.y, fma(-f0, s.c3.x, s.a[JJ + 3]));
    s.d0 = readlane_f64(s.a[JJ + 2], JJ + 2);
    s.e = readlane_f64(s.a[JJ + 2], JJ + 3);
    s.d1 = readlane_f64(s.a[JJ + 3], JJ + 3);
    W.colp[buf ^ 1][r] = make_double2(s.a[JJ + 2], s.a[JJ + 3]);
    __builtin_amdgcn_wave_barrier();
    if constexpr (JJ + 4 < 64) {
      s.c2 = colp[buf ^ 1][JJ + 4];
      s.c3 = colp[buf ^ 1][JJ + 5];
    }
    if constexpr (NB > 0) {
#pragma unroll
      for (int q = 0; q < FS_CHUNK; ++q)
        if (JJ + 4 + q < 64) ct[0][q] = colp[buf][JJ + 4 + q];
    }
    fs_fence();
    // B: the next pair's scalars
    {
      const double rdet = recip(s.d0 * s.d1 - s.e * s.e);
      const double un0 = s.a[JJ + 2], un1 = s.a[JJ + 3];
      s.f0 = fma(un0, s.d1, -un1 * s.e) * rdet;
      s.f1 = fma(un1, s.d0, -un0 * s.e) * rdet;
    }
    // C
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const int t0 = JJ + 4 + k * FS_CHUNK;
      if (k + 1 < NB) {
#pragma unroll
        for (int q = 0; q < FS_CHUNK; ++q)
          if (t0 + FS_CHUNK + q < 64) ct[(k + 1) & 1][q] = colp[buf][t0 + FS_CHUNK + q];
      }
#pragma unroll
      for (int q = 0; q < FS_CHUNK; ++q)
        if (t0 + q < 64) {
          s.a[t0 + q] = fma(-f1, ct[k & 1][q].y, fma(-f0, ct[k & 1][q].x, s.a[t0 + q]));
          asm volatile("" : "+v"(s.a[t0 + q]));   // (pins the update into this chunk)
        }
      fs_fence();
    }
  }
  const double rd0j = recip(d0j);
  s.a[JJ + 1] -= u0 * (ej * rd0j);
  // columns JJ, JJ+1 are final: scaled into T (off the chain)
  const double dn = readlane_f64(s.a[JJ + 1], JJ + 1);
  bad |= !(d0j > 0.0 && isfinite(d0j)) || !(dn > 0.0 && isfinite(dn));
  const double rs0 = rsqrt_nr(d0j), rs1 = rsqrt_nr(dn);
  *reinterpret_cast<double2*>(&T[r][JJ]) =
      make_double2(JJ <= r ? s.a[JJ] * rs0 : 0.0, JJ + 1 <= r ? s.a[JJ + 1] * rs1 : 0.0);
  if (r == 0) *reinterpret_cast<double2*>(&W.rsv[JJ]) = make_double2(rs0, rs1);
  // every 16 columns: the row block's L columns and scalings are in LDS
  // (LDS operations of one wave complete in order)
  if constexpr ((JJ + 2) % 16 == 0) {
    if (prog != nullptr && r == 0) *reinterpret_cast<volatile int*>(prog) = JJ + 2;
  }
}
template <int... P>
__device__ __forceinline__ void fs_pairs(FsState& s, double (*T)[LDP], CholLds& W, double2 (*colp)[CB], int r,
                                         bool& bad, int* prog, std::integer_sequence<int, P...>) {
  (fs_pair<2 * P>(s, T, W, colp, r, bad, prog), ...);
}
__device__ __forceinline__ void full_sweep64(double (*T)[LDP], CholLds& W, int* prog = nullptr) {
  const int r = ctid() & 63;
  int zo = 0;
  asm volatile("" : "+v"(zo));
  double2 (*colp)[CB] = reinterpret_cast<double2 (*)[CB]>(&W.colp[0][zo]);
  FsState s;
  {
    const double2* src = reinterpret_cast<const double2*>(&T[r][0]);
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      const double2 v = src[k];
      s.a[2 * k] = v.x;
      s.a[2 * k + 1] = v.y;
    }
  }
  W.colp[0][r] = make_double2(s.a[0], s.a[1]);
  __builtin_amdgcn_wave_barrier();
  s.c2 = colp[0][2];
  s.c3 = colp[0][3];
  s.d0 = readlane_f64(s.a[0], 0);
  s.e = readlane_f64(s.a[0], 1);
  s.d1 = readlane_f64(s.a[1], 1);
  {
    const double rdet = recip(s.d0 * s.d1 - s.e * s.e);
    s.f0 = fma(s.a[0], s.d1, -s.a[1] * s.e) * rdet;
    s.f1 = fma(s.a[1], s.d0, -s.a[0] * s.e) * rdet;
  }
  bool bad = false;
  fs_pairs(s, T, W, colp, r, bad, prog, std::make_integer_sequence<int, 32>{});
  if (bad && r == 0) W.bad = 1;
}

// waves 1..3: X = L^-1 row block by row block behind the sweep
__device__ __forceinline__ void wait_lds(int* p, int v) {
  while (__builtin_amdgcn_readfirstlane(*reinterpret_cast<volatile int*>(p)) < v) __builtin_amdgcn_s_sleep(1);
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void set_lds(int* p, int v) {
  asm volatile("" ::: "memory");
  if ((ctid() & 63) == 0) *reinterpret_cast<volatile int*>(p) = v;
}
template <int ZLD>
__device__ __forceinline__ void fs_inverse(double (*T)[LDP], double (*X)[LDP], double (*Z)[ZLD], CholLds& W,
                                           int* prog, int* fl) {
  const int w = cwave();
  if (w == 1) {
    wait_lds(prog, 16);
    diag_inverse16(T, W.rsv, X, 0, CB);
    set_lds(&fl[0], 1);
    wait_lds(prog, 32);
    diag_inverse16(T, W.rsv, X, 1, CB);
    inv_offdiag_sum(T, X, Z, 1, 0, 0);
    inv_offdiag_fin(X, Z, 1, 0, 0);
    set_lds(&fl[1], 1);
    wait_lds(prog, 64);
    diag_inverse16(T, W.rsv, X, 3, CB);
  } else if (w == 2) {
    wait_lds(prog, 48);
    diag_inverse16(T, W.rsv, X, 2, CB);
    wait_lds(&fl[1], 1);
    inv_offdiag_sum(T, X, Z, 2, 0, 16);
    inv_offdiag_fin(X, Z, 2, 0, 16);
    inv_offdiag_sum(T, X, Z, 2, 1, 16);
    inv_offdiag_fin(X, Z, 2, 1, 16);
    set_lds(&fl[2], 1);
  } else if (w == 3) {
    wait_lds(&fl[2], 1);
    for (int q = 0; q < 3; ++q) inv_offdiag_sum(T, X, Z, 3, q, 16 + 16 * q);
  }
}
// the tail (after a barrier): X_3q = -X_33 Z_q by waves 1..3
template <int ZLD>
__device__ __forceinline__ void fs_inverse_fin(double (*X)[LDP], double (*Z)[ZLD]) {
  const int w = cwave();
  if (w >= 1) inv_offdiag_fin(X, Z, 3, w - 1, 16 * w);
}

template <int V>
__global__ __launch_bounds__(256) void k_probe(const double* __restrict__ A, double* __restrict__ out,
                                               unsigned long long* __restrict__ cyc, int reps) {
  __shared__ double T[CB][LDP];
  __shared__ double T0[CB][LDP];
  __shared__ double X[CB][LDP];
  __shared__ double Z[CB][LDP];
  __shared__ CholLds W;
  __shared__ int prog[1], fl[4];
  const int tid = threadIdx.x, w = tid >> 6;
  for (int e = tid; e < CB * CB; e += 256) T0[e / CB][e % CB] = (e % CB <= e / CB) ? A[e] : 0.0;
  __syncthreads();
  unsigned long long tot = 0, mn = ~0ull;
  for (int rep = 0; rep < reps; ++rep) {
    for (int e = tid; e < CB * CB; e += 256) T[e / CB][e % CB] = T0[e / CB][e % CB];
    if (tid == 0) { W.bad = 0; prog[0] = 0; fl[0] = fl[1] = fl[2] = fl[3] = 0; }
    __syncthreads();
    const unsigned long long t0 = stamp();
    if (V == 0) {
      factor_invert_blk<1>(T, X, Z, W, CB, CB);
    } else if (V == 1) {
      if (w == 0) full_sweep64(T, W);
      __syncthreads();
    } else {
      if (w == 0) full_sweep64(T, W, prog);
      else fs_inverse(T, X, Z, W, prog, fl);
      __syncthreads();
      fs_inverse_fin(X, Z);
      __syncthreads();
    }
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
  std::vector<double> G(64 * 80), A(64 * 64);
  for (auto& v : G) v = N01(rng);
  for (int i = 0; i < 64; ++i)
    for (int j = 0; j < 64; ++j) {
      double s = 0;
      for (int k = 0; k < 80; ++k) s += G[i * 80 + k] * G[j * 80 + k];
      A[i * 64 + j] = s / 80 + (i == j ? 1.0 : 0.0);
    }
  // CPU Cholesky (long double)
  std::vector<long double> Lc(64 * 64, 0.0L);
  for (int j = 0; j < 64; ++j) {
    long double s = A[j * 64 + j];
    for (int k = 0; k < j; ++k) s -= Lc[j * 64 + k] * Lc[j * 64 + k];
    Lc[j * 64 + j] = sqrtl(s);
    for (int i = j + 1; i < 64; ++i) {
      long double t = A[i * 64 + j];
      for (int k = 0; k < j; ++k) t -= Lc[i * 64 + k] * Lc[j * 64 + k];
      Lc[i * 64 + j] = t / Lc[j * 64 + j];
    }
  }
  double *dA, *dO;
  unsigned long long* dC;
  hipMalloc(&dA, 8 * 4096);
  hipMalloc(&dO, 16 * 4096);
  hipMalloc(&dC, 32);
  hipMemcpy(dA, A.data(), 8 * 4096, hipMemcpyHostToDevice);
  std::vector<double> o(2 * 4096);
  auto run = [&](auto kern, const char* name, bool inv) {
    hipLaunchKernelGGL(kern, dim3(1), dim3(256), 0, 0, dA, dO, dC, 64);
    if (hipDeviceSynchronize() != hipSuccess) { printf("%s: launch failed\n", name); return; }
    unsigned long long c[3];
    hipMemcpy(c, dC, 24, hipMemcpyDeviceToHost);
    hipMemcpy(o.data(), dO, 16 * 4096, hipMemcpyDeviceToHost);
    double el = 0, ei = 0;
    for (int i = 0; i < 64; ++i)
      for (int j = 0; j <= i; ++j) el = std::fmax(el, std::fabs((double)(o[i * 64 + j] - Lc[i * 64 + j])));
    if (inv) {   // | X L - I |
      for (int i = 0; i < 64; ++i)
        for (int j = 0; j <= i; ++j) {
          long double s = 0;
          for (int k = j; k <= i; ++k) s += (long double)o[4096 + i * 64 + k] * Lc[k * 64 + j];
          ei = std::fmax(ei, std::fabs((double)(s - (i == j ? 1.0L : 0.0L))));
        }
    }
    printf("%-40s avg %7llu  min %7llu cycles  max|L - L_cpu| %.2e  max|XL - I| %.2e  bad %llu\n", name, c[0], c[1],
           el, ei, c[2]);
  };
  run(k_probe<0>, "V0 product factor + inverse", true);
  run(k_probe<1>, "V1 64-column register sweep (no inverse)", false);
  run(k_probe<2>, "V2 register sweep + pipelined inverse", true);
  return 0;
}

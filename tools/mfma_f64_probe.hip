// mfma_f64_probe.hip — issue rate of v_mfma_f64_16x16x4_f64 on gfx950 with
// NACC independent accumulators per wave (registers only, no memory in the
// loop), for 1..4 waves per SIMD and the whole chip.  Sizes the split
// Cholesky's tile GEMMs (bundleadjustment_amd/csrc/ba_chol_split.hip).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I bundleadjustment_amd/csrc tools/mfma_f64_probe.hip -o tools/mfma_f64_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(1024) void k_probe(double* out, int iters) {
  d4 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = d4{0.0, 0.0, 0.0, 0.0};
  double x = 1.0 + 1e-9 * threadIdx.x, y = 1.0 - 1e-9 * threadIdx.x;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc[i], 0, 0, 0);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NACC>
static void run(double* d, int blocks, int threads, int iters) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(k_probe<NACC>, dim3(blocks), dim3(threads), 0, 0, d, iters);
  hipEventRecord(a);
  hipLaunchKernelGGL(k_probe<NACC>, dim3(blocks), dim3(threads), 0, 0, d, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double mf = (double)blocks * (threads / 64) * iters * NACC;   // MFMAs
  const double fl = mf * 2048.0;
  printf("NACC %2d  blocks %5d x %4d threads: %8.3f ms  %7.2f TF/s  %.1f ns per MFMA per wave\n", NACC, blocks, threads,
         ms, fl / ms / 1e9, ms * 1e6 / ((double)iters * NACC));
}

int tile_main();
int main() {
  double* d;
  hipMalloc(&d, sizeof(double) * 1024 * 4096);
  const int it = 4000;
  // one workgroup of 4 waves (one per SIMD) on one CU
  run<4>(d, 1, 256, it);
  run<8>(d, 1, 256, it);
  run<16>(d, 1, 256, it);
  // two waves per SIMD
  run<4>(d, 1, 512, it);
  // whole chip: 256 CUs x 4 SIMDs x 1 / 2 waves
  run<4>(d, 256, 256, it);
  run<8>(d, 256, 256, it);
  run<4>(d, 512, 256, it);
  run<4>(d, 1024, 256, it);
  run<8>(d, 1024, 256, it);
  return tile_main();
}

// ---- the split Cholesky tile GEMM (ba_chol.h mfma_xyT_64_add) in isolation:
// MODE 0: the MFMA loop alone over LDS tiles; 1: + the per-panel LDS put of
// two register-staged tiles and its two barriers; LDS sized as k_chol_upd
// (79 KB: two workgroups per CU).
#include "ba_chol.h"
template <int MODE>
__global__ __launch_bounds__(256) void k_tile_loop(double* out, int reps) {
  __shared__ double S0[bahip::CB][bahip::LDP];
  __shared__ double S1[bahip::CB][bahip::LDP];
  __shared__ double Zs[bahip::CB][18];
  for (int e = threadIdx.x; e < bahip::CB * bahip::LDP; e += 256) {
    (&S0[0][0])[e] = 1.0 + 1e-6 * e;
    (&S1[0][0])[e] = 1.0 - 1e-6 * e;
  }
  if (threadIdx.x < bahip::CB) Zs[threadIdx.x][0] = 0.0;
  bahip::TileRaw t;
  for (int it = 0; it < 8; ++it) t.v[it] = make_double2(1.0 + threadIdx.x, 2.0);
  t.mask = 0xffffu;
  __syncthreads();
  bahip::d4 acc[2][2];
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b) acc[a][b] = bahip::d4{0.0, 0.0, 0.0, 0.0};
  for (int r = 0; r < reps; ++r) {
    if (MODE == 1) {
      __syncthreads();
      bahip::tile_put_masked(S0, t);
      bahip::tile_put_masked(S1, t);
      __syncthreads();
    }
    bahip::mfma_xyT_64_add(S0, S1, acc);
  }
  double s = Zs[0][0];
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b) s += acc[a][b][0] + acc[a][b][1] + acc[a][b][2] + acc[a][b][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
template <int MODE>
static void run_tile(double* d, int blocks, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(k_tile_loop<MODE>, dim3(blocks), dim3(256), 0, 0, d, reps);
  hipEventRecord(a);
  hipLaunchKernelGGL(k_tile_loop<MODE>, dim3(blocks), dim3(256), 0, 0, d, reps);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double fl = 2.0 * 64 * 64 * 64 * (double)reps * blocks;
  printf("tile loop mode %d (%s), %4d workgroups x %d panels: %8.3f ms  %6.2f TF/s  %.2f us per panel per workgroup\n",
         MODE, MODE ? "MFMA + put" : "MFMA only", blocks, reps, ms, fl / ms / 1e9, ms * 1e3 / reps);
}
int tile_main() {
  double* d;
  hipMalloc(&d, sizeof(double) * 256 * 4096);
  for (int blocks : {1, 256, 512}) {
    run_tile<0>(d, blocks, 200);
    run_tile<1>(d, blocks, 200);
  }
  return 0;
}

// mfma_f64_probe.hip — issue rate of v_mfma_f64_16x16x4_f64 on gfx950 with
// NACC independent accumulators per wave (registers only, no memory in the
// loop), for 1..4 waves per SIMD and the whole chip.  Sizes the split
// Cholesky's tile GEMMs (bundleadjustment_amd/csrc/ba_chol_split.hip).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mfma_f64_probe.hip -o tools/mfma_f64_probe
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
  return 0;
}

// lat_probe.hip — dependent-chain latencies of the instructions on the
// Cholesky column chain (one wave, s_memtime cycles per link):
// fp64 FMA / MUL, v_rcp_f64, DPP row_newbcast broadcast, LDS write->read
// broadcast, v_readlane broadcast, f64 MFMA 16x16x4 (dependent and
// independent accumulators), and the issue rate of independent fp64 FMAs.
//   hipcc --offload-arch=gfx950 -O3 tools/lat_probe.hip -o tools/lat_probe
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kN = 512;
typedef double d4 __attribute__((ext_vector_type(4)));

template <int J>
__device__ __forceinline__ double bcast16(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0x150 + J, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x150 + J, 0xf, 0xf, false);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const long long bits = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_readlane((int)bits, lane);
  const int hi = __builtin_amdgcn_readlane((int)(bits >> 32), lane);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}

template <int MODE>
__global__ void k_lat(double* out, unsigned long long* cyc, double a, double b) {
  __shared__ double buf[2][64];
  const int lane = threadIdx.x;
  double v = lane * 1e-3 + 1.0, w = v + 0.5, x2 = v + 0.25, x3 = v + 0.125;
  double y[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) y[q] = v + q;
  d4 acc = {v, v, v, v}, acc2 = acc, acc3 = acc, acc4 = acc;
  buf[0][lane] = v;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 8
  for (int i = 0; i < kN; ++i) {
    if (MODE == 0) v = fma(v, a, b);                       // dependent FMA
    else if (MODE == 1) v = v * a;                         // dependent MUL
    else if (MODE == 2) v = __builtin_amdgcn_rcp(v) + b;   // rcp + add
    else if (MODE == 3) v = fma(bcast16<5>(v), a, b);      // DPP broadcast + FMA
    else if (MODE == 4) {                                  // LDS write -> broadcast read + FMA (one wave)
      buf[i & 1][lane] = v;
      v = fma(buf[i & 1][5], a, b);
    } else if (MODE == 5) v = fma(readlane_f64(v, 5), a, b);   // readlane + FMA
    else if (MODE == 6) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(v, w, acc, 0, 0, 0);   // dependent MFMA
    else if (MODE == 7) {                                  // 4 independent MFMA chains
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(v, w, acc, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(w, v, acc2, 0, 0, 0);
      acc3 = __builtin_amdgcn_mfma_f64_16x16x4f64(x2, v, acc3, 0, 0, 0);
      acc4 = __builtin_amdgcn_mfma_f64_16x16x4f64(x3, v, acc4, 0, 0, 0);
    } else if (MODE == 8) {                                // 8 independent FMA chains (issue rate)
#pragma unroll
      for (int q = 0; q < 8; ++q) y[q] = fma(y[q], a, b);
    } else if (MODE == 9) {                                // 8 independent DPP broadcasts + FMA
#pragma unroll
      for (int q = 0; q < 8; ++q) y[q] = fma(bcast16<3>(y[q]), a, b);
    } else if (MODE == 10) {                               // rsq + 2 Newton (the pivot reciprocal)
      double r = __builtin_amdgcn_rsq(v);
      const double h = 0.5 * v;
      r = fma(r, fma(-h * r, r, 0.5), r);
      r = fma(r, fma(-h * r, r, 0.5), r);
      v = r + b;
    } else if (MODE == 11) {                               // rcp + 2 Newton
      double r = __builtin_amdgcn_rcp(v);
      double e = fma(-v, r, 1.0);
      r = fma(r, e, r);
      e = fma(-v, r, 1.0);
      v = fma(r, e, r) + b;
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = v;
#pragma unroll
  for (int q = 0; q < 8; ++q) s += y[q];
  s += acc[0] + acc[1] + acc[2] + acc[3] + acc2[0] + acc3[1] + acc4[2];
  out[lane] = s;
  if (lane == 0) cyc[MODE] = t1 - t0;
}

int main() {
  double* out;
  unsigned long long* cyc;
  hipMalloc(&out, 64 * sizeof(double));
  hipMalloc(&cyc, 16 * sizeof(unsigned long long));
  const char* names[] = {"fma f64 dep",        "mul f64 dep",        "rcp f64 + add dep",  "dpp bcast + fma dep",
                         "lds w->r bcast + fma", "readlane + fma dep", "mfma f64 16x16x4 dep", "mfma f64 x4 indep (per 4)",
                         "fma f64 x8 indep (per 8)", "dpp+fma x8 indep (per 8)", "rsq + 2 newton dep", "rcp + 2 newton dep"};
  unsigned long long h[16];
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k_lat<0>, dim3(1), dim3(64), 0, 0, out, cyc, 0.999, 1e-3);
    hipLaunchKernelGGL(k_lat<1>, dim3(1), dim3(64), 0, 0, out, cyc, 0.999, 1e-3);
    hipLaunchKernelGGL(k_lat<2>, dim3(1), dim3(64), 0, 0, out, cyc, 0.999, 1e-3);
    hipLaunchKernelGGL(k_lat<3>, dim3(1), dim3(64), 0, 0, out, cyc, 0.999, 1e-3);
    hipLaunchKernelGGL(k_lat<4>, dim3(1), dim3(64), 0, 0, out, cyc, 0.999, 1e-3);
    hipLaunchKernelGGL(k_lat<5>, dim3(1), dim3(64), 0, 0, out, cyc, 0.999, 1e-3);
    hipLaunchKernelGGL(k_lat<6>, dim3(1), dim3(64), 0, 0, out, cyc, 0.999, 1e-3);
    hipLaunchKernelGGL(k_lat<7>, dim3(1), dim3(64), 0, 0, out, cyc, 0.999, 1e-3);
    hipLaunchKernelGGL(k_lat<8>, dim3(1), dim3(64), 0, 0, out, cyc, 0.999, 1e-3);
    hipLaunchKernelGGL(k_lat<9>, dim3(1), dim3(64), 0, 0, out, cyc, 0.999, 1e-3);
    hipLaunchKernelGGL(k_lat<10>, dim3(1), dim3(64), 0, 0, out, cyc, 0.999, 1e-3);
    hipLaunchKernelGGL(k_lat<11>, dim3(1), dim3(64), 0, 0, out, cyc, 0.999, 1e-3);
    if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
  }
  hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  for (int m = 0; m < 12; ++m) printf("%-28s %8.1f cycles/link\n", names[m], (double)h[m] / kN);
  return 0;
}

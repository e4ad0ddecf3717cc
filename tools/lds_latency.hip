// lds_latency.hip — micro-benchmark of the serial LDS broadcast round trip
// (write -> barrier -> read -> dependent fp64 op) that bounds the column
// chain of the diagonal-block factorization.  Prints cycles per round.
//   hipcc --offload-arch=gfx950 -O3 tools/lds_latency.hip -o tools/lds_latency
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kRounds = 1024;

template <int MODE>
__global__ void k_round(double* out, unsigned long long* cyc) {
  __shared__ double buf[2][256];
  const int tid = threadIdx.x;
  double v = tid * 1e-3;
  buf[0][tid] = v;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < kRounds; ++i) {
    const int b = i & 1;
    if (MODE == 0) {                 // barrier only
      __syncthreads();
    } else if (MODE == 1) {          // write own slot, barrier, read neighbour, dependent FMA
      buf[b][tid] = v;
      __syncthreads();
      v = fma(buf[b][(tid + 64) & 255], 0.5, v);
    } else if (MODE == 2) {          // same plus a division on the chain
      buf[b][tid] = v;
      __syncthreads();
      v = fma(buf[b][(tid + 64) & 255], 1.0 / (v + 3.0), v);
    } else if (MODE == 3) {          // no barrier: single-wave exchange (launch 64 threads)
      buf[b][tid] = v;
      __builtin_amdgcn_s_waitcnt(0xc07f);
      v = fma(buf[b][(tid + 1) & 63], 0.5, v);
    } else if (MODE == 4) {          // read-only dependent chain (LDS latency)
      v = buf[0][((int)v & 1) + tid] + v;
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[tid] = v;
  if (tid == 0) cyc[0] = t1 - t0;
}

int main() {
  double* out;
  unsigned long long* cyc;
  hipMalloc(&out, 256 * sizeof(double));
  hipMalloc(&cyc, sizeof(unsigned long long));
  const char* names[] = {"barrier only (256 thr)", "write+barrier+read+fma (256 thr)",
                         "write+barrier+read+div+fma (256 thr)", "write+waitcnt+read (64 thr, no barrier)",
                         "dependent LDS read chain (256 thr)"};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int mode = 0; mode < 5; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      const int threads = mode == 3 ? 64 : 256;
      hipEventRecord(e0);
      switch (mode) {
        case 0: hipLaunchKernelGGL(k_round<0>, dim3(1), dim3(threads), 0, 0, out, cyc); break;
        case 1: hipLaunchKernelGGL(k_round<1>, dim3(1), dim3(threads), 0, 0, out, cyc); break;
        case 2: hipLaunchKernelGGL(k_round<2>, dim3(1), dim3(threads), 0, 0, out, cyc); break;
        case 3: hipLaunchKernelGGL(k_round<3>, dim3(1), dim3(threads), 0, 0, out, cyc); break;
        case 4: hipLaunchKernelGGL(k_round<4>, dim3(1), dim3(threads), 0, 0, out, cyc); break;
      }
      hipEventRecord(e1);
      hipDeviceSynchronize();
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      unsigned long long c;
      hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
      if (rep == 1) printf("%-45s %8.1f cycles/round  (kernel %.1f us, %.2f GHz-equivalent)\n", names[mode],
                         (double)c / kRounds, ms * 1e3, c / (ms * 1e6));
    }
  }
  return 0;
}

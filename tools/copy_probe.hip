// copy_probe.hip — diagnostic: device copy bandwidth of 1 GiB buffers (past
// the 256-MiB Infinity Cache) for the shapes ba_stream_copy could use:
// plain vs non-temporal 16-B accesses, 1 or 4 loads in flight per lane, and
// the grid size.  Reports read + write bytes / time.
//   hipcc --offload-arch=gfx950 -O3 -o tools/copy_probe tools/copy_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d2 __attribute__((ext_vector_type(2)));

template <bool NT, int U>
__global__ __launch_bounds__(256) void copy_k(const d2* __restrict__ a, d2* __restrict__ b, size_t n2) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n2; i += U * stride) {
    d2 v[U];
#pragma unroll
    for (int q = 0; q < U; ++q) v[q] = NT ? __builtin_nontemporal_load(a + i + q * stride) : a[i + q * stride];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      if (NT) __builtin_nontemporal_store(v[q], b + i + q * stride);
      else b[i + q * stride] = v[q];
    }
  }
  for (; i < n2; i += stride) b[i] = a[i];
}

int main() {
  const size_t bytes = (size_t)1 << 30, n2 = bytes / 16;
  d2 *a, *b;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) { printf("alloc failed\n"); return 1; }
  hipMemset(a, 0, bytes);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](const char* nm, auto kern, int g) {
    hipLaunchKernelGGL(kern, dim3(g), dim3(256), 0, 0, (const d2*)a, b, n2);
    hipEventRecord(e0);
    for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(kern, dim3(g), dim3(256), 0, 0, (const d2*)a, b, n2);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-18s g=%6d  %7.1f GB/s\n", nm, g, 2.0 * bytes * 10 / (ms * 1e-3) / 1e9);
  };
  for (int g : {1024, 8192, 65536, 131072, 262144}) {
    run("plain u1", copy_k<false, 1>, g);
    run("plain u4", copy_k<false, 4>, g);
    run("nt u1", copy_k<true, 1>, g);
    run("nt u4", copy_k<true, 4>, g);
  }
  if (hipDeviceSynchronize() != hipSuccess) { printf("failed\n"); return 1; }
  return 0;
}

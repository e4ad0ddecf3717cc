// hbm_probe.hip — diagnostic: HBM ceilings for the store/load shapes the LM
// kernels use (160-B observation records, 1 M records = 160 MB).
//   write_flat   : grid-stride dwordx4 stores, 1 KiB per wave instruction
//   write_rec    : one 160-B record per lane (10 dwordx4 at 160-B stride)
//   write_stage  : row-per-lane record staged through wave-private LDS, then
//                  1 KiB-per-instruction stores (no workgroup barrier)
//   read_flat    : grid-stride dwordx4 loads (sum)
//   copy_flat    : dwordx4 load + store
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/hbm_probe tools/hbm_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int kRec = 20;  // doubles per record

__global__ __launch_bounds__(256) void write_flat(double2* __restrict__ o, size_t n2, double v) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256) o[i] = make_double2(v, v + i);
}
__global__ __launch_bounds__(256) void write_rec(double* __restrict__ o, int nrec, double v) {
  for (int r = blockIdx.x * 256 + threadIdx.x; r < nrec; r += gridDim.x * 256) {
    double2* d = reinterpret_cast<double2*>(o + (size_t)r * kRec);
#pragma unroll
    for (int k = 0; k < kRec / 2; ++k) d[k] = make_double2(v + k, v * r);
  }
}
template <int WAVES>
__global__ __launch_bounds__(WAVES * 64) void write_stage(double* __restrict__ o, int nrec, double v) {
  __shared__ double st[WAVES][64 * (kRec + 1)];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double* s = st[w];
  const int gw = blockIdx.x * WAVES + w, nw = gridDim.x * WAVES;
  for (int base = gw * 64; base < nrec; base += nw * 64) {
    const int r = base + lane;
#pragma unroll
    for (int k = 0; k < kRec; ++k) s[lane * (kRec + 1) + k] = v + k + r;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    const int nr = min(64, nrec - base);
    double2* d = reinterpret_cast<double2*>(o + (size_t)base * kRec);
#pragma unroll
    for (int it = 0; it < kRec / 2; ++it) {
      const int e = it * 64 + lane, rr = e / (kRec / 2), f = 2 * (e - rr * (kRec / 2));
      if (rr < nr) d[e] = make_double2(s[rr * (kRec + 1) + f], s[rr * (kRec + 1) + f + 1]);
    }
    __builtin_amdgcn_wave_barrier();
  }
}
__global__ __launch_bounds__(256) void read_flat(const double2* __restrict__ a, size_t n2, double* out) {
  double s = 0;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256) { double2 t = a[i]; s += t.x + t.y; }
  if (s == 12345.678) out[0] = s;
}
__global__ __launch_bounds__(256) void copy_flat(const double2* __restrict__ a, double2* __restrict__ o, size_t n2) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256) o[i] = a[i];
}

template <class F>
static float timeit(F f, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  f(); f();
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int i = 0; i < reps; ++i) f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main() {
  const int nrec = 1000000;
  const size_t bytes = (size_t)nrec * kRec * 8, n2 = bytes / 16;
  double *a, *o, *out;
  CK(hipMalloc(&a, bytes)); CK(hipMalloc(&o, bytes)); CK(hipMalloc(&out, 64));
  CK(hipMemset(a, 0, bytes));
  const int reps = 50;
  auto rep = [&](const char* name, float ms, double mb) { printf("%-28s %8.2f us  %7.1f GB/s\n", name, ms * 1e3, mb / (ms * 1e-3) / 1e9); };
  for (int g : {1024, 2048, 4096, 8192}) {
    char nm[64];
    snprintf(nm, 64, "write_flat g=%d", g);
    rep(nm, timeit([&] { hipLaunchKernelGGL(write_flat, dim3(g), dim3(256), 0, 0, (double2*)o, n2, 1.0); }, reps), bytes);
    snprintf(nm, 64, "write_rec g=%d", g);
    rep(nm, timeit([&] { hipLaunchKernelGGL(write_rec, dim3(g), dim3(256), 0, 0, o, nrec, 1.0); }, reps), bytes);
    snprintf(nm, 64, "read_flat g=%d", g);
    rep(nm, timeit([&] { hipLaunchKernelGGL(read_flat, dim3(g), dim3(256), 0, 0, (const double2*)a, n2, out); }, reps), bytes);
    snprintf(nm, 64, "copy_flat g=%d", g);
    rep(nm, timeit([&] { hipLaunchKernelGGL(copy_flat, dim3(g), dim3(256), 0, 0, (const double2*)a, (double2*)o, n2); }, reps), 2.0 * bytes);
  }
  for (int g : {256, 512, 1024, 2048}) {
    char nm[64];
    snprintf(nm, 64, "write_stage4 g=%d", g);
    rep(nm, timeit([&] { hipLaunchKernelGGL(write_stage<4>, dim3(g), dim3(256), 0, 0, o, nrec, 1.0); }, reps), bytes);
    snprintf(nm, 64, "write_stage8 g=%d", g);
    rep(nm, timeit([&] { hipLaunchKernelGGL(write_stage<8>, dim3(g), dim3(512), 0, 0, o, nrec, 1.0); }, reps), bytes);
  }
  CK(hipDeviceSynchronize());
  return 0;
}

// ba_reduce.h — fixed-order (bitwise reproducible) wave / workgroup
// reductions shared by the CDNA4 kernels (wave64: shuffles, then LDS).
#pragma once
#include <hip/hip_runtime.h>

#include "ba_kernels.h"

namespace bahip {

// ---------------------------------------------------------------------------
// reductions
// ---------------------------------------------------------------------------
__device__ inline double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  return v;
}
__device__ inline double wave_max(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_down(v, off, 64));
  return v;
}
// Block-wide sum of NV values per thread (fixed order).  Result valid in
// thread 0: out[k].  lds must hold NV * (blockDim/64) doubles.
template <int NV>
__device__ inline void block_sum(double (&v)[NV], double* lds, double (&out)[NV]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const double s = wave_sum(v[k]);
    if (lane == 0) lds[k * 16 + w] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      double s = 0.0;
      for (int i = 0; i < nw; ++i) s += lds[k * 16 + i];
      out[k] = s;
    }
  }
  __syncthreads();
}
__device__ inline double block_max1(double v, double* lds) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_max(v);
  if (lane == 0) lds[w] = v;
  __syncthreads();
  double m = 0.0;
  if (threadIdx.x == 0) for (int i = 0; i < nw; ++i) m = fmax(m, lds[i]);
  __syncthreads();
  return m;
}

__device__ inline double* part_of(double* part, int slot) { return part + (size_t)slot * kMaxBlocks; }

// Workgroup sum of NV values per thread whose result every thread receives
// (fixed order: wave shuffle tree, then the waves in index order).  lds must
// hold NV * 16 doubles.
template <int NV>
__device__ inline void block_allsum(double (&v)[NV], double* lds) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const double s = wave_sum(v[k]);
    if (lane == 0) lds[k * 16 + w] = s;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    double s = 0.0;
    for (int i = 0; i < nw; ++i) s += lds[k * 16 + i];
    v[k] = s;
  }
  __syncthreads();
}

// One per-observation Schur block W_o (6x3, 18 values) -> fp64 registers;
// stored fp64 (144 B) or, with BA_MIXED_FP32, fp32 (72 B).
__device__ inline void load_w18(const double* __restrict__ Wm, size_t o, double (&w)[18]) {
  const double2* s = reinterpret_cast<const double2*>(Wm + o * 18);
#pragma unroll
  for (int k = 0; k < 9; ++k) { const double2 t = s[k]; w[2 * k] = t.x; w[2 * k + 1] = t.y; }
}
__device__ inline void load_w18(const float* __restrict__ Wm, size_t o, double (&w)[18]) {
  const float2* s = reinterpret_cast<const float2*>(Wm + o * 18);
#pragma unroll
  for (int k = 0; k < 9; ++k) { const float2 t = s[k]; w[2 * k] = (double)t.x; w[2 * k + 1] = (double)t.y; }
}

}  // namespace bahip

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

// Value pair c (values 2c, 2c+1) of a run of contiguous W records.
__device__ inline void w_pair(const double* __restrict__ base, int c, double& x, double& y) {
  const double2 t = reinterpret_cast<const double2*>(base)[c]; x = t.x; y = t.y;
}
__device__ inline void w_pair(const float* __restrict__ base, int c, double& x, double& y) {
  const float2 t = reinterpret_cast<const float2*>(base)[c]; x = (double)t.x; y = (double)t.y;
}

// Sum over the observations [o0, o1) of one point of W_o^T x_{vc(o)}
// (3-vector), by a group of kPtLanes consecutive lanes.  Lane gl of the group
// takes the value pairs gl, gl + kPtLanes, ... of the point's contiguous W
// records (9 pairs per record), so one wavefront load instruction reads whole
// 256-B (fp64) segments instead of 64 records 1.4 KB apart -- every cache
// line is requested once.  Fixed-order xor reduction inside the group: all
// lanes of the group get the same (deterministic) sum.
#ifndef BA_PT_LANES
#define BA_PT_LANES 16
#endif
constexpr int kPtLanes = BA_PT_LANES;
// UNROLL: four pairs per round with every load issued first (the PCG point
// passes: C5 shard +2.6 %); the back substitution keeps the one-pair loop
// (the unrolled form measured 37.8 -> 41.9 us there at C3)
template <bool UNROLL, typename WT>
__device__ inline void point_wtx(const WT* __restrict__ Wm, const int* __restrict__ obs_vc,
                                 const double* __restrict__ xv, int o0, int o1, int gl, double (&s)[3]) {
  const WT* base = Wm + (size_t)o0 * 18;
  const int nch = 9 * (o1 - o0);
  double s0 = 0.0, s1 = 0.0, s2 = 0.0;
  // value pair c: its W loads, then its camera index, then the two x values
  // (fixed cameras: W_o = 0); four pairs per round with every load issued
  // before the first product (the chain W / index -> x -> FMA of one pair at
  // a time left the lanes latency-bound); same summation order
  auto add = [&](double t0, double t1, int f, const double* xc) {
    // values i0 = 2f, i1 = 2f + 1 of W_o: row i / 3, column i % 3
    const int i0 = 2 * f, i1 = i0 + 1;
    const double p0 = t0 * xc[i0 / 3], p1 = t1 * xc[i1 / 3];
    const int b0 = i0 % 3, b1 = i1 % 3;
    s0 += b0 == 0 ? p0 : (b1 == 0 ? p1 : 0.0);
    s1 += b0 == 1 ? p0 : (b1 == 1 ? p1 : 0.0);
    s2 += b0 == 2 ? p0 : (b1 == 2 ? p1 : 0.0);
  };
  int c = gl;
  if (UNROLL)
  for (; c + 3 * kPtLanes < nch; c += 4 * kPtLanes) {
    double t[4][2];
    int f[4];
    const double* xc[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) w_pair(base, c + u * kPtLanes, t[u][0], t[u][1]);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int cu = c + u * kPtLanes, k = cu / 9;
      f[u] = cu - 9 * k;
      xc[u] = xv + 6 * max(obs_vc[o0 + k], 0);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) add(t[u][0], t[u][1], f[u], xc[u]);
  }
  for (; c < nch; c += kPtLanes) {
    double t0, t1;
    w_pair(base, c, t0, t1);
    const int k = c / 9;
    add(t0, t1, c - 9 * k, xv + 6 * max(obs_vc[o0 + k], 0));
  }
#pragma unroll
  for (int m = kPtLanes / 2; m > 0; m >>= 1) {
    s0 += __shfl_xor(s0, m, kPtLanes);
    s1 += __shfl_xor(s1, m, kPtLanes);
    s2 += __shfl_xor(s2, m, kPtLanes);
  }
  s[0] = s0; s[1] = s1; s[2] = s2;
}

}  // namespace bahip

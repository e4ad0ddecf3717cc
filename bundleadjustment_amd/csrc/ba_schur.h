// ba_schur.h — device pieces of the explicit Schur complement (DENSE_SCHUR,
// compact W records) shared by the pair pass (ba_kernels.hip
// k_schur_pairs_cd, k_cam_schur_diag_cd, k_cam_fold_diag) and the
// overlapped factorisation (ba_chol_persist.hip), which forms the same S
// entries with the same arithmetic in the same order.
#pragma once
#include <hip/hip_runtime.h>

#include "ba_kernels.h"
#include "ba_reduce.h"

namespace bahip {

// compact W records (k_obs_w_rc<double, true>, described there): 16 doubles
constexpr int kWcRec = 16;
// the camera constants of the compact records: Jc's scaled translation
// columns are f (A_row,k - pr_row B_k), A_row,k = s_{3+k} K_{3k+row},
// B_k = s_{3+k} K_{3k+2}
struct WcCam {
  double a0[3], a1[3], b[3];
  __device__ void load(const DevProblem& P, const double* __restrict__ scale_c, int v) {
    const int c = P.cam_of_vc[v];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const double st = scale_c[(size_t)v * 6 + 3 + k];
      a0[k] = st * (double)P.K[9 * c + 3 * k];
      a1[k] = st * (double)P.K[9 * c + 3 * k + 1];
      b[k] = st * (double)P.K[9 * c + 3 * k + 2];
    }
  }
};
struct WcRaw { double r[kWcRec]; };
__device__ inline WcRaw wc_fetch(const double* __restrict__ Wc, int o) {
  WcRaw w;
  const double2* s = reinterpret_cast<const double2*>(Wc + (size_t)o * kWcRec);
#pragma unroll
  for (int k = 0; k < kWcRec / 2; ++k) { const double2 t = s[k]; w.r[2 * k] = t.x; w.r[2 * k + 1] = t.y; }
  return w;
}
// c = Jc s_c (rows c0, c1) of a compact record
__device__ inline void wc_rows(const WcRaw& w, const WcCam& m, double (&c0)[6], double (&c1)[6]) {
  const double pr0 = w.r[6], pr1 = w.r[7], f = w.r[8];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    c0[k] = w.r[k];
    c1[k] = w.r[3 + k];
    c0[3 + k] = f * (m.a0[k] - pr0 * m.b[k]);
    c1[3 + k] = f * (m.a1[k] - pr1 * m.b[k]);
  }
}

// LDS-DMA: one 16-B piece per lane, lane-linear at lds_dst (global_load_lds_dwordx4)
__device__ __forceinline__ void glds16(const double* src, double* lds_dst) {
  __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)lds_dst, 16, 0, 0);
}

// PL lanes per camera-pair block (64 / PL blocks per wave; PL = 16 by
// default, BA_PAIR_LANES selects 8 or 32): each lane accumulates every PL-th
// pair, then a log2(PL)-stage xor reduction inside the lane group
#ifndef BA_PAIRS_IDX2
#define BA_PAIRS_IDX2 1
#endif
#ifndef BA_PAIR_LANES
#define BA_PAIR_LANES 16
#endif
constexpr int kPairLanes = BA_PAIR_LANES;

// one camera slice (v, slice g of G) by one wave: the per-lane sums
__device__ __forceinline__ void diag_cd_wave(const DevProblem& P, const double* __restrict__ Wc,
                                             const double* __restrict__ scale_c, const double* __restrict__ u,
                                             int v, int g, int G, double* rbuf, double* ubuf, double (&acc)[27]) {
  WcCam m;
  m.load(P, scale_c, v);
#pragma unroll
  for (int k = 0; k < 27; ++k) acc[k] = 0.0;
  const int a0 = P.cam_off[v], a1 = P.cam_off[v + 1];
  const int len = (a1 - a0 + G - 1) / G;
  const int i0 = min(a1, a0 + g * len), i1 = min(a1, i0 + len);
  const int lane = threadIdx.x & 63;
  const int swr = (lane >> 1) & 7;
  auto issue = [&](int2 op) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int q = (lane >> 3) + 8 * k;
      const int oq = __shfl(op.x, q);
      glds16(Wc + (size_t)oq * kWcRec + 2 * ((lane & 7) ^ ((q >> 1) & 7)), rbuf + k * 128);
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int q = (lane >> 1) + 32 * k;
      const int pq = __shfl(op.y, q);
      glds16(u + 4 * (size_t)pq + 2 * (lane & 1), ubuf + k * 128);
    }
  };
  const int nr = (i1 - i0 + 63) >> 6;   // rounds (uniform)
  int i = i0 + lane;
  int2 op = i < i1 ? P.cam_op[i] : make_int2(0, 0);
  int2 opn = i + 64 < i1 ? P.cam_op[i + 64] : make_int2(0, 0);
  if (nr > 0) issue(op);
  for (int r = 0; r < nr; ++r, i += 64) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this round's DMA has landed
    WcRaw w;
    const double* rr = rbuf + lane * kWcRec;
#pragma unroll
    for (int p = 0; p < kWcRec / 2; ++p) {
      const double2 t = *reinterpret_cast<const double2*>(rr + 2 * (p ^ swr));
      w.r[2 * p] = t.x;
      w.r[2 * p + 1] = t.y;
    }
    const double2 u01 = *reinterpret_cast<const double2*>(ubuf + 4 * lane);
    const double u2 = ubuf[4 * lane + 2];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // read out before the refill
    if (r + 1 < nr) {
      issue(opn);
      opn = i + 128 < i1 ? P.cam_op[i + 128] : make_int2(0, 0);
    }
    if (i < i1) {
      double c0[6], c1[6];
      wc_rows(w, m, c0, c1);
      const double* z0 = w.r + 9;
      const double* z1 = w.r + 12;
      const double m00 = z0[0] * z0[0] + z0[1] * z0[1] + z0[2] * z0[2];
      const double m01 = z0[0] * z1[0] + z0[1] * z1[1] + z0[2] * z1[2];
      const double m11 = z1[0] * z1[0] + z1[1] * z1[1] + z1[2] * z1[2];
      const double zu0 = z0[0] * u01.x + z0[1] * u01.y + z0[2] * u2;
      const double zu1 = z1[0] * u01.x + z1[1] * u01.y + z1[2] * u2;
      double n0[6], n1[6];
#pragma unroll
      for (int b = 0; b < 6; ++b) {
        n0[b] = m00 * c0[b] + m01 * c1[b];
        n1[b] = m01 * c0[b] + m11 * c1[b];
      }
      int t = 0;
#pragma unroll
      for (int a = 0; a < 6; ++a) {
#pragma unroll
        for (int b = 0; b <= a; ++b) acc[t++] += c0[a] * n0[b] + c1[a] * n1[b];
      }
#pragma unroll
      for (int a = 0; a < 6; ++a) acc[21 + a] += c0[a] * zu0 + c1[a] * zu1;
    }
  }
}

// S_cc = s Hcc s + D^2 - (the G slices of -sum W W^T), b_c likewise: entry e
// = (camera, 27 entries) (k_cam_fold_diag, or the extra workgroups of the
// pair pass's launch).  SC1: the overlapped factorisation's form — the
// slices (written by other workgroups of the same launch) read, and S
// written, through agent-scope atomic accesses (sc1: at the memory side),
// and the Cholesky failure slots left to the factorisation, which clears
// them itself; the same arithmetic
template <bool SC1 = false>
__device__ __forceinline__ void cam_fold_diag_entry(const DevProblem& P, const double* __restrict__ cpart, int nsl,
                                                    const double* __restrict__ Hcc, const double* __restrict__ gc,
                                                    const double* __restrict__ scale_c,
                                                    const double* __restrict__ diag_c, double radius,
                                                    double* __restrict__ S, double* __restrict__ scal, int e) {
  // no fma contraction: the fused and the exchange path (k_cam_fold +
  // k_cam_add_diag) must round identically
#pragma clang fp contract(off)
  if (!SC1 && e == 0) { scal[SL_CHOL_BAD] = 0.0; scal[SL_CHOL_SPIN] = 0.0; }   // the Cholesky that follows flags failures here
  if (e >= P.nvc * 27) return;
  const int v = e / 27, k = e - v * 27;
  double acc = 0.0;
  for (int sl = 0; sl < nsl; ++sl) {
    const double* src = cpart + ((size_t)sl * P.nvc + v) * 27 + k;
    if constexpr (SC1) acc += __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else acc += *src;
  }
  const size_t ld = (size_t)P.ld;
  double* dst;
  double val;
  if (k < 21) {
    int a = 0;
    while ((a + 1) * (a + 2) / 2 <= k) ++a;
    const int b = k - a * (a + 1) / 2;
    double h = Hcc[(size_t)v * 21 + k] * scale_c[(size_t)v * 6 + a] * scale_c[(size_t)v * 6 + b];
    if (a == b) {
      const double D = sqrt(diag_c[(size_t)v * 6 + a] / radius);
      h += D * D;
    }
    dst = S + (size_t)(6 * v + a) * ld + 6 * v + b;
    val = -acc + h;
  } else {
    const int a = k - 21;
    dst = S + (size_t)P.n * ld + 6 * v + a;
    val = -acc + gc[(size_t)v * 6 + a] * scale_c[(size_t)v * 6 + a];
  }
  if constexpr (SC1) __hip_atomic_store(dst, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *dst = val;
}
// the S entry (row, col) that fold entry k of camera v writes
__device__ __forceinline__ void fold_entry_pos(int n, int v, int k, int& row, int& col) {
  if (k < 21) {
    int a = 0;
    while ((a + 1) * (a + 2) / 2 <= k) ++a;
    row = 6 * v + a;
    col = 6 * v + k - a * (a + 1) / 2;
  } else {
    row = n;
    col = 6 * v + k - 21;
  }
}

}  // namespace bahip

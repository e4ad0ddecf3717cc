#pragma once
// ba_chol.h — dense blocked Cholesky of the reduced camera system on gfx950.
//
// The reference solves the reduced camera system of DENSE_SCHUR with a dense
// Cholesky (Eigen LLT; Optimizer.cpp:85).  Here the (n+1) x n lower
// trapezoid A (row n = right-hand side b) is factored in 64-wide block
// columns into a separate lower-trapezoidal L (row n of L = z = L^-1 b).
//
// One launch per block step k ("look-ahead"), grid = lower tiles of the
// trailing matrix (64 x 64, MFMA f64 16x16x4 contractions):
//   tile (0,0) [critical]:  P = A_{k+1,k} V_k^T  (-> L), C = A_{k+1,k+1} - P P^T,
//                           factor C = L L^T and invert it (V_{k+1} = L^-1)
//   tile (I,J) [others]:    P_I = A_{I,k} V_k^T, P_J = A_{J,k} V_k^T,
//                           A_{IJ} -= P_I P_J^T ; the J = k+1 column also
//                           stores P_I = L_{I,k}
// so the serial chain per 64 columns is one panel GEMM, one tile update and
// the 64-column factor + inverse of the critical workgroup.  Back
// substitution L^T y = z then uses the explicit V_K (no triangular solves).
#include "ba_kernels.h"

namespace bahip {

constexpr int CB = 64;           // block size
#ifndef BA_LDP
#define BA_LDP (CB + 2)   // (diagnostic builds may pad differently: tools/chol_bench A/B, profiles/r06_v13_*)
#endif
constexpr int LDP = BA_LDP;      // padded LDS row (doubles): conflict-free MFMA operand reads (16 rows x 4 k per wave)

typedef double d4 __attribute__((ext_vector_type(4)));

// threadIdx.x through an opaque copy: the index arithmetic derived from it is
// formed where it is used instead of being hoisted, as loop invariants, out
// of the persistent kernel's block-column loop (where ~120 such values stayed
// live, in AGPRs, for the whole kernel); the wave index stays uniform
__device__ __forceinline__ int ctid() {
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}
__device__ __forceinline__ int cwave() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// Diagnostic build only (tools/chol_bench.hip defines BA_CHOL_STAMPS): the
// critical workgroup records s_memtime at phase boundaries into g_stamps.
#ifdef BA_CHOL_STAMPS
__device__ unsigned long long g_stamps[64];
__device__ int g_stamp_on = 1;   // the persistent kernel records one chosen step only
#define CHOL_STAMP(i)                                                                         \
  do {                                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    unsigned long long t_;                                                                    \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    if (threadIdx.x == 0 && g_stamp_on) g_stamps[i] = t_;                                     \
  } while (0)
#else
#define CHOL_STAMP(i) do {} while (0)
#endif

// Device-coherent (sc1) buffer loads / stores and the epoch-flag hand-offs of
// the in-launch dataflows (persistent factorisation, split form's panels):
// a value published by one CU is read by another, on any XCD.
typedef unsigned int u4 __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t Rsrc;
constexpr int kAuxSc1 = 16;                    // buffer-instruction cache policy: sc1

__device__ __forceinline__ Rsrc make_rsrc(const void* base, size_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ double2 ld_sc1(Rsrc r, size_t byte_off) {
  const u4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)byte_off, 0, kAuxSc1);
  return __builtin_bit_cast(double2, v);
}
__device__ __forceinline__ void st_sc1(Rsrc r, size_t byte_off, double2 x) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, x), r, (int)byte_off, 0, kAuxSc1);
}

// drain this wave's stores, join the workgroup, one lane raises the flag
__device__ __forceinline__ void publish(unsigned* flag, unsigned epoch) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // EVERY storing wave
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flag, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the same with the 8 tile loads of tile_fetch_sc1 issued after the stores
// still in flight: vector memory operations complete in issue order, so
// vmcnt(8) drains exactly the stores
__device__ __forceinline__ void publish_before_loads(unsigned* flag, unsigned epoch) {
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (threadIdx.x == 0) __hip_atomic_store(flag, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// lane 0 polls (relaxed, bounded), the barrier releases the workgroup.
// Returns false in thread 0 if the bound was hit (the failure is reported by
// thread 0 alone; other threads return true)
__device__ __forceinline__ bool wait_flag(const unsigned* flag, unsigned epoch, unsigned spin_max) {
  bool ok = true;
  if (threadIdx.x == 0) {
    unsigned it = 0;
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch) {
      if (++it >= spin_max) { ok = false; break; }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  return ok;
}

// Stage a 64x64 block M[r0 + i][c0 + j] (i < rmax - r0, j < cmax - c0, else
// 0) into LDS: tile_load issues the 8 16-B loads of a thread, tile_put
// writes them to LDS — several tiles' loads go out before the first store.
// Branch-free (a load under a divergent branch gets its own vmcnt(0) wait,
// which serialised the 24 loads of the critical stage): every lane loads a
// 16-B pair from a clamped in-range address and zeroes what is outside the
// tile.  LOWER: pairs strictly above the diagonal are redirected to the
// row's diagonal pair (a line another lane fetches anyway) and zeroed.
// Needs ld even and cmax - c0 >= 2 (n = 6 * cameras).
struct TileRegs { double2 v[8]; };
template <bool LOWER = false>
__device__ inline TileRegs tile_fetch(const double* __restrict__ M, size_t ld, int r0, int c0, int rmax, int cmax) {
  TileRegs t;
  const int tid = ctid();
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int e = tid + 256 * it;          // 2048 double2
    const int i = e >> 5, j = (e & 31) * 2;
    const bool up = LOWER && j > i;
    const int ri = r0 + i, cj = c0 + (up ? (i & ~1) : j);
    const int ric = min(ri, rmax - 1), cjc = min(cj, cmax - 2) & ~1;
    const double2 v = *reinterpret_cast<const double2*>(M + (size_t)ric * ld + cjc);
    const bool rok = ri < rmax && !up;
    t.v[it].x = (rok && cj < cmax) ? v.x : 0.0;
    t.v[it].y = (rok && cj + 1 < cmax) ? v.y : 0.0;
  }
  return t;
}
__device__ inline void tile_put(double (*D)[LDP], const TileRegs& t) {
  const int tid = ctid();
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int e = tid + 256 * it;
    const int i = e >> 5, j = (e & 31) * 2;
    D[i][j] = t.v[it].x;
    D[i][j + 1] = t.v[it].y;
  }
}
// The same staging in two halves for a pipelined consumer: tile_fetch_raw
// only issues the loads (the out-of-tile zeroing is a per-element mask,
// computed from indices, applied by tile_put_masked) — with the selects of
// tile_fetch next to the loads, the compiler waits for the loads right there,
// and the next operand tiles' loads never overlapped the current MFMAs.
struct TileRaw { double2 v[8]; unsigned mask; };
__device__ inline TileRaw tile_fetch_raw(const double* __restrict__ M, size_t ld, int r0, int c0, int rmax, int cmax) {
  TileRaw t;
  t.mask = 0;
  const int tid = ctid();
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int e = tid + 256 * it;
    const int i = e >> 5, j = (e & 31) * 2;
    const int ri = r0 + i, cj = c0 + j;
    const int ric = min(ri, rmax - 1), cjc = min(cj, cmax - 2) & ~1;
    t.v[it] = *reinterpret_cast<const double2*>(M + (size_t)ric * ld + cjc);
    const bool rok = ri < rmax;
    t.mask |= ((rok && cj < cmax) ? 1u : 0u) << (2 * it);
    t.mask |= ((rok && cj + 1 < cmax) ? 2u : 0u) << (2 * it);
  }
  return t;
}
__device__ inline void tile_put_masked(double (*D)[LDP], const TileRaw& t) {
  const int tid = ctid();
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int e = tid + 256 * it;
    const int i = e >> 5, j = (e & 31) * 2;
    D[i][j] = (t.mask >> (2 * it)) & 1u ? t.v[it].x : 0.0;
    D[i][j + 1] = (t.mask >> (2 * it)) & 2u ? t.v[it].y : 0.0;
  }
}
// tile_fetch with sc1 loads: the same clamped, branch-free
// addresses and the same zeroing, so the staged tile is identical
template <bool LOWER = false>
__device__ inline TileRegs tile_fetch_sc1(Rsrc r, size_t ld, int r0, int c0, int rmax, int cmax) {
  TileRegs t;
  const int tid = ctid();
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int e = tid + 256 * it;
    const int i = e >> 5, j = (e & 31) * 2;
    const bool up = LOWER && j > i;
    const int ri = r0 + i, cj = c0 + (up ? (i & ~1) : j);
    const int ric = min(ri, rmax - 1), cjc = min(cj, cmax - 2) & ~1;
    const double2 v = ld_sc1(r, ((size_t)ric * ld + cjc) * sizeof(double));
    const bool rok = ri < rmax && !up;
    t.v[it].x = (rok && cj < cmax) ? v.x : 0.0;
    t.v[it].y = (rok && cj + 1 < cmax) ? v.y : 0.0;
  }
  return t;
}

__device__ inline void stage64(double (*D)[LDP], const double* __restrict__ M, size_t ld, int r0, int c0, int rmax,
                               int cmax) {
  tile_put(D, tile_fetch(M, ld, r0, c0, rmax, cmax));
}

// C (64x64, distributed as 4 waves x 2x2 MFMA tiles of 16x16) = sum_k Xs[i][k] Ys[j][k]
__device__ inline void mfma_xyT_64(const double (*Xs)[LDP], const double (*Ys)[LDP], d4 acc[2][2]) {
  const int lane = ctid() & 63, w = cwave();
  const int r0 = (w >> 1) * 32, c0 = (w & 1) * 32;
  const int li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
  for (int k0 = 0; k0 < CB; k0 += 4) {
    const double x0 = Xs[r0 + li][k0 + lk], x1 = Xs[r0 + 16 + li][k0 + lk];
    const double y0 = Ys[c0 + li][k0 + lk], y1 = Ys[c0 + 16 + li][k0 + lk];
    acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(x0, y0, acc[0][0], 0, 0, 0);
    acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(x0, y1, acc[0][1], 0, 0, 0);
    acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(x1, y0, acc[1][0], 0, 0, 0);
    acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(x1, y1, acc[1][1], 0, 0, 0);
  }
}

// the same product added to acc (a rank-K update accumulated over K / 64 tiles)
__device__ inline void mfma_xyT_64_add(const double (*Xs)[LDP], const double (*Ys)[LDP], d4 acc[2][2]) {
  const int lane = ctid() & 63, w = cwave();
  const int r0 = (w >> 1) * 32, c0 = (w & 1) * 32;
  const int li = lane & 15, lk = lane >> 4;
#pragma unroll 4
  for (int k0 = 0; k0 < CB; k0 += 4) {
    const double x0 = Xs[r0 + li][k0 + lk], x1 = Xs[r0 + 16 + li][k0 + lk];
    const double y0 = Ys[c0 + li][k0 + lk], y1 = Ys[c0 + 16 + li][k0 + lk];
    acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(x0, y0, acc[0][0], 0, 0, 0);
    acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(x0, y1, acc[0][1], 0, 0, 0);
    acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(x1, y0, acc[1][0], 0, 0, 0);
    acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(x1, y1, acc[1][1], 0, 0, 0);
  }
}

// Lower 16x16 tiles (ti >= tj) of C = sum_k Xs[i][k] Xs[j][k] (a symmetric
// product): 10 tiles over 4 waves (3, 3, 2, 2) instead of 16 (4 each).
__device__ inline int lower_tiles_of(int w, int (*tl)[2]) {
  constexpr int T[10][2] = {{0, 0}, {1, 0}, {1, 1}, {2, 0}, {2, 1}, {2, 2}, {3, 0}, {3, 1}, {3, 2}, {3, 3}};
  const int first = w == 0 ? 0 : (w == 1 ? 3 : (w == 2 ? 6 : 8));
  const int cnt = w < 2 ? 3 : 2;
  for (int q = 0; q < 3; ++q) { tl[q][0] = T[first + min(q, cnt - 1)][0]; tl[q][1] = T[first + min(q, cnt - 1)][1]; }
  return cnt;
}
__device__ inline void mfma_xxT_lower_sub(const double (*Xs)[LDP], double (*D)[LDP]) {
  const int lane = ctid() & 63, w = cwave();
  const int li = lane & 15, lk = lane >> 4;
  int tl[3][2];
  const int cnt = lower_tiles_of(w, tl);
  d4 acc[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) acc[q] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
  for (int k0 = 0; k0 < CB; k0 += 4) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      if (q < cnt) {
        const double x = Xs[16 * tl[q][0] + li][k0 + lk];
        const double y = Xs[16 * tl[q][1] + li][k0 + lk];
        acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc[q], 0, 0, 0);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 3; ++q)
    if (q < cnt)
#pragma unroll
      for (int g = 0; g < 4; ++g) D[16 * tl[q][0] + lk + 4 * g][16 * tl[q][1] + li] -= acc[q][g];
}

// The same product split for the critical path: the tiles (w, 0) of
// column 0 first (one per wave: all the first sub-panel sweep reads), the
// other six lower tiles (two per wave for waves 1..3) while wave 0 sweeps.
// Each tile accumulates over k in the order of mfma_xxT_lower_sub (bitwise
// the same C).
__device__ inline void mfma_xxT_tile(const double (*Xs)[LDP], double (*D)[LDP], int ti, int tj) {
  const int lane = ctid() & 63;
  const int li = lane & 15, lk = lane >> 4;
  d4 acc = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
  for (int k0 = 0; k0 < CB; k0 += 4) {
    const double x = Xs[16 * ti + li][k0 + lk];
    const double y = Xs[16 * tj + li][k0 + lk];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc, 0, 0, 0);
  }
#pragma unroll
  for (int g = 0; g < 4; ++g) D[16 * ti + lk + 4 * g][16 * tj + li] -= acc[g];
}
__device__ inline void mfma_xxT_col0(const double (*Xs)[LDP], double (*D)[LDP]) {
  mfma_xxT_tile(Xs, D, cwave(), 0);
}
__device__ inline void mfma_xxT_rest(const double (*Xs)[LDP], double (*D)[LDP]) {
  constexpr int T[6][2] = {{1, 1}, {2, 1}, {2, 2}, {3, 1}, {3, 2}, {3, 3}};
  const int w = cwave();
  if (w == 0) return;
#pragma unroll
  for (int h = 0; h < 2; ++h) mfma_xxT_tile(Xs, D, T[2 * (w - 1) + h][0], T[2 * (w - 1) + h][1]);
}

// P = Xs V^T with V lower triangular (V[j][k] = 0 for k > j): wave w owns
// the row strip 16w..16w+15, and output column tile bc needs only k <
// 16 (bc + 1) -> 40 MFMAs per wave (the square product: 64).
// acc[bc] element g: row 16w + (lane >> 4) + 4g, col 16bc + (lane & 15).
__device__ inline void mfma_xVT_strip(const double (*Xs)[LDP], const double (*Vs)[LDP], d4 acc[4]) {
  const int lane = ctid() & 63, w = cwave();
  const int li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int bc = 0; bc < 4; ++bc) acc[bc] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int k0 = 0; k0 < CB; k0 += 4) {
    const double x = Xs[16 * w + li][k0 + lk];
#pragma unroll
    for (int bc = 0; bc < 4; ++bc)
      if (k0 < 16 * (bc + 1)) acc[bc] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, Vs[16 * bc + li][k0 + lk], acc[bc], 0, 0, 0);
  }
}

// accumulator element (a, b, reg) -> tile-local (row, col); v_mfma_f64_16x16x4
// D layout: col = lane & 15, row = (lane >> 4) + 4 * reg
__device__ inline void acc_pos(int a, int b, int reg, int* row, int* col) {
  const int lane = ctid() & 63, w = cwave();
  *row = (w >> 1) * 32 + 16 * a + (lane >> 4) + 4 * reg;
  *col = (w & 1) * 32 + 16 * b + (lane & 15);
}

// Dst (LDS) = acc (op: 0 store, 1 Dst = Dst - acc)
__device__ inline void acc_to_lds(double (*D)[LDP], const d4 acc[2][2], int op) {
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        int rr, cc;
        acc_pos(a, b, g, &rr, &cc);
        if (op == 0) D[rr][cc] = acc[a][b][g];
        else D[rr][cc] -= acc[a][b][g];
      }
}

// Store rows [0, m) x cols [0, w) of an LDS tile to global (coalesced).
__device__ inline void lds_to_global(const double (*Sx)[LDP], double* __restrict__ G, size_t ld, int r0, int c0,
                                     int m, int w) {
  for (int e = ctid(); e < CB * CB; e += 256) {
    const int i = e / CB, j = e % CB;
    if (i < m && j < w) G[(size_t)(r0 + i) * ld + c0 + j] = Sx[i][j];
  }
}

// Factor + inverse of the diagonal 64-block, the serial heart of the solve.
//
// T (LDS) holds the lower part of the block (b columns, m <= 64 rows; rows
// b..m-1 are extra panel rows: the rhs row of the last step).  It is
// factored in four 16-column sub-panels (right-looking, blocked):
//   sweep  16 column steps, division-free (LDL^T form): column j and the
//          pivot row j of U (unscaled inverse of the sub-panel's 16x16
//          diagonal block) are published to double-buffered LDS, one
//          barrier, then every row r > j does  f = a_rj / d_j,
//          a_rt -= f a_tj (t in the sub-panel, t > j),  U_r -= f U_j.
//          Thread (r = tid >> 2, q = tid & 3) owns a_{r, c0+4q..c0+4q+3}.
//   scale  L_rt = a_rt / sqrt(d_t), L_tt = sqrt(d_t); X_pp = U / sqrt(d_r)
//   update trailing rows/cols: T_RS -= L_{R,p} L_{S,p}^T, 16x16 MFMA tiles.
// then the off-diagonal blocks of X = L^-1 follow by block distance:
//   X_ip = -X_ii sum_{k=p}^{i-1} L_ik X_kp   (MFMA, 3 rounds).
// Per column the chain is one barrier, one LDS round trip and one
// reciprocal; the O(b^3) work runs on MFMA.  (A full-width register sweep
// measured ~1300 cycles per column: its 16+16 broadcast reads per thread
// saturate LDS bandwidth; this one reads 6 doubles per thread per column.)
// On exit T holds L (b columns, rows < m) and X holds L^-1 (b x b).
struct CholLds {
  double2 colp[2][CB];     // column-pair broadcast of the sub-panel sweep
  double rsv[CB];          // 1/sqrt(pivot) broadcast for the final scaling
  int bad;
};

// 1/d to ~1 ulp: hardware reciprocal + two Newton steps
__device__ __forceinline__ double recip(double d) {
  double y = __builtin_amdgcn_rcp(d);
  double e = fma(-d, y, 1.0);
  y = fma(y, e, y);
  e = fma(-d, y, 1.0);
  return fma(y, e, y);
}

// 1/sqrt(d) to ~1 ulp: hardware estimate + two Newton steps (IEEE sqrt and
// division are long instruction sequences on the column chain)
__device__ __forceinline__ double rsqrt_nr(double d) {
  double y = __builtin_amdgcn_rsq(d);
  const double h = 0.5 * d;
  y = fma(y, fma(-h * y, y, 0.5), y);
  return fma(y, fma(-h * y, y, 0.5), y);
}

// D (16x16, MFMA accumulator layout) += sgn * sum_{k < K} Xs[xr + i][xc + k] * Ys[yr + j][yc + k]
template <int K>
__device__ __forceinline__ d4 mfma_tile(d4 acc, const double (*Xs)[LDP], int xr, int xc, const double (*Ys)[LDP],
                                        int yr, int yc, double sgn) {
  const int lane = ctid() & 63, li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int k0 = 0; k0 < K; k0 += 4) {
    const double x = sgn * Xs[xr + li][xc + k0 + lk];
    const double y = Ys[yr + li][yc + k0 + lk];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc, 0, 0, 0);
  }
  return acc;
}

// same with the second operand transposed: Ys[yr + k][yc + j]
template <int K, int YLD = LDP>
__device__ __forceinline__ d4 mfma_tile_n(d4 acc, const double (*Xs)[LDP], int xr, int xc, const double (*Ys)[YLD],
                                          int yr, int yc, double sgn) {
  const int lane = ctid() & 63, li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int k0 = 0; k0 < K; k0 += 4) {
    const double x = sgn * Xs[xr + li][xc + k0 + lk];
    const double y = Ys[yr + k0 + lk][yc + li];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc, 0, 0, 0);
  }
  return acc;
}

__device__ __forceinline__ d4 tile_load(const double (*S)[LDP], int r0, int c0) {
  const int lane = ctid() & 63;
  d4 v;
#pragma unroll
  for (int g = 0; g < 4; ++g) v[g] = S[r0 + (lane >> 4) + 4 * g][c0 + (lane & 15)];
  return v;
}

template <int SLD = LDP>
__device__ __forceinline__ void tile_store(double (*S)[SLD], int r0, int c0, d4 v) {
  const int lane = ctid() & 63;
#pragma unroll
  for (int g = 0; g < 4; ++g) S[r0 + (lane >> 4) + 4 * g][c0 + (lane & 15)] = v[g];
}

__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const long long bits = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane(static_cast<int>(bits), lane);
  const int hi = __builtin_amdgcn_readlane(static_cast<int>(bits >> 32), lane);
  return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned int>(lo));
}

// 16-column sub-panel sweep by ONE wave (lane = row, registers = columns):
// no barriers on the chain; each column is broadcast through LDS by the
// same wave (LDS is in order per wave).  Division-free: f_r = a_rj / d_j, a_rt -= f_r a_tj (t > j).
// The pivots d_t end up on the diagonal (a_tt), so the scaling
// 1/sqrt(d_t) is computed once per lane in parallel and broadcast.
// Writes the scaled L columns c0..c0+15 (rows c0..m-1) into T.
//
// Columns are eliminated in pairs (2 x 2 pivot block B of the updated
// matrix): [f0, f1]_r = [a_rj, a_r,j+1] B^-1 and a_rt -= f0 a_tj + f1 a_t,j+1
// for t > j+1 — the same Schur complement as two 1 x 1 steps, with one
// reciprocal per pair on the chain.  Column j+1 is then brought to its 1 x 1
// form (a_r,j+1 -= a_rj e / d_j) off the chain, so the final scaling and
// the pivots on the diagonal are those of the column-by-column sweep.
// Per pair the chain is: B by readlane from its two lanes -> det, reciprocal
// -> f -> update of the NEXT pair's two columns; the other columns' entries
// of the pivot columns travel through LDS one pair ahead (wave_barrier keeps
// the publish ahead of the reads), off the chain.  Measured per 16 columns
// (tools/sweep_probe.hip): ~3.4k cycles with B through LDS too.
__device__ __forceinline__ void panel_sweep(double (*T)[LDP], CholLds& W, int c0, int b, int m) {
  // the row index is made opaque here, so that the sweep's row masks are
  // formed per sweep instead of being hoisted out of the caller's loops
  // (in the persistent kernel they would stay live, as spilled SGPRs, across
  // its whole block-column loop)
  const int r = ctid() & 63;
  // likewise the broadcast reads' base (an opaque zero in the column index):
  // with compile-time c0 their LDS addresses are constants, and hoisted out
  // of the loops they held one VGPR each for the whole kernel
  int zo = 0;
  asm volatile("" : "+v"(zo));
  double2 (*colp)[CB] = reinterpret_cast<double2 (*)[CB]>(&W.colp[0][zo]);
  double a[16];
  {  // row r, columns c0..c0+15: 8 unconditional 16-B reads, then selects
    const double2* src = reinterpret_cast<const double2*>(&T[r][c0]);
    double2 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = src[k];
#pragma unroll
    for (int cc = 0; cc < 16; ++cc) {
      const int t = c0 + cc;
      const double x = (cc & 1) ? v[cc >> 1].y : v[cc >> 1].x;
      a[cc] = (r >= c0 && r < m && t < b && (t <= r || r >= b)) ? x : 0.0;
    }
  }
  CHOL_STAMP(30 + c0 / 16 * 4);
  W.colp[0][r] = make_double2(a[0], a[1]);
  __builtin_amdgcn_wave_barrier();
  double2 ct[16];
#pragma unroll
  for (int t = 2; t < 16; ++t) ct[t] = colp[0][c0 + t];
  // the pivot block of the first pair from its two rows' lanes (readlane: no
  // LDS round trip on the chain; the same bits an LDS broadcast carries)
  double d0 = readlane_f64(a[0], c0), e = readlane_f64(a[0], c0 + 1), d1 = readlane_f64(a[1], c0 + 1);
  double rdet = recip(d0 * d1 - e * e), rd0 = recip(d0);
#pragma unroll
  for (int jj = 0; jj < 16; jj += 2) {
    const int j = c0 + jj;
    if (j + 1 >= b) break;                   // uniform: a last single column needs no update
    const int buf = (jj >> 1) & 1;
    // (no row mask: rows r <= j + 1 and r >= m update only entries that are
    // never read again — strictly-upper ones, or rows outside the tile — and
    // the final store masks them; every row > j + 1 of the tile computes
    // exactly what the masked form computed)
    const double u0 = a[jj], u1 = a[jj + 1];
    const double f0 = fma(u0, d1, -u1 * e) * rdet;
    const double f1 = fma(u1, d0, -u0 * e) * rdet;
    const double ej = e, rd0j = rd0;
    if (jj + 2 < 16) {
      // the chain: the next pair's two columns, then its pivot block
      a[jj + 2] = fma(-f1, ct[jj + 2].y, fma(-f0, ct[jj + 2].x, a[jj + 2]));
      a[jj + 3] = fma(-f1, ct[jj + 3].y, fma(-f0, ct[jj + 3].x, a[jj + 3]));
      if (j + 3 < b) {
        d0 = readlane_f64(a[jj + 2], j + 2);
        e = readlane_f64(a[jj + 2], j + 3);
        d1 = readlane_f64(a[jj + 3], j + 3);
        rdet = recip(d0 * d1 - e * e);
        rd0 = recip(d0);
      }
      // off the chain (their latency hides under it): the later columns'
      // pivot-column entries through LDS one pair ahead (wave_barrier keeps
      // the publish ahead of the reads) and their updates
      double2 ctn[16];
      if (jj + 4 < 16) {
        W.colp[buf ^ 1][r] = make_double2(a[jj + 2], a[jj + 3]);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int t = jj + 4; t < 16; ++t) ctn[t] = colp[buf ^ 1][c0 + t];
      }
#pragma unroll
      for (int t = jj + 4; t < 16; ++t) a[t] = fma(-f1, ct[t].y, fma(-f0, ct[t].x, a[t]));
#pragma unroll
      for (int t = jj + 4; t < 16; ++t) ct[t] = ctn[t];
    }
    // column j+1 to its 1 x 1 form (rows r > j; lane j+1 gets the pivot
    // d1 - e^2/d0; unmasked like the updates above)
    a[jj + 1] -= u0 * (ej * rd0j);
  }
  CHOL_STAMP(31 + c0 / 16 * 4);
  // own pivot (lanes c0..c0+15): d_r = a_rr
  double d_own = 1.0;
#pragma unroll
  for (int cc = 0; cc < 16; ++cc)
    if (r == c0 + cc) d_own = a[cc];
  const bool own = r >= c0 && r < c0 + 16;
  if (own && r < b && !(d_own > 0.0 && isfinite(d_own))) W.bad = 1;
  const double rs_own = rsqrt_nr(d_own);
  // broadcast the 16 scalings through LDS (in order within the wave); they
  // stay there as 1 / L_tt for the diagonal-block inverse
  if (own) W.rsv[r] = rs_own;
  __builtin_amdgcn_sched_barrier(0);
  double rs[16];
  {
    const double2* src = reinterpret_cast<const double2*>(&W.rsv[c0]);
#pragma unroll
    for (int k = 0; k < 8; ++k) { const double2 x = src[k]; rs[2 * k] = x.x; rs[2 * k + 1] = x.y; }
  }
  if (r >= c0 && r < m) {
    double2* dst = reinterpret_cast<double2*>(&T[r][c0]);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      double lv[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int cc = 2 * k + h, t = c0 + cc;
        lv[h] = (t < b && t <= r) ? a[cc] * rs[cc] : 0.0;   // t == r: sqrt(d_t) = d_t / sqrt(d_t)
      }
      dst[k] = make_double2(lv[0], lv[1]);
    }
  }
}

// X_pp = L_pp^-1 for one 16x16 diagonal block p by the calling wave: lane
// c < 16 solves L_pp x = e_c by column-oriented forward substitution (x_k
// final -> every later row's sum takes its term at once), so the chain per
// row is one multiply and one FMA; L values are uniform LDS broadcasts, the
// next column read one step ahead; 1/L_ii is the sweep's 1/sqrt(d_i), no
// divisions.  The sums run over k in the same order as a row-oriented
// substitution (fma(-L_ik, x_k, s), k ascending).  (The row-oriented form has
// a 120-FMA chain: ~5.7k cycles on the critical path of the last row block.)
__device__ __forceinline__ void diag_inverse16(const double (*T)[LDP], const double* rinv, double (*X)[LDP], int p,
                                               int b) {
  const int c = ctid() & 63;
  const int c0 = 16 * p;
  if (c0 >= b || c >= 16) return;
  // (uniform reads from an opaque base: see panel_sweep)
  int zo = 0;
  asm volatile("" : "+v"(zo));
  T = reinterpret_cast<const double (*)[LDP]>(&T[0][zo]);
  double ri[16];
  {
    const double2* src = reinterpret_cast<const double2*>(&rinv[c0]);
#pragma unroll
    for (int k = 0; k < 8; ++k) { const double2 v = src[k]; ri[2 * k] = v.x; ri[2 * k + 1] = v.y; }
  }
  double acc[16], col[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = (i == c) ? 1.0 : 0.0;
#pragma unroll
  for (int i = 1; i < 16; ++i) col[i] = T[c0 + i][c0];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    double nxt[16];
#pragma unroll
    for (int i = k + 2; i < 16; ++i) nxt[i] = T[c0 + i][c0 + k + 1];
    const double xk = (c0 + k < b) ? acc[k] * ri[k] : 0.0;
    acc[k] = xk;
#pragma unroll
    for (int i = k + 1; i < 16; ++i) acc[i] = fma(-col[i], xk, acc[i]);
#pragma unroll
    for (int i = k + 2; i < 16; ++i) col[i] = nxt[i];
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) X[c0 + i][c0 + c] = acc[i];
}

// Z_q (16x16, rows zr.. of Z; Z's row stride ZLD) = sum_{k=q}^{p-1} L_pk X_kq, by the calling wave
template <int ZLD>
__device__ __forceinline__ void inv_offdiag_sum(const double (*T)[LDP], const double (*X)[LDP], double (*Z)[ZLD],
                                                int p, int q, int zr) {
  d4 acc = d4{0.0, 0.0, 0.0, 0.0};
  for (int k = q; k < p; ++k) acc = mfma_tile_n<16>(acc, T, 16 * p, 16 * k, X, 16 * k, 16 * q, 1.0);
  tile_store<ZLD>(Z, zr, 0, acc);
}
// X_pq = -X_pp Z_q
template <int ZLD>
__device__ __forceinline__ void inv_offdiag_fin(double (*X)[LDP], const double (*Z)[ZLD], int p, int q, int zr) {
  d4 acc = d4{0.0, 0.0, 0.0, 0.0};
  acc = mfma_tile_n<16, ZLD>(acc, X, 16 * p, 16 * p, Z, zr, 0, -1.0);
  tile_store(X, 16 * p, 16 * q, acc);
}

// Row block p of X = L^-1 by ONE wave (diagonal block, then the blocks
// (p, q < p) from the finished rows above); Z rows 16 zw.. are its scratch.
// LDS operations of one wave complete in order, so no barrier inside.
template <int ZLD>
__device__ __forceinline__ void inverse_rowblock(const double (*T)[LDP], const double* rinv, double (*X)[LDP],
                                                 double (*Z)[ZLD], int p, int b, int zw) {
  diag_inverse16(T, rinv, X, p, b);
  for (int q = 0; q < p; ++q) {
    inv_offdiag_sum(T, X, Z, p, q, 16 * zw);
    inv_offdiag_fin(X, Z, p, q, 16 * zw);
  }
}

// Factor the 64x64 block in four 16-column sub-panels (wave 0 sweeps, all
// waves apply the trailing updates) and form X = L^-1 row block by row block:
// row block p - 1 (wave 1) overlaps the sweep of sub-panel p, so only the
// last row block follows the factorization (its off-diagonal sums spread
// over waves 1..3).
// Pc != nullptr: T is final in its column-0 tiles only; waves 1..3 apply
// the rest of C = T - Pc Pc^T (mfma_xxT_rest) during the first sweep (Pc
// must stay intact until the first sub-panel's barrier: Z aliases it only
// from sub-panel 1 on).
// Z: inverse scratch, rows 16..63 used (row stride ZLD >= 16).  X may alias
// Pc (written from the second sub-panel on).
// Hook: work for waves 2 and 3 while wave 0 sweeps sub-panel p = 1, 2, 3 and
// wave 1 inverts row block p - 1 (the persistent factorisation prefetches its
// next panel tile there); the per-step kernels pass none.
// hook.land(): waves 2 and 3 again, in the inverse tail beside wave 0's last
// diagonal inverse; hook.finish(): waves 2 and 3 at the end of the tail.
struct NoFactorHook {
  __device__ void operator()(int) const {}
  __device__ void land() const {}
  __device__ void finish() const {}
};
// A workgroup barrier for LDS only: every hand-off inside the factor goes
// through LDS, and __syncthreads' release fence would also drain every global
// load and store in flight (the persistent factorisation's next-panel
// prefetch, V's row blocks stored as they complete)
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
// FULL: b = m = CB (every block but the last): the sub-panel loop is
// unrolled, so the sweeps' row predicates and LDS offsets are compile-time
// (tools/sweep_probe.hip: a sweep with run-time c0 / b / m costs ~800 more
// cycles of its ~3.5k).
template <bool FULL, int ZLD, class Hook>
__device__ __forceinline__ void factor_invert_impl(double (*T)[LDP], double (*X)[LDP], double (*Z)[ZLD], CholLds& W,
                                                   int b, int m, const double (*Pc)[LDP], const Hook& hook) {
  if constexpr (FULL) { b = CB; m = CB; }
  const int w = cwave();
  lds_barrier();
  CHOL_STAMP(2);
  int last = 0;
  // one trailing-update tile (ti, ts) -= (sub-panel c0 columns) products
  auto upd_tile = [&](int ti, int ts, int c0) {
    d4 acc = tile_load(T, 16 * ti, 16 * ts);
    acc = mfma_tile<16>(acc, T, 16 * ti, c0, T, 16 * ts, c0, -1.0);
    tile_store(T, 16 * ti, 16 * ts, acc);
  };
  auto subpanel = [&](const int p) {
    const int c0 = 16 * p;
    last = p;
    if (w == 0) panel_sweep(T, W, c0, b, m);
    else if (w == 1 && p > 0) inverse_rowblock(T, W.rsv, X, Z, p - 1, b, 1);
    else if (p == 0 && Pc != nullptr) mfma_xxT_rest(Pc, T);
    else if (p >= 1) {
      // FULL: sub-panel 0's updates of tiles (3, 2) and (3, 3), which only
      // sub-panels 2 and 3 read, run here beside the sweep of sub-panel 1
      // (waves 2, 3) instead of as a second round before it; each tile
      // still takes its sub-panel-0 update before its sub-panel-1 one
      if constexpr (FULL) {
        if (p == 1) upd_tile(3, w == 2 ? 2 : 3, 0);
      }
      hook(p);
    }
    CHOL_STAMP(10 + 2 * p);
    lds_barrier();
    if constexpr (FULL) {
      if (p == 0) {   // the tiles the next sweeps read first: one round
        const int ti = w == 0 ? 1 : (w == 1 ? 2 : (w == 2 ? 2 : 3));
        const int ts = w == 2 ? 2 : 1;
        upd_tile(ti, ts, c0);
        lds_barrier();
        CHOL_STAMP(11 + 2 * p);
        return;
      }
    }
    // trailing update of the remaining sub-panels: tiles (i, s), p < s <= i
    {
      const int nt = 3 - p;                  // tile rows below the sub-panel
      const int ntiles = nt * (nt + 1) / 2;
      for (int e = w; e < ntiles; e += 4) {
        int i = 0, s2 = e;
        while (s2 > i) { s2 -= i + 1; ++i; }  // e -> (i, s2), s2 <= i
        const int ti = p + 1 + i, ts = p + 1 + s2;
        if (16 * ti >= m || 16 * ts >= b) continue;
        d4 acc = tile_load(T, 16 * ti, 16 * ts);
        acc = mfma_tile<16>(acc, T, 16 * ti, c0, T, 16 * ts, c0, -1.0);
        tile_store(T, 16 * ti, 16 * ts, acc);
      }
    }
    lds_barrier();
    CHOL_STAMP(11 + 2 * p);
  };
  if constexpr (FULL) {
#pragma unroll
    for (int p = 0; p < 4; ++p) subpanel(p);
  } else {
#pragma unroll 1
    for (int p = 0; p < 4 && 16 * p < b; ++p) subpanel(p);
  }
  CHOL_STAMP(3);
  // last row block: diagonal inverse (wave 0) beside the sums Z_q (wave q + 1)
  // and the landing of the hook's loads (waves 2, 3: under wave 0's chain)
  if (w == 0) diag_inverse16(T, W.rsv, X, last, b);
  else if (w - 1 < last) inv_offdiag_sum(T, X, Z, last, w - 1, 16 * w);
  if (w >= 2) hook.land();
  CHOL_STAMP(40);
  lds_barrier();
  CHOL_STAMP(41);
  if (w >= 1 && w - 1 < last) inv_offdiag_fin(X, Z, last, w - 1, 16 * w);
  if (w >= 2) hook.finish();
  lds_barrier();
  CHOL_STAMP(4);
}
// KIND: 1 = the caller guarantees b = m = CB, 0 = the general form, -1 =
// chosen at run time (two copies of the code)
template <int KIND = -1, int ZLD = LDP, class Hook = NoFactorHook>
__device__ void factor_invert_blk(double (*T)[LDP], double (*X)[LDP], double (*Z)[ZLD], CholLds& W, int b, int m,
                                  const double (*Pc)[LDP] = nullptr, const Hook& hook = Hook{}) {
  if constexpr (KIND == 1) factor_invert_impl<true>(T, X, Z, W, b, m, Pc, hook);
  else if constexpr (KIND == 0) factor_invert_impl<false>(T, X, Z, W, b, m, Pc, hook);
  else if (b == CB && m == CB) factor_invert_impl<true>(T, X, Z, W, b, m, Pc, hook);
  else factor_invert_impl<false>(T, X, Z, W, b, m, Pc, hook);
}

}  // namespace bahip

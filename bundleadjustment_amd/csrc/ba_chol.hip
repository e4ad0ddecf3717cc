// ba_chol.hip — dense blocked Cholesky of the reduced camera system on gfx950.
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
constexpr int LDP = CB + 2;      // padded LDS row (doubles): conflict-free MFMA operand reads (16 rows x 4 k per wave)

typedef double d4 __attribute__((ext_vector_type(4)));

// Diagnostic build only (tools/chol_bench.hip defines BA_CHOL_STAMPS): the
// critical workgroup records s_memtime at phase boundaries into g_stamps.
#ifdef BA_CHOL_STAMPS
__device__ unsigned long long g_stamps[64];
#define CHOL_STAMP(i)                                                                         \
  do {                                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    unsigned long long t_;                                                                    \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    if (threadIdx.x == 0) g_stamps[i] = t_;                                                   \
  } while (0)
#else
#define CHOL_STAMP(i) do {} while (0)
#endif

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
  const int tid = threadIdx.x;
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
  const int tid = threadIdx.x;
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int e = tid + 256 * it;
    const int i = e >> 5, j = (e & 31) * 2;
    D[i][j] = t.v[it].x;
    D[i][j + 1] = t.v[it].y;
  }
}
__device__ inline void stage64(double (*D)[LDP], const double* __restrict__ M, size_t ld, int r0, int c0, int rmax,
                               int cmax) {
  tile_put(D, tile_fetch(M, ld, r0, c0, rmax, cmax));
}

// C (64x64, distributed as 4 waves x 2x2 MFMA tiles of 16x16) = sum_k Xs[i][k] Ys[j][k]
__device__ inline void mfma_xyT_64(const double (*Xs)[LDP], const double (*Ys)[LDP], d4 acc[2][2]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
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
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
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

// P = Xs V^T with V lower triangular (V[j][k] = 0 for k > j): wave w owns
// the row strip 16w..16w+15, and output column tile bc needs only k <
// 16 (bc + 1) -> 40 MFMAs per wave (the square product: 64).
// acc[bc] element g: row 16w + (lane >> 4) + 4g, col 16bc + (lane & 15).
__device__ inline void mfma_xVT_strip(const double (*Xs)[LDP], const double (*Vs)[LDP], d4 acc[4]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
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
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
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
  for (int e = threadIdx.x; e < CB * CB; e += 256) {
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
  const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int k0 = 0; k0 < K; k0 += 4) {
    const double x = sgn * Xs[xr + li][xc + k0 + lk];
    const double y = Ys[yr + li][yc + k0 + lk];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc, 0, 0, 0);
  }
  return acc;
}

// same with the second operand transposed: Ys[yr + k][yc + j]
template <int K>
__device__ __forceinline__ d4 mfma_tile_n(d4 acc, const double (*Xs)[LDP], int xr, int xc, const double (*Ys)[LDP],
                                          int yr, int yc, double sgn) {
  const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int k0 = 0; k0 < K; k0 += 4) {
    const double x = sgn * Xs[xr + li][xc + k0 + lk];
    const double y = Ys[yr + k0 + lk][yc + li];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc, 0, 0, 0);
  }
  return acc;
}

__device__ __forceinline__ d4 tile_load(const double (*S)[LDP], int r0, int c0) {
  const int lane = threadIdx.x & 63;
  d4 v;
#pragma unroll
  for (int g = 0; g < 4; ++g) v[g] = S[r0 + (lane >> 4) + 4 * g][c0 + (lane & 15)];
  return v;
}

__device__ __forceinline__ void tile_store(double (*S)[LDP], int r0, int c0, d4 v) {
  const int lane = threadIdx.x & 63;
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
// Per pair the chain is: LDS read of B -> det, reciprocal -> f -> update of
// the NEXT pair's two columns -> LDS publish (sched_barriers keep the publish
// and the next reads ahead of the remaining updates).  Measured per 16
// columns (tools/chol_bench.hip): 1 x 1 pivots ~5.7k cycles.
__device__ __forceinline__ void panel_sweep(double (*T)[LDP], CholLds& W, int c0, int b, int m) {
  const int r = threadIdx.x & 63;
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
  __builtin_amdgcn_sched_barrier(0);
  double2 q0 = W.colp[0][c0], q1 = W.colp[0][c0 + 1];
  double2 ct[16];
#pragma unroll
  for (int t = 2; t < 16; ++t) ct[t] = W.colp[0][c0 + t];
#pragma unroll
  for (int jj = 0; jj < 16; jj += 2) {
    const int j = c0 + jj;
    if (j + 1 >= b) break;                   // uniform: a last single column needs no update
    const int buf = (jj >> 1) & 1;
    const double d0 = q0.x, e = q1.x, d1 = q1.y;
    const double rdet = recip(d0 * d1 - e * e);
    const bool row = r > j + 1 && r < m;
    const double u0 = a[jj], u1 = a[jj + 1];
    const double f0 = row ? fma(u0, d1, -u1 * e) * rdet : 0.0;
    const double f1 = row ? fma(u1, d0, -u0 * e) * rdet : 0.0;
    if (jj + 2 < 16) {
      a[jj + 2] = fma(-f1, ct[jj + 2].y, fma(-f0, ct[jj + 2].x, a[jj + 2]));
      a[jj + 3] = fma(-f1, ct[jj + 3].y, fma(-f0, ct[jj + 3].x, a[jj + 3]));
      W.colp[buf ^ 1][r] = make_double2(a[jj + 2], a[jj + 3]);
      __builtin_amdgcn_sched_barrier(0);
      const double2 q0n = W.colp[buf ^ 1][c0 + jj + 2], q1n = W.colp[buf ^ 1][c0 + jj + 3];
      double2 ctn[16];
#pragma unroll
      for (int t = jj + 4; t < 16; ++t) ctn[t] = W.colp[buf ^ 1][c0 + t];
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = jj + 4; t < 16; ++t) a[t] = fma(-f1, ct[t].y, fma(-f0, ct[t].x, a[t]));
      q0 = q0n;
      q1 = q1n;
#pragma unroll
      for (int t = jj + 4; t < 16; ++t) ct[t] = ctn[t];
    }
    // column j+1 to its 1 x 1 form (rows r > j; lane j+1 gets the pivot d1 - e^2/d0)
    if (r > j && r < m) a[jj + 1] -= u0 * (e * recip(d0));
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

// X_pp = L_pp^-1 for the four 16x16 diagonal blocks, one wave each (lane
// c < 16 solves L_pp x = e_c by forward substitution; L values are uniform
// LDS broadcasts; 1/L_ii is the sweep's 1/sqrt(d_i), no divisions).
__device__ __forceinline__ void diag_inverse16(const double (*T)[LDP], const double* rinv, double (*X)[LDP], int b) {
  const int w = threadIdx.x >> 6, c = threadIdx.x & 15;
  const int c0 = 16 * w;
  if (c0 >= b || (threadIdx.x & 63) >= 16) return;
  double x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    double s = (i == c) ? 1.0 : 0.0;
#pragma unroll
    for (int k = 0; k < i; ++k) s -= T[c0 + i][c0 + k] * x[k];
    x[i] = (c0 + i < b) ? s * rinv[c0 + i] : 0.0;   // rinv = 1 / L_ii from the sweep
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) X[c0 + i][c0 + c] = x[i];
}

__device__ void factor_invert_blk(double (*T)[LDP], double (*X)[LDP], double (*Z)[LDP], CholLds& W, int b, int m) {
  const int w = threadIdx.x >> 6;
  __syncthreads();
  CHOL_STAMP(2);
  for (int p = 0; p < 4; ++p) {
    const int c0 = 16 * p;
    if (c0 >= b) break;                      // uniform
    if (w == 0) panel_sweep(T, W, c0, b, m);
    CHOL_STAMP(10 + 2 * p);
    __syncthreads();
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
    __syncthreads();
    CHOL_STAMP(11 + 2 * p);
  }
  CHOL_STAMP(3);
  diag_inverse16(T, W.rsv, X, b);
  CHOL_STAMP(40);
  __syncthreads();
  CHOL_STAMP(41);
  // off-diagonal blocks of X = L^-1, by block distance dd
  for (int dd = 1; dd < 4; ++dd) {
    const int i = dd + w, pp = w;            // wave w: block (dd + w, w)
    const bool act = i < 4 && 16 * i < b;
    if (act) {
      d4 acc = d4{0.0, 0.0, 0.0, 0.0};
      for (int k = pp; k < i; ++k) acc = mfma_tile_n<16>(acc, T, 16 * i, 16 * k, X, 16 * k, 16 * pp, 1.0);
      tile_store(Z, 16 * w, 0, acc);
    }
    __syncthreads();
    if (act) {
      d4 acc = d4{0.0, 0.0, 0.0, 0.0};
      acc = mfma_tile_n<16>(acc, X, 16 * i, 16 * i, Z, 16 * w, 0, -1.0);
      tile_store(X, 16 * i, 16 * pp, acc);
    }
    __syncthreads();
  }
  CHOL_STAMP(4);
}

// One block step.  k < 0: factor block 0 only (grid 1x1).
//   A    working matrix ((n+1) x ld), trailing part updated in place
//   L    output factor ((n+1) x ld)
//   Vbuf [T][64][64] inverses of the diagonal blocks
// SPLIT (large systems): the panel L_{I,k} = A_{I,k} V_k^T was formed and
// stored by k_chol_panel just before; every tile reads it from L, so a tile
// does one GEMM instead of three (the fused form recomputes P_I, P_J per
// tile: 3x the flops and ~2.5x the bytes, which dominate once the trailing
// matrix has thousands of tiles).
template <bool SPLIT>
__global__ __launch_bounds__(256) void k_chol_step(double* __restrict__ A, double* __restrict__ L, int ld, int n,
                                                   int k, double* __restrict__ Vbuf, double* __restrict__ scal) {
  const int I = blockIdx.y, J = blockIdx.x;
  if (J > I) return;
  __shared__ double S0[CB][LDP];
  __shared__ double S1[CB][LDP];
  __shared__ double S2[CB][LDP];
  __shared__ CholLds cw;
  const int nrows = n + 1;
  const size_t lds = (size_t)ld;
  const int s = (k + 1) * CB;                 // first row/col of the trailing matrix
  const int kc = k * CB;                      // column offset of block k
  const int kb = k >= 0 ? min(CB, n - kc) : 0;
  const int r0 = s + I * CB, c0 = s + J * CB;
  const double* Vk = k >= 0 ? Vbuf + (size_t)k * CB * CB : nullptr;
  if (I == 0 && J == 0) {
    // ---- critical workgroup: next diagonal block
    const int b = min(CB, n - s);             // its order
    const int m = min(CB, nrows - s);         // rows in the tile (b or b + 1 with the rhs row)
    CHOL_STAMP(0);
    if (SPLIT && k >= 0) {
      const TileRegs tA = tile_fetch<true>(A, lds, s, s, nrows, s + b);   // A_{k+1,k+1} (+ rhs row)
      const TileRegs tP = tile_fetch(L, lds, s, kc, nrows, kc + kb);      // L_{k+1,k} (k_chol_panel)
      tile_put(S0, tA);
      tile_put(S1, tP);
      __syncthreads();
      mfma_xxT_lower_sub(S1, S0);            // C = A - P P^T (lower tiles)
    } else if (k >= 0) {
      // the three tiles' loads all in flight before the first LDS store
      const TileRegs tA = tile_fetch<true>(A, lds, s, s, nrows, s + b);   // A_{k+1,k+1} (+ rhs row)
      const TileRegs tP = tile_fetch(A, lds, s, kc, nrows, kc + kb);      // A_{k+1,k}
      const TileRegs tV = tile_fetch<true>(Vk, CB, 0, 0, CB, CB);         // V_k (lower triangular)
      tile_put(S0, tA);
      tile_put(S1, tP);
      tile_put(S2, tV);
      __syncthreads();
      CHOL_STAMP(20);
      d4 acc[4];
      mfma_xVT_strip(S1, S2, acc);           // P = A_{k+1,k} V_k^T
      __syncthreads();
      CHOL_STAMP(21);
      // P -> LDS, and L_{k+1,k} straight from the accumulators (16
      // consecutive columns per 16 lanes); the stores drain while the
      // factorization runs
      {
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
        for (int bc = 0; bc < 4; ++bc)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int rr = 16 * w + (lane >> 4) + 4 * g, cc = 16 * bc + (lane & 15);
            S1[rr][cc] = acc[bc][g];
            if (rr < m && cc < kb) L[(size_t)(s + rr) * ld + kc + cc] = acc[bc][g];
          }
      }
      __syncthreads();
      CHOL_STAMP(22);
      mfma_xxT_lower_sub(S1, S0);            // C = A - P P^T (lower tiles)
      CHOL_STAMP(23);
    } else {
      stage64(S0, A, lds, s, s, nrows, s + b);
    }
    if (threadIdx.x == 0) cw.bad = 0;
    CHOL_STAMP(1);
    factor_invert_blk(S0, S2, S1, cw, b, m);   // rows b..m-1 (rhs) come out as L rows too
    CHOL_STAMP(5);
    __syncthreads();
    // only V_{k+1} and the rhs row of L leave the workgroup: the diagonal L
    // block itself is never read again (back substitution uses V)
    {
      double2* Vd = reinterpret_cast<double2*>(Vbuf + (size_t)(k + 1) * CB * CB);
      for (int e2 = threadIdx.x; e2 < CB * CB / 2; e2 += 256) {
        const int i = (2 * e2) / CB, j = (2 * e2) % CB;
        double v[2];
#pragma unroll
        for (int h = 0; h < 2; ++h)
          v[h] = (j + h <= i && i < b && j + h < b) ? S2[i][j + h] : (i == j + h ? 1.0 : 0.0);
        Vd[e2] = make_double2(v[0], v[1]);
      }
      if (m > b)
        for (int j = threadIdx.x; j < b; j += 256) L[(size_t)(s + b) * ld + s + j] = S0[b][j];
    }
    CHOL_STAMP(6);
    if (threadIdx.x == 0 && cw.bad) scal[SL_CHOL_BAD] += 1.0;
    return;
  }
  // ---- trailing tile (I, J) != (0, 0)
  if (k < 0) return;
  if (r0 >= nrows || c0 >= n) return;
  if (SPLIT) {
    const TileRegs tI = tile_fetch(L, lds, r0, kc, nrows, kc + kb);   // L_{I,k}
    if (I != J) {
      const TileRegs tJ = tile_fetch(L, lds, c0, kc, n, kc + kb);     // L_{J,k}
      tile_put(S1, tJ);
    }
    tile_put(S0, tI);
    __syncthreads();
    d4 acc[2][2];
    mfma_xyT_64(S0, I != J ? S1 : S0, acc);
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          int rr, cc;
          acc_pos(a, b, g, &rr, &cc);
          const int ri = r0 + rr, cj = c0 + cc;
          if (ri < nrows && cj < n && cj <= ri) A[(size_t)ri * ld + cj] -= acc[a][b][g];
        }
    return;
  }
  stage64(S2, Vk, CB, 0, 0, CB, CB);
  stage64(S0, A, lds, r0, kc, nrows, kc + kb);   // A_{I,k}
  if (I != J) stage64(S1, A, lds, c0, kc, n, kc + kb);  // A_{J,k}
  __syncthreads();
  d4 acc[2][2];
  mfma_xyT_64(S0, S2, acc);                  // P_I
  d4 accJ[2][2];
  if (I != J) mfma_xyT_64(S1, S2, accJ);     // P_J
  __syncthreads();
  acc_to_lds(S0, acc, 0);
  if (I != J) acc_to_lds(S1, accJ, 0);
  __syncthreads();
  const int mI = min(CB, nrows - r0);
  if (J == 0) lds_to_global(S0, L, lds, r0, kc, mI, kb);   // L_{I,k} final
  mfma_xyT_64(S0, I != J ? S1 : S0, acc);    // P_I P_J^T
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        int rr, cc;
        acc_pos(a, b, g, &rr, &cc);
        const int ri = r0 + rr, cj = c0 + cc;
        if (ri < nrows && cj < n && cj <= ri) A[(size_t)ri * ld + cj] -= acc[a][b][g];
      }
}

// ---------------------------------------------------------------------------
// back substitution L^T y = z (z = row n of L) as a dataflow over block
// columns: workgroup K owns y_K = V_K^T (z_K - sum_{J>K} L_JK^T y_J).  It
// folds in the contribution of every y_J (J = T-1 .. K+1) as soon as
// workgroup J has published it, prefetching the L_JK tile before it polls,
// so the serial chain per block is one hand-off plus two 64x64 GEMVs (the
// single-workgroup sweep it replaces was bound by one CU pulling all of L:
// 152 us at n = 1194).
//
// Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility): producer =
// plain stores of y_K -> every storing wave s_waitcnt vmcnt(0) -> barrier ->
// one lane: agent release fence -> vmcnt(0) -> relaxed agent flag store;
// consumer = one lane polls the flag (relaxed, agent, s_sleep) -> agent
// acquire fence -> vmcnt(0) -> barrier -> plain loads.  Flags are zeroed
// by a memset node before every launch; spins are bounded (a missing
// producer sets the failure slot instead of hanging the GPU).
// ---------------------------------------------------------------------------
constexpr long kSpinMax = 1L << 26;

__device__ inline void flag_publish(int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// returns false if the spin bound was hit
__device__ inline bool flag_wait(int* flag, int* lds_ok) {
  if (threadIdx.x == 0) {
    long it = 0;
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0 && it < kSpinMax) {
      __builtin_amdgcn_s_sleep(1);
      ++it;
    }
    *lds_ok = it < kSpinMax;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  return *lds_ok != 0;
}

__global__ __launch_bounds__(256) void k_back_flow(const double* __restrict__ A, const double* __restrict__ Lm,
                                                   int ld, int n, const double* __restrict__ Vall,
                                                   double* __restrict__ y, int* __restrict__ flags,
                                                   double* __restrict__ scal) {
  __shared__ double zs[CB];
  __shared__ double ys[CB];
  __shared__ double part[4][CB];
  __shared__ int ok;
  const int K = blockIdx.x, tid = threadIdx.x;
  const int T = (n + CB - 1) / CB;
  const int s0 = K * CB, bsz = min(CB, n - s0);
  const size_t lds = (size_t)ld;
  // thread (j = tid & 63, h = tid >> 6) sums rows i = h, h + 4, ... of a tile
  const int j = tid & 63, h = tid >> 6;
  if (n % CB == 0 && K == T - 1) {
    // the rhs row starts a tile row of its own: no step factored it into
    // z_K, the last trailing update left A_{n,K}; z_K = V_K A_{n,K}^T
    if (tid < CB) ys[tid] = A[(size_t)n * lds + s0 + tid];
    __syncthreads();
    const double* V = Vall + (size_t)K * CB * CB;
    double t = 0.0;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int i = h + 4 * q;
      t += V[(size_t)j * CB + i] * ys[i];
    }
    part[h][j] = t;
    __syncthreads();
    if (tid < CB) zs[tid] = (part[0][tid] + part[1][tid]) + (part[2][tid] + part[3][tid]);
    __syncthreads();
  } else if (tid < CB) {
    zs[tid] = tid < bsz ? Lm[(size_t)n * lds + s0 + tid] : 0.0;
  }
  double acc = 0.0;
  bool good = true;
  for (int J = T - 1; J > K; --J) {
    const int sJ = J * CB, bJ = min(CB, n - sJ);
    double lv[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {   // L[sJ + i][s0 + j], i = h + 4 q (prefetched before the poll)
      const int i = h + 4 * q;
      lv[q] = (i < bJ && j < bsz) ? Lm[(size_t)(sJ + i) * lds + s0 + j] : 0.0;
    }
    good = flag_wait(flags + J, &ok) && good;
    if (tid < CB) ys[tid] = tid < bJ ? y[sJ + tid] : 0.0;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 16; ++q) acc += lv[q] * ys[h + 4 * q];
    __syncthreads();
  }
  part[h][j] = acc;
  __syncthreads();
  if (tid < CB) zs[tid] -= (part[0][tid] + part[1][tid]) + (part[2][tid] + part[3][tid]);
  __syncthreads();
  // y_K[j] = sum_{i >= j} V[i][j] z[i]
  {
    const double* V = Vall + (size_t)K * CB * CB;
    double t = 0.0;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int i = h + 4 * q;
      t += V[(size_t)i * CB + j] * zs[i];
    }
    part[h][j] = t;
  }
  __syncthreads();
  if (tid < CB && tid < bsz) y[s0 + tid] = (part[0][tid] + part[1][tid]) + (part[2][tid] + part[3][tid]);
  flag_publish(flags + K);
  if (tid == 0 && !good) scal[SL_CHOL_BAD] += 1.0;
}

// Panel of block step k (SPLIT mode): L_{I,k} = A_{I,k} V_k^T for every tile
// row I > k (the rhs row included), one workgroup per tile row.
__global__ __launch_bounds__(256) void k_chol_panel(const double* __restrict__ A, double* __restrict__ L, int ld,
                                                    int n, int k, const double* __restrict__ Vbuf) {
  __shared__ double S0[CB][LDP];
  __shared__ double S2[CB][LDP];
  const int nrows = n + 1;
  const size_t lds = (size_t)ld;
  const int kc = k * CB, kb = min(CB, n - kc);
  const int r0 = (k + 1) * CB + blockIdx.x * CB;
  if (r0 >= nrows) return;
  const TileRegs tA = tile_fetch(A, lds, r0, kc, nrows, kc + kb);
  const TileRegs tV = tile_fetch<true>(Vbuf + (size_t)k * CB * CB, CB, 0, 0, CB, CB);
  tile_put(S0, tA);
  tile_put(S2, tV);
  __syncthreads();
  d4 acc[4];
  mfma_xVT_strip(S0, S2, acc);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, m = min(CB, nrows - r0);
#pragma unroll
  for (int bc = 0; bc < 4; ++bc)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int rr = 16 * w + (lane >> 4) + 4 * g, cc = 16 * bc + (lane & 15);
      if (rr < m && cc < kb) L[(size_t)(r0 + rr) * ld + kc + cc] = acc[bc][g];
    }
}

// Block columns from which the split (panel + update) form is used: below it
// the fused step's trailing tiles hide behind the critical workgroup and one
// launch per step is cheaper (C3: 19 block columns); above it the trailing
// GEMMs dominate (C4: 94).
constexpr int kCholSplitBlocks = 24;

void launch_cholesky_solve2(const DevProblem& P, const DevWork& W, hipStream_t s) {
  const int n = P.n;
  if (n == 0) return;
  const int nrows = n + 1;
  const int T = (n + CB - 1) / CB;
  const bool split = T >= kCholSplitBlocks;
  hipLaunchKernelGGL(k_chol_step<false>, dim3(1, 1), dim3(256), 0, s, W.S, W.Lf, P.ld, n, -1, W.Vbuf, W.scal);
  for (int k = 0; k + 1 < T; ++k) {
    const int st = (k + 1) * CB;
    const int tr = (nrows - st + CB - 1) / CB, tc = (n - st + CB - 1) / CB;
    if (split) {
      hipLaunchKernelGGL(k_chol_panel, dim3(tr), dim3(256), 0, s, W.S, W.Lf, P.ld, n, k, W.Vbuf);
      hipLaunchKernelGGL(k_chol_step<true>, dim3(tc, tr), dim3(256), 0, s, W.S, W.Lf, P.ld, n, k, W.Vbuf, W.scal);
    } else {
      hipLaunchKernelGGL(k_chol_step<false>, dim3(tc, tr), dim3(256), 0, s, W.S, W.Lf, P.ld, n, k, W.Vbuf, W.scal);
    }
  }
  (void)hipMemsetAsync(W.flags, 0, sizeof(int) * T, s);
  hipLaunchKernelGGL(k_back_flow, dim3(T), dim3(256), 0, s, W.S, W.Lf, P.ld, n, W.Vbuf, W.y, W.flags, W.scal);
}

}  // namespace bahip

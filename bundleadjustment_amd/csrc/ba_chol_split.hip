// ba_chol_split.hip — split form of the dense Cholesky block step for large
// reduced systems (>= kCholSplitBlocks block columns, e.g. C4's 6000 rows):
// k_chol_panel forms L_{I,k} = A_{I,k} V_k^T once per tile row, then every
// trailing tile does a single GEMM.  Its own translation unit, so the fused
// step of ba_chol.hip keeps its code generation (a shared template changed
// the inlining of the critical workgroup's factor_invert_blk).
#include "ba_chol.h"

namespace bahip {

// One block step.  k < 0: factor block 0 only (grid 1x1).
//   A    working matrix ((n+1) x ld), trailing part updated in place
//   L    output factor ((n+1) x ld)
//   Vbuf [T][64][64] inverses of the diagonal blocks
// SPLIT (large systems): the panel L_{I,k} = A_{I,k} V_k^T was formed and
// stored by k_chol_panel just before; every tile reads it from L, so a tile
// does one GEMM instead of three (the fused form recomputes P_I, P_J per
// tile: 3x the flops and ~2.5x the bytes, which dominate once the trailing
// matrix has thousands of tiles).
// Grid: the lower tiles only, linear id -> (I, J <= I) (tile 0 = the
// critical block); a rhs-only last tile row (n % 64 == 0) follows them.
__device__ inline void split_tile_of(int lin, int tc, int& I, int& J) {
  const int tri = tc * (tc + 1) / 2;
  if (lin >= tri) { I = tc; J = lin - tri; return; }
  int i = (int)((sqrt(8.0 * lin + 1.0) - 1.0) * 0.5);
  while (i * (i + 1) / 2 > lin) --i;
  while ((i + 1) * (i + 2) / 2 <= lin) ++i;
  I = i;
  J = lin - i * (i + 1) / 2;
}
// The critical workgroup of block step k: C = A_{k+1,k+1} - L_{k+1,k}
// L_{k+1,k}^T (the panel from k_chol_panel; k < 0: block 0 as it is), then
// factor_invert_blk; V_{k+1} and the rhs row of L leave the workgroup.
__device__ __forceinline__ void split_critical(double* __restrict__ A, double* __restrict__ L, int ld, int n, int k,
                                               double* __restrict__ Vbuf, double* __restrict__ scal,
                                               double (*S0)[LDP], double (*S1)[LDP], double (*Zs)[18], CholLds& cw) {
  const int nrows = n + 1;
  const size_t lds = (size_t)ld;
  const int s = (k + 1) * CB;
  const int kc = k * CB;
  const int kb = k >= 0 ? min(CB, n - kc) : 0;
  // ---- critical workgroup: next diagonal block
  const int b = min(CB, n - s);             // its order
  const int m = min(CB, nrows - s);         // rows in the tile (b or b + 1 with the rhs row)
  CHOL_STAMP(0);
  if (k >= 0) {
    const TileRegs tA = tile_fetch<true>(A, lds, s, s, nrows, s + b);   // A_{k+1,k+1} (+ rhs row)
    const TileRegs tP = tile_fetch(L, lds, s, kc, nrows, kc + kb);      // L_{k+1,k} (k_chol_panel)
    tile_put(S0, tA);
    tile_put(S1, tP);
    __syncthreads();
    mfma_xxT_col0(S1, S0);                 // C = A - P P^T: column 0 now, the rest beside the first sweep
  } else {
    stage64(S0, A, lds, s, s, nrows, s + b);
  }
  if (threadIdx.x == 0) cw.bad = 0;
  CHOL_STAMP(1);
  factor_invert_blk<-1, 18>(S0, S1, Zs, cw, b, m, k >= 0 ? S1 : nullptr);   // rows b..m-1 (rhs) come out as L rows too
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
        v[h] = (j + h <= i && i < b && j + h < b) ? S1[i][j + h] : (i == j + h ? 1.0 : 0.0);
      Vd[e2] = make_double2(v[0], v[1]);
    }
    if (m > b)
      for (int j = threadIdx.x; j < b; j += 256) L[(size_t)(s + b) * ld + s + j] = S0[b][j];
  }
  CHOL_STAMP(6);
  if (threadIdx.x == 0 && cw.bad) scal[SL_CHOL_BAD] += 1.0;
}

__global__ __launch_bounds__(256) void k_chol_step_split(double* __restrict__ A, double* __restrict__ L, int ld, int n,
                                                   int k, double* __restrict__ Vbuf, double* __restrict__ scal) {
  int I, J;
  split_tile_of(blockIdx.x, (n - (k + 1) * CB + CB - 1) / CB, I, J);
  // two tiles + a narrow inverse scratch (78 KB: two workgroups per CU, so
  // one tile's operand loads overlap another's MFMAs); the critical
  // workgroup forms the block inverse in S1 once C = A - P P^T consumed it
  __shared__ double S0[CB][LDP];
  __shared__ double S1[CB][LDP];
  __shared__ double Zs[CB][18];
  __shared__ CholLds cw;
  const int nrows = n + 1;
  const size_t lds = (size_t)ld;
  const int s = (k + 1) * CB;                 // first row/col of the trailing matrix
  const int kc = k * CB;                      // column offset of block k
  const int kb = k >= 0 ? min(CB, n - kc) : 0;
  const int r0 = s + I * CB, c0 = s + J * CB;
  if (I == 0 && J == 0) {
    split_critical(A, L, ld, n, k, Vbuf, scal, S0, S1, Zs, cw);
    return;
  }
  // ---- trailing tile (I, J) != (0, 0)
  if (k < 0) return;
  if (r0 >= nrows || c0 >= n) return;
  const TileRegs tI = tile_fetch(L, lds, r0, kc, nrows, kc + kb);   // L_{I,k}
  TileRegs tJ;
  if (I != J) tJ = tile_fetch(L, lds, c0, kc, n, kc + kb);          // L_{J,k}
  // the A tile (read-modify-write target) is loaded with the operands, so
  // its latency hides behind the staging and the MFMAs (clamped addresses,
  // unconditional loads)
  double av[2][2][4];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        int rr, cc;
        acc_pos(a, b, g, &rr, &cc);
        av[a][b][g] = A[(size_t)min(r0 + rr, nrows - 1) * ld + min(c0 + cc, n - 1)];
      }
  if (I != J) tile_put(S1, tJ);
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
        if (ri < nrows && cj < n && cj <= ri) A[(size_t)ri * ld + cj] = av[a][b][g] - acc[a][b][g];
      }
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

// ---- grouped form (default): the trailing matrix takes the panels of a
// group of 4 block columns as ONE rank-256 update per tile instead of four
// rank-64 ones, so a trailing tile is read and written once per 4 block steps
// (A's read-modify-write traffic / 4; each tile's operand tiles come from L,
// which the L2 / Infinity Cache serves).  The chain keeps its one-step
// look-ahead: block step k forms panel k (k_chol_panel) and then launches
// k_chol_upd with the critical workgroup (diagonal block k + 1, panel k) and
// tile tasks A_IJ -= sum_{p in [pa, pb)} L_Ip L_Jp^T in up to 4 segments:
//   (i)   within group G = k / 4: columns (k + 1 .. 4G + 3], all rows, panel k
//         (the column k + 1 itself below the diagonal too);
//   (ii)  the next group's first diagonal tile D = (4G + 4, 4G + 4): panels
//         [4G - 4, 4G + 1) at k = 4G (group G - 1 and panel 4G), else panel k;
//         the critical workgroup applies panel 4G + 3 to it at k = 4G + 3;
//   (iii) k = 4G + 3: group G to the next group's columns [4G + 4, 4G + 8)
//         (their diagonal D excepted), due before panel 4G + 4;
//   (iv)  k = 4G + j, j < 3: a third of group G - 1's update of the columns
//         >= 4G + 4 (D excepted), column-ordered — due from step 4G + 7 on.
// Every tile (I, J) so receives the panels p < J exactly once before panel J
// (or diagonal block J) is formed, and no two tasks of one launch write the
// same tile.  Bitwise deterministic; not bitwise the rank-64 form (the sums
// are grouped differently): parity is against the oracle, as before.
struct CholUpdSeg {
  int ja, jb;      // block columns [ja, jb)
  int pa, pb;      // panels [pa, pb)
  int xd;          // column whose diagonal tile the segment skips (-1: none)
  int diag;        // 1: the diagonal tiles only
  int cnt;         // tiles
};
struct CholUpd {
  int k, nseg, TR;
  CholUpdSeg seg[4];
};

__host__ __device__ __forceinline__ int upd_col_tiles(const CholUpdSeg& g, int J, int TR) {
  return g.diag ? 1 : TR - J - (J == g.xd ? 1 : 0);
}

// A_IJ -= sum_{p in [pa, pb)} L_Ip L_Jp^T: operand tiles of panel p + 1 are
// fetched into registers while panel p's MFMAs run; A is read once, written once
__device__ __forceinline__ void upd_tile(double* __restrict__ A, const double* __restrict__ L, int ld, int n, int I,
                                         int J, int pa, int pb, double (*S0)[LDP], double (*S1)[LDP]) {
  const int nrows = n + 1;
  const size_t lds = (size_t)ld;
  const int r0 = I * CB, c0 = J * CB;
  const bool off = I != J;
  TileRegs tI = tile_fetch(L, lds, r0, pa * CB, nrows, min(pa * CB + CB, n));
  TileRegs tJ;
  if (off) tJ = tile_fetch(L, lds, c0, pa * CB, n, min(pa * CB + CB, n));
  double av[2][2][4];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        int rr, cc;
        acc_pos(a, b, g, &rr, &cc);
        av[a][b][g] = A[(size_t)min(r0 + rr, nrows - 1) * ld + min(c0 + cc, n - 1)];
      }
  d4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
  for (int p = pa; p < pb; ++p) {
    if (p > pa) __syncthreads();             // the previous panel's MFMAs are done with the tiles
    tile_put(S0, tI);
    if (off) tile_put(S1, tJ);
    __syncthreads();
    if (p + 1 < pb) {
      const int kc = (p + 1) * CB, ke = min(kc + CB, n);
      tI = tile_fetch(L, lds, r0, kc, nrows, ke);
      if (off) tJ = tile_fetch(L, lds, c0, kc, n, ke);
    }
    mfma_xyT_64_add(S0, off ? S1 : S0, acc);
  }
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        int rr, cc;
        acc_pos(a, b, g, &rr, &cc);
        const int ri = r0 + rr, cj = c0 + cc;
        if (ri < nrows && cj < n && cj <= ri) A[(size_t)ri * ld + cj] = av[a][b][g] - acc[a][b][g];
      }
}

// Grid: 1 (critical) + the segments' tiles.
__global__ __launch_bounds__(256) void k_chol_upd(double* __restrict__ A, double* __restrict__ L, int ld, int n,
                                                  double* __restrict__ Vbuf, double* __restrict__ scal, CholUpd u) {
  __shared__ double S0[CB][LDP];
  __shared__ double S1[CB][LDP];
  __shared__ double Zs[CB][18];
  __shared__ CholLds cw;
  if (blockIdx.x == 0) {
    split_critical(A, L, ld, n, u.k, Vbuf, scal, S0, S1, Zs, cw);
    return;
  }
  int b = blockIdx.x - 1, sg = 0;
  while (sg < u.nseg && b >= u.seg[sg].cnt) b -= u.seg[sg++].cnt;
  if (sg >= u.nseg) return;
  const CholUpdSeg g = u.seg[sg];
  int J = g.ja;
  for (; J < g.jb; ++J) {
    const int c = upd_col_tiles(g, J, u.TR);
    if (b < c) break;
    b -= c;
  }
  if (J >= g.jb) return;
  const int I = g.diag ? J : J + (J == g.xd ? 1 : 0) + b;
  upd_tile(A, L, ld, n, I, J, g.pa, g.pb, S0, S1);
}

// The segments of block step k (T block columns, TR tile rows).
static CholUpd chol_upd_plan(int k, int T, int TR) {
  CholUpd u{};
  u.k = k;
  u.TR = TR;
  const int G = k / 4, r = k % 4, D = 4 * G + 4;
  auto add = [&](int ja, int jb, int pa, int pb, int xd, int diag) {
    jb = std::min(jb, T);
    if (ja >= jb) return;
    CholUpdSeg g{ja, jb, pa, pb, xd, diag, 0};
    for (int J = ja; J < jb; ++J) g.cnt += diag ? 1 : TR - J - (J == xd ? 1 : 0);
    if (g.cnt > 0) u.seg[u.nseg++] = g;
  };
  if (r < 3) {
    add(k + 1, 4 * G + 4, k, k + 1, k + 1, 0);                          // (i)
    add(D, D + 1, r == 0 ? std::max(0, 4 * G - 4) : k, k + 1, -1, 1);    // (ii)
    if (G >= 1 && D < T) {                                               // (iv)
      // column-ordered thirds of the tiles of columns [D, T)
      long tot = 0;
      for (int J = D; J < T; ++J) tot += TR - J - (J == D ? 1 : 0);
      int ja = D, jb = D;
      long acc = 0;
      for (int J = D; J < T; ++J) {
        const long before = acc;
        acc += TR - J - (J == D ? 1 : 0);
        if (before * 3 < tot * r) ja = J + 1;
        if (before * 3 < tot * (r + 1)) jb = J + 1;
      }
      add(ja, jb, 4 * G - 4, 4 * G, D, 0);
    }
  } else {
    add(D, D + 4, 4 * G, 4 * G + 4, D, 0);                               // (iii)
  }
  return u;
}

static int chol_grouped() {
  static const int on = [] {
    const char* e = getenv("BA_CHOL_GROUP");
    return e && e[0] == '0' ? 0 : 1;
  }();
  return on;
}

void launch_chol_split_step(double* A, double* L, int ld, int n, int k, int tc, int tr, double* Vbuf, double* scal,
                            hipStream_t s) {
  hipLaunchKernelGGL(k_chol_panel, dim3(tr), dim3(256), 0, s, A, L, ld, n, k, Vbuf);
  if (chol_grouped()) {
    const int T = (n + CB - 1) / CB, TR = (n + 1 + CB - 1) / CB;
    const CholUpd u = chol_upd_plan(k, T, TR);
    int grid = 1;
    for (int g = 0; g < u.nseg; ++g) grid += u.seg[g].cnt;
    hipLaunchKernelGGL(k_chol_upd, dim3(grid), dim3(256), 0, s, A, L, ld, n, Vbuf, scal, u);
    return;
  }
  const int ntiles = tc * (tc + 1) / 2 + (tr > tc ? tc : 0);   // lower tiles (+ a rhs-only tile row)
  hipLaunchKernelGGL(k_chol_step_split, dim3(ntiles), dim3(256), 0, s, A, L, ld, n, k, Vbuf, scal);
}

}  // namespace bahip

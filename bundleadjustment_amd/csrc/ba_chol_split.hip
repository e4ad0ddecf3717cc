// ba_chol_split.hip — the dense Cholesky of large reduced systems (>=
// kCholSplitBlocks block columns, e.g. C4's 6000 rows), in three forms that
// share one host-planned task table (chol_split_plan) and are bitwise equal:
//   flow (default)  k_chol_flow: the whole factorisation as one dataflow
//                   launch, a chain workgroup for the diagonal blocks and the
//                   tile tasks, synchronised by epoch-tagged flags;
//   fused           per block step, k_chol_upd: the critical workgroup and the
//                   step's tile tasks, whose column tasks form the next panel;
//   panels          the same with k_chol_panel launches (BA_CHOL_FUSE=0);
// and the round-5 rank-64 form (k_chol_step_split, BA_CHOL_RANK=0), where
// every trailing tile takes every panel.  DESIGN.md section 15.2.  Its own
// translation unit, so the fused step of ba_chol.hip keeps its code
// generation (a shared template changed the inlining of the critical
// workgroup's factor_invert_blk; here the calls force it inline).
#include "ba_chol.h"

#include <algorithm>
#include <cstdlib>
#include <vector>

namespace bahip {

// The rank-64 form: one block step.  k < 0: factor block 0 only (grid 1x1).
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
// vflag (fused panels, k_chol_upd): V_{k+1} leaves by device-coherent
// stores and vflag[k + 1] = epoch publishes it to the column tasks of the
// same launch.
template <bool FLOW = false>
__device__ __forceinline__ void split_critical(double* __restrict__ A, double* __restrict__ L, int ld, int n, int k,
                                               double* __restrict__ Vbuf, double* __restrict__ scal,
                                               double (*S0)[LDP], double (*S1)[LDP], double (*Zs)[18], CholLds& cw,
                                               unsigned* vflag = nullptr, unsigned epoch = 0) {
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
    // (FLOW: both tiles were written in this launch — device-coherent loads)
    const Rsrc rA = make_rsrc(A, (size_t)nrows * ld * sizeof(double));
    const Rsrc rL = make_rsrc(L, (size_t)nrows * ld * sizeof(double));
    const TileRegs tA = FLOW ? tile_fetch_sc1<true>(rA, lds, s, s, nrows, s + b)
                             : tile_fetch<true>(A, lds, s, s, nrows, s + b);   // A_{k+1,k+1} (+ rhs row)
    const TileRegs tP = FLOW ? tile_fetch_sc1(rL, lds, s, kc, nrows, kc + kb)
                             : tile_fetch(L, lds, s, kc, nrows, kc + kb);      // L_{k+1,k} (k_chol_panel)
    tile_put(S0, tA);
    tile_put(S1, tP);
    __syncthreads();
    mfma_xxT_col0(S1, S0);                 // C = A - P P^T: column 0 now, the rest beside the first sweep
  } else {
    stage64(S0, A, lds, s, s, nrows, s + b);
  }
  if (threadIdx.x == 0) cw.bad = 0;
  CHOL_STAMP(1);
  // (forced inline: with three kernels calling it the inliner kept one out-of-line copy —
  // an s_swappc call that took every caller to 248+ VGPRs, one workgroup per CU)
  [[clang::always_inline]] factor_invert_blk<-1, 18>(S0, S1, Zs, cw, b, m, k >= 0 ? S1 : nullptr);   // rows b..m-1 (rhs) come out as L rows too
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
      if (vflag) st_sc1(make_rsrc(Vbuf, (size_t)(k + 2) * CB * CB * sizeof(double)),
                        ((size_t)(k + 1) * CB * CB + 2 * (size_t)e2) * sizeof(double), make_double2(v[0], v[1]));
      else Vd[e2] = make_double2(v[0], v[1]);
    }
    if (m > b)
      for (int j = threadIdx.x; j < b; j += 256) L[(size_t)(s + b) * ld + s + j] = S0[b][j];
  }
  if (vflag) publish(&vflag[k + 1], epoch);
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

// A_IJ -= sum_{p in [pa, pb)} L_Ip L_Jp^T: operand tiles of panel p + 1 are
// fetched into registers while panel p's MFMAs run; A is read once, written
// once (not at all for an empty range).
// vflag (a column task of the fused form, J = k + 1): the updated tile then
// forms its panel L_IJ = A_IJ V_J^T, as k_chol_panel would in the next step —
// V_J comes from this launch's critical workgroup (vflag[J] = epoch).
// FLOW (k_chol_flow, one launch for the whole factorisation): the tile, its
// operand panels and V are produced by other tasks of the same launch — the
// task first waits on their flags (tile: its previous range's tag; panels:
// the column tasks that formed them), reads and writes them device-coherent,
// and publishes its own tile (and panel) when done.
__device__ __forceinline__ unsigned flow_tag(unsigned epoch, int p) { return epoch * 4096u + (unsigned)p; }
// Diagnostic build only (tools/chol_bench with -DBA_CHOL_FLOW_TRACE): per
// flow task, s_memrealtime (100 MHz) at start, after its waits, at the end,
// and the hardware id (XCC / SE / CU) it ran on; tools/flow_trace.py.
#ifdef BA_CHOL_FLOW_TRACE
__device__ unsigned long long g_ftrace[1 << 16][4];
__shared__ unsigned flow_slot;   // 0: the chain; 1 + ticket: a tile task
#define FLOW_STAMP(i)                                                                               \
  do {                                                                                              \
    if (threadIdx.x == 0 && flow_slot < (1u << 16)) g_ftrace[flow_slot][i] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
__device__ unsigned long long g_fchain[4096][6];   // the chain: each step's inputs ready / V published / phases
#define CHAIN_STAMP(k, i)                                                                           \
  do {                                                                                              \
    if (threadIdx.x == 0 && (k) < 4096) g_fchain[k][i] = __builtin_amdgcn_s_memrealtime();          \
  } while (0)
#define FLOW_SLOT(v) do { if (threadIdx.x == 0) flow_slot = (v); } while (0)
#else
#define FLOW_STAMP(i) do {} while (0)
#define CHAIN_STAMP(k, i) do {} while (0)
#define FLOW_SLOT(v) do {} while (0)
#endif
__device__ __forceinline__ TileRaw tile_fetch_raw_sc1(Rsrc r, size_t ld, int r0, int c0, int rmax, int cmax) {
  TileRaw t;
  t.mask = 0;
  const int tid = ctid();
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int e = tid + 256 * it;
    const int i = e >> 5, j = (e & 31) * 2;
    const int ri = r0 + i, cj = c0 + j;
    const int ric = min(ri, rmax - 1), cjc = min(cj, cmax - 2) & ~1;
    t.v[it] = ld_sc1(r, ((size_t)ric * ld + cjc) * sizeof(double));
    const bool rok = ri < rmax;
    t.mask |= ((rok && cj < cmax) ? 1u : 0u) << (2 * it);
    t.mask |= ((rok && cj + 1 < cmax) ? 2u : 0u) << (2 * it);
  }
  return t;
}
// thread 0 polls every flag the task needs, then one barrier; false (thread
// 0) if a bound was hit
struct FlowFlags { unsigned* tflag; unsigned* pflag; unsigned epoch; unsigned spin_max; int T; };
__device__ __forceinline__ bool flow_poll(const unsigned* f, unsigned want, unsigned spin_max) {
  unsigned it = 0;
  while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != want) {
    if (++it >= spin_max) return false;
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}
__device__ __forceinline__ bool flow_wait(const FlowFlags& ff, int I, int J, int pa, int pb) {
  bool ok = true;
  if (threadIdx.x == 0) {
    if (pa > 0) ok &= flow_poll(&ff.tflag[I * ff.T + J], flow_tag(ff.epoch, pa), ff.spin_max);
    for (int p = max(pa, 1); p < pb; ++p) {   // (panel 0 precedes the launch)
      ok &= flow_poll(&ff.pflag[I * ff.T + p], ff.epoch, ff.spin_max);
      if (I != J) ok &= flow_poll(&ff.pflag[J * ff.T + p], ff.epoch, ff.spin_max);
    }
  }
  __syncthreads();
  return ok;
}

template <bool FLOW = false>
__device__ __forceinline__ bool upd_tile(double* __restrict__ A, double* __restrict__ L, int ld, int n, int I,
                                         int J, int pa, int pb, double (*S0)[LDP], double (*S1)[LDP],
                                         const unsigned* vflag = nullptr, unsigned epoch = 0, unsigned spin_max = 0,
                                         const double* __restrict__ Vbuf = nullptr, const FlowFlags* ff = nullptr) {
  const int nrows = n + 1;
  const size_t lds = (size_t)ld;
  const int r0 = I * CB, c0 = J * CB;
  const bool off = I != J;
  bool ok = true;
  if (FLOW) ok = flow_wait(*ff, I, J, pa, pb);
  if (FLOW) FLOW_STAMP(1);
  const Rsrc rL = make_rsrc(L, (size_t)nrows * ld * sizeof(double));
  TileRaw tI, tJ;
  if (pb > pa) {
    if (FLOW) {
      tI = tile_fetch_raw_sc1(rL, lds, r0, pa * CB, nrows, min(pa * CB + CB, n));
      if (off) tJ = tile_fetch_raw_sc1(rL, lds, c0, pa * CB, n, min(pa * CB + CB, n));
    } else {
      tI = tile_fetch_raw(L, lds, r0, pa * CB, nrows, min(pa * CB + CB, n));
      if (off) tJ = tile_fetch_raw(L, lds, c0, pa * CB, n, min(pa * CB + CB, n));
    }
  }
  double av[2][2][4];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        int rr, cc;
        acc_pos(a, b, g, &rr, &cc);
        const size_t off_a = (size_t)min(r0 + rr, nrows - 1) * ld + min(c0 + cc, n - 1);
        av[a][b][g] = FLOW ? __hip_atomic_load(A + off_a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : A[off_a];
      }
  d4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
  for (int p = pa; p < pb; ++p) {
    if (p > pa) __syncthreads();             // the previous panel's MFMAs are done with the tiles
    tile_put_masked(S0, tI);
    if (off) tile_put_masked(S1, tJ);
    __syncthreads();
    if (p + 1 < pb) {
      const int kc = (p + 1) * CB, ke = min(kc + CB, n);
      if (FLOW) {
        tI = tile_fetch_raw_sc1(rL, lds, r0, kc, nrows, ke);
        if (off) tJ = tile_fetch_raw_sc1(rL, lds, c0, kc, n, ke);
      } else {
        tI = tile_fetch_raw(L, lds, r0, kc, nrows, ke);
        if (off) tJ = tile_fetch_raw(L, lds, c0, kc, n, ke);
      }
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
        if (pb > pa && ri < nrows && cj < n && cj <= ri) {
          if (FLOW) __hip_atomic_store(A + (size_t)ri * ld + cj, av[a][b][g] - acc[a][b][g], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
          else A[(size_t)ri * ld + cj] = av[a][b][g] - acc[a][b][g];
        }
      }
  if (FLOW && pb > pa) publish(&ff->tflag[I * ff->T + J], flow_tag(ff->epoch, pb));
  if (!vflag) return ok;
  // ---- the panel: S0 = the updated tile (bitwise what k_chol_panel reloads)
  if (pb > pa) __syncthreads();               // the last MFMAs are done with S0 / S1
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        int rr, cc;
        acc_pos(a, b, g, &rr, &cc);
        const int ri = r0 + rr, cj = c0 + cc;
        S0[rr][cc] = (ri < nrows && cj < n) ? av[a][b][g] - acc[a][b][g] : 0.0;
      }
  ok &= wait_flag(&vflag[J], epoch, spin_max);
  tile_put(S1, tile_fetch_sc1<true>(make_rsrc(Vbuf, (size_t)(J + 1) * CB * CB * sizeof(double)), CB, J * CB, 0,
                                    (J + 1) * CB, CB));
  __syncthreads();
  d4 pacc[4];
  mfma_xVT_strip(S0, S1, pacc);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, m = min(CB, nrows - r0), kb = min(CB, n - c0);
#pragma unroll
  for (int bc = 0; bc < 4; ++bc)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int rr = 16 * w + (lane >> 4) + 4 * g, cc = 16 * bc + (lane & 15);
      if (rr < m && cc < kb) {
        if (FLOW) __hip_atomic_store(L + (size_t)(r0 + rr) * ld + c0 + cc, pacc[bc][g], __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
        else L[(size_t)(r0 + rr) * ld + c0 + cc] = pacc[bc][g];
      }
    }
  if (FLOW) publish(&ff->pflag[I * ff->T + J], ff->epoch);
  return ok;
}

// ---- scheduled form (default): a host-planned task table replaces the
// per-step "every trailing tile takes panel k" update.  A task is one tile
// and a contiguous range of panels, A_IJ -= sum_{p in [pa, pb)} L_Ip L_Jp^T,
// so a tile is read and written once per range instead of once per panel
// (ranges of up to `rank` panels: 4 -> a quarter of the rank-64 form's tile
// read-modify-write traffic; the operand tiles come from L through the
// L2 / Infinity Cache).  The chain keeps its one-step look-ahead: block step
// k forms panel k (k_chol_panel) and then launches k_chol_upd with the
// critical workgroup (diagonal block k + 1, panel k) and the step's tasks.
// Plan (chol_split_plan, host, once per order):
//  - a tile (I, J) takes the panels p < J (a diagonal tile: p < J - 1, the
//    critical workgroup applies panel J - 1), in order, each exactly once;
//  - due: an off-diagonal tile of column J by the launch of step J - 1 (panel
//    J is formed next), a diagonal tile by step J - 2; a due tile takes all
//    its remaining available panels in one task;
//  - the rest is spread evenly over the steps: each launch takes the least
//    work (in panels) that still meets every later due step if the steps
//    after it work at that same rate, filled earliest-due first with tasks
//    of `rank` panels (or a tile's last, shorter range) — right-looking's
//    front-loaded trailing work becomes a steady background the chain's
//    serial steps hide.
// At most one task per tile per launch; bitwise deterministic for a given
// order (not bitwise the rank-64 form: the sums are grouped differently —
// parity is against the oracle, as before).
struct CholSplitPlan {
  std::vector<int4> tasks;   // {I, J, pa, pb}, step-major
  std::vector<int> off;      // step k's tasks: [off[k], off[k + 1])
};
static void chol_split_plan(int T, int TR, int rank, double budget, CholSplitPlan& P) {
  P.tasks.clear();
  P.off.assign(std::max(T, 1), 0);
  if (T < 2) return;
  struct Tile { int I, J, a, need, due; };
  std::vector<Tile> tl;
  for (int J = 1; J < T; ++J)
    for (int I = J; I < TR; ++I) {
      const int need = I == J ? J - 1 : J;
      if (need > 0) tl.push_back({I, J, 0, need, I == J ? J - 2 : J - 1});
    }
  // earliest due first; within a due step, column then row order
  std::sort(tl.begin(), tl.end(), [](const Tile& x, const Tile& y) {
    return x.due != y.due ? x.due < y.due : (x.J != y.J ? x.J < y.J : x.I < y.I);
  });
  std::vector<long> due_work(T, 0);
  for (const Tile& t : tl) due_work[t.due] += t.need;
  for (int k = 0; k + 1 < T; ++k) {
    P.off[k] = (int)P.tasks.size();
    long spent = 0;
    // due tasks first (the longest first), then the background
    const size_t first = P.tasks.size();
    for (Tile& t : tl) {
      // (every off-diagonal tile of column k + 1 gets a column task — the
      // fused form's panel — even with nothing left to apply)
      const bool col = t.I != t.J;
      if (t.due != k || (t.a >= t.need && !col)) continue;
      P.tasks.push_back(make_int4(t.I | (col ? 1 << 20 : 0), t.J, t.a, t.need));
      spent += t.need - t.a;
      due_work[t.due] -= t.need - t.a;
      t.a = t.need;
    }
    // column tasks first (the next step waits on their panels), longest first
    std::stable_sort(P.tasks.begin() + first, P.tasks.end(), [](const int4& x, const int4& y) {
      const int px = (x.x >> 20) & 1, py = (y.x >> 20) & 1;
      return px != py ? px > py : x.w - x.z > y.w - y.z;
    });
    // the least constant rate that meets every later due step, given that a
    // tile advances by at most `rank` panels per launch: by step s a tile
    // must have done all but rank x (due - s) of its remaining panels
    double rate = 0;
    for (int s = k + 1; s + 1 < T; ++s) {
      long req = 0;
      for (const Tile& t : tl)
        if (t.due > k && t.a < t.need) req += std::max(0L, (long)(t.need - t.a) - (long)rank * std::max(0, t.due - s));
      rate = std::max(rate, (double)req / (double)(s - k + 1));
    }
    const double target = budget * rate;   // this launch's share (the due work above is in it too)
    // least laxity first: a tile whose remaining ranges need every step left
    // before its due step goes now whatever the share (a tile advances by at
    // most `rank` panels per launch), then the share fills earliest-due first
    struct Cand { int slack, idx; };
    std::vector<Cand> cand;
    for (int i = 0; i < (int)tl.size(); ++i) {
      const Tile& t = tl[i];
      if (t.due <= k || t.a >= t.need) continue;
      const int avail = std::min(t.need, k + 1) - t.a;   // panels <= k exist
      const int take = std::min(avail, rank);
      if (take <= 0 || (take < rank && t.a + take < t.need)) continue;   // a full range, or the tile's last
      const int left = t.due - k, needed = (t.need - t.a + rank - 1) / rank;   // (the due step takes the rest)
      cand.push_back({left - needed, i});
    }
    std::stable_sort(cand.begin(), cand.end(), [](const Cand& x, const Cand& y) { return x.slack < y.slack; });
    for (const Cand& c : cand) {
      if (c.slack > 0 && spent >= target) continue;   // (earliest-due order within a slack: tl's order)
      Tile& t = tl[c.idx];
      const int take = std::min(std::min(t.need, k + 1) - t.a, rank);
      P.tasks.push_back(make_int4(t.I, t.J, t.a, t.a + take));
      spent += take;
      due_work[t.due] -= take;
      t.a += take;
    }
  }
  P.off[T - 1] = (int)P.tasks.size();
}

// Grid: 1 (critical) + the step's tasks {I | panel << 20, J, pa, pb}.
// vflag (the fused form): the critical workgroup publishes V_{k+1}, and the
// column tasks (panel bit) of column k + 1 form their panels after their
// updates; without it the panel bit is ignored (k_chol_panel forms them in
// the next step).
__global__ __launch_bounds__(256) void k_chol_upd(double* __restrict__ A, double* __restrict__ L, int ld, int n, int k,
                                                  double* __restrict__ Vbuf, double* __restrict__ scal,
                                                  const int4* __restrict__ tasks, unsigned* vflag, unsigned epoch,
                                                  unsigned spin_max) {
  __shared__ double S0[CB][LDP];
  __shared__ double S1[CB][LDP];
  __shared__ double Zs[CB][18];
  __shared__ CholLds cw;
  if (blockIdx.x == 0) {
    if (k >= -1) split_critical(A, L, ld, n, k, Vbuf, scal, S0, S1, Zs, cw, vflag, epoch);   // (k = -2: tasks only, tools/chol_bench)
    return;
  }
  const int4 t = tasks[blockIdx.x - 1];
  const bool pan = vflag && ((t.x >> 20) & 1);
  const bool ok = upd_tile(A, L, ld, n, t.x & 0xfffff, t.y, t.z, t.w, S0, S1, pan ? vflag : nullptr, epoch, spin_max,
                           Vbuf);
  if (threadIdx.x == 0 && !ok) atomicAdd(&scal[SL_CHOL_SPIN], 1.0);   // (V never came: the caller redoes the step unfused)
}

// The flow form's chain: ONE workgroup (the list's first entry) factors every
// diagonal block in turn, k = 0 .. T - 2 (d = k + 1).  It keeps V_k (cleaned,
// as stored) in registers from its own previous step and forms the panel row
// it needs itself, P = L_{d,k} = A_{d,k} V_k^T (bitwise what the column task
// of tile (d, k) stores: the same tile values, V and MFMA strip), so a step
// waits only on the two tiles' tags — tile (d, k) and the diagonal tile
// holding panels < k — instead of on another task's panel after V_k (the
// critical-task chain handed V_k out, waited for the column task to form and
// publish L_{d,k}, and reloaded it: ~8 us per step).  Then C = A_dd - P P^T,
// factor_invert_blk, V_d out (device-coherent) and vflag[d].
__device__ __forceinline__ bool flow_chain(double* __restrict__ A, double* __restrict__ L, int ld, int n,
                                           double* __restrict__ Vbuf, double* __restrict__ scal,
                                           double (*S0)[LDP], double (*S1)[LDP], double (*Zs)[18], CholLds& cw,
                                           unsigned* vflag, const unsigned* tflag, unsigned epoch, unsigned spin_max,
                                           int T) {
  const int nrows = n + 1;
  const size_t lds = (size_t)ld;
  const Rsrc rA = make_rsrc(A, (size_t)nrows * ld * sizeof(double));
  const Rsrc rV = make_rsrc(Vbuf, (size_t)(T + 1) * CB * CB * sizeof(double));
  bool ok = true;
  TileRegs tV = tile_fetch<true>(Vbuf, CB, 0, 0, CB, CB);   // V_0 (the launch before)
  for (int k = 0; k + 1 < T; ++k) {
    const int d = k + 1, s = d * CB, kc = k * CB;
    const int kb = min(CB, n - kc), b = min(CB, n - s), m = min(CB, nrows - s);
    if (threadIdx.x == 0 && k > 0) {
      ok &= flow_poll(&tflag[d * T + k], flow_tag(epoch, k), spin_max);   // A_{d,k}: panels < k
      ok &= flow_poll(&tflag[d * T + d], flow_tag(epoch, k), spin_max);   // A_dd: panels < k
    }
    __syncthreads();                                                       // (and the previous step's LDS reads are done)
    CHAIN_STAMP(k, 0);
    const TileRegs tAk = tile_fetch_sc1(rA, lds, s, kc, nrows, kc + kb);
    const TileRegs tA = tile_fetch_sc1<true>(rA, lds, s, s, nrows, s + b);
    tile_put(S1, tV);
    tile_put(S0, tAk);
    __syncthreads();
    CHAIN_STAMP(k, 2);
    d4 pacc[4];
    mfma_xVT_strip(S0, S1, pacc);
    __syncthreads();
    {
      const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
      for (int bc = 0; bc < 4; ++bc)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int rr = 16 * w + (lane >> 4) + 4 * g, cc = 16 * bc + (lane & 15);
          S1[rr][cc] = (rr < m && cc < kb) ? pacc[bc][g] : 0.0;   // (as the stored panel, reloaded)
        }
    }
    tile_put(S0, tA);
    __syncthreads();
    CHAIN_STAMP(k, 3);
    mfma_xxT_col0(S1, S0);
    if (threadIdx.x == 0) cw.bad = 0;
    [[clang::always_inline]] factor_invert_blk<-1, 18>(S0, S1, Zs, cw, b, m, S1);
    __syncthreads();
    CHAIN_STAMP(k, 4);
    for (int it = 0; it < 8; ++it) {
      const int e2 = threadIdx.x + 256 * it;
      const int i = (2 * e2) / CB, j = (2 * e2) % CB;
      double v[2];
#pragma unroll
      for (int h = 0; h < 2; ++h)
        v[h] = (j + h <= i && i < b && j + h < b) ? S1[i][j + h] : (i == j + h ? 1.0 : 0.0);
      tV.v[it] = make_double2(v[0], v[1]);
      st_sc1(rV, ((size_t)d * CB * CB + 2 * (size_t)e2) * sizeof(double), tV.v[it]);
    }
    if (m > b)
      for (int j = threadIdx.x; j < b; j += 256) L[(size_t)(s + b) * ld + s + j] = S0[b][j];
    publish(&vflag[d], epoch);
    CHAIN_STAMP(k, 1);
    if (threadIdx.x == 0 && cw.bad) scal[SL_CHOL_BAD] += 1.0;
  }
  return ok;
}

// ---- flow form (default): the whole factorisation in ONE launch.  The task
// list is the scheduled form's, step by step, each step led by its critical
// workgroup (bit 21, y = k); every task waits on the flags of what it reads
// (FLOW above; the critical: its diagonal tile's tag and its panel row) and
// publishes what it writes.  A task waits only on tasks before it in the
// list, which the in-order dispatch has placed on the device before it, so
// the grid needs no co-residency (as k_back_flow).  The steps overlap: a
// step's background tasks run beside the next steps' chain, and no launch
// boundary drains the device between steps.  Same arithmetic per task as
// the per-step launches: bitwise the same factor.
// Block 0 is the chain workgroup (flow_chain); block 1 + i runs task i.
// (Measured and not kept: giving the chain a CU of its own — a workgroup the
// dispatcher placed beside it waited there, the others drew tasks from an
// atomic ticket counter: the chain's factor went from 14 to 11.5 us, but its
// inputs came later (13.9 vs 6.7 us median wait) and n = 6000 took 2.9 vs
// 2.6 ms; profiles/r06_v9_chol_flow_ab.txt.)
__global__ __launch_bounds__(256, 2) void k_chol_flow(double* __restrict__ A, double* __restrict__ L, int ld, int n,
                                                      double* __restrict__ Vbuf, double* __restrict__ scal,
                                                      const int4* __restrict__ tasks, unsigned* vflag, unsigned* tflag,
                                                      unsigned* pflag, unsigned epoch, unsigned spin_max, int T) {
  __shared__ double S0[CB][LDP];
  __shared__ double S1[CB][LDP];
  __shared__ double Zs[CB][18];
  __shared__ CholLds cw;
  FLOW_SLOT(blockIdx.x);
  FLOW_STAMP(0);
  bool ok;
  if (blockIdx.x == 0) {
    FLOW_STAMP(1);
    ok = flow_chain(A, L, ld, n, Vbuf, scal, S0, S1, Zs, cw, vflag, tflag, epoch, spin_max, T);
  } else {
    const int4 t = tasks[blockIdx.x - 1];
    const FlowFlags ff{tflag, pflag, epoch, spin_max, T};
    ok = upd_tile<true>(A, L, ld, n, t.x & 0xfffff, t.y, t.z, t.w, S0, S1, ((t.x >> 20) & 1) ? vflag : nullptr, epoch,
                        spin_max, Vbuf, &ff);
  }
  FLOW_STAMP(2);
  if (threadIdx.x == 0 && !ok) atomicAdd(&scal[SL_CHOL_SPIN], 1.0);   // (the caller redoes the step per step)
}

// (the switches are read when a system is set up: ensure_dense, tools/chol_bench)
int chol_split_rank() {
  const char* e = getenv("BA_CHOL_RANK");
  const int v = e ? atoi(e) : 4;
  return v < 0 ? 4 : v;   // 0: the rank-64 form (k_chol_step_split)
}
static double chol_split_budget() {
  const char* e = getenv("BA_CHOL_BUDGET");
  const double v = e ? atof(e) : 1.0;
  return v > 0 ? v : 1.0;
}

// The task table of an order-n system (device copy + host step offsets).
void chol_split_tasks(int n, std::vector<int4>& tasks, std::vector<int>& off) {
  const int T = (n + CB - 1) / CB, TR = (n + 1 + CB - 1) / CB;
  CholSplitPlan P;
  chol_split_plan(T, TR, std::max(1, chol_split_rank()), chol_split_budget(), P);
  tasks.swap(P.tasks);
  off.swap(P.off);
}
// ... as the flow form's one list: the chain workgroup first (flow_chain),
// then the tile tasks.  A tile task waits only on tasks before it (its tile's
// previous range, the column tasks that formed its panels) and on V from the
// chain; the chain waits, at step k, on the tasks that finish tiles (k+1, k)
// and (k+1, k+1) — which come before every task waiting on V_{k+1} or later
// (their due steps precede), so the in-order dispatch never fills the device
// with tasks the chain's next V would release while one it needs is still
// queued.  Within that, the order is a priority: a step's background tasks
// (tiles due more than lag + 1 steps later) move behind the next `lag` steps'
// chain-bound tasks (BA_CHOL_FLOW_LAG, default 1; 0: step order).
void chol_flow_tasks(const std::vector<int4>& tasks, const std::vector<int>& off, std::vector<int4>& flow) {
  const int T = (int)off.size();
  const char* e = getenv("BA_CHOL_FLOW_LAG");
  const int lag = e ? std::max(0, atoi(e)) : 1;
  // the tasks on the tiles next to the diagonal (I - J <= 2: the chain's own
  // inputs and the panel rows they are formed from) go `lead` steps ahead
  // (BA_CHOL_FLOW_LEAD; the chain still waited ~6 us per step for them: the
  // latency is the hand-offs themselves, not the dispatch order)
  const char* e2 = getenv("BA_CHOL_FLOW_LEAD");
  const int lead = e2 ? std::max(0, atoi(e2)) : 0;   // (2, 4, 8 measured slower: 2.66, 2.67, 2.73 vs 2.60 ms)
  int TR = T;
  for (const int4& t : tasks) TR = std::max(TR, (t.x & 0xfffff) + 1);
  struct E { int4 t; double level; };
  std::vector<E> es;
  std::vector<int> last((size_t)TR * T, -1), colt((size_t)TR * T, -1);
  const double eps = 1e-6;
  for (int k = 0; k + 1 < T; ++k) {
    for (int i = off[k]; i < off[k + 1]; ++i) {
      const int4 t = tasks[i];
      const int I = t.x & 0xfffff, J = t.y;
      const bool col = (t.x >> 20) & 1;
      const int due = I == J ? J - 2 : J - 1;
      const bool chain = col || due <= k + lag + 1;
      double lv = I - J <= 2 ? k - lead + 0.125 : (chain ? k + 0.25 : k + lag + 0.5);
      const int prev = last[(size_t)I * T + J];
      if (t.z > 0 && prev >= 0) lv = std::max(lv, es[prev].level + eps);
      for (int p = std::max(t.z, 1); p < t.w; ++p) {
        if (colt[(size_t)I * T + p] >= 0) lv = std::max(lv, es[colt[(size_t)I * T + p]].level + eps);
        if (colt[(size_t)J * T + p] >= 0) lv = std::max(lv, es[colt[(size_t)J * T + p]].level + eps);
      }
      const int idx = (int)es.size();
      es.push_back({t, lv});
      if (t.w > t.z) last[(size_t)I * T + J] = idx;
      if (col) colt[(size_t)I * T + J] = idx;
    }
  }
  std::stable_sort(es.begin(), es.end(), [](const E& a, const E& b) { return a.level < b.level; });
  flow.clear();
  for (const E& x : es) flow.push_back(x.t);   // (the chain workgroup, flow_chain, is block 0 beside them)
}
int chol_split_flow() {
  const char* e = getenv("BA_CHOL_FLOW");
  return e && e[0] == '0' ? 0 : 1;
}
void launch_chol_flow(double* A, double* L, int ld, int n, double* Vbuf, double* scal, const int4* ftask, int nftask,
                      unsigned* vflag, unsigned* tflag, unsigned* pflag, unsigned epoch, hipStream_t s) {
  const int T = (n + CB - 1) / CB, tr = (n + 1 - CB + CB - 1) / CB;
  const char* e = getenv("BA_CHOL_SPIN_MAX");
  const unsigned spin = e && atoi(e) > 0 ? (unsigned)atoi(e) : (1u << 17);
  hipLaunchKernelGGL(k_chol_panel, dim3(tr), dim3(256), 0, s, A, L, ld, n, 0, Vbuf);   // panel 0
  hipLaunchKernelGGL(k_chol_flow, dim3(1 + nftask), dim3(256), 0, s, A, L, ld, n, Vbuf, scal, ftask, vflag, tflag,
                     pflag, epoch, spin, T);
}

int chol_split_fused() {
  const char* e = getenv("BA_CHOL_FUSE");
  return e && e[0] == '0' ? 0 : 1;
}

// Block step k of the split form.  tasks == null: the rank-64 form.  vflag
// (the fused form): panel k was formed by step k - 1's column tasks (k = 0:
// k_chol_panel here), else k_chol_panel forms it now.
void launch_chol_split_step(double* A, double* L, int ld, int n, int k, int tc, int tr, double* Vbuf, double* scal,
                            const int4* tasks, const int* off, unsigned* vflag, unsigned epoch, hipStream_t s) {
  if (!vflag || !tasks || k == 0) hipLaunchKernelGGL(k_chol_panel, dim3(tr), dim3(256), 0, s, A, L, ld, n, k, Vbuf);
  if (tasks) {
    const char* e = getenv("BA_CHOL_SPIN_MAX");   // (diagnostics: a small bound exercises the fallback)
    const unsigned spin = e && atoi(e) > 0 ? (unsigned)atoi(e) : (1u << 17);
    hipLaunchKernelGGL(k_chol_upd, dim3(1 + off[k + 1] - off[k]), dim3(256), 0, s, A, L, ld, n, k, Vbuf, scal,
                       tasks + off[k], vflag, epoch, spin);
    return;
  }
  const int ntiles = tc * (tc + 1) / 2 + (tr > tc ? tc : 0);   // lower tiles (+ a rhs-only tile row)
  hipLaunchKernelGGL(k_chol_step_split, dim3(ntiles), dim3(256), 0, s, A, L, ld, n, k, Vbuf, scal);
}

}  // namespace bahip

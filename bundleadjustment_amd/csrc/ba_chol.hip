// ba_chol.hip — dense Cholesky of the reduced camera system (DENSE_SCHUR):
// the fused block step (critical workgroup + trailing tiles, one launch per
// 64-column block) and the dataflow back substitution; helpers in
// ba_chol.h, the split form for large systems in ba_chol_split.hip.
#include "ba_chol.h"

namespace bahip {

// One block step.  k < 0: factor block 0 only (grid 1x1).
//   A    working matrix ((n+1) x ld), trailing part updated in place
//   L    output factor ((n+1) x ld)
//   Vbuf [T][64][64] inverses of the diagonal blocks
//   U    update accumulator ((n+1) x ld): a trailing tile's updates are summed
//        from zero, U = ((0 - u_0) - u_1) - ..., and its last update writes
//        A + U into A (the persistent form's order, ba_chol_persist.hip)
__global__ __launch_bounds__(256) void k_chol_step(double* __restrict__ A, double* __restrict__ L, int ld, int n,
                                                   int k, double* __restrict__ Vbuf, double* __restrict__ scal,
                                                   double* __restrict__ U) {
  // XCD-aware tile order: workgroup b runs on XCD b % 8 (round-robin
  // dispatch).  The tiles (1,0) and (1,1) produce A_{k+2,k+1} and
  // A_{k+2,k+2}, the next launch's critical inputs; they take linear ids 8
  // and 16 so they run on the critical workgroup's XCD (id 0) and the next
  // critical workgroup stages them from that XCD's L2.
  int I = blockIdx.y, J = blockIdx.x;
  {
    const int gx = gridDim.x, G = gx * gridDim.y;
    if (k >= 0 && G > 16) {
      const int a = gx, bb = gx + 1;                    // natural ids of (1,0), (1,1)
      const int x = bb == 8 ? a : (bb == a ? 8 : bb);   // swap(8, a) applied to bb
      int lin = blockIdx.y * gx + blockIdx.x;
      lin = lin == 16 ? x : (lin == x ? 16 : lin);      // swap(16, x)
      lin = lin == 8 ? a : (lin == a ? 8 : lin);        // swap(8, a)
      I = lin / gx;
      J = lin - I * gx;
    }
  }
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
    if (k >= 0) {
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
      mfma_xxT_col0(S1, S0);                 // C = A - P P^T: column 0 now, the rest beside the first sweep
      CHOL_STAMP(23);
    } else {
      stage64(S0, A, lds, s, s, nrows, s + b);
    }
    if (threadIdx.x == 0) cw.bad = 0;
    CHOL_STAMP(1);
    factor_invert_blk(S0, S2, S1, cw, b, m, k >= 0 ? S1 : nullptr);   // rows b..m-1 (rhs) come out as L rows too
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
  // this tile's last update (absolute column k + 1 + J): step k + J off the
  // diagonal, k + J - 1 on it (its update k + J is the next critical
  // workgroup's C = A - P P^T) — i.e. relative column 0, resp. tile (1, 1)
  const bool last = I == J ? J == 1 : J == 0;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        int rr, cc;
        acc_pos(a, b, g, &rr, &cc);
        const int ri = r0 + rr, cj = c0 + cc;
        if (ri < nrows && cj < n && cj <= ri) {
          const size_t o = (size_t)ri * ld + cj;
          const double u = (k == 0 ? 0.0 : U[o]) - acc[a][b][g];
          if (last) A[o] = A[o] + u;
          else U[o] = u;
        }
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
// Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility: the
// data-tagged granule form, its hand-off table's handoff-1to1 row): every
// element of y_K travels as one 16-B granule {value, epoch} written by ONE
// write-through store (global_store_dwordx4 sc1); each consumer lane polls
// its element's granule with 16-B sc1 loads until the tag matches, so the
// value arrives with its flag (one fabric round trip per hop, no separate
// flag, no L2 write-back or L1 invalidate).  The epoch (launch counter,
// never 0) tags the latest publish, so nothing is reset between launches;
// spins are bounded (a missing producer sets the failure slot instead of
// hanging the GPU).  The plain y (read by later kernels) is stored too.
// ---------------------------------------------------------------------------
constexpr long kSpinMax = 1L << 24;
typedef int gi4 __attribute__((ext_vector_type(4)));

//
// The trailing s_nop 1 is part of the protocol.  hipcc treats an asm
// statement as opaque and pads none of its hazards: without the nop the
// compiler's next VALU may overwrite the store's data registers before the
// 16-B store has read them (the VMEM-store-data hazard of stores wider than
// 8 B; cdna_hip_programming.md §5.7 item 1).  Round 2's "V_K in registers"
// variant hit exactly this: its register allocation put the y address into
// the {epoch, 0} half of the granule's registers on the very next
// instruction (v_lshl_add_u64 v[2:3] right after global_store_dwordx4 ...
// v[0:3]), the granule went out with a wrong tag, and the consumers spun to
// kSpinMax.  The shipping allocation happened to reuse no data register.
__device__ inline void gran_store(double* g, double v, int epoch) {
  const long long b = __double_as_longlong(v);
  const gi4 d = {(int)b, (int)(b >> 32), epoch, 0};
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(g), "v"(d) : "memory");
}
// waits for the granule of `epoch`; false if the spin bound was hit.  The
// load and its wait are one statement with an early-clobber output, so the
// compiler never sees the destination before the data has landed.
__device__ inline bool gran_wait(const double* g, int epoch, double& v) {
  gi4 d;
  long it = 0;
  while (true) {
    asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=&v"(d) : "v"(g) : "memory");
    if (d.z == epoch || it >= kSpinMax) break;
    __builtin_amdgcn_s_sleep(1);
    ++it;
  }
  v = __longlong_as_double(((long long)d.y << 32) | (unsigned)d.x);
  return d.z == epoch;
}

__global__ __launch_bounds__(256) void k_back_flow(const double* __restrict__ A, const double* __restrict__ Lm,
                                                   int ld, int n, const double* __restrict__ Vall,
                                                   double* __restrict__ y, double* __restrict__ yg, int epoch,
                                                   double* __restrict__ scal) {
  __shared__ double zs[CB];
  __shared__ double ys[CB];
  __shared__ double part[4][CB];
  __shared__ int bad;
  // producers first: workgroup K waits on every J > K, and low block ids are
  // dispatched first, so block b takes K = T - 1 - b (if the grid cannot be
  // resident at once, the waiting consumers are then the ones still queued)
  const int T = (n + CB - 1) / CB;
  const int K = T - 1 - (int)blockIdx.x, tid = threadIdx.x;
  const int s0 = K * CB, bsz = min(CB, n - s0);
  const size_t lds = (size_t)ld;
  // thread (j = tid & 63, h = tid >> 6) sums rows i = h, h + 4, ... of a tile
  const int j = tid & 63, h = tid >> 6;
  if (tid == 0) bad = 0;
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
      t += (i <= j ? V[(size_t)j * CB + i] : 0.0) * ys[i];   // (V lower triangular; the persistent form leaves its upper blocks unwritten)
    }
    part[h][j] = t;
    __syncthreads();
    if (tid < CB) zs[tid] = (part[0][tid] + part[1][tid]) + (part[2][tid] + part[3][tid]);
    __syncthreads();
  } else if (tid < CB) {
    zs[tid] = tid < bsz ? Lm[(size_t)n * lds + s0 + tid] : 0.0;
  }
  // V_K (the column block this thread needs for y_K) is loaded before the
  // hand-off loop, so the final product after the last hand-off reads only
  // registers and LDS
  double vk[16];
  {
    const double* V = Vall + (size_t)K * CB * CB;
#pragma unroll
    for (int q = 0; q < 16; ++q) vk[q] = h + 4 * q >= j ? V[(size_t)(h + 4 * q) * CB + j] : 0.0;   // (lower triangle only)
  }
  double acc = 0.0;
  for (int J = T - 1; J > K; --J) {
    const int sJ = J * CB, bJ = min(CB, n - sJ);
    double lv[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {   // L[sJ + i][s0 + j], i = h + 4 q (prefetched before the poll)
      const int i = h + 4 * q;
      lv[q] = (i < bJ && j < bsz) ? Lm[(size_t)(sJ + i) * lds + s0 + j] : 0.0;
    }
    if (tid < CB) {
      double v = 0.0;
      if (tid < bJ && !gran_wait(yg + 2 * (size_t)(sJ + tid), epoch, v)) bad = 1;
      ys[tid] = v;
    }
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
    double t = 0.0;
#pragma unroll
    for (int q = 0; q < 16; ++q) t += vk[q] * zs[h + 4 * q];
    part[h][j] = t;
  }
  __syncthreads();
  if (tid < CB && tid < bsz) {
    const double val = (part[0][tid] + part[1][tid]) + (part[2][tid] + part[3][tid]);
    gran_store(yg + 2 * (size_t)(s0 + tid), val, epoch);
    y[s0 + tid] = val;
  }
  if (tid == 0 && bad) scal[SL_CHOL_SPIN] += 1.0;   // (a granule that never came: not a pivot failure)
}

// Workgroups of k_back_flow the device holds at once (occupancy API x CUs).
// The dataflow needs no co-residency for progress (workgroup K waits only
// on J > K, i.e. on lower block ids, which are dispatched first), but a grid
// that fits keeps every hop a pure hand-off; ensure_dense refuses a system
// whose T block columns exceed this (ba_solver.hip).
int back_flow_capacity(int device) {
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(k_back_flow), 256, 0) !=
          hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
    return -1;
  return per_cu * cus;
}

// split-form block step (ba_chol_split.hip)
void launch_chol_split_step(double* A, double* L, int ld, int n, int k, int tc, int tr, double* Vbuf, double* scal,
                            const int4* tasks, const int* off, unsigned* vflag, unsigned epoch, hipStream_t s);

// Block columns from which the split (panel + update) form is used: below it
// the fused step's trailing tiles hide behind the critical workgroup and one
// launch per step is cheaper (C3: 19 block columns); above it the trailing
// GEMMs dominate (C4: 94).
constexpr int kCholSplitBlocks = 24;
int chol_split_blocks() { return kCholSplitBlocks; }

void launch_chol_flow(double* A, double* L, int ld, int n, double* Vbuf, double* scal, const int4* ftask, int nftask,
                      unsigned* vflag, unsigned* tflag, unsigned* pflag, unsigned epoch, hipStream_t s);

// the persistent form (ba_chol_persist.hip)
void launch_chol_persist(double* A, double* L, int ld, int n, double* Vbuf, double* scal, unsigned* flags,
                         unsigned epoch, hipStream_t s);

void launch_chol_persist_ov(const DevProblem& P, const DevWork& W, OvPlan& plan, double radius, int epoch,
                            hipStream_t s, bool pass_only);
void launch_cholesky_solve_ov(const DevProblem& P, const DevWork& W, OvPlan& plan, double radius, int epoch,
                              hipStream_t s, bool pass_only) {
  const int n = P.n, T = (n + CB - 1) / CB;
  launch_chol_persist_ov(P, W, plan, radius, epoch, s, pass_only);
  if (pass_only) return;
  hipLaunchKernelGGL(k_back_flow, dim3(T), dim3(256), 0, s, W.S, W.Lf, P.ld, n, W.Vbuf, W.y, W.yg, epoch, W.scal);
}

void launch_cholesky_solve2(const DevProblem& P, const DevWork& W, int epoch, hipStream_t s) {
  const int n = P.n;
  if (n == 0) return;
  const int nrows = n + 1;
  const int T = (n + CB - 1) / CB;
  const bool split = T >= kCholSplitBlocks;
  if (W.chol_persist && !split) {
    launch_chol_persist(W.S, W.Lf, P.ld, n, W.Vbuf, W.scal, W.cflags, (unsigned)epoch, s);
    hipLaunchKernelGGL(k_back_flow, dim3(T), dim3(256), 0, s, W.S, W.Lf, P.ld, n, W.Vbuf, W.y, W.yg, epoch, W.scal);
    return;
  }
  hipLaunchKernelGGL(k_chol_step, dim3(1, 1), dim3(256), 0, s, W.S, W.Lf, P.ld, n, -1, W.Vbuf, W.scal, W.Ubuf);
  if (split && W.chol_flow) {
    const size_t TR = (size_t)(nrows + CB - 1) / CB;
    launch_chol_flow(W.S, W.Lf, P.ld, n, W.Vbuf, W.scal, W.ftask, W.nftask, W.cflags, W.tflag, W.tflag + TR * T,
                     (unsigned)epoch, s);
    hipLaunchKernelGGL(k_back_flow, dim3(T), dim3(256), 0, s, W.S, W.Lf, P.ld, n, W.Vbuf, W.y, W.yg, epoch, W.scal);
    return;
  }
  for (int k = 0; k + 1 < T; ++k) {
    const int st = (k + 1) * CB;
    const int tr = (nrows - st + CB - 1) / CB, tc = (n - st + CB - 1) / CB;
    if (split) {
      launch_chol_split_step(W.S, W.Lf, P.ld, n, k, tc, tr, W.Vbuf, W.scal, W.ctask, W.ctask_off,
                             W.chol_fuse ? W.cflags : nullptr, (unsigned)epoch, s);
    } else {
      hipLaunchKernelGGL(k_chol_step, dim3(tc, tr), dim3(256), 0, s, W.S, W.Lf, P.ld, n, k, W.Vbuf, W.scal, W.Ubuf);
    }
  }
  hipLaunchKernelGGL(k_back_flow, dim3(T), dim3(256), 0, s, W.S, W.Lf, P.ld, n, W.Vbuf, W.y, W.yg, epoch, W.scal);
}


}  // namespace bahip

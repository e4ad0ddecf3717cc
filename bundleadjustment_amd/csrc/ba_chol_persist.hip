// ba_chol_persist.hip — the dense Cholesky of the reduced camera system
// (DENSE_SCHUR, Optimizer.cpp:85) as ONE persistent launch with look-ahead,
// for systems whose lower tiles fit the chip (C3: 19 block columns, 171
// workgroups).  Same arithmetic as the per-step launches of ba_chol.hip
// (k_chol_step), in the same order per tile, so L and the block inverses V
// come out bitwise identical; only the orchestration differs:
//
//   workgroup 0 (critical)  for c = 0 .. T-1: stage A_{c,c-1} and the
//       diagonal tile A_{c,c} once their workers have published them,
//       P = A_{c,c-1} V_{c-1}^T (V_{c-1} never leaves its LDS), C = A_cc -
//       P P^T, factor + invert C -> V_c, publish V_c.
//   workgroup w > 0 (worker) owns ONE lower tile (I, J), J >= 1, in
//       registers for the whole factorisation and applies the panel
//       updates k = 0 .. J-1 (J-2 on the diagonal: the last one is the
//       critical workgroup's C = A - P P^T) as soon as V_k and the tiles
//       (I, k), (J, k) are final, then publishes its tile.
//
// The per-step form paid, on every one of its T launches, the critical
// workgroup's re-staging of V_k and the serialisation of the launch
// boundary; here the chain per block column is: two tile fetches, the panel
// GEMM, C, the factor.  The trailing updates of step k run beside the
// factor of block k+1 (look-ahead), on the other CUs.
//
// Hand-offs (MI355X_MICROARCH.md, visibility, valid-forms table row 1; the
// publish/consume recipe of cdna_hip_programming.md Guideline 16, R1):
// every handed-off byte (published tiles of A, V_c) is stored write-through
// (16-B buffer stores with sc1), every storing wave drains (s_waitcnt
// vmcnt(0)) before the workgroup barrier, ONE lane then stores the flag
// (relaxed agent-scope atomic); the consumer's wave 0 polls the flag
// (relaxed agent-scope loads + s_sleep), the workgroup barrier releases the
// other waves, and EVERY load of handed-off bytes is a 16-B sc1 buffer load.
// Flags carry the factorisation's epoch (never 0, never reset).  Spins are
// bounded: a missing producer (e.g. a grid that could not be resident beside
// another process's work) sets SL_CHOL_SPIN instead of hanging the GPU; the
// host then redoes the step with the per-step launches.  Every workgroup of the
// grid must be resident at once: the host checks the occupancy first
// (chol_persist_fits) and otherwise runs the per-step launches.
#include "ba_chol.h"
#include "ba_schur.h"

namespace bahip {

// diagnostic build (tools/chol_bench.hip, BA_CHOL_STAMPS): s_memtime of the
// critical workgroup's phases per block column
#ifdef BA_CHOL_STAMPS
__device__ unsigned long long g_pstamps[64][8];
__device__ unsigned long long g_prt[64][8];       // the same stamps in s_memrealtime (100 MHz, chip-wide)
__device__ unsigned long long g_wstamps[64][6];   // worker (J+1, J), its last update (s_memrealtime)
__device__ unsigned long long g_estamps[64][2];   // end_step: entered, V stores issued (s_memtime)
#define WSTAMP(j, i)                                                                          \
  do {                                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    unsigned long long t_;                                                                    \
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");            \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    if (threadIdx.x == 0 && (j) < 64) g_wstamps[j][i] = t_;                                   \
  } while (0)
#define PSTAMP(c, i)                                                                          \
  do {                                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    unsigned long long t_;                                                                    \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    if (threadIdx.x == 0 && (c) < 64) g_pstamps[c][i] = t_;                                   \
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");            \
    if (threadIdx.x == 0 && (c) < 64) g_prt[c][i] = t_;                                       \
  } while (0)
#else
#define PSTAMP(c, i) do {} while (0)
#define WSTAMP(j, i) do {} while (0)
#endif

// diagnostic build (tools/ov_trace.py, BA_OV_TRACE): s_memrealtime (100 MHz)
// of the overlapped form's events: [0] the critical workgroup's start,
// [8 + t] tile t formed (pflag raised), [512 + c] / [768 + c] the critical's
// step c start / its inputs staged, [1024 + b] / [1536 + b] / [2048 + b]
// workgroup b's last item taken / own tile formed (seen) / own tile published
#ifdef BA_OV_TRACE
__device__ unsigned long long g_ovt[4096];
#define OVT(i)                                                                                \
  do {                                                                                        \
    unsigned long long t_;                                                                    \
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");            \
    if ((threadIdx.x & 63) == 0 && (i) < 4096) g_ovt[i] = t_;                                 \
  } while (0)
extern "C" int ba_debug_ov_trace(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ovt), sizeof(unsigned long long) * (n < 4096 ? n : 4096)) ==
                 hipSuccess
             ? 0
             : 2;
}
#else
#define OVT(i) do {} while (0)
#endif

constexpr unsigned kPersistSpin = 1u << 17;   // ~0.2 s of polls: far beyond any real wait (~20 us)
// (BA_CHOL_SPIN_MAX, diagnostics: a smaller bound, e.g. 1, so that the
// spin-fallback path of ba_solve runs; tests/test_gpu_parity.py)
constexpr int kOvCams = 200;                   // overlapped form: variable cameras of the LDS camera table (kLinLdsCams)
constexpr int kOvFar = 4;                      // overlapped form: a worker takes items while >= this many steps from its last update

// (tile_fetch_sc1: ba_chol.h)
// the same tile as tile_fetch_sc1 in two halves: the raw 16-B loads (clamped
// addresses) now, the zeroing when the tile goes to LDS.  The masks read the
// loaded registers, so formed at the fetch they made the compiler wait for
// the loads right there (the diagonal tile's ~2k-cycle round trip on the
// chain, before the panel GEMM it was meant to hide under)
template <bool LOWER = false>
__device__ inline TileRegs tile_issue_sc1(Rsrc r, size_t ld, int r0, int c0, int rmax, int cmax) {
  TileRegs t;
  const int tid = ctid();
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int e = tid + 256 * it;
    const int i = e >> 5, j = (e & 31) * 2;
    const bool up = LOWER && j > i;
    const int ri = r0 + i, cj = c0 + (up ? (i & ~1) : j);
    const int ric = min(ri, rmax - 1), cjc = min(cj, cmax - 2) & ~1;
    t.v[it] = ld_sc1(r, ((size_t)ric * ld + cjc) * sizeof(double));
  }
  return t;
}
template <bool LOWER = false>
__device__ inline void tile_put_masked(double (*D)[LDP], const TileRegs& t, int r0, int c0, int rmax, int cmax) {
  const int tid = ctid();
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int e = tid + 256 * it;
    const int i = e >> 5, j = (e & 31) * 2;
    const bool up = LOWER && j > i;
    const int ri = r0 + i, cj = c0 + (up ? (i & ~1) : j);
    const bool rok = ri < rmax && !up;
    D[i][j] = (rok && cj < cmax) ? t.v[it].x : 0.0;
    D[i][j + 1] = (rok && cj + 1 < cmax) ? t.v[it].y : 0.0;
  }
}

// (publish, publish_before_loads, wait_flag, make_rsrc, ld_sc1, st_sc1: ba_chol.h)

// The overlapped form (OvArgs::on): the reduced system S is formed INSIDE
// the launch, by the workgroups that do not yet hold a tile — the pair blocks
// of k_schur_pairs_cd, the diagonal slices of k_cam_schur_diag_cd and the
// fold of k_cam_fold_diag, as work items handed out in tile-column order
// (the order the factorisation consumes S), with the same arithmetic in the
// same order per S entry, so S (and with it L) is bitwise the serial form's.
//   items: per XCD (blockIdx & 7) a queue of wave-sized work items — a pair
//       item is 4 camera-pair blocks (16 lanes each, as k_schur_pairs_cd), a
//       diagonal item is one (camera, slice) of diag_cd_wave; the wave that
//       completes a camera's last slice folds it.  Each item stores its S
//       entries write-through (agent-scope atomic stores: sc1), drains, and
//       counts itself into every tile it wrote (cnt); the contribution that
//       completes a tile raises the tile's pflag.
//   workers (tile owners) take items until their own tile column comes up
//       in their queue, then wait for their tile's pflag and factor as
//       before; the critical workgroup waits for pflag of the tiles no worker
//       owns (column 0 and (1, 1)); extra workgroups past the workers
//       ("helpers") only take items.
// Counters and tickets are cumulative over the launches (pe = the launch
// count): nothing is reset, and every wave draws exactly one failing ticket
// per launch, so queue x's tickets of launch pe start at qbase[x] = (pe - 1)
// (items_x + 4 waves x its workgroups).  Items never wait, so the pass always
// completes; a missing tile is a bounded spin like any other hand-off.
struct OvArgs {
  int on = 0;
  int pass_only = 0;         // (diagnostics, ba_debug_blocks: every workgroup only takes items; no factorisation)
  int worker_items = 0;      // (diagnostics, BA_OV_WORKERS: 0 items between updates, 2 none)
  int far = kOvFar;          // (BA_OV_FAR: the distance from its last update below which a worker takes no item)
  DevProblem P;
  const int4* blocks;
  const int2* pairs;
  const double* Wc;          // compact W records (k_obs_w_rc<double, true>)
  const double* scale_c;
  const double* u;           // [np][4] u_p (diagonal slices)
  const double* Hcc;
  const double* gc;
  const double* diag_c;
  double radius;
  double* cpart;             // [G][nvc][27] slices
  int G;
  // item i: irec[4 i .. 4 i + 3], one int4 per 16-lane group: a pair item's
  // blocks {I, J, start, end} (no block: zeros), or a diagonal item's
  // {-1 - (v G + g), 0, 0, 0} first
  const int4* irec;
  const int* item_col;       // the tile column each item belongs to
  const unsigned* tgt;       // [TR][T] contributions per tile and launch
  unsigned* cnt;             // [TR][T] contributions (cumulative)
  unsigned* cam_cnt;         // [nvc] slices done (cumulative)
  unsigned* q;               // [8] tickets drawn (cumulative)
  unsigned* pflag;           // [TR][T] tile formed: the factorisation epoch
  int ioff[9];               // queue x's items: [ioff[x], ioff[x+1])
  unsigned qbase[8];
  unsigned pe;
};

struct PersistArgs {
  double* A;         // working matrix ((n+1) x ld)
  double* L;         // output factor
  double* Vbuf;      // [T][64][64] diagonal-block inverses
  double* scal;
  unsigned* flags;   // [T] V_c published | [TR][T] tile (I, J) published
  int ld, n, T, TR;
  unsigned epoch;
  unsigned spin_max;   // polls per hand-off before SL_CHOL_SPIN (kPersistSpin)
  OvArgs ov;           // ov.on: S formed inside the launch
};

// worker w (>= 1) -> its tile (I, J): tiles with J >= 1 and I >= J, in
// column order, without the diagonal tile (1, 1) (no update reaches it
// before the critical workgroup's)
__device__ inline bool worker_tile(int w, int T, int TR, int& I, int& J) {
  int idx = w - 1;
  for (int j = 1; j < T; ++j) {
    const int first = j == 1 ? 2 : j;   // (1, 1) has no worker
    const int cnt = TR - first;
    if (idx < cnt) { I = first + idx; J = j; return true; }
    idx -= cnt;
  }
  return false;
}

// V_c's lower 16x16 blocks [blk0, blk0 + nblk) in row-block order ((0,0),
// (1,0), (1,1), (2,0), ...) from LDS to Vbuf (write-through, 16-B pieces,
// row-contiguous), by the nthr threads with index t
__device__ __forceinline__ void store_v_blocks(Rsrc rV, size_t vbase, const double (*X)[LDP], int blk0, int nblk,
                                               int t, int nthr) {
  for (int e = t; e < nblk * 16 * 8; e += nthr) {
    const int blk = blk0 + (e >> 7), rr = (e >> 3) & 15, cc = (e & 7) * 2;
    const int bi = blk < 1 ? 0 : (blk < 3 ? 1 : (blk < 6 ? 2 : 3));
    const int bj = blk - bi * (bi + 1) / 2;
    const int i = 16 * bi + rr, j = 16 * bj + cc;
#ifndef BA_CHOL_NO_VSTORE
    st_sc1(rV, vbase + ((size_t)i * CB + j) * sizeof(double), make_double2(X[i][j], X[i][j + 1]));
#endif
  }
}

// The next panel tile A_{c+1,c} into S3 by waves 2 and 3 (each wave one half,
// 32 rows), spread over the factor so that no global round trip lands on a
// sub-panel barrier: p = 1 polls the worker's flag (one relaxed load, no
// spin); p = 2 fetches the half if the flag was seen, else polls again and
// fetches at once when it is up; p = 3 polls if needed and only ISSUES the
// loads, which land in LDS at the end of the inverse tail (finish()).  A half
// still missing then is fetched at the next step's start.  (The worker of
// A_{c+1,c} publishes it ~30k cycles after V_{c-1}: in sub-panel 3 mostly,
// tools/chol_bench.hip.)  ok[w - 2]: 0 not yet, 2 flag seen, 1 landed in S3
// (only lane 0 of the owning wave writes it; LDS is in order within the wave).
struct PanelPrefetch {
  Rsrc rA;
  size_t ld;
  const unsigned* flag;   // nullptr: column 0, never updated (always ready)
  unsigned epoch;
  double (*S3)[LDP];
  int* ok;
  int r0, kc, nrows, cmax;
  int c;                  // diagnostics (BA_CHOL_STAMPS): the step, for the fetch-phase record
  const unsigned* dflag;  // the next diagonal tile's flag (nullptr: no worker, ready)
  int* dready;            // finish(): that flag seen up (polled once by wave 2)
  // V_c's row blocks 0..2, final before the last sub-panel's sweep ends
  // (row block q by wave 1 beside sweep q + 1): stored here, under wave 0's
  // chain — row blocks 0, 1 in sub-panel 3, row block 2 in the inverse tail
  // — so that the end of the step stores only row block 3 (4 of the 10 lower
  // blocks; the stores and the diagonal tile's loads behind them were ~3.5k
  // cycles of the step's chain, tools/chol_bench.hip)
  Rsrc rV;
  size_t vbase;           // byte offset of V_c in Vbuf
  const double (*X)[LDP];
  mutable double2 v[16];  // loads in flight between p = 3 and land()
  mutable bool pending = false;
  __device__ bool poll() const {
    if (!flag) return true;
    const unsigned f = (ctid() & 63) == 0 ? __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                               : 0u;
    return __builtin_amdgcn_readfirstlane(f) == epoch;
  }
  // this wave's 32 rows x 32 pairs = 1024 pairs, 16 per lane
  __device__ void issue() const {
    const int w = cwave(), lane = ctid() & 63, hr = 32 * (w - 2);
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int e = lane + 64 * it;
      const int i = hr + (e >> 5), j = (e & 31) * 2;
      const int ri = r0 + i, cj = kc + j;
      const int ric = min(ri, nrows - 1), cjc = min(cj, cmax - 2) & ~1;
      v[it] = ld_sc1(rA, ((size_t)ric * ld + cjc) * sizeof(double));
    }
  }
  __device__ void land(int p) const {
    const int w = cwave(), lane = ctid() & 63, hr = 32 * (w - 2);
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int e = lane + 64 * it, i = hr + (e >> 5), j = (e & 31) * 2;
      const int ri = r0 + i, cj = kc + j;
      const bool rok = ri < nrows;
      S3[i][j] = (rok && cj < cmax) ? v[it].x : 0.0;
      S3[i][j + 1] = (rok && cj + 1 < cmax) ? v[it].y : 0.0;
    }
    if (lane == 0) ok[w - 2] = 1;
#ifdef BA_CHOL_STAMPS
    if (lane == 0 && w == 2 && c < 64) g_pstamps[c][7] = (unsigned long long)p;   // sub-panel of the fetch
#endif
  }
  __device__ void operator()(int p) const {
    const int w = cwave(), lane = ctid() & 63;   // w = 2 or 3
    if (p == 3) store_v_blocks(rV, vbase, X, 0, 3, ctid() - 128, 128);
    const int st = __builtin_amdgcn_readfirstlane(ok[w - 2]);   // 0 at p = 1 (reset at the step start)
    if (st == 1) return;
    if (st == 0) {
      if (!poll()) return;
      if (p == 1) {
        if (lane == 0) ok[w - 2] = 2;
        return;
      }
    }
    issue();
    if (p == 2) land(p);
    else pending = true;
  }
  __device__ void land() const {
    if (pending) land(3);
    pending = false;
    store_v_blocks(rV, vbase, X, 3, 3, ctid() - 128, 128);
  }
  __device__ void finish() const {
    if (pending) land(3);
    if (cwave() == 2) {
      bool up = true;
      if (dflag) {
        const unsigned f = (ctid() & 63) == 0
                               ? __hip_atomic_load(dflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                               : 0u;
        up = __builtin_amdgcn_readfirstlane(f) == epoch;
      }
      if ((ctid() & 63) == 0) *dready = up ? 1 : 0;
    }
  }
};

// ---------------------------------------------------------------- overlapped S
// one tile's contribution counted; the one that completes the tile raises pflag
__device__ __forceinline__ void ov_count(const OvArgs& o, int t, unsigned epoch) {
  const unsigned old = __hip_atomic_fetch_add(&o.cnt[t], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (old + 1u == o.pe * o.tgt[t]) {
    __hip_atomic_store(&o.pflag[t], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#ifdef BA_OV_TRACE
    unsigned long long t_;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");
    if (8 + t < 512) g_ovt[8 + t] = t_;
#endif
  }
}

// LDS-DMA issued by inline asm (the pair item's pipeline): the compiler,
// which does not see these loads, then neither counts them nor inserts the
// vmcnt(0) it puts before any LDS access that may follow an LDS-DMA
// intrinsic (that wait would drain the second round at every round).  Every
// wait on them is explicit.  M0 = the wave's LDS byte address; nothing else
// in this kernel's pair path touches M0.
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return __builtin_amdgcn_readfirstlane((unsigned)(size_t)(__attribute__((address_space(3))) const void*)p);
}
// (M0 is a reserved register: clang warns on the clobber, which the compiler
// honours — it re-sets M0 before each of its own uses)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void adma16(const void* src, unsigned lds) {   // 16 B per lane, lane-linear
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(lds) : "memory", "m0");
}
__device__ __forceinline__ void adma4(const void* src, unsigned lds) {    // 4 B per lane, lane-linear
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(src), "s"(lds) : "memory", "m0");
}
#pragma clang diagnostic pop

// one pair item by one wave: 4 camera-pair blocks, 16 lanes each — the lanes,
// pairs, products and xor reduction of k_schur_pairs_cd (bitwise its S
// blocks).  The records go through LDS by LDS-DMA as there, two rounds in
// flight (region: 2 x (row, partner) x 64 records = 32 KB): the
// factorisation's one workgroup per CU leaves each wave alone on its SIMD, so
// the second round is what hides the gather latency.  The pair indices come
// by LDS-DMA too, three rounds ahead (islot: 4 x 64 {x, y}), so no register
// is ever loaded in flight.  Round t requests round t + 3's indices (2
// pieces, if that round exists) and round t + 2's records (16 pieces, if it
// exists); so behind round t's records there are round t + 2's indices and
// round t + 1's records, and behind round t + 2's indices round t + 1's
// records: vmcnt(16) waits for both while round t + 1 exists, vmcnt(0) at
// the last round.
__device__ __forceinline__ void ov_pair_item(const OvArgs& o, int4 blk, const WcCam* ctab, double* region, int* islot,
                                             double* S, size_t ld, int T, unsigned epoch) {
  constexpr int PL = kPairLanes;
  static_assert(64 / PL == 4, "a pair item is 4 blocks per wave");
  const int lane = threadIdx.x & 63, sl = lane & (PL - 1);
  const bool live = blk.w > blk.z;
  const WcCam& mI = ctab[blk.x];   // (the workgroup's LDS camera table)
  const WcCam& mJ = ctab[blk.y];
  const int swr = (lane >> 1) & 7;
  const int len = blk.w - blk.z;
  int nit = len > sl ? (len - sl + PL - 1) / PL : 0;
#pragma unroll
  for (int x = 32; x >= 1; x >>= 1) nit = max(nit, __shfl_xor(nit, x));
  nit = __builtin_amdgcn_readfirstlane(nit);   // (a uniform loop)
  const int e0 = blk.z + sl;
  // round t's buffers: records (row at +0, partner at +64 records), indices
  // (x at +0, y at +64 ints)
  auto rbuf = [&](int t) { return region + (t & 1) * (128 * kWcRec); };
  auto ibuf = [&](int t) { return islot + (t & 3) * 128; };
  auto req_idx = [&](int t) {   // round t's pair of this lane -> ibuf(t)
    const int2* p = o.pairs + max(min(e0 + t * PL, blk.w - 1), 0);
    const int* ib = ibuf(t);
    adma4(&p->x, lds_addr(ib));
    adma4(&p->y, lds_addr(ib + 64));
  };
  auto req_rec = [&](int t) {   // round t's records (its indices in ibuf(t)) -> rbuf(t)
    const int* ib = ibuf(t);
    const int2 pr = make_int2(ib[lane], ib[64 + lane]);
    double* rb = rbuf(t);
    const unsigned lr = lds_addr(rb), lp = lds_addr(rb + 64 * kWcRec);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int q = (lane >> 3) + 8 * i;
      const int ra = __shfl(pr.x, q), rq = __shfl(pr.y, q);
      const int sp = 2 * ((lane & 7) ^ ((q >> 1) & 7));
      adma16(o.Wc + (size_t)ra * kWcRec + sp, lr + i * 1024);
      adma16(o.Wc + (size_t)rq * kWcRec + sp, lp + i * 1024);
    }
  };
  auto read_rec = [&](const double* buf) {
    WcRaw w;
    const double* r = buf + lane * kWcRec;
#pragma unroll
    for (int p = 0; p < kWcRec / 2; ++p) {
      const double2 t = *reinterpret_cast<const double2*>(r + 2 * (p ^ swr));
      w.r[2 * p] = t.x;
      w.r[2 * p + 1] = t.y;
    }
    return w;
  };
  double acc[36];
#pragma unroll
  for (int k = 0; k < 36; ++k) acc[k] = 0.0;
  // prologue: indices of rounds 0, 1 (waited), records 0, indices 2, records 1
  req_idx(0);
  if (nit > 1) req_idx(1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  req_rec(0);
  if (nit > 2) req_idx(2);
  if (nit > 1) req_rec(1);
  for (int t = 0; t < nit; ++t) {
    if (t + 1 < nit) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const WcRaw wa = read_rec(rbuf(t));
    const WcRaw wb = read_rec(rbuf(t) + 64 * kWcRec);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // read out before the refill
    if (t + 3 < nit) req_idx(t + 3);
    if (t + 2 < nit) req_rec(t + 2);
    if (e0 + t * PL < blk.w) {
      double ca0[6], ca1[6], cb0[6], cb1[6];
      wc_rows(wa, mI, ca0, ca1);
      wc_rows(wb, mJ, cb0, cb1);
      const double* za0 = wa.r + 9;
      const double* za1 = wa.r + 12;
      const double* zb0 = wb.r + 9;
      const double* zb1 = wb.r + 12;
      const double m00 = za0[0] * zb0[0] + za0[1] * zb0[1] + za0[2] * zb0[2];
      const double m01 = za0[0] * zb1[0] + za0[1] * zb1[1] + za0[2] * zb1[2];
      const double m10 = za1[0] * zb0[0] + za1[1] * zb0[1] + za1[2] * zb0[2];
      const double m11 = za1[0] * zb1[0] + za1[1] * zb1[1] + za1[2] * zb1[2];
      double n0[6], n1[6];
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        n0[j] = m00 * cb0[j] + m01 * cb1[j];
        n1[j] = m10 * cb0[j] + m11 * cb1[j];
      }
#pragma unroll
      for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < 6; ++j) acc[i * 6 + j] += ca0[i] * n0[j] + ca1[i] * n1[j];
    }
  }
#pragma unroll
  for (int k = 0; k < 36; ++k) {
    double v = acc[k];
#pragma unroll
    for (int x = PL / 2; x >= 1; x >>= 1) v += __shfl_xor(v, x, PL);
    acc[k] = v;
  }
  if (live) {
    const int I = blk.x, Jb = blk.y;   // I > Jb (no point observed twice by one camera in this form)
#pragma unroll
    for (int k = 0; k < 36; ++k) {
      if ((k % PL) != sl) continue;
      const int i = k / 6, j = k % 6;
      __hip_atomic_store(S + (size_t)(6 * I + i) * ld + 6 * Jb + j, -acc[k], __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the S stores are done
  if (live && sl == 0) {
    const int r0 = (6 * blk.x) >> 6, r1 = (6 * blk.x + 5) >> 6;
    const int c0 = (6 * blk.y) >> 6, c1 = (6 * blk.y + 5) >> 6;
    ov_count(o, r0 * T + c0, epoch);
    if (c1 != c0) ov_count(o, r0 * T + c1, epoch);
    if (r1 != r0) {
      ov_count(o, r1 * T + c0, epoch);
      if (c1 != c0) ov_count(o, r1 * T + c1, epoch);
    }
  }
}

// one diagonal item by one wave: camera slice (v, g) of diag_cd_wave (the
// one-wave sum of the pair launch's diagonal workgroups), stored to cpart;
// the wave that stores a camera's last slice folds it (k_cam_fold_diag's
// entries, lanes 0..26)
__device__ __forceinline__ void ov_diag_item(const OvArgs& o, int unit, double* region, double* S, int T,
                                          unsigned epoch) {
  const int lane = threadIdx.x & 63;
  const int nvc = o.P.nvc;
  const int v = unit / o.G, g = unit - v * o.G;
  double acc[27];
  diag_cd_wave(o.P, o.Wc, o.scale_c, o.u, v, g, o.G, region, region + 64 * kWcRec, acc);
  double tot[27];
#pragma unroll
  for (int k = 0; k < 27; ++k) tot[k] = 0.0 + wave_sum(acc[k]);   // (block_sum's value for one wave)
  if (lane == 0) {
    double* dst = o.cpart + ((size_t)g * nvc + v) * 27;
#pragma unroll
    for (int k = 0; k < 27; ++k) __hip_atomic_store(dst + k, tot[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  unsigned old = 0;
  if (lane == 0) old = __hip_atomic_fetch_add(&o.cam_cnt[v], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  old = __builtin_amdgcn_readfirstlane(old);
  if (old + 1u != o.pe * (unsigned)o.G) return;
  // the fold of camera v
  if (lane < 27)
    cam_fold_diag_entry<true>(o.P, o.cpart, o.G, o.Hcc, o.gc, o.scale_c, o.diag_c, o.radius, S, nullptr,
                              v * 27 + lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane < 27) {
    int row, col;
    fold_entry_pos(o.P.n, v, lane, row, col);
    ov_count(o, (row >> 6) * T + (col >> 6), epoch);
  }
}

// queue x: a ticket (wave-uniform); false: the queue is exhausted (this wave's
// one failing draw of the launch)
__device__ __forceinline__ bool ov_draw(const OvArgs& o, int x, int& item) {
  unsigned t = 0;
  if ((threadIdx.x & 63) == 0) t = __hip_atomic_fetch_add(&o.q[x], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  t = __builtin_amdgcn_readfirstlane(t) - o.qbase[x];
  const unsigned nq = (unsigned)(o.ioff[x + 1] - o.ioff[x]);
  if (t >= nq) return false;
  item = o.ioff[x] + (int)t;
  return true;
}
__device__ __forceinline__ void ov_run(const OvArgs& o, int item, const WcCam* ctab, double* region, int* islot,
                                       double* S, size_t ld, int T, unsigned epoch) {
  const int4 mine = o.irec[4 * (size_t)item + ((threadIdx.x & 63) >> 4)];
  const int head = __builtin_amdgcn_readfirstlane(mine.x);   // (lanes 0..15: the item's first record)
  if (head >= 0) ov_pair_item(o, mine, ctab, region, islot, S, ld, T, epoch);
  else ov_diag_item(o, -1 - head, region, S, T, epoch);
}
// items until the queue is exhausted; this wave's failing draw is the last.
// (Drawing the next ticket as the current item starts, to hide the atomic's
// round trip, measured slower: a wave busy with its item then holds the next
// one, and the early tile columns completed later — C3 pass alone 236 vs
// 221 us, tile (0, 0) formed at 47 vs 38 us: profiles/r06_v5_ov_prefetch_ab.txt)
__device__ __forceinline__ void ov_take(const OvArgs& o, const WcCam* ctab, double* region, int* islot, double* S,
                                        size_t ld, int T, unsigned epoch) {
  const int x = blockIdx.x & 7;
  int item;
  while (ov_draw(o, x, item)) ov_run(o, item, ctab, region, islot, S, ld, T, epoch);
}

// block 0: the critical workgroup, block w > 0: worker w
__global__ __launch_bounds__(256) void k_chol_persist(PersistArgs a) {
  // S0..S3; S3: the next panel tile A_{c+1,c}, prefetched during the factor.
  // (Overlapped form: before a workgroup takes up its tile, its waves' 32-KB
  // slices of this array are the work items' LDS-DMA rounds)
  __shared__ __attribute__((aligned(16))) double Sall[4][CB][LDP];
  double (*S0)[LDP] = Sall[0];
  double (*S1)[LDP] = Sall[1];
  double (*S2)[LDP] = Sall[2];
  double (*S3)[LDP] = Sall[3];
  __shared__ int pref_ok[2];
  __shared__ int dready[1];        // the next diagonal tile's flag was up at the factor's end
  __shared__ CholLds cw;
  const int n = a.n, nrows = n + 1, T = a.T;
  const size_t ld = (size_t)a.ld;
  const Rsrc rA = make_rsrc(a.A, (size_t)nrows * ld * sizeof(double));
  const Rsrc rV = make_rsrc(a.Vbuf, (size_t)(T + 1) * CB * CB * sizeof(double));
  unsigned* vflag = a.flags;
  unsigned* tflag = a.flags + T;
  bool bad = false;    // a non-positive pivot
  bool spin = false;   // a hand-off spin bound hit
  double* region = &Sall[0][0][0] + (size_t)(threadIdx.x >> 6) * (4 * 64 * kWcRec);   // this wave's 32 KB
  __shared__ __attribute__((aligned(16))) int ov_islot[4][4][128];                        // its pair-index slots
  int* islot = ov_islot[threadIdx.x >> 6][0];
  __shared__ WcCam ov_ctab[kOvCams];   // (overlapped form: the pair items' camera constants)
  const OvArgs& ov = a.ov;
  if (ov.on && (blockIdx.x != 0 || ov.pass_only)) {   // (the critical workgroup takes items only at its end, and fills it then)
    for (int v = threadIdx.x; v < ov.P.nvc; v += 256) ov_ctab[v].load(ov.P, ov.scale_c, v);
    __syncthreads();
  }
  // tiles no worker owns (column 0, and (1, 1)) are final once formed: with
  // the overlapped form their pflag, else ready from before the launch
  auto formed = [&](int I, int J) -> const unsigned* { return ov.on ? &ov.pflag[I * T + J] : nullptr; };
  // roles (pass-only diagnostics: none); then every workgroup's items (its
  // waves' failing draws, and whatever is left) — one copy of the item code
  bool drew_fail = false;   // (overlapped form: this wave's failing draw)
  int I = 0, J = 0;
  const bool worker = !ov.pass_only && blockIdx.x != 0 && worker_tile(blockIdx.x, T, a.TR, I, J);
  if (blockIdx.x == 0 && !ov.pass_only) {
    // ---------------- critical workgroup: the diagonal chain
    if (threadIdx.x == 0) { pref_ok[0] = 0; pref_ok[1] = 0; dready[0] = 0; }
    if (ov.on) OVT(0);
    if (ov.on && threadIdx.x == 0) {   // (the serial form's fold clears them before the launch)
      __hip_atomic_store(&a.scal[SL_CHOL_BAD], 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&a.scal[SL_CHOL_SPIN], 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // the end of step cp: V_cp cleaned in place (zero above the diagonal,
    // identity rows past b: exactly the Vbuf image the per-step form
    // re-stages) for the next panel GEMM, stored write-through and published
    // to the workers (their trailing updates of step cp, and with them the
    // next panel and diagonal tiles, wait for it).  The loop is rotated: this
    // runs at the start of iteration cp + 1, so that the next diagonal tile's
    // loads (issued here behind the V stores when its flag was up at the end
    // of the factor, hook.finish) are consumed in the same iteration — tD is
    // never live across the loop's back edge.
    auto end_step = [&](int cp) {
      const int sp = cp * CB, bp = min(CB, n - sp), mp = min(CB, nrows - sp);
#ifdef BA_CHOL_STAMPS
      {
        __builtin_amdgcn_sched_barrier(0);
        unsigned long long t_;
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");
        __builtin_amdgcn_sched_barrier(0);
        if (threadIdx.x == 0 && cp < 64) g_estamps[cp][0] = t_;
      }
#endif
      if (bp == CB) {
        // a full block: only the lower block triangle (10 of 16 blocks) is
        // read again — the panel products skip the upper blocks, k_back_flow
        // masks them — and the diagonal blocks already hold exact zeros
        // above the diagonal (diag_inverse16): no clean-up pass, 5 / 8 of
        // the stores; row blocks 0..2 went out during the factor (the
        // prefetch hook) unless this was the last block column
        // (the upper blocks' Vbuf entries stay stale, unread)
        const bool hooked = cp + 1 < T;
        store_v_blocks(rV, (size_t)cp * CB * CB * sizeof(double), S2, hooked ? 6 : 0, hooked ? 4 : 10, ctid(), 256);
        bad |= cw.bad != 0;
#ifdef BA_CHOL_STAMPS
        {
          __builtin_amdgcn_sched_barrier(0);
          unsigned long long t_;
          asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");
          __builtin_amdgcn_sched_barrier(0);
          if (threadIdx.x == 0 && cp < 64) g_estamps[cp][1] = t_;
        }
#endif
        return;
      }
      for (int e2 = ctid(); e2 < CB * CB / 2; e2 += 256) {
        const int i = (2 * e2) / CB, j = (2 * e2) % CB;
        double v[2];
#pragma unroll
        for (int h = 0; h < 2; ++h)
          v[h] = (j + h <= i && i < bp && j + h < bp) ? S2[i][j + h] : (i == j + h ? 1.0 : 0.0);
        S2[i][j] = v[0];
        S2[i][j + 1] = v[1];
        st_sc1(rV, ((size_t)cp * CB * CB + 2 * (size_t)e2) * sizeof(double), make_double2(v[0], v[1]));
      }
      if (mp > bp)
        for (int j = ctid(); j < bp; j += 256) a.L[(size_t)(sp + bp) * ld + sp + j] = S0[bp][j];
      bad |= cw.bad != 0;
    };
    for (int c = 0; c < T; ++c) {
      const int s = c * CB;
      const int b = min(CB, n - s);
      const int m = min(CB, nrows - s);
      bool have_diag = false;
      TileRegs tD;
      if (c > 0) {
        end_step(c - 1);
        // A_{c,c}: in flight from here when its worker had published it by
        // the end of the factor (S0 is rewritten only at the panel GEMM,
        // after L's last read above); the V drain waits for the stores only
        have_diag = dready[0] != 0;
        if (have_diag) {
          asm volatile("" ::: "memory");   // (the loads after the V stores)
          tD = tile_issue_sc1<true>(rA, ld, s, s, nrows, s + b);
        }
        PSTAMP(c - 1, 6);
        if (have_diag) publish_before_loads(&vflag[c - 1], a.epoch);
        else publish(&vflag[c - 1], a.epoch);
      }
      PSTAMP(c, 0);
      if (ov.on && threadIdx.x < 64) OVT(512 + c);
#ifdef BA_CHOL_STAMPS
      if (threadIdx.x == 0) g_stamp_on = c == T / 2;   // the factor's inner stamps: one mid step
      if (threadIdx.x == 0 && c < 64) g_pstamps[c][7] = 0;
#endif
      if (c == 0) {
        if (ov.on) {                               // formed in this launch
          spin |= !wait_flag(formed(0, 0), a.epoch, a.spin_max);
          tile_put(S0, tile_fetch_sc1(rA, ld, 0, 0, nrows, b));
        } else {
          stage64(S0, a.A, ld, 0, 0, nrows, b);   // written before the launch
        }
      } else {
        const int k = c - 1, kc = k * CB, kb = min(CB, n - kc);
        // A_{c,k} final (its worker; column 0 is never updated): prefetched
        // into S3 during the last factor when published by then, else fetched
        // here; the diagonal tile after the updates k' <= c - 2 (no worker for
        // c = 1), unless already in flight, is fetched into registers here;
        // it lands behind the panel GEMM
        const bool have_pref = pref_ok[0] == 1 && pref_ok[1] == 1;   // (read after the factor's last barrier)
        if (!have_pref) {
          if (k >= 1) spin |= !wait_flag(&tflag[c * T + k], a.epoch, a.spin_max);
          else if (ov.on) spin |= !wait_flag(formed(c, 0), a.epoch, a.spin_max);
          const TileRegs tP = tile_fetch_sc1(rA, ld, s, kc, nrows, kc + kb);   // A_{c,k}
          tile_put(S3, tP);
        }
        // (its barrier also covers S3; the plain form is an LDS-only
        // barrier, so the diagonal tile's loads stay in flight across it)
        if (c >= 2 && !have_diag) spin |= !wait_flag(&tflag[c * T + c], a.epoch, a.spin_max);
        else if (c == 1 && ov.on && !have_diag) spin |= !wait_flag(formed(1, 1), a.epoch, a.spin_max);
        else lds_barrier();
        if (threadIdx.x == 0) { pref_ok[0] = 0; pref_ok[1] = 0; dready[0] = 0; }
        PSTAMP(c, 1);
        if (ov.on && threadIdx.x < 64) OVT(768 + c);
        if (!have_diag) tD = tile_issue_sc1<true>(rA, ld, s, s, nrows, s + b);   // A_{c,c} (+ rhs row), in flight
        PSTAMP(c, 2);
        d4 acc[4];
        mfma_xVT_strip(S3, S2, acc);            // P = A_{c,k} V_k^T (V_k: S2, from the last iteration)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the diagonal tile has landed
        tile_put_masked<true>(S0, tD, s, s, nrows, s + b);
        // P = L_{c,k} to the factor: here only without a worker (c+1, c),
        // which otherwise stores the same product (its P_J) off this chain
        const bool store_l = c + 1 >= a.TR;
        {
          const int lane = ctid() & 63, w = cwave();
#pragma unroll
          for (int bc = 0; bc < 4; ++bc)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const int rr = 16 * w + (lane >> 4) + 4 * g, cc = 16 * bc + (lane & 15);
              S1[rr][cc] = acc[bc][g];
              if (store_l && rr < m && cc < kb) a.L[(size_t)(s + rr) * ld + kc + cc] = acc[bc][g];
            }
        }
        __syncthreads();
        PSTAMP(c, 3);
        mfma_xxT_col0(S1, S0);                  // C = A - P P^T: column 0 now, the rest beside the first sweep
      }
      if (threadIdx.x == 0) cw.bad = 0;
      PSTAMP(c, 4);
      if (c + 1 < T) {
        // next step's panel tile A_{c+1,c}: final once its worker published
        // it (column 0: from before the launch)
        const PanelPrefetch pf{rA, ld, c >= 1 ? &tflag[(c + 1) * T + c] : formed(1, 0), a.epoch, S3, pref_ok,
                               (c + 1) * CB, c * CB, nrows, c * CB + min(CB, n - c * CB), c,
                               c + 1 >= 2 ? &tflag[(c + 1) * T + c + 1] : formed(1, 1), dready,
                               rV, (size_t)c * CB * CB * sizeof(double), S2};
        // (inlined: as a call its prefetch hook object would live in scratch)
        [[clang::always_inline]] factor_invert_blk<1>(S0, S2, S1, cw, b, m, c > 0 ? S1 : nullptr, pf);   // b = m = CB before the last block
      } else {
        factor_invert_blk<0>(S0, S2, S1, cw, b, m, c > 0 ? S1 : nullptr);
      }
      __syncthreads();
      PSTAMP(c, 5);
    }
    end_step(T - 1);
    PSTAMP(T - 1, 6);
    publish(&vflag[T - 1], a.epoch);
    if (threadIdx.x == 0 && bad) atomicAdd(&a.scal[SL_CHOL_BAD], 1.0);
    if (threadIdx.x == 0 && spin) atomicAdd(&a.scal[SL_CHOL_SPIN], 1.0);
#ifdef BA_CHOL_STAMPS
    if (threadIdx.x == 0) g_stamp_on = 1;
#endif
    if (ov.on) {   // (its camera table, for the items it may still find)
      __syncthreads();
      for (int v = threadIdx.x; v < ov.P.nvc; v += 256) ov_ctab[v].load(ov.P, ov.scale_c, v);
    }
  } else if (worker) {

    // ---------------- worker: one lower tile (I, J), J >= 1 (or a helper)
    // The tile's updates accumulate from zero, own = ((0 - u_0) - u_1) - ...,
    // and the tile itself is added at the end, A + own (k_chol_step keeps the
    // same order through its U buffer, so both forms round alike): a worker
    // needs its tile only for its last update.  Overlapped form: while update k
    // is not ready and this tile is at least kOvFar block steps from its last
    // update, the waves take work items (one each per round); near it, and
    // once the queue is empty, the worker only factors.
    const bool diag = I == J;
    const int r0 = I * CB, c0 = J * CB;
    const int mI = min(CB, nrows - r0);
    double own[2][2][4];   // (the MFMA accumulator layout, acc_pos)
  #pragma unroll
    for (int x = 0; x < 2; ++x)
  #pragma unroll
      for (int y = 0; y < 2; ++y)
  #pragma unroll
        for (int g = 0; g < 4; ++g) own[x][y][g] = 0.0;
    const int kmax = diag ? J - 2 : J - 1;
    const bool stamp = I == J + 1;   // (diagnostics: the next-panel tiles' last update)
    // the panel tiles A_{I,k}, A_{J,k} of update k are final long before V_k
    // (their workers finished update k - 1 one step earlier): they are staged
    // while V_k is awaited, so only V_k's fetch follows its flag
    auto stage_panels = [&](int k) {
      const int kc = k * CB, kb = min(CB, n - kc);
      if (k >= 1) {
        spin |= !wait_flag(&tflag[I * T + k], a.epoch, a.spin_max);
        if (!diag) spin |= !wait_flag(&tflag[J * T + k], a.epoch, a.spin_max);
      } else if (ov.on) {   // column 0: formed in this launch, never updated
        spin |= !wait_flag(formed(I, 0), a.epoch, a.spin_max);
        if (!diag) spin |= !wait_flag(formed(J, 0), a.epoch, a.spin_max);
      }
      const TileRegs tI = tile_fetch_sc1(rA, ld, r0, kc, nrows, kc + kb);        // A_{I,k}
      TileRegs tJ;
      if (!diag) tJ = tile_fetch_sc1(rA, ld, c0, kc, n, kc + kb);              // A_{J,k}
      tile_put(S0, tI);
      if (!diag) tile_put(S1, tJ);
    };
    __shared__ int ov_sh[2];   // (overlapped form: update k ready | the queue is empty)
    bool no_items = !ov.on || ov.worker_items != 0;
    if (threadIdx.x == 0) ov_sh[1] = 0;
    auto up = [&](const unsigned* f) {
      return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == a.epoch;
    };
    bool staged = false;
    if (kmax >= 0 && (no_items || J < ov.far)) {
      stage_panels(0);
      staged = true;
    }
    for (int k = 0; k <= kmax;) {
      if (!no_items && J - k >= ov.far) {
        if (threadIdx.x == 0) {
          bool r = up(&vflag[k]);
          if (r) r = k >= 1 ? up(&tflag[I * T + k]) && (diag || up(&tflag[J * T + k]))
                            : up(formed(I, 0)) && (diag || up(formed(J, 0)));
          ov_sh[0] = r ? 1 : 0;
        }
        __syncthreads();
        const bool ready = ov_sh[0] != 0;
        if (!ready) {
          int item;
          if (ov_draw(ov, blockIdx.x & 7, item)) {
            ov_run(ov, item, ov_ctab, region, islot, a.A, ld, T, a.epoch);
          } else {
            drew_fail = true;
            if ((threadIdx.x & 63) == 0) ov_sh[1] = 1;
          }
          __syncthreads();
          no_items = ov_sh[1] != 0;
          continue;
        }
        __syncthreads();   // (ov_sh[0] is read)
      }
      if (!staged) stage_panels(k);
      spin |= !wait_flag(&vflag[k], a.epoch, a.spin_max);
      if (stamp && k == kmax) WSTAMP(J, 0);
      tile_put(S2, tile_fetch_sc1(rV, CB, k * CB, 0, (k + 1) * CB, CB));          // V_k (stored cleaned)
      __syncthreads();
      if (stamp && k == kmax) WSTAMP(J, 1);
      // the tile itself, for the last update: in flight under its GEMMs
      // (overlapped: formed in this launch, sc1 loads)
      double av[2][2][4];
      if (k == kmax) {
        if (ov.on) spin |= !wait_flag(&ov.pflag[I * T + J], a.epoch, a.spin_max);
        if (ov.on && threadIdx.x < 64) OVT(1536 + blockIdx.x);
  #pragma unroll
        for (int x = 0; x < 2; ++x)
  #pragma unroll
          for (int y = 0; y < 2; ++y)
  #pragma unroll
            for (int g = 0; g < 4; ++g) {
              int rr, cc;
              acc_pos(x, y, g, &rr, &cc);
              const size_t off = (size_t)min(r0 + rr, nrows - 1) * ld + min(c0 + cc, n - 1);
              av[x][y][g] = ov.on ? __hip_atomic_load(a.A + off, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : a.A[off];
            }
      }
      // P_I = A_{I,k} V_k^T, P_J likewise: V_k is lower triangular, so the
      // strip products skip its zero blocks (40 instead of 64 MFMAs per wave;
      // the skipped terms are exact zeros, so the sums are those of the full
      // product)
      d4 sI[4], sJ[4];
      mfma_xVT_strip(S0, S2, sI);
      if (!diag) mfma_xVT_strip(S1, S2, sJ);
      __syncthreads();
      if (stamp && k == kmax) WSTAMP(J, 2);
      {
        const int lane = ctid() & 63, wv = cwave();
  #pragma unroll
        for (int bc = 0; bc < 4; ++bc)
  #pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int rr = 16 * wv + (lane >> 4) + 4 * g, cc = 16 * bc + (lane & 15);
            S0[rr][cc] = sI[bc][g];
            if (!diag) S1[rr][cc] = sJ[bc][g];
            if (J == k + 1) S3[rr][cc] = sI[bc][g];   // L_{I,k} final: stored after the publish
          }
      }
      __syncthreads();
      d4 acc[2][2];
      mfma_xyT_64(S0, diag ? S0 : S1, acc);      // P_I P_J^T
  #pragma unroll
      for (int x = 0; x < 2; ++x)
  #pragma unroll
        for (int y = 0; y < 2; ++y)
  #pragma unroll
          for (int g = 0; g < 4; ++g) own[x][y][g] -= acc[x][y][g];
      if (k == kmax) {
  #pragma unroll
        for (int x = 0; x < 2; ++x)
  #pragma unroll
          for (int y = 0; y < 2; ++y)
  #pragma unroll
            for (int g = 0; g < 4; ++g) own[x][y][g] = av[x][y][g] + own[x][y][g];
      }
      __syncthreads();                           // S0..S2 are restaged next
      if (stamp && k == kmax) WSTAMP(J, 3);
      ++k;
      staged = false;
      if (k <= kmax && (no_items || J - k < ov.far)) {
        stage_panels(k);
        staged = true;
      }
    }
    // publish the tile (lower part; pairs that start on or left of the
    // diagonal on a diagonal tile): through S0, as row-contiguous 16-B sc1 stores
  #pragma unroll
    for (int x = 0; x < 2; ++x)
  #pragma unroll
      for (int y = 0; y < 2; ++y)
  #pragma unroll
        for (int g = 0; g < 4; ++g) {
          int rr, cc;
          acc_pos(x, y, g, &rr, &cc);
          S0[rr][cc] = own[x][y][g];
        }
    __syncthreads();
    for (int e2 = ctid(); e2 < CB * CB / 2; e2 += 256) {
      const int i = (2 * e2) / CB, j = (2 * e2) % CB;
      const int ri = r0 + i, cj = c0 + j;
      if (ri < nrows && cj < n && (!diag || j <= i))   // n = 6 cameras: even, whole pairs
        st_sc1(rA, ((size_t)ri * ld + cj) * sizeof(double), make_double2(S0[i][j], S0[i][j + 1]));
    }
    publish(&tflag[I * T + J], a.epoch);
    if (stamp) WSTAMP(J, 4);
    if (ov.on && threadIdx.x < 64) OVT(2048 + blockIdx.x);
    // L_{I,J-1} (the last update of an off-diagonal tile: J == k + 1) to the
    // factor, after the publish: no in-kernel reader, and its drain would
    // otherwise sit in the barriers before the tile's hand-off
    if (!diag && kmax == J - 1) lds_to_global(S3, a.L, ld, r0, kmax * CB, mI, min(CB, n - kmax * CB));
    // the worker (J+1, J) also stores P_J = L_{J,J-1}, the critical
    // workgroup's panel product of step J (bitwise the same: the same tiles
    // through the same strip product; block row J has no rhs row here)
    if (I == J + 1) lds_to_global(S1, a.L, ld, c0, kmax * CB, CB, min(CB, n - kmax * CB));
    if (threadIdx.x == 0 && bad) atomicAdd(&a.scal[SL_CHOL_BAD], 1.0);
    if (threadIdx.x == 0 && spin) atomicAdd(&a.scal[SL_CHOL_SPIN], 1.0);
  }
  // ---------------- every workgroup: items (helpers: all of theirs), then
  // each wave's one failing draw of the launch
  if (ov.on) {
    __syncthreads();
    if (!drew_fail) ov_take(ov, ov_ctab, region, islot, a.A, ld, T, a.epoch);
    if (!worker && blockIdx.x != 0 && threadIdx.x < 64) OVT(1024 + blockIdx.x);
  }
}

// grid of the persistent factorisation: 1 critical + one worker per tile
int chol_persist_grid(int n) {
  const int T = (n + CB - 1) / CB, TR = (n + 1 + CB - 1) / CB;
  int w = 0;
  for (int j = 1; j < T; ++j) w += TR - (j == 1 ? 2 : j);
  return 1 + w;
}

// every workgroup of the grid resident at once (the dataflow spins)?
bool chol_persist_fits(int device, int n) {
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(k_chol_persist), 256, 0) !=
          hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
    return false;
  return chol_persist_grid(n) <= per_cu * cus;
}

int chol_persist_capacity(int device) {
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(k_chol_persist), 256, 0) !=
          hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
    return -1;
  return per_cu * cus;
}

// the overlapped form: one launch of plan.grid workgroups forms S (pairs,
// diagonal slices, fold at this step's radius) and factors it
void launch_chol_persist_ov(const DevProblem& P, const DevWork& W, OvPlan& plan, double radius, int epoch,
                            hipStream_t s, bool pass_only) {
  const int n = P.n, T = (n + CB - 1) / CB, TR = (n + 1 + CB - 1) / CB;
  PersistArgs a;
  a.A = W.S; a.L = W.Lf; a.Vbuf = W.Vbuf; a.scal = W.scal; a.flags = W.cflags;
  a.ld = P.ld; a.n = n; a.T = T; a.TR = TR;
  a.epoch = (unsigned)epoch;
  const char* e = getenv("BA_CHOL_SPIN_MAX");   // (read per launch: tests switch it)
  a.spin_max = e && atoi(e) > 0 ? (unsigned)atoi(e) : kPersistSpin;
  OvArgs& o = a.ov;
  o.on = 1;
  o.pass_only = pass_only ? 1 : 0;
  const char* we = getenv("BA_OV_WORKERS");
  o.worker_items = we ? atoi(we) : 0;
  const char* fe = getenv("BA_OV_FAR");
  o.far = fe && atoi(fe) > 0 ? atoi(fe) : kOvFar;
  o.P = P;
  o.blocks = W.blocks; o.pairs = W.pairs; o.Wc = W.W; o.scale_c = W.scale_c; o.u = W.u;
  o.Hcc = W.Hcc; o.gc = W.gc; o.diag_c = W.diag_c; o.radius = radius;
  o.cpart = W.cpart; o.G = W.cam_split;
  o.irec = plan.irec; o.item_col = plan.item_col; o.tgt = plan.tgt;
  o.cnt = plan.ctr;
  o.cam_cnt = plan.ctr + (size_t)TR * T;
  o.q = o.cam_cnt + P.nvc;
  o.pflag = o.q + 8;
  const unsigned pe = ++plan.launches;
  o.pe = pe;
  for (int x = 0; x < 9; ++x) o.ioff[x] = plan.ioff[x];
  for (int x = 0; x < 8; ++x) {
    const unsigned nwg = (unsigned)((plan.grid - x + 7) / 8);   // workgroups b = x mod 8
    const unsigned D = (unsigned)(plan.ioff[x + 1] - plan.ioff[x]) + 4u * nwg;   // tickets per launch
    o.qbase[x] = (pe - 1u) * D;
  }
  hipLaunchKernelGGL(k_chol_persist, dim3(plan.grid), dim3(256), 0, s, a);
}

void launch_chol_persist(double* A, double* L, int ld, int n, double* Vbuf, double* scal, unsigned* flags,
                         unsigned epoch, hipStream_t s) {
  PersistArgs a;
  a.A = A; a.L = L; a.Vbuf = Vbuf; a.scal = scal; a.flags = flags;
  a.ld = ld; a.n = n;
  a.T = (n + CB - 1) / CB;
  a.TR = (n + 1 + CB - 1) / CB;
  a.epoch = epoch;
  const char* e = getenv("BA_CHOL_SPIN_MAX");   // (read per launch: tests switch it)
  a.spin_max = e && atoi(e) > 0 ? (unsigned)atoi(e) : kPersistSpin;
  hipLaunchKernelGGL(k_chol_persist, dim3(chol_persist_grid(n)), dim3(256), 0, s, a);
}

}  // namespace bahip

// ba_pcg.hip — ITERATIVE_SCHUR on gfx950: preconditioned conjugate gradients
// on the implicit reduced camera system.
//
// Ceres semantics restated (iterative_schur_complement_solver.cc,
// implicit_schur_complement.cc, conjugate_gradients_solver.cc; the oracle's
// iterative_schur_solve is the CPU statement of the same algorithm):
//
//   (S x)_c = A_c x_c - sum_{o in c} W_o v_{p(o)},   v_p = sum_{o in p} W_o^T x_{c(o)},
//   A_c = s_c Hcc_c s_c + D_c^2
//
// with W_o = diag(s_c) Jc^T Jp diag(s_p) L_p^-T (6x3, the same per-observation
// blocks the DENSE_SCHUR path builds) — never forming S.  One matvec is two
// HBM passes over W: a point pass (observations contiguous per point) and a
// camera pass (observations gathered per camera, sliced over workgroups).
// Everything on the camera side (6 nvc entries: A x, preconditioner,
// dot products, the CG recurrences and Ceres' termination tests) is one
// 1024-thread workgroup up to 1024 cameras (one launch per CG iteration,
// fixed-order reductions without grid barriers) and three thread-per-camera
// grid kernels beyond.  Multi-GPU: each rank
// holds a point shard; the camera slices of every matvec are summed with one
// RCCL all-reduce of 6 nvc x slices doubles (ba_solver.hip); all other CG
// state is replicated and evolves identically on every rank.
//
// All reductions are fixed-order: results are bitwise reproducible.
#include "ba_kernels.h"
#include "ba_device.h"
#include "ba_reduce.h"

namespace bahip {

// k_pcg_update (one workgroup, one thread per camera) up to this many
// cameras, the grid kernels past
// it: at 1000 cameras the one workgroup's strided Adiag / Minv reads go
// through one CU (~35 us per working launch); C4 3893 -> 3898 M-obs/s with the
// grid kernels (profiles/r05_v10_pcg_update_form_ab.txt)
constexpr int kPcgOneWg = 256;

// LDS hand-off between the lanes of one wave (in-order DS operations)
__device__ inline void wave_lds_sync_pcg() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

__device__ inline bool zero_or_inf(double x) { return x == 0.0 || isinf(x); }   // ceres IsZeroOrInfinity

// lower-triangle index of (a, b), a >= b
__device__ inline int tri(int a, int b) { return a * (a + 1) / 2 + b; }

// y = A x for a symmetric 6x6 block stored as its lower 21 entries
__device__ inline void sym6_mul(const double* __restrict__ A, const double (&x)[6], double (&y)[6]) {
#pragma unroll
  for (int a = 0; a < 6; ++a) {
    double v = 0.0;
#pragma unroll
    for (int b = 0; b < 6; ++b) v += A[a >= b ? tri(a, b) : tri(b, a)] * x[b];
    y[a] = v;
  }
}

// Inverse of an SPD 6x6 block (lower 21) by LLT + two triangular solves
// against I (Eigen selfadjointView().llt().solve(Identity), as Ceres'
// BlockRandomAccessDiagonalMatrix::Invert).  Returns false if not PD.
__device__ inline bool spd6_inverse(const double (&M)[21], double* __restrict__ out /*36, row-major*/) {
  double L[21];
  bool ok = true;
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    double d = M[tri(j, j)];
#pragma unroll
    for (int t = 0; t < j; ++t) d -= L[tri(j, t)] * L[tri(j, t)];
    ok = ok && d > 0.0;
    d = sqrt(d);
    L[tri(j, j)] = d;
#pragma unroll
    for (int i = j + 1; i < 6; ++i) {
      double v = M[tri(i, j)];
#pragma unroll
      for (int t = 0; t < j; ++t) v -= L[tri(i, t)] * L[tri(j, t)];
      L[tri(i, j)] = v / d;
    }
  }
#pragma unroll
  for (int col = 0; col < 6; ++col) {
    double z[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      double v = i == col ? 1.0 : 0.0;
#pragma unroll
      for (int t = 0; t < i; ++t) v -= L[tri(i, t)] * z[t];
      z[i] = v / L[tri(i, i)];
    }
#pragma unroll
    for (int i = 5; i >= 0; --i) {
      double v = z[i];
#pragma unroll
      for (int t = i + 1; t < 6; ++t) v -= L[tri(t, i)] * z[t];
      z[i] = v / L[tri(i, i)];
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) out[i * 6 + col] = z[i];
  }
  return ok;
}

__device__ inline void mat6_mul(const double* __restrict__ M, const double (&x)[6], double (&y)[6]) {
#pragma unroll
  for (int a = 0; a < 6; ++a) {
    double v = 0.0;
#pragma unroll
    for (int b = 0; b < 6; ++b) v += M[a * 6 + b] * x[b];
    y[a] = v;
  }
}

__device__ inline void load6(const double* __restrict__ p, double (&v)[6]) {
#pragma unroll
  for (int a = 0; a < 6; ++a) v[a] = p[a];
}
__device__ inline void store6(double* __restrict__ p, const double (&v)[6]) {
#pragma unroll
  for (int a = 0; a < 6; ++a) p[a] = v[a];
}

__device__ inline void pcg_stop(double* st, double* scal, int term, int iters) {
  if (threadIdx.x == 0) {
    st[PS_DONE] = 1.0;
    st[PS_TERM] = term;
    st[PS_ITER] = iters;
    if (term == PCG_FAILURE) scal[SL_CHOL_BAD] = 1.0;   // linear solver failure -> invalid step
  }
}

// ---------------------------------------------------------------------------
// Schur-Jacobi cross terms of a point observed twice by one camera:
// Sd_c -= W_a W_b^T + W_b W_a^T (lower), one thread per camera (fixed order)
// ---------------------------------------------------------------------------
template <typename WT>
__global__ __launch_bounds__(256) void k_pcg_dup(DevProblem P, const int* __restrict__ dup_off,
                                                 const int2* __restrict__ dup_pairs, const WT* __restrict__ Wm,
                                                 double* __restrict__ Sd) {
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= P.nvc) return;
  for (int i = dup_off[v]; i < dup_off[v + 1]; ++i) {
    const int2 pr = dup_pairs[i];
    double wa[18], wb[18];
    load_w18(Wm, (size_t)pr.x, wa);
    load_w18(Wm, (size_t)pr.y, wb);
    for (int a = 0; a < 6; ++a)
      for (int b = 0; b <= a; ++b) {
        double s = 0.0;
        for (int t = 0; t < 3; ++t) s += wa[a * 3 + t] * wb[b * 3 + t] + wb[a * 3 + t] * wa[b * 3 + t];
        Sd[(size_t)v * 27 + tri(a, b)] -= s;
      }
  }
}

// Sum of nb per-block partials, in a fixed order, returned to every thread
// of the workgroup (wave 0 folds lane-strided, then the wave tree).
__device__ inline double fold_part(const double* __restrict__ pp, int nb, double* lds1) {
  if (threadIdx.x < 64) {
    double v = 0.0;
    for (int i = threadIdx.x; i < nb; i += 64) v += pp[i];
    v = wave_sum(v);
    if (threadIdx.x == 0) lds1[0] = v;
  }
  __syncthreads();
  const double t = lds1[0];
  __syncthreads();
  return t;
}

// ---------------------------------------------------------------------------
// setup (thread per camera): A_c = s Hcc s + D^2, preconditioner block
// M_c = A_c (JACOBI) or A_c + Sd_c (SCHUR_JACOBI) inverted, rhs
// b_c = Sd_c[rhs] + s g_c; x = 0, r = b, z = M r, p = z; per-block partials
// of |b|^2, r.z and non-PD blocks.  k_pcg_setup_fin then applies ceres'
// norm_b == 0 exit and the first iteration's rho test.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_pcg_setup(DevProblem P, const double* __restrict__ Sd,
                                                   const double* __restrict__ Hcc, const double* __restrict__ gc,
                                                   const double* __restrict__ scale_c,
                                                   const double* __restrict__ diag_c, double radius, int schur_jacobi,
                                                   double* __restrict__ Adiag, double* __restrict__ Minv,
                                                   double* __restrict__ b, double* __restrict__ x,
                                                   double* __restrict__ r, double* __restrict__ z,
                                                   double* __restrict__ p, double* __restrict__ ppart) {
  __shared__ double lds[3 * 16];
  double acc[3] = {0.0, 0.0, 0.0};   // |b|^2, r.z, bad blocks
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v < P.nvc) {
    double s[6], D2[6];
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      s[a] = scale_c[(size_t)v * 6 + a];
      const double D = sqrt(diag_c[(size_t)v * 6 + a] / radius);
      D2[a] = D * D;
    }
    double A[21], M[21];
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
      for (int c = 0; c <= a; ++c) {
        const int k = tri(a, c);
        double h = Hcc[(size_t)v * 21 + k] * s[a] * s[c];   // same arithmetic as k_cam_add_diag
        if (a == c) h += D2[a];
        A[k] = h;
        M[k] = schur_jacobi ? Sd[(size_t)v * 27 + k] + h : h;
      }
#pragma unroll
    for (int k = 0; k < 21; ++k) Adiag[(size_t)v * 21 + k] = A[k];
    double* mi = Minv + (size_t)v * 36;
    if (!spd6_inverse(M, mi)) acc[2] += 1.0;
    double bv[6], zv[6];
#pragma unroll
    for (int a = 0; a < 6; ++a) bv[a] = Sd[(size_t)v * 27 + 21 + a] + gc[(size_t)v * 6 + a] * s[a];
    mat6_mul(mi, bv, zv);
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      const size_t i = (size_t)v * 6 + a;
      b[i] = bv[a]; r[i] = bv[a]; x[i] = 0.0; z[i] = zv[a]; p[i] = zv[a];
      acc[0] += bv[a] * bv[a];
      acc[1] += bv[a] * zv[a];
    }
  }
  double tot[3];
  block_sum<3>(acc, lds, tot);
  if (threadIdx.x == 0)
#pragma unroll
    for (int k = 0; k < 3; ++k) ppart[k * kMaxBlocks + blockIdx.x] = tot[k];
}

__global__ __launch_bounds__(64) void k_pcg_setup_fin(const double* __restrict__ ppart, int nb,
                                                      double* __restrict__ scal) {
  __shared__ double lds[1];
  double* st = scal + kNumSlots;
  const double bb = fold_part(ppart, nb, lds);
  const double rz = fold_part(ppart + kMaxBlocks, nb, lds);
  const double bad = fold_part(ppart + 2 * kMaxBlocks, nb, lds);
  if (threadIdx.x == 0) {
    st[PS_RHO] = st[PS_RHO1] = 1.0; st[PS_Q0] = st[PS_Q01] = -0.0; st[PS_ALPHA] = 0.0; st[PS_NORM_B] = sqrt(bb);
    st[PS_ITER] = 0.0; st[PS_DONE] = 0.0; st[PS_TERM] = PCG_NO_CONVERGENCE;
    st[PS_AAPP] = 0.0; st[PS_AAPP_IT] = 0.0;
    scal[SL_CHOL_BAD] = 0.0;   // linear-solver failure flag of this step
    scal[SL_CHOL_SPIN] = 0.0;  // (a dense step's spin on this context must not fail this one)
  }
  if (sqrt(bb) == 0.0) { pcg_stop(st, scal, PCG_SUCCESS, 0); return; }   // x = 0
  // iteration 1 starts: rho = r.z (an indefinite / singular preconditioner
  // block yields a non-finite rho: stop as a failure, the step is invalid
  // either way)
  if (zero_or_inf(rz) || isnan(rz) || bad != 0.0) { pcg_stop(st, scal, PCG_FAILURE, 1); return; }
  if (threadIdx.x == 0) st[PS_RHO] = st[PS_RHO1] = rz;
}

// ---------------------------------------------------------------------------
// matvec, point pass: v_p = sum_{o in p} W_o^T x_{c(o)}  (thread per point)
// ---------------------------------------------------------------------------
template <typename WT>
__global__ __launch_bounds__(256) void k_pcg_point(DevProblem P, const WT* __restrict__ Wm,
                                                   const double* __restrict__ xv, double* __restrict__ vpt,
                                                   const double* __restrict__ st) {
  if (st[PS_DONE] != 0.0) return;
  // kPtLanes lanes per point (point_wtx); fixed cameras and fixed points
  // carry W_o = 0 (k_obs_w): no branches
  const int gl = threadIdx.x & (kPtLanes - 1), gpb = blockDim.x / kPtLanes;
  for (int p = blockIdx.x * gpb + threadIdx.x / kPtLanes; p < P.np; p += gridDim.x * gpb) {
    double w[3];
    point_wtx<true>(Wm, P.obs_vc, xv, P.pt_off[p], P.pt_off[p + 1], gl, w);
    if (gl < 3) vpt[3 * (size_t)p + gl] = gl == 0 ? w[0] : (gl == 1 ? w[1] : w[2]);
  }
}

// ---------------------------------------------------------------------------
// matvec, camera pass: slice g of camera v: sum_{o in slice} W_o v_{p(o)}
// ---------------------------------------------------------------------------
template <typename WT>
__global__ __launch_bounds__(256) void k_pcg_cam(DevProblem P, const WT* __restrict__ Wm,
                                                 const double* __restrict__ vpt, double* __restrict__ tpart,
                                                 const double* __restrict__ st) {
  if (st[PS_DONE] != 0.0) return;
  __shared__ double lds[6 * 16];
  const int v = blockIdx.x, g = blockIdx.y, G = gridDim.y;
  const int a0 = P.cam_off[v], a1 = P.cam_off[v + 1];
  const int len = (a1 - a0 + G - 1) / G;
  const int i0 = min(a1, a0 + g * len), i1 = min(a1, i0 + len);
  double acc[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    const int2 op = P.cam_op[i];   // fixed points: W_o = 0, v_p = 0
    const int o = op.x, p = op.y;
    double wv[18];
    load_w18(Wm, (size_t)o, wv);
    const double u0 = vpt[3 * (size_t)p], u1 = vpt[3 * (size_t)p + 1], u2 = vpt[3 * (size_t)p + 2];
#pragma unroll
    for (int a = 0; a < 6; ++a) acc[a] += wv[a * 3] * u0 + wv[a * 3 + 1] * u1 + wv[a * 3 + 2] * u2;
  }
  double tot[6];
  block_sum<6>(acc, lds, tot);
  if (threadIdx.x == 0) {
    double* dst = tpart + ((size_t)g * P.nvc + v) * 6;
#pragma unroll
    for (int a = 0; a < 6; ++a) dst[a] = tot[a];
  }
}

// Matvec with per-observation products (point-major, coalesced): the point
// pass also forms t_o = W_o v_p for the point's observations (the group has
// just read those W records: the re-read hits the caches) and stores them
// contiguously [no][6]; the camera pass then gathers 48-B t_o instead of the
// 144-B W_o and the point's v_p.
template <typename WT>
__global__ __launch_bounds__(256) void k_pcg_point_t(DevProblem P, const WT* __restrict__ Wm,
                                                     const double* __restrict__ xv, double* __restrict__ tobs,
                                                     const double* __restrict__ st) {
  if (st[PS_DONE] != 0.0) return;
  const int gl = threadIdx.x & (kPtLanes - 1), gpb = blockDim.x / kPtLanes;
  for (int p = blockIdx.x * gpb + threadIdx.x / kPtLanes; p < P.np; p += gridDim.x * gpb) {
    const int o0 = P.pt_off[p], o1 = P.pt_off[p + 1];
    double w[3];
    point_wtx<true>(Wm, P.obs_vc, xv, o0, o1, gl, w);
    for (int o = o0 + gl; o < o1; o += kPtLanes) {
      double wv[18];
      load_w18(Wm, (size_t)o, wv);
      double2* d = reinterpret_cast<double2*>(tobs + 6 * (size_t)o);
#pragma unroll
      for (int a = 0; a < 6; a += 2)
        d[a / 2] = make_double2(wv[a * 3] * w[0] + wv[a * 3 + 1] * w[1] + wv[a * 3 + 2] * w[2],
                                wv[a * 3 + 3] * w[0] + wv[a * 3 + 4] * w[1] + wv[a * 3 + 5] * w[2]);
    }
  }
}
__global__ __launch_bounds__(256) void k_pcg_cam_t(DevProblem P, const double* __restrict__ tobs,
                                                   double* __restrict__ tpart, const double* __restrict__ st) {
  if (st[PS_DONE] != 0.0) return;
  __shared__ double lds[6 * 16];
  const int v = blockIdx.x, g = blockIdx.y, G = gridDim.y;
  const int a0 = P.cam_off[v], a1 = P.cam_off[v + 1];
  const int len = (a1 - a0 + G - 1) / G;
  const int i0 = min(a1, a0 + g * len), i1 = min(a1, i0 + len);
  double acc[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    const double2* t = reinterpret_cast<const double2*>(tobs + 6 * (size_t)P.cam_op[i].x);
#pragma unroll
    for (int k = 0; k < 3; ++k) { const double2 x = t[k]; acc[2 * k] += x.x; acc[2 * k + 1] += x.y; }
  }
  double tot[6];
  block_sum<6>(acc, lds, tot);
  if (threadIdx.x == 0) {
    double* dst = tpart + ((size_t)g * P.nvc + v) * 6;
#pragma unroll
    for (int a = 0; a < 6; ++a) dst[a] = tot[a];
  }
}

// k_pcg_cam_t with the 48-B products gathered into LDS by LDS-DMA: a round of
// 64 observations is 192 16-B pieces, three wave-instructions whose lane l
// fetches piece (l + 64 k) mod 3 of record (l + 64 k) / 3, so the records
// land contiguously (record q at 48 q B) and an instruction touches ~21
// records instead of 64; each lane then reads its record with three
// conflict-free ds_read_b128 (stride 12 dwords).  Thread t still sums the
// observations i0 + t + 256 j in order: bitwise k_pcg_cam_t.
__device__ __forceinline__ void glds16p(const double* src, double* lds_dst) {
  __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)lds_dst, 16, 0, 0);
}
__global__ __launch_bounds__(256) void k_pcg_cam_td(DevProblem P, const double* __restrict__ tobs,
                                                    double* __restrict__ tpart, const double* __restrict__ st) {
  if (st[PS_DONE] != 0.0) return;
  __shared__ double lds[6 * 16];
  __shared__ __attribute__((aligned(16))) double tb[4][64 * 6];
  const int v = blockIdx.x, g = blockIdx.y, G = gridDim.y;
  const int a0 = P.cam_off[v], a1 = P.cam_off[v + 1];
  const int len = (a1 - a0 + G - 1) / G;
  const int i0 = min(a1, a0 + g * len), i1 = min(a1, i0 + len);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double* buf = tb[w];
  auto issue = [&](int o) {   // o: this lane's observation (any valid index when unused)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int e = lane + 64 * k, q = e / 3, pc = e - 3 * q;
      const int oq = __shfl(o, q);
      glds16p(tobs + 6 * (size_t)oq + 2 * pc, buf + 128 * k);
    }
  };
  double acc[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  // rounds of this wave: observations i0 + 64 w + lane + 256 r
  const int first = i0 + 64 * w;
  const int nr = first < i1 ? (i1 - first + 255) / 256 : 0;   // (uniform per wave)
  int i = first + lane;
  int on = i < i1 ? P.cam_op[i].x : 0;
  if (nr > 0) issue(on);
  on = i + 256 < i1 ? P.cam_op[i + 256].x : 0;
  for (int r = 0; r < nr; ++r, i += 256) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this round's DMA has landed
    const double2* t = reinterpret_cast<const double2*>(buf + 6 * lane);
    const double2 x0 = t[0], x1 = t[1], x2 = t[2];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // read out before the refill
    if (r + 1 < nr) {
      issue(on);
      on = i + 512 < i1 ? P.cam_op[i + 512].x : 0;
    }
    if (i < i1) {
      acc[0] += x0.x; acc[1] += x0.y;
      acc[2] += x1.x; acc[3] += x1.y;
      acc[4] += x2.x; acc[5] += x2.y;
    }
  }
  double tot[6];
  block_sum<6>(acc, lds, tot);
  if (threadIdx.x == 0) {
    double* dst = tpart + ((size_t)g * P.nvc + v) * 6;
#pragma unroll
    for (int a = 0; a < 6; ++a) dst[a] = tot[a];
  }
}

// Point pass over point-aligned chunks of <= 64 observations, one wave per
// chunk (ensure_pcg builds the chunk list; points with more than 64
// observations keep k_pcg_point / k_pcg_point_t).  The chunk's W records
// arrive as contiguous 8-B-per-lane wave loads (512 B per instruction)
// through the wave's LDS slot; each lane then forms W_o^T x_c for its own
// observation from LDS, and a segmented inclusive scan over the lanes (a
// fixed order for a given layout) sums each point's run, whose last lane
// stores v_p.  TOUT: every lane then takes its point's v_p back (shuffle
// from the run's last lane) and forms t_o = W_o v_p, stored as contiguous
// wave stores.  (k_pcg_point_t's value-pair loop issued ~4 loads per 8-16 B
// of W and re-read every record for t_o: 3.4 TB/s at C4.)
// PC: the 16-value rank-2 records of k_obs_w_rc<.., PC> (W_o = c^T Z: c's
// scaled rotation columns, its four nonzero translation entries, Z):
// W_o^T x = Z^T (c x), W_o v = c^T (Z v).  A record is 8 units (8 units of
// 16 B fp64, of 8 B fp32): at that even stride the per-lane record reads
// would conflict, so the units of record r sit XOR-swizzled in the slot
// (unit k at k ^ ((r >> SH) & 7), SH = 1 fp64 / 2 fp32: the records of one
// LDS row pass then cover distinct banks).
template <typename WT, bool TOUT, bool PC = false>
__global__ __launch_bounds__(256) void k_pcg_point_seg(DevProblem P, const int2* __restrict__ chunks, int nchunks,
                                                       const WT* __restrict__ Wm, const double* __restrict__ xv,
                                                       double* __restrict__ vpt, double* __restrict__ tobs,
                                                       const double* __restrict__ st) {
  static_assert(!PC || TOUT, "rank-2 records: the products");
  if (st[PS_DONE] != 0.0) return;
  constexpr int REC = PC ? 16 : 18;
  // fp64: 16-B units (a record is 9, 16-B aligned; the per-lane 144-B record
  // reads from LDS are ds_read_b128 at 9 slots' stride: every 16-lane group
  // hits 16 distinct slots).  fp32 (72-B records, 8-B aligned): 8-B units
  using U = typename std::conditional<sizeof(WT) == 8, uint4, unsigned long long>::type;
  constexpr int UN = REC * (int)sizeof(WT) / (int)sizeof(U);   // units per record: 9 (PC: 8)
  constexpr int SH = sizeof(WT) == 8 ? 1 : 2;
  // the slot position of unit e of the chunk (identity unless PC)
  auto spos = [](int e) { return PC ? (e & ~7) | ((e & 7) ^ ((e >> (3 + SH)) & 7)) : e; };
  __shared__ __attribute__((aligned(16))) U stage[4][64 * UN];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // the products leave through the wave's own slot: its records are in
  // registers by then (LDS operations of a wave complete in order), so the
  // slot is free, and without a second array 4 (fp64 18-value: 4, was 3)
  // workgroups fit a CU's LDS
  static_assert(64 * UN * sizeof(U) >= 64 * 6 * sizeof(double), "products fit the slot");
  double* tstw = reinterpret_cast<double*>(&stage[w][0]);
  // fp32: the next chunk's W units are loaded one chunk ahead, into
  // registers, so that their latency runs under this chunk's arithmetic and
  // scan (C5 shard 4.20 -> 4.09 ms per LM iteration).  fp64: the 36 VGPRs
  // this needs cost occupancy (C4 seg pass 300 -> 547 us): loaded in place
  constexpr bool PF = sizeof(WT) == 4;
  const int cstride = gridDim.x * 4;
  auto fetch = [&](int c, U (&u)[UN], int2& crr) {
    crr = chunks[c];
    const U* src = reinterpret_cast<const U*>(Wm + (size_t)crr.x * REC);
    const int nu = (crr.y - crr.x) * UN;
#pragma unroll
    for (int k = 0; k < UN; ++k) {
      const int e = k * 64 + lane;
      if (e < nu) u[k] = src[e];
    }
  };
  int ch = blockIdx.x * 4 + w;
  U nxt[PF ? UN : 1];
  int2 ncr = make_int2(0, 0);
  if constexpr (PF) {
    if (ch < nchunks) fetch(ch, nxt, ncr);
  }
  for (; ch < nchunks; ch += cstride) {   // (uniform per wave)
    const int2 cr = PF ? ncr : chunks[ch];
    const int o0 = cr.x, n = cr.y - cr.x;
    const int nu = n * UN;
    if constexpr (PF) {
#pragma unroll
      for (int k = 0; k < UN; ++k) {
        const int e = k * 64 + lane;
        if (e < nu) stage[w][spos(e)] = nxt[k];
      }
      if (ch + cstride < nchunks) fetch(ch + cstride, nxt, ncr);
    } else {
      const U* src = reinterpret_cast<const U*>(Wm + (size_t)o0 * REC);
#pragma unroll
      for (int k = 0; k < UN; ++k) {
        const int e = k * 64 + lane;
        if (e < nu) stage[w][spos(e)] = src[e];
      }
    }
    const bool live = lane < n;
    const int o = o0 + min(lane, n - 1);
    const int vc = P.obs_vc[o];
    const int pt = live ? P.obs_pt[o] : -1;
    const double2* xc = reinterpret_cast<const double2*>(xv + 6 * (size_t)max(vc, 0));
    const double2 x01 = xc[0], x23 = xc[1], x45 = xc[2];
    const double x[6] = {x01.x, x01.y, x23.x, x23.y, x45.x, x45.y};
    wave_lds_sync_pcg();
    double wr[REC];
    {
      const int rl = min(lane, n - 1);
      const U* ru = &stage[w][0] + (size_t)rl * UN;
      U ur[UN];
#pragma unroll
      for (int k = 0; k < UN; ++k) ur[k] = ru[PC ? k ^ ((rl >> SH) & 7) : k];
      const WT* r = reinterpret_cast<const WT*>(ur);
#pragma unroll
      for (int k = 0; k < REC; ++k) wr[k] = (double)r[k];
    }
    double v[3];
    if constexpr (PC) {
      // y = c x (c0[4] = c1[3] = 0), v = Z^T y
      double wp[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) wp[k] = wr[k];
      pc_v(wp, x, live, v);
    } else {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        double a = 0.0;
#pragma unroll
        for (int b = 0; b < 6; ++b) a += wr[b * 3 + k] * x[b];
        v[k] = live ? a : 0.0;
      }
    }
    // segmented inclusive scan: runs of equal pt (the chunk holds whole points)
    const int ptp = __shfl_up(pt, 1, 64);
    const bool head = lane == 0 || pt != ptp;
    const unsigned long long heads = __ballot(head);
    const unsigned long long upto = lane == 63 ? ~0ull : ((1ull << (lane + 1)) - 1);
    const int s0 = 63 - __clzll(heads & upto);   // this lane's run head
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      double y[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) y[k] = __shfl_up(v[k], off, 64);
      if (lane - off >= s0) {
#pragma unroll
        for (int k = 0; k < 3; ++k) v[k] += y[k];
      }
    }
    const unsigned long long after = heads & ~upto;   // heads past this lane
    const int last = after ? __ffsll((long long)after) - 2 : n - 1;   // this run's last lane
    if (live && lane == last) {
#pragma unroll
      for (int k = 0; k < 3; ++k) vpt[3 * (size_t)pt + k] = v[k];
    }
    if constexpr (TOUT) {
      double vp[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) vp[k] = __shfl(v[k], last, 64);
      {   // (three 16-B LDS stores at 3 slots' stride: conflict-free)
        double tv[6];
        if constexpr (PC) {   // q = Z v_p, t_o = c^T q
          double wp[16];
#pragma unroll
          for (int k = 0; k < 16; ++k) wp[k] = wr[k];
          pc_t(wp, vp, tv);
        } else {
#pragma unroll
          for (int a = 0; a < 6; ++a) tv[a] = wr[a * 3] * vp[0] + wr[a * 3 + 1] * vp[1] + wr[a * 3 + 2] * vp[2];
        }
        double2* td = reinterpret_cast<double2*>(&tstw[lane * 6]);
#pragma unroll
        for (int a = 0; a < 3; ++a) td[a] = make_double2(tv[2 * a], tv[2 * a + 1]);
      }
      wave_lds_sync_pcg();
      double2* dst = reinterpret_cast<double2*>(tobs + 6 * (size_t)o0);
      const double2* tsrc = reinterpret_cast<const double2*>(&tstw[0]);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int e = k * 64 + lane;
        if (e < 3 * n) dst[e] = tsrc[e];
      }
    }
    wave_lds_sync_pcg();   // (the slots are rewritten by the next chunk)
  }
}

// Sum of the G matvec slices of camera v entry a, in slice order (the same
// order in k_pcg_tfold, so the exchange path, which folds the slices before
// its all-reduce, rounds exactly like the single-rank path)
__device__ inline double slice_sum(const double* __restrict__ tpart, int G, int nvc, int v, int a) {
  double t = tpart[(size_t)v * 6 + a];
  for (int g = 1; g < G; ++g) t += tpart[((size_t)g * nvc + v) * 6 + a];
  return t;
}

// S y for camera v from its A block and the matvec slices of y
__device__ inline void schur_row(const double* __restrict__ Adiag, const double* __restrict__ tpart, int G, int nvc,
                                 int v, const double (&y)[6], double (&out)[6]) {
  sym6_mul(Adiag + (size_t)v * 21, y, out);
#pragma unroll
  for (int a = 0; a < 6; ++a) out[a] -= slice_sum(tpart, G, nvc, v, a);
}

// Exchange path: fold the G slices into slice 0 before the all-reduce, so
// every CG iteration sends one 6 nvc vector (not G of them).
__global__ __launch_bounds__(256) void k_pcg_tfold(int nvc, int G, double* __restrict__ tpart,
                                                   const double* __restrict__ st) {
  if (st[PS_DONE] != 0.0) return;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= 6 * nvc) return;
  const int v = e / 6, a = e - 6 * v;
  const double t = slice_sum(tpart, G, nvc, v, a);
  tpart[e] = t;
}

// ---------------------------------------------------------------------------
// camera-side CG iteration (one workgroup), ceres ConjugateGradientsSolver:
//   q = S p; pq = p.q (<= 0 or inf: NO_CONVERGENCE, stop); alpha = rho / pq
//   (inf: FAILURE); x += alpha p; r -= alpha q  (every 10th: r = b - S x);
//   Q1 = -x.(b + r); zeta = it (Q1 - Q0) / Q1 < q_tol: SUCCESS; it >= max:
//   NO_CONVERGENCE; then iteration it+1 begins: z = M r, rho' = r.z,
//   beta = rho' / rho (zero or inf: FAILURE), p = z + beta p.
// ---------------------------------------------------------------------------
// nvc <= kPcgOneWg: one camera per thread, its vectors held in registers
// across the phases (every load issued at the start, each vector stored once;
// the per-phase re-reads of the loop form cost a dependent L2 round trip per
// phase: C4 shard 15.4 us per launch).  The same operations per camera in the
// same order and the same workgroup sums: bitwise the loop form.
__global__ __launch_bounds__(kPcgOneWg) void k_pcg_update(DevProblem P, int mode, int it, PcgOpts o, int G,
                                                            const double* __restrict__ Adiag,
                                                            const double* __restrict__ Minv,
                                                            const double* __restrict__ b, double* __restrict__ x,
                                                            double* __restrict__ r, double* __restrict__ z,
                                                            double* __restrict__ p, double* __restrict__ q,
                                                            const double* __restrict__ tpart,
                                                            double* __restrict__ scal) {
  __shared__ double lds[2 * 16];
  double* st = scal + kNumSlots;
  if (st[PS_DONE] != 0.0) return;
  const int nvc = P.nvc;
  const int v = threadIdx.x;
  const bool on = v < nvc;
  const size_t o6 = 6 * (size_t)(on ? v : 0);
  double pv[6] = {0, 0, 0, 0, 0, 0}, xv[6] = {0, 0, 0, 0, 0, 0};
  double rv[6] = {0, 0, 0, 0, 0, 0}, bv[6] = {0, 0, 0, 0, 0, 0};
  if (on) {
    load6(p + o6, pv);
    load6(x + o6, xv);
    load6(b + o6, bv);
    if (mode != 2) load6(r + o6, rv);
  }
  double alpha;
  if (mode != 2) {
    double acc[1] = {0.0};
    double qv[6] = {0, 0, 0, 0, 0, 0};
    if (on) {
      schur_row(Adiag, tpart, G, nvc, v, pv, qv);
      store6(q + o6, qv);
#pragma unroll
      for (int a = 0; a < 6; ++a) acc[0] += pv[a] * qv[a];
    }
    block_allsum<1>(acc, lds);
    const double pq = acc[0], rho = st[PS_RHO];
    if (pq <= 0.0 || isinf(pq)) { pcg_stop(st, scal, PCG_NO_CONVERGENCE, it); return; }
    alpha = rho / pq;
    if (isinf(alpha) || isnan(alpha)) { pcg_stop(st, scal, PCG_FAILURE, it); return; }
    if (on) {
#pragma unroll
      for (int a = 0; a < 6; ++a) xv[a] = xv[a] + alpha * pv[a];
      store6(x + o6, xv);
    }
    if (threadIdx.x == 0) { st[PS_AAPP] = alpha; st[PS_AAPP_IT] = it; }   // x moved (k_pcg_vacc)
    if (mode == 1) {
      if (threadIdx.x == 0) st[PS_ALPHA] = alpha;
      return;
    }
#pragma unroll
    for (int a = 0; a < 6; ++a) rv[a] = rv[a] - alpha * qv[a];
  } else {
    alpha = st[PS_ALPHA];
    if (on) {
      double sx[6];
      schur_row(Adiag, tpart, G, nvc, v, xv, sx);
#pragma unroll
      for (int a = 0; a < 6; ++a) rv[a] = bv[a] - sx[a];
    }
  }
  double acc[1] = {0.0};
  if (on) {
    store6(r + o6, rv);
#pragma unroll
    for (int a = 0; a < 6; ++a) acc[0] += xv[a] * (bv[a] + rv[a]);
  }
  block_allsum<1>(acc, lds);
  const double Q1 = -1.0 * acc[0];
  const double Q0 = st[PS_Q0];
  const double zeta = it * (Q1 - Q0) / Q1;
  if (zeta < o.q_tolerance && it >= o.min_iter) { pcg_stop(st, scal, PCG_SUCCESS, it); return; }
  if (it >= o.max_iter) { pcg_stop(st, scal, PCG_NO_CONVERGENCE, it); return; }
  // iteration it + 1
  double racc[1] = {0.0};
  double zv[6] = {0, 0, 0, 0, 0, 0};
  if (on) {
    mat6_mul(Minv + (size_t)v * 36, rv, zv);
    store6(z + o6, zv);
#pragma unroll
    for (int a = 0; a < 6; ++a) racc[0] += rv[a] * zv[a];
  }
  block_allsum<1>(racc, lds);
  const double rho_new = racc[0], rho = st[PS_RHO];
  if (zero_or_inf(rho_new) || isnan(rho_new)) { pcg_stop(st, scal, PCG_FAILURE, it + 1); return; }
  const double beta = rho_new / rho;
  if (zero_or_inf(beta)) { pcg_stop(st, scal, PCG_FAILURE, it + 1); return; }
  if (on) {
#pragma unroll
    for (int a = 0; a < 6; ++a) pv[a] = zv[a] + beta * pv[a];
    store6(p + o6, pv);
  }
  if (threadIdx.x == 0) {
    st[PS_RHO] = rho_new;
    st[PS_Q0] = Q1;
    st[PS_ITER] = it;
  }
}

// ---------------------------------------------------------------------------
// The same CG iteration for larger camera counts (nvc > kPcgOneWg): three
// grid kernels, thread per camera; each block folds the previous kernel's
// per-block partials itself (fixed order: every block reaches the same
// decisions), block 0 records the state.
//   k_pcg_q:  q = S p, partials p.q                              (modes 0, 1)
//   k_pcg_xr: alpha, x += alpha p [mode 1 stops here], r update,
//             z = M r, partials x.(b + r), r.z                  (modes 0, 1, 2)
//   k_pcg_p:  termination tests, rho', beta, p = z + beta p
// ---------------------------------------------------------------------------
// rho and Q0 of CG iteration it (grid kernels): parity slots
__device__ inline int rho_slot(int it) { return (it & 1) ? PS_RHO1 : PS_RHO; }
__device__ inline int q0_slot(int it) { return (it & 1) ? PS_Q01 : PS_Q0; }

__global__ __launch_bounds__(256) void k_pcg_q(DevProblem P, int G, const double* __restrict__ Adiag,
                                               const double* __restrict__ p, double* __restrict__ q,
                                               const double* __restrict__ tpart, double* __restrict__ ppart,
                                               const double* __restrict__ st) {
  if (st[PS_DONE] != 0.0) return;
  __shared__ double lds[16];
  double acc[1] = {0.0};
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v < P.nvc) {
    double pv[6], qv[6];
    load6(p + 6 * (size_t)v, pv);
    schur_row(Adiag, tpart, G, P.nvc, v, pv, qv);
    store6(q + 6 * (size_t)v, qv);
#pragma unroll
    for (int a = 0; a < 6; ++a) acc[0] += pv[a] * qv[a];
  }
  double tot[1];
  block_sum<1>(acc, lds, tot);
  if (threadIdx.x == 0) ppart[blockIdx.x] = tot[0];
}

__global__ __launch_bounds__(256) void k_pcg_xr(DevProblem P, int mode, int it, int G,
                                                const double* __restrict__ Adiag, const double* __restrict__ Minv,
                                                const double* __restrict__ b, double* __restrict__ x,
                                                double* __restrict__ r, double* __restrict__ z,
                                                const double* __restrict__ p, const double* __restrict__ q,
                                                const double* __restrict__ tpart, double* __restrict__ ppart,
                                                double* __restrict__ scal) {
  double* st = scal + kNumSlots;
  if (st[PS_DONE] != 0.0) return;
  __shared__ double lds[2 * 16];
  const int nb = gridDim.x;
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = v < P.nvc;
  double alpha;
  if (mode != 2) {
    const double pq = fold_part(ppart, nb, lds), rho = st[rho_slot(it)];
    if (pq <= 0.0 || isinf(pq)) { if (blockIdx.x == 0) pcg_stop(st, scal, PCG_NO_CONVERGENCE, it); return; }
    alpha = rho / pq;
    if (isinf(alpha) || isnan(alpha)) { if (blockIdx.x == 0) pcg_stop(st, scal, PCG_FAILURE, it); return; }
    if (live)
#pragma unroll
      for (int a = 0; a < 6; ++a) x[6 * (size_t)v + a] = x[6 * (size_t)v + a] + alpha * p[6 * (size_t)v + a];
    if (blockIdx.x == 0 && threadIdx.x == 0) { st[PS_AAPP] = alpha; st[PS_AAPP_IT] = it; }   // (k_pcg_vacc)
    if (mode == 1) {
      if (blockIdx.x == 0 && threadIdx.x == 0) st[PS_ALPHA] = alpha;
      return;
    }
  } else {
    alpha = st[PS_ALPHA];
  }
  double acc[2] = {0.0, 0.0};
  if (live) {
    double rv[6], xv[6], zv[6];
    load6(x + 6 * (size_t)v, xv);
    if (mode == 2) {
      double sx[6];
      schur_row(Adiag, tpart, G, P.nvc, v, xv, sx);
#pragma unroll
      for (int a = 0; a < 6; ++a) rv[a] = b[6 * (size_t)v + a] - sx[a];
    } else {
#pragma unroll
      for (int a = 0; a < 6; ++a) rv[a] = r[6 * (size_t)v + a] - alpha * q[6 * (size_t)v + a];
    }
    store6(r + 6 * (size_t)v, rv);
    mat6_mul(Minv + (size_t)v * 36, rv, zv);
    store6(z + 6 * (size_t)v, zv);
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      acc[0] += xv[a] * (b[6 * (size_t)v + a] + rv[a]);
      acc[1] += rv[a] * zv[a];
    }
  }
  double tot[2];
  block_sum<2>(acc, lds, tot);
  if (threadIdx.x == 0) {
    ppart[kMaxBlocks + blockIdx.x] = tot[0];
    ppart[2 * kMaxBlocks + blockIdx.x] = tot[1];
  }
}

__global__ __launch_bounds__(256) void k_pcg_p(DevProblem P, int it, PcgOpts o, const double* __restrict__ z,
                                               double* __restrict__ p, const double* __restrict__ ppart,
                                               double* __restrict__ scal) {
  double* st = scal + kNumSlots;
  if (st[PS_DONE] != 0.0) return;
  __shared__ double lds[1];
  const int nb = gridDim.x;
  const double Q1 = -1.0 * fold_part(ppart + kMaxBlocks, nb, lds);
  const double rho_new = fold_part(ppart + 2 * kMaxBlocks, nb, lds);
  const double Q0 = st[q0_slot(it)], rho = st[rho_slot(it)];
  const double zeta = it * (Q1 - Q0) / Q1;
  const bool lead = blockIdx.x == 0;
  if (zeta < o.q_tolerance && it >= o.min_iter) { if (lead) pcg_stop(st, scal, PCG_SUCCESS, it); return; }
  if (it >= o.max_iter) { if (lead) pcg_stop(st, scal, PCG_NO_CONVERGENCE, it); return; }
  if (zero_or_inf(rho_new) || isnan(rho_new)) { if (lead) pcg_stop(st, scal, PCG_FAILURE, it + 1); return; }
  const double beta = rho_new / rho;
  if (zero_or_inf(beta)) { if (lead) pcg_stop(st, scal, PCG_FAILURE, it + 1); return; }
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v < P.nvc)
#pragma unroll
    for (int a = 0; a < 6; ++a) p[6 * (size_t)v + a] = z[6 * (size_t)v + a] + beta * p[6 * (size_t)v + a];
  if (lead && threadIdx.x == 0) {
    st[rho_slot(it + 1)] = rho_new;   // the other parity: blocks of this launch still read rho, Q0
    st[q0_slot(it + 1)] = Q1;
    st[PS_ITER] = it;
  }
}

// The points' accumulated products: y = sum_k alpha_k p_k (x starts at 0), so
// vpt(y) = sum_k alpha_k vpt(p_k) by linearity — the back substitution's
// u_p - sum_o W_o^T y_c without a pass over the observations (W.pacc).  set:
// the residual reset's matvec of y itself (skipped once the CG has stopped:
// that matvec did not run).  Otherwise fold alpha vpt when the update of
// iteration `it` moved x (PS_AAPP_IT), from zero at it = 1.
// (four doubles per thread as two 16-B pieces, grid-stride: 35 -> 14.6 us per
// working launch at C4, profiles/r05_final_c4full_kernel_stats.csv)
__global__ __launch_bounds__(256) void k_pcg_vacc(int n3, int it, int set, const double* __restrict__ st,
                                                  const double* __restrict__ vpt, double* __restrict__ vacc) {
  const bool done = st[PS_DONE] != 0.0;
  const bool moved = st[PS_AAPP_IT] == (double)it;
  const double al = st[PS_AAPP];
  if (set ? done : (!moved && it != 1)) return;   // (nothing to write)
  auto one = [&](double v, double a) { return set ? v : (moved ? (it == 1 ? 0.0 : a) + al * v : 0.0); };
  const int n4 = n3 >> 2;
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += gridDim.x * blockDim.x) {
    const double2* v2 = reinterpret_cast<const double2*>(vpt) + 2 * q;
    double2* a2 = reinterpret_cast<double2*>(vacc) + 2 * q;
    const double2 v0 = v2[0], v1 = v2[1];
    double2 a0 = make_double2(0.0, 0.0), a1 = make_double2(0.0, 0.0);
    if (!set && it != 1) { a0 = a2[0]; a1 = a2[1]; }
    a2[0] = make_double2(one(v0.x, a0.x), one(v0.y, a0.y));
    a2[1] = make_double2(one(v1.x, a1.x), one(v1.y, a1.y));
  }
  if (blockIdx.x == 0 && (int)threadIdx.x < (n3 & 3)) {
    const int e = 4 * n4 + threadIdx.x;
    vacc[e] = one(vpt[e], (!set && it != 1) ? vacc[e] : 0.0);
  }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
void launch_pcg_vacc(const DevProblem& P, const DevWork& W, int it, bool set, hipStream_t s) {
  const int n3 = 3 * P.np;
  if (n3 == 0) return;
  const int g = std::max(1, std::min((n3 / 4 + 255) / 256, 2048));
  hipLaunchKernelGGL(k_pcg_vacc, dim3(g), dim3(256), 0, s, n3, it, set ? 1 : 0, W.scal + kNumSlots,
                     W.vpt, W.vacc);
}
void launch_pcg_dup(const DevProblem& P, const DevWork& W, hipStream_t s) {
  if (P.nvc == 0) return;
  if (W.w32)
    hipLaunchKernelGGL(k_pcg_dup<float>, dim3((P.nvc + 255) / 256), dim3(256), 0, s, P, W.dup_off, W.dup_pairs, W.Wf,
                       W.Sd);
  else
    hipLaunchKernelGGL(k_pcg_dup<double>, dim3((P.nvc + 255) / 256), dim3(256), 0, s, P, W.dup_off, W.dup_pairs, W.W,
                       W.Sd);
}
void launch_pcg_setup(const DevProblem& P, const DevWork& W, double radius, const PcgOpts& o, hipStream_t s) {
  const int nb = (P.nvc + 255) / 256;
  hipLaunchKernelGGL(k_pcg_setup, dim3(nb), dim3(256), 0, s, P, W.Sd, W.Hcc, W.gc, W.scale_c, W.diag_c, radius,
                     o.schur_jacobi, W.Adiag, W.Minv, W.pb, W.y, W.pr, W.pz, W.pp, W.ppart);
  hipLaunchKernelGGL(k_pcg_setup_fin, dim3(1), dim3(64), 0, s, W.ppart, nb, W.scal);
}
void launch_pcg_matvec(const DevProblem& P, const DevWork& W, const double* vec, hipStream_t s) {
  const double* st = W.scal + kNumSlots;
  if (W.npchunks > 0) {   // point-aligned chunks of <= 64 observations (k_pcg_point_seg)
    const int g = std::max(1, std::min((W.npchunks + 3) / 4, 16384));
    if (W.tobs) {
      if (W.pcgjf)   // (the records formed in the pass itself, no W)
        launch_pcg_point_jf(P, W, vec, s);
      else if (W.pcgc && W.w32)   // (the 16-value rank-2 records)
        hipLaunchKernelGGL((k_pcg_point_seg<float, true, true>), dim3(g), dim3(256), 0, s, P, W.pchunks, W.npchunks,
                           W.Wf, vec, W.vpt, W.tobs, st);
      else if (W.pcgc)
        hipLaunchKernelGGL((k_pcg_point_seg<double, true, true>), dim3(g), dim3(256), 0, s, P, W.pchunks, W.npchunks,
                           W.W, vec, W.vpt, W.tobs, st);
      else if (W.w32)
        hipLaunchKernelGGL((k_pcg_point_seg<float, true>), dim3(g), dim3(256), 0, s, P, W.pchunks, W.npchunks, W.Wf,
                           vec, W.vpt, W.tobs, st);
      else
        hipLaunchKernelGGL((k_pcg_point_seg<double, true>), dim3(g), dim3(256), 0, s, P, W.pchunks, W.npchunks, W.W,
                           vec, W.vpt, W.tobs, st);
      // the products gathered into LDS by LDS-DMA: 152 -> 149 us at C4
      hipLaunchKernelGGL(k_pcg_cam_td, dim3(P.nvc, W.pcg_G), dim3(256), 0, s, P, W.tobs, W.tpart, st);
      return;
    }
    if (W.w32) {
      hipLaunchKernelGGL((k_pcg_point_seg<float, false>), dim3(g), dim3(256), 0, s, P, W.pchunks, W.npchunks, W.Wf,
                         vec, W.vpt, nullptr, st);
      hipLaunchKernelGGL(k_pcg_cam<float>, dim3(P.nvc, W.pcg_G), dim3(256), 0, s, P, W.Wf, W.vpt, W.tpart, st);
    } else {
      hipLaunchKernelGGL((k_pcg_point_seg<double, false>), dim3(g), dim3(256), 0, s, P, W.pchunks, W.npchunks, W.W,
                         vec, W.vpt, nullptr, st);
      hipLaunchKernelGGL(k_pcg_cam<double>, dim3(P.nvc, W.pcg_G), dim3(256), 0, s, P, W.W, W.vpt, W.tpart, st);
    }
    return;
  }
  if (W.tobs) {
    if (W.w32)
      hipLaunchKernelGGL(k_pcg_point_t<float>, dim3(pt_group_grid(P.np)), dim3(256), 0, s, P, W.Wf, vec, W.tobs, st);
    else
      hipLaunchKernelGGL(k_pcg_point_t<double>, dim3(pt_group_grid(P.np)), dim3(256), 0, s, P, W.W, vec, W.tobs, st);
    hipLaunchKernelGGL(k_pcg_cam_t, dim3(P.nvc, W.pcg_G), dim3(256), 0, s, P, W.tobs, W.tpart, st);
    return;
  }
  if (W.w32) {
    hipLaunchKernelGGL(k_pcg_point<float>, dim3(pt_group_grid(P.np)), dim3(256), 0, s, P, W.Wf, vec, W.vpt, st);
    hipLaunchKernelGGL(k_pcg_cam<float>, dim3(P.nvc, W.pcg_G), dim3(256), 0, s, P, W.Wf, W.vpt, W.tpart, st);
  } else {
    hipLaunchKernelGGL(k_pcg_point<double>, dim3(pt_group_grid(P.np)), dim3(256), 0, s, P, W.W, vec, W.vpt, st);
    hipLaunchKernelGGL(k_pcg_cam<double>, dim3(P.nvc, W.pcg_G), dim3(256), 0, s, P, W.W, W.vpt, W.tpart, st);
  }
}
void launch_pcg_tfold(const DevProblem& P, const DevWork& W, hipStream_t s) {
  if (W.pcg_G <= 1 || P.nvc == 0) return;
  hipLaunchKernelGGL(k_pcg_tfold, dim3((6 * P.nvc + 255) / 256), dim3(256), 0, s, P.nvc, W.pcg_G, W.tpart,
                     W.scal + kNumSlots);
}
void launch_pcg_update(const DevProblem& P, const DevWork& W, int mode, int it, const PcgOpts& o, hipStream_t s) {
  // (after launch_pcg_tfold the slices are folded into slice 0: G = 1)
  const int G = W.pcg_folded ? 1 : W.pcg_G;
  if (P.nvc <= kPcgOneWg) {   // one workgroup: one launch per CG iteration
    // (kPcgOneWg threads: the workgroup sums add the waves in index order, so
    // the 1024-thread launch this replaced, whose extra waves added zeros,
    // rounded identically)
    hipLaunchKernelGGL(k_pcg_update, dim3(1), dim3(kPcgOneWg), 0, s, P, mode, it, o, G, W.Adiag, W.Minv,
                       W.pb, W.y, W.pr, W.pz, W.pp, W.pq, W.tpart, W.scal);
    return;
  }
  const int nb = (P.nvc + 255) / 256;
  const double* st = W.scal + kNumSlots;
  if (mode != 2)
    hipLaunchKernelGGL(k_pcg_q, dim3(nb), dim3(256), 0, s, P, G, W.Adiag, W.pp, W.pq, W.tpart, W.ppart, st);
  hipLaunchKernelGGL(k_pcg_xr, dim3(nb), dim3(256), 0, s, P, mode, it, G, W.Adiag, W.Minv, W.pb, W.y, W.pr,
                     W.pz, W.pp, W.pq, W.tpart, W.ppart, W.scal);
  if (mode != 1) hipLaunchKernelGGL(k_pcg_p, dim3(nb), dim3(256), 0, s, P, it, o, W.pz, W.pp, W.ppart, W.scal);
}

}  // namespace bahip

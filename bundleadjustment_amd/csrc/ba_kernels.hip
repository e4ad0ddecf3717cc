// ba_kernels.hip — CDNA4 (gfx950, wave64) kernels of one Levenberg-Marquardt
// iteration of the reference's Ceres DENSE_SCHUR bundle adjustment
// (ba_project/src/ba/Optimizer.cpp:80-90, 216-333; Optimizer.h:49-194),
// re-designed for MI355X:
//
//   linearise  (per observation, HBM stream)   r, J  (Huber-corrected)
//   assemble   (per point / per camera)        Hpp, gp, Hcc, gc, scaling, LM diag
//   eliminate  (per point / per observation)   L^-1 of (Hpp + D), W = E L^-T
//   reduce     (per camera, per camera pair)   S = A_cc - sum W W^T, rhs
//   factor     (dense blocked Cholesky)        S = L L^T, forward folded in
//   candidate  (per point, HBM stream)         back-substitution, model cost
//                                              change, candidate cost
//
// Every reduction is a fixed-order tree (wave shuffles + LDS, then a
// fixed-order fold of per-block partials): results are bitwise reproducible
// run to run.  No floating-point atomics anywhere.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include <hip/hip_ext.h>

#include "ba_kernels.h"
#include "ba_device.h"
#include "ba_reduce.h"
#include "ba_schur.h"
#include "../../include/ba_hip.h"   // ba_termination codes (batched pose-only solve)

namespace bahip {

// Non-temporal 16-B / 8-B stores for the per-observation record streams (JR
// from the linearisation, W from the elimination): measured in the LM
// pipeline, they keep the records from displacing (and writing back) the
// previous phases' dirty lines in the caches on the write path —
// k_linearize_lds_t 44.1 -> 40.3 us at C3, whole iteration +0.5 %.
typedef double ntd2 __attribute__((ext_vector_type(2)));
typedef float ntf2 __attribute__((ext_vector_type(2)));
__device__ inline void nt_store(double2* p, double2 v) {
  ntd2 t = {v.x, v.y};
  __builtin_nontemporal_store(t, reinterpret_cast<ntd2*>(p));
}
__device__ inline void nt_store(float2* p, float2 v) {
  ntf2 t = {v.x, v.y};
  __builtin_nontemporal_store(t, reinterpret_cast<ntf2*>(p));
}

int grid_for(int n) {
  int g = (n + kThreads - 1) / kThreads;
  if (g < 1) g = 1;
  return g > kMaxBlocks ? kMaxBlocks : g;
}
int pt_group_grid(int np) { return grid_for((int)std::min<long long>((long long)np * kPtLanes, 1LL << 30)); }


// Per-camera work is split over W.cam_split <= kCamSplit workgroups (one workgroup per
// camera leaves CUs idle and is latency bound).  Each slice stores its 27
// block sums; a second kernel adds the slices in slice order (deterministic;
// the kernel boundary makes the slices visible across XCDs — an in-kernel
// last-block fold needs agent-scope release fences, which write back the L2
// and measured 2x slower).
__device__ inline void cam_slice_store(const double (&tot)[27], double* __restrict__ cpart, int v, int nvc) {
  if (threadIdx.x == 0) {
    double* dst = cpart + ((size_t)blockIdx.y * nvc + v) * 27;
#pragma unroll
    for (int k = 0; k < 27; ++k) dst[k] = tot[k];
  }
}

// fold the slices: mode 0 -> Hcc (21) / gc (6); mode 1 -> S diagonal block
// (-sum W W^T, lower) and rhs row (-sum W u); mode 2 -> the same 27 values
// into a compact per-camera array (ITERATIVE_SCHUR)
__global__ __launch_bounds__(256) void k_cam_fold(DevProblem P, const double* __restrict__ cpart, int nsl, int mode,
                                                  double* __restrict__ Hcc, double* __restrict__ gc,
                                                  double* __restrict__ S) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= P.nvc * 27) return;
  const int v = e / 27, k = e - v * 27;
  double acc = 0.0;
  for (int sl = 0; sl < nsl; ++sl) acc += cpart[((size_t)sl * P.nvc + v) * 27 + k];
  if (mode == 0) {
    if (k < 21) Hcc[(size_t)v * 21 + k] = acc;
    else gc[(size_t)v * 6 + (k - 21)] = acc;
  } else if (mode == 2) {   // compact [nvc][27] (ITERATIVE_SCHUR: diagonal Schur blocks + rhs, no dense S)
    S[(size_t)v * 27 + k] = -acc;
  } else {
    const size_t ld = (size_t)P.ld;
    if (k < 21) {
      int a2 = 0;
      while ((a2 + 1) * (a2 + 2) / 2 <= k) ++a2;
      const int b2 = k - a2 * (a2 + 1) / 2;
      S[(size_t)(6 * v + a2) * ld + 6 * v + b2] = -acc;
    } else {
      S[(size_t)P.n * ld + 6 * v + (k - 21)] = -acc;
    }
  }
}

// observation range of slice blockIdx.y of camera v
__device__ inline void cam_slice(const DevProblem& P, int v, int& i0, int& i1) {
  const int a = P.cam_off[v], b = P.cam_off[v + 1];
  const int len = (b - a + (int)gridDim.y - 1) / (int)gridDim.y;
  i0 = min(b, a + (int)blockIdx.y * len);
  i1 = min(b, i0 + len);
}

// ---------------------------------------------------------------------------
// camera records: R, dR/dw (forward derivative of ceres' Rodrigues), t, K
// ---------------------------------------------------------------------------
// One 64-lane block per camera; every lane evaluates the (cheap) Rodrigues
// duals and writes the record entries e = lane, lane + 64 (short critical
// path: a thread per camera serialises ~90 dependent stores).
__device__ inline double cam_rec_entry(int e, const double* w, const double* t, const double* Kd, const D3* R,
                                       const double* R0, bool deriv) {
  if (e < 9) return deriv ? R[e].a : R0[e];
  if (e < 36) { const int k = (e - 9) / 9, i = (e - 9) % 9; return deriv ? R[i].d[k] : 0.0; }
  if (e < 39) return t[e - 36];
  if (e < 48) return Kd[e - 39];
  if (!deriv) return 0.0;
  const int l = e - kRecL;
  if (l < 36) {   // K M, M = R or dR/dw_k, col-major
    const int m = l / 9, idx = l % 9, col = idx / 3, row = idx % 3;
    double M0, M1, M2;
    if (m == 0) { M0 = R[col * 3].a; M1 = R[col * 3 + 1].a; M2 = R[col * 3 + 2].a; }
    else { M0 = R[col * 3].d[m - 1]; M1 = R[col * 3 + 1].d[m - 1]; M2 = R[col * 3 + 2].d[m - 1]; }
    return Kd[row] * M0 + Kd[3 + row] * M1 + Kd[6 + row] * M2;
  }
  if (l < 39) { const int row = l - 36; return Kd[row] * t[0] + Kd[3 + row] * t[1] + Kd[6 + row] * t[2]; }
  return 0.0;
}

__global__ __launch_bounds__(64) void k_cam_prep(int nc, const double* __restrict__ cams, const float* __restrict__ K,
                                                 const uint8_t* __restrict__ cam_fixed, const float* __restrict__ extr,
                                                 double* __restrict__ rec, int deriv) {
  const int c = blockIdx.x, lane = threadIdx.x;
  if (c >= nc) return;
  double* o = rec + (size_t)c * kCamRec;
  double Kd[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) Kd[k] = (double)K[9 * c + k];
  if (cam_fixed && cam_fixed[c]) {
    const float* E = extr + 16 * c;
    for (int e = lane; e < kCamRec; e += 64) {
      double v = 0.0;
      if (e < 16) v = (double)E[e];
      else if (e >= kRecK && e < kRecK + 9) v = Kd[e - kRecK];
      else if (deriv && e >= kRecL) {
        const int l = e - kRecL;
        if (l < 12) {   // K E(0:3, col)
          const int col = l / 3, row = l % 3;
          v = Kd[row] * (double)E[col * 4] + Kd[3 + row] * (double)E[col * 4 + 1] + Kd[6 + row] * (double)E[col * 4 + 2];
        } else if (l < 16) {
          v = (double)E[(l - 12) * 4 + 3];
        }
      }
      o[e] = v;
    }
    return;
  }
  const double w[3] = {cams[6 * c], cams[6 * c + 1], cams[6 * c + 2]};
  const double t[3] = {cams[6 * c + 3], cams[6 * c + 4], cams[6 * c + 5]};
  D3 R[9];
  double R0[9];
  if (deriv) angle_axis_to_R_d3(w, R);
  else angle_axis_to_R(w, R0);
  for (int e = lane; e < kCamRec; e += 64) o[e] = cam_rec_entry(e, w, t, Kd, R, R0, deriv != 0);
}

// Project one observation; value only.  Returns residual (u,v) in r.
__device__ inline void project_value(const double* __restrict__ cr, bool cvar, double X0, double X1, double X2,
                                     float2 uv, double r[2]) {
  double p[3];
  if (cvar) {
#pragma unroll
    for (int i = 0; i < 3; ++i) p[i] = cr[kRecR + i] * X0 + cr[kRecR + 3 + i] * X1 + cr[kRecR + 6 + i] * X2 + cr[kRecT + i];
  } else {
    double ph[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) ph[i] = X0 * cr[i] + X1 * cr[4 + i] + X2 * cr[8 + i] + cr[12 + i];
    p[0] = ph[0] / ph[3]; p[1] = ph[1] / ph[3]; p[2] = ph[2] / ph[3];
  }
  const double* Kc = cr + kRecK;
  double q[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) q[i] = p[0] * Kc[i] + p[1] * Kc[3 + i] + p[2] * Kc[6 + i];
  r[0] = q[0] / q[2] - (double)uv.x;
  r[1] = q[1] / q[2] - (double)uv.y;
}

// ---------------------------------------------------------------------------
// Per-observation Jacobian/residual record (AoS, 20 doubles = 160 B):
//   [0..5]  Jc row 0   [6..11] Jc row 1   [12..14] Jp row 0   [15..17] Jp row 1
//   [18] r0  [19] r1          (Huber-corrected)
// One record per observation in (point, camera) order: the per-point and
// per-observation passes stream it, the per-camera passes gather whole
// records (1-2 cache lines each instead of 14 scattered SoA lines).
// ---------------------------------------------------------------------------
constexpr int kJR = 20;
constexpr int kStageLd = kJR + 1;   // LDS row stride of staged records
// Storage: the record is split in two arrays inside the JR buffer so that
// readers of one half fetch only that half's cache lines:
//   JA = JR           [no][JA]  fields 0..11 (camera rows: 96 B)
//                               (+ 18..19 when JA = 14: the residual again)
//   JB = JR + JA no   [no][8]   fields 12..19 (point rows + residual: 64 B)
// JA = 12 up to kLinLdsCams cameras.  Beyond, JA = 14: k_cam_assemble's
// camera-order gathers then read one 112-B record (~1.75 lines) instead of
// 96 B plus a JB line (~2.5 lines) — C5 shard +1.6 %; at C3 the 16 B/obs of
// extra writes cost more than the gathers save (profiles/r02_v7_ab_jr_*).
// JA = 16 (BA_JA_SMALL=16: 128-B records, one line per k_cam_assemble
// gather) measured slower still at C3: k_linearize +5..7 us against the
// gathers it saves (profiles/r02_s3_ab_ja16.txt).
constexpr int kJB = 8;
constexpr int kFJB = 12;   // record field of the first JB slot
#ifndef BA_JA_SMALL
#define BA_JA_SMALL 12
#endif
constexpr int jr_ja(bool many_cams) { return many_cams ? 14 : BA_JA_SMALL; }
// JA slot k -> record field (slots 12.. repeat the residual: 12/14 -> r0, 13/15 -> r1)
__device__ __forceinline__ int ja_field(int k) { return k < 12 ? k : 18 + ((k - 12) & 1); }
template <int JA>
__device__ inline const double* jr_a(const double* JR, int o) { return JR + (size_t)o * JA; }
template <int JA>
__device__ inline const double* jr_b(const double* JR, int no, int o) {
  return JR + (size_t)JA * no + (size_t)o * kJB;
}
// the 64 records of the chunk at `base` as JA/2 + 4 coalesced 1 KiB wave
// loads, indices clamped (unconditional loads); non-temporal: each chunk is
// read once per kernel (measured +0.9 % per LM iteration)
template <int JA>
__device__ inline void jr_chunk_load(const double* __restrict__ JR, int no, int base, int lane,
                                     double2 (&t)[JA / 2 + kJB / 2]) {
  const double2* A2 = reinterpret_cast<const double2*>(JR);
  const double2* B2 = reinterpret_cast<const double2*>(JR + (size_t)JA * no);
  const int lastA = (JA / 2) * no - 1, lastB = (kJB / 2) * no - 1;
#pragma unroll
  for (int it = 0; it < JA / 2; ++it) {
    const ntd2 x = __builtin_nontemporal_load(reinterpret_cast<const ntd2*>(&A2[min((JA / 2) * base + it * 64 + lane, lastA)]));
    t[it] = make_double2(x.x, x.y);
  }
#pragma unroll
  for (int it = 0; it < kJB / 2; ++it) {
    const ntd2 x = __builtin_nontemporal_load(reinterpret_cast<const ntd2*>(&B2[min((kJB / 2) * base + it * 64 + lane, lastB)]));
    t[JA / 2 + it] = make_double2(x.x, x.y);
  }
}
// scatter them into the wave's LDS rows (record fields 0..19, stride kStageLd;
// a JA copy of the residual is dropped, JB's lands in fields 18..19)
template <int JA>
__device__ inline void jr_chunk_stage(double* st, int lane, const double2 (&t)[JA / 2 + kJB / 2]) {
#pragma unroll
  for (int it = 0; it < JA / 2; ++it) {
    const int e = it * 64 + lane, r = e / (JA / 2), f = 2 * (e - r * (JA / 2));
    if (JA == 12 || f < 12) {
      st[r * kStageLd + f] = t[it].x;
      st[r * kStageLd + f + 1] = t[it].y;
    }
  }
#pragma unroll
  for (int it = 0; it < kJB / 2; ++it) {
    const int e = it * 64 + lane, r = e / (kJB / 2), f = kFJB + 2 * (e - r * (kJB / 2));
    st[r * kStageLd + f] = t[JA / 2 + it].x;
    st[r * kStageLd + f + 1] = t[JA / 2 + it].y;
  }
}

// ---------------------------------------------------------------------------
// linearisation: one thread per observation (sorted by point)
// ---------------------------------------------------------------------------
// Camera access for the linearisation: the K-folded table (kRecL, 40
// doubles, read as 20 16-B loads) and K (float-valued) from the block's LDS
// copy of the camera table.
// LDS row: lin table (40) + variable flag (slot 40) + pad; stride 42 doubles
// keeps rows 16-B aligned and spreads random cameras over the 16 bank
// groups of ds_read_b128
constexpr int kTblRec = kLin + 2;
struct CamLds {
  const double* r;
  const float* k;
  __device__ bool var() const { return r[kLin] != 0.0; }
  __device__ void load(double (&t)[kLin]) const {
    const double2* s = reinterpret_cast<const double2*>(r);
#pragma unroll
    for (int k = 0; k < kLin / 2; ++k) { const double2 u = s[k]; t[2 * k] = u.x; t[2 * k + 1] = u.y; }
  }
  __device__ double K(int i) const { return (double)k[i]; }
};
// camera row as an indexable value: a register copy
struct RowRegs {
  double t[kLin];
  __device__ double operator[](int i) const { return t[i]; }
};
template <class Cam>
__device__ inline RowRegs cam_row(const Cam& cr) { RowRegs R; cr.load(R.t); return R; }

// Many cameras (nc > kLinLdsCams): the 704-B camera records no longer fit the
// LDS and, past ~5k cameras, not even one XCD's L2 (C5: 7 MB of records,
// ~4.8 GB of per-observation record gathers served by the Infinity Cache).
// Instead every observation gathers its camera's compact 128-B record (one
// cache line, the whole table L2-resident) and rebuilds the K-folded terms in
// registers: the dual-number Rodrigues of k_cam_prep (same functions, same
// arithmetic), cheap next to the HBM stream.  The per-camera scalars of the
// Rodrigues (theta = |w|, 1 / (2 theta), 1 / theta, cos, sin) are formed
// once per camera by k_cam_compact and travel in the record, so the
// per-observation work has no sqrt, divide or sin / cos on its chain.
//   [0..2] w (variable) | camera index in [0] (fixed); [3..5] t;
//   [6..10] K as 9 floats (float-valued Matrix3f) + the variable flag as
//   float 9; [11..15] theta, 1/(2 theta), 1/theta, cos theta, sin theta
//   (theta = 0: the small-angle branch)
constexpr int kCRec = 16;
constexpr int kCRecK = 6, kCRecTh = 11;
struct CamRcPre {
  double2 v[kCRec / 2];
};
struct CamRc {   // unpacked compact record; lin_obs(CamRc) forms the table terms itself
  double w[3], t[3], Kd[9], th[5];
  int cidx;
  bool v;
  __device__ bool var() const { return v; }
  __device__ double K(int i) const { return Kd[i]; }
};
struct CamRcOf {
  const double* crec;
  const float* extr;
};
// prefetch / construct hooks of lin_waves: table-based camera accessors take
// the camera index itself; CamRcOf prefetches the compact record one chunk
// ahead and rebuilds the table at use
template <class F>
__device__ inline int cam_pre(const F&, int c) { return c; }
template <class F>
__device__ inline auto cam_make(const F& f, int c) { return f(c); }
__device__ inline CamRcPre cam_pre(const CamRcOf& f, int c) {
  CamRcPre q;
  const double2* s = reinterpret_cast<const double2*>(f.crec + (size_t)c * kCRec);
#pragma unroll
  for (int k = 0; k < kCRec / 2; ++k) q.v[k] = s[k];
  return q;
}
__device__ inline CamRc cam_make(const CamRcOf&, const CamRcPre& q) {
  CamRc C;
  double rv[kCRec];
#pragma unroll
  for (int k = 0; k < kCRec / 2; ++k) { rv[2 * k] = q.v[k].x; rv[2 * k + 1] = q.v[k].y; }
#pragma unroll
  for (int k = 0; k < 3; ++k) { C.w[k] = rv[k]; C.t[k] = rv[3 + k]; }
  float kf[10];
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, rv[kCRecK + k]);
    kf[2 * k] = __builtin_bit_cast(float, (unsigned)b);
    kf[2 * k + 1] = __builtin_bit_cast(float, (unsigned)(b >> 32));
  }
#pragma unroll
  for (int k = 0; k < 9; ++k) C.Kd[k] = (double)kf[k];
#pragma unroll
  for (int k = 0; k < 5; ++k) C.th[k] = rv[kCRecTh + k];
  C.cidx = (int)rv[0];
  C.v = kf[9] != 0.0f;
  return C;
}

// ceres::AngleAxisToRotationMatrix on duals (angle_axis_to_R_d3) with the
// value-only scalars of theta taken from the record: theta, 1 / (2 theta)
// (dsqrt), 1 / theta (the three quotients) and cos / sin (dcos, dsin) are the
// same operations on the same operand, so the result is the same
__device__ __forceinline__ void angle_axis_to_R_d3_pre(const double w[3], const double th[5], D3 R[9]) {
  const D3 a0 = mk(w[0], 1, 0, 0), a1 = mk(w[1], 0, 1, 0), a2 = mk(w[2], 0, 0, 1);
  if (th[0] > 0.0) {
    const D3 theta2 = a0 * a0 + a1 * a1 + a2 * a2;
    const double ti = th[1], gi = th[2], cs = th[3], sn = th[4];
    const D3 theta = mk(th[0], theta2.d[0] * ti, theta2.d[1] * ti, theta2.d[2] * ti);
    auto quot = [&](D3 f) {
      const double fg = f.a * gi;
      return mk(fg, (f.d[0] - fg * theta.d[0]) * gi, (f.d[1] - fg * theta.d[1]) * gi, (f.d[2] - fg * theta.d[2]) * gi);
    };
    const D3 wx = quot(a0), wy = quot(a1), wz = quot(a2);
    const double ns = -sn;
    const D3 c = mk(cs, ns * theta.d[0], ns * theta.d[1], ns * theta.d[2]);
    const D3 s = mk(sn, cs * theta.d[0], cs * theta.d[1], cs * theta.d[2]);
    const D3 oc = rsub(1.0, c);
    R[0] = c + wx * wx * oc;
    R[1] = wz * s + wx * wy * oc;
    R[2] = -(wy * s) + wx * wz * oc;
    R[3] = wx * wy * oc - wz * s;
    R[4] = c + wy * wy * oc;
    R[5] = wx * s + wy * wz * oc;
    R[6] = wy * s + wx * wz * oc;
    R[7] = -(wx * s) + wy * wz * oc;
    R[8] = c + wz * wz * oc;
  } else {
    R[0] = mk(1, 0, 0, 0); R[1] = a2;             R[2] = -a1;
    R[3] = -a2;            R[4] = mk(1, 0, 0, 0); R[5] = a0;
    R[6] = a1;             R[7] = -a0;            R[8] = mk(1, 0, 0, 0);
  }
}

// compact camera records for CamRcOf (thread per camera)
__global__ __launch_bounds__(256) void k_cam_compact(DevProblem P, const double* __restrict__ cams,
                                                     double* __restrict__ crec) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= P.nc) return;
  const bool var = P.vc[c] >= 0;
  double* o = crec + (size_t)c * kCRec;
  double w[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) w[k] = var ? cams[6 * c + k] : 0.0;
#pragma unroll
  for (int k = 0; k < 6; ++k) o[k] = var ? cams[6 * c + k] : (k == 0 ? (double)c : 0.0);
  float kf[10];
#pragma unroll
  for (int k = 0; k < 9; ++k) kf[k] = P.K[9 * c + k];
  kf[9] = var ? 1.0f : 0.0f;
#pragma unroll
  for (int k = 0; k < 5; ++k)
    o[kCRecK + k] = __builtin_bit_cast(double, ((unsigned long long)__builtin_bit_cast(unsigned, kf[2 * k + 1]) << 32) |
                                                   __builtin_bit_cast(unsigned, kf[2 * k]));
  // the scalars of angle_axis_to_R_d3: theta2.a of the duals is w.w
  const D3 a0 = mk(w[0], 1, 0, 0), a1 = mk(w[1], 0, 1, 0), a2 = mk(w[2], 0, 0, 1);
  const D3 theta2 = a0 * a0 + a1 * a1 + a2 * a2;
  double th[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  if (var && theta2.a > 2.220446049250313080847e-16) {
    const double t = sqrt(theta2.a);
    th[0] = t;
    th[1] = 1.0 / (2.0 * t);
    th[2] = 1.0 / t;
    th[3] = cos(t);
    th[4] = sin(t);
  }
#pragma unroll
  for (int k = 0; k < 5; ++k) o[kCRecTh + k] = th[k];
}

// r, J (Huber-corrected) of one observation into out[20]; returns rho.
// AngleReprojectionError (Optimizer.h:54-76) / PointOnlyReprojectionError
// (Optimizer.h:96-107) with the chain rule of their Jets:
//   q = K (R X + t),  dq/dw_k = K dR_k X,  dq/dt = K,  dq/dX = K R
//   fixed: q = K E(0:3) [X;1] / w,  w = E(3) [X;1],  dq/dX = (K E - q e3) / w
//   r = q01 / q2 - uv,  dr/d* = (dq01 - r' dq2) / q2,  Huber corrector sqrt(rho')
template <class Cam>
__device__ inline double lin_obs(const DevProblem& P, const Cam& cr, bool cvar, bool pvar, double X0, double X1,
                                 double X2, float2 uv, double (&out)[kJR], bool& fin, double* prf = nullptr) {
  const auto T = cam_row(cr);
  double q[3], iw = 1.0;
  if (cvar) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
      q[i] = T[kLinKR + i] * X0 + T[kLinKR + 3 + i] * X1 + T[kLinKR + 6 + i] * X2 + T[kLinKt + i];
  } else {
    const double wv = T[kLinE3] * X0 + T[kLinE3 + 1] * X1 + T[kLinE3 + 2] * X2 + T[kLinE3 + 3];
    iw = 1.0 / wv;
#pragma unroll
    for (int i = 0; i < 3; ++i)
      q[i] = (T[kLinKE + i] * X0 + T[kLinKE + 3 + i] * X1 + T[kLinKE + 6 + i] * X2 + T[kLinKE + 9 + i]) * iw;
  }
  const double iq = 1.0 / q[2];
  const double pr0 = q[0] * iq, pr1 = q[1] * iq;
  const double r0 = pr0 - (double)uv.x, r1 = pr1 - (double)uv.y;
  double scale;
  const double rho = huber(r0 * r0 + r1 * r1, P.huber_a, P.huber_b, &scale);
  const double f = iq * scale;
  fin = isfinite(r0) && isfinite(r1) && isfinite(f);
  if (prf) { prf[0] = pr0; prf[1] = pr1; prf[2] = f; }   // (k_obs_w_rc's compact records)
  if (cvar) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int b = kLinKdR + 9 * k;
      const double d0 = T[b] * X0 + T[b + 3] * X1 + T[b + 6] * X2;
      const double d1 = T[b + 1] * X0 + T[b + 4] * X1 + T[b + 7] * X2;
      const double d2 = T[b + 2] * X0 + T[b + 5] * X1 + T[b + 8] * X2;
      out[k] = (d0 - pr0 * d2) * f;
      out[6 + k] = (d1 - pr1 * d2) * f;
      const double k2 = cr.K(3 * k + 2);
      out[3 + k] = (cr.K(3 * k) - pr0 * k2) * f;
      out[9 + k] = (cr.K(3 * k + 1) - pr1 * k2) * f;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 12; ++k) out[k] = 0.0;
  }
  if (pvar) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      double d0, d1, d2;
      if (cvar) {
        d0 = T[kLinKR + 3 * k]; d1 = T[kLinKR + 3 * k + 1]; d2 = T[kLinKR + 3 * k + 2];
      } else {
        const double e = T[kLinE3 + k];
        d0 = (T[kLinKE + 3 * k] - q[0] * e) * iw;
        d1 = (T[kLinKE + 3 * k + 1] - q[1] * e) * iw;
        d2 = (T[kLinKE + 3 * k + 2] - q[2] * e) * iw;
      }
      out[12 + k] = (d0 - pr0 * d2) * f;
      out[15 + k] = (d1 - pr1 * d2) * f;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 6; ++k) out[12 + k] = 0.0;
  }
  out[18] = r0 * scale;
  out[19] = r1 * scale;
#pragma unroll
  for (int k = 0; k < 18; ++k) fin = fin && isfinite(out[k]);
  return rho;
}

// The same record from a compact camera (CamRc): the Jets' evaluation order
// itself — p = R X + t on duals of w, q = K p, dq/dX = K R — with R and its
// w-derivatives from the dual Rodrigues of k_cam_prep.  Fixed cameras read
// their float extrinsic.  lin_obs_rc: the part after the dual Rodrigues (R
// given), so that camera-major kernels form R once per camera (CamRcR) and
// point-major ones per observation — the same operations either way.
__device__ inline double lin_obs_rc(const DevProblem& P, const D3* R, const double* t, const double* Kd, int cidx,
                                    bool cvar, bool pvar, double X0, double X1, double X2, float2 uv,
                                    double (&out)[kJR], bool& fin, double* prf) {
  double q[3], dq[3][3], dX[3][3], iw = 1.0;   // dq/dw_k [k][row], dq/dX_col [col][row]
  if (cvar) {
    D3 p[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const D3 a = R[i], b = R[3 + i], c = R[6 + i];
      p[i] = mk(a.a * X0 + b.a * X1 + c.a * X2 + t[i], a.d[0] * X0 + b.d[0] * X1 + c.d[0] * X2,
                a.d[1] * X0 + b.d[1] * X1 + c.d[1] * X2, a.d[2] * X0 + b.d[2] * X1 + c.d[2] * X2);
    }
#pragma unroll
    for (int row = 0; row < 3; ++row) {
      q[row] = Kd[row] * p[0].a + Kd[3 + row] * p[1].a + Kd[6 + row] * p[2].a;
#pragma unroll
      for (int k = 0; k < 3; ++k) dq[k][row] = Kd[row] * p[0].d[k] + Kd[3 + row] * p[1].d[k] + Kd[6 + row] * p[2].d[k];
#pragma unroll
      for (int col = 0; col < 3; ++col)
        dX[col][row] = Kd[row] * R[col * 3].a + Kd[3 + row] * R[col * 3 + 1].a + Kd[6 + row] * R[col * 3 + 2].a;
    }
  } else {
    const float* E = P.extr + 16 * cidx;
    double e3[4], KE[12];
#pragma unroll
    for (int l = 0; l < 12; ++l) {
      const int col = l / 3, row = l % 3;
      KE[l] = Kd[row] * (double)E[col * 4] + Kd[3 + row] * (double)E[col * 4 + 1] + Kd[6 + row] * (double)E[col * 4 + 2];
    }
#pragma unroll
    for (int l = 0; l < 4; ++l) e3[l] = (double)E[l * 4 + 3];
    const double wv = e3[0] * X0 + e3[1] * X1 + e3[2] * X2 + e3[3];
    iw = 1.0 / wv;
#pragma unroll
    for (int i = 0; i < 3; ++i) q[i] = (KE[i] * X0 + KE[3 + i] * X1 + KE[6 + i] * X2 + KE[9 + i]) * iw;
#pragma unroll
    for (int col = 0; col < 3; ++col)
#pragma unroll
      for (int row = 0; row < 3; ++row) dX[col][row] = (KE[3 * col + row] - q[row] * e3[col]) * iw;
  }
  const double iq = 1.0 / q[2];
  const double pr0 = q[0] * iq, pr1 = q[1] * iq;
  const double r0 = pr0 - (double)uv.x, r1 = pr1 - (double)uv.y;
  double scale;
  const double rho = huber(r0 * r0 + r1 * r1, P.huber_a, P.huber_b, &scale);
  const double f = iq * scale;
  fin = isfinite(r0) && isfinite(r1) && isfinite(f);
  if (prf) { prf[0] = pr0; prf[1] = pr1; prf[2] = f; }
  if (cvar) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      out[k] = (dq[k][0] - pr0 * dq[k][2]) * f;
      out[6 + k] = (dq[k][1] - pr1 * dq[k][2]) * f;
      const double k2 = Kd[3 * k + 2];
      out[3 + k] = (Kd[3 * k] - pr0 * k2) * f;
      out[9 + k] = (Kd[3 * k + 1] - pr1 * k2) * f;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 12; ++k) out[k] = 0.0;
  }
  if (pvar) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      out[12 + k] = (dX[k][0] - pr0 * dX[k][2]) * f;
      out[15 + k] = (dX[k][1] - pr1 * dX[k][2]) * f;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 6; ++k) out[12 + k] = 0.0;
  }
  out[18] = r0 * scale;
  out[19] = r1 * scale;
#pragma unroll
  for (int k = 0; k < 18; ++k) fin = fin && isfinite(out[k]);
  return rho;
}
__device__ inline double lin_obs(const DevProblem& P, const CamRc& cr, bool cvar, bool pvar, double X0, double X1,
                                 double X2, float2 uv, double (&out)[kJR], bool& fin, double* prf = nullptr) {
  D3 R[9];
  if (cvar) angle_axis_to_R_d3_pre(cr.w, cr.th, R);
  return lin_obs_rc(P, R, cr.t, cr.Kd, cr.cidx, cvar, pvar, X0, X1, X2, uv, out, fin, prf);
}
// a compact camera with its dual Rodrigues formed (camera-major kernels)
struct CamRcR {
  D3 R[9];
  double t[3], Kd[9];
  int cidx;
  bool v;
  __device__ void make(const CamRc& c) {
    if (c.v) angle_axis_to_R_d3_pre(c.w, c.th, R);
#pragma unroll
    for (int k = 0; k < 3; ++k) t[k] = c.t[k];
#pragma unroll
    for (int k = 0; k < 9; ++k) Kd[k] = c.Kd[k];
    cidx = c.cidx;
    v = c.v;
  }
  __device__ bool var() const { return v; }
};
__device__ inline double lin_obs(const DevProblem& P, const CamRcR& cr, bool cvar, bool pvar, double X0, double X1,
                                 double X2, float2 uv, double (&out)[kJR], bool& fin, double* prf = nullptr) {
  return lin_obs_rc(P, cr.R, cr.t, cr.Kd, cr.cidx, cvar, pvar, X0, X1, X2, uv, out, fin, prf);
}
// the compact record of camera c, unpacked (one 128-B line)
__device__ inline CamRc cam_rc(const double* __restrict__ crec, int c) {
  return cam_make(CamRcOf{crec, nullptr}, cam_pre(CamRcOf{crec, nullptr}, c));
}

// Wave body: every wave owns chunks of 64 consecutive observations (grid
// stride over chunks), computes one record per lane, stages the records in a
// wave-private LDS slot of ROWS rows (row stride 21 doubles: conflict-free
// b64 writes; ROWS = 32 stages the chunk in two rounds to leave LDS for more
// waves) and stores them as contiguous 1 KiB wave stores.  No workgroup
// barrier: waves drift apart, so one wave's store burst overlaps the others'
// arithmetic (measured ceiling of this store shape: tools/hbm_probe.hip
// write_stage, 6.4 TB/s; a row-per-lane 160-B record store: 3.3 TB/s).
// Indices are loaded three chunks ahead, the gathered point data two chunks
// ahead of the arithmetic.
// LDS hand-off between the lanes of one wave: DS operations of a wave
// execute in order, so a compiler barrier is enough (a wavefront-scope
// fence made the waitcnt pass drain vmcnt before every LDS read)
__device__ inline void wave_lds_sync() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

// MODE (diagnostics only, tools/lin_probe.hip): 0 product; 1 no global
// stores; 2 no arithmetic (records = a sum of the camera row); 3 table fill
// only; 4 loads only; 5 arithmetic only (no stage, no stores); 6 = 5 with
// every lane on camera 1 (broadcast table reads)
struct NoInit {
  __device__ void operator()() const {}
};
// init(): block-wide setup (e.g. building the LDS camera table) run by every
// thread after the prologue loads are issued, so it overlaps their latency
template <int JA, int WAVES, int ROWS, class CamOf, int MODE = 0, class Init = NoInit>
__device__ inline void lin_waves(const DevProblem& P, const double* __restrict__ pts, double* __restrict__ JR,
                                 double* stage_all, const CamOf& cam_of, double (&acc)[2], const Init& init = Init{}) {
  static_assert(ROWS == 64 || ROWS == 32, "stage rows");
  if (P.no == 0) { init(); return; }   // (the clamped prefetch indices need no >= 1)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double* stage = stage_all + w * (ROWS * kStageLd);
  const int step = gridDim.x * WAVES * 64;
  int base = (blockIdx.x * WAVES + w) * 64;
  // loads are unconditional (index clamped to the last observation): no
  // branches around them, so the waitcnt pass can keep them in flight
  auto load_idx = [&](int o, int& c, int& p, float2& uv) {
    const int oc = min(o, P.no - 1);
    c = P.obs_cam[oc]; p = P.obs_pt[oc]; uv = P.uv[oc];
  };
  auto load_pt = [&](int, int p, double (&X)[3], uint8_t& pv) {
    X[0] = pts[3 * p]; X[1] = pts[3 * p + 1]; X[2] = pts[3 * p + 2]; pv = P.pt_var[p];
  };
  // pipeline: chunk i computes while the point data of chunk i+2 and the
  // indices of chunk i+3 are in flight (loads queue behind the store bursts
  // of all waves of the CU: several microseconds under load)
  int c, p, c1, p1, c2, p2;
  float2 uv, uv1, uv2;
  double X[3], X1[3];
  uint8_t pv, pv1;
  load_idx(base + lane, c, p, uv);
  load_idx(base + step + lane, c1, p1, uv1);
  load_idx(base + 2 * step + lane, c2, p2, uv2);
  load_pt(base + lane, p, X, pv);
  load_pt(base + step + lane, p1, X1, pv1);
  init();
  // compact-record cameras are prefetched one chunk ahead; table cameras are
  // read at use (their index is all that travels)
  constexpr bool kPre = std::is_same<CamOf, CamRcOf>::value;
  auto q = cam_pre(cam_of, kPre ? c : 0);
  for (; base < P.no; base += step) {
    const int o = base + lane;
    double X2[3];
    uint8_t pv2;
    load_pt(o + 2 * step, p2, X2, pv2);
    int c3, p3;
    float2 uv3;
    load_idx(o + 3 * step, c3, p3, uv3);
    const auto qn = cam_pre(cam_of, kPre ? c1 : 0);
    double out[kJR];
    if (MODE == 4) {   // loads only
      acc[0] += X[0] + X[1] + X[2] + uv.x + pv + c;
      c = c1; p = p1; uv = uv1;
      c1 = c2; p1 = p2; uv1 = uv2;
      c2 = c3; p2 = p3; uv2 = uv3;
      X[0] = X1[0]; X[1] = X1[1]; X[2] = X1[2]; pv = pv1;
      X1[0] = X2[0]; X1[1] = X2[1]; X1[2] = X2[2]; pv1 = pv2;
      q = qn;
      continue;
    }
    {
      const bool live = o < P.no;
      const auto cam = [&] {
        if constexpr (kPre) return cam_make(cam_of, q);
        else return cam_of(c);
      }();
      if constexpr (MODE == 2) {
        const auto T = cam_row(cam);
        double sum = X[0] + uv.x;
#pragma unroll
        for (int k = 0; k < kLin; ++k) sum += T[k];
#pragma unroll
        for (int k = 0; k < kJR; ++k) out[k] = sum + k;
      } else if constexpr (MODE >= 5) {   // arithmetic only: no stage, no stores
        bool fin;
        const auto cam2 = cam_of(MODE == 6 ? 1 : c);
        const double rho = lin_obs(P, cam2, cam2.var(), pv != 0, X[0], X[1], X[2], uv, out, fin);
        double sum = 0.0;
#pragma unroll
        for (int k = 0; k < kJR; ++k) sum += out[k];
        if (live) { acc[0] += 0.5 * rho; acc[1] += sum; }
      } else {
        bool fin;
        const double rho = lin_obs(P, cam, cam.var(), pv != 0, X[0], X[1], X[2], uv, out, fin);
        if (live) { acc[0] += 0.5 * rho; acc[1] += fin ? 0.0 : 1.0; }
      }
    }
    if constexpr (MODE >= 5) {
      c = c1; p = p1; uv = uv1;
      c1 = c2; p1 = p2; uv1 = uv2;
      c2 = c3; p2 = p3; uv2 = uv3;
      X[0] = X1[0]; X[1] = X1[1]; X[2] = X1[2]; pv = pv1;
      X1[0] = X2[0]; X1[1] = X2[1]; X1[2] = X2[2]; pv1 = pv2;
      q = qn;
      continue;
    }
    const int nrec = min(64, P.no - base);
    double2* dA = reinterpret_cast<double2*>(JR) + (size_t)(JA / 2) * base;
    double2* dB = reinterpret_cast<double2*>(JR + (size_t)JA * P.no) + (size_t)(kJB / 2) * base;
#pragma unroll
    for (int h = 0; h < 64 / ROWS; ++h) {
      // all LDS reads into distinct registers first, then the stores: a
      // store's data registers may not be overwritten before it completes
      // (the waitcnt pass inserts vmcnt(0)), so reusing one register
      // quadruple per store serialises the stores
      if (ROWS == 64 || (lane >= h * ROWS && lane < (h + 1) * ROWS)) {
        double* row = stage + (lane - h * ROWS) * kStageLd;
#pragma unroll
        for (int k = 0; k < kJR; ++k) row[k] = out[k];
      }
      wave_lds_sync();
      // JA: ROWS * JA/2 double2 (JA = 14 with ROWS = 32: the last wave load is half used)
      constexpr int EA = ROWS * (JA / 2), NA = (EA + 63) / 64, NB = ROWS * (kJB / 2) / 64;
      double2 va[NA], vb[NB];
#pragma unroll
      for (int it = 0; it < NA; ++it) {
        const int e = min(it * 64 + lane, EA - 1), r = e / (JA / 2), f = ja_field(2 * (e - r * (JA / 2)));
        va[it] = make_double2(stage[r * kStageLd + f], stage[r * kStageLd + f + 1]);
      }
#pragma unroll
      for (int it = 0; it < NB; ++it) {
        const int e = it * 64 + lane, r = e / (kJB / 2), f = kFJB + 2 * (e - r * (kJB / 2));
        vb[it] = make_double2(stage[r * kStageLd + f], stage[r * kStageLd + f + 1]);
      }
      wave_lds_sync();
      double2* dAh = dA + h * ROWS * (JA / 2);
      double2* dBh = dB + h * ROWS * (kJB / 2);
      if (MODE == 1) {
#pragma unroll
        for (int it = 0; it < NA; ++it)
          if (va[it].x == 1234.5678) dAh[it * 64 + lane] = va[it];
#pragma unroll
        for (int it = 0; it < NB; ++it)
          if (vb[it].x == 1234.5678) dBh[it * 64 + lane] = vb[it];
      } else if (h * ROWS + ROWS <= nrec) {   // full: unconditional stores
#pragma unroll
        for (int it = 0; it < NA; ++it)
          if (EA % 64 == 0 || it * 64 + lane < EA) nt_store(&dAh[it * 64 + lane], va[it]);
#pragma unroll
        for (int it = 0; it < NB; ++it) nt_store(&dBh[it * 64 + lane], vb[it]);
      } else {
#pragma unroll
        for (int it = 0; it < NA; ++it) {
          const int e = it * 64 + lane;
          if (e < EA && h * ROWS + e / (JA / 2) < nrec) dAh[e] = va[it];
        }
#pragma unroll
        for (int it = 0; it < NB; ++it) {
          const int e = it * 64 + lane;
          if (h * ROWS + e / (kJB / 2) < nrec) dBh[e] = vb[it];
        }
      }
    }
    c = c1; p = p1; uv = uv1;
    c1 = c2; p1 = p2; uv1 = uv2;
    c2 = c3; p2 = p3; uv2 = uv3;
    X[0] = X1[0]; X[1] = X1[1]; X[2] = X1[2]; pv = pv1;
    X1[0] = X2[0]; X1[1] = X2[1]; X1[2] = X2[2]; pv1 = pv2;
    q = qn;
  }
}

__global__ __launch_bounds__(256) void k_linearize_rc(DevProblem P, const double* __restrict__ crec,
                                                      const double* __restrict__ pts, double* __restrict__ JR,
                                                      double* __restrict__ part) {
  __shared__ double lds[2 * 16];
  __shared__ double stage[4 * 64 * kStageLd];
  double acc[2] = {0.0, 0.0};  // cost, bad
  lin_waves<jr_ja(true), 4, 64>(P, pts, JR, stage, CamRcOf{crec, P.extr}, acc);
  double tot[2];
  block_sum<2>(acc, lds, tot);
  if (threadIdx.x == 0) {
    part_of(part, SL_COST)[blockIdx.x] = tot[0];
    part_of(part, SL_LIN_BAD)[blockIdx.x] = tot[1];
  }
}

// Small camera sets (nc <= kLinLdsCams): the whole camera table lives in
// LDS, so the per-observation camera gathers hit LDS instead of the texture
// path (the gathers, 24 x 16 B per lane from random cameras, saturate the
// TA: measured 46 % issue stalls).  One 512-thread block per CU.
constexpr int kLinLdsThreads = 512;
constexpr int kLinLdsCams = kLinLdsCamsHost;
// Camera table -> LDS, every global load of the fill issued before the
// first LDS store (one round trip; an element-wise loop serialises ~16 L2
// round trips in the block prologue).
template <int NT>
__device__ inline void fill_lin_table(const DevProblem& P, const double* __restrict__ rec, double* tbl, float* ktb) {
  constexpr int kPer2 = (kLinLdsCams * (kLin / 2) + NT - 1) / NT;
  constexpr int kPerK = (kLinLdsCams * 9 + NT - 1) / NT;
  const int n2 = P.nc * (kLin / 2), nk = P.nc * 9;
  double2 v[kPer2];
  float kv[kPerK];
  // unconditional loads (clamped indices): a load under a branch gets its
  // own vmcnt(0) wait
#pragma unroll
  for (int i = 0; i < kPer2; ++i) {
    const int e = min((int)threadIdx.x + i * NT, n2 - 1);
    const int c = e / (kLin / 2), k2 = e - c * (kLin / 2);
    v[i] = reinterpret_cast<const double2*>(rec + (size_t)c * kCamRec + kRecL)[k2];
  }
#pragma unroll
  for (int i = 0; i < kPerK; ++i) kv[i] = P.K[min((int)threadIdx.x + i * NT, nk - 1)];   // float-valued (Matrix3f)
  const int c0 = threadIdx.x;
  const double flag = P.vc[min(c0, P.nc - 1)] >= 0 ? 1.0 : 0.0;
#pragma unroll
  for (int i = 0; i < kPer2; ++i) {
    const int e = threadIdx.x + i * NT;
    if (e < n2) {
      const int c = e / (kLin / 2), k2 = e - c * (kLin / 2);
      reinterpret_cast<double2*>(tbl + c * kTblRec)[k2] = v[i];
    }
  }
#pragma unroll
  for (int i = 0; i < kPerK; ++i) {
    const int e = threadIdx.x + i * NT;
    if (e < nk) ktb[e] = kv[i];
  }
  if (c0 < P.nc) { tbl[c0 * kTblRec + kLin] = flag; tbl[c0 * kTblRec + kLin + 1] = 0.0; }
  __syncthreads();
}

// NT threads per block (one block per CU: the camera table fills most of
// the LDS), stage rows ROWS per wave.
// HOOK: the table fill runs after the first chunks' loads are issued
template <int NT, int ROWS, int MODE = 0, bool HOOK = false>
__global__ __launch_bounds__(NT) void k_linearize_lds_t(DevProblem P, const double* __restrict__ rec,
                                                        const double* __restrict__ pts, double* __restrict__ JR,
                                                        double* __restrict__ part) {
  __shared__ double lds[2 * 16];
  __shared__ double stage[(NT / 64) * ROWS * kStageLd];
  __shared__ __attribute__((aligned(16))) double tbl[kLinLdsCams * kTblRec];
  __shared__ float ktb[kLinLdsCams * 9];
  if (!HOOK) fill_lin_table<NT>(P, rec, tbl, ktb);
  double acc[2] = {0.0, 0.0};
  auto cam_of = [&](int c) { return CamLds{tbl + c * kTblRec, ktb + c * 9}; };
  auto init = [&] { if (HOOK) fill_lin_table<NT>(P, rec, tbl, ktb); };
  if (MODE != 3) lin_waves<jr_ja(false), NT / 64, ROWS, decltype(cam_of), MODE>(P, pts, JR, stage, cam_of, acc, init);
  double tot[2];
  block_sum<2>(acc, lds, tot);
  if (threadIdx.x == 0) {
    part_of(part, SL_COST)[blockIdx.x] = tot[0];
    part_of(part, SL_LIN_BAD)[blockIdx.x] = tot[1];
  }
}
#ifndef BA_LIN_ROWS
#define BA_LIN_ROWS 64
#endif
constexpr int kLinNT = 512, kLinRows = BA_LIN_ROWS;    // product configuration (tools/lin_probe.hip)

// ---------------------------------------------------------------------------
// point blocks: Hpp (xx,xy,xz,yy,yz,zz), gp, jacobi scale, LM diagonal, norms
// ---------------------------------------------------------------------------
// kPaLanes lanes per point: lane l of the group sums observations o0 + l,
// o0 + l + kPaLanes, ... (adjacent lanes read adjacent 64-B JB records, one
// 256-B segment per load instruction and group), then a fixed-order xor
// reduction inside the group; lane 0 of the group finishes the point.
constexpr int kPaLanes = 4;
template <int JA>
__global__ __launch_bounds__(256) void k_point_assemble(DevProblem P, const double* __restrict__ JR,
                                                        const double* __restrict__ pts, double* __restrict__ Hpp,
                                                        double* __restrict__ gp, double* __restrict__ scale_p,
                                                        double* __restrict__ diag_p, int compute_scale,
                                                        double min_diag, double max_diag, double* __restrict__ part) {
  __shared__ double lds[3 * 16];
  double acc[2] = {0.0, 0.0};  // gn2, xn2
  double gmax = 0.0;
  const size_t np = (size_t)P.np;
  const int sl = threadIdx.x & (kPaLanes - 1);
  const int g0 = (blockIdx.x * blockDim.x + threadIdx.x) / kPaLanes, gs = gridDim.x * blockDim.x / kPaLanes;
  for (int p = g0; p < P.np; p += gs) {      // uniform inside a lane group
    if (!P.pt_var[p]) continue;
    double H[6] = {0, 0, 0, 0, 0, 0}, g[3] = {0, 0, 0};
    const int o0 = P.pt_off[p], o1 = P.pt_off[p + 1];
    for (int o = o0 + sl; o < o1; o += kPaLanes) {
      const double2* s = reinterpret_cast<const double2*>(jr_b<JA>(JR, P.no, o));
      const double2 t0 = s[0], t1 = s[1], t2 = s[2], t3 = s[3];
      const double jp[2][3] = {{t0.x, t0.y, t1.x}, {t1.y, t2.x, t2.y}};
      const double rr[2] = {t3.x, t3.y};
#pragma unroll
      for (int row = 0; row < 2; ++row) {
        const double a = jp[row][0], b = jp[row][1], c = jp[row][2];
        H[0] += a * a; H[1] += a * b; H[2] += a * c; H[3] += b * b; H[4] += b * c; H[5] += c * c;
        g[0] += a * rr[row]; g[1] += b * rr[row]; g[2] += c * rr[row];
      }
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) {
#pragma unroll
      for (int x = kPaLanes / 2; x >= 1; x >>= 1) H[k] += __shfl_xor(H[k], x, kPaLanes);
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
#pragma unroll
      for (int x = kPaLanes / 2; x >= 1; x >>= 1) g[k] += __shfl_xor(g[k], x, kPaLanes);
    }
    if (sl != 0) continue;
#pragma unroll
    for (int k = 0; k < 6; ++k) Hpp[k * np + p] = H[k];
    const double hd[3] = {H[0], H[3], H[5]};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      gp[k * np + p] = g[k];
      double s;
      if (compute_scale) {
        s = 1.0 / (1.0 + sqrt(hd[k]));
        scale_p[k * np + p] = s;
      } else {
        s = scale_p[k * np + p];
      }
      diag_p[k * np + p] = fmin(fmax(hd[k] * s * s, min_diag), max_diag);
      const double x = pts[3 * p + k];
      const double d = x - (x + (-g[k]));
      gmax = fmax(gmax, fabs(d));
      acc[0] += d * d;
      acc[1] += x * x;
    }
  }
  double out[2];
  block_sum<2>(acc, lds, out);
  const double m = block_max1(gmax, lds + 32);
  if (threadIdx.x == 0) {
    part_of(part, SL_GN2_P)[blockIdx.x] = out[0];
    part_of(part, SL_XN2_P)[blockIdx.x] = out[1];
    part_of(part, SL_GMAX_P)[blockIdx.x] = m;
  }
}

// ---------------------------------------------------------------------------
// camera blocks: one workgroup per active variable camera, Hcc (21, lower
// row-major) and gc (6), gathering its observations' records.
// ---------------------------------------------------------------------------
// (one workgroup per camera: splitting it measured slower — the pass is
// bound by the gathered record reads, 256 B fetched per 112 B used)
// Hcc (lower 21) and gc per camera, slice blockIdx.y of its observations;
// two observations in flight per thread (the camera-order index is one load
// ahead of the record gathers)
template <int JA>
__device__ inline void cam_acc_jr(const double* __restrict__ JR, int no, int o, double (&acc)[27]) {
  const double2* s = reinterpret_cast<const double2*>(jr_a<JA>(JR, o));
  double jc[12];
#pragma unroll
  for (int k = 0; k < 6; ++k) { const double2 t = s[k]; jc[2 * k] = t.x; jc[2 * k + 1] = t.y; }
  // JA = 14: the residual copy in the same record, else JB's
  const double2 rt = JA >= 14 ? s[6] : reinterpret_cast<const double2*>(jr_b<JA>(JR, no, o))[3];
  const double rr[2] = {rt.x, rt.y};
#pragma unroll
  for (int row = 0; row < 2; ++row) {
    const double* j = jc + 6 * row;
    int t = 0;
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
      for (int b = 0; b <= a; ++b) acc[t++] += j[a] * j[b];
#pragma unroll
    for (int a = 0; a < 6; ++a) acc[21 + a] += j[a] * rr[row];
  }
}
template <int NT, int JA>
__global__ __launch_bounds__(NT) void k_cam_assemble(DevProblem P, const double* __restrict__ JR,
                                                     double* __restrict__ cpart, double* __restrict__ Hcc,
                                                     double* __restrict__ gc) {
  __shared__ double lds[27 * 16];
  const int v = blockIdx.x;
  double acc[27];
#pragma unroll
  for (int k = 0; k < 27; ++k) acc[k] = 0.0;
  int i0, i1;
  cam_slice(P, v, i0, i1);
  const int bd = blockDim.x;
  for (int i = i0 + threadIdx.x; i < i1; i += 2 * bd) {
    const bool two = i + bd < i1;
    const int oa = P.cam_op[i].x, ob = P.cam_op[two ? i + bd : i].x;
    cam_acc_jr<JA>(JR, P.no, oa, acc);
    if (two) cam_acc_jr<JA>(JR, P.no, ob, acc);
  }
  double out[27];
  block_sum<27>(acc, lds, out);
  if (gridDim.y == 1) {   // one slice per camera: final sums
    if (threadIdx.x == 0) {
#pragma unroll
      for (int k = 0; k < 21; ++k) Hcc[(size_t)v * 21 + k] = out[k];
#pragma unroll
      for (int k = 0; k < 6; ++k) gc[(size_t)v * 6 + k] = out[21 + k];
    }
    return;
  }
  cam_slice_store(out, cpart, v, P.nvc);
}

__device__ inline int tri(int a, int b) { return a * (a + 1) / 2 + b; }  // a >= b

// (bx, nbx: this workgroup's index and the workgroup count of the pass, so
// that the pass can ride in another kernel's launch: k_point_elim_norms)
__device__ __forceinline__ void cam_norms_body(const DevProblem& P, const double* __restrict__ cams,
                                               const double* __restrict__ Hcc, const double* __restrict__ gc,
                                               double* __restrict__ scale_c, double* __restrict__ diag_c,
                                               int compute_scale, double min_diag, double max_diag,
                                               double* __restrict__ part, int bx, int nbx) {
  __shared__ double lds[3 * 16];
  double acc[2] = {0.0, 0.0};
  double gmax = 0.0;
  for (int v = bx * blockDim.x + threadIdx.x; v < P.nvc; v += nbx * blockDim.x) {
    const int c = P.cam_of_vc[v];
    for (int a = 0; a < 6; ++a) {
      const double h = Hcc[(size_t)v * 21 + tri(a, a)];
      double s;
      if (compute_scale) {
        s = 1.0 / (1.0 + sqrt(h));
        scale_c[(size_t)v * 6 + a] = s;
      } else {
        s = scale_c[(size_t)v * 6 + a];
      }
      diag_c[(size_t)v * 6 + a] = fmin(fmax(h * s * s, min_diag), max_diag);
      const double x = cams[6 * c + a], g = gc[(size_t)v * 6 + a];
      const double d = x - (x + (-g));
      gmax = fmax(gmax, fabs(d));
      acc[0] += d * d;
      acc[1] += x * x;
    }
  }
  double out[2];
  block_sum<2>(acc, lds, out);
  const double m = block_max1(gmax, lds + 32);
  if (threadIdx.x == 0) {
    part_of(part, SL_GN2_C)[bx] = out[0];
    part_of(part, SL_XN2_C)[bx] = out[1];
    part_of(part, SL_GMAX_C)[bx] = m;
  }
}
__global__ __launch_bounds__(256) void k_cam_norms(DevProblem P, const double* __restrict__ cams, const double* __restrict__ Hcc,
                                                   const double* __restrict__ gc, double* __restrict__ scale_c,
                                                   double* __restrict__ diag_c, int compute_scale, double min_diag,
                                                   double max_diag, double* __restrict__ part) {
  cam_norms_body(P, cams, Hcc, gc, scale_c, diag_c, compute_scale, min_diag, max_diag, part, blockIdx.x, gridDim.x);
}

// ---------------------------------------------------------------------------
// point elimination: per point (one thread)
//   A = s Hpp s + D^2 (D = sqrt(diag / radius), ceres lm_diagonal_), L L^T = A,
//   store L^-1 and u = L^-1 (s g)
// ---------------------------------------------------------------------------
// prec (optional: the camera-major J-free kernels of a step): one 128-B
// record per point with what k_obs_w_cam / k_cam_schur_diag_rc gather: X, the
// variable flag, s_p, L_p^-1, u_p
constexpr int kPRec = 16;
__device__ __forceinline__ void point_elim_body(const DevProblem& P, const double* __restrict__ Hpp,
                                                const double* __restrict__ gp, const double* __restrict__ scale_p,
                                                const double* __restrict__ diag_p, double radius,
                                                double* __restrict__ Linv, double* __restrict__ u,
                                                double* __restrict__ part, const double* __restrict__ pts,
                                                double* __restrict__ prec, int bx, int nbx) {
  __shared__ double lds[16];
  // prec: the wave's 64 records leave through LDS as contiguous 1 KiB wave
  // stores (a 128-B record per lane is store-issue bound); row stride 17
  __shared__ double pst[(kThreads / 64) * 64 * (kPRec + 1)];
  double acc[1] = {0.0};
  const size_t np = (size_t)P.np;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double* ps = pst + w * 64 * (kPRec + 1);
  for (int pb = bx * blockDim.x; pb < P.np; pb += nbx * blockDim.x) {   // (uniform in the workgroup)
    const int p = pb + threadIdx.x;
    double rv[kPRec];
    if (p < P.np && !P.pt_var[p]) {   // zeros: the camera-side gathers then need no point flag (W_o = 0 there too)
#pragma unroll
      for (int k = 0; k < 6; ++k) Linv[k * np + p] = 0.0;
#pragma unroll
      for (int k = 0; k < 4; ++k) u[4 * (size_t)p + k] = 0.0;
      if (prec) {
        rv[0] = pts[3 * (size_t)p]; rv[1] = pts[3 * (size_t)p + 1]; rv[2] = pts[3 * (size_t)p + 2];
#pragma unroll
        for (int k = 3; k < kPRec; ++k) rv[k] = 0.0;
      }
    } else if (p < P.np) {
      double s[3], D2[3], gs[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        s[k] = scale_p[k * np + p];
        const double D = sqrt(diag_p[k * np + p] / radius);
        D2[k] = D * D;
        gs[k] = gp[k * np + p] * s[k];
      }
      const double h00 = Hpp[0 * np + p] * s[0] * s[0] + D2[0];
      const double h10 = Hpp[1 * np + p] * s[0] * s[1];
      const double h20 = Hpp[2 * np + p] * s[0] * s[2];
      const double h11 = Hpp[3 * np + p] * s[1] * s[1] + D2[1];
      const double h21 = Hpp[4 * np + p] * s[1] * s[2];
      const double h22 = Hpp[5 * np + p] * s[2] * s[2] + D2[2];
      bool ok = h00 > 0.0;
      const double l00 = sqrt(h00);
      const double l10 = h10 / l00, l20 = h20 / l00;
      const double d11 = h11 - l10 * l10;
      ok = ok && d11 > 0.0;
      const double l11 = sqrt(d11);
      const double l21 = (h21 - l20 * l10) / l11;
      const double d22 = h22 - l20 * l20 - l21 * l21;
      ok = ok && d22 > 0.0;
      const double l22 = sqrt(d22);
      const double i00 = 1.0 / l00, i11 = 1.0 / l11, i22 = 1.0 / l22;
      const double i10 = -(l10 * i00) * i11;
      const double i21 = -(l21 * i11) * i22;
      const double i20 = -(l20 * i00 + l21 * i10) * i22;
      Linv[0 * np + p] = i00; Linv[1 * np + p] = i10; Linv[2 * np + p] = i11;
      Linv[3 * np + p] = i20; Linv[4 * np + p] = i21; Linv[5 * np + p] = i22;
      // u AoS [np][4] (one 32-B sector per point for the camera-side gathers)
      const double u0 = i00 * gs[0];
      const double u1 = i10 * gs[0] + i11 * gs[1];
      const double u2 = i20 * gs[0] + i21 * gs[1] + i22 * gs[2];
      u[4 * (size_t)p + 0] = u0;
      u[4 * (size_t)p + 1] = u1;
      u[4 * (size_t)p + 2] = u2;
      u[4 * (size_t)p + 3] = 0.0;
      if (prec) {
        rv[0] = pts[3 * (size_t)p]; rv[1] = pts[3 * (size_t)p + 1]; rv[2] = pts[3 * (size_t)p + 2]; rv[3] = 1.0;
        rv[4] = s[0]; rv[5] = s[1]; rv[6] = s[2]; rv[7] = i00;
        rv[8] = i10; rv[9] = i11; rv[10] = i20; rv[11] = i21;
        rv[12] = i22; rv[13] = u0; rv[14] = u1; rv[15] = u2;
      }
      acc[0] += ok ? 0.0 : 1.0;
    }
    if (prec) {   // (uniform)
      if (p < P.np) {
#pragma unroll
        for (int k = 0; k < kPRec; ++k) ps[lane * (kPRec + 1) + k] = rv[k];
      }
      wave_lds_sync();
      const int p0 = pb + w * 64;   // the wave's first point
      const int nrec = min(64, P.np - p0);
      double2* dst = reinterpret_cast<double2*>(prec + (size_t)max(p0, 0) * kPRec);
#pragma unroll
      for (int it = 0; it < kPRec / 2; ++it) {
        const int e = it * 64 + lane, r = e >> 3, f = 2 * (e & 7);
        if (r < nrec) dst[e] = make_double2(ps[r * (kPRec + 1) + f], ps[r * (kPRec + 1) + f + 1]);
      }
      wave_lds_sync();
    }
  }
  double out[1];
  block_sum<1>(acc, lds, out);
  if (threadIdx.x == 0) part_of(part, SL_ELIM_BAD)[bx] = out[0];
}
__global__ __launch_bounds__(256) void k_point_elim(DevProblem P, const double* __restrict__ Hpp,
                                                    const double* __restrict__ gp, const double* __restrict__ scale_p,
                                                    const double* __restrict__ diag_p, double radius,
                                                    double* __restrict__ Linv, double* __restrict__ u,
                                                    double* __restrict__ part, const double* __restrict__ pts,
                                                    double* __restrict__ prec) {
  point_elim_body(P, Hpp, gp, scale_p, diag_p, radius, Linv, u, part, pts, prec, blockIdx.x, gridDim.x);
}
// k_point_elim with the camera-side norms of the linearisation it follows
// (k_cam_norms) as the first workgroups of the same launch (dispatched
// first: the norms' serial camera loop runs beside the points): the two
// passes share no data (point blocks vs camera blocks, distinct scalar
// slots), and the norms' slots are folded only with the step's scalars
// (single rank, deferred fold).  One ~6-us launch fewer per LM iteration;
// each workgroup runs exactly the arithmetic of its separate launch.
__global__ __launch_bounds__(256) void k_point_elim_norms(DevProblem P, const double* __restrict__ Hpp,
                                                          const double* __restrict__ gp,
                                                          const double* __restrict__ scale_p,
                                                          const double* __restrict__ diag_p, double radius,
                                                          double* __restrict__ Linv, double* __restrict__ u,
                                                          double* __restrict__ part, const double* __restrict__ pts,
                                                          double* __restrict__ prec, int nbp, NormsFold nf) {
  const int nbn = (int)gridDim.x - nbp;
  if ((int)blockIdx.x < nbn)
    cam_norms_body(P, nf.cams, nf.Hcc, nf.gc, nf.scale_c, nf.diag_c, nf.compute_scale, nf.min_diag, nf.max_diag, part,
                   blockIdx.x, nbn);
  else
    point_elim_body(P, Hpp, gp, scale_p, diag_p, radius, Linv, u, part, pts, prec, blockIdx.x - nbn, nbp);
}

// ---------------------------------------------------------------------------
// W per observation with a variable camera and a variable point:
//   W_o = diag(s_c) Jc^T Jp diag(s_p) L_p^-T     (6x3, AoS [no][18])
// Wave-private chunks of 64 observations: the chunk's JR records arrive as
// 10 contiguous 1 KiB wave loads through the wave's LDS slot, the 64 W
// records leave as 9 contiguous 1 KiB wave stores through the same slot
// (row-per-lane 144-B stores are store-issue bound: tools/hbm_probe.hip).
// Camera scales come from an LDS table (nc <= kLinLdsCams) or global.
// ---------------------------------------------------------------------------
constexpr int kWRec = 18;
template <bool TBL, typename WT>
__global__ __launch_bounds__(512) void k_obs_w(DevProblem P, const double* __restrict__ JR,
                                               const double* __restrict__ scale_c, const double* __restrict__ scale_p,
                                               const double* __restrict__ Linv, WT* __restrict__ W) {
  using V2 = typename std::conditional<sizeof(WT) == 8, double2, float2>::type;
  constexpr int WAVES = 8;
  constexpr int JA = jr_ja(!TBL);
  __shared__ double stage[WAVES * 64 * kStageLd];
  __shared__ double sct[TBL ? kLinLdsCams * 6 : 1];
  if (TBL) {
    for (int e = threadIdx.x; e < P.nc * 6; e += 512) {
      const int c = e / 6, a = e - 6 * c;
      const int v = P.vc[c];
      sct[e] = v >= 0 ? scale_c[(size_t)v * 6 + a] : 0.0;
    }
    __syncthreads();
  }
  // Required before the prologue below: it issues loads at indices clamped to
  // P.no - 1 (obs_cam, the JR chunk, the factors), which are out of bounds
  // (index -1) for a rank shard without observations.
  if (P.no == 0) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double* st = stage + w * (64 * kStageLd);
  const int step = gridDim.x * WAVES * 64;
  const size_t np = (size_t)P.np;
  // pipeline (every load unconditional, indices clamped): the indices of
  // chunk i+2 and the JR records + per-camera / per-point factors of chunk
  // i+1 are in flight while chunk i computes (issued at use, each chunk waited
  // for its index -> camera -> scale chain)
  struct Fac {
    double sc[6], sp[3], li[6];
    bool live;
  };
  auto load_idx = [&](int b, int& c, int& p) {
    const int oc = min(b + lane, P.no - 1);
    c = P.obs_cam[oc]; p = P.obs_pt[oc];
  };
  auto load_fac = [&](int b, int c, int p, Fac& f) {
    const int v = P.vc[c];
    f.live = b + lane < P.no && v >= 0 && P.pt_var[p];
#pragma unroll
    for (int a = 0; a < 6; ++a) f.sc[a] = TBL ? sct[c * 6 + a] : scale_c[(size_t)max(v, 0) * 6 + a];
#pragma unroll
    for (int k = 0; k < 3; ++k) f.sp[k] = scale_p[k * np + p];
#pragma unroll
    for (int k = 0; k < 6; ++k) f.li[k] = Linv[k * np + p];
  };
  int base = (blockIdx.x * WAVES + w) * 64;
  int ci0, pi0, ci1, pi1;
  load_idx(base, ci0, pi0);
  load_idx(base + step, ci1, pi1);
  double2 t[JA / 2 + kJB / 2];
  jr_chunk_load<JA>(JR, P.no, min(base, P.no - 1), lane, t);
  Fac fc;
  load_fac(base, ci0, pi0, fc);
  for (; base < P.no; base += step) {
    const int nb = base + step;
    int ci2, pi2;
    load_idx(nb + step, ci2, pi2);
    double2 tn[JA / 2 + kJB / 2];
    jr_chunk_load<JA>(JR, P.no, min(nb, P.no - 1), lane, tn);
    Fac fn;
    load_fac(nb, ci1, pi1, fn);
    const bool live = fc.live;
    double sc[6];
#pragma unroll
    for (int a = 0; a < 6; ++a) sc[a] = fc.sc[a];
    const double s0 = fc.sp[0], s1 = fc.sp[1], s2 = fc.sp[2];
    const double i00 = fc.li[0], i10 = fc.li[1], i11 = fc.li[2];
    const double i20 = fc.li[3], i21 = fc.li[4], i22 = fc.li[5];
    jr_chunk_stage<JA>(st, lane, t);
    wave_lds_sync();
    double j[18];
#pragma unroll
    for (int k = 0; k < 18; ++k) j[k] = st[lane * kStageLd + k];
    wave_lds_sync();
    const double jp0[3] = {j[12] * s0, j[13] * s1, j[14] * s2};
    const double jp1[3] = {j[15] * s0, j[16] * s1, j[17] * s2};
    double wv[18];
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      const double c0 = j[a] * sc[a], c1 = j[6 + a] * sc[a];
      const double e0 = c0 * jp0[0] + c1 * jp1[0];
      const double e1 = c0 * jp0[1] + c1 * jp1[1];
      const double e2 = c0 * jp0[2] + c1 * jp1[2];
      wv[a * 3 + 0] = live ? e0 * i00 : 0.0;
      wv[a * 3 + 1] = live ? e0 * i10 + e1 * i11 : 0.0;
      wv[a * 3 + 2] = live ? e0 * i20 + e1 * i21 + e2 * i22 : 0.0;
    }
#pragma unroll
    for (int k = 0; k < kWRec; ++k) st[lane * kStageLd + k] = wv[k];
    wave_lds_sync();
    constexpr int NIT = kWRec / 2;   // 9 x 1 KiB (fp64) / 9 x 512 B (fp32)
    V2 ov[NIT];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int e = it * 64 + lane;
      const int r = e / (kWRec / 2), f = 2 * (e - r * (kWRec / 2));
      ov[it].x = (WT)st[r * kStageLd + f];
      ov[it].y = (WT)st[r * kStageLd + f + 1];
    }
    wave_lds_sync();
    V2* dst = reinterpret_cast<V2*>(W + (size_t)base * kWRec);
    const int nrec = min(64, P.no - base);
    if (nrec == 64) {
#pragma unroll
      for (int it = 0; it < NIT; ++it) nt_store(&dst[it * 64 + lane], ov[it]);
    } else {
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        const int e = it * 64 + lane;
        if (e / (kWRec / 2) < nrec) dst[e] = ov[it];
      }
    }
#pragma unroll
    for (int k = 0; k < JA / 2 + kJB / 2; ++k) t[k] = tn[k];
    fc = fn;
    ci1 = ci2; pi1 = pi2;
  }
}

// ---------------------------------------------------------------------------
// back-substitution, kPtLanes lanes per point (all points; fixed / unobserved
// points keep x' = x):  y_p = L^-T (u_p - sum W_o^T y_c) ; d_p = s_p (-y_p)
// ---------------------------------------------------------------------------
template <typename WT>
__global__ __launch_bounds__(256) void k_backsub(DevProblem P, const double* __restrict__ pts,
                                                 double* __restrict__ pts_c, double* __restrict__ delta_p,
                                                 const WT* __restrict__ W, const double* __restrict__ u,
                                                 const double* __restrict__ Linv, const double* __restrict__ y,
                                                 const double* __restrict__ scale_p, double* __restrict__ part) {
  __shared__ double lds[2 * 16];
  double acc[2] = {0.0, 0.0};  // step2, step_bad (lane 0 of each point group)
  const size_t np = (size_t)P.np;
  const int gl = threadIdx.x & (kPtLanes - 1), gpb = blockDim.x / kPtLanes;
  for (int p = blockIdx.x * gpb + threadIdx.x / kPtLanes; p < P.np; p += gridDim.x * gpb) {
    // kPtLanes lanes per point (point_wtx); fixed cameras carry W_o = 0
    double wy[3] = {0.0, 0.0, 0.0};
    const bool var = P.pt_var[p];
    if (var) point_wtx<false>(W, P.obs_vc, y, P.pt_off[p], P.pt_off[p + 1], gl, wy);
    if (gl != 0) continue;
    const double X[3] = {pts[3 * p], pts[3 * p + 1], pts[3 * p + 2]};
    double dX[3] = {0.0, 0.0, 0.0}, Xc[3] = {X[0], X[1], X[2]};
    if (var) {
      const double w[3] = {u[4 * p] - wy[0], u[4 * p + 1] - wy[1], u[4 * p + 2] - wy[2]};
      const double i00 = Linv[0 * np + p], i10 = Linv[1 * np + p], i11 = Linv[2 * np + p];
      const double i20 = Linv[3 * np + p], i21 = Linv[4 * np + p], i22 = Linv[5 * np + p];
      const double yp[3] = {i00 * w[0] + i10 * w[1] + i20 * w[2], i11 * w[1] + i21 * w[2], i22 * w[2]};
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        dX[k] = (-yp[k]) * scale_p[k * np + p];
        Xc[k] = X[k] + dX[k];
        const double e = X[k] - Xc[k];
        acc[0] += e * e;
        if (!isfinite(dX[k])) acc[1] += 1.0;
      }
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) { pts_c[3 * p + k] = Xc[k]; delta_p[3 * p + k] = dX[k]; }
  }
  double out[2];
  block_sum<2>(acc, lds, out);
  if (threadIdx.x == 0) {
    part_of(part, SL_STEP2_P)[blockIdx.x] = out[0];
    part_of(part, SL_STEP_BAD)[blockIdx.x] += out[1];
  }
}

// ---------------------------------------------------------------------------
// model cost change + candidate cost, one lane per observation:
//   Jd = Jc d_c + Jp d_p ; m += Jd.(r + Jd/2)    (model_cost_change = -sum m)
//   candidate residual at (camera', X') -> Huber cost
// ---------------------------------------------------------------------------
// Same with the camera table (value-only candidate records + the camera
// step) and the observation records staged in LDS: the JR records of a
// chunk are read with contiguous 16-B-per-lane loads, the per-observation
// camera data comes from LDS (nc <= kLinLdsCams).
constexpr int kCandRec = 22;   // R (9) t (3) | extrinsic (16); camera step (6) at 16..21
// entry e of the candidate camera table (value-only records + the step)
__device__ inline double cand_entry(const DevProblem& P, const double* __restrict__ rec_c,
                                    const double* __restrict__ delta_c, int e) {
  const int c = e / kCandRec, k = e - c * kCandRec;
  const bool fixed = P.cam_fixed && P.cam_fixed[c];
  const int vc = P.vc[c];
  const double* src;
  bool zero = false;
  if (k < 16) {
    src = rec_c + (size_t)c * kCamRec + (fixed ? k : (k < 9 ? kRecR + k : kRecT + min(k - 9, 2)));
    zero = !fixed && k >= 12;
  } else {
    src = delta_c + (size_t)max(vc, 0) * 6 + (k - 16);
    zero = vc < 0;
  }
  const double x = *src;
  return zero ? 0.0 : x;
}
// the same table in global memory for nc > kLinLdsCams (176 B per camera:
// L2-resident up to ~20k cameras, where the 704-B records are not)
__global__ __launch_bounds__(256) void k_cand_table(DevProblem P, const double* __restrict__ rec_c,
                                                    const double* __restrict__ delta_c, double* __restrict__ tbl) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < P.nc * kCandRec) tbl[e] = cand_entry(P, rec_c, delta_c, e);
}
// NT threads per block; GTBL: camera table in global memory (gtbl, K = P.K),
// else filled into LDS (nc <= kLinLdsCams)
template <int NT, bool GTBL>
__global__ __launch_bounds__(NT) void k_candidate_lds(DevProblem P, const double* __restrict__ JR,
                                                      const double* __restrict__ delta_c,
                                                      const double* __restrict__ delta_p,
                                                      const double* __restrict__ rec_c,
                                                      const double* __restrict__ pts_c, const double* __restrict__ gtbl,
                                                      double* __restrict__ part) {
  constexpr int JA = jr_ja(GTBL);
  __shared__ double lds[3 * 16];
  __shared__ double stage[NT * kStageLd];
  __shared__ double tbl_s[GTBL ? 1 : kLinLdsCams * kCandRec];
  __shared__ float ktb_s[GTBL ? 1 : kLinLdsCams * 9];
  const double* tbl;
  const float* ktb;
  if constexpr (GTBL) {
    tbl = gtbl;
    ktb = P.K;
  } else {  // camera table: every load issued before the first LDS store (clamped, unconditional)
    constexpr int kPer = (kLinLdsCams * kCandRec + NT - 1) / NT;
    constexpr int kPerK = (kLinLdsCams * 9 + NT - 1) / NT;
    const int n = P.nc * kCandRec, nk = P.nc * 9;
    double v[kPer];
    float kv[kPerK];
#pragma unroll
    for (int i = 0; i < kPer; ++i) v[i] = cand_entry(P, rec_c, delta_c, min((int)threadIdx.x + i * NT, n - 1));
#pragma unroll
    for (int i = 0; i < kPerK; ++i) kv[i] = P.K[min((int)threadIdx.x + i * NT, nk - 1)];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = threadIdx.x + i * NT;
      if (e < n) tbl_s[e] = v[i];
    }
#pragma unroll
    for (int i = 0; i < kPerK; ++i) {
      const int e = threadIdx.x + i * NT;
      if (e < nk) ktb_s[e] = kv[i];
    }
    tbl = tbl_s;
    ktb = ktb_s;
  }
  __syncthreads();   // table ready
  double acc[3] = {0.0, 0.0, 0.0};  // mneg, ccost, cand_bad
  // wave-private chunks of 64 observations: the chunk's 64 records are read
  // as 10 contiguous 1 KiB wave loads (one chunk ahead) into the wave's LDS
  // slot, then each lane consumes its own record (no workgroup barrier).
  // Loads are unconditional with clamped indices (no waitcnt drains).
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int WAVES = NT / 64;
  double* st = stage + w * (64 * kStageLd);
  const int step = gridDim.x * WAVES * 64;
  int base = (blockIdx.x * WAVES + w) * 64;
  if (P.no == 0) base = P.no;
  double2 t[JA / 2 + kJB / 2];
  int c = 0, p = 0;
  float2 uv = make_float2(0.f, 0.f);
  // GTBL: the lane's camera record (176 B, 16-B aligned) and K are gathered
  // one chunk ahead into registers, beside the next chunk's JR loads (read at
  // use, each chunk waited one L2 round trip for them)
  struct CandCam {
    double2 r[kCandRec / 2];
    float k[9];
  };
  auto cam_load = [&](int cc, CandCam& q) {
    if constexpr (GTBL) {
      const double2* s2 = reinterpret_cast<const double2*>(tbl + (size_t)cc * kCandRec);
#pragma unroll
      for (int i = 0; i < kCandRec / 2; ++i) q.r[i] = s2[i];
#pragma unroll
      for (int i = 0; i < 9; ++i) q.k[i] = ktb[(size_t)cc * 9 + i];
    }
  };
  CandCam cq;
  if (base < P.no) {
    jr_chunk_load<JA>(JR, P.no, base, lane, t);
    const int oc = min(base + lane, P.no - 1);
    c = P.obs_cam[oc]; p = P.obs_pt[oc]; uv = P.uv[oc];
    cam_load(c, cq);
  }
  for (; base < P.no; base += step) {
    const int o = base + lane;
    // stage this chunk's records
    jr_chunk_stage<JA>(st, lane, t);
    const double dp0 = delta_p[3 * p], dp1 = delta_p[3 * p + 1], dp2 = delta_p[3 * p + 2];
    const double X0 = pts_c[3 * p], X1 = pts_c[3 * p + 1], X2 = pts_c[3 * p + 2];
    const bool cfix = P.cam_fixed && P.cam_fixed[c];
    // next chunk's records and indices (in flight during this chunk)
    const int nb = base + step;
    int cn = c, pn = p;
    float2 uvn = uv;
    CandCam cqn;
    if (nb < P.no) {
      jr_chunk_load<JA>(JR, P.no, nb, lane, t);
      const int oc = min(nb + lane, P.no - 1);
      cn = P.obs_cam[oc]; pn = P.obs_pt[oc]; uvn = P.uv[oc];
      cam_load(cn, cqn);
    }
    wave_lds_sync();
    {
      const double* j = st + lane * kStageLd;
      double crv[GTBL ? kCandRec : 1];
      if constexpr (GTBL) {
#pragma unroll
        for (int i = 0; i < kCandRec / 2; ++i) { crv[2 * i] = cq.r[i].x; crv[2 * i + 1] = cq.r[i].y; }
      }
      const double* cr = GTBL ? crv : tbl + c * kCandRec;
      double jd0 = 0.0, jd1 = 0.0;
#pragma unroll
      for (int a2 = 0; a2 < 6; ++a2) { jd0 += j[a2] * cr[16 + a2]; jd1 += j[6 + a2] * cr[16 + a2]; }
      jd0 += j[12] * dp0 + j[13] * dp1 + j[14] * dp2;
      jd1 += j[15] * dp0 + j[16] * dp1 + j[17] * dp2;
      const double mneg = jd0 * (j[18] + jd0 / 2.0) + jd1 * (j[19] + jd1 / 2.0);
      double pc[3];
      if (!cfix) {
#pragma unroll
        for (int i = 0; i < 3; ++i) pc[i] = cr[i] * X0 + cr[3 + i] * X1 + cr[6 + i] * X2 + cr[9 + i];
      } else {
        double ph[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) ph[i] = X0 * cr[i] + X1 * cr[4 + i] + X2 * cr[8 + i] + cr[12 + i];
        pc[0] = ph[0] / ph[3]; pc[1] = ph[1] / ph[3]; pc[2] = ph[2] / ph[3];
      }
      const float* Kc = GTBL ? cq.k : ktb + c * 9;
      double q[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) q[i] = pc[0] * (double)Kc[i] + pc[1] * (double)Kc[3 + i] + pc[2] * (double)Kc[6 + i];
      const double rc0 = q[0] / q[2] - (double)uv.x, rc1 = q[1] / q[2] - (double)uv.y;
      double sc;
      const double rho = huber(rc0 * rc0 + rc1 * rc1, P.huber_a, P.huber_b, &sc);
      if (o < P.no) {
        acc[0] += mneg;
        acc[1] += 0.5 * rho;
        if (!isfinite(rc0) || !isfinite(rc1)) acc[2] += 1.0;
      }
    }
    wave_lds_sync();
    c = cn; p = pn; uv = uvn;
    if constexpr (GTBL) cq = cqn;
  }
  double out[3];
  block_sum<3>(acc, lds, out);
  if (threadIdx.x == 0) {
    part_of(part, SL_MCC_NEG)[blockIdx.x] = out[0];
    part_of(part, SL_CCOST)[blockIdx.x] = out[1];
    part_of(part, SL_CAND_BAD)[blockIdx.x] = out[2];
  }
}


// ---------------------------------------------------------------------------
// diagonal Schur blocks and rhs (local part): one workgroup per camera
//   S_cc = -sum W W^T (lower 21) ; b_c = -sum W u_p
// ---------------------------------------------------------------------------
// NT threads per camera slice
template <typename WT, int NT = 256>
__global__ __launch_bounds__(NT) void k_cam_schur_diag(DevProblem P, const WT* __restrict__ W,
                                                        const double* __restrict__ u, double* __restrict__ S,
                                                        double* __restrict__ cpart) {
  __shared__ double lds[27 * 16];
  const int v = blockIdx.x;
  double acc[27];
#pragma unroll
  for (int k = 0; k < 27; ++k) acc[k] = 0.0;
  int i0, i1;
  cam_slice(P, v, i0, i1);
  // observations of fixed points carry W = 0 and u = 0 (k_obs_w,
  // k_point_elim): no flag needed; (o, p) pairs in camera order
  auto add = [&](const double (&w)[18], double u0, double u1, double u2) {
    int t = 0;
#pragma unroll
    for (int a = 0; a < 6; ++a) {
#pragma unroll
      for (int b = 0; b <= a; ++b) acc[t++] += w[a * 3] * w[b * 3] + w[a * 3 + 1] * w[b * 3 + 1] + w[a * 3 + 2] * w[b * 3 + 2];
    }
#pragma unroll
    for (int a = 0; a < 6; ++a) acc[21 + a] += w[a * 3] * u0 + w[a * 3 + 1] * u1 + w[a * 3 + 2] * u2;
  };
  for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    const int2 op = P.cam_op[i];
    double w[18];
    load_w18(W, (size_t)op.x, w);
    const double2 u01 = *reinterpret_cast<const double2*>(u + 4 * (size_t)op.y);
    add(w, u01.x, u01.y, u[4 * (size_t)op.y + 2]);
  }
  double tot[27];
  block_sum<27>(acc, lds, tot);
  cam_slice_store(tot, cpart, v, P.nvc);
}

// ---------------------------------------------------------------------------
// off-diagonal Schur blocks: one wave per camera pair block (I >= J), lanes
// stride over its observation pairs, fixed-order shuffle reduction.
//   S_IJ (rows I, cols J) = -sum W_oI W_oJ^T
// ---------------------------------------------------------------------------
__device__ inline void load_w(const double* __restrict__ W, int o, double (&w)[18]) {
  const double2* s = reinterpret_cast<const double2*>(W + (size_t)o * 18);
#pragma unroll
  for (int k = 0; k < 9; ++k) { const double2 t = s[k]; w[2 * k] = t.x; w[2 * k + 1] = t.y; }
}
__device__ inline void acc_pair(double (&acc)[36], const double (&a)[18], const double (&b)[18]) {
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j)
      acc[i * 6 + j] += a[i * 3] * b[j * 3] + a[i * 3 + 1] * b[j * 3 + 1] + a[i * 3 + 2] * b[j * 3 + 2];
}

// PL lanes per block (64 / PL blocks per wave; PL = 16 by default,
// BA_PAIR_LANES selects 8 or 32): each lane accumulates every PL-th pair
// (two pairs' gathers in flight), then a log2(PL)-stage xor reduction inside
// the lane group; all PL lanes then hold the sums and store 36/PL each.
__global__ __launch_bounds__(256) void k_schur_pairs(DevProblem P, const int4* __restrict__ blocks,
                                                     const int* __restrict__ xoff, const int2* __restrict__ pairs,
                                                     const double* __restrict__ W, double* __restrict__ S) {
  constexpr int PL = kPairLanes, BPW = 64 / PL;
  const int lane = threadIdx.x & 63, sl = lane & (PL - 1), sub = lane / PL;
  // XCD-aware order: workgroups b and b + 8 share an XCD (round-robin
  // dispatch).  XCD x owns the block range [xoff[x], xoff[x+1]) (the rows I
  // of S with I mod 8 = x, ascending) and its workgroups sweep it in rounds,
  // so the W rows of the few cameras I active on an XCD are re-read from its
  // L2 by the ~9 blocks (I, J) each observation contributes to.  gridDim.x is
  // a multiple of 8.
  const int xcd = blockIdx.x & 7, wx = blockIdx.x >> 3, nwx = gridDim.x >> 3;
  const int r0 = xoff[xcd], r1 = xoff[xcd + 1];
  const int wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
  const size_t ld = (size_t)P.ld;
  for (int base = r0 + (wx * nwv + wv) * BPW; base < r1; base += nwx * nwv * BPW) {
    const int bi = base + sub;
    const bool live = bi < r1;
    const int4 blk = live ? blocks[bi] : make_int4(0, 0, 0, 0);
    double acc[36];
#pragma unroll
    for (int k = 0; k < 36; ++k) acc[k] = 0.0;
    int e = blk.z + sl;
    for (; e + PL < blk.w; e += 2 * PL) {
      const int2 p0 = pairs[e], p1 = pairs[e + PL];
      double a0[18], b0[18], a1[18], b1[18];
      load_w(W, p0.x, a0); load_w(W, p0.y, b0);
      load_w(W, p1.x, a1); load_w(W, p1.y, b1);
      acc_pair(acc, a0, b0);
      acc_pair(acc, a1, b1);
    }
    if (e < blk.w) {
      const int2 p0 = pairs[e];
      double a0[18], b0[18];
      load_w(W, p0.x, a0); load_w(W, p0.y, b0);
      acc_pair(acc, a0, b0);
    }
#pragma unroll
    for (int k = 0; k < 36; ++k) {
      double v = acc[k];
#pragma unroll
      for (int x = PL / 2; x >= 1; x >>= 1) v += __shfl_xor(v, x, PL);
      acc[k] = v;
    }
    if (live) {
      const int I = blk.x, Jb = blk.y;
#pragma unroll
      for (int k = 0; k < 36; ++k) {
        if ((k % PL) != sl) continue;
        const int i = k / 6, j = k % 6;
        if (I != Jb) S[(size_t)(6 * I + i) * ld + 6 * Jb + j] = -acc[k];
        else if (j <= i) S[(size_t)(6 * I + i) * ld + 6 * I + j] -= acc[k];  // duplicate obs of one point by one camera
      }
    }
  }
}

// k_schur_pairs on compact records (the same blocks, lanes and reduction):
//   W_a W_b^T = c_a^T M c_b,  M = Z_a Z_b^T (2 x 2)
// the partner record is one 128-B line (W: two) and is fetched one pair
// ahead; the row camera's record is an L2 hit.
// (Measured and not kept: the row camera's record one pair ahead as well,
// with the camera constants re-read from LDS per pair to keep 2 waves per
// SIMD: 168 vs 165 us, profiles/r03_v13_ab_pairs_ca.txt.)

// (236 VGPRs: 2 waves per SIMD; forcing 3 or 4 spills 109 / 262 VGPRs)
__global__ __launch_bounds__(256) void k_schur_pairs_c(DevProblem P, const int4* __restrict__ blocks,
                                                       const int* __restrict__ xoff, const int2* __restrict__ pairs,
                                                       const double* __restrict__ Wc,
                                                       const double* __restrict__ scale_c, double* __restrict__ S) {
  // the camera constants of every variable camera in LDS (dynamic: 72 B per
  // camera, 14.4 KB at 200 cameras), read per pair (registers)
  extern __shared__ WcCam ctab[];
  for (int v = threadIdx.x; v < P.nvc; v += blockDim.x) ctab[v].load(P, scale_c, v);
  __syncthreads();
  constexpr int PL = kPairLanes, BPW = 64 / PL;
  const int lane = threadIdx.x & 63, sl = lane & (PL - 1), sub = lane / PL;
  const int xcd = blockIdx.x & 7, wx = blockIdx.x >> 3, nwx = gridDim.x >> 3;
  const int r0 = xoff[xcd], r1 = xoff[xcd + 1];
  const int wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
  const size_t ld = (size_t)P.ld;
  for (int base = r0 + (wx * nwv + wv) * BPW; base < r1; base += nwx * nwv * BPW) {
    const int bi = base + sub;
    const bool live = bi < r1;
    const int4 blk = live ? blocks[bi] : make_int4(0, 0, 0, 0);
    const WcCam& mI = ctab[blk.x];
    const WcCam& mJ = ctab[blk.y];
    double acc[36];
#pragma unroll
    for (int k = 0; k < 36; ++k) acc[k] = 0.0;
    int e = blk.z + sl;
    WcRaw nb;                 // the partner record one pair ahead
    int2 pr = make_int2(0, 0);
    if (e < blk.w) {
      pr = pairs[e];
      nb = wc_fetch(Wc, pr.y);
    }
#if BA_PAIRS_IDX2
    // the pair indices two pairs ahead: the next partner's fetch then waits
    // for no index load of its own iteration (one latency per pair, not two)
    int2 pn = make_int2(0, 0);
    if (e + PL < blk.w) pn = pairs[e + PL];
#endif
    for (; e < blk.w; e += PL) {
      const WcRaw wa = wc_fetch(Wc, pr.x);   // row camera I's record: re-read from L2 by the camera's blocks
      const WcRaw wb = nb;                    // column camera J's
      if (e + PL < blk.w) {
#if BA_PAIRS_IDX2
        pr = pn;
        nb = wc_fetch(Wc, pr.y);
        if (e + 2 * PL < blk.w) pn = pairs[e + 2 * PL];
#else
        pr = pairs[e + PL];
        nb = wc_fetch(Wc, pr.y);
#endif
      }
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
#pragma unroll
    for (int k = 0; k < 36; ++k) {
      double v = acc[k];
#pragma unroll
      for (int x = PL / 2; x >= 1; x >>= 1) v += __shfl_xor(v, x, PL);
      acc[k] = v;
    }
    if (live) {
      const int I = blk.x, Jb = blk.y;
#pragma unroll
      for (int k = 0; k < 36; ++k) {
        if ((k % PL) != sl) continue;
        const int i = k / 6, j = k % 6;
        if (I != Jb) S[(size_t)(6 * I + i) * ld + 6 * Jb + j] = -acc[k];
        else if (j <= i) S[(size_t)(6 * I + i) * ld + 6 * I + j] -= acc[k];  // duplicate obs of one point by one camera
      }
    }
  }
}

// k_schur_pairs_c with the two records of every pair gathered into LDS by
// LDS-DMA (global_load_lds_dwordx4) instead of per-lane 16-B register loads.
// A per-lane record load touches 64 different lines per wave-instruction (8
// instructions per record); here 8 lanes fetch one record's eight 16-B
// pieces, so an instruction covers 8 whole lines.  The pieces land
// lane-linear (record q at q * 128 B), with the piece order XOR-swizzled by
// (q >> 1) & 7 through the SOURCE address, so that the per-lane record reads
// (ds_read_b128, 16-lane groups) are conflict-free.  One buffer per wave:
// the next pair's records are requested right after this pair's are read out
// of LDS, and arrive during its arithmetic.  Same lanes, pairs, products and
// reduction as k_schur_pairs_c: bitwise the same S.
constexpr int kPairsDmaLds = 4 * 2 * 64 * kWcRec * (int)sizeof(double);   // 64 KB: 4 waves x (row, partner) x 64 records
// the diagonal Schur slices in the pair pass's launch (pairs_take_diag);
// BA_DIAG_IN_PAIRS=0 (read per step: tests compare the two forms bitwise)
// keeps the separate diagonal launch (A/B: profiles/r05_v12_diag_in_pairs_ab.txt)

__global__ __launch_bounds__(64) void k_cam_schur_diag_cd(DevProblem P, const double* __restrict__ Wc,
                                                          const double* __restrict__ scale_c,
                                                          const double* __restrict__ u, double* __restrict__ cpart) {
  __shared__ double lds[27 * 16];
  __shared__ __attribute__((aligned(16))) double rbuf[64 * kWcRec];
  __shared__ __attribute__((aligned(16))) double ubuf[64 * 4];
  double acc[27];
  diag_cd_wave(P, Wc, scale_c, u, blockIdx.x, blockIdx.y, gridDim.y, rbuf, ubuf, acc);
  double tot[27];
  block_sum<27>(acc, lds, tot);
  cam_slice_store(tot, cpart, blockIdx.x, P.nvc);
}

// FoldArgs (nsl > 0): workgroups past pgrid run the diagonal fold
// (cam_fold_diag_entry) instead of pairs — independent of the pairs (other S
// blocks) when no point has two observations by one camera
struct FoldArgs {
  const double* cpart;
  int nsl;
  const double* Hcc;
  const double* gc;
  const double* diag_c;
  double radius;
  double* scal;
  // G > 0: those workgroups run the diagonal slices instead (four waves, each
  // one (camera, slice) of k_cam_schur_diag_cd into cpart), independent of the
  // pairs; the fold then follows in its own launch
  const double* u = nullptr;
  int G = 0;
};
// CTAB: the camera constants in an LDS table (<= ~220 variable cameras);
// else (1000 cameras: 72 KB of table beside the 64 KB of records would leave
// one workgroup per CU) each block's two cameras' constants in registers,
// loaded with the block — the same values, so the same S bitwise
template <bool CTAB>
__global__ __launch_bounds__(256) void k_schur_pairs_cd(DevProblem P, const int4* __restrict__ blocks,
                                                        const int* __restrict__ xoff, const int2* __restrict__ pairs,
                                                        const double* __restrict__ Wc,
                                                        const double* __restrict__ scale_c, double* __restrict__ S,
                                                        int pgrid, FoldArgs fa) {
  extern __shared__ double dsm[];
  if ((int)blockIdx.x >= pgrid) {
    if (fa.G > 0) {
      const int wv = threadIdx.x >> 6;
      const int unit = ((int)blockIdx.x - pgrid) * (int)(blockDim.x >> 6) + wv;
      if (unit >= P.nvc * fa.G) return;
      const int v = unit / fa.G, g = unit - v * fa.G;
      double* rb = dsm + (size_t)wv * 2 * 64 * kWcRec;
      double acc[27];
      diag_cd_wave(P, Wc, scale_c, fa.u, v, g, fa.G, rb, rb + 64 * kWcRec, acc);
      double tot[27];
#pragma unroll
      for (int k = 0; k < 27; ++k) tot[k] = 0.0 + wave_sum(acc[k]);   // (block_sum's value for one wave)
      if ((threadIdx.x & 63) == 0) {
        double* dst = const_cast<double*>(fa.cpart) + ((size_t)g * P.nvc + v) * 27;
#pragma unroll
        for (int k = 0; k < 27; ++k) dst[k] = tot[k];
      }
      return;
    }
    cam_fold_diag_entry(P, fa.cpart, fa.nsl, fa.Hcc, fa.gc, scale_c, fa.diag_c, fa.radius, S, fa.scal,
                        ((int)blockIdx.x - pgrid) * blockDim.x + threadIdx.x);
    return;
  }
  WcCam* ctab = reinterpret_cast<WcCam*>(dsm + kPairsDmaLds / (int)sizeof(double));
  if constexpr (CTAB) {
    for (int v = threadIdx.x; v < P.nvc; v += blockDim.x) ctab[v].load(P, scale_c, v);
    __syncthreads();
  }
  constexpr int PL = kPairLanes, BPW = 64 / PL;
  const int lane = threadIdx.x & 63, sl = lane & (PL - 1), sub = lane / PL;
  const int xcd = blockIdx.x & 7, wx = blockIdx.x >> 3, nwx = pgrid >> 3;
  const int r0 = xoff[xcd], r1 = xoff[xcd + 1];
  const int wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
  double* rbuf = dsm + (size_t)wv * 2 * 64 * kWcRec;   // row camera's records [64][16]
  double* pbuf = rbuf + 64 * kWcRec;                    // partner records
  const int swr = (lane >> 1) & 7;                      // this lane's record: piece p at slot p ^ swr
  const size_t ld = (size_t)P.ld;
  // the 8 DMA pieces of this lane: record q = (lane >> 3) + 8 i, source piece
  // (lane & 7) ^ ((q >> 1) & 7), destination slot lane & 7
  auto issue = [&](int2 pr) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int q = (lane >> 3) + 8 * i;
      const int ra = __shfl(pr.x, q), rb = __shfl(pr.y, q);
      const int sp = 2 * ((lane & 7) ^ ((q >> 1) & 7));
      glds16(Wc + (size_t)ra * kWcRec + sp, rbuf + i * 128);
      glds16(Wc + (size_t)rb * kWcRec + sp, pbuf + i * 128);
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
  for (int base = r0 + (wx * nwv + wv) * BPW; base < r1; base += nwx * nwv * BPW) {
    const int bi = base + sub;
    const bool live = bi < r1;
    const int4 blk = live ? blocks[bi] : make_int4(0, 0, 0, 0);
    WcCam mI, mJ;
    if constexpr (CTAB) {
      mI = ctab[blk.x];
      mJ = ctab[blk.y];
    } else {
      mI.load(P, scale_c, blk.x);
      mJ.load(P, scale_c, blk.y);
    }
    double acc[36];
#pragma unroll
    for (int k = 0; k < 36; ++k) acc[k] = 0.0;
    // pairs per lane, wave maximum (the loop below is wave-uniform)
    const int len = blk.w - blk.z;
    int nit = len > sl ? (len - sl + PL - 1) / PL : 0;
#pragma unroll
    for (int x = 32; x >= 1; x >>= 1) nit = max(nit, __shfl_xor(nit, x));
    int e = blk.z + sl;
    int2 pr = e < blk.w ? pairs[e] : make_int2(0, 0);
    int2 pn = e + PL < blk.w ? pairs[e + PL] : make_int2(0, 0);
    if (nit > 0) issue(pr);
    for (int t = 0; t < nit; ++t, e += PL) {
      // this pair's DMA has landed (the compiler does not order LDS reads
      // after an LDS-DMA on its own)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const WcRaw wa = read_rec(rbuf);
      const WcRaw wb = read_rec(pbuf);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // read out before the buffers are refilled
      if (t + 1 < nit) {
        issue(pn);
        pn = e + 2 * PL < blk.w ? pairs[e + 2 * PL] : make_int2(0, 0);
      }
      if (e < blk.w) {
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
      const int I = blk.x, Jb = blk.y;
#pragma unroll
      for (int k = 0; k < 36; ++k) {
        if ((k % PL) != sl) continue;
        const int i = k / 6, j = k % 6;
        if (I != Jb) S[(size_t)(6 * I + i) * ld + 6 * Jb + j] = -acc[k];
        else if (j <= i) S[(size_t)(6 * I + i) * ld + 6 * I + j] -= acc[k];  // duplicate obs of one point by one camera
      }
    }
  }
}

// S_cc += s Hcc s + D^2 ;  b_c += s * g_c      (after any cross-rank reduction)
// one thread per (camera, entry): 21 lower entries of the diagonal block and
// 6 rhs entries (a thread per camera serialised ~50 dependent accesses)
__global__ __launch_bounds__(256) void k_cam_add_diag(DevProblem P, const double* __restrict__ Hcc,
                                                      const double* __restrict__ gc, const double* __restrict__ scale_c,
                                                      const double* __restrict__ diag_c, double radius,
                                                      double* __restrict__ S, double* __restrict__ scal) {
  // no fma contraction: the fused and the exchange path (k_cam_fold +
  // k_cam_add_diag) must round identically
#pragma clang fp contract(off)
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e == 0) { scal[SL_CHOL_BAD] = 0.0; scal[SL_CHOL_SPIN] = 0.0; }   // the Cholesky that follows flags failures here
  if (e >= P.nvc * 27) return;
  const int v = e / 27, k = e - v * 27;
  const size_t ld = (size_t)P.ld;
  if (k < 21) {
    int a = 0;
    while ((a + 1) * (a + 2) / 2 <= k) ++a;
    const int b = k - a * (a + 1) / 2;
    double h = Hcc[(size_t)v * 21 + k] * scale_c[(size_t)v * 6 + a] * scale_c[(size_t)v * 6 + b];
    if (a == b) {
      const double D = sqrt(diag_c[(size_t)v * 6 + a] / radius);
      h += D * D;
    }
    S[(size_t)(6 * v + a) * ld + 6 * v + b] += h;
  } else {
    const int a = k - 21;
    S[(size_t)P.n * ld + 6 * v + a] += gc[(size_t)v * 6 + a] * scale_c[(size_t)v * 6 + a];
  }
}

// single rank: k_cam_fold (mode 1) and k_cam_add_diag in one pass,
//   S_cc = -sum_slices + s Hcc s + D^2 ;  b_c = -sum_slices + s g_c
// (k_schur_pairs' duplicate-observation terms land on the diagonal after)
__global__ __launch_bounds__(256) void k_cam_fold_diag(DevProblem P, const double* __restrict__ cpart, int nsl,
                                                       const double* __restrict__ Hcc, const double* __restrict__ gc,
                                                       const double* __restrict__ scale_c,
                                                       const double* __restrict__ diag_c, double radius,
                                                       double* __restrict__ S, double* __restrict__ scal) {
  cam_fold_diag_entry(P, cpart, nsl, Hcc, gc, scale_c, diag_c, radius, S, scal, blockIdx.x * blockDim.x + threadIdx.x);
}

// ---------------------------------------------------------------------------
// candidate cameras: x' = x + s * (-y), value-only records at x'
// ---------------------------------------------------------------------------
// one 64-lane block per camera: lanes 0..5 form the step, every lane
// evaluates the (cheap) Rodrigues and writes record entries lane, lane + 64
// Hcc, gc != nullptr (the block form of the model cost change, k_point_step_rc
// ACC): + gc^T dc + dc^T Hcc dc / 2 per variable camera into SL_MCC_NEG
__global__ __launch_bounds__(64) void k_cam_candidate(DevProblem P, const double* __restrict__ cams,
                                                      const double* __restrict__ y, const double* __restrict__ scale_c,
                                                      double* __restrict__ cams_c, double* __restrict__ delta_c,
                                                      double* __restrict__ rec_c, double* __restrict__ part,
                                                      const double* __restrict__ Hcc, const double* __restrict__ gc) {
  __shared__ double lds[3 * 16];
  const int lane = threadIdx.x;
  double acc[3] = {0.0, 0.0, 0.0};  // step2, bad, model terms
  for (int c = blockIdx.x; c < P.nc; c += gridDim.x) {
    const int v = P.vc[c];
    if (Hcc && v >= 0 && lane == 0) {
      double d[6];
#pragma unroll
      for (int a = 0; a < 6; ++a) d[a] = (-y[6 * v + a]) * scale_c[(size_t)v * 6 + a];
      const double* h = Hcc + (size_t)v * 21;
      double dhd = 0.0, gd = 0.0;
      int t = 0;
#pragma unroll
      for (int a = 0; a < 6; ++a) {
#pragma unroll
        for (int b = 0; b < a; ++b) dhd += 2.0 * h[t++] * d[a] * d[b];
        dhd += h[t++] * d[a] * d[a];
        gd += gc[(size_t)v * 6 + a] * d[a];
      }
      acc[2] += gd + 0.5 * dhd;
    }
    double xc[6];
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      const double x = cams[6 * c + a];
      double d = 0.0;
      if (v >= 0) d = (-y[6 * v + a]) * scale_c[(size_t)v * 6 + a];
      xc[a] = v >= 0 ? x + d : x;
      if (lane == a && v >= 0) {
        delta_c[(size_t)v * 6 + a] = d;
        const double e = x - xc[a];
        acc[0] += e * e;
        if (!isfinite(d)) acc[1] += 1.0;
      }
    }
#pragma unroll
    for (int a = 0; a < 6; ++a)
      if (lane == a) cams_c[6 * c + a] = xc[a];
    double* o = rec_c + (size_t)c * kCamRec;
    const bool fixed = P.cam_fixed && P.cam_fixed[c];
    double R[9];
    if (!fixed) angle_axis_to_R(xc, R);
    for (int e = lane; e < kRecL; e += 64) {
      double val = 0.0;
      if (e >= kRecK && e < kRecK + 9) val = (double)P.K[9 * c + e - kRecK];
      else if (fixed) val = e < 16 ? (double)P.extr[16 * c + e] : 0.0;
      else if (e < 9) val = R[e];
      else if (e >= kRecT && e < kRecT + 3) val = xc[3 + e - kRecT];
      else if (e < kRecK) continue;   // dR/dw: not used at a candidate point
      o[e] = val;
    }
  }
  double out[3];
  block_sum<3>(acc, lds, out);
  if (threadIdx.x == 0) {
    part_of(part, SL_STEP2_C)[blockIdx.x] = out[0];
    part_of(part, SL_STEP_BAD)[blockIdx.x] += out[1];
    if (Hcc) part_of(part, SL_MCC_NEG)[blockIdx.x] += out[2];
  }
}

// Raw residuals (no loss) at given records, for ba_eval_residuals.
__global__ __launch_bounds__(256) void k_residuals(DevProblem P, const double* __restrict__ rec,
                                                   const double* __restrict__ pts, double* __restrict__ rr) {
  for (int o = blockIdx.x * blockDim.x + threadIdx.x; o < P.no; o += gridDim.x * blockDim.x) {
    const int c = P.obs_cam[o], p = P.obs_pt[o];
    double res[2];
    project_value(rec + (size_t)c * kCamRec, !(P.cam_fixed && P.cam_fixed[c]), pts[3 * p], pts[3 * p + 1],
                  pts[3 * p + 2], P.uv[o], res);
    rr[2 * o] = res[0];
    rr[2 * o + 1] = res[1];
  }
}

// Fold partials -> scalars (fixed order), then clear the partials.  One
// wave per slot (kNumSlots waves), no workgroup barrier: each lane folds a
// fixed strided subset, then a fixed-order shuffle tree.
// one 64-lane workgroup per slot (the slots' 16-KB folds run on separate
// CUs; as waves of one workgroup they all went through one CU)
//
// PUB (the scalar record of ba_ctx::publish_scalars folded into the same
// launch): every workgroup then takes a ticket after its slot (agent-scope
// release fence first), and the last one acquires and does what
// k_publish_scalars does: the record into the pinned host-mapped copy,
// system-scope release, then the sequence number.  The ticket is reset by
// that workgroup for the next launch (stream order).
struct ReducePub {
  double* host = nullptr;
  int n = 0;
  unsigned* host_seq = nullptr;
  unsigned seq = 0;
  unsigned* ticket = nullptr;
};
__device__ __forceinline__ void reduce_slot(double* __restrict__ part, double* __restrict__ scal, int slot, int lane,
                                            bool is_max) {
  double* pp = part + (size_t)slot * kMaxBlocks;
  constexpr int PER = kMaxBlocks / 64;
  double v[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) v[i] = pp[i * 64 + lane];
#pragma unroll
  for (int i = 0; i < PER; ++i) pp[i * 64 + lane] = 0.0;
  double x = 0.0;
  if (is_max) {
#pragma unroll
    for (int i = 0; i < PER; ++i) x = fmax(x, v[i]);
    x = wave_max(x);
  } else {
#pragma unroll
    for (int i = 0; i < PER; ++i) x += v[i];
    x = wave_sum(x);
  }
  if (lane == 0) scal[slot] = x;
}
template <bool PUB>
__global__ __launch_bounds__(64) void k_reduce(double* __restrict__ part, double* __restrict__ scal,
                                               uint32_t sum_mask, uint32_t max_mask, ReducePub pub) {
  const int slot = blockIdx.x, lane = threadIdx.x & 63;
  const bool is_sum = (sum_mask >> slot) & 1u, is_max = (max_mask >> slot) & 1u;
  if (is_sum || is_max) reduce_slot(part, scal, slot, lane, is_max);
  if (!PUB) return;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");   // this slot before the ticket
  unsigned t = 0;
  if (lane == 0) t = __hip_atomic_fetch_add(pub.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  t = __builtin_amdgcn_readfirstlane(t);
  if (t != gridDim.x - 1) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // every slot after it
  for (int i = lane; i < pub.n; i += 64) pub.host[i] = scal[i];
  if (lane == 0) *pub.ticket = 0u;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // system scope: the record reaches host memory first
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) __hip_atomic_store(pub.host_seq, pub.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
// ---------------------------------------------------------------------------
// J-free iteration (nc <= kLinLdsCams, the camera table fits the LDS).
//
// The per-observation Jacobian costs ~18 us of arithmetic at C3 but 176 B of
// HBM writes plus 4 x 160 B of re-reads per observation when it is
// materialised (k_linearize -> JR -> k_point_assemble, k_cam_assemble,
// k_obs_w, k_candidate_lds: ~0.8 GB per LM iteration).  Here every consumer
// recomputes r and J from the camera table (LDS), the point and the pixel with
// the same lin_obs() (same operations on the same operands: bitwise the JR
// values), so J never leaves the registers:
//   k_lin_point       r, J, Huber, cost + the point blocks Hpp / gp, scaling,
//                     LM diagonal, gradient norms (k_linearize + k_point_assemble)
//   k_cam_assemble_rc Hcc / gc per camera, the camera's table row in registers
//   k_obs_w_rc        W_o = s_c Jc^T Jp s_p L_p^-T
//   k_point_step_rc   back substitution, model cost change J d . (r + J d / 2)
//                     and candidate cost
// Per point / camera the sums run in the order of the JR kernels they replace.
// ---------------------------------------------------------------------------
// a variable camera's table row held in registers (the camera of a whole
// workgroup in k_cam_assemble_rc)
struct CamRegs {
  double t[kLin];
  double k[9];
  __device__ bool var() const { return true; }
  __device__ void load(double (&o)[kLin]) const {
#pragma unroll
    for (int i = 0; i < kLin; ++i) o[i] = t[i];
  }
  __device__ double K(int i) const { return k[i]; }
};

// LANES lanes per point (lane l of a group takes the point's observations l,
// l + LANES, ...; fixed-order xor fold inside the group); the next
// observation's indices and pixel, and the group's next point, are loaded one
// step ahead (clamped, unconditional loads).  The cameras from the LDS copy
// of the records' lin tables (nc <= kLinLdsCams; beyond: k_lin_point_d)
template <int NT, int LANES>
// pxv: the points as 32-B records {X, variable flag} for the camera-major
// consumers (k_cam_assemble_rc: one sector per gathered point)
__global__ __launch_bounds__(NT) void k_lin_point(DevProblem P, const double* __restrict__ rec,
                                                  const double* __restrict__ pts, double* __restrict__ Hpp,
                                                  double* __restrict__ gp, double* __restrict__ scale_p,
                                                  double* __restrict__ diag_p, int compute_scale, double min_diag,
                                                  double max_diag, double* __restrict__ part,
                                                  double* __restrict__ pxv) {
  __shared__ double lds[5 * 16];
  __shared__ __attribute__((aligned(16))) double tbl[kLinLdsCams * kTblRec];
  __shared__ float ktb[kLinLdsCams * 9];
  fill_lin_table<NT>(P, rec, tbl, ktb);
  double acc[4] = {0.0, 0.0, 0.0, 0.0};   // cost, bad, gn2, xn2
  double gmax = 0.0;
  const size_t np = (size_t)P.np;
  const int sl = threadIdx.x & (LANES - 1);
  const int g0 = (blockIdx.x * NT + threadIdx.x) / LANES, gs = gridDim.x * NT / LANES;
  const int lastp = max(P.np - 1, 0), lasto = max(P.no - 1, 0);
  // the group's point p and its data, one point ahead (np = 0: no prologue,
  // pt_off has a single entry)
  int p = P.np > 0 ? g0 : P.np;
  if (P.np > 0) {
  // (prologue and loop)
  int pc = min(p, lastp);
  int o0 = P.pt_off[pc], o1 = P.pt_off[pc + 1];
  double X0 = pts[3 * pc], X1 = pts[3 * pc + 1], X2 = pts[3 * pc + 2];
  bool pv = P.pt_var[pc] != 0;
  for (; p < P.np; p += gs) {     // uniform inside a lane group
    const int pn = min(p + gs, lastp);
    const int o0n = P.pt_off[pn], o1n = P.pt_off[pn + 1];
    const double Y0 = pts[3 * pn], Y1 = pts[3 * pn + 1], Y2 = pts[3 * pn + 2];
    const bool pvn = P.pt_var[pn] != 0;
    double H[6] = {0, 0, 0, 0, 0, 0}, g[3] = {0, 0, 0};
    int o = o0 + sl;
    int oc = min(o, lasto);
    int c = P.obs_cam[oc];
    float2 uv = P.uv[oc];
    for (; o < o1; o += LANES) {
      const int on = min(o + LANES, lasto);
      const int cn = P.obs_cam[on];
      const float2 uvn = P.uv[on];
      double out[kJR];
      bool fin;
      const CamLds cam{tbl + c * kTblRec, ktb + c * 9};
      const double rho = lin_obs(P, cam, cam.var(), pv, X0, X1, X2, uv, out, fin);
      acc[0] += 0.5 * rho;
      acc[1] += fin ? 0.0 : 1.0;
      // k_point_assemble's accumulation of the JB record (Jp rows, r)
      const double jp[2][3] = {{out[12], out[13], out[14]}, {out[15], out[16], out[17]}};
      const double rr[2] = {out[18], out[19]};
#pragma unroll
      for (int row = 0; row < 2; ++row) {
        const double a = jp[row][0], b = jp[row][1], cc = jp[row][2];
        H[0] += a * a; H[1] += a * b; H[2] += a * cc; H[3] += b * b; H[4] += b * cc; H[5] += cc * cc;
        g[0] += a * rr[row]; g[1] += b * rr[row]; g[2] += cc * rr[row];
      }
      c = cn;
      uv = uvn;
    }
    if (pv) {
#pragma unroll
      for (int k = 0; k < 6; ++k) {
#pragma unroll
        for (int x = LANES / 2; x >= 1; x >>= 1) H[k] += __shfl_xor(H[k], x, LANES);
      }
#pragma unroll
      for (int k = 0; k < 3; ++k) {
#pragma unroll
        for (int x = LANES / 2; x >= 1; x >>= 1) g[k] += __shfl_xor(g[k], x, LANES);
      }
      if (sl == 0) {
#pragma unroll
        for (int k = 0; k < 6; ++k) Hpp[k * np + p] = H[k];
        const double hd[3] = {H[0], H[3], H[5]};
        const double Xk[3] = {X0, X1, X2};
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          gp[k * np + p] = g[k];
          double s;
          if (compute_scale) {
            s = 1.0 / (1.0 + sqrt(hd[k]));
            scale_p[k * np + p] = s;
          } else {
            s = scale_p[k * np + p];
          }
          diag_p[k * np + p] = fmin(fmax(hd[k] * s * s, min_diag), max_diag);
          const double x = Xk[k];
          const double d = x - (x + (-g[k]));
          gmax = fmax(gmax, fabs(d));
          acc[2] += d * d;
          acc[3] += x * x;
        }
      }
    }
    if (sl == 0) {
      double2* d = reinterpret_cast<double2*>(pxv + 4 * (size_t)p);
      d[0] = make_double2(X0, X1);
      d[1] = make_double2(X2, pv ? 1.0 : 0.0);
    }
    o0 = o0n; o1 = o1n;
    X0 = Y0; X1 = Y1; X2 = Y2;
    pv = pvn;
  }
  }
  double tot[4];
  block_sum<4>(acc, lds, tot);
  const double m = block_max1(gmax, lds + 64);
  if (threadIdx.x == 0) {
    part_of(part, SL_COST)[blockIdx.x] = tot[0];
    part_of(part, SL_LIN_BAD)[blockIdx.x] = tot[1];
    part_of(part, SL_GN2_P)[blockIdx.x] = tot[2];
    part_of(part, SL_XN2_P)[blockIdx.x] = tot[3];
    part_of(part, SL_GMAX_P)[blockIdx.x] = m;
  }
}

// k_lin_point beyond kLinLdsCams cameras: the compact camera records
// (k_cam_compact; the dual Rodrigues per observation) gathered by LDS-DMA
// (8 lanes per 128-B record, a wave-instruction touching 8 records instead of
// 64; pieces XOR-swizzled through the source address as in k_schur_pairs_cd)
// one observation round ahead — across point boundaries too: the last round
// of a point requests the first cameras of the lane's next point.  The DMA
// needs every lane of the wave, so the point and observation loops run in
// wave-uniform rounds (a lane past its point's observations, or past the
// points, computes nothing).  Per lane the same lin_obs on the same record
// values and the same accumulation order as per-lane register gathers.
template <int NT, int LANES>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_lin_point_d(DevProblem P, const double* __restrict__ crec,
                                                    const double* __restrict__ pts, double* __restrict__ Hpp,
                                                    double* __restrict__ gp, double* __restrict__ scale_p,
                                                    double* __restrict__ diag_p, int compute_scale, double min_diag,
                                                    double max_diag, double* __restrict__ part,
                                                    double* __restrict__ pxv) {
  __shared__ double lds[5 * 16];
  __shared__ __attribute__((aligned(16))) double cbuf[NT / 64][64 * kCRec];
  const int lane = threadIdx.x & 63;
  double* cb = cbuf[threadIdx.x >> 6];
  const int swr = (lane >> 1) & 7;
  auto issue = [&](int cc) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int q = (lane >> 3) + 8 * k;
      const int cq = __shfl(cc, q);
      glds16(crec + (size_t)cq * kCRec + 2 * ((lane & 7) ^ ((q >> 1) & 7)), cb + k * 128);
    }
  };
  auto fetch = [&]() {
    CamRcPre q;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this round's records have landed
#pragma unroll
    for (int k = 0; k < kCRec / 2; ++k) q.v[k] = *reinterpret_cast<const double2*>(cb + lane * kCRec + 2 * (k ^ swr));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // read out before the next request
    return q;
  };
  double acc[4] = {0.0, 0.0, 0.0, 0.0};   // cost, bad, gn2, xn2
  double gmax = 0.0;
  const size_t np = (size_t)P.np;
  const int sl = threadIdx.x & (LANES - 1);
  const int g0 = (blockIdx.x * NT + threadIdx.x) / LANES, gs = gridDim.x * NT / LANES;
  const int lastp = max(P.np - 1, 0), lasto = max(P.no - 1, 0);
  if (P.np > 0 && P.no > 0) {
    int p = g0;
    int pc = min(p, lastp);
    int o0 = P.pt_off[pc], o1 = P.pt_off[pc + 1];
    double X0 = pts[3 * pc], X1 = pts[3 * pc + 1], X2 = pts[3 * pc + 2];
    bool pv = P.pt_var[pc] != 0;
    int c = P.obs_cam[min(o0 + sl, lasto)];
    float2 uv = P.uv[min(o0 + sl, lasto)];
    issue(c);
    while (__any(p < P.np)) {   // wave-uniform point rounds
      const bool livep = p < P.np;
      const int pn = min(p + gs, lastp);
      const int o0n = P.pt_off[pn], o1n = P.pt_off[pn + 1];
      const double Y0 = pts[3 * pn], Y1 = pts[3 * pn + 1], Y2 = pts[3 * pn + 2];
      const bool pvn = P.pt_var[pn] != 0;
      const int onp = min(o0n + sl, lasto);   // the next point's first observation of this lane
      const int cnp = P.obs_cam[onp];
      const float2 uvnp = P.uv[onp];
      double H[6] = {0, 0, 0, 0, 0, 0}, g[3] = {0, 0, 0};
      int cnt = livep && o1 - o0 > sl ? (o1 - o0 - sl + LANES - 1) / LANES : 0;
#pragma unroll
      for (int x = 32; x >= 1; x >>= 1) cnt = max(cnt, __shfl_xor(cnt, x));
      int o = o0 + sl;
      if (cnt == 0) {   // (keep one request in flight: the next point's)
        (void)fetch();
        issue(cnp);
        uv = uvnp;
      }
      for (int t = 0; t < cnt; ++t) {
        const CamRcPre q = fetch();
        const bool more = t + 1 < cnt;
        const int on = min(o + LANES, lasto);
        const int cn = more ? P.obs_cam[on] : cnp;
        const float2 uvn = more ? P.uv[on] : uvnp;
        issue(cn);
        if (livep && o < o1) {
          const CamRc cam = cam_make(CamRcOf{crec, nullptr}, q);
          double out[kJR];
          bool fin;
          const double rho = lin_obs(P, cam, cam.var(), pv, X0, X1, X2, uv, out, fin);
          acc[0] += 0.5 * rho;
          acc[1] += fin ? 0.0 : 1.0;
          const double jp[2][3] = {{out[12], out[13], out[14]}, {out[15], out[16], out[17]}};
          const double rr[2] = {out[18], out[19]};
#pragma unroll
          for (int row = 0; row < 2; ++row) {
            const double a = jp[row][0], b = jp[row][1], cc = jp[row][2];
            H[0] += a * a; H[1] += a * b; H[2] += a * cc; H[3] += b * b; H[4] += b * cc; H[5] += cc * cc;
            g[0] += a * rr[row]; g[1] += b * rr[row]; g[2] += cc * rr[row];
          }
        }
        uv = uvn;
        o += LANES;
      }
      if (livep && pv) {
#pragma unroll
        for (int k = 0; k < 6; ++k) {
#pragma unroll
          for (int x = LANES / 2; x >= 1; x >>= 1) H[k] += __shfl_xor(H[k], x, LANES);
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) {
#pragma unroll
          for (int x = LANES / 2; x >= 1; x >>= 1) g[k] += __shfl_xor(g[k], x, LANES);
        }
        if (sl == 0) {
#pragma unroll
          for (int k = 0; k < 6; ++k) Hpp[k * np + p] = H[k];
          const double hd[3] = {H[0], H[3], H[5]};
          const double Xk[3] = {X0, X1, X2};
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            gp[k * np + p] = g[k];
            double s;
            if (compute_scale) {
              s = 1.0 / (1.0 + sqrt(hd[k]));
              scale_p[k * np + p] = s;
            } else {
              s = scale_p[k * np + p];
            }
            diag_p[k * np + p] = fmin(fmax(hd[k] * s * s, min_diag), max_diag);
            const double x = Xk[k];
            const double d = x - (x + (-g[k]));
            gmax = fmax(gmax, fabs(d));
            acc[2] += d * d;
            acc[3] += x * x;
          }
        }
      }
      if (livep && sl == 0) {
        double2* d = reinterpret_cast<double2*>(pxv + 4 * (size_t)p);
        d[0] = make_double2(X0, X1);
        d[1] = make_double2(X2, pv ? 1.0 : 0.0);
      }
      o0 = o0n; o1 = o1n;
      X0 = Y0; X1 = Y1; X2 = Y2;
      pv = pvn;
      p += gs;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the last (unread) request
  }
  double tot[4];
  block_sum<4>(acc, lds, tot);
  const double m = block_max1(gmax, lds + 64);
  if (threadIdx.x == 0) {
    part_of(part, SL_COST)[blockIdx.x] = tot[0];
    part_of(part, SL_LIN_BAD)[blockIdx.x] = tot[1];
    part_of(part, SL_GN2_P)[blockIdx.x] = tot[2];
    part_of(part, SL_XN2_P)[blockIdx.x] = tot[3];
    part_of(part, SL_GMAX_P)[blockIdx.x] = m;
  }
}

// Hcc (lower 21) and gc per variable camera, its observations in camera order
// (k_cam_assemble's order: thread i takes i0 + tid, i0 + tid + NT, ...)
// TB = 2: rec is the compact records crec (the camera's dual Rodrigues once
// per workgroup: CamRcR), else the camera records (lin table in registers).
// pxv: k_lin_point's 32-B point records {X, variable flag}; the pixels come
// in camera order (uv_cm)
template <int NT, int TB = 0>
__global__ __launch_bounds__(NT) void k_cam_assemble_rc(DevProblem P, const double* __restrict__ rec,
                                                        const double* __restrict__ pxv, double* __restrict__ cpart,
                                                        double* __restrict__ Hcc, double* __restrict__ gc) {
  __shared__ double lds[27 * 16];
  // TB 2: the camera's dual Rodrigues and K once per workgroup, in LDS and
  // read at use (uniform broadcasts; an opaque per-observation offset keeps
  // the reads from being hoisted into registers: 196 -> fewer VGPRs, more
  // waves per SIMD)
  __shared__ CamRcR scam;
  const int v = blockIdx.x;
  const int c = P.cam_of_vc[v];
  CamRegs cam;
  if constexpr (TB == 2) {
    if (threadIdx.x == 0) scam.make(cam_rc(rec, c));
    __syncthreads();
  } else {
    const double2* s2 = reinterpret_cast<const double2*>(rec + (size_t)c * kCamRec + kRecL);
#pragma unroll
    for (int k = 0; k < kLin / 2; ++k) { const double2 u = s2[k]; cam.t[2 * k] = u.x; cam.t[2 * k + 1] = u.y; }
#pragma unroll
    for (int k = 0; k < 9; ++k) cam.k[k] = (double)P.K[9 * c + k];   // float-valued (Matrix3f)
  }
  double acc[27];
#pragma unroll
  for (int k = 0; k < 27; ++k) acc[k] = 0.0;
  int i0, i1;
  cam_slice(P, v, i0, i1);
  for (int i = i0 + threadIdx.x; i < i1; i += NT) {
    const int p = P.cam_op[i].y;
    const double2* xr = reinterpret_cast<const double2*>(pxv + 4 * (size_t)p);
    const double2 x01 = xr[0], x2v = xr[1];
    double out[kJR];
    bool fin;
    if constexpr (TB == 2) {
      int zo = 0;
      asm volatile("" : "+v"(zo));
      const CamRcR& cl = *reinterpret_cast<const CamRcR*>(reinterpret_cast<const char*>(&scam) + zo);
      (void)lin_obs(P, cl, true, x2v.y != 0.0, x01.x, x01.y, x2v.x, P.uv_cm[i], out, fin);
    } else {
      (void)lin_obs(P, cam, true, x2v.y != 0.0, x01.x, x01.y, x2v.x, P.uv_cm[i], out, fin);
    }
    // cam_acc_jr on the record: Jc rows (0..11) and the residual (18, 19)
    const double rr[2] = {out[18], out[19]};
#pragma unroll
    for (int row = 0; row < 2; ++row) {
      const double* j = out + 6 * row;
      int t = 0;
#pragma unroll
      for (int a = 0; a < 6; ++a)
#pragma unroll
        for (int b = 0; b <= a; ++b) acc[t++] += j[a] * j[b];
#pragma unroll
      for (int a = 0; a < 6; ++a) acc[21 + a] += j[a] * rr[row];
    }
  }
  double out27[27];
  block_sum<27>(acc, lds, out27);
  if (gridDim.y == 1) {
    if (threadIdx.x == 0) {
#pragma unroll
      for (int k = 0; k < 21; ++k) Hcc[(size_t)v * 21 + k] = out27[k];
#pragma unroll
      for (int k = 0; k < 6; ++k) gc[(size_t)v * 6 + k] = out27[21 + k];
    }
    return;
  }
  cam_slice_store(out27, cpart, v, P.nvc);
}

// W_o from recomputed J (k_obs_w<true, WT> with the JR chunk replaced by
// lin_obs; the records leave through the same wave-private LDS staging).
//
// COMPACT (J-free fp64 DENSE_SCHUR): W_o = c^T Z is rank 2 (c = Jc s_c, 2 x 6;
// Z = Jp s_p L_p^-T, 2 x 3) and the translation columns of Jc are
// (K_k - pr K_k2) f (lin_obs): the record keeps the scaled rotation columns
// of c, pr0, pr1, f and Z — 15 doubles in one 128-B line instead of W's
// 144 B, which straddle two.  The camera-side consumers (k_cam_schur_diag_c,
// k_schur_pairs_c) gather one line per observation and form their products
// through the 2 x 2 inner matrices Z Z'^T (WcCam: the camera's K and
// translation scalings).
//
// PC (ITERATIVE_SCHUR, intrinsics without skew: K01 = K10 = K20 = K21 = 0):
// the same rank-2 form for the PCG point pass, self-contained — c's scaled
// rotation columns, the four nonzero scaled translation entries c0[3],
// c0[5], c1[4], c1[5] (c0[4] = (K01 - pr0 K21) f and c1[3] = (K10 - pr1 K20)
// f are exact zeros there), then Z: 16 values, one 128-B line (fp64) instead
// of 144 B, with no per-camera constants to gather (k_pcg_point_seg<.., PC>)
constexpr int kObsWRcWaves = 6;   // table + K + scales + 6 staging slots fit the 160 KB LDS
// TB: 0 the LDS copy of the camera table, 3 (nc > kLinLdsCams) rec is the
// compact records crec, gathered by LDS-DMA (below); the camera scalings are
// then read from scale_c
// WAVES: waves per workgroup.  The LDS-table form (TB 0) holds one 148-KB
// workgroup per CU: 6.  The global-source forms need ~230 VGPRs (two waves per
// SIMD): a 6-wave workgroup then leaves a CU at one workgroup, 6 waves, where
// two 4-wave workgroups fill its 8 slots (kObsWRcWavesG; C5 shard +0.9 %,
// C4 unchanged: profiles/r04_v18_obsw_waves_ab.txt)
constexpr int kObsWRcWavesG = 4;
template <typename WT, bool COMPACT = false, int TB = 0, bool PC = false, int WAVES = kObsWRcWaves>
// pxv: k_lin_point's 32-B point records {X, variable flag} (one aligned
// 32-B read per observation instead of 24 B of X plus the flag byte)
__global__ __launch_bounds__(64 * WAVES) void k_obs_w_rc(DevProblem P, const double* __restrict__ rec,
                                                                const double* __restrict__ pxv,
                                                                const double* __restrict__ scale_c,
                                                                const double* __restrict__ scale_p,
                                                                const double* __restrict__ Linv, WT* __restrict__ W) {
  using V2 = typename std::conditional<sizeof(WT) == 8, double2, float2>::type;
  constexpr int NT = 64 * WAVES;
  __shared__ double stage[WAVES * 64 * kStageLd];
  __shared__ __attribute__((aligned(16))) double tbl[TB ? 2 : kLinLdsCams * kTblRec];
  __shared__ float ktb[TB ? 1 : kLinLdsCams * 9];
  __shared__ double sct[TB ? 1 : kLinLdsCams * 6];
  if constexpr (!TB) {
    fill_lin_table<NT>(P, rec, tbl, ktb);   // (ends with a barrier)
    for (int e = threadIdx.x; e < P.nc * 6; e += NT) {
      const int c = e / 6, a = e - 6 * c;
      const int v = P.vc[c];
      sct[e] = v >= 0 ? scale_c[(size_t)v * 6 + a] : 0.0;
    }
    __syncthreads();
  }
  if (P.no == 0) return;   // (the clamped prefetch indices below need no >= 1)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double* st = stage + w * (64 * kStageLd);
  const int step = gridDim.x * WAVES * 64;
  const size_t np = (size_t)P.np;
  int base = (blockIdx.x * WAVES + w) * 64;
  // indices one chunk ahead (clamped, unconditional)
  int oc = min(base + lane, P.no - 1);
  int c = P.obs_cam[oc], p = P.obs_pt[oc];
  float2 uv = P.uv[oc];
  // TB 3: the compact records gathered by LDS-DMA into the wave's
  // staging slot, 8 lanes per 128-B record (pieces XOR-swizzled through the
  // source address, as k_schur_pairs_cd): a wave-instruction touches 8
  // records instead of 64.  The next chunk's records are requested after
  // this chunk's W records have left the slot, ahead of their stores
  static_assert(!(COMPACT && PC), "one record form");
  constexpr int NST = (COMPACT || PC ? kWcRec : kWRec) / 2;   // store instructions per chunk
  auto crec_issue = [&](int cc) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int q = (lane >> 3) + 8 * k;
      const int cq = __shfl(cc, q);
      glds16(rec + (size_t)cq * kCRec + 2 * ((lane & 7) ^ ((q >> 1) & 7)), st + k * 128);
    }
  };
  if constexpr (TB == 3) {
    crec_issue(c);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (the first chunk's; later ones: below)
  }
  for (; base < P.no; base += step) {
    CamRcPre crp;
    if constexpr (TB == 3) {
      // this chunk's records have landed; the previous chunk's NST stores,
      // issued after them, may still be in flight (in-order completion; only
      // a full chunk is followed by a request, and it stores NST times)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NST) : "memory");
      const int swr = (lane >> 1) & 7;
#pragma unroll
      for (int k = 0; k < kCRec / 2; ++k) crp.v[k] = *reinterpret_cast<const double2*>(st + lane * kCRec + 2 * (k ^ swr));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // out of the slot before the W staging
    }
    const int nb = base + step;
    const int ocn = min(nb + lane, P.no - 1);
    const int cn = P.obs_cam[ocn], pn = P.obs_pt[ocn];
    const float2 uvn = P.uv[ocn];
    const int v = P.vc[c];
    const double2* xr = reinterpret_cast<const double2*>(pxv + 4 * (size_t)p);
    const double2 x01 = xr[0], x2v = xr[1];
    const bool pv = x2v.y != 0.0;
    const bool live = base + lane < P.no && v >= 0 && pv;
    const double X0 = x01.x, X1 = x01.y, X2 = x2v.x;
    const double s0 = scale_p[p], s1 = scale_p[np + p], s2 = scale_p[2 * np + p];
    const double i00 = Linv[p], i10 = Linv[np + p], i11 = Linv[2 * np + p];
    const double i20 = Linv[3 * np + p], i21 = Linv[4 * np + p], i22 = Linv[5 * np + p];
    double j[kJR];
    bool fin;
    double prf[3];
    double sc[6];
    static_assert(TB == 0 || TB == 3, "camera source: LDS table or DMA-gathered compact records");
    if constexpr (TB == 3) {
      {
        const CamRc cam = cam_make(CamRcOf{rec, nullptr}, crp);
        (void)lin_obs(P, cam, v >= 0, pv, X0, X1, X2, uv, j, fin, prf);
      }
      // (v < 0: the record is zero, !live).  Three 16-B gathers, not six
      // 8-B ones: each touches a random camera's line per lane, so the
      // instruction count is what the address path pays for
      const double2* sv = reinterpret_cast<const double2*>(scale_c + (size_t)max(v, 0) * 6);
#pragma unroll
      for (int a = 0; a < 3; ++a) { const double2 x = sv[a]; sc[2 * a] = x.x; sc[2 * a + 1] = x.y; }
    } else {
      const CamLds cam{tbl + c * kTblRec, ktb + c * 9};
      (void)lin_obs(P, cam, cam.var(), pv, X0, X1, X2, uv, j, fin, prf);
#pragma unroll
      for (int a = 0; a < 6; ++a) sc[a] = sct[c * 6 + a];
    }
    const double jp0[3] = {j[12] * s0, j[13] * s1, j[14] * s2};
    const double jp1[3] = {j[15] * s0, j[16] * s1, j[17] * s2};
    constexpr int REC = COMPACT || PC ? kWcRec : kWRec;
    double wv[REC];
    if constexpr (PC) {
      pc_record(j, sc, {s0, s1, s2}, {i00, i10, i11, i20, i21, i22}, live, wv);
    } else if constexpr (COMPACT) {
      const double z[6] = {jp0[0] * i00, jp0[0] * i10 + jp0[1] * i11, jp0[0] * i20 + jp0[1] * i21 + jp0[2] * i22,
                           jp1[0] * i00, jp1[0] * i10 + jp1[1] * i11, jp1[0] * i20 + jp1[1] * i21 + jp1[2] * i22};
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        wv[a] = live ? j[a] * sc[a] : 0.0;
        wv[3 + a] = live ? j[6 + a] * sc[a] : 0.0;
        wv[6 + a] = live ? prf[a] : 0.0;   // pr0, pr1, f
      }
#pragma unroll
      for (int k = 0; k < 6; ++k) wv[9 + k] = live ? z[k] : 0.0;
      wv[15] = 0.0;
    } else {
#pragma unroll
      for (int a = 0; a < 6; ++a) {
        const double c0 = j[a] * sc[a], c1 = j[6 + a] * sc[a];
        const double e0 = c0 * jp0[0] + c1 * jp1[0];
        const double e1 = c0 * jp0[1] + c1 * jp1[1];
        const double e2 = c0 * jp0[2] + c1 * jp1[2];
        wv[a * 3 + 0] = live ? e0 * i00 : 0.0;
        wv[a * 3 + 1] = live ? e0 * i10 + e1 * i11 : 0.0;
        wv[a * 3 + 2] = live ? e0 * i20 + e1 * i21 + e2 * i22 : 0.0;
      }
    }
#pragma unroll
    for (int k = 0; k < REC; ++k) st[lane * kStageLd + k] = wv[k];
    wave_lds_sync();
    constexpr int NIT = REC / 2;
    V2 ov[NIT];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int e = it * 64 + lane;
      const int r = e / (REC / 2), f = 2 * (e - r * (REC / 2));
      ov[it].x = (WT)st[r * kStageLd + f];
      ov[it].y = (WT)st[r * kStageLd + f + 1];
    }
    wave_lds_sync();
    if constexpr (TB == 3) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the W records are out of the slot
      if (nb < P.no) crec_issue(cn);
    }
    V2* dst = reinterpret_cast<V2*>(W + (size_t)base * REC);
    const int nrec = min(64, P.no - base);
    if (nrec == 64) {
#pragma unroll
      for (int it = 0; it < NIT; ++it) nt_store(&dst[it * 64 + lane], ov[it]);
    } else {
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        const int e = it * 64 + lane;
        if (e / (REC / 2) < nrec) dst[e] = ov[it];
      }
    }
    c = cn; p = pn; uv = uvn;
  }
}

// PCG point pass without W (ITERATIVE_SCHUR beyond kLinLdsCams cameras, the
// rank-2 record conditions of k_obs_w_rc<.., PC> met): each lane forms its
// observation's 16-value record c, Z from the compact camera record as
// k_obs_w_rc<WT, false, 3, true> forms it (pc_record; rounded to WT, the
// stored record's values), then runs k_pcg_point_seg<WT, true, true>'s
// arithmetic on it (pc_v, the segmented per-point sum, pc_t) over the same
// point-aligned chunks.  What it trades: per LM iteration k_obs_w_rc's 128-B
// (fp64) record per observation, written once and read by every CG
// iteration (C4: 1.28 GB written, 1.28 GB read per matvec), against lin_obs
// once per matvec.  Per chunk two records per lane arrive by LDS-DMA, 8
// lanes per record (a wave-instruction touching 8 records, not 64): the
// compact camera record and the point record prec of k_point_elim (X, flag,
// s_p, L_p^-1) — the camera record one chunk ahead, the point record
// requested once its values are out of the slot (after lin_obs: holding them
// across lin_obs spilled registers).  The products leave through a third
// slot.  (Measured at C4: 520 us per working launch against 394 for
// k_pcg_point_seg on the stored records; without its stores 456: it runs at
// two waves per SIMD on lin_obs' ~250 VGPRs, latency-bound, not at the VALU
// or HBM limit.)
template <typename WT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_pcg_point_jf(
    DevProblem P, const int2* __restrict__ chunks, int nchunks, const double* __restrict__ crec,
    const double* __restrict__ prec, const double* __restrict__ scale_c, const double* __restrict__ xv,
    double* __restrict__ vpt, double* __restrict__ tobs, const double* __restrict__ st) {
  if (st[PS_DONE] != 0.0) return;
  static_assert(kCRec == 16 && kPRec == 16, "16-double records");
  __shared__ __attribute__((aligned(16))) double cbuf[4][64 * 16];
  __shared__ __attribute__((aligned(16))) double pbuf[4][64 * 16];
  __shared__ __attribute__((aligned(16))) double tbuf[4][64 * 6];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double* cb = cbuf[w];
  double* pb = pbuf[w];
  double* tst = tbuf[w];
  const int swr = (lane >> 1) & 7;
  auto issue = [&](const double* base, int idx, double* slot) {   // record idx of this lane into slot
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int q = (lane >> 3) + 8 * k;
      const int iq = __shfl(idx, q);
      glds16(base + (size_t)iq * 16 + 2 * ((lane & 7) ^ ((q >> 1) & 7)), slot + k * 128);
    }
  };
  auto piece = [&](const double* slot, int k) {   // piece k of this lane's record
    return *reinterpret_cast<const double2*>(slot + lane * 16 + 2 * (k ^ swr));
  };
  const int cs = gridDim.x * 4;
  int ch = blockIdx.x * 4 + w;
  if (ch >= nchunks) return;   // (uniform per wave; no workgroup barrier below)
  int2 cr = chunks[ch];
  int2 crn = ch + cs < nchunks ? chunks[ch + cs] : cr;
  int o = cr.x + min(lane, cr.y - cr.x - 1);
  int c = P.obs_cam[o], p = P.obs_pt[o], vc = P.obs_vc[o];
  float2 uv = P.uv[o];
  issue(crec, c, cb);
  issue(prec, p, pb);
  for (;;) {
    const int o0 = cr.x, n = cr.y - cr.x;
    double sc[6], x[6];   // s_c, x_c (L2-resident gathers)
    {
      const double2* sv = reinterpret_cast<const double2*>(scale_c + (size_t)max(vc, 0) * 6);
      const double2* xc = reinterpret_cast<const double2*>(xv + 6 * (size_t)max(vc, 0));
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        const double2 u = sv[a], y = xc[a];
        sc[2 * a] = u.x; sc[2 * a + 1] = u.y;
        x[2 * a] = y.x; x[2 * a + 1] = y.y;
      }
    }
    // the next chunk's indices
    const bool more = ch + cs < nchunks;
    const int on = crn.x + min(lane, crn.y - crn.x - 1);
    const int cn = P.obs_cam[on], pn = P.obs_pt[on], vcn = P.obs_vc[on];
    const float2 uvn = P.uv[on];
    const int2 crnn = ch + 2 * cs < nchunks ? chunks[ch + 2 * cs] : crn;
    CamRcPre crp;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this chunk's records have landed
#pragma unroll
    for (int k = 0; k < 8; ++k) crp.v[k] = piece(cb, k);
    const double2 x01 = piece(pb, 0), x2v = piece(pb, 1);   // X, the variable flag
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // read out before the next request
    if (more) issue(crec, cn, cb);
    const bool inl = lane < n;
    const bool pv = x2v.y != 0.0;
    const bool live = inl && vc >= 0 && pv;
    double j[kJR];
    {
      bool fin;
      double prf[3];
      const CamRc cam = cam_make(CamRcOf{crec, nullptr}, crp);
      (void)lin_obs(P, cam, vc >= 0, pv, x01.x, x01.y, x2v.x, uv, j, fin, prf);
    }
    double sp[3], li[6];   // s_p, L_p^-1 (prec[4..12])
    {
      const double2 q2 = piece(pb, 2), q3 = piece(pb, 3), q4 = piece(pb, 4), q5 = piece(pb, 5), q6 = piece(pb, 6);
      sp[0] = q2.x; sp[1] = q2.y; sp[2] = q3.x;
      li[0] = q3.y; li[1] = q4.x; li[2] = q4.y; li[3] = q5.x; li[4] = q5.y; li[5] = q6.x;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (more) issue(prec, pn, pb);
    // the record (k_obs_w_rc<.., PC>), rounded as stored
    double wr[16];
    {
      double wv[16];
      pc_record(j, sc, sp, li, live, wv);
#pragma unroll
      for (int k = 0; k < 16; ++k) wr[k] = (double)(WT)wv[k];
    }
    // k_pcg_point_seg<WT, true, true> from here
    double v[3];
    pc_v(wr, x, inl, v);
    const int pt = inl ? p : -1;
    const int ptp = __shfl_up(pt, 1, 64);
    const bool head = lane == 0 || pt != ptp;
    const unsigned long long heads = __ballot(head);
    const unsigned long long upto = lane == 63 ? ~0ull : ((1ull << (lane + 1)) - 1);
    const int h0 = 63 - __clzll(heads & upto);   // this lane's run head
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      double y[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) y[k] = __shfl_up(v[k], off, 64);
      if (lane - off >= h0) {
#pragma unroll
        for (int k = 0; k < 3; ++k) v[k] += y[k];
      }
    }
    const unsigned long long after = heads & ~upto;
    const int last = after ? __ffsll((long long)after) - 2 : n - 1;   // this run's last lane
    if (inl && lane == last) {
#pragma unroll
      for (int k = 0; k < 3; ++k) vpt[3 * (size_t)pt + k] = v[k];
    }
    {
      double vp[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) vp[k] = __shfl(v[k], last, 64);
      double tv[6];
      pc_t(wr, vp, tv);
      double2* td = reinterpret_cast<double2*>(&tst[lane * 6]);
#pragma unroll
      for (int a = 0; a < 3; ++a) td[a] = make_double2(tv[2 * a], tv[2 * a + 1]);
    }
    wave_lds_sync();
    {
      double2* dst = reinterpret_cast<double2*>(tobs + 6 * (size_t)o0);
      const double2* tsrc = reinterpret_cast<const double2*>(tst);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int e = k * 64 + lane;
        if (e < 3 * n) dst[e] = tsrc[e];
      }
    }
    wave_lds_sync();   // (the product slot is rewritten by the next chunk)
    if (!more) break;
    ch += cs;
    cr = crn; crn = crnn;
    o = on; c = cn; p = pn; vc = vcn; uv = uvn;
  }
}

// The diagonal Schur blocks and the reduced rhs per camera, J-free
// (k_cam_schur_diag without W): the camera's table row (or its compact
// record's dual Rodrigues) in registers, per observation the point's
// 128-B record (prec: X, s_p, L_p^-1, u_p) and the pixel in camera order,
// W_o formed as k_obs_w_rc forms it and consumed at once:
//   -sum W W^T (lower 21), -sum W u_p (6).  W32: W_o rounded to fp32 first
// (BA_MIXED_FP32: the preconditioner and the rhs see the stored fp32 blocks).
// Replaces a 72 / 144-B gather per observation from the point-major W.
template <int NT, int TB, bool W32>
__global__ __launch_bounds__(NT) void k_cam_schur_diag_rc(DevProblem P, const double* __restrict__ rec,
                                                          const double* __restrict__ prec,
                                                          const double* __restrict__ scale_c,
                                                          double* __restrict__ cpart) {
  __shared__ double lds[27 * 16];
  const int v = blockIdx.x;
  const int c = P.cam_of_vc[v];
  // (the camera in registers: its LDS form, as k_cam_assemble_rc's, drops
  // 244 -> 204 VGPRs, still two waves per SIMD; three spill 35)
  typename std::conditional<TB == 2, CamRcR, CamRegs>::type cam;
  if constexpr (TB == 2) {
    cam.make(cam_rc(rec, c));
  } else {
    const double2* s2 = reinterpret_cast<const double2*>(rec + (size_t)c * kCamRec + kRecL);
#pragma unroll
    for (int k = 0; k < kLin / 2; ++k) { const double2 q = s2[k]; cam.t[2 * k] = q.x; cam.t[2 * k + 1] = q.y; }
#pragma unroll
    for (int k = 0; k < 9; ++k) cam.k[k] = (double)P.K[9 * c + k];
  }
  double sc[6];
#pragma unroll
  for (int a = 0; a < 6; ++a) sc[a] = scale_c[(size_t)v * 6 + a];
  double acc[27];
#pragma unroll
  for (int k = 0; k < 27; ++k) acc[k] = 0.0;
  int i0, i1;
  cam_slice(P, v, i0, i1);
  for (int i = i0 + threadIdx.x; i < i1; i += NT) {
    const int p = P.cam_op[i].y;
    double r[kPRec];
    {
      const double2* q = reinterpret_cast<const double2*>(prec + (size_t)p * kPRec);
#pragma unroll
      for (int k = 0; k < kPRec / 2; ++k) { const double2 t = q[k]; r[2 * k] = t.x; r[2 * k + 1] = t.y; }
    }
    const bool pv = r[3] != 0.0;
    double j[kJR];
    bool fin;
    (void)lin_obs(P, cam, true, pv, r[0], r[1], r[2], P.uv_cm[i], j, fin);
    const double s0 = r[4], s1 = r[5], s2 = r[6];
    const double i00 = r[7], i10 = r[8], i11 = r[9], i20 = r[10], i21 = r[11], i22 = r[12];
    const double jp0[3] = {j[12] * s0, j[13] * s1, j[14] * s2};
    const double jp1[3] = {j[15] * s0, j[16] * s1, j[17] * s2};
    double w[kWRec];
#pragma unroll
    for (int a = 0; a < 6; ++a) {   // k_obs_w_rc's arithmetic
      const double c0 = j[a] * sc[a], c1 = j[6 + a] * sc[a];
      const double e0 = c0 * jp0[0] + c1 * jp1[0];
      const double e1 = c0 * jp0[1] + c1 * jp1[1];
      const double e2 = c0 * jp0[2] + c1 * jp1[2];
      double w0 = pv ? e0 * i00 : 0.0;
      double w1 = pv ? e0 * i10 + e1 * i11 : 0.0;
      double w2 = pv ? e0 * i20 + e1 * i21 + e2 * i22 : 0.0;
      if constexpr (W32) { w0 = (double)(float)w0; w1 = (double)(float)w1; w2 = (double)(float)w2; }
      w[a * 3 + 0] = w0; w[a * 3 + 1] = w1; w[a * 3 + 2] = w2;
    }
    const double u0 = r[13], u1 = r[14], u2 = r[15];
    int t = 0;
#pragma unroll
    for (int a = 0; a < 6; ++a) {   // k_cam_schur_diag's accumulation
#pragma unroll
      for (int b = 0; b <= a; ++b) acc[t++] += w[a * 3] * w[b * 3] + w[a * 3 + 1] * w[b * 3 + 1] + w[a * 3 + 2] * w[b * 3 + 2];
    }
#pragma unroll
    for (int a = 0; a < 6; ++a) acc[21 + a] += w[a * 3] * u0 + w[a * 3 + 1] * u1 + w[a * 3 + 2] * u2;
  }
  double tot[27];
  block_sum<27>(acc, lds, tot);
  cam_slice_store(tot, cpart, v, P.nvc);
}

// k_cam_schur_diag on compact records (W W^T = c^T (Z Z^T) c, W u = c^T (Z u)),
// the records and u gathered into LDS by LDS-DMA (as k_schur_pairs_cd: 8
// lanes per 128-B record, 2 per 32-B u record, pieces XOR-swizzled through
// the source address), one wave per workgroup (a thread has ~10
// observations at C3; at 256 threads ~2.5 and the 27-value reduction was a
// third of the instructions, profiles/r03_v12_pmc_sq.txt).  The next round's
// observation indices are loaded one round ahead, its DMA issued right after
// this round's records are read out of LDS.

// Back substitution of the points fused with the model cost change and the
// candidate cost (J-free; replaces k_backsub + a candidate pass).  Per point,
// LANES lanes (k_lin_point's layout):
//   pass 1  v = sum_o Jp_o^T (Jc_o dc_o) over the point's observations (J
//           recomputed at x), folded in the group; then
//           w = u_p + L_p^-1 (s_p o v) = u_p - sum_o W_o^T y_c  (W_o = s_c Jc^T
//           Jp s_p L_p^-T and s_c o y_c = -dc: the same step without reading
//           the 144-B W records), y_p = L_p^-T w, d_p = -s_p o y_p, x'_p.
//   pass 2  J d . (r + J d / 2) (Jc dc, Jp and r kept from pass 1 for the
//           lane's first KC observations, J again past them) and the
//           candidate residual at (camera', x'_p) per observation.
// TB 2 (nc > kLinLdsCams): rec is the compact records crec, rec_c the
// global candidate table ctbl (k_cand_table)
// ACC (ITERATIVE_SCHUR, W.pacc): no J at all.  Pass 1 is w = u_p - vacc_p
// (vacc = vpt(y), accumulated over the CG iterations: k_pcg_vacc); the model
// cost change is taken from the blocks instead of per observation:
//   (J d)^T (r + J d / 2) summed = g^T d + d^T H d / 2 with
//   d^T H d = sum_c dc^T Hcc dc + sum_p dp^T Hpp dp + 2 sum_p dp^T v_p,
//   v_p = sum_o Jp^T Jc dc = -(L_p vacc_p) / s_p, so dp^T v_p = yp^T (L_p vacc_p)
// — the point terms here (per point, Hpp and gp of the linearisation), the
// camera terms in k_cam_candidate (mcc_cam).  The same quantity as Ceres'
// per-residual sum, up to rounding.  Pass 2 is the candidate cost alone.
template <int NT, int LANES, int KC = 3, int TB = 0, bool ACC = false>
__global__ __launch_bounds__(NT) void k_point_step_rc(DevProblem P, const double* __restrict__ rec,
                                                      const double* __restrict__ pts,
                                                      const double* __restrict__ delta_c,
                                                      const double* __restrict__ rec_c, const double* __restrict__ u,
                                                      const double* __restrict__ Linv,
                                                      const double* __restrict__ scale_p, double* __restrict__ pts_c,
                                                      double* __restrict__ delta_p, double* __restrict__ part,
                                                      const double* __restrict__ vacc = nullptr,
                                                      const double* __restrict__ Hpp = nullptr,
                                                      const double* __restrict__ gp = nullptr) {
  __shared__ double lds[5 * 16];
  __shared__ __attribute__((aligned(16))) double tbl[TB ? 2 : kLinLdsCams * kTblRec];
  __shared__ float ktb[TB ? 1 : kLinLdsCams * 9];
  __shared__ __attribute__((aligned(16))) double ctb_s[TB ? 2 : kLinLdsCams * kCandRec];
  if constexpr (!TB) {
    fill_lin_table<NT>(P, rec, tbl, ktb);
    const int n = P.nc * kCandRec;
    for (int e = threadIdx.x; e < n; e += NT) ctb_s[e] = cand_entry(P, rec_c, delta_c, e);
    __syncthreads();
  }
  // the candidate rows (176 B, 16-B aligned) are read as 16-B pieces: beyond
  // 200 cameras each per-lane read touches a random camera's line, so the
  // number of read instructions is what the address path pays for
  const double* ctb = TB ? rec_c : ctb_s;
  auto row16 = [&](int c, int k0, double* dst, int n2) {   // entries k0 .. k0 + 2 n2 - 1 of row c
    const double2* s2 = reinterpret_cast<const double2*>(ctb + (size_t)c * kCandRec + k0);
    for (int k = 0; k < n2; ++k) { const double2 x = s2[k]; dst[2 * k] = x.x; dst[2 * k + 1] = x.y; }
  };
  double acc[5] = {0.0, 0.0, 0.0, 0.0, 0.0};   // step2, step_bad, mneg, ccost, cand_bad
  const size_t np = (size_t)P.np;
  const int sl = threadIdx.x & (LANES - 1);
  const int g0 = (blockIdx.x * NT + threadIdx.x) / LANES, gs = gridDim.x * NT / LANES;
  const int lastp = max(P.np - 1, 0), lasto = max(P.no - 1, 0);
  auto lin = [&](int c, bool pv, double X0, double X1, double X2, float2 uv, double (&j)[kJR]) {
    bool fin;
    if constexpr (TB == 2) {
      const CamRc cam = cam_rc(rec, c);
      (void)lin_obs(P, cam, cam.var(), pv, X0, X1, X2, uv, j, fin);
    } else {
      const CamLds cam{tbl + c * kTblRec, ktb + c * 9};
      (void)lin_obs(P, cam, cam.var(), pv, X0, X1, X2, uv, j, fin);
    }
  };
  int p = P.np > 0 ? g0 : P.np;
  if (P.np > 0) {
    int pc = min(p, lastp);
    int o0 = P.pt_off[pc], o1 = P.pt_off[pc + 1];
    double X0 = pts[3 * pc], X1 = pts[3 * pc + 1], X2 = pts[3 * pc + 2];
    bool pv = P.pt_var[pc] != 0;
    for (; p < P.np; p += gs) {   // uniform inside a lane group
      const int pn = min(p + gs, lastp);
      const int o0n = P.pt_off[pn], o1n = P.pt_off[pn + 1];
      const double Y0 = pts[3 * pn], Y1 = pts[3 * pn + 1], Y2 = pts[3 * pn + 2];
      const bool pvn = P.pt_var[pn] != 0;
      double dX[3] = {0.0, 0.0, 0.0};
      // the first KC observations of the lane keep what pass 2 needs from
      // pass 1's J (Jc dc, Jp, r: 10 doubles), so pass 2 recomputes J only
      // past them (points with more than LANES * KC observations) and for
      // fixed points (no pass 1)
      double kc[ACC ? 1 : KC][10];
      if (ACC && pv) {
        // w = u_p - vpt_p(y), the point step and its model-cost terms (lane 0)
        const double s0 = scale_p[p], s1 = scale_p[np + p], s2 = scale_p[2 * np + p];
        const double i00 = Linv[p], i10 = Linv[np + p], i11 = Linv[2 * np + p];
        const double i20 = Linv[3 * np + p], i21 = Linv[4 * np + p], i22 = Linv[5 * np + p];
        const double a0 = vacc[3 * (size_t)p], a1 = vacc[3 * (size_t)p + 1], a2 = vacc[3 * (size_t)p + 2];
        const double w0 = u[4 * p] - a0, w1 = u[4 * p + 1] - a1, w2 = u[4 * p + 2] - a2;
        const double yp[3] = {i00 * w0 + i10 * w1 + i20 * w2, i11 * w1 + i21 * w2, i22 * w2};
        const double sp[3] = {s0, s1, s2};
#pragma unroll
        for (int k = 0; k < 3; ++k) dX[k] = (-yp[k]) * sp[k];
        if (sl == 0) {
          // t = L_p vacc_p (L_p^-1 t = vacc_p)
          const double t0 = a0 / i00;
          const double t1 = (a1 - i10 * t0) / i11;
          const double t2 = (a2 - i20 * t0 - i21 * t1) / i22;
          const double h00 = Hpp[p], h10 = Hpp[np + p], h20 = Hpp[2 * np + p];
          const double h11 = Hpp[3 * np + p], h21 = Hpp[4 * np + p], h22 = Hpp[5 * np + p];
          const double hd0 = h00 * dX[0] + h10 * dX[1] + h20 * dX[2];
          const double hd1 = h10 * dX[0] + h11 * dX[1] + h21 * dX[2];
          const double hd2 = h20 * dX[0] + h21 * dX[1] + h22 * dX[2];
          const double gd = gp[p] * dX[0] + gp[np + p] * dX[1] + gp[2 * np + p] * dX[2];
          const double dhd = dX[0] * hd0 + dX[1] * hd1 + dX[2] * hd2;
          const double ytv = yp[0] * t0 + yp[1] * t1 + yp[2] * t2;
          acc[2] += gd + 0.5 * dhd + ytv;
        }
      } else if (!ACC && pv) {
        // pass 1: v = sum Jp^T (Jc dc)
        double v0 = 0.0, v1 = 0.0, v2 = 0.0;
        int o = o0 + sl;
        int oc = min(o, lasto);
        int c = P.obs_cam[oc];
        float2 uv = P.uv[oc];
        auto obs1 = [&](double (&keep)[10], bool store) {
          const int on = min(o + LANES, lasto);
          const int cn = P.obs_cam[on];
          const float2 uvn = P.uv[on];
          double j[kJR];
          lin(c, true, X0, X1, X2, uv, j);
          double dc[6];   // the camera step (0 for a fixed camera)
          row16(c, 16, dc, 3);
          double t0 = 0.0, t1 = 0.0;
#pragma unroll
          for (int a = 0; a < 6; ++a) { t0 += j[a] * dc[a]; t1 += j[6 + a] * dc[a]; }
          v0 += j[12] * t0 + j[15] * t1;
          v1 += j[13] * t0 + j[16] * t1;
          v2 += j[14] * t0 + j[17] * t1;
          if (store) {
            keep[0] = t0; keep[1] = t1;
#pragma unroll
            for (int k = 0; k < 8; ++k) keep[2 + k] = j[12 + k];
          }
          c = cn;
          uv = uvn;
          o += LANES;
        };
#pragma unroll
        for (int k = 0; k < KC; ++k)
          if (o < o1) obs1(kc[k], true);
        while (o < o1) obs1(kc[0], false);
#pragma unroll
        for (int x = LANES / 2; x >= 1; x >>= 1) {
          v0 += __shfl_xor(v0, x, LANES);
          v1 += __shfl_xor(v1, x, LANES);
          v2 += __shfl_xor(v2, x, LANES);
        }
        const double s0 = scale_p[p], s1 = scale_p[np + p], s2 = scale_p[2 * np + p];
        const double i00 = Linv[p], i10 = Linv[np + p], i11 = Linv[2 * np + p];
        const double i20 = Linv[3 * np + p], i21 = Linv[4 * np + p], i22 = Linv[5 * np + p];
        const double z0 = s0 * v0, z1 = s1 * v1, z2 = s2 * v2;
        const double w0 = u[4 * p] + i00 * z0;
        const double w1 = u[4 * p + 1] + (i10 * z0 + i11 * z1);
        const double w2 = u[4 * p + 2] + (i20 * z0 + i21 * z1 + i22 * z2);
        const double yp[3] = {i00 * w0 + i10 * w1 + i20 * w2, i11 * w1 + i21 * w2, i22 * w2};
        const double sp[3] = {s0, s1, s2};
#pragma unroll
        for (int k = 0; k < 3; ++k) dX[k] = (-yp[k]) * sp[k];
      }
      const double Xc[3] = {X0 + dX[0], X1 + dX[1], X2 + dX[2]};
      if (sl == 0) {
        const double Xk[3] = {X0, X1, X2};
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          pts_c[3 * p + k] = pv ? Xc[k] : Xk[k];
          delta_p[3 * p + k] = dX[k];
          if (pv) {
            const double e = Xk[k] - Xc[k];
            acc[0] += e * e;
            if (!isfinite(dX[k])) acc[1] += 1.0;
          }
        }
      }
      // pass 2: model cost change and candidate cost per observation
      {
        int o = o0 + sl;
        int oc = min(o, lasto);
        int c = P.obs_cam[oc];
        float2 uv = P.uv[oc];
        // keep: pass 1's values of this observation (nullptr: J again)
        auto obs2 = [&](const double* keep) {
          const int on = min(o + LANES, lasto);
          const int cn = P.obs_cam[on];
          const float2 uvn = P.uv[on];
          const bool cfix = P.cam_fixed && P.cam_fixed[c];
          // k_candidate_lds' arithmetic
          double jd0 = 0.0, jd1 = 0.0, jp[6], r0 = 0.0, r1 = 0.0;
          if constexpr (ACC) {
            (void)jp;
          } else if (keep) {
            jd0 = keep[0]; jd1 = keep[1];
#pragma unroll
            for (int k = 0; k < 6; ++k) jp[k] = keep[2 + k];
            r0 = keep[8]; r1 = keep[9];
          } else {
            double j[kJR];
            lin(c, pv, X0, X1, X2, uv, j);
            jd0 = 0.0; jd1 = 0.0;
            double dc[6];
            row16(c, 16, dc, 3);
#pragma unroll
            for (int a2 = 0; a2 < 6; ++a2) { jd0 += j[a2] * dc[a2]; jd1 += j[6 + a2] * dc[a2]; }
#pragma unroll
            for (int k = 0; k < 6; ++k) jp[k] = j[12 + k];
            r0 = j[18]; r1 = j[19];
          }
          double mneg = 0.0;
          if constexpr (!ACC) {
            jd0 += jp[0] * dX[0] + jp[1] * dX[1] + jp[2] * dX[2];
            jd1 += jp[3] * dX[0] + jp[4] * dX[1] + jp[5] * dX[2];
            mneg = jd0 * (r0 + jd0 / 2.0) + jd1 * (r1 + jd1 / 2.0);
          }
          double pcand[3];
          if (!cfix) {
            double cr[12];
            row16(c, 0, cr, 6);
#pragma unroll
            for (int i = 0; i < 3; ++i) pcand[i] = cr[i] * Xc[0] + cr[3 + i] * Xc[1] + cr[6 + i] * Xc[2] + cr[9 + i];
          } else {
            double cr[16];
            row16(c, 0, cr, 8);
            double ph[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) ph[i] = Xc[0] * cr[i] + Xc[1] * cr[4 + i] + Xc[2] * cr[8 + i] + cr[12 + i];
            pcand[0] = ph[0] / ph[3]; pcand[1] = ph[1] / ph[3]; pcand[2] = ph[2] / ph[3];
          }
          // TB 2: K from the compact record (the same floats as P.K, packed
          // two per double at kCRecK: three 16-B reads instead of nine 4-B)
          float kq[12];
          if constexpr (TB == 2) {
            const double2* s2 = reinterpret_cast<const double2*>(rec + (size_t)c * kCRec + kCRecK);
#pragma unroll
            for (int k = 0; k < 3; ++k) {
              const double2 x = s2[k];
              const unsigned long long a = __builtin_bit_cast(unsigned long long, x.x);
              const unsigned long long b = __builtin_bit_cast(unsigned long long, x.y);
              kq[4 * k] = __builtin_bit_cast(float, (unsigned)a);
              kq[4 * k + 1] = __builtin_bit_cast(float, (unsigned)(a >> 32));
              kq[4 * k + 2] = __builtin_bit_cast(float, (unsigned)b);
              kq[4 * k + 3] = __builtin_bit_cast(float, (unsigned)(b >> 32));
            }
          }
          const float* Kc = TB == 2 ? kq : ktb + c * 9;
          double q[3];
#pragma unroll
          for (int i = 0; i < 3; ++i)
            q[i] = pcand[0] * (double)Kc[i] + pcand[1] * (double)Kc[3 + i] + pcand[2] * (double)Kc[6 + i];
          const double rc0 = q[0] / q[2] - (double)uv.x, rc1 = q[1] / q[2] - (double)uv.y;
          double sc;
          const double rho = huber(rc0 * rc0 + rc1 * rc1, P.huber_a, P.huber_b, &sc);
          if constexpr (!ACC) acc[2] += mneg;
          acc[3] += 0.5 * rho;
          if (!isfinite(rc0) || !isfinite(rc1)) acc[4] += 1.0;
          c = cn;
          uv = uvn;
          o += LANES;
        };
        if (!ACC && pv) {
#pragma unroll
          for (int k = 0; k < KC; ++k)
            if (o < o1) obs2(kc[ACC ? 0 : k]);
        }
        while (o < o1) obs2(nullptr);
      }
      o0 = o0n; o1 = o1n;
      X0 = Y0; X1 = Y1; X2 = Y2;
      pv = pvn;
    }
  }
  double tot[5];
  block_sum<5>(acc, lds, tot);
  if (threadIdx.x == 0) {
    part_of(part, SL_STEP2_P)[blockIdx.x] = tot[0];
    part_of(part, SL_STEP_BAD)[blockIdx.x] += tot[1];
    if (ACC) part_of(part, SL_MCC_NEG)[blockIdx.x] += tot[2];   // (k_cam_candidate's camera terms are there)
    else part_of(part, SL_MCC_NEG)[blockIdx.x] = tot[2];
    part_of(part, SL_CCOST)[blockIdx.x] = tot[3];
    part_of(part, SL_CAND_BAD)[blockIdx.x] = tot[4];
  }
}

void launch_cam_prep(const DevProblem& P, const double* cams, double* rec, bool deriv, hipStream_t s) {
  if (P.nc == 0) return;
  hipLaunchKernelGGL(k_cam_prep, dim3(P.nc), dim3(64), 0, s, P.nc, cams, P.K, P.cam_fixed, P.extr, rec,
                     deriv ? 1 : 0);
}
// one 512-thread block per CU for the LDS-table kernels
static int lds_grid(int n) {
  static int n_cu = 0;
  if (n_cu == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0)
      n_cu = 256;
  }
  int g = (n + kLinLdsThreads - 1) / kLinLdsThreads;
  return g < 1 ? 1 : (g > n_cu ? n_cu : g);
}

// camera source of the J-free kernels: 0 the LDS copy of the records' lin
// tables (nc <= kLinLdsCams), 2 beyond: the compact records crec (each
// observation forms its camera's dual Rodrigues from them)
static int jr_tab(const DevProblem& P, const DevWork& W) { return W.jrfree && P.nc > kLinLdsCams ? 2 : 0; }
void launch_lin_prep(const DevProblem& P, const DevWork& W, hipStream_t s) {
  if (P.nc > kLinLdsCams) {   // (the JR path's k_linearize_rc reads them too)
    hipLaunchKernelGGL(k_cam_compact, dim3((P.nc + 255) / 256), dim3(256), 0, s, P, W.cams, W.crec);
    return;
  }
  launch_cam_prep(P, W.cams, W.rec, true, s);
}
// the W writers have a 16-value PCG record form (k_obs_w_rc<.., PC>) for the
// LDS camera table (TB 0) and the DMA-gathered compact records (TB 3)
bool obs_w_pc_ok(const DevProblem&, const DevWork& W) { return W.jrfree; }
void launch_linearize(const DevProblem& P, const DevWork& W, hipStream_t s, hipEvent_t t0, hipEvent_t t1) {
  // t0 / t1 (optional): start / stop of the kernel's execution, stamped by
  // hipExtLaunchKernel itself (no separate event records around the launch)
  if (W.jrfree) return;   // J-free: r and J are formed inside k_lin_point (launch_point_assemble)
  launch_linearize_jr(P, W, s, t0, t1);
}
// the JR-writing linearisation (also ba_linearize's read-back in J-free mode)
void launch_linearize_jr(const DevProblem& P, const DevWork& W, hipStream_t s, hipEvent_t t0, hipEvent_t t1) {
  if (P.nc > 0 && P.nc <= kLinLdsCams) {
    hipExtLaunchKernelGGL((k_linearize_lds_t<kLinNT, kLinRows>), dim3(lds_grid(P.no)), dim3(kLinNT), 0, s, t0, t1, 0,
                          P, (const double*)W.rec, (const double*)W.pts, W.JR, W.part);
    return;
  }
  // (J-free beyond kLinLdsCams cameras, ba_linearize's read-back: the
  // compact-record kernel forms the camera terms in the order of the J-free
  // consumers, so the records are bitwise what they compute)
  hipExtLaunchKernelGGL(k_linearize_rc, dim3(grid_for(P.no)), dim3(kThreads), 0, s, t0, t1, 0, P,
                        (const double*)W.crec, (const double*)W.pts, W.JR, W.part);
}
void launch_point_assemble(const DevProblem& P, const DevWork& W, bool compute_scale, double min_diag,
                           double max_diag, hipStream_t s, hipEvent_t t0, hipEvent_t t1) {
  if (W.jrfree) {   // r, J, cost and the point blocks in one pass (J never materialised)
    // 2 lanes per point, 256 threads: 30.7 us at C3 vs 32.4 at 4 lanes and 38
    // at 512 threads; lazy table reads 42.5 (profiles/r03_v4_ab_lin_point.txt).
    // Two 74-KB-LDS workgroups per CU at most: a grid of that size,
    // grid-stride over the points (no second round of table fills)
    const int want = (int)std::min<long long>(((long long)P.np * 2 + 255) / 256, 1LL << 30);
    if (jr_tab(P, W)) {
      // beyond 200 cameras the compact camera records by LDS-DMA (wave-uniform
      // point rounds): C5 shard 386.5 -> 331.3 us against per-lane register
      // gathers, C4 2883 -> 2896 M-obs/s (profiles/r04_v11_ab_lp_dma.txt)
      const int g = std::max(1, std::min(want, kMaxBlocks));
      hipExtLaunchKernelGGL((k_lin_point_d<256, 2>), dim3(g), dim3(256), 0, s, t0, t1, 0, P, (const double*)W.crec,
                            (const double*)W.pts, W.Hpp, W.gp, W.scale_p, W.diag_p, compute_scale ? 1 : 0, min_diag,
                            max_diag, W.part, W.pxv);
      return;
    }
    const int g = std::max(1, std::min(want, 2 * lds_grid(1 << 30)));
    hipExtLaunchKernelGGL((k_lin_point<256, 2>), dim3(g), dim3(256), 0, s, t0, t1, 0, P, (const double*)W.rec,
                          (const double*)W.pts, W.Hpp, W.gp, W.scale_p, W.diag_p, compute_scale ? 1 : 0, min_diag,
                          max_diag, W.part, W.pxv);
    return;
  }
  const bool many = P.nc > kLinLdsCams;
  hipLaunchKernelGGL((many ? k_point_assemble<jr_ja(true)> : k_point_assemble<jr_ja(false)>),
                     dim3(grid_for((int)std::min<long long>((long long)P.np * kPaLanes, 1LL << 30))),
                     dim3(kThreads), 0, s, P, W.JR, W.pts, W.Hpp, W.gp,
                     W.scale_p, W.diag_p, compute_scale ? 1 : 0, min_diag, max_diag, W.part);
}
void launch_cam_assemble(const DevProblem& P, const DevWork& W, hipStream_t s) {
  if (P.nvc == 0) return;
  if (W.jrfree) {
    // one 512-thread workgroup per camera: 30.6 us vs 37 / 49 us at 2 / 4
    // slices, 32.5 us at 256 threads x 2 (profiles/r03_v13_ab_pairs_ca.txt)
    const dim3 g(P.nvc);
    if (jr_tab(P, W) == 2) {
      // (the compact records: the camera's dual Rodrigues once per
      // workgroup).  Threads per camera by its observations (~8 per thread):
      // at 10k cameras x 1250 observations a 512-thread workgroup had 2.4
      // per thread and the per-workgroup setup and 27-value reduction
      // dominated (C5 shard 642 us)
      const int per = (int)std::max<long long>(1, (long long)P.no / std::max(P.nvc, 1));
      const int t = per >= 8 * 512 ? 512 : (per >= 8 * 256 ? 256 : (per >= 8 * 128 ? 128 : 64));
      const double* cr = W.crec;
      if (t == 512)
        hipLaunchKernelGGL((k_cam_assemble_rc<512, 2>), g, dim3(512), 0, s, P, cr, (const double*)W.pxv, W.cpart, W.Hcc, W.gc);
      else if (t == 256)
        hipLaunchKernelGGL((k_cam_assemble_rc<256, 2>), g, dim3(256), 0, s, P, cr, (const double*)W.pxv, W.cpart, W.Hcc, W.gc);
      else if (t == 128)
        hipLaunchKernelGGL((k_cam_assemble_rc<128, 2>), g, dim3(128), 0, s, P, cr, (const double*)W.pxv, W.cpart, W.Hcc, W.gc);
      else
        hipLaunchKernelGGL((k_cam_assemble_rc<64, 2>), g, dim3(64), 0, s, P, cr, (const double*)W.pxv, W.cpart, W.Hcc, W.gc);
    } else {
      hipLaunchKernelGGL(k_cam_assemble_rc<512>, g, dim3(512), 0, s, P, (const double*)W.rec, (const double*)W.pxv,
                         W.cpart, W.Hcc, W.gc);
    }
    return;
  }
  const bool many = P.nc > kLinLdsCams;   // JR layout (jr_ja)
  // one 512-thread workgroup per camera: measured faster than slicing at C3
  // (57 vs 66 us at 8 slices) and at C5 (where 2048 / nvc < 1 anyway); 54 us
  // at 512 threads, 57 at 256 / 1024
  hipLaunchKernelGGL((many ? k_cam_assemble<512, jr_ja(true)> : k_cam_assemble<512, jr_ja(false)>), dim3(P.nvc),
                     dim3(512), 0, s, P, W.JR, W.cpart, W.Hcc, W.gc);
}
NormsFold norms_fold(const DevWork& W, bool compute_scale, double min_diag, double max_diag) {
  return NormsFold{W.cams, W.Hcc, W.gc, W.scale_c, W.diag_c, compute_scale ? 1 : 0, min_diag, max_diag};
}
void launch_cam_norms(const DevProblem& P, const DevWork& W, bool compute_scale, double min_diag, double max_diag,
                      hipStream_t s) {
  hipLaunchKernelGGL(k_cam_norms, dim3(grid_for(P.nvc)), dim3(kThreads), 0, s, P, W.cams, W.Hcc, W.gc, W.scale_c,
                     W.diag_c, compute_scale ? 1 : 0, min_diag, max_diag, W.part);
}
void launch_point_elim(const DevProblem& P, const DevWork& W, double radius, hipStream_t s, const NormsFold* nf) {
  double* prec = W.jdiag ? W.prec : nullptr;
  if (nf) {
    const int nbp = grid_for(P.np);
    hipLaunchKernelGGL(k_point_elim_norms, dim3(nbp + grid_for(P.nvc)), dim3(kThreads), 0, s, P, W.Hpp, W.gp,
                       W.scale_p, W.diag_p, radius, W.Linv, W.u, W.part, (const double*)W.pts, prec, nbp, *nf);
  } else {
    hipLaunchKernelGGL(k_point_elim, dim3(grid_for(P.np)), dim3(kThreads), 0, s, P, W.Hpp, W.gp, W.scale_p, W.diag_p,
                       radius, W.Linv, W.u, W.part, (const double*)W.pts, prec);
  }
  if (P.no == 0) return;
  if (W.pcgjf) return;   // (no W: the PCG point pass forms the records itself)
  if (jr_tab(P, W)) {
    // the compact camera records gathered by LDS-DMA through the W staging
    // slot (C5 shard 707 -> 568 us against register gathers), 64.5 KB of
    // staging LDS: two 4-wave workgroups per CU at ~230 VGPRs (C5 shard
    // 3346-3349 vs 3315-3320 M-obs/s for one 6-wave workgroup,
    // profiles/r04_v18_obsw_waves_ab.txt)
    constexpr int WG = kObsWRcWavesG;
    const int g = std::min(2 * lds_grid(1 << 30), std::max(1, (P.no + 64 * WG - 1) / (64 * WG)));
    const double* src = W.crec;
    const dim3 b(64 * WG);
    if (W.pcgc && W.w32)
      hipLaunchKernelGGL((k_obs_w_rc<float, false, 3, true, WG>), dim3(g), b, 0, s, P, src, (const double*)W.pxv,
                         W.scale_c, W.scale_p, W.Linv, W.Wf);
    else if (W.pcgc)
      hipLaunchKernelGGL((k_obs_w_rc<double, false, 3, true, WG>), dim3(g), b, 0, s, P, src, (const double*)W.pxv,
                         W.scale_c, W.scale_p, W.Linv, W.W);
    else if (W.w32)
      hipLaunchKernelGGL((k_obs_w_rc<float, false, 3, false, WG>), dim3(g), b, 0, s, P, src, (const double*)W.pxv,
                         W.scale_c, W.scale_p, W.Linv, W.Wf);
    else if (W.wcompact)   // (DENSE_SCHUR up to kWcCamsHost variable cameras: the compact records)
      hipLaunchKernelGGL((k_obs_w_rc<double, true, 3, false, WG>), dim3(g), b, 0, s, P, src, (const double*)W.pxv,
                         W.scale_c, W.scale_p, W.Linv, W.W);
    else
      hipLaunchKernelGGL((k_obs_w_rc<double, false, 3, false, WG>), dim3(g), b, 0, s, P, src, (const double*)W.pxv,
                         W.scale_c, W.scale_p, W.Linv, W.W);
    return;
  }
  if (W.jrfree) {   // one 148-KB-LDS workgroup per CU
    const int g = lds_grid(P.no);
    if (W.pcgc && W.w32)
      hipLaunchKernelGGL((k_obs_w_rc<float, false, 0, true>), dim3(g), dim3(64 * kObsWRcWaves), 0, s, P,
                         (const double*)W.rec, (const double*)W.pxv, W.scale_c, W.scale_p, W.Linv, W.Wf);
    else if (W.pcgc)
      hipLaunchKernelGGL((k_obs_w_rc<double, false, 0, true>), dim3(g), dim3(64 * kObsWRcWaves), 0, s, P,
                         (const double*)W.rec, (const double*)W.pxv, W.scale_c, W.scale_p, W.Linv, W.W);
    else if (W.w32)
      hipLaunchKernelGGL(k_obs_w_rc<float>, dim3(g), dim3(64 * kObsWRcWaves), 0, s, P, (const double*)W.rec,
                         (const double*)W.pxv, W.scale_c, W.scale_p, W.Linv, W.Wf);
    else if (W.wcompact)
      hipLaunchKernelGGL((k_obs_w_rc<double, true>), dim3(g), dim3(64 * kObsWRcWaves), 0, s, P, (const double*)W.rec,
                         (const double*)W.pxv, W.scale_c, W.scale_p, W.Linv, W.W);
    else
      hipLaunchKernelGGL(k_obs_w_rc<double>, dim3(g), dim3(64 * kObsWRcWaves), 0, s, P, (const double*)W.rec,
                         (const double*)W.pxv, W.scale_c, W.scale_p, W.Linv, W.W);
    return;
  }
  const int g = lds_grid(P.no);
  if (W.w32) {
    if (P.nc <= kLinLdsCams)
      hipLaunchKernelGGL((k_obs_w<true, float>), dim3(g), dim3(512), 0, s, P, W.JR, W.scale_c, W.scale_p, W.Linv, W.Wf);
    else
      hipLaunchKernelGGL((k_obs_w<false, float>), dim3(g), dim3(512), 0, s, P, W.JR, W.scale_c, W.scale_p, W.Linv, W.Wf);
  } else {
    if (P.nc <= kLinLdsCams)
      hipLaunchKernelGGL((k_obs_w<true, double>), dim3(g), dim3(512), 0, s, P, W.JR, W.scale_c, W.scale_p, W.Linv, W.W);
    else
      hipLaunchKernelGGL((k_obs_w<false, double>), dim3(g), dim3(512), 0, s, P, W.JR, W.scale_c, W.scale_p, W.Linv, W.W);
  }
}
void launch_pcg_point_jf(const DevProblem& P, const DevWork& W, const double* vec, hipStream_t s) {
  const double* st = W.scal + kNumSlots;
  // (two 4-wave workgroups per CU at ~250 VGPRs, 76 KB of LDS each: a grid of
  // that size, chunk-stride)
  const int g = std::max(1, std::min((W.npchunks + 3) / 4, 2 * lds_grid(1 << 30)));
  if (W.w32)
    hipLaunchKernelGGL(k_pcg_point_jf<float>, dim3(g), dim3(256), 0, s, P, W.pchunks, W.npchunks,
                       (const double*)W.crec, (const double*)W.prec, W.scale_c, vec, W.vpt, W.tobs, st);
  else
    hipLaunchKernelGGL(k_pcg_point_jf<double>, dim3(g), dim3(256), 0, s, P, W.pchunks, W.npchunks,
                       (const double*)W.crec, (const double*)W.prec, W.scale_c, vec, W.vpt, W.tobs, st);
}
// camera slices of the diagonal pass
int cam_split_count(const DevWork& W) { return W.cam_split; }
void launch_cam_schur_diag(const DevProblem& P, const DevWork& W, hipStream_t s, double* compact, double radius,
                           bool skip_fold) {
  if (P.nvc == 0) return;
  const int sl = cam_split_count(W);
  // threads per camera slice by its observations (~8 per thread): 256, or
  // 128 at C5's 1250 observations per camera
  const int per = (int)std::max<long long>(1, (long long)P.no / std::max(P.nvc * sl, 1));
  const bool t128 = per < 8 * 256;
  if (W.jdiag) {   // J-free (no W read): the camera's row in registers, the point records gathered
    const dim3 g(P.nvc, sl);
    const int tb = jr_tab(P, W) == 2 ? 2 : 0;
    const double* src = tb == 2 ? (const double*)W.crec : (const double*)W.rec;
    const double* pr = W.prec;
#define BA_DIAG_RC(NT_, TB_, W32_) \
    hipLaunchKernelGGL((k_cam_schur_diag_rc<NT_, TB_, W32_>), g, dim3(NT_), 0, s, P, src, pr, W.scale_c, W.cpart)
    if (tb == 2) {
      if (t128) { if (W.w32) BA_DIAG_RC(128, 2, true); else BA_DIAG_RC(128, 2, false); }
      else { if (W.w32) BA_DIAG_RC(256, 2, true); else BA_DIAG_RC(256, 2, false); }
    } else {
      if (t128) { if (W.w32) BA_DIAG_RC(128, 0, true); else BA_DIAG_RC(128, 0, false); }
      else { if (W.w32) BA_DIAG_RC(256, 0, true); else BA_DIAG_RC(256, 0, false); }
    }
#undef BA_DIAG_RC
  } else if (W.w32 && t128)
    hipLaunchKernelGGL((k_cam_schur_diag<float, 128>), dim3(P.nvc, sl), dim3(128), 0, s, P, W.Wf, W.u, W.S, W.cpart);
  else if (W.w32)
    hipLaunchKernelGGL(k_cam_schur_diag<float>, dim3(P.nvc, sl), dim3(kThreads), 0, s, P, W.Wf, W.u, W.S, W.cpart);
  else if (W.wcompact) {
    // compact records + 32-B u records gathered by LDS-DMA, two lanes each,
    // 64-thread workgroups: 46.6 -> 37.9 us against the register gathers at
    // C3 (profiles/r04_v8_ab_diag_dma.txt; 64 threads: 49 vs 65.5 us at 256,
    // profiles/r03_v13_ab_diag_nt.txt)
    hipLaunchKernelGGL(k_cam_schur_diag_cd, dim3(P.nvc, sl), dim3(64), 0, s, P, W.W, W.scale_c, W.u, W.cpart);
  }
  else
    hipLaunchKernelGGL(k_cam_schur_diag<double>, dim3(P.nvc, sl), dim3(kThreads), 0, s, P, W.W, W.u, W.S, W.cpart);
  if (skip_fold) return;   // (the pair pass's launch folds: launch_schur_pairs)
  if (!compact && radius > 0.0) {   // single rank: the LM diagonal goes in with the fold
    hipLaunchKernelGGL(k_cam_fold_diag, dim3((P.nvc * 27 + 255) / 256), dim3(256), 0, s, P, W.cpart, sl, W.Hcc,
                       W.gc, W.scale_c, W.diag_c, radius, W.S, W.scal);
    return;
  }
  hipLaunchKernelGGL(k_cam_fold, dim3((P.nvc * 27 + 255) / 256), dim3(256), 0, s, P, W.cpart, sl,
                     compact ? 2 : 1, W.Hcc,
                     W.gc, compact ? compact : W.S);
}
// the diagonal fold (k_cam_fold_diag) can ride in the pair pass's launch
// (one launch fewer: C3 1517-1556 vs 1494-1512 M-obs/s,
// profiles/r04_v14_ab_fusions_psdma.txt)
bool pairs_take_fold(const DevProblem& P, const DevWork& W) {
  return W.nblocks > 0 && W.wcompact && kPairsDmaLds + sizeof(WcCam) * (size_t)P.nvc <= 80 * 1024;
}
void launch_cam_fold_diag(const DevProblem& P, const DevWork& W, double radius, hipStream_t s) {
  hipLaunchKernelGGL(k_cam_fold_diag, dim3((P.nvc * 27 + 255) / 256), dim3(256), 0, s, P, W.cpart,
                     cam_split_count(W), W.Hcc, W.gc, W.scale_c, W.diag_c, radius, W.S, W.scal);
}
bool pairs_take_diag(const DevProblem& P, const DevWork& W) {
  const char* e = getenv("BA_DIAG_IN_PAIRS");
  return !(e && e[0] == '0') && pairs_take_fold(P, W) && !W.jdiag && !W.w32 && P.nvc > 0;
}
// ... beyond the LDS camera table (k_schur_pairs_cd<false>, 1000 cameras):
// the diagonal slices' waves use the same 64 KB of DMA buffers, so they ride
// there too (the fold then follows in its own launch)
bool pairs_take_diag_nt(const DevProblem& P, const DevWork& W) {
  const char* e = getenv("BA_DIAG_IN_PAIRS");
  const char* de = getenv("BA_PAIRS_DMA");
  return !(e && e[0] == '0') && !(de && de[0] == '0') && W.nblocks > 0 && W.wcompact && !pairs_take_fold(P, W) &&
         !W.jdiag && !W.w32 && P.nvc > 0;
}
void launch_schur_pairs(const DevProblem& P, const DevWork& W, hipStream_t s, double fold_radius, bool with_diag) {
  if (W.nblocks == 0) return;
  // 16 blocks per workgroup (4 waves of 4) over the largest XCD range, at
  // most 2048 workgroups (256 sweeping the ranges in rounds ties it:
  // profiles/r02_v7_ab_pairs_grid_np.txt)
  const int* xoff = W.xoff;
  int grid = 8 * ((W.xmax + 15) / 16);
  if (grid == 0) return;
  if (grid > 2048) grid = 2048;
  grid = (grid + 7) / 8 * 8;   // k_schur_pairs' XCD ranges need a multiple of 8
  // the LDS-DMA gather form while its 64 KB + the camera constants fit half
  // the LDS (two workgroups per CU): C3 159 -> 121 us, 1409-1424 -> 1487-1503
  // M-obs/s (profiles/r04_v7_ab_pairs_dma.txt); beyond, the register form
  const size_t ctab_bytes = sizeof(WcCam) * (size_t)P.nvc;
  const bool ctab = kPairsDmaLds + ctab_bytes <= 80 * 1024;
  const char* de = getenv("BA_PAIRS_DMA");   // (0: the register gathers beyond the LDS camera table; A/B)
  if (W.wcompact && !ctab && !(de && de[0] == '0')) {
    // 1000 cameras (C4): LDS-DMA gathers with the camera constants per block
    // in registers
    FoldArgs fa{W.cpart, 0, W.Hcc, W.gc, W.diag_c, 0.0, W.scal};
    int fgrid = 0;
    if (with_diag) {   // the diagonal slices ride in this launch (dispatched last: they fill the pairs' tail)
      fa.u = W.u;
      fa.G = cam_split_count(W);
      fgrid = (P.nvc * fa.G + 3) / 4;
    }
    hipLaunchKernelGGL(k_schur_pairs_cd<false>, dim3(grid + fgrid), dim3(256), kPairsDmaLds, s, P, W.blocks, xoff,
                       W.pairs, W.W, W.scale_c, W.S, grid, fa);
  }
  else if (W.wcompact && ctab) {
    FoldArgs fa{W.cpart, 0, W.Hcc, W.gc, W.diag_c, fold_radius, W.scal};
    int fgrid = 0;
    if (with_diag) {   // the diagonal slices ride in this launch (dispatched last: they fill the pairs' tail)
      fa.u = W.u;
      fa.G = cam_split_count(W);
      fgrid = (P.nvc * fa.G + 3) / 4;
    } else if (fold_radius > 0.0) {   // the diagonal fold rides in this launch
      fa.nsl = cam_split_count(W);
      fgrid = (P.nvc * 27 + 255) / 256;
    }
    hipLaunchKernelGGL(k_schur_pairs_cd<true>, dim3(grid + fgrid), dim3(256), kPairsDmaLds + ctab_bytes, s, P, W.blocks,
                       xoff, W.pairs, W.W, W.scale_c, W.S, grid, fa);
  }
  else if (W.wcompact)
    hipLaunchKernelGGL(k_schur_pairs_c, dim3(grid), dim3(256), ctab_bytes, s, P, W.blocks, xoff,
                       W.pairs, W.W, W.scale_c, W.S);
  else
    hipLaunchKernelGGL(k_schur_pairs, dim3(grid), dim3(256), 0, s, P, W.blocks, xoff, W.pairs, W.W, W.S);
}
// one workgroup per row of S: row i < n holds its lower part (j <= i), row n
// the rhs (all n entries)
__global__ __launch_bounds__(256) void k_pack_lower(int n, int ld, double* __restrict__ S, double* __restrict__ pk,
                                                    double* __restrict__ scal, int pack) {
  const int i = blockIdx.x;
  if (i == 0 && threadIdx.x == 0) {   // the elimination-failure count travels in the last slot
    const size_t tail = (size_t)n * (n + 1) / 2 + n;
    if (pack) pk[tail] = scal[SL_ELIM_BAD];
    else scal[SL_ELIM_BAD] = pk[tail];
  }
  const size_t off = (size_t)i * (i + 1) / 2;   // row n: n(n+1)/2, the rhs
  const int len = i < n ? i + 1 : n;
  double* row = S + (size_t)i * ld;
  for (int j = threadIdx.x; j < len; j += blockDim.x) {
    if (pack) pk[off + j] = row[j];
    else row[j] = pk[off + j];
  }
}
void launch_pack_lower(const DevProblem& P, const DevWork& W, bool pack, hipStream_t s) {
  if (P.n == 0) return;
  hipLaunchKernelGGL(k_pack_lower, dim3(P.n + 1), dim3(256), 0, s, P.n, P.ld, W.S, W.Spk, W.scal, pack ? 1 : 0);
}
__global__ __launch_bounds__(256) void k_zero_blocks(int ld, const int2* __restrict__ eb, int nb,
                                                     double* __restrict__ S) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nb * 36) return;
  const int2 b = eb[e / 36];
  const int k = e % 36;
  S[(size_t)(6 * b.x + k / 6) * ld + 6 * b.y + k % 6] = 0.0;
}
void launch_zero_blocks(const DevProblem& P, const DevWork& W, hipStream_t s) {
  if (W.neblocks == 0) return;
  hipLaunchKernelGGL(k_zero_blocks, dim3((W.neblocks * 36 + 255) / 256), dim3(256), 0, s, P.ld, W.eblocks, W.neblocks,
                     W.S);
}
void launch_cam_add_diag(const DevProblem& P, const DevWork& W, double radius, hipStream_t s) {
  if (P.nvc == 0) return;
  hipLaunchKernelGGL(k_cam_add_diag, dim3((P.nvc * 27 + 255) / 256), dim3(256), 0, s, P, W.Hcc, W.gc, W.scale_c,
                     W.diag_c, radius, W.S, W.scal);
}
void launch_cam_candidate(const DevProblem& P, const DevWork& W, hipStream_t s) {
  if (P.nc == 0) return;
  // (the camera terms of the block-form model cost change: once over the
  // ranks, on rank 0 — SL_MCC_NEG is summed across them)
  const bool mc = W.pacc && W.mcc_cam;
  hipLaunchKernelGGL(k_cam_candidate, dim3(P.nc < kMaxBlocks ? P.nc : kMaxBlocks), dim3(64), 0, s, P, W.cams, W.y,
                     W.scale_c, W.cams_c, W.delta_c, W.rec_c, W.part, mc ? (const double*)W.Hcc : nullptr,
                     mc ? (const double*)W.gc : nullptr);
}
// J-free: back substitution + model cost change + candidate cost in one
// point-major pass (k_point_step_rc; separate back substitution and
// candidate kernels measured 1126 vs 1151 M-obs/s at C3, r03_v5_ab.txt)
void launch_backsub_candidate(const DevProblem& P, const DevWork& W, hipStream_t s) {
  if (jr_tab(P, W)) {
    // compact camera records: the candidate table (value-only records + the
    // camera step) from k_cam_candidate's records first
    hipLaunchKernelGGL(k_cand_table, dim3((P.nc * kCandRec + 255) / 256), dim3(256), 0, s, P, W.rec_c, W.delta_c,
                       W.ctbl);
    constexpr int NT = 512, L = 4;
    const int want = (int)std::min<long long>(((long long)P.np * L + NT - 1) / NT, 1LL << 30);
    const int g = std::max(1, std::min(want, kMaxBlocks));
    if (W.pacc)
      hipLaunchKernelGGL((k_point_step_rc<NT, L, 3, 2, true>), dim3(g), dim3(NT), 0, s, P, (const double*)W.crec,
                         (const double*)W.pts, W.delta_c, (const double*)W.ctbl, W.u, W.Linv, W.scale_p, W.pts_c,
                         W.delta_p, W.part, (const double*)W.vacc, (const double*)W.Hpp, (const double*)W.gp);
    else
      hipLaunchKernelGGL((k_point_step_rc<NT, L, 3, 2>), dim3(g), dim3(NT), 0, s, P, (const double*)W.crec,
                         (const double*)W.pts, W.delta_c, (const double*)W.ctbl, W.u, W.Linv, W.scale_p, W.pts_c,
                         W.delta_p, W.part);
    return;
  }
  if (W.jrfree) {
    // (fp32 W storage too: without W.pacc the back substitution is exact in
    // fp64 from J, as the oracle's fp32-W mode restates it; with it, the
    // accumulated products carry the stored fp32 blocks, as the matvec, the
    // rhs and the preconditioner do)
    constexpr int NT = 512, L = 4;
    const int want = (int)std::min<long long>(((long long)P.np * L + NT - 1) / NT, 1LL << 30);
    const int g = std::max(1, std::min(want, lds_grid(1 << 30)));   // one 110-KB-LDS workgroup per CU
    if (W.pacc)
      hipLaunchKernelGGL((k_point_step_rc<NT, L, 3, 0, true>), dim3(g), dim3(NT), 0, s, P, (const double*)W.rec,
                         (const double*)W.pts, W.delta_c, W.rec_c, W.u, W.Linv, W.scale_p, W.pts_c, W.delta_p, W.part,
                         (const double*)W.vacc, (const double*)W.Hpp, (const double*)W.gp);
    else
      hipLaunchKernelGGL((k_point_step_rc<NT, L>), dim3(g), dim3(NT), 0, s, P, (const double*)W.rec,
                         (const double*)W.pts, W.delta_c, W.rec_c, W.u, W.Linv, W.scale_p, W.pts_c, W.delta_p, W.part);
    return;
  }
  if (W.w32)
    hipLaunchKernelGGL(k_backsub<float>, dim3(pt_group_grid(P.np)), dim3(kThreads), 0, s, P, W.pts, W.pts_c, W.delta_p,
                       W.Wf, W.u, W.Linv, W.y, W.scale_p, W.part);
  else
    hipLaunchKernelGGL(k_backsub<double>, dim3(pt_group_grid(P.np)), dim3(kThreads), 0, s, P, W.pts, W.pts_c, W.delta_p,
                       W.W, W.u, W.Linv, W.y, W.scale_p, W.part);
  if (P.nc <= kLinLdsCams) {
    const int g = lds_grid(P.no);
    hipLaunchKernelGGL((k_candidate_lds<kLinLdsThreads, false>), dim3(g), dim3(kLinLdsThreads), 0, s, P, W.JR,
                       W.delta_c, W.delta_p, W.rec_c, W.pts_c, nullptr, W.part);
    return;
  }
  hipLaunchKernelGGL(k_cand_table, dim3((P.nc * kCandRec + 255) / 256), dim3(256), 0, s, P, W.rec_c, W.delta_c,
                     W.ctbl);
  hipLaunchKernelGGL((k_candidate_lds<256, true>), dim3(grid_for(P.no)), dim3(256), 0, s, P, W.JR, W.delta_c,
                     W.delta_p, W.rec_c, W.pts_c, W.ctbl, W.part);
}
// STREAM-style copy for the measured bandwidth figure (ba_stream_copy):
// non-temporal 16-B loads and stores, one per lane, grid up to one lane per
// element (tools/copy_probe.hip, 1 GiB: 5.95 TB/s at 65536 workgroups vs
// 5.1 with four per lane at 8192)
__global__ __launch_bounds__(256) void k_stream_copy(const double2* __restrict__ a, double2* __restrict__ b, size_t n2) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += stride)
    __builtin_nontemporal_store(__builtin_nontemporal_load(reinterpret_cast<const ntd2*>(a + i)),
                                reinterpret_cast<ntd2*>(b + i));
}
int jr_ja_host(int nc) { return jr_ja(nc > kLinLdsCams); }
void launch_stream_copy(const double* a, double* b, size_t n2, hipStream_t s) {
  if (n2 == 0) return;
  const size_t g = std::min<size_t>((n2 + 255) / 256, 262144);
  hipLaunchKernelGGL(k_stream_copy, dim3((unsigned)g), dim3(256), 0, s, reinterpret_cast<const double2*>(a),
                     reinterpret_cast<double2*>(b), n2);
}
void launch_reduce(const DevWork& W, uint32_t sum_mask, uint32_t max_mask, hipStream_t s) {
  hipLaunchKernelGGL(k_reduce<false>, dim3(kNumSlots), dim3(64), 0, s, W.part, W.scal, sum_mask, max_mask,
                     ReducePub{});
}
void launch_reduce_publish(const DevWork& W, uint32_t sum_mask, uint32_t max_mask, double* host, int n,
                           unsigned* host_seq, unsigned seq, unsigned* ticket, hipStream_t s) {
  hipLaunchKernelGGL(k_reduce<true>, dim3(kNumSlots), dim3(64), 0, s, W.part, W.scal, sum_mask, max_mask,
                     ReducePub{host, n, host_seq, seq, ticket});
}
void launch_residuals(const DevProblem& P, const double* rec, const double* pts, double* r_raw, hipStream_t s) {
  hipLaunchKernelGGL(k_residuals, dim3(grid_for(P.no)), dim3(kThreads), 0, s, P, rec, pts, r_raw);
}

}  // namespace bahip

// ===========================================================================
// Batched pose-only LM: the solve of
// MotionOnlyBAOptimizerAngles::optimizeCameraPose (Optimizer.cpp:417-457)
// for many frames per launch.  One problem = one camera, constant points
// (PoseOnlyAngleReprojectionError, Optimizer.h:163-182), HuberLoss.
//
// One wavefront per problem runs the WHOLE trust-region loop in-kernel: the
// 6x6 normal equations are wave reductions (xor butterfly: every lane holds
// the bitwise-identical total, so the LM bookkeeping runs lane-uniform in
// registers), the 6x6 Cholesky and the accept/reject logic are the host
// loop of solve() (ba_solver.hip) restated per wave.  Per LM iteration ONE
// pass over the observations: model cost change from J(x), candidate cost
// at x', and the linearisation at x' (speculative: adopted when the step is
// accepted, exactly what a separate linearize(x') pass would produce).
// Latency-bound by design (10^2-10^3 observations per problem): no host
// round trip, no launch per iteration.
// ===========================================================================
namespace bahip {

__device__ inline double wave_allsum(double v) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// K-folded derivative table of camera x (lin table, kLin entries) into LDS;
// every lane evaluates the dual Rodrigues (uniform) and writes its entries.
__device__ inline void pose_table(const double x[6], const double Kd[9], double* tbl) {
  D3 R[9];
  angle_axis_to_R_d3(x, R);
  const int lane = threadIdx.x & 63;
  for (int e = lane; e < kLin; e += 64) tbl[e] = cam_rec_entry(kRecL + e, x, x + 3, Kd, R, nullptr, true);
  if (lane == 0) { tbl[kLin] = 1.0; tbl[kLin + 1] = 0.0; }
  wave_lds_sync();
}

// accumulate the 2x6 camera block of one observation: H (21 lower, row-major), g (6)
__device__ inline void pose_acc(const double (&out)[kJR], double (&H)[21], double (&g)[6]) {
#pragma unroll
  for (int row = 0; row < 2; ++row) {
    const double* j = out + 6 * row;
    int t = 0;
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
      for (int b = 0; b <= a; ++b) H[t++] += j[a] * j[b];
#pragma unroll
    for (int a = 0; a < 6; ++a) g[a] += j[a] * out[18 + row];
  }
}

__global__ __launch_bounds__(64) void k_pose_batch(int nprob, const int* __restrict__ off,
                                                   const double* __restrict__ cams_in, const float* __restrict__ Kf,
                                                   const double* __restrict__ Xw, const float2* __restrict__ uvs,
                                                   double huber_a, PoseOpts o, double* __restrict__ cams_out,
                                                   double* __restrict__ summ) {
  __shared__ double tb[2][kLin + 2];
  __shared__ float ks[9];
  const int prob = blockIdx.x, lane = threadIdx.x;
  if (prob >= nprob) return;
  const int o0 = off[prob], o1 = off[prob + 1];
  DevProblem P{};
  P.huber_a = huber_a;
  P.huber_b = huber_a * huber_a;
  double x[6], Kd[9];
#pragma unroll
  for (int a = 0; a < 6; ++a) x[a] = cams_in[6 * prob + a];
#pragma unroll
  for (int k = 0; k < 9; ++k) Kd[k] = (double)Kf[9 * prob + k];
  if (lane < 9) ks[lane] = Kf[9 * prob + lane];
  int cur = 0;
  pose_table(x, Kd, tb[cur]);

  // ---- linearisation at x (iteration 0)
  double H[21], g[6], cost = 0.0, bad = 0.0;
#pragma unroll
  for (int k = 0; k < 21; ++k) H[k] = 0.0;
#pragma unroll
  for (int a = 0; a < 6; ++a) g[a] = 0.0;
  for (int ob = o0 + lane; ob < o1; ob += 64) {
    double out[kJR];
    bool fin;
    const double rho = lin_obs(P, CamLds{tb[cur], ks}, true, false, Xw[3 * ob], Xw[3 * ob + 1], Xw[3 * ob + 2],
                               uvs[ob], out, fin);
    cost += 0.5 * rho;
    bad += fin ? 0.0 : 1.0;
    pose_acc(out, H, g);
  }
#pragma unroll
  for (int k = 0; k < 21; ++k) H[k] = wave_allsum(H[k]);
#pragma unroll
  for (int a = 0; a < 6; ++a) g[a] = wave_allsum(g[a]);
  cost = wave_allsum(cost);
  bad = wave_allsum(bad);
  const bool empty = o1 <= o0;

  double s[6], dg[6];
  auto norms = [&](double& gmax, double& gnorm, double& xnorm) {
    double gn2 = 0.0, xn2 = 0.0;
    gmax = 0.0;
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      const double h = H[tri(a, a)];
      dg[a] = fmin(fmax(h * s[a] * s[a], o.min_diag), o.max_diag);
      const double d = x[a] - (x[a] + (-g[a]));
      gmax = fmax(gmax, fabs(d));
      gn2 += d * d;
      xn2 += x[a] * x[a];
    }
    gnorm = sqrt(gn2);
    xnorm = sqrt(xn2);
  };
#pragma unroll
  for (int a = 0; a < 6; ++a) s[a] = o.jacobi ? 1.0 / (1.0 + sqrt(H[tri(a, a)])) : 1.0;
  double gmax = 0.0, gnorm = 0.0, xnorm = 0.0;
  double x_cost = cost;
  const double initial_cost = cost;
  int iteration = 0, nsucc = 0, nunsucc = 0, termination = BA_NO_CONVERGENCE;
  if (empty) {   // no residual block touches the camera: nothing to solve
    gmax = 0.0;
    xnorm = 0.0;
  } else {
    norms(gmax, gnorm, xnorm);
  }
  if (!(bad == 0.0 && isfinite(cost))) {
    termination = BA_FAILURE;
  } else {
    double radius = o.r0, decrease = 2.0;
    int consecutive_invalid = 0;
    bool last_success = true;
    while (true) {
      if (iteration >= o.max_iter) { termination = BA_NO_CONVERGENCE; break; }
      if (last_success && gmax <= o.gtol) { termination = BA_CONVERGENCE; break; }
      if (radius <= o.rmin) { termination = BA_CONVERGENCE; break; }
      ++iteration;
      // ---- reduced system (the camera block itself): S = s H s + D^2, b = s g
      double L[21], y[6];
      bool chol_ok = true;
      {
        int t = 0;
#pragma unroll
        for (int a = 0; a < 6; ++a)
#pragma unroll
          for (int b = 0; b <= a; ++b, ++t) {
            double h = H[t] * s[a] * s[b];
            if (a == b) {
              const double D = sqrt(dg[a] / radius);
              h += D * D;
            }
            L[t] = h;
          }
        // LL^T in place (row-major lower), then forward / back substitution
#pragma unroll
        for (int j = 0; j < 6; ++j) {
          double d = L[tri(j, j)];
#pragma unroll
          for (int k = 0; k < j; ++k) d -= L[tri(j, k)] * L[tri(j, k)];
          if (!(d > 0.0 && isfinite(d))) chol_ok = false;
          const double lj = sqrt(d);
          L[tri(j, j)] = lj;
#pragma unroll
          for (int i = j + 1; i < 6; ++i) {
            double v = L[tri(i, j)];
#pragma unroll
            for (int k = 0; k < j; ++k) v -= L[tri(i, k)] * L[tri(j, k)];
            L[tri(i, j)] = v / lj;
          }
        }
        double z[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          double v = g[i] * s[i];
#pragma unroll
          for (int k = 0; k < i; ++k) v -= L[tri(i, k)] * z[k];
          z[i] = v / L[tri(i, i)];
        }
#pragma unroll
        for (int i = 5; i >= 0; --i) {
          double v = z[i];
#pragma unroll
          for (int k = i + 1; k < 6; ++k) v -= L[tri(k, i)] * y[k];
          y[i] = v / L[tri(i, i)];
        }
      }
      double xc[6], dl[6], step2 = 0.0;
      bool step_bad = false;
#pragma unroll
      for (int a = 0; a < 6; ++a) {
        dl[a] = (-y[a]) * s[a];
        xc[a] = x[a] + dl[a];
        const double e = x[a] - xc[a];
        step2 += e * e;
        if (!isfinite(dl[a])) step_bad = true;
      }
      // ---- one pass: model cost change (J at x), candidate cost, linearisation at x'
      const int nxt = cur ^ 1;
      pose_table(xc, Kd, tb[nxt]);
      double Rc[9];
      angle_axis_to_R(xc, Rc);
      double mneg = 0.0, ccost = 0.0, cbad = 0.0, H2[21], g2[6], cost2 = 0.0, bad2 = 0.0;
#pragma unroll
      for (int k = 0; k < 21; ++k) H2[k] = 0.0;
#pragma unroll
      for (int a = 0; a < 6; ++a) g2[a] = 0.0;
      for (int ob = o0 + lane; ob < o1; ob += 64) {
        const double X0 = Xw[3 * ob], X1 = Xw[3 * ob + 1], X2 = Xw[3 * ob + 2];
        const float2 uv = uvs[ob];
        double out[kJR];
        bool fin;
        lin_obs(P, CamLds{tb[cur], ks}, true, false, X0, X1, X2, uv, out, fin);
        double jd0 = 0.0, jd1 = 0.0;
#pragma unroll
        for (int a = 0; a < 6; ++a) { jd0 += out[a] * dl[a]; jd1 += out[6 + a] * dl[a]; }
        mneg += jd0 * (out[18] + jd0 / 2.0) + jd1 * (out[19] + jd1 / 2.0);
        // candidate residual, value-only record at x' (k_candidate's arithmetic)
        double pc[3], q[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) pc[i] = Rc[i] * X0 + Rc[3 + i] * X1 + Rc[6 + i] * X2 + xc[3 + i];
#pragma unroll
        for (int i = 0; i < 3; ++i) q[i] = pc[0] * Kd[i] + pc[1] * Kd[3 + i] + pc[2] * Kd[6 + i];
        const double rc0 = q[0] / q[2] - (double)uv.x, rc1 = q[1] / q[2] - (double)uv.y;
        double sc;
        ccost += 0.5 * huber(rc0 * rc0 + rc1 * rc1, P.huber_a, P.huber_b, &sc);
        if (!isfinite(rc0) || !isfinite(rc1)) cbad += 1.0;
        // linearisation at x' (used if the step is accepted)
        const double rho2 = lin_obs(P, CamLds{tb[nxt], ks}, true, false, X0, X1, X2, uv, out, fin);
        cost2 += 0.5 * rho2;
        bad2 += fin ? 0.0 : 1.0;
        pose_acc(out, H2, g2);
      }
      mneg = wave_allsum(mneg);
      ccost = wave_allsum(ccost);
      cbad = wave_allsum(cbad);
      const double mcc = -mneg;
      const bool valid = chol_ok && !step_bad && mcc > 0.0;
      if (!valid) {
        if (++consecutive_invalid >= o.max_invalid) { termination = BA_FAILURE; break; }
        radius = radius / decrease;
        decrease *= 2.0;
        last_success = false;
        ++nunsucc;
        continue;
      }
      consecutive_invalid = 0;
      if (sqrt(step2) <= o.ptol * (xnorm + o.ptol)) { termination = BA_CONVERGENCE; break; }
      const double cand_cost = (cbad > 0.0 || !isfinite(ccost)) ? 1.7976931348623157e308 : ccost;
      const double cost_change = x_cost - cand_cost;
      if (fabs(cost_change) <= o.ftol * x_cost) { termination = BA_CONVERGENCE; break; }
      const double rel = cand_cost >= 1.7976931348623157e308 ? -1.7976931348623157e308 : (x_cost - cand_cost) / mcc;
      if (rel > o.min_rel) {
#pragma unroll
        for (int k = 0; k < 21; ++k) H[k] = wave_allsum(H2[k]);
#pragma unroll
        for (int a = 0; a < 6; ++a) { g[a] = wave_allsum(g2[a]); x[a] = xc[a]; }
        cost = wave_allsum(cost2);
        bad = wave_allsum(bad2);
        cur = nxt;
        if (!(bad == 0.0 && isfinite(cost))) { termination = BA_FAILURE; x_cost = cost; break; }
        x_cost = cost;
        norms(gmax, gnorm, xnorm);
        const double t3 = 2.0 * rel - 1.0;
        radius = fmin(o.rmax, radius / fmax(1.0 / 3.0, 1.0 - t3 * t3 * t3));
        decrease = 2.0;
        last_success = true;
        ++nsucc;
      } else {
        radius = radius / decrease;
        decrease *= 2.0;
        last_success = false;
        ++nunsucc;
      }
    }
  }
  if (lane < 6) cams_out[6 * prob + lane] = x[lane];
  if (lane == 0) {
    double* sm = summ + 8 * prob;
    sm[0] = initial_cost;
    sm[1] = x_cost;
    sm[2] = iteration;
    sm[3] = nsucc;
    sm[4] = nunsucc;
    sm[5] = termination;
    sm[6] = gmax;
    sm[7] = 0.0;
  }
}

void launch_pose_batch(int nprob, const int* off, const double* cams_in, const float* K, const double* X,
                       const float2* uv, double huber_a, const PoseOpts& o, double* cams_out, double* summ,
                       hipStream_t s) {
  if (nprob <= 0) return;
  hipLaunchKernelGGL(k_pose_batch, dim3(nprob), dim3(64), 0, s, nprob, off, cams_in, K, X, uv, huber_a, o, cams_out,
                     summ);
}

__global__ __launch_bounds__(64) void k_publish_scalars(const double* __restrict__ scal, double* __restrict__ host,
                                                        int n, unsigned* __restrict__ host_seq, unsigned seq) {
  for (int i = threadIdx.x; i < n; i += 64) host[i] = scal[i];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // system scope: the record reaches host memory first
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(host_seq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
void launch_publish_scalars(const double* scal, double* host, int n, unsigned* host_seq, unsigned seq, hipStream_t s) {
  hipLaunchKernelGGL(k_publish_scalars, dim3(1), dim3(64), 0, s, scal, host, n, host_seq, seq);
}

}  // namespace bahip

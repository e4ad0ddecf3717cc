// ba_solver.hip — host side of libba_hip.so: problem structure, device
// workspace, the Levenberg-Marquardt driver and the extern "C" ABI
// (include/ba_hip.h).
//
// The driver restates ceres::TrustRegionMinimizer + LevenbergMarquardtStrategy
// with the options of BAOptimizer::configureSolver (reference
// ba_project/src/ba/Optimizer.cpp:80-90) and drives the CDNA4 kernels of
// ba_kernels.hip.  Per LM iteration the host reads back one small scalar
// record (cost, model cost change, norms, failure counts) to take Ceres'
// accept / reject / terminate decisions; all vectors stay in HBM.
//
// Multi-GPU: every rank owns a disjoint set of points with all their
// observations; cameras are replicated.  RCCL all-reduces (over xGMI) the
// per-camera blocks after linearisation, the dense reduced camera system
// after point elimination, and the scalar record after the candidate pass.
// All ranks then take identical decisions.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <numeric>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/ba_hip.h"
#include "ba_device.h"
#include "ba_kernels.h"

using namespace bahip;

namespace {

struct BaError {
  int code;
  std::string msg;
};

#define HIP_OK(expr)                                                                                  \
  do {                                                                                                \
    hipError_t _e = (expr);                                                                           \
    if (_e != hipSuccess)                                                                             \
      throw BaError{_e == hipErrorOutOfMemory ? BA_ERR_OUT_OF_MEMORY : BA_ERR_DEVICE,                 \
                    std::string(#expr) + ": " + hipGetErrorString(_e)};                               \
  } while (0)
#define NCCL_OK(expr)                                                                                 \
  do {                                                                                                \
    ncclResult_t _r = (expr);                                                                         \
    if (_r != ncclSuccess) throw BaError{BA_ERR_COMM, std::string(#expr) + ": " + ncclGetErrorString(_r)}; \
  } while (0)

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

struct ba_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  hipEvent_t ev[7] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};   // [2..5]: two r+J stamp pairs, [6]: scalar blit
  int rj_slot = 0;   // the stamp pair of the next timed linearisation (bench)
  // the device linearisation state is at the candidate of the last step (a
  // speculative linearisation, enqueued behind the step's scalar record)
  bool lin_at_cand = false;

  // multi-GPU
  int nranks = 1, rank = 0;
  ncclComm_t comm = nullptr;
  // host-staged transport (ba_comm_init_host: tests of the multi-rank path
  // with several ranks on one GPU, where RCCL refuses duplicate devices)
  ba_host_allreduce_fn host_fn = nullptr;
  void* host_user = nullptr;
  std::vector<double> host_buf;

  // problem
  bool have_problem = false;
  int nc = 0, np = 0, no = 0, nvc = 0, n = 0, ld = 0;
  std::vector<int> perm;         // sorted obs -> caller obs
  std::vector<int> chol_off;     // split Cholesky task table: host step offsets (W.ctask_off)
  std::vector<int> cam_of_vc;
  std::vector<uint8_t> cam_fixed_h;
  double huber_a = 0.0;
  DevProblem P{};
  DevWork W{};
  std::vector<void*> allocs;     // device buffers of the current problem
  double* h_scal = nullptr;      // pinned scalar record (device-mapped, coherent)
  double* d_hscal = nullptr;     // its device address
  unsigned* h_seq = nullptr;     // the record's sequence number (after the record), host / device address
  unsigned* d_hseq = nullptr;
  unsigned* d_ticket = nullptr;  // k_reduce<true>'s last-workgroup ticket (zero between launches)
  unsigned scal_seq = 0;
  char* pose_buf = nullptr;      // ba_solve_pose_batch device staging (grown on demand)
  size_t pose_cap = 0;
  std::vector<char> pose_host;

  // host copies of the sorted structure, kept for the lazily built
  // linear-solver structures (Schur pair lists / PCG duplicate pairs)
  std::vector<int> h_pt_off, h_obs_cam, h_vc;
  std::vector<uint8_t> h_pt_var;
  bool have_dense = false, have_pcg = false;
  int chol_epoch = 0;   // launches of the back substitution (hand-off flag values)
  // scalar slots whose fold a linearisation left to the step enqueued right
  // behind it (single rank: one k_reduce for both records)
  uint32_t pend_sum = 0, pend_max = 0;
  // the camera-side norms pass of such a linearisation, left to ride in the
  // step's point-elimination launch (launch_point_elim's NormsFold)
  bool norms_pend = false;
  bahip::NormsFold norms_args{};
  // a pending norms pass as its own launch (before any fold of its slots)
  void flush_norms() {
    if (!norms_pend) return;
    norms_pend = false;
    bahip::launch_cam_norms(P, W, norms_args.compute_scale != 0, norms_args.min_diag, norms_args.max_diag, stream);
  }
  const bahip::NormsFold* take_norms() {
    if (!norms_pend) return nullptr;
    norms_pend = false;
    return &norms_args;
  }
  void clear_pending() { pend_sum = pend_max = 0; norms_pend = false; }
  bool dup_diag = false;   // the dense pair list has diagonal blocks (duplicate observations)
  bool k_plain = false;    // every camera's K without skew, row 2 = (0, 0, k22) (set_problem)
  size_t pcg_ndup = 0;     // ITERATIVE_SCHUR duplicate (camera, point) pairs (ensure_pcg)
  double* tobs_buf = nullptr;   // [no][6] ITERATIVE_SCHUR per-observation products (allocated on first use)
  int max_no = 0;               // largest observation count over the ranks (collective matvec-path choice)

  // solver state
  std::vector<ba_iteration> log;
  std::vector<double> bench_ms;   // host wall time of each iteration of the last ba_bench_iterations
  bool scale_valid = false;
  double t_lin = 0.0, t_solve = 0.0;

  template <typename T>
  T* dalloc(size_t count) {
    if (count == 0) count = 1;
    void* p = nullptr;
    HIP_OK(hipMalloc(&p, count * sizeof(T)));
    allocs.push_back(p);
    return static_cast<T*>(p);
  }
  void dfree(void* p) {
    if (!p) return;
    auto it = std::find(allocs.begin(), allocs.end(), p);
    if (it != allocs.end()) allocs.erase(it);
    if (stream) (void)hipStreamSynchronize(stream);
    (void)hipFree(p);
  }
  template <typename T>
  T* upload(const std::vector<T>& v) {
    T* d = dalloc<T>(v.size());
    if (!v.empty()) HIP_OK(hipMemcpyAsync(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, stream));
    return d;
  }
  void free_problem() {
    if (stream) (void)hipStreamSynchronize(stream);
    for (void* p : allocs) (void)hipFree(p);
    allocs.clear();
    have_problem = have_dense = have_pcg = false;
    tobs_buf = nullptr;
    scale_valid = false;
    log.clear();
  }

  // collectives on the data path: with more than one rank, or forced on a
  // one-rank communicator (BA_FORCE_COLLECTIVES=1: tests of the exchange path
  // on a single GPU, where the all-reduce is the identity)
  bool force_coll = false;
  bool has_comm() const { return comm || host_fn; }
  bool coll() const { return has_comm() && (nranks > 1 || force_coll); }
  void allreduce(double* d, size_t count, ncclRedOp_t op = ncclSum) {
    if (!has_comm() || count == 0) return;   // a 1-rank communicator still runs the collectives (tests)
    if (host_fn) {   // stage through the host and the caller's transport
      host_buf.resize(count);
      HIP_OK(hipMemcpyAsync(host_buf.data(), d, sizeof(double) * count, hipMemcpyDeviceToHost, stream));
      HIP_OK(hipStreamSynchronize(stream));
      if (host_fn(host_user, host_buf.data(), (int64_t)count, op == ncclMax ? 1 : 0) != 0)
        throw BaError{BA_ERR_COMM, "host all-reduce callback failed"};
      HIP_OK(hipMemcpyAsync(d, host_buf.data(), sizeof(double) * count, hipMemcpyHostToDevice, stream));
      // host_buf is pageable and reused by the next call: wait for the copy
      // (test transport, latency irrelevant)
      HIP_OK(hipStreamSynchronize(stream));
      return;
    }
    NCCL_OK(ncclAllReduce(d, d, count, ncclDouble, op, comm, stream));
  }
  // host values (set_problem structure, bench timing); one device scratch
  // buffer, grown on demand and kept for the context's lifetime
  double* hv_scratch = nullptr;
  size_t hv_cap = 0;
  void allreduce_host_values(double* v, size_t count, int op) {
    if (!has_comm() || count == 0) return;
    if (count > hv_cap) {
      if (hv_scratch) { (void)hipStreamSynchronize(stream); (void)hipFree(hv_scratch); hv_scratch = nullptr; hv_cap = 0; }
      HIP_OK(hipMalloc(&hv_scratch, sizeof(double) * count));
      hv_cap = count;
    }
    HIP_OK(hipMemcpyAsync(hv_scratch, v, sizeof(double) * count, hipMemcpyHostToDevice, stream));
    allreduce(hv_scratch, count, op == 1 ? ncclMax : ncclSum);
    HIP_OK(hipMemcpyAsync(v, hv_scratch, sizeof(double) * count, hipMemcpyDeviceToHost, stream));
    HIP_OK(hipStreamSynchronize(stream));
  }
  // The scalar record to the host: a one-workgroup kernel stores it into the
  // pinned, device-mapped record and then a sequence number (system-scope
  // release), and the host spins on that number, instead of a D2H blit and
  // a stream synchronisation (whose wake-up left ~20 us of idle device
  // between an LM step and the next linearisation).  A device error or a
  // missing number (bounded wait) falls back to the synchronisation, which
  // reports it.  BA_SCAL_SPIN=0: the blit + synchronisation (A/B).
  // publish_scalars() enqueues the record's transfer, wait_scalars() waits
  // for it (work enqueued in between keeps the device busy meanwhile)
  void read_scalars() {
    publish_scalars();
    wait_scalars();
  }
  bool scal_spin() const { return spin && d_hscal; }
  // per-call switches (read at every ba_solve / ba_bench_iterations entry, so
  // tests can A/B them in one process): BA_SPEC_LIN=0 turns the speculative
  // linearisation off, BA_SCAL_SPIN=0 the spin-published scalar record
  bool spec_lin = true, spin = true;
  void read_env() {
    const char* e = std::getenv("BA_SPEC_LIN");
    spec_lin = !(e && e[0] == '0');
    e = std::getenv("BA_SCAL_SPIN");
    spin = !(e && e[0] == '0');
  }
  void publish_scalars() {
    const size_t cnt = kNumSlots + kPcgState;
    flush_norms();
    if (!scal_spin()) {
      if (pend_sum | pend_max) bahip::launch_reduce(W, pend_sum, pend_max, stream);
      pend_sum = pend_max = 0;
      HIP_OK(hipMemcpyAsync(h_scal, W.scal, sizeof(double) * cnt, hipMemcpyDeviceToHost, stream));
      HIP_OK(hipEventRecord(ev[6], stream));
      return;
    }
    // scalars still to be folded (pend_*: the step's and the deferred
    // linearisation's, single rank): one launch folds and publishes them
    if ((pend_sum | pend_max) && d_ticket) {
      bahip::launch_reduce_publish(W, pend_sum, pend_max, d_hscal, (int)cnt, d_hseq, ++scal_seq, d_ticket, stream);
      pend_sum = pend_max = 0;
    } else {
      if (pend_sum | pend_max) bahip::launch_reduce(W, pend_sum, pend_max, stream);
      pend_sum = pend_max = 0;
      bahip::launch_publish_scalars(W.scal, d_hscal, (int)cnt, d_hseq, ++scal_seq, stream);
    }
    HIP_OK(hipGetLastError());
  }
  void wait_scalars() {
    if (!scal_spin()) {
      HIP_OK(hipEventSynchronize(ev[6]));
      return;
    }
    const unsigned seq = scal_seq;
    const double t0 = now_s();
    for (unsigned it = 1;; ++it) {
      if (__atomic_load_n(h_seq, __ATOMIC_ACQUIRE) == seq) return;
      if ((it & 1023u) == 0 && now_s() - t0 > 2.0) break;
    }
    HIP_OK(hipStreamSynchronize(stream));   // (raises a device error)
    if (__atomic_load_n(h_seq, __ATOMIC_ACQUIRE) != seq)
      throw BaError{BA_ERR_DEVICE, "scalar record: sequence number not received"};
  }
};

namespace {

// ---------------------------------------------------------------------------
// structure build
// ---------------------------------------------------------------------------
void set_problem(ba_ctx* ctx, const ba_problem* pb) {
  if (!pb) throw BaError{BA_ERR_INVALID_ARGUMENT, "problem is NULL"};
  const int nc = pb->n_cams, np = pb->n_pts, no = pb->n_obs;
  if (nc < 0 || np < 0 || no < 0) throw BaError{BA_ERR_INVALID_ARGUMENT, "negative size"};
  if ((nc > 0 && (!pb->cams || !pb->K)) || (np > 0 && !pb->pts) ||
      (no > 0 && (!pb->obs_cam || !pb->obs_pt || !pb->obs_uv)))
    throw BaError{BA_ERR_INVALID_ARGUMENT, "missing array"};
  bool any_fixed = false;
  for (int c = 0; c < nc; ++c) any_fixed |= (pb->cam_fixed && pb->cam_fixed[c]);
  if (any_fixed && !pb->cam_fixed_extr) throw BaError{BA_ERR_INVALID_ARGUMENT, "cam_fixed_extr required for fixed cameras"};
  for (int o = 0; o < no; ++o) {
    if (pb->obs_cam[o] < 0 || pb->obs_cam[o] >= nc || pb->obs_pt[o] < 0 || pb->obs_pt[o] >= np)
      throw BaError{BA_ERR_INVALID_ARGUMENT, "observation index out of range at obs " + std::to_string(o)};
  }
  ctx->free_problem();
  HIP_OK(hipSetDevice(ctx->device));
  ctx->nc = nc; ctx->np = np; ctx->no = no;
  ctx->huber_a = pb->huber_a;
  ctx->cam_fixed_h.assign(nc, 0);
  for (int c = 0; c < nc; ++c) ctx->cam_fixed_h[c] = pb->cam_fixed ? pb->cam_fixed[c] : 0;
  std::vector<uint8_t> pt_fixed(np, 0);
  for (int p = 0; p < np; ++p) pt_fixed[p] = pb->pt_fixed ? pb->pt_fixed[p] : 0;

  // sort observations by (point, camera, caller index): counting sort by point
  std::vector<int> pt_off(np + 1, 0);
  for (int o = 0; o < no; ++o) pt_off[pb->obs_pt[o] + 1]++;
  for (int p = 0; p < np; ++p) pt_off[p + 1] += pt_off[p];
  std::vector<int> perm(no);
  {
    std::vector<int> fill(pt_off.begin(), pt_off.end() - 1);
    for (int o = 0; o < no; ++o) perm[fill[pb->obs_pt[o]]++] = o;
    for (int p = 0; p < np; ++p) {
      auto b = perm.begin() + pt_off[p], e = perm.begin() + pt_off[p + 1];
      if (e - b > 1)
        std::stable_sort(b, e, [&](int a, int c) { return pb->obs_cam[a] < pb->obs_cam[c]; });
    }
  }
  // active blocks
  std::vector<int> vc(nc, -1);
  std::vector<uint8_t> pt_var(np, 0), cam_used(nc, 0);
  for (int o = 0; o < no; ++o) {
    const int c = pb->obs_cam[o], p = pb->obs_pt[o];
    if (!ctx->cam_fixed_h[c]) cam_used[c] = 1;
    if (!pt_fixed[p]) pt_var[p] = 1;
  }
  if (ctx->coll() && nc > 0) {
    // the reduced system spans the union of the ranks' observed cameras
    std::vector<double> u(nc);
    for (int c = 0; c < nc; ++c) u[c] = cam_used[c];
    ctx->allreduce_host_values(u.data(), nc, 1);
    for (int c = 0; c < nc; ++c) cam_used[c] = u[c] != 0.0;
  }
  ctx->max_no = no;
  if (ctx->coll()) {
    // every rank takes the same matvec path (ITERATIVE_SCHUR), chosen from the
    // largest shard: identical kernels and rounding on every rank
    double h = (double)no;
    ctx->allreduce_host_values(&h, 1, 1);
    ctx->max_no = (int)h;
  }
  ctx->cam_of_vc.clear();
  for (int c = 0; c < nc; ++c)
    if (cam_used[c]) { vc[c] = (int)ctx->cam_of_vc.size(); ctx->cam_of_vc.push_back(c); }
  const int nvc = (int)ctx->cam_of_vc.size();
  ctx->nvc = nvc;
  ctx->n = 6 * nvc;
  ctx->ld = ctx->n;

  std::vector<int> obs_cam(no), obs_pt(no);
  std::vector<float2> uv(no);
  for (int s = 0; s < no; ++s) {
    const int o = perm[s];
    obs_cam[s] = pb->obs_cam[o];
    obs_pt[s] = pb->obs_pt[o];
    uv[s] = make_float2(pb->obs_uv[2 * o], pb->obs_uv[2 * o + 1]);
  }
  // observations by variable camera (increasing sorted index)
  std::vector<int> cam_off(nvc + 1, 0);
  for (int s = 0; s < no; ++s) if (vc[obs_cam[s]] >= 0) cam_off[vc[obs_cam[s]] + 1]++;
  for (int v = 0; v < nvc; ++v) cam_off[v + 1] += cam_off[v];
  std::vector<int> cam_obs(cam_off[nvc]);
  {
    std::vector<int> fill(cam_off.begin(), cam_off.end() - 1);
    for (int s = 0; s < no; ++s) if (vc[obs_cam[s]] >= 0) cam_obs[fill[vc[obs_cam[s]]]++] = s;
  }
  // ---- device upload
  DevProblem& P = ctx->P;
  P = DevProblem{};
  P.nc = nc; P.np = np; P.no = no; P.nvc = nvc; P.n = ctx->n; P.ld = ctx->ld;
  P.huber_a = pb->huber_a;
  P.huber_b = pb->huber_a * pb->huber_a;
  P.obs_cam = ctx->upload(obs_cam);
  P.obs_pt = ctx->upload(obs_pt);
  P.uv = ctx->upload(uv);
  P.pt_off = ctx->upload(pt_off);
  P.cam_off = ctx->upload(cam_off);
  {
    std::vector<int2> cam_op(cam_obs.size());
    for (size_t i = 0; i < cam_obs.size(); ++i) cam_op[i] = make_int2(cam_obs[i], obs_pt[cam_obs[i]]);
    P.cam_op = ctx->upload(cam_op);
    std::vector<float2> uv_cm(cam_obs.size());
    for (size_t i = 0; i < cam_obs.size(); ++i) uv_cm[i] = uv[cam_obs[i]];
    P.uv_cm = ctx->upload(uv_cm);
  }
  P.vc = ctx->upload(vc);
  {
    std::vector<int> obs_vc(no);
    for (int o = 0; o < no; ++o) obs_vc[o] = vc[obs_cam[o]];
    P.obs_vc = ctx->upload(obs_vc);
  }
  P.cam_of_vc = ctx->upload(ctx->cam_of_vc);
  P.cam_fixed = ctx->upload(ctx->cam_fixed_h);
  P.pt_var = ctx->upload(pt_var);
  P.K = ctx->upload(std::vector<float>(pb->K, pb->K + 9 * (size_t)nc));
  ctx->k_plain = true;   // no skew, row 2 = (0, 0, k22): the 16-value PCG records apply
  for (int c = 0; c < nc; ++c) {
    const float* k = pb->K + 9 * (size_t)c;   // column-major
    if (k[1] != 0.0f || k[2] != 0.0f || k[3] != 0.0f || k[5] != 0.0f) ctx->k_plain = false;
  }
  {
    std::vector<float> ex(16 * (size_t)nc, 0.0f);
    if (pb->cam_fixed_extr)
      for (int c = 0; c < nc; ++c)
        if (ctx->cam_fixed_h[c]) std::memcpy(&ex[16 * (size_t)c], pb->cam_fixed_extr + 16 * (size_t)c, 16 * sizeof(float));
    P.extr = ctx->upload(ex);
  }
  DevWork& W = ctx->W;
  W = DevWork{};
  W.cams = ctx->upload(std::vector<double>(pb->cams, pb->cams + 6 * (size_t)nc));
  W.pts = ctx->upload(std::vector<double>(pb->pts, pb->pts + 3 * (size_t)np));
  W.cams_c = ctx->dalloc<double>(6 * (size_t)nc);
  W.pts_c = ctx->dalloc<double>(3 * (size_t)np);
  W.rec = ctx->dalloc<double>((size_t)kCamRec * nc);
  W.rec_c = ctx->dalloc<double>((size_t)kCamRec * nc);
  W.crec = ctx->dalloc<double>((size_t)16 * nc);
  W.ctbl = ctx->dalloc<double>((size_t)22 * nc);
  // J-free iteration: r and J are recomputed by every consumer and never
  // stored (camera tables in LDS up to 200 cameras, the compact 128-B camera
  // records beyond: each observation forms its camera's dual Rodrigues from
  // them); BA_JR=1 forces the JR-materialising kernels (A/B,
  // diagnostics).  JR is then allocated only for ba_linearize's read-back.
  {
    const char* e = std::getenv("BA_JR");
    W.jrfree = nc > 0 && !(e && e[0] == '1');
  }
  W.JR = W.jrfree ? nullptr : ctx->dalloc<double>((size_t)(bahip::jr_ja_host(nc) + 8) * no);   // JA [no][jr_ja] + JB [no][8] (ba_kernels.hip)
  W.delta_p = ctx->dalloc<double>(3 * (size_t)np);
  W.pxv = ctx->dalloc<double>(4 * (size_t)np);
  W.Hpp = ctx->dalloc<double>(6 * (size_t)np);
  W.gp = ctx->dalloc<double>(3 * (size_t)np);
  W.scale_p = ctx->dalloc<double>(3 * (size_t)np);
  W.diag_p = ctx->dalloc<double>(3 * (size_t)np);
  W.Linv = ctx->dalloc<double>(6 * (size_t)np);
  W.u = ctx->dalloc<double>(4 * (size_t)np);
  // Hcc | gc | scalar slots | PCG state in one allocation: the camera blocks
  // and the point-side sums cross ranks in one all-reduce
  {
    double* hx = ctx->dalloc<double>(27 * (size_t)nvc + kNumSlots + kPcgState);
    W.Hcc = hx;
    W.gc = hx + 21 * (size_t)nvc;
    W.scal = hx + 27 * (size_t)nvc;
  }
  W.scale_c = ctx->dalloc<double>(6 * (size_t)nvc);
  W.diag_c = ctx->dalloc<double>(6 * (size_t)nvc);
  W.delta_c = ctx->dalloc<double>(6 * (size_t)nvc);
  W.W = nullptr;   // per-observation Schur blocks: allocated by the first solve (fp64 or fp32)
  W.Wf = nullptr;
  W.y = ctx->dalloc<double>(std::max(ctx->n, 1));
  W.part = ctx->dalloc<double>((size_t)kNumSlots * kMaxBlocks);
  W.cam_split = nvc > 0 ? std::min(kCamSplit, std::max(1, 2048 / nvc)) : 1;
  W.cpart = ctx->dalloc<double>((size_t)W.cam_split * 27 * std::max(nvc, 1));

  HIP_OK(hipMemsetAsync(W.part, 0, sizeof(double) * kNumSlots * kMaxBlocks, ctx->stream));
  HIP_OK(hipMemsetAsync(W.scal, 0, sizeof(double) * (kNumSlots + kPcgState), ctx->stream));
  HIP_OK(hipStreamSynchronize(ctx->stream));
  ctx->perm.swap(perm);
  ctx->h_pt_off.swap(pt_off);
  ctx->h_obs_cam.swap(obs_cam);
  ctx->h_vc.swap(vc);
  ctx->h_pt_var.swap(pt_var);
  ctx->have_problem = true;
}

// The overlapped form's plan (ba_kernels.h OvPlan, ba_chol_persist.hip
// OvArgs): every S entry of the lower tiles is rewritten each step (no empty
// camera pair, no point observed twice by one camera), the persistent grid
// fits, and the launch takes every CU.  Work items per XCD queue in tile-column
// order: for each tile column, the diagonal slices of its cameras (dealt
// round-robin over the queues), then its pair blocks in row-major order, cut
// into 8 contiguous runs of equal pair count (one per queue: the runs of a
// column are formed side by side) and grouped 4 to an item.
void build_overlap_plan(ba_ctx* ctx, const std::vector<int4>& blocks) {
  DevWork& W = ctx->W;
  W.ov = OvPlan{};
  const int n = ctx->n, nvc = ctx->nvc, G = W.cam_split;
  const int T = (n + 63) / 64, TR = (n + 1 + 63) / 64;
  if (!W.chol_persist || nvc == 0 || nvc > bahip::kLinLdsCamsHost || ctx->dup_diag || W.s_memset || W.neblocks != 0)
    return;
  const int cap = bahip::chol_persist_capacity(ctx->device);
  int grid = 1;
  for (int j = 1; j < T; ++j) grid += TR - (j == 1 ? 2 : j);   // (chol_persist_grid)
  // (at least one helper per XCD queue: a queue's last items are then always
  // taken, whatever the workers are waiting for)
  if (cap < grid + 8) return;
  grid = cap;
  std::vector<unsigned> tgt((size_t)TR * T, 0);
  auto tile = [&](int r, int c) { return (size_t)(r >> 6) * T + (c >> 6); };
  std::vector<std::vector<int>> colblk(T);
  for (size_t b = 0; b < blocks.size(); ++b) {
    const int I = blocks[b].x, J = blocks[b].y;
    if (I <= J) return;   // (a diagonal pair block: not this form)
    colblk[(6 * J) >> 6].push_back((int)b);
    const int r0 = 6 * I, c0 = 6 * J;
    std::vector<size_t> ts = {tile(r0, c0), tile(r0, c0 + 5), tile(r0 + 5, c0), tile(r0 + 5, c0 + 5)};
    std::sort(ts.begin(), ts.end());
    ts.erase(std::unique(ts.begin(), ts.end()), ts.end());
    for (size_t t : ts) ++tgt[t];
  }
  for (int v = 0; v < nvc; ++v)
    for (int k = 0; k < 27; ++k) {
      int row, col;
      if (k < 21) {
        int a = 0;
        while ((a + 1) * (a + 2) / 2 <= k) ++a;
        row = 6 * v + a;
        col = 6 * v + k - a * (a + 1) / 2;
      } else {
        row = n;
        col = 6 * v + k - 21;
      }
      ++tgt[tile(row, col)];
    }
  for (int I = 0; I < TR; ++I)
    for (int J = 0; J < T && J <= I; ++J)
      if (tgt[(size_t)I * T + J] == 0) return;   // (a lower tile nothing writes)
  std::vector<int4> items[8];
  std::vector<int> icol[8];
  int unit_rr = 0;
  const char* fe = std::getenv("BA_OV_FIRST_COLS");
  const int first_cols = fe ? std::max(0, atoi(fe)) : 0;
  for (int tc = 0; tc < T; ++tc) {
    for (int v = 0; v < nvc; ++v) {
      if ((6 * v) >> 6 != tc) continue;
      for (int g = 0; g < G; ++g) {
        const int x = unit_rr++ & 7;
        items[x].push_back(make_int4(-1 - (v * G + g), 0, 0, 0));
        for (int q = 1; q < 4; ++q) items[x].push_back(make_int4(0, 0, 0, 0));
        icol[x].push_back(tc);
      }
    }
    const std::vector<int>& cb = colblk[tc];
    long long tot = 0;
    for (int b : cb) tot += blocks[b].w - blocks[b].z;
    size_t k = 0;
    long long acc = 0;
    for (int x = 0; x < 8; ++x) {
      const long long until = tot * (x + 1) / 8;
      std::vector<int> run;
      while (k < cb.size() && (acc < until || x == 7)) {
        acc += blocks[cb[k]].w - blocks[cb[k]].z;
        run.push_back(cb[k++]);
      }
      // (BA_OV_FIRST_COLS, default 0: the first columns one block to an item,
      // meant to start the chain sooner — measured slower, C3 0.64 ms with
      // column 0 alone, 0.97 with every column, vs 0.58: an item's fixed cost
      // outweighs its length; profiles/r06_v11_ov_first_cols_ab.txt)
      const int per = tc < first_cols ? 1 : 4;
      for (size_t r = 0; r < run.size(); r += per) {
        for (int q = 0; q < 4; ++q)
          items[x].push_back(q < per && r + q < run.size() ? blocks[run[r + q]] : make_int4(0, 0, 0, 0));
        icol[x].push_back(tc);
      }
    }
  }
  std::vector<int4> all;
  std::vector<int> allc;
  OvPlan& P = W.ov;
  for (int x = 0; x < 8; ++x) {
    P.ioff[x] = (int)allc.size();
    all.insert(all.end(), items[x].begin(), items[x].end());
    allc.insert(allc.end(), icol[x].begin(), icol[x].end());
  }
  P.ioff[8] = (int)allc.size();
  P.irec = ctx->upload(all);
  P.item_col = ctx->upload(allc);
  P.tgt = ctx->upload(tgt);
  const size_t nctr = 2 * (size_t)TR * T + nvc + 8;   // cnt | cam_cnt | q | pflag
  P.ctr = ctx->dalloc<unsigned>(nctr);
  HIP_OK(hipMemsetAsync(P.ctr, 0, sizeof(unsigned) * nctr, ctx->stream));
  P.grid = grid;
  P.launches = 0;
  P.ok = true;
}

// DENSE_SCHUR structures (built on the first dense solve): the dense reduced
// system S / factor Lf (16 n^2 bytes), Cholesky block inverses, and the Schur
// pair lists.
void ensure_dense(ba_ctx* ctx) {
  if (ctx->have_dense) return;
  const int np = ctx->np, nvc = ctx->nvc;
  const std::vector<int>& pt_off = ctx->h_pt_off;
  const std::vector<int>& obs_cam = ctx->h_obs_cam;
  const std::vector<int>& vc = ctx->h_vc;
  const std::vector<uint8_t>& pt_var = ctx->h_pt_var;
  // Schur pair lists: for every variable point, every pair of its observations
  // by variable cameras contributes W_a W_b^T to block (vc_a, vc_b), vc_a >= vc_b.
  std::vector<int4> blocks;
  std::vector<int2> pairs;
  {
    struct PE { int64_t key; int a, b; };
    std::vector<PE> pe;
    size_t est = 0;
    for (int p = 0; p < np; ++p) if (pt_var[p]) { const size_t k = pt_off[p + 1] - pt_off[p]; est += k * (k - 1) / 2; }
    pe.reserve(est);
    std::vector<int> lst;
    for (int p = 0; p < np; ++p) {
      if (!pt_var[p]) continue;
      lst.clear();
      for (int s = pt_off[p]; s < pt_off[p + 1]; ++s) if (vc[obs_cam[s]] >= 0) lst.push_back(s);
      for (size_t i = 0; i < lst.size(); ++i)
        for (size_t j = 0; j < i; ++j) {
          const int a = lst[i], b = lst[j];        // vc[a] >= vc[b] (sorted by camera)
          const int I = vc[obs_cam[a]], J = vc[obs_cam[b]];
          const int64_t key = (int64_t)I * nvc + J;
          pe.push_back({key, a, b});
          if (I == J) pe.push_back({key, b, a});    // duplicate camera on one point
        }
    }
    // stable counting/radix by key keeps point order inside a block
    std::stable_sort(pe.begin(), pe.end(), [](const PE& x, const PE& y) { return x.key < y.key; });
    pairs.resize(pe.size());
    for (size_t i = 0; i < pe.size(); ++i) {
      pairs[i] = make_int2(pe[i].a, pe[i].b);
      if (i == 0 || pe[i].key != pe[i - 1].key) {
        if (!blocks.empty()) blocks.back().w = (int)i;
        blocks.push_back(make_int4((int)(pe[i].key / nvc), (int)(pe[i].key % nvc), (int)i, 0));
      }
    }
    if (!blocks.empty()) blocks.back().w = (int)pe.size();
  }
  {
    const int T = (ctx->n + 63) / 64, cap = bahip::back_flow_capacity(ctx->device);
    if (cap < 0) throw BaError{BA_ERR_DEVICE, "occupancy query for the back substitution failed"};
    if (T > cap)
      throw BaError{BA_ERR_INVALID_ARGUMENT, "DENSE_SCHUR: " + std::to_string(T) + " block columns exceed the " +
                                                 std::to_string(cap) + " resident back-substitution workgroups; "
                                                 "use ITERATIVE_SCHUR"};
  }
  DevWork& W = ctx->W;
  W.S = ctx->dalloc<double>((size_t)(ctx->n + 1) * std::max(ctx->ld, 1));
  W.Lf = ctx->dalloc<double>((size_t)(ctx->n + 1) * std::max(ctx->ld, 1));
  W.Ubuf = (ctx->n + 63) / 64 < bahip::chol_split_blocks()
               ? ctx->dalloc<double>((size_t)(ctx->n + 1) * std::max(ctx->ld, 1)) : nullptr;
  W.Vbuf = ctx->dalloc<double>((size_t)((ctx->n + 63) / 64 + 1) * 64 * 64);
  W.ctask = nullptr;
  W.ctask_off = nullptr;
  std::vector<int4> tasks_h;
  if ((ctx->n + 63) / 64 >= bahip::chol_split_blocks() && bahip::chol_split_rank() > 0) {
    bahip::chol_split_tasks(ctx->n, tasks_h, ctx->chol_off);
    W.ctask = ctx->upload(tasks_h);
    W.ctask_off = ctx->chol_off.data();
  }
  W.chol_fuse = W.ctask && bahip::chol_split_fused();
  W.chol_flow = false;
  W.ftask = nullptr;
  W.nftask = 0;
  W.tflag = nullptr;
  if (W.ctask && bahip::chol_split_flow() &&
      (size_t)(ctx->n + 1) * std::max(ctx->ld, 1) * sizeof(double) < ((size_t)1 << 31)) {   // (32-bit buffer offsets)
    std::vector<int4> flow;
    bahip::chol_flow_tasks(tasks_h, ctx->chol_off, flow);
    W.ftask = ctx->upload(flow);
    W.nftask = (int)flow.size();
    const size_t T = (ctx->n + 63) / 64, TR = (ctx->n + 1 + 63) / 64;
    W.tflag = ctx->dalloc<unsigned>(2 * TR * T);
    HIP_OK(hipMemsetAsync(W.tflag, 0, sizeof(unsigned) * 2 * TR * T, ctx->stream));
    W.chol_flow = true;
  }
  W.yg = ctx->dalloc<double>(2 * (size_t)std::max(ctx->n, 1));
  {
    // persistent factorisation (one launch) when the per-step form would not
    // split and the whole grid is resident; BA_CHOL_PERSIST=0 forces the
    // per-step launches (A/B).  Not with the host-staged transport: its ranks
    // may share one GPU, and their persistent grids need not all fit at once
    // (a spin bound would then be hit on some ranks only, and the ranks'
    // steps would diverge)
    const int T = (ctx->n + 63) / 64, TR = (ctx->n + 1 + 63) / 64;
    const char* env = std::getenv("BA_CHOL_PERSIST");
    W.chol_persist = ctx->n > 0 && T < bahip::chol_split_blocks() && !(env && env[0] == '0') && !ctx->host_fn &&
                     bahip::chol_persist_fits(ctx->device, ctx->n);
    const size_t nf = (size_t)T + (size_t)TR * T;
    W.cflags = ctx->dalloc<unsigned>(nf);
    HIP_OK(hipMemsetAsync(W.cflags, 0, sizeof(unsigned) * std::max<size_t>(nf, 1), ctx->stream));
  }
  W.Spk = nullptr;
  // diagonal pair blocks (a point observed twice by one camera) update the
  // S diagonal after the fold: the LM diagonal is then added after them
  // (separate k_cam_add_diag), in the order the exchange path uses
  ctx->dup_diag = std::any_of(blocks.begin(), blocks.end(), [](const int4& b) { return b.x == b.y; });
  // k_schur_pairs*: XCD x sweeps the blocks [xoff[x], xoff[x+1]): equal
  // contiguous ranges of the row-major list (bands of rows: C3 165 vs 188 us
  // for an interleave)
  std::vector<int> xoff(9, 0);
  {
    const int R = ((int)blocks.size() + 7) / 8;
    for (int x = 0; x <= 8; ++x) xoff[x] = std::min((int)blocks.size(), x * R);
    W.xmax = R;
  }
  W.blocks = ctx->upload(blocks);
  W.nblocks = (int)blocks.size();
  W.xoff = ctx->upload(xoff);
  W.pairs = ctx->upload(pairs);
  HIP_OK(hipMemsetAsync(W.yg, 0, sizeof(double) * 2 * (size_t)std::max(ctx->n, 1), ctx->stream));
  // S is rewritten every step (diagonal blocks, rhs and every co-observed
  // block); the rest of the lower triangle must be re-zeroed (the Cholesky
  // updates it in place): a list of those blocks, or a memset when they are
  // the majority
  {
    const size_t nlow = (size_t)nvc * (nvc - (nvc > 0 ? 1 : 0)) / 2;
    const size_t nfull = (size_t)std::count_if(blocks.begin(), blocks.end(), [](const int4& b) { return b.x != b.y; });
    const size_t nempty = nlow - nfull;
    W.s_memset = nempty > nfull || nempty > (size_t)(1 << 22);
    W.neblocks = 0;
    W.eblocks = nullptr;
    if (!W.s_memset && nempty > 0) {
      std::vector<uint8_t> used(nlow, 0);
      auto lid = [](size_t I, size_t J) { return I * (I - 1) / 2 + J; };   // I > J
      for (const int4& b : blocks) if (b.x != b.y) used[lid(b.x, b.y)] = 1;
      std::vector<int2> eb;
      eb.reserve(nempty);
      for (int I = 1; I < nvc; ++I)
        for (int J = 0; J < I; ++J) if (!used[lid(I, J)]) eb.push_back(make_int2(I, J));
      W.eblocks = ctx->upload(eb);
      W.neblocks = (int)eb.size();
    }
  }
  HIP_OK(hipMemsetAsync(W.S, 0, sizeof(double) * (size_t)(ctx->n + 1) * std::max(ctx->ld, 1), ctx->stream));
  build_overlap_plan(ctx, blocks);
  HIP_OK(hipStreamSynchronize(ctx->stream));
  ctx->have_dense = true;
}

// ITERATIVE_SCHUR structures: compact diagonal blocks, preconditioner, CG
// vectors, matvec scratch, and the (rare) pairs of observations of one point
// by one camera, whose cross terms belong to the Schur-Jacobi diagonal block.
void ensure_pcg(ba_ctx* ctx) {
  if (ctx->have_pcg) return;
  const int np = ctx->np, nvc = ctx->nvc;
  const size_t n = (size_t)std::max(ctx->n, 1);
  DevWork& W = ctx->W;
  W.pcg_G = W.cam_split;
  W.Sd = ctx->dalloc<double>(27 * (size_t)std::max(nvc, 1));
  W.Adiag = ctx->dalloc<double>(21 * (size_t)std::max(nvc, 1));
  W.Minv = ctx->dalloc<double>(36 * (size_t)std::max(nvc, 1));
  W.pb = ctx->dalloc<double>(n);
  W.pr = ctx->dalloc<double>(n);
  W.pz = ctx->dalloc<double>(n);
  W.pp = ctx->dalloc<double>(n);
  W.pq = ctx->dalloc<double>(n);
  W.vpt = ctx->dalloc<double>(3 * (size_t)std::max(np, 1));
  W.vacc = ctx->dalloc<double>(3 * (size_t)std::max(np, 1));
  // a point with no observation never gets a vpt entry (the point passes
  // store it at the end of a point's run), but k_pcg_vacc folds every point:
  // zeros, so such a point's accumulated product and step stay 0
  HIP_OK(hipMemsetAsync(W.vpt, 0, sizeof(double) * 3 * (size_t)std::max(np, 1), ctx->stream));
  HIP_OK(hipMemsetAsync(W.vacc, 0, sizeof(double) * 3 * (size_t)std::max(np, 1), ctx->stream));
  W.tpart = ctx->dalloc<double>((size_t)W.pcg_G * 6 * std::max(nvc, 1));
  W.ppart = ctx->dalloc<double>(3 * (size_t)kMaxBlocks);
  if ((nvc + 255) / 256 > kMaxBlocks) throw BaError{BA_ERR_INVALID_ARGUMENT, "too many cameras for ITERATIVE_SCHUR"};
  std::vector<int> dup_off(nvc + 1, 0);
  std::vector<int2> dup;
  {
    std::vector<std::vector<int2>> per(nvc);
    for (int p = 0; p < np; ++p) {
      if (!ctx->h_pt_var[p]) continue;
      for (int a = ctx->h_pt_off[p]; a < ctx->h_pt_off[p + 1]; ++a)
        for (int b = a + 1; b < ctx->h_pt_off[p + 1] && ctx->h_obs_cam[b] == ctx->h_obs_cam[a]; ++b) {
          const int v = ctx->h_vc[ctx->h_obs_cam[a]];
          if (v >= 0) per[v].push_back(make_int2(a, b));
        }
    }
    for (int v = 0; v < nvc; ++v) {
      dup_off[v + 1] = dup_off[v] + (int)per[v].size();
      dup.insert(dup.end(), per[v].begin(), per[v].end());
    }
  }
  W.dup_off = ctx->upload(dup_off);
  W.dup_pairs = ctx->upload(dup);
  ctx->pcg_ndup = dup.size();
  {
    // point-aligned chunks of <= 64 observations for the PCG point pass
    // (k_pcg_point_seg); BA_PCG_SEG=0 keeps the value-pair passes
    const char* e = std::getenv("BA_PCG_SEG");
    std::vector<int2> ch;
    bool ok = !(e && e[0] == '0');
    int start = 0;
    for (int p = 0; p < np && ok; ++p) {
      const int a = ctx->h_pt_off[p], b = ctx->h_pt_off[p + 1];
      if (b - a > 64) { ok = false; break; }
      if (b - start > 64) { ch.push_back(make_int2(start, a)); start = a; }
    }
    if (ok && ctx->no > start) ch.push_back(make_int2(start, ctx->no));
    W.npchunks = ok ? (int)ch.size() : 0;
    W.pchunks = ok && !ch.empty() ? ctx->upload(ch) : nullptr;
    if (!W.pchunks) W.npchunks = 0;
  }
  HIP_OK(hipStreamSynchronize(ctx->stream));
  ctx->have_pcg = true;
}

// ---------------------------------------------------------------------------
// LM phases
// ---------------------------------------------------------------------------
struct LinResult { double cost, gmax, gnorm, xnorm; bool ok; };

constexpr uint32_t bit(int s) { return 1u << s; }

// Linearisation phase: enqueue (no host sync) / read back.  The solver
// enqueues the next trust-region step right behind an accepted step's
// linearisation and reads both records with one host sync (the step is
// wasted only when the new gradient ends the solve).
// defer_reduce: a step_enqueue follows before the next read_scalars and
// folds this linearisation's scalars with its own (single rank only)
void linearize_enqueue(ba_ctx* ctx, bool compute_scale, double min_diag, double max_diag, bool time_rj = false,
                       bool defer_reduce = false) {
  const hipStream_t s = ctx->stream;
  DevProblem& P = ctx->P;
  DevWork& W = ctx->W;
  ctx->lin_at_cand = false;
  launch_lin_prep(P, W, s);
  // time_rj: kernel execution stamps from the launch itself (bench roofline),
  // into the stamp pair ctx->rj_slot
  hipEvent_t e0 = time_rj ? ctx->ev[2 + 2 * ctx->rj_slot] : nullptr, e1 = time_rj ? ctx->ev[3 + 2 * ctx->rj_slot] : nullptr;
  launch_linearize(P, W, s, e0, e1);
  // (J-free: the timed residual + Jacobian kernel is k_lin_point, launched here)
  launch_point_assemble(P, W, compute_scale, min_diag, max_diag, s, W.jrfree ? e0 : nullptr, W.jrfree ? e1 : nullptr);
  launch_cam_assemble(P, W, s);
  // point-side scalars: folded here when they must be all-reduced before
  // cam_norms, else together with the camera-side ones (one launch less)
  const uint32_t lin_sum = bit(SL_COST) | bit(SL_LIN_BAD) | bit(SL_GN2_P) | bit(SL_XN2_P);
  if (ctx->coll()) launch_reduce(W, lin_sum, bit(SL_GMAX_P), s);
  if (ctx->coll()) {
    // Hcc, gc, COST, LIN_BAD, GN2_P, XN2_P (contiguous), then the max
    ctx->allreduce(W.Hcc, 27 * (size_t)ctx->nvc + SL_GMAX_P);
    ctx->allreduce(W.scal + SL_GMAX_P, 1, ncclMax);
  }
  // deferred fold (single rank): the norms ride in the step's point
  // elimination (BA_NORMS_FOLD=0: their own launch here)
  const char* nfe = getenv("BA_NORMS_FOLD");   // (read per call: tests switch it)
  const bool norms_fold_on = !(nfe && nfe[0] == '0');
  if (defer_reduce && !ctx->coll() && norms_fold_on) {
    ctx->norms_pend = true;
    ctx->norms_args = norms_fold(W, compute_scale, min_diag, max_diag);
  } else {
    ctx->norms_pend = false;
    launch_cam_norms(P, W, compute_scale, min_diag, max_diag, s);
  }
  const uint32_t sum_mask = bit(SL_GN2_C) | bit(SL_XN2_C) | (ctx->coll() ? 0u : lin_sum);
  const uint32_t max_mask = bit(SL_GMAX_C) | (ctx->coll() ? 0u : bit(SL_GMAX_P));
  if (defer_reduce && !ctx->coll()) {
    ctx->pend_sum |= sum_mask;
    ctx->pend_max |= max_mask;
  } else {
    launch_reduce(W, sum_mask, max_mask, s);
  }
  if (compute_scale) ctx->scale_valid = true;
}

// after ctx->read_scalars()
LinResult lin_result(ba_ctx* ctx) {
  const double* h = ctx->h_scal;
  LinResult r;
  r.cost = h[SL_COST];
  r.gmax = std::max(h[SL_GMAX_P], h[SL_GMAX_C]);
  r.gnorm = std::sqrt(h[SL_GN2_P] + h[SL_GN2_C]);
  r.xnorm = std::sqrt(h[SL_XN2_P] + h[SL_XN2_C]);
  r.ok = h[SL_LIN_BAD] == 0.0 && std::isfinite(r.cost);
  return r;
}

LinResult linearize(ba_ctx* ctx, bool compute_scale, double min_diag, double max_diag) {
  // a fresh start (solve / bench entry): folds still pending belong to work
  // an earlier call abandoned (e.g. the speculative linearisation behind a
  // solve's last step) and must not be folded into this record
  ctx->clear_pending();
  linearize_enqueue(ctx, compute_scale, min_diag, max_diag);
  ctx->read_scalars();
  return lin_result(ctx);
}

struct StepResult { bool linear_ok; double mcc, cand_cost, step_norm; int ls_iters; bool spin; };

// DENSE_SCHUR: explicit reduced camera system (form_reduced_dense) + dense
// Cholesky
// Returns true when S is left to the factorisation's launch (the overlapped
// form, launch_cholesky_solve_ov: single rank, compact W records, the
// persistent factorisation; BA_CHOL_OVERLAP=0, read per step, or
// allow_ov = false keeps the separate pair / diagonal / fold launches)
bool form_reduced_dense(ba_ctx* ctx, double radius, bool allow_ov = true) {
  const hipStream_t s = ctx->stream;
  DevProblem& P = ctx->P;
  DevWork& W = ctx->W;
  ensure_dense(ctx);
  const char* oe = getenv("BA_CHOL_OVERLAP");
  const bool ov = allow_ov && !(oe && oe[0] == '0') && W.ov.ok && W.chol_persist && !ctx->coll() && !ctx->dup_diag &&
                  radius > 0.0 && W.wcompact && !W.jdiag && !W.w32 && ctx->n > 0;
  if (ov) {
    launch_point_elim(P, W, radius, s, ctx->take_norms());
    return true;
  }
  if (ctx->n > 0) {
    if (W.s_memset) HIP_OK(hipMemsetAsync(W.S, 0, sizeof(double) * (size_t)(ctx->n + 1) * ctx->ld, s));
    else launch_zero_blocks(P, W, s);
  }
  launch_point_elim(P, W, radius, s, ctx->take_norms());
  // single rank, no diagonal pair blocks: the LM diagonal goes in with the
  // fold (same operation order as the exchange path's, bitwise)
  const bool fused_diag = !ctx->coll() && !ctx->dup_diag;
  // ... and that fold rides in the pair pass's launch when it can (one
  // launch fewer; the fold writes only the diagonal blocks and the rhs)
  const bool fold_in_pairs = fused_diag && radius > 0.0 && pairs_take_fold(P, W);
  if ((fold_in_pairs && pairs_take_diag(P, W)) || (fused_diag && radius > 0.0 && pairs_take_diag_nt(P, W))) {
    // ... or rather the diagonal slices ride in it (dispatched after the pair
    // workgroups, they fill the pass's tail) and the fold follows
    launch_schur_pairs(P, W, s, 0.0, true);
    launch_cam_fold_diag(P, W, radius, s);
  } else {
    launch_cam_schur_diag(P, W, s, nullptr, fused_diag ? radius : 0.0, fold_in_pairs);
    launch_schur_pairs(P, W, s, fold_in_pairs ? radius : 0.0);
  }
  if (ctx->coll()) launch_reduce(W, bit(SL_ELIM_BAD), 0, s);   // else folded with the step scalars
  if (ctx->coll()) {
    // only the lower triangle and the rhs row of S carry data: all-reduce
    // them packed (n(n+1)/2 + n doubles instead of (n+1) n)
    // (+1: the elimination-failure count rides along)
    const size_t npk = (size_t)ctx->n * (ctx->n + 1) / 2 + ctx->n;
    if (!W.Spk) W.Spk = ctx->dalloc<double>(npk + 1);
    launch_pack_lower(P, W, true, s);
    ctx->allreduce(W.Spk, npk + 1);
    launch_pack_lower(P, W, false, s);
  }
  if (!fused_diag) launch_cam_add_diag(P, W, radius, s);   // (after the exchange)
  return false;
}
void reduced_solve_dense(ba_ctx* ctx, double radius) {
  if (form_reduced_dense(ctx, radius))
    launch_cholesky_solve_ov(ctx->P, ctx->W, ctx->W.ov, radius, ++ctx->chol_epoch, ctx->stream);
  else
    launch_cholesky_solve2(ctx->P, ctx->W, ++ctx->chol_epoch, ctx->stream);
}

// ITERATIVE_SCHUR: implicit Schur complement + PCG (ba_pcg.hip).  The host
// enqueues CG iterations in batches and reads the device-side state record
// between batches (the kernels of iterations past termination return at
// once); every rank enqueues the same sequence, so the RCCL all-reduce of
// each matvec's camera slices stays matched.  Returns the CG iteration count.
int reduced_solve_pcg(ba_ctx* ctx, double radius, const ba_options& o) {
  const hipStream_t s = ctx->stream;
  DevProblem& P = ctx->P;
  DevWork& W = ctx->W;
  ensure_pcg(ctx);
  {
    // per-observation products t_o = W_o v_p: the camera pass then reads 48 B
    // per observation instead of gathering 144 + 24 B.  With the point-aligned
    // chunks (k_pcg_point_seg forms t_o from the W it has just staged, the
    // camera pass gathers them by LDS-DMA) always: C4 shard 1998-2029 ->
    // 2091-2098 M-obs/s (profiles/r04_v13_ab_pcg_t_c4shard.txt).  Without
    // them (k_pcg_point_t re-reads W) only when the fp64 W outgrows the
    // 256-MiB Infinity Cache (C5 shard +2.7 %; below it the extra pass lost
    // ~0.7 %).  BA_PCG_T=0 / 1 (diagnostics) forces it off / on.
    const char* fe = getenv("BA_PCG_T");   // (read per solve: tests switch it)
    const int force = fe ? atoi(fe) : -1;
    // (the Infinity-Cache test uses the largest rank's shard; the chunk and
    // duplicate-pair tests below are per rank, so ranks may run different
    // matvec forms: that changes only the rounding of each rank's own
    // contribution, which is all-reduced before anything is decided, so the
    // ranks' decisions stay identical)
    const bool big = 144.0 * (double)ctx->max_no > 256.0 * 1024 * 1024;
    const bool use_t = force >= 0 ? force != 0 : W.npchunks > 0 || (big && !W.w32);
    if (use_t && !ctx->tobs_buf) ctx->tobs_buf = ctx->dalloc<double>(6 * (size_t)std::max(ctx->no, 1));
    if (!use_t && ctx->tobs_buf) { ctx->dfree(ctx->tobs_buf); ctx->tobs_buf = nullptr; }   // 48 B/obs back
    W.tobs = use_t ? ctx->tobs_buf : nullptr;
  }
  PcgOpts po{o.eta, o.min_linear_solver_iterations, std::max(1, o.max_linear_solver_iterations),
             o.preconditioner_type == BA_SCHUR_JACOBI ? 1 : 0};
  launch_point_elim(P, W, radius, s, ctx->take_norms());
  launch_cam_schur_diag(P, W, s, W.Sd);
  if (po.schur_jacobi && ctx->pcg_ndup > 0) launch_pcg_dup(P, W, s);   // (this rank's duplicate pairs)
  // exchange path: one 6 nvc vector per matvec crosses the ranks (the
  // camera slices are folded first, in the order the single-rank update
  // folds them, so both paths round identically).  The point-elimination
  // failure count is folded and all-reduced with the step's scalars at its
  // end (step_enqueue): a failed elimination on any rank makes the all-reduced
  // products non-finite, so every rank's CG stops alike and the step is
  // rejected on every rank (one collective fewer per LM iteration)
  const size_t tcount = (size_t)6 * ctx->nvc;
  W.pcg_folded = ctx->coll();
  if (ctx->coll()) ctx->allreduce(W.Sd, 27 * (size_t)ctx->nvc);
  if (ctx->nvc == 0) {
    if (W.pacc && P.np > 0) HIP_OK(hipMemsetAsync(W.vacc, 0, sizeof(double) * 3 * (size_t)P.np, s));   // (y = 0)
    // k_pcg_setup_fin, which clears them otherwise, does not run: a spin or
    // pivot failure left by an earlier DENSE_SCHUR solve of this context must
    // not be read back as this step's
    HIP_OK(hipMemsetAsync(W.scal + SL_CHOL_SPIN, 0, sizeof(double), s));
    HIP_OK(hipMemsetAsync(W.scal + SL_CHOL_BAD, 0, sizeof(double), s));
    return 0;
  }
  launch_pcg_setup(P, W, radius, po, s);
  int it = 0, batch = 4;
  for (;;) {
    for (int k = 0; k < batch && it < po.max_iter; ++k) {
      ++it;
      launch_pcg_matvec(P, W, W.pp, s);
      if (ctx->coll()) { launch_pcg_tfold(P, W, s); ctx->allreduce(W.tpart, tcount); }
      if (it % 10 == 0) {   // ceres residual_reset_period: r = b - S x
        launch_pcg_update(P, W, 1, it, po, s);
        launch_pcg_matvec(P, W, W.y, s);
        if (W.pacc) launch_pcg_vacc(P, W, it, true, s);   // vpt(y) itself
        if (ctx->coll()) { launch_pcg_tfold(P, W, s); ctx->allreduce(W.tpart, tcount); }
        launch_pcg_update(P, W, 2, it, po, s);
      } else {
        launch_pcg_update(P, W, 0, it, po, s);
        if (W.pacc) launch_pcg_vacc(P, W, it, false, s);
      }
    }
    ctx->read_scalars();
    if (ctx->h_scal[kNumSlots + PS_DONE] != 0.0 || it >= po.max_iter) break;
    batch = std::min(2 * batch, 32);
  }
  return (int)ctx->h_scal[kNumSlots + PS_ITER];
}

// Trust-region step phase: enqueue (the PCG reads its state record between
// batches of CG iterations) / read back.  Returns the linear-solver iterations.
// the per-observation Schur blocks of a step: fp32 or fp64, compact records,
// camera-major copies
void step_w_storage(ba_ctx* ctx, const ba_options& o) {
  DevWork& W = ctx->W;
  W.w32 = o.precision == BA_MIXED_FP32;
  if (W.w32 && !W.Wf) W.Wf = ctx->dalloc<float>(18 * (size_t)ctx->no);
  if (!W.w32 && !W.W) W.W = ctx->dalloc<double>(18 * (size_t)ctx->no);
  {
    // compact W records (ba_kernels.hip k_obs_w_rc<double, true>): the
    // J-free fp64 DENSE_SCHUR iteration with the fused point step (the only
    // W readers are then k_cam_schur_diag_c and k_schur_pairs_c);
    // BA_WCOMPACT=0 (diagnostics, read per solve) keeps the 18-double blocks
    const char* e = getenv("BA_WCOMPACT");
    W.wcompact = W.jrfree && ctx->nvc <= bahip::kWcCamsHost && !W.w32 && o.linear_solver == BA_DENSE_SCHUR &&
                 !(e && e[0] == '0');
  }
  {
    // the diagonal Schur blocks J-free (k_cam_schur_diag_rc) where they would
    // gather the 18-value W (ITERATIVE_SCHUR, or DENSE_SCHUR without compact
    // records): C4 3.53 vs 3.74 ms with the W-reading pass
    // (profiles/r04_v4_jdiag_tscat_ab.txt)
    W.jdiag = W.jrfree && !W.wcompact;
    if (W.jdiag && !W.prec) W.prec = ctx->dalloc<double>(16 * (size_t)std::max(ctx->np, 1));
    // the PCG point pass over the 16-value rank-2 records (k_obs_w_rc<.., PC>:
    // 128 B per observation fp64, 64 B fp32): only where nothing else reads
    // W — the diagonal blocks J-free, the fused point step, the products t_o,
    // no duplicate (camera, point) pairs, every point in the point-aligned
    // chunks — and K without skew.  BA_PCG_PC=0
    // (read per solve) keeps the 18-value records
    W.pcgc = false;
    const char* pe = getenv("BA_PCG_PC");
    const char* te = getenv("BA_PCG_T");
    if (!(pe && pe[0] == '0') && o.linear_solver == BA_ITERATIVE_SCHUR && W.jdiag && ctx->k_plain &&
        obs_w_pc_ok(ctx->P, W) && !(te && te[0] == '0')) {
      ensure_pcg(ctx);
      W.pcgc = W.npchunks > 0 && ctx->pcg_ndup == 0;
    }
    // fp64 beyond the LDS camera table (compact camera records): the point
    // pass forms those records itself instead of reading them
    // (k_pcg_point_jf, no W): C4 fixed radius 2.82 vs 3.14 ms per LM
    // iteration, along the trajectory 3.66 vs 3.89, C4 shard 0.50 vs 0.56;
    // with fp32 W (64-B records) the stored records win (C5 shard 3.65 vs
    // 3.81 ms: profiles/r05_v5_pcg_jfree_ab.txt).  BA_PCG_JF=0 / 1 (read per
    // solve) forces it off / on
    // the back substitution from the CG's accumulated point products (no J in
    // k_point_step_rc: k_pcg_vacc, the block-form model cost change).  With
    // fp32 W (MIXED_FP32) the products carry the stored fp32 blocks into the
    // back substitution as they carry them into the CG (a relative 1e-7
    // perturbation of the point step; the costs stay within the oracle
    // comparisons' 1e-9).  BA_PCG_PACC=0 (read per solve) recomputes J per
    // observation, in fp64
    W.pacc = false;
    const char* ae = getenv("BA_PCG_PACC");
    if (o.linear_solver == BA_ITERATIVE_SCHUR && W.jrfree && !(ae && ae[0] == '0')) {
      ensure_pcg(ctx);
      W.pacc = W.npchunks > 0;
    }
    W.mcc_cam = ctx->rank == 0;
    const char* je = getenv("BA_PCG_JF");
    const bool jf_ok = W.pcgc && ctx->P.nc > bahip::kLinLdsCamsHost;
    W.pcgjf = jf_ok && (je ? je[0] != '0' : !W.w32);
  }
}
int step_enqueue(ba_ctx* ctx, double radius, const ba_options& o) {
  const hipStream_t s = ctx->stream;
  DevProblem& P = ctx->P;
  DevWork& W = ctx->W;
  step_w_storage(ctx, o);
  // (SL_CHOL_BAD is cleared by k_cam_add_diag / k_pcg_setup_fin, the first
  // kernels that may set it, so no separate memset per step)
  int ls_iters = 1;
  if (o.linear_solver == BA_ITERATIVE_SCHUR) ls_iters = reduced_solve_pcg(ctx, radius, o);
  else reduced_solve_dense(ctx, radius);
  launch_cam_candidate(P, W, s);
  launch_backsub_candidate(P, W, s);
  // (DENSE_SCHUR under collectives: the elimination failures already
  // crossed the ranks with the packed S)
  const bool pcg = o.linear_solver == BA_ITERATIVE_SCHUR;
  const uint32_t step_sum = bit(SL_MCC_NEG) | bit(SL_CCOST) | bit(SL_STEP2_P) | bit(SL_CAND_BAD) | bit(SL_STEP_BAD) |
                            bit(SL_STEP2_C) | (ctx->coll() && !pcg ? 0u : bit(SL_ELIM_BAD));
  if (!ctx->coll()) {
    // folded by the scalar record's publish that follows every step
    // (ba_ctx::publish_scalars: one launch for the fold and the record)
    ctx->pend_sum |= step_sum;
    return ls_iters;
  }
  launch_reduce(W, step_sum | ctx->pend_sum, ctx->pend_max, s);
  ctx->pend_sum = ctx->pend_max = 0;
  if (ctx->coll()) {
    // MCC_NEG, CCOST, STEP2_P, CAND_BAD, STEP_BAD, CHOL_SPIN (+ ELIM_BAD: ITERATIVE_SCHUR)
    ctx->allreduce(W.scal + SL_MCC_NEG, pcg ? 7 : 6);
  }
  return ls_iters;
}

// after ctx->read_scalars()
StepResult step_result(ba_ctx* ctx, int ls_iters) {
  const double* h = ctx->h_scal;
  StepResult r;
  r.linear_ok = h[SL_ELIM_BAD] == 0.0 && h[SL_CHOL_BAD] == 0.0 && h[SL_STEP_BAD] == 0.0;
  r.mcc = -h[SL_MCC_NEG];
  r.cand_cost = h[SL_CAND_BAD] > 0.0 || !std::isfinite(h[SL_CCOST]) ? std::numeric_limits<double>::max() : h[SL_CCOST];
  r.step_norm = std::sqrt(h[SL_STEP2_P] + h[SL_STEP2_C]);
  r.ls_iters = ls_iters;
  r.spin = h[SL_CHOL_SPIN] != 0.0;
  return r;
}

void accept_candidate(ba_ctx* ctx) {
  std::swap(ctx->W.cams, ctx->W.cams_c);
  std::swap(ctx->W.pts, ctx->W.pts_c);
}

// Speculative linearisation at the last step's candidate, enqueued behind
// the step's scalar record: it runs while the host reads the record and
// decides, and it is the next iteration's linearisation when the step is
// accepted (the common case).  A rejected step re-linearises at x
// (ctx->lin_at_cand); the values are the same either way.  With collectives
// too: every rank enqueues the same linearisation (identical decisions), so
// the all-reduces keep one order across the ranks.  BA_SPEC_LIN=0: off
// (ba_ctx::read_env).
void spec_lin_enqueue(ba_ctx* ctx, const ba_options& o) {
  if (!ctx->spec_lin) return;
  // the kernels read W.cams / W.pts: point them at the candidate for the
  // enqueue only (restored on every exit, a throw included)
  struct Swap {
    ba_ctx* c;
    explicit Swap(ba_ctx* x) : c(x) { accept_candidate(c); }
    ~Swap() { accept_candidate(c); }
  } swap(ctx);
  linearize_enqueue(ctx, false, o.min_lm_diagonal, o.max_lm_diagonal, false, true);
  ctx->lin_at_cand = true;
}

void check_options(const ba_options& o) {
  if (o.linear_solver != BA_DENSE_SCHUR && o.linear_solver != BA_ITERATIVE_SCHUR)
    throw BaError{BA_ERR_INVALID_ARGUMENT, "unknown linear_solver " + std::to_string(o.linear_solver)};
  if (o.linear_solver == BA_ITERATIVE_SCHUR &&
      ((o.preconditioner_type != BA_JACOBI && o.preconditioner_type != BA_SCHUR_JACOBI) ||
       o.max_linear_solver_iterations < 1 || o.min_linear_solver_iterations < 0 || !(o.eta > 0.0)))
    throw BaError{BA_ERR_INVALID_ARGUMENT, "invalid ITERATIVE_SCHUR options"};
  if (o.precision != BA_FP64 && o.precision != BA_MIXED_FP32)
    throw BaError{BA_ERR_INVALID_ARGUMENT, "unknown precision " + std::to_string(o.precision)};
  if (o.precision == BA_MIXED_FP32 && o.linear_solver != BA_ITERATIVE_SCHUR)
    throw BaError{BA_ERR_INVALID_ARGUMENT, "BA_MIXED_FP32 requires BA_ITERATIVE_SCHUR"};
}

// ---------------------------------------------------------------------------
// ceres TrustRegionMinimizer (LM, monotonic) restated over the device phases
// ---------------------------------------------------------------------------
void solve(ba_ctx* ctx, const ba_options* opt, ba_summary* sum) {
  if (!ctx->have_problem) throw BaError{BA_ERR_NO_PROBLEM, "ba_solve before ba_set_problem"};
  ba_options o;
  if (opt) o = *opt; else ba_default_options(&o);
  check_options(o);
  ctx->read_env();
  const double t0 = now_s();
  ctx->log.clear();
  ctx->t_lin = ctx->t_solve = 0.0;
  ba_summary S{};
  auto push = [&](const ba_iteration& it) { ctx->log.push_back(it); };
  double radius = o.initial_trust_region_radius, decrease_factor = 2.0;
  int consecutive_invalid = 0;

  double tl = now_s();
  LinResult L = linearize(ctx, o.jacobi_scaling != 0, o.min_lm_diagonal, o.max_lm_diagonal);
  ctx->t_lin += now_s() - tl;
  if (!o.jacobi_scaling) {
    // scale = 1: write ones (kernels always read scale arrays)
    std::vector<double> ones(3 * (size_t)ctx->np, 1.0), onesc(6 * (size_t)ctx->nvc, 1.0);
    HIP_OK(hipMemcpy(ctx->W.scale_p, ones.data(), ones.size() * sizeof(double), hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(ctx->W.scale_c, onesc.data(), onesc.size() * sizeof(double), hipMemcpyHostToDevice));
    L = linearize(ctx, false, o.min_lm_diagonal, o.max_lm_diagonal);
  }
  S.initial_cost = L.cost;
  if (!L.ok) {
    S.final_cost = L.cost;
    S.termination_type = BA_FAILURE;
    S.total_time_s = now_s() - t0;
    if (sum) *sum = S;
    return;
  }
  {
    ba_iteration it{};
    it.iteration = 0; it.step_is_valid = 1; it.step_is_successful = 1;
    it.cost = L.cost; it.gradient_max_norm = L.gmax; it.gradient_norm = L.gnorm;
    it.trust_region_radius = radius;
    it.iteration_time_s = now_s() - t0;
    push(it);
  }
  double x_cost = L.cost, x_norm = L.xnorm, gmax = L.gmax, gnorm = L.gnorm;
  int iteration = 0;
  int termination = BA_NO_CONVERGENCE;
  bool last_success = true;
  auto can_continue = [&]() {
    if (iteration >= o.max_num_iterations) { termination = BA_NO_CONVERGENCE; return false; }
    if (last_success && gmax <= o.gradient_tolerance) { termination = BA_CONVERGENCE; return false; }
    if (radius <= o.min_trust_region_radius) { termination = BA_CONVERGENCE; return false; }
    return true;
  };
  // a step enqueued right behind the last accepted step's linearisation
  // (its record arrived with the linearisation's): used if the solve goes on
  bool have_step = false;
  ctx->clear_pending();   // (an earlier solve may have thrown between the two enqueues)
  int spec_ls = 0;
  while (can_continue()) {
    const double ti = now_s();
    ++iteration;
    ba_iteration it{};
    it.iteration = iteration;
    double ts = now_s();
    int ls = spec_ls;
    if (!have_step) {
      // (after a rejected or invalid step the speculative linearisation at
      // its candidate replaced the one at x)
      if (ctx->lin_at_cand) linearize_enqueue(ctx, false, o.min_lm_diagonal, o.max_lm_diagonal, false, true);
      ls = step_enqueue(ctx, radius, o);
      ctx->publish_scalars();
      spec_lin_enqueue(ctx, o);
      ctx->wait_scalars();
    }
    have_step = false;
    StepResult st = step_result(ctx, ls);
    if (st.spin) {
      // a hand-off of the persistent factorisation never came (its grid
      // could not be fully resident, e.g. beside another process's kernels):
      // not a pivot failure.  Redo the step with the per-step launches (and
      // keep them for this context).  A spin of the per-step form's back
      // substitution (k_back_flow) has no fallback: BA_ERR_DEVICE.  Under
      // collectives the spin slot is all-reduced with the step's scalars, so
      // every rank redoes (or throws) together.
      if (!ctx->W.chol_persist && !ctx->W.chol_fuse && !ctx->W.chol_flow)
        throw BaError{BA_ERR_DEVICE, "dense Cholesky: a hand-off spin bound was hit"};
      ctx->W.chol_persist = false;
      ctx->W.chol_flow = false;   // (the split form's one-launch dataflow: per-step launches instead,
      ctx->W.chol_fuse = false;   //  and their in-launch panels: k_chol_panel launches)
      if (ctx->lin_at_cand) linearize_enqueue(ctx, false, o.min_lm_diagonal, o.max_lm_diagonal, false, true);
      ls = step_enqueue(ctx, radius, o);
      ctx->read_scalars();
      st = step_result(ctx, ls);
      if (st.spin) throw BaError{BA_ERR_DEVICE, "dense Cholesky: a hand-off spin bound was hit"};
    }
    ctx->t_solve += now_s() - ts;
    it.linear_solver_iterations = st.ls_iters;
    const bool valid = st.linear_ok && st.mcc > 0.0;
    it.model_cost_change = st.mcc;
    if (!valid) {
      if (++consecutive_invalid >= o.max_num_consecutive_invalid_steps) { termination = BA_FAILURE; break; }
      radius = radius / decrease_factor;
      decrease_factor *= 2.0;
      it.cost = x_cost; it.gradient_max_norm = gmax; it.gradient_norm = gnorm;
      it.trust_region_radius = radius; it.step_is_valid = 0; it.step_is_successful = 0;
      last_success = false;
      S.num_unsuccessful_steps++;
      it.iteration_time_s = now_s() - ti;
      push(it);
      continue;
    }
    consecutive_invalid = 0;
    it.step_norm = st.step_norm;
    if (st.step_norm <= o.parameter_tolerance * (x_norm + o.parameter_tolerance)) { termination = BA_CONVERGENCE; break; }
    const double cost_change = x_cost - st.cand_cost;
    it.cost_change = cost_change;
    if (std::fabs(cost_change) <= o.function_tolerance * x_cost) { termination = BA_CONVERGENCE; break; }
    const double rel = st.cand_cost >= std::numeric_limits<double>::max() ? std::numeric_limits<double>::lowest()
                                                                          : (x_cost - st.cand_cost) / st.mcc;
    it.relative_decrease = rel;
    if (rel > o.min_relative_decrease) {
      accept_candidate(ctx);
      radius = std::min(o.max_trust_region_radius, radius / std::max(1.0 / 3.0, 1.0 - std::pow(2.0 * rel - 1.0, 3)));
      decrease_factor = 2.0;
      tl = now_s();
      // speculate: the next step at the new radius, unless the loop ends on
      // grounds already known (iteration cap, radius floor)
      const bool spec = iteration < o.max_num_iterations && radius > o.min_trust_region_radius;
      // the linearisation at the new x: already enqueued behind the step
      // (spec_lin_enqueue; its scalars are pending), else now
      if (!ctx->lin_at_cand) linearize_enqueue(ctx, false, o.min_lm_diagonal, o.max_lm_diagonal, false, spec);
      ctx->lin_at_cand = false;
      if (spec) {
        spec_ls = step_enqueue(ctx, radius, o);
      } else if (ctx->pend_sum | ctx->pend_max) {
        ctx->flush_norms();
        launch_reduce(ctx->W, ctx->pend_sum, ctx->pend_max, ctx->stream);
        ctx->pend_sum = ctx->pend_max = 0;
      }
      ctx->publish_scalars();
      if (spec) spec_lin_enqueue(ctx, o);
      ctx->wait_scalars();
      L = lin_result(ctx);
      have_step = spec;
      ctx->t_lin += now_s() - tl;
      if (!L.ok) { termination = BA_FAILURE; x_cost = L.cost; break; }
      x_cost = L.cost; x_norm = L.xnorm; gmax = L.gmax; gnorm = L.gnorm;
      last_success = true;
      S.num_successful_steps++;
      it.cost = x_cost; it.step_is_successful = 1;
    } else {
      radius = radius / decrease_factor;
      decrease_factor *= 2.0;
      last_success = false;
      S.num_unsuccessful_steps++;
      it.cost = st.cand_cost; it.step_is_successful = 0;
    }
    it.gradient_max_norm = gmax; it.gradient_norm = gnorm; it.trust_region_radius = radius; it.step_is_valid = 1;
    it.iteration_time_s = now_s() - ti;
    push(it);
  }
  S.final_cost = x_cost;
  S.termination_type = termination;
  S.num_iterations = iteration;
  S.total_time_s = now_s() - t0;
  S.linearize_time_s = ctx->t_lin;
  S.solve_time_s = ctx->t_solve;
  if (sum) *sum = S;
}

void get_params(ba_ctx* ctx, double* cams, double* pts) {
  if (!ctx->have_problem) throw BaError{BA_ERR_NO_PROBLEM, "no problem"};
  if (cams && ctx->nc) HIP_OK(hipMemcpy(cams, ctx->W.cams, 6 * sizeof(double) * ctx->nc, hipMemcpyDeviceToHost));
  if (pts && ctx->np) HIP_OK(hipMemcpy(pts, ctx->W.pts, 3 * sizeof(double) * ctx->np, hipMemcpyDeviceToHost));
}

}  // namespace

// ============================================================================
// extern "C" ABI
// ============================================================================
template <typename F>
static int guarded(ba_ctx* ctx, F&& f) {
  try {
    f();
    return BA_OK;
  } catch (const BaError& e) {
    if (ctx) ctx->err = e.msg;
    return e.code;
  } catch (const std::exception& e) {
    if (ctx) ctx->err = e.what();
    return BA_ERR_DEVICE;
  } catch (...) {
    if (ctx) ctx->err = "unknown error";
    return BA_ERR_DEVICE;
  }
}

extern "C" {

int ba_abi_version(void) { return BA_ABI_VERSION; }

// ba_default_options: host/ba_options.cpp (plain C++, shared with the sanitizer build)

int ba_create(ba_ctx** out, int device) {
  if (!out) return BA_ERR_INVALID_ARGUMENT;
  *out = nullptr;
  ba_ctx* ctx = new ba_ctx();
  try {
    int ndev = 0;
    HIP_OK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) throw BaError{BA_ERR_INVALID_ARGUMENT, "invalid device " + std::to_string(device)};
    ctx->device = device;
    HIP_OK(hipSetDevice(device));
    HIP_OK(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
    for (auto& e : ctx->ev) HIP_OK(hipEventCreate(&e));
    {
      const size_t rec = sizeof(double) * (kNumSlots + kPcgState);
      HIP_OK(hipHostMalloc(&ctx->h_scal, rec + 64, hipHostMallocMapped | hipHostMallocCoherent));
      std::memset(ctx->h_scal, 0, rec + 64);
      ctx->h_seq = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(ctx->h_scal) + rec);
      void* d = nullptr;
      HIP_OK(hipHostGetDevicePointer(&d, ctx->h_scal, 0));
      ctx->d_hscal = static_cast<double*>(d);
      ctx->d_hseq = reinterpret_cast<unsigned*>(static_cast<char*>(d) + rec);
      HIP_OK(hipMalloc(&ctx->d_ticket, 64));
      HIP_OK(hipMemset(ctx->d_ticket, 0, 64));
    }
  } catch (const BaError& e) {
    std::fprintf(stderr, "ba_create: %s\n", e.msg.c_str());
    delete ctx;
    return e.code;
  }
  *out = ctx;
  return BA_OK;
}

int ba_destroy(ba_ctx* ctx) {
  if (!ctx) return BA_OK;
  (void)hipSetDevice(ctx->device);
  ctx->free_problem();
  if (ctx->comm) ncclCommDestroy(ctx->comm);
  for (auto& e : ctx->ev) if (e) (void)hipEventDestroy(e);
  if (ctx->h_scal) (void)hipHostFree(ctx->h_scal);
  if (ctx->d_ticket) (void)hipFree(ctx->d_ticket);
  if (ctx->pose_buf) (void)hipFree(ctx->pose_buf);
  if (ctx->hv_scratch) (void)hipFree(ctx->hv_scratch);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return BA_OK;
}

const char* ba_last_error(const ba_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int ba_comm_unique_id(char id[128]) {
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  if (!id) return BA_ERR_INVALID_ARGUMENT;
  ncclUniqueId uid;
  if (ncclGetUniqueId(&uid) != ncclSuccess) return BA_ERR_COMM;
  std::memcpy(id, &uid, 128);
  return BA_OK;
}

int ba_comm_init(ba_ctx* ctx, const char id[128], int nranks, int rank) {
  if (!ctx || !id || nranks < 1 || rank < 0 || rank >= nranks) return BA_ERR_INVALID_ARGUMENT;
  return guarded(ctx, [&] {
    HIP_OK(hipSetDevice(ctx->device));
    if (ctx->comm) { ncclCommDestroy(ctx->comm); ctx->comm = nullptr; }
    ctx->host_fn = nullptr;
    ctx->nranks = nranks;
    ctx->rank = rank;
    ncclUniqueId uid;
    std::memcpy(&uid, id, 128);
    NCCL_OK(ncclCommInitRank(&ctx->comm, nranks, uid, rank));
    const char* fc = getenv("BA_FORCE_COLLECTIVES");
    ctx->force_coll = fc && atoi(fc) != 0;
  });
}

int ba_comm_allreduce_host(ba_ctx* ctx, double* values, int n, int op) {
  if (!ctx || n < 0 || (n > 0 && !values) || (op != 0 && op != 1)) return BA_ERR_INVALID_ARGUMENT;
  return guarded(ctx, [&] {
    if (!ctx->has_comm()) return;
    HIP_OK(hipSetDevice(ctx->device));
    double zero = 0.0;
    ctx->allreduce_host_values(n > 0 ? values : &zero, n > 0 ? (size_t)n : 1, op);   // n = 0: a barrier
  });
}

int ba_comm_init_host(ba_ctx* ctx, ba_host_allreduce_fn fn, void* user, int nranks, int rank) {
  if (!ctx || !fn || nranks < 1 || rank < 0 || rank >= nranks) return BA_ERR_INVALID_ARGUMENT;
  return guarded(ctx, [&] {
    if (ctx->comm) { ncclCommDestroy(ctx->comm); ctx->comm = nullptr; }
    ctx->host_fn = fn;
    ctx->host_user = user;
    ctx->nranks = nranks;
    ctx->rank = rank;
    const char* fc = getenv("BA_FORCE_COLLECTIVES");
    ctx->force_coll = fc && atoi(fc) != 0;
  });
}

int ba_set_problem(ba_ctx* ctx, const ba_problem* problem) {
  if (!ctx) return BA_ERR_INVALID_ARGUMENT;
  return guarded(ctx, [&] { set_problem(ctx, problem); });
}

int ba_set_params(ba_ctx* ctx, const double* cams, const double* pts) {
  if (!ctx) return BA_ERR_INVALID_ARGUMENT;
  return guarded(ctx, [&] {
    if (!ctx->have_problem) throw BaError{BA_ERR_NO_PROBLEM, "no problem"};
    if (cams && ctx->nc) HIP_OK(hipMemcpy(ctx->W.cams, cams, 6 * sizeof(double) * ctx->nc, hipMemcpyHostToDevice));
    if (pts && ctx->np) HIP_OK(hipMemcpy(ctx->W.pts, pts, 3 * sizeof(double) * ctx->np, hipMemcpyHostToDevice));
    // the Jacobi scaling belongs to the old parameters (ceres evaluates it at
    // the start of every solve): ba_bench_iterations must recompute it
    ctx->scale_valid = false;
  });
}

int ba_solve(ba_ctx* ctx, const ba_options* opt, ba_summary* summary) {
  if (!ctx) return BA_ERR_INVALID_ARGUMENT;
  return guarded(ctx, [&] { HIP_OK(hipSetDevice(ctx->device)); solve(ctx, opt, summary); });
}

int ba_get_params(ba_ctx* ctx, double* cams, double* pts) {
  if (!ctx) return BA_ERR_INVALID_ARGUMENT;
  return guarded(ctx, [&] { get_params(ctx, cams, pts); });
}

int ba_get_iteration_log(ba_ctx* ctx, ba_iteration* out, int n) {
  if (!ctx) return -BA_ERR_INVALID_ARGUMENT;
  const int avail = (int)ctx->log.size();
  if (out && n > 0) std::memcpy(out, ctx->log.data(), sizeof(ba_iteration) * std::min(n, avail));
  return avail;
}

int ba_eval_residuals(ba_ctx* ctx, double* r, double* cost) {
  if (!ctx) return BA_ERR_INVALID_ARGUMENT;
  return guarded(ctx, [&] {
    if (!ctx->have_problem) throw BaError{BA_ERR_NO_PROBLEM, "no problem"};
    HIP_OK(hipSetDevice(ctx->device));
    const int no = ctx->no;
    double* d_r = nullptr;
    HIP_OK(hipMalloc(&d_r, sizeof(double) * 2 * std::max(no, 1)));
    launch_cam_prep(ctx->P, ctx->W.cams, ctx->W.rec_c, false, ctx->stream);
    launch_residuals(ctx->P, ctx->W.rec_c, ctx->W.pts, d_r, ctx->stream);
    std::vector<double> rs(2 * (size_t)no);
    HIP_OK(hipMemcpyAsync(rs.data(), d_r, sizeof(double) * 2 * no, hipMemcpyDeviceToHost, ctx->stream));
    HIP_OK(hipStreamSynchronize(ctx->stream));
    (void)hipFree(d_r);
    double c = 0.0;
    const double a = ctx->huber_a, b = a * a;
    for (int s = 0; s < no; ++s) {
      const int o = ctx->perm[s];
      if (r) { r[2 * o] = rs[2 * s]; r[2 * o + 1] = rs[2 * s + 1]; }
      double sc;
      c += 0.5 * huber(rs[2 * s] * rs[2 * s] + rs[2 * s + 1] * rs[2 * s + 1], a, b, &sc);
    }
    if (cost) *cost = c;
  });
}

int ba_linearize(ba_ctx* ctx, double* r, double* J, double* cost) {
  if (!ctx) return BA_ERR_INVALID_ARGUMENT;
  return guarded(ctx, [&] {
    if (!ctx->have_problem) throw BaError{BA_ERR_NO_PROBLEM, "no problem"};
    HIP_OK(hipSetDevice(ctx->device));
    ba_options o;
    ba_default_options(&o);
    LinResult L = linearize(ctx, true, o.min_lm_diagonal, o.max_lm_diagonal);
    const int no = ctx->no;
    if (ctx->W.jrfree) {   // the iteration never stores J: write the records once for the read-back
      if (!ctx->W.JR) ctx->W.JR = ctx->dalloc<double>((size_t)(bahip::jr_ja_host(ctx->P.nc) + 8) * no);
      bahip::launch_linearize_jr(ctx->P, ctx->W, ctx->stream);
      // its cost partials are not this call's result (k_lin_point's were): fold
      // and clear them so no later reduction counts them
      launch_reduce(ctx->W, bit(SL_COST) | bit(SL_LIN_BAD), 0, ctx->stream);
      HIP_OK(hipStreamSynchronize(ctx->stream));
    }
    // record layout of ba_kernels.hip: JA [no][ja] (Jc rows; ja = 14: then r
    // again) then JB [no][8] (Jp rows, r)
    const int ja = bahip::jr_ja_host(ctx->P.nc);
    std::vector<double> rec((size_t)(ja + 8) * no);
    HIP_OK(hipMemcpy(rec.data(), ctx->W.JR, sizeof(double) * rec.size(), hipMemcpyDeviceToHost));
    for (int s = 0; s < no; ++s) {
      const int o2 = ctx->perm[s];
      const double* qa = &rec[(size_t)s * ja];
      const double* qb = &rec[(size_t)ja * no + (size_t)s * 8];
      // bit patterns, not values: a NaN residual (zero depth) is still a
      // faithful copy of itself
      if (ja >= 14 && (std::memcmp(&qa[12], &qb[6], 2 * sizeof(double)) != 0))
        throw BaError{BA_ERR_DEVICE, "JR: the two residual copies differ"};
      if (r) { r[2 * o2] = qb[6]; r[2 * o2 + 1] = qb[7]; }
      if (J)
        for (int row = 0; row < 2; ++row) {
          for (int k = 0; k < 6; ++k) J[(size_t)o2 * 18 + row * 9 + k] = qa[row * 6 + k];
          for (int k = 0; k < 3; ++k) J[(size_t)o2 * 18 + row * 9 + 6 + k] = qb[row * 3 + k];
        }
    }
    if (cost) *cost = L.cost;
  });
}

int ba_prune(ba_ctx* ctx, const ba_prune_problem* p, uint8_t* result) {
  if (!ctx) return BA_ERR_INVALID_ARGUMENT;
  return guarded(ctx, [&] {
    if (!p || p->n_cams < 0 || p->n_obs < 0) throw BaError{BA_ERR_INVALID_ARGUMENT, "ba_prune: bad sizes"};
    const int nc = p->n_cams, no = p->n_obs;
    if (no == 0) return;
    if (!p->extr || !p->cam_center || !p->K || !p->obs_cam || !p->obs_X || !p->obs_uv || !p->obs_inv_sigma ||
        !p->obs_dist || !result)
      throw BaError{BA_ERR_INVALID_ARGUMENT, "ba_prune: null array"};
    for (int o = 0; o < no; ++o)
      if (p->obs_cam[o] < 0 || p->obs_cam[o] >= nc)
        throw BaError{BA_ERR_INVALID_ARGUMENT, "ba_prune: obs_cam[" + std::to_string(o) + "] out of range"};
    HIP_OK(hipSetDevice(ctx->device));
    // one staging buffer: cameras (16 + 3 + 9 floats) then pairs (1 int + 3 + 2 + 1 + 2 floats + 1 byte)
    const size_t cam_b = sizeof(float) * 28 * (size_t)nc, obs_b = sizeof(float) * 9 * (size_t)no;
    const size_t bytes = cam_b + obs_b + sizeof(int) * (size_t)no + (size_t)no;
    char* d = nullptr;
    HIP_OK(hipMalloc(&d, bytes));
    std::vector<char> h(bytes - (size_t)no);
    size_t off = 0;
    auto put = [&](const void* src, size_t n) { std::memcpy(h.data() + off, src, n); off += n; };
    put(p->extr, sizeof(float) * 16 * nc);
    put(p->cam_center, sizeof(float) * 3 * nc);
    put(p->K, sizeof(float) * 9 * nc);
    put(p->obs_X, sizeof(float) * 3 * no);
    put(p->obs_uv, sizeof(float) * 2 * no);
    put(p->obs_inv_sigma, sizeof(float) * no);
    put(p->obs_dist, sizeof(float) * 2 * no);
    put(p->obs_cam, sizeof(int) * no);
    auto f = [&](size_t o) { return reinterpret_cast<const float*>(d + o); };
    const size_t oX = cam_b, oUV = oX + sizeof(float) * 3 * no, oS = oUV + sizeof(float) * 2 * no,
                 oD = oS + sizeof(float) * no, oC = oD + sizeof(float) * 2 * no, oR = oC + sizeof(int) * no;
    HIP_OK(hipMemcpyAsync(d, h.data(), h.size(), hipMemcpyHostToDevice, ctx->stream));
    launch_prune(no, f(0), f(sizeof(float) * 16 * nc), f(sizeof(float) * 19 * nc),
                 reinterpret_cast<const int*>(d + oC), f(oX), f(oUV), f(oS), f(oD),
                 reinterpret_cast<uint8_t*>(d + oR), ctx->stream);
    HIP_OK(hipGetLastError());
    HIP_OK(hipMemcpyAsync(result, d + oR, (size_t)no, hipMemcpyDeviceToHost, ctx->stream));
    HIP_OK(hipStreamSynchronize(ctx->stream));
    (void)hipFree(d);
  });
}

int ba_solve_pose_batch(ba_ctx* ctx, const ba_pose_batch* b, const ba_options* opt, double* cams_out,
                        ba_summary* summaries) {
  if (!ctx) return BA_ERR_INVALID_ARGUMENT;
  return guarded(ctx, [&] {
    if (!b || b->n_problems < 0) throw BaError{BA_ERR_INVALID_ARGUMENT, "ba_solve_pose_batch: bad batch"};
    const int n = b->n_problems;
    if (n == 0) return;
    if (!b->obs_offset || !b->cams || !b->K || !cams_out)
      throw BaError{BA_ERR_INVALID_ARGUMENT, "ba_solve_pose_batch: null array"};
    if (b->obs_offset[0] != 0) throw BaError{BA_ERR_INVALID_ARGUMENT, "ba_solve_pose_batch: obs_offset[0] != 0"};
    for (int i = 0; i < n; ++i)
      if (b->obs_offset[i + 1] < b->obs_offset[i])
        throw BaError{BA_ERR_INVALID_ARGUMENT, "ba_solve_pose_batch: obs_offset decreases at " + std::to_string(i)};
    const int no = b->obs_offset[n];
    if (no > 0 && (!b->pts || !b->obs_uv)) throw BaError{BA_ERR_INVALID_ARGUMENT, "ba_solve_pose_batch: null array"};
    ba_options o;
    if (opt) o = *opt; else ba_default_options(&o);
    PoseOpts po{o.max_num_iterations, o.max_num_consecutive_invalid_steps, o.jacobi_scaling,
                o.function_tolerance, o.gradient_tolerance, o.parameter_tolerance, o.initial_trust_region_radius,
                o.max_trust_region_radius, o.min_trust_region_radius, o.min_relative_decrease, o.min_lm_diagonal,
                o.max_lm_diagonal};
    const double t0 = now_s();
    HIP_OK(hipSetDevice(ctx->device));
    // one staging buffer, 16-B aligned sections: inputs (uploaded), then outputs
    auto al = [](size_t x) { return (x + 15) & ~size_t(15); };
    const size_t s_off = al(sizeof(int) * (n + 1)), s_cam = al(sizeof(double) * 6 * n), s_K = al(sizeof(float) * 9 * n),
                 s_X = al(sizeof(double) * 3 * (size_t)no), s_uv = al(sizeof(float) * 2 * (size_t)no);
    const size_t in_b = s_off + s_cam + s_K + s_X + s_uv;
    const size_t out_b = s_cam + al(sizeof(double) * 8 * n);
    if (in_b + out_b > ctx->pose_cap) {
      if (ctx->pose_buf) (void)hipFree(ctx->pose_buf);
      ctx->pose_buf = nullptr;
      ctx->pose_cap = 0;
      HIP_OK(hipMalloc(&ctx->pose_buf, in_b + out_b));
      ctx->pose_cap = in_b + out_b;
    }
    std::vector<char>& h = ctx->pose_host;
    h.assign(in_b + out_b, 0);
    size_t at = 0;
    auto put = [&](const void* src, size_t nb, size_t sec) { if (nb) std::memcpy(h.data() + at, src, nb); at += sec; };
    put(b->obs_offset, sizeof(int) * (n + 1), s_off);
    put(b->cams, sizeof(double) * 6 * n, s_cam);
    put(b->K, sizeof(float) * 9 * n, s_K);
    put(b->pts, sizeof(double) * 3 * (size_t)no, s_X);
    put(b->obs_uv, sizeof(float) * 2 * (size_t)no, s_uv);
    char* d = ctx->pose_buf;
    HIP_OK(hipMemcpyAsync(d, h.data(), in_b, hipMemcpyHostToDevice, ctx->stream));
    const int* d_off = reinterpret_cast<const int*>(d);
    const double* d_cam = reinterpret_cast<const double*>(d + s_off);
    const float* d_K = reinterpret_cast<const float*>(d + s_off + s_cam);
    const double* d_X = reinterpret_cast<const double*>(d + s_off + s_cam + s_K);
    const float2* d_uv = reinterpret_cast<const float2*>(d + s_off + s_cam + s_K + s_X);
    double* d_out = reinterpret_cast<double*>(d + in_b);
    double* d_sum = reinterpret_cast<double*>(d + in_b + s_cam);
    launch_pose_batch(n, d_off, d_cam, d_K, d_X, d_uv, b->huber_a, po, d_out, d_sum, ctx->stream);
    HIP_OK(hipGetLastError());
    HIP_OK(hipMemcpyAsync(h.data() + in_b, d + in_b, out_b, hipMemcpyDeviceToHost, ctx->stream));
    HIP_OK(hipStreamSynchronize(ctx->stream));
    std::memcpy(cams_out, h.data() + in_b, sizeof(double) * 6 * n);
    if (summaries) {
      const double* sm = reinterpret_cast<const double*>(h.data() + in_b + s_cam);
      const double wall = now_s() - t0;
      for (int i = 0; i < n; ++i) {
        ba_summary S{};
        S.initial_cost = sm[8 * i];
        S.final_cost = sm[8 * i + 1];
        S.num_iterations = (int)sm[8 * i + 2];
        S.num_successful_steps = (int)sm[8 * i + 3];
        S.num_unsuccessful_steps = (int)sm[8 * i + 4];
        S.termination_type = (int)sm[8 * i + 5];
        S.total_time_s = wall;
        summaries[i] = S;
      }
    }
  });
}

int ba_debug_blocks(ba_ctx* ctx, double radius, double* Hpp, double* gp, double* Hcc, double* gc, double* S,
                    double* rhs, int* n_out) {
  if (!ctx || !(radius > 0.0)) return BA_ERR_INVALID_ARGUMENT;
  return guarded(ctx, [&] {
    if (!ctx->have_problem) throw BaError{BA_ERR_NO_PROBLEM, "no problem"};
    HIP_OK(hipSetDevice(ctx->device));
    ba_options o;
    ba_default_options(&o);   // DENSE_SCHUR, fp64
    ctx->read_env();
    // iteration 0's linearisation (Jacobi scaling from it), then the step's
    // reduced system without its factorisation
    const LinResult L = linearize(ctx, true, o.min_lm_diagonal, o.max_lm_diagonal);
    if (!L.ok) throw BaError{BA_ERR_DEVICE, "linearisation not finite"};
    step_w_storage(ctx, o);
    // BA_DEBUG_OV_PASS=1: S from the overlapped form's work items (a launch
    // that only forms S), else from the separate pair / diagonal / fold passes
    const char* dv = getenv("BA_DEBUG_OV_PASS");
    const bool want_ov = dv && dv[0] == '1';
    if (form_reduced_dense(ctx, radius, want_ov))
      launch_cholesky_solve_ov(ctx->P, ctx->W, ctx->W.ov, radius, ++ctx->chol_epoch, ctx->stream, true);
    else if (want_ov)
      throw BaError{BA_ERR_INVALID_ARGUMENT, "BA_DEBUG_OV_PASS: the overlapped form does not apply to this problem"};
    const hipStream_t st = ctx->stream;
    const int np = ctx->np, nc = ctx->nc, nvc = ctx->nvc, n = ctx->n;
    HIP_OK(hipStreamSynchronize(st));
    if (Hpp || gp) {
      std::vector<double> h(6 * (size_t)np), g(3 * (size_t)np);
      HIP_OK(hipMemcpy(h.data(), ctx->W.Hpp, h.size() * sizeof(double), hipMemcpyDeviceToHost));
      HIP_OK(hipMemcpy(g.data(), ctx->W.gp, g.size() * sizeof(double), hipMemcpyDeviceToHost));
      for (int p = 0; p < np; ++p) {   // (SoA [k][np] on the device; fixed points: not written)
        const bool v = ctx->h_pt_var[p] != 0;
        for (int k = 0; k < 6; ++k) if (Hpp) Hpp[6 * (size_t)p + k] = v ? h[(size_t)k * np + p] : 0.0;
        for (int k = 0; k < 3; ++k) if (gp) gp[3 * (size_t)p + k] = v ? g[(size_t)k * np + p] : 0.0;
      }
    }
    if (Hcc || gc) {
      std::vector<double> h(27 * (size_t)std::max(nvc, 1));
      if (nvc) HIP_OK(hipMemcpy(h.data(), ctx->W.Hcc, 27 * (size_t)nvc * sizeof(double), hipMemcpyDeviceToHost));
      if (Hcc) std::fill(Hcc, Hcc + 21 * (size_t)nc, 0.0);
      if (gc) std::fill(gc, gc + 6 * (size_t)nc, 0.0);
      for (int v = 0; v < nvc; ++v) {
        const int c = ctx->cam_of_vc[v];
        for (int k = 0; k < 21; ++k) if (Hcc) Hcc[21 * (size_t)c + k] = h[21 * (size_t)v + k];
        for (int k = 0; k < 6; ++k) if (gc) gc[6 * (size_t)c + k] = h[21 * (size_t)nvc + 6 * (size_t)v + k];
      }
    }
    if (S || rhs) {
      std::vector<double> m((size_t)(n + 1) * std::max(ctx->ld, 1));
      if (n) HIP_OK(hipMemcpy(m.data(), ctx->W.S, m.size() * sizeof(double), hipMemcpyDeviceToHost));
      for (int i = 0; i < n; ++i) {
        if (S) for (int j = 0; j < n; ++j) S[(size_t)i * n + j] = j <= i ? m[(size_t)i * ctx->ld + j] : 0.0;
        if (rhs) rhs[i] = m[(size_t)n * ctx->ld + i];
      }
    }
    if (n_out) *n_out = n;
  });
}

int ba_synchronize(ba_ctx* ctx) {
  if (!ctx) return BA_ERR_INVALID_ARGUMENT;
  return guarded(ctx, [&] { HIP_OK(hipStreamSynchronize(ctx->stream)); });
}

int ba_bench_iteration_times(ba_ctx* ctx, double* ms, int n) {
  if (!ctx) return BA_ERR_INVALID_ARGUMENT;
  const int m = (int)ctx->bench_ms.size();
  for (int i = 0; i < std::min(n, m) && ms; ++i) ms[i] = ctx->bench_ms[i];
  return m;
}

int ba_stream_copy(ba_ctx* ctx, size_t bytes, int reps, double* gbs) {
  if (!ctx || reps < 1 || bytes < 16 || !gbs) return BA_ERR_INVALID_ARGUMENT;
  return guarded(ctx, [&] {
    HIP_OK(hipSetDevice(ctx->device));
    const size_t n2 = bytes / 16;
    double *a = nullptr, *b = nullptr;
    HIP_OK(hipMalloc(&a, n2 * 16));
    if (hipMalloc(&b, n2 * 16) != hipSuccess) {
      (void)hipFree(a);
      throw BaError{BA_ERR_OUT_OF_MEMORY, "ba_stream_copy: hipMalloc"};
    }
    struct Free {
      double *a, *b;
      ~Free() { (void)hipFree(a); (void)hipFree(b); }
    } fr{a, b};
    HIP_OK(hipMemsetAsync(a, 0, n2 * 16, ctx->stream));
    bahip::launch_stream_copy(a, b, n2, ctx->stream);   // warm-up
    HIP_OK(hipGetLastError());
    HIP_OK(hipEventRecord(ctx->ev[0], ctx->stream));
    for (int r = 0; r < reps; ++r) bahip::launch_stream_copy(a, b, n2, ctx->stream);
    HIP_OK(hipEventRecord(ctx->ev[1], ctx->stream));
    HIP_OK(hipEventSynchronize(ctx->ev[1]));
    float ms = 0.0f;
    HIP_OK(hipEventElapsedTime(&ms, ctx->ev[0], ctx->ev[1]));
    *gbs = 2.0 * 16.0 * (double)n2 * reps / ((double)ms * 1e-3) / 1e9;
  });
}

int ba_bench_iterations(ba_ctx* ctx, const ba_options* opt, int iters, double radius, double* ms_per_iter,
                        double* ms_rj_kernel, double* linear_iters) {
  if (!ctx || iters < 1) return BA_ERR_INVALID_ARGUMENT;
  return guarded(ctx, [&] {
    if (!ctx->have_problem) throw BaError{BA_ERR_NO_PROBLEM, "no problem"};
    HIP_OK(hipSetDevice(ctx->device));
    ba_options o;
    if (opt) o = *opt; else ba_default_options(&o);
    check_options(o);
    ctx->clear_pending();
    if (!ctx->scale_valid) linearize(ctx, true, o.min_lm_diagonal, o.max_lm_diagonal);
    double rj_total = 0.0;
    long ls_total = 0;
    ctx->read_env();
    const bool spec = ctx->spec_lin;
    const bool trj = ms_rj_kernel != nullptr;   // event pair around the r+J kernel
    HIP_OK(hipEventRecord(ctx->ev[0], ctx->stream));
    ctx->rj_slot = 0;
    ctx->bench_ms.assign(iters, 0.0);
    double th = now_s();
    if (spec) linearize_enqueue(ctx, false, o.min_lm_diagonal, o.max_lm_diagonal, trj, true);
    for (int i = 0; i < iters; ++i) {
      // the solver's steady state after an accepted step: the step, its
      // scalar record, and the next linearisation (spec_lin_enqueue) behind
      // it while the host reads the record; K linearisations and K steps
      // (BA_SPEC_LIN=0: linearisation + step, then the read)
      const int slot = ctx->rj_slot;
      if (!spec) linearize_enqueue(ctx, false, o.min_lm_diagonal, o.max_lm_diagonal, trj, true);
      const int ls = step_enqueue(ctx, radius, o);
      ctx->publish_scalars();
      if (spec && i + 1 < iters) {
        ctx->rj_slot ^= 1;
        linearize_enqueue(ctx, false, o.min_lm_diagonal, o.max_lm_diagonal, trj, true);
      }
      ctx->wait_scalars();
      if (ctx->h_scal[SL_CHOL_SPIN] != 0.0) throw BaError{BA_ERR_DEVICE, "dense Cholesky: a hand-off spin bound was hit"};
      {   // (the iteration's record has arrived: its host wall time)
        const double t = now_s();
        ctx->bench_ms[i] = (t - th) * 1e3;
        th = t;
      }
      const StepResult st = step_result(ctx, ls);
      if (trj) {
        float rj = 0.0f;
        HIP_OK(hipEventSynchronize(ctx->ev[3 + 2 * slot]));
        HIP_OK(hipEventElapsedTime(&rj, ctx->ev[2 + 2 * slot], ctx->ev[3 + 2 * slot]));
        rj_total += rj;
      }
      ls_total += st.ls_iters;
    }
    HIP_OK(hipEventRecord(ctx->ev[1], ctx->stream));
    HIP_OK(hipEventSynchronize(ctx->ev[1]));
    float total = 0.0f;
    HIP_OK(hipEventElapsedTime(&total, ctx->ev[0], ctx->ev[1]));
    if (ms_per_iter) *ms_per_iter = total / iters;
    if (ms_rj_kernel) *ms_rj_kernel = rj_total / iters;
    if (linear_iters) *linear_iters = (double)ls_total / iters;
  });
}

}  // extern "C"

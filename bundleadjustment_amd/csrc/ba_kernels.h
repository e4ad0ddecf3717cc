// ba_kernels.h — launch interface of the CDNA4 (gfx950) kernels of one LM
// iteration.  See DESIGN.md §3 for the data layout and the per-kernel
// roofline.  All arrays live in HBM, observations sorted by (point, camera).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

namespace bahip {

constexpr int kThreads = 256;
constexpr int kMaxBlocks = 2048;        // grid cap of the streaming kernels
constexpr int kCamSplit = 8;            // workgroups per camera in k_cam_schur_diag

// Scalar reduction slots (device buffer d_scal[kNumSlots]).
enum Slot {
  SL_COST = 0,      // robustified cost at x (linearisation)
  SL_LIN_BAD,       // non-finite residual / jacobian count
  SL_GN2_P,         // sum (x - (x - g))^2 over point params
  SL_XN2_P,         // sum x^2 over active point params
  SL_GMAX_P,        // max |x - (x - g)| over point params
  // (COST..XN2_P are contiguous and follow Hcc, gc in memory: one sum
  // all-reduce carries all of them across ranks)
  SL_MCC_NEG,       // sum (J d)^T (r + J d / 2)  (model_cost_change = -this)
  SL_CCOST,         // robustified cost at the candidate point
  SL_STEP2_P,       // sum (x - x')^2 over point params
  SL_CAND_BAD,      // non-finite candidate residual count
  SL_STEP_BAD,      // non-finite step component count (linear solver failure)
  SL_CHOL_SPIN,     // a hand-off spin bound of the dataflow Cholesky / back substitution was hit (not a pivot failure)
  // (MCC_NEG..CHOL_SPIN are contiguous: one all-reduce per step under
  // collectives, so every rank sees every rank's spin and they decide alike)
  SL_ELIM_BAD,      // failed 3x3 point-block Cholesky count
  SL_GMAX_C, SL_GN2_C, SL_XN2_C, SL_STEP2_C,
  SL_CHOL_BAD,      // non-positive pivot in the reduced camera system
  kNumSlots
};

struct DevProblem {
  int nc, np, no, nvc;       // cameras, points, observations, active variable cameras
  int n;                     // reduced system order 6*nvc
  int ld;                    // leading dimension of the dense reduced matrix
  double huber_a, huber_b;
  const int* obs_cam;        // [no]  sorted by (point, camera)
  const int* obs_pt;         // [no]
  const float2* uv;          // [no]
  const int* pt_off;         // [np+1] CSR of observations by point
  const int* cam_off;        // [nvc+1] CSR of observations by active variable camera
  const int2* cam_op;        // [..] (sorted observation, its point) grouped by camera
  const float2* uv_cm;       // [..] the pixel of each cam_op entry (camera-major copy of uv: streamed, not gathered)
  const int* vc;             // [nc] compact variable-camera index or -1
  const int* obs_vc;         // [no] vc of each observation's camera (one load instead of two dependent ones)
  const int* cam_of_vc;      // [nvc] camera id of a compact index
  const uint8_t* cam_fixed;  // [nc]
  const uint8_t* pt_var;     // [np] 1 = variable point with >=1 residual
  const float* K;            // [9*nc]
  const float* extr;         // [16*nc] (fixed cameras)
};

// The reduced system formed inside the persistent factorisation's launch
// (ba_chol_persist.hip, OvArgs): per-XCD queues of wave-sized work items in
// tile-column order, per-tile contribution counts, cumulative counters.
// Built once per problem (ba_solver.hip ensure_overlap).
struct OvPlan {
  bool ok = false;                   // built, and the problem qualifies
  const int4* irec = nullptr;        // [items][4]: a pair item's 4 blocks {I, J, start, end} (zeros: none),
                                     //   or {-1 - (v G + g), 0, 0, 0} first: a diagonal slice
  const int* item_col = nullptr;     // tile column of each item
  const unsigned* tgt = nullptr;     // [TR][T] contributions per tile and launch
  unsigned* ctr = nullptr;           // cnt [TR][T] | cam_cnt [nvc] | q [8] | pflag [TR][T]: zeroed once, cumulative
  int ioff[9] = {0};                 // queue x: items [ioff[x], ioff[x+1])
  int grid = 0;                      // workgroups of the launch (every CU: critical + workers + helpers)
  unsigned launches = 0;             // overlapped launches so far (pe of the next one - 1)
};

// Device workspace pointers (see ba_solver.hip for sizes).
struct DevWork {
  double* cams;  double* pts;        // x
  double* cams_c; double* pts_c;     // candidate x'
  double* rec;   double* rec_c;      // camera records at x / x'
  double* crec;                      // [nc][16] compact camera records (w, t, K, flag, theta terms) for > kLinLdsCams cameras
  double* ctbl;                      // [nc][22] candidate camera table for > kLinLdsCams cameras
  bool jrfree;                       // J-free iteration: consumers recompute J, JR unused (camera table in LDS up to kLinLdsCams cameras, crec beyond)
  double* JR;                        // JA [no][JA] (Jc rows 0..1; JA = 14 beyond kLinLdsCams cameras: + r again), then JB [no][8] (Jp rows 3+3, r 2)
  double* delta_p;                   // [np][3] point step (scaled back)
  double* Hpp;   double* gp;         // [6][np], [3][np]
  double* scale_p; double* diag_p;   // [3][np]
  double* Linv;  double* u;          // [6][np], [np][4] (AoS, last entry 0)
  double* Hcc;   double* gc;         // [nvc][21], [nvc][6]
  double* scale_c; double* diag_c;   // [nvc][6]
  double* delta_c;                   // [nvc][6]
  double* W;                         // [no][18]  (E L^-T per observation), fp64
  double* prec;                      // [np][16] point record of the J-free diagonal blocks: X (3), var flag, s_p (3), L_p^-1 (6), u_p
  double* pxv;                       // [np][4] the linearisation point {X, var flag} (k_lin_point; camera-major gathers)
  bool jdiag;                        // the diagonal Schur blocks J-free (k_cam_schur_diag_rc: prec gathered, W not read)
  float* Wf;                         // [no][18]  the same in fp32 (BA_MIXED_FP32)
  bool w32;                          // W blocks stored in Wf
  bool wcompact;                     // W as 128-B compact records (J-free fp64 DENSE_SCHUR; ba_kernels.hip)
  double* S;                         // [(n+1) x ld] reduced system, row n = rhs (working matrix)
  double* Lf;                        // [(n+1) x ld] Cholesky factor, row n = L^-1 rhs
  double* Ubuf;                      // [(n+1) x ld] the per-step Cholesky's update accumulator (< kCholSplitBlocks block columns)
  double* Spk;                       // [n(n+1)/2 + n] packed lower triangle + rhs of S (multi-rank exchange)
  double* y;                         // [n] reduced solution
  double* Vbuf;                      // [ceil(n/64)][64][64] inverses of the diagonal Cholesky blocks
  const int4* ctask;                 // split Cholesky task table {I, J, pa, pb} (>= kCholSplitBlocks block columns; null: rank-64 form)
  const int* ctask_off;              // host: step k's tasks [ctask_off[k], ctask_off[k+1])
  bool chol_fuse;                    // split form: column tasks form the next panel in-launch (flags: cflags[0, T))
  bool chol_flow;                    // split form: the whole factorisation as one dataflow launch (k_chol_flow)
  const int4* ftask; int nftask;     // ... its task list
  unsigned* tflag;                   // ... [TR][T] tile tags, [TR][T] panel flags (epoch-tagged, zeroed once)
  double* yg;                        // [n][2] back-substitution hand-off granules {y, epoch} (zeroed once)
  unsigned* cflags;                  // [T + TR*T] persistent-Cholesky hand-off flags (epoch-tagged, zeroed once)
  bool chol_persist;                 // the factorisation runs as one persistent launch (ba_chol_persist.hip)
  OvPlan ov;                         // ... with S formed in the same launch (the overlapped form)
  const int4* blocks; int nblocks;   // off-diagonal Schur blocks {I, J, start, end}, camera rows interleaved over the XCDs
  const int* xoff;                   // [9] k_schur_pairs* block range of XCD x: [xoff[x], xoff[x+1])
  int xmax;                          // largest XCD range
  const int2* eblocks; int neblocks; // lower off-diagonal blocks {I, J} with no observation pair
  bool s_memset;                     // many empty blocks: memset S instead
  const int2* pairs;                 // observation pairs per block
  double* cpart;                     // [cam_split][nvc][27] per-slice camera sums
  int cam_split;                     // workgroups per camera of the per-camera gathers (>= 2048 in total, <= kCamSplit)
  double* part;                      // [kNumSlots][kMaxBlocks]
  double* scal;                      // [kNumSlots + kPcgState]: scalar slots, then the PCG state record
  // ITERATIVE_SCHUR (allocated on first use; x of the CG is y above)
  double* Sd;                        // [nvc][27] diagonal Schur blocks (lower 21) + reduced rhs (6)
  double* Adiag;                     // [nvc][21] s Hcc s + D^2 (lower)
  double* Minv;                      // [nvc][36] preconditioner block inverses
  double* pb; double* pr; double* pz; double* pp; double* pq;   // [n] CG vectors
  double* vpt;                       // [np][3] point-side products of one implicit matvec
  double* vacc;                      // [np][3] sum over the CG iterations of alpha_k vpt(p_k) = vpt(y): the
                                     // back substitution's E^T dc term without J (W.pacc; k_pcg_vacc)
  bool pacc = false;
  bool mcc_cam = true;               // this rank adds the camera terms of the block-form model cost change (rank 0)
  double* tobs;                      // [no][6] per-observation products W_o v_p (null: gather W in the camera pass)
  double* tpart;                     // [pcg_G][nvc][6] camera-side slices of one implicit matvec
  double* ppart;                     // [3][kMaxBlocks] per-block partials of the camera-side kernels
  int pcg_G;
  const int2* pchunks;               // point-aligned observation chunks of <= 64 {start, end} (the PCG point pass)
  // ITERATIVE_SCHUR point-pass records in the 16-value rank-2 form
  // (k_obs_w_rc<.., PC>, k_pcg_point_seg<.., PC>; step_w_storage decides)
  bool pcgc = false;
  // the PCG point pass forms the rank-2 records itself from the compact camera
  // records (k_pcg_point_jf): no W written or read (step_w_storage decides)
  bool pcgjf = false;
  int npchunks;                      // 0: a point has more than 64 observations (value-pair point pass)
  bool pcg_folded;                   // exchange path: slices folded into slice 0 before the all-reduce
  const int* dup_off;                // [nvc+1] per variable camera: pairs of observations of one
  const int2* dup_pairs;             //   point by that camera (Schur-Jacobi diagonal cross terms)
};

// PCG state record at scal + kNumSlots (doubles)
// (PS_RHO1 / PS_Q01: the odd-iteration copies of rho and Q0 of the grid
// kernels, whose lead block must not overwrite a value the other blocks of
// the same launch still read)
// PS_AAPP / PS_AAPP_IT: the step length of the last CG iteration that moved x,
// and that iteration (k_pcg_vacc folds it into the points' accumulated
// products)
enum PcgState { PS_RHO = 0, PS_Q0, PS_ALPHA, PS_NORM_B, PS_ITER, PS_DONE, PS_TERM, PS_RHO1, PS_Q01, PS_AAPP, PS_AAPP_IT,
                kPcgState };
enum PcgTerm { PCG_SUCCESS = 0, PCG_NO_CONVERGENCE = 1, PCG_FAILURE = 2 };
struct PcgOpts { double q_tolerance; int min_iter, max_iter, schur_jacobi; };

// --- launchers (all asynchronous on `s`) ---
void launch_cam_prep(const DevProblem& P, const double* cams, double* rec, bool deriv, hipStream_t s);
void launch_lin_prep(const DevProblem& P, const DevWork& W, hipStream_t s);   // camera tables for launch_linearize
// t0 / t1: optional events stamped at the start / end of the kernel's execution
void launch_linearize(const DevProblem& P, const DevWork& W, hipStream_t s, hipEvent_t t0 = nullptr,
                      hipEvent_t t1 = nullptr);
void launch_point_assemble(const DevProblem& P, const DevWork& W, bool compute_scale, double min_diag,
                           double max_diag, hipStream_t s, hipEvent_t t0 = nullptr, hipEvent_t t1 = nullptr);
// the JR-writing linearisation (launch_linearize in JR mode; ba_linearize's read-back in J-free mode)
void launch_linearize_jr(const DevProblem& P, const DevWork& W, hipStream_t s, hipEvent_t t0 = nullptr,
                         hipEvent_t t1 = nullptr);
void launch_cam_assemble(const DevProblem& P, const DevWork& W, hipStream_t s);
void launch_cam_norms(const DevProblem& P, const DevWork& W, bool compute_scale, double min_diag, double max_diag,
                      hipStream_t s);
// the camera-side norms pass (k_cam_norms) as extra workgroups of another launch
struct NormsFold {
  const double* cams;
  const double* Hcc;
  const double* gc;
  double* scale_c;
  double* diag_c;
  int compute_scale;
  double min_diag, max_diag;
};
NormsFold norms_fold(const DevWork& W, bool compute_scale, double min_diag, double max_diag);
// + W = E L^-T; nf: k_cam_norms rides in the point elimination's launch
void launch_point_elim(const DevProblem& P, const DevWork& W, double radius, hipStream_t s,
                       const NormsFold* nf = nullptr);
// compact != nullptr: write the diagonal blocks + rhs to compact[nvc][27]
// instead of the dense S (ITERATIVE_SCHUR); radius > 0 (dense, single
// rank): add s Hcc s + D^2 and s g_c in the same pass (no launch_cam_add_diag)
void launch_cam_schur_diag(const DevProblem& P, const DevWork& W, hipStream_t s, double* compact = nullptr,
                           double radius = 0.0, bool skip_fold = false);
void launch_schur_pairs(const DevProblem& P, const DevWork& W, hipStream_t s, double fold_radius = 0.0,
                        bool with_diag = false);
bool pairs_take_fold(const DevProblem& P, const DevWork& W);
bool pairs_take_diag(const DevProblem& P, const DevWork& W);
bool pairs_take_diag_nt(const DevProblem& P, const DevWork& W);   // ... beyond the LDS camera table
void launch_cam_fold_diag(const DevProblem& P, const DevWork& W, double radius, hipStream_t s);
void launch_cam_add_diag(const DevProblem& P, const DevWork& W, double radius, hipStream_t s);
// ba_chol.hip; epoch: per-context launch counter (>= 1) tagging the
// back substitution's hand-off flags
void launch_cholesky_solve2(const DevProblem& P, const DevWork& W, int epoch, hipStream_t s);
// zero the lower Schur blocks no observation pair writes (the Cholesky
// leaves its updates there)
void launch_zero_blocks(const DevProblem& P, const DevWork& W, hipStream_t s);
// S <-> W.Spk: lower triangle row by row (offset i(i+1)/2), then the rhs row
void launch_pack_lower(const DevProblem& P, const DevWork& W, bool pack, hipStream_t s);
void launch_cam_candidate(const DevProblem& P, const DevWork& W, hipStream_t s);
void launch_backsub_candidate(const DevProblem& P, const DevWork& W, hipStream_t s);
// ITERATIVE_SCHUR (ba_pcg.hip): implicit Schur complement + PCG
void launch_pcg_setup(const DevProblem& P, const DevWork& W, double radius, const PcgOpts& o, hipStream_t s);
void launch_pcg_dup(const DevProblem& P, const DevWork& W, hipStream_t s);   // Schur-Jacobi cross terms
// one implicit matvec (point pass + camera pass) of vec into W.tpart
void launch_pcg_matvec(const DevProblem& P, const DevWork& W, const double* vec, hipStream_t s);
// the J-free point pass of one implicit matvec (W.pcgjf): v_p into W.vpt, t_o into W.tobs
void launch_pcg_point_jf(const DevProblem& P, const DevWork& W, const double* vec, hipStream_t s);
// W.pacc: after a CG update (set = false) W.vacc += alpha vpt when iteration
// `it` moved x (W.vacc = alpha vpt at it = 1); after the residual reset's
// matvec of y (set = true) W.vacc = vpt
void launch_pcg_vacc(const DevProblem& P, const DevWork& W, int it, bool set, hipStream_t s);
// exchange path: fold the matvec's camera slices into slice 0 (one 6 nvc all-reduce)
void launch_pcg_tfold(const DevProblem& P, const DevWork& W, hipStream_t s);
// mode 0: full CG iteration; 1: up to the x update; 2: residual reset from W.tpart = matvec(x)
void launch_pcg_update(const DevProblem& P, const DevWork& W, int mode, int it, const PcgOpts& o, hipStream_t s);

// Fold the partials of `slots` (bitmask) into d_scal; kernels producing
// partials always use grid = nblocks_of(...)
void launch_reduce(const DevWork& W, uint32_t sum_mask, uint32_t max_mask, hipStream_t s);
// the same, then (last workgroup) the scalar record to the host as launch_publish_scalars
void launch_reduce_publish(const DevWork& W, uint32_t sum_mask, uint32_t max_mask, double* host, int n,
                           unsigned* host_seq, unsigned seq, unsigned* ticket, hipStream_t s);
int back_flow_capacity(int device);
int chol_persist_capacity(int device);   // resident k_chol_persist workgroups (occupancy x CUs; -1: query failed)
// the persistent factorisation with S formed in the same launch (W.S holds
// nothing on entry): pairs, diagonal slices and fold of this step at radius
// (pass_only, diagnostics: S formed by that launch's work items, nothing factored)
void launch_cholesky_solve_ov(const DevProblem& P, const DevWork& W, OvPlan& plan, double radius, int epoch,
                              hipStream_t s, bool pass_only = false);
bool obs_w_pc_ok(const DevProblem& P, const DevWork& W);   // k_obs_w_rc has the PCG record form for this source
bool chol_persist_fits(int device, int n);   // every workgroup of k_chol_persist resident at once
void chol_split_tasks(int n, std::vector<int4>& tasks, std::vector<int>& off);   // the split form's task table
int chol_split_rank();
int chol_split_fused();                      // BA_CHOL_FUSE (default 1)
int chol_split_flow();                       // BA_CHOL_FLOW (default 1)
void chol_flow_tasks(const std::vector<int4>& tasks, const std::vector<int>& off, std::vector<int4>& flow);                       // panels per split-Cholesky task (BA_CHOL_RANK, default 4; 0: rank-64 form)
int chol_split_blocks();                     // block columns from which the split step form is used   // resident k_back_flow workgroups (-1: query failed)
constexpr int kLinLdsCamsHost = 200;   // = kLinLdsCams (ba_kernels.hip): cameras the LDS camera table holds
constexpr int kWcCamsHost = 1024;      // variable cameras of the compact-W DENSE_SCHUR pair pass
int jr_ja_host(int nc);   // JA stride of the JR records for nc cameras (12 or 14)
void launch_stream_copy(const double* a, double* b, size_t n2, hipStream_t s);
// the scalar record into pinned host memory, then its sequence number
// (system-scope release): ba_solver.hip read_scalars
void launch_publish_scalars(const double* scal, double* host, int n, unsigned* host_seq, unsigned seq, hipStream_t s);
void launch_residuals(const DevProblem& P, const double* rec, const double* pts, double* r_raw, hipStream_t s);

// pruneCorrespondences per (keyframe, keypoint) pair (ba_prune.hip)
void launch_prune(int n, const float* extr, const float* center, const float* K, const int* obs_cam, const float* X,
                  const float* uv, const float* inv_sigma, const float* dist, uint8_t* out, hipStream_t s);

// batched pose-only LM, one wavefront per problem (ba_kernels.hip)
struct PoseOpts {
  int max_iter, max_invalid, jacobi;
  double ftol, gtol, ptol, r0, rmax, rmin, min_rel, min_diag, max_diag;
};
void launch_pose_batch(int nprob, const int* off, const double* cams_in, const float* K, const double* X,
                       const float2* uv, double huber_a, const PoseOpts& o, double* cams_out, double* summ,
                       hipStream_t s);

int grid_for(int n);
int pt_group_grid(int np);   // grid of the kPtLanes-lanes-per-point kernels

}  // namespace bahip

/*
 * ba_hip.h — C-ABI of libba_hip.so, the MI355X-native replacement for the
 * reference's Ceres Problem/Solve bundle-adjustment path.
 *
 * Reference seam being replaced (MatteoWohlrapp/BundleAdjustment,
 * ba_project/src/ba):
 *   ceres::Problem problem;                                 Optimizer.cpp:229
 *   problem.AddResidualBlock(cost, HuberLoss(sqrt(5.991)),  Optimizer.cpp:312-329
 *                            cam6*, pt3*)                   (also :486-490, :645-691)
 *   configureSolver(options)  -> LM, DENSE_SCHUR, ...       Optimizer.cpp:80-90
 *   ceres::Solve(options, &problem, &summary)               Optimizer.cpp:242, 442, 570
 *
 * Conventions (match the reference's parameter layout, Optimizer.h:54-76):
 *   camera block  double[6] = [wx, wy, wz, tx, ty, tz]: world->camera,
 *                 angle-axis + translation, additive update (no manifold).
 *   point block   double[3] world position.
 *   K             float[9]  column-major 3x3 (Eigen Matrix3f storage).
 *   fixed camera  float[16] column-major 4x4 world->camera extrinsic, used
 *                 exactly like PointOnlyReprojectionError (Optimizer.h:96-107).
 *   observation   (camera index, point index, float2 pixel).
 *   Residual kind per observation (chosen like prepareConstraints,
 *   Optimizer.cpp:306-329 / 472-490 / 668-691):
 *     camera variable, point variable -> AngleReprojectionError      (2x[6,3])
 *     camera fixed,    point variable -> PointOnlyReprojectionError  (2x[3])
 *     camera variable, point fixed    -> PoseOnlyAngleReprojectionError (2x[6])
 *     both fixed                      -> constant block (cost only)
 *   Each residual carries ceres::HuberLoss(huber_a) (huber_a <= 0: no loss).
 *
 * Error behaviour: no exceptions cross the ABI.  Every call returns a status
 * (BA_OK == 0); ba_last_error(ctx) describes the last failure.  Solver
 * non-convergence is NOT an error: it is reported in ba_summary exactly like
 * ceres::Solver::Summary::termination_type (which the reference ignores).
 *
 * Threading: a ba_ctx is not thread-safe; use one context per calling thread.
 * All calls block until their results are on the host.
 */
#ifndef BA_HIP_H_
#define BA_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BA_ABI_VERSION 2

enum ba_status {
  BA_OK = 0,
  BA_ERR_INVALID_ARGUMENT = 1,
  BA_ERR_DEVICE = 2,          /* HIP runtime / kernel failure */
  BA_ERR_OUT_OF_MEMORY = 3,
  BA_ERR_NO_PROBLEM = 4,      /* ba_solve before ba_set_problem */
  BA_ERR_COMM = 5             /* RCCL failure */
};

enum ba_termination {          /* ceres::TerminationType subset */
  BA_CONVERGENCE = 0,
  BA_NO_CONVERGENCE = 1,
  BA_FAILURE = 2
};

enum ba_linear_solver {
  BA_DENSE_SCHUR = 0,          /* ceres::DENSE_SCHUR (Optimizer.cpp:85): explicit reduced camera
                                  system, dense Cholesky (MFMA) */
  BA_ITERATIVE_SCHUR = 1       /* ceres::ITERATIVE_SCHUR: implicit Schur complement + PCG
                                  (C5 scale; one 6C all-reduce per CG step) */
};

enum ba_preconditioner {       /* ceres::PreconditionerType (ITERATIVE_SCHUR only) */
  BA_JACOBI = 0,               /* ceres default: block diagonal of F'F + D^2 */
  BA_SCHUR_JACOBI = 1          /* block diagonal of the Schur complement */
};

enum ba_precision {
  BA_FP64 = 0,                 /* everything fp64 (the reference's Jets are double) */
  BA_MIXED_FP32 = 1            /* ITERATIVE_SCHUR: fp32 storage of the per-observation Schur
                                  blocks W read by every CG step; fp64 accumulation and CG vectors */
};

typedef struct ba_ctx ba_ctx;

/* Problem description (caller-owned host SoA; copied to the device by
 * ba_set_problem).  Replaces the AddResidualBlock loop of prepareConstraints. */
typedef struct {
  int32_t n_cams, n_pts, n_obs, reserved;
  const double*  cams;            /* [6*n_cams]                             */
  const uint8_t* cam_fixed;       /* [n_cams] 1 = constant (may be NULL)    */
  const float*   cam_fixed_extr;  /* [16*n_cams] col-major; read for fixed cams (may be NULL if none) */
  const float*   K;               /* [9*n_cams] col-major                   */
  const double*  pts;             /* [3*n_pts]                              */
  const uint8_t* pt_fixed;        /* [n_pts] 1 = constant (may be NULL)     */
  const int32_t* obs_cam;         /* [n_obs]                                */
  const int32_t* obs_pt;          /* [n_obs]                                */
  const float*   obs_uv;          /* [2*n_obs]                              */
  double huber_a;                 /* sqrt(5.991) in the reference           */
} ba_problem;

/* ceres::Solver::Options fields the reference touches (configureSolver,
 * Optimizer.cpp:80-90) plus the Ceres defaults it inherits. */
typedef struct {
  int32_t max_num_iterations;                 /* m_nMaxItPerBA (Optimizer.h:203,212) */
  int32_t max_num_consecutive_invalid_steps;  /* 5  */
  int32_t jacobi_scaling;                     /* 1  */
  int32_t linear_solver;                      /* BA_DENSE_SCHUR */
  double function_tolerance;                  /* 1e-6  */
  double gradient_tolerance;                  /* 1e-10 */
  double parameter_tolerance;                 /* 1e-8  */
  double initial_trust_region_radius;         /* 1e4   */
  double max_trust_region_radius;             /* 1e16  */
  double min_trust_region_radius;             /* 1e-32 */
  double min_relative_decrease;               /* 1e-3  */
  double min_lm_diagonal;                     /* 1e-6  */
  double max_lm_diagonal;                     /* 1e32  */
  /* ITERATIVE_SCHUR (ceres::Solver::Options defaults; unused by DENSE_SCHUR) */
  int32_t preconditioner_type;                /* BA_JACOBI */
  int32_t max_linear_solver_iterations;       /* 500 */
  int32_t min_linear_solver_iterations;       /* 0   */
  int32_t precision;                          /* BA_FP64 */
  double eta;                                 /* 1e-1: CG q_tolerance (LevenbergMarquardtStrategy) */
} ba_options;

/* ceres::Solver::Summary subset */
typedef struct {
  double initial_cost;
  double final_cost;
  int32_t num_iterations;
  int32_t num_successful_steps;
  int32_t num_unsuccessful_steps;
  int32_t termination_type;        /* enum ba_termination */
  double total_time_s;             /* wall time of ba_solve */
  double linearize_time_s;         /* device time: residual+Jacobian+assembly */
  double solve_time_s;             /* device time: Schur + reduced solve + back-sub + candidate */
} ba_summary;

/* ceres::IterationSummary subset (one record per minimizer iteration,
 * iteration 0 = initial evaluation). */
typedef struct {
  int32_t iteration;
  int32_t step_is_valid;
  int32_t step_is_successful;
  int32_t linear_solver_iterations; /* CG iterations (ITERATIVE_SCHUR), 1 for DENSE_SCHUR */
  double cost;
  double cost_change;
  double gradient_max_norm;
  double gradient_norm;
  double step_norm;
  double relative_decrease;
  double trust_region_radius;
  double model_cost_change;
  double iteration_time_s;
} ba_iteration;

int ba_abi_version(void);
void ba_default_options(ba_options* opt);       /* Ceres defaults, max_num_iterations = 50 */

/* Context on one HIP device (the process's GPU).  Owns device buffers, the
 * HIP stream and (after ba_comm_init) the RCCL communicator. */
int ba_create(ba_ctx** ctx, int device);
int ba_destroy(ba_ctx* ctx);
const char* ba_last_error(const ba_ctx* ctx);

/* Multi-GPU (points sharded across ranks; cameras replicated).  Every rank
 * calls ba_comm_init with the same 128-byte id produced by ba_comm_unique_id
 * on rank 0 (exchange it with any host transport, e.g. torch.distributed).
 * Per LM iteration the ranks all-reduce the camera-side system over RCCL. */
int ba_comm_unique_id(char id[128]);
int ba_comm_init(ba_ctx* ctx, const char id[128], int nranks, int rank);

/* Host-visible collective over the context's communicator (RCCL): in-place
 * reduction of n doubles across ranks (op 0 = sum, 1 = max); blocks until the
 * result is on the host.  With n = 0 it is a barrier.  Without a
 * communicator it is the identity.  Used for the bench's max-over-ranks
 * timing, so no second GPU runtime is needed for host-side rendezvous. */
int ba_comm_allreduce_host(ba_ctx* ctx, double* values, int n, int op);

/* Host-staged transport for the same exchange (test hook, not the product
 * path): every all-reduce of the multi-rank LM iteration is copied to the
 * host and handed to fn(user, values, n, op) (op 0 = sum, 1 = max; in place;
 * return 0 on success), e.g. torch.distributed over gloo.  It lets several
 * ranks share one GPU — RCCL refuses duplicate devices — so the multi-rank
 * HIP path (packing, folding, replicated decisions) runs on a 1-GPU box.
 * Replaces any RCCL communicator of the context. */
typedef int (*ba_host_allreduce_fn)(void* user, double* values, int64_t n, int op);
int ba_comm_init_host(ba_ctx* ctx, ba_host_allreduce_fn fn, void* user, int nranks, int rank);

/* Copy a problem to the device and build its (fixed) structure. */
int ba_set_problem(ba_ctx* ctx, const ba_problem* problem);

/* Replace the parameter values of the current problem (same structure). */
int ba_set_params(ba_ctx* ctx, const double* cams, const double* pts);

/* Levenberg-Marquardt with DENSE_SCHUR or ITERATIVE_SCHUR (ceres::Solve
 * semantics; opt->linear_solver). */
int ba_solve(ba_ctx* ctx, const ba_options* opt, ba_summary* summary);

/* Current parameters (after ba_solve: the returned minimum). */
int ba_get_params(ba_ctx* ctx, double* cams, double* pts);

/* Iteration log of the last ba_solve: copies min(n, available) records,
 * returns the number available (or <0 on error). */
int ba_get_iteration_log(ba_ctx* ctx, ba_iteration* out, int n);

/* Raw functor residuals r[2*n_obs] in caller observation order and the total
 * robustified cost 0.5*sum(rho) (used for pruning and tests). */
int ba_eval_residuals(ba_ctx* ctx, double* r, double* cost);

/* Linearisation at the current parameters in caller order: Huber-corrected
 * residuals r[2*n_obs] and Jacobian J[n_obs][2][9] (camera 6 | point 3;
 * zero blocks for constant parameter blocks).  Test/inspection entry point. */
int ba_linearize(ba_ctx* ctx, double* r, double* J, double* cost);

/* pruneCorrespondences (BAOptimizer, Optimizer.cpp:6-79) for a batch of
 * (keyframe, keypoint) pairs, evaluated in float like the reference:
 *   c = hnormalized(extr * [X;1]); outlier if c.z <= 0;
 *   outlier if |X - cam_center| > max_dist or < min_dist;
 *   outlier if |hnormalized(K c) - uv| * inv_sigma > 5.991 (a norm, not a
 *   squared norm: Optimizer.cpp:56-59); otherwise inlier.
 * Operation order (fixed here; Eigen's is not pinned): matrix-vector products
 * accumulate column by column, norms as sqrt((x*x + y*y) + z*z), no fused
 * multiply-adds, IEEE division and square root.
 * The caller selects which pairs to evaluate (considerOutlier) and applies
 * the results with Frame::setOutlier / setInlier. */
typedef struct {
  int32_t n_cams, n_obs;
  const float*   extr;            /* [16*n_cams] col-major world->camera = getPose().inverse() */
  const float*   cam_center;      /* [3*n_cams]  getWorldPos()                   */
  const float*   K;               /* [9*n_cams]  col-major getIntrinsics()      */
  const int32_t* obs_cam;         /* [n_obs]                                     */
  const float*   obs_X;           /* [3*n_obs]   MapPoint::getPosition()          */
  const float*   obs_uv;          /* [2*n_obs]   getKeypoint(i)->pt               */
  const float*   obs_inv_sigma;   /* [n_obs]     (float)(1.0 / pow(1.2, octave))  */
  const float*   obs_dist;        /* [2*n_obs]   getMinDistance, getMaxDistance   */
} ba_prune_problem;

enum ba_prune_result {
  BA_INLIER = 0,
  BA_OUTLIER_BEHIND = 1,          /* camspacePos.z() <= 0        (Optimizer.cpp:36-41) */
  BA_OUTLIER_DEPTH = 2,           /* outside [minDist, maxDist]  (:43-51) */
  BA_OUTLIER_CHI2 = 3             /* reprojection test           (:53-64) */
};

/* result[n_obs] receives a ba_prune_result per pair (runs on the device). */
int ba_prune(ba_ctx* ctx, const ba_prune_problem* problem, uint8_t* result);

/* Batched frame-to-frame pose-only solves.
 * Replaces, per frame, the ceres::Problem + ceres::Solve of
 * MotionOnlyBAOptimizerAngles::optimizeCameraPose (Optimizer.cpp:417-442;
 * residuals from MotionOnlyBAOptimizerAngles::prepareConstraints,
 * Optimizer.cpp:459-498: PoseOnlyAngleReprojectionError, Optimizer.h:163-182,
 * with HuberLoss(huber_a)).  Problem i owns observations
 * [obs_offset[i], obs_offset[i+1]) against its own camera; the points are
 * constant.  Same Levenberg-Marquardt semantics as ba_solve on the
 * equivalent one-camera problem (options and termination rules included),
 * but the whole trust-region loop of every problem runs in one kernel
 * launch (one wavefront per problem), so a frame costs one host round trip
 * instead of two per LM iteration.  cams_out[6*i] receives the solution
 * (may alias cams); summaries[i] (may be NULL) the per-problem summary
 * (time fields: the batch's wall time). */
typedef struct {
  int32_t n_problems;
  int32_t reserved;
  const int32_t* obs_offset;      /* [n_problems + 1], obs_offset[0] = 0, non-decreasing */
  const double*  cams;            /* [6*n_problems] initial [w, t] (world->camera)      */
  const float*   K;               /* [9*n_problems] col-major                           */
  const double*  pts;             /* [3*obs_offset[n]] constant world points (float values
                                     of MapPoint::getPosition in the reference)          */
  const float*   obs_uv;          /* [2*obs_offset[n]]                                  */
  double huber_a;                 /* sqrt(5.991); <= 0: no loss                         */
} ba_pose_batch;

int ba_solve_pose_batch(ba_ctx* ctx, const ba_pose_batch* batch, const ba_options* opt, double* cams_out,
                        ba_summary* summaries);

/* Test / inspection entry point: the state inside ceres::Solve's
 * SchurComplementSolver (Optimizer.cpp:242, DENSE_SCHUR) for one step.
 * Linearises at the current parameters with iteration-0 Jacobi scaling, then
 * forms the reduced camera system at trust-region radius `radius` with the
 * very kernels a solve's step runs (J-free consumers, compact or 18-double W
 * records, LDS or global camera tables: whatever the problem size selects),
 * without factoring it, and copies out (caller indices; any pointer may be
 * NULL):
 *   Hpp[6*n_pts]  J_p^T J_p per point (xx, xy, xz, yy, yz, zz; unscaled,
 *                 Huber-corrected J; zero for constant points),
 *   gp[3*n_pts]   J_p^T r,
 *   Hcc[21*n_cams] J_c^T J_c (lower triangle, row-major: (a, b), b <= a),
 *   gc[6*n_cams]  J_c^T r (zero for constant / unobserved cameras),
 *   S[n*n]        the reduced system s_c (Hcc - sum W W^T) s_c + D^2 as the
 *                 Cholesky receives it (row-major, lower triangle; upper 0),
 *   rhs[n]        its right-hand side,
 * with n = *n_out = 6 x the observed variable cameras in increasing camera
 * index (Jacobi-scaled columns, as Ceres' DENSE_SCHUR forms them). */
int ba_debug_blocks(ba_ctx* ctx, double radius, double* Hpp, double* gp, double* Hcc, double* gc, double* S,
                    double* rhs, int* n_out);

/* Blocks until all device work of the context is done. */
int ba_synchronize(ba_ctx* ctx);

/* Timing hooks for bench.py: one LM iteration = linearise + assemble + Schur
 * + reduced solve (opt->linear_solver; NULL = defaults) + back-substitution +
 * candidate evaluation at a fixed trust-region radius (no accept/reject
 * bookkeeping).  Runs `iters` iterations on the context's stream and returns
 * the device-measured (HIP events) average milliseconds of the whole
 * iteration and of the residual+Jacobian kernel alone, and the mean number
 * of linear-solver iterations per LM iteration (may be NULL).  ms_rj_kernel
 * NULL: no event pair around the kernel (each pair's packets idle the device
 * ~5 us per iteration; bench.py times the kernel in a second pass). */
int ba_bench_iterations(ba_ctx* ctx, const ba_options* opt, int iters, double radius, double* ms_per_iter,
                        double* ms_rj_kernel, double* linear_iters);

/* Host wall time (ms) of each LM iteration of the last ba_bench_iterations
 * call: from one iteration's scalar record reaching the host to the next's
 * (the first from the call's start).  Copies min(n, available) values and
 * returns the number available (bench.py reports their median, BASELINE.md
 * §2, beside the mean over the timed region). */
int ba_bench_iteration_times(ba_ctx* ctx, double* ms, int n);

/* Measured copy bandwidth of the context's device ("also
 * report a measured STREAM-copy figure" beside the 8 TB/s peak): a
 * non-temporal 16-B load / store copy of `bytes` (rounded down to 16 B)
 * between two device buffers, `reps` timed launches after one warm-up, HIP
 * events on the context's stream.  *gbs = 2 * bytes * reps / time (read +
 * write).  Diagnostic; no reference counterpart. */
int ba_stream_copy(ba_ctx* ctx, size_t bytes, int reps, double* gbs);

#ifdef __cplusplus
}
#endif
#endif /* BA_HIP_H_ */

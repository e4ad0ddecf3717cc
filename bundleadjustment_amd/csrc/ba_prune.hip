// ba_prune.hip — pruneCorrespondences (Optimizer.cpp:6-79) as a per-pair
// device kernel.  The reference runs it on the host in float after every
// outer BA round; the result bits are observable output, so the arithmetic
// is pinned: round-to-nearest intrinsics (no contraction into FMAs), IEEE
// division and square root, and the operation order documented for ba_prune
// in include/ba_hip.h.
#include "ba_kernels.h"

namespace bahip {

__global__ __launch_bounds__(256) void k_prune(int n, const float* __restrict__ extr,
                                               const float* __restrict__ center, const float* __restrict__ K,
                                               const int* __restrict__ obs_cam, const float* __restrict__ X,
                                               const float* __restrict__ uv, const float* __restrict__ inv_sigma,
                                               const float* __restrict__ dist, uint8_t* __restrict__ out) {
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= n) return;
  const int c = obs_cam[o];
  const float* e = extr + 16 * c;
  const float x0 = X[3 * o], x1 = X[3 * o + 1], x2 = X[3 * o + 2];
  // camspacePos = (extr * X.homogeneous()).hnormalized()      (Optimizer.cpp:33)
  float v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
    v[i] = __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(e[i], x0), __fmul_rn(e[4 + i], x1)), __fmul_rn(e[8 + i], x2)),
                     e[12 + i]);
  const float cz = __fdiv_rn(v[2], v[3]);
  if (cz <= 0.0f) { out[o] = 1; return; }                        // :36-41
  const float cx = __fdiv_rn(v[0], v[3]), cy = __fdiv_rn(v[1], v[3]);
  // worldDist = |X - frame->getWorldPos()|                       :44-51
  const float* ctr = center + 3 * c;
  const float d0 = __fsub_rn(x0, ctr[0]), d1 = __fsub_rn(x1, ctr[1]), d2 = __fsub_rn(x2, ctr[2]);
  const float wd = __fsqrt_rn(__fadd_rn(__fadd_rn(__fmul_rn(d0, d0), __fmul_rn(d1, d1)), __fmul_rn(d2, d2)));
  if (wd > dist[2 * o + 1] || wd < dist[2 * o]) { out[o] = 2; return; }
  // projPos = (intr * camspacePos).hnormalized(); |projPos - kp| * invSigma > 5.991   :53-64
  const float* k = K + 9 * c;
  float q[3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
    q[i] = __fadd_rn(__fadd_rn(__fmul_rn(k[i], cx), __fmul_rn(k[3 + i], cy)), __fmul_rn(k[6 + i], cz));
  const float e0 = __fsub_rn(__fdiv_rn(q[0], q[2]), uv[2 * o]);
  const float e1 = __fsub_rn(__fdiv_rn(q[1], q[2]), uv[2 * o + 1]);
  const float nrm = __fsqrt_rn(__fadd_rn(__fmul_rn(e0, e0), __fmul_rn(e1, e1)));
  const float chi = __fmul_rn(nrm, inv_sigma[o]);
  const float thresh = 5.991;                                     // float chiThresh = 5.991
  out[o] = chi > thresh ? 3 : 0;
}

void launch_prune(int n, const float* extr, const float* center, const float* K, const int* obs_cam, const float* X,
                  const float* uv, const float* inv_sigma, const float* dist, uint8_t* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_prune, dim3((n + 255) / 256), dim3(256), 0, s, n, extr, center, K, obs_cam, X, uv, inv_sigma,
                     dist, out);
}

}  // namespace bahip

// halfspace_kernels.hip — batched Constraints::FindHalfSpaces (reference
// src/constraints.cpp:116-265) on gfx950.
//
// The reference walks one LaserScan sequentially with a small state machine whose quirks
// (stale `hi` when a new gap opens, so single-beam gaps are never recorded; the (-1,-1)
// "gap" recorded when the window opens on a short beam; int/float buffer comparison) decide
// which gap wins. Those quirks make the winner depend on the scan order, so each scan is
// processed by one lane exactly in reference order; the batch (one scan per candidate
// scenario / QP) supplies the parallelism. The per-beam float arithmetic is written with
// explicit round-to-nearest intrinsics so hipcc cannot contract it into FMAs that the x86
// reference build does not use. Output is the f110qp_solve_batch half-space layout
// hs[b] = (a1, b1, c1+0.5, a2, b2, c2+0.5) in float32.
#include <hip/hip_runtime.h>

#include "f110qp_kernels.h"

namespace f110qp {

__global__ __launch_bounds__(256) void half_space_kernel(int B, const float* __restrict__ states,
                                                         const float* __restrict__ ranges,
                                                         int nr, float angle_min, float angle_inc,
                                                         float angle_max, float thresh,
                                                         float divider, float buffer,
                                                         float* __restrict__ hs, int* gap_lo,
                                                         int* gap_hi) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float* r = ranges + (size_t)b * nr;
  int num_scans = (int)(__fadd_rn(__fdiv_rn(__fsub_rn(angle_max, angle_min), angle_inc), 1.0f));
  if (num_scans > nr) num_scans = nr;
  int max_gap = -1, best_lo = 0, best_hi = 0, lo = -1, hi = -1;
  bool in_gap = false;
  const float lim = __fdiv_rn(1.571f, divider);
  for (int ii = 0; ii < num_scans; ii++) {
    const float angle = __fadd_rn(angle_min, __fmul_rn((float)ii, angle_inc));
    if (angle > -lim && angle < lim) {
      if (r[ii] > thresh) {
        if (in_gap) hi = ii;
        else { lo = ii; in_gap = true; }
      } else {
        in_gap = false;
      }
      if (hi - lo > max_gap) { max_gap = hi - lo; best_hi = hi; best_lo = lo; }
    }
  }
  if ((float)(best_hi - best_lo) > __fmul_rn(2.0f, buffer)) {
    best_hi = (int)((float)best_hi - buffer);
    best_lo = (int)((float)best_lo + buffer);
  }
  if (gap_lo) gap_lo[b] = best_lo;
  if (gap_hi) gap_hi[b] = best_hi;
  float* o = hs + (size_t)b * 6;
  if (best_lo < 0 || best_hi < 0 || best_lo >= nr || best_hi >= nr) {
    const float nanv = __int_as_float(0x7fc00000);
    for (int j = 0; j < 6; j++) o[j] = nanv;
    return;
  }
  const double poseX = (double)states[3 * b + 0], poseY = (double)states[3 * b + 1];
  const float cur = states[3 * b + 2];
  const float ang1 = __fadd_rn(__fadd_rn(angle_min, __fmul_rn((float)best_lo, angle_inc)), cur);
  const float ang2 = __fadd_rn(__fadd_rn(angle_min, __fmul_rn((float)best_hi, angle_inc)), cur);
  const float p1x = (float)__dadd_rn(__dmul_rn((double)r[best_lo], cos((double)ang1)), poseX);
  const float p1y = (float)__dadd_rn(__dmul_rn((double)r[best_lo], sin((double)ang1)), poseY);
  const float p2x = (float)__dadd_rn(__dmul_rn((double)r[best_hi], cos((double)ang2)), poseX);
  const float p2y = (float)__dadd_rn(__dmul_rn((double)r[best_hi], sin((double)ang2)), poseY);
  const float px = (float)poseX, py = (float)poseY;
  float a1 = __fsub_rn(py, p1y), b1 = __fsub_rn(p1x, px);
  float c1 = __fsub_rn(__fmul_rn(px, p1y), __fmul_rn(py, p1x));
  if (__fadd_rn(__fadd_rn(__fmul_rn(a1, p2x), __fmul_rn(b1, p2y)), c1) < 0.f) {
    a1 = -a1; b1 = -b1; c1 = -c1;
  }
  float a2 = __fsub_rn(py, p2y), b2 = __fsub_rn(p2x, px);
  float c2 = __fsub_rn(__fmul_rn(px, p2y), __fmul_rn(py, p2x));
  if (__fadd_rn(__fadd_rn(__fmul_rn(a2, p1x), __fmul_rn(b2, p1y)), c2) < 0.f) {
    a2 = -a2; b2 = -b2; c2 = -c2;
  }
  o[0] = a1; o[1] = b1; o[2] = (float)((double)c1 + 0.5);
  o[3] = a2; o[4] = b2; o[5] = (float)((double)c2 + 0.5);
}

hipError_t launch_half_spaces(int B, const float* states, const float* ranges, int nr,
                              float angle_min, float angle_inc, float angle_max, float thresh,
                              float divider, float buffer, float* hs, int* gap_lo, int* gap_hi,
                              hipStream_t s) {
  if (B <= 0) return hipSuccess;
  const int threads = 256;
  hipLaunchKernelGGL(half_space_kernel, dim3((B + threads - 1) / threads), dim3(threads), 0, s,
                     B, states, ranges, nr, angle_min, angle_inc, angle_max, thresh, divider,
                     buffer, hs, gap_lo, gap_hi);
  return hipGetLastError();
}

}  // namespace f110qp

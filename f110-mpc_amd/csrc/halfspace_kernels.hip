// halfspace_kernels.hip — batched Constraints::FindHalfSpaces (reference
// src/constraints.cpp:116-265) on gfx950: ONE WAVEFRONT PER SCAN.
//
// The reference walks one LaserScan sequentially with a small state machine (lo, hi, in_gap,
// max_gap) whose quirks decide which gap wins: a gap's `hi` is stale when the next gap opens, so
// a single-beam gap is never recorded; the record is taken after every in-window beam with a
// strict '>' (the first gap of the maximal length wins); and when the field-of-view window opens
// on a short beam the initial (lo, hi) = (-1, -1) is recorded as a gap of length 0. Written
// over the window's open beams (in window and range > ftg_thresh) that machine has a closed
// form, which this kernel evaluates in parallel:
//   * for an open beam p inside a run of open beams that started at s < p, the record compares
//     p - s (for p = s the stale hi makes it negative); the answer is the FIRST beam p attaining
//     the maximum of p - s, i.e. the end of the first longest run of >= 2 beams, (lo, hi) = (s, p);
//   * with no run of >= 2 beams: (-1, -1) if the window's first beam is closed, else the
//     initial (0, 0) (also when no beam falls in the window).
// A wave streams its scan in 64-beam blocks (lane j loads beam 64 k + j: coalesced 256 B per
// wave instruction; a 1,080-beam scan is one round trip, every block in flight at once), turns the open flags into 64-bit ballots,
// finds run starts with shifts of the ballot (the carry of block k-1's top beam included) and
// the start of each lane's run as the highest start bit at or below it (or the last start of an
// earlier block, a wave-uniform scalar). Each lane keeps the best key (p - s) << 16 | (65535 - p)
// as an UNSIGNED 32-bit value (p - s <= 65534, so the key never overflows; 0 = no run) (larger
// run first, then the earlier beam); one wave max-reduction ends the scan. Lane 0 then
// evaluates the endpoints and the two half-spaces with the reference's float/double types.
// FP contraction is off for the whole kernel body (hipcc fuses a*b+c into an FMA by default and
// does so even through the __fmul_rn/__fadd_rn helpers, which are plain operators inlined from
// the HIP headers; the x86 reference build does not fuse: with fusion 18% of the end points came
// out one float ulp off), so the reference's float/double expressions are written as they are. Output is the f110qp_solve_batch half-space
// layout hs[b] = (a1, b1, c1+0.5, a2, b2, c2+0.5) in float32; a scan without a gap (the
// reference reads ranges[-1] there) gives NaN.
#include <hip/hip_runtime.h>

#include "f110qp_kernels.h"

namespace f110qp {

constexpr int kHsWaves = 4;   // scans (waves) per 256-thread workgroup
constexpr int kHsBatch = 24;  // 64-beam blocks loaded per lane before they are consumed (1,536 beams)

__device__ __forceinline__ unsigned wave_max_u32(unsigned v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = max(v, (unsigned)__shfl_xor((int)v, o));
  return v;
}

__global__ __launch_bounds__(256) void half_space_kernel(int B, const float* __restrict__ states,
                                                         const float* __restrict__ ranges,
                                                         int nr, float angle_min, float angle_inc,
                                                         float angle_max, float thresh,
                                                         float divider, float buffer,
                                                         float* __restrict__ hs, int* gap_lo,
                                                         int* gap_hi) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * kHsWaves + (threadIdx.x >> 6);
  if (b >= B) return;  // whole waves only
  const float* r = ranges + (size_t)b * nr;
  // the pose is only needed by the tail: loaded now, its latency hides behind the scan
  const float st0 = states[3 * b + 0], st1 = states[3 * b + 1], st2 = states[3 * b + 2];
  // num_scans = (angle_max - angle_min) / angle_increment + 1 in float, truncated (:118)
  int num_scans = (int)((angle_max - angle_min) / angle_inc + 1.0f);
  if (num_scans > nr) num_scans = nr;
  const float lim = 1.571f / divider;  // :135
  const int nblk = num_scans > 0 ? (num_scans + 63) / 64 : 0;
  unsigned best = 0u;         // per-lane best key (0: no run of >= 2 beams)
  int last_start = -1;        // last run start in the blocks before k (wave-uniform)
  bool top_open = false;      // beam 64 k - 1 open (wave-uniform)
  int w0 = -1;                // first in-window beam (wave-uniform)
  bool w0_open = false;
  float v[kHsBatch];  // the last batch of blocks stays in registers for the tail
#pragma unroll
  for (int j = 0; j < kHsBatch; j++) v[j] = 0.f;
  const unsigned last = (unsigned)(num_scans - 1);
  for (int k0 = 0; k0 < nblk; k0 += kHsBatch) {
    // unconditional loads (clamped index): no exec masking; a 32-bit offset from the scan's
    // wave-uniform base (one min and one shift per load)
#pragma unroll
    for (int j = 0; j < kHsBatch; j++) v[j] = r[min((unsigned)(64 * (k0 + j) + lane), last)];
    // fully unrolled (a wave-uniform guard per block instead of a break: the break kept the loop
    // rolled, v[j] then went through dynamic register indexing)
#pragma unroll
    for (int j = 0; j < kHsBatch; j++) {
      const int k = k0 + j;
      if (k >= nblk) continue;
      const int p = 64 * k + lane;
      const float angle = angle_min + (float)p * angle_inc;  // :133
      const bool inwin = p < num_scans && angle > -lim && angle < lim;
      const bool open = inwin && v[j] > thresh;  // :138
      const unsigned long long W = __builtin_amdgcn_ballot_w64(inwin), M = __builtin_amdgcn_ballot_w64(open);
      if (w0 < 0 && W) {
        const int t = __builtin_ctzll(W);
        w0 = 64 * k + t;
        w0_open = (M >> t) & 1ull;
      }
      // run starts: open beams whose predecessor is not open
      const unsigned long long S = M & ~((M << 1) | (top_open ? 1ull : 0ull));
      const unsigned long long upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
      const unsigned long long Sb = S & upto;
      const int s = Sb ? 64 * k + 63 - __builtin_clzll(Sb) : last_start;
      if (open && s < p) best = max(best, ((unsigned)(p - s) << 16) | (unsigned)(65535 - p));
      if (S) last_start = 64 * k + 63 - __builtin_clzll(S);
      top_open = (M >> 63) & 1ull;
    }
  }
  best = wave_max_u32(best);
  // The tail runs on every lane with the same values (a partially masked wave runs ~2.4x slower
  // on a loaded CU, tools/microbench/contention.hip); lane 0 stores.
  int best_lo, best_hi;
  if (best != 0u) {
    best_hi = 65535 - (int)(best & 0xffffu);
    best_lo = best_hi - (int)(best >> 16);
  } else if (w0 >= 0 && !w0_open) {
    best_lo = best_hi = -1;  // the initial (lo, hi) recorded on the window's first (short) beam
  } else {
    best_lo = best_hi = 0;
  }
  if ((float)(best_hi - best_lo) > 2.0f * buffer) {  // :173-177 (int vs float buffer_)
    best_hi = (int)((float)best_hi - buffer);
    best_lo = (int)((float)best_lo + buffer);
  }
  if (lane == 0 && gap_lo) gap_lo[b] = best_lo;
  if (lane == 0 && gap_hi) gap_hi[b] = best_hi;
  float* o = hs + (size_t)b * 6;
  if (best_lo < 0 || best_hi < 0 || best_lo >= nr || best_hi >= nr) {  // wave-uniform
    const float nanv = __int_as_float(0x7fc00000);
    if (lane == 0)
      for (int j = 0; j < 6; j++) o[j] = nanv;
    return;
  }
  const double poseX = (double)st0, poseY = (double)st1;
  const float cur = st2;
  const float ang1 = angle_min + (float)best_lo * angle_inc + cur;  // :179-180
  const float ang2 = angle_min + (float)best_hi * angle_inc + cur;
  // even lanes evaluate the first end point's cos/sin, odd lanes the second (::cos/::sin(double))
  double sl, cl;
  sincos((double)((lane & 1) ? ang2 : ang1), &sl, &cl);
  const double s1 = __shfl(sl, 0), c1d = __shfl(cl, 0);
  const double s2 = __shfl(sl, 1), c2d = __shfl(cl, 1);
  // ranges[best_lo], ranges[best_hi]: from the registers of the last batch when the scan fits
  // one batch (1,536 beams), else re-read (L2). An empty window (num_scans <= 0: no block was
  // loaded, (lo, hi) = (0, 0)) reads ranges[0] as the reference does.
  float rlo, rhi;
  if (nblk >= 1 && nblk <= kHsBatch) {
    const int klo = best_lo >> 6, khi = best_hi >> 6;
    float vlo = 0.f, vhi = 0.f;
#pragma unroll
    for (int j = 0; j < kHsBatch; j++) {
      vlo = (j == klo) ? v[j] : vlo;
      vhi = (j == khi) ? v[j] : vhi;
    }
    rlo = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, vlo), best_lo & 63));
    rhi = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, vhi), best_hi & 63));
  } else {
    rlo = r[best_lo];
    rhi = r[best_hi];
  }
  const float p1x = (float)((double)rlo * c1d + poseX);  // :181-185
  const float p1y = (float)((double)rlo * s1 + poseY);
  const float p2x = (float)((double)rhi * c2d + poseX);
  const float p2y = (float)((double)rhi * s2 + poseY);
  const float px = (float)poseX, py = (float)poseY;
  float a1 = py - p1y, b1 = p1x - px;  // :233-253
  float c1 = px * p1y - py * p1x;
  if (a1 * p2x + b1 * p2y + c1 < 0.f) {
    a1 = -a1; b1 = -b1; c1 = -c1;
  }
  float a2 = py - p2y, b2 = p2x - px;
  float c2 = px * p2y - py * p2x;
  if (a2 * p1x + b2 * p1y + c2 < 0.f) {
    a2 = -a2; b2 = -b2; c2 = -c2;
  }
  if (lane == 0) {
    o[0] = a1; o[1] = b1; o[2] = (float)((double)c1 + 0.5);  // :255-264
    o[3] = a2; o[4] = b2; o[5] = (float)((double)c2 + 0.5);
  }
}

hipError_t launch_half_spaces(int B, const float* states, const float* ranges, int nr,
                              float angle_min, float angle_inc, float angle_max, float thresh,
                              float divider, float buffer, float* hs, int* gap_lo, int* gap_hi,
                              hipStream_t s) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(half_space_kernel, dim3((B + kHsWaves - 1) / kHsWaves), dim3(64 * kHsWaves), 0, s,
                     B, states, ranges, nr, angle_min, angle_inc, angle_max, thresh, divider,
                     buffer, hs, gap_lo, gap_hi);
  return hipGetLastError();
}

}  // namespace f110qp

// f110qp_kernels.hip — dispatch of the solve kernel (solve_kernel.h) by horizon and row set.
//
// NUM = 2N rounded up to the instantiated variable counts: one register row per lane up to
// NUM = 64 (N <= 32, the reference default N = 30 included), two rows for NUM = 80 / 96
// (N <= 48; BASELINE config C4 is N = 40). GAP selects the kernel with follow-the-gap rows.
#include <hip/hip_runtime.h>

#include "f110qp_kernels.h"

namespace f110qp {

template <int NUM, bool GAP>
hipError_t launch_t(const KParams& P, int B, const float* x0, const float* ul, const float* xr,
                    const float* hs, float* uo, float* xo, int* st, int* its, double* Hd,
                    double* gd, const WarmState& ws, const int* list, const int* count, int grid,
                    const ObjOut& oo, hipStream_t s);  // solve_inst.hip
template <int NUM, bool GAP>
hipError_t launch_prep_t(const KParams& P, int B, const float* x0, const float* ul,
                         const float* xr, const float* hs, const WarmState& ws, const int* leader,
                         hipStream_t s);  // solve_inst.hip

template <bool GAP>
static hipError_t launch_g(const KParams& P, int B, const float* x0, const float* ul,
                           const float* xr, const float* hs, float* uo, float* xo, int* st,
                           int* its, double* Hd, double* gd, const WarmState& ws, const int* list,
                           const int* count, int grid, const ObjOut& oo, hipStream_t s) {
  const int NU = 2 * P.N;
#define F110QP_CASE(NUM)                                                                    \
  if (NU <= NUM)                                                                            \
    return launch_t<NUM, GAP>(P, B, x0, ul, xr, hs, uo, xo, st, its, Hd, gd, ws, list, count, \
                              grid, oo, s);
  F110QP_CASE(8) F110QP_CASE(16) F110QP_CASE(24) F110QP_CASE(32) F110QP_CASE(40)
  F110QP_CASE(48) F110QP_CASE(56) F110QP_CASE(64) F110QP_CASE(80) F110QP_CASE(96)
#undef F110QP_CASE
  return hipErrorInvalidValue;
}

// Gap-row screen after a box-only lane solve: a QP whose box optimum keeps every gap row of stages
// 1..N strictly satisfied has that point as its optimum with the gap rows (adding constraints that
// hold at the unique minimiser of a strictly convex QP does not move it), so its lane outputs stand.
// Every other QP goes to the wave kernel's GI: a gap row violated or within the margin, the stage-0
// rows violated (constant rows, x0 on both lines by constraints.cpp:233-246; violated, the wedge is
// infeasible), a non-SOLVED box status, non-finite values. The margin is 1e-6 of the row's terms:
// ~8x the float rounding of the stored x (absolute coordinates) plus the row's float data. This
// kernel serves the sequential lane kernel's batches (from stored float x); the segmented kernel
// evaluates the same test in its output sweep, in fp64. Output: the GI priority of each QP (0: the
// box optimum stands, else 1 + the violated rows; 1 for the stage-0 / status cases).
__global__ __launch_bounds__(256) void gap_screen_kernel(const int B, const int N,
                                                         const float* __restrict__ x0g,
                                                         const float* __restrict__ hsg,
                                                         const float* __restrict__ xo,
                                                         const int* __restrict__ status,
                                                         int* __restrict__ prio) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  const double px = (double)x0g[3 * b], py = (double)x0g[3 * b + 1];
  const float* xb = xo + (size_t)b * (N + 1) * 3;
  bool ok0 = status[b] == F110QP_SOLVED_ID;
  int nv = 0;
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const double a = (double)hsg[6 * b + 3 * h], bb = (double)hsg[6 * b + 3 * h + 1],
                 c = (double)hsg[6 * b + 3 * h + 2];
    ok0 = ok0 && (a * px + bb * py >= -c - 1e-9);  // stage 0: constant rows
    for (int i = 1; i <= N; i++) {
      const double x = (double)xb[3 * i], y = (double)xb[3 * i + 1];
      const double ax = a * x, by = bb * y;
      nv += !(ax + by + c >= 1e-6 * (1.0 + fabs(ax) + fabs(by) + fabs(c)));
    }
  }
  prio[b] = !ok0 ? 1 : (nv > 0 ? 1 + nv : 0);
}

// The GI list in priority order, heavy first (one workgroup; a counting sort over the priorities
// 1..kPrioMax by LDS histogram, scan and scatter): a QP's GI chain grows with the gap rows its box
// optimum violates, and a long chain that starts late in the dispatch adds its whole length to
// the launch (an atomic append in the lane kernel's wave completion order put them late; same-box
// A/B on C3: step 236-242 -> 225 us with this order).
constexpr int kPrioMax = 127;
__global__ __launch_bounds__(1024) void gap_order_kernel(const int B, const int* __restrict__ prio,
                                                         int* __restrict__ count, int* __restrict__ list,
                                                         int* __restrict__ zero) {
  __shared__ int hist[kPrioMax + 1];
  __shared__ int off[2][kPrioMax + 1];
  const int t = threadIdx.x;
  if (t <= kPrioMax) hist[t] = 0;
  // the first kHold x 1,024 priorities stay in registers for the scatter (one global read of them)
  constexpr int kHold = 8;
  int held[kHold];
#pragma unroll
  for (int k = 0; k < kHold; k++) {
    const int b = t + 1024 * k;
    held[k] = b < B ? min(prio[b], kPrioMax) : 0;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kHold; k++)
    if (held[k] > 0) atomicAdd(&hist[held[k]], 1);
  for (int b = t + 1024 * kHold; b < B; b += 1024) {
    const int p = min(prio[b], kPrioMax);
    if (p > 0) atomicAdd(&hist[p], 1);
  }
  __syncthreads();
  // descending offsets (the highest priority first): an inclusive scan over r = kPrioMax - p in
  // LDS, log2(128) barrier-separated steps, independent of the wavefront width (round-5 ADVICE: the
  // two 64-lane shuffle scans assumed wave64)
  const int r = kPrioMax - t;  // thread t < 128 scans priority kPrioMax - t (priority 0 counts none)
  if (t <= kPrioMax) off[0][t] = (r > 0) ? hist[r] : 0;
  __syncthreads();
  int src = 0;
#pragma unroll
  for (int d = 1; d <= kPrioMax; d <<= 1) {
    if (t <= kPrioMax) off[src ^ 1][t] = off[src][t] + (t >= d ? off[src][t - d] : 0);
    src ^= 1;
    __syncthreads();
  }
  if (t <= kPrioMax) {
    const int inc = off[src][t];
    hist[t] = inc;  // (hist is free again) inclusive prefix in scan order
    if (t == kPrioMax) {
      *count = inc;
      if (zero) *zero = 0;  // the re-check count the GI kernel appends to next
    }
  }
  __syncthreads();
  // exclusive offset of priority p at off[0][kPrioMax + 1 - p]: the QPs of every priority above p,
  // i.e. the inclusive prefix at scan index kPrioMax - p - 1 (0 for the top priority)
  if (t >= 1 && t <= kPrioMax) off[0][t] = (t >= 2) ? hist[t - 2] : 0;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kHold; k++)
    if (held[k] > 0) list[atomicAdd(&off[0][kPrioMax + 1 - held[k]], 1)] = t + 1024 * k;
  for (int b = t + 1024 * kHold; b < B; b += 1024) {
    const int p = min(prio[b], kPrioMax);
    if (p > 0) list[atomicAdd(&off[0][kPrioMax + 1 - p], 1)] = b;
  }
}

// The re-check list holding every QP of the call in order (the test build's F110QP_RECHECK_ALL route)
__global__ __launch_bounds__(256) void list_all_kernel(const int B, int* __restrict__ count,
                                                       int* __restrict__ list) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b < B) list[b] = b;
  if (b == 0) *count = B;
}

// The completion signal costs every workgroup of the call's last kernel a system-scope fence (an L2
// write-back of its XCD) and an arrival on one device word: a win up to a few hundred of them, a loss
// beyond (tools/sync_batch_probe.py, dev_sync against launch + stream synchronize: 128 waves 32.0
// against 36.7 us, 512 waves 51.2 against 39.1, 4,096 waves 174 against 109). So only calls whose last
// kernel has at most kSignalMaxGrid workgroups are armed; the others synchronise the stream, whose
// end-of-kernel release writes each L2 back once.
constexpr int kSignalMaxGrid = 256;
bool launch_signals(const KParams& P, int B, int backend, const float* hs, const LaneWork& lw) {
  if (B <= 0) return false;
  long grid;
  if (hs) {
    grid = B < 256 ? B : 256;  // the fp64 re-check's grid (launch_gap_recheck)
  } else if (backend == BACKEND_LANE) {
    const int S = lane_segments(P, B, lw);
    if (S > 1) {
      const long L = 64 / S;
      grid = (((long)B << (lane_seg_starts(P, B, S, lw) == 2 ? 1 : 0)) + L - 1) / L;
    } else {
      const long L = lane_qps_per_wave(B, lw.qpw);
      grid = (B + L - 1) / L;
    }
  } else {
    grid = B;  // one wave per QP
  }
  return grid <= kSignalMaxGrid;
}

hipError_t launch_solve(const KParams& P, int B, const float* x0, const float* ul,
                        const float* xr, const float* hs, float* uo, float* xo, int* st,
                        int* its, const WarmState& ws, int backend, const LaneWork& lw,
                        const ObjOut& oo_in, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  ObjOut oo = oo_in;
  if (!launch_signals(P, B, backend, hs, lw)) oo.sig_host = nullptr;  // several kernels: no signal
  if (hs) {
    // Gap rows. With the screen: the box-only lane solve of every QP (the segmented kernel
    // evaluates the screen in its output sweep, in fp64, and writes each QP's GI priority; the
    // sequential kernel leaves it to gap_screen_kernel), the GI list heavy first (gap_order_kernel,
    // which also zeroes the re-check count), GI over it (grid B: the waves past the device-side
    // count exit at once). Without: GI for every QP. Either way the GI kernel appends the QPs it
    // does not certify (SOLVED) to the re-check list, and the fp64 GI re-checks them.
    const HandLayout H(lw.hand, B);
    hipError_t e = hipSuccess;
    ObjOut base = oo;  // the kernels before the re-check never raise the completion signal
    base.sig_host = nullptr;
    if (lw.recheck_all) {  // test build: the re-check's own answer for every QP (no screen, no fp32 GI)
      hipLaunchKernelGGL(list_all_kernel, dim3((B + 255) / 256), dim3(256), 0, s, B, H.c_rc, H.rc);
      if ((e = hipGetLastError()) != hipSuccess) return e;
      return launch_gap_recheck(P, B, x0, ul, xr, hs, uo, xo, st, its, H.rc, H.c_rc, oo, s);
    }
    ObjOut go = base;
    go.rc_count = H.c_rc;
    go.rc_list = H.rc;
    if (lw.screen) {
      const bool fused = lane_segments(P, B, lw) > 1;
      ObjOut so = base;
      if (fused) {
        so.scr_hs = hs;
        so.scr_prio = H.prio;
      }
      if ((e = launch_lane(P, B, x0, ul, xr, uo, xo, st, its, WarmState(), lw, so, s)) != hipSuccess) return e;
      if (!fused) {
        hipLaunchKernelGGL(gap_screen_kernel, dim3((B + 255) / 256), dim3(256), 0, s, B, P.N, x0, hs, xo, st, H.prio);
        if ((e = hipGetLastError()) != hipSuccess) return e;
      }
      hipLaunchKernelGGL(gap_order_kernel, dim3(1), dim3(1024), 0, s, B, H.prio, H.c_list, H.list, H.c_rc);
      if ((e = hipGetLastError()) != hipSuccess) return e;
      e = launch_g<true>(P, B, x0, ul, xr, hs, uo, xo, st, its, nullptr, nullptr, WarmState(), H.list, H.c_list, B,
                         go, s);
    } else {
      if ((e = hipMemsetAsync(H.c_rc, 0, sizeof(int), s)) != hipSuccess) return e;
      e = launch_g<true>(P, B, x0, ul, xr, hs, uo, xo, st, its, nullptr, nullptr, ws, nullptr, nullptr, B, go, s);
    }
    if (e != hipSuccess) return e;
    return launch_gap_recheck(P, B, x0, ul, xr, hs, uo, xo, st, its, H.rc, H.c_rc, oo, s);
  }
  if (backend == BACKEND_LANE) return launch_lane(P, B, x0, ul, xr, uo, xo, st, its, ws, lw, oo, s);
  return launch_g<false>(P, B, x0, ul, xr, hs, uo, xo, st, its, nullptr, nullptr, ws, nullptr,
                         nullptr, B, oo, s);
}

template <bool GAP>
static hipError_t launch_prep_g(const KParams& P, int B, const float* x0, const float* ul,
                                const float* xr, const float* hs, const WarmState& ws,
                                const int* leader, hipStream_t s) {
  const int NU = 2 * P.N;
#define F110QP_CASE(NUM) \
  if (NU <= NUM) return launch_prep_t<NUM, GAP>(P, B, x0, ul, xr, hs, ws, leader, s);
  F110QP_CASE(8) F110QP_CASE(16) F110QP_CASE(24) F110QP_CASE(32) F110QP_CASE(40)
  F110QP_CASE(48) F110QP_CASE(56) F110QP_CASE(64) F110QP_CASE(80) F110QP_CASE(96)
#undef F110QP_CASE
  return hipErrorInvalidValue;
}

// leader[g] = smallest b with group[b] == g (leader pre-filled with 0x7f7f7f7f = "none")
__global__ __launch_bounds__(256) void group_mark_kernel(const int B, const int* __restrict__ group,
                                                         const int G, int* __restrict__ leader) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b < B) {
    const int g = group[b];
    if (g >= 0 && g < G) atomicMin(leader + g, b);
  }
}

hipError_t launch_solve_grouped(const KParams& P, int B, const float* x0, const float* ul,
                                const float* xr, const float* hs, float* uo, float* xo, int* st,
                                int* its, const WarmState& gws, int* leader, int backend,
                                const LaneWork& lw, const ObjOut& oo, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  if (backend == BACKEND_LANE || (hs && (lw.screen || lw.recheck_all)))  // per-QP Riccati: nothing to share
    return launch_solve(P, B, x0, ul, xr, hs, uo, xo, st, its, WarmState(), backend, lw, oo, s);
  hipError_t e = hipMemsetAsync(leader, 0x7f, (size_t)gws.ngroups * sizeof(int), s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(group_mark_kernel, dim3((B + 255) / 256), dim3(256), 0, s, B, gws.group,
                     gws.ngroups, leader);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  e = hs ? launch_prep_g<true>(P, B, x0, ul, xr, hs, gws, leader, s)
         : launch_prep_g<false>(P, B, x0, ul, xr, hs, gws, leader, s);
  if (e != hipSuccess) return e;
  if (hs) {
    const HandLayout H(lw.hand, B);
    ObjOut go = oo;
    go.sig_host = nullptr;  // (grouped calls are never armed; only the re-check could signal)
    go.rc_count = H.c_rc;
    go.rc_list = H.rc;
    if ((e = hipMemsetAsync(H.c_rc, 0, sizeof(int), s)) != hipSuccess) return e;
    e = launch_g<true>(P, B, x0, ul, xr, hs, uo, xo, st, its, nullptr, nullptr, gws, nullptr, nullptr, B, go, s);
    if (e != hipSuccess) return e;
    return launch_gap_recheck(P, B, x0, ul, xr, hs, uo, xo, st, its, H.rc, H.c_rc, oo, s);
  }
  return launch_g<false>(P, B, x0, ul, xr, hs, uo, xo, st, its, nullptr, nullptr, gws, nullptr, nullptr, B, oo, s);
}

hipError_t launch_condense_debug(const KParams& P, int B, const float* x0, const float* ul,
                                 const float* xr, double* Hd, double* gd, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  return launch_g<false>(P, B, x0, ul, xr, nullptr, nullptr, nullptr, nullptr, nullptr, Hd, gd,
                         WarmState(), nullptr, nullptr, B, ObjOut(), s);
}

// ---- per-scenario selection (f110qp_select_dev) --------------------------------------------
// Two passes of 64-bit atomics over one grid-stride launch each: (1) the group minimum of the
// solved members' cost bits (a non-negative double orders like its bit pattern), (2) the smallest
// member index attaining it. Exact (no rounding of the cost into a packed key) and
// deterministic; O(B) with one atomic per QP and pass.
__global__ __launch_bounds__(256) void select_init_kernel(int G, unsigned long long* __restrict__ bits,
                                                          int* __restrict__ winner) {
  const int g = blockIdx.x * 256 + threadIdx.x;
  if (g < G) {
    bits[g] = 0x7ff0000000000000ull;  // +inf: no solved member yet
    winner[g] = 0x7fffffff;
  }
}

__device__ __forceinline__ bool select_eligible(int b, const int* group, int G, const double* cost,
                                                const int* status, int* gout, unsigned long long* cb) {
  const int g = group[b];
  const double c = cost[b];
  if (g < 0 || g >= G || status[b] != F110QP_SOLVED_ID || !(c >= 0.0) || !(c < 1.0e308)) return false;
  *gout = g;
  *cb = (unsigned long long)__double_as_longlong(c + 0.0);  // -0.0 -> +0.0
  return true;
}

__global__ __launch_bounds__(256) void select_min_kernel(int B, const int* __restrict__ group, int G,
                                                         const double* __restrict__ cost,
                                                         const int* __restrict__ status,
                                                         unsigned long long* __restrict__ bits) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  int g;
  unsigned long long cb;
  if (b < B && select_eligible(b, group, G, cost, status, &g, &cb)) atomicMin(bits + g, cb);
}

__global__ __launch_bounds__(256) void select_arg_kernel(int B, const int* __restrict__ group, int G,
                                                         const double* __restrict__ cost,
                                                         const int* __restrict__ status,
                                                         const unsigned long long* __restrict__ bits,
                                                         int* __restrict__ winner) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  int g;
  unsigned long long cb;
  if (b < B && select_eligible(b, group, G, cost, status, &g, &cb) && cb == bits[g])
    atomicMin(winner + g, b);
}

__global__ __launch_bounds__(256) void select_fin_kernel(int G, const unsigned long long* __restrict__ bits,
                                                         int* __restrict__ winner, double* __restrict__ best) {
  const int g = blockIdx.x * 256 + threadIdx.x;
  if (g < G) {
    const bool none = winner[g] == 0x7fffffff;
    if (none) winner[g] = -1;
    // best aliases bits (same 8-byte slots): the value is read before it is overwritten
    const double v = __longlong_as_double((long long)bits[g]);
    if (best) best[g] = v;
  }
}

hipError_t launch_select(int B, const int* group, int G, const double* cost, const int* status,
                         int* winner, double* best, hipStream_t s) {
  if (G <= 0) return hipSuccess;
  // the minimum bits live in `best` (G doubles, caller-provided) and become the best cost
  unsigned long long* bits = reinterpret_cast<unsigned long long*>(best);
  hipLaunchKernelGGL(select_init_kernel, dim3((G + 255) / 256), dim3(256), 0, s, G, bits, winner);
  if (B > 0) {
    hipLaunchKernelGGL(select_min_kernel, dim3((B + 255) / 256), dim3(256), 0, s, B, group, G, cost, status, bits);
    hipLaunchKernelGGL(select_arg_kernel, dim3((B + 255) / 256), dim3(256), 0, s, B, group, G, cost, status, bits,
                       winner);
  }
  hipLaunchKernelGGL(select_fin_kernel, dim3((G + 255) / 256), dim3(256), 0, s, G, bits, winner, best);
  return hipGetLastError();
}

}  // namespace f110qp

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
                    hipStream_t s);  // solve_inst.hip
template <int NUM, bool GAP>
hipError_t launch_prep_t(const KParams& P, int B, const float* x0, const float* ul,
                         const float* xr, const float* hs, const WarmState& ws, const int* leader,
                         hipStream_t s);  // solve_inst.hip

template <bool GAP>
static hipError_t launch_g(const KParams& P, int B, const float* x0, const float* ul,
                           const float* xr, const float* hs, float* uo, float* xo, int* st,
                           int* its, double* Hd, double* gd, const WarmState& ws, const int* list,
                           const int* count, int grid, hipStream_t s) {
  const int NU = 2 * P.N;
#define F110QP_CASE(NUM)                                                                    \
  if (NU <= NUM)                                                                            \
    return launch_t<NUM, GAP>(P, B, x0, ul, xr, hs, uo, xo, st, its, Hd, gd, ws, list, count, \
                              grid, s);
  F110QP_CASE(8) F110QP_CASE(16) F110QP_CASE(24) F110QP_CASE(32) F110QP_CASE(40)
  F110QP_CASE(48) F110QP_CASE(56) F110QP_CASE(64) F110QP_CASE(80) F110QP_CASE(96)
#undef F110QP_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_solve(const KParams& P, int B, const float* x0, const float* ul,
                        const float* xr, const float* hs, float* uo, float* xo, int* st,
                        int* its, const WarmState& ws, int backend, const LaneWork& lw,
                        hipStream_t s) {
  if (B <= 0) return hipSuccess;
  if (hs)
    return launch_g<true>(P, B, x0, ul, xr, hs, uo, xo, st, its, nullptr, nullptr, ws, nullptr,
                          nullptr, B, s);
  if (backend == BACKEND_LANE) return launch_lane(P, B, x0, ul, xr, uo, xo, st, its, ws, lw, s);
  return launch_g<false>(P, B, x0, ul, xr, hs, uo, xo, st, its, nullptr, nullptr, ws, nullptr,
                         nullptr, B, s);
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
                                const LaneWork& lw, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  if (!hs && backend == BACKEND_LANE)  // per-QP Riccati: nothing to share
    return launch_solve(P, B, x0, ul, xr, hs, uo, xo, st, its, WarmState(), backend, lw, s);
  hipError_t e = hipMemsetAsync(leader, 0x7f, (size_t)gws.ngroups * sizeof(int), s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(group_mark_kernel, dim3((B + 255) / 256), dim3(256), 0, s, B, gws.group,
                     gws.ngroups, leader);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  e = hs ? launch_prep_g<true>(P, B, x0, ul, xr, hs, gws, leader, s)
         : launch_prep_g<false>(P, B, x0, ul, xr, hs, gws, leader, s);
  if (e != hipSuccess) return e;
  return hs ? launch_g<true>(P, B, x0, ul, xr, hs, uo, xo, st, its, nullptr, nullptr, gws, nullptr,
                             nullptr, B, s)
            : launch_g<false>(P, B, x0, ul, xr, hs, uo, xo, st, its, nullptr, nullptr, gws,
                              nullptr, nullptr, B, s);
}

hipError_t launch_condense_debug(const KParams& P, int B, const float* x0, const float* ul,
                                 const float* xr, double* Hd, double* gd, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  return launch_g<false>(P, B, x0, ul, xr, nullptr, nullptr, nullptr, nullptr, nullptr, Hd, gd,
                         WarmState(), nullptr, nullptr, B, s);
}

}  // namespace f110qp

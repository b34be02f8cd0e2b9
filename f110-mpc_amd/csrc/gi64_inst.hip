// gi64_inst.hip — the fp64 re-check of gap-row QPs (gi64_kernel.h). The Makefile compiles this file
// once per variable count (-DF110QP_GI64_NUM=.., in parallel) and once for the launch over the
// re-check list (-DF110QP_GI64_LAUNCH); -DF110QP_GI64_ALL builds everything in one unit.
#if defined(F110QP_GI64_NUM) || defined(F110QP_GI64_ALL)
#include "gi64_kernel.h"
#else
#include "f110qp_kernels.h"
#endif

namespace f110qp {

#if defined(F110QP_GI64_NUM) || defined(F110QP_GI64_ALL)
#define F110QP_GI64_INSTANTIATE(NUM)                                                                   \
  template hipError_t launch_gi64_t<NUM>(const KParams&, int, const float*, const float*, const float*, \
                                         const float*, float*, float*, int*, int*, const int*,          \
                                         const int*, const ObjOut&, hipStream_t);
#ifdef F110QP_GI64_ALL
F110QP_GI64_INSTANTIATE(8) F110QP_GI64_INSTANTIATE(16) F110QP_GI64_INSTANTIATE(24) F110QP_GI64_INSTANTIATE(32)
F110QP_GI64_INSTANTIATE(40) F110QP_GI64_INSTANTIATE(48) F110QP_GI64_INSTANTIATE(56) F110QP_GI64_INSTANTIATE(64)
F110QP_GI64_INSTANTIATE(80) F110QP_GI64_INSTANTIATE(96)
#else
F110QP_GI64_INSTANTIATE(F110QP_GI64_NUM)
#endif
#endif

#if defined(F110QP_GI64_LAUNCH) || defined(F110QP_GI64_ALL)
// Grid of the re-check: a grid-stride loop over the device-side count processes every listed QP,
// whatever the grid. One workgroup per CU (256 on the MI355X; the N = 48 instantiation's 154 KiB of
// LDS fits one per CU anyway), so a long list (stiff batches list a few percent of their QPs at
// ~170 us per heavy QP) spreads over the whole chip instead of 1/8 of it. A call whose list is
// empty (the usual case) costs the launch of workgroups that read a zero count and exit: 4.7 us at
// 256 workgroups against 4.45 at 32 on C3 (rocprof, round 5).
#ifndef F110QP_RECHECK_GRID
#define F110QP_RECHECK_GRID 256
#endif
constexpr int kRecheckGrid = F110QP_RECHECK_GRID;

template <int NUM>
hipError_t launch_gi64_t(const KParams& P, int grid, const float* x0, const float* ul, const float* xr,
                         const float* hs, float* uo, float* xo, int* st, int* its, const int* list,
                         const int* count, const ObjOut& oo, hipStream_t s);  // one object per NUM

hipError_t launch_gap_recheck(const KParams& P, int B, const float* x0, const float* ul, const float* xr,
                              const float* hs, float* uo, float* xo, int* st, int* its, const int* list,
                              const int* count, const ObjOut& oo, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  const int grid = B < kRecheckGrid ? B : kRecheckGrid;
  ObjOut o = oo;
  o.rc_count = nullptr;
  o.rc_list = nullptr;
  const int NU = 2 * P.N;
#define F110QP_CASE(NUM) \
  if (NU <= NUM) return launch_gi64_t<NUM>(P, grid, x0, ul, xr, hs, uo, xo, st, its, list, count, o, s);
  F110QP_CASE(8) F110QP_CASE(16) F110QP_CASE(24) F110QP_CASE(32) F110QP_CASE(40)
  F110QP_CASE(48) F110QP_CASE(56) F110QP_CASE(64) F110QP_CASE(80) F110QP_CASE(96)
#undef F110QP_CASE
  return hipErrorInvalidValue;
}
#endif

}  // namespace f110qp

// lane_ipm_inst.hip — the interior-point lane kernel for QPs with gap rows (lane_ipm_kernel.h):
// its launch policy (segments per QP) and the instantiations.
#include "lane_ipm_kernel.h"

namespace f110qp {

// Horizon segments per QP: S in {2, 4, 8, 16} cutting N into segments of >= 2 stages, the grid's
// resident waves within the CU's 160 KiB of LDS (ipm_lds_bytes per wave) and <= 4 waves per CU;
// among those the shortest per-iteration chain by the instruction model ceil(N / S) x ~1,000
// cycles of stage work + (S - 1) x ~500 of segment steps. 0: no segmentation fits (the wave
// kernel solves the batch). F110QP_LANE_SEG forces S where it fits.
int lane_ipm_segments(const KParams& P, int B, const LaneWork& lw) {
  const int N = P.N;
  auto fits = [&](int S) {
    if (N / S < 2) return false;
    const size_t waves = ((size_t)B * S + 63) / 64;
    const size_t per_cu = (waves + 255) / 256;
    return per_cu <= 4 && per_cu * ipm_lds_bytes(N, S) <= 160 * 1024;
  };
  if (lw.seg == 2 || lw.seg == 4 || lw.seg == 8 || lw.seg == 16) return fits(lw.seg) ? lw.seg : 0;
  int best = 0;
  double cbest = 1e30;
  for (int S = 2; S <= 16; S <<= 1) {
    if (!fits(S)) continue;
    const double c = 1000.0 * ((N + S - 1) / S) + 500.0 * (S - 1);
    if (c < cbest) {
      best = S;
      cbest = c;
    }
  }
  return best;
}

template <bool ROT>
static hipError_t ipm_s(int S, const KParams& P, int B, const float* x0, const float* ul, const float* xr,
                        const float* hs, float* uo, float* xo, int* st, int* its, int* list, int* count,
                        const IpmKnobs& kn, const ObjOut& oo, hipStream_t s, const int* ql, const int* qc, int rc) {
  switch (S) {
    case 2: return launch_lane_ipm_t<2, ROT>(P, B, x0, ul, xr, hs, uo, xo, st, its, list, count, kn, oo, s, ql, qc, rc);
    case 4: return launch_lane_ipm_t<4, ROT>(P, B, x0, ul, xr, hs, uo, xo, st, its, list, count, kn, oo, s, ql, qc, rc);
    case 8: return launch_lane_ipm_t<8, ROT>(P, B, x0, ul, xr, hs, uo, xo, st, its, list, count, kn, oo, s, ql, qc, rc);
    case 16: return launch_lane_ipm_t<16, ROT>(P, B, x0, ul, xr, hs, uo, xo, st, its, list, count, kn, oo, s, ql, qc, rc);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_lane_ipm(const KParams& P, int B, const float* x0, const float* ul, const float* xr,
                           const float* hs, float* uo, float* xo, int* st, int* its, const LaneWork& lw,
                           const ObjOut& oo, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  const bool rot = lw.rot && P.q[0] == P.q[1];
  const int S = lane_ipm_segments(P, B, lw);
  const HandLayout H(lw.hand, B);
  return rot ? ipm_s<true>(S, P, B, x0, ul, xr, hs, uo, xo, st, its, H.list, H.c_list, lw.ipm, oo, s, nullptr,
                           nullptr, 0)
             : ipm_s<false>(S, P, B, x0, ul, xr, hs, uo, xo, st, its, H.list, H.c_list, lw.ipm, oo, s, nullptr,
                            nullptr, 0);
}

// Re-check of the wave kernel's gap-row QPs that are not SOLVED (status 2, -2, -3, -10): list them,
// then run the interior point over the list in fp64; a polished point (KKT-checked) becomes SOLVED,
// a Farkas certificate PRIMAL_INFEASIBLE, anything else keeps the wave kernel's answer. At most
// kRecheckCap list items are re-checked (one wave per CU at S = 4, N = 20). Count HandLayout::c_rc,
// list HandLayout::list (or `flagged`); zeroed: the caller already cleared the count.
constexpr int kRecheckCap = 4096;
hipError_t launch_gap_recheck(const KParams& P, int B, const float* x0, const float* ul, const float* xr,
                              const float* hs, float* uo, float* xo, int* st, int* its, const LaneWork& lw,
                              const ObjOut& oo, hipStream_t s, bool zeroed, const int* flagged) {
  if (B <= 0 || !lw.hand) return hipSuccess;
  const int cap = B < kRecheckCap ? B : kRecheckCap;
  LaneWork l2 = lw;
  l2.seg = 0;
  const int S = lane_ipm_segments(P, cap, l2);
  if (S == 0) return hipSuccess;  // no segmentation fits this horizon: the wave kernel's answer stands
  hipError_t e = hipSuccess;
  const HandLayout H(lw.hand, B);
  const int* list = flagged ? flagged : H.list;
  if (!flagged) {
    if (!zeroed && (e = hipMemsetAsync(H.c_rc, 0, sizeof(int), s)) != hipSuccess) return e;
    hipLaunchKernelGGL(ipm_flag_kernel, dim3((B + 255) / 256), dim3(256), 0, s, B, st, H.c_rc, H.list);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  const bool rot = lw.rot && P.q[0] == P.q[1];
  // grid of `cap` QPs; the kernel reads the count and idle waves exit at once
  return rot ? ipm_s<true>(S, P, cap, x0, ul, xr, hs, uo, xo, st, its, nullptr, nullptr, lw.ipm, oo, s,
                           list, H.c_rc, 1)
             : ipm_s<false>(S, P, cap, x0, ul, xr, hs, uo, xo, st, its, nullptr, nullptr, lw.ipm, oo, s,
                            list, H.c_rc, 1);
}

}  // namespace f110qp

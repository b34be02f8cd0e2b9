// lane_ipm_inst.hip — the interior-point lane kernel for QPs with gap rows (lane_ipm_kernel.h):
// its launch policy (segments per QP) and the instantiations.
#include "lane_ipm_kernel.h"

namespace f110qp {

// Horizon segments per QP: S in {2, 4, 8} cutting N into segments of >= 2 stages, the grid's
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
  if (lw.seg == 2 || lw.seg == 4 || lw.seg == 8) return fits(lw.seg) ? lw.seg : 0;
  int best = 0;
  double cbest = 1e30;
  for (int S = 2; S <= 8; S <<= 1) {
    if (!fits(S)) continue;
    const double c = 1000.0 * ((N + S - 1) / S) + 500.0 * (S - 1);
    if (c < cbest) {
      best = S;
      cbest = c;
    }
  }
  return best;
}

hipError_t launch_lane_ipm(const KParams& P, int B, const float* x0, const float* ul, const float* xr,
                           const float* hs, float* uo, float* xo, int* st, int* its, const LaneWork& lw,
                           const ObjOut& oo, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  const bool rot = lw.rot && P.q[0] == P.q[1];
  int* count = lw.hand;
  int* list = lw.hand + 1;
  switch (lane_ipm_segments(P, B, lw)) {
    case 2: return rot ? launch_lane_ipm_t<2, true>(P, B, x0, ul, xr, hs, uo, xo, st, its, list, count, lw.ipm, oo, s)
                       : launch_lane_ipm_t<2, false>(P, B, x0, ul, xr, hs, uo, xo, st, its, list, count, lw.ipm, oo, s);
    case 4: return rot ? launch_lane_ipm_t<4, true>(P, B, x0, ul, xr, hs, uo, xo, st, its, list, count, lw.ipm, oo, s)
                       : launch_lane_ipm_t<4, false>(P, B, x0, ul, xr, hs, uo, xo, st, its, list, count, lw.ipm, oo, s);
    case 8: return rot ? launch_lane_ipm_t<8, true>(P, B, x0, ul, xr, hs, uo, xo, st, its, list, count, lw.ipm, oo, s)
                       : launch_lane_ipm_t<8, false>(P, B, x0, ul, xr, hs, uo, xo, st, its, list, count, lw.ipm, oo, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace f110qp

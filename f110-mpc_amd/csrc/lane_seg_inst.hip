// lane_seg_inst.hip — instantiations of the segmented lane kernel (lane_seg_kernel.h): S = 2, 4, 8
// horizon segments per QP (64 / S QPs per wave), heading frame and general frame. Compiled twice
// (Makefile): F110QP_SEG_SCR = 0 the box-only kernels, 1 the variants with the gap-row screen in
// the output sweep (f110qp_kernels.hip), as two objects that build in parallel; F110QP_SEG_ALL
// (the stamps build) instantiates both here.
#include "lane_seg_kernel.h"

#ifndef F110QP_SEG_SCR
#define F110QP_SEG_SCR 0
#endif

namespace f110qp {
#define F110QP_SEG_INST(S, ROT, SCR)                                                                \
  template hipError_t launch_lane_seg_t<S, ROT, SCR>(const KParams&, int, const float*, const float*, \
                                                     const float*, float*, float*, int*, int*,       \
                                                     const WarmState&, const LaneWork&, const ObjOut&, \
                                                     hipStream_t);
#define F110QP_SEG_INST_ALL(SCR) \
  F110QP_SEG_INST(2, true, SCR)  \
  F110QP_SEG_INST(2, false, SCR) \
  F110QP_SEG_INST(4, true, SCR)  \
  F110QP_SEG_INST(4, false, SCR) \
  F110QP_SEG_INST(8, true, SCR)  \
  F110QP_SEG_INST(8, false, SCR)
#if defined(F110QP_SEG_ALL) || F110QP_SEG_SCR == 0
F110QP_SEG_INST_ALL(false)
#endif
#if defined(F110QP_SEG_ALL) || F110QP_SEG_SCR == 1
F110QP_SEG_INST_ALL(true)
#endif
#undef F110QP_SEG_INST_ALL
#undef F110QP_SEG_INST

#if defined(F110QP_SEG_ALL) || F110QP_SEG_SCR == 0
int lane_seg_scratch(const KParams& P, int B, int S, const LaneWork& lw) {
  return seg_scratch_mode(P, seg_twin(P, B, S, lw) ? 2 * B : B, S, lw);
}
int lane_seg_starts(const KParams& P, int B, int S, const LaneWork& lw) { return seg_twin(P, B, S, lw) ? 2 : 1; }
#endif
}  // namespace f110qp

// lane_seg_inst.hip — instantiations of the segmented lane kernel (lane_seg_kernel.h): S = 2, 4, 8
// horizon segments per QP (64 / S QPs per wave), heading frame and general frame.
#include "lane_seg_kernel.h"

namespace f110qp {
#define F110QP_SEG_INST(S, ROT)                                                                \
  template hipError_t launch_lane_seg_t<S, ROT>(const KParams&, int, const float*, const float*, \
                                                const float*, float*, float*, int*, int*,       \
                                                const WarmState&, const LaneWork&, const ObjOut&, \
                                                hipStream_t);
F110QP_SEG_INST(2, true)
F110QP_SEG_INST(2, false)
F110QP_SEG_INST(4, true)
F110QP_SEG_INST(4, false)
F110QP_SEG_INST(8, true)
F110QP_SEG_INST(8, false)
#undef F110QP_SEG_INST

int lane_seg_scratch(const KParams& P, int B, int S, const LaneWork& lw) { return seg_scratch_mode(P, B, S, lw); }
}  // namespace f110qp

// lane_inst.hip — instantiations of the lane kernel (lane_kernel.h) for one QPs-per-wave value
// F110QP_LQ (compiled once per value by the Makefile, so make -j builds them in parallel): LDS
// fp64, LDS fp32, HBM fp32 and HBM fp64 Riccati scratch, each in the heading frame (q0 == q1)
// and in the general one, with fp64 or float references in LDS (DREF).
#include "lane_kernel.h"

#ifndef F110QP_LQ
#error "F110QP_LQ (QPs per wave) must be defined"
#endif

namespace f110qp {
#define F110QP_INST(ST, SLDS)                                                                  \
  F110QP_INST_R(ST, SLDS, true, true)                                                          \
  F110QP_INST_R(ST, SLDS, false, true)                                                         \
  F110QP_INST_R(ST, SLDS, true, false)                                                         \
  F110QP_INST_R(ST, SLDS, false, false)
#define F110QP_INST_R(ST, SLDS, ROT, DREF)                                                     \
  template hipError_t launch_lane_t<ST, SLDS, F110QP_LQ, ROT, DREF>(                           \
      const KParams&, int, const float*, const float*, const float*, float*, float*, int*, int*, \
      const WarmState&, const LaneWork&, const ObjOut&, size_t, hipStream_t);
F110QP_INST(double, true)
F110QP_INST(float, true)
F110QP_INST(float, false)
F110QP_INST(double, false)
#undef F110QP_INST
#undef F110QP_INST_R
}  // namespace f110qp

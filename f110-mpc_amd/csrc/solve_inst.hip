// solve_inst.hip — explicit instantiations of the solve kernel (solve_kernel.h).
//
// The Makefile compiles this file once per (NUM, GAP) pair (-DF110QP_NUM=.. -DF110QP_GAP=..)
// so the 20 instantiations build in parallel; the diagnostic stamps build compiles it once with
// -DF110QP_ALL_INST (the per-wave stamp buffer must live in a single translation unit).
#include "solve_kernel.h"

#define F110QP_INSTANTIATE(NUM, GAP)                                                           \
  template hipError_t f110qp::launch_t<NUM, GAP>(                                              \
      const KParams&, int, const float*, const float*, const float*, const float*, float*,      \
      float*, int*, int*, double*, double*, const WarmState&, const int*, const int*, int,       \
      const ObjOut&, hipStream_t);                                                             \
  template hipError_t f110qp::launch_prep_t<NUM, GAP>(const KParams&, int, const float*,       \
                                                      const float*, const float*, const float*,  \
                                                      const WarmState&, const int*, hipStream_t);

#ifdef F110QP_ALL_INST
#define F110QP_BOTH(NUM) F110QP_INSTANTIATE(NUM, false) F110QP_INSTANTIATE(NUM, true)
F110QP_BOTH(8) F110QP_BOTH(16) F110QP_BOTH(24) F110QP_BOTH(32) F110QP_BOTH(40)
F110QP_BOTH(48) F110QP_BOTH(56) F110QP_BOTH(64) F110QP_BOTH(80) F110QP_BOTH(96)
#else
F110QP_INSTANTIATE(F110QP_NUM, F110QP_GAP)
#endif

#ifdef F110QP_STAMPS
extern "C" int f110qp_read_stamps(unsigned long long* host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(f110qp::g_stamps),
                                  (size_t)n * f110qp::kStampSlots * sizeof(unsigned long long));
}
#endif

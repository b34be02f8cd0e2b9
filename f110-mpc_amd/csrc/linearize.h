// linearize.h — Model::Linearize on the device, fp64 (reference src/model.cpp:30-59; L = 0.3302f
// at :32; dt is the float MPC::dt_). Shared by the wave kernel (solve_kernel.h) and the
// assembly-parity hook (assemble_kernel.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace f110qp {

struct Lin {
  double th0, a02, a12, b00, b10, b20, b21, c0, c1, c2;
};

__device__ __forceinline__ Lin linearize(double th, double v, double d, float dtf) {
  const double dt = (double)dtf;
  const double L = (double)0.3302f;
  double sn, cs, sd, cd;
  sincos(th, &sn, &cs);
  sincos(d, &sd, &cd);
  const double sec2 = 1.0 / (cd * cd);  // pow(cos(d), -2)
  Lin M;
  M.th0 = th;
  M.a02 = -1 * v * sn * dt;           // :42
  M.a12 = v * cs * dt;                // :43
  M.b00 = cs * dt;                    // :48
  M.b10 = sn * dt;                    // :49
  M.b20 = (sd / cd) * dt / L;         // :50 tan(d)
  M.b21 = v * sec2 * dt / L;          // :51
  M.c0 = v * th * sn * dt;            // :53
  M.c1 = -1 * v * th * cs * dt;       // :54
  M.c2 = -1 * d * v * sec2 * dt / L;  // :55
  return M;
}

}  // namespace f110qp

// assemble_kernel.hip — the assembly-parity hook f110qp_assemble_debug_dev: one instance's QP in
// the reference's OSQP form, (P, q, A, l, u) in CSC exactly as MPC holds it after
// MPC::Update's CreateGradientVector / UpdateLinearConstraintMatrix / Update{Lower,Upper}Bound
// (src/mpc.cpp:77-80, layouts :208-306), computed on the device from the same inputs and the
// same fp64 Model::Linearize the solve kernel uses (linearize.h). The solve kernels never build
// this sparse form (they condense it, or sweep it stage by stage); the hook lets a test check
// the product's reading of the reference QP — the explicit zeros of the dense 3x3 / 3x2 blocks,
// the placeholder all-ones gap block of stage 0 (:238-241, never updated: the update loop starts
// at ii = 1, :267), the terminal gradient reusing x_ref[N-1] (:228), the +-INFTY gap bounds of
// the shipped code (:279-300) or the documented C3 semantic — entry by entry.
#include <hip/hip_runtime.h>

#include "f110qp_kernels.h"
#include "linearize.h"

namespace f110qp {

constexpr double kInfty = 1e30;  // OsqpEigen::INFTY (constraints.cpp:15,17; mpc.cpp:279-298)

// One thread: a debug path, not a hot one.
__global__ __launch_bounds__(64) void assemble_kernel(const KParams P, const float* __restrict__ x0g,
                                                      const float* __restrict__ ulg,
                                                      const float* __restrict__ xrg,
                                                      const float* __restrict__ hsg, int gap_active,
                                                      int* Pc, int* Pr, double* Pv, double* q, int* Ac,
                                                      int* Ar, double* Av, double* l, double* u) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const int N = P.N, ns = 3 * (N + 1), n = ns + 2 * N;
  const int gap0 = ns, inp0 = ns + 2 * (N + 1);
  const double x0[3] = {(double)x0g[0], (double)x0g[1], (double)x0g[2]};
  const Lin M = linearize(x0[2], (double)ulg[0], (double)ulg[1], P.dt);
  // A = I + E (E at (0,2), (1,2)), B, C of model.cpp:42-55, row-major
  const double A[9] = {1.0, 0.0, M.a02, 0.0, 1.0, M.a12, 0.0, 0.0, 1.0};
  const double Bm[6] = {M.b00, 0.0, M.b10, 0.0, M.b20, M.b21};
  const double Cv[3] = {M.c0, M.c1, M.c2};
  double hz[6] = {0, 0, 0, 0, 0, 0};
  if (hsg)
    for (int k = 0; k < 6; k++) hz[k] = (double)hsg[k];
  // P = blkdiag(Q x (N+1), R x N), dense blocks with explicit zeros (SparseBlockInit, :308-319)
  int nz = 0;
  for (int j = 0; j < n; j++) {
    Pc[j] = nz;
    if (j < ns) {
      const int bk = j / 3, c = j % 3;
      for (int rr = 0; rr < 3; rr++) { Pr[nz] = 3 * bk + rr; Pv[nz] = (rr == c) ? P.q[c] : 0.0; nz++; }
    } else {
      const int k = (j - ns) / 2, a = (j - ns) % 2;
      for (int rr = 0; rr < 2; rr++) { Pr[nz] = ns + 2 * k + rr; Pv[nz] = (rr == a) ? P.r[a] : 0.0; nz++; }
    }
  }
  Pc[n] = nz;
  // q (CreateGradientVector, :221-229): -Q x_ref[i] for i < N, the terminal stage reuses x_ref[N-1]
  for (int i = 0; i <= N; i++) {
    const int ri = i < N ? i : N - 1;
    const float* r = xrg + (size_t)ri * 3;
    for (int c = 0; c < 3; c++) q[3 * i + c] = -1 * P.q[c] * (double)r[c];
  }
  for (int k = 0; k < N; k++)
    for (int a = 0; a < 2; a++) q[ns + 2 * k + a] = -1 * P.r[a] * P.udes[a];
  // A (CreateLinearConstraintMatrix + UpdateLinearConstraintMatrix, :231-273)
  nz = 0;
  for (int j = 0; j < n; j++) {
    Ac[j] = nz;
    if (j < ns) {
      const int i = j / 3, c = j % 3;
      Ar[nz] = 3 * i + c; Av[nz] = -1; nz++;  // SparseBlockEye(-1), :244
      if (i < N)
        for (int rr = 0; rr < 3; rr++) { Ar[nz] = 3 * (i + 1) + rr; Av[nz] = A[rr * 3 + c]; nz++; }  // :247,269
      for (int h = 0; h < 2; h++) {  // gap rows :241,249,271
        const double coef = (i == 0 && !gap_active) ? 1.0 : (c == 2 ? 0.0 : hz[3 * h + c]);
        Ar[nz] = gap0 + 2 * i + h; Av[nz] = coef; nz++;
      }
    } else {
      const int k = (j - ns) / 2, a = (j - ns) % 2;
      for (int rr = 0; rr < 3; rr++) { Ar[nz] = 3 * (k + 1) + rr; Av[nz] = Bm[rr * 2 + a]; nz++; }  // :248,270
      Ar[nz] = inp0 + 2 * k + a; Av[nz] = 1; nz++;  // :253
    }
  }
  Ac[n] = nz;
  // l, u (:275-306): -x0 and -C on the dynamics rows, the gap rows, the input box
  for (int c = 0; c < 3; c++) { l[c] = -x0[c]; u[c] = -x0[c]; }
  for (int i = 1; i <= N; i++)
    for (int c = 0; c < 3; c++) { l[3 * i + c] = -Cv[c]; u[3 * i + c] = -Cv[c]; }
  for (int i = 0; i <= N; i++)
    for (int h = 0; h < 2; h++) {
      l[gap0 + 2 * i + h] = gap_active ? -hz[3 * h + 2] : -kInfty;  // :297-298 (commented upstream)
      u[gap0 + 2 * i + h] = kInfty;
    }
  for (int k = 0; k < N; k++)
    for (int a = 0; a < 2; a++) {
      l[inp0 + 2 * k + a] = (double)P.umin[a];
      u[inp0 + 2 * k + a] = (double)P.umax[a];
    }
}

hipError_t launch_assemble(const KParams& P, const float* x0, const float* ul, const float* xr,
                           const float* hs, int gap_active, int* Pc, int* Pr, double* Pv, double* q,
                           int* Ac, int* Ar, double* Av, double* l, double* u, hipStream_t s) {
  hipLaunchKernelGGL(assemble_kernel, dim3(1), dim3(64), 0, s, P, x0, ul, xr, hs, gap_active, Pc, Pr,
                     Pv, q, Ac, Ar, Av, l, u);
  return hipGetLastError();
}

}  // namespace f110qp

// solve_kernel.h — the MI355X (gfx950) hot path of the f110-mpc control tick (kernel templates;
// instantiated per (NUM, GAP) in solve_inst.hip, dispatched from f110qp_kernels.hip).
//
// One 64-lane wavefront per QP instance (one workgroup = one wave), B instances per launch.
// Per instance, fused in one launch:
//   1. Model::Linearize                      (reference src/model.cpp:30-59)      fp64, uniform
//   2. condensing of the tick's QP           (src/mpc.cpp:208-306)                closed form
//      The dynamics rows x_{i+1} = A x_i + B u_i + C are eliminated. A = I + E with E^2 = 0
//      (model.cpp:42-46), so Gamma's entries are affine in the stage distance and every
//      Hessian entry H = R + Gamma'Q Gamma is an O(1) polynomial sum: each lane builds its
//      rows of H in registers with no GEMM.
//   3. W = H^-1 by a symmetric Gauss-Jordan sweep, rows in VGPRs, pivot rows broadcast
//      by readlane.
//   4. the QP solve that OSQP does in the reference (src/mpc.cpp:133): a primal-dual active
//      set warm start (box rows) handed to a dual active-set method (Goldfarb-Idnani,
//      range-space form) on the condensed problem. The Cholesky factor of S_A = N_A' W N_A
//      lives in LDS; with gap rows the active normals' W n_j and S_A do too (box rows read
//      them straight from W). The triangular solves walk the active slots with one lane per
//      slot and readlane broadcasts. Box rows (mpc.cpp:253,281,290) and follow-the-gap rows
//      (mpc.cpp:249,271,297-298) are the constraint set.
//   5. two steps of iterative refinement whose residuals are evaluated in fp64 by an adjoint
//      (costate) recursion written as wave prefix/suffix scans, then an fp64 feasibility
//      re-check that re-enters step 4 if needed. Exact optimum to ~1e-9, not OSQP's 1e-3.
//   6. u* and the state rollout x* (MPC::UpdateSolvedTrajectory, mpc.cpp:145-159).
// Everything is recentred on (x0, y0): the dynamics and cost are translation invariant in
// (x, y) (model.cpp:42-55), which keeps fp32 exact to ~1e-6 for |x| ~ 50 m.
//
// Lane layout. Decision variable v = 2k + a (stage k, a = 0 speed, 1 steering) lives in
// lane v mod 64, register row r = v / 64: horizons N <= 32 use one row per lane (R = 1), N <=
// 48 two (R = 2, BASELINE config C4 is N = 40). Every per-variable quantity is an [R] register
// array, prefix/suffix scans carry across rows, active slots follow the same map.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "f110qp_kernels.h"

#include "linearize.h"

namespace f110qp {

// Diagnostic build only (-DF110QP_STAMPS): per-phase s_memtime deltas of every wave, read back
// with f110qp_read_stamps(). The shipped library never executes a stamp.
#ifdef F110QP_STAMPS
constexpr int kStampSlots = 16;
__device__ unsigned long long g_stamps[65536 * kStampSlots];  // stamps build: one TU (all instantiations)
#define STAMP(var) unsigned long long var = __builtin_amdgcn_s_memtime()
#define STAMP_SET(var) var = __builtin_amdgcn_s_memtime()
#define STAMP_ACC(acc, since) acc += __builtin_amdgcn_s_memtime() - (since)
#else
#define STAMP(var)
#define STAMP_SET(var)
#define STAMP_ACC(acc, since)
#endif

// ------------------------------------------------------------------------------------------
// wave helpers (64 lanes). Cross-lane traffic uses DPP (row shifts / quad permutes /
// row broadcasts) and readlane, never LDS: every helper is a handful of VALU instructions.
// They must be called from wave-uniform control flow (all 64 lanes active): readlane of an
// EXEC-disabled lane returns a stale register, and DPP treats disabled sources as invalid.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void wsync() { __syncthreads(); }

// DPP controls (gfx9 family encodings)
constexpr int DPP_ROW_SHR1 = 0x111, DPP_ROW_SHR2 = 0x112, DPP_ROW_SHR4 = 0x114, DPP_ROW_SHR8 = 0x118;
constexpr int DPP_ROW_BCAST15 = 0x142, DPP_ROW_BCAST31 = 0x143;
constexpr int DPP_QUAD_XOR1 = 0xB1;  // quad_perm [1,0,3,2]
constexpr int DPP_QUAD_XOR2 = 0x4E;  // quad_perm [2,3,0,1]
constexpr int DPP_QUAD_ODD = 0xF5;   // quad_perm [1,1,3,3]: every lane gets lane|1
constexpr int DPP_ROW_HALF_MIRROR = 0x141, DPP_ROW_MIRROR = 0x140;

template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ int dpp_i(int v) {  // lanes without a source read 0
  return __builtin_amdgcn_update_dpp(0, v, CTRL, ROWMASK, 0xf, false);
}
template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(dpp_i<CTRL, ROWMASK>(__float_as_int(v)));
}
template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ double dpp_d(double v) {
  int2 p = *reinterpret_cast<int2*>(&v);
  p.x = dpp_i<CTRL, ROWMASK>(p.x);
  p.y = dpp_i<CTRL, ROWMASK>(p.y);
  return *reinterpret_cast<double*>(&p);
}
// full-permutation DPPs (every lane has a source)
template <int CTRL>
__device__ __forceinline__ float perm_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xf, 0xf, false));
}
template <int CTRL>
__device__ __forceinline__ int perm_i(int v) {
  return __builtin_amdgcn_mov_dpp(v, CTRL, 0xf, 0xf, false);
}
template <int CTRL>
__device__ __forceinline__ double perm_d(double v) {
  int2 p = *reinterpret_cast<int2*>(&v);
  p.x = __builtin_amdgcn_mov_dpp(p.x, CTRL, 0xf, 0xf, false);
  p.y = __builtin_amdgcn_mov_dpp(p.y, CTRL, 0xf, 0xf, false);
  return *reinterpret_cast<double*>(&p);
}

__device__ __forceinline__ float readlane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ int readlane_i(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ double readlane_d(double v, int l) {
  int2 p = *reinterpret_cast<int2*>(&v);
  p.x = __builtin_amdgcn_readlane(p.x, l);
  p.y = __builtin_amdgcn_readlane(p.y, l);
  return *reinterpret_cast<double*>(&p);
}

// row r of a per-lane register array, r wave-uniform at run time
template <int R, typename T>
__device__ __forceinline__ T pick(const T (&x)[R], int r) {
  T v = x[0];
#pragma unroll
  for (int i = 1; i < R; i++) v = (r == i) ? x[i] : v;
  return v;
}
// value of slot / variable j (lane j mod 64, row j / 64), j wave-uniform
template <int R>
__device__ __forceinline__ float rl_f(const float (&x)[R], int j) {
  return readlane_f(pick<R>(x, j >> 6), j & 63);
}
template <int R>
__device__ __forceinline__ int rl_i(const int (&x)[R], int j) {
  return readlane_i(pick<R>(x, j >> 6), j & 63);
}

// inclusive prefix sum over the 64 lanes (row shifts, then row broadcasts 15 and 31)
__device__ __forceinline__ float scan_incl(float x) {
  x += dpp_f<DPP_ROW_SHR1>(x);
  x += dpp_f<DPP_ROW_SHR2>(x);
  x += dpp_f<DPP_ROW_SHR4>(x);
  x += dpp_f<DPP_ROW_SHR8>(x);
  x += dpp_f<DPP_ROW_BCAST15, 0xa>(x);
  x += dpp_f<DPP_ROW_BCAST31, 0xc>(x);
  return x;
}
__device__ __forceinline__ double scan_incl(double x) {
  x += dpp_d<DPP_ROW_SHR1>(x);
  x += dpp_d<DPP_ROW_SHR2>(x);
  x += dpp_d<DPP_ROW_SHR4>(x);
  x += dpp_d<DPP_ROW_SHR8>(x);
  x += dpp_d<DPP_ROW_BCAST15, 0xa>(x);
  x += dpp_d<DPP_ROW_BCAST31, 0xc>(x);
  return x;
}
__device__ __forceinline__ float lane63(float v) { return readlane_f(v, 63); }
__device__ __forceinline__ double lane63(double v) { return readlane_d(v, 63); }

// inclusive prefix over all 64R variables (variable order = row-major over (r, lane))
template <int R, typename T>
__device__ __forceinline__ void scan_incl_R(T (&x)[R]) {
  T carry = T(0);
#pragma unroll
  for (int r = 0; r < R; r++) {
    const T p = scan_incl(x[r]);
    x[r] = p + carry;
    if (r + 1 < R) carry += lane63(p);
  }
}
// inclusive suffix over all 64R variables: total - inclusive prefix + own
template <int R, typename T>
__device__ __forceinline__ void scan_suffix_incl_R(T (&x)[R]) {
  T p[R];
#pragma unroll
  for (int r = 0; r < R; r++) p[r] = x[r];
  scan_incl_R<R>(p);
  const T tot = lane63(p[R - 1]);
#pragma unroll
  for (int r = 0; r < R; r++) x[r] = tot - p[r] + x[r];
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
  return lane63(scan_incl(v));
}

// value of lane|1 (the steering lane of the stage pair)
__device__ __forceinline__ float odd_lane(float v) { return perm_f<DPP_QUAD_ODD>(v); }
__device__ __forceinline__ double odd_lane(double v) { return perm_d<DPP_QUAD_ODD>(v); }

// argmin of (val, idx) over the wave, result uniform; ties -> smaller idx
__device__ __forceinline__ void amin_step(float& v, int& i, float ov, int oi) {
  const bool take = (ov < v) || (ov == v && oi < i);
  v = take ? ov : v;
  i = take ? oi : i;
}
__device__ __forceinline__ void wave_argmin(float& val, int& idx) {
  amin_step(val, idx, perm_f<DPP_QUAD_XOR1>(val), perm_i<DPP_QUAD_XOR1>(idx));
  amin_step(val, idx, perm_f<DPP_QUAD_XOR2>(val), perm_i<DPP_QUAD_XOR2>(idx));
  amin_step(val, idx, perm_f<DPP_ROW_HALF_MIRROR>(val), perm_i<DPP_ROW_HALF_MIRROR>(idx));
  amin_step(val, idx, perm_f<DPP_ROW_MIRROR>(val), perm_i<DPP_ROW_MIRROR>(idx));
  float v0 = readlane_f(val, 0);
  int i0 = readlane_i(idx, 0);
  amin_step(v0, i0, readlane_f(val, 16), readlane_i(idx, 16));
  amin_step(v0, i0, readlane_f(val, 32), readlane_i(idx, 32));
  amin_step(v0, i0, readlane_f(val, 48), readlane_i(idx, 48));
  val = v0;
  idx = i0;
}

// Forward rollout of u (one value per variable) in fp64. Returns, for each row, the
// recentred state after the variable's stage k (i = k+1) in both lanes of the stage.
template <int R>
__device__ __forceinline__ void rollout_f64(const Lin& M, int lane, const double (&u)[R],
                                            double (&px)[R], double (&py)[R], double (&th)[R]) {
  const int a = lane & 1;
  const double beta = a ? M.b21 : M.b20;
  double s1[R], s2[R], s3[R];
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int k = 32 * r + (lane >> 1);
    s1[r] = beta * u[r];
    s2[r] = (double)k * s1[r];
    s3[r] = a ? 0.0 : u[r];
  }
  scan_incl_R<R>(s1);
  scan_incl_R<R>(s2);
  scan_incl_R<R>(s3);
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int k = 32 * r + (lane >> 1);
    const double P1 = odd_lane(s1[r]), P2 = odd_lane(s2[r]), V = odd_lane(s3[r]);
    const double i = (double)(k + 1);
    th[r] = M.th0 + i * M.c2 + P1;
    const double sth = i * M.th0 + M.c2 * (i * (i - 1.0) * 0.5) + (i - 1.0) * P1 - P2;
    px[r] = i * M.c0 + M.a02 * sth + M.b00 * V;
    py[r] = i * M.c1 + M.a12 * sth + M.b10 * V;
  }
}

// The linearisation's coefficients the fp32 GI uses, converted once and held in scalar registers
// (the GI loop read the fp64 Lin from LDS and converted it on every rollout and normal)
struct LinF {
  float a02, a12, b00, b10, b20, b21;
};
__device__ __forceinline__ float sgpr_f(float v) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}
__device__ __forceinline__ LinF lin_f32(const Lin& M) {
  LinF f;
  f.a02 = sgpr_f((float)M.a02); f.a12 = sgpr_f((float)M.a12);
  f.b00 = sgpr_f((float)M.b00); f.b10 = sgpr_f((float)M.b10);
  f.b20 = sgpr_f((float)M.b20); f.b21 = sgpr_f((float)M.b21);
  return f;
}

// Linear part of the rollout (Gamma w, zero initial state, no affine term), fp32.
template <int R>
__device__ __forceinline__ void rollout_lin_f32(const LinF& M, int lane, const float (&w)[R],
                                                float (&X)[R], float (&Y)[R]) {
  const int a = lane & 1;
  const float beta = a ? M.b21 : M.b20;
  const float a02 = M.a02, a12 = M.a12, b00 = M.b00, b10 = M.b10;
  float s1[R], s2[R], s3[R];
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int k = 32 * r + (lane >> 1);
    s1[r] = beta * w[r];
    s2[r] = (float)k * s1[r];
    s3[r] = a ? 0.f : w[r];
  }
  scan_incl_R<R>(s1);
  scan_incl_R<R>(s2);
  scan_incl_R<R>(s3);
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int k = 32 * r + (lane >> 1);
    const float P1 = odd_lane(s1[r]), P2 = odd_lane(s2[r]), V = odd_lane(s3[r]);
    const float sth = (float)k * P1 - P2;  // (i-1)P1 - P2 with i = k+1
    X[r] = a02 * sth + b00 * V;
    Y[r] = a12 * sth + b10 * V;
  }
}

template <int R>
__device__ __forceinline__ void rollout_lin_f32(const Lin& M, int lane, const float (&w)[R],
                                                float (&X)[R], float (&Y)[R]) {
  const LinF f = {(float)M.a02, (float)M.a12, (float)M.b00, (float)M.b10, (float)M.b20, (float)M.b21};
  rollout_lin_f32<R>(f, lane, w, X, Y);
}

// Gradient of the tracking objective (mpc.cpp:208-229 cost) minus the gap-row multiplier
// terms, at u, by the costate recursion lambda_i = Q(x_i - r_i) - mu_i n_i + A' lambda_{i+1},
// written as suffix scans. px,py,th are the variable-stage states from rollout_f64.
template <int R>
__device__ __forceinline__ void grad_f64(const Lin& M, const KParams& P, int lane, int N,
                                         const double (&u)[R], const double (&px)[R],
                                         const double (&py)[R], const double (&th)[R],
                                         const double (&rx)[R], const double (&ry)[R],
                                         const double (&rth)[R], const double (&gmx)[R],
                                         const double (&gmy)[R], double (&g)[R]) {
  const int a = lane & 1;
  double ex[R], ey[R], et[R], lx[R], ly[R];
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int k = 32 * r + (lane >> 1);
    const bool contrib = (a == 1) && (k < N);
    const double i = (double)(k + 1);
    ex[r] = contrib ? P.q[0] * (px[r] - rx[r]) - gmx[r] : 0.0;
    ey[r] = contrib ? P.q[1] * (py[r] - ry[r]) - gmy[r] : 0.0;
    et[r] = contrib ? P.q[2] * (th[r] - rth[r]) : 0.0;
    lx[r] = i * ex[r];
    ly[r] = i * ey[r];
  }
  scan_suffix_incl_R<R>(ex);
  scan_suffix_incl_R<R>(lx);
  scan_suffix_incl_R<R>(ey);
  scan_suffix_incl_R<R>(ly);
  scan_suffix_incl_R<R>(et);
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int k = 32 * r + (lane >> 1);
    const double i = (double)(k + 1);
    const double lth = et[r] + M.a02 * (lx[r] - i * ex[r]) + M.a12 * (ly[r] - i * ey[r]);
    const double gv = a ? (P.r[1] * (u[r] - P.udes[1]) + M.b21 * lth)
                        : (P.r[0] * (u[r] - P.udes[0]) + M.b00 * ex[r] + M.b10 * ey[r] + M.b20 * lth);
    g[r] = (k < N) ? gv : 0.0;
  }
}

// H y in fp64 (H = R + Gamma'Q Gamma, the condensed Hessian): the linear rollout of y and the
// costate of its Q-weighted states (grad_f64 with no reference, no affine term and no u_des).
template <int R>
__device__ __forceinline__ void hv_f64(const Lin& M, const KParams& P, int lane, int N,
                                       const double (&y)[R], double (&hy)[R]) {
  Lin ML = M;
  ML.th0 = 0.0; ML.c0 = 0.0; ML.c1 = 0.0; ML.c2 = 0.0;
  double px[R], py[R], th[R];
  rollout_f64<R>(ML, lane, y, px, py, th);
  const int a = lane & 1;
  double ex[R], ey[R], et[R], lx[R], ly[R];
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int k = 32 * r + (lane >> 1);
    const bool contrib = (a == 1) && (k < N);
    const double i = (double)(k + 1);
    ex[r] = contrib ? P.q[0] * px[r] : 0.0;
    ey[r] = contrib ? P.q[1] * py[r] : 0.0;
    et[r] = contrib ? P.q[2] * th[r] : 0.0;
    lx[r] = i * ex[r];
    ly[r] = i * ey[r];
  }
  scan_suffix_incl_R<R>(ex);
  scan_suffix_incl_R<R>(lx);
  scan_suffix_incl_R<R>(ey);
  scan_suffix_incl_R<R>(ly);
  scan_suffix_incl_R<R>(et);
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int k = 32 * r + (lane >> 1);
    const double i = (double)(k + 1);
    const double lth = et[r] + ML.a02 * (lx[r] - i * ex[r]) + ML.a12 * (ly[r] - i * ey[r]);
    const double hv = a ? (P.r[1] * y[r] + ML.b21 * lth)
                        : (P.r[0] * y[r] + ML.b00 * ex[r] + ML.b10 * ey[r] + ML.b20 * lth);
    hy[r] = (k < N) ? hv : 0.0;
  }
}

// ------------------------------------------------------------------------------------------
// shared memory of one wave / one QP
// ------------------------------------------------------------------------------------------
template <int NUM, bool GAP>
struct Smem {
  static constexpr int R = (NUM + 63) / 64;
  static constexpr int VN = 64 * R;      // per-variable vectors (one entry per lane and row)
  static constexpr int NST = NUM / 2 + 1;  // stages 0..N
  // W = H^-1, row-major (symmetric: row p == column p). Rows padded to NUM + 4: matvec_W reads a
  // lane's own row as float4, and a stride of NUM + 4 words puts 16 such lanes on distinct banks
  alignas(16) float W[NUM][NUM + 4];
  float L[NUM][NUM + 1];           // Cholesky factor of S_A (lower), slots x slots
  // gap rows only: V[slot][var] = W n_slot. With box rows alone V and S_A = N_A' W N_A are
  // signed entries of W (n_j = +-e_var) and are read from W directly.
  alignas(16) float V[GAP ? NUM : 1][NUM + 4];  // rows padded as W's (row reads in float4)
  alignas(16) float vec[VN];       // broadcast scratch (one entry per variable)
  float vec2[VN];
  float stX[NST], stY[NST];        // per-stage linear rollout (stage 1..N)
  double rx[VN], ry[VN];           // recentred reference of the variable's stage (fp64: x_ref - x0
                                   // of two floats is not always a float)
  float rth[VN];
  double cmult[3 * VN];            // multiplier per constraint id (fp64: the refinement's)
  alignas(16) float prow[NUM];     // box PDAS: pivot row of T broadcast (pivot_T)
  alignas(16) float yb[NUM];       // box PDAS: right-hand side broadcast (matvec_T)
  double d64[VN];
  double sx64[NST], sy64[NST];
  Lin M;                           // linearisation of this QP (uniform)
};

// constraint ids: id = 3*var + t, t = 0 box lower (n = e_var), 1 box upper (n = -e_var),
// 2 gap row (stage var/2+1, side var&1)
__device__ __forceinline__ float box_sign(int id) { return (id - 3 * (id / 3) == 0) ? 1.f : -1.f; }

constexpr int kTriBlock = 8;  // steps per block of the triangular solves (loads hoisted)

// l = L^-1 v, one lane per active slot (slot j: lane j mod 64, row j / 64); L read from LDS.
// A plain q-step loop: the slot count is uniform, each step is mul -> readlane -> fma.
template <int NUM, bool GAP, int R>
__device__ __forceinline__ void tri_forward(Smem<NUM, GAP>& sm, int lane, int q,
                                            const float (&rdiag)[R], const float (&v)[R],
                                            float (&lv)[R]) {
  float acc[R];
  const float* Lrow[R];
#pragma unroll
  for (int r = 0; r < R; r++) {
    acc[r] = v[r];
    lv[r] = 0.f;
    const int row = 64 * r + lane;
    Lrow[r] = sm.L[row < NUM ? row : NUM - 1];
  }
  const int q0 = q < 64 ? q : 64;
  // blocks of kTriBlock steps with the block's L loads issued first, off the dependent
  // mul -> readlane -> fma chain (readlane is convergent: the compiler does not runtime-unroll
  // the rolled loop, whose every step then waits for its own LDS load)
  int kk = 0;
  for (; kk + kTriBlock <= q0; kk += kTriBlock) {
    float lb[kTriBlock][R];
#pragma unroll
    for (int j = 0; j < kTriBlock; j++)
#pragma unroll
      for (int r = 0; r < R; r++) lb[j][r] = Lrow[r][kk + j];
#pragma unroll
    for (int j = 0; j < kTriBlock; j++) {
      const float t = acc[0] * rdiag[0];
      const float lk = readlane_f(t, kk + j);
      lv[0] = (lane == kk + j) ? t : lv[0];
#pragma unroll
      for (int r = 0; r < R; r++) acc[r] = fmaf(-lb[j][r], lk, acc[r]);
    }
  }
  for (; kk < q0; kk++) {
    const float t = acc[0] * rdiag[0];
    const float lk = readlane_f(t, kk);
    lv[0] = (lane == kk) ? t : lv[0];
#pragma unroll
    for (int r = 0; r < R; r++) acc[r] = fmaf(-Lrow[r][kk], lk, acc[r]);
  }
  if constexpr (R > 1) {
    for (int kk = 64; kk < q; kk++) {
      const float t = acc[1] * rdiag[1];
      const float lk = readlane_f(t, kk - 64);
      lv[1] = (lane == kk - 64) ? t : lv[1];
#pragma unroll
      for (int r = 1; r < R; r++) acc[r] = fmaf(-Lrow[r][kk], lk, acc[r]);
    }
  }
}

// r = L^-T l (backward substitution, column-oriented)
template <int NUM, bool GAP, int R>
__device__ __forceinline__ void tri_backward(Smem<NUM, GAP>& sm, int lane, int q,
                                             const float (&rdiag)[R], const float (&l)[R],
                                             float (&out)[R]) {
  float acc[R];
  int col[R];
#pragma unroll
  for (int r = 0; r < R; r++) {
    acc[r] = l[r];
    out[r] = 0.f;
    const int c = 64 * r + lane;
    col[r] = c < NUM ? c : NUM - 1;
  }
  if constexpr (R > 1) {
    for (int jj = q - 1; jj >= 64; jj--) {
      const float t = acc[1] * rdiag[1];
      const float rj = readlane_f(t, jj - 64);
      out[1] = (lane == jj - 64) ? t : out[1];
#pragma unroll
      for (int r = 0; r < R; r++) acc[r] = fmaf(-sm.L[jj][col[r]], rj, acc[r]);
    }
  }
  const int q0 = q < 64 ? q : 64;
  int jj = q0 - 1;
  for (; jj - kTriBlock + 1 >= 0; jj -= kTriBlock) {  // blocks as in tri_forward
    float lb[kTriBlock];
#pragma unroll
    for (int j = 0; j < kTriBlock; j++) lb[j] = sm.L[jj - j][col[0]];
#pragma unroll
    for (int j = 0; j < kTriBlock; j++) {
      const float t = acc[0] * rdiag[0];
      const float rj = readlane_f(t, jj - j);
      out[0] = (lane == jj - j) ? t : out[0];
      acc[0] = fmaf(-lb[j], rj, acc[0]);
    }
  }
  for (; jj >= 0; jj--) {
    const float t = acc[0] * rdiag[0];
    const float rj = readlane_f(t, jj);
    out[0] = (lane == jj) ? t : out[0];
    acc[0] = fmaf(-sm.L[jj][col[0]], rj, acc[0]);
  }
}

// Delete slot kd from S_A = L L' (q slots before the call; rd = this lane's 1/L[j][j]).
// The rows below kd move up one; each of them then carries one entry right of its diagonal,
// which q - 1 - kd Givens rotations on the column pairs (j, j + 1) remove: the updated factor in
// O(q^2) work and q - 1 - kd short dependent steps (hypot -> readlane -> 4 FMAs), instead of the
// O(q^3) refactorisation of S_A with its q dependent column steps. After the shift every lane
// touches only its own row, so the rotation loop needs no barrier.
template <int NUM, bool GAP, int R>
__device__ __forceinline__ void chol_delete(Smem<NUM, GAP>& sm, int lane, int q, int kd,
                                            float (&rd)[R]) {
  constexpr int kChunk = 8;
  for (int c0 = 0; c0 < q; c0 += kChunk) {  // row s <- row s + 1 (columns 0..s + 1)
    float t[R][kChunk];
#pragma unroll
    for (int r = 0; r < R; r++) {
      const int row = 64 * r + lane;
      const bool mv = row >= kd && row < q - 1;
#pragma unroll
      for (int cc = 0; cc < kChunk; cc++) {
        const int c = c0 + cc;
        t[r][cc] = (mv && c < q && c <= row + 1) ? sm.L[row + 1][c] : 0.f;
      }
    }
    wsync();
#pragma unroll
    for (int r = 0; r < R; r++) {
      const int row = 64 * r + lane;
      const bool mv = row >= kd && row < q - 1;
#pragma unroll
      for (int cc = 0; cc < kChunk; cc++) {
        const int c = c0 + cc;
        if (mv && c < q && c <= row + 1) sm.L[row][c] = t[r][cc];
      }
    }
    wsync();
  }
  float carry[R];  // this row's entry in column j (rotated so far)
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int row = 64 * r + lane;
    carry[r] = (row >= kd && row < q - 1) ? sm.L[row < NUM ? row : NUM - 1][kd] : 0.f;
  }
  for (int j = kd; j < q - 1; j++) {
    float y[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
      const int row = 64 * r + lane;
      y[r] = (row >= j && row < q - 1) ? sm.L[row][j + 1] : 0.f;
    }
    const float a = rl_f<R>(carry, j), b = rl_f<R>(y, j);
    const float h = sqrtf(a * a + b * b);
    const float ih = 1.f / h;  // one division per rotation (cs, sn and the new 1 / L[j][j])
    const float cs = a * ih, sn = b * ih;
#pragma unroll
    for (int r = 0; r < R; r++) {
      const int row = 64 * r + lane;
      if (row > j && row < q - 1) {
        sm.L[row][j] = fmaf(cs, carry[r], sn * y[r]);
        carry[r] = fmaf(cs, y[r], -sn * carry[r]);
      }
      if (row == j) {
        sm.L[row][j] = h;
        rd[r] = ih;
      }
    }
  }
}

// y = W x with x in sm.vec; W symmetric so the lane reads column v (consecutive addresses
// across lanes, conflict free). Variables >= NUM get 0.
#ifndef F110QP_MATVEC_SPLIT
#define F110QP_MATVEC_SPLIT 1
#endif
template <int NUM, bool GAP, int R>
__device__ __forceinline__ void matvec_W(Smem<NUM, GAP>& sm, int lane, float (&y)[R]) {
  int c[R];
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int v = 64 * r + lane;
    c[r] = v < NUM ? v : NUM - 1;
    y[r] = 0.f;
  }
#if F110QP_MATVEC_SPLIT
  // y_c = sum_j W[c][j] x_j over the lane's own row (W symmetric): four entries of the row and of
  // the broadcast x per 16-B LDS read, four independent accumulator chains (the column form was
  // NUM dependent FMAs and 2 NUM LDS reads per call, one call per GI step)
  static_assert(NUM % 4 == 0, "matvec_W reads in float4");
  float y1[R], y2[R], y3[R];
  const float4* wr[R];
#pragma unroll
  for (int r = 0; r < R; r++) {
    y1[r] = 0.f; y2[r] = 0.f; y3[r] = 0.f;
    wr[r] = reinterpret_cast<const float4*>(sm.W[c[r]]);
  }
  const float4* x4 = reinterpret_cast<const float4*>(sm.vec);
#pragma unroll
  for (int j = 0; j < NUM / 4; j++) {
    const float4 xj = x4[j];
#pragma unroll
    for (int r = 0; r < R; r++) {
      const float4 wv = wr[r][j];
      y[r] = fmaf(wv.x, xj.x, y[r]);
      y1[r] = fmaf(wv.y, xj.y, y1[r]);
      y2[r] = fmaf(wv.z, xj.z, y2[r]);
      y3[r] = fmaf(wv.w, xj.w, y3[r]);
    }
  }
#pragma unroll
  for (int r = 0; r < R; r++) y[r] = (y[r] + y1[r]) + (y2[r] + y3[r]);
#else
#pragma unroll
  for (int j = 0; j < NUM; j++) {
    const float xj = sm.vec[j];
#pragma unroll
    for (int r = 0; r < R; r++) y[r] = fmaf(sm.W[j][c[r]], xj, y[r]);
  }
#endif
#pragma unroll
  for (int r = 0; r < R; r++) y[r] = (64 * r + lane < NUM) ? y[r] : 0.f;
}

// n_j' w for the active slot with id slot_id (w in sm.vec2 by variable, gap rows from the
// per-stage linear rollout in sm.stX/stY).
template <int NUM, bool GAP>
__device__ __forceinline__ float slot_dot(Smem<NUM, GAP>& sm, int slot_id, float ga0, float ga1,
                                          float gb0, float gb1) {
  const int owner = slot_id / 3, t = slot_id - 3 * owner;
  if (t == 0) return sm.vec2[owner];
  if (t == 1) return -sm.vec2[owner];
  const int st = (owner >> 1) + 1;
  return ((owner & 1) ? ga1 : ga0) * sm.stX[st] + ((owner & 1) ? gb1 : gb0) * sm.stY[st];
}

// column c of V[j] = W n_j for uniform slot j with id sid_j
template <int NUM, bool GAP>
__device__ __forceinline__ float vcol(Smem<NUM, GAP>& sm, int j, int sid_j, int c) {
  if constexpr (GAP) return sm.V[j][c];
  else return box_sign(sid_j) * sm.W[sid_j / 3][c];
}

// One pivot of the symmetric sweep operator (Goodnight 1979) on the rows held by this lane:
//   a_ij -= a_ip a_pj / a_pp ; a_ip /= a_pp ; a_pj /= a_pp ; a_pp = -1/a_pp.
// The pivot row is broadcast by readlane; the pivot row's own update folds into the common FMA
// with f = 1 - 1/a_pp. After all pivots the rows hold -H^-1. P is a template constant so every
// register index is static (no scratch).
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NUM, int R, int P>
__device__ __forceinline__ void sweep_step(float (&hrow)[R][NUM], int lane) {
  constexpr int PR = P / 64, PL = P % 64;
  // pivot row broadcast by readlane (lane PL, static register index) -> SGPR operands
  float rk[NUM];
#pragma unroll
  for (int j = 0; j < NUM; j++) rk[j] = readlane_f(hrow[PR][j], PL);
  const float inv = __builtin_amdgcn_rcpf(rk[P]);  // 1 ulp; the fp64 refinement absorbs it
#pragma unroll
  for (int r = 0; r < R; r++) {
    const bool piv = (r == PR) && (lane == PL);
    const float hp = hrow[r][P];
    const float f = piv ? (1.f - inv) : hp * inv;
    const f32x2 nf = {-f, -f};
#pragma unroll
    for (int j = 0; j < NUM; j += 2) {  // packed FMA over column pairs (v_pk_fma_f32)
      const f32x2 rr = {rk[j], rk[j + 1]};
      f32x2 h = {hrow[r][j], hrow[r][j + 1]};
      h = __builtin_elementwise_fma(nf, rr, h);
      hrow[r][j] = h.x;
      hrow[r][j + 1] = h.y;
    }
    hrow[r][P] = piv ? -inv : hp * inv;
  }
}

template <int NUM, int R, int P>
struct Sweep {
  static __device__ __forceinline__ void run(float (&hrow)[R][NUM], int lane) {
    sweep_step<NUM, R, P>(hrow, lane);
    Sweep<NUM, R, P + 1>::run(hrow, lane);
  }
};
template <int NUM, int R>
struct Sweep<NUM, R, NUM> {
  static __device__ __forceinline__ void run(float (&)[R][NUM], int) {}
};

// ---- box rows: the partially swept Hessian T (rows in registers) --------------------------
// T = SWP_F(H), the sweep of H on the free set F: T_FF = -(H_FF)^-1, T_FA = H_FF^-1 H_FA and
// T_AA = H_AA - H_AF H_FF^-1 H_FA (the full sweep above leaves F = all, T = -H^-1). Moving one
// variable k between F and the active set A is one sweep (sg = +1, A -> F) or reverse sweep
// (sg = -1, F -> A) pivot on k: a rank-1 update of the register rows, no factorization, and a
// box-constrained solve of a guess A is one product with T (matvec_T).
// The pivot row is broadcast through LDS with its entry k replaced by T_kk - sg, so the common
// FMA leaves sg * T_ik / T_kk in column k of every other row. The pivot lane zeroes its own row
// first, so the same FMA (f = -sg / T_kk) writes sg T_kj / T_kk there exactly (folding it in as
// T_kj - (1 - sg / T_kk) T_kj cancels when |T_kk| >> 1: 5e-4 relative on stiff QPs); its
// diagonal entry then ends sg away from -1/T_kk: the exact diagonal is carried in dg, and ed
// (+-1 or 0, exact in fp32) records the offset of the register copy, which matvec_T removes.
template <int NUM, bool GAP, int R>
__device__ __forceinline__ void pivot_T(Smem<NUM, GAP>& sm, float (&h)[R][NUM], float (&dg)[R],
                                        float (&ed)[R], int lane, const int (&vv)[R], int k,
                                        float sg) {
  const int kl = k & 63, kr = k >> 6;
  if (lane == kl) {
#pragma unroll
    for (int r = 0; r < R; r++) {
      if (r == kr) {
#pragma unroll
        for (int j = 0; j < NUM; j += 4) {
          *reinterpret_cast<f32x4*>(&sm.prow[j]) = f32x4{h[r][j], h[r][j + 1], h[r][j + 2], h[r][j + 3]};
          h[r][j] = 0.f; h[r][j + 1] = 0.f; h[r][j + 2] = 0.f; h[r][j + 3] = 0.f;
        }
        sm.prow[k] = dg[r] - sg;
      }
    }
  }
  wsync();
  float rk[NUM];
#pragma unroll
  for (int j = 0; j < NUM; j += 4) {
    const f32x4 v4 = *reinterpret_cast<const f32x4*>(&sm.prow[j]);
    rk[j] = v4.x; rk[j + 1] = v4.y; rk[j + 2] = v4.z; rk[j + 3] = v4.w;
  }
  float tk[R];  // T_ki = T_ik (symmetric) of this lane's rows
#pragma unroll
  for (int r = 0; r < R; r++) tk[r] = (vv[r] < NUM) ? sm.prow[vv[r]] : 0.f;
  const float inv = __builtin_amdgcn_rcpf(readlane_f(pick<R>(dg, kr), kl));
#pragma unroll
  for (int r = 0; r < R; r++) {
    const bool piv = (r == kr) && (lane == kl);
    const float f = piv ? -sg * inv : tk[r] * inv;  // pivot row zeroed above: sg T_kj / T_kk exactly
    const f32x2 nf = {-f, -f};
#pragma unroll
    for (int j = 0; j < NUM; j += 2) {
      f32x2 x = {h[r][j], h[r][j + 1]};
      x = __builtin_elementwise_fma(nf, f32x2{rk[j], rk[j + 1]}, x);
      h[r][j] = x.x;
      h[r][j + 1] = x.y;
    }
    dg[r] = piv ? -inv : fmaf(-f, tk[r], dg[r]);
    ed[r] = piv ? sg : ed[r];  // register diagonal sg (T_kk - sg) / T_kk = sg - 1/T_kk
  }
  wsync();  // prow is rewritten by the next pivot
}

// x = T y (y one entry per variable, zero outside the valid rows)
template <int NUM, bool GAP, int R>
__device__ __forceinline__ void matvec_T(Smem<NUM, GAP>& sm, const float (&h)[R][NUM],
                                         const float (&ed)[R], const int (&vv)[R],
                                         const float (&y)[R], float (&x)[R]) {
#pragma unroll
  for (int r = 0; r < R; r++)
    if (vv[r] < NUM) sm.yb[vv[r]] = y[r];
  wsync();
  float yb[NUM];
#pragma unroll
  for (int j = 0; j < NUM; j += 4) {
    const f32x4 v4 = *reinterpret_cast<const f32x4*>(&sm.yb[j]);
    yb[j] = v4.x; yb[j + 1] = v4.y; yb[j + 2] = v4.z; yb[j + 3] = v4.w;
  }
#pragma unroll
  for (int r = 0; r < R; r++) {
    f32x2 a0 = {0.f, 0.f}, a1 = {0.f, 0.f};
#pragma unroll
    for (int j = 0; j < NUM; j += 4) {
      a0 = __builtin_elementwise_fma(f32x2{h[r][j], h[r][j + 1]}, f32x2{yb[j], yb[j + 1]}, a0);
      a1 = __builtin_elementwise_fma(f32x2{h[r][j + 2], h[r][j + 3]}, f32x2{yb[j + 2], yb[j + 3]}, a1);
    }
    x[r] = fmaf(-ed[r], y[r], (a0.x + a0.y) + (a1.x + a1.y));
  }
  wsync();  // yb is rewritten by the next product
}

// fp64 iterative refinement of the fp32 solve (steps 4a/5): each step evaluates the residual in
// fp64 (rollout + adjoint) and corrects through the fp32 T / W. Stiff problems (large dt x N: H's
// condition number grows like (N dt v)^2) contract more slowly per step; the fuzz test over the
// ABI's range (dt 0.05, N = 40) needed more than the two steps that suffice at the shipped
// dt = 0.01, so up to four, stopping once the fp32 correction is at its noise level.
constexpr int kRefineSteps = 4;
constexpr float kRefineTol = 2e-6f;
// GI's final point (gap rows): refined until its fp64 KKT residual is small (at most kRefineMax
// residual evaluations), then certified by duality. For a point u that satisfies every row and
// holds its active rows to 1e-9 relative (fp64), with the multipliers mu+ = max(mu, 0) of its
// active rows and rho = H u + g - N_A mu+: |u - u*'|_H^2 <= rho'W rho (W = H^-1) for the optimum
// u*' of the reference QP with each row bound moved by u's own residual on it (<= 1e-9 relative:
// a backward error far below the float32 rounding of the inputs), and |e|_2 <= |e|_H / sqrt(lambda)
// with lambda = min(r) <= lambda_min(H) (H = R + Gamma'Q Gamma). SOLVED when rho'W rho, bounded
// from above in fp64 (an fp64 Hessian product corrects the fp32 W's product, hv_f64), is <=
// lambda (kCertTauW max(1, |u|_inf))^2. The W-norm keeps the bound at sqrt(kappa(H)) times the
// rounding of an exact point, where |rho|_2 / lambda would be kappa times (stiff QPs, kappa ~ 4e5
// at N = 48, dt = 0.05). Anything else is SOLVED_INACCURATE and goes to the fp64 re-check
// (gi64_kernel.h).
constexpr int kRefineMax = 8;
constexpr double kCertTauW = 1e-6;
// box path's fp64 PDAS (step 4a'): passes, HIK passes before the least-index rule, flips pivoted
// in place before T is rebuilt, refinement steps and tolerance per pass
constexpr int kHikPasses = 8;
constexpr int kIncPivots = 8;
constexpr int kRobSteps = 12;
constexpr float kRobTol = 1e-9f;     // converged
constexpr float kRobTight = 1e-14f;  // keep going to fp64 level: the multipliers r1_A = (Hu + g)_A
                                     // carry ||H_AF|| times the error left in u_F
template <int NUM>
constexpr int kRobPasses = kHikPasses + NUM;

template <int NUM, bool GAP>
__device__ __forceinline__ void solve_qp(Smem<NUM, GAP>& sm, const int b, const KParams& P,
                                         const float* __restrict__ x0g,
                                         const float* __restrict__ ulg,
                                         const float* __restrict__ xrg,
                                         const float* __restrict__ hsg,
                                         float* __restrict__ uout,
                                         float* __restrict__ xout,
                                         int* __restrict__ status_out,
                                         int* __restrict__ iters_out,
                                         double* __restrict__ Hdbg,
                                         double* __restrict__ gdbg,
                                         const WarmState& ws, const ObjOut& oo,
                                         const int prep_slot = -1) {
  constexpr int R = (NUM + 63) / 64;
  const int lane = threadIdx.x;
  const int N = P.N;
  const int NU = 2 * N;
  const int a = lane & 1;    // 0 = speed v, 1 = steering
  int vv[R], kk[R], cl[R];   // variable, its input stage, clamped LDS column
  bool valid[R];
#pragma unroll
  for (int r = 0; r < R; r++) {
    vv[r] = 64 * r + lane;
    kk[r] = vv[r] >> 1;
    valid[r] = vv[r] < NU;
    cl[r] = vv[r] < NUM ? vv[r] : NUM - 1;
  }

  STAMP(t_start);
#ifdef F110QP_STAMPS
  unsigned long long acc_refine = 0, acc_s1 = 0, acc_w = 0, acc_vj = 0, acc_tri = 0, acc_z = 0,
                     acc_step = 0, acc_upd = 0, acc_pdas = 0;
#endif
  // ---- 1. inputs + Model::Linearize ----------------------------------------------------
  const float fX0 = x0g[3 * b + 0], fY0 = x0g[3 * b + 1], fTH0 = x0g[3 * b + 2];
  const float ul0 = ulg[2 * b + 0], ul1 = ulg[2 * b + 1];
  const double X0 = (double)fX0, Y0 = (double)fY0;
  // The reference point of each variable's state stage (i = k+1; the terminal stage reuses
  // x_ref[N-1], mpc.cpp:228) is loaded here and consumed after the inverse: H depends only on
  // the linearisation point, so the load latency hides behind the Hessian and the sweep.
  float xrv[R][3], x00[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int r = 0; r < R; r++) {
    xrv[r][0] = 0.f; xrv[r][1] = 0.f; xrv[r][2] = 0.f;
    if (valid[r]) {
      const int ri = (kk[r] + 1 < N) ? kk[r] + 1 : N - 1;
      const float* xr = xrg + ((size_t)b * P.xr_stride + ri) * 3;
      xrv[r][0] = xr[0]; xrv[r][1] = xr[1]; xrv[r][2] = xr[2];
    }
  }
  if (lane == 0) {
    const float* xq = xrg + (size_t)b * P.xr_stride * 3;
    x00[0] = xq[0]; x00[1] = xq[1]; x00[2] = xq[2];
  }
  {
    const Lin M = linearize((double)fTH0, (double)ul0, (double)ul1, P.dt);
    if (lane == 0) sm.M = M;
  }
  const float umin0 = P.umin[0], umin1 = P.umin[1], umax0 = P.umax[0], umax1 = P.umax[1];
  float lb[R], ub[R];
#pragma unroll
  for (int r = 0; r < R; r++) {
    lb[r] = valid[r] ? (a ? umin1 : umin0) : -3.0e38f;
    ub[r] = valid[r] ? (a ? umax1 : umax0) : 3.0e38f;
  }
  const float il0 = 1.f / (1.f + fabsf(umin0)), il1 = 1.f / (1.f + fabsf(umin1));
  const float iu0 = 1.f / (1.f + fabsf(umax0)), iu1 = 1.f / (1.f + fabsf(umax1));

  // gap rows: a*x + b*y >= -(c+0.5) (constraints.cpp:255-264, mpc.cpp:297-298), recentred
  float ga0 = 0.f, ga1 = 0.f, gb0 = 0.f, gb1 = 0.f;
  double gbeta0 = 0.0, gbeta1 = 0.0;
  bool infeasible0 = false;
  if (GAP) {
    const float* h6 = hsg + 6 * b;
    ga0 = h6[0]; gb0 = h6[1]; ga1 = h6[3]; gb1 = h6[4];
    gbeta0 = -(double)h6[2] - (double)ga0 * X0 - (double)gb0 * Y0;
    gbeta1 = -(double)h6[5] - (double)ga1 * X0 - (double)gb1 * Y0;
    // the stage-0 rows are constant (x0 lies on both lines): infeasible only if violated
    if (gbeta0 > 1e-9 * (1.0 + fabs((double)h6[2])) || gbeta1 > 1e-9 * (1.0 + fabs((double)h6[5])))
      infeasible0 = true;
    if (!(isfinite(gbeta0) && isfinite(gbeta1))) infeasible0 = true;
  }
  wsync();

  // W cache: per slot b (warm start), per group (grouped mode), or the group slot a prepare
  // launch fills (prep_slot >= 0). Does the cached W belong to this linearisation point?
  const bool warm = ws.W != nullptr && Hdbg == nullptr;
  const bool grp = ws.group != nullptr;
  const bool prep = prep_slot >= 0;
  int wslot = b;
  if (grp) {
    const int g = __builtin_amdgcn_readfirstlane(ws.group[b]);
    wslot = (g >= 0 && g < ws.ngroups) ? g : -1;
  }
  if (prep) wslot = prep_slot;
  bool whit = false, wvalid = false;
  if (warm && !prep && wslot >= 0) {
    const unsigned* key = ws.key + 4 * wslot;
    wvalid = key[3] == 1u;
    whit = wvalid && key[0] == __float_as_uint(fTH0) && key[1] == __float_as_uint(ul0) &&
           key[2] == __float_as_uint(ul1);
  }
  // previous tick's active set seeds the PDAS guess only when the linearisation point repeats:
  // on the closed-loop C5 stream (theta0 changes every tick) a stale seed measured 1.62 vs 1.49
  // equality solves per QP cold, since its pivots must be undone
  const bool seed_act = ws.act != nullptr && !grp && whit;
  STAMP(t_lin);
  // ---- 2a. (run after the inverse) non-finite check, recentred references, gradient at u = 0
  // by the fp64 adjoint, and the free response of the gap rows
  bool numerical = false;
  float cgap[R], gnorm = 1.f;
  auto inputs_and_gradient = [&]() {
    // non-finite data -> F110QP_NUMERICAL with NaN outputs (e.g. the NaN x_ref the planning
    // stage emits for a scenario without a valid candidate, where the reference skips
    // MPC::Update)
    bool bad = !(isfinite(fX0) && isfinite(fY0) && isfinite(fTH0) && isfinite(ul0) && isfinite(ul1));
    if (lane == 0) bad = bad || !(isfinite(x00[0]) && isfinite(x00[1]) && isfinite(x00[2]));
    const Lin M = sm.M;
    double zero[R], px0[R], py0[R], th0s[R], rxd[R], ryd[R], rthd[R], g64[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
      if (valid[r]) bad = bad || !(isfinite(xrv[r][0]) && isfinite(xrv[r][1]) && isfinite(xrv[r][2]));
      zero[r] = 0.0;
      rxd[r] = valid[r] ? (double)xrv[r][0] - X0 : 0.0;  // recentred in fp64
      ryd[r] = valid[r] ? (double)xrv[r][1] - Y0 : 0.0;
      rthd[r] = (double)xrv[r][2];
      sm.rx[vv[r]] = rxd[r]; sm.ry[vv[r]] = ryd[r]; sm.rth[vv[r]] = xrv[r][2];
      cgap[r] = 0.f;
    }
    numerical = __ballot(bad) != 0ull;
    rollout_f64<R>(M, lane, zero, px0, py0, th0s);
    // cross-lane helpers run with all 64 lanes active (variables >= 2N contribute zeros)
    grad_f64<R>(M, P, lane, N, zero, px0, py0, th0s, rxd, ryd, rthd, zero, zero, g64);
#pragma unroll
    for (int r = 0; r < R; r++) {
      const double gv = valid[r] ? g64[r] : 0.0;
      sm.vec[vv[r]] = (float)gv;
      if (Hdbg && valid[r]) gdbg[(size_t)b * NU + vv[r]] = gv;
    }
    if (GAP) {
      const double gah = a ? ga1 : ga0, gbh = a ? gb1 : gb0, gbe = a ? gbeta1 : gbeta0;
#pragma unroll
      for (int r = 0; r < R; r++) cgap[r] = (float)(gah * px0[r] + gbh * py0[r] - gbe);  // slack = a X + b Y + cgap
      gnorm = (float)sqrt(gah * gah + gbh * gbh) + 1.f;
    }
    wsync();
  };

  STAMP(t_hess);
  STAMP(t_inv);
  float hrow[R][NUM];  // condensed Hessian rows, swept in place to T = -H^-1 (box path keeps it)
  // ---- 2b. condensed Hessian rows (closed form, fp32) -------------------------------------
  // Row v = (k, a), column w = (l, b). For l <= k the stages that see both inputs are
  // i = k+1..N (T = N-k of them), and Gamma_i[:, w] is affine in the stage distance, so
  //   H[v][w] = C0_b + C1_b * (k - l)
  // with four per-row constants (sums of 1, t, t^2 over the T stages). The entries with
  // l > k are the transpose: every lane publishes its lower rows and reads column v back.
  // hd = the diagonal of this lane's rows (the exact pivot values pivot_T carries). Also
  // rebuilt by the box path's fp64 PDAS for a fresh T (step 4a').
  auto build_H = [&](float (&hd)[R]) __attribute__((always_inline)) {
    // The row constants and entries are formed in fp64 and rounded once: in fp32 the sums
    // C0 + C1 (k - l) cancel (|C1 (k - l)| ~ 1e5 against entries ~ 1) and on stiff QPs
    // (kappa(H) ~ 4e5 at N = 48, dt = 0.05) that error alone made -H^-1 a divergent
    // preconditioner for the fp64 refinement; correctly rounded entries keep it at ~1e-3.
    const Lin M = sm.M;
    const double q0 = P.q[0], q1 = P.q[1], q2 = P.q[2];
    const double ra = a ? P.r[1] : P.r[0];
    const double beta_a = a ? M.b21 : M.b20;
    const double pxa = a ? 0.0 : M.b00, pya = a ? 0.0 : M.b10;  // dk = 0 in this regime
    const double sxa = M.a02 * beta_a, sya = M.a12 * beta_a;
    double C0[R][2], C1[R][2];
    bool stiff = false;
#pragma unroll
    for (int r = 0; r < R; r++) {
      const double T = (double)(N - kk[r]);
      const double S1 = T * (T - 1.0) * 0.5;
      const double S2 = (T - 1.0) * T * (2.0 * T - 1.0) * (1.0 / 6.0);
      const double Ux = T * pxa + sxa * S1, Vx = pxa * S1 + sxa * S2;
      const double Uy = T * pya + sya * S1, Vy = pya * S1 + sya * S2;
#pragma unroll
      for (int bb = 0; bb < 2; bb++) {
        const double beta_b = bb ? M.b21 : M.b20;
        const double ax_b = bb ? 0.0 : M.b00, ay_b = bb ? 0.0 : M.b10;
        const double sxb = M.a02 * beta_b, syb = M.a12 * beta_b;
        C0[r][bb] = q0 * (ax_b * Ux + sxb * Vx) + q1 * (ay_b * Uy + syb * Vy) + q2 * T * beta_a * beta_b;
        C1[r][bb] = q0 * sxb * Ux + q1 * syb * Uy;
      }
      // a row cancels in fp32 when |C1| (k - l) reaches its diagonal's magnitude
      const double dg = (a ? C0[r][1] : C0[r][0]) + ra;
      stiff |= valid[r] && (fabs(C1[r][0]) + fabs(C1[r][1])) * (double)N > 4.0 * fabs(dg);
    }
    // fp32 entries for box-only QPs of one register row (N <= 32) when no row cancels (the
    // shipped dt = 0.01: |C1| N is a few percent of the diagonal; the round-2 formation), fp64
    // entries rounded once otherwise (wave-uniform). The gap kernel always takes fp64: GI's
    // final fp64 check at N = 40 rejected a point built on fp32 entries (test_horizons_gap[40]).
    if (!GAP && R == 1 && __ballot(stiff) == 0ull) {
      float C0f[R][2], C1f[R][2];
#pragma unroll
      for (int r = 0; r < R; r++)
#pragma unroll
        for (int bb = 0; bb < 2; bb++) {
          C0f[r][bb] = (float)C0[r][bb];
          C1f[r][bb] = (float)C1[r][bb];
        }
#pragma unroll
      for (int r = 0; r < R; r++) {
        if (vv[r] < NUM) {
#pragma unroll
          for (int w = 0; w < NUM; w++) {
            const int l = w >> 1, bb = w & 1;
            sm.L[vv[r]][w] = fmaf(C1f[r][bb], (float)(kk[r] - l), C0f[r][bb]);
          }
        }
      }
      wsync();
#pragma unroll
      for (int r = 0; r < R; r++) {
#pragma unroll
        for (int w = 0; w < NUM; w++) {
          const int l = w >> 1, bb = w & 1;
          float h;
          if (w == vv[r]) h = (float)(C0[r][bb] + ra);
          else h = (l <= kk[r]) ? fmaf(C1f[r][bb], (float)(kk[r] - l), C0f[r][bb]) : sm.L[w][cl[r]];
          const bool ok = valid[r] && (w < NU);
          hrow[r][w] = ok ? h : (w == vv[r] ? 1.f : 0.f);
        }
      }
    } else {
#pragma unroll
      for (int r = 0; r < R; r++) {
        if (vv[r] < NUM) {
#pragma unroll
          for (int w = 0; w < NUM; w++) {
            const int l = w >> 1, bb = w & 1;  // exchange via L: row stride NUM + 1, conflict-free
            sm.L[vv[r]][w] = (float)fma(C1[r][bb], (double)(kk[r] - l), C0[r][bb]);
          }
        }
      }
      wsync();
#pragma unroll
      for (int r = 0; r < R; r++) {
#pragma unroll
        for (int w = 0; w < NUM; w++) {
          const int l = w >> 1, bb = w & 1;
          float h;
          if (w == vv[r]) h = (float)(C0[r][bb] + ra);
          else h = (l <= kk[r]) ? (float)fma(C1[r][bb], (double)(kk[r] - l), C0[r][bb]) : sm.L[w][cl[r]];
          const bool ok = valid[r] && (w < NU);
          hrow[r][w] = ok ? h : (w == vv[r] ? 1.f : 0.f);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < R; r++)
      hd[r] = vv[r] < NUM ? (valid[r] ? (float)((a ? C0[r][1] : C0[r][0]) + ra) : 1.f) : 0.f;
    wsync();
  };
  if (whit) {
    // ---- 2b/3 (cache hit): W from the slot / group cache, no Hessian, no sweep ----------
    const float* Wc = ws.W + (size_t)wslot * NU * NU;
#pragma unroll
    for (int r = 0; r < R; r++) {
      if (vv[r] >= NUM) continue;
#pragma unroll 4
      for (int j = 0; j < NUM; j++) {
        float wv = (j == vv[r]) ? 1.f : 0.f;
        if (j < NU && valid[r]) wv = Wc[(size_t)j * NU + vv[r]];
        sm.W[j][vv[r]] = wv;
      }
    }
    wsync();
#pragma unroll
    for (int r = 0; r < R; r++)
#pragma unroll
      for (int j = 0; j < NUM; j++) hrow[r][j] = (vv[r] < NUM) ? -sm.W[j][vv[r]] : 0.f;
  } else {
  float hd[R];
  build_H(hd);
  if (Hdbg) {  // debug/parity hook: dump H and g, no solve
    inputs_and_gradient();
#pragma unroll
    for (int r = 0; r < R; r++) {
      if (valid[r]) {
#pragma unroll
        for (int w = 0; w < NUM; w++)
          if (w < NU) Hdbg[((size_t)b * NU + vv[r]) * NU + w] = (double)hrow[r][w];
      }
    }
    return;
  }
  STAMP_SET(t_hess);
  // ---- 3. W = H^-1 : symmetric sweep (Goodnight), rows in registers -----------------------
  // Jacobi scaling around the sweep: sweep D H D (unit diagonal, every later pivot <= 1) and
  // scale back, W = D (D H D)^-1 D. The sweep folds the pivot row's update into the common FMA
  // (f = 1 - 1/a_pp), which loses ~eps |a_pp| of that row relative; with pivots <= 1 nothing
  // cancels. Unscaled, stiff QPs (H_kk ~ 8e3 at N = 48, dt = 0.05) got W rows 5e-4 off and the
  // fp64 refinement through W contracted by only 0.25 per step.
  {
    float dsc[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
      dsc[r] = (vv[r] < NUM && hd[r] > 0.f) ? __builtin_amdgcn_rsqf(hd[r]) : 1.f;
      if (vv[r] < NUM) sm.yb[vv[r]] = dsc[r];
    }
    wsync();
    auto scale_rows = [&]() __attribute__((always_inline)) {
#pragma unroll
      for (int j = 0; j < NUM; j += 4) {
        const f32x4 d4 = *reinterpret_cast<const f32x4*>(&sm.yb[j]);
#pragma unroll
        for (int r = 0; r < R; r++) {
          hrow[r][j] *= dsc[r] * d4.x; hrow[r][j + 1] *= dsc[r] * d4.y;
          hrow[r][j + 2] *= dsc[r] * d4.z; hrow[r][j + 3] *= dsc[r] * d4.w;
        }
      }
    };
    scale_rows();
    Sweep<NUM, R, 0>::run(hrow, lane);
    scale_rows();
    wsync();
  }
#pragma unroll
  for (int r = 0; r < R; r++) {
    if (vv[r] < NUM) {
#pragma unroll
      for (int j = 0; j < NUM; j++) sm.W[j][vv[r]] = -hrow[r][j];  // -H^-1 (symmetric: stored by column, conflict-free)
    }
  }
  wsync();
  if (warm && wslot >= 0 && (prep || !grp)) {  // prime the slot / group cache (coalesced:
    float* Wc = ws.W + (size_t)wslot * NU * NU;        // lane v writes column v of every row)
    for (int j = 0; j < NU; j++) {
#pragma unroll
      for (int r = 0; r < R; r++)
        if (valid[r]) Wc[(size_t)j * NU + vv[r]] = sm.W[j][cl[r]];
    }
    if (lane == 0) {
      unsigned* key = ws.key + 4 * wslot;
      key[0] = __float_as_uint(fTH0);
      key[1] = __float_as_uint(ulg[2 * b + 0]);
      key[2] = __float_as_uint(ulg[2 * b + 1]);
      key[3] = 1u;
    }
  }
  wsync();
  if (prep) return;  // prepare launch: the group's W is published, no solve
  }  // !whit

  STAMP_SET(t_inv);
  inputs_and_gradient();
  // GAP: steepest-edge ranking of the gap rows in GI's step 1. A gap row of stage k+1
  // (mpc.cpp:249,271) is n_j'u >= beta_j with n_j = Gamma_{k+1}'(a, b, 0), which by A = I + E
  // (model.cpp:42-51) is n_j = alpha u + beta (k p - r) on the inputs of stages <= k, with
  // u = [speed input], p = (b20 | b21) by input, r = stage * p. Its W-norm n_j'W n_j then follows
  // from six block moments M_xy(k) = sum_{w,v of stages <= k} x_w W_wv y_v (x, y in {u, p, r}),
  // which one pass over each lane's row of W and six wave prefix scans give for every k. Ranking
  // the violated gap rows by slack / sqrt(n_j'W n_j) instead of slack / |(a, b)| cut the GI
  // iterations of the bench's C3 batch from max 58 / p99 21 to 34 / 17 (numpy model of this
  // loop, box rows kept at slack / (1 + |bound|)): C3's time is its slowest QP's GI chain.
  float gsc[R];
#pragma unroll
  for (int r = 0; r < R; r++) gsc[r] = 0.f;
  if constexpr (GAP) {
    const Lin M = sm.M;
    double T[6][R];  // per variable w: its part of the moments uu, up, ur, pp, pr, rr
#pragma unroll
    for (int r = 0; r < R; r++) {
      const int kw = kk[r];
      const double pw = valid[r] ? (a ? M.b21 : M.b20) : 0.0, uw = (valid[r] && a == 0) ? 1.0 : 0.0;
      const double rw = kw * pw;
      float RPu = 0.f, RPp = 0.f, RPr = 0.f, SSu = 0.f, SSp = 0.f, SSr = 0.f;
      const float fb20 = (float)M.b20, fb21 = (float)M.b21;
      for (int x = 0; x < NUM; x++) {  // W[w][x] = sm.W[x][w]: consecutive lanes, conflict free
        const float wx = (x <= 2 * kw + 1) ? sm.W[x][cl[r]] : 0.f;
        const int kx = x >> 1;
        const float px = (x & 1) ? fb21 : fb20, ux = (x & 1) ? 0.f : 1.f, rx = (float)kx * px;
        RPu = fmaf(wx, ux, RPu); RPp = fmaf(wx, px, RPp); RPr = fmaf(wx, rx, RPr);
        const float ws = (kx == kw) ? wx : 0.f;
        SSu = fmaf(ws, ux, SSu); SSp = fmaf(ws, px, SSp); SSr = fmaf(ws, rx, SSr);
      }
      // pairs (w, x) with stage(x) <= stage(w) from row w, pairs with stage(w) < stage(x) from row x
      const double Su = RPu - SSu, Sp = RPp - SSp, Sr = RPr - SSr;
      T[0][r] = uw * RPu + uw * Su;
      T[1][r] = uw * RPp + pw * Su;
      T[2][r] = uw * RPr + rw * Su;
      T[3][r] = pw * RPp + pw * Sp;
      T[4][r] = pw * RPr + rw * Sp;
      T[5][r] = rw * RPr + rw * Sr;
    }
#pragma unroll
    for (int m = 0; m < 6; m++) scan_incl_R<R>(T[m]);
#pragma unroll
    for (int r = 0; r < R; r++) {
      double Mm[6];
#pragma unroll
      for (int m = 0; m < 6; m++) Mm[m] = odd_lane(T[m][r]);  // stage k's moments sit in lane 2k+1
      const double ah = a ? ga1 : ga0, bh = a ? gb1 : gb0;
      const double al = ah * M.b00 + bh * M.b10, be = ah * M.a02 + bh * M.a12, k = (double)kk[r];
      const double c = al * al * Mm[0] + 2.0 * al * be * (k * Mm[1] - Mm[2]) +
                       be * be * (k * k * Mm[3] - 2.0 * k * Mm[4] + Mm[5]);
      gsc[r] = (valid[r] && c > 0.0) ? (float)(1.0 / sqrt(c)) : 1.f / gnorm;
    }
  }
  STAMP(t_grad);
  // ---- 4. active set -----------------------------------------------------------------------
  float xv[R];           // GI iterate (fp32)
  float xunc[R];         // GI's start, the unconstrained optimum -W g (the negative-multiplier re-entry)
  int actf[R];           // bit t set when constraint 3*v+t is active
  int slot_id[R];        // constraint id of active slot (64r + lane), -1 if none
  float mult[R];         // its multiplier
  float rdiag[R];        // 1 / L[slot][slot]
#pragma unroll
  for (int r = 0; r < R; r++) { xv[r] = 0.f; actf[r] = 0; slot_id[r] = -1; mult[r] = 0.f; rdiag[r] = 0.f; }
  int q = 0;
  int it = 0;
  const int max_iter = P.max_iter;
  int status = numerical ? F110QP_NUMERICAL_ID
                         : (infeasible0 ? F110QP_PRIMAL_INFEASIBLE_ID : F110QP_SOLVED_ID);
  int reentries = 0;
  double u64[R];
#pragma unroll
  for (int r = 0; r < R; r++) u64[r] = 0.0;
  bool final_ok = false;
  bool gi_start = true;  // GI starts from the unconstrained point (x = -W g)
  int forced_p = -1;     // violated row found by the fp64 re-check
  float forced_sp = 0.f;
  bool inexact = false;  // GI's final check failed: SOLVED_INACCURATE

  // ---- box rows: fp64 machinery of steps 4a' and 6 (T, its set, the fp64 point) ----------
  float dg[R], ed[R];   // exact diagonal of T / offset of its register copy (pivot_T)
  int act[R], nact[R];  // 0 free, 1 at the lower bound, 2 at the upper bound
#pragma unroll
  for (int r = 0; r < R; r++) { dg[r] = 0.f; ed[r] = 0.f; act[r] = 0; nact[r] = 0; }
  // r1 = H u + g at u64 (fp64 rollout and costate); the references are re-read from LDS so
  // that nothing of this rare path stays live across the fp32 loop above
  auto residual = [&](double (&r1)[R]) __attribute__((always_inline)) {
    const Lin M = sm.M;
    double rxd[R], ryd[R], rthd[R], zero[R], px[R], py[R], th[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
      rxd[r] = sm.rx[vv[r]]; ryd[r] = sm.ry[vv[r]]; rthd[r] = sm.rth[vv[r]];
      zero[r] = 0.0;
    }
    rollout_f64<R>(M, lane, u64, px, py, th);
    grad_f64<R>(M, P, lane, N, u64, px, py, th, rxd, ryd, rthd, zero, zero, r1);
  };
  // u_F += T_FF r1_F (r1 = H u + g in fp64) until max |du| <= tight; converged if <= loose
  // (past `steps`, up to steps_max while each step still halves the correction). Converged:
  // the last correction <= loose and the error it leaves, ~ |du|^2 / |du_prev| at the observed
  // contraction, <= 1e-8: a slowly contracting T (stiff QP) keeps refining instead of stopping
  // at a 2e-6 step that still leaves ~1e-6 in u.
  auto refine = [&](int steps, float tight, float loose, int steps_max) __attribute__((always_inline)) -> bool {
    float adx = 3.0e38f, prev = 3.0e38f;
    bool conv = false;
    for (int rs = 0; rs < steps_max; rs++) {
      double r1[R];
      residual(r1);
      float y[R], dx[R];
#pragma unroll
      for (int r = 0; r < R; r++) y[r] = (valid[r] && !act[r]) ? (float)r1[r] : 0.f;
      matvec_T<NUM, GAP, R>(sm, hrow, ed, vv, y, dx);
      float mx = 0.f;
#pragma unroll
      for (int r = 0; r < R; r++) {
        const bool fr = valid[r] && !act[r];
        if (fr) u64[r] += (double)dx[r];
        const float m = fr ? fabsf(dx[r]) : 0.f;
        mx = fmaxf(mx, (m == m) ? m : 3.0e38f);  // a NaN correction never converges
      }
      int dummy = 0;
      mx = -mx;
      wave_argmin(mx, dummy);  // -max |dx|
      adx = -mx;
      conv = adx <= loose && adx * adx <= 1e-8f * prev;
      if (adx <= tight && conv) break;
      if (rs + 1 >= steps && !(adx < 0.5f * prev)) break;
      prev = adx;
    }
    return conv;
  };
  // T for the current set from H: forward sweeps of the free variables only
  // (Jacobi-scaled like the full sweep: T^ = SWP_F(D H D) has T_FF = D T^_FF D, T_FA = D T^_FA
  // D^-1, T_AA = D^-1 T^_AA D^-1, i.e. entry (i, j) times s_i s_j with s = d on F, 1/d on A.
  // Unscaled, fp32 elimination of the stiff H (entries ~8e3, lambda_min ~0.4) left T_FF 10% off
  // and the refinement through it diverged.)
  auto fresh_T = [&]() __attribute__((always_inline)) {
    build_H(dg);
    float dsc[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
      ed[r] = 0.f;
      dsc[r] = (vv[r] < NUM && dg[r] > 0.f) ? __builtin_amdgcn_rsqf(dg[r]) : 1.f;
      if (vv[r] < NUM) sm.yb[vv[r]] = dsc[r];
    }
    wsync();
    auto scale = [&]() __attribute__((always_inline)) {  // h_ij *= s_i s_j from sm.yb
#pragma unroll
      for (int j = 0; j < NUM; j += 4) {
        const f32x4 d4 = *reinterpret_cast<const f32x4*>(&sm.yb[j]);
#pragma unroll
        for (int r = 0; r < R; r++) {
          const float si = sm.yb[vv[r] < NUM ? vv[r] : 0];
          hrow[r][j] *= si * d4.x; hrow[r][j + 1] *= si * d4.y;
          hrow[r][j + 2] *= si * d4.z; hrow[r][j + 3] *= si * d4.w;
        }
      }
    };
    scale();
#pragma unroll
    for (int r = 0; r < R; r++) dg[r] *= dsc[r] * dsc[r];
#pragma unroll
    for (int r0 = 0; r0 < R; r0++) {
      unsigned long long m = __ballot(valid[r0] && act[r0] == 0);
      while (m) {
        const int bit = __builtin_ctzll(m);
        m &= m - 1;
        pivot_T<NUM, GAP, R>(sm, hrow, dg, ed, lane, vv, 64 * r0 + bit, 1.f);
      }
    }
    float s[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
      s[r] = (valid[r] && act[r]) ? 1.f / dsc[r] : dsc[r];
      if (vv[r] < NUM) sm.yb[vv[r]] = s[r];
    }
    wsync();
    scale();
#pragma unroll
    for (int r = 0; r < R; r++) {
      dg[r] *= s[r] * s[r];
      ed[r] *= s[r] * s[r];
    }
    wsync();
  };
  // exact KKT re-check at u64: nact = act with every violator flipped; any violation?
  // Both tests in primal units: a free variable past its bound by more than 1e-9 (1 + |b|),
  // an active one whose wrong-sign multiplier would move it by more than that once freed
  // (|r1| / T_ii, T_ii = the Schur complement H_ii - H_iF H_FF^-1 H_Fi carried in dg): a
  // multiplier tolerance in gradient units let a near-degenerate bound of a stiff QP stay
  // active with an error of |r1| / curvature ~ 1e-3 in u.
  auto kkt_violated = [&]() __attribute__((always_inline)) -> bool {
    double r1f[R];
    residual(r1f);
    bool any = false;
#pragma unroll
    for (int r = 0; r < R; r++) {
      nact[r] = act[r];
      if (!valid[r]) continue;
      if (act[r]) {
        const double bnd = act[r] == 1 ? (double)lb[r] : (double)ub[r];
        const double lam = act[r] == 1 ? r1f[r] : -r1f[r];  // >= 0 at the optimum
        if (!(lam >= -1e-9 * (1.0 + fabs(bnd)) * fmax((double)dg[r], 0.0))) nact[r] = 0;
      } else {
        const double s0 = (u64[r] - (double)lb[r]) / (1.0 + fabs((double)lb[r]));
        const double s1 = ((double)ub[r] - u64[r]) / (1.0 + fabs((double)ub[r]));
        nact[r] = s0 < -1e-9 ? 1 : (s1 < -1e-9 ? 2 : 0);
      }
      any = any || (nact[r] != act[r]);
    }
    return __ballot(any) != 0ull;
  };

  // ---- 4a. box rows only: primal-dual active set (Hintermueller-Ito-Kunisch) on T ----------
  // Each pass solves the equality QP of the current guess A with one product x = T y
  // (y = g on F, -bound on A): u_F = x_F, and the bound multipliers are lambda_A = g_A - x_A
  // (lambda = Hu + g). The next guess follows from the multipliers and the bounds; each
  // variable that enters or leaves A is one pivot of T. On these QPs the optimal set is
  // reached in <= 5 passes (P.pdas_max = 10); step 4a' then refines and certifies it in fp64.
  // (Measured and not kept for the gap-row kernel: the same box PDAS first,
  // then GI from its set for the violated gap rows: C3 327 -> 451 us, the GI steps are the gap
  // rows themselves and the extra code halves that kernel's occupancy.)
  if constexpr (!GAP) {
    if (status == F110QP_SOLVED_ID) {
      STAMP(t_pdas);
      float gr[R], u[R], lam[R];
#pragma unroll
      for (int r = 0; r < R; r++) {
        dg[r] = (vv[r] < NUM) ? -sm.W[vv[r]][vv[r]] : 0.f;
        ed[r] = 0.f;
        gr[r] = valid[r] ? sm.vec[vv[r]] : 0.f;
        u[r] = 0.f;
        lam[r] = 0.f;
        act[r] = 0;
        if (seed_act && valid[r]) {  // previous tick's active bounds seed the first guess
          const unsigned long long lo_m = ws.act[2 * (R * b + r)], hi_m = ws.act[2 * (R * b + r) + 1];
          act[r] = ((lo_m >> lane) & 1ull) ? 1 : (((hi_m >> lane) & 1ull) ? 2 : 0);
        }
      }
#pragma unroll
      for (int r0 = 0; r0 < R; r0++) {
        unsigned long long m = __ballot(act[r0] != 0);
        while (m) {
          const int bit = __builtin_ctzll(m);
          m &= m - 1;
          pivot_T<NUM, GAP, R>(sm, hrow, dg, ed, lane, vv, 64 * r0 + bit, -1.f);
        }
      }
      bool converged = false;
      for (int pit = 0; pit < P.pdas_max; pit++) {
        float y[R], x[R];
#pragma unroll
        for (int r = 0; r < R; r++)
          y[r] = !valid[r] ? 0.f : (act[r] == 1 ? -lb[r] : (act[r] == 2 ? -ub[r] : gr[r]));
        matvec_T<NUM, GAP, R>(sm, hrow, ed, vv, y, x);
        int nact[R];
        bool any_changed = false;
#pragma unroll
        for (int r = 0; r < R; r++) {
          u[r] = !valid[r] ? 0.f : (act[r] == 1 ? lb[r] : (act[r] == 2 ? ub[r] : x[r]));
          lam[r] = (valid[r] && act[r]) ? gr[r] - x[r] : 0.f;
          const float myu = act[r] == 1 ? lam[r] : (act[r] == 2 ? -lam[r] : 0.f);
          const bool nlo = valid[r] && ((act[r] == 1 ? myu : 0.f) + (lb[r] - u[r]) > 0.f);
          const bool nhi = valid[r] && !nlo && ((act[r] == 2 ? myu : 0.f) + (u[r] - ub[r]) > 0.f);
          nact[r] = nlo ? 1 : (nhi ? 2 : 0);
          any_changed = any_changed || (__ballot(nact[r] != act[r]) != 0);
        }
        if (!any_changed) { converged = true; it = pit + 1; break; }
#pragma unroll
        for (int r0 = 0; r0 < R; r0++) {
          unsigned long long enter = __ballot(act[r0] == 0 && nact[r0] != 0);
          unsigned long long leave = __ballot(act[r0] != 0 && nact[r0] == 0);
          while (enter) {
            const int bit = __builtin_ctzll(enter);
            enter &= enter - 1;
            pivot_T<NUM, GAP, R>(sm, hrow, dg, ed, lane, vv, 64 * r0 + bit, -1.f);
          }
          while (leave) {
            const int bit = __builtin_ctzll(leave);
            leave &= leave - 1;
            pivot_T<NUM, GAP, R>(sm, hrow, dg, ed, lane, vv, 64 * r0 + bit, 1.f);
          }
        }
#pragma unroll
        for (int r = 0; r < R; r++) act[r] = nact[r];
      }
      if (!converged) it = P.pdas_max;
      STAMP_ACC(acc_pdas, t_pdas);
      // ---- 4a'. acceptance in fp64, and the fp64 PDAS behind it ----------------------------
      // The fp32 fixed point is refined in fp64 (residual from the fp64 rollout and costate,
      // correction through T on F) and accepted only if the refinement converged and the exact
      // re-check holds: every free variable inside its box, every active bound's multiplier
      // r1 = (H u + g)_A of the right sign (lower: r1 >= 0, upper: r1 <= 0). Otherwise the same
      // PDAS continues on the fp64 values: HIK updates (every violator flips) for kHikPasses
      // passes, then one flip per pass, the least-index violator (Murty's rule, finite for SPD H),
      // each pass's equality solve refined to kRobTol. A few flips pivot T in place; more, or a
      // refinement that stalls, rebuild T from H by forward sweeps of the free set only: reverse
      // sweeps out of the full inverse lose T's accuracy on stiff H (condition number ~ (N dt v)^2:
      // 4e5 at N = 48, dt = 0.05, where the fp32 set of a bang-bang optimum, 95 of 96 bounds
      // active, was wrong or its refinement stalled). No fixed point within kRobPasses -> GI from
      // the unconstrained point, whose own final check reports SOLVED_INACCURATE, never a wrong
      // SOLVED.
      STAMP(t_ref0);
      {
#pragma unroll
        for (int r = 0; r < R; r++)
          u64[r] = !valid[r] ? 0.0 : (act[r] == 1 ? (double)lb[r] : (act[r] == 2 ? (double)ub[r] : (double)u[r]));
        bool ref_ok = converged && refine(kRefineSteps, kRefineTol, kRefineTol, kRobSteps);
        bool fresh = false, accept = false;
        int pass = 0;
        for (;;) {
          if (ref_ok && !kkt_violated()) { accept = true; break; }
          if (pass >= kRobPasses<NUM> || it >= max_iter) break;
          if (!ref_ok) {
            if (fresh) break;  // a fresh T stalls too
            fresh_T();
            fresh = true;
          } else {
            if (pass >= kHikPasses) {  // least-index violator only
              int first = 0x7fffffff;
#pragma unroll
              for (int r0 = R - 1; r0 >= 0; r0--) {
                const unsigned long long m = __ballot(nact[r0] != act[r0]);
                if (m) first = 64 * r0 + __builtin_ctzll(m);
              }
#pragma unroll
              for (int r = 0; r < R; r++)
                if (vv[r] != first) nact[r] = act[r];
            }
            int nchg = 0;
#pragma unroll
            for (int r0 = 0; r0 < R; r0++) nchg += __popcll(__ballot(nact[r0] != act[r0]));
            if (nchg > kIncPivots) {
#pragma unroll
              for (int r = 0; r < R; r++) act[r] = nact[r];
              fresh_T();
              fresh = true;
            } else {
#pragma unroll
              for (int r0 = 0; r0 < R; r0++) {
                unsigned long long enter = __ballot(act[r0] == 0 && nact[r0] != 0);
                unsigned long long leave = __ballot(act[r0] != 0 && nact[r0] == 0);
                while (enter) {
                  const int bit = __builtin_ctzll(enter);
                  enter &= enter - 1;
                  pivot_T<NUM, GAP, R>(sm, hrow, dg, ed, lane, vv, 64 * r0 + bit, -1.f);
                }
                while (leave) {
                  const int bit = __builtin_ctzll(leave);
                  leave &= leave - 1;
                  pivot_T<NUM, GAP, R>(sm, hrow, dg, ed, lane, vv, 64 * r0 + bit, 1.f);
                }
              }
#pragma unroll
              for (int r = 0; r < R; r++) act[r] = nact[r];
              fresh = false;
            }
#pragma unroll
            for (int r = 0; r < R; r++)
              if (valid[r]) u64[r] = act[r] == 1 ? (double)lb[r] : (act[r] == 2 ? (double)ub[r] : u64[r]);
            pass++;
            it++;
          }
          ref_ok = refine(3, kRobTight, kRobTol, kRobSteps);
        }
        STAMP_ACC(acc_refine, t_ref0);
        if (accept) {
          final_ok = true;
#pragma unroll
          for (int r = 0; r < R; r++) actf[r] = act[r];  // bit0 lower, bit1 upper
        }
        // else: GI from the unconstrained point (gi_start)
      }
    }
  }
  if (gi_start && !final_ok) {
    // x = -W g  (g in sm.vec)
    matvec_W<NUM, GAP, R>(sm, lane, xv);
#pragma unroll
    for (int r = 0; r < R; r++) {
      xv[r] = valid[r] ? -xv[r] : 0.f;
      xunc[r] = xv[r];
    }
    wsync();
#pragma unroll
    for (int r = 0; r < R; r++) actf[r] = 0;
  }

  const bool gi_fallback = !final_ok && status == F110QP_SOLVED_ID;  // box rows: behind the fp64 PDAS
  const LinF MF = lin_f32(sm.M);  // fp32 coefficients for GI's rollouts and normals
  // ---- 4b. dual active set (Goldfarb-Idnani, range space) ---------------------------------
  while (status == F110QP_SOLVED_ID && !final_ok) {
    // ---- step 1: most violated inactive constraint (fp32, scaled) ----
    STAMP(t_s1);
    int p;
    float sp;
    if (forced_p >= 0) {
      p = forced_p;
      sp = forced_sp;
      forced_p = -1;
    } else {
      float X[R], Y[R];
      if (GAP) rollout_lin_f32<R>(MF, lane, xv, X, Y);
      // Gap rows first (P.gap_first): a violated gap row enters before any box row; numpy model of
      // the GI loop on the C3 batch (tests/diag_gi_selection_model.py rules): max 34 -> 30
      // iterations, p99 17 either way. Otherwise one ranking over all rows.
      const bool gf = GAP && P.gap_first;
      float best = 0.f, bestG = 0.f;
      int bid = 0x7fffffff, bidG = 0x7fffffff;
      float sraw = 0.f, srawG = 0.f;  // raw slack of this lane's best candidate (box / gap class)
#pragma unroll
      for (int r = 0; r < R; r++) {
        if (!valid[r]) continue;
        const int v = vv[r];
        const float s0 = xv[r] - lb[r], s1 = ub[r] - xv[r];
        // scaled slacks s / (1 + |bound|); the bound of a variable is its input's, so the two
        // scales are wave-uniform per lane parity (a reciprocal multiply, no fp32 division)
        const float v0 = s0 * (a ? il1 : il0), v1 = s1 * (a ? iu1 : iu0);
        if (!(actf[r] & 1) && v0 < -1e-6f && v0 < best) { best = v0; bid = 3 * v; sraw = s0; }
        if (!(actf[r] & 2) && v1 < -1e-6f && v1 < best) { best = v1; bid = 3 * v + 1; sraw = s1; }
        if (GAP) {
          const float s2 = (a ? ga1 : ga0) * X[r] + (a ? gb1 : gb0) * Y[r] + cgap[r];
          const float v2 = s2 * gsc[r];  // ranked by the W-norm (steepest edge), thresholded as before
          const bool c2 = !(actf[r] & 4) && s2 < -1e-6f * gnorm;
          if (gf) {
            if (c2 && v2 < bestG) { bestG = v2; bidG = 3 * v + 2; srawG = s2; }
          } else if (c2 && v2 < best) {
            best = v2; bid = 3 * v + 2; sraw = s2;
          }
        }
      }
      int bid_w = 0x7fffffff;
      float sraw_w = sraw;
      if (gf) {
        float bg = bestG;
        bid_w = bidG;
        wave_argmin(bg, bid_w);
        sraw_w = srawG;
      }
      if (bid_w == 0x7fffffff) {
        float best_w = best;
        bid_w = bid;
        wave_argmin(best_w, bid_w);
        sraw_w = sraw;
      }
      if (bid_w != 0x7fffffff) {
        p = bid_w;
        sp = readlane_f(sraw_w, (bid_w / 3) & 63);
      } else {
        // ---- 5. refinement in fp64, feasibility re-check, certificate ----
        // Newton steps on the equality KKT system of the final set (fp64 residuals, corrections
        // through the fp32 W and factor; the multipliers kept in fp64 in sm.cmult) until the fp64
        // residual certifies the point (kRefineMax, kCertTauW), then every inactive row in fp64.
        STAMP(t_ref0);
#pragma unroll
        for (int r = 0; r < R; r++) {
          sm.cmult[3 * vv[r]] = 0.0;
          sm.cmult[3 * vv[r] + 1] = 0.0;
          sm.cmult[3 * vv[r] + 2] = 0.0;
        }
        wsync();
        float umaxf = 0.f;
#pragma unroll
        for (int r = 0; r < R; r++) {
          if (64 * r + lane < q) sm.cmult[slot_id[r]] = (double)mult[r];
          u64[r] = valid[r] ? (double)xv[r] : 0.0;
          umaxf = fmaxf(umaxf, valid[r] ? fabsf(xv[r]) : 0.f);
        }
        {
          int dummy = 0;
          umaxf = -umaxf;
          wave_argmin(umaxf, dummy);
          umaxf = -umaxf;
        }
        const double ctol = kCertTauW * fmax(1.0, (double)umaxf);
        const double thr2 = fmin(P.r[0], P.r[1]) * ctol * ctol;  // bound on rho'W rho
        const Lin M = sm.M;
        double rxd[R], ryd[R], rthd[R];
#pragma unroll
        for (int r = 0; r < R; r++) { rxd[r] = sm.rx[vv[r]]; ryd[r] = sm.ry[vv[r]]; rthd[r] = sm.rth[vv[r]]; }
        double px[R], py[R], th[R];
        // r1 = H u + g - N_A mu at u64 (fp64 rollout and costate), mu from sm.cmult (clamped at 0
        // with `clamp`); px / py / th the rollout of u64
        auto kkt_res = [&](bool clamp, double (&r1)[R]) __attribute__((always_inline)) {
          rollout_f64<R>(M, lane, u64, px, py, th);
          double gmx[R], gmy[R];  // gap multipliers of the variable's stage (sides 0,1)
#pragma unroll
          for (int r = 0; r < R; r++) {
            gmx[r] = 0.0; gmy[r] = 0.0;
            if (GAP) {
              double m0 = sm.cmult[3 * (vv[r] & ~1) + 2], m1 = sm.cmult[3 * (vv[r] | 1) + 2];
              if (clamp) { m0 = fmax(m0, 0.0); m1 = fmax(m1, 0.0); }
              gmx[r] = m0 * ga0 + m1 * ga1;
              gmy[r] = m0 * gb0 + m1 * gb1;
            }
          }
          grad_f64<R>(M, P, lane, N, u64, px, py, th, rxd, ryd, rthd, gmx, gmy, r1);
#pragma unroll
          for (int r = 0; r < R; r++) {
            double ml = sm.cmult[3 * vv[r]], mu = sm.cmult[3 * vv[r] + 1];
            if (clamp) { ml = fmax(ml, 0.0); mu = fmax(mu, 0.0); }
            r1[r] = valid[r] ? r1[r] - ml + mu : 0.0;
          }
        };
        // r2_j = n_j'u - b_j on the active rows (fp64, from sm.d64 / sx64 / sy64); active rows must
        // hold with equality. Returns max |r2_j| / scale over the slots (wave-uniform).
        auto act_res = [&](float (&r2)[R]) __attribute__((always_inline)) -> float {
          float r2n = 0.f;
#pragma unroll
          for (int r = 0; r < R; r++) {
            r2[r] = 0.f;
            if (64 * r + lane < q) {
              const int owner = slot_id[r] / 3, t = slot_id[r] - 3 * owner;
              double r2d, sc;
              if (t == 0) {
                const double bd = (double)((owner & 1) ? umin1 : umin0);
                r2d = sm.d64[owner] - bd;
                sc = 1.0 + fabs(bd);
              } else if (t == 1) {
                const double bd = (double)((owner & 1) ? umax1 : umax0);
                r2d = bd - sm.d64[owner];
                sc = 1.0 + fabs(bd);
              } else {
                const int st = (owner >> 1) + 1;
                r2d = (owner & 1) ? ((double)ga1 * sm.sx64[st] + (double)gb1 * sm.sy64[st] - gbeta1)
                                  : ((double)ga0 * sm.sx64[st] + (double)gb0 * sm.sy64[st] - gbeta0);
                sc = (double)gnorm;
              }
              r2[r] = (float)r2d;
              r2n = fmaxf(r2n, (float)(fabs(r2d) / sc));
            }
          }
          int dummy = 0;
          r2n = -r2n;
          wave_argmin(r2n, dummy);
          return -r2n;
        };
        float prev = 3.0e38f;
        // the last residual evaluation when the refinement stopped on its own test: with no negative
        // multiplier it is the certificate's clamped residual at the same point (reused below)
        double r1k[R];
        float w1k[R];
        bool refok = false;
#pragma unroll
        for (int r = 0; r < R; r++) { r1k[r] = 0.0; w1k[r] = 0.f; }
        for (int rs = 0; rs < kRefineMax; rs++) {
          wsync();
          double r1[R];
          kkt_res(false, r1);
#pragma unroll
          for (int r = 0; r < R; r++) {
            sm.d64[vv[r]] = u64[r];
            if (GAP && a == 1 && kk[r] < N) { sm.sx64[kk[r] + 1] = px[r]; sm.sy64[kk[r] + 1] = py[r]; }
            sm.vec[vv[r]] = (float)r1[r];
          }
          wsync();
          // w1 = W r1 (the correction's first product) and the residual's W-norm r1'W r1
          float w1[R];
          matvec_W<NUM, GAP, R>(sm, lane, w1);
          double rsq = 0.0;
#pragma unroll
          for (int r = 0; r < R; r++) rsq += valid[r] ? r1[r] * (double)w1[r] : 0.0;
          rsq = wave_sum(rsq);
          float r2[R];
          const float r2n = act_res(r2);
          if (rsq <= 0.25 * thr2 && r2n <= 1e-9f) {  // small enough: the certificate decides below
#pragma unroll
            for (int r = 0; r < R; r++) { r1k[r] = r1[r]; w1k[r] = w1[r]; }
            refok = true;
            break;
          }
          if (rs + 1 == kRefineMax) break;
          // v1_j = n_j' w1 (= V_j' r1 with the gap rows' stored V_j = W n_j: r1 is still in sm.vec
          // from the W product, so no rollout of w1 and no barrier)
          float rhs[R], lv[R], du[R];
          if constexpr (GAP) {
            const float4* x4 = reinterpret_cast<const float4*>(sm.vec);
#pragma unroll
            for (int r = 0; r < R; r++) {
              const int sl = 64 * r + lane;
              const float4* v4 = reinterpret_cast<const float4*>(sm.V[sl < NUM ? sl : NUM - 1]);
              float d0 = 0.f, d1 = 0.f, d2 = 0.f, d3 = 0.f;
#pragma unroll
              for (int j4 = 0; j4 < NUM / 4; j4++) {
                const float4 xr4 = x4[j4], vr4 = v4[j4];
                d0 = fmaf(vr4.x, xr4.x, d0);
                d1 = fmaf(vr4.y, xr4.y, d1);
                d2 = fmaf(vr4.z, xr4.z, d2);
                d3 = fmaf(vr4.w, xr4.w, d3);
              }
              rhs[r] = (sl < q) ? ((d0 + d1) + (d2 + d3)) - r2[r] : 0.f;
            }
          } else {
#pragma unroll
            for (int r = 0; r < R; r++) sm.vec2[vv[r]] = w1[r];
            wsync();
#pragma unroll
            for (int r = 0; r < R; r++)
              rhs[r] = (64 * r + lane < q) ? slot_dot<NUM, GAP>(sm, slot_id[r], ga0, ga1, gb0, gb1) - r2[r] : 0.f;
          }
          // du = S^-1 rhs ; dx = -w1 + sum_j du_j V[j]
          tri_forward<NUM, GAP, R>(sm, lane, q, rdiag, rhs, lv);
          tri_backward<NUM, GAP, R>(sm, lane, q, rdiag, lv, du);
          float dx[R];
#pragma unroll
          for (int r = 0; r < R; r++) dx[r] = -w1[r];
          int j = 0;
          if constexpr (GAP) {  // V rows in blocks, loads first (as the GI step's z update)
            for (; j + kTriBlock <= q; j += kTriBlock) {
              float vb[kTriBlock][R];
#pragma unroll
              for (int jb = 0; jb < kTriBlock; jb++)
#pragma unroll
                for (int r = 0; r < R; r++) vb[jb][r] = sm.V[j + jb][cl[r]];
#pragma unroll
              for (int jb = 0; jb < kTriBlock; jb++) {
                const float duj = rl_f<R>(du, j + jb);
#pragma unroll
                for (int r = 0; r < R; r++) dx[r] = fmaf(duj, vb[jb][r], dx[r]);
              }
            }
          }
          for (; j < q; j++) {
            const float duj = rl_f<R>(du, j);
            const int sj = GAP ? 0 : rl_i<R>(slot_id, j);
#pragma unroll
            for (int r = 0; r < R; r++) dx[r] = fmaf(duj, vcol<NUM, GAP>(sm, j, sj, cl[r]), dx[r]);
          }
          float adx = 0.f;
#pragma unroll
          for (int r = 0; r < R; r++) {
            if (valid[r]) u64[r] += (double)dx[r];
            adx = fmaxf(adx, valid[r] ? fabsf(dx[r]) : 0.f);
          }
          wsync();
#pragma unroll
          for (int r = 0; r < R; r++)
            if (64 * r + lane < q) sm.cmult[slot_id[r]] += (double)du[r];
          int dummy = 0;
          adx = -adx;
          wave_argmin(adx, dummy);  // -max |dx|
          adx = -adx;
          if (rs >= 2 && !(adx < 0.5f * prev)) break;  // stalled: not certifiable here
          prev = adx;
        }
        wsync();
#pragma unroll
        for (int r = 0; r < R; r++)
          if (64 * r + lane < q) mult[r] = (float)sm.cmult[slot_id[r]];
        // fp64 feasibility check of every inactive row at the refined point
        rollout_f64<R>(M, lane, u64, px, py, th);
        float best64 = 0.f, sp64 = 0.f;
        int bid64 = 0x7fffffff;
#pragma unroll
        for (int r = 0; r < R; r++) {
          if (!valid[r]) continue;
          const int v = vv[r];
          const double s0 = u64[r] - (double)lb[r], s1 = (double)ub[r] - u64[r];
          const float v0 = (float)(s0 / (1.0 + fabs((double)lb[r])));
          const float v1 = (float)(s1 / (1.0 + fabs((double)ub[r])));
          if (!(actf[r] & 1) && v0 < -1e-9f && v0 < best64) { best64 = v0; bid64 = 3 * v; sp64 = (float)s0; }
          if (!(actf[r] & 2) && v1 < -1e-9f && v1 < best64) { best64 = v1; bid64 = 3 * v + 1; sp64 = (float)s1; }
          if (GAP) {
            const double s2 = a ? ((double)ga1 * px[r] + (double)gb1 * py[r] - gbeta1)
                                : ((double)ga0 * px[r] + (double)gb0 * py[r] - gbeta0);
            const float v2 = (float)(s2 / (double)gnorm);
            if (!(actf[r] & 4) && v2 < -1e-9f && v2 < best64) { best64 = v2; bid64 = 3 * v + 2; sp64 = (float)s2; }
          }
        }
        wave_argmin(best64, bid64);
        STAMP_ACC(acc_refine, t_ref0);
        if (bid64 == 0x7fffffff || reentries >= 4) {
          // certificate: every row holds (fp64, the test above), evaluated at the final u64 with
          // the multipliers clamped at 0 whatever the refinement did (a negative multiplier's pull
          // stays in the residual, in primal units / lambda)
          bool cert = false;
          bool neg = false;
#pragma unroll
          for (int r = 0; r < R; r++) neg = neg || (64 * r + lane < q && sm.cmult[slot_id[r]] < 0.0);
          if (bid64 == 0x7fffffff) {
            // With mu+ = max(mu, 0) on the active rows and rho = H u + g - N_A mu+, u is the exact
            // optimum of the QP whose gradient is g - rho and whose row bounds are moved by u's own
            // residuals on them (active rows to n_j'u, rows u violates to n_j'u: at most the 1e-9
            // relative of the tests here, far below the float32 rounding of the inputs), and the
            // optimum u*' of that QP with the true gradient g is within |u - u*'|_H^2 <= rho'W rho
            // (its duality gap at the dual point mu+), so |u - u*'|_2^2 <= rho'W rho / lambda
            // (lambda = min r <= lambda_min(H)). rho'W rho is bounded from above in fp64 whatever
            // the accuracy of the fp32 W (kappa ~ 4e5 on the stiff corners): with y = W rho (the
            // fp32 product) and r = rho - H y (fp64 Hessian product, hv_f64),
            //   rho'H^-1 rho = y'(2 rho - H y) + r'H^-1 r <= y'(2 rho - H y) + |r|_2^2 / lambda,
            // with one correction y += W r when that bound is loose (round-5 ADVICE: the fp32
            // estimate of rho'W rho is no longer what certifies). A first-order bound in the rows'
            // residuals against the unmoved bounds would need the optimal multipliers; the
            // duality gap charges them as 2 mu+ s, which measured 1e4-1e6 times the threshold on
            // exact points and is not used.
            double r1c[R];
            float wc[R];
            float r2nc = 0.f;  // (the refinement's own test held the active rows to 1e-9)
            if (refok && __ballot(neg) == 0ull) {
#pragma unroll
              for (int r = 0; r < R; r++) { r1c[r] = r1k[r]; wc[r] = w1k[r]; }
            } else {
              wsync();
              kkt_res(true, r1c);
#pragma unroll
              for (int r = 0; r < R; r++) {
                sm.d64[vv[r]] = u64[r];
                if (GAP && a == 1 && kk[r] < N) { sm.sx64[kk[r] + 1] = px[r]; sm.sy64[kk[r] + 1] = py[r]; }
                sm.vec[vv[r]] = (float)r1c[r];
              }
              wsync();
              float r2c[R];
              matvec_W<NUM, GAP, R>(sm, lane, wc);
              r2nc = act_res(r2c);
            }
            const double lam = fmin(P.r[0], P.r[1]);
            double ycr[R];
#pragma unroll
            for (int r = 0; r < R; r++) ycr[r] = valid[r] ? (double)wc[r] : 0.0;
            double bound = 0.0;
            for (int pass = 0; pass < 2; pass++) {
              double hy[R], rr[R];
              hv_f64<R>(M, P, lane, N, ycr, hy);
              double t1 = 0.0, t2 = 0.0;
#pragma unroll
              for (int r = 0; r < R; r++) {
                rr[r] = valid[r] ? r1c[r] - hy[r] : 0.0;
                t1 += valid[r] ? ycr[r] * (2.0 * r1c[r] - hy[r]) : 0.0;
                t2 += rr[r] * rr[r];
              }
              t1 = wave_sum(t1);
              t2 = wave_sum(t2);
              bound = t1 + t2 / lam;
              // decided: certified, or even a perfect y (bound -> t1) could not certify
              if (pass == 1 || bound <= thr2 || t1 > thr2) break;
              wsync();
#pragma unroll
              for (int r = 0; r < R; r++) sm.vec[vv[r]] = (float)rr[r];
              wsync();
              float dy[R];
              matvec_W<NUM, GAP, R>(sm, lane, dy);
#pragma unroll
              for (int r = 0; r < R; r++) ycr[r] += valid[r] ? (double)dy[r] : 0.0;
            }
            cert = bound >= 0.0 && bound <= thr2 && r2nc <= 1e-9f;
          }
          if constexpr (GAP) {
            // Negative-multiplier re-entry: the refined set holds a row with a negative multiplier
            // (fp32 GI kept a row it should have released; the clamped residual then fails the
            // bound). Drop the most negative, re-solve the equality QP of the remaining set for its
            // multipliers, S_A mu = -s_A(x_unc) (dropping again while one is negative), and continue
            // GI from the dual-feasible x = x_unc + sum mu_j V_j, instead of sending the QP to the
            // fp64 re-check (one heavy QP there costs ~170 us on the C3 launch).
            if (!cert && bid64 == 0x7fffffff && reentries < 4 && __ballot(neg) != 0ull) {
              float mneg = 0.f;
              int kd = 0x7fffffff;
#pragma unroll
              for (int r = 0; r < R; r++) {
                const int sl = 64 * r + lane;
                if (sl < q) {
                  const float m = (float)sm.cmult[slot_id[r]];
                  if (m < mneg) { mneg = m; kd = sl; }
                }
              }
              wave_argmin(mneg, kd);
              // slacks of the rows at x_unc, by variable: box rows from x_unc itself, gap rows from
              // its linear rollout
              {
                float X[R], Y[R];
                rollout_lin_f32<R>(MF, lane, xunc, X, Y);
                wsync();
#pragma unroll
                for (int r = 0; r < R; r++) {
                  sm.vec[vv[r]] = (a ? ga1 : ga0) * X[r] + (a ? gb1 : gb0) * Y[r] + cgap[r];
                  sm.vec2[vv[r]] = xunc[r];
                }
                wsync();
              }
              float mu[R];
#pragma unroll
              for (int r = 0; r < R; r++) mu[r] = mult[r];
              while (kd != 0x7fffffff) {
                const int did = rl_i<R>(slot_id, kd);
                const int down = did / 3;
#pragma unroll
                for (int r = 0; r < R; r++)
                  if (vv[r] == down) actf[r] &= ~(1 << (did - 3 * down));
                int sid_n[R];
#pragma unroll
                for (int r = 0; r < R; r++) {
                  sid_n[r] = __shfl_down(slot_id[r], 1, 64);
                  if (r + 1 < R) {
                    const int s_next = readlane_i(slot_id[r + 1 < R ? r + 1 : r], 0);
                    if (lane == 63) sid_n[r] = s_next;
                  }
                }
#pragma unroll
                for (int r = 0; r < R; r++) {
                  const int sl = 64 * r + lane;
                  if (sl >= kd && sl < q - 1) slot_id[r] = sid_n[r];
                  if (sl == q - 1) slot_id[r] = -1;
                }
#pragma unroll
                for (int r = 0; r < R; r++)
                  if (vv[r] < NUM)
                    for (int j = kd; j < q - 1; j++) sm.V[j][vv[r]] = sm.V[j + 1][vv[r]];
                chol_delete<NUM, GAP, R>(sm, lane, q, kd, rdiag);
                q--;
                wsync();
                // multipliers of the equality QP on the remaining set
                float rhs[R], lv[R];
#pragma unroll
                for (int r = 0; r < R; r++) {
                  rhs[r] = 0.f;
                  if (64 * r + lane < q) {
                    const int owner = slot_id[r] / 3, t = slot_id[r] - 3 * owner;
                    const float xo = sm.vec2[owner];
                    const float sl = t == 0 ? xo - ((owner & 1) ? umin1 : umin0)
                                   : (t == 1 ? ((owner & 1) ? umax1 : umax0) - xo : sm.vec[owner]);
                    rhs[r] = -sl;
                  }
                }
                tri_forward<NUM, GAP, R>(sm, lane, q, rdiag, rhs, lv);
                tri_backward<NUM, GAP, R>(sm, lane, q, rdiag, lv, mu);
                mneg = 0.f;
                kd = 0x7fffffff;
#pragma unroll
                for (int r = 0; r < R; r++) {
                  const int sl = 64 * r + lane;
                  if (sl < q && mu[r] < mneg) { mneg = mu[r]; kd = sl; }
                }
                wave_argmin(mneg, kd);
                it++;
              }
#pragma unroll
              for (int r = 0; r < R; r++) {
                mult[r] = (64 * r + lane < q) ? mu[r] : 0.f;
                xv[r] = xunc[r];
              }
              for (int j = 0; j < q; j++) {
                const float mj = rl_f<R>(mu, j);
#pragma unroll
                for (int r = 0; r < R; r++) xv[r] = fmaf(mj, sm.V[j][cl[r]], xv[r]);
              }
#pragma unroll
              for (int r = 0; r < R; r++) xv[r] = valid[r] ? xv[r] : 0.f;
              reentries++;
              forced_p = -1;
              wsync();
              continue;
            }
          }
          inexact = !cert;
          final_ok = true;
          break;
        }
        reentries++;
        forced_p = bid64;
        forced_sp = readlane_f(sp64, (bid64 / 3) & 63);
#pragma unroll
        for (int r = 0; r < R; r++) xv[r] = valid[r] ? (float)u64[r] : 0.f;
        continue;
      }
    }

    STAMP_ACC(acc_s1, t_s1);
    const int pown = p / 3, pt = p - 3 * pown;
    float uplus_new = 0.f;  // multiplier of the candidate p
    // ---- step 2: add p (possibly after drops) ----
    for (;;) {
      STAMP(t_a);
      if (++it > max_iter) { status = F110QP_MAX_ITER_ID; break; }
      // w = W n_p ; nw = n_p' W n_p
      float w[R], nw;
      if (pt < 2) {
        const float sg = (pt == 0) ? 1.f : -1.f;
#pragma unroll
        for (int r = 0; r < R; r++) w[r] = (vv[r] < NUM) ? sg * sm.W[pown][vv[r]] : 0.f;
        nw = sm.W[pown][pown];
      } else {
        const int ip = (pown >> 1) + 1, h = pown & 1;
        const float ah = h ? ga1 : ga0, bh = h ? gb1 : gb0;
        float np[R];
#pragma unroll
        for (int r = 0; r < R; r++) {
          np[r] = 0.f;
          if (valid[r] && kk[r] < ip) {
            const float d = (float)(ip - 1 - kk[r]);
            if (a == 0) np[r] = ah * (MF.b00 + MF.a02 * MF.b20 * d) + bh * (MF.b10 + MF.a12 * MF.b20 * d);
            else np[r] = (ah * MF.a02 + bh * MF.a12) * MF.b21 * d;
          }
          sm.vec[vv[r]] = np[r];
        }
        wsync();
        matvec_W<NUM, GAP, R>(sm, lane, w);
        float s = 0.f;
#pragma unroll
        for (int r = 0; r < R; r++) s += np[r] * w[r];
        nw = wave_sum(s);
      }
      STAMP_ACC(acc_w, t_a);
      STAMP(t_b);
      // v_j = n_j' W n_p for the active slots
      float vj[R];
      if constexpr (GAP) {
        // = V_j' n_p (W symmetric, V_j = W n_j stored at slot j's add): a box candidate reads one
        // entry of each V row, a gap candidate dots the slot's row with n_p, still in sm.vec from
        // the W product; no rollout of w, no LDS round trip through stX / stY and no barrier
        if (pt < 2) {
          const float sg = (pt == 0) ? 1.f : -1.f;
#pragma unroll
          for (int r = 0; r < R; r++) {
            const int sl = 64 * r + lane;
            vj[r] = (sl < q) ? sg * sm.V[sl < NUM ? sl : NUM - 1][pown] : 0.f;
          }
        } else {
          const float4* x4 = reinterpret_cast<const float4*>(sm.vec);
#pragma unroll
          for (int r = 0; r < R; r++) {
            const int sl = 64 * r + lane;
            const float4* v4 = reinterpret_cast<const float4*>(sm.V[sl < NUM ? sl : NUM - 1]);
            float d0 = 0.f, d1 = 0.f, d2 = 0.f, d3 = 0.f;
#pragma unroll
            for (int j4 = 0; j4 < NUM / 4; j4++) {
              const float4 xv4 = x4[j4], vv4 = v4[j4];
              d0 = fmaf(vv4.x, xv4.x, d0);
              d1 = fmaf(vv4.y, xv4.y, d1);
              d2 = fmaf(vv4.z, xv4.z, d2);
              d3 = fmaf(vv4.w, xv4.w, d3);
            }
            vj[r] = (sl < q) ? (d0 + d1) + (d2 + d3) : 0.f;
          }
        }
      } else {
#pragma unroll
        for (int r = 0; r < R; r++) sm.vec2[vv[r]] = w[r];
        wsync();
#pragma unroll
        for (int r = 0; r < R; r++)
          vj[r] = (64 * r + lane < q) ? slot_dot<NUM, GAP>(sm, slot_id[r], ga0, ga1, gb0, gb1) : 0.f;
      }
      STAMP_ACC(acc_vj, t_b);
      STAMP(t_c);
      // l = L^-1 v ; r = L^-T l  (r = S_A^-1 N_A' W n_p : dual step direction)
      float lv[R], rr[R];
      tri_forward<NUM, GAP, R>(sm, lane, q, rdiag, vj, lv);
      float lls = 0.f;
#pragma unroll
      for (int r = 0; r < R; r++) lls += (64 * r + lane < q) ? lv[r] * lv[r] : 0.f;
      const float ll = wave_sum(lls);
      tri_backward<NUM, GAP, R>(sm, lane, q, rdiag, lv, rr);
      STAMP_ACC(acc_tri, t_c);
      STAMP(t_d);
      // z = w - sum_j r_j V[j]  (primal step direction)
      float z[R], z2[R];  // two accumulator chains (even / odd slots of a block)
#pragma unroll
      for (int r = 0; r < R; r++) { z[r] = w[r]; z2[r] = 0.f; }
      int j = 0;
      if constexpr (GAP) {  // V rows in blocks: the block's loads first (see tri_forward)
        for (; j + kTriBlock <= q; j += kTriBlock) {
          float vb[kTriBlock][R];
#pragma unroll
          for (int jb = 0; jb < kTriBlock; jb++)
#pragma unroll
            for (int r = 0; r < R; r++) vb[jb][r] = sm.V[j + jb][cl[r]];
#pragma unroll
          for (int jb = 0; jb < kTriBlock; jb++) {
            const float rj = rl_f<R>(rr, j + jb);
#pragma unroll
            for (int r = 0; r < R; r++) {
              if (jb & 1) z2[r] = fmaf(-rj, vb[jb][r], z2[r]);
              else z[r] = fmaf(-rj, vb[jb][r], z[r]);
            }
          }
        }
      }
#pragma unroll
      for (int r = 0; r < R; r++) z[r] += z2[r];
      for (; j < q; j++) {
        const float rj = rl_f<R>(rr, j);
        const int sj = GAP ? 0 : rl_i<R>(slot_id, j);
#pragma unroll
        for (int r = 0; r < R; r++) z[r] = fmaf(-rj, vcol<NUM, GAP>(sm, j, sj, cl[r]), z[r]);
      }
      const float pivv = nw - ll;  // = z' n_p, the new Schur pivot
      STAMP_ACC(acc_z, t_d);
      STAMP(t_e);
      // partial step t1 (blocking multiplier k1)
      float t1 = 3.0e38f;
      int k1 = 0x7fffffff;
#pragma unroll
      for (int r = 0; r < R; r++) {
        const int s = 64 * r + lane;
        if (s < q && rr[r] > 0.f) {
          // (v_rcp: the ratio only ranks the blocking slot and sets the partial step, whose point
          // the fp64 refinement corrects; an IEEE division is ~10 dependent instructions)
          const float tr = mult[r] * __builtin_amdgcn_rcpf(rr[r]);
          if (tr < t1) { t1 = tr; k1 = s; }
        }
      }
      wave_argmin(t1, k1);
      const bool dep = !(pivv > 1e-5f * nw);  // n_p (numerically) in span of the active set
      const float t2 = dep ? 3.0e38f : -sp / pivv;
      const float t = fminf(t1, t2);
      if (t >= 3.0e38f) { status = F110QP_PRIMAL_INFEASIBLE_ID; break; }
#pragma unroll
      for (int r = 0; r < R; r++)
        if (64 * r + lane < q) mult[r] -= t * rr[r];
      uplus_new += t;
      bool add = false;
      if (!dep) {
#pragma unroll
        for (int r = 0; r < R; r++)
          if (valid[r]) xv[r] = fmaf(t, z[r], xv[r]);
        sp = fmaf(t, pivv, sp);
        add = (t2 <= t1);
      }
      wsync();
      STAMP_ACC(acc_step, t_e);
      STAMP(t_f);
      if (add) {
        if (q >= NUM) { status = F110QP_MAX_ITER_ID; break; }
#pragma unroll
        for (int r = 0; r < R; r++) {
          const int s = 64 * r + lane;
          if (GAP && vv[r] < NUM) sm.V[q][vv[r]] = w[r];
          if (s < q) sm.L[q][s] = lv[r];
          if (s == q) {
            slot_id[r] = p;
            mult[r] = uplus_new;
            rdiag[r] = 1.f / sqrtf(pivv);
          }
          if (vv[r] == pown) actf[r] |= (1 << pt);
        }
        if (lane == 0) sm.L[q][q] = sqrtf(pivv);
        q++;
        wsync();
        STAMP_ACC(acc_upd, t_f);
        break;
      }
      // drop slot k1, then retry p
      {
        const int kd = k1;
        const int did = rl_i<R>(slot_id, kd);
        const int down = did / 3;
#pragma unroll
        for (int r = 0; r < R; r++)
          if (vv[r] == down) actf[r] &= ~(1 << (did - 3 * down));
        // slots kd+1..q-1 move down by one (lane shift, carrying across register rows)
        int sid_n[R];
        float mul_n[R];
#pragma unroll
        for (int r = 0; r < R; r++) {
          sid_n[r] = __shfl_down(slot_id[r], 1, 64);
          mul_n[r] = __shfl_down(mult[r], 1, 64);
          if (r + 1 < R) {
            const int s_next = readlane_i(slot_id[r + 1 < R ? r + 1 : r], 0);
            const float m_next = readlane_f(mult[r + 1 < R ? r + 1 : r], 0);
            if (lane == 63) { sid_n[r] = s_next; mul_n[r] = m_next; }
          }
        }
#pragma unroll
        for (int r = 0; r < R; r++) {
          const int s = 64 * r + lane;
          if (s >= kd && s < q - 1) { slot_id[r] = sid_n[r]; mult[r] = mul_n[r]; }
          if (s == q - 1) { slot_id[r] = -1; mult[r] = 0.f; }
        }
        if (GAP) {
          // remove slot kd from V (rows): every lane moves only its own column
#pragma unroll
          for (int r = 0; r < R; r++)
            if (vv[r] < NUM)
              for (int j = kd; j < q - 1; j++) sm.V[j][vv[r]] = sm.V[j + 1][vv[r]];
        }
        chol_delete<NUM, GAP, R>(sm, lane, q, kd, rdiag);
        q--;
        wsync();
      }
    }
  }

  STAMP(t_gi);
  if constexpr (!GAP) {
    // box rows: GI's point is certified like the PDAS one, in fp64 (its set, a fresh T, the
    // refined point, the exact KKT check); and a box (u_min <= u_max, checked at create) is never
    // empty, so GI's infeasibility there is a numerical breakdown
    if (gi_fallback && final_ok && status == F110QP_SOLVED_ID) {
#pragma unroll
      for (int r = 0; r < R; r++) act[r] = (actf[r] & 1) ? 1 : ((actf[r] & 2) ? 2 : 0);
      fresh_T();
      const bool conv = refine(3, kRobTight, kRobTol, kRobSteps);
      inexact = !conv || kkt_violated();
    }
    if (gi_fallback && status == F110QP_PRIMAL_INFEASIBLE_ID) status = F110QP_NUMERICAL_ID;
  }
  // ---- 6. outputs ---------------------------------------------------------------------------
  if (status == F110QP_SOLVED_ID && !final_ok) status = F110QP_MAX_ITER_ID;
  if (status == F110QP_SOLVED_ID && inexact) status = F110QP_SOLVED_INACCURATE_ID;
  const bool ok = (status == F110QP_SOLVED_ID) || (status == F110QP_SOLVED_INACCURATE_ID);
  {
    double uo[R], px[R], py[R], th[R];
#pragma unroll
    for (int r = 0; r < R; r++) uo[r] = (ok && valid[r]) ? u64[r] : 0.0;
    rollout_f64<R>(sm.M, lane, uo, px, py, th);
    const float nanv = __int_as_float(0x7fc00000);
    float* xo = xout + (size_t)b * 3 * (N + 1);
    if (lane == 0) {
      xo[0] = ok ? fX0 : nanv;
      xo[1] = ok ? fY0 : nanv;
      xo[2] = ok ? fTH0 : nanv;
    }
#pragma unroll
    for (int r = 0; r < R; r++) {
      if (valid[r]) uout[(size_t)b * NU + vv[r]] = ok ? (float)u64[r] : nanv;
      if (valid[r] && a == 1) {
        xo[3 * (kk[r] + 1) + 0] = ok ? (float)(px[r] + X0) : nanv;
        xo[3 * (kk[r] + 1) + 1] = ok ? (float)(py[r] + Y0) : nanv;
        xo[3 * (kk[r] + 1) + 2] = ok ? (float)th[r] : nanv;
      }
    }
    if (oo.obj || oo.cost) {
      // objective (fp64): cost = sum_{i=0..N} 1/2|x_i - r_i|_Q^2 + sum 1/2|u - u_des|_R^2 (r_N =
      // x_ref[N-1], mpc.cpp:228; odd lanes hold stage kk+1, lane 0 stage 0), and OSQP's
      // 1/2 z'Pz + q'z = cost - 1/2 sum r_i'Q r_i - N/2 u_des'R u_des (world coordinates)
      const double q0 = P.q[0], q1 = P.q[1], q2 = P.q[2];
      double J = 0.0, Cr = 0.0;
#pragma unroll
      for (int r = 0; r < R; r++) {
        if (!valid[r]) continue;
        const double ra = a ? P.r[1] : P.r[0], uda = a ? P.udes[1] : P.udes[0];
        J += 0.5 * ra * (uo[r] - uda) * (uo[r] - uda);
        if (a == 1) {
          const double dx = px[r] - sm.rx[vv[r]], dy = py[r] - sm.ry[vv[r]];
          const double rth = (double)sm.rth[vv[r]], dth = th[r] - rth;
          J += 0.5 * (q0 * dx * dx + q1 * dy * dy + q2 * dth * dth);
          const double wx = sm.rx[vv[r]] + X0, wy = sm.ry[vv[r]] + Y0;
          Cr += 0.5 * (q0 * wx * wx + q1 * wy * wy + q2 * rth * rth);
        }
      }
      if (lane == 0) {  // stage 0: x_0 = x0 (fixed by the dynamics rows) against x_ref[0]
        const double e0 = X0 - (double)x00[0], e1 = Y0 - (double)x00[1], e2 = (double)fTH0 - (double)x00[2];
        J += 0.5 * (q0 * e0 * e0 + q1 * e1 * e1 + q2 * e2 * e2);
        const double w0 = x00[0], w1 = x00[1], w2 = x00[2];
        Cr += 0.5 * (q0 * w0 * w0 + q1 * w1 * w1 + q2 * w2 * w2);
      }
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) {
        J += __shfl_xor(J, o);
        Cr += __shfl_xor(Cr, o);
      }
      const double Cu = 0.5 * (double)N * (P.r[0] * P.udes[0] * P.udes[0] + P.r[1] * P.udes[1] * P.udes[1]);
      const double dnan = __longlong_as_double(0x7ff8000000000000ll);
      if (lane == 0 && oo.cost) oo.cost[b] = ok ? J : dnan;
      if (lane == 0 && oo.obj) oo.obj[b] = ok ? J - Cr - Cu : dnan;
    }
  }
  if (lane == 0) {
    status_out[b] = status;
    if (iters_out) iters_out[b] = it;
    // re-check list: every answer GI did not certify (an uncertified point, its cap, an
    // infeasibility found by the fp32 GI); non-finite data and a violated stage-0 row are exact
    if (oo.rc_list && status != F110QP_SOLVED_ID && !numerical && !infeasible0)
      oo.rc_list[atomicAdd(oo.rc_count, 1)] = b;
  }
  if (ws.act != nullptr && !grp && Hdbg == nullptr) {
#pragma unroll
    for (int r = 0; r < R; r++) {
      const unsigned long long lo_m = __ballot(ok && valid[r] && (actf[r] & 1));
      const unsigned long long hi_m = __ballot(ok && valid[r] && (actf[r] & 2));
      if (lane == 0) {
        ws.act[2 * (R * b + r)] = lo_m;
        ws.act[2 * (R * b + r) + 1] = hi_m;
      }
    }
  }
#ifdef F110QP_STAMPS
  STAMP(t_end);
  if (lane == 0 && b < 65536) {
    unsigned long long* o = g_stamps + (size_t)b * kStampSlots;
    o[0] = t_lin - t_start; o[1] = t_grad - t_inv; o[2] = t_hess - t_lin; o[3] = t_inv - t_hess;
    o[4] = t_gi - t_grad - acc_refine; o[5] = acc_refine; o[6] = t_end - t_gi; o[7] = t_end - t_start;
    o[8] = acc_s1; o[9] = acc_pdas + acc_w; o[10] = acc_vj; o[11] = acc_tri; o[12] = acc_z; o[13] = acc_step;
    o[14] = acc_upd; o[15] = it;
  }
#endif
}

// One QP per workgroup (= one wave). With `list` the grid walks the index list instead
// (count read on the device): the lane-per-QP kernel hands its non-converged QPs over this way.
template <int NUM, bool GAP>
#ifdef F110QP_SOLVE_WPE  // measurement knob: occupancy hint for the register allocator
#define F110QP_SOLVE_ATTR __attribute__((amdgpu_waves_per_eu(F110QP_SOLVE_WPE, F110QP_SOLVE_WPE)))
#else
#define F110QP_SOLVE_ATTR
#endif
__global__ __launch_bounds__(64) F110QP_SOLVE_ATTR void solve_kernel(const KParams P, const int B,
                                                   const float* __restrict__ x0g,
                                                   const float* __restrict__ ulg,
                                                   const float* __restrict__ xrg,
                                                   const float* __restrict__ hsg,
                                                   float* __restrict__ uout,
                                                   float* __restrict__ xout,
                                                   int* __restrict__ status_out,
                                                   int* __restrict__ iters_out,
                                                   double* __restrict__ Hdbg,
                                                   double* __restrict__ gdbg,
                                                   const WarmState ws,
                                                   const int* __restrict__ list,
                                                   const int* __restrict__ count,
                                                   const ObjOut oo) {
  __shared__ Smem<NUM, GAP> sm;
  const int n = list ? __builtin_amdgcn_readfirstlane(*count) : B;
  // XCD-aware order: workgroup i runs on XCD i mod 8, so with one workgroup per QP each XCD
  // takes a contiguous range of QPs and the 128-B lines of x_ref / u / x are fetched and
  // written back by one L2 only (a plain order splits every line over 8 L2s).
  const bool xcd = (list == nullptr) && ((int)gridDim.x == B);
  const int per = B >> 3, rem = B & 7;
  for (int item = blockIdx.x; item < n; item += gridDim.x) {
    const int xi = item & 7;
    const int b = list ? __builtin_amdgcn_readfirstlane(list[item])
                       : (xcd ? xi * per + (xi < rem ? xi : rem) + (item >> 3) : item);
    solve_qp<NUM, GAP>(sm, b, P, x0g, ulg, xrg, hsg, uout, xout, status_out, iters_out, Hdbg,
                       gdbg, ws, oo);
    wsync();
  }
  signal_call_done(oo);  // a synchronous box-only call's completion word (f110qp_kernels.h)
}

// Grouped mode, prepare launch: one wave per group builds the closed-form Hessian and the swept
// inverse of the group's leader (the smallest member index; none -> the slot is marked empty)
// and publishes W and the key of its linearisation point (theta0, v, delta) to the group slot.
template <int NUM, bool GAP>
__global__ __launch_bounds__(64) void group_prep_kernel(const KParams P, const int G,
                                                        const float* __restrict__ x0g,
                                                        const float* __restrict__ ulg,
                                                        const float* __restrict__ xrg,
                                                        const float* __restrict__ hsg,
                                                        const WarmState ws,
                                                        const int* __restrict__ leader,
                                                        const int B) {
  __shared__ Smem<NUM, GAP> sm;
  const int g = blockIdx.x;
  const int b = __builtin_amdgcn_readfirstlane(leader[g]);
  if (b < 0 || b >= B) {
    if (threadIdx.x == 0) ws.key[4 * g + 3] = 0u;
    return;
  }
  solve_qp<NUM, GAP>(sm, b, P, x0g, ulg, xrg, hsg, nullptr, nullptr, nullptr, nullptr, nullptr,
                     nullptr, ws, ObjOut(), g);
}

// ------------------------------------------------------------------------------------------
// launch of one instantiation
// ------------------------------------------------------------------------------------------
template <int NUM, bool GAP>
hipError_t launch_t(const KParams& P, int B, const float* x0, const float* ul, const float* xr,
                    const float* hs, float* uo, float* xo, int* st, int* its, double* Hd,
                    double* gd, const WarmState& ws, const int* list, const int* count, int grid,
                    const ObjOut& oo, hipStream_t s) {
  hipLaunchKernelGGL((solve_kernel<NUM, GAP>), dim3(grid), dim3(64), 0, s, P, B, x0, ul, xr, hs,
                     uo, xo, st, its, Hd, gd, ws, list, count, oo);
  return hipGetLastError();
}

template <int NUM, bool GAP>
hipError_t launch_prep_t(const KParams& P, int B, const float* x0, const float* ul,
                         const float* xr, const float* hs, const WarmState& ws, const int* leader,
                         hipStream_t s) {
  if (ws.ngroups <= 0) return hipSuccess;
  hipLaunchKernelGGL((group_prep_kernel<NUM, GAP>), dim3(ws.ngroups), dim3(64), 0, s, P,
                     ws.ngroups, x0, ul, xr, hs, ws, leader, B);
  return hipGetLastError();
}

}  // namespace f110qp

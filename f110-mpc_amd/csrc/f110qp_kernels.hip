// f110qp_kernels.hip — the MI355X (gfx950) hot path of the f110-mpc control tick.
//
// One 64-lane wavefront per QP instance (one workgroup = one wave), B instances per launch.
// Per instance, fused in one launch:
//   1. Model::Linearize                      (reference src/model.cpp:30-59)      fp64, uniform
//   2. condensing of the tick's QP           (src/mpc.cpp:208-306)                closed form
//      The dynamics rows x_{i+1} = A x_i + B u_i + C are eliminated. A = I + E with E^2 = 0
//      (model.cpp:42-46), so Gamma's entries are affine in the stage distance and every
//      Hessian entry H = R + Gamma'Q Gamma is an O(1) polynomial sum: lane v builds row v of
//      H in registers with no GEMM.
//   3. W = H^-1 by a symmetric Gauss-Jordan sweep, rows in VGPRs, pivot rows broadcast
//      through LDS.
//   4. the QP solve that OSQP does in the reference (src/mpc.cpp:133): a dual active-set
//      method (Goldfarb-Idnani, range-space form) on the condensed problem. The active
//      normals' W n_j and the Cholesky factor of S_A = N_A' W N_A live in LDS; the
//      triangular solves walk the active slots with one lane per slot and readlane
//      broadcasts. Box rows (mpc.cpp:253,281,290) and follow-the-gap rows
//      (mpc.cpp:249,271,297-298) are the constraint set.
//   5. two steps of iterative refinement whose residuals are evaluated in fp64 by an adjoint
//      (costate) recursion written as wave prefix/suffix scans, then an fp64 feasibility
//      re-check that re-enters step 4 if needed. Exact optimum to ~1e-9, not OSQP's 1e-3.
//   6. u* and the state rollout x* (MPC::UpdateSolvedTrajectory, mpc.cpp:145-159).
// Everything is recentred on (x0, y0): the dynamics and cost are translation invariant in
// (x, y) (model.cpp:42-55), which keeps fp32 exact to ~1e-6 for |x| ~ 50 m.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "f110qp_kernels.h"

namespace f110qp {

// Diagnostic build only (-DF110QP_STAMPS): per-phase s_memtime deltas of every wave, read back
// with f110qp_read_stamps(). The shipped library never executes a stamp.
#ifdef F110QP_STAMPS
constexpr int kStampSlots = 16;
__device__ unsigned long long g_stamps[65536 * kStampSlots];
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

// inclusive prefix sum over the 64 lanes (row shifts, then row broadcasts 15 and 31)
__device__ __forceinline__ float scan_incl(float x, int) {
  x += dpp_f<DPP_ROW_SHR1>(x);
  x += dpp_f<DPP_ROW_SHR2>(x);
  x += dpp_f<DPP_ROW_SHR4>(x);
  x += dpp_f<DPP_ROW_SHR8>(x);
  x += dpp_f<DPP_ROW_BCAST15, 0xa>(x);
  x += dpp_f<DPP_ROW_BCAST31, 0xc>(x);
  return x;
}
__device__ __forceinline__ double scan_incl(double x, int) {
  x += dpp_d<DPP_ROW_SHR1>(x);
  x += dpp_d<DPP_ROW_SHR2>(x);
  x += dpp_d<DPP_ROW_SHR4>(x);
  x += dpp_d<DPP_ROW_SHR8>(x);
  x += dpp_d<DPP_ROW_BCAST15, 0xa>(x);
  x += dpp_d<DPP_ROW_BCAST31, 0xc>(x);
  return x;
}
// inclusive suffix sum: total - inclusive prefix + own
template <typename T>
__device__ __forceinline__ T scan_suffix_incl(T x, int lane) {
  const T p = scan_incl(x, lane);
  T tot;
  if constexpr (sizeof(T) == 8) tot = readlane_d(p, 63);
  else tot = readlane_f(p, 63);
  return tot - p + x;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
  const T p = scan_incl(v, 0);
  if constexpr (sizeof(T) == 8) return readlane_d(p, 63);
  else return readlane_f(p, 63);
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

// ------------------------------------------------------------------------------------------
// linearised model, fp64 (model.cpp:30-59; L = 0.3302f at :32; dt is the float MPC::dt_)
// ------------------------------------------------------------------------------------------
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

// Forward rollout of u (one value per lane, lane = variable 2k+a) in fp64.
// Returns the recentred state after stage k (i = k+1) in both lanes of the stage.
__device__ __forceinline__ void rollout_f64(const Lin& M, int lane, double uval, double& px,
                                            double& py, double& th) {
  const int k = lane >> 1, a = lane & 1;
  const double beta = a ? M.b21 : M.b20;
  double s1 = beta * uval;
  double s2 = (double)k * s1;
  double s3 = a ? 0.0 : uval;
  s1 = scan_incl(s1, lane);
  s2 = scan_incl(s2, lane);
  s3 = scan_incl(s3, lane);
  const double P1 = odd_lane(s1), P2 = odd_lane(s2), V = odd_lane(s3);
  const double i = (double)(k + 1);
  th = M.th0 + i * M.c2 + P1;
  const double sth = i * M.th0 + M.c2 * (i * (i - 1.0) * 0.5) + (i - 1.0) * P1 - P2;
  px = i * M.c0 + M.a02 * sth + M.b00 * V;
  py = i * M.c1 + M.a12 * sth + M.b10 * V;
}

// Linear part of the rollout (Gamma w, zero initial state, no affine term), fp32.
__device__ __forceinline__ void rollout_lin_f32(float a02, float a12, float b00, float b10,
                                                float b20, float b21, int lane, float w,
                                                float& X, float& Y) {
  const int k = lane >> 1, a = lane & 1;
  const float beta = a ? b21 : b20;
  float s1 = beta * w;
  float s2 = (float)k * s1;
  float s3 = a ? 0.f : w;
  s1 = scan_incl(s1, lane);
  s2 = scan_incl(s2, lane);
  s3 = scan_incl(s3, lane);
  const float P1 = odd_lane(s1), P2 = odd_lane(s2), V = odd_lane(s3);
  const float sth = (float)k * P1 - P2;  // (i-1)P1 - P2 with i = k+1
  X = a02 * sth + b00 * V;
  Y = a12 * sth + b10 * V;
}

// Gradient of the tracking objective (mpc.cpp:208-229 cost) minus the gap-row multiplier
// terms, at u, by the costate recursion lambda_i = Q(x_i - r_i) - mu_i n_i + A' lambda_{i+1},
// written as suffix scans. px,py,th are the lane-stage states from rollout_f64.
__device__ __forceinline__ double grad_f64(const Lin& M, const KParams& P, int lane, int N,
                                           double uval, double px, double py, double th,
                                           double rx, double ry, double rth, double gmx,
                                           double gmy) {
  const int k = lane >> 1, a = lane & 1;
  const bool contrib = (a == 1) && (k < N);
  const double i = (double)(k + 1);
  double ex = contrib ? P.q[0] * (px - rx) - gmx : 0.0;
  double ey = contrib ? P.q[1] * (py - ry) - gmy : 0.0;
  double et = contrib ? P.q[2] * (th - rth) : 0.0;
  double lx = i * ex, ly = i * ey;
  ex = scan_suffix_incl(ex, lane);
  lx = scan_suffix_incl(lx, lane);
  ey = scan_suffix_incl(ey, lane);
  ly = scan_suffix_incl(ly, lane);
  et = scan_suffix_incl(et, lane);
  const double lth = et + M.a02 * (lx - i * ex) + M.a12 * (ly - i * ey);
  const double g = a ? (P.r[1] * (uval - P.udes[1]) + M.b21 * lth)
                     : (P.r[0] * (uval - P.udes[0]) + M.b00 * ex + M.b10 * ey + M.b20 * lth);
  return (k < N) ? g : 0.0;
}

// ------------------------------------------------------------------------------------------
// shared memory of one wave / one QP
// ------------------------------------------------------------------------------------------
template <int NUM>
struct Smem {
  // first and 16-B aligned: small immediate offsets, ds_read_b128 broadcasts in the sweep
  alignas(16) float colbuf[2][64];  // sweep: pivot column all-gather (double buffered)
  alignas(16) float W[NUM][NUM];    // W = H^-1, row-major (symmetric: row p == column p)
  float V[NUM][NUM];       // V[slot][var] = W n_slot
  float S[NUM][NUM + 1];   // S_A = N_A' W N_A
  float L[NUM][NUM + 1];   // Cholesky factor of S_A (lower)
  float vec[64];           // broadcast scratch (one entry per lane)
  float vec2[64];
  float stX[33], stY[33];  // per-stage linear rollout (stage 1..N)
  float rx[64], ry[64], rth[64];  // recentred reference of the lane's stage
  float cmult[3 * 64];     // multiplier per constraint id
  int ids[64];             // PDAS: constraint id of each active slot
  float pmu[64];           // PDAS: multiplier of each variable's active bound
  double d64[64];
  double sx64[33], sy64[33];
  Lin M;                   // linearisation of this QP (uniform)
};

// l = L^-1 v, one lane per active slot (v, l in lane j for slot j < q); L read from LDS.
// A plain q-step loop: the slot count is uniform, each step is mul -> readlane -> fma.
template <int NUM>
__device__ __forceinline__ float tri_forward(Smem<NUM>& sm, int lane, int q, float rdiag,
                                             float v) {
  float acc = v, lv = 0.f;
  const int row = lane < NUM ? lane : NUM - 1;
  for (int kk = 0; kk < q; kk++) {
    const float t = acc * rdiag;
    const float lk = readlane_f(t, kk);
    lv = (lane == kk) ? t : lv;
    acc = fmaf(-sm.L[row][kk], lk, acc);
  }
  return lv;
}

// r = L^-T l (backward substitution, column-oriented)
template <int NUM>
__device__ __forceinline__ float tri_backward(Smem<NUM>& sm, int lane, int q, float rdiag,
                                              float l) {
  float acc = l, r = 0.f;
  const int col = lane < NUM ? lane : NUM - 1;
  for (int jj = q - 1; jj >= 0; jj--) {
    const float t = acc * rdiag;
    const float rj = readlane_f(t, jj);
    r = (lane == jj) ? t : r;
    acc = fmaf(-sm.L[jj][col], rj, acc);
  }
  return r;
}

// L = chol(S_A) of the q active slots (left-looking, one lane per row, S and L in LDS).
// Returns this lane's 1/L[lane][lane] (unchanged value `rd` for lanes >= q).
template <int NUM>
__device__ __forceinline__ float chol_slots(Smem<NUM>& sm, int lane, int q, float rd) {
  for (int c = 0; c < q; c++) {
    float s = 0.f;
    if (lane < q && lane >= c) {
      float s0 = sm.S[lane][c], s1 = 0.f, s2 = 0.f, s3 = 0.f;
      int i2 = 0;
      for (; i2 + 4 <= c; i2 += 4) {  // four independent chains: the LDS reads pipeline
        s0 = fmaf(-sm.L[lane][i2 + 0], sm.L[c][i2 + 0], s0);
        s1 = fmaf(-sm.L[lane][i2 + 1], sm.L[c][i2 + 1], s1);
        s2 = fmaf(-sm.L[lane][i2 + 2], sm.L[c][i2 + 2], s2);
        s3 = fmaf(-sm.L[lane][i2 + 3], sm.L[c][i2 + 3], s3);
      }
      for (; i2 < c; i2++) s0 = fmaf(-sm.L[lane][i2], sm.L[c][i2], s0);
      s = (s0 + s1) + (s2 + s3);
    }
    const float dcc = sqrtf(readlane_f(s, c));
    if (lane < q && lane >= c) sm.L[lane][c] = (lane == c) ? dcc : s / dcc;
    if (lane == c) rd = 1.f / dcc;
    wsync();
  }
  return rd;
}

// y_lane = sum_j W[lane][j] x_j with x in sm.vec; W symmetric so lane reads column `lane`
// (consecutive addresses across lanes, conflict free). Lanes >= NUM return 0.
template <int NUM>
__device__ __forceinline__ float matvec_W(Smem<NUM>& sm, int lane) {
  const int c = lane < NUM ? lane : NUM - 1;
  float y = 0.f;
#pragma unroll
  for (int j = 0; j < NUM; j++) y = fmaf(sm.W[j][c], sm.vec[j], y);
  return lane < NUM ? y : 0.f;
}

// n_j' w for the active slot held by this lane (w in sm.vec2 by variable, gap rows from the
// per-stage linear rollout in sm.stX/stY).
template <int NUM>
__device__ __forceinline__ float slot_dot(Smem<NUM>& sm, int slot_id, float ga0, float ga1,
                                          float gb0, float gb1) {
  const int owner = slot_id / 3, t = slot_id - 3 * owner;
  if (t == 0) return sm.vec2[owner];
  if (t == 1) return -sm.vec2[owner];
  const int st = (owner >> 1) + 1;
  return ((owner & 1) ? ga1 : ga0) * sm.stX[st] + ((owner & 1) ? gb1 : gb0) * sm.stY[st];
}

// One pivot of the symmetric sweep operator (Goodnight 1979) on the row held by this lane:
//   a_ij -= a_ip a_pj / a_pp ; a_ip /= a_pp ; a_pj /= a_pp ; a_pp = -1/a_pp.
// The pivot column is all-gathered through LDS; the pivot row's own update folds into the common FMA with
// f = 1 - 1/a_pp. After all pivots the rows hold -H^-1. P is a template constant so every
// register index is static (no scratch).
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int NUM, int P>
__device__ __forceinline__ void sweep_step(Smem<NUM>& sm, float (&hrow)[NUM], int lane) {
  // pivot row broadcast by readlane (lane P, static register index) -> SGPR operands
  float rk[NUM];
#pragma unroll
  for (int j = 0; j < NUM; j++) rk[j] = readlane_f(hrow[j], P);
  const float inv = __builtin_amdgcn_rcpf(rk[P]);  // 1 ulp; the fp64 refinement absorbs it
  const bool piv = (lane == P);
  const float hp = hrow[P];
  const float f = piv ? (1.f - inv) : hp * inv;
  const f32x2 nf = {-f, -f};
#pragma unroll
  for (int j = 0; j < NUM; j += 2) {  // packed FMA over column pairs (v_pk_fma_f32)
    const f32x2 r = {rk[j], rk[j + 1]};
    f32x2 h = {hrow[j], hrow[j + 1]};
    h = __builtin_elementwise_fma(nf, r, h);
    hrow[j] = h.x;
    hrow[j + 1] = h.y;
  }
  hrow[P] = piv ? -inv : hp * inv;
}

template <int NUM, int P>
struct Sweep {
  static __device__ __forceinline__ void run(Smem<NUM>& sm, float (&hrow)[NUM], int lane) {
    sweep_step<NUM, P>(sm, hrow, lane);
    Sweep<NUM, P + 1>::run(sm, hrow, lane);
  }
};
template <int NUM>
struct Sweep<NUM, NUM> {
  static __device__ __forceinline__ void run(Smem<NUM>&, float (&)[NUM], int) {}
};

// constraint ids: id = 3*owner_lane + t, t = 0 box lower, 1 box upper, 2 gap (stage owner/2+1,
// side owner&1)

template <int NUM, bool GAP>
__global__ __launch_bounds__(64) void solve_kernel(const KParams P, const int B,
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
                                                   const WarmState ws) {
  __shared__ Smem<NUM> sm;
  const int b = blockIdx.x;
  if (b >= B) return;
  const int lane = threadIdx.x;
  const int N = P.N;
  const int NU = 2 * N;
  const int k = lane >> 1;   // input stage of this lane's variable
  const int a = lane & 1;    // 0 = speed v, 1 = steering
  const bool valid = lane < NU;

  STAMP(t_start);
#ifdef F110QP_STAMPS
  unsigned long long acc_refine = 0, acc_s1 = 0, acc_w = 0, acc_vj = 0, acc_tri = 0, acc_z = 0,
                     acc_step = 0, acc_upd = 0, acc_pdas = 0;
#endif
  // ---- 1. inputs + Model::Linearize ----------------------------------------------------
  const float fX0 = x0g[3 * b + 0], fY0 = x0g[3 * b + 1], fTH0 = x0g[3 * b + 2];
  const double X0 = (double)fX0, Y0 = (double)fY0;
  {
    const Lin M = linearize((double)fTH0, (double)ulg[2 * b + 0], (double)ulg[2 * b + 1], P.dt);
    if (lane == 0) sm.M = M;
    // reference point of the lane's state stage i = k+1 (terminal reuses x_ref[N-1],
    // mpc.cpp:228). (x_ref - x0) of two floats within a few metres is exact in fp32.
    float rx = 0.f, ry = 0.f, rth = 0.f;
    if (valid) {
      const int ri = (k + 1 < N) ? k + 1 : N - 1;
      const float* xr = xrg + ((size_t)b * N + ri) * 3;
      rx = (float)((double)xr[0] - X0);
      ry = (float)((double)xr[1] - Y0);
      rth = xr[2];
    }
    sm.rx[lane] = rx; sm.ry[lane] = ry; sm.rth[lane] = rth;
  }
  const float umin0 = P.umin[0], umin1 = P.umin[1], umax0 = P.umax[0], umax1 = P.umax[1];
  const float lb = valid ? (a ? umin1 : umin0) : -3.0e38f;
  const float ub = valid ? (a ? umax1 : umax0) : 3.0e38f;

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

  // warm start: does the cached W of this slot belong to the same linearisation point?
  const bool warm = ws.W != nullptr && Hdbg == nullptr;
  bool whit = false, wvalid = false;
  if (warm) {
    const unsigned* kk = ws.key + 4 * b;
    wvalid = kk[3] == 1u;
    whit = wvalid && kk[0] == __float_as_uint(fTH0) && kk[1] == __float_as_uint(ulg[2 * b + 0]) &&
           kk[2] == __float_as_uint(ulg[2 * b + 1]);
  }
  STAMP(t_lin);
  // ---- 2a. gradient at u = 0 (fp64 adjoint) and the free response ------------------------
  float cgap = 0.f, gnorm = 1.f;
  {
    const Lin M = sm.M;
    double px0, py0, th0s;
    rollout_f64(M, lane, 0.0, px0, py0, th0s);
    // cross-lane helpers run with all 64 lanes active (lanes >= 2N contribute zeros)
    const double g64a = grad_f64(M, P, lane, N, 0.0, px0, py0, th0s, (double)sm.rx[lane],
                                 (double)sm.ry[lane], (double)sm.rth[lane], 0.0, 0.0);
    const double g64 = valid ? g64a : 0.0;
    sm.vec[lane] = (float)g64;
    if (Hdbg && valid) gdbg[(size_t)b * NU + lane] = g64;
    if (GAP) {
      const double gah = a ? ga1 : ga0, gbh = a ? gb1 : gb0, gbe = a ? gbeta1 : gbeta0;
      cgap = (float)(gah * px0 + gbh * py0 - gbe);  // slack = a X + b Y + cgap
      gnorm = (float)sqrt(gah * gah + gbh * gbh) + 1.f;
    }
  }

  STAMP(t_grad);
  STAMP(t_hess);
  STAMP(t_inv);
  if (whit) {
    // ---- 2b/3 (warm hit): W from the slot cache, no Hessian, no sweep ------------------
    const float g32w = sm.vec[lane];
    const float* Wc = ws.W + (size_t)b * NU * NU;
    const int cl = lane < NUM ? lane : NUM - 1;
#pragma unroll 4
    for (int j = 0; j < NUM; j++) {
      float wv = (j == lane) ? 1.f : 0.f;
      if (j < NU && valid) wv = Wc[(size_t)j * NU + lane];
      if (lane < NUM) sm.W[j][cl] = wv;
    }
    wsync();
    sm.vec[lane] = g32w;
    wsync();
  } else {
  // ---- 2b. condensed Hessian row (closed form, fp32) --------------------------------------
  // Row v = (k, a), column w = (l, b). For l <= k the stages that see both inputs are
  // i = k+1..N (T = N-k of them), and Gamma_i[:, w] is affine in the stage distance, so
  //   H[v][w] = C0_b + C1_b * (k - l)
  // with four per-lane constants (sums of 1, t, t^2 over the T stages). The entries with
  // l > k are the transpose: every lane publishes its lower row and reads column v back.
  float hrow[NUM];
  {
    const Lin M = sm.M;
    const float fa02 = (float)M.a02, fa12 = (float)M.a12, fb00 = (float)M.b00;
    const float fb10 = (float)M.b10, fb20 = (float)M.b20, fb21 = (float)M.b21;
    const float q0 = (float)P.q[0], q1 = (float)P.q[1], q2 = (float)P.q[2];
    const float ra = a ? (float)P.r[1] : (float)P.r[0];
    const float T = (float)(N - k);
    const float S1 = T * (T - 1.f) * 0.5f;
    const float S2 = (T - 1.f) * T * (2.f * T - 1.f) * (1.f / 6.f);
    const float beta_a = a ? fb21 : fb20;
    const float pxa = a ? 0.f : fb00, pya = a ? 0.f : fb10;  // dk = 0 in this regime
    const float sxa = fa02 * beta_a, sya = fa12 * beta_a;
    const float Ux = T * pxa + sxa * S1, Vx = pxa * S1 + sxa * S2;
    const float Uy = T * pya + sya * S1, Vy = pya * S1 + sya * S2;
    float C0[2], C1[2];
#pragma unroll
    for (int bb = 0; bb < 2; bb++) {
      const float beta_b = bb ? fb21 : fb20;
      const float ax_b = bb ? 0.f : fb00, ay_b = bb ? 0.f : fb10;
      const float sxb = fa02 * beta_b, syb = fa12 * beta_b;
      C0[bb] = q0 * (ax_b * Ux + sxb * Vx) + q1 * (ay_b * Uy + syb * Vy) + q2 * T * beta_a * beta_b;
      C1[bb] = q0 * sxb * Ux + q1 * syb * Uy;
    }
    float lower[NUM];
#pragma unroll
    for (int w = 0; w < NUM; w++) {
      const int l = w >> 1, bb = w & 1;
      lower[w] = fmaf(C1[bb], (float)(k - l), C0[bb]);
    }
    if (lane < NUM) {
#pragma unroll
      for (int w = 0; w < NUM; w++) sm.W[lane][w] = lower[w];
    }
    wsync();
    const int cl = lane < NUM ? lane : NUM - 1;
#pragma unroll
    for (int w = 0; w < NUM; w++) {
      const int l = w >> 1;
      float h = (l <= k) ? lower[w] : sm.W[w][cl];
      if (w == lane) h += ra;
      const bool ok = valid && (w < NU);
      hrow[w] = ok ? h : (w == lane ? 1.f : 0.f);
    }
    wsync();
  }
  if (Hdbg) {  // debug/parity hook: dump H (g was written above), no solve
    if (valid) {
#pragma unroll
      for (int w = 0; w < NUM; w++)
        if (w < NU) Hdbg[((size_t)b * NU + lane) * NU + w] = (double)hrow[w];
    }
    return;
  }
  const float g32 = sm.vec[lane];
  wsync();
  STAMP_SET(t_hess);
  // ---- 3. W = H^-1 : symmetric sweep (Goodnight), row `lane` in registers ----------------
  sm.colbuf[0][lane] = hrow[0];
  Sweep<NUM, 0>::run(sm, hrow, lane);
  if (lane < NUM) {
#pragma unroll
    for (int j = 0; j < NUM; j++) sm.W[lane][j] = -hrow[j];  // the sweep leaves -H^-1
  }
  wsync();
  sm.vec[lane] = g32;
  if (warm) {  // prime the slot cache (coalesced: lane v writes column v of every row)
    float* Wc = ws.W + (size_t)b * NU * NU;
    const int cl = lane < NUM ? lane : NUM - 1;
    for (int j = 0; j < NU; j++)
      if (valid) Wc[(size_t)j * NU + lane] = sm.W[j][cl];
    if (lane == 0) {
      unsigned* kk = ws.key + 4 * b;
      kk[0] = __float_as_uint(fTH0);
      kk[1] = __float_as_uint(ulg[2 * b + 0]);
      kk[2] = __float_as_uint(ulg[2 * b + 1]);
      kk[3] = 1u;
    }
  }
  wsync();
  }  // !whit

  STAMP_SET(t_inv);
  // ---- 4. dual active set (Goldfarb-Idnani, range space) ---------------------------------
  // x = -W g  (g in sm.vec)
  float xv = valid ? -matvec_W<NUM>(sm, lane) : 0.f;
  wsync();

  int actf = 0;          // bit t set when constraint 3*lane+t is active
  int slot_id = -1;      // constraint id of active slot `lane`
  float mult = 0.f;      // its multiplier
  float rdiag = 0.f;     // 1 / L[lane][lane]
  int q = 0;
  int it = 0;
  const int max_iter = P.max_iter;
  int status = infeasible0 ? F110QP_PRIMAL_INFEASIBLE_ID : F110QP_SOLVED_ID;
  int reentries = 0;
  double u64 = 0.0;
  bool final_ok = false;
  int forced_p = -1;     // violated row found by the fp64 re-check
  float forced_sp = 0.f;

  // ---- 4a. box rows only: primal-dual active set warm start (Hintermueller-Ito-Kunisch) ----
  // Each pass solves the equality QP of the current guess by one Schur solve with S_A =
  // W[A][A] and re-guesses A from the multipliers and the bounds; on these QPs it reaches
  // the optimal set in <= 5 passes (one-at-a-time GI needs one pass per active bound). Its
  // fixed point is a valid GI state (independent normals, positive multipliers), so the GI
  // loop below only confirms it, and resumes from it if the fp64 re-check finds a violated
  // row. No convergence within kPdasMaxIter passes -> plain GI from the unconstrained point.
  if (!GAP && status == F110QP_SOLVED_ID) {
    STAMP(t_pdas);
    constexpr int kPdasMaxIter = 10;
    const float uunc = xv;
    sm.vec[lane] = uunc;
    const int cl = lane < NUM ? lane : NUM - 1;
    int act = 0;           // 0 free, 1 at the lower bound, 2 at the upper bound
    if (warm && wvalid && valid) {  // previous tick's active bounds seed the first guess
      const unsigned long long lo_m = ws.act[2 * b], hi_m = ws.act[2 * b + 1];
      act = ((lo_m >> lane) & 1ull) ? 1 : (((hi_m >> lane) & 1ull) ? 2 : 0);
    }
    int qn = 0;            // slots of the current guess (slot j held by lane j)
    int svar = 0;          // slot lane: its variable
    float ssg = 1.f;       // slot lane: +1 lower bound row (n = e), -1 upper bound row (n = -e)
    float rdp = 0.f;       // slot lane: 1 / L[j][j]
    bool converged = false;
    float u = uunc, mu = 0.f;
    bool seeded = __ballot(act != 0) != 0;  // warm guess: build its slots before the first solve
    for (int pit = 0; pit < kPdasMaxIter; pit++) {
      if (seeded) {
        seeded = false;
        const unsigned long long mask = __ballot(act != 0);
        qn = __popcll(mask);
        const int myslot = __builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32),
                                                     __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0));
        if (act) sm.ids[myslot] = 3 * lane + (act == 2 ? 1 : 0);
        wsync();
        const int sid = (lane < qn) ? sm.ids[lane] : 0;
        svar = sid / 3;
        ssg = (sid - 3 * svar == 0) ? 1.f : -1.f;
        if (lane < qn)
          for (int l = 0; l < qn; l++) {
            const int idl = sm.ids[l];
            const int vl = idl / 3;
            sm.S[lane][l] = ssg * ((idl - 3 * vl == 0) ? 1.f : -1.f) * sm.W[svar][vl];
          }
        wsync();
        rdp = chol_slots<NUM>(sm, lane, qn, 0.f);
      }
      // solve the equality QP of the current slots: mu = S^-1 (b - N'u_unc), u = u_unc + W N mu
      float rhs = 0.f;
      if (lane < qn) {
        const float bj = (ssg > 0.f) ? ((svar & 1) ? umin1 : umin0) : -((svar & 1) ? umax1 : umax0);
        rhs = bj - ssg * sm.vec[svar];
      }
      const float lvp = tri_forward<NUM>(sm, lane, qn, rdp, rhs);
      mu = tri_backward<NUM>(sm, lane, qn, rdp, lvp);
      u = uunc;
      for (int j = 0; j < qn; j++) u = fmaf(readlane_f(mu * ssg, j), sm.W[readlane_i(svar, j)][cl], u);
      if (lane < qn) sm.pmu[svar] = mu;
      wsync();
      const float myu = act ? sm.pmu[lane] : 0.f;
      const bool nlo = valid && ((act == 1 ? myu : 0.f) + (lb - u) > 0.f);
      const bool nhi = valid && !nlo && ((act == 2 ? myu : 0.f) + (u - ub) > 0.f);
      const int nact = nlo ? 1 : (nhi ? 2 : 0);
      const unsigned long long changed = __ballot(nact != act);
      if (!changed) { converged = true; it = pit + 1; break; }
      if (qn == 0 || __ballot(act != 0 && nact != act)) {
        // first guess, or a slot leaves / flips side: build slots and chol(S_A) from scratch
        const unsigned long long mask = __ballot(nact != 0);
        qn = __popcll(mask);
        const int myslot = __builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32),
                                                     __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0));
        if (nact) sm.ids[myslot] = 3 * lane + (nact == 2 ? 1 : 0);
        wsync();
        const int sid = (lane < qn) ? sm.ids[lane] : 0;
        svar = sid / 3;
        ssg = (sid - 3 * svar == 0) ? 1.f : -1.f;
        if (lane < qn)
          for (int l = 0; l < qn; l++) {
            const int idl = sm.ids[l];
            const int vl = idl / 3;
            sm.S[lane][l] = ssg * ((idl - 3 * vl == 0) ? 1.f : -1.f) * sm.W[svar][vl];
          }
        wsync();
        rdp = chol_slots<NUM>(sm, lane, qn, 0.f);
      } else {
        // only additions: append each new bound as a slot with one forward solve
        // (incremental Cholesky row l = L^-1 S[q][:q], L[q][q] = sqrt(S[q][q] - l'l))
        unsigned long long addm = changed;
        while (addm) {
          const int v = __builtin_ctzll(addm);
          addm &= addm - 1;
          const int na = readlane_i(nact, v);
          const float sg = (na == 1) ? 1.f : -1.f;
          const float sv = (lane < qn) ? sg * ssg * sm.W[v][svar] : 0.f;
          const float lrow = tri_forward<NUM>(sm, lane, qn, rdp, sv);
          const float ll = wave_sum(lane < qn ? lrow * lrow : 0.f);
          const float dnew = sqrtf(sm.W[v][v] - ll);
          if (lane < qn) sm.L[qn][lane] = lrow;
          if (lane == qn) {
            sm.L[qn][qn] = dnew;
            svar = v;
            ssg = sg;
            rdp = 1.f / dnew;
          }
          if (lane == 0) sm.ids[qn] = 3 * v + (na == 2 ? 1 : 0);
          qn++;
          wsync();
        }
      }
      act = nact;
    }
    if (converged) {
      // hand the active set to the GI state: slots, multipliers, W n_j, S_A, chol(S_A)
      q = qn;
      slot_id = (lane < qn) ? 3 * svar + (ssg > 0.f ? 0 : 1) : -1;
      mult = (lane < qn) ? fmaxf(mu, 0.f) : 0.f;
      rdiag = (lane < qn) ? rdp : 0.f;
      actf = act;  // bit0 lower, bit1 upper
      if (lane < NUM)
        for (int j = 0; j < qn; j++) {
          const int vj = readlane_i(svar, j);
          sm.V[j][lane] = readlane_f(ssg, j) * sm.W[vj][lane];
        }
      if (lane < qn)
        for (int l = 0; l < qn; l++) {
          const int vl = readlane_i(svar, l);
          sm.S[lane][l] = ssg * readlane_f(ssg, l) * sm.W[svar][vl];
        }
      xv = valid ? u : 0.f;
      wsync();
    }
    STAMP_ACC(acc_pdas, t_pdas);
  }

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
      float X = 0.f, Y = 0.f;
      if (GAP) {
        const Lin& M = sm.M;
        rollout_lin_f32((float)M.a02, (float)M.a12, (float)M.b00, (float)M.b10, (float)M.b20,
                        (float)M.b21, lane, xv, X, Y);
      }
      float best = 0.f;
      int bid = 0x7fffffff;
      float sraw = 0.f;
      if (valid) {
        const float s0 = xv - lb, s1 = ub - xv;
        const float v0 = s0 / (1.f + fabsf(lb)), v1 = s1 / (1.f + fabsf(ub));
        if (!(actf & 1) && v0 < -1e-6f && v0 < best) { best = v0; bid = 3 * lane; sraw = s0; }
        if (!(actf & 2) && v1 < -1e-6f && v1 < best) { best = v1; bid = 3 * lane + 1; sraw = s1; }
        if (GAP) {
          const float s2 = (a ? ga1 : ga0) * X + (a ? gb1 : gb0) * Y + cgap;
          const float v2 = s2 / gnorm;
          if (!(actf & 4) && v2 < -1e-6f && v2 < best) { best = v2; bid = 3 * lane + 2; sraw = s2; }
        }
      }
      wave_argmin(best, bid);
      if (bid != 0x7fffffff) {
        p = bid;
        sp = readlane_f(sraw, bid / 3);
      } else {
        // ---- 5. refinement in fp64 + exact feasibility re-check ----
        STAMP(t_ref0);
        sm.cmult[3 * lane] = 0.f;
        sm.cmult[3 * lane + 1] = 0.f;
        sm.cmult[3 * lane + 2] = 0.f;
        wsync();
        if (lane < q) sm.cmult[slot_id] = mult;
        u64 = valid ? (double)xv : 0.0;
        const Lin M = sm.M;
        const double rxd = sm.rx[lane], ryd = sm.ry[lane], rthd = sm.rth[lane];
        double px, py, th;
        for (int rs = 0; rs < 2; rs++) {
          wsync();
          rollout_f64(M, lane, u64, px, py, th);
          double gmx = 0, gmy = 0;  // gap multipliers of this lane's stage (sides 0,1)
          if (GAP) {
            const double m0 = (double)sm.cmult[3 * (lane & ~1) + 2];
            const double m1 = (double)sm.cmult[3 * (lane | 1) + 2];
            gmx = m0 * ga0 + m1 * ga1;
            gmy = m0 * gb0 + m1 * gb1;
          }
          const double r1a = grad_f64(M, P, lane, N, u64, px, py, th, rxd, ryd, rthd, gmx, gmy);
          double r1 = valid ? r1a : 0.0;
          if (valid) r1 += -(double)sm.cmult[3 * lane] + (double)sm.cmult[3 * lane + 1];
          sm.d64[lane] = u64;
          if (GAP && a == 1 && k < N) { sm.sx64[k + 1] = px; sm.sy64[k + 1] = py; }
          sm.vec[lane] = (float)r1;
          wsync();
          // r2_j = n_j'u - b_j on the active rows (fp64)
          float r2 = 0.f;
          if (lane < q) {
            const int owner = slot_id / 3, t = slot_id - 3 * owner;
            if (t == 0) r2 = (float)(sm.d64[owner] - (double)((owner & 1) ? umin1 : umin0));
            else if (t == 1) r2 = (float)((double)((owner & 1) ? umax1 : umax0) - sm.d64[owner]);
            else {
              const int st = (owner >> 1) + 1;
              r2 = (owner & 1) ? (float)((double)ga1 * sm.sx64[st] + (double)gb1 * sm.sy64[st] - gbeta1)
                               : (float)((double)ga0 * sm.sx64[st] + (double)gb0 * sm.sy64[st] - gbeta0);
            }
          }
          // w1 = W r1 ; v1_j = n_j' w1
          const float w1 = matvec_W<NUM>(sm, lane);
          sm.vec2[lane] = w1;
          if (GAP) {
            float X1, Y1;
            rollout_lin_f32((float)M.a02, (float)M.a12, (float)M.b00, (float)M.b10,
                            (float)M.b20, (float)M.b21, lane, valid ? w1 : 0.f, X1, Y1);
            if (a == 1 && k < N) { sm.stX[k + 1] = X1; sm.stY[k + 1] = Y1; }
          }
          wsync();
          const float rhs = (lane < q) ? slot_dot<NUM>(sm, slot_id, ga0, ga1, gb0, gb1) - r2 : 0.f;
          // du = S^-1 rhs ; dx = -w1 + sum_j du_j V[j]
          const float lv = tri_forward<NUM>(sm, lane, q, rdiag, rhs);
          const float du = tri_backward<NUM>(sm, lane, q, rdiag, lv);
          float dx = -w1;
          const int cl = lane < NUM ? lane : NUM - 1;
          for (int j = 0; j < q; j++) dx = fmaf(readlane_f(du, j), sm.V[j][cl], dx);
          if (valid) u64 += (double)dx;
          mult += du;
          wsync();
          if (lane < q) sm.cmult[slot_id] = mult;
          // a second step only if the first correction was not already at fp32 noise level
          float adx = valid ? fabsf(dx) : 0.f;
          int dummy = 0;
          adx = -adx;
          wave_argmin(adx, dummy);  // -max |dx|
          if (-adx <= 1e-5f) break;
        }
        wsync();
        // fp64 feasibility check of every inactive row at the refined point
        rollout_f64(M, lane, u64, px, py, th);
        float best64 = 0.f, sp64 = 0.f;
        int bid64 = 0x7fffffff;
        if (valid) {
          const double s0 = u64 - (double)lb, s1 = (double)ub - u64;
          const float v0 = (float)(s0 / (1.0 + fabs((double)lb)));
          const float v1 = (float)(s1 / (1.0 + fabs((double)ub)));
          if (!(actf & 1) && v0 < -1e-9f && v0 < best64) { best64 = v0; bid64 = 3 * lane; sp64 = (float)s0; }
          if (!(actf & 2) && v1 < -1e-9f && v1 < best64) { best64 = v1; bid64 = 3 * lane + 1; sp64 = (float)s1; }
          if (GAP) {
            const double s2 = a ? ((double)ga1 * px + (double)gb1 * py - gbeta1)
                                : ((double)ga0 * px + (double)gb0 * py - gbeta0);
            const float v2 = (float)(s2 / (double)gnorm);
            if (!(actf & 4) && v2 < -1e-9f && v2 < best64) { best64 = v2; bid64 = 3 * lane + 2; sp64 = (float)s2; }
          }
        }
        wave_argmin(best64, bid64);
        STAMP_ACC(acc_refine, t_ref0);
        if (bid64 == 0x7fffffff || reentries >= 4) {
          final_ok = true;
          break;
        }
        reentries++;
        forced_p = bid64;
        forced_sp = readlane_f(sp64, bid64 / 3);
        xv = valid ? (float)u64 : 0.f;
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
      float w, nw;
      if (pt < 2) {
        const float sg = (pt == 0) ? 1.f : -1.f;
        w = (lane < NUM) ? sg * sm.W[pown][lane] : 0.f;
        nw = sm.W[pown][pown];
      } else {
        const int ip = (pown >> 1) + 1, h = pown & 1;
        const float ah = h ? ga1 : ga0, bh = h ? gb1 : gb0;
        const Lin& M = sm.M;
        float np = 0.f;
        if (valid && k < ip) {
          const float d = (float)(ip - 1 - k);
          const float fa02 = (float)M.a02, fa12 = (float)M.a12;
          if (a == 0) np = ah * ((float)M.b00 + fa02 * (float)M.b20 * d) + bh * ((float)M.b10 + fa12 * (float)M.b20 * d);
          else np = (ah * fa02 + bh * fa12) * (float)M.b21 * d;
        }
        sm.vec[lane] = np;
        wsync();
        w = matvec_W<NUM>(sm, lane);
        nw = wave_sum(np * w);
      }
      STAMP_ACC(acc_w, t_a);
      STAMP(t_b);
      // v_j = n_j' w for the active slots
      sm.vec2[lane] = w;
      if (GAP) {
        const Lin& M = sm.M;
        float Xw, Yw;
        rollout_lin_f32((float)M.a02, (float)M.a12, (float)M.b00, (float)M.b10, (float)M.b20,
                        (float)M.b21, lane, valid ? w : 0.f, Xw, Yw);
        if (a == 1 && k < N) { sm.stX[k + 1] = Xw; sm.stY[k + 1] = Yw; }
      }
      wsync();
      const float vj = (lane < q) ? slot_dot<NUM>(sm, slot_id, ga0, ga1, gb0, gb1) : 0.f;
      STAMP_ACC(acc_vj, t_b);
      STAMP(t_c);
      // l = L^-1 v ; r = L^-T l  (r = S_A^-1 N_A' W n_p : dual step direction)
      const float lv = tri_forward<NUM>(sm, lane, q, rdiag, vj);
      const float ll = wave_sum(lane < q ? lv * lv : 0.f);
      const float r = tri_backward<NUM>(sm, lane, q, rdiag, lv);
      STAMP_ACC(acc_tri, t_c);
      STAMP(t_d);
      // z = w - sum_j r_j V[j]  (primal step direction)
      float z = w;
      const int cl = lane < NUM ? lane : NUM - 1;
      for (int j = 0; j < q; j++) z = fmaf(-readlane_f(r, j), sm.V[j][cl], z);
      const float pivv = nw - ll;  // = z' n_p, the new Schur pivot
      STAMP_ACC(acc_z, t_d);
      STAMP(t_e);
      // partial step t1 (blocking multiplier k1)
      float t1 = 3.0e38f;
      int k1 = 0x7fffffff;
      if (lane < q && r > 0.f) { t1 = mult / r; k1 = lane; }
      wave_argmin(t1, k1);
      const bool dep = !(pivv > 1e-5f * nw);  // n_p (numerically) in span of the active set
      const float t2 = dep ? 3.0e38f : -sp / pivv;
      const float t = fminf(t1, t2);
      if (t >= 3.0e38f) { status = F110QP_PRIMAL_INFEASIBLE_ID; break; }
      if (lane < q) mult -= t * r;
      uplus_new += t;
      bool add = false;
      if (!dep) {
        if (valid) xv = fmaf(t, z, xv);
        sp = fmaf(t, pivv, sp);
        add = (t2 <= t1);
      }
      wsync();
      STAMP_ACC(acc_step, t_e);
      STAMP(t_f);
      if (add) {
        if (q >= NUM) { status = F110QP_MAX_ITER_ID; break; }
        if (lane < NUM) sm.V[q][lane] = w;
        if (lane < q) {
          sm.S[q][lane] = vj;
          sm.S[lane][q] = vj;
          sm.L[q][lane] = lv;
        }
        if (lane == 0) {
          sm.S[q][q] = nw;
          sm.L[q][q] = sqrtf(pivv);
        }
        if (lane == q) {
          slot_id = p;
          mult = uplus_new;
          rdiag = 1.f / sqrtf(pivv);
        }
        if (lane == pown) actf |= (1 << pt);
        q++;
        wsync();
        STAMP_ACC(acc_upd, t_f);
        break;
      }
      // drop slot k1, then retry p
      {
        const int kd = k1;
        const int did = readlane_i(slot_id, kd);
        if (lane == did / 3) actf &= ~(1 << (did - 3 * (did / 3)));
        const int sid_n = __shfl_down(slot_id, 1, 64);
        const float mul_n = __shfl_down(mult, 1, 64);
        if (lane >= kd && lane < q - 1) { slot_id = sid_n; mult = mul_n; }
        if (lane == q - 1) { slot_id = -1; mult = 0.f; }
        // remove slot kd from V (rows) and S (row and column): every lane moves only its own
        // column (V, S rows) or its own row (S columns), so there is no cross-lane hazard
        if (lane < NUM) {
          for (int j = kd; j < q - 1; j++) {
            sm.V[j][lane] = sm.V[j + 1][lane];
            sm.S[j][lane] = sm.S[j + 1][lane];
          }
        }
        wsync();
        if (lane < q - 1)
          for (int i2 = kd; i2 < q - 1; i2++) sm.S[lane][i2] = sm.S[lane][i2 + 1];
        q--;
        wsync();
        rdiag = chol_slots<NUM>(sm, lane, q, rdiag);
      }
    }
  }

  STAMP(t_gi);
  // ---- 6. outputs ---------------------------------------------------------------------------
  if (status == F110QP_SOLVED_ID && !final_ok) status = F110QP_MAX_ITER_ID;
  const bool ok = (status == F110QP_SOLVED_ID);
  double px, py, th;
  rollout_f64(sm.M, lane, (ok && valid) ? u64 : 0.0, px, py, th);
  const float nanv = __int_as_float(0x7fc00000);
  if (valid) uout[(size_t)b * NU + lane] = ok ? (float)u64 : nanv;
  float* xo = xout + (size_t)b * 3 * (N + 1);
  if (lane == 0) {
    xo[0] = ok ? fX0 : nanv;
    xo[1] = ok ? fY0 : nanv;
    xo[2] = ok ? fTH0 : nanv;
  }
  if (valid && a == 1) {
    xo[3 * (k + 1) + 0] = ok ? (float)(px + X0) : nanv;
    xo[3 * (k + 1) + 1] = ok ? (float)(py + Y0) : nanv;
    xo[3 * (k + 1) + 2] = ok ? (float)th : nanv;
  }
  if (lane == 0) {
    status_out[b] = status;
    if (iters_out) iters_out[b] = it;
  }
  if (warm) {
    const unsigned long long lo_m = __ballot(ok && valid && (actf & 1));
    const unsigned long long hi_m = __ballot(ok && valid && (actf & 2));
    if (lane == 0) {
      ws.act[2 * b] = lo_m;
      ws.act[2 * b + 1] = hi_m;
    }
  }
#ifdef F110QP_STAMPS
  STAMP(t_end);
  if (lane == 0 && b < 65536) {
    unsigned long long* o = g_stamps + (size_t)b * kStampSlots;
    o[0] = t_lin - t_start; o[1] = t_grad - t_lin; o[2] = t_hess - t_grad; o[3] = t_inv - t_hess;
    o[4] = t_gi - t_inv - acc_refine; o[5] = acc_refine; o[6] = t_end - t_gi; o[7] = t_end - t_start;
    o[8] = acc_s1; o[9] = acc_w; o[10] = acc_vj; o[11] = acc_tri; o[12] = acc_z; o[13] = acc_step;
    o[14] = acc_upd; o[15] = it; o[8] += 0; o[13] += 0; o[12] += 0; (void)acc_pdas;
    o[9] = acc_pdas;
  }
#endif
}

// ------------------------------------------------------------------------------------------
// launch
// ------------------------------------------------------------------------------------------
template <int NUM, bool GAP>
static hipError_t launch_t(const KParams& P, int B, const float* x0, const float* ul,
                           const float* xr, const float* hs, float* uo, float* xo, int* st,
                           int* its, double* Hd, double* gd, const WarmState& ws, hipStream_t s) {
  hipLaunchKernelGGL((solve_kernel<NUM, GAP>), dim3(B), dim3(64), 0, s, P, B, x0, ul, xr, hs, uo,
                     xo, st, its, Hd, gd, ws);
  return hipGetLastError();
}

template <bool GAP>
static hipError_t launch_g(const KParams& P, int B, const float* x0, const float* ul,
                           const float* xr, const float* hs, float* uo, float* xo, int* st,
                           int* its, double* Hd, double* gd, const WarmState& ws, hipStream_t s) {
  const int NU = 2 * P.N;
  if (NU <= 8) return launch_t<8, GAP>(P, B, x0, ul, xr, hs, uo, xo, st, its, Hd, gd, ws, s);
  if (NU <= 16) return launch_t<16, GAP>(P, B, x0, ul, xr, hs, uo, xo, st, its, Hd, gd, ws, s);
  if (NU <= 24) return launch_t<24, GAP>(P, B, x0, ul, xr, hs, uo, xo, st, its, Hd, gd, ws, s);
  if (NU <= 32) return launch_t<32, GAP>(P, B, x0, ul, xr, hs, uo, xo, st, its, Hd, gd, ws, s);
  if (NU <= 40) return launch_t<40, GAP>(P, B, x0, ul, xr, hs, uo, xo, st, its, Hd, gd, ws, s);
  if (NU <= 48) return launch_t<48, GAP>(P, B, x0, ul, xr, hs, uo, xo, st, its, Hd, gd, ws, s);
  if (NU <= 56) return launch_t<56, GAP>(P, B, x0, ul, xr, hs, uo, xo, st, its, Hd, gd, ws, s);
  if (NU <= 64) return launch_t<64, GAP>(P, B, x0, ul, xr, hs, uo, xo, st, its, Hd, gd, ws, s);
  return hipErrorInvalidValue;
}

hipError_t launch_solve(const KParams& P, int B, const float* x0, const float* ul,
                        const float* xr, const float* hs, float* uo, float* xo, int* st,
                        int* its, const WarmState& ws, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  if (hs) return launch_g<true>(P, B, x0, ul, xr, hs, uo, xo, st, its, nullptr, nullptr, ws, s);
  return launch_g<false>(P, B, x0, ul, xr, hs, uo, xo, st, its, nullptr, nullptr, ws, s);
}

hipError_t launch_condense_debug(const KParams& P, int B, const float* x0, const float* ul,
                                 const float* xr, double* Hd, double* gd, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  return launch_g<false>(P, B, x0, ul, xr, nullptr, nullptr, nullptr, nullptr, nullptr, Hd, gd,
                         WarmState(), s);
}

}  // namespace f110qp

#ifdef F110QP_STAMPS
extern "C" int f110qp_read_stamps(unsigned long long* host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(f110qp::g_stamps),
                                  (size_t)n * f110qp::kStampSlots * sizeof(unsigned long long));
}
#endif

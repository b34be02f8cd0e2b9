// gi64_kernel.h — the fp64 re-check of gap-row QPs: the Goldfarb-Idnani dual active set in fp64
// on the condensed QP, one workgroup per QP of a device-side list (the QPs whose wave-kernel
// answer its fp64 certificate did not accept, solve_kernel.h step 5).
//
// Reference: the QP of src/mpc.cpp:208-306 with the gap rows of :249,271 (C3 semantic :297-298),
// which OSQP solves in c_float = double (:133-142). The algorithm and its rules are the oracle's
// (the CPU oracle's gi_solve, test infrastructure): the most violated row by raw slack with tolerance
// 1e-11 (1 + |b| + |x_unc|_inf), ties to the oracle's row order (box rows by variable, lower before
// upper, then the gap rows by stage and side), a dependent row when the new Schur pivot is
// <= 1e-12 n'Wn, at most 20 (n + m) iterations. So the re-check reaches the oracle's verdict on the
// QPs where the fp32 GI of the wave kernel cannot be certified (stiff corners: dt = 0.05, N = 33..48).
//
// Per QP, in a workgroup of 64 ceil(2 NUM / 64) threads:
//   1. thread t < NUM: row t of H (fp64, the closed form of solve_kernel.h build_H); then the
//      Jacobi-scaled symmetric sweep (Goodnight) with each row in the registers of two threads
//      (half a row each) and the pivot row through LDS (double buffered, one barrier per pivot):
//      W = H^-1 stored to LDS;
//   2. wave 0 alone (the other waves wait at the item's closing barrier; wave 0 synchronises with
//      wave-scope fences only): GI from the unconstrained point, fp64 throughout — w = W n_p, the
//      Cholesky factor of S_A = N_A' W N_A in LDS (rows appended, slots deleted by Givens rotations),
//      z = W (n_p - N_A r) with N_A r by the adjoint (costate) scans, no stored W n_j;
//   3. the final set's equality QP solved afresh from W and the factor, then the certificate of
//      the wave kernel (solve_kernel.h kCertTauW): every row within 1e-9 (1 + |b| + |x|_inf), and
//      with the residual rho = H u + g - N_A mu+ (mu clamped at 0), rho'W rho (bounded from above
//      in fp64 through an fp64 Hessian product) <= lambda (tau max(1, |u|_inf))^2, lambda = min(R)
//      <= lambda_min(H): rho'W rho bounds |u - u*'|_H^2 (the duality gap at mu+) for the optimum u*'
//      of the QP whose row bounds are moved by u's own residuals on them (<= the 1e-9 tolerance),
//      so |u - u*'|_2 <= tau max(1, |u|_inf) and the QP is SOLVED, else SOLVED_INACCURATE; an empty
//      feasible set PRIMAL_INFEASIBLE, the cap MAX_ITER, non-finite data NUMERICAL. u*, x* (fp64
//      rollout) and obj / cost are written.
#pragma once
#include "solve_kernel.h"

namespace f110qp {

// rho'W rho <= lambda_min(R) (kCertTau max(1, |u|_inf))^2 certifies |u - u*|_2 <= kCertTau max(1, |u|_inf)
constexpr double kCertTau = 1e-6;

template <int NUM>
struct G64Smem {
  static constexpr int R = (NUM + 63) / 64;
  static constexpr int VN = 64 * R;
  static constexpr int NST = NUM / 2 + 1;
  double W[NUM][NUM];       // W = H^-1 (symmetric): lane v reads W[j][v] (conflict free)
  double L[NUM][NUM + 1];   // Cholesky factor of S_A (lower), slots x slots; sweep pivot rows
  double vec[VN];           // broadcast vector (matvec input, slot gathers)
  double cid[3 * VN];       // a value per constraint id (dual step r, multipliers)
  double stX[NST], stY[NST];  // per-stage linear rollout of a vector (stages 1..N)
  double rx[VN], ry[VN], rth[VN];  // recentred reference of each variable's stage
  double dsc[VN];           // Jacobi scaling of the sweep
  Lin M;
};

// wave-scope ordering of LDS accesses (wave 0 runs GI while the other waves wait at a barrier)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// argmin of (val, key) over the wave (ties -> smaller key), result uniform
__device__ __forceinline__ void wave_argmin_d(double& val, int& key) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const double ov = __shfl_xor(val, o, 64);
    const int ok = __shfl_xor(key, o, 64);
    const bool take = (ov < val) || (ov == val && ok < key);
    val = take ? ov : val;
    key = take ? ok : key;
  }
}
__device__ __forceinline__ double wave_max_d(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}
template <int R>
__device__ __forceinline__ double rl_d(const double (&x)[R], int j) {
  return readlane_d(pick<R>(x, j >> 6), j & 63);
}

// g = Gamma_x' ex + Gamma_y' ey on the inputs: ex / ey per stage i = k+1 on the odd lanes of
// stage pair k (zero elsewhere), by the costate suffix scans of solve_kernel.h grad_f64.
template <int R>
__device__ __forceinline__ void adjoint_xy(const Lin& M, int lane, double (&ex)[R], double (&ey)[R],
                                           double (&g)[R]) {
  const int a = lane & 1;
  double lx[R], ly[R];
#pragma unroll
  for (int r = 0; r < R; r++) {
    const double i = (double)(32 * r + (lane >> 1) + 1);
    lx[r] = i * ex[r];
    ly[r] = i * ey[r];
  }
  scan_suffix_incl_R<R>(ex);
  scan_suffix_incl_R<R>(lx);
  scan_suffix_incl_R<R>(ey);
  scan_suffix_incl_R<R>(ly);
#pragma unroll
  for (int r = 0; r < R; r++) {
    const double i = (double)(32 * r + (lane >> 1) + 1);
    const double lth = M.a02 * (lx[r] - i * ex[r]) + M.a12 * (ly[r] - i * ey[r]);
    g[r] = a ? M.b21 * lth : M.b00 * ex[r] + M.b10 * ey[r] + M.b20 * lth;
  }
}

template <int NUM>
__device__ void gi64_qp(G64Smem<NUM>& sm, const int b, const KParams& P, const float* __restrict__ x0g,
                        const float* __restrict__ ulg, const float* __restrict__ xrg,
                        const float* __restrict__ hsg, float* __restrict__ uout, float* __restrict__ xout,
                        int* __restrict__ status_out, int* __restrict__ iters_out, const ObjOut& oo) {
  constexpr int R = (NUM + 63) / 64;
  const int t = threadIdx.x;
  const int N = P.N;
  const int NU = 2 * N;
  const float fX0 = x0g[3 * b + 0], fY0 = x0g[3 * b + 1], fTH0 = x0g[3 * b + 2];
  const float ul0 = ulg[2 * b + 0], ul1 = ulg[2 * b + 1];
  const Lin M0 = linearize((double)fTH0, (double)ul0, (double)ul1, P.dt);
  // the exact verdicts (non-finite data, a violated stage-0 row) need no solve: uniform per QP,
  // so the whole workgroup skips the inverse
  bool early;
  {
    const float* xq = xrg + (size_t)b * P.xr_stride * 3;
    bool nf = !(isfinite(fX0) && isfinite(fY0) && isfinite(fTH0) && isfinite(ul0) && isfinite(ul1));
    for (int i = 0; i < 3 * N; i++) nf = nf || !isfinite(xq[i]);
    const float* h6e = hsg + 6 * b;
    const double be0 = -(double)h6e[2] - (double)h6e[0] * (double)fX0 - (double)h6e[1] * (double)fY0;
    const double be1 = -(double)h6e[5] - (double)h6e[3] * (double)fX0 - (double)h6e[4] * (double)fY0;
    const bool inf0 = !(isfinite(be0) && isfinite(be1)) || be0 > 1e-9 * (1.0 + fabs((double)h6e[2])) ||
                      be1 > 1e-9 * (1.0 + fabs((double)h6e[5]));
    early = nf || inf0;
  }

  // ---- 1. H row t (fp64 closed form, solve_kernel.h build_H), sweep to W = H^-1 ----------------
  if (!early) {
    const int kt = t >> 1, at = t & 1;
    const bool vt = t < NU;
    double C0[2] = {0.0, 0.0}, C1[2] = {0.0, 0.0}, hd = 1.0;
    if (vt) {
      const double q0 = P.q[0], q1 = P.q[1], q2 = P.q[2];
      const double beta_a = at ? M0.b21 : M0.b20;
      const double pxa = at ? 0.0 : M0.b00, pya = at ? 0.0 : M0.b10;
      const double sxa = M0.a02 * beta_a, sya = M0.a12 * beta_a;
      const double T = (double)(N - kt);
      const double S1 = T * (T - 1.0) * 0.5;
      const double S2 = (T - 1.0) * T * (2.0 * T - 1.0) * (1.0 / 6.0);
      const double Ux = T * pxa + sxa * S1, Vx = pxa * S1 + sxa * S2;
      const double Uy = T * pya + sya * S1, Vy = pya * S1 + sya * S2;
#pragma unroll
      for (int bb = 0; bb < 2; bb++) {
        const double beta_b = bb ? M0.b21 : M0.b20;
        const double ax_b = bb ? 0.0 : M0.b00, ay_b = bb ? 0.0 : M0.b10;
        const double sxb = M0.a02 * beta_b, syb = M0.a12 * beta_b;
        C0[bb] = q0 * (ax_b * Ux + sxb * Vx) + q1 * (ay_b * Uy + syb * Vy) + q2 * T * beta_a * beta_b;
        C1[bb] = q0 * sxb * Ux + q1 * syb * Uy;
      }
      hd = C0[at] + (at ? P.r[1] : P.r[0]);
    }
    // entries (t, w) for w <= t and their mirror (w, t): every entry written by one thread
    if (t < NUM) {
      if (vt) {
        for (int w = 0; w <= t; w++) {
          const int l = w >> 1, bb = w & 1;
          const double h = (w == t) ? hd : fma(C1[bb], (double)(kt - l), C0[bb]);
          sm.W[t][w] = h;
          sm.W[w][t] = h;
        }
      } else {  // padding variables: identity rows and columns
        for (int w = 0; w < NUM; w++) {
          sm.W[t][w] = (w == t) ? 1.0 : 0.0;
          sm.W[w][t] = (w == t) ? 1.0 : 0.0;
        }
      }
      sm.dsc[t] = (hd > 0.0) ? 1.0 / sqrt(hd) : 1.0;
    }
    __syncthreads();
    // the sweep: two threads per row (HN = NUM / 2 columns each, 2 NUM threads): a whole fp64
    // row in one thread's registers spilled at NUM = 96
    constexpr int HN = NUM / 2;
    const int row = t >> 1, c0 = (t & 1) * HN;
    const bool rv = row < NUM;
    double a[HN];
    const double dr = rv ? sm.dsc[row] : 1.0;
#pragma unroll
    for (int j = 0; j < HN; j++) a[j] = rv ? sm.W[c0 + j][row] * dr * sm.dsc[c0 + j] : 0.0;
    // symmetric sweep (Goodnight): a_pp <- -1/a_pp, a_pj <- a_pj / a_pp, a_ip <- a_ip / a_pp,
    // a_ij <- a_ij - a_ip a_pj / a_pp; the pivot row through LDS (row p of L, double buffered:
    // the writers of pivot p + 2 pass the barrier of pivot p + 1 only after every read of p)
    for (int p = 0; p < NUM; p++) {
      double* pr = sm.L[p & 1];
      if (row == p) {
#pragma unroll
        for (int j = 0; j < HN; j++) pr[c0 + j] = a[j];
      }
      __syncthreads();
      const double inv = 1.0 / pr[p];
      const double f = (rv ? pr[row] : 0.0) * inv;  // a_rp / a_pp (symmetric)
      const bool piv = row == p;
#pragma unroll
      for (int j = 0; j < HN; j++) {
        const double pj = pr[c0 + j];
        const double upd = piv ? pj * inv : fma(-f, pj, a[j]);
        a[j] = (c0 + j == p) ? (piv ? -inv : f) : upd;
      }
    }
    __syncthreads();  // every pivot row read before W is overwritten
    if (rv) {
#pragma unroll
      for (int j = 0; j < HN; j++) sm.W[c0 + j][row] = -a[j] * dr * sm.dsc[c0 + j];
    }
    if (t == 0) sm.M = M0;
    __syncthreads();
  }
  if (t >= 64) return;  // the GI loop runs in wave 0

  // ---- 2. inputs, gradient at u = 0, unconstrained point ----------------------------------------
  const int lane = t;
  const int a = lane & 1;
  const Lin M = M0;
  int vv[R], kk[R], cl[R];
  bool valid[R];
#pragma unroll
  for (int r = 0; r < R; r++) {
    vv[r] = 64 * r + lane;
    kk[r] = vv[r] >> 1;
    valid[r] = vv[r] < NU;
    cl[r] = vv[r] < NUM ? vv[r] : NUM - 1;
  }
  const double X0 = (double)fX0, Y0 = (double)fY0;
  bool bad = !(isfinite(fX0) && isfinite(fY0) && isfinite(fTH0) && isfinite(ul0) && isfinite(ul1));
  float x00[3] = {0.f, 0.f, 0.f};
  if (lane == 0) {
    const float* xq = xrg + (size_t)b * P.xr_stride * 3;
    x00[0] = xq[0]; x00[1] = xq[1]; x00[2] = xq[2];
    bad = bad || !(isfinite(x00[0]) && isfinite(x00[1]) && isfinite(x00[2]));
  }
  double rxd[R], ryd[R], rthd[R];
#pragma unroll
  for (int r = 0; r < R; r++) {
    rxd[r] = 0.0; ryd[r] = 0.0; rthd[r] = 0.0;
    if (valid[r]) {
      const int ri = (kk[r] + 1 < N) ? kk[r] + 1 : N - 1;  // terminal stage reuses x_ref[N-1] (mpc.cpp:228)
      const float* xr = xrg + ((size_t)b * P.xr_stride + ri) * 3;
      const float f0 = xr[0], f1 = xr[1], f2 = xr[2];
      bad = bad || !(isfinite(f0) && isfinite(f1) && isfinite(f2));
      rxd[r] = (double)f0 - X0;
      ryd[r] = (double)f1 - Y0;
      rthd[r] = (double)f2;
    }
    sm.rx[vv[r]] = rxd[r]; sm.ry[vv[r]] = ryd[r]; sm.rth[vv[r]] = rthd[r];
  }
  // gap rows a x + b y >= -(c + 0.5) (constraints.cpp:255-264, mpc.cpp:297-298), recentred
  const float* h6 = hsg + 6 * b;
  const double ga0 = h6[0], gb0 = h6[1], ga1 = h6[3], gb1 = h6[4];
  const double gbeta0 = -(double)h6[2] - ga0 * X0 - gb0 * Y0;
  const double gbeta1 = -(double)h6[5] - ga1 * X0 - gb1 * Y0;
  // the stage-0 rows are constant (x0 lies on both lines): infeasible only if violated; a
  // non-finite row is the wave kernel's empty-set verdict too
  bool infeasible0 = gbeta0 > 1e-9 * (1.0 + fabs((double)h6[2])) || gbeta1 > 1e-9 * (1.0 + fabs((double)h6[5]));
  if (!(isfinite(gbeta0) && isfinite(gbeta1))) infeasible0 = true;
  const bool numerical = __ballot(bad) != 0ull;
  const double gah = a ? ga1 : ga0, gbh = a ? gb1 : gb0, gbe = a ? gbeta1 : gbeta0;
  const double lb0 = P.umin[0], lb1 = P.umin[1], ub0 = P.umax[0], ub1 = P.umax[1];
  double lb[R], ub[R], gcon[R], g[R];
  {
    double zero[R], px0[R], py0[R], th0s[R];
#pragma unroll
    for (int r = 0; r < R; r++) zero[r] = 0.0;
    rollout_f64<R>(M, lane, zero, px0, py0, th0s);
    grad_f64<R>(M, P, lane, N, zero, px0, py0, th0s, rxd, ryd, rthd, zero, zero, g);
#pragma unroll
    for (int r = 0; r < R; r++) {
      lb[r] = a ? lb1 : lb0;
      ub[r] = a ? ub1 : ub0;
      g[r] = valid[r] ? g[r] : 0.0;
      // the oracle's b of this variable's gap row (stage kk+1, side a): -c - a f_x - b f_y (world)
      gcon[r] = gbe - gah * px0[r] - gbh * py0[r];
    }
  }
  // x = -W g
  auto matvec_W = [&](double (&y)[R]) __attribute__((always_inline)) {  // y = W vec
#pragma unroll
    for (int r = 0; r < R; r++) y[r] = 0.0;
    for (int j = 0; j < NU; j++) {
      const double xj = sm.vec[j];
#pragma unroll
      for (int r = 0; r < R; r++) y[r] = fma(sm.W[j][cl[r]], xj, y[r]);
    }
#pragma unroll
    for (int r = 0; r < R; r++) y[r] = valid[r] ? y[r] : 0.0;
  };
  double x[R];
#pragma unroll
  for (int r = 0; r < R; r++) sm.vec[vv[r]] = g[r];
  wave_sync();
  matvec_W(x);
#pragma unroll
  for (int r = 0; r < R; r++) x[r] = -x[r];
  double xscale = 0.0;
#pragma unroll
  for (int r = 0; r < R; r++) xscale = fmax(xscale, fabs(x[r]));
  xscale = wave_max_d(xscale);

  // ---- 3. Goldfarb-Idnani with the oracle's rules, fp64 ----------------------------------------
  int actf[R], slot_id[R];
  double mult[R], rdiag[R];
#pragma unroll
  for (int r = 0; r < R; r++) { actf[r] = 0; slot_id[r] = -1; mult[r] = 0.0; rdiag[r] = 0.0; }
  int q = 0, it = 0;
  int status = numerical ? F110QP_NUMERICAL_ID : (infeasible0 ? F110QP_PRIMAL_INFEASIBLE_ID : F110QP_SOLVED_ID);
  const int max_iter = 20 * (NU + 2 * NU + NU);  // 20 (n + m), m = 2 nu box + 2N gap rows
  // normal of row id pid = 3 v + t at this lane's variables
  auto normal = [&](int pid, double (&np)[R]) __attribute__((always_inline)) {
    const int pown = pid / 3, pt = pid - 3 * pown;
#pragma unroll
    for (int r = 0; r < R; r++) {
      np[r] = 0.0;
      if (pt < 2) {
        np[r] = (vv[r] == pown) ? (pt == 0 ? 1.0 : -1.0) : 0.0;
      } else {
        const int ip = (pown >> 1) + 1;  // stage of the row
        const double ah = (pown & 1) ? ga1 : ga0, bh = (pown & 1) ? gb1 : gb0;
        if (valid[r] && kk[r] < ip) {
          const double d = (double)(ip - 1 - kk[r]);
          np[r] = a ? (ah * M.a02 + bh * M.a12) * M.b21 * d
                    : ah * (M.b00 + M.a02 * M.b20 * d) + bh * (M.b10 + M.a12 * M.b20 * d);
        }
      }
    }
  };
  // per-stage positions of the linear rollout of w (in sm.stX / stY) and w per variable (sm.vec)
  Lin ML = M;
  ML.th0 = 0.0; ML.c0 = 0.0; ML.c1 = 0.0; ML.c2 = 0.0;
  auto publish = [&](const double (&w)[R]) __attribute__((always_inline)) {
    double X[R], Y[R], Th[R];
    rollout_f64<R>(ML, lane, w, X, Y, Th);
#pragma unroll
    for (int r = 0; r < R; r++) {
      sm.vec[vv[r]] = w[r];
      if (a == 1 && kk[r] < N) { sm.stX[kk[r] + 1] = X[r]; sm.stY[kk[r] + 1] = Y[r]; }
    }
    wave_sync();
  };
  auto slot_dot = [&](int sid) __attribute__((always_inline)) -> double {  // n_sid' w (published)
    const int own = sid / 3, tt = sid - 3 * own;
    if (tt == 0) return sm.vec[own];
    if (tt == 1) return -sm.vec[own];
    const int st = (own >> 1) + 1;
    return ((own & 1) ? ga1 : ga0) * sm.stX[st] + ((own & 1) ? gb1 : gb0) * sm.stY[st];
  };
  // sum_j c_j n_j over the active slots (c per slot lane) at this lane's variables: box rows
  // directly, gap rows by the adjoint scans (through the per-id table sm.cid)
  auto nsum = [&](const double (&c)[R], double (&out)[R]) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < R; r++) {
      sm.cid[3 * vv[r]] = 0.0; sm.cid[3 * vv[r] + 1] = 0.0; sm.cid[3 * vv[r] + 2] = 0.0;
    }
    wave_sync();
#pragma unroll
    for (int r = 0; r < R; r++)
      if (64 * r + lane < q) sm.cid[slot_id[r]] = c[r];
    wave_sync();
    double ex[R], ey[R], gg[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
      ex[r] = 0.0; ey[r] = 0.0;
      if (a == 1 && kk[r] < N) {  // odd lane of stage pair kk: the rows of stage kk + 1
        const double c0 = sm.cid[3 * (vv[r] & ~1) + 2], c1 = sm.cid[3 * (vv[r] | 1) + 2];
        ex[r] = c0 * ga0 + c1 * ga1;
        ey[r] = c0 * gb0 + c1 * gb1;
      }
    }
    adjoint_xy<R>(M, lane, ex, ey, gg);
#pragma unroll
    for (int r = 0; r < R; r++)
      out[r] = valid[r] ? gg[r] + sm.cid[3 * vv[r]] - sm.cid[3 * vv[r] + 1] : 0.0;
    wave_sync();
  };

  while (status == F110QP_SOLVED_ID) {
    // ---- step 1: most violated inactive row (raw slack, oracle tolerance and order) ----
    double px[R], py[R], th[R];
    rollout_f64<R>(M, lane, x, px, py, th);
    double best = 0.0;
    int bkey = 0x7fffffff;
#pragma unroll
    for (int r = 0; r < R; r++) {
      if (!valid[r]) continue;
      const int v = vv[r];
      const double s0 = x[r] - lb[r], s1 = ub[r] - x[r];
      const double tol0 = 1e-11 * (1.0 + fabs(lb[r]) + xscale), tol1 = 1e-11 * (1.0 + fabs(ub[r]) + xscale);
      // oracle order: box lower 2v, box upper 2v + 1, gap row (stage k+1, side a) 2 NU + v
      if (!(actf[r] & 1) && s0 < -tol0 && (s0 < best || (s0 == best && 2 * v < bkey))) { best = s0; bkey = 2 * v; }
      if (!(actf[r] & 2) && s1 < -tol1 && (s1 < best || (s1 == best && 2 * v + 1 < bkey))) { best = s1; bkey = 2 * v + 1; }
      const double s2 = gah * px[r] + gbh * py[r] - gbe;
      const double tol2 = 1e-11 * (1.0 + fabs(gcon[r]) + xscale);
      if (!(actf[r] & 4) && s2 < -tol2 && (s2 < best || (s2 == best && 2 * NU + v < bkey))) { best = s2; bkey = 2 * NU + v; }
    }
    wave_argmin_d(best, bkey);
    if (bkey == 0x7fffffff) break;  // no violated row: optimal
    const int p = bkey < 2 * NU ? 3 * (bkey >> 1) + (bkey & 1) : 3 * (bkey - 2 * NU) + 2;
    const int pown = p / 3, ptt = p - 3 * pown;
    double sp = best;
    double uplus = 0.0;  // multiplier of the candidate p
    double np[R];
    normal(p, np);
    // ---- step 2: add p, possibly after drops ----
    for (;;) {
      if (++it > max_iter) { status = F110QP_MAX_ITER_ID; break; }
      double w[R];
#pragma unroll
      for (int r = 0; r < R; r++) sm.vec[vv[r]] = np[r];
      wave_sync();
      matvec_W(w);  // w = W n_p
      wave_sync();
      double s = 0.0;
#pragma unroll
      for (int r = 0; r < R; r++) s += np[r] * w[r];
      const double nw = wave_sum(s);
      publish(w);
      double vj[R], lv[R], rr[R];
#pragma unroll
      for (int r = 0; r < R; r++) vj[r] = (64 * r + lane < q) ? slot_dot(slot_id[r]) : 0.0;
      // lv = L^-1 v (the new factor row), ll = |lv|^2, rr = L^-T lv = S^-1 v (dual direction)
#pragma unroll
      for (int r = 0; r < R; r++) lv[r] = vj[r];
      for (int j = 0; j < q; j++) {
        const double xj = rl_d<R>(lv, j) * rl_d<R>(rdiag, j);
#pragma unroll
        for (int r = 0; r < R; r++) {
          const int sl = 64 * r + lane;
          if (sl > j && sl < q) lv[r] = fma(-sm.L[sl][j], xj, lv[r]);
          if (sl == j) lv[r] = xj;
        }
      }
      double lls = 0.0;
#pragma unroll
      for (int r = 0; r < R; r++) lls += (64 * r + lane < q) ? lv[r] * lv[r] : 0.0;
      const double ll = wave_sum(lls);
#pragma unroll
      for (int r = 0; r < R; r++) rr[r] = lv[r];
      for (int j = q - 1; j >= 0; j--) {
        const double xj = rl_d<R>(rr, j) * rl_d<R>(rdiag, j);
#pragma unroll
        for (int r = 0; r < R; r++) {
          const int sl = 64 * r + lane;
          if (sl < j) rr[r] = fma(-sm.L[j][sl], xj, rr[r]);
          if (sl == j) rr[r] = xj;
        }
      }
      // z = W (n_p - N_A rr)
      double nr[R], z[R];
      nsum(rr, nr);
#pragma unroll
      for (int r = 0; r < R; r++) sm.vec[vv[r]] = np[r] - nr[r];
      wave_sync();
      matvec_W(z);
      wave_sync();
      const double pivv = nw - ll;  // = z'n_p, the new Schur pivot
      // partial step t1 (blocking multiplier k1, the first on ties as the oracle)
      double t1 = __longlong_as_double(0x7ff0000000000000ll);
      int k1 = 0x7fffffff;
#pragma unroll
      for (int r = 0; r < R; r++) {
        const int sl = 64 * r + lane;
        if (sl < q && rr[r] > 0.0) {
          const double tr = mult[r] / rr[r];
          if (tr < t1) { t1 = tr; k1 = sl; }
        }
      }
      wave_argmin_d(t1, k1);
      const bool indep = q < NU && pivv > 1e-12 * nw;
      const double t2 = indep ? -sp / pivv : __longlong_as_double(0x7ff0000000000000ll);
      const double tt = fmin(t1, t2);
      if (!isfinite(tt)) { status = F110QP_PRIMAL_INFEASIBLE_ID; break; }
#pragma unroll
      for (int r = 0; r < R; r++)
        if (64 * r + lane < q) mult[r] = fma(-tt, rr[r], mult[r]);
      uplus += tt;
      bool add = false;
      if (indep) {
#pragma unroll
        for (int r = 0; r < R; r++) x[r] = fma(tt, z[r], x[r]);
        sp = fma(tt, pivv, sp);
        add = t2 <= t1;
      }
      if (add) {
#pragma unroll
        for (int r = 0; r < R; r++) {
          const int sl = 64 * r + lane;
          if (sl < q) sm.L[q][sl] = lv[r];
          if (sl == q) {
            slot_id[r] = p;
            mult[r] = uplus;
            rdiag[r] = 1.0 / sqrt(pivv);
          }
          if (vv[r] == pown) actf[r] |= (1 << ptt);
        }
        if (lane == 0) sm.L[q][q] = sqrt(pivv);
        q++;
        wave_sync();
        break;
      }
      // drop slot k1 (a dependent p keeps its multiplier and is retried, as the oracle)
      {
        const int kd = k1;
        const int did = rl_i<R>(slot_id, kd);
        const int down = did / 3;
#pragma unroll
        for (int r = 0; r < R; r++)
          if (vv[r] == down) actf[r] &= ~(1 << (did - 3 * down));
        int sid_n[R];
        double mul_n[R];
#pragma unroll
        for (int r = 0; r < R; r++) {
          sid_n[r] = __shfl_down(slot_id[r], 1, 64);
          mul_n[r] = __shfl_down(mult[r], 1, 64);
          if (r + 1 < R) {
            const int s_next = readlane_i(slot_id[r + 1 < R ? r + 1 : r], 0);
            const double m_next = readlane_d(mult[r + 1 < R ? r + 1 : r], 0);
            if (lane == 63) { sid_n[r] = s_next; mul_n[r] = m_next; }
          }
        }
#pragma unroll
        for (int r = 0; r < R; r++) {
          const int sl = 64 * r + lane;
          if (sl >= kd && sl < q - 1) { slot_id[r] = sid_n[r]; mult[r] = mul_n[r]; }
          if (sl == q - 1) { slot_id[r] = -1; mult[r] = 0.0; }
        }
        // S_A without row / column kd = (L without row kd)(L without row kd)': rows kd+1..q-1 move
        // up (each lane its own row, column by column: iteration c touches column c only), then
        // Givens rotations on the column pairs (j, j + 1), j = kd..q-2, clear the superdiagonal of
        // the Hessenberg rows (row j's diagonal becomes hypot > 0) and column q-1 empties
        for (int c = 0; c < q; c++) {
#pragma unroll
          for (int r = 0; r < R; r++) {
            const int row = 64 * r + lane;
            if (row >= kd && row < q - 1) sm.L[row][c] = (c <= row + 1) ? sm.L[row + 1][c] : 0.0;
          }
        }
        wave_sync();
        for (int j = kd; j < q - 1; j++) {
          const double aa = sm.L[j][j], bb2 = sm.L[j][j + 1];
          const double hh = sqrt(aa * aa + bb2 * bb2);
          const double cs = aa / hh, sn = bb2 / hh;
          wave_sync();
#pragma unroll
          for (int r = 0; r < R; r++) {
            const int row = 64 * r + lane;
            if (row >= j && row < q - 1) {
              const double cj = sm.L[row][j], cj1 = sm.L[row][j + 1];
              sm.L[row][j] = cs * cj + sn * cj1;
              sm.L[row][j + 1] = cs * cj1 - sn * cj;
            }
          }
          wave_sync();
        }
        q--;
#pragma unroll
        for (int r = 0; r < R; r++) {
          const int sl = 64 * r + lane;
          rdiag[r] = (sl < q) ? 1.0 / sm.L[sl][sl] : 0.0;
        }
        wave_sync();
      }
    }
  }

  // ---- 4. the final set's equality QP solved afresh, certificate, outputs -------------------------
  // x and mu accumulate the rounding of every GI step; the optimum of the final set is recomputed
  // from W and the factor: S_A mu = b_A + N_A' W g, x = W (N_A mu - g)
  if (status == F110QP_SOLVED_ID && q > 0) {
    double wg[R], v[R];
#pragma unroll
    for (int r = 0; r < R; r++) sm.vec[vv[r]] = g[r];
    wave_sync();
    matvec_W(wg);
    wave_sync();
    publish(wg);
#pragma unroll
    for (int r = 0; r < R; r++) {
      v[r] = 0.0;
      if (64 * r + lane < q) {
        const int sid = slot_id[r], own = sid / 3, tt = sid - 3 * own;
        const double bj = tt == 0 ? ((own & 1) ? lb1 : lb0) : (tt == 1 ? -((own & 1) ? ub1 : ub0) : 0.0);
        v[r] = slot_dot(sid) + bj;
      }
    }
    wave_sync();
    // the gap rows' b (the oracle's -c - a f_x - b f_y) through the per-id table
#pragma unroll
    for (int r = 0; r < R; r++) sm.cid[3 * vv[r] + 2] = gcon[r];
    wave_sync();
#pragma unroll
    for (int r = 0; r < R; r++)
      if (64 * r + lane < q && slot_id[r] % 3 == 2) v[r] += sm.cid[slot_id[r]];
    wave_sync();
    for (int j = 0; j < q; j++) {  // v <- L^-1 v
      const double xj = rl_d<R>(v, j) * rl_d<R>(rdiag, j);
#pragma unroll
      for (int r = 0; r < R; r++) {
        const int sl = 64 * r + lane;
        if (sl > j && sl < q) v[r] = fma(-sm.L[sl][j], xj, v[r]);
        if (sl == j) v[r] = xj;
      }
    }
    for (int j = q - 1; j >= 0; j--) {  // v <- L^-T v = mu
      const double xj = rl_d<R>(v, j) * rl_d<R>(rdiag, j);
#pragma unroll
      for (int r = 0; r < R; r++) {
        const int sl = 64 * r + lane;
        if (sl < j) v[r] = fma(-sm.L[j][sl], xj, v[r]);
        if (sl == j) v[r] = xj;
      }
    }
    double nm[R];
    nsum(v, nm);
#pragma unroll
    for (int r = 0; r < R; r++) {
      sm.vec[vv[r]] = nm[r] - g[r];
      if (64 * r + lane < q) mult[r] = v[r];
    }
    wave_sync();
    matvec_W(x);
    wave_sync();
  }
  double px[R], py[R], th[R];
  rollout_f64<R>(M, lane, x, px, py, th);
  if (status == F110QP_SOLVED_ID) {
    double umax = 0.0;
    bool viol = false;
#pragma unroll
    for (int r = 0; r < R; r++) {
      if (!valid[r]) continue;
      umax = fmax(umax, fabs(x[r]));
    }
    umax = wave_max_d(umax);
#pragma unroll
    for (int r = 0; r < R; r++) {
      if (!valid[r]) continue;
      const double tol = 1e-9;
      viol |= x[r] - lb[r] < -tol * (1.0 + fabs(lb[r]) + umax);
      viol |= ub[r] - x[r] < -tol * (1.0 + fabs(ub[r]) + umax);
      viol |= gah * px[r] + gbh * py[r] - gbe < -tol * (1.0 + fabs(gcon[r]) + umax);
    }
    // rho = H u + g - N_A mu+ (fp64 rollout and costate), mu clamped at 0
    double mup[R], nmu[R], gu[R], zero[R];
#pragma unroll
    for (int r = 0; r < R; r++) { mup[r] = (64 * r + lane < q) ? fmax(mult[r], 0.0) : 0.0; zero[r] = 0.0; }
    nsum(mup, nmu);
    grad_f64<R>(M, P, lane, N, x, px, py, th, rxd, ryd, rthd, zero, zero, gu);
    double rho[R], wr[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
      rho[r] = valid[r] ? gu[r] - nmu[r] : 0.0;
      sm.vec[vv[r]] = rho[r];
    }
    wave_sync();
    matvec_W(wr);
    wave_sync();
    // rho'W rho from above in fp64: y = W rho, rho'H^-1 rho <= y'(2 rho - H y) + |rho - H y|^2 / lambda
    const double lam = fmin(P.r[0], P.r[1]);
    double hy[R];
    hv_f64<R>(M, P, lane, N, wr, hy);
    double t1 = 0.0, t2 = 0.0;
#pragma unroll
    for (int r = 0; r < R; r++) {
      const double rr = valid[r] ? rho[r] - hy[r] : 0.0;
      t1 += valid[r] ? wr[r] * (2.0 * rho[r] - hy[r]) : 0.0;
      t2 += rr * rr;
    }
    const double rs = wave_sum(t1) + wave_sum(t2) / lam;
    const double ctol = kCertTau * fmax(1.0, umax);
    const bool cert = !(__ballot(viol) != 0ull) && rs >= 0.0 && rs <= lam * ctol * ctol;
    if (!cert) status = F110QP_SOLVED_INACCURATE_ID;
  }
  const bool ok = (status == F110QP_SOLVED_ID) || (status == F110QP_SOLVED_INACCURATE_ID);
  {
    const float nanv = __int_as_float(0x7fc00000);
    float* xo = xout + (size_t)b * 3 * (N + 1);
    if (lane == 0) {
      xo[0] = ok ? fX0 : nanv;
      xo[1] = ok ? fY0 : nanv;
      xo[2] = ok ? fTH0 : nanv;
    }
#pragma unroll
    for (int r = 0; r < R; r++) {
      if (valid[r]) uout[(size_t)b * NU + vv[r]] = ok ? (float)x[r] : nanv;
      if (valid[r] && a == 1) {
        xo[3 * (kk[r] + 1) + 0] = ok ? (float)(px[r] + X0) : nanv;
        xo[3 * (kk[r] + 1) + 1] = ok ? (float)(py[r] + Y0) : nanv;
        xo[3 * (kk[r] + 1) + 2] = ok ? (float)th[r] : nanv;
      }
    }
    if (oo.obj || oo.cost) {  // as solve_kernel.h's output sweep (mpc.cpp:208-229 objective)
      const double q0 = P.q[0], q1 = P.q[1], q2 = P.q[2];
      double J = 0.0, Cr = 0.0;
#pragma unroll
      for (int r = 0; r < R; r++) {
        if (!valid[r]) continue;
        const double ra = a ? P.r[1] : P.r[0], uda = a ? P.udes[1] : P.udes[0];
        J += 0.5 * ra * (x[r] - uda) * (x[r] - uda);
        if (a == 1) {
          const double dx = px[r] - rxd[r], dy = py[r] - ryd[r], dth = th[r] - rthd[r];
          J += 0.5 * (q0 * dx * dx + q1 * dy * dy + q2 * dth * dth);
          const double wx = rxd[r] + X0, wy = ryd[r] + Y0;
          Cr += 0.5 * (q0 * wx * wx + q1 * wy * wy + q2 * rthd[r] * rthd[r]);
        }
      }
      if (lane == 0) {
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
  }
}

// One workgroup per list item, a grid-stride loop over the device-side count: every listed QP is
// re-checked whatever the grid. Each item ends at a workgroup barrier that the waves other than
// wave 0 wait at while wave 0 runs GI.
template <int NUM>
__global__ __launch_bounds__(64 * ((2 * NUM + 63) / 64)) void gi64_kernel(const KParams P, const float* __restrict__ x0g,
                                                                   const float* __restrict__ ulg,
                                                                   const float* __restrict__ xrg,
                                                                   const float* __restrict__ hsg,
                                                                   float* __restrict__ uout,
                                                                   float* __restrict__ xout,
                                                                   int* __restrict__ status_out,
                                                                   int* __restrict__ iters_out,
                                                                   const int* __restrict__ list,
                                                                   const int* __restrict__ count,
                                                                   const ObjOut oo) {
  __shared__ G64Smem<NUM> sm;
  const int n = __builtin_amdgcn_readfirstlane(*count);
  for (int item = blockIdx.x; item < n; item += gridDim.x) {
    const int b = __builtin_amdgcn_readfirstlane(list[item]);
    gi64_qp<NUM>(sm, b, P, x0g, ulg, xrg, hsg, uout, xout, status_out, iters_out, oo);
    __syncthreads();
  }
  signal_call_done(oo, (int)blockIdx.x < n);  // the completion word of a synchronous gap-row call
}

template <int NUM>
hipError_t launch_gi64_t(const KParams& P, int grid, const float* x0, const float* ul, const float* xr,
                         const float* hs, float* uo, float* xo, int* st, int* its, const int* list,
                         const int* count, const ObjOut& oo, hipStream_t s) {
  hipLaunchKernelGGL((gi64_kernel<NUM>), dim3(grid), dim3(64 * ((2 * NUM + 63) / 64)), 0, s, P, x0, ul, xr, hs, uo,
                     xo, st, its, list, count, oo);
  return hipGetLastError();
}

}  // namespace f110qp

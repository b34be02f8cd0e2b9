// lane_ipm_kernel.h — the lane back end for QPs WITH the follow-the-gap rows (BASELINE configs[2],
// C3): a Mehrotra predictor-corrector interior point whose every Newton system is one Riccati
// factorisation on the partitioned horizon of lane_seg_kernel.h (one QP per S lanes, each lane
// one segment of m = N / S stages), finished by an OSQP-style polish that makes the answer exact.
//
// The QP (recentred on x0; rotated into the heading frame when ROT; mpc.cpp:208-306 with the C3
// gap semantic of mpc.cpp:297-298):
//   min sum_{i<N} 1/2|x_i - r_i|_Q^2 + 1/2|x_N - r_{N-1}|_Q^2 + sum_i 1/2|u_i - ud|_R^2
//   s.t. x_{i+1} = A x_i + B u_i + C (model.cpp:42-55), x_0 = 0,
//        lb <= u_i <= ub (constraints.cpp:19,21), nu_k' x_{i+1} >= beta_k (k = 0, 1;
//        mpc.cpp:249,271: the two half-spaces of FindHalfSpaces, rows normalised).
// Stage i owns six inequality rows, c_i = (u0 - lb0, ub0 - u0, u1 - lb1, ub1 - u1,
// nu_0'x_{i+1} - beta_0, nu_1'x_{i+1} - beta_1), each with a slack s > 0 and a multiplier z > 0.
// The primal iterate keeps x = rollout(u), so each Newton step is an LQ problem in (dx, du) with
//   R~_i = R + diag(Sig_0 + Sig_1, Sig_2 + Sig_3),  Q~_{i+1} = Q + sum_k Sig_{4+k} nu_k nu_k'
// (Sig = z / s: the rank-2 gap term on the state's (x, y) block, a diagonal on the inputs) and the
// linear terms grad f + D'e, e_j = Sig_j (c_j - s_j) [+ (ds_aff dz_aff - sigma mu)_j / s_j]. One
// backward sweep factors it (K_i, H_i^-1, the lam-gains F_i of the segment coupling) and solves
// the predictor; the corrector and the polish re-use the factor with linear-only sweeps. The
// segment ends are lane_seg_kernel.h's two-point recursion (the Riccati over the segments once
// per factor, then a vector-only pass per further right-hand side).
//
// Polish (OSQP's `polish`, here the exit test): once a QP's mu is small it guesses the active rows
// A = {z > 1e4 s} and solves the equality QP on them by an augmented Lagrangian on the SAME factor
// (penalty Sig_j, multipliers started at z_j; inactive rows act as proximal terms that vanish at
// convergence): two linear-only solves. The QP is SOLVED when every inactive row holds
// (c >= -tol), every active row holds with equality (|c| <= tol) and carries a multiplier >= -tol:
// the KKT conditions of the reference QP, checked in fp64 on the point that is returned. A QP the
// interior point has not polished after IpmKnobs::max_iter iterations (primal infeasible, or a stalled
// path) goes on the hand-over list: the wave kernel's Goldfarb-Idnani loop solves it or proves
// infeasibility (status -3), exactly as before. Design model: tests/diag_ipm_model.py.
// The factor 1e4 (IpmKnobs::act_sig, was 1): a degenerate row whose z and s both go to zero
// (z ~ s ~ sqrt(mu)) carries Sig ~ 1, too small a penalty for the two AL steps to pin it, and
// with z > s it failed the multiplier sign test at every iterate (an N = 48 gap QP that neither
// this polish nor GI certified; numpy model first: acceptance up on 4 test batches at 1e2..1e6
// with no accuracy change; on the device, at S = 16, 1e4 accepted it and 1e2 did not); such a
// row is taken as inactive, and an active row's penalty is then large enough for the two AL
// steps' convergence test to mean stationarity.
//
// Layout: LDS per wave, lane-major rows (every access one conflict-free 64-lane row), fp64:
// references [3m][64], per-stage fields [m][kIpmNF][64], the segment-end state [39][64].
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "f110qp_kernels.h"

namespace f110qp {

// per-stage fields (doubles)
enum : int {
  kFXn = 0,     // x_{i+1} (3)
  kFU = 3,      // u_i (2)
  kFS = 5,      // slacks (6)
  kFZ = 11,     // multipliers (6)
  kFK = 17,     // K_i (6)
  kFHi = 23,    // H_i^-1 (3: 00, 01, 11)
  kFFl = 26,    // lam-gains F_i = -H_i^-1 W_i' (6)
  kFk = 32,     // k_i of the current right-hand side (2)
  kFDsDz = 34,  // predictor ds * dz (6)
  kFDu = 40,    // corrector du (2)
  kFDxn = 42,   // corrector dx_{i+1} (3)
  kFUp = 45,    // polish u (2)
  kFXnp = 47,   // polish x_{i+1} (3)
  kIpmNF = 50
};
constexpr int kIpmSegState = 39;  // Mn 6, Zi 9, T 9, Phi 9, Gam 6

constexpr size_t ipm_lds_bytes(int N, int S) {
  return (size_t)64 * 8 * ((size_t)((N + S - 1) / S) * (3 + kIpmNF) + (S > 1 ? kIpmSegState : 0));
}

#ifndef F110QP_IPM_WPE
#define F110QP_IPM_WPE 1
#endif

template <int M>
struct IpmTag {
  static constexpr int value = M;
};

// one Newton step: ~1e-15 relative, enough for the slack inverses of the Newton systems
__device__ __forceinline__ double ipm_rcp1(double v) {
  const double r = __builtin_amdgcn_rcp(v);
  return fma(r, fma(-v, r, 1.0), r);
}

__device__ __forceinline__ double ipm_rcp(double v) {
  double r = __builtin_amdgcn_rcp(v);
  r = fma(r, fma(-v, r, 1.0), r);
  r = fma(r, fma(-v, r, 1.0), r);
  return r;
}

template <int S, bool ROT>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(F110QP_IPM_WPE, F110QP_IPM_WPE))) void lane_ipm_kernel(
    const KParams P, const int B, const float* __restrict__ x0g, const float* __restrict__ ulg,
    const float* __restrict__ xrg, const float* __restrict__ hsg, float* __restrict__ uout,
    float* __restrict__ xout, int* __restrict__ status_out, int* __restrict__ iters_out,
    int* __restrict__ hand_list, int* __restrict__ hand_count, const IpmKnobs kn, const ObjOut oo,
    const int* __restrict__ qlist, const int* __restrict__ qcount, const int recheck) {
  constexpr int L = 64 / S;  // QPs per wave
  constexpr int NF = kIpmNF;
  extern __shared__ __attribute__((aligned(16))) double ipm_smem[];
  const int lane = threadIdx.x;
  const int sl = lane & (L - 1);
  const int seg = lane / L;
  // list mode (qlist): the wave takes list items b0 .. b0 + L - 1 of the device list (the wave
  // kernel's flagged QPs); otherwise QPs b0 .. b0 + L - 1 of the batch
  const int nb = qlist ? __builtin_amdgcn_readfirstlane(*qcount) : B;
  const int b0 = blockIdx.x * L;
  if (b0 >= nb) return;  // wave-uniform: an empty part of the list
  const int nq = (nb - b0) < L ? (nb - b0) : L;
  const int slot = sl < nq ? sl : 0;  // a missing QP's lanes duplicate QP 0 of the wave
  const bool owner = sl < nq;
  const bool qowner = owner && seg == 0;
  const int b = qlist ? qlist[b0 + slot] : b0 + slot;
  const int N = P.N;
  const int q = N / S, rem = N - q * S;
  const int m = q + (seg < rem ? 1 : 0);
  const int s0 = seg * q + (seg < rem ? seg : rem);
  const int mM = q + (rem > 0 ? 1 : 0);
  const bool top = seg == S - 1;
  const int up = (lane + L) & 63, dn = (lane - L) & 63;

  double* const r64 = ipm_smem + lane;                   // [3 mM][64]
  double* const fs = ipm_smem + 3 * mM * 64 + lane;      // [mM][NF][64]
  double* const ss = ipm_smem + (3 + NF) * mM * 64 + lane;  // [39][64]
  auto F = [&](int t, int f) -> double& { return fs[(t * NF + f) * 64]; };

  const float fX0 = x0g[3 * b + 0], fY0 = x0g[3 * b + 1], fTH0 = x0g[3 * b + 2];
  const float fv = ulg[2 * b + 0], fd = ulg[2 * b + 1];
  const float h00 = hsg[6 * b + 0], h01 = hsg[6 * b + 1], h02 = hsg[6 * b + 2];
  const float h10 = hsg[6 * b + 3], h11 = hsg[6 * b + 4], h12 = hsg[6 * b + 5];
  // ---- stage the wave's reference paths (float, [3N][L]) into the stage-field region, as
  // lane_seg_kernel.h (no EXEC-masked region) ----
  {
    float* stg = reinterpret_cast<float*>(ipm_smem + 3 * mM * 64);
    const int n3 = 3 * N, S3 = 3 * P.xr_stride, tot = nq * n3;
    const float* src = xrg + (qlist ? (size_t)0 : (size_t)b0 * S3);
    const int dq = 64 / n3, dc = 64 - dq * n3;
    int qq = lane / n3, c = lane - (lane / n3) * n3;
    const int junk = n3 * L + lane;
    const size_t last_off = (size_t)(qlist ? qlist[b0 + nq - 1] : nq - 1) * S3 + (n3 - 1);
    constexpr int kChunk = 16;
    for (int e0 = 0; e0 < tot; e0 += kChunk * 64) {
      float vbuf[kChunk];
      int dst[kChunk];
#pragma unroll
      for (int j = 0; j < kChunk; j++) {
        const bool in = e0 + j * 64 + lane < tot;
        dst[j] = in ? c * L + qq : junk;
        vbuf[j] = src[in ? (size_t)(qlist ? qlist[b0 + qq] : qq) * S3 + c : last_off];
        qq += dq;
        c += dc;
        const bool wrap = c >= n3;
        c -= wrap ? n3 : 0;
        qq += wrap ? 1 : 0;
      }
#pragma unroll
      for (int j = 0; j < kChunk; j++) stg[dst[j]] = vbuf[j];
    }
    __syncthreads();
  }

  // ---- per-lane QP data (Model::Linearize, model.cpp:30-59) ----
  const double X0 = (double)fX0, Y0 = (double)fY0;
  const double th0 = (double)fTH0;
  const double v = (double)fv, d = (double)fd;
  const double dt = (double)P.dt;
  const double Lw = (double)0.3302f;
  double sn, cs, sd, cd;
  sincos(th0, &sn, &cs);
  sincos(d, &sd, &cd);
  const double sec2 = 1.0 / (cd * cd);
  const double a02 = ROT ? 0.0 : -1 * v * sn * dt;                    // model.cpp:42
  const double a12 = ROT ? v * dt : v * cs * dt;                      // :43
  const double b00 = ROT ? dt : cs * dt, b10 = ROT ? 0.0 : sn * dt;   // :48-49
  const double b20 = (sd / cd) * dt / Lw, b21 = v * sec2 * dt / Lw;   // :50-51
  const double c0r = v * th0 * sn * dt, c1r = -1 * v * th0 * cs * dt;  // :53-54
  const double c2 = -1 * d * v * sec2 * dt / Lw;                      // :55
  const double c0 = ROT ? 0.0 : c0r + a02 * th0, c1 = ROT ? 0.0 : c1r + a12 * th0;
  const double q0 = P.q[0], q1 = P.q[1], q2 = P.q[2], r0 = P.r[0], r1 = P.r[1];
  const double ud0 = P.udes[0], ud1 = P.udes[1];
  const double lb0 = (double)P.umin[0], lb1 = (double)P.umin[1];
  const double ub0 = (double)P.umax[0], ub1 = (double)P.umax[1];
  // gap rows (constraints.cpp:255-264: l = (a, b, c + 0.5), a x + b y >= -(c + 0.5)), recentred
  // on (X0, Y0), in the lane's frame, normalised
  double n0s, n0n, be0, n1s, n1n, be1;
  bool gapbad;
  {
    const double A0 = h00, Bb0 = h01, A1 = h10, Bb1 = h11;
    const double nr0 = sqrt(A0 * A0 + Bb0 * Bb0), nr1 = sqrt(A1 * A1 + Bb1 * Bb1);
    gapbad = !(nr0 > 1e-300) || !(nr1 > 1e-300);
    const double i0 = gapbad ? 0.0 : 1.0 / nr0, i1 = gapbad ? 0.0 : 1.0 / nr1;
    n0s = (ROT ? A0 * cs + Bb0 * sn : A0) * i0;
    n0n = (ROT ? Bb0 * cs - A0 * sn : Bb0) * i0;
    n1s = (ROT ? A1 * cs + Bb1 * sn : A1) * i1;
    n1n = (ROT ? Bb1 * cs - A1 * sn : Bb1) * i1;
    be0 = (-(double)h02 - A0 * X0 - Bb0 * Y0) * i0;
    be1 = (-(double)h12 - A1 * X0 - Bb1 * Y0) * i1;
  }
  const double sc0 = 1.0 + fabs(lb0), sc1 = 1.0 + fabs(ub0), sc2 = 1.0 + fabs(lb1), sc3 = 1.0 + fabs(ub1);
  const double sc4 = 1.0 + fabs(be0), sc5 = 1.0 + fabs(be1);

  // references of the lane's stages: recentred (ROT: rotated) fp64, lane-major (the float staging
  // sits in the stage-field region, past the fp64 rows: no overlap)
  bool nonfin = false;
  {
    const float* stg = reinterpret_cast<const float*>(ipm_smem + 3 * mM * 64);
    for (int t = 0; t < m; t++) {
      const int i = s0 + t;
      const float fx = stg[(3 * i + 0) * L + slot], fy = stg[(3 * i + 1) * L + slot];
      const float ft = stg[(3 * i + 2) * L + slot];
      nonfin |= !(isfinite(fx) && isfinite(fy) && isfinite(ft));
      const double dx = (double)fx - X0, dy = (double)fy - Y0;
      r64[(3 * t + 0) * 64] = ROT ? cs * dx + sn * dy : dx;
      r64[(3 * t + 1) * 64] = ROT ? cs * dy - sn * dx : dy;
      r64[(3 * t + 2) * 64] = (double)ft - th0;
    }
    __syncthreads();  // the staging region becomes the stage fields
  }
  // terminal reference x_ref[N-1] (mpc.cpp:228): the last stage of the top segment
  const int toplane = (lane | (63 & ~(L - 1))) & 63;
  const double rNx = __shfl(r64[(3 * (m - 1) + 0) * 64], toplane);
  const double rNy = __shfl(r64[(3 * (m - 1) + 1) * 64], toplane);
  const double rNt = __shfl(r64[(3 * (m - 1) + 2) * 64], toplane);

  auto fold = [&](unsigned long long mk) {
#pragma unroll
    for (int k = L; k < 64; k <<= 1) mk |= mk >> k;
    return mk;
  };
  auto qsum = [&](double x) {
#pragma unroll
    for (int k = L; k < 64; k <<= 1) x += __shfl_xor(x, k, 64);
    return x;
  };
  auto qmin = [&](double x) {
#pragma unroll
    for (int k = L; k < 64; k <<= 1) x = fmin(x, __shfl_xor(x, k, 64));
    return x;
  };
  const bool bad = !(isfinite(X0) && isfinite(Y0) && isfinite(th0) && isfinite(v) && isfinite(d)) ||
                   !(isfinite(n0s) && isfinite(n0n) && isfinite(be0) && isfinite(n1s) && isfinite(n1n) &&
                     isfinite(be1)) ||
                   ((fold(__ballot(nonfin)) >> sl) & 1ull);
  // degenerate half-space normals: no interior point; the wave kernel's GI takes the QP
  const bool handover0 = !bad && gapbad;

  // ---- initial point: u = box centre, x = rollout(u), s = max(c, s_floor), z = 1 ----
  const double um0 = 0.5 * (lb0 + ub0), um1 = 0.5 * (lb1 + ub1);
  double xs0 = 0.0, xs1 = 0.0, xs2 = 0.0;  // the segment's start state x_{s0}
  {
    // segment map of the rollout: x_e = A^m x_s + psi, A^m = I + m E (E^2 = 0, model.cpp:42-46)
    double p0 = 0.0, p1 = 0.0, p2 = 0.0;
    for (int t = 0; t < m; t++) {
      const double n0 = ROT ? p0 + b00 * um0 : p0 + a02 * p2 + b00 * um0 + c0;
      const double n1 = ROT ? p1 + a12 * p2 : p1 + a12 * p2 + b10 * um0 + c1;
      const double n2 = p2 + b20 * um0 + b21 * um1 + c2;
      p0 = n0; p1 = n1; p2 = n2;
    }
    const double md = (double)m;
    if constexpr (S > 1) {
#pragma unroll 1
      for (int it = 0; it < S - 1; it++) {
        const double e0 = top ? 0.0 : xs0 + md * a02 * xs2 + p0;
        const double e1 = top ? 0.0 : xs1 + md * a12 * xs2 + p1;
        const double e2 = top ? 0.0 : xs2 + p2;
        xs0 = __shfl(e0, dn);
        xs1 = __shfl(e1, dn);
        xs2 = __shfl(e2, dn);
      }
    }
    double x0 = xs0, x1 = xs1, x2 = xs2;
    for (int t = 0; t < m; t++) {
      const double n0 = ROT ? x0 + b00 * um0 : x0 + a02 * x2 + b00 * um0 + c0;
      const double n1 = ROT ? x1 + a12 * x2 : x1 + a12 * x2 + b10 * um0 + c1;
      const double n2 = x2 + b20 * um0 + b21 * um1 + c2;
      x0 = n0; x1 = n1; x2 = n2;
      F(t, kFXn + 0) = x0; F(t, kFXn + 1) = x1; F(t, kFXn + 2) = x2;
      F(t, kFU + 0) = um0; F(t, kFU + 1) = um1;
      const double cg0 = n0s * x0 + n0n * x1 - be0, cg1 = n1s * x0 + n1n * x1 - be1;
      const double sf = kn.s_floor;
      F(t, kFS + 0) = fmax(um0 - lb0, sf); F(t, kFS + 1) = fmax(ub0 - um0, sf);
      F(t, kFS + 2) = fmax(um1 - lb1, sf); F(t, kFS + 3) = fmax(ub1 - um1, sf);
      F(t, kFS + 4) = fmax(cg0, sf); F(t, kFS + 5) = fmax(cg1, sf);
#pragma unroll
      for (int j = 0; j < 6; j++) {
        F(t, kFZ + j) = 1.0;
        F(t, kFDsDz + j) = 0.0;
      }
      F(t, kFDu + 0) = 0.0; F(t, kFDu + 1) = 0.0;
      F(t, kFDxn + 0) = 0.0; F(t, kFDxn + 1) = 0.0; F(t, kFDxn + 2) = 0.0;
    }
  }

  const double mrows = 6.0 * (double)N;
  bool done = bad || handover0;
  int iters = 0;

  // stage quantities shared by the sweeps
  // constraint values of stage t at (u, xn)
  auto cvals = [&](double u0, double u1, double x0, double x1, double* c) {
    c[0] = u0 - lb0; c[1] = ub0 - u0; c[2] = u1 - lb1; c[3] = ub1 - u1;
    c[4] = n0s * x0 + n0n * x1 - be0;
    c[5] = n1s * x0 + n1n * x1 - be1;
  };

  // ---- one backward Riccati step (factor or linear-only) ----
  // state: P (sym), p, Phi, psi, Gam. Linear-only sweeps (FAC = false) carry p and psi only.
  double P00, P01, P02, P11, P12, P22, p0, p1, p2;
  double F00, F01, F02, F10, F11, F12, F20, F21, F22;
  double s0v, s1v, s2v, G00, G01, G02, G11, G12, G22;

  // segment ends, full (after the factor sweep): Riccati over the segments; stores Mn, Zi, T,
  // Phi, Gam in the segment-state rows and returns lam_j, dx_s.
  auto seg_full = [&](double& lm0, double& lm1, double& lm2, double& dx0, double& dx1, double& dx2) {
    if (top) {
      F00 = F01 = F02 = F10 = F11 = F12 = F20 = F21 = F22 = 0.0;
      s0v = s1v = s2v = 0.0;
      G00 = G01 = G02 = G11 = G12 = G22 = 0.0;
    }
    lm0 = lm1 = lm2 = 0.0;
    dx0 = dx1 = dx2 = 0.0;
    if constexpr (S > 1) {
      double M00 = P00, M01 = P01, M02 = P02, M11 = P11, M12 = P12, M22 = P22;
      double mm0 = p0, mm1 = p1, mm2 = p2;
      double T00 = 0, T01 = 0, T02 = 0, T10 = 0, T11 = 0, T12 = 0, T20 = 0, T21 = 0, T22 = 0;
      double t0 = 0, t1 = 0, t2 = 0;
      double N00 = 0, N01 = 0, N02 = 0, N11 = 0, N12 = 0, N22 = 0;
      double Z00i = 0, Z01i = 0, Z02i = 0, Z10i = 0, Z11i = 0, Z12i = 0, Z20i = 0, Z21i = 0, Z22i = 0;
#pragma unroll 1
      for (int it = 0; it < S - 1; it++) {
        N00 = __shfl(M00, up); N01 = __shfl(M01, up); N02 = __shfl(M02, up);
        N11 = __shfl(M11, up); N12 = __shfl(M12, up); N22 = __shfl(M22, up);
        const double n0 = __shfl(mm0, up), n1 = __shfl(mm1, up), n2 = __shfl(mm2, up);
        const double Z00 = 1.0 - (N00 * G00 + N01 * G01 + N02 * G02);
        const double Z01 = -(N00 * G01 + N01 * G11 + N02 * G12);
        const double Z02 = -(N00 * G02 + N01 * G12 + N02 * G22);
        const double Z10 = -(N01 * G00 + N11 * G01 + N12 * G02);
        const double Z11 = 1.0 - (N01 * G01 + N11 * G11 + N12 * G12);
        const double Z12 = -(N01 * G02 + N11 * G12 + N12 * G22);
        const double Z20 = -(N02 * G00 + N12 * G01 + N22 * G02);
        const double Z21 = -(N02 * G01 + N12 * G11 + N22 * G12);
        const double Z22 = 1.0 - (N02 * G02 + N12 * G12 + N22 * G22);
        const double A00 = Z11 * Z22 - Z12 * Z21, A01 = Z02 * Z21 - Z01 * Z22, A02 = Z01 * Z12 - Z02 * Z11;
        const double A10 = Z12 * Z20 - Z10 * Z22, A11 = Z00 * Z22 - Z02 * Z20, A12 = Z02 * Z10 - Z00 * Z12;
        const double A20 = Z10 * Z21 - Z11 * Z20, A21 = Z01 * Z20 - Z00 * Z21, A22 = Z00 * Z11 - Z01 * Z10;
        const double zdet = Z00 * A00 + Z01 * A10 + Z02 * A20;
        const double iz = ipm_rcp(zdet);
        Z00i = iz * A00; Z01i = iz * A01; Z02i = iz * A02;
        Z10i = iz * A10; Z11i = iz * A11; Z12i = iz * A12;
        Z20i = iz * A20; Z21i = iz * A21; Z22i = iz * A22;
        const double U00 = N00 * F00 + N01 * F10 + N02 * F20, U01 = N00 * F01 + N01 * F11 + N02 * F21;
        const double U02 = N00 * F02 + N01 * F12 + N02 * F22;
        const double U10 = N01 * F00 + N11 * F10 + N12 * F20, U11 = N01 * F01 + N11 * F11 + N12 * F21;
        const double U12 = N01 * F02 + N11 * F12 + N12 * F22;
        const double U20 = N02 * F00 + N12 * F10 + N22 * F20, U21 = N02 * F01 + N12 * F11 + N22 * F21;
        const double U22 = N02 * F02 + N12 * F12 + N22 * F22;
        const double w0 = N00 * s0v + N01 * s1v + N02 * s2v + n0;
        const double w1 = N01 * s0v + N11 * s1v + N12 * s2v + n1;
        const double w2 = N02 * s0v + N12 * s1v + N22 * s2v + n2;
        T00 = Z00i * U00 + Z01i * U10 + Z02i * U20; T01 = Z00i * U01 + Z01i * U11 + Z02i * U21;
        T02 = Z00i * U02 + Z01i * U12 + Z02i * U22;
        T10 = Z10i * U00 + Z11i * U10 + Z12i * U20; T11 = Z10i * U01 + Z11i * U11 + Z12i * U21;
        T12 = Z10i * U02 + Z11i * U12 + Z12i * U22;
        T20 = Z20i * U00 + Z21i * U10 + Z22i * U20; T21 = Z20i * U01 + Z21i * U11 + Z22i * U21;
        T22 = Z20i * U02 + Z21i * U12 + Z22i * U22;
        t0 = Z00i * w0 + Z01i * w1 + Z02i * w2;
        t1 = Z10i * w0 + Z11i * w1 + Z12i * w2;
        t2 = Z20i * w0 + Z21i * w1 + Z22i * w2;
        M00 = P00 + F00 * T00 + F10 * T10 + F20 * T20;
        M01 = P01 + F00 * T01 + F10 * T11 + F20 * T21;
        M02 = P02 + F00 * T02 + F10 * T12 + F20 * T22;
        M11 = P11 + F01 * T01 + F11 * T11 + F21 * T21;
        M12 = P12 + F01 * T02 + F11 * T12 + F21 * T22;
        M22 = P22 + F02 * T02 + F12 * T12 + F22 * T22;
        mm0 = p0 + F00 * t0 + F10 * t1 + F20 * t2;
        mm1 = p1 + F01 * t0 + F11 * t1 + F21 * t2;
        mm2 = p2 + F02 * t0 + F12 * t1 + F22 * t2;
      }
#pragma unroll 1
      for (int it = 0; it < S - 1; it++) {
        const double l0 = T00 * dx0 + T01 * dx1 + T02 * dx2 + t0;
        const double l1 = T10 * dx0 + T11 * dx1 + T12 * dx2 + t1;
        const double l2 = T20 * dx0 + T21 * dx1 + T22 * dx2 + t2;
        const double e0 = F00 * dx0 + F01 * dx1 + F02 * dx2 + s0v + G00 * l0 + G01 * l1 + G02 * l2;
        const double e1 = F10 * dx0 + F11 * dx1 + F12 * dx2 + s1v + G01 * l0 + G11 * l1 + G12 * l2;
        const double e2 = F20 * dx0 + F21 * dx1 + F22 * dx2 + s2v + G02 * l0 + G12 * l1 + G22 * l2;
        dx0 = __shfl(e0, dn);
        dx1 = __shfl(e1, dn);
        dx2 = __shfl(e2, dn);
      }
      lm0 = top ? 0.0 : T00 * dx0 + T01 * dx1 + T02 * dx2 + t0;
      lm1 = top ? 0.0 : T10 * dx0 + T11 * dx1 + T12 * dx2 + t1;
      lm2 = top ? 0.0 : T20 * dx0 + T21 * dx1 + T22 * dx2 + t2;
      const double st[kIpmSegState] = {N00, N01, N02, N11, N12, N22, Z00i, Z01i, Z02i, Z10i, Z11i, Z12i, Z20i,
                                       Z21i, Z22i, T00, T01, T02, T10, T11, T12, T20, T21, T22, F00, F01,
                                       F02, F10, F11, F12, F20, F21, F22, G00, G01, G02, G11, G12, G22};
#pragma unroll
      for (int e = 0; e < kIpmSegState; e++) ss[e * 64] = st[e];
    }
  };
  // segment ends, vector-only (after a linear sweep: p = a_s, psi of this right-hand side)
  auto seg_vec = [&](double& lm0, double& lm1, double& lm2, double& dx0, double& dx1, double& dx2) {
    lm0 = lm1 = lm2 = 0.0;
    dx0 = dx1 = dx2 = 0.0;
    if constexpr (S > 1) {
      double st[kIpmSegState];
#pragma unroll
      for (int e = 0; e < kIpmSegState; e++) st[e] = ss[e * 64];
      const double N00 = st[0], N01 = st[1], N02 = st[2], N11 = st[3], N12 = st[4], N22 = st[5];
      const double Z00i = st[6], Z01i = st[7], Z02i = st[8], Z10i = st[9], Z11i = st[10], Z12i = st[11];
      const double Z20i = st[12], Z21i = st[13], Z22i = st[14];
      const double T00 = st[15], T01 = st[16], T02 = st[17], T10 = st[18], T11 = st[19], T12 = st[20];
      const double T20 = st[21], T21 = st[22], T22 = st[23];
      const double H00 = st[24], H01 = st[25], H02 = st[26], H10 = st[27], H11 = st[28], H12 = st[29];
      const double H20 = st[30], H21 = st[31], H22 = st[32];  // Phi (top: 0)
      const double K00 = st[33], K01 = st[34], K02 = st[35], K11 = st[36], K12 = st[37], K22 = st[38];  // Gam
      if (top) s0v = s1v = s2v = 0.0;
      double mm0 = p0, mm1 = p1, mm2 = p2, t0 = 0.0, t1 = 0.0, t2 = 0.0;
#pragma unroll 1
      for (int it = 0; it < S - 1; it++) {
        const double n0 = __shfl(mm0, up), n1 = __shfl(mm1, up), n2 = __shfl(mm2, up);
        const double w0 = N00 * s0v + N01 * s1v + N02 * s2v + n0;
        const double w1 = N01 * s0v + N11 * s1v + N12 * s2v + n1;
        const double w2 = N02 * s0v + N12 * s1v + N22 * s2v + n2;
        t0 = Z00i * w0 + Z01i * w1 + Z02i * w2;
        t1 = Z10i * w0 + Z11i * w1 + Z12i * w2;
        t2 = Z20i * w0 + Z21i * w1 + Z22i * w2;
        mm0 = p0 + H00 * t0 + H10 * t1 + H20 * t2;
        mm1 = p1 + H01 * t0 + H11 * t1 + H21 * t2;
        mm2 = p2 + H02 * t0 + H12 * t1 + H22 * t2;
      }
#pragma unroll 1
      for (int it = 0; it < S - 1; it++) {
        const double l0 = T00 * dx0 + T01 * dx1 + T02 * dx2 + t0;
        const double l1 = T10 * dx0 + T11 * dx1 + T12 * dx2 + t1;
        const double l2 = T20 * dx0 + T21 * dx1 + T22 * dx2 + t2;
        const double e0 = H00 * dx0 + H01 * dx1 + H02 * dx2 + s0v + K00 * l0 + K01 * l1 + K02 * l2;
        const double e1 = H10 * dx0 + H11 * dx1 + H12 * dx2 + s1v + K01 * l0 + K11 * l1 + K12 * l2;
        const double e2 = H20 * dx0 + H21 * dx1 + H22 * dx2 + s2v + K02 * l0 + K12 * l1 + K22 * l2;
        dx0 = __shfl(e0, dn);
        dx1 = __shfl(e1, dn);
        dx2 = __shfl(e2, dn);
      }
      lm0 = top ? 0.0 : T00 * dx0 + T01 * dx1 + T02 * dx2 + t0;
      lm1 = top ? 0.0 : T10 * dx0 + T11 * dx1 + T12 * dx2 + t1;
      lm2 = top ? 0.0 : T20 * dx0 + T21 * dx1 + T22 * dx2 + t2;
    }
  };

  // the right-hand sides: MODE 0 predictor (factor sweep), 1 corrector, 2 polish 1, 3 polish 2
  // e_j of stage t: the pull-back D'e of the linear term (grad f + D'e)
  double smu = 0.0;  // sigma mu of the corrector

  // the step of the previous iteration (alpha_prev along the stored corrector direction, or the
  // polished point), applied as the next factor sweep reads the stage (the update pass fused in)
  double alpha_prev = 0.0;
  bool pol_prev = false;
  // (branch free: every operand is loaded and the polished point selected, no EXEC-masked loads)
  auto step_x = [&](int t, double& x0, double& x1, double& x2) {
    const double p0 = F(t, kFXnp + 0), p1 = F(t, kFXnp + 1), p2 = F(t, kFXnp + 2);
    const double a0 = F(t, kFXn + 0) + alpha_prev * F(t, kFDxn + 0);
    const double a1 = F(t, kFXn + 1) + alpha_prev * F(t, kFDxn + 1);
    const double a2 = F(t, kFXn + 2) + alpha_prev * F(t, kFDxn + 2);
    x0 = pol_prev ? p0 : a0;
    x1 = pol_prev ? p1 : a1;
    x2 = pol_prev ? p2 : a2;
  };
  auto step_stage = [&](int t, double& u0, double& u1, double& x0, double& x1, double& x2, double* sv,
                        double* zv) {
    double cc[6];
    const double ou0 = F(t, kFU), ou1 = F(t, kFU + 1);
    const double ox0 = F(t, kFXn), ox1 = F(t, kFXn + 1), ox2 = F(t, kFXn + 2);
    cvals(ou0, ou1, ox0, ox1, cc);
    const double du0 = F(t, kFDu), du1 = F(t, kFDu + 1);
    const double d0 = F(t, kFDxn), d1 = F(t, kFDxn + 1), d2 = F(t, kFDxn + 2);
    const double dc[6] = {du0, -du0, du1, -du1, n0s * d0 + n0n * d1, n1s * d0 + n1n * d1};
#pragma unroll
    for (int j = 0; j < 6; j++) {
      const double sj = F(t, kFS + j), zj = F(t, kFZ + j);
      const double is = ipm_rcp1(sj);
      const double ds = dc[j] + cc[j] - sj;
      const double dz = -zj - (F(t, kFDsDz + j) - smu) * is - zj * is * ds;
      sv[j] = sj + alpha_prev * ds;
      zv[j] = zj + alpha_prev * dz;
      F(t, kFS + j) = sv[j];
      F(t, kFZ + j) = zv[j];
    }
    const double pu0 = F(t, kFUp + 0), pu1 = F(t, kFUp + 1);
    const double px0 = F(t, kFXnp + 0), px1 = F(t, kFXnp + 1), px2 = F(t, kFXnp + 2);
    u0 = pol_prev ? pu0 : ou0 + alpha_prev * du0;
    u1 = pol_prev ? pu1 : ou1 + alpha_prev * du1;
    x0 = pol_prev ? px0 : ox0 + alpha_prev * d0;
    x1 = pol_prev ? px1 : ox1 + alpha_prev * d1;
    x2 = pol_prev ? px2 : ox2 + alpha_prev * d2;
    F(t, kFU + 0) = u0; F(t, kFU + 1) = u1;
    F(t, kFXn + 0) = x0; F(t, kFXn + 1) = x1; F(t, kFXn + 2) = x2;
  };

  // backward sweep. FAC: factor + predictor right-hand side. Otherwise linear-only with MODE.
  // xs_cur: the segment start state of the point the linear terms are evaluated at.
  auto backward = [&](auto fac_tag, auto mode_tag, double xb0, double xb1, double xb2, double& szs) {
    constexpr bool FAC = decltype(fac_tag)::value != 0;
    constexpr int MODE = decltype(mode_tag)::value;
    const bool usep = MODE == 3;
    // terminal: the top segment carries x_N's cost Q (x_N - r_{N-1}) (mpc.cpp:228)
    {
      double xN0 = F(m - 1, (usep ? kFXnp : kFXn) + 0), xN1 = F(m - 1, (usep ? kFXnp : kFXn) + 1);
      double xN2 = F(m - 1, (usep ? kFXnp : kFXn) + 2);
      if constexpr (FAC) step_x(m - 1, xN0, xN1, xN2);
      if constexpr (FAC) {
        P00 = top ? q0 : 0.0; P01 = 0.0; P02 = 0.0; P11 = top ? q1 : 0.0; P12 = 0.0; P22 = top ? q2 : 0.0;
        F00 = 1.0; F01 = 0.0; F02 = 0.0; F10 = 0.0; F11 = 1.0; F12 = 0.0; F20 = 0.0; F21 = 0.0; F22 = 1.0;
        G00 = G01 = G02 = G11 = G12 = G22 = 0.0;
      }
      p0 = top ? q0 * (xN0 - rNx) : 0.0;
      p1 = top ? q1 * (xN1 - rNy) : 0.0;
      p2 = top ? q2 * (xN2 - rNt) : 0.0;
      s0v = s1v = s2v = 0.0;
    }
    szs = 0.0;
#pragma unroll 1
    for (int t = m - 1; t >= 0; t--) {
      // the point: u_i, x_{i+1} (polish 2: the polish iterate), x_i for the Q-gradient. The factor
      // sweep first applies the previous iteration's step (step_stage: the update pass fused in)
      const int fu = usep ? kFUp : kFU, fx = usep ? kFXnp : kFXn;
      double u0, u1, xn0, xn1, xi0, xi1, xi2, sv[6], zv[6];
      if constexpr (FAC) {
        double xn2;
        step_stage(t, u0, u1, xn0, xn1, xn2, sv, zv);
        double y0, y1, y2;
        step_x(t > 0 ? t - 1 : 0, y0, y1, y2);  // clamped: loaded for every stage, then selected
        xi0 = t > 0 ? y0 : xb0; xi1 = t > 0 ? y1 : xb1; xi2 = t > 0 ? y2 : xb2;
      } else {
        u0 = F(t, fu); u1 = F(t, fu + 1);
        xn0 = F(t, fx); xn1 = F(t, fx + 1);
        const int tp = t > 0 ? t - 1 : 0;
        const double y0 = F(tp, fx), y1 = F(tp, fx + 1), y2 = F(tp, fx + 2);
        xi0 = t > 0 ? y0 : xb0; xi1 = t > 0 ? y1 : xb1; xi2 = t > 0 ? y2 : xb2;
#pragma unroll
        for (int j = 0; j < 6; j++) {
          sv[j] = F(t, kFS + j);
          zv[j] = F(t, kFZ + j);
        }
      }
      const double ri0 = r64[(3 * t + 0) * 64], ri1 = r64[(3 * t + 1) * 64], ri2 = r64[(3 * t + 2) * 64];
      double cc[6], e[6], sg[6];
      cvals(u0, u1, xn0, xn1, cc);
#pragma unroll
      for (int j = 0; j < 6; j++) {
        const double sj = sv[j], zj = zv[j];
        const double is = ipm_rcp1(sj);
        sg[j] = zj * is;
        if constexpr (MODE == 0) {
          e[j] = sg[j] * (cc[j] - sj);
          szs += sj * zj;
        } else if constexpr (MODE == 1) {
          e[j] = sg[j] * (cc[j] - sj) + (F(t, kFDsDz + j) - smu) * is;
        } else if constexpr (MODE == 2) {
          e[j] = zj > kn.act_sig * sj ? sg[j] * cc[j] - zj : 0.0;
        } else {
          e[j] = zj > kn.act_sig * sj ? 2.0 * sg[j] * cc[j] - zj : 0.0;
        }
      }
      // x_{i+1}'s gap rows: Hessian (FAC) and linear term
      if constexpr (FAC) {
        P00 += sg[4] * n0s * n0s + sg[5] * n1s * n1s;
        P01 += sg[4] * n0s * n0n + sg[5] * n1s * n1n;
        P11 += sg[4] * n0n * n0n + sg[5] * n1n * n1n;
      }
      p0 += n0s * e[4] + n1s * e[5];
      p1 += n0n * e[4] + n1n * e[5];
      const double gu0 = r0 * (u0 - ud0) + e[0] - e[1], gu1 = r1 * (u1 - ud1) + e[2] - e[3];
      const double gq0 = q0 * (xi0 - ri0), gq1 = q1 * (xi1 - ri1), gq2 = q2 * (xi2 - ri2);
      const double h0 = ROT ? gu0 + b00 * p0 + b20 * p2 : gu0 + b00 * p0 + b10 * p1 + b20 * p2;
      const double h1 = gu1 + b21 * p2;
      double K00, K01, K02, K10, K11, K12, I00, I01, I11;
      if constexpr (FAC) {
        const double pb0 = ROT ? P00 * b00 + P02 * b20 : P00 * b00 + P01 * b10 + P02 * b20;
        const double pb1 = ROT ? P01 * b00 + P12 * b20 : P01 * b00 + P11 * b10 + P12 * b20;
        const double pb2 = ROT ? P02 * b00 + P22 * b20 : P02 * b00 + P12 * b10 + P22 * b20;
        const double pc0 = P02 * b21, pc1 = P12 * b21, pc2 = P22 * b21;
        const double H00 = r0 + sg[0] + sg[1] + (ROT ? b00 * pb0 + b20 * pb2 : b00 * pb0 + b10 * pb1 + b20 * pb2);
        const double H01 = b21 * pb2;
        const double H11 = r1 + sg[2] + sg[3] + b21 * pc2;
        const double X00 = pb0, X01 = pb1;
        const double X02 = ROT ? pb2 + a12 * pb1 : pb2 + a02 * pb0 + a12 * pb1;
        const double X10 = pc0, X11 = pc1;
        const double X12 = ROT ? pc2 + a12 * pc1 : pc2 + a02 * pc0 + a12 * pc1;
        const double det = H00 * H11 - H01 * H01;
        const double idet = ipm_rcp(det);
        I00 = H11 * idet; I11 = H00 * idet; I01 = -H01 * idet;
        K00 = -(I00 * X00 + I01 * X10); K01 = -(I00 * X01 + I01 * X11); K02 = -(I00 * X02 + I01 * X12);
        K10 = -(I01 * X00 + I11 * X10); K11 = -(I01 * X01 + I11 * X11); K12 = -(I01 * X02 + I11 * X12);
        F(t, kFK + 0) = K00; F(t, kFK + 1) = K01; F(t, kFK + 2) = K02;
        F(t, kFK + 3) = K10; F(t, kFK + 4) = K11; F(t, kFK + 5) = K12;
        F(t, kFHi + 0) = I00; F(t, kFHi + 1) = I01; F(t, kFHi + 2) = I11;
        // P = Q + A'PA + X'K
        const double e0 = ROT ? P02 + a12 * P01 : P02 + a02 * P00 + a12 * P01;
        const double e1 = ROT ? P12 + a12 * P11 : P12 + a02 * P01 + a12 * P11;
        const double e2 = ROT ? P22 + a12 * P12 : P22 + a02 * P02 + a12 * P12;
        const double Y22 = ROT ? q2 + e2 + a12 * e1 : q2 + e2 + a02 * e0 + a12 * e1;
        // closed-loop map of the segment (Phi = Phi_{i+1} on entry): W = Phi B, Fl = -H^-1 W'
        const double W00 = ROT ? F00 * b00 + F02 * b20 : F00 * b00 + F01 * b10 + F02 * b20;
        const double W10 = ROT ? F10 * b00 + F12 * b20 : F10 * b00 + F11 * b10 + F12 * b20;
        const double W20 = ROT ? F20 * b00 + F22 * b20 : F20 * b00 + F21 * b10 + F22 * b20;
        const double W01 = F02 * b21, W11 = F12 * b21, W21 = F22 * b21;
        const double L00 = -(I00 * W00 + I01 * W01), L01 = -(I00 * W10 + I01 * W11);
        const double L02 = -(I00 * W20 + I01 * W21);
        const double L10 = -(I01 * W00 + I11 * W01), L11 = -(I01 * W10 + I11 * W11);
        const double L12 = -(I01 * W20 + I11 * W21);
        F(t, kFFl + 0) = L00; F(t, kFFl + 1) = L01; F(t, kFFl + 2) = L02;
        F(t, kFFl + 3) = L10; F(t, kFFl + 4) = L11; F(t, kFFl + 5) = L12;
        G00 += W00 * L00 + W01 * L10;
        G01 += W00 * L01 + W01 * L11;
        G02 += W00 * L02 + W01 * L12;
        G11 += W10 * L01 + W11 * L11;
        G12 += W10 * L02 + W11 * L12;
        G22 += W20 * L02 + W21 * L12;
        const double n02 = (ROT ? F02 + a12 * F01 : F02 + a02 * F00 + a12 * F01) + W00 * K02 + W01 * K12;
        const double n12 = (ROT ? F12 + a12 * F11 : F12 + a02 * F10 + a12 * F11) + W10 * K02 + W11 * K12;
        const double n22 = (ROT ? F22 + a12 * F21 : F22 + a02 * F20 + a12 * F21) + W20 * K02 + W21 * K12;
        F00 += W00 * K00 + W01 * K10; F01 += W00 * K01 + W01 * K11;
        F10 += W10 * K00 + W11 * K10; F11 += W10 * K01 + W11 * K11;
        F20 += W20 * K00 + W21 * K10; F21 += W20 * K01 + W21 * K11;
        F02 = n02; F12 = n12; F22 = n22;
        const double nP00 = q0 + P00 + X00 * K00 + X10 * K10;
        const double nP01 = P01 + X00 * K01 + X10 * K11;
        const double nP02 = e0 + X00 * K02 + X10 * K12;
        const double nP11 = q1 + P11 + X01 * K01 + X11 * K11;
        const double nP12 = e1 + X01 * K02 + X11 * K12;
        const double nP22 = Y22 + X02 * K02 + X12 * K12;
        P00 = nP00; P01 = nP01; P02 = nP02; P11 = nP11; P12 = nP12; P22 = nP22;
      } else {
        K00 = F(t, kFK + 0); K01 = F(t, kFK + 1); K02 = F(t, kFK + 2);
        K10 = F(t, kFK + 3); K11 = F(t, kFK + 4); K12 = F(t, kFK + 5);
        I00 = F(t, kFHi + 0); I01 = F(t, kFHi + 1); I11 = F(t, kFHi + 2);
      }
      const double k0 = -(I00 * h0 + I01 * h1), k1 = -(I01 * h0 + I11 * h1);
      F(t, kFk + 0) = k0; F(t, kFk + 1) = k1;
      // psi += W k = Fl' h
      s0v += F(t, kFFl + 0) * h0 + F(t, kFFl + 3) * h1;
      s1v += F(t, kFFl + 1) * h0 + F(t, kFFl + 4) * h1;
      s2v += F(t, kFFl + 2) * h0 + F(t, kFFl + 5) * h1;
      // p = gq + A'p + K'h
      const double np0 = gq0 + p0 + K00 * h0 + K10 * h1;
      const double np1 = gq1 + p1 + K01 * h0 + K11 * h1;
      const double np2 = gq2 + (ROT ? p2 + a12 * p1 : p2 + a02 * p0 + a12 * p1) + K02 * h0 + K12 * h1;
      p0 = np0; p1 = np1; p2 = np2;
    }
  };

  // forward sweep of a Newton direction from dx_s: du = K dx + k + Fl lam, dx' = A dx + B du.
  // fn(t, du0, du1, dxn0, dxn1, dxn2) sees every stage.
  auto forward = [&](double dx0, double dx1, double dx2, double lm0, double lm1, double lm2, auto fn) {
#pragma unroll 1
    for (int t = 0; t < m; t++) {
      const double du0 = F(t, kFK + 0) * dx0 + F(t, kFK + 1) * dx1 + F(t, kFK + 2) * dx2 + F(t, kFk + 0) +
                         F(t, kFFl + 0) * lm0 + F(t, kFFl + 1) * lm1 + F(t, kFFl + 2) * lm2;
      const double du1 = F(t, kFK + 3) * dx0 + F(t, kFK + 4) * dx1 + F(t, kFK + 5) * dx2 + F(t, kFk + 1) +
                         F(t, kFFl + 3) * lm0 + F(t, kFFl + 4) * lm1 + F(t, kFFl + 5) * lm2;
      const double n0 = ROT ? dx0 + b00 * du0 : dx0 + a02 * dx2 + b00 * du0;
      const double n1 = ROT ? dx1 + a12 * dx2 : dx1 + a12 * dx2 + b10 * du0;
      const double n2 = dx2 + b20 * du0 + b21 * du1;
      dx0 = n0; dx1 = n1; dx2 = n2;
      fn(t, du0, du1, dx0, dx1, dx2);
    }
  };

  const int max_it = kn.max_iter;
  for (int it = 0; it < max_it; it++) {
    if (__ballot(!done) == 0ull) break;
    // ---- 1. factor + predictor right-hand side ----
    double szs;
    backward(IpmTag<1>{}, IpmTag<0>{}, xs0, xs1, xs2, szs);
    const double mu = qsum(szs) / mrows;
    double lm0, lm1, lm2, dx0, dx1, dx2;
    seg_full(lm0, lm1, lm2, dx0, dx1, dx2);
    // ---- 2. predictor forward: step to the boundary and the affine complementarity ----
    double amin = 1.0, sa = 0.0, sb = 0.0;
    forward(dx0, dx1, dx2, lm0, lm1, lm2, [&](int t, double du0, double du1, double d0, double d1, double d2) {
      double cc[6];
      cvals(F(t, kFU), F(t, kFU + 1), F(t, kFXn), F(t, kFXn + 1), cc);
      const double dc[6] = {du0, -du0, du1, -du1, n0s * d0 + n0n * d1, n1s * d0 + n1n * d1};
#pragma unroll
      for (int j = 0; j < 6; j++) {
        const double sj = F(t, kFS + j), zj = F(t, kFZ + j);
        const double is = ipm_rcp1(sj);
        const double ds = dc[j] + cc[j] - sj;
        const double dz = -zj - zj * is * ds;
        const double rs = -sj * __builtin_amdgcn_rcp(ds), rz = -zj * __builtin_amdgcn_rcp(dz);
        amin = fmin(amin, fmin(ds < 0.0 ? rs : 1.0, dz < 0.0 ? rz : 1.0));
        sa += sj * dz + zj * ds;
        sb += ds * dz;
        F(t, kFDsDz + j) = ds * dz;
      }
    });
    const double aaff = qmin(amin);
    const double sza = qsum(sa), szb = qsum(sb);
    const double muaff = fmax((mu * mrows + aaff * sza + aaff * aaff * szb) / mrows, 0.0);
    const double rat = muaff / fmax(mu, 1e-300);
    const double sigma = fmin(rat * rat * rat, 1.0);
    smu = sigma * mu;

    // ---- 3. polish: the equality QP on the guessed active rows, on this factor ----
    const bool want_pol = !done && mu < kn.pol_mu && !kn.debug;
    bool pol_ok = false;
    double xp0 = xs0, xp1 = xs1, xp2 = xs2;
    if (__ballot(want_pol) != 0ull) {
      double dz_;
      backward(IpmTag<0>{}, IpmTag<2>{}, xs0, xs1, xs2, dz_);
      seg_vec(lm0, lm1, lm2, dx0, dx1, dx2);
      xp0 = xs0 + dx0; xp1 = xs1 + dx1; xp2 = xs2 + dx2;
      forward(dx0, dx1, dx2, lm0, lm1, lm2, [&](int t, double du0, double du1, double d0, double d1, double d2) {
        F(t, kFUp + 0) = F(t, kFU + 0) + du0;
        F(t, kFUp + 1) = F(t, kFU + 1) + du1;
        F(t, kFXnp + 0) = F(t, kFXn + 0) + d0;
        F(t, kFXnp + 1) = F(t, kFXn + 1) + d1;
        F(t, kFXnp + 2) = F(t, kFXn + 2) + d2;
      });
      backward(IpmTag<0>{}, IpmTag<3>{}, xp0, xp1, xp2, dz_);
      seg_vec(lm0, lm1, lm2, dx0, dx1, dx2);
      xp0 += dx0; xp1 += dx1; xp2 += dx2;
      bool ok = true;
      forward(dx0, dx1, dx2, lm0, lm1, lm2, [&](int t, double du0, double du1, double d0, double d1, double d2) {
        const double pu0 = F(t, kFUp + 0), pu1 = F(t, kFUp + 1);
        const double px0 = F(t, kFXnp + 0), px1 = F(t, kFXnp + 1), px2 = F(t, kFXnp + 2);
        double c1v[6], c2v[6];
        cvals(pu0, pu1, px0, px1, c1v);
        cvals(pu0 + du0, pu1 + du1, px0 + d0, px1 + d1, c2v);
        F(t, kFUp + 0) = pu0 + du0;
        F(t, kFUp + 1) = pu1 + du1;
        F(t, kFXnp + 0) = px0 + d0;
        F(t, kFXnp + 1) = px1 + d1;
        F(t, kFXnp + 2) = px2 + d2;
        const double scl[6] = {sc0, sc1, sc2, sc3, sc4, sc5};
        // the second augmented-Lagrangian step must have converged (stationarity of the point)
        // (bitwise: no EXEC-masked region per test)
        ok = ok & (fabs(du0) <= kn.tolp * (1.0 + fabs(pu0))) & (fabs(du1) <= kn.tolp * (1.0 + fabs(pu1))) &
             (fabs(d0) <= kn.tolp * (1.0 + fabs(px0))) & (fabs(d1) <= kn.tolp * (1.0 + fabs(px1))) &
             (fabs(d2) <= kn.tolp * (1.0 + fabs(px2)));
#pragma unroll
        for (int j = 0; j < 6; j++) {
          const double sj = F(t, kFS + j), zj = F(t, kFZ + j);
          const bool act = zj > kn.act_sig * sj;
          const double sgj = zj * ipm_rcp1(sj);
          const double y2 = zj - sgj * (c1v[j] + c2v[j]);
          const bool oka = (y2 >= -kn.told) & (fabs(c2v[j]) <= kn.tolp * scl[j]);
          const bool oki = c2v[j] >= -kn.tolp * scl[j];
          ok = ok & (act ? oka : oki);
        }
      });
      const bool qfail = (fold(__ballot(!ok)) >> sl) & 1ull;
      pol_ok = want_pol && !qfail;
    }

    // ---- 4. corrector: linear-only sweep on the same factor ----
    backward(IpmTag<0>{}, IpmTag<1>{}, xs0, xs1, xs2, szs);
    seg_vec(lm0, lm1, lm2, dx0, dx1, dx2);
    amin = 1.0;
    forward(dx0, dx1, dx2, lm0, lm1, lm2, [&](int t, double du0, double du1, double d0, double d1, double d2) {
      double cc[6];
      cvals(F(t, kFU), F(t, kFU + 1), F(t, kFXn), F(t, kFXn + 1), cc);
      const double dc[6] = {du0, -du0, du1, -du1, n0s * d0 + n0n * d1, n1s * d0 + n1n * d1};
#pragma unroll
      for (int j = 0; j < 6; j++) {
        const double sj = F(t, kFS + j), zj = F(t, kFZ + j);
        const double is = ipm_rcp1(sj);
        const double ds = dc[j] + cc[j] - sj;
        const double dz = -zj - (F(t, kFDsDz + j) - smu) * is - zj * is * ds;
        const double rs = -sj * __builtin_amdgcn_rcp(ds), rz = -zj * __builtin_amdgcn_rcp(dz);
        amin = fmin(amin, fmin(ds < 0.0 ? rs : 1.0, dz < 0.0 ? rz : 1.0));
      }
      F(t, kFDu + 0) = du0; F(t, kFDu + 1) = du1;
      F(t, kFDxn + 0) = d0; F(t, kFDxn + 1) = d1; F(t, kFDxn + 2) = d2;
    });
    const double alpha = (done || pol_ok) ? 0.0 : fmin(1.0, kn.tau * qmin(amin));
    // ---- 5. the step: applied by the next factor sweep (or the final pass below) ----
    alpha_prev = alpha;
    pol_prev = pol_ok;
    xs0 = pol_ok ? xp0 : xs0 + alpha * dx0;
    xs1 = pol_ok ? xp1 : xs1 + alpha * dx1;
    xs2 = pol_ok ? xp2 : xs2 + alpha * dx2;
    if (pol_ok) {
      done = true;
      iters = it + 1;
    }
  }

  // the pending step of the last iteration
#pragma unroll 1
  for (int t = 0; t < m; t++) {
    double u0, u1, x0, x1, x2, sv[6], zv[6];
    step_stage(t, u0, u1, x0, x1, x2, sv, zv);
  }

  const bool solved = (done && !bad && !handover0 && iters > 0) || (kn.debug && !bad);

  // ---- infeasibility certificate (Farkas) for the QPs the interior point did not polish ----
  // On an empty feasible set the multipliers of the gap rows grow without bound; y = z_gap /
  // max z_gap then nearly annihilates the reachable set. For ANY y >= 0 the bound
  //   max_{u in box} y'c_gap(x(u)) = y'c_gap(u_k) + sum_i sum_a [max(g_ia lb_a, g_ia ub_a) - g_ia u_ia],
  //   g_i = B' G_{i+1},  G_{i+1} = sum_k y_ik nu_k + A' G_{i+2}  (the costate of y'c_gap, dynamics
  //   model.cpp:42-51, rows mpc.cpp:249,271)
  // is exact (c_gap is affine in u); a negative value proves that no input in the box satisfies
  // every gap row: PRIMAL_INFEASIBLE, as OSQP reports it. Checked in fp64 on every QP still open.
  bool infeas = false;
  {
    const bool open_qp = !solved && !bad && !handover0;
    if (__ballot(open_qp) != 0ull) {
      double ym = 0.0;
      for (int t = 0; t < m; t++) ym = fmax(ym, fmax(F(t, kFZ + 4), F(t, kFZ + 5)));
#pragma unroll
      for (int k = L; k < 64; k <<= 1) ym = fmax(ym, __shfl_xor(ym, k, 64));
      const double iy = ym > 0.0 ? 1.0 / ym : 0.0;
      // the segment's own contribution to the costate at its start (incoming G = 0)
      double G0 = 0.0, G1 = 0.0, G2 = 0.0, val = 0.0;
      for (int t = m - 1; t >= 0; t--) {
        const double y0 = F(t, kFZ + 4) * iy, y1 = F(t, kFZ + 5) * iy;
        const double xn0 = F(t, kFXn), xn1 = F(t, kFXn + 1);
        val += y0 * (n0s * xn0 + n0n * xn1 - be0) + y1 * (n1s * xn0 + n1n * xn1 - be1);
        G0 += y0 * n0s + y1 * n1s;
        G1 += y0 * n0n + y1 * n1n;
        G2 = ROT ? G2 + a12 * G1 : G2 + a02 * G0 + a12 * G1;  // A' G
      }
      // incoming costate from the segments above: G_in(j) = (A')^m_{j+1} G_in(j+1) + local(j+1)
      double gi0 = 0.0, gi1 = 0.0, gi2 = 0.0;
      if constexpr (S > 1) {
        const double md = (double)m;
#pragma unroll 1
        for (int it2 = 0; it2 < S - 1; it2++) {
          const double o0 = gi0 + G0, o1 = gi1 + G1;
          const double o2 = gi2 + (ROT ? md * a12 * gi1 : md * (a02 * gi0 + a12 * gi1)) + G2;
          const double r0_ = __shfl(o0, up), r1_ = __shfl(o1, up), r2_ = __shfl(o2, up);
          gi0 = top ? 0.0 : r0_;
          gi1 = top ? 0.0 : r1_;
          gi2 = top ? 0.0 : r2_;
        }
      }
      // g_i = B' G_{i+1} with the incoming costate, and the box maximum of each input term
      double box = 0.0;
      {
        double c0_ = gi0, c1_ = gi1, c2_ = gi2;
        for (int t = m - 1; t >= 0; t--) {
          const double y0 = F(t, kFZ + 4) * iy, y1 = F(t, kFZ + 5) * iy;
          c0_ += y0 * n0s + y1 * n1s;
          c1_ += y0 * n0n + y1 * n1n;
          const double g0 = ROT ? b00 * c0_ + b20 * c2_ : b00 * c0_ + b10 * c1_ + b20 * c2_;
          const double g1 = b21 * c2_;
          const double u0 = F(t, kFU), u1 = F(t, kFU + 1);
          box += fmax(g0 * lb0, g0 * ub0) - g0 * u0 + fmax(g1 * lb1, g1 * ub1) - g1 * u1;
          c2_ = ROT ? c2_ + a12 * c1_ : c2_ + a02 * c0_ + a12 * c1_;
        }
      }
      const double cert = qsum(val + box);
      infeas = open_qp && ym > 0.0 && cert < -1e-9;
    }
  }

  // ---- outputs: the polished point (fp64) in the reference frame ----
  // hand-over: open QPs without a certificate go to the wave kernel's GI (normal mode); in the
  // re-check mode (the wave kernel's flagged QPs) only a polished or certified answer is written
  const bool hand = !bad && !solved && !infeas && !recheck;
  const bool wr = recheck ? (solved || infeas) : !hand;
  const float nanv = __int_as_float(0x7fc00000);
  float* uo = uout + (size_t)b * 2 * N;
  float* xo = xout + (size_t)b * 3 * (N + 1);
  if (qowner && wr) {
    xo[0] = solved ? fX0 : nanv;
    xo[1] = solved ? fY0 : nanv;
    xo[2] = solved ? fTH0 : nanv;
  }
  const bool want_obj = oo.obj || oo.cost;
  double J = 0.0, Cr = 0.0;
  auto qterm = [&](double rx, double ry, double rt, double e0, double e1, double e2) {
    const double d0 = e0 - rx, d1 = e1 - ry, d2 = e2 - rt;
    J += 0.5 * (q0 * d0 * d0 + q1 * d1 * d1 + q2 * d2 * d2);
    const double wx = (ROT ? cs * rx - sn * ry : rx) + X0, wy = (ROT ? sn * rx + cs * ry : ry) + Y0;
    const double wt = rt + th0;
    Cr += 0.5 * (q0 * wx * wx + q1 * wy * wy + q2 * wt * wt);
  };
  {
    double x0 = xs0, x1 = xs1, x2 = xs2;
    for (int t = 0; t < m; t++) {
      const int i = s0 + t;
      const double u0 = F(t, kFU), u1 = F(t, kFU + 1);
      if (want_obj) {
        qterm(r64[(3 * t) * 64], r64[(3 * t + 1) * 64], r64[(3 * t + 2) * 64], x0, x1, x2);
        J += 0.5 * (r0 * (u0 - ud0) * (u0 - ud0) + r1 * (u1 - ud1) * (u1 - ud1));
      }
      x0 = F(t, kFXn); x1 = F(t, kFXn + 1); x2 = F(t, kFXn + 2);
      if (owner && wr) {
        uo[2 * i] = solved ? (float)u0 : nanv;
        uo[2 * i + 1] = solved ? (float)u1 : nanv;
        const double ox = ROT ? cs * x0 - sn * x1 : x0, oy = ROT ? sn * x0 + cs * x1 : x1;
        xo[3 * i + 3] = solved ? (float)(ox + X0) : nanv;
        xo[3 * i + 4] = solved ? (float)(oy + Y0) : nanv;
        xo[3 * i + 5] = solved ? (float)(x2 + th0) : nanv;
      }
    }
    if (want_obj && top) qterm(rNx, rNy, rNt, x0, x1, x2);  // x_N against x_ref[N-1]
  }
  if (want_obj) {
    J = qsum(J);
    Cr = qsum(Cr);
    const double Cu = 0.5 * (double)N * (r0 * ud0 * ud0 + r1 * ud1 * ud1);
    const double dnan = __longlong_as_double(0x7ff8000000000000ll);
    if (qowner && wr && oo.cost) oo.cost[b] = solved ? J : dnan;
    if (qowner && wr && oo.obj) oo.obj[b] = solved ? J - Cr - Cu : dnan;
  }
  if (qowner) {
    if (hand) {
      const int idx = atomicAdd(hand_count, 1);
      hand_list[idx] = b;
    } else if (wr) {
      status_out[b] = bad ? F110QP_NUMERICAL_ID : (solved ? F110QP_SOLVED_ID : F110QP_PRIMAL_INFEASIBLE_ID);
      if (iters_out) iters_out[b] = bad ? 0 : (solved ? iters : kn.max_iter);
    }
  }
}

// The wave kernel's QPs with gap rows that it did not certify (SOLVED_INACCURATE, MAX_ITER) or
// declared infeasible / numerically broken: the list the interior point re-checks in fp64.
__global__ __launch_bounds__(256) void ipm_flag_kernel(const int B, const int* __restrict__ status,
                                                      int* __restrict__ count, int* __restrict__ list) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b < B) {
    const int s = status[b];
    if (s != F110QP_SOLVED_ID) list[atomicAdd(count, 1)] = b;
  }
}

template <int S, bool ROT>
hipError_t launch_lane_ipm_t(const KParams& P, int B, const float* x0, const float* ul, const float* xr,
                             const float* hs, float* uo, float* xo, int* st, int* its, int* list, int* count,
                             const IpmKnobs& kn, const ObjOut& oo, hipStream_t s, const int* qlist = nullptr,
                             const int* qcount = nullptr, int recheck = 0) {
  constexpr int L = 64 / S;
  const int waves = (B + L - 1) / L;
  const size_t lds = ipm_lds_bytes(P.N, S);
  auto kern = &lane_ipm_kernel<S, ROT>;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(kern, dim3(waves), dim3(64), lds, s, P, B, x0, ul, xr, hs, uo, xo, st, its, list,
                     count, kn, oo, qlist, qcount, recheck);
  return hipGetLastError();
}

}  // namespace f110qp

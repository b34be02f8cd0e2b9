// lane_seg_kernel.h — the lane back end for batches that leave lanes over: ONE QP PER S LANES,
// each lane owning one of S horizon segments (a partitioned, parallel-in-time Riccati).
//
// lane_kernel.h solves L <= 64 QPs per wave and, below 64 QPs per wave, runs 64 / L identical
// copies of each QP to keep EXEC full: a QP's time is its serial chain of N backward Riccati
// stages + N forward stages per PDAS pass (mpc.cpp:244-248 block-tridiagonal KKT walked
// strictly in sequence). Here the S = 64 / L lanes of a QP split the horizon into segments
// [s_j, e_j) of m = N / S stages and every pass runs:
//
// 1. backward, all segments at once: the masked Riccati step of lane_kernel.h over the lane's m
//    stages, with the terminal value V_e(x_e) = lam_j' x_e (lam_j: the multiplier of the coupling
//    x_e^(j) = x_s^(j+1), unknown yet; the last segment keeps the true terminal cost, mpc.cpp:228),
//    and alongside it the affine map of the segment's closed loop x_e = Phi x_s + psi + Gam lam_j:
//      W = Phi_{i+1} B,  F_i = -S_i^-1 W'  (the lam-gain of u_i, S_i^-1 the masked inverse),
//      psi_i = W k_i + Phi_{i+1} C + psi_{i+1},  Gam_i = Gam_{i+1} + W F_i,
//      Phi_i = Phi_{i+1} A + W K_i             (Phi_e = I, psi_e = 0, Gam_e = 0).
//    At the segment start V_s(x) = 1/2 x'P_s x + (a_s + Phi' lam_j)' x + const.
// 2. the segment ends: the coupling conditions x_s^(j+1) = Phi_j x_s^(j) + psi_j + Gam_j lam_j and
//    lam_{j-1} = P_j x_s^(j) + a_j + Phi_j' lam_j (x_s^(0) = 0) are an S-stage LQ two-point
//    boundary problem, solved by a Riccati recursion over the segments, lam_{j-1} = M_j x + m_j:
//      T_j = (I - M_{j+1} Gam_j)^-1 M_{j+1} Phi_j,  t_j = (I - M_{j+1} Gam_j)^-1 (M_{j+1} psi_j + m_{j+1}),
//      M_j = P_j + Phi_j' T_j,  m_j = a_j + Phi_j' t_j,   then lam_j = T_j x_s^(j) + t_j forward.
//    (I - M Gam has eigenvalues >= 1: M is positive definite, Gam negative semidefinite.) Every
//    lane runs every step on its own data with its neighbour's (M, m) / x_e from a lane shuffle;
//    the top segment's (Phi, psi, Gam) are zeroed so that its lane reproduces (P, a) and hands
//    x_e = 0 to segment 0 round the ring: S - 1 identical steps each way, no selects.
// 3. refresh, all segments: the lam-part of the feed-forward, p^lam_e = lam_j,
//    k_i += -S_i^-1 B' p^lam_{i+1},  p^lam_i = A' p^lam_{i+1} + K_i' B' p^lam_{i+1}
//    (the p-recursion of the Riccati step restricted to its lam-dependent part).
// 4. forward, all segments: lane_kernel.h's sweep from x_s^(j) with the costate
//    P_s x_s + a_s + p^lam_s: rollout, costate carried forward, PDAS re-guess per stage.
// A pass's result equals the sequential pass's up to rounding (tests/diag_segment_riccati_model.py:
// 1.8e-15 relative on random masks), so the PDAS iterates, the single-flip rule (the first
// violation over the whole horizon: a min over the QP's lanes) and the stopping test are
// lane_kernel.h's. Per pass the chain is m stages of ~(200 + 120 + 30) instructions plus
// 2 (S - 1) segment steps instead of N stages of ~255.
//
// Layout (fp64 throughout): lane l = S slot + j works on QP L w + slot, segment j (a QP's segments
// are adjacent lanes: its segment-end exchanges stay inside a quad at S <= 4). LDS per wave,
// lane-major so that every access is one conflict-free 64-lane row: references [3m][64] (recentred,
// rotated), PDAS state [m][64] int, Riccati scratch [m][11][64] (K 6, k 2, S^-1 3); the float
// staging of the references borrows the scratch region.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "f110qp_kernels.h"

namespace f110qp {

// Diagnostic build only (-DF110QP_STAMPS on lane_seg_inst.hip): per-wave cycles of the setup, each
// pass phase and the output, read back with f110qp_read_seg_stamps(). Never in the shipped library.
#ifdef F110QP_STAMPS
constexpr int kSegStampSlots = 16;
__device__ unsigned long long g_sstamps[4096 * kSegStampSlots];
#define SSTAMP(var) const unsigned long long var = __builtin_amdgcn_s_memtime()
#define SACC(acc, since) acc += __builtin_amdgcn_s_memtime() - (since)
#else
#define SSTAMP(var)
#define SACC(acc, since)
#endif

// LDS bytes per wave of the segmented kernel for horizon N split into S segments (rows for the
// longest segment, ceil(N / S) stages)
// FST: the scratch keeps the lam-gains F_i (6) instead of S_i^-1 (3): 14 doubles per stage
// F32: references and Riccati scratch held as float (the fp64 arithmetic is unchanged): 60 instead
// of 116 bytes per stage and lane, so 16,384 x N = 40 QPs per GPU fit at S = 4 (DESIGN.md 2b')
// + the per-wave tables of the active-state codes (kSegTabBytes: the backward sweep's bound values
// and free masks, the fp64-scratch forward sweep's re-guess thresholds, 16 codes x 8 doubles each)
constexpr size_t kSegTabBytes = 16 * 8 * 8;
constexpr size_t seg_lds_bytes(int N, int S, bool fst = false, bool f32 = false) {
  return (size_t)((N + S - 1) / S) * 64 * (3 * (f32 ? 4 : 8) + 4 + (fst ? 14 : 11) * (f32 ? 4 : 8)) +
         (f32 ? 1 : 2) * kSegTabBytes;
}

template <int M>
struct SegMode {
  static constexpr int value = M;
};

// Lane-adjacent segments (lane = S slot + segment): the segment ring of a QP is S consecutive lanes,
// so the segment-end exchanges are DPP moves (VALU) instead of ds_bpermute round trips through the
// LDS crossbar: quad permutes at S <= 4, at S = 8 two row shifts and a select (an 8-lane group is
// half a DPP row). A lane only ever reads lanes of its own QP.
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, true);  // (an invalid source lane reads 0)
}
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = (unsigned)dpp_i<CTRL>((int)(unsigned)b);
  const unsigned hi = (unsigned)dpp_i<CTRL>((int)(unsigned)(b >> 32));
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
// the value of segment + 1 (seg_up) / segment - 1 (seg_dn) of the lane's QP, round the QP's ring
template <int S>
__device__ __forceinline__ double seg_up(double v, int lane) {
  static_assert(S == 2 || S == 4 || S == 8, "segments per QP: 2, 4 or 8");
  if constexpr (S == 2) return dpp_d<0xB1>(v);       // quad_perm [1, 0, 3, 2]
  else if constexpr (S == 4) return dpp_d<0x39>(v);  // quad_perm [1, 2, 3, 0]
  else {  // row_shl:1; the top segment's lane takes 0 instead of the ring's wrap: its own
          // (Phi, psi, Gam) are zero in the segment-end recursion, so what it receives only
          // matters as a non-finite value (a neighbouring QP's lane), and 0 is what it computes
          // with anyway (one DPP move and a select per dword instead of two moves and a select)
    const double b = dpp_d<0x101>(v);
    return (lane & 7) == 7 ? 0.0 : b;
  }
}
template <int S>
__device__ __forceinline__ double seg_dn(double v, int lane) {
  if constexpr (S == 2) return dpp_d<0xB1>(v);
  else if constexpr (S == 4) return dpp_d<0x93>(v);  // quad_perm [3, 0, 1, 2]
  else {  // row_shr:1; segment 0 takes 0: the ring hands it the top segment's x_e, which is 0
    const double b = dpp_d<0x111>(v);
    return (lane & 7) == 0 ? 0.0 : b;
  }
}

#ifndef F110QP_SEG_NEWTON
#define F110QP_SEG_NEWTON 2  // Newton steps after v_rcp_f64 in the masked 2x2 inverse (knob; 1
                             // measured no change: C5 30.2, C2 27.3, C4 shard 63.7 us)
#endif
// unroll factor of the backward stage loop: 2 lets a stage's closed-loop map (Phi, psi, Gam)
// overlap the next stage's Riccati step; same-box A/B C5 30.2 -> 29.6 us, C2 27.4 -> 26.9 at
// S = 4, C4 shard (S = 8, m = 5) 63.6 -> 64.1, so S = 8 keeps 1 (knob F110QP_SEG_BW_UNROLL)
#ifndef F110QP_SEG_BW_UNROLL
#define F110QP_SEG_BW_UNROLL (S <= 4 ? 2 : 1)
#endif
#ifndef F110QP_SEG_WPE
// waves-per-EU hint: 2 (<= 256 VGPRs; the grid still runs one wave per SIMD or CU) schedules
// better than 1: same-box A/B C5 31.2 -> 30.6 us, C2 on the lane back end 28.3 -> 27.7, C4 shard
// neutral (tools/ab_seg_variant.sh)
#define F110QP_SEG_WPE 2
#endif
template <int S, bool ROT, bool FST, typename ST = double, bool SCR = false, bool TWIN = false, bool EVEN = false>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(F110QP_SEG_WPE, F110QP_SEG_WPE))) void lane_seg_kernel(
    const KParams P, const int B, const float* __restrict__ x0g, const float* __restrict__ ulg,
    const float* __restrict__ xrg, float* __restrict__ uout, float* __restrict__ xout,
    int* __restrict__ status_out, int* __restrict__ iters_out, const WarmState ws, const int kmax,
    const ObjOut oo) {
  constexpr int twin = TWIN ? 1 : 0;
  constexpr int L = 64 / S;  // QPs per wave
  // the kernel arguments the staging address needs, in SGPRs before anything else: hipcc loads
  // kernel arguments next to their first use, which put two dependent kernarg round trips in
  // front of the staging loads
  constexpr int NV = FST ? 14 : 11;  // scratch doubles per stage: K 6, k 2, then F 6 or S^-1 3
  extern __shared__ __attribute__((aligned(16))) double seg_smem[];
  const int lane = threadIdx.x;
  const int sl = lane / S;         // QP slot of the wave
  const int seg = lane & (S - 1);  // segment: the QP's S segments are S consecutive lanes
  // twin = 1: every QP is solved from two PDAS starts at once, adjacent slots 2b (cold) and 2b + 1
  // (the speed bound nearest u_des active on the first half of the horizon); the QP is done when
  // either start has converged, and the converged one (the cold one on a tie) writes the outputs.
  // Both end at the same exact optimum; the pass count is the smaller one (launch_lane_seg_t)
  const int b0 = blockIdx.x * L;                 // first (virtual) QP of the wave
  const int VB = B << twin;
  const int nq = (VB - b0) < L ? (VB - b0) : L;
  // a missing QP's lanes duplicate QP 0 of the wave (twin: the start of the same parity, so that a
  // duplicate's sibling lane is a duplicate of its sibling start)
  const int slot = sl < nq ? sl : (sl & twin);
  const bool owner0 = sl < nq;         // stores the outputs of its segment's stages ...
  const bool qowner0 = owner0 && seg == 0;
  const int vq = b0 + slot;
  const bool var = (vq & twin) != 0;   // ... if its start is the one that converged (owner below)
  const int b = vq >> twin;
  const int N = P.N;
  // segments of q or q + 1 stages (the first N mod S ones longer); LDS rows for the longest
  // EVEN (S divides N, the launcher's choice): every segment has q stages, so the stage loops run
  // on a wave-uniform count (scalar loop control and LDS strides instead of per-lane ones)
  const int q = N / S, rem = EVEN ? 0 : N - q * S;
  const int m = EVEN ? q : q + (seg < rem ? 1 : 0);
  const int s0 = EVEN ? seg * q : seg * q + (seg < rem ? seg : rem);
  const int mM = EVEN ? q : q + (rem > 0 ? 1 : 0);
  const bool top = seg == S - 1;

  SSTAMP(t_start);
#ifdef F110QP_STAMPS
  unsigned long long acc_bw = 0, acc_dual = 0, acc_ref = 0, acc_fw = 0, t_setup = 0, npass = 0;
  unsigned long long t_out_loop = 0;  // the output sweep's stage loop
#endif
  constexpr bool F32 = sizeof(ST) == 4;
  char* const lbase = reinterpret_cast<char*>(seg_smem);
  const size_t o_ap = (size_t)3 * mM * 64 * sizeof(ST), o_sc = o_ap + (size_t)mM * 64 * 4;
  ST* const r64 = reinterpret_cast<ST*>(lbase) + lane;                     // [3mM][64]
  int* const ap = reinterpret_cast<int*>(lbase + o_ap) + lane;             // [mM][64]
  ST* const sc = reinterpret_cast<ST*>(lbase + o_sc) + lane;               // [mM][NV][64]
  // code tables (wave-uniform base; a lane reads the entry of its own stage's state code)
  double* const btab = reinterpret_cast<double*>(lbase + o_sc + (size_t)mM * NV * 64 * sizeof(ST));
  double* const ftab = btab + 16 * 8;  // (ST = double only)

  // per-QP inputs and the warm-start traffic switch (warm_traffic), issued before the staging loads
  const float fX0 = x0g[3 * b + 0], fY0 = x0g[3 * b + 1], fTH0 = x0g[3 * b + 2];
  const float fv = ulg[2 * b + 0], fd = ulg[2 * b + 1];
  const unsigned wlast = warm_last_hit(ws);
  // ---- stage the wave's reference paths (float, [3N][L]) into the scratch region ----
  // Element e = q 3N + c of the wave's nq rows (row stride 3 xr_stride in HBM) goes to
  // stg[c L + q]. (q, c) advance by 64 elements per step without a division, every load reads a
  // valid address (clamped) and every store lands (past the staged rows for e >= tot), so the
  // loop has no EXEC-masked region: ~11 instructions per element instead of ~50 (ISA).
  // (Issuing chunk 0 first and the linearisation under its loads measured no gain: C2 23.4 against
  // 23.1 us, C5 30.9 against 30.4, same box.) Twin starts: row q of the wave is QP (b0 >> 1) + q.
  // Twin starts: the two starts of a QP share its row, staged once ([3N][L / 2] QP rows)
  constexpr int LR = L >> twin;
  {
    float* stg = reinterpret_cast<float*>(lbase + o_sc);
    const int nqr = (nq + twin) >> twin;  // QP rows of the wave (b0 is even with twin starts)
    const int n3 = 3 * N, S3 = 3 * P.xr_stride, tot = nqr * n3;
    const int rb0 = b0 >> twin;
    const float* src = xrg + (size_t)rb0 * S3;
    const int dq = 64 / n3, dc = 64 - dq * n3;
    int q = lane / n3, c = lane - (lane / n3) * n3;
    const int junk = n3 * LR + lane;                 // inside the scratch rows, never read
    const int last_off = (nqr - 1) * S3 + (n3 - 1);  // a valid element
    // C5 and the C4 shard stage 960 floats per wave, the twin kernels 480: one round trip
    constexpr int kChunk = TWIN ? 8 : 16;
    for (int e0 = 0; e0 < tot; e0 += kChunk * 64) {
      float vbuf[kChunk];
      int dst[kChunk];
#pragma unroll
      for (int j = 0; j < kChunk; j++) {
        const bool in = e0 + j * 64 + lane < tot;
        dst[j] = in ? c * LR + q : junk;
        vbuf[j] = src[in ? q * S3 + c : last_off];
        q += dq;
        c += dc;
        const bool wrap = c >= n3;
        c -= wrap ? n3 : 0;
        q += wrap ? 1 : 0;
      }
#pragma unroll
      for (int j = 0; j < kChunk; j++) stg[dst[j]] = vbuf[j];
    }
    __syncthreads();
  }
  // the warm-start key, when this call moves warm traffic (its round trip overlaps the staging)
  const bool wt = warm_traffic(ws, wlast);
  unsigned key0 = 0u, key1 = 0u, key2 = 0u, key3 = 0u;
  uint2 wst = make_uint2(0u, 0u);  // this wave's warm counters (f110qp_warm_hits), updated at the end
  if (wt) {
    if (ws.stats) wst = *reinterpret_cast<const uint2*>(ws.stats + 2 * (size_t)blockIdx.x);
    const uint4 k4 = *reinterpret_cast<const uint4*>(ws.key + 4 * (size_t)b);
    key0 = k4.x; key1 = k4.y; key2 = k4.z; key3 = k4.w;
  }

  SSTAMP(t_stg);
  // ---- per-lane QP data (Model::Linearize, model.cpp:30-59), as lane_kernel.h ----
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
  // PDAS flip tolerances of lane_kernel.h: fp64 scratch 1e-10 (scaled) in every pass; fp32
  // scratch (gains rounded to ~1e-7) exact compares in the PDAS passes and 1e-6 / 1e-5 in the
  // single-flip passes, where a degenerate bound then settles
  const double ptT = F32 ? 0.0 : 1e-10, gtT = F32 ? 0.0 : 1e-10;
  const double ptL = F32 ? 1e-6 : 1e-10, gtL = F32 ? 1e-5 : 1e-10;
  const double lbe0 = lb0 - ptT * (1.0 + fabs(lb0)), ube0 = ub0 + ptT * (1.0 + fabs(ub0));
  const double lbe1 = lb1 - ptT * (1.0 + fabs(lb1)), ube1 = ub1 + ptT * (1.0 + fabs(ub1));
  const double gtol0 = gtT * (1.0 + r0 * (1.0 + fabs(lb0) + fabs(ub0)));
  const double gtol1 = gtT * (1.0 + r1 * (1.0 + fabs(lb1) + fabs(ub1)));
  const double lbl0 = lb0 - ptL * (1.0 + fabs(lb0)), ubl0 = ub0 + ptL * (1.0 + fabs(ub0));
  const double lbl1 = lb1 - ptL * (1.0 + fabs(lb1)), ubl1 = ub1 + ptL * (1.0 + fabs(ub1));
  const double gtoll0 = gtL * (1.0 + r0 * (1.0 + fabs(lb0) + fabs(ub0)));
  const double gtoll1 = gtL * (1.0 + r1 * (1.0 + fabs(lb1) + fabs(ub1)));

  SSTAMP(t_lin);
  // references of the lane's stages: recentred (ROT: rotated) fp64, lane-major; a non-finite
  // entry flags the QP (one ballot folded over its segment lanes)
  // (the loop runs to the wave-uniform mM: a lane of a shorter segment converts one stage of the
  // next segment, or of the staging's junk rows on the top segment, into a row it never reads, so
  // the loop has no EXEC-masked exits; its flag only counts stages < m)
  bool nonfin = false;
  {
    const float* stg = reinterpret_cast<const float*>(lbase + o_sc);
    const int row = slot >> twin;
    for (int t = 0; t < mM; t++) {
      const int i = s0 + t;
      const float fx = stg[(3 * i + 0) * LR + row], fy = stg[(3 * i + 1) * LR + row];
      const float ft = stg[(3 * i + 2) * LR + row];
      nonfin |= (t < m) & !(isfinite(fx) && isfinite(fy) && isfinite(ft));
      const double dx = (double)fx - X0, dy = (double)fy - Y0;
      r64[(3 * t + 0) * 64] = ROT ? cs * dx + sn * dy : dx;
      r64[(3 * t + 1) * 64] = ROT ? cs * dy - sn * dx : dy;
      r64[(3 * t + 2) * 64] = (double)ft - th0;
    }
    // the active-state code tables: code c holds input a's state (c >> 2a) & 3 (0 free, 1 lower,
    // 2 upper). btab[c] = (bA0, bA1, fm0, fm1, 1 - fm0, 1 - fm1, fm0 fm1, 0): the fixed inputs'
    // bound values and the free masks of the masked 2 x 2 solve (products with 0 / 1 instead of
    // ~20 selects per backward stage; the first four are read a stage ahead). ftab[c] = per input
    // the forward sweep's re-guess thresholds and masks (fp64 scratch: one set of tolerances for
    // both pass kinds)
    if (lane < 16) {
      const int cA = lane & 3, cB = (lane >> 2) & 3;
      const double fA = cA == 0 ? 1.0 : 0.0, fB = cB == 0 ? 1.0 : 0.0;
      double* e = btab + 8 * lane;
      e[0] = cA == 0 ? 0.0 : (cA == 1 ? lb0 : ub0);
      e[1] = cB == 0 ? 0.0 : (cB == 1 ? lb1 : ub1);
      e[2] = fA; e[3] = fB; e[4] = 1.0 - fA; e[5] = 1.0 - fB; e[6] = fA * fB; e[7] = 0.0;
      if constexpr (!F32) {
        // per input (lo, hi, fm, 1 - fm): the re-guess tests y = fm u - (1 - fm) g against
        // y < lo (lower) and y > hi (upper); free: y = u in (lbe, ube); at the lower bound: y = -g,
        // stays while -g < gtol; at the upper: y = -g, stays while -g > -gtol
        const double inf = __builtin_inf();
        double* f = ftab + 8 * lane;
        f[0] = cA == 0 ? lbe0 : (cA == 1 ? gtol0 : -inf); f[1] = cA == 0 ? ube0 : (cA == 2 ? -gtol0 : inf);
        f[2] = fA; f[3] = 1.0 - fA;
        f[4] = cB == 0 ? lbe1 : (cB == 1 ? gtol1 : -inf); f[5] = cB == 0 ? ube1 : (cB == 2 ? -gtol1 : inf);
        f[6] = fB; f[7] = 1.0 - fB;
      }
    }
    __syncthreads();  // the staging region becomes the Riccati scratch
  }
  SSTAMP(t_conv);
  // terminal reference x_ref[N-1] (mpc.cpp:228): the last stage of the top segment
  const double rNx = __shfl(r64[(3 * (m - 1) + 0) * 64], lane | (S - 1));
  const double rNy = __shfl(r64[(3 * (m - 1) + 1) * 64], lane | (S - 1));
  const double rNt = __shfl(r64[(3 * (m - 1) + 2) * 64], lane | (S - 1));
  SSTAMP(t_rn);

  // warm start: previous tick's active bounds when the slot's (theta0, v, steer) bits repeat
  const int R = (2 * N + 63) / 64;
  const unsigned kth = __float_as_uint(fTH0), kv = __float_as_uint(fv), kd = __float_as_uint(fd);
  {
#ifdef F110QP_SEG_SEED_ANY  // measurement knob: seed from the slot's previous set on any key
                            // (measured C5 31.2 -> 34.9 us: the stale set costs passes)
    const bool hit = wt && key3 != 0u;
#else
    const bool hit = wt && key3 != 0u && key0 == kth && key1 == kv && key2 == kd;
#endif
    unsigned long long lw = 0, hw = 0;
    if (wt) {  // (wave-uniform: a call that moves no warm state skips the mask window)
      if (ws.hit_call && __ballot(hit) != 0ull && lane == 0) *ws.hit_call = ws.call;
      wst.x += (unsigned)__popcll(__ballot(hit && qowner0 && !var));  // hits (one lane per QP)
      unsigned long long lo0 = 0, lo1 = 0, hi0 = 0, hi1 = 0;
      if (hit) {
        lo0 = ws.act[2 * R * b];
        hi0 = ws.act[2 * R * b + 1];
        if (R > 1) {
          lo1 = ws.act[2 * (R * b + 1)];
          hi1 = ws.act[2 * (R * b + 1) + 1];
        }
      }
      // the lane's 2m mask bits start at bit 2 s0 of the 128-bit pair (hi word : lo word)
      const int sh = 2 * s0;
      auto window = [&](unsigned long long w0, unsigned long long w1) {
        return sh >= 64 ? (w1 >> (sh - 64)) : (sh == 0 ? w0 : ((w0 >> sh) | (w1 << (64 - sh))));
      };
      lw = window(lo0, lo1);
      hw = window(hi0, hi1);
    }
    // the twin start: the speed bound u_des sits on, active on the first half of the horizon (on
    // the C2 / C5 workloads the optimum holds the speed on its upper bound over a prefix of the
    // horizon that cold PDAS finds a few stages per pass: numpy model of the kernel's PDAS, the
    // slowest QP's passes 4-5 -> 3-4 over eight C2 batches and six C5 ticks; launch_lane_seg_t
    // enables it only when u_des is on a speed bound)
    const int sv = ud0 >= ub0 ? 2 : (ud0 <= lb0 ? 1 : 0);
    const bool tw = var && !hit;
    // per input: 1 lower, 2 upper, 0 free; the lower bound wins. To the wave-uniform mM (rows
    // t >= m of a shorter segment are never read): no EXEC-masked loop exits
    for (int t = 0; t < mM; t++) {
      const unsigned l2 = (unsigned)(lw >> (2 * t)) & 3u, h2 = (unsigned)(hw >> (2 * t)) & 3u & ~l2;
      const int a = (int)((l2 & 1u) | ((h2 & 1u) << 1) | ((l2 & 2u) << 1) | ((h2 & 2u) << 2));
      ap[t * 64] = (tw && 2 * (s0 + t) < N) ? sv : a;
    }
  }
  SSTAMP(t_mask);

  // whether any of the lane's QP's S lanes has its bit set in a ballot
  auto qany = [&](unsigned long long mk) { return ((mk >> (sl * S)) & ((1ull << S) - 1ull)) != 0ull; };
  const bool bad = !(isfinite(X0) && isfinite(Y0) && isfinite(th0) && isfinite(v) && isfinite(d)) ||
                   qany(__ballot(nonfin));
  bool done = bad;
  int iters = 0;
  // the segment's start state and terminal multiplier lam_j of the current pass (kept for the
  // output sweep)
  double xs0 = 0.0, xs1 = 0.0, xs2 = 0.0, lm0 = 0.0, lm1 = 0.0, lm2 = 0.0;


  const int max_pass = P.pass_cap > 0 ? P.pass_cap : (P.max_iter > kmax ? P.max_iter : kmax);
#ifdef F110QP_STAMPS
  t_setup = __builtin_amdgcn_s_memtime() - t_start;
#endif
  for (int pass = 0; pass < max_pass; pass++) {
    // a QP is finished when one of its starts is (twin: the sibling start is S lanes over). The
    // shuffle runs on every lane: under a short-circuit || the done lanes are off in EXEC, and a
    // permute reads nothing from an inactive source lane
    if constexpr (TWIN) {
      const int sib = __shfl_xor((int)done, S, 64);
      if (__ballot(!(done || sib != 0)) == 0ull) break;
    } else {
      if (__ballot(!done) == 0ull) break;
    }
    const bool single = pass >= kmax;
#ifdef F110QP_STAMPS
    npass++;
#endif
    SSTAMP(t_bw);
    // ---- 1. backward over the segment: Riccati + the closed-loop map (Phi, psi, Gam) ----
    double P00 = top ? q0 : 0.0, P01 = 0.0, P02 = 0.0, P11 = top ? q1 : 0.0, P12 = 0.0;
    double P22 = top ? q2 : 0.0;
    double p0 = top ? -q0 * rNx : 0.0, p1 = top ? -q1 * rNy : 0.0, p2 = top ? -q2 * rNt : 0.0;
    double F00 = 1.0, F01 = 0.0, F02 = 0.0, F10 = 0.0, F11 = 1.0, F12 = 0.0, F20 = 0.0, F21 = 0.0;
    double F22 = 1.0;  // Phi
    double s0v = 0.0, s1v = 0.0, s2v = 0.0;  // psi
    double G00 = 0.0, G01 = 0.0, G02 = 0.0, G11 = 0.0, G12 = 0.0, G22 = 0.0;  // Gam (symmetric)
    {
      int nst = ap[(m - 1) * 64];
      // the next stage's code-table entry (bA0, bA1, fm0, fm1), read one stage ahead: the masked
      // solve needs it right after H, which the previous stage's P already gives
      double nb0 = btab[8 * nst], nb1 = btab[8 * nst + 1], nf0 = btab[8 * nst + 2], nf1 = btab[8 * nst + 3];
      double rx = r64[(3 * (m - 1) + 0) * 64], ry = r64[(3 * (m - 1) + 1) * 64];
      double rt = r64[(3 * (m - 1) + 2) * 64];
      constexpr int kBwUnroll = F110QP_SEG_BW_UNROLL;
#pragma unroll kBwUnroll
      for (int t = m - 1; t >= 0; t--) {
        ST* s = sc + t * NV * 64;
        const double bA0 = nb0, bA1 = nb1, fm0 = nf0, fm1 = nf1;
        const int tn = t > 0 ? t - 1 : 0;
        nst = ap[tn * 64];
        const double rxi = rx, ryi = ry, rti = rt;
        rx = r64[(3 * tn + 0) * 64];
        ry = r64[(3 * tn + 1) * 64];
        rt = r64[(3 * tn + 2) * 64];
        const double g0 = ROT ? P02 * c2 + p0 : P00 * c0 + P01 * c1 + P02 * c2 + p0;
        const double g1 = ROT ? P12 * c2 + p1 : P01 * c0 + P11 * c1 + P12 * c2 + p1;
        const double g2 = ROT ? P22 * c2 + p2 : P02 * c0 + P12 * c1 + P22 * c2 + p2;
        const double pb0 = ROT ? P00 * b00 + P02 * b20 : P00 * b00 + P01 * b10 + P02 * b20;
        const double pb1 = ROT ? P01 * b00 + P12 * b20 : P01 * b00 + P11 * b10 + P12 * b20;
        const double pb2 = ROT ? P02 * b00 + P22 * b20 : P02 * b00 + P12 * b10 + P22 * b20;
        const double pc0 = P02 * b21, pc1 = P12 * b21, pc2 = P22 * b21;
        const double H00 = ROT ? r0 + b00 * pb0 + b20 * pb2 : r0 + b00 * pb0 + b10 * pb1 + b20 * pb2;
        const double H01 = b21 * pb2;
        const double H11 = r1 + b21 * pc2;
        const double X00 = pb0, X01 = pb1;
        const double X02 = ROT ? pb2 + a12 * pb1 : pb2 + a02 * pb0 + a12 * pb1;
        const double X10 = pc0, X11 = pc1;
        const double X12 = ROT ? pc2 + a12 * pc1 : pc2 + a02 * pc0 + a12 * pc1;
        const double h0 = ROT ? -r0 * ud0 + b00 * g0 + b20 * g2
                              : -r0 * ud0 + b00 * g0 + b10 * g1 + b20 * g2;
        const double h1 = -r1 * ud1 + b21 * g2;
        const double e0 = ROT ? P02 + a12 * P01 : P02 + a02 * P00 + a12 * P01;
        const double e1 = ROT ? P12 + a12 * P11 : P12 + a02 * P01 + a12 * P11;
        const double e2 = ROT ? P22 + a12 * P12 : P22 + a02 * P02 + a12 * P12;
        const double Y00 = q0 + P00, Y01 = P01, Y11 = q1 + P11, Y02 = e0, Y12 = e1;
        const double Y22 = ROT ? q2 + e2 + a12 * e1 : q2 + e2 + a02 * e0 + a12 * e1;
        const double hx0 = -q0 * rxi + g0, hx1 = -q1 * ryi + g1;
        const double hx2 = ROT ? -q2 * rti + g2 + a12 * g1 : -q2 * rti + g2 + a02 * g0 + a12 * g1;
        // the stage's masked 2 x 2 solve from its code's table entry: M = the free block of H with
        // ones on the fixed diagonal, S^-1 rows of the fixed inputs zero (exact: products with 0 / 1)
        {
          const double* tb = btab + 8 * nst;
          nb0 = tb[0]; nb1 = tb[1]; nf0 = tb[2]; nf1 = tb[3];
        }
        const double om0 = 1.0 - fm0, om1 = 1.0 - fm1, fm01 = fm0 * fm1;
        const double M00 = fm0 * H00 + om0, M11 = fm1 * H11 + om1, M01 = fm01 * H01;
        const double det = M00 * M11 - M01 * M01;
        double idet = __builtin_amdgcn_rcp(det);
#pragma unroll
        for (int nt = 0; nt < F110QP_SEG_NEWTON; nt++) idet = fma(idet, fma(-det, idet, 1.0), idet);
        const double I00 = fm0 * (M11 * idet), I11 = fm1 * (M00 * idet);
        const double I01 = -M01 * idet;
        const double K00 = -I00 * X00 - I01 * X10, K01 = -I00 * X01 - I01 * X11;
        const double K02 = -I00 * X02 - I01 * X12;
        const double K10 = -I01 * X00 - I11 * X10, K11 = -I01 * X01 - I11 * X11;
        const double K12 = -I01 * X02 - I11 * X12;
        const double w0 = h0 + H00 * bA0 + H01 * bA1, w1 = h1 + H01 * bA0 + H11 * bA1;
        const double k0 = bA0 - (I00 * w0 + I01 * w1), k1 = bA1 - (I01 * w0 + I11 * w1);
        s[0] = K00; s[64] = K01; s[2 * 64] = K02; s[3 * 64] = K10; s[4 * 64] = K11;
        s[5 * 64] = K12; s[6 * 64] = k0; s[7 * 64] = k1;
        if constexpr (!FST) {
          s[8 * 64] = I00; s[9 * 64] = I01; s[10 * 64] = I11;
        }
        P00 = Y00 + X00 * K00 + X10 * K10;
        P01 = Y01 + X00 * K01 + X10 * K11;
        P02 = Y02 + X00 * K02 + X10 * K12;
        P11 = Y11 + X01 * K01 + X11 * K11;
        P12 = Y12 + X01 * K02 + X11 * K12;
        P22 = Y22 + X02 * K02 + X12 * K12;
        p0 = hx0 + X00 * k0 + X10 * k1;
        p1 = hx1 + X01 * k0 + X11 * k1;
        p2 = hx2 + X02 * k0 + X12 * k1;
        // closed-loop map of the segment (Phi = Phi_{i+1} on entry)
        const double W00 = ROT ? F00 * b00 + F02 * b20 : F00 * b00 + F01 * b10 + F02 * b20;  // Phi B
        const double W10 = ROT ? F10 * b00 + F12 * b20 : F10 * b00 + F11 * b10 + F12 * b20;
        const double W20 = ROT ? F20 * b00 + F22 * b20 : F20 * b00 + F21 * b10 + F22 * b20;
        const double W01 = F02 * b21, W11 = F12 * b21, W21 = F22 * b21;
        // lam-gain of u_i: Fl = -S^-1 W'
        // (written as -a b - c d: the negation folds into the fma's source modifiers, where
        // -(a b + c d) cost a v_xor per entry)
        const double L00 = -I00 * W00 - I01 * W01, L01 = -I00 * W10 - I01 * W11;
        const double L02 = -I00 * W20 - I01 * W21;
        const double L10 = -I01 * W00 - I11 * W01, L11 = -I01 * W10 - I11 * W11;
        const double L12 = -I01 * W20 - I11 * W21;
        if constexpr (FST) {
          s[8 * 64] = L00; s[9 * 64] = L01; s[10 * 64] = L02;
          s[11 * 64] = L10; s[12 * 64] = L11; s[13 * 64] = L12;
        }
        // psi += W k + Phi C
        s0v += W00 * k0 + W01 * k1 + (ROT ? F02 * c2 : F00 * c0 + F01 * c1 + F02 * c2);
        s1v += W10 * k0 + W11 * k1 + (ROT ? F12 * c2 : F10 * c0 + F11 * c1 + F12 * c2);
        s2v += W20 * k0 + W21 * k1 + (ROT ? F22 * c2 : F20 * c0 + F21 * c1 + F22 * c2);
        // Gam += W Fl
        G00 += W00 * L00 + W01 * L10;
        G01 += W00 * L01 + W01 * L11;
        G02 += W00 * L02 + W01 * L12;
        G11 += W10 * L01 + W11 * L11;
        G12 += W10 * L02 + W11 * L12;
        G22 += W20 * L02 + W21 * L12;
        // Phi = Phi A + W K  (A = I + E, E = a02 e_0 e_2' + a12 e_1 e_2')
        const double n02 = (ROT ? F02 + a12 * F01 : F02 + a02 * F00 + a12 * F01) + W00 * K02 + W01 * K12;
        const double n12 = (ROT ? F12 + a12 * F11 : F12 + a02 * F10 + a12 * F11) + W10 * K02 + W11 * K12;
        const double n22 = (ROT ? F22 + a12 * F21 : F22 + a02 * F20 + a12 * F21) + W20 * K02 + W21 * K12;
        F00 += W00 * K00 + W01 * K10; F01 += W00 * K01 + W01 * K11;
        F10 += W10 * K00 + W11 * K10; F11 += W10 * K01 + W11 * K11;
        F20 += W20 * K00 + W21 * K10; F21 += W20 * K01 + W21 * K11;
        F02 = n02; F12 = n12; F22 = n22;
      }
    }
    SACC(acc_bw, t_bw);
    SSTAMP(t_dual);
    // ---- 2. the segment ends: Riccati over the segments, then lam_j, x_s^(j) forward ----
    // the top segment hands (P, a) up the chain and x_e = 0 round the ring to segment 0
    if (top) {
      F00 = F01 = F02 = F10 = F11 = F12 = F20 = F21 = F22 = 0.0;
      s0v = s1v = s2v = 0.0;
      G00 = G01 = G02 = G11 = G12 = G22 = 0.0;
    }
    lm0 = lm1 = lm2 = 0.0;
    xs0 = xs1 = xs2 = 0.0;
    if constexpr (S > 1) {
      double M00 = P00, M01 = P01, M02 = P02, M11 = P11, M12 = P12, M22 = P22;
      double m0 = p0, m1 = p1, m2 = p2;
      double T00 = 0, T01 = 0, T02 = 0, T10 = 0, T11 = 0, T12 = 0, T20 = 0, T21 = 0, T22 = 0;
      double t0 = 0, t1 = 0, t2 = 0;
#pragma unroll 1
      for (int it = 0; it < S - 1; it++) {
        const double N00 = seg_up<S>(M00, lane), N01 = seg_up<S>(M01, lane), N02 = seg_up<S>(M02, lane);
        const double N11 = seg_up<S>(M11, lane), N12 = seg_up<S>(M12, lane), N22 = seg_up<S>(M22, lane);
        const double n0 = seg_up<S>(m0, lane), n1 = seg_up<S>(m1, lane), n2 = seg_up<S>(m2, lane);
        // Z = I - Mn Gam
        const double Z00 = 1.0 - (N00 * G00 + N01 * G01 + N02 * G02);
        const double Z01 = -(N00 * G01 + N01 * G11 + N02 * G12);
        const double Z02 = -(N00 * G02 + N01 * G12 + N02 * G22);
        const double Z10 = -(N01 * G00 + N11 * G01 + N12 * G02);
        const double Z11 = 1.0 - (N01 * G01 + N11 * G11 + N12 * G12);
        const double Z12 = -(N01 * G02 + N11 * G12 + N12 * G22);
        const double Z20 = -(N02 * G00 + N12 * G01 + N22 * G02);
        const double Z21 = -(N02 * G01 + N12 * G11 + N22 * G12);
        const double Z22 = 1.0 - (N02 * G02 + N12 * G12 + N22 * G22);
        // Z^-1 by the adjugate
        const double A00 = Z11 * Z22 - Z12 * Z21, A01 = Z02 * Z21 - Z01 * Z22, A02 = Z01 * Z12 - Z02 * Z11;
        const double A10 = Z12 * Z20 - Z10 * Z22, A11 = Z00 * Z22 - Z02 * Z20, A12 = Z02 * Z10 - Z00 * Z12;
        const double A20 = Z10 * Z21 - Z11 * Z20, A21 = Z01 * Z20 - Z00 * Z21, A22 = Z00 * Z11 - Z01 * Z10;
        const double zdet = Z00 * A00 + Z01 * A10 + Z02 * A20;
        double iz = __builtin_amdgcn_rcp(zdet);
        iz = fma(iz, fma(-zdet, iz, 1.0), iz);
        iz = fma(iz, fma(-zdet, iz, 1.0), iz);
        // Y = Z^-1 Mn is symmetric ((I - N G)^-1 N = N (I - G N)^-1 for symmetric N, G): six
        // entries, then T = Y Phi and t = Y psi + Z^-1 mn (15 fewer fp64 operations per step than
        // T = Z^-1 (Mn Phi))
        const double Y00 = iz * (A00 * N00 + A01 * N01 + A02 * N02);
        const double Y01 = iz * (A00 * N01 + A01 * N11 + A02 * N12);
        const double Y02 = iz * (A00 * N02 + A01 * N12 + A02 * N22);
        const double Y11 = iz * (A10 * N01 + A11 * N11 + A12 * N12);
        const double Y12 = iz * (A10 * N02 + A11 * N12 + A12 * N22);
        const double Y22 = iz * (A20 * N02 + A21 * N12 + A22 * N22);
        T00 = Y00 * F00 + Y01 * F10 + Y02 * F20; T01 = Y00 * F01 + Y01 * F11 + Y02 * F21;
        T02 = Y00 * F02 + Y01 * F12 + Y02 * F22;
        T10 = Y01 * F00 + Y11 * F10 + Y12 * F20; T11 = Y01 * F01 + Y11 * F11 + Y12 * F21;
        T12 = Y01 * F02 + Y11 * F12 + Y12 * F22;
        T20 = Y02 * F00 + Y12 * F10 + Y22 * F20; T21 = Y02 * F01 + Y12 * F11 + Y22 * F21;
        T22 = Y02 * F02 + Y12 * F12 + Y22 * F22;
        const double an0 = A00 * n0 + A01 * n1 + A02 * n2, an1 = A10 * n0 + A11 * n1 + A12 * n2;
        const double an2 = A20 * n0 + A21 * n1 + A22 * n2;
        t0 = Y00 * s0v + Y01 * s1v + Y02 * s2v + iz * an0;
        t1 = Y01 * s0v + Y11 * s1v + Y12 * s2v + iz * an1;
        t2 = Y02 * s0v + Y12 * s1v + Y22 * s2v + iz * an2;
        // M = P + Phi' T, m = a + Phi' t
        M00 = P00 + F00 * T00 + F10 * T10 + F20 * T20;
        M01 = P01 + F00 * T01 + F10 * T11 + F20 * T21;
        M02 = P02 + F00 * T02 + F10 * T12 + F20 * T22;
        M11 = P11 + F01 * T01 + F11 * T11 + F21 * T21;
        M12 = P12 + F01 * T02 + F11 * T12 + F21 * T22;
        M22 = P22 + F02 * T02 + F12 * T12 + F22 * T22;
        m0 = p0 + F00 * t0 + F10 * t1 + F20 * t2;
        m1 = p1 + F01 * t0 + F11 * t1 + F21 * t2;
        m2 = p2 + F02 * t0 + F12 * t1 + F22 * t2;
      }
#pragma unroll 1
      for (int it = 0; it < S - 1; it++) {
        const double l0 = T00 * xs0 + T01 * xs1 + T02 * xs2 + t0;
        const double l1 = T10 * xs0 + T11 * xs1 + T12 * xs2 + t1;
        const double l2 = T20 * xs0 + T21 * xs1 + T22 * xs2 + t2;
        const double e0 = F00 * xs0 + F01 * xs1 + F02 * xs2 + s0v + G00 * l0 + G01 * l1 + G02 * l2;
        const double e1 = F10 * xs0 + F11 * xs1 + F12 * xs2 + s1v + G01 * l0 + G11 * l1 + G12 * l2;
        const double e2 = F20 * xs0 + F21 * xs1 + F22 * xs2 + s2v + G02 * l0 + G12 * l1 + G22 * l2;
        xs0 = seg_dn<S>(e0, lane);
        xs1 = seg_dn<S>(e1, lane);
        xs2 = seg_dn<S>(e2, lane);
      }
      lm0 = top ? 0.0 : T00 * xs0 + T01 * xs1 + T02 * xs2 + t0;
      lm1 = top ? 0.0 : T10 * xs0 + T11 * xs1 + T12 * xs2 + t1;
      lm2 = top ? 0.0 : T20 * xs0 + T21 * xs1 + T22 * xs2 + t2;
    }
    SACC(acc_dual, t_dual);
    SSTAMP(t_ref);
    // ---- 3. refresh: the lam-part of the feed-forward, backward over the segment ----
    // (FST: nothing to refresh; the forward sweep adds F_i lam_j to k_i and the costate at the
    // segment start takes p^lam_s = Phi_s' lam_j. Phi's top-lane zeroing is harmless: lam = 0 there.)
    double pl0 = lm0, pl1 = lm1, pl2 = lm2;
    if constexpr (FST) {
      pl0 = F00 * lm0 + F10 * lm1 + F20 * lm2;
      pl1 = F01 * lm0 + F11 * lm1 + F21 * lm2;
      pl2 = F02 * lm0 + F12 * lm1 + F22 * lm2;
    }
    if constexpr (S > 1 && !FST) {
      // stage t - 1's values are loaded while stage t computes (clamped: no branch)
      double nr[11];
#pragma unroll
      for (int e = 0; e < 11; e++) nr[e] = sc[((m - 1) * NV + e) * 64];
      for (int t = m - 1; t >= 0; t--) {
        ST* s = sc + t * NV * 64;
        const double K00 = nr[0], K01 = nr[1], K02 = nr[2], K10 = nr[3], K11 = nr[4];
        const double K12 = nr[5], k0 = nr[6], k1 = nr[7];
        const double I00 = nr[8], I01 = nr[9], I11 = nr[10];
        {
          const ST* sn1 = sc + (t > 0 ? t - 1 : 0) * NV * 64;
#pragma unroll
          for (int e = 0; e < 11; e++) nr[e] = sn1[e * 64];
        }
        const double bp0 = ROT ? b00 * pl0 + b20 * pl2 : b00 * pl0 + b10 * pl1 + b20 * pl2;  // B' p
        const double bp1 = b21 * pl2;
        s[6 * 64] = k0 - (I00 * bp0 + I01 * bp1);
        s[7 * 64] = k1 - (I01 * bp0 + I11 * bp1);
        const double n0 = pl0 + K00 * bp0 + K10 * bp1, n1 = pl1 + K01 * bp0 + K11 * bp1;
        pl2 = (ROT ? pl2 + a12 * pl1 : pl2 + a02 * pl0 + a12 * pl1) + K02 * bp0 + K12 * bp1;
        pl0 = n0; pl1 = n1;
      }
    }
    SACC(acc_ref, t_ref);
    SSTAMP(t_fw);
    // ---- 4. forward over the segment: rollout, costate, PDAS re-guess ----
    // Two instantiations as in lane_kernel.h: plain PDAS passes (MODE 0) store the re-guessed
    // state as it is; single-flip passes (MODE 1) take the segment's first change only and
    // remember it (stage, replaced state) for the min over the QP's lanes below.
    bool changed = false;
    int fi = N;       // single-flip passes: this segment's first flip (stage) ...
    int fold_st = 0;  // ... and the state it replaced
    auto forward = [&](auto mode_tag) {
      constexpr int MODE = decltype(mode_tag)::value;
      double x0 = xs0, x1 = xs1, x2 = xs2;
      double l0 = P00 * x0 + P01 * x1 + P02 * x2 + p0 + pl0;  // costate at x_s
      double l1 = P01 * x0 + P11 * x1 + P12 * x2 + p1 + pl1;
      double l2 = P02 * x0 + P12 * x1 + P22 * x2 + p2 + pl2;
      bool flipped = false;
      double rx = r64[0], ry = r64[64], rt = r64[2 * 64];
      int old_n = ap[0];
      constexpr int NG = FST ? 14 : 8;
      double ng[NG];  // stage t + 1's gains, loaded while stage t computes
#pragma unroll
      for (int e = 0; e < NG; e++) ng[e] = sc[e * 64];
      // unrolled by 2: same-box A/B C5 29.6 -> 29.3 us, C2 27.0 -> 26.5, C4 shard neutral
#pragma unroll 2
      for (int t = 0; t < m; t++) {
        const double K00 = ng[0], K01 = ng[1], K02 = ng[2], K10 = ng[3], K11 = ng[4];
        const double K12 = ng[5];
        const double k0 = FST ? ng[6] + ng[8] * lm0 + ng[9] * lm1 + ng[10] * lm2 : ng[6];
        const double k1 = FST ? ng[7] + ng[11] * lm0 + ng[12] * lm1 + ng[13] * lm2 : ng[7];
        {
          const ST* sn1 = sc + (t + 1 < m ? t + 1 : m - 1) * NV * 64;
#pragma unroll
          for (int e = 0; e < NG; e++) ng[e] = sn1[e * 64];
        }
        const int old = old_n;
        const double rxi = rx, ryi = ry, rti = rt;
        {
          const int tn = t + 1 < m ? t + 1 : m - 1;
          old_n = ap[tn * 64];
          rx = r64[(3 * tn + 0) * 64];
          ry = r64[(3 * tn + 1) * 64];
          rt = r64[(3 * tn + 2) * 64];
        }
        const double u0 = K00 * x0 + K01 * x1 + K02 * x2 + k0;
        const double u1 = K10 * x0 + K11 * x1 + K12 * x2 + k1;
        const double w0 = l0 - q0 * (x0 - rxi), w1 = l1 - q1 * (x1 - ryi);
        const double w2 = l2 - q2 * (x2 - rti);
        l0 = w0; l1 = w1; l2 = ROT ? w2 - a12 * w1 : w2 - a02 * w0 - a12 * w1;
        const double g0 = ROT ? r0 * (u0 - ud0) + b00 * l0 + b20 * l2
                              : r0 * (u0 - ud0) + b00 * l0 + b10 * l1 + b20 * l2;
        const double g1 = r1 * (u1 - ud1) + b21 * l2;
        int st = MODE ? old : 0;
        const double* tf = ftab + 8 * old;  // (fp64 scratch) the old state's test thresholds
#pragma unroll
        for (int a = 0; a < 2; a++) {
          const int ca = (old >> (2 * a)) & 3;
          const double u = a ? u1 : u0, g = a ? g1 : g0;
          bool nlo, nhi;
          if constexpr (!F32) {
            // (the two tests exclude each other: lbe < ube, and a bound input has one test)
            const double y = tf[4 * a + 2] * u - tf[4 * a + 3] * g;
            nlo = y < tf[4 * a];
            nhi = y > tf[4 * a + 1];
          } else {
            const double gta = MODE ? (a ? gtoll1 : gtoll0) : (a ? gtol1 : gtol0);
            const double lbx = MODE ? (a ? lbl1 : lbl0) : (a ? lbe1 : lbe0);
            const double ubx = MODE ? (a ? ubl1 : ubl0) : (a ? ube1 : ube0);
            nlo = ((ca == 1) & (g > -gta)) | ((ca == 0) & (u < lbx));
            nhi = !nlo & (((ca == 2) & (g < gta)) | ((ca == 0) & (u > ubx)));
          }
          const int nca = (int)nlo | ((int)nhi << 1);
          if constexpr (MODE == 0) {
            st |= nca << (2 * a);
          } else {
            const bool take = (nca != ca) & !flipped;
            st = take ? ((st & ~(3 << (2 * a))) | (nca << (2 * a))) : st;
            flipped |= take;
          }
        }
        const bool ch = st != old;
        if constexpr (MODE == 1) {
          fi = (ch & (fi == N)) ? s0 + t : fi;
          fold_st = (ch & (fi == s0 + t)) ? old : fold_st;
        }
        changed |= ch;
        ap[t * 64] = st;
        const double nx0 = ROT ? x0 + b00 * u0 : x0 + a02 * x2 + b00 * u0 + c0;
        const double nx1 = ROT ? x1 + a12 * x2 : x1 + a12 * x2 + b10 * u0 + c1;
        const double nx2 = x2 + b20 * u0 + b21 * u1 + c2;
        x0 = nx0; x1 = nx1; x2 = nx2;
      }
    };
    if (single) forward(SegMode<1>{});
    else forward(SegMode<0>{});
    // single-flip passes keep only the QP's first flip over the whole horizon
    if (single) {
      int mn = fi;
#pragma unroll
      for (int k = 1; k < S; k <<= 1) {
        const int o = __shfl_xor(mn, k, 64);
        mn = o < mn ? o : mn;
      }
      if (fi < N && fi != mn) {
        ap[(fi - s0) * 64] = fold_st;
        changed = false;
      }
    }
    const bool qchanged = qany(__ballot(changed));
    SACC(acc_fw, t_fw);
    if (!qchanged && !done) {
      done = true;
      iters = pass + 1;
    }
  }

  SSTAMP(t_out);
  // the start whose outputs stand: the one that converged first (a converged start keeps its
  // iteration count while its wave sweeps on), the cold one on a tie or when neither converged
  bool owner = owner0, qowner = qowner0;
  if constexpr (TWIN) {
    const bool sdone = __shfl_xor((int)done, S, 64) != 0;
    const int sibit = __shfl_xor(iters, S, 64);
    const bool win = var ? (done && (!sdone || iters < sibit)) : (done ? (!sdone || iters <= sibit) : !sdone);
    owner = owner0 && win;
    qowner = qowner0 && win;
  }
  // ---- output sweep: u* = K x + k from the final gains, x* by the fp64 rollout ----
  const bool solved = done && !bad;
  const float nanv = __int_as_float(0x7fc00000);
  float* uo = uout + (size_t)b * 2 * N;
  float* xo = xout + (size_t)b * 3 * (N + 1);
  if (qowner) {
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
  // gap-row box screen (f110qp_kernels.hip, AUTO gap calls): the box optimum is the optimum with
  // the gap rows too when it keeps every row of stages 1..N with a margin of 1e-6 of the row's
  // terms (evaluated here on the fp64 rollout in world coordinates) and the constant stage-0 rows
  // hold; any other QP goes on the list for GI. A template variant (SCR): the box-only kernels
  // keep their code (a runtime test cost C2 26.7 -> 27.5 us, same box)
  double ga0 = 0.0, gb0 = 0.0, gc0 = 0.0, ga1 = 0.0, gb1 = 0.0, gc1 = 0.0;
  if constexpr (SCR) {
    const float* h6 = oo.scr_hs + 6 * (size_t)b;
    ga0 = h6[0]; gb0 = h6[1]; gc0 = h6[2]; ga1 = h6[3]; gb1 = h6[4]; gc1 = h6[5];
  }
  int nviol = 0;  // gap rows of this lane's stages the box optimum violates (or within the margin)
  SSTAMP(t_ol0);
  {
    double x0 = xs0, x1 = xs1, x2 = xs2;
    for (int t = 0; t < m; t++) {
      const int i = s0 + t;
      const ST* s = sc + t * NV * 64;
      const double K00 = s[0], K01 = s[64], K02 = s[2 * 64], K10 = s[3 * 64], K11 = s[4 * 64];
      const double K12 = s[5 * 64];
      const double k0 = FST ? s[6 * 64] + s[8 * 64] * lm0 + s[9 * 64] * lm1 + s[10 * 64] * lm2 : s[6 * 64];
      const double k1 = FST ? s[7 * 64] + s[11 * 64] * lm0 + s[12 * 64] * lm1 + s[13 * 64] * lm2 : s[7 * 64];
      // fp32 scratch: clamp a free input that sits outside its box by the single-flip tolerance
      const double u0 = F32 ? fmin(fmax(K00 * x0 + K01 * x1 + K02 * x2 + k0, lb0), ub0)
                            : K00 * x0 + K01 * x1 + K02 * x2 + k0;
      const double u1 = F32 ? fmin(fmax(K10 * x0 + K11 * x1 + K12 * x2 + k1, lb1), ub1)
                            : K10 * x0 + K11 * x1 + K12 * x2 + k1;
      if (want_obj) {
        qterm(r64[(3 * t) * 64], r64[(3 * t + 1) * 64], r64[(3 * t + 2) * 64], x0, x1, x2);
        J += 0.5 * (r0 * (u0 - ud0) * (u0 - ud0) + r1 * (u1 - ud1) * (u1 - ud1));
      }
      const double nx0 = ROT ? x0 + b00 * u0 : x0 + a02 * x2 + b00 * u0 + c0;
      const double nx1 = ROT ? x1 + a12 * x2 : x1 + a12 * x2 + b10 * u0 + c1;
      const double nx2 = x2 + b20 * u0 + b21 * u1 + c2;
      x0 = nx0; x1 = nx1; x2 = nx2;
      if constexpr (SCR) {
        const double wx = (ROT ? cs * x0 - sn * x1 : x0) + X0, wy = (ROT ? sn * x0 + cs * x1 : x1) + Y0;
        const double ta0 = ga0 * wx, tb0 = gb0 * wy, ta1 = ga1 * wx, tb1 = gb1 * wy;
        nviol += !(ta0 + tb0 + gc0 >= 1e-6 * (1.0 + fabs(ta0) + fabs(tb0) + fabs(gc0)));
        nviol += !(ta1 + tb1 + gc1 >= 1e-6 * (1.0 + fabs(ta1) + fabs(tb1) + fabs(gc1)));
      }
      if (owner) {
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
  SACC(t_out_loop, t_ol0);
  if (want_obj) {
#pragma unroll
    for (int k = 1; k < S; k <<= 1) {
      J += __shfl_xor(J, k, 64);
      Cr += __shfl_xor(Cr, k, 64);
    }
    const double Cu = 0.5 * (double)N * (r0 * ud0 * ud0 + r1 * ud1 * ud1);
    const double dnan = __longlong_as_double(0x7ff8000000000000ll);
    if (qowner && oo.cost) oo.cost[b] = solved ? J : dnan;
    if (qowner && oo.obj) oo.obj[b] = solved ? J - Cr - Cu : dnan;
  }
  if constexpr (SCR) {
    // the QP's violation count over its S lanes; GI priority 1 + count (the list is ordered by it,
    // heavy first: gap_order_kernel), 1 for a violated stage-0 row or a box solve that failed
#pragma unroll
    for (int k = 1; k < S; k <<= 1) nviol += __shfl_xor(nviol, k, 64);
    const bool ok0 = (ga0 * X0 + gb0 * Y0 >= -gc0 - 1e-9) & (ga1 * X0 + gb1 * Y0 >= -gc1 - 1e-9);
    if (qowner) oo.scr_prio[b] = (!solved || !ok0) ? 1 : (nviol > 0 ? 1 + nviol : 0);
  }
  if (qowner) {
    status_out[b] = bad ? F110QP_NUMERICAL_ID : (done ? F110QP_SOLVED_ID : F110QP_MAX_ITER_ID);
    if (iters_out) iters_out[b] = bad ? 0 : (done ? iters : max_pass);
  }
  if (wt) {  // active set of this solution for the next tick (OR over the segments)
    // the lane's 2m bits (input a of stage t at bit 2t + a), placed at bit 2 s0 of the pair
    unsigned long long lw = 0, hw = 0;
    for (int t = 0; t < m; t++) {
      const unsigned st = (unsigned)ap[t * 64];
      const unsigned l2 = (st & 1u) | ((st >> 1) & 2u), h2 = ((st >> 1) & 1u) | ((st >> 2) & 2u);
      lw |= (unsigned long long)l2 << (2 * t);
      hw |= (unsigned long long)h2 << (2 * t);
    }
    const int sh = 2 * s0;
    unsigned long long lo0 = sh < 64 ? lw << sh : 0ull, hi0 = sh < 64 ? hw << sh : 0ull;
    unsigned long long lo1 = sh == 0 ? 0ull : (sh < 64 ? lw >> (64 - sh) : lw << (sh - 64));
    unsigned long long hi1 = sh == 0 ? 0ull : (sh < 64 ? hw >> (64 - sh) : hw << (sh - 64));
#pragma unroll
    for (int k = 1; k < S; k <<= 1) {
      lo0 |= __shfl_xor(lo0, k, 64);
      hi0 |= __shfl_xor(hi0, k, 64);
      lo1 |= __shfl_xor(lo1, k, 64);
      hi1 |= __shfl_xor(hi1, k, 64);
    }
    if (qowner) {
      ws.act[2 * R * b] = lo0;
      ws.act[2 * R * b + 1] = hi0;
      if (R > 1) {
        ws.act[2 * (R * b + 1)] = lo1;
        ws.act[2 * (R * b + 1) + 1] = hi1;
      }
      unsigned* key = ws.key + 4 * b;
      key[0] = kth; key[1] = kv; key[2] = kd; key[3] = 2u;
    }
    // the wave's own counters (no atomics on one address: 256 waves x 2 of them measured ~3 us on
    // a stream whose keys hit every call)
    if (ws.stats && lane == 0) {
      *reinterpret_cast<uint2*>(ws.stats + 2 * (size_t)blockIdx.x) = make_uint2(wst.x, wst.y + 1u);
    }
  }
#ifdef F110QP_STAMPS
  if (lane == 0 && blockIdx.x < 4096) {
    unsigned long long* o = g_sstamps + (size_t)blockIdx.x * kSegStampSlots;
    const unsigned long long t_end = __builtin_amdgcn_s_memtime();
    o[0] = t_setup; o[1] = acc_bw; o[2] = acc_dual; o[3] = acc_ref; o[4] = acc_fw;
    o[5] = t_end - t_out; o[6] = npass; o[7] = t_end - t_start;
    o[8] = t_stg - t_start; o[9] = t_lin - t_stg; o[10] = t_conv - t_lin; o[11] = t_setup - (t_conv - t_start);
    o[12] = t_rn - t_conv; o[13] = t_mask - t_rn; o[14] = t_setup - (t_mask - t_start); o[15] = t_out_loop;
  }
#endif
  signal_call_done(oo);  // a synchronous call's completion word (f110qp_kernels.h)
}

// Scratch of the segmented kernel for a batch: 1 fp64 (the lam-gains kept when they fit), 2 fp32
// (references and scratch as float) when fp64 does not fit the CU's 160 KiB at the grid's waves
// per CU (the float grid may then take more than one dispatch round), or when forced (lw.seg32:
// F110QP_LANE_SEG_F32=1); 0 if neither fits.
inline int seg_scratch_mode(const KParams& P, int B, int S, const LaneWork& lw) {
  const size_t waves = ((size_t)B * S + 63) / 64;
  const size_t per_cu = (waves + 255) / 256;
  const bool f64 = per_cu * seg_lds_bytes(P.N, S, false) <= 160 * 1024;
  const bool f32 = seg_lds_bytes(P.N, S, false, true) <= 160 * 1024;  // in one or more rounds
  if (lw.seg32 && f32) return 2;
  return f64 ? 1 : (f32 ? 2 : 0);
}

// Twin starts (lane_seg_kernel<..., TWIN = true>): each QP solved from the cold start and from the
// speed bound u_des sits on held over the first half of the horizon, in adjacent slots of one wave.
// Taken when u_des is on a speed bound (the shipped params.yaml:42,46: des_vel = umax), the doubled
// grid is at most two waves per CU and the lam-gain (FST) scratch of those waves fits a CU's LDS:
// C2 (1,024 QPs, 128 waves) 26.4 -> 23.4 us. C5 (4,096, 512 waves, two per CU) measured 28.8 ->
// 30.9 while the segment ends went through ds_bpermute, and 28.95 -> 28.55 us (cold 28.84 -> 28.3)
// with the DPP exchanges (same box; its slowest tick's passes 5 -> 4). lw.twin = 0 (test build,
// F110QP_LANE_TWIN=0) turns it off.
#ifndef F110QP_TWIN_MAX_WAVES
#define F110QP_TWIN_MAX_WAVES 512  // (measurement builds: tools/build_seg_variant.sh -D...)
#endif
constexpr long kTwinMaxWaves = F110QP_TWIN_MAX_WAVES;
inline bool seg_twin(const KParams& P, int B, int S, const LaneWork& lw) {
  if (!lw.twin || !(P.udes[0] >= (double)P.umax[0] || P.udes[0] <= (double)P.umin[0])) return false;
  const long waves2 = (2L * B * S + 63) / 64;
  const long per_cu = (waves2 + 255) / 256;
  return waves2 <= kTwinMaxWaves && seg_scratch_mode(P, 2 * B, S, lw) == 1 && lw.dref &&
         per_cu * seg_lds_bytes(P.N, S, true) <= 160 * 1024;  // the FST kernel, all waves resident
}

template <int S, bool ROT, bool SCR>
hipError_t launch_lane_seg_t(const KParams& P, int B, const float* x0, const float* ul, const float* xr,
                             float* uo, float* xo, int* st, int* its, const WarmState& ws,
                             const LaneWork& lw, const ObjOut& oo, hipStream_t s) {
  constexpr int L = 64 / S;
  const int twin = seg_twin(P, B, S, lw) ? 1 : 0;  // (one wave per CU at most: FST fits)
  const int waves = ((B << twin) + L - 1) / L;
  const int mode = seg_scratch_mode(P, B << twin, S, lw);
  // the lam-gains stored (FST, no refresh sweep: measured C5 30.5 -> see DESIGN.md 2b') when the
  // resident waves' LDS holds 14 doubles per stage, else the refresh sweep (11); lw.dref = 0
  // forces the refresh (test hook, F110QP_LANE_DREF=0)
  const size_t per_cu = ((size_t)waves + 255) / 256;
  const bool fst = mode == 1 && lw.dref && per_cu * seg_lds_bytes(P.N, S, true) <= 160 * 1024;
  auto go1 = [&](auto kern, size_t lds) -> hipError_t {
    if (lds > 64 * 1024) {
      hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(kern, dim3(waves), dim3(64), lds, s, P, B, x0, ul, xr, uo, xo, st, its, ws,
                       lw.kmax, oo);
    return hipGetLastError();
  };
  const bool even = P.N % S == 0;  // equal segments: the EVEN instantiation
#define F110QP_SEG_GO(FST_, ST_, TWIN_, LDS_)                                              \
  (even ? go1(&lane_seg_kernel<S, ROT, FST_, ST_, SCR, TWIN_, true>, LDS_)                 \
        : go1(&lane_seg_kernel<S, ROT, FST_, ST_, SCR, TWIN_, false>, LDS_))
  if (twin) return F110QP_SEG_GO(true, double, true, seg_lds_bytes(P.N, S, true));
  if (mode == 2) return F110QP_SEG_GO(false, float, false, seg_lds_bytes(P.N, S, false, true));
  return fst ? F110QP_SEG_GO(true, double, false, seg_lds_bytes(P.N, S, true))
             : F110QP_SEG_GO(false, double, false, seg_lds_bytes(P.N, S, false));
#undef F110QP_SEG_GO
}

}  // namespace f110qp

#ifdef F110QP_STAMPS
extern "C" int f110qp_read_seg_stamps(unsigned long long* host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(f110qp::g_sstamps),
                                  (size_t)n * f110qp::kSegStampSlots * sizeof(unsigned long long));
}
#endif

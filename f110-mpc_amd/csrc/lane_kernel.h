// lane_kernel.h — the throughput path: ONE LANE PER QP (up to 64 box-constrained QPs per wave).
//
// The reference solves, per control tick, the sparse QP of MPC::Update (src/mpc.cpp:69-143):
// min sum_i 1/2 |x_i - r_i|_Q^2 + 1/2 |u_i - u_des|_R^2 subject to the dynamics rows
// x_{i+1} = A x_i + B u_i + C (mpc.cpp:244-248,299,305; A, B, C from Model::Linearize,
// model.cpp:30-59, the same at every stage) and the input box rows (mpc.cpp:253,281,290).
// With the gap rows inactive (the shipped bounds, mpc.cpp:296-300) that is a box-constrained
// linear-quadratic regulator, and its exact optimum comes from a primal-dual active set on the
// inputs where every pass is two sweeps over the horizon:
//   backward i = N-1..0 : one Riccati step with the stage's fixed inputs masked out (branch
//                         free): K_i, k_i to scratch; P_i = Hxx + Hux' K_i, p_i = hx + Hux' k_i.
//                         With x_0 = 0 (recentred) the costate at stage 0 is lambda_0 = p_0.
//   forward  i = 0..N-1 : u_i = K_i x_i + k_i, x_{i+1} = A x_i + B u_i + C, and the costate
//                         carried FORWARD: lambda_{i+1} = A'^-1 (lambda_i - Q(x_i - r_i)) with
//                         A'^-1 = I - E' (A = I + E, E^2 = 0, model.cpp:42-46) — the adjoint
//                         equation lambda_i = Q(x_i - r_i) + A' lambda_{i+1} solved for its
//                         successor, exact because lambda_i = P_i x_i + p_i on the solution of
//                         the masked problem. The gradient R(u_i - u_des) + B' lambda_{i+1}
//                         gives the bound multipliers and the PDAS re-guess of stage i.
// A forward sweep that changes nothing certifies the KKT conditions (active bounds with
// non-negative multipliers, inactive inputs inside the box); its gains (kept in the scratch)
// give u* and x* in a last output sweep. Everything is fp64 in registers, recentred on
// (x0, y0, theta0) like the wave kernel, so the result is the exact optimum to ~1e-12 (to
// ~1e-7 with fp32 scratch).
//
// Layout: a wave solves L QPs (L = 1..64, a power of two): lane l of workgroup w works on QP
// b = L w + (l mod L), so for L < 64 every QP is computed by 64 / L lanes in lock step; only
// the first (the owner) stores results. Keeping EXEC full is deliberate: on gfx950 a wave whose
// EXEC mask is partial runs ~2.4x slower once its CU hosts one wave per SIMD, while full waves
// do not (tools/microbench/contention.hip) — the same reason a lane whose
// QP has converged keeps sweeping (its sweeps reproduce the same K, u and set: idempotent)
// until the whole wave is done, and why the output sweep runs once for all lanes at the end.
// The duplicates write the same values to the same LDS/HBM slots as their owner (measured free).
// A wave's time is its slowest QP's passes times the cost of one sweep at one wave per SIMD, so
// L is the smallest power of two that fits the batch in <= 256 waves (one per CU; measured
// faster than one per SIMD at 1,024 - 8,192 QPs, and a second wave on a SIMD halves both, the
// fp64 pipe being saturated by one): small batches spread over the whole chip and each wave
// waits for the maximum pass count of fewer QPs. The wave's L
// reference paths are contiguous in HBM; they are staged once into LDS transposed ([i][c][L],
// conflict free), every load of the wave in flight at once. K_i, k_i (backward -> forward; u_i
// are recomputed from them in the output sweep) go through a per-wave scratch, [stage][8][L]
// in LDS when the resident waves fit, else [stage][L][8] in an HBM workspace read through a
// prefetch ring;
// the per-stage PDAS state sits in LDS. No cross-lane traffic at all except the wave-uniform
// "any lane still iterating" vote.
// Convergence: PDAS (every violated complementarity condition flips at once) for kmax passes;
// a lane still changing after that flips only its FIRST violation per pass (stage-major,
// input-minor order: the least-index single principal pivoting of Murty / Bard, finite for
// box-constrained QPs with a positive definite Hessian, Judice & Pires 1989), so every QP is
// solved inside this one launch; P.max_iter passes bound it (status MAX_ITER, NaN outputs).
//
// This header holds the kernel template; lane_inst.hip instantiates it per QPs-per-wave value
// LQ (a compile-time stride: every LDS / scratch offset is an immediate, which removed ~45
// address instructions per stage and pass), lane_launch.hip picks the instantiation.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "f110qp_kernels.h"

namespace f110qp {

// Diagnostic build only (-DF110QP_STAMPS): per-wave cycles of each sweep type, read back with
// f110qp_read_lane_stamps(). The shipped library never executes a stamp.
#ifdef F110QP_STAMPS
constexpr int kLaneStampSlots = 8;
__device__ unsigned long long g_lstamps[4096 * kLaneStampSlots];  // one TU per stamps build
#define LSTAMP(var) const unsigned long long var = __builtin_amdgcn_s_memtime()
#define LACC(acc, since) acc += __builtin_amdgcn_s_memtime() - (since)
#else
#define LSTAMP(var)
#define LACC(acc, since)
#endif

// stages of scratch loaded ahead in the forward and output sweeps: HBM latency is several
// stages of compute, LDS latency (~60 cycles at one wave per SIMD) less than one
#ifndef F110QP_LANE_RING_LDS
#define F110QP_LANE_RING_LDS 1  // measured: 1 vs 2 stages ahead, C4 shard 184.3 -> 178.9 us, C5 64.6 -> 61.5
#endif
#ifndef F110QP_LANE_RING_HBM
#define F110QP_LANE_RING_HBM 4
#endif
#ifndef F110QP_LANE_NEWTON
#define F110QP_LANE_NEWTON 2  // Newton steps after v_rcp_f64 in the masked 2x2 inverse
#endif
template <bool SLDS>
constexpr int ring_depth() { return SLDS ? F110QP_LANE_RING_LDS : F110QP_LANE_RING_HBM; }


template <int M>
struct ModeTag {
  static constexpr int value = M;
};

// Scratch of the Riccati passes: ST = double or float, in LDS (SLDS) or in the HBM workspace.
// Occupancy hint for the register allocator / scheduler: 2 waves per SIMD for the LDS-scratch
// kernels (the grid still runs one wave per SIMD or CU; the 256-VGPR budget gave a better
// schedule: C4 shard 179.2 -> 172.4 us, C5 61.1 -> 60.0), 1 for the HBM-scratch ones (2
// measured C4 248.9 -> 251.7). F110QP_LANE_WPE overrides both (measurement knob).
#ifdef F110QP_LANE_WPE
#define F110QP_LANE_ATTR __attribute__((amdgpu_waves_per_eu(F110QP_LANE_WPE, F110QP_LANE_WPE)))
#else
#define F110QP_LANE_ATTR __attribute__((amdgpu_waves_per_eu(SLDS ? 2 : 1, SLDS ? 2 : 1)))
#endif
template <typename ST, bool SLDS, int L, bool ROT, bool DREF>
__global__ __launch_bounds__(64) F110QP_LANE_ATTR void lane_kernel(const KParams P, const int B,
                                                  const float* __restrict__ x0g,
                                                  const float* __restrict__ ulg,
                                                  const float* __restrict__ xrg,
                                                  float* __restrict__ uout,
                                                  float* __restrict__ xout,
                                                  int* __restrict__ status_out,
                                                  int* __restrict__ iters_out,
                                                  double* __restrict__ scr,
                                                  const WarmState ws, const int kmax,
                                                  const ObjOut oo) {
  extern __shared__ __attribute__((aligned(16))) float xr_s[];  // [3N][L] x_ref, transposed
  // DREF: the references are kept as recentred (and, ROT, rotated) fp64 offsets [3N][L] at the
  // start of LDS, converted once after staging; the float staging then sits in the upper half
  // of that region (stage i's doubles end at byte 24 (i + 1) L, below the floats of stage i + 1
  // at 12 N L + 12 (i + 1) L, so the in-order conversion never overwrites an unread float).
  // Layout: DREF [3N][L] fp64 refs | (SLDS) scratch | [N][L] state; else [3N][L] float refs |
  // [N][L] state | (SLDS) scratch.
  float* const stg = DREF ? xr_s + 3 * P.N * L : xr_s;
  LSTAMP(t_start);
#ifdef F110QP_STAMPS
  unsigned long long acc_bw = 0, acc_fw = 0, acc_out = 0, t_setup = 0, npass = 0;
#endif
  constexpr int kRing = ring_depth<SLDS>();
  const int lane = threadIdx.x;
  const int b0 = blockIdx.x * L;
  const int nq = (B - b0) < L ? (B - b0) : L;  // QPs of this wave (>= 1)
  int slot = lane & (L - 1);
  if (slot >= nq) slot = 0;                     // duplicate of a QP that exists
  const bool owner = lane < nq;                 // stores the results of QP b
  const int b = b0 + slot;
  const int N = P.N;
  const int n3 = 3 * N;
  const int R = (2 * N + 63) / 64;  // register-row count of the wave kernel's act layout
  const unsigned wlast = warm_last_hit(ws);  // the warm-start traffic switch (warm_traffic)

  // ---- stage the wave's reference paths (nq rows of 3S floats, the first 3N of each used) ---
  // Linear, coalesced sweep over the rows' first 3N entries (element e = q 3N + c -> stg[c L + q],
  // transposed). (q, c) advance by 64 elements per step without a division, every load reads a
  // valid address (clamped) and only the last chunk predicates its stores, so the full chunks
  // have no EXEC-masked region: ~18 instructions per element instead of ~50 (ISA). All loads of
  // a chunk per lane are issued before the first LDS write.
  {
    const int S3 = 3 * P.xr_stride;  // floats per QP in x_ref (>= 3N)
    const int tot = nq * n3;
    const float* src = xrg + (size_t)b0 * S3;
    const int dq = 64 / n3, dc = 64 - dq * n3;
    int q = lane / n3, c = lane - (lane / n3) * n3;
    const int last_off = (nq - 1) * S3 + (n3 - 1);
    constexpr int kChunk = 8;
    for (int e0 = 0; e0 < tot; e0 += kChunk * 64) {
      float vbuf[kChunk];
      int dst[kChunk];
#pragma unroll
      for (int j = 0; j < kChunk; j++) {
        const bool in = e0 + j * 64 + lane < tot;
        dst[j] = in ? c * L + q : -1;
        vbuf[j] = src[in ? q * S3 + c : last_off];
        q += dq;
        c += dc;
        const bool wrap = c >= n3;
        c -= wrap ? n3 : 0;
        q += wrap ? 1 : 0;
      }
      if (e0 + kChunk * 64 <= tot) {  // wave-uniform
#pragma unroll
        for (int j = 0; j < kChunk; j++) stg[dst[j]] = vbuf[j];
      } else {
#pragma unroll
        for (int j = 0; j < kChunk; j++)
          if (dst[j] >= 0) stg[dst[j]] = vbuf[j];
      }
    }
    __syncthreads();
  }
  // warm start: the slot's key and active-set masks when this call moves warm traffic (wlast
  // arrived with the staging loads); the masks unconditionally, so that no second dependent round
  // trip follows the key compare
  const bool wt = warm_traffic(ws, wlast);
  uint4 wkey = make_uint4(0u, 0u, 0u, 0u);
  unsigned long long wact[4] = {0ull, 0ull, 0ull, 0ull};
  uint2 wst = make_uint2(0u, 0u);  // this wave's warm counters (f110qp_warm_hits), updated at the end
  if (wt) {
    if (ws.stats) wst = *reinterpret_cast<const uint2*>(ws.stats + 2 * (size_t)blockIdx.x);
    wkey = *reinterpret_cast<const uint4*>(ws.key + 4 * (size_t)b);
    wact[0] = ws.act[2 * R * b];
    wact[1] = ws.act[2 * R * b + 1];
    if (R > 1) {
      wact[2] = ws.act[2 * (R * b + 1)];
      wact[3] = ws.act[2 * (R * b + 1) + 1];
    }
  }
  // a non-finite reference entry flags the QP: each lane scans its QP's staged row (~10
  // instructions per entry; a ballot per staged element measured more at C4 and c2_big sizes)
  bool nonfin = false;
  for (int e = 0; e < n3; e++) nonfin |= !isfinite(stg[e * L + slot]);

  // ---- per-lane QP data (Model::Linearize, model.cpp:30-59; fp64 of the float inputs) ----
  const double X0 = (double)x0g[3 * b + 0], Y0 = (double)x0g[3 * b + 1];
  const float fTH0 = x0g[3 * b + 2];
  const double th0 = (double)fTH0;
  const double v = (double)ulg[2 * b + 0], d = (double)ulg[2 * b + 1];
  const double dt = (double)P.dt;
  const double Lw = (double)0.3302f;
  double sn, cs, sd, cd;
  sincos(th0, &sn, &cs);
  sincos(d, &sd, &cd);
  const double sec2 = 1.0 / (cd * cd);
  // ROT (q0 == q1, the shipped params.yaml:1-2): the (x, y) offsets are expressed in the frame
  // of the heading th0, s = cs dx + sn dy, n = cs dy - sn dx. Q = diag(q0, q0, q2) is invariant
  // under that rotation and A = I + E, B become A = I + (v dt) e_n e_th', B = [dt 0; 0 0; b20 b21]
  // (the rotated model.cpp:42-51 with cs^2 + sn^2 = 1): four zero entries that drop ~20 fp64
  // operations of the backward Riccati stage and ~6 of the forward one.
  const double a02 = ROT ? 0.0 : -1 * v * sn * dt;                         // :42
  const double a12 = ROT ? v * dt : v * cs * dt;                           // :43
  const double b00 = ROT ? dt : cs * dt, b10 = ROT ? 0.0 : sn * dt;        // :48-49
  const double b20 = (sd / cd) * dt / Lw, b21 = v * sec2 * dt / Lw;        // :50-51
  const double c0r = v * th0 * sn * dt, c1r = -1 * v * th0 * cs * dt;     // :53-54
  const double c2 = -1 * d * v * sec2 * dt / Lw;                           // :55
  // The state is recentred on x0 = (X0, Y0, th0): translation invariance in (x, y) and, for the
  // heading, x_{i+1} = x_i + a02 th_i + ... + c0 = x_i + a02 (th_i - th0) + ... + (c0 + a02 th0).
  // c0 + a02 th0 is zero up to rounding (model.cpp:42,53); keeping it as computed stays exact.
  // (In the rotated frame both are exactly zero in exact arithmetic and dropped.)
  const double c0 = ROT ? 0.0 : c0r + a02 * th0, c1 = ROT ? 0.0 : c1r + a12 * th0;
  const double q0 = P.q[0], q1 = P.q[1], q2 = P.q[2], r0 = P.r[0], r1 = P.r[1];
  const double ud0 = P.udes[0], ud1 = P.udes[1];
  const double lb0 = (double)P.umin[0], lb1 = (double)P.umin[1];
  const double ub0 = (double)P.umax[0], ub1 = (double)P.umax[1];
  // PDAS flip tolerances (scaled): a free input enters its bound only when it is outside by more
  // than ptol, a fixed one leaves only when its multiplier is below -gtol, so that a degenerate
  // bound (zero multiplier: u_des on a bound and the reference tracked exactly) cannot flip free ->
  // bound -> free on rounding noise. fp64 gains: 1e-10 (noise ~1e-15), every pass. fp32 gains
  // (u carry ~1e-7 relative noise): exact compares in the PDAS passes (the accuracy of round 2),
  // 1e-6 / 1e-5 in the single-flip passes after kmax, where a degenerate QP then settles (its
  // KKT point exact to ~ptol, well inside the 1e-4 parity bound).
  constexpr bool F32 = sizeof(ST) == 4;
  constexpr double kPtT = F32 ? 0.0 : 1e-10, kGtT = F32 ? 0.0 : 1e-10;  // PDAS passes
  constexpr double kPtL = F32 ? 1e-6 : 1e-10, kGtL = F32 ? 1e-5 : 1e-10;  // single-flip passes
  auto tols = [&](bool loose, double& l0, double& u0, double& l1, double& u1, double& g0, double& g1) {
    const double pt = loose ? kPtL : kPtT, gt = loose ? kGtL : kGtT;
    l0 = lb0 - pt * (1.0 + fabs(lb0)); u0 = ub0 + pt * (1.0 + fabs(ub0));
    l1 = lb1 - pt * (1.0 + fabs(lb1)); u1 = ub1 + pt * (1.0 + fabs(ub1));
    g0 = gt * (1.0 + r0 * (1.0 + fabs(lb0) + fabs(ub0)));
    g1 = gt * (1.0 + r1 * (1.0 + fabs(lb1) + fabs(ub1)));
  };

  // scratch slot (i, e) of this QP: sp[8 L i + e ES] (LDS [stage][8][L]: ES = L; HBM
  // [stage][L][8]: ES = 1); the PDAS state of stage i (2 bits
  // per input: 0 free, 1 lower bound, 2 upper bound) at ap[i * L].
  // LDS: [3N][L] references, [N][L] PDAS state, then (SLDS) the [N][8][L] Riccati scratch
  double* const r64 = reinterpret_cast<double*>(xr_s) + slot;  // DREF only
  constexpr int ES = SLDS ? L : 1;  // stride of a stage's 8 gains in the scratch
  ST* sp;
  int* ap;
  if constexpr (SLDS) {
    sp = reinterpret_cast<ST*>(xr_s + (DREF ? 6 : 4) * N * L) + slot;
    ap = DREF ? reinterpret_cast<int*>(reinterpret_cast<ST*>(xr_s + 6 * N * L) + 8 * N * L) + slot
              : reinterpret_cast<int*>(xr_s + 3 * N * L) + slot;
  } else {
    // HBM: [stage][lane][8], a lane's 8 gains contiguous (two or four 16-B accesses per stage
    // instead of eight 4/8-B ones; 32-B aligned: the workspace is hipMalloc'ed)
    sp = static_cast<ST*>(__builtin_assume_aligned(
        reinterpret_cast<ST*>(scr) + (size_t)blockIdx.x * N * 8 * L + (size_t)slot * 8, 32));
    ap = reinterpret_cast<int*>(xr_s + (DREF ? 6 : 3) * N * L) + slot;
  }
  const unsigned kth = __float_as_uint(fTH0), kv = __float_as_uint(ulg[2 * b + 0]);
  const unsigned kd = __float_as_uint(ulg[2 * b + 1]);
  {
    // previous tick's active bounds seed the first pass (C5) when the slot's linearisation point
    // (theta0, v, steer bits) repeats: on the closed-loop stream, where it changes every tick, a
    // stale seed measured 1.61 vs 1.49 passes per QP cold. Key valid flag: 1 = written by the
    // wave kernel with its W = H^-1, 2 = by this kernel (act masks only, never a W for the wave
    // kernel to reuse).
    const bool hit = wkey.w != 0u && wkey.x == kth && wkey.y == kv && wkey.z == kd;
    if (ws.hit_call && __ballot(hit) != 0ull && lane == 0) *ws.hit_call = ws.call;
    wst.x += (unsigned)__popcll(__ballot(hit && owner));  // hits (owner lanes), stored at the end
    const unsigned long long lo0 = hit ? wact[0] : 0ull, hi0 = hit ? wact[1] : 0ull;
    const unsigned long long lo1 = hit ? wact[2] : 0ull, hi1 = hit ? wact[3] : 0ull;
    // (a cold start from the free set beats seeding the inputs whose u_des sits on a bound:
    // measured +0.5 PDAS passes per QP with the seed on the C2/C4 workloads)
    // stage i's two bits sit at bit 2i of the 128-bit (row 1 : row 0) masks: shifted out two at a
    // time (per input: 1 lower, 2 upper, 0 free; the lower bound wins)
    unsigned long long lw = lo0, hw = hi0;
    for (int i = 0; i < N; i++) {
      if (i == 32) {
        lw = lo1;
        hw = hi1;
      }
      const unsigned l2 = (unsigned)lw & 3u, h2 = (unsigned)hw & 3u & ~l2;
      ap[i * L] = (int)((l2 & 1u) | ((h2 & 1u) << 1) | ((l2 & 2u) << 1) | ((h2 & 2u) << 2));
      lw >>= 2;
      hw >>= 2;
    }
  }
  // recentred (ROT: rotated) reference of stage i from the float staging
  auto ref_f = [&](int i, double& rx, double& ry, double& rt) {
    const double dx = (double)stg[(3 * i + 0) * L + slot] - X0;
    const double dy = (double)stg[(3 * i + 1) * L + slot] - Y0;
    if constexpr (ROT) {
      rx = cs * dx + sn * dy;
      ry = cs * dy - sn * dx;
    } else {
      rx = dx;
      ry = dy;
    }
    rt = (double)stg[(3 * i + 2) * L + slot] - th0;
  };
  if constexpr (DREF) {  // once per kernel instead of once per stage and sweep
    for (int i = 0; i < N; i++) {
      double rx, ry, rt;
      ref_f(i, rx, ry, rt);
      r64[(3 * i + 0) * L] = rx;
      r64[(3 * i + 1) * L] = ry;
      r64[(3 * i + 2) * L] = rt;
    }
  }
  auto ref = [&](int i, double& rx, double& ry, double& rt) {
    if constexpr (DREF) {
      rx = r64[(3 * i + 0) * L];
      ry = r64[(3 * i + 1) * L];
      rt = r64[(3 * i + 2) * L];
    } else {
      ref_f(i, rx, ry, rt);
    }
  };

  // non-finite data -> F110QP_NUMERICAL with NaN outputs (e.g. the planning stage's NaN x_ref
  // of a scenario without a valid candidate, where the reference skips MPC::Update). Such a
  // lane keeps sweeping (NaN) in lock step but never holds the wave back.
  const bool bad = !(isfinite(X0) && isfinite(Y0) && isfinite(th0) && isfinite(v) && isfinite(d)) || nonfin;
  bool done = bad;
  int iters = 0;
#ifdef F110QP_STAMPS
  t_setup = __builtin_amdgcn_s_memtime() - t_start;
#endif
  // Rounds: a Riccati sweep for the current active set (backward), then the forward sweep that
  // rolls out u_i, x_i and carries the costate to re-guess the set (PDAS; after kmax passes
  // one flip per pass, the least-index rule). No change certifies the KKT conditions and the
  // u_i the forward sweep left in the scratch are the solution; a converged lane's further
  // sweeps reproduce them exactly.
  const int max_pass = P.pass_cap > 0 ? P.pass_cap : (P.max_iter > kmax ? P.max_iter : kmax);
  for (int pass = 0; pass < max_pass; pass++) {
    if (__ballot(!done) == 0ull) break;
    const bool single = pass >= kmax;
#ifdef F110QP_STAMPS
    npass++;
#endif
    LSTAMP(t_bw);
    {
      // ---- Riccati backward sweep ---------------------------------------------------------
      double rx, ry, rt;
      ref(N - 1, rx, ry, rt);  // terminal stage reuses x_ref[N-1] (mpc.cpp:228)
      double P00 = q0, P01 = 0.0, P02 = 0.0, P11 = q1, P12 = 0.0, P22 = q2;
      double p0 = -q0 * rx, p1 = -q1 * ry, p2 = -q2 * rt;
      int nst = ap[(N - 1) * L];
      for (int i = N - 1; i >= 0; i--) {
        ST* s = sp + (size_t)i * 8 * L;
        const int sti = nst;
        const int inx = i > 0 ? i - 1 : 0;  // clamped: loads without a branch (no register copies)
        nst = ap[inx * L];
        const double rxi = rx, ryi = ry, rti = rt;
        ref(inx, rx, ry, rt);  // next stage's reference, loaded a stage ahead
        // Riccati step of stage i against V_{i+1}(x) = 1/2 x'Px + p'x
        // (ROT: the terms of the zero entries a02, b10, c0, c1 are not formed at all)
        const double g0 = ROT ? P02 * c2 + p0 : P00 * c0 + P01 * c1 + P02 * c2 + p0;  // P C + p
        const double g1 = ROT ? P12 * c2 + p1 : P01 * c0 + P11 * c1 + P12 * c2 + p1;
        const double g2 = ROT ? P22 * c2 + p2 : P02 * c0 + P12 * c1 + P22 * c2 + p2;
        const double pb0 = ROT ? P00 * b00 + P02 * b20 : P00 * b00 + P01 * b10 + P02 * b20;  // P B[:,0]
        const double pb1 = ROT ? P01 * b00 + P12 * b20 : P01 * b00 + P11 * b10 + P12 * b20;
        const double pb2 = ROT ? P02 * b00 + P22 * b20 : P02 * b00 + P12 * b10 + P22 * b20;
        const double pc0 = P02 * b21, pc1 = P12 * b21, pc2 = P22 * b21;  // P B[:,1]
        const double H00 = ROT ? r0 + b00 * pb0 + b20 * pb2 : r0 + b00 * pb0 + b10 * pb1 + b20 * pb2;  // R + B'PB
        const double H01 = b21 * pb2;
        const double H11 = r1 + b21 * pc2;
        // Hux = B'PA: row a = ((PB_a)_0, (PB_a)_1, (PB_a)_2 + a02 (PB_a)_0 + a12 (PB_a)_1)
        const double X00 = pb0, X01 = pb1;
        const double X02 = ROT ? pb2 + a12 * pb1 : pb2 + a02 * pb0 + a12 * pb1;
        const double X10 = pc0, X11 = pc1;
        const double X12 = ROT ? pc2 + a12 * pc1 : pc2 + a02 * pc0 + a12 * pc1;
        const double h0 = ROT ? -r0 * ud0 + b00 * g0 + b20 * g2
                              : -r0 * ud0 + b00 * g0 + b10 * g1 + b20 * g2;  // -R ud + B'g
        const double h1 = -r1 * ud1 + b21 * g2;
        // Hxx = Q + A'PA, hx = -Q r + A'g
        const double e0 = ROT ? P02 + a12 * P01 : P02 + a02 * P00 + a12 * P01;
        const double e1 = ROT ? P12 + a12 * P11 : P12 + a02 * P01 + a12 * P11;
        const double e2 = ROT ? P22 + a12 * P12 : P22 + a02 * P02 + a12 * P12;
        const double Y00 = q0 + P00, Y01 = P01, Y11 = q1 + P11, Y02 = e0, Y12 = e1;
        const double Y22 = ROT ? q2 + e2 + a12 * e1 : q2 + e2 + a02 * e0 + a12 * e1;
        const double hx0 = -q0 * rxi + g0, hx1 = -q1 * ryi + g1;
        const double hx2 = ROT ? -q2 * rti + g2 + a12 * g1 : -q2 * rti + g2 + a02 * g0 + a12 * g1;
        // masked 2x2 solve over the free inputs of the stage (fixed ones sit on their bound)
        const int ca0 = sti & 3, ca1 = (sti >> 2) & 3;
        const bool f0 = ca0 == 0, f1 = ca1 == 0;
        const double bA0 = f0 ? 0.0 : (ca0 == 1 ? lb0 : ub0);
        const double bA1 = f1 ? 0.0 : (ca1 == 1 ? lb1 : ub1);
        const double M00 = f0 ? H00 : 1.0, M11 = f1 ? H11 : 1.0, M01 = (f0 && f1) ? H01 : 0.0;
        const double det = M00 * M11 - M01 * M01;  // > 0: R + B'PB is positive definite
        double idet = __builtin_amdgcn_rcp(det);   // + two Newton steps: full fp64
#pragma unroll
        for (int nt = 0; nt < F110QP_LANE_NEWTON; nt++) idet = fma(idet, fma(-det, idet, 1.0), idet);
        const double I00 = f0 ? M11 * idet : 0.0, I11 = f1 ? M00 * idet : 0.0;
        const double I01 = (f0 && f1) ? -M01 * idet : 0.0;
        const double K00 = -I00 * X00 - I01 * X10, K01 = -I00 * X01 - I01 * X11;
        const double K02 = -I00 * X02 - I01 * X12;
        const double K10 = -I01 * X00 - I11 * X10, K11 = -I01 * X01 - I11 * X11;
        const double K12 = -I01 * X02 - I11 * X12;
        const double w0 = h0 + H00 * bA0 + H01 * bA1, w1 = h1 + H01 * bA0 + H11 * bA1;
        const double k0 = bA0 - (I00 * w0 + I01 * w1), k1 = bA1 - (I01 * w0 + I11 * w1);
        s[0] = (ST)K00; s[ES] = (ST)K01; s[2 * ES] = (ST)K02; s[3 * ES] = (ST)K10;
        s[4 * ES] = (ST)K11; s[5 * ES] = (ST)K12; s[6 * ES] = (ST)k0; s[7 * ES] = (ST)k1;
        // V_i: P = Hxx + Hux' K, p = hx + Hux' k
        P00 = Y00 + X00 * K00 + X10 * K10;
        P01 = Y01 + X00 * K01 + X10 * K11;
        P02 = Y02 + X00 * K02 + X10 * K12;
        P11 = Y11 + X01 * K01 + X11 * K11;
        P12 = Y12 + X01 * K02 + X11 * K12;
        P22 = Y22 + X02 * K02 + X12 * K12;
        p0 = hx0 + X00 * k0 + X10 * k1;
        p1 = hx1 + X01 * k0 + X11 * k1;
        p2 = hx2 + X02 * k0 + X12 * k1;
      }
      LACC(acc_bw, t_bw);
      LSTAMP(t_fw);
      // ---- forward sweep: u_i = K_i x_i + k_i, x_{i+1} = A x_i + B u_i + C, costate and the
      // PDAS re-guess. K_i, k_i come through a ring of kRing stages loaded ahead; the ring
      // index is static inside the unrolled group.
      bool changed = false;
      if constexpr (SLDS) {
        // (LDS-scratch kernels instantiate the sweep twice: plain PDAS passes (MODE 0) take the
        // re-guessed state as it is, single-flip passes (MODE 1) keep only the first change of the
        // sweep — no per-stage flag logic in the common case: C4 shard 171.4 -> 163.6 us, C5 60.5
        // -> 57.5. The HBM-scratch kernels keep the inline sweep with the runtime flag below: the
        // lambda form measured C4 254 -> 276-280 us and 65,536 x N=20 109 -> 117-121 there, same
        // box.)
        auto forward = [&](auto mode_tag) -> bool {
        constexpr int MODE = decltype(mode_tag)::value;
        double lbe0, ube0, lbe1, ube1, gtol0, gtol1;
        tols(MODE == 1, lbe0, ube0, lbe1, ube1, gtol0, gtol1);
        bool changed = false;
        bool flipped = false;  // single-flip passes: the first violation of this sweep is taken
        {
          double x0 = 0.0, x1 = 0.0, x2 = 0.0;  // recentred x_0
          double l0 = p0, l1 = p1, l2 = p2;      // lambda_0 = P_0 x_0 + p_0 = p_0
          ST rg[kRing][8];
  #pragma unroll
          for (int t = 0; t < kRing; t++)
            if (t < N) {
  #pragma unroll
              for (int e = 0; e < 8; e++) rg[t][e] = sp[(size_t)t * 8 * L + e * ES];
            }
          double rx, ry, rt;
          ref(0, rx, ry, rt);
          int old_n = ap[0];
          for (int i0 = 0; i0 < N; i0 += kRing) {
  #pragma unroll
            for (int t = 0; t < kRing; t++) {
              const int i = i0 + t;
              if (i < N) {
                ST* s = sp + (size_t)i * 8 * L;
                const double K00 = rg[t][0], K01 = rg[t][1], K02 = rg[t][2], K10 = rg[t][3];
                const double K11 = rg[t][4], K12 = rg[t][5], k0 = rg[t][6], k1 = rg[t][7];
                {  // clamped loads: no branch, no register copies for the skipped case
                  const ST* sa = sp + (size_t)(i + kRing < N ? i + kRing : N - 1) * 8 * L;
  #pragma unroll
                  for (int e = 0; e < 8; e++) rg[t][e] = sa[e * ES];
                }
                const int old = old_n;
                const double rxi = rx, ryi = ry, rti = rt;
                {  // next stage's state and reference, loaded a stage ahead
                  const int inx = i + 1 < N ? i + 1 : N - 1;
                  old_n = ap[inx * L];
                  ref(inx, rx, ry, rt);
                }
                const double u0 = K00 * x0 + K01 * x1 + K02 * x2 + k0;
                const double u1 = K10 * x0 + K11 * x1 + K12 * x2 + k1;
                // lambda_{i+1} = (I - E')(lambda_i - Q(x_i - r_i))
                const double w0 = l0 - q0 * (x0 - rxi), w1 = l1 - q1 * (x1 - ryi);
                const double w2 = l2 - q2 * (x2 - rti);
                l0 = w0; l1 = w1; l2 = ROT ? w2 - a12 * w1 : w2 - a02 * w0 - a12 * w1;
                // gradient of the objective in u_i: g = R(u - ud) + B' lambda_{i+1}
                const double g0 = ROT ? r0 * (u0 - ud0) + b00 * l0 + b20 * l2
                                      : r0 * (u0 - ud0) + b00 * l0 + b10 * l1 + b20 * l2;
                const double g1 = r1 * (u1 - ud1) + b21 * l2;
                // PDAS re-guess (Hintermueller-Ito-Kunisch, c = 1), both inputs of the stage:
                // the multiplier of an active lower bound is g, of an active upper bound -g
                int st = MODE ? old : 0;
  #pragma unroll
                for (int a = 0; a < 2; a++) {
                  const int ca = (old >> (2 * a)) & 3;
                  const double u = a ? u1 : u0, g = a ? g1 : g0;
                  // a fixed input sits exactly on its bound (k carries the bound, its K row is
                  // zero), so the HIK test reduces to the multiplier's sign for a fixed input and
                  // to the bound test for a free one — both with a small tolerance, so that a
                  // degenerate bound (zero multiplier, e.g. u_des on a bound and the reference
                  // tracked exactly) cannot flip free -> bound -> free on rounding noise
                  // (bitwise, every compare evaluated: no EXEC-masked region per input and stage)
                  const double gt = a ? gtol1 : gtol0;
                  const bool nlo = ((ca == 1) & (g > -gt)) | ((ca == 0) & (u < (a ? lbe1 : lbe0)));
                  const bool nhi = !nlo & (((ca == 2) & (g < gt)) | ((ca == 0) & (u > (a ? ube1 : ube0))));
                  const int nca = (int)nlo | ((int)nhi << 1);
                  if constexpr (MODE == 0) {
                    st |= nca << (2 * a);
                  } else {
                    const bool take = (nca != ca) & !((MODE == 1 || single) & flipped);
                    st = take ? ((st & ~(3 << (2 * a))) | (nca << (2 * a))) : st;
                    flipped |= take;
                  }
                }
                changed |= (st != old);
                ap[i * L] = st;  // unconditional: an unchanged state rewrites its own value
                const double nx0 = ROT ? x0 + b00 * u0 : x0 + a02 * x2 + b00 * u0 + c0;
                const double nx1 = ROT ? x1 + a12 * x2 : x1 + a12 * x2 + b10 * u0 + c1;
                const double nx2 = x2 + b20 * u0 + b21 * u1 + c2;
                x0 = nx0; x1 = nx1; x2 = nx2;
              }
            }
          }
        }
        return changed;
        };
        changed = single ? forward(ModeTag<1>{}) : forward(ModeTag<0>{});
      } else {
        bool flipped = false;  // single-flip passes: the first violation of this sweep is taken
        double lbe0, ube0, lbe1, ube1, gtol0, gtol1;
        tols(single, lbe0, ube0, lbe1, ube1, gtol0, gtol1);
        {
          double x0 = 0.0, x1 = 0.0, x2 = 0.0;  // recentred x_0
          double l0 = p0, l1 = p1, l2 = p2;      // lambda_0 = P_0 x_0 + p_0 = p_0
          ST rg[kRing][8];
  #pragma unroll
          for (int t = 0; t < kRing; t++)
            if (t < N) {
  #pragma unroll
              for (int e = 0; e < 8; e++) rg[t][e] = sp[(size_t)t * 8 * L + e * ES];
            }
          double rx, ry, rt;
          ref(0, rx, ry, rt);
          int old_n = ap[0];
          for (int i0 = 0; i0 < N; i0 += kRing) {
  #pragma unroll
            for (int t = 0; t < kRing; t++) {
              const int i = i0 + t;
              if (i < N) {
                ST* s = sp + (size_t)i * 8 * L;
                const double K00 = rg[t][0], K01 = rg[t][1], K02 = rg[t][2], K10 = rg[t][3];
                const double K11 = rg[t][4], K12 = rg[t][5], k0 = rg[t][6], k1 = rg[t][7];
                {  // clamped loads: no branch, no register copies for the skipped case
                  const ST* sa = sp + (size_t)(i + kRing < N ? i + kRing : N - 1) * 8 * L;
  #pragma unroll
                  for (int e = 0; e < 8; e++) rg[t][e] = sa[e * ES];
                }
                const int old = old_n;
                const double rxi = rx, ryi = ry, rti = rt;
                {  // next stage's state and reference, loaded a stage ahead
                  const int inx = i + 1 < N ? i + 1 : N - 1;
                  old_n = ap[inx * L];
                  ref(inx, rx, ry, rt);
                }
                const double u0 = K00 * x0 + K01 * x1 + K02 * x2 + k0;
                const double u1 = K10 * x0 + K11 * x1 + K12 * x2 + k1;
                // lambda_{i+1} = (I - E')(lambda_i - Q(x_i - r_i))
                const double w0 = l0 - q0 * (x0 - rxi), w1 = l1 - q1 * (x1 - ryi);
                const double w2 = l2 - q2 * (x2 - rti);
                l0 = w0; l1 = w1; l2 = ROT ? w2 - a12 * w1 : w2 - a02 * w0 - a12 * w1;
                // gradient of the objective in u_i: g = R(u - ud) + B' lambda_{i+1}
                const double g0 = ROT ? r0 * (u0 - ud0) + b00 * l0 + b20 * l2
                                      : r0 * (u0 - ud0) + b00 * l0 + b10 * l1 + b20 * l2;
                const double g1 = r1 * (u1 - ud1) + b21 * l2;
                // PDAS re-guess (Hintermueller-Ito-Kunisch, c = 1), both inputs of the stage:
                // the multiplier of an active lower bound is g, of an active upper bound -g
                int st = old;
  #pragma unroll
                for (int a = 0; a < 2; a++) {
                  const int ca = (old >> (2 * a)) & 3;
                  const double u = a ? u1 : u0, g = a ? g1 : g0;
                  // a fixed input sits exactly on its bound (k carries the bound, its K row is
                  // zero), so the HIK test reduces to the multiplier's sign for a fixed input and
                  // to the bound test for a free one — both with a small tolerance, so that a
                  // degenerate bound (zero multiplier, e.g. u_des on a bound and the reference
                  // tracked exactly) cannot flip free -> bound -> free on rounding noise
                  // (bitwise, every compare evaluated: no EXEC-masked region per input and stage)
                  const double gt = a ? gtol1 : gtol0;
                  const bool nlo = ((ca == 1) & (g > -gt)) | ((ca == 0) & (u < (a ? lbe1 : lbe0)));
                  const bool nhi = !nlo & (((ca == 2) & (g < gt)) | ((ca == 0) & (u > (a ? ube1 : ube0))));
                  const int nca = (int)nlo | ((int)nhi << 1);
                  const bool take = (nca != ca) & !(single & flipped);
                  st = take ? ((st & ~(3 << (2 * a))) | (nca << (2 * a))) : st;
                  flipped |= take;
                }
                changed |= (st != old);
                ap[i * L] = st;  // unconditional: an unchanged state rewrites its own value
                const double nx0 = ROT ? x0 + b00 * u0 : x0 + a02 * x2 + b00 * u0 + c0;
                const double nx1 = ROT ? x1 + a12 * x2 : x1 + a12 * x2 + b10 * u0 + c1;
                const double nx2 = x2 + b20 * u0 + b21 * u1 + c2;
                x0 = nx0; x1 = nx1; x2 = nx2;
              }
            }
          }
        }
      }
      LACC(acc_fw, t_fw);
      if (!changed && !done) {  // KKT point: the gains of this pass (in the scratch) give u*
        done = true;
        iters = pass + 1;  // equality-QP solves incl. the confirming one
      }
    }
  }
  // ---- output sweep, every lane at once: x* by the fp64 rollout of u* ----
  LSTAMP(t_out);
  {
    const bool solved = done && !bad;
    const float nanv = __int_as_float(0x7fc00000);
    float* uo = uout + (size_t)b * 2 * N;
    float* xo = xout + (size_t)b * 3 * (N + 1);
    if (owner) {
      xo[0] = solved ? x0g[3 * b + 0] : nanv;  // x*_0 = x0 exactly, as the dynamics rows fix it
      xo[1] = solved ? x0g[3 * b + 1] : nanv;
      xo[2] = solved ? fTH0 : nanv;
    }
    // u* = K_i x_i + k_i from the gains of the last backward sweep (the set of the converged
    // pass: a converged lane's later sweeps rewrote the same gains), the same expression the
    // forward sweep evaluated — so the forward sweeps store no u (2 of 10 scratch values per
    // stage and pass) and this sweep reads the 8 gains once.
    double x0 = 0.0, x1 = 0.0, x2 = 0.0;
    ST ur[kRing][8];
#pragma unroll
    for (int t = 0; t < kRing; t++)
      if (t < N) {
#pragma unroll
        for (int e = 0; e < 8; e++) ur[t][e] = sp[(size_t)t * 8 * L + e * ES];
      }
    for (int i0 = 0; i0 < N; i0 += kRing) {
#pragma unroll
      for (int t = 0; t < kRing; t++) {
        const int i = i0 + t;
        if (i < N) {
          const double K00 = ur[t][0], K01 = ur[t][1], K02 = ur[t][2], K10 = ur[t][3];
          const double K11 = ur[t][4], K12 = ur[t][5], k0 = ur[t][6], k1 = ur[t][7];
          if (i + kRing < N) {
            const ST* s = sp + (size_t)(i + kRing) * 8 * L;
#pragma unroll
            for (int e = 0; e < 8; e++) ur[t][e] = s[e * ES];
          }
          // fp32 gains: a free input may sit outside its box by the single-flip tolerance
          // (1e-6 scaled); the output clamps it, x* is the rollout of the clamped u*
          const double u0 = F32 ? fmin(fmax(K00 * x0 + K01 * x1 + K02 * x2 + k0, lb0), ub0)
                                : K00 * x0 + K01 * x1 + K02 * x2 + k0;
          const double u1 = F32 ? fmin(fmax(K10 * x0 + K11 * x1 + K12 * x2 + k1, lb1), ub1)
                                : K10 * x0 + K11 * x1 + K12 * x2 + k1;
          const double nx0 = ROT ? x0 + b00 * u0 : x0 + a02 * x2 + b00 * u0 + c0;
          const double nx1 = ROT ? x1 + a12 * x2 : x1 + a12 * x2 + b10 * u0 + c1;
          const double nx2 = x2 + b20 * u0 + b21 * u1 + c2;
          x0 = nx0; x1 = nx1; x2 = nx2;
          if (owner) {
            uo[2 * i] = solved ? (float)u0 : nanv;
            uo[2 * i + 1] = solved ? (float)u1 : nanv;
            const double ox = ROT ? cs * x0 - sn * x1 : x0, oy = ROT ? sn * x0 + cs * x1 : x1;
            xo[3 * i + 3] = solved ? (float)(ox + X0) : nanv;
            xo[3 * i + 4] = solved ? (float)(oy + Y0) : nanv;
            xo[3 * i + 5] = solved ? (float)(x2 + th0) : nanv;
          }
        }
      }
    }
    if (owner) {
      // OSQP status ids: solved; no KKT point within max_pass passes -> max-iter
      status_out[b] = bad ? F110QP_NUMERICAL_ID : (done ? F110QP_SOLVED_ID : F110QP_MAX_ITER_ID);
      if (iters_out) iters_out[b] = bad ? 0 : (done ? iters : max_pass);
    }
  }
  LACC(acc_out, t_out);
  if (oo.obj || oo.cost) {
    // objective of the solution (fp64): cost = sum_{i=0..N} 1/2|x_i - r_i|_Q^2 + sum 1/2|u_i - u_des|_R^2
    // (r_N = x_ref[N-1], mpc.cpp:228) by one more rollout from the final gains, and OSQP's
    // 1/2 z'Pz + q'z = cost - 1/2 sum r_i'Q r_i - N/2 u_des'R u_des (world coordinates). In the
    // heading frame Q = diag(q0, q0, q2) is rotation invariant, so the tracking term is taken there.
    const bool solved = done && !bad;
    double x0 = 0.0, x1 = 0.0, x2 = 0.0, J = 0.0, Cr = 0.0;
    auto qterm = [&](int i, double e0, double e1, double e2) {
      double rx, ry, rt;
      ref(i, rx, ry, rt);
      const double d0 = e0 - rx, d1 = e1 - ry, d2 = e2 - rt;
      J += 0.5 * (q0 * d0 * d0 + q1 * d1 * d1 + q2 * d2 * d2);
      const double wx = (ROT ? cs * rx - sn * ry : rx) + X0, wy = (ROT ? sn * rx + cs * ry : ry) + Y0;
      const double wt = rt + th0;
      Cr += 0.5 * (q0 * wx * wx + q1 * wy * wy + q2 * wt * wt);
    };
    qterm(0, 0.0, 0.0, 0.0);
    for (int i = 0; i < N; i++) {
      const ST* s = sp + (size_t)i * 8 * L;
      const double K00 = s[0], K01 = s[ES], K02 = s[2 * ES], K10 = s[3 * ES];
      const double K11 = s[4 * ES], K12 = s[5 * ES], k0 = s[6 * ES], k1 = s[7 * ES];
      const double u0 = F32 ? fmin(fmax(K00 * x0 + K01 * x1 + K02 * x2 + k0, lb0), ub0)
                            : K00 * x0 + K01 * x1 + K02 * x2 + k0;
      const double u1 = F32 ? fmin(fmax(K10 * x0 + K11 * x1 + K12 * x2 + k1, lb1), ub1)
                            : K10 * x0 + K11 * x1 + K12 * x2 + k1;
      J += 0.5 * (r0 * (u0 - ud0) * (u0 - ud0) + r1 * (u1 - ud1) * (u1 - ud1));
      const double nx0 = ROT ? x0 + b00 * u0 : x0 + a02 * x2 + b00 * u0 + c0;
      const double nx1 = ROT ? x1 + a12 * x2 : x1 + a12 * x2 + b10 * u0 + c1;
      const double nx2 = x2 + b20 * u0 + b21 * u1 + c2;
      x0 = nx0; x1 = nx1; x2 = nx2;
      qterm(i + 1 < N ? i + 1 : N - 1, x0, x1, x2);
    }
    const double Cu = 0.5 * (double)N * (r0 * ud0 * ud0 + r1 * ud1 * ud1);
    const double nanv = __longlong_as_double(0x7ff8000000000000ll);
    if (owner && oo.cost) oo.cost[b] = solved ? J : nanv;
    if (owner && oo.obj) oo.obj[b] = solved ? J - Cr - Cu : nanv;
  }
  if (owner && wt) {  // active set of this solution for the next tick
    unsigned long long lo0 = 0, lo1 = 0, hi0 = 0, hi1 = 0;
    for (int i = 0; i < N; i++) {
      const unsigned st = (unsigned)ap[i * L];
      const unsigned long long l2 = (st & 1u) | ((st >> 1) & 2u), h2 = ((st >> 1) & 1u) | ((st >> 2) & 2u);
      const int sh = 2 * (i & 31);
      if (i < 32) {
        lo0 |= l2 << sh;
        hi0 |= h2 << sh;
      } else {
        lo1 |= l2 << sh;
        hi1 |= h2 << sh;
      }
    }
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
  if (ws.stats && wt && lane == 0) {
    *reinterpret_cast<uint2*>(ws.stats + 2 * (size_t)blockIdx.x) = make_uint2(wst.x, wst.y + 1u);
  }
#ifdef F110QP_STAMPS
  if (lane == 0 && blockIdx.x < 4096) {
    unsigned long long* o = g_lstamps + (size_t)blockIdx.x * kLaneStampSlots;
    o[0] = t_setup; o[1] = acc_bw; o[2] = acc_fw; o[3] = 0; o[4] = acc_out;
    o[5] = npass; o[6] = __builtin_amdgcn_s_memtime() - t_start; o[7] = 0;
  }
#endif
  signal_call_done(oo);  // a synchronous call's completion word (f110qp_kernels.h)
}

template <typename ST, bool SLDS, int L, bool ROT, bool DREF>
hipError_t launch_lane_t(const KParams& P, int B, const float* x0, const float* ul, const float* xr,
                         float* uo, float* xo, int* st, int* its, const WarmState& ws,
                         const LaneWork& lw, const ObjOut& oo, size_t lds, hipStream_t s) {
  const int waves = (B + L - 1) / L;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&lane_kernel<ST, SLDS, L, ROT, DREF>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((lane_kernel<ST, SLDS, L, ROT, DREF>), dim3(waves), dim3(64), lds, s, P, B, x0, ul, xr,
                     uo, xo, st, its, lw.scratch, ws, lw.kmax, oo);
  return hipGetLastError();
}

}  // namespace f110qp

#if defined(F110QP_STAMPS) && defined(F110QP_LANE_ALL)
extern "C" int f110qp_read_lane_stamps(unsigned long long* host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(f110qp::g_lstamps),
                                  (size_t)n * f110qp::kLaneStampSlots * sizeof(unsigned long long));
}
#endif

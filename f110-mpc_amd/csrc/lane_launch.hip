// lane_launch.hip — the lane back end's launch policy: QPs per wave L and the scratch placement,
// dispatched to the per-L instantiations of lane_kernel.h (lane_inst.hip). With F110QP_LANE_ALL
// (the -DF110QP_STAMPS diagnostic build) this one file instantiates every variant itself.
#ifdef F110QP_LANE_ALL
#include "lane_kernel.h"
#else
#include <hip/hip_runtime.h>

#include "f110qp_kernels.h"
#endif

namespace f110qp {

template <int S, bool ROT, bool SCR>
hipError_t launch_lane_seg_t(const KParams& P, int B, const float* x0, const float* ul, const float* xr,
                             float* uo, float* xo, int* st, int* its, const WarmState& ws,
                             const LaneWork& lw, const ObjOut& oo, hipStream_t s);  // lane_seg_inst.hip
// LDS per wave of the segmented kernel with fp64 / fp32 references and scratch (lane_seg_kernel.h
// seg_lds_bytes without the lam-gains, with its 1 KiB state-code tables: two with fp64 scratch)
constexpr size_t seg_lds_per_wave(int N, int S, bool f32 = false) {
  return (size_t)((N + S - 1) / S) * 64 * (3 * (f32 ? 4 : 8) + 4 + 11 * (f32 ? 4 : 8)) + (f32 ? 1 : 2) * 1024;
}

// Horizon segments per QP (lane_seg_kernel.h). A batch whose waves leave SIMDs idle (the QPs fit
// in fewer than one wave per SIMD at 64 / S QPs per wave) splits every QP's horizon over S lanes
// instead of running 64 / L identical copies of it. S cuts N into segments of >= 2 stages (of
// floor(N / S) or one more), the grid stays within two waves per SIMD (2,048 waves) and a wave's
// segmented LDS fits the CU (fp64 references and scratch when the whole grid is resident with
// them, else float ones, possibly in more than one dispatch round: 16,384 x N = 40 runs S = 4 on
// fp32 scratch in one round, 32,768 x N = 40 in two, round 4). Among those the launch takes the S with the shortest per-pass chain by the
// instruction model of DESIGN.md 2b': sequential N x ~255 instructions, segmented ceil(N / S) x
// ~350 + (S - 1) x ~230 (the two segment recursions). A forced QPs-per-wave or scratch placement
// keeps lane_kernel.h.
int lane_segments(const KParams& P, int B, const LaneWork& lw) {
  const int N = P.N;
  // dispatch rounds of the segmented grid: waves per CU over the waves the CU's 160 KiB of LDS
  // holds at once (fp64 scratch when the whole grid is resident with it, else float); 0 = no fit
  // the cost multiplier is rounds x resident waves per SIMD (a second wave on a SIMD shares its
  // fp64 issue slots: the kernels are VALU-issue bound)
  auto rounds = [&](int S) -> int {
    if (N / S < 2) return 0;
    const size_t waves = ((size_t)B * S + 63) / 64;
    const size_t per_cu = (waves + 255) / 256;
    if (per_cu > 8) return 0;
    size_t resident = per_cu;
    if (per_cu * seg_lds_per_wave(N, S) > 160 * 1024) {
      resident = (160 * 1024) / seg_lds_per_wave(N, S, true);
      if (resident < 1) return 0;
      if (resident > per_cu) resident = per_cu;
    }
    const size_t r = (per_cu + resident - 1) / resident;
    return (int)(r * ((resident + 3) / 4));
  };
  if (lw.seg == 1) return 1;
  if (lw.seg == 2 || lw.seg == 4 || lw.seg == 8) return rounds(lw.seg) > 0 ? lw.seg : 1;
  if (lw.qpw != 0 || (lw.mode != 0 && lw.mode != 1)) return 1;
  int best = 1;
  double cbest = 255.0 * N;
  for (int S = 2; S <= 8; S <<= 1) {
    const int r = rounds(S);
    if (r == 0) continue;
    // per-pass chain x dispatch rounds (the sequential kernel keeps its grid resident: HBM scratch)
    const double c = r * (350.0 * ((N + S - 1) / S) + 230.0 * (S - 1));
    if (c < cbest) {
      best = S;
      cbest = c;
    }
  }
  return best;
}

#ifndef F110QP_LANE_ALL
template <typename ST, bool SLDS, int L, bool ROT, bool DREF>
hipError_t launch_lane_t(const KParams& P, int B, const float* x0, const float* ul, const float* xr,
                         float* uo, float* xo, int* st, int* its, const WarmState& ws,
                         const LaneWork& lw, const ObjOut& oo, size_t lds, hipStream_t s);  // lane_inst.hip
#endif

// QPs per wave: the smallest power of two (<= 64) that fits the batch in kLaneTargetWaves waves
// (one per CU).
int lane_qps_per_wave(int B, int qpw) {
  if (qpw >= 1 && qpw <= 64 && (qpw & (qpw - 1)) == 0) return qpw;
  int L = 1;
  while (L < 64 && (B + L - 1) / L > kLaneTargetWaves) L <<= 1;
  return L;
}

// the heading-frame variant when Q's (x, y) weights are equal (lane_kernel.h, ROT), with the
// references converted once to fp64 in LDS (DREF: 12 N L more bytes per wave than the float
// references) when the grid runs one wave per CU. Measured: C4 shard 8,192 x N=40 195.8 ->
// 184.6 us, C5 66.9 -> 65.3; at four waves per CU (65,536 x N=20) 107.0 -> 109.1, so not there.
template <typename ST, bool SLDS, int L, bool DREF>
static hipError_t launch_rot_d(const KParams& P, int B, const float* x0, const float* ul,
                               const float* xr, float* uo, float* xo, int* st, int* its,
                               const WarmState& ws, const LaneWork& lw, const ObjOut& oo, size_t lds,
                               hipStream_t s) {
  if (lw.rot && P.q[0] == P.q[1])
    return launch_lane_t<ST, SLDS, L, true, DREF>(P, B, x0, ul, xr, uo, xo, st, its, ws, lw, oo, lds, s);
  return launch_lane_t<ST, SLDS, L, false, DREF>(P, B, x0, ul, xr, uo, xo, st, its, ws, lw, oo, lds, s);
}
template <typename ST, bool SLDS, int L>
static hipError_t launch_rot(const KParams& P, int B, const float* x0, const float* ul,
                             const float* xr, float* uo, float* xo, int* st, int* its,
                             const WarmState& ws, const LaneWork& lw, const ObjOut& oo, size_t lds,
                             hipStream_t s) {
  const size_t ldsd = lds + (size_t)P.N * L * 12;
  const size_t per_cu = (((size_t)B + L - 1) / L + 255) / 256;
  if (lw.dref && per_cu == 1 && ldsd <= 160 * 1024)
    return launch_rot_d<ST, SLDS, L, true>(P, B, x0, ul, xr, uo, xo, st, its, ws, lw, oo, ldsd, s);
  return launch_rot_d<ST, SLDS, L, false>(P, B, x0, ul, xr, uo, xo, st, its, ws, lw, oo, lds, s);
}

// Scratch placement of the lane kernel for a batch (lane_mode 0 = auto; 1/2/3/4 force LDS fp64 /
// LDS fp32 / HBM fp64 / HBM fp32): auto puts the scratch in LDS when every wave of the grid is
// resident with it (waves per CU x its LDS within the CU's 160 KiB): fp64 if that fits, else
// fp32; otherwise fp32 in the HBM workspace (the waves then stay resident on the 16 N L bytes of
// references + state alone). With the state recentred on x0 the fp32 gains and trajectories stay
// within ~1e-7 of the exact optimum (tests/test_gpu_parity.py::test_lane_backend_scratch_modes).
static int scratch_mode(const KParams& P, int B, int L, int mode) {
  const size_t N = (size_t)P.N;
  const size_t base = N * L * (12 + 4);  // references + PDAS state
  const size_t lds64 = base + N * 8 * L * sizeof(double), lds32 = base + N * 8 * L * sizeof(float);
  const size_t cap = 160 * 1024;
  if (mode == 0) {
    const size_t waves = ((size_t)B + L - 1) / L;
    const size_t per_cu = (waves + 255) / 256;
    mode = per_cu * lds64 <= cap ? 1 : per_cu * lds32 <= cap ? 2 : 4;
  }
  if (mode == 1 && lds64 > cap) mode = 3;
  if (mode == 2 && lds32 > cap) mode = 4;
  return mode;
}

int lane_scratch_mode(const KParams& P, int B, const LaneWork& lw) {
  return scratch_mode(P, B, lane_qps_per_wave(B, lw.qpw), lw.mode);
}

template <int L>
static hipError_t launch_lq(const KParams& P, int B, const float* x0, const float* ul, const float* xr,
                            float* uo, float* xo, int* st, int* its, const WarmState& ws,
                            const LaneWork& lw, const ObjOut& oo, hipStream_t s) {
  const size_t N = (size_t)P.N;
  const size_t base = N * L * (12 + 4);
  const size_t lds64 = base + N * 8 * L * sizeof(double), lds32 = base + N * 8 * L * sizeof(float);
  switch (scratch_mode(P, B, L, lw.mode)) {
    case 1: return launch_rot<double, true, L>(P, B, x0, ul, xr, uo, xo, st, its, ws, lw, oo, lds64, s);
    case 2: return launch_rot<float, true, L>(P, B, x0, ul, xr, uo, xo, st, its, ws, lw, oo, lds32, s);
    case 3: return launch_rot<double, false, L>(P, B, x0, ul, xr, uo, xo, st, its, ws, lw, oo, base, s);
    default: return launch_rot<float, false, L>(P, B, x0, ul, xr, uo, xo, st, its, ws, lw, oo, base, s);
  }
}

// LDS per wave: the staged references (12 N L B) + PDAS state (4 N L B) + Riccati scratch
// (8 N L sizeof(ST)) (lane_mode 0 = auto; 1/2/3/4 force LDS fp64 / LDS fp32 / HBM fp64 / HBM
// fp32).
hipError_t launch_lane(const KParams& P, int B, const float* x0, const float* ul,
                       const float* xr, float* uo, float* xo, int* st, int* its,
                       const WarmState& ws, const LaneWork& lw, const ObjOut& oo, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  const bool rot = lw.rot && P.q[0] == P.q[1];
  const bool scr = oo.scr_hs != nullptr;  // the gap-row screen variant (f110qp_kernels.hip)
#define F110QP_SEG_CASE(S)                                                                        \
  case S:                                                                                         \
    return scr ? (rot ? launch_lane_seg_t<S, true, true>(P, B, x0, ul, xr, uo, xo, st, its, ws, lw, oo, s)  \
                      : launch_lane_seg_t<S, false, true>(P, B, x0, ul, xr, uo, xo, st, its, ws, lw, oo, s)) \
               : (rot ? launch_lane_seg_t<S, true, false>(P, B, x0, ul, xr, uo, xo, st, its, ws, lw, oo, s) \
                      : launch_lane_seg_t<S, false, false>(P, B, x0, ul, xr, uo, xo, st, its, ws, lw, oo, s));
  switch (lane_segments(P, B, lw)) {
    F110QP_SEG_CASE(2)
    F110QP_SEG_CASE(4)
    F110QP_SEG_CASE(8)
    default: break;
  }
#undef F110QP_SEG_CASE
  switch (lane_qps_per_wave(B, lw.qpw)) {
    case 1: return launch_lq<1>(P, B, x0, ul, xr, uo, xo, st, its, ws, lw, oo, s);
    case 2: return launch_lq<2>(P, B, x0, ul, xr, uo, xo, st, its, ws, lw, oo, s);
    case 4: return launch_lq<4>(P, B, x0, ul, xr, uo, xo, st, its, ws, lw, oo, s);
    case 8: return launch_lq<8>(P, B, x0, ul, xr, uo, xo, st, its, ws, lw, oo, s);
    case 16: return launch_lq<16>(P, B, x0, ul, xr, uo, xo, st, its, ws, lw, oo, s);
    case 32: return launch_lq<32>(P, B, x0, ul, xr, uo, xo, st, its, ws, lw, oo, s);
    default: return launch_lq<64>(P, B, x0, ul, xr, uo, xo, st, its, ws, lw, oo, s);
  }
}

}  // namespace f110qp

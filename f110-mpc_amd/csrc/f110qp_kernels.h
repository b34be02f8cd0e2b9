// f110qp_kernels.h — internal launch interface between the C ABI (f110qp_api.cpp) and the
// gfx950 kernels (f110qp_kernels.hip, halfspace_kernels.hip). Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>

namespace f110qp {

// per-QP status ids (== F110QP_* in include/f110qp.h)
constexpr int F110QP_SOLVED_ID = 1;
constexpr int F110QP_SOLVED_INACCURATE_ID = 2;
constexpr int F110QP_MAX_ITER_ID = -2;
constexpr int F110QP_PRIMAL_INFEASIBLE_ID = -3;
constexpr int F110QP_NUMERICAL_ID = -10;

// Kernel-side copy of f110qp_config (passed by value in kernarg memory).
struct KParams {
  int N;          // horizon
  float dt;       // MPC::dt_ (float)
  double q[3];    // diag Q
  double r[2];    // diag R
  double udes[2]; // desired input
  float umin[2];  // input lower bounds
  float umax[2];  // input upper bounds
  int max_iter;   // active-set iteration cap
  int xr_stride;  // points per QP in x_ref (>= N; the reference passes its whole miniPath)
  int pdas_max;   // PDAS passes of the wave kernel's box path before its GI loop takes over
  int pass_cap = 0;  // lane kernels: passes per launch (0: max_iter; measurement knob F110QP_LANE_PASSCAP)
  int gap_first = 1;  // wave GI with gap rows: a violated gap row is added before any box row
};

// Warm-start state of a context (all null = cold solve). Per QP slot b of the batch:
//   W[b]   the cached W = H^-1 (2N x 2N, fp32) of the last solve of slot b,
//   key[b] the float bits of (theta0, v_lin, delta_lin) it was built for + a valid flag,
//   act[b] the active bounds at the last solution, per register row r of the lane map
//          (R = ceil(2N/64) rows): bit lane of act[2(R b + r)] lower, act[2(R b + r) + 1] upper.
// H depends only on the linearisation point (model.cpp:30-59), so a key hit reuses W exactly.
// Grouped mode (f110qp_solve_grouped*) reuses W/key as a per-GROUP cache instead: group[b] in
// [0, ngroups) names QP b's scenario, a prepare launch fills W[g]/key[g] from one member of each
// group, and every QP whose (theta0, v_lin, delta_lin) bits match its group's key skips the
// Hessian and the inverse (a QP that does not match builds its own: grouping never changes a
// result, the group's W is bit-identical to the one the QP would build).
struct WarmState {
  float* W = nullptr;
  unsigned* key = nullptr;
  unsigned long long* act = nullptr;
  const int* group = nullptr;
  int ngroups = 0;
  // lane back ends: the context's call counter (from 1) and a device int holding the last call in
  // which a wave saw a key hit (see warm_traffic)
  unsigned* hit_call = nullptr;
  unsigned call = 0;  // wraps after 2^32 calls: compared by unsigned difference only
  // lane back ends: cumulative counters per wave w (f110qp_warm_hits), stats[2w] QPs whose key hit,
  // stats[2w + 1] calls that moved warm traffic; read and written by the wave itself, only in a
  // call that moves the traffic
  unsigned* stats = nullptr;
};

// Whether a lane-back-end wave moves warm-start traffic in this call (loads its QPs' keys and masks,
// writes them back). On the closed-loop stream (configs[4]) theta0 changes every tick, so no key
// ever hits, and that traffic measured 0.7 us per call (0.55 the write-back, 0.15 the key loads:
// C5 kernel 29.2 against 28.5 cold). It runs while a hit was seen within the last kWarmRecent
// calls, and on two probe calls in every kWarmProbe (the first writes keys, the second can hit),
// so a stream whose linearisation points repeat turns it back on within kWarmProbe calls. Without
// hit_call (grouped / wave paths): always.
constexpr int kWarmRecent = 2, kWarmProbe = 32;
__device__ __forceinline__ unsigned warm_last_hit(const WarmState& ws) {  // load early, test late
  return ws.hit_call ? __builtin_nontemporal_load(ws.hit_call) : 0u;
}
__device__ __forceinline__ bool warm_traffic(const WarmState& ws, unsigned last) {
  if (!ws.act || !ws.key) return false;
  if (!ws.hit_call) return true;
  return ws.call - last <= (unsigned)kWarmRecent || ws.call % (unsigned)kWarmProbe <= 1u;
}

// LaneWork::hand for a call of B gap-row QPs: kHandInts(B) = 3 B + 4 ints, the two counts first
// (padded to four ints), then three B-int arrays.
struct HandLayout {
  int* c_list;  // [0] the screen's GI list count
  int* c_rc;    // [1] the fp64 re-check's count (the wave kernel appends its non-SOLVED QPs)
  int* list;    // [4, 4 + B) the screen's GI list, heavy first
  int* prio;    // [4 + B, 4 + 2B) screen: GI priority per QP
  int* rc;      // [4 + 2B, 4 + 3B) the re-check list
  HandLayout(int* h, int B)
      : c_list(h), c_rc(h + 1), list(h + 4), prio(h + 4 + (size_t)B), rc(h + 4 + 2 * (size_t)B) {}
};
constexpr size_t kHandInts(int B) { return 3 * (size_t)B + 4; }

// Workspace of the lane-per-QP kernel (lane_kernel.h): the HBM Riccati scratch when it does
// not stay in LDS (ceil(B/L) x N x 8 x L doubles at most, L QPs per wave <= 64).
struct LaneWork {
  double* scratch = nullptr;
  int kmax = 16;  // PDAS passes (all violations flip) before single flips (least index)
  int mode = 0;   // scratch: 0 auto, 1 LDS fp64, 2 LDS fp32, 3 HBM fp64, 4 HBM fp32 (workspace)
  int qpw = 0;    // QPs per wave: 0 auto (lane_qps_per_wave), else a power of two <= 64
  int rot = 1;    // 1: heading-frame kernel when q0 == q1 (lane_kernel.h ROT); 0: general frame
  int dref = 1;   // 1: fp64 references in LDS when the resident waves fit (DREF); 0: float
  int seg = 0;    // horizon segments per QP (lane_seg_kernel.h): 0 auto, 1 off, 2 / 4 / 8 forced
  int seg32 = 0;  // segmented kernel: 1 forces float references and Riccati scratch in LDS
  int twin = 1;   // segmented kernel: two PDAS starts per QP where the grid leaves SIMDs idle
  int* hand = nullptr;  // gap rows: counts + per-QP lists (HandLayout, kHandInts(B) ints)
  int screen = 0;       // gap rows: box solve on the lane kernel first, GI only for the QPs whose
                        // box optimum violates a gap row (f110qp_kernels.hip)
  int recheck_all = 0;  // gap rows, test build only: every QP through the fp64 re-check alone
};

// Optional per-QP objective outputs (fp64, computed in the kernels' output sweeps from the fp64
// solution): obj[b] = OSQP's objective 1/2 z'Pz + q'z of the reference QP (mpc.cpp:208-229;
// OSQP drops the constant), cost[b] = the same plus that constant
// 1/2 sum_i r_i'Q r_i + N/2 u_des'R u_des, i.e. sum 1/2|x_i - r_i|_Q^2 + 1/2|u_i - u_des|_R^2 >= 0.
struct ObjOut {
  double* obj = nullptr;
  double* cost = nullptr;
  // gap-row box screen fused into the segmented lane kernel's output sweep (f110qp_kernels.hip):
  // the half-spaces, and per QP the GI priority it writes (0: the box optimum stands; else 1 + the
  // gap rows it violates; null: no screen)
  const float* scr_hs = nullptr;
  int* scr_prio = nullptr;
  // wave kernel, gap rows: QPs it does not report SOLVED are appended here for the fp64 re-check
  // (count + list; null: the re-check flags them itself)
  int* rc_count = nullptr;
  int* rc_list = nullptr;
  // completion signal of a synchronous call, raised by its last kernel (signal_call_done): every
  // workgroup arrives on sig_count once its stores are visible at system scope; the last one
  // re-zeroes the count and writes sig_seq to sig_host (the pinned host word the calling thread
  // polls). null: none
  unsigned* sig_host = nullptr;
  unsigned* sig_count = nullptr;
  unsigned sig_seq = 0;
};

// whether launch_solve's kernels for this call raise ObjOut's completion signal (every ungrouped
// call: its last kernel is a lane, wave or re-check kernel that signals); the caller synchronises
// the stream otherwise
bool launch_signals(const KParams& P, int B, int backend, const float* hs, const LaneWork& lw);

// The completion signal at the very end of a call's last kernel (ObjOut::sig_*): every wave's
// stores visible at system scope (zero-copy outputs in pinned host memory; device outputs written
// back from this XCD's L2), then one arrival per workgroup (after a barrier when it has several
// waves); the last arrival re-zeroes the count for the next call and publishes the call's number
// to the host word the caller polls (f110qp_api.cpp wait_done). Every workgroup must reach it; one
// that stored nothing (wrote = false: a re-check workgroup past the list) skips the fence, whose L2
// write-back walk is what makes a burst of them costly.
__device__ __forceinline__ void signal_call_done(const ObjOut& oo, bool wrote = true) {
  if (!oo.sig_host) return;
  if (wrote) __threadfence_system();
  if (blockDim.x > 64) __syncthreads();
  if (threadIdx.x != 0) return;
  if (gridDim.x == 1) {  // one workgroup: no arrival count to go through
    __hip_atomic_store(oo.sig_host, oo.sig_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  const unsigned arrived = __hip_atomic_fetch_add(oo.sig_count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
  if (arrived + 1u == gridDim.x) {
    __hip_atomic_store(oo.sig_count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(oo.sig_host, oo.sig_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// waves the lane kernel's grid aims for (one per CU of the MI355X's 256)
constexpr int kLaneTargetWaves = 256;
int lane_qps_per_wave(int B, int qpw);
// scratch placement the lane launch picks for a batch: 1 LDS fp64, 2 LDS fp32, 3 HBM fp64, 4 HBM fp32
int lane_scratch_mode(const KParams& P, int B, const LaneWork& lw);
// horizon segments per QP the lane launch picks for a batch (1 = lane_kernel.h, one QP per lane
// group of 64 / L identical lanes; S > 1 = lane_seg_kernel.h, 64 / S QPs per wave)
int lane_segments(const KParams& P, int B, const LaneWork& lw);
// scratch of the segmented kernel at S segments: 1 LDS fp64, 2 LDS fp32 (lane_seg_kernel.h)
int lane_seg_scratch(const KParams& P, int B, int S, const LaneWork& lw);
// PDAS starts per QP of the segmented kernel at S segments: 2 with the twin start (lane_seg_kernel.h)
int lane_seg_starts(const KParams& P, int B, int S, const LaneWork& lw);

// fp64 re-check of the gap-row QPs the wave kernel did not report SOLVED (its certificate
// failed, or GI ended infeasible / at its cap): the fp64 Goldfarb-Idnani of gi64_kernel.h over
// the device-side list (count, list: HandLayout c_rc / rc), every listed QP, its outputs rewritten.
hipError_t launch_gap_recheck(const KParams& P, int B, const float* x0, const float* u_lin,
                              const float* x_ref, const float* hs, float* u_out, float* x_out,
                              int* status, int* iters, const int* list, const int* count,
                              const ObjOut& oo, hipStream_t stream);

enum Backend { BACKEND_WAVE = 0, BACKEND_LANE = 1 };

// Solve B QPs. hs == nullptr -> box-only kernels (gap rows inactive). backend LANE: box rows, the
// lane-per-QP Riccati/PDAS kernel alone (one launch, no hand-over). Gap rows: lw.screen, the box
// solve on the lane kernel, GI for the QPs whose box optimum violates a gap row; else GI for every
// QP; then the fp64 re-check of what GI did not certify.
hipError_t launch_solve(const KParams& P, int B, const float* x0, const float* u_lin,
                        const float* x_ref, const float* hs, float* u_out, float* x_out,
                        int* status, int* iters, const WarmState& warm, int backend,
                        const LaneWork& lw, const ObjOut& oo, hipStream_t stream);

// The lane-per-QP kernel alone (box rows).
hipError_t launch_lane(const KParams& P, int B, const float* x0, const float* u_lin,
                       const float* x_ref, float* u_out, float* x_out, int* status, int* iters,
                       const WarmState& warm, const LaneWork& lw, const ObjOut& oo,
                       hipStream_t stream);

// Grouped solve: leader (smallest member) of every group, W = H^-1 per group from its leader,
// then the solve (wave back end; the lane back end has no factor to share and ignores groups).
// ws.W/ws.key hold ngroups slots, leader ngroups ints.
hipError_t launch_solve_grouped(const KParams& P, int B, const float* x0, const float* u_lin,
                                const float* x_ref, const float* hs, float* u_out, float* x_out,
                                int* status, int* iters, const WarmState& gws, int* leader,
                                int backend, const LaneWork& lw, const ObjOut& oo,
                                hipStream_t stream);

// Per-scenario selection (the argmin of src/project.cpp:125-136 taken over the
// QP costs): winner[g] = the smallest b with group[b] == g, status[b] == SOLVED and the minimal
// cost[b]; -1 when the group has no solved member. best[g] = that cost (+inf if none).
hipError_t launch_select(int B, const int* group, int G, const double* cost, const int* status,
                         int* winner, double* best, hipStream_t stream);

// Dump the condensed H (B x 2N x 2N) and g (B x 2N) as built by the solve kernel.
hipError_t launch_condense_debug(const KParams& P, int B, const float* x0, const float* u_lin,
                                 const float* x_ref, double* H, double* g, hipStream_t stream);

// One instance's (P, q, A, l, u) in the reference's CSC layout (assemble_kernel.hip).
hipError_t launch_assemble(const KParams& P, const float* x0, const float* u_lin, const float* x_ref,
                           const float* hs, int gap_active, int* Pc, int* Pr, double* Pv, double* q,
                           int* Ac, int* Ar, double* Av, double* l, double* u, hipStream_t stream);

// Planning stage (plan_kernels.hip): grid size, candidate count / length, float params.
struct PlanKParams {
  int G;            // grid_blocks_ = size_ / discrete_
  int T;            // candidates (steer_discrete + 1)
  int P;            // points per candidate (traj_discrete)
  float discrete;   // occ_discrete
  float dilation;   // occ_dilation
  float lookahead;  // Trajectory::lookahead
};

hipError_t launch_plan(const PlanKParams& K, int B, const double* pose, const float* ranges,
                       int nr, float angle_min, float angle_inc, float angle_max,
                       const double* table, const double* wp, int W, unsigned char* grid_out,
                       unsigned char* valid_out, int* best_global, int* best_traj, float* x_ref,
                       float* x0, int* status, hipStream_t stream);

// Batched FindHalfSpaces (constraints.cpp:116-265), one wave per scan.
hipError_t launch_half_spaces(int B, const float* states, const float* ranges, int num_ranges,
                              float angle_min, float angle_inc, float angle_max, float thresh,
                              float divider, float buffer, float* hs, int* gap_lo, int* gap_hi,
                              hipStream_t stream);

}  // namespace f110qp

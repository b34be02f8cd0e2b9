// f110qp_api.cpp — the C ABI (include/f110qp.h) over the gfx950 kernels.
//
// Host-side responsibilities only: argument validation, the device workspace of a context,
// H2D/D2H for the host-pointer entry points, and Constraints::FindHalfSpaces for one scan
// (reference src/constraints.cpp:116-265) for callers that hold a single LaserScan.
// No C++ exception crosses this boundary.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "f110qp.h"
#include "f110qp_kernels.h"

namespace {

thread_local std::string g_last_error = "";

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  return fail(F110QP_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

// Device buffer that only grows (freed with its owner).
struct DevBuf {
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  void* p = nullptr;
  size_t bytes = 0;
  hipError_t ensure(size_t n) {
    if (n <= bytes) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    hipError_t e = hipMalloc(&p, n);
    if (e == hipSuccess) bytes = n;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
};

// Pinned, device-visible (fine-grained, coherent) host buffer that only grows.
struct HostBuf {
  HostBuf() = default;
  HostBuf(const HostBuf&) = delete;
  HostBuf& operator=(const HostBuf&) = delete;
  ~HostBuf() { release(); }
  void* p = nullptr;  // host address
  void* d = nullptr;  // device address of the same memory
  size_t bytes = 0;
  hipError_t ensure(size_t n) {
    if (n <= bytes) return hipSuccess;
    release();
    hipError_t e = hipHostMalloc(&p, n, hipHostMallocCoherent | hipHostMallocMapped);
    if (e != hipSuccess) { p = nullptr; return e; }
    e = hipHostGetDevicePointer(&d, p, 0);
    if (e != hipSuccess) { release(); return e; }
    bytes = n;
    return hipSuccess;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = d = nullptr;
    bytes = 0;
  }
};

// Host-pointer calls of up to this many QPs (the per-tick call of the host MPC class) let the
// kernel read its inputs from and write its outputs to the pinned staging buffers directly
// (zero-copy over PCIe): one launch and one synchronisation per call, no copy engine.
constexpr int kZeroCopyMaxBatch = 64;

}  // namespace

struct f110qp_ctx {
  f110qp_config cfg;
  f110qp::KParams kp;
  HostBuf hin, hout;  // host-pointer entry point: packed pinned staging [x0|u_lin|x_ref|hs], [u|x|st|it]
  DevBuf din, dout;   // their device copies for batches above kZeroCopyMaxBatch
  DevBuf wW, wkey, wact;  // warm-start slot state (config.warm_start)
  int warm_batch = 0;     // batch size the warm state was laid out for
  unsigned warm_calls = 0;  // warm calls since the state was laid out (WarmState::call, wraps)
  unsigned warm_prev[2] = {0u, 0u};  // the counters at the last f110qp_warm_hits
  hipStream_t warm_stream = nullptr;  // stream of the last warm call
  DevBuf gW, gkey, glead;    // grouped mode: W = H^-1, key and leader per group
  DevBuf dgrp;               // host-pointer grouped calls: device copy of the group ids
  DevBuf lscr;               // lane back end: HBM Riccati scratch (when not in LDS)
  DevBuf hand;               // gap rows: counts and lists (f110qp::HandLayout, kHandInts(B) ints)
  int lane_kmax = 16;        // lane back end: PDAS passes before single (least-index) flips
  int lane_mode = 0;         // lane scratch placement (LaneWork::mode)
  int lane_qpw = 0;          // lane QPs per wave (LaneWork::qpw, 0 = auto)
  int lane_rot = 1;          // lane heading-frame kernel when q0 == q1 (LaneWork::rot)
  int lane_dref = 1;         // lane fp64 references in LDS when they fit (LaneWork::dref)
  int lane_seg = 0;          // lane horizon segments per QP (LaneWork::seg: 0 auto, 1 off, 2/4/8)
  int lane_seg32 = 0;        // segmented kernel: force fp32 references + scratch (LaneWork::seg32)
  int lane_twin = 1;         // segmented kernel: twin PDAS starts where they fit (LaneWork::twin)
  int gap_screen = -1;      // gap rows, AUTO: box screen on the lane kernel (-1 by batch, 0 off, 1 on)
  int recheck_all = 0;      // gap rows: every QP of a call through the fp64 re-check alone (test build)
  HostBuf hsig;              // synchronous calls: the completion word they poll (wait_done)
  DevBuf dsig;               // its kernel's wave arrival count (zeroed once, re-zeroed by the kernel)
  unsigned sig_seq = 0;      // number of the last signalled call (the value the kernel publishes)
  int sig_poll = 1;          // 0: synchronous calls synchronise the stream (test build, F110QP_SIG_POLL=0)
  hipStream_t stream = nullptr;
  hipStream_t last_gap_stream = nullptr;  // stream of the last gap-row call (f110qp_last_recheck_count)
  int last_gap_batch = 0;                 // its batch (0: no gap-row call yet)
};

#ifdef F110QP_TEST_HOOKS
// Test / measurement build only (lib_test/libf110qp.so, -DF110QP_TEST_HOOKS): create-time knobs read
// from the environment that force one kernel variant or rule of the dispatch, so the tests reach every
// code path AUTO does not pick at their sizes. The product library (lib/libf110qp.so) reads no
// environment variable: its behaviour is the config alone (the reference's solver settings are fixed
// in code, src/mpc.cpp:98-99).
static int env_int(const char* name, int lo, int hi, int* out) {
  const char* e = std::getenv(name);
  if (!e) return 0;
  const int v = std::atoi(e);
  if (v < lo || v > hi) return 0;
  *out = v;
  return 1;
}

static void test_hooks(f110qp_ctx* c) {
  // PDAS passes of the lane back end before single least-index flips (0: single flips from pass 1)
  env_int("F110QP_LANE_KMAX", 0, 64, &c->lane_kmax);
  // QPs per wave of the lane back end (power of two <= 64)
  int v;
  if (env_int("F110QP_LANE_QPW", 1, 64, &v) && (v & (v - 1)) == 0) c->lane_qpw = v;
  // lane scratch: 1 LDS fp64, 2 LDS fp32, 3 HBM fp64, 4 HBM fp32
  env_int("F110QP_LANE_MODE", 0, 4, &c->lane_mode);
  // 0: general-frame lane kernel even when q0 == q1
  if (env_int("F110QP_LANE_ROT", 0, 1, &v)) c->lane_rot = v;
  // 0: float references in LDS (no fp64 DREF array)
  if (env_int("F110QP_LANE_DREF", 0, 1, &v)) c->lane_dref = v;
  // horizon segments per QP (0 auto, 1 off, 2 / 4 / 8 forced where the horizon and the LDS allow)
  if (env_int("F110QP_LANE_SEG", 0, 8, &v) && (v == 0 || v == 1 || v == 2 || v == 4 || v == 8)) c->lane_seg = v;
  // 1: the segmented kernel's float references and scratch
  if (env_int("F110QP_LANE_SEG_F32", 0, 1, &v)) c->lane_seg32 = v;
  // 0: one PDAS start per QP in the segmented kernel (the twin start off)
  if (env_int("F110QP_LANE_TWIN", 0, 1, &v)) c->lane_twin = v;
  // gap rows: the box screen on (1) / off (0) at every batch size
  if (env_int("F110QP_GAP_SCREEN", 0, 1, &v)) c->gap_screen = v;
  // wave GI: 0 picks gap and box candidates by one ranking
  if (env_int("F110QP_GI_GAPFIRST", 0, 1, &v)) c->kp.gap_first = v;
  // lane kernels: PDAS passes per launch (measurement of the pass distribution: MAX_ITER past it)
  env_int("F110QP_LANE_PASSCAP", 1, 999, &c->kp.pass_cap);
  // wave kernel's box PDAS passes (0: GI from the unconstrained point)
  env_int("F110QP_PDAS_MAX", 0, 64, &c->kp.pdas_max);
  // gap rows: every QP of a call through the fp64 re-check (gi64_kernel.h) alone, no screen and no
  // fp32 GI: the re-check's own answers, for its parity tests
  if (env_int("F110QP_RECHECK_ALL", 0, 1, &v)) c->recheck_all = v;
  // 0: synchronous calls wait with hipStreamSynchronize, not on the kernel's completion word
  if (env_int("F110QP_SIG_POLL", 0, 1, &v)) c->sig_poll = v;
}
#endif

// Synchronous calls whose work is one kernel that raises the completion signal (f110qp::launch_signals:
// the box-only solve on the segmented lane kernel, the per-tick call) wait for that kernel's last
// wave to write the call's number to a pinned host word instead of synchronising the stream: the
// hipStreamSynchronize round trip measured 12.2 us p50 against 6.5 us for the polled word on an
// empty kernel (tools/microbench/flag_latency.hip). Arms the signal in *oo when the
// call's kernels raise it; *armed false: the caller synchronises the stream.
static int arm_signal(f110qp_ctx* c, int batch, int backend, const float* h, const f110qp::LaneWork& lw,
                      hipStream_t s, f110qp::ObjOut* oo, bool* armed) {
  *armed = false;
  if (!c->sig_poll || !f110qp::launch_signals(c->kp, batch, backend, h, lw)) return F110QP_OK;
  if (!c->hsig.p) {
    hipError_t e = c->hsig.ensure(64);
    if (e != hipSuccess) return hip_fail(e, "hipHostMalloc completion word");
    if ((e = c->dsig.ensure(64)) != hipSuccess) return hip_fail(e, "hipMalloc arrival count");
    if ((e = hipMemsetAsync(c->dsig.p, 0, 64, s)) != hipSuccess) return hip_fail(e, "hipMemsetAsync arrival count");
    __atomic_store_n((unsigned*)c->hsig.p, c->sig_seq, __ATOMIC_RELEASE);
  }
  oo->sig_host = (unsigned*)c->hsig.d;
  oo->sig_count = (unsigned*)c->dsig.p;
  oo->sig_seq = ++c->sig_seq;
  *armed = true;
  return F110QP_OK;
}

// Waits for the call armed by arm_signal (or synchronises the stream when it was not armed). The
// poll reads only the word (a hipStreamQuery inside the usual 10-15 us wait delayed the answer by
// its own cost and made the call bimodal); after kPollWindow it hands over to hipStreamSynchronize,
// so a stalled call does not keep a core spinning and a kernel that faults (no word) is reported by
// its HIP error (a gap-row call of 256 QPs, ~245 us, lost 7 us when the hand-over came at 200 us).
// A drained stream without the word is an error, not a wait.
constexpr auto kPollWindow = std::chrono::microseconds(1000);
static int wait_done(f110qp_ctx* c, hipStream_t s, bool armed) {
  if (armed) {
    const unsigned seq = c->sig_seq;
    const unsigned* w = (const unsigned*)c->hsig.p;
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned k = 1;; k++) {
      if (__atomic_load_n(w, __ATOMIC_ACQUIRE) == seq) return F110QP_OK;
      if ((k & 255u) == 0 && std::chrono::steady_clock::now() - t0 > kPollWindow) break;
      __builtin_ia32_pause();
    }
  }
  const hipError_t e = hipStreamSynchronize(s);
  if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
  if (armed && __atomic_load_n((const unsigned*)c->hsig.p, __ATOMIC_ACQUIRE) != c->sig_seq)
    return fail(F110QP_ERR_HIP, "solve kernel finished without its completion signal");
  return F110QP_OK;
}

extern "C" {

int f110qp_version(void) { return F110QP_API_VERSION; }

const char* f110qp_last_error(void) { return g_last_error.c_str(); }

void f110qp_default_config(f110qp_config* c, int horizon) {
  if (!c) return;
  std::memset(c, 0, sizeof(*c));
  c->horizon = horizon;  // params.yaml:12 (reference default 30)
  c->dt = 0.01f;         // params.yaml:13
  c->q[0] = 10.0; c->q[1] = 10.0; c->q[2] = 0.0;  // params.yaml:1-3
  c->r[0] = 0.10; c->r[1] = 5.0;                  // params.yaml:5-6
  c->u_des[0] = 4.5; c->u_des[1] = 0.0;           // params.yaml:42-43
  c->u_min[0] = 3.0f; c->u_min[1] = -0.43f;       // params.yaml:47, constraints.cpp:21
  c->u_max[0] = 4.5f; c->u_max[1] = 0.43f;        // params.yaml:46, constraints.cpp:19
  c->gap_mode = F110QP_GAP_INACTIVE;
  c->max_iter = 0;
  c->device = 0;
  c->warm_start = 0;
  c->backend = F110QP_BACKEND_AUTO;
  c->x_ref_points = 0;
}

static int validate_config(const f110qp_config* c) {
  if (!c) return fail(F110QP_ERR_INVALID, "config is NULL");
  if (c->horizon < 1 || c->horizon > F110QP_MAX_HORIZON)
    return fail(F110QP_ERR_INVALID, "horizon must be in [1, 48] (one wave holds 2N inputs in <= 2 register rows)");
  if (!(c->dt > 0.f) || !std::isfinite(c->dt)) return fail(F110QP_ERR_INVALID, "dt must be > 0");
  for (int i = 0; i < 3; i++)
    if (!(c->q[i] >= 0.0)) return fail(F110QP_ERR_INVALID, "Q must be >= 0");
  for (int i = 0; i < 2; i++) {
    if (!(c->r[i] > 0.0)) return fail(F110QP_ERR_INVALID, "R must be > 0 (strictly convex QP)");
    if (!(c->u_min[i] <= c->u_max[i])) return fail(F110QP_ERR_INVALID, "u_min > u_max");
  }
  if (c->gap_mode != F110QP_GAP_INACTIVE && c->gap_mode != F110QP_GAP_ACTIVE)
    return fail(F110QP_ERR_INVALID, "gap_mode must be 0 (gap rows inactive) or 1 (active)");
  if (c->max_iter < 0) return fail(F110QP_ERR_INVALID, "max_iter must be >= 0");
  if (c->warm_start != 0 && c->warm_start != 1) return fail(F110QP_ERR_INVALID, "warm_start must be 0 or 1");
  if (c->x_ref_points != 0 && c->x_ref_points < c->horizon)
    return fail(F110QP_ERR_INVALID, "x_ref_points must be 0 (= horizon) or >= horizon");
  if (c->backend < F110QP_BACKEND_AUTO || c->backend > F110QP_BACKEND_LANE)
    return fail(F110QP_ERR_INVALID, "backend must be 0 (auto), 1 (wave) or 2 (lane)");
  return F110QP_OK;
}

int f110qp_create(f110qp_ctx** out, const f110qp_config* cfg) {
  if (!out) return fail(F110QP_ERR_INVALID, "ctx out-pointer is NULL");
  *out = nullptr;
  int rc = validate_config(cfg);
  if (rc) return rc;
  f110qp_ctx* c = new (std::nothrow) f110qp_ctx();
  if (!c) return fail(F110QP_ERR_ALLOC, "out of host memory");
  c->cfg = *cfg;
  f110qp::KParams& k = c->kp;
  k.N = cfg->horizon;
  k.dt = cfg->dt;
  for (int i = 0; i < 3; i++) k.q[i] = cfg->q[i];
  for (int i = 0; i < 2; i++) {
    k.r[i] = cfg->r[i];
    k.udes[i] = cfg->u_des[i];
    k.umin[i] = cfg->u_min[i];
    k.umax[i] = cfg->u_max[i];
  }
  k.pdas_max = 10;
#ifdef F110QP_TEST_HOOKS
  test_hooks(c);
#endif
  const int nu = 2 * cfg->horizon;
  k.max_iter = cfg->max_iter > 0 ? cfg->max_iter : 8 * (nu + (cfg->gap_mode ? nu : 0)) + 16;
  k.xr_stride = cfg->x_ref_points > 0 ? cfg->x_ref_points : cfg->horizon;
  *out = c;
  return F110QP_OK;
}

void f110qp_destroy(f110qp_ctx* c) {
  if (!c) return;
  // a synchronous call returns on its completion word while its kernel may still be retiring: let
  // it finish before the word and the arrival count are freed (the caller's stream may be gone)
  if (c->sig_seq) (void)hipDeviceSynchronize();
  c->hsig.release(); c->dsig.release();
  c->hin.release(); c->hout.release(); c->din.release(); c->dout.release();
  c->wW.release(); c->wkey.release(); c->wact.release();
  c->lscr.release();
  c->hand.release();
  c->gW.release(); c->gkey.release(); c->glead.release(); c->dgrp.release();
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

static int check_batch_args(f110qp_ctx* c, int batch, const void* x0, const void* ul,
                            const void* xr, const void* hs, const void* uo, const void* xo,
                            const void* st) {
  if (!c) return fail(F110QP_ERR_INVALID, "ctx is NULL");
  if (batch < 0) return fail(F110QP_ERR_INVALID, "batch < 0");
  if (batch == 0) return F110QP_OK;
  if (!x0 || !ul || !xr || !uo || !xo || !st)
    return fail(F110QP_ERR_INVALID, "x0/u_lin/x_ref/u_out/x_out/status must be non-NULL");
  if (c->cfg.gap_mode == F110QP_GAP_ACTIVE && !hs)
    return fail(F110QP_ERR_INVALID, "gap_mode ACTIVE needs the halfspace array");
  if (batch > (1 << 30) / 64) return fail(F110QP_ERR_INVALID, "batch too large");
  return F110QP_OK;
}

// Warm-start slot state for a batch of `batch` QPs (allocated and zeroed on first use and
// whenever the batch size changes; zero keys = no valid entry).
static int warm_state(f110qp_ctx* c, int batch, hipStream_t s, f110qp::WarmState* ws) {
  *ws = f110qp::WarmState();
  if (!c->cfg.warm_start) return F110QP_OK;
  const size_t B = (size_t)batch, nu = 2 * (size_t)c->cfg.horizon;
  const size_t rows = (nu + 63) / 64;  // register rows per lane (act masks: 2 x 64 bits per row)
  hipError_t e;
  // keys (16 B per QP), then the lane back ends' last-hit call (warm_traffic) and the cumulative
  // traffic-call and hit counters (f110qp_warm_hits)
  const size_t wbytes = B * 16 + 16 + 8 * (B + 1);  // keys, last-hit call, per-wave counters
  if ((e = c->wW.ensure(B * nu * nu * 4)) || (e = c->wkey.ensure(wbytes)) ||
      (e = c->wact.ensure(B * 16 * rows)))
    return hip_fail(e, "hipMalloc warm-start state");
  if (c->warm_batch != batch) {
    if ((e = hipMemsetAsync(c->wkey.p, 0, wbytes, s)) || (e = hipMemsetAsync(c->wact.p, 0, B * 16 * rows, s)))
      return hip_fail(e, "hipMemsetAsync warm-start state");
    c->warm_batch = batch;
    c->warm_calls = 0;
    c->warm_prev[0] = c->warm_prev[1] = 0;
  }
  ws->W = (float*)c->wW.p;
  ws->key = (unsigned*)c->wkey.p;
  ws->act = (unsigned long long*)c->wact.p;
  ws->hit_call = (unsigned*)((char*)c->wkey.p + B * 16);
  ws->stats = (unsigned*)((char*)c->wkey.p + B * 16 + 16);  // per wave: hits, traffic calls
  ws->call = ++c->warm_calls;
  c->warm_stream = s;
  return F110QP_OK;
}

// The back end a call of `batch` QPs runs on (what AUTO resolves to). Box rows: the lane back end
// from F110QP_LANE_MIN_BATCH[_WIDE]. Gap rows: the wave kernel's GI (AUTO, WAVE), behind the box
// screen on the lane kernel for AUTO batches >= F110QP_GAP_SCREEN_MIN_BATCH; LANE: the box screen
// on the lane kernel for every batch (GI for the QPs it does not clear).
static int resolve_backend(f110qp_ctx* c, int batch, bool grouped) {
  const bool gap = c->cfg.gap_mode == F110QP_GAP_ACTIVE;
  int be = c->cfg.backend;
  if (gap)  // LANE: the screen path (never grouped or warm-started: those run GI on the wave kernel)
    return be == F110QP_BACKEND_LANE && !grouped && !c->cfg.warm_start ? F110QP_BACKEND_LANE : F110QP_BACKEND_WAVE;
  if (be == F110QP_BACKEND_AUTO) {
    const int min_b = grouped ? (c->cfg.horizon <= 32 ? F110QP_LANE_MIN_BATCH_GROUPED
                                                      : F110QP_LANE_MIN_BATCH_GROUPED_WIDE)
                              : (c->cfg.horizon <= 32 ? F110QP_LANE_MIN_BATCH : F110QP_LANE_MIN_BATCH_WIDE);
    const bool small = !grouped && c->cfg.horizon <= 32 && batch <= F110QP_LANE_MAX_SMALL_BATCH;
    be = (batch >= min_b || small) ? F110QP_BACKEND_LANE : F110QP_BACKEND_WAVE;
  }
  return be;
}

// Gap rows: does the call take the box screen on the lane kernel first (backend LANE, or AUTO from
// F110QP_GAP_SCREEN_MIN_BATCH; ungrouped, no warm-start state)?
static bool gap_screen(const f110qp_ctx* c, int batch, bool grouped) {
  if (c->cfg.gap_mode != F110QP_GAP_ACTIVE || grouped || c->cfg.warm_start) return false;
  if (c->cfg.backend == F110QP_BACKEND_LANE) return true;
  if (c->cfg.backend != F110QP_BACKEND_AUTO || c->gap_screen == 0) return false;
  return c->gap_screen == 1 || batch >= F110QP_GAP_SCREEN_MIN_BATCH;
}

// Back end of a call and, for the lane back end (or the gap screen), its workspace.
static int lane_work(f110qp_ctx* c, int batch, hipStream_t s, int* backend, f110qp::LaneWork* lw,
                     bool grouped = false) {
  *lw = f110qp::LaneWork();
  lw->kmax = c->lane_kmax;
  lw->mode = c->lane_mode;
  lw->qpw = c->lane_qpw;
  lw->rot = c->lane_rot;
  lw->dref = c->lane_dref;
  lw->seg = c->lane_seg;
  lw->seg32 = c->lane_seg32;
  lw->twin = c->lane_twin;
  *backend = resolve_backend(c, batch, grouped) == F110QP_BACKEND_LANE ? f110qp::BACKEND_LANE
                                                                      : f110qp::BACKEND_WAVE;
  hipError_t e;
  if (c->cfg.gap_mode == F110QP_GAP_ACTIVE) {
    // counts and lists of the screen's GI list and of the fp64 re-check
    if ((e = c->hand.ensure(f110qp::kHandInts(batch) * sizeof(int))) != hipSuccess)
      return hip_fail(e, "hipMalloc gap-row lists");
    lw->hand = (int*)c->hand.p;
    lw->recheck_all = c->recheck_all;
    lw->screen = gap_screen(c, batch, grouped) && !c->recheck_all;
    c->last_gap_stream = s;
    c->last_gap_batch = batch;
    if (!lw->screen) return F110QP_OK;
  } else if (*backend == f110qp::BACKEND_WAVE) {
    return F110QP_OK;
  }
  // HBM scratch of ceil(B/L) waves x N stages x 8 values x L lanes (<= (B + 63) x N x 8 doubles)
  const size_t N = (size_t)c->cfg.horizon;
  e = c->lscr.ensure(((size_t)batch + 63) * N * 8 * sizeof(double));
  if (e != hipSuccess) return hip_fail(e, "hipMalloc lane workspace");
  lw->scratch = (double*)c->lscr.p;
  return F110QP_OK;
}

int f110qp_last_recheck_count(f110qp_ctx* c, int* count) {
  if (!c || !count) return fail(F110QP_ERR_INVALID, "ctx / count is NULL");
  *count = 0;
  if (c->cfg.gap_mode != F110QP_GAP_ACTIVE || c->last_gap_batch == 0 || !c->hand.p) return F110QP_OK;
  hipError_t e = hipStreamSynchronize(c->last_gap_stream);
  if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
  const f110qp::HandLayout H((int*)c->hand.p, c->last_gap_batch);
  if ((e = hipMemcpy(count, H.c_rc, sizeof(int), hipMemcpyDeviceToHost)) != hipSuccess)
    return hip_fail(e, "hipMemcpy re-check count");
  return F110QP_OK;
}

int f110qp_warm_hits(f110qp_ctx* c, int* traffic, int* hits) {
  if (!c || !traffic || !hits) return fail(F110QP_ERR_INVALID, "ctx / traffic / hits is NULL");
  *traffic = 0;
  *hits = 0;
  if (!c->cfg.warm_start || c->warm_batch == 0 || !c->wkey.p) return F110QP_OK;
  hipError_t e = hipStreamSynchronize(c->warm_stream);
  if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
  // per-wave counters (hits, traffic calls) of every wave of the lane launches: every wave of a call
  // counts the same traffic, wave 0 is the call's count; the hits sum over the waves
  const size_t nw = (size_t)c->warm_batch + 1;
  std::vector<unsigned> st(2 * nw);
  if ((e = hipMemcpy(st.data(), (char*)c->wkey.p + (size_t)c->warm_batch * 16 + 16, st.size() * sizeof(unsigned),
                     hipMemcpyDeviceToHost)))
    return hip_fail(e, "hipMemcpy warm-start counters");
  unsigned hsum = 0;
  for (size_t w = 0; w < nw; w++) hsum += st[2 * w];
  *traffic = (int)(st[1] - c->warm_prev[0]);
  *hits = (int)(hsum - c->warm_prev[1]);
  c->warm_prev[0] = st[1];
  c->warm_prev[1] = hsum;
  return F110QP_OK;
}

int f110qp_test_build(void) {
#ifdef F110QP_TEST_HOOKS
  return 1;
#else
  return 0;
#endif
}

int f110qp_sync_signals(f110qp_ctx* c, unsigned* count) {
  if (!c || !count) return fail(F110QP_ERR_INVALID, "ctx / count is NULL");
  *count = c->sig_seq;
  return F110QP_OK;
}

int f110qp_warm_reset(f110qp_ctx* c) {
  if (!c) return fail(F110QP_ERR_INVALID, "ctx is NULL");
  c->warm_batch = 0;  // the next call re-zeroes the slot keys
  return F110QP_OK;
}

int f110qp_solve_batch_dev(f110qp_ctx* c, int batch, const float* x0, const float* ul,
                           const float* xr, const float* hs, float* uo, float* xo, int* st,
                           int* it, void* stream) {
  return f110qp_solve_batch_ex_dev(c, batch, x0, ul, xr, hs, uo, xo, st, it, nullptr, nullptr, stream);
}

// device-pointer solve; sync: wait for it before returning (the completion word where the call's
// kernel raises it, else the stream)
static int solve_dev(f110qp_ctx* c, int batch, const float* x0, const float* ul, const float* xr,
                     const float* hs, float* uo, float* xo, int* st, int* it, double* obj,
                     double* cost, hipStream_t s, bool sync) {
  int rc = check_batch_args(c, batch, x0, ul, xr, hs, uo, xo, st);
  if (rc || batch == 0) return rc;
  const float* h = (c->cfg.gap_mode == F110QP_GAP_ACTIVE) ? hs : nullptr;
  f110qp::WarmState ws;
  rc = warm_state(c, batch, s, &ws);
  if (rc) return rc;
  int backend;
  f110qp::LaneWork lw;
  rc = lane_work(c, batch, s, &backend, &lw);
  if (rc) return rc;
  f110qp::ObjOut oo;
  oo.obj = obj;
  oo.cost = cost;
  bool armed = false;
  if (sync && (rc = arm_signal(c, batch, backend, h, lw, s, &oo, &armed))) return rc;
  hipError_t e = f110qp::launch_solve(c->kp, batch, x0, ul, xr, h, uo, xo, st, it, ws, backend, lw, oo, s);
  if (e != hipSuccess) return hip_fail(e, "solve kernel launch");
  return sync ? wait_done(c, s, armed) : F110QP_OK;
}

int f110qp_solve_batch_dev_sync(f110qp_ctx* c, int batch, const float* x0, const float* ul,
                                const float* xr, const float* hs, float* uo, float* xo, int* st,
                                int* it, void* stream) {
  return solve_dev(c, batch, x0, ul, xr, hs, uo, xo, st, it, nullptr, nullptr, (hipStream_t)stream, true);
}

int f110qp_solve_batch_ex_dev(f110qp_ctx* c, int batch, const float* x0, const float* ul,
                              const float* xr, const float* hs, float* uo, float* xo, int* st,
                              int* it, double* obj, double* cost, void* stream) {
  return solve_dev(c, batch, x0, ul, xr, hs, uo, xo, st, it, obj, cost, (hipStream_t)stream, false);
}

// Per-group W cache of a grouped call (grows only; every call re-fills the slots it uses).
static int group_state(f110qp_ctx* c, const int* group, int num_groups, f110qp::WarmState* gws,
                       int** leader) {
  const size_t G = (size_t)num_groups, nu = 2 * (size_t)c->cfg.horizon;
  hipError_t e;
  if ((e = c->gW.ensure(G * nu * nu * 4)) || (e = c->gkey.ensure(G * 16)) || (e = c->glead.ensure(G * 4)))
    return hip_fail(e, "hipMalloc group state");
  *gws = f110qp::WarmState();
  gws->W = (float*)c->gW.p;
  gws->key = (unsigned*)c->gkey.p;
  gws->group = group;
  gws->ngroups = num_groups;
  *leader = (int*)c->glead.p;
  return F110QP_OK;
}

static int check_groups(const int* group, int num_groups, int batch) {
  if (!group) return fail(F110QP_ERR_INVALID, "group is NULL");
  (void)batch;
  if (num_groups < 1 || num_groups > (1 << 22)) return fail(F110QP_ERR_INVALID, "num_groups must be in [1, 2^22]");
  return F110QP_OK;
}

int f110qp_solve_grouped_dev(f110qp_ctx* c, int batch, const float* x0, const float* ul,
                             const float* xr, const float* hs, const int* group, int num_groups,
                             float* uo, float* xo, int* st, int* it, void* stream) {
  return f110qp_solve_grouped_ex_dev(c, batch, x0, ul, xr, hs, group, num_groups, uo, xo, st, it,
                                     nullptr, nullptr, stream);
}

int f110qp_solve_grouped_ex_dev(f110qp_ctx* c, int batch, const float* x0, const float* ul,
                                const float* xr, const float* hs, const int* group, int num_groups,
                                float* uo, float* xo, int* st, int* it, double* obj, double* cost,
                                void* stream) {
  int rc = check_batch_args(c, batch, x0, ul, xr, hs, uo, xo, st);
  if (rc || batch == 0) return rc;
  if ((rc = check_groups(group, num_groups, batch))) return rc;
  const float* h = (c->cfg.gap_mode == F110QP_GAP_ACTIVE) ? hs : nullptr;
  f110qp::WarmState gws;
  int* leader;
  if ((rc = group_state(c, group, num_groups, &gws, &leader))) return rc;
  int backend;
  f110qp::LaneWork lw;
  if ((rc = lane_work(c, batch, (hipStream_t)stream, &backend, &lw, true))) return rc;
  f110qp::ObjOut oo;
  oo.obj = obj;
  oo.cost = cost;
  hipError_t e = f110qp::launch_solve_grouped(c->kp, batch, x0, ul, xr, h, uo, xo, st, it, gws,
                                              leader, backend, lw, oo, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "grouped solve launch");
  return F110QP_OK;
}

static int solve_host(f110qp_ctx* c, int batch, const float* x0, const float* ul, const float* xr,
                      const float* hs, const int* group, int num_groups, float* uo, float* xo,
                      int* st, int* it, double* obj, double* cost);

int f110qp_solve_batch(f110qp_ctx* c, int batch, const float* x0, const float* ul,
                       const float* xr, const float* hs, float* uo, float* xo, int* st,
                       int* it) {
  return solve_host(c, batch, x0, ul, xr, hs, nullptr, 0, uo, xo, st, it, nullptr, nullptr);
}

int f110qp_solve_batch_ex(f110qp_ctx* c, int batch, const float* x0, const float* ul,
                          const float* xr, const float* hs, float* uo, float* xo, int* st,
                          int* it, double* obj, double* cost) {
  return solve_host(c, batch, x0, ul, xr, hs, nullptr, 0, uo, xo, st, it, obj, cost);
}

int f110qp_solve_grouped(f110qp_ctx* c, int batch, const float* x0, const float* ul,
                         const float* xr, const float* hs, const int* group, int num_groups,
                         float* uo, float* xo, int* st, int* it) {
  return f110qp_solve_grouped_ex(c, batch, x0, ul, xr, hs, group, num_groups, uo, xo, st, it,
                                 nullptr, nullptr);
}

int f110qp_solve_grouped_ex(f110qp_ctx* c, int batch, const float* x0, const float* ul,
                            const float* xr, const float* hs, const int* group, int num_groups,
                            float* uo, float* xo, int* st, int* it, double* obj, double* cost) {
  if (batch > 0) {
    const int rc = check_groups(group, num_groups, batch);
    if (rc) return rc;
  }
  return solve_host(c, batch, x0, ul, xr, hs, group, num_groups, uo, xo, st, it, obj, cost);
}

int f110qp_backend_info(f110qp_ctx* c, int batch, int grouped, int* backend, int* qps_per_wave,
                        int* scratch) {
  if (!c) return fail(F110QP_ERR_INVALID, "ctx is NULL");
  if (batch < 1) return fail(F110QP_ERR_INVALID, "batch must be >= 1");
  f110qp::LaneWork lw;
  lw.mode = c->lane_mode;
  lw.qpw = c->lane_qpw;
  lw.seg = c->lane_seg;
  const int be = resolve_backend(c, batch, grouped != 0);
  const bool lane = be == F110QP_BACKEND_LANE;  // gap rows: the box screen's lane solve
  const int segs = lane ? f110qp::lane_segments(c->kp, batch, lw) : 1;
  if (backend) *backend = be;
  if (qps_per_wave) *qps_per_wave = lane ? (segs > 1 ? 64 / segs : f110qp::lane_qps_per_wave(batch, lw.qpw)) : 1;
  lw.seg32 = c->lane_seg32;
  lw.twin = c->lane_twin;
  if (scratch)
    *scratch = !lane ? 0 : segs > 1 ? f110qp::lane_seg_scratch(c->kp, batch, segs, lw)
                                    : f110qp::lane_scratch_mode(c->kp, batch, lw);
  return F110QP_OK;
}

int f110qp_lane_segments(f110qp_ctx* c, int batch, int* segments) {
  if (!c || !segments) return fail(F110QP_ERR_INVALID, "ctx / segments is NULL");
  if (batch < 1) return fail(F110QP_ERR_INVALID, "batch must be >= 1");
  int be = 0;
  const int rc = f110qp_backend_info(c, batch, 0, &be, nullptr, nullptr);
  if (rc) return rc;
  f110qp::LaneWork lw;
  lw.mode = c->lane_mode;
  lw.qpw = c->lane_qpw;
  lw.seg = c->lane_seg;
  if (be != F110QP_BACKEND_LANE) *segments = 1;
  else *segments = f110qp::lane_segments(c->kp, batch, lw);
  return F110QP_OK;
}

int f110qp_lane_starts(f110qp_ctx* c, int batch, int* starts) {
  if (!c || !starts) return fail(F110QP_ERR_INVALID, "ctx / starts is NULL");
  if (batch < 1) return fail(F110QP_ERR_INVALID, "batch must be >= 1");
  int segs = 1;
  const int rc = f110qp_lane_segments(c, batch, &segs);
  if (rc) return rc;
  f110qp::LaneWork lw;
  lw.mode = c->lane_mode;
  lw.qpw = c->lane_qpw;
  lw.seg = c->lane_seg;
  lw.seg32 = c->lane_seg32;
  lw.twin = c->lane_twin;
  *starts = segs > 1 ? f110qp::lane_seg_starts(c->kp, batch, segs, lw) : 1;
  return F110QP_OK;
}

int f110qp_gap_screen(f110qp_ctx* c, int batch, int* on) {
  if (!c || !on) return fail(F110QP_ERR_INVALID, "ctx / on is NULL");
  if (batch < 1) return fail(F110QP_ERR_INVALID, "batch must be >= 1");
  *on = gap_screen(c, batch, false);
  return F110QP_OK;
}

int f110qp_select_dev(int batch, const int* group, int num_groups, const double* cost,
                      const int* status, int* winner, double* best_cost, void* stream) {
  if (batch < 0 || num_groups < 0) return fail(F110QP_ERR_INVALID, "batch / num_groups < 0");
  if (num_groups == 0) return F110QP_OK;
  if (!winner || !best_cost || (batch > 0 && (!group || !cost || !status)))
    return fail(F110QP_ERR_INVALID, "NULL pointer argument");
  hipError_t e = f110qp::launch_select(batch, group, num_groups, cost, status, winner, best_cost,
                                       (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "select kernel launch");
  return F110QP_OK;
}

}  // extern "C"

static int solve_host(f110qp_ctx* c, int batch, const float* x0, const float* ul, const float* xr,
                      const float* hs, const int* group, int num_groups, float* uo, float* xo,
                      int* st, int* it, double* obj, double* cost) {
  int rc = check_batch_args(c, batch, x0, ul, xr, hs, uo, xo, st);
  if (rc || batch == 0) return rc;
  hipError_t e = hipSetDevice(c->cfg.device);
  if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  if (!c->stream) {
    e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) return hip_fail(e, "hipStreamCreate");
  }
  const int N = c->cfg.horizon;
  const bool gap = c->cfg.gap_mode == F110QP_GAP_ACTIVE;
  const size_t B = (size_t)batch;
  const size_t S = (size_t)c->kp.xr_stride;
  const size_t s_x0 = B * 3 * 4, s_ul = B * 2 * 4, s_xr = B * S * 3 * 4, s_hs = B * 6 * 4;
  const size_t s_uo = B * N * 2 * 4, s_xo = B * (N + 1) * 3 * 4, s_st = B * 4;
  // packed layouts (every size a multiple of 4 bytes): in = x0 | u_lin | x_ref | halfspace,
  // out = u | x | status | iters | obj | cost (the doubles 8-byte aligned)
  const size_t o_ul = s_x0, o_xr = o_ul + s_ul, o_hs = o_xr + s_xr, in_bytes = o_hs + (gap ? s_hs : 0);
  const size_t o_xo = s_uo, o_st = o_xo + s_xo, o_it = o_st + s_st;
  const size_t o_ob = (o_it + s_st + 7) & ~(size_t)7, s_ob = B * 8;
  const size_t o_co = o_ob + (obj ? s_ob : 0);
  const size_t out_bytes = o_co + (cost ? s_ob : 0);
  if ((e = c->hin.ensure(in_bytes)) || (e = c->hout.ensure(out_bytes)))
    return hip_fail(e, "hipHostMalloc staging");
  char* hi = (char*)c->hin.p;
  std::memcpy(hi, x0, s_x0);
  std::memcpy(hi + o_ul, ul, s_ul);
  std::memcpy(hi + o_xr, xr, s_xr);
  if (gap) std::memcpy(hi + o_hs, hs, s_hs);
  hipStream_t s = c->stream;
  const bool zc = batch <= kZeroCopyMaxBatch;
  char* di = (char*)c->hin.d;
  char* dq = (char*)c->hout.d;
  if (!zc) {
    if ((e = c->din.ensure(in_bytes)) || (e = c->dout.ensure(out_bytes)))
      return hip_fail(e, "hipMalloc workspace");
    di = (char*)c->din.p;
    dq = (char*)c->dout.p;
    if ((e = hipMemcpyAsync(di, c->hin.p, in_bytes, hipMemcpyHostToDevice, s)))
      return hip_fail(e, "hipMemcpyAsync H2D");
  }
  int backend;
  f110qp::LaneWork lw;
  f110qp::ObjOut oo;
  bool armed = false;
  oo.obj = obj ? (double*)(dq + o_ob) : nullptr;
  oo.cost = cost ? (double*)(dq + o_co) : nullptr;
  if (group) {
    if ((e = c->dgrp.ensure(B * 4)) || (e = hipMemcpyAsync(c->dgrp.p, group, B * 4, hipMemcpyHostToDevice, s)))
      return hip_fail(e, "group ids H2D");
    f110qp::WarmState gws;
    int* leader;
    if ((rc = group_state(c, (const int*)c->dgrp.p, num_groups, &gws, &leader))) return rc;
    if ((rc = lane_work(c, batch, s, &backend, &lw, true))) return rc;
    e = f110qp::launch_solve_grouped(c->kp, batch, (const float*)di, (const float*)(di + o_ul),
                                     (const float*)(di + o_xr), gap ? (const float*)(di + o_hs) : nullptr,
                                     (float*)dq, (float*)(dq + o_xo), (int*)(dq + o_st),
                                     (int*)(dq + o_it), gws, leader, backend, lw, oo, s);
  } else {
    f110qp::WarmState ws;
    if ((rc = warm_state(c, batch, s, &ws))) return rc;
    if ((rc = lane_work(c, batch, s, &backend, &lw))) return rc;
    // zero-copy: the kernel's stores are the outputs the host reads, so its completion word ends
    // the wait (staged batches wait for the D2H copy on the stream)
    if (zc && (rc = arm_signal(c, batch, backend, gap ? (const float*)(di + o_hs) : nullptr, lw, s, &oo, &armed)))
      return rc;
    e = f110qp::launch_solve(c->kp, batch, (const float*)di, (const float*)(di + o_ul),
                             (const float*)(di + o_xr), gap ? (const float*)(di + o_hs) : nullptr,
                             (float*)dq, (float*)(dq + o_xo), (int*)(dq + o_st), (int*)(dq + o_it),
                             ws, backend, lw, oo, s);
  }
  if (e != hipSuccess) return hip_fail(e, "solve kernel launch");
  if (!zc && (e = hipMemcpyAsync(c->hout.p, dq, out_bytes, hipMemcpyDeviceToHost, s)))
    return hip_fail(e, "hipMemcpyAsync D2H");
  if ((rc = wait_done(c, s, armed))) return rc;
  const char* ho = (const char*)c->hout.p;
  std::memcpy(uo, ho, s_uo);
  std::memcpy(xo, ho + o_xo, s_xo);
  std::memcpy(st, ho + o_st, s_st);
  if (it) std::memcpy(it, ho + o_it, s_st);
  if (obj) std::memcpy(obj, ho + o_ob, s_ob);
  if (cost) std::memcpy(cost, ho + o_co, s_ob);
  return F110QP_OK;
}

extern "C" {

int f110qp_condense_debug_dev(f110qp_ctx* c, int batch, const float* x0, const float* ul,
                              const float* xr, double* H, double* g, void* stream) {
  if (!c) return fail(F110QP_ERR_INVALID, "ctx is NULL");
  if (batch < 0) return fail(F110QP_ERR_INVALID, "batch < 0");
  if (batch == 0) return F110QP_OK;
  if (!x0 || !ul || !xr || !H || !g) return fail(F110QP_ERR_INVALID, "NULL pointer argument");
  hipError_t e = f110qp::launch_condense_debug(c->kp, batch, x0, ul, xr, H, g,
                                               (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "condense kernel launch");
  return F110QP_OK;
}

int f110qp_qp_dims(int N, int* n, int* m, int* nnz_P, int* nnz_A) {
  if (N < 1 || N > F110QP_MAX_HORIZON) return fail(F110QP_ERR_INVALID, "horizon must be in [1, 48]");
  if (n) *n = 5 * N + 3;              // 3(N+1) states + 2N inputs (mpc.cpp:26-28)
  if (m) *m = 7 * N + 5;              // dynamics + gap + input rows (mpc.cpp:29)
  if (nnz_P) *nnz_P = 9 * (N + 1) + 4 * N;
  if (nnz_A) *nnz_A = 26 * N + 9;
  return F110QP_OK;
}

int f110qp_assemble_debug_dev(f110qp_ctx* c, const float* x0, const float* ul, const float* xr,
                              const float* hs, int* Pc, int* Pr, double* Pv, double* q, int* Ac,
                              int* Ar, double* Av, double* l, double* u, void* stream) {
  if (!c) return fail(F110QP_ERR_INVALID, "ctx is NULL");
  if (!x0 || !ul || !xr || !Pc || !Pr || !Pv || !q || !Ac || !Ar || !Av || !l || !u)
    return fail(F110QP_ERR_INVALID, "NULL pointer argument");
  const int gap = c->cfg.gap_mode == F110QP_GAP_ACTIVE;
  if (gap && !hs) return fail(F110QP_ERR_INVALID, "gap_mode ACTIVE needs the halfspace array");
  hipError_t e = f110qp::launch_assemble(c->kp, x0, ul, xr, hs, gap, Pc, Pr, Pv, q, Ac, Ar, Av, l, u,
                                         (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "assemble kernel launch");
  return F110QP_OK;
}

// Constraints::FindHalfSpaces (src/constraints.cpp:116-265) for one scan, host code with the
// reference's float32 member types; the ROS marker publish (:191-229) is not reproduced.
int f110qp_find_half_spaces(const double state[3], const float* ranges, int nr, float angle_min,
                            float angle_inc, float angle_max, float ftg_thresh, float divider,
                            float buffer, double l1[3], double l2[3]) {
  if (!state || !ranges || !l1 || !l2 || nr <= 0)
    return fail(F110QP_ERR_INVALID, "NULL pointer or empty scan");
  int num_scans = (int)((angle_max - angle_min) / angle_inc + 1);
  if (num_scans > nr) num_scans = nr;
  int max_gap = -1, best_lo = 0, best_hi = 0, lo = -1, hi = -1;
  bool in_gap = false;
  const float lim = 1.571f / divider;
  for (int ii = 0; ii < num_scans; ii++) {
    const float angle = angle_min + ii * angle_inc;
    if (angle > -lim && angle < lim) {
      if (ranges[ii] > ftg_thresh) {
        if (in_gap) hi = ii;
        else { lo = ii; in_gap = true; }
      } else {
        in_gap = false;
      }
      if (hi - lo > max_gap) { max_gap = hi - lo; best_hi = hi; best_lo = lo; }
    }
  }
  if (best_hi - best_lo > 2 * buffer) {
    best_hi = (int)(best_hi - buffer);
    best_lo = (int)(best_lo + buffer);
  }
  if (best_lo < 0 || best_hi < 0 || best_lo >= nr || best_hi >= nr)
    return fail(F110QP_ERR_INVALID, "scan holds no gap (reference reads ranges[-1] here)");
  const double poseX = state[0], poseY = state[1];
  const float cur = (float)state[2];
  const float ang1 = angle_min + best_lo * angle_inc + cur;
  const float ang2 = angle_min + best_hi * angle_inc + cur;
  const float p1x = (float)(ranges[best_lo] * std::cos((double)ang1) + poseX);
  const float p1y = (float)(ranges[best_lo] * std::sin((double)ang1) + poseY);
  const float p2x = (float)(ranges[best_hi] * std::cos((double)ang2) + poseX);
  const float p2y = (float)(ranges[best_hi] * std::sin((double)ang2) + poseY);
  const float px = (float)poseX, py = (float)poseY;
  float a1 = py - p1y, b1 = p1x - px, c1 = px * p1y - py * p1x;
  if (a1 * p2x + b1 * p2y + c1 < 0) { a1 = -a1; b1 = -b1; c1 = -c1; }
  float a2 = py - p2y, b2 = p2x - px, c2 = px * p2y - py * p2x;
  if (a2 * p1x + b2 * p1y + c2 < 0) { a2 = -a2; b2 = -b2; c2 = -c2; }
  l1[0] = a1; l1[1] = b1; l1[2] = (double)c1 + 0.5;
  l2[0] = a2; l2[1] = b2; l2[2] = (double)c2 + 0.5;
  return F110QP_OK;
}

int f110qp_find_half_spaces_dev(int batch, const float* states, const float* ranges, int nr,
                                float angle_min, float angle_inc, float angle_max,
                                float ftg_thresh, float divider, float buffer, float* hs,
                                int* gap_lo, int* gap_hi, void* stream) {
  if (batch < 0 || nr <= 0 || nr > 65535) return fail(F110QP_ERR_INVALID, "bad batch / num_ranges (1..65535)");
  if (batch == 0) return F110QP_OK;
  if (!states || !ranges || !hs) return fail(F110QP_ERR_INVALID, "NULL pointer argument");
  if (!(angle_inc > 0.f)) return fail(F110QP_ERR_INVALID, "angle_increment must be > 0");
  hipError_t e = f110qp::launch_half_spaces(batch, states, ranges, nr, angle_min, angle_inc,
                                            angle_max, ftg_thresh, divider, buffer, hs, gap_lo,
                                            gap_hi, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "half-space kernel launch");
  return F110QP_OK;
}

}  // extern "C"

// ---- planning stage -----------------------------------------------------------------------

static int validate_plan(const f110qp_plan_config* c, int* G);

extern "C" {

void f110qp_default_plan_config(f110qp_plan_config* c) {
  if (!c) return;
  std::memset(c, 0, sizeof(*c));
  c->size = 10;            // params.yaml:16
  c->discrete = 0.1f;      // params.yaml:17
  c->dilation = 0.15f;     // params.yaml:18
  c->lookahead = 2.5f;     // params.yaml:63
  c->speed_max = 4.5;      // params.yaml:46 (umax)
  c->steer_max = 0.4;      // params.yaml:60
  c->steer_discrete = 30;  // params.yaml:59
  c->traj_discrete = 50;   // params.yaml:61
  c->dt = 0.01;            // params.yaml:13
}

static int validate_plan(const f110qp_plan_config* c, int* G) {
  if (!c) return fail(F110QP_ERR_INVALID, "plan config is NULL");
  if (!(c->discrete > 0.f) || c->size <= 0 || !(c->dilation >= 0.f))
    return fail(F110QP_ERR_INVALID, "occupancy grid size/discrete/dilation");
  const int g = (int)((float)c->size / c->discrete);  // occupancy_grid.cpp:9
  if (g < 1 || g > 200) return fail(F110QP_ERR_INVALID, "grid_blocks must be in [1, 200]");
  if (c->steer_discrete < 1 || c->steer_discrete > 255 || c->traj_discrete < 2 || c->traj_discrete > 1024)
    return fail(F110QP_ERR_INVALID, "steer_discrete in [1, 255], traj_discrete in [2, 1024]");
  *G = g;
  return F110QP_OK;
}

// Traj_Plan::generate_traj_table (trajectory_planner.cpp:26-72) with Model::simulate_dynamics
// (model.cpp:61-75, CAR_LENGTH = 0.35), doubles as the reference's State/Input.
int f110qp_traj_table(const f110qp_plan_config* c, double* table) {
  int G;
  int rc = validate_plan(c, &G);
  if (rc) return rc;
  if (!table) return fail(F110QP_ERR_INVALID, "table is NULL");
  const double ds = 2 * +c->steer_max / c->steer_discrete;  // :31
  const int T = c->steer_discrete + 1, P = c->traj_discrete;
  const double CAR_LENGTH = 0.35;
  for (int i = 0; i < T; i++) {
    const double steer = -c->steer_max + i * ds;  // :43
    const double v = c->speed_max;
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    double* row = table + (size_t)i * P * 3;
    row[0] = s0; row[1] = s1; row[2] = s2;  // k == 0 (:54)
    for (int k = 1; k < P; k++) {
      const volatile double d0 = v * std::cos(s2), d1 = v * std::sin(s2);
      const volatile double d2 = std::tan(steer) * v / CAR_LENGTH;
      const volatile double e0 = d0 * c->dt, e1 = d1 * c->dt, e2 = d2 * c->dt;  // dynamics*dt
      s0 = s0 + e0; s1 = s1 + e1; s2 = s2 + e2;
      row[3 * k] = s0; row[3 * k + 1] = s1; row[3 * k + 2] = s2;
    }
  }
  return T;
}

// Trajectory::ReadCSV (trajectory.cpp:18-55): getline(',') then getline() and stof of each.
int f110qp_parse_waypoints(const char* text, double* wp, int max_n, int* n_out) {
  if (!text || !wp || !n_out || max_n < 0) return fail(F110QP_ERR_INVALID, "NULL argument");
  std::string buf;
  int n = 0;
  const char* s = text;
  std::string xs, ys;
  // temp.push_back(pair<float,float>(stof(coordX), stof(coordY)))
  std::vector<float> tx, ty;
  while (*s) {
    const char* comma = std::strchr(s, ',');
    if (!comma) break;
    xs.assign(s, comma - s);
    const char* eol = std::strchr(comma + 1, '\n');
    ys.assign(comma + 1, eol ? (size_t)(eol - comma - 1) : std::strlen(comma + 1));
    char* e1;
    char* e2;
    const float x = std::strtof(xs.c_str(), &e1);
    const float y = std::strtof(ys.c_str(), &e2);
    if (e1 == xs.c_str() || e2 == ys.c_str()) return fail(F110QP_ERR_INVALID, "stof: no conversion");
    tx.push_back(x);
    ty.push_back(y);
    s = eol ? eol + 1 : comma + 1 + std::strlen(comma + 1);
  }
  const unsigned int cnt = (unsigned int)tx.size();
  for (unsigned int i = 0; i < cnt && (int)i < max_n; i++) {
    const unsigned int prev = (i - 1) % cnt;  // :42-43 (unsigned wrap for i = 0)
    const float x = tx[i], y = ty[i];
    wp[3 * i] = x;
    wp[3 * i + 1] = y;
    wp[3 * i + 2] = (float)std::atan2((double)(y - ty[prev]), (double)(x - tx[prev]));  // :46
    n++;
  }
  *n_out = n;
  return F110QP_OK;
}

int f110qp_plan_batch_dev(const f110qp_plan_config* c, int batch, const double* pose,
                          const float* ranges, int nr, float angle_min, float angle_inc,
                          float angle_max, const double* table, const double* wp, int W,
                          unsigned char* grid, unsigned char* valid, int* best_global,
                          int* best_traj, float* x_ref, float* x0, int* status, void* stream) {
  int G;
  int rc = validate_plan(c, &G);
  if (rc) return rc;
  if (batch < 0 || nr <= 0 || W < 0) return fail(F110QP_ERR_INVALID, "bad batch / num_ranges / num_waypoints");
  if (batch == 0) return F110QP_OK;
  if (!pose || !ranges || !table || (W > 0 && !wp) || !best_global || !best_traj || !x_ref || !x0 || !status)
    return fail(F110QP_ERR_INVALID, "NULL pointer argument");
  if (!(angle_inc > 0.f)) return fail(F110QP_ERR_INVALID, "angle_increment must be > 0");
  f110qp::PlanKParams K;
  K.G = G;
  K.T = c->steer_discrete + 1;
  K.P = c->traj_discrete;
  K.discrete = c->discrete;
  K.dilation = c->dilation;
  K.lookahead = c->lookahead;
  hipError_t e = f110qp::launch_plan(K, batch, pose, ranges, nr, angle_min, angle_inc, angle_max,
                                     table, wp, W, grid, valid, best_global, best_traj, x_ref, x0,
                                     status, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "plan kernel launch");
  return F110QP_OK;
}

}  // extern "C"

namespace {
// device staging of f110qp_plan_batch, one set per host thread
struct PlanBufs {
  DevBuf pose, ranges, table, wp, grid, valid, bg, bt, xr, x0, st;
  hipStream_t stream = nullptr;
  ~PlanBufs() {
    if (stream) (void)hipStreamDestroy(stream);
  }
};
thread_local PlanBufs g_plan;
}  // namespace

extern "C" int f110qp_plan_batch(const f110qp_plan_config* c, int batch, const double* pose,
                                 const float* ranges, int nr, float angle_min, float angle_inc,
                                 float angle_max, const double* table, const double* wp, int W,
                                 unsigned char* grid, unsigned char* valid, int* best_global,
                                 int* best_traj, float* x_ref, float* x0, int* status) {
  int G;
  int rc = validate_plan(c, &G);
  if (rc) return rc;
  if (batch < 0 || nr <= 0 || W < 0) return fail(F110QP_ERR_INVALID, "bad batch / num_ranges / num_waypoints");
  if (batch == 0) return F110QP_OK;
  if (!pose || !ranges || !table || (W > 0 && !wp) || !best_global || !best_traj || !x_ref || !x0 || !status)
    return fail(F110QP_ERR_INVALID, "NULL pointer argument");
  PlanBufs& pb = g_plan;
  hipError_t e;
  if (!pb.stream && (e = hipStreamCreateWithFlags(&pb.stream, hipStreamNonBlocking)))
    return hip_fail(e, "hipStreamCreate");
  const size_t B = (size_t)batch, T = (size_t)c->steer_discrete + 1, P = (size_t)c->traj_discrete;
  const size_t s_pose = B * 4 * 8, s_r = B * nr * 4, s_tab = T * P * 3 * 8, s_wp = (size_t)W * 2 * 8;
  const size_t s_grid = B * G * G, s_valid = B * T, s_i = B * 4, s_xr = B * P * 3 * 4, s_x0 = B * 3 * 4;
  if ((e = pb.pose.ensure(s_pose)) || (e = pb.ranges.ensure(s_r)) || (e = pb.table.ensure(s_tab)) ||
      (e = pb.wp.ensure(s_wp ? s_wp : 8)) || (grid && (e = pb.grid.ensure(s_grid))) ||
      (valid && (e = pb.valid.ensure(s_valid))) || (e = pb.bg.ensure(s_i)) || (e = pb.bt.ensure(s_i)) ||
      (e = pb.xr.ensure(s_xr)) || (e = pb.x0.ensure(s_x0)) || (e = pb.st.ensure(s_i)))
    return hip_fail(e, "hipMalloc plan workspace");
  hipStream_t s = pb.stream;
  if ((e = hipMemcpyAsync(pb.pose.p, pose, s_pose, hipMemcpyHostToDevice, s)) ||
      (e = hipMemcpyAsync(pb.ranges.p, ranges, s_r, hipMemcpyHostToDevice, s)) ||
      (e = hipMemcpyAsync(pb.table.p, table, s_tab, hipMemcpyHostToDevice, s)) ||
      (W > 0 && (e = hipMemcpyAsync(pb.wp.p, wp, s_wp, hipMemcpyHostToDevice, s))))
    return hip_fail(e, "hipMemcpyAsync H2D");
  rc = f110qp_plan_batch_dev(c, batch, (const double*)pb.pose.p, (const float*)pb.ranges.p, nr, angle_min,
                             angle_inc, angle_max, (const double*)pb.table.p, (const double*)pb.wp.p, W,
                             grid ? (unsigned char*)pb.grid.p : nullptr,
                             valid ? (unsigned char*)pb.valid.p : nullptr, (int*)pb.bg.p, (int*)pb.bt.p,
                             (float*)pb.xr.p, (float*)pb.x0.p, (int*)pb.st.p, s);
  if (rc) return rc;
  if ((e = hipMemcpyAsync(best_global, pb.bg.p, s_i, hipMemcpyDeviceToHost, s)) ||
      (e = hipMemcpyAsync(best_traj, pb.bt.p, s_i, hipMemcpyDeviceToHost, s)) ||
      (e = hipMemcpyAsync(x_ref, pb.xr.p, s_xr, hipMemcpyDeviceToHost, s)) ||
      (e = hipMemcpyAsync(x0, pb.x0.p, s_x0, hipMemcpyDeviceToHost, s)) ||
      (e = hipMemcpyAsync(status, pb.st.p, s_i, hipMemcpyDeviceToHost, s)) ||
      (grid && (e = hipMemcpyAsync(grid, pb.grid.p, s_grid, hipMemcpyDeviceToHost, s))) ||
      (valid && (e = hipMemcpyAsync(valid, pb.valid.p, s_valid, hipMemcpyDeviceToHost, s))))
    return hip_fail(e, "hipMemcpyAsync D2H");
  if ((e = hipStreamSynchronize(s))) return hip_fail(e, "hipStreamSynchronize");
  return F110QP_OK;
}

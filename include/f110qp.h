/*
 * f110qp.h — C ABI of the MI355X batched MPC/QP solver for the f110-mpc control tick.
 *
 * Drop-in boundary. In the reference the per-tick hot path is
 *   MPC::Update (src/mpc.cpp:69-143)
 *     Model::Linearize            (src/model.cpp:30-59)
 *     Constraints::FindHalfSpaces (src/constraints.cpp:116-265)
 *     MPC::CreateGradientVector / Update{LinearConstraintMatrix,Lower,Upper}Bound
 *                                 (src/mpc.cpp:221-306)
 *     OsqpEigen::Solver::{updateGradient, updateLinearConstraintsMatrix, updateBounds,
 *                         initSolver, solve, getSolution}  (src/mpc.cpp:81-142,
 *                         solver_ member at include/f110-mpc/mpc.h:63)
 * f110qp_solve_batch[_dev] replaces that whole sequence for B ticks/candidates at once:
 * linearisation, condensing, the QP solve and the (u*, x*) extraction of
 * MPC::UpdateSolvedTrajectory (src/mpc.cpp:145-159) run in one HIP launch on gfx950.
 *
 * Conventions
 *  - Plain C: no C++ exceptions cross this boundary; every entry point returns an int
 *    (F110QP_OK = 0, negative = error; details from f110qp_last_error()).
 *  - The caller owns every buffer. *_dev entry points take device pointers and a
 *    hipStream_t (passed as void*) and are asynchronous on that stream; the host-pointer
 *    entry points are synchronous.
 *  - One f110qp_ctx per host thread. A ctx owns its device workspace, so the calls made on
 *    one ctx must be ordered (one stream, or synchronised between streams).
 *  - Layouts (row-major, float32):
 *      x0        [B][3]      (x, y, ori)           State  (include/f110-mpc/state.h:10-45)
 *      u_lin     [B][2]      (v, steer_ang)        Input  (include/f110-mpc/input.h:11-34)
 *      x_ref     [B][S][3]   desired states, S = x_ref_points (default N); states 0..N-1 are
 *                            read (the reference reads the first N of its 50-point mini path;
 *                            stage N reuses x_ref[N-1], mpc.cpp:228)
 *      halfspace [B][2][3]   (l1, l2) = (a, b, c+0.5) from FindHalfSpaces, or NULL
 *      u_out     [B][N][2]   u*_k = z[3(N+1)+2k .. +1]            (mpc.cpp:148-157)
 *      x_out     [B][N+1][3] x*_k = z[3k .. 3k+2]                 (mpc.cpp:167-169)
 *      status    [B]         F110QP_SOLVED / _PRIMAL_INFEASIBLE / _MAX_ITER / _NUMERICAL
 *                            (OSQP codes)
 *      iters     [B]         active-set iterations (may be NULL): box-only QPs on either back end
 *                            count the equality-QP solves of the primal-dual active set including
 *                            the final one that confirms the KKT point (0 would mean none ran);
 *                            QPs the wave back end hands to its Goldfarb-Idnani loop (gap rows,
 *                            or a box PDAS that did not settle) count GI iterations instead
 *      obj       [B] double  (the *_ex entry points; may be NULL) OSQP's objective value
 *                            1/2 z'Pz + q'z of the solved QP (osqp_info::obj_val; P, q of
 *                            mpc.cpp:208-229), computed in fp64 on the device
 *      cost      [B] double  (*_ex; may be NULL) the same objective WITH the constant OSQP drops:
 *                            sum_i 1/2|x_i - x_ref_i|_Q^2 + sum_k 1/2|u_k - u_des|_R^2 >= 0
 *                            (= obj + 1/2 sum_i x_ref_i'Q x_ref_i + N/2 u_des'R u_des). Candidates
 *                            with different references are compared on `cost`: obj carries the
 *                            reference-dependent constant -1/2 sum x_ref'Q x_ref.
 *    On a non-SOLVED status u_out/x_out hold NaN (obj/cost too), as OSQP's solution does on
 *    failure, with one exception: F110QP_SOLVED_INACCURATE returns the finite but uncertified
 *    point (u, x, obj, cost written; see the status below).
 */
#ifndef F110QP_H
#define F110QP_H

#ifdef __cplusplus
extern "C" {
#endif

#define F110QP_API_VERSION 6

/* return codes */
#define F110QP_OK 0
#define F110QP_ERR_INVALID -1     /* bad argument / unsupported configuration */
#define F110QP_ERR_HIP -2         /* HIP runtime error (no device, launch failure, ...) */
#define F110QP_ERR_ALLOC -3

/* per-QP status codes (values follow OSQP's status ids) */
#define F110QP_SOLVED 1
#define F110QP_SOLVED_INACCURATE 2 /* a point whose fp64 certificate failed (box rows: the KKT  */
                                  /* check in primal units; gap rows: the duality-gap bound     */
                                  /* below, also after the fp64 Goldfarb-Idnani re-check): u,   */
                                  /* x, obj, cost                                               */
                                  /* are written but not certified, and f110qp_select_dev never */
                                  /* picks it. Its active set may seed the next warm start (a   */
                                  /* seed is only a first guess; every solve is certified on    */
                                  /* its own).                                                  */
#define F110QP_MAX_ITER -2
#define F110QP_PRIMAL_INFEASIBLE -3
#define F110QP_NUMERICAL -10      /* non-finite data or factorisation breakdown */

/* gap (follow-the-gap half-space) row semantics, src/mpc.cpp:279-300 */
#define F110QP_GAP_INACTIVE 0     /* as shipped: gap rows bounded by +-OsqpEigen::INFTY */
#define F110QP_GAP_ACTIVE 1       /* a*x+b*y >= -(c+0.5) on stages 1..N (mpc.cpp:297-298) */

/* solver back ends (f110qp_config.backend) */
#define F110QP_BACKEND_AUTO 0     /* lane-per-QP for box-only batches >= F110QP_LANE_MIN_BATCH  */
                                  /* or <= F110QP_LANE_MAX_SMALL_BATCH (N <= 32), and >=       */
                                  /* F110QP_LANE_MIN_BATCH_WIDE (N > 32)                       */
#define F110QP_BACKEND_WAVE 1     /* one wavefront per QP: condensed W = H^-1 + PDAS/GI         */
#define F110QP_BACKEND_LANE 2     /* one lane per QP: Riccati/PDAS in fp64; with gap rows the   */
                                  /* box screen at every batch size: the lane solve of the box- */
                                  /* only problem, the wave kernel's GI for the QPs whose box   */
                                  /* optimum violates a gap row (no warm state, ungrouped)      */
/* Gap rows: the wave kernel's GI (AUTO: behind the box screen from
 * F110QP_GAP_SCREEN_MIN_BATCH QPs); GI's final point is certified in fp64, and every QP it does not
 * certify is re-checked in the same call by an fp64 Goldfarb-Idnani with the oracle's rules
 * (SOLVED, PRIMAL_INFEASIBLE, MAX_ITER or SOLVED_INACCURATE from there). What SOLVED certifies on
 * this path: every row holds to 1e-9 (1 + |b| + |u|_inf) in fp64, and |u - u*'|_2 <= 1e-6
 * max(1, |u|_inf) for the exact optimum u*' of the reference QP with each row bound moved by u's own
 * residual on it (a backward error <= that 1e-9 relative, below the float32 rounding of the
 * inputs): the duality gap at the clamped multipliers, rho'W rho / min(R) with rho = Hu + g - N_A mu+,
 * rho'W rho bounded from above in fp64. The distance to the optimum of the unmoved QP also depends
 * on that QP's sensitivity to its bounds, which is not bounded here (tests: within 4e-8 of the
 * oracle's exact optimum on every gap-row case).
 * AUTO thresholds, measured on MI355X (kernel us, DESIGN.md section 6, round 3: the lane back end
 * with the partitioned-horizon kernel below one wave per SIMD, the wave back end with its fp64
 * certification). N = 20 (C2 recipe, cold): wave 27.3 vs lane 30.6 at 512 (before the last
 * segmented-kernel changes), 28.5 vs 27.7 at 1,024, 53.1 vs 36.3 at 2,048, 93.0 vs 37.0 at
 * 3,072. N = 30: 94.8 vs 77.9 at 2,048. N = 40: wave 223 vs lane 45.7 at 256, 365 vs 46.1 at
 * 512, 428 vs 53.7 at 768: the lane back end from one QP on.
 * Grouped calls use the same thresholds: the wave back end's per-group W saves its inverse but
 * its per-QP active-set phase still dominates (C4 candidate sets: 8,192 x N=40 grouped wave
 * 1,041 us vs lane 240 us, round 2). */
#define F110QP_LANE_MIN_BATCH 1024
#define F110QP_LANE_MIN_BATCH_WIDE 1
/* ... and, at N <= 32, batches of at most this many QPs (the single QP of MPC::Update): the
 * partitioned-horizon lane kernel splits each horizon over S = 4 lanes and beats the wave kernel's
 * one-QP chain (round 4, kernel us, N = 20: B = 1 lane 10.3 vs wave 19.3, B = 4 20.5 vs 23.9,
 * B = 16 25.8 vs 25.5, B = 64 30.8 vs 25.2; tools/latency_probe.py) */
#define F110QP_LANE_MAX_SMALL_BATCH 8
/* Gap rows (gap_mode ACTIVE), AUTO, ungrouped, no warm start, batches of at least this many QPs:
 * the box-only problem is solved on the lane back end first, and only the QPs whose box optimum
 * leaves a gap row violated (or within a 1e-6 margin) go to the wave kernel's GI; the others'
 * lane outputs are the optimum with the gap rows as well (round 4: 57% of the C3 batch). Results
 * are the exact optimum either way; the iteration count is the lane PDAS passes for screened QPs. */
#define F110QP_GAP_SCREEN_MIN_BATCH 1024
#define F110QP_LANE_MIN_BATCH_GROUPED F110QP_LANE_MIN_BATCH
#define F110QP_LANE_MIN_BATCH_GROUPED_WIDE F110QP_LANE_MIN_BATCH_WIDE

#define F110QP_MAX_HORIZON 48  /* 2N <= 96 decision variables: two register rows per lane */

typedef struct f110qp_ctx f110qp_ctx;

typedef struct {
  int horizon;      /* N; params.yaml:12 ("/horizon"), 1..F110QP_MAX_HORIZON (48)     */
  float dt;         /* params.yaml:13, held as float MPC::dt_ (include/f110-mpc/mpc.h:46) */
  double q[3];      /* diag Q: q0,q1,q2 (params.yaml:1-3; mpc.cpp:20-24)                 */
  double r[2];      /* diag R: r0,r1 (params.yaml:5-6)                                    */
  double u_des[2];  /* des_vel, des_steer (params.yaml:42-43; mpc.cpp:18-19)              */
  float u_min[2];   /* (umin, -0.43f) constraints.cpp:21                                  */
  float u_max[2];   /* (umax,  0.43f) constraints.cpp:19                                  */
  int gap_mode;     /* F110QP_GAP_INACTIVE | F110QP_GAP_ACTIVE                            */
  int max_iter;     /* active-set iteration cap per QP (0 = default 8*(2N+2N))             */
  int device;       /* HIP device ordinal used by the host-pointer entry points            */
  int warm_start;   /* 1: keep per-slot state across calls (OsqpEigen setWarmStart(true),   */
                    /*    mpc.cpp:98): the factor W = H^-1 is reused when a slot's          */
                    /*    linearisation point (theta0, v, steer) is bit-identical to its    */
                    /*    previous call's, and the previous active set seeds the solve.    */
                    /*    Slot b of call t+1 continues slot b of call t (same batch size). */
                    /*    The lane back ends move this state only while keys hit (within  */
                    /*    the last 2 calls, or on 2 probe calls in every 32).             */
                    /*    A stream whose linearisation point changes every tick (the      */
                    /*    closed loop of configs[4]: theta0 follows the plant) never hits: */
                    /*    its solves are cold solves (no factor or active set is reused;  */
                    /*    the previous tick's active set measured a worse seed than none, */
                    /*    DESIGN.md 2b). f110qp_warm_hits reports what a call reused.      */
  int backend;      /* F110QP_BACKEND_AUTO | _WAVE | _LANE (both give the exact optimum)    */
  int x_ref_points; /* points per QP in x_ref, >= N (0 = N). MPC::Update receives the whole   */
                    /* miniPath and reads its first N states (mpc.cpp:223-228): pass the      */
                    /* planner's [B][P][3] x_ref with x_ref_points = P                        */
} f110qp_config;

/* Library / ABI version (F110QP_API_VERSION). */
int f110qp_version(void);
/* Message of the last error on this thread (never NULL). */
const char* f110qp_last_error(void);

/* Defaults of params.yaml + constraints.cpp:19,21 for horizon N.
 * Replaces the getParam block of MPC::MPC (src/mpc.cpp:5-24) and Constraints::Constraints
 * (src/constraints.cpp:7-21). */
void f110qp_default_config(f110qp_config* cfg, int horizon);

/* Create a solver context (device workspace). Replaces the lazy OsqpEigen workspace set-up
 * of MPC::Update's first call (src/mpc.cpp:96-131). */
int f110qp_create(f110qp_ctx** ctx, const f110qp_config* cfg);
void f110qp_destroy(f110qp_ctx* ctx);

/* Solve B independent ticks (host pointers, synchronous). Replaces, per instance,
 * MPC::Update's Linearize + gradient/constraint/bound updates + solver_.solve() +
 * getSolution (src/mpc.cpp:69-143) and UpdateSolvedTrajectory (src/mpc.cpp:145-159).
 * Up to 64 QPs the kernel reads the inputs from and writes the outputs to pinned host staging
 * (zero-copy), and the call returns on its last kernel's completion word (f110qp_sync_signals);
 * larger batches are staged through device memory and wait for the stream. */
int f110qp_solve_batch(f110qp_ctx* ctx, int batch, const float* x0, const float* u_lin,
                       const float* x_ref, const float* halfspace, float* u_out, float* x_out,
                       int* status, int* iters);

/* Same on device pointers, enqueued on `stream` (a hipStream_t, NULL = default stream). */
int f110qp_solve_batch_dev(f110qp_ctx* ctx, int batch, const float* x0, const float* u_lin,
                           const float* x_ref, const float* halfspace, float* u_out,
                           float* x_out, int* status, int* iters, void* stream);

/* f110qp_solve_batch_dev, then a wait until the results are in device memory: one call per
 * control tick for a caller that needs the answer before it returns, as solver_.solve() +
 * getSolution do in MPC::Update (src/mpc.cpp:133-142). When the call's last kernel (lane or wave
 * kernel; for gap rows the fp64 re-check) has at most 256 workgroups, the call waits on the
 * completion word that kernel writes from its last wave or workgroup after a system-scope fence:
 * the outputs are then visible to any stream and to the host, and the kernel may still be retiring
 * on `stream` when this returns. Larger launches synchronise `stream`. */
int f110qp_solve_batch_dev_sync(f110qp_ctx* ctx, int batch, const float* x0, const float* u_lin,
                                const float* x_ref, const float* halfspace, float* u_out,
                                float* x_out, int* status, int* iters, void* stream);

/* Grouped solve: the candidates of one control tick share their linearisation point.
 * Model::Linearize depends only on (theta0, v, delta) (src/model.cpp:30-59), so the candidate
 * mini-paths of one pose (src/project.cpp:76-113) share A, B, C, the condensed Hessian H and
 * W = H^-1: only the gradient differs (the proposal's `group` argument, 8(b)).
 *   group [B]   scenario id of each QP in [0, num_groups); ids need not be contiguous or sorted.
 * One W per group is built from its first member; every member whose (x0[b][2], u_lin[b]) bits
 * equal that member's reuses it, any other QP (or an id outside [0, num_groups)) builds its own.
 * Grouping therefore never changes a result: the output is bit-identical to
 * f110qp_solve_batch[_dev] on the wave back end. The lane back end (chosen by AUTO at and above
 * F110QP_LANE_MIN_BATCH_GROUPED[_WIDE]) ignores the groups (only its first, cold pass has
 * group-invariant Riccati matrices: <= ~4% of a C4 launch). Grouped
 * calls neither use nor update the warm-start state. Same layouts and conventions as above. */
int f110qp_solve_grouped(f110qp_ctx* ctx, int batch, const float* x0, const float* u_lin,
                         const float* x_ref, const float* halfspace, const int* group,
                         int num_groups, float* u_out, float* x_out, int* status, int* iters);
int f110qp_solve_grouped_dev(f110qp_ctx* ctx, int batch, const float* x0, const float* u_lin,
                             const float* x_ref, const float* halfspace, const int* group,
                             int num_groups, float* u_out, float* x_out, int* status, int* iters,
                             void* stream);

/* Same as f110qp_solve_batch[_dev] / f110qp_solve_grouped[_dev], plus the per-QP objective
 * `obj` and `cost` (see Layouts; either may be NULL). The objective is what
 * OsqpEigen::Solver::solve() leaves in osqp_info::obj_val after src/mpc.cpp:133. */
int f110qp_solve_batch_ex(f110qp_ctx* ctx, int batch, const float* x0, const float* u_lin,
                          const float* x_ref, const float* halfspace, float* u_out, float* x_out,
                          int* status, int* iters, double* obj, double* cost);
int f110qp_solve_batch_ex_dev(f110qp_ctx* ctx, int batch, const float* x0, const float* u_lin,
                              const float* x_ref, const float* halfspace, float* u_out,
                              float* x_out, int* status, int* iters, double* obj, double* cost,
                              void* stream);
int f110qp_solve_grouped_ex(f110qp_ctx* ctx, int batch, const float* x0, const float* u_lin,
                            const float* x_ref, const float* halfspace, const int* group,
                            int num_groups, float* u_out, float* x_out, int* status, int* iters,
                            double* obj, double* cost);
int f110qp_solve_grouped_ex_dev(f110qp_ctx* ctx, int batch, const float* x0, const float* u_lin,
                                const float* x_ref, const float* halfspace, const int* group,
                                int num_groups, float* u_out, float* x_out, int* status,
                                int* iters, double* obj, double* cost, void* stream);

/* Per-scenario selection on the device: the candidate argmin of
 * project::OdomCallback (src/project.cpp:125-136), taken over the QP costs of each scenario's
 * candidates instead of the end-point distance. winner[g] = the smallest b with group[b] == g,
 * status[b] == F110QP_SOLVED and the minimal cost[b] (exact, deterministic), or -1 when the
 * scenario has no solved candidate; best_cost[g] = that cost (+inf if none). group/cost/status
 * [batch], winner/best_cost [num_groups], device pointers, async on stream. Across GPUs, the
 * per-rank (best_cost, winner) pairs reduce with a min-loc all-reduce (f110qp/shard.py). */
int f110qp_select_dev(int batch, const int* group, int num_groups, const double* cost,
                      const int* status, int* winner, double* best_cost, void* stream);

/* The launch a solve call of `batch` QPs on this context makes (grouped != 0: the grouped entry
 * points): backend = F110QP_BACKEND_WAVE or _LANE (what AUTO resolves to), qps_per_wave (lane:
 * QPs per 64-lane wavefront; wave: 1) and scratch (lane: 1 LDS fp64, 2 LDS fp32, 3 HBM fp64,
 * 4 HBM fp32 Riccati gain scratch; the partitioned-horizon kernel uses 1 or 2 (float references
 * and scratch where fp64 does not fit); wave: 0). With gap rows, LANE means the box screen's lane
 * solve (F110QP_BACKEND_LANE). Any pointer may be NULL. */
int f110qp_backend_info(f110qp_ctx* ctx, int batch, int grouped, int* backend, int* qps_per_wave,
                        int* scratch);

/* Horizon segments per QP of that launch: 1, or S = 2 / 4 / 8 when the lane back end splits each
 * QP's horizon over S lanes (partitioned Riccati; batches too small to give every SIMD a wave of
 * distinct QPs; with gap rows on the lane back end: the box screen's solve).
 * The result is the exact optimum either way. */
int f110qp_lane_segments(f110qp_ctx* ctx, int batch, int* segments);

/* PDAS starts per QP of that launch: 2 when the partitioned-horizon kernel solves each QP from two
 * starts at once (the cold one and the speed bound u_des sits on held over the first half of the
 * horizon; taken when u_des is on a speed bound and the doubled grid still leaves no SIMD with
 * two waves), else 1. The first start to converge gives the answer: the same exact optimum, in the
 * smaller of the two pass counts (DESIGN.md 2b'). */
int f110qp_lane_starts(f110qp_ctx* ctx, int batch, int* starts);

/* on = 1 when a gap-row call of `batch` QPs takes the box screen (F110QP_GAP_SCREEN_MIN_BATCH):
 * the lane back end solves the box-only problem, the wave kernel's GI only the QPs whose box
 * optimum does not keep every gap row (an ungrouped solve call; replaces nothing in the reference:
 * a query of this library's dispatch, like f110qp_backend_info). */
int f110qp_gap_screen(f110qp_ctx* ctx, int batch, int* on);

/* Forget the warm-start state of every slot (the next call solves cold). */
int f110qp_warm_reset(f110qp_ctx* ctx);

/* What the solve calls on this context did with the warm-start state (config.warm_start) since
 * the previous f110qp_warm_hits (or since the state was laid out for the batch size): *traffic =
 * the calls that loaded and stored the slots' keys and active sets (the lane back ends skip both
 * while no key hits, see warm_start), *hits = the QPs whose slot key equalled their linearisation
 * point, i.e. that started from the slot's previous active set. Counted by the lane back ends'
 * kernels (the wave back end reports 0); synchronises with the last warm call's stream; both 0
 * without warm_start. */
int f110qp_warm_hits(f110qp_ctx* ctx, int* traffic, int* hits);

/* Gap rows: how many QPs the last gap-row solve call on this context sent to the fp64
 * Goldfarb-Idnani re-check (the QPs whose fp32 GI answer the fp64
 * certificate did not accept). Synchronises with that call's stream; 0 before any gap-row call. */
int f110qp_last_recheck_count(f110qp_ctx* ctx, int* count);

/* How many synchronous calls on this context (f110qp_solve_batch_dev_sync, and the host-pointer
 * calls of at most 64 QPs, whose kernel stores the outputs into pinned host memory) waited on the
 * kernel's completion word instead of synchronising the stream: the calls whose last kernel (lane or
 * wave kernel, for gap rows the fp64 re-check) has at most 256 workgroups, which publishes the
 * call's number to a pinned host word after a system-scope fence (single-QP latency).
 * Larger launches, host-pointer calls of more than 64 QPs and the grouped calls synchronise the
 * stream. */
int f110qp_sync_signals(f110qp_ctx* ctx, unsigned* count);

/* 1 for the test / measurement build (lib_test/libf110qp.so, -DF110QP_TEST_HOOKS), whose
 * f110qp_create also reads create-time F110QP_* knobs from the environment that force kernel
 * variants for the tests; 0 for the product library, which reads no environment variable. */
int f110qp_test_build(void);

/* Debug/parity hook: the condensed Hessian H [B][2N][2N] and gradient g [B][2N] exactly as
 * the solve kernel builds them on the device (float64), for comparison with the CPU oracle's
 * condensing of the reference QP (src/mpc.cpp:208-306). Device pointers, async on stream. */
int f110qp_condense_debug_dev(f110qp_ctx* ctx, int batch, const float* x0, const float* u_lin,
                              const float* x_ref, double* H_out, double* g_out, void* stream);

/* Sizes of the reference's OSQP problem for horizon N (src/mpc.cpp:26-29): n = 5N+3 variables,
 * m = 7N+5 constraints, and the stored nonzeros of P (9(N+1) + 4N) and A (26N + 9), explicit
 * zeros of the dense blocks included. Returns F110QP_OK or F110QP_ERR_INVALID. */
int f110qp_qp_dims(int horizon, int* n, int* m, int* nnz_P, int* nnz_A);

/* Assembly-parity hook: ONE instance's QP exactly as
 * MPC::Update leaves it for OsqpEigen (src/mpc.cpp:77-80, layouts :208-306), computed on the
 * device from x0[3], u_lin[2], x_ref[S][3] (S = x_ref_points) and halfspace[6] (NULL: zeros) with
 * the solve kernels' Model::Linearize: P (CSC: colptr[n+1], rowind/val[nnz_P]), q[n], A (CSC:
 * colptr[n+1], rowind/val[nnz_A]), l[m], u[m]; +-1e30 = OsqpEigen::INFTY. gap_mode INACTIVE gives
 * the shipped rows (stage-0 all-ones placeholder block, +-INFTY bounds), ACTIVE the C3 semantic.
 * Device pointers, async on stream. */
int f110qp_assemble_debug_dev(f110qp_ctx* ctx, const float* x0, const float* u_lin,
                              const float* x_ref, const float* halfspace, int* P_colptr,
                              int* P_rowind, double* P_val, double* q, int* A_colptr, int* A_rowind,
                              double* A_val, double* l, double* u, void* stream);

/* Constraints::FindHalfSpaces (src/constraints.cpp:116-265) for one scan, host code.
 * state[3] = (x, y, ori); writes l1[3], l2[3] = (a, b, c+0.5). Returns F110QP_OK, or
 * F110QP_ERR_INVALID when the scan holds no gap (the reference then reads ranges[-1]). */
int f110qp_find_half_spaces(const double state[3], const float* ranges, int num_ranges,
                            float angle_min, float angle_increment, float angle_max,
                            float ftg_thresh, float divider, float buffer, double l1[3],
                            double l2[3]);

/* Batched FindHalfSpaces on the device, one wavefront per scan (num_ranges <= 65535, angle_increment
 * > 0): scans [B][num_ranges], states [B][3] -> hs [B][2][3]
 * (float32, the f110qp_solve_batch halfspace layout); gap_lo/gap_hi [B] may be NULL. */
int f110qp_find_half_spaces_dev(int batch, const float* states, const float* ranges,
                                int num_ranges, float angle_min, float angle_increment,
                                float angle_max, float ftg_thresh, float divider, float buffer,
                                float* hs_out, int* gap_lo, int* gap_hi, void* stream);

/* ---- planning stage in front of MPC::Update (src/project.cpp:73-152) ----------------------- */

typedef struct {
  int size;            /* occ_size, params.yaml:16 (OccGrid::size_ is int)                    */
  float discrete;      /* occ_discrete, params.yaml:17 (float)                                  */
  float dilation;      /* occ_dilation, params.yaml:18 (float)                                  */
  float lookahead;     /* lookahead, params.yaml:63 (Trajectory::lookahead is float)            */
  double speed_max;    /* umax as Traj_Plan reads it, params.yaml:46                            */
  double steer_max;    /* steer_max, params.yaml:60                                             */
  int steer_discrete;  /* params.yaml:59: T = steer_discrete + 1 candidates                     */
  int traj_discrete;   /* params.yaml:61: P points per candidate                               */
  double dt;           /* params.yaml:13 (Traj_Plan::dt is double)                              */
} f110qp_plan_config;

/* params.yaml defaults of the planning stage. */
void f110qp_default_plan_config(f110qp_plan_config* cfg);

/* Traj_Plan::generate_traj_table (src/trajectory_planner.cpp:26-72), host code: table
 * [T][P][3] doubles (car frame). Returns T (> 0) or a negative error code. */
int f110qp_traj_table(const f110qp_plan_config* cfg, double* table);

/* Trajectory::ReadCSV (src/trajectory.cpp:18-55) on CSV text in memory: wp[n][3] = (x, y, ori)
 * with the reference's float parsing and its (0u - 1) % n predecessor of point 0. Writes the
 * count to *n; returns F110QP_OK or F110QP_ERR_INVALID. */
int f110qp_parse_waypoints(const char* text, double* wp, int max_n, int* n);

/* The planning branch of project::OdomCallback (src/project.cpp:73-152) for B scenarios on the
 * device, one workgroup each: OccGrid::FillOccGrid of the scenario's LaserScan
 * (src/occupancy_grid.cpp:55-88), the collision check of the T candidates, the lookahead
 * waypoint (src/trajectory.cpp:81-126) and the nearest valid end point. Device pointers:
 *   pose [B][4] doubles (x, y, qz, qw; planar odometry pose), ranges [B][num_ranges],
 *   table [T][P][3] (f110qp_traj_table), waypoints [W][2] (x, y);
 * outputs: x_ref [B][P][3] = the chosen candidate in the map frame with ori 0 (miniPath_,
 * src/project.cpp:149-152; NaN without a candidate), x0 [B][3] = (x, y, GetCarOrientation)
 * for f110qp_solve_batch_dev, best_traj / best_global [B], status [B] (0 ok, 1 no valid
 * candidate — the reference returns before MPC, 2 no waypoint ahead — the reference throws);
 * valid [B][T] and grid [B][G][G] (G = size / discrete) may be NULL. */
int f110qp_plan_batch_dev(const f110qp_plan_config* cfg, int batch, const double* pose,
                          const float* ranges, int num_ranges, float angle_min,
                          float angle_increment, float angle_max, const double* table,
                          const double* waypoints, int num_waypoints, unsigned char* grid,
                          unsigned char* valid, int* best_global, int* best_traj, float* x_ref,
                          float* x0, int* status, void* stream);

/* Same on host pointers (synchronous; device buffers are cached per host thread). table and
 * waypoints are host arrays too. Used by the ROS-free host mirror for one scenario per tick. */
int f110qp_plan_batch(const f110qp_plan_config* cfg, int batch, const double* pose,
                      const float* ranges, int num_ranges, float angle_min, float angle_increment,
                      float angle_max, const double* table, const double* waypoints,
                      int num_waypoints, unsigned char* grid, unsigned char* valid,
                      int* best_global, int* best_traj, float* x_ref, float* x0, int* status);

#ifdef __cplusplus
}
#endif
#endif /* F110QP_H */

/*
 * f110_oracle.h — CPU restatement of the f110-mpc hot path (TEST INFRASTRUCTURE ONLY).
 *
 * This header belongs to the checker, not to the product. Only tests/, the
 * smoke() entry and bench.py's cpu_baseline leg may load the library built
 * from it. The shipped path (f110-mpc_amd/, include/f110qp.h) never links it.
 *
 * Everything is float64 unless a reference quirk forces float32 (FindHalfSpaces,
 * the float-typed params dt_, L, u bounds). Each function cites the reference
 * file:line it restates (paths relative to the reference repository root).
 *
 * Parity status: the reference publishes no tests, fixtures or solver outputs
 * and cannot be built here (ROS1 + Eigen3 + OsqpEigen + OSQP are absent), so the
 * QP *solution* parity is pinned to the exact optimum, certified by a KKT check
 * on the reference's own sparse formulation (f110o_kkt_residuals), not to
 * OSQP's (eps=1e-3) output. Linearize is pinned to known-answer vectors derived
 * from src/model.cpp:30-59 (tests/golden/linearize_kat.json).
 */
#ifndef F110_ORACLE_H
#define F110_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

#define F110O_INFTY 1e30 /* OsqpEigen::INFTY == OSQP_INFTY (constraints.cpp:15, mpc.cpp:279) */

/* Status codes (mirror include/f110qp.h) */
#define F110O_SOLVED 1
#define F110O_PRIMAL_INFEASIBLE -3
#define F110O_MAX_ITER -2
#define F110O_UNCERTIFIED -99 /* GI ended on a point that fails its own feasibility re-check */

typedef struct {
  int horizon;        /* params.yaml:12 (reference default 30) */
  float dt;           /* params.yaml:13; stored as float MPC::dt_ (mpc.h:46) */
  double q[3];        /* q0,q1,q2  params.yaml:1-3 */
  double r[2];        /* r0,r1     params.yaml:5-6 */
  double u_des[2];    /* des_vel, des_steer params.yaml:42-43 */
  float u_min[2];     /* (umin, -0.43f)  constraints.cpp:21 */
  float u_max[2];     /* (umax,  0.43f)  constraints.cpp:19 */
} f110o_params;

void f110o_default_params(f110o_params* p, int horizon);

/* model.cpp:30-59. A row-major 3x3, B row-major 3x2, C 3. */
void f110o_linearize(double theta, double v, double delta, double dt, double A[9], double B[6],
                     double C[3]);
/* model.cpp:61-75 (CAR_LENGTH = 0.35, model.cpp:2). */
void f110o_simulate_dynamics(const double s[3], const double u[2], double dt, double out[3]);

/* constraints.cpp:116-265 with float32 semantics. Writes l1,l2 = (a,b,c+0.5) as doubles
 * (Constraints::l1_/l2_ are VectorXd), plus the chosen (post-buffer) gap indices.
 * Quirk (i): when no gap exists best_lo = best_hi = -1 and the reference reads ranges[-1]
 * (UB); here that case returns -1 and leaves l1/l2 untouched. */
int f110o_find_half_spaces(const double state[3], const float* ranges, int num_ranges,
                           float angle_min, float angle_increment, float angle_max,
                           float ftg_thresh, float divider, float buffer, double l1[3],
                           double l2[3], int* best_lo, int* best_hi);
/* the same with the float overload of cos / sin at :182-186 (float_trig = 1), see f110_oracle.c */
int f110o_find_half_spaces_trig(const double state[3], const float* ranges, int num_ranges,
                           float angle_min, float angle_increment, float angle_max,
                           float ftg_thresh, float divider, float buffer, double l1[3],
                           double l2[3], int* best_lo, int* best_hi, int float_trig);

/* Dimensions of the reference QP (mpc.cpp:26-29). */
int f110o_num_variables(int horizon);
int f110o_num_constraints(int horizon);
int f110o_nnz_P(int horizon);
int f110o_nnz_A(int horizon);

/* mpc.cpp:208-306: the exact OSQP data (P, q, A, l, u) of one tick, CSC (Eigen column-major,
 * explicit zeros kept exactly as SparseBlockInit inserts them).
 *   x0[3], u_lin[2], x_ref[N*3], hs[6] = (l1, l2) or NULL (treated as zeros),
 *   gap_active = 0: reference-shipped bounds (gap rows +-INFTY, row block 0 all-ones)
 *   gap_active = 1: config-C3 semantic (gap rows l = -(c+0.5), u = +INFTY, all blocks [a b 0]).
 * Output arrays must be sized with the f110o_nnz_* / dims helpers. */
int f110o_assemble(const f110o_params* prm, const double x0[3], const double u_lin[2],
                   const double* x_ref, const double* hs, int gap_active, int* P_colptr,
                   int* P_rowind, double* P_val, double* q, int* A_colptr, int* A_rowind,
                   double* A_val, double* l, double* u);

/* Condensed problem of one tick (dynamics rows eliminated): H [2N*2N] row-major, g [2N],
 * objective 0.5 u'Hu + g'u (+ const), built from an explicit Gamma (float64). */
int f110o_condense(const f110o_params* prm, const double x0[3], const double u_lin[2],
                   const double* x_ref, double* H_out, double* g_out);

/* Exact solve of the tick's QP (condensed, dual active-set, float64) and the OSQP-layout
 * primal z (n) and dual y (m) reconstructed on the full formulation.
 *   u_out[N*2], x_out[(N+1)*3] (may be NULL), z_out[n], y_out[m] (may be NULL).
 * Returns F110O_SOLVED, F110O_PRIMAL_INFEASIBLE or F110O_MAX_ITER.
 * *n_active (may be NULL) = active inequality constraints at the optimum. */
int f110o_solve(const f110o_params* prm, const double x0[3], const double u_lin[2],
                const double* x_ref, const double* hs, int gap_active, double* u_out,
                double* x_out, double* z_out, double* y_out, double* obj_out, int* n_active);

/* KKT residuals of (z, y) on the assembled sparse QP:
 *   res[0] = ||P z + q + A'y||_inf, res[1] = primal infeasibility ||Az - proj_[l,u](Az)||_inf,
 *   res[2] = dual sign / complementarity violation. */
void f110o_kkt_residuals(const f110o_params* prm, const double x0[3], const double u_lin[2],
                         const double* x_ref, const double* hs, int gap_active, const double* z,
                         const double* y, double res[3]);

/* Batched exact solve (OpenMP over instances). Float inputs in the f110qp ABI layout.
 * Returns the number of instances with status SOLVED. */
int f110o_solve_batch(const f110o_params* prm, int batch, const float* x0, const float* u_lin,
                      const float* x_ref, const float* hs, int gap_active, double* u_out,
                      double* x_out, int* status, int num_threads);
int f110o_solve_batch_obj(const f110o_params* prm, int batch, const float* x0, const float* u_lin,
                          const float* x_ref, const float* hs, int gap_active, double* u_out,
                          double* x_out, int* status, double* obj_out, int num_threads);

/* OSQP-0.6-default-settings ADMM on the sparse formulation (CPU baseline; see osqp_admm.c). */
typedef struct {
  double rho, sigma, alpha, eps_abs, eps_rel;
  int max_iter, check_termination, scaling, adaptive_rho, warm_start;
} f110o_admm_settings;
void f110o_admm_default_settings(f110o_admm_settings* s);
int f110o_admm_solve(const f110o_params* prm, const f110o_admm_settings* s, const double x0[3],
                     const double u_lin[2], const double* x_ref, const double* hs, int gap_active,
                     double* z_inout, double* y_inout, int* iters);
int f110o_admm_solve_batch(const f110o_params* prm, const f110o_admm_settings* s, int batch,
                           const float* x0, const float* u_lin, const float* x_ref,
                           const float* hs, int gap_active, double* u_out, int* status,
                           int* iters, int num_threads);
/* single-QP ticks on the calling thread (C1 baseline): ns_out[t] per tick; exact = 1 -> f110o_solve */
int f110o_tick_latency(const f110o_params* prm, const f110o_admm_settings* s, int exact, int batch,
                       const float* x0, const float* u_lin, const float* x_ref, const float* hs,
                       int gap_active, int ticks, double* ns_out);

/* ---- planning stage in front of MPC::Update (plan_oracle.c; project.cpp:64-152) ---------- */
typedef struct {
  int size;            /* occ_size (OccGrid::size_ int), params.yaml:16 */
  float discrete;      /* occ_discrete (float), params.yaml:17 */
  float dilation;      /* occ_dilation (float), params.yaml:18 */
  float lookahead;     /* lookahead (Trajectory::lookahead float), params.yaml:63 */
  double speed_max;    /* umax as read by Traj_Plan (double), params.yaml:46 */
  double steer_max;    /* steer_max (double), params.yaml:60 */
  int steer_discrete;  /* params.yaml:59 (T = steer_discrete + 1 candidates) */
  int traj_discrete;   /* params.yaml:61 (P points per candidate) */
  double dt;           /* params.yaml:13 (Traj_Plan::dt double) */
} f110o_plan_params;

void f110o_default_plan_params(f110o_plan_params* p);
int f110o_grid_blocks(const f110o_plan_params* p);
/* trajectory_planner.cpp:26-72: table[T][P][3] (car frame, double); returns T */
int f110o_traj_table(const f110o_plan_params* p, double* table);
/* transforms.cpp:44-47 for pose = (x, y, qz, qw) */
float f110o_car_orientation(const double pose[4]);
/* the float dilation offsets of occupancy_grid.cpp:77-78; returns their count */
int f110o_dilation_offsets(const f110o_plan_params* p, float* offs, int max_n);
/* occupancy_grid.cpp:55-88: grid[G][G] (row = y cell), occ_offset_ */
void f110o_fill_occ_grid(const f110o_plan_params* p, const double pose[4], const float* ranges,
                         int nr, float angle_min, float angle_inc, float angle_max,
                         unsigned char* grid, float off[2]);
/* project.cpp:73-152 + trajectory.cpp:81-126: valid[T], best waypoint / candidate, the chosen
 * candidate in the map frame x_ref[P][3] (ori 0) and the MPC state x0. waypoints[W][2].
 * Returns 0, 1 (no valid candidate: the reference returns before MPC) or 2 (no waypoint ahead:
 * the reference throws on waypoints_.at(-1)). */
int f110o_plan(const f110o_plan_params* p, const double pose[4], const unsigned char* grid,
               const float off[2], const double* table, const double* waypoints, int W,
               unsigned char* valid, int* best_global, int* best_traj, float* x_ref,
               float x0[3]);
/* trajectory.cpp:18-55 on CSV text: wp[n][3] = (x, y, ori); returns n */
int f110o_parse_waypoints(const char* text, double* wp, int max_n);

#ifdef __cplusplus
}
#endif
#endif

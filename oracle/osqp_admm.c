/*
 * osqp_admm.c — restatement of OSQP 0.6's ADMM with its default settings, as the reference
 * calls it (TEST INFRASTRUCTURE / CPU BASELINE ONLY; never linked by the product).
 *
 * The reference solves each tick with OsqpEigen -> OSQP (src/mpc.cpp:83-142; settings only
 * warm_start = true, verbose = false at :98-99). OSQP is third-party and absent here (its
 * version is not pinned: bare find_package in CMakeLists.txt:21-22; the API usage points to
 * OsqpEigen <= 0.7 / OSQP 0.6.x). This file restates OSQP's published algorithm (Stellato et
 * al., "OSQP: an operator splitting solver for quadratic programs", Math. Prog. Comp. 2020,
 * and the 0.6 defaults) on the reference's own QP data (f110o_assemble):
 *   - modified Ruiz equilibration, scaling = 10 passes, plus cost scaling c;
 *   - rho = 0.1 (x1e3 on equality rows l == u, rho_min on loose rows), sigma = 1e-6,
 *     alpha = 1.6, eps_abs = eps_rel = 1e-3, eps_prim_inf = 1e-4, max_iter = 4000,
 *     check_termination = 25, polish off, unscaled termination;
 *   - adaptive rho with the deterministic interval 4 x check_termination = 100 (OSQP's rule
 *     when the timing-based interval is not used), tolerance x5;
 *   - the KKT system [P + sigma I, A'; A, -diag(1/rho)] factored by LDL' each time rho changes
 *     and once per tick (the reference changes A every tick, so OSQP re-scales and re-factors).
 *     QDLDL with an AMD ordering is replaced by a banded LDL' in a stage-interleaved ordering
 *     of the MPC KKT (bandwidth 17 at any horizon): the same O(n) factor cost class.
 */
#define _POSIX_C_SOURCE 199309L
#include <math.h>
#include <time.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "f110_oracle.h"

#define RHO_MIN 1e-6
#define RHO_MAX 1e6
#define RHO_EQ_OVER_RHO_INEQ 1e3
#define RHO_TOL 1e-4
#define MIN_SCALING 1e-4
#define MAX_SCALING 1e4
#define ADAPTIVE_RHO_TOLERANCE 5.0
#define ADAPTIVE_RHO_MULTIPLE_TERMINATION 4

void f110o_admm_default_settings(f110o_admm_settings* s) {
  s->rho = 0.1;
  s->sigma = 1e-6;
  s->alpha = 1.6;
  s->eps_abs = 1e-3;
  s->eps_rel = 1e-3;
  s->max_iter = 4000;
  s->check_termination = 25;
  s->scaling = 10;
  s->adaptive_rho = 1;
  s->warm_start = 1;
}

static double limit_scaling(double v) {
  if (v < MIN_SCALING) return 1.0;
  if (v > MAX_SCALING) return MAX_SCALING;
  return v;
}

typedef struct {
  int n, m, nk, bw;
  /* scaled data (CSC, P full symmetric) */
  int *Pc, *Pr, *Ac, *Ar;
  double *Pv, *Av, *q, *l, *u;
  double *D, *E, c;
  /* KKT in band form: perm[k] = original index of KKT unknown at position k */
  int *perm, *iperm;
  double* band; /* (nk) x (bw+1): band[k*(bw+1) + d] = K[k][k-d] (lower) */
  double* dvec; /* LDL' diagonal */
  double *rho_vec, *rho_inv, rho;
} admm_ws;

/* stage-interleaved ordering of the KKT unknowns: [x_i, dyn_i, gap_i, u_i, inp_i]_i */
static void kkt_order(int N, int* perm) {
  const int ns = 3 * (N + 1), n = ns + 2 * N;
  const int gap0 = n + ns, inp0 = n + ns + 2 * (N + 1);
  int k = 0;
  for (int i = 0; i <= N; i++) {
    for (int c = 0; c < 3; c++) perm[k++] = 3 * i + c;        /* x_i */
    for (int c = 0; c < 3; c++) perm[k++] = n + 3 * i + c;    /* dynamics rows of stage i */
    for (int h = 0; h < 2; h++) perm[k++] = gap0 + 2 * i + h; /* gap rows of stage i */
    if (i < N) {
      for (int a = 0; a < 2; a++) perm[k++] = ns + 2 * i + a; /* u_i */
      for (int a = 0; a < 2; a++) perm[k++] = inp0 + 2 * i + a; /* input rows of u_i */
    }
  }
}

static void band_set(admm_ws* w, int i, int j, double v) { /* original KKT indices */
  int a = w->iperm[i], b = w->iperm[j];
  if (a < b) { int t = a; a = b; b = t; }
  w->band[(size_t)a * (w->bw + 1) + (a - b)] += v;
}

static int factor_kkt(admm_ws* w, double sigma) {
  const int nk = w->nk, bw = w->bw, ld = bw + 1;
  memset(w->band, 0, (size_t)nk * ld * sizeof(double));
  for (int j = 0; j < w->n; j++) {
    for (int p = w->Pc[j]; p < w->Pc[j + 1]; p++)
      if (w->Pr[p] >= j) band_set(w, w->Pr[p], j, w->Pv[p]);
    band_set(w, j, j, sigma);
    for (int p = w->Ac[j]; p < w->Ac[j + 1]; p++) band_set(w, w->n + w->Ar[p], j, w->Av[p]);
  }
  for (int i = 0; i < w->m; i++) band_set(w, w->n + i, w->n + i, -w->rho_inv[i]);
  /* in-place banded LDL': band holds L (unit lower, below diagonal) and d on the diagonal */
  double* B = w->band;
  for (int j = 0; j < nk; j++) {
    double d = B[(size_t)j * ld];
    const int k0 = j - bw > 0 ? j - bw : 0;
    for (int k = k0; k < j; k++) {
      const double Ljk = B[(size_t)j * ld + (j - k)];
      d -= Ljk * Ljk * w->dvec[k];
    }
    if (d == 0.0 || !isfinite(d)) return -1;
    w->dvec[j] = d;
    const int i1 = j + bw < nk - 1 ? j + bw : nk - 1;
    for (int i = j + 1; i <= i1; i++) {
      double s = B[(size_t)i * ld + (i - j)];
      const int kk0 = i - bw > k0 ? i - bw : k0;
      for (int k = kk0; k < j; k++) s -= B[(size_t)i * ld + (i - k)] * B[(size_t)j * ld + (j - k)] * w->dvec[k];
      B[(size_t)i * ld + (i - j)] = s / d;
    }
  }
  return 0;
}

static void solve_kkt(const admm_ws* w, double* rhs /* original order, in/out */, double* tmp) {
  const int nk = w->nk, bw = w->bw, ld = bw + 1;
  for (int k = 0; k < nk; k++) tmp[k] = rhs[w->perm[k]];
  for (int i = 0; i < nk; i++) {
    const int k0 = i - bw > 0 ? i - bw : 0;
    double s = tmp[i];
    for (int k = k0; k < i; k++) s -= w->band[(size_t)i * ld + (i - k)] * tmp[k];
    tmp[i] = s;
  }
  for (int i = 0; i < nk; i++) tmp[i] /= w->dvec[i];
  for (int i = nk - 1; i >= 0; i--) {
    const int i1 = i + bw < nk - 1 ? i + bw : nk - 1;
    double s = tmp[i];
    for (int k = i + 1; k <= i1; k++) s -= w->band[(size_t)k * ld + (k - i)] * tmp[k];
    tmp[i] = s;
  }
  for (int k = 0; k < nk; k++) rhs[w->perm[k]] = tmp[k];
}

static void set_rho_vec(admm_ws* w) {
  for (int i = 0; i < w->m; i++) {
    double r;
    if (w->l[i] < -F110O_INFTY * MIN_SCALING && w->u[i] > F110O_INFTY * MIN_SCALING) r = RHO_MIN;
    else if (w->u[i] - w->l[i] < RHO_TOL) r = RHO_EQ_OVER_RHO_INEQ * w->rho;
    else r = w->rho;
    w->rho_vec[i] = r;
    w->rho_inv[i] = 1.0 / r;
  }
}

/* Ruiz equilibration (OSQP scale_data) */
static void scale_data(admm_ws* w, int passes) {
  const int n = w->n, m = w->m;
  double* Dt = (double*)malloc(n * sizeof(double));
  double* Et = (double*)malloc((m > 0 ? m : 1) * sizeof(double));
  for (int j = 0; j < n; j++) w->D[j] = 1.0;
  for (int i = 0; i < m; i++) w->E[i] = 1.0;
  w->c = 1.0;
  for (int it = 0; it < passes; it++) {
    for (int j = 0; j < n; j++) Dt[j] = 0.0;
    for (int i = 0; i < m; i++) Et[i] = 0.0;
    for (int j = 0; j < n; j++) {
      for (int p = w->Pc[j]; p < w->Pc[j + 1]; p++) Dt[j] = fmax(Dt[j], fabs(w->Pv[p]));
      for (int p = w->Ac[j]; p < w->Ac[j + 1]; p++) {
        Dt[j] = fmax(Dt[j], fabs(w->Av[p]));
        Et[w->Ar[p]] = fmax(Et[w->Ar[p]], fabs(w->Av[p]));
      }
    }
    for (int j = 0; j < n; j++) Dt[j] = 1.0 / sqrt(limit_scaling(Dt[j]));
    for (int i = 0; i < m; i++) Et[i] = 1.0 / sqrt(limit_scaling(Et[i]));
    for (int j = 0; j < n; j++) {
      for (int p = w->Pc[j]; p < w->Pc[j + 1]; p++) w->Pv[p] *= Dt[w->Pr[p]] * Dt[j];
      for (int p = w->Ac[j]; p < w->Ac[j + 1]; p++) w->Av[p] *= Et[w->Ar[p]] * Dt[j];
      w->q[j] *= Dt[j];
      w->D[j] *= Dt[j];
    }
    for (int i = 0; i < m; i++) w->E[i] *= Et[i];
    /* cost scaling */
    double mean = 0.0, qn = 0.0;
    for (int j = 0; j < n; j++) {
      double cm = 0.0;
      for (int p = w->Pc[j]; p < w->Pc[j + 1]; p++) cm = fmax(cm, fabs(w->Pv[p]));
      mean += cm;
      qn = fmax(qn, fabs(w->q[j]));
    }
    mean /= n;
    double ct = fmax(mean, limit_scaling(qn));
    ct = 1.0 / limit_scaling(ct);
    for (int p = 0; p < w->Pc[n]; p++) w->Pv[p] *= ct;
    for (int j = 0; j < n; j++) w->q[j] *= ct;
    w->c *= ct;
  }
  for (int i = 0; i < m; i++) {
    if (w->l[i] > -F110O_INFTY) w->l[i] *= w->E[i];
    if (w->u[i] < F110O_INFTY) w->u[i] *= w->E[i];
  }
  free(Dt);
  free(Et);
}

static double inf_norm(const double* v, int k) {
  double r = 0.0;
  for (int i = 0; i < k; i++) r = fmax(r, fabs(v[i]));
  return r;
}

int f110o_admm_solve(const f110o_params* prm, const f110o_admm_settings* s, const double x0[3],
                     const double u_lin[2], const double* x_ref, const double* hs, int gap_active,
                     double* z_inout, double* y_inout, int* iters) {
  const int N = prm->horizon, n = f110o_num_variables(N), m = f110o_num_constraints(N);
  admm_ws w;
  memset(&w, 0, sizeof(w));
  w.n = n; w.m = m; w.nk = n + m;
  w.Pc = (int*)malloc((n + 1) * sizeof(int)); w.Pr = (int*)malloc(f110o_nnz_P(N) * sizeof(int));
  w.Ac = (int*)malloc((n + 1) * sizeof(int)); w.Ar = (int*)malloc(f110o_nnz_A(N) * sizeof(int));
  w.Pv = (double*)malloc(f110o_nnz_P(N) * sizeof(double));
  w.Av = (double*)malloc(f110o_nnz_A(N) * sizeof(double));
  w.q = (double*)malloc(n * sizeof(double));
  w.l = (double*)malloc(m * sizeof(double)); w.u = (double*)malloc(m * sizeof(double));
  w.D = (double*)malloc(n * sizeof(double)); w.E = (double*)malloc(m * sizeof(double));
  w.perm = (int*)malloc(w.nk * sizeof(int)); w.iperm = (int*)malloc(w.nk * sizeof(int));
  w.rho_vec = (double*)malloc(m * sizeof(double)); w.rho_inv = (double*)malloc(m * sizeof(double));
  w.dvec = (double*)malloc(w.nk * sizeof(double));
  f110o_assemble(prm, x0, u_lin, x_ref, hs, gap_active, w.Pc, w.Pr, w.Pv, w.q, w.Ac, w.Ar, w.Av, w.l, w.u);
  kkt_order(N, w.perm);
  for (int k = 0; k < w.nk; k++) w.iperm[w.perm[k]] = k;
  /* bandwidth of the permuted KKT pattern */
  int bw = 0;
  for (int j = 0; j < n; j++) {
    for (int p = w.Pc[j]; p < w.Pc[j + 1]; p++) bw = fmax(bw, abs(w.iperm[w.Pr[p]] - w.iperm[j]));
    for (int p = w.Ac[j]; p < w.Ac[j + 1]; p++) bw = fmax(bw, abs(w.iperm[n + w.Ar[p]] - w.iperm[j]));
  }
  w.bw = bw;
  w.band = (double*)malloc((size_t)w.nk * (bw + 1) * sizeof(double));
  if (s->scaling > 0) scale_data(&w, s->scaling);
  else {
    for (int j = 0; j < n; j++) w.D[j] = 1.0;
    for (int i = 0; i < m; i++) w.E[i] = 1.0;
    w.c = 1.0;
  }
  w.rho = s->rho;
  set_rho_vec(&w);
  int status = F110O_MAX_ITER;
  double *x = (double*)calloc(n, sizeof(double)), *z = (double*)calloc(m, sizeof(double));
  double *y = (double*)calloc(m, sizeof(double)), *xp = (double*)malloc(n * sizeof(double));
  double *zp = (double*)malloc(m * sizeof(double)), *rhs = (double*)malloc(w.nk * sizeof(double));
  double *tmp = (double*)malloc(w.nk * sizeof(double)), *zt = (double*)malloc(m * sizeof(double));
  double *Ax = (double*)malloc(m * sizeof(double)), *Px = (double*)malloc(n * sizeof(double));
  double *Aty = (double*)malloc(n * sizeof(double)), *dy = (double*)malloc(m * sizeof(double));
  double *yprev = (double*)malloc(m * sizeof(double));
  if (s->warm_start && z_inout && y_inout) { /* warm start from an unscaled (x, y) */
    for (int j = 0; j < n; j++) x[j] = z_inout[j] / w.D[j];
    for (int i = 0; i < m; i++) y[i] = y_inout[i] * w.c / w.E[i];
    for (int i = 0; i < m; i++) z[i] = 0.0;
    for (int j = 0; j < n; j++)
      for (int p = w.Ac[j]; p < w.Ac[j + 1]; p++) z[w.Ar[p]] += w.Av[p] * x[j];
  }
  if (factor_kkt(&w, s->sigma)) { status = -10; goto done; }
  const int rho_interval = ADAPTIVE_RHO_MULTIPLE_TERMINATION * s->check_termination;
  int it;
  for (it = 1; it <= s->max_iter; it++) {
    memcpy(xp, x, n * sizeof(double));
    memcpy(zp, z, m * sizeof(double));
    memcpy(yprev, y, m * sizeof(double));
    for (int j = 0; j < n; j++) rhs[j] = s->sigma * xp[j] - w.q[j];
    for (int i = 0; i < m; i++) rhs[n + i] = zp[i] - w.rho_inv[i] * y[i];
    solve_kkt(&w, rhs, tmp);
    for (int i = 0; i < m; i++) zt[i] = zp[i] + w.rho_inv[i] * (rhs[n + i] - y[i]);
    for (int j = 0; j < n; j++) x[j] = s->alpha * rhs[j] + (1.0 - s->alpha) * xp[j];
    for (int i = 0; i < m; i++) {
      const double zr = s->alpha * zt[i] + (1.0 - s->alpha) * zp[i];
      double zz = zr + w.rho_inv[i] * y[i];
      zz = zz < w.l[i] ? w.l[i] : (zz > w.u[i] ? w.u[i] : zz);
      z[i] = zz;
      y[i] += w.rho_vec[i] * (zr - zz);
    }
    const int check = (s->check_termination && it % s->check_termination == 0) || it == s->max_iter;
    const int adapt = s->adaptive_rho && it % rho_interval == 0;
    if (!check && !adapt) continue;
    /* residuals on the unscaled problem */
    for (int i = 0; i < m; i++) Ax[i] = 0.0;
    for (int j = 0; j < n; j++) { Px[j] = 0.0; Aty[j] = 0.0; }
    for (int j = 0; j < n; j++) {
      for (int p = w.Pc[j]; p < w.Pc[j + 1]; p++) Px[w.Pr[p]] += w.Pv[p] * x[j];
      for (int p = w.Ac[j]; p < w.Ac[j + 1]; p++) {
        Ax[w.Ar[p]] += w.Av[p] * x[j];
        Aty[j] += w.Av[p] * y[w.Ar[p]];
      }
    }
    double prim = 0, axn = 0, zn = 0, dual = 0, pxn = 0, atyn = 0, qn = 0;
    for (int i = 0; i < m; i++) {
      prim = fmax(prim, fabs((Ax[i] - z[i]) / w.E[i]));
      axn = fmax(axn, fabs(Ax[i] / w.E[i]));
      zn = fmax(zn, fabs(z[i] / w.E[i]));
    }
    for (int j = 0; j < n; j++) {
      const double s1 = 1.0 / (w.c * w.D[j]);
      dual = fmax(dual, fabs((Px[j] + w.q[j] + Aty[j]) * s1));
      pxn = fmax(pxn, fabs(Px[j] * s1));
      atyn = fmax(atyn, fabs(Aty[j] * s1));
      qn = fmax(qn, fabs(w.q[j] * s1));
    }
    if (check) {
      const double ep = s->eps_abs + s->eps_rel * fmax(axn, zn);
      const double ed = s->eps_abs + s->eps_rel * fmax(pxn, fmax(atyn, qn));
      if (prim < ep && dual < ed) { status = F110O_SOLVED; break; }
      /* primal infeasibility certificate (unscaled dy = E dy_scaled) */
      for (int i = 0; i < m; i++) dy[i] = (y[i] - yprev[i]) * w.E[i];
      const double dyn = inf_norm(dy, m);
      if (dyn > 1e-4 * 1e-4) {
        double atdy = 0.0, sup = 0.0;
        for (int j = 0; j < n; j++) {
          double t = 0.0;
          for (int p = w.Ac[j]; p < w.Ac[j + 1]; p++) t += w.Av[p] * (y[w.Ar[p]] - yprev[w.Ar[p]]);
          atdy = fmax(atdy, fabs(t / w.D[j]));
        }
        for (int i = 0; i < m; i++) {
          const double ui = w.u[i] < F110O_INFTY * MIN_SCALING ? w.u[i] / w.E[i] : 0.0;
          const double li = w.l[i] > -F110O_INFTY * MIN_SCALING ? w.l[i] / w.E[i] : 0.0;
          if (dy[i] > 0) { if (w.u[i] >= F110O_INFTY * MIN_SCALING) { sup = INFINITY; break; } sup += ui * dy[i]; }
          else if (dy[i] < 0) { if (w.l[i] <= -F110O_INFTY * MIN_SCALING) { sup = INFINITY; break; } sup += li * dy[i]; }
        }
        if (atdy <= 1e-4 * dyn && sup <= -1e-4 * dyn) { status = F110O_PRIMAL_INFEASIBLE; break; }
      }
    }
    if (adapt) {
      const double pr = prim / (fmax(axn, zn) + 1e-10);
      const double du = dual / (fmax(pxn, fmax(atyn, qn)) + 1e-10);
      double rn = w.rho * sqrt(pr / (du + 1e-10));
      rn = fmin(fmax(rn, RHO_MIN), RHO_MAX);
      if (rn > w.rho * ADAPTIVE_RHO_TOLERANCE || rn < w.rho / ADAPTIVE_RHO_TOLERANCE) {
        w.rho = rn;
        set_rho_vec(&w);
        if (factor_kkt(&w, s->sigma)) { status = -10; break; }
      }
    }
  }
  if (iters) *iters = it > s->max_iter ? s->max_iter : it;
  if (z_inout) for (int j = 0; j < n; j++) z_inout[j] = status == F110O_SOLVED ? x[j] * w.D[j] : NAN;
  if (y_inout) for (int i = 0; i < m; i++) y_inout[i] = y[i] * w.E[i] / w.c;
done:
  free(w.Pc); free(w.Pr); free(w.Ac); free(w.Ar); free(w.Pv); free(w.Av); free(w.q); free(w.l);
  free(w.u); free(w.D); free(w.E); free(w.perm); free(w.iperm); free(w.rho_vec); free(w.rho_inv);
  free(w.dvec); free(w.band);
  free(x); free(z); free(y); free(xp); free(zp); free(rhs); free(tmp); free(zt); free(Ax); free(Px);
  free(Aty); free(dy); free(yprev);
  return status;
}

int f110o_admm_solve_batch(const f110o_params* prm, const f110o_admm_settings* s, int batch,
                           const float* x0, const float* u_lin, const float* x_ref,
                           const float* hs, int gap_active, double* u_out, int* status,
                           int* iters, int num_threads) {
  const int N = prm->horizon, n = f110o_num_variables(N), ns = 3 * (N + 1);
  int nsolved = 0;
#ifdef _OPENMP
  if (num_threads > 0) omp_set_num_threads(num_threads);
#pragma omp parallel for schedule(dynamic, 8) reduction(+ : nsolved)
#endif
  for (int b = 0; b < batch; b++) {
    double xx[3], uu[2], hh[6];
    double* xr = (double*)malloc(3 * N * sizeof(double));
    double* z = (double*)malloc(n * sizeof(double));
    for (int k = 0; k < 3; k++) xx[k] = x0[3 * b + k];
    for (int k = 0; k < 2; k++) uu[k] = u_lin[2 * b + k];
    for (int k = 0; k < 3 * N; k++) xr[k] = x_ref[(size_t)b * 3 * N + k];
    if (hs) for (int k = 0; k < 6; k++) hh[k] = hs[6 * b + k];
    f110o_admm_settings cold = *s;
    cold.warm_start = 0; /* independent QPs of a batch: cold start */
    int it = 0;
    const int st = f110o_admm_solve(prm, &cold, xx, uu, xr, hs ? hh : NULL, gap_active, z, NULL, &it);
    if (u_out) for (int k = 0; k < 2 * N; k++) u_out[(size_t)b * 2 * N + k] = z[ns + k];
    if (status) status[b] = st;
    if (iters) iters[b] = it;
    nsolved += st == F110O_SOLVED;
    free(xr);
    free(z);
  }
  return nsolved;
}

/* C1 CPU baseline (BASELINE configs[0]): single-QP control ticks on the CALLING
 * thread, one core, as MPC::Update solves one QP per odometry tick (src/mpc.cpp:133,
 * src/project.cpp:188). Tick t solves instance t % batch; ns_out[t] = wall nanoseconds of that
 * tick's whole solve (set-up + factorisation + iterations + solution), clock_gettime MONOTONIC.
 * exact = 0: the OSQP-0.6-defaults ADMM restatement (cold per tick, as the batch baseline);
 * exact = 1: the exact condensed active-set oracle. Returns the number of SOLVED ticks. */
int f110o_tick_latency(const f110o_params* prm, const f110o_admm_settings* s, int exact, int batch,
                       const float* x0, const float* u_lin, const float* x_ref, const float* hs,
                       int gap_active, int ticks, double* ns_out) {
  const int N = prm->horizon, n = f110o_num_variables(N);
  double* xr = (double*)malloc(3 * N * sizeof(double));
  double* z = (double*)malloc(n * sizeof(double));
  double* u = (double*)malloc(2 * N * sizeof(double));
  double* x = (double*)malloc(3 * (N + 1) * sizeof(double));
  int nsolved = 0;
  f110o_admm_settings cold = *s;
  cold.warm_start = 0;
  for (int t = 0; t < ticks; t++) {
    const int b = t % batch;
    double xx[3], uu[2], hh[6];
    for (int k = 0; k < 3; k++) xx[k] = x0[3 * b + k];
    for (int k = 0; k < 2; k++) uu[k] = u_lin[2 * b + k];
    for (int k = 0; k < 3 * N; k++) xr[k] = x_ref[(size_t)b * 3 * N + k];
    if (hs) for (int k = 0; k < 6; k++) hh[k] = hs[6 * b + k];
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    int st, it = 0;
    if (exact)
      st = f110o_solve(prm, xx, uu, xr, hs ? hh : NULL, gap_active, u, x, NULL, NULL, NULL, NULL);
    else
      st = f110o_admm_solve(prm, &cold, xx, uu, xr, hs ? hh : NULL, gap_active, z, NULL, &it);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    ns_out[t] = (double)(t1.tv_sec - t0.tv_sec) * 1e9 + (double)(t1.tv_nsec - t0.tv_nsec);
    nsolved += st == F110O_SOLVED;
  }
  free(xr); free(z); free(u); free(x);
  return nsolved;
}

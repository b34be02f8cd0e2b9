/*
 * f110_oracle.c — CPU restatement of the f110-mpc MPC tick (TEST INFRASTRUCTURE ONLY).
 *
 * Checker for the HIP product path: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load liboracle.so. Citations are reference file:line.
 *
 * Contents
 *   - Model::Linearize / simulate_dynamics          src/model.cpp:30-75
 *   - Constraints::FindHalfSpaces (float32 quirks)  src/constraints.cpp:116-265
 *   - MPC QP assembly (P,q,A,l,u, CSC)              src/mpc.cpp:26-29, 208-340
 *   - exact solve: condensed QP + dual active set (Goldfarb-Idnani, range-space form),
 *     float64, followed by reconstruction of OSQP's (z, y) on the full formulation and a
 *     KKT certificate on the reference's own sparse QP (the optimum is unique: min eig of the
 *     condensed Hessian >= min(R) > 0).
 */
#include "f110_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------------------------ */
/* params                                                                                      */
/* ------------------------------------------------------------------------------------------ */
void f110o_default_params(f110o_params* p, int horizon) {
  /* params.yaml:1-13,42-47 ; constraints.cpp:19,21 */
  p->horizon = horizon;
  p->dt = 0.01f;
  p->q[0] = 10.0; p->q[1] = 10.0; p->q[2] = 0.0;
  p->r[0] = 0.10; p->r[1] = 5.0;
  p->u_des[0] = 4.5; p->u_des[1] = 0.0;
  p->u_min[0] = 3.0f; p->u_min[1] = -0.43f;
  p->u_max[0] = 4.5f; p->u_max[1] = 0.43f;
}

int f110o_num_variables(int N) { return 3 * (N + 1) + 2 * N; }            /* mpc.cpp:26-28 */
int f110o_num_constraints(int N) { return 3 * (N + 1) + 2 * (N + 1) + 2 * N; } /* mpc.cpp:29 */
int f110o_nnz_P(int N) { return 9 * (N + 1) + 4 * N; }
int f110o_nnz_A(int N) { return 26 * N + 9; }

/* ------------------------------------------------------------------------------------------ */
/* model                                                                                       */
/* ------------------------------------------------------------------------------------------ */
void f110o_linearize(double th, double v, double d, double dt, double A[9], double B[6],
                     double C[3]) {
  const float L = 0.3302f; /* model.cpp:32 */
  const double sec2 = pow(cos(d), -2);
  memset(A, 0, 9 * sizeof(double));
  memset(B, 0, 6 * sizeof(double));
  A[0 * 3 + 2] = -1 * v * sin(th) * dt; /* :42 */
  A[1 * 3 + 2] = v * cos(th) * dt;      /* :43 */
  A[0] = 1; A[4] = 1; A[8] = 1;         /* :44-46 */
  B[0 * 2 + 0] = cos(th) * dt;          /* :48 */
  B[1 * 2 + 0] = sin(th) * dt;          /* :49 */
  B[2 * 2 + 0] = tan(d) * dt / L;       /* :50 */
  B[2 * 2 + 1] = v * sec2 * dt / L;     /* :51 */
  C[0] = v * th * sin(th) * dt;         /* :53 */
  C[1] = -1 * v * th * cos(th) * dt;    /* :54 */
  C[2] = -1 * d * v * sec2 * dt / L;    /* :55 */
}

void f110o_simulate_dynamics(const double s[3], const double u[2], double dt, double out[3]) {
  const double CAR_LENGTH = 0.35; /* model.cpp:2 */
  double dyn0 = u[0] * cos(s[2]);
  double dyn1 = u[0] * sin(s[2]);
  double dyn2 = tan(u[1]) * u[0] / CAR_LENGTH; /* model.cpp:67-69 */
  out[0] = s[0] + dyn0 * dt;
  out[1] = s[1] + dyn1 * dt;
  out[2] = s[2] + dyn2 * dt; /* :71-75 */
}

/* ------------------------------------------------------------------------------------------ */
/* follow-the-gap half spaces (constraints.cpp:116-265), float32 members as in the class     */
/* ------------------------------------------------------------------------------------------ */
/* float_trig selects the overload the reference's unqualified cos(angle1) / sin(angle1) on a float
 * angle (:182-186) resolves to: 0 = ::cos(double) (the C library function; the restatement's
 * default), 1 = the float overload std::cos(float) (= cosf, the product ranges * cosf in float),
 * which the libstdc++ <math.h> wrapper puts in the global namespace when some header of the ROS /
 * Eigen include chain pulls it in. Which one the reference build gets cannot be checked here
 * (ROS and Eigen are absent); tests/test_halfspace_overload.py measures the difference. */
int f110o_find_half_spaces_trig(const double state[3], const float* ranges, int nr, float angle_min,
                                float angle_inc, float angle_max, float ftg_thresh, float divider,
                                float buffer, double l1[3], double l2[3], int* out_lo, int* out_hi,
                                int float_trig);

int f110o_find_half_spaces(const double state[3], const float* ranges, int nr, float angle_min,
                           float angle_inc, float angle_max, float ftg_thresh, float divider,
                           float buffer, double l1[3], double l2[3], int* out_lo, int* out_hi) {
  return f110o_find_half_spaces_trig(state, ranges, nr, angle_min, angle_inc, angle_max, ftg_thresh,
                                     divider, buffer, l1, l2, out_lo, out_hi, 0);
}

int f110o_find_half_spaces_trig(const double state[3], const float* ranges, int nr, float angle_min,
                                float angle_inc, float angle_max, float ftg_thresh, float divider,
                                float buffer, double l1[3], double l2[3], int* out_lo, int* out_hi,
                                int float_trig) {
  int num_scans = (int)((angle_max - angle_min) / angle_inc + 1); /* :118 */
  if (num_scans > nr) num_scans = nr;
  int max_gap = -1, best_lo = 0, best_hi = 0, lo = -1, hi = -1; /* :119-123 */
  double poseX = state[0], poseY = state[1];
  float current_angle = (float)state[2]; /* :127 */
  int in_gap = 0;
  for (int ii = 0; ii < num_scans; ii++) {
    float angle = angle_min + ii * angle_inc; /* :133 */
    if (angle > -1.571f / divider && angle < 1.571f / divider) { /* :135 */
      if (ranges[ii] > ftg_thresh) {                            /* :138 */
        if (in_gap) hi = ii;
        else { lo = ii; in_gap = 1; }
      } else {
        in_gap = 0;
        if (hi - lo > max_gap) { max_gap = hi - lo; best_hi = hi; best_lo = lo; }
      }
      if (hi - lo > max_gap) { max_gap = hi - lo; best_hi = hi; best_lo = lo; } /* :162-167 */
    }
  }
  if (best_hi - best_lo > 2 * buffer) { /* :173-177 (int compared with float buffer_) */
    best_hi = (int)(best_hi - buffer);
    best_lo = (int)(best_lo + buffer);
  }
  if (out_lo) *out_lo = best_lo;
  if (out_hi) *out_hi = best_hi;
  if (best_lo < 0 || best_hi < 0 || best_lo >= nr || best_hi >= nr) return -1; /* quirk (i) */
  float angle1 = angle_min + best_lo * angle_inc + current_angle; /* :179 */
  float angle2 = angle_min + best_hi * angle_inc + current_angle; /* :180 */
  float p1x, p1y, p2x, p2y;
  if (!float_trig) {
    p1x = (float)(ranges[best_lo] * cos((double)angle1) + poseX); /* :182 */
    p1y = (float)(ranges[best_lo] * sin((double)angle1) + poseY); /* :183 */
    p2x = (float)(ranges[best_hi] * cos((double)angle2) + poseX); /* :185 */
    p2y = (float)(ranges[best_hi] * sin((double)angle2) + poseY); /* :186 */
  } else { /* float overload: float product, then + double pose */
    const float t1x = ranges[best_lo] * cosf(angle1), t1y = ranges[best_lo] * sinf(angle1);
    const float t2x = ranges[best_hi] * cosf(angle2), t2y = ranges[best_hi] * sinf(angle2);
    p1x = (float)((double)t1x + poseX);
    p1y = (float)((double)t1y + poseY);
    p2x = (float)((double)t2x + poseX);
    p2y = (float)((double)t2y + poseY);
  }
  float px = (float)poseX, py = (float)poseY;                         /* :188-189 */
  float a1 = py - p1y, b1 = p1x - px, c1 = px * p1y - py * p1x;       /* :233-235 */
  if (a1 * p2x + b1 * p2y + c1 < 0) { a1 = -a1; b1 = -b1; c1 = -c1; } /* :237-242 */
  float a2 = py - p2y, b2 = p2x - px, c2 = px * p2y - py * p2x;       /* :244-246 */
  if (a2 * p1x + b2 * p1y + c2 < 0) { a2 = -a2; b2 = -b2; c2 = -c2; } /* :248-253 */
  l1[0] = a1; l1[1] = b1; l1[2] = (double)c1 + 0.5; /* :258-260 */
  l2[0] = a2; l2[1] = b2; l2[2] = (double)c2 + 0.5; /* :262-264 */
  return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* assembly (mpc.cpp:208-340)                                                                  */
/* ------------------------------------------------------------------------------------------ */
static void ref_point(const double* x_ref, int N, int i, double r[3]) {
  /* CreateGradientVector: stages 0..N-1 use x_ref[i], terminal uses x_ref[N-1] (mpc.cpp:223-228) */
  int k = i < N ? i : N - 1;
  r[0] = x_ref[3 * k + 0]; r[1] = x_ref[3 * k + 1]; r[2] = x_ref[3 * k + 2];
}

int f110o_assemble(const f110o_params* prm, const double x0[3], const double ulin[2],
                   const double* x_ref, const double* hs, int gap_active, int* Pc, int* Pr,
                   double* Pv, double* q, int* Ac, int* Ar, double* Av, double* l, double* u) {
  const int N = prm->horizon, ns = 3 * (N + 1), n = ns + 2 * N;
  const int gap0 = ns, inp0 = ns + 2 * (N + 1);
  double A[9], B[6], C[3];
  f110o_linearize(x0[2], ulin[0], ulin[1], (double)prm->dt, A, B, C);
  double hz[6] = {0, 0, 0, 0, 0, 0};
  if (hs) memcpy(hz, hs, sizeof(hz));
  /* P = blkdiag(Q x (N+1), R x N), dense blocks incl. explicit zeros (mpc.cpp:208-219) */
  int nz = 0;
  for (int j = 0; j < n; j++) {
    Pc[j] = nz;
    if (j < ns) {
      int b = j / 3, c = j % 3;
      for (int rr = 0; rr < 3; rr++) { Pr[nz] = 3 * b + rr; Pv[nz] = (rr == c) ? prm->q[c] : 0.0; nz++; }
    } else {
      int k = (j - ns) / 2, a = (j - ns) % 2;
      for (int rr = 0; rr < 2; rr++) { Pr[nz] = ns + 2 * k + rr; Pv[nz] = (rr == a) ? prm->r[a] : 0.0; nz++; }
    }
  }
  Pc[n] = nz;
  /* q (mpc.cpp:221-229) */
  for (int i = 0; i <= N; i++) {
    double r[3];
    ref_point(x_ref, N, i, r);
    for (int c = 0; c < 3; c++) q[3 * i + c] = -1 * prm->q[c] * r[c];
  }
  for (int k = 0; k < N; k++)
    for (int a = 0; a < 2; a++) q[ns + 2 * k + a] = -1 * prm->r[a] * prm->u_des[a];
  /* A (mpc.cpp:231-273) */
  nz = 0;
  for (int j = 0; j < n; j++) {
    Ac[j] = nz;
    if (j < ns) {
      int i = j / 3, c = j % 3;
      Ar[nz] = 3 * i + c; Av[nz] = -1; nz++; /* SparseBlockEye(-1) :244 */
      if (i < N)
        for (int rr = 0; rr < 3; rr++) { Ar[nz] = 3 * (i + 1) + rr; Av[nz] = A[rr * 3 + c]; nz++; } /* :247,269 */
      for (int h = 0; h < 2; h++) { /* gap rows :241,249,271 */
        double coef;
        if (i == 0 && !gap_active) coef = 1.0; /* placeholder ones never updated (:241, loop from ii=1) */
        else coef = (c == 2) ? 0.0 : hz[3 * h + c];
        Ar[nz] = gap0 + 2 * i + h; Av[nz] = coef; nz++;
      }
    } else {
      int k = (j - ns) / 2, a = (j - ns) % 2;
      for (int rr = 0; rr < 3; rr++) { Ar[nz] = 3 * (k + 1) + rr; Av[nz] = B[rr * 2 + a]; nz++; } /* :248,270 */
      Ar[nz] = inp0 + 2 * k + a; Av[nz] = 1; nz++; /* :253 */
    }
  }
  Ac[n] = nz;
  /* bounds (mpc.cpp:275-306) */
  for (int c = 0; c < 3; c++) { l[c] = -x0[c]; u[c] = -x0[c]; }
  for (int i = 1; i <= N; i++)
    for (int c = 0; c < 3; c++) { l[3 * i + c] = -C[c]; u[3 * i + c] = -C[c]; }
  for (int i = 0; i <= N; i++)
    for (int h = 0; h < 2; h++) {
      l[gap0 + 2 * i + h] = gap_active ? -hz[3 * h + 2] : -F110O_INFTY; /* :297-298 (commented) */
      u[gap0 + 2 * i + h] = F110O_INFTY;
    }
  for (int k = 0; k < N; k++)
    for (int a = 0; a < 2; a++) {
      l[inp0 + 2 * k + a] = (double)prm->u_min[a];
      u[inp0 + 2 * k + a] = (double)prm->u_max[a];
    }
  return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* dense linear algebra helpers (small, column-agnostic row-major)                            */
/* ------------------------------------------------------------------------------------------ */
static int chol(double* a, int n, int lda) { /* in-place lower Cholesky, returns 0 on success */
  for (int j = 0; j < n; j++) {
    double s = a[j * lda + j];
    for (int k = 0; k < j; k++) s -= a[j * lda + k] * a[j * lda + k];
    if (!(s > 0)) return -1;
    double d = sqrt(s);
    a[j * lda + j] = d;
    for (int i = j + 1; i < n; i++) {
      double t = a[i * lda + j];
      for (int k = 0; k < j; k++) t -= a[i * lda + k] * a[j * lda + k];
      a[i * lda + j] = t / d;
    }
  }
  return 0;
}
static void lsolve(const double* L, int n, int lda, double* x) {
  for (int i = 0; i < n; i++) {
    double t = x[i];
    for (int k = 0; k < i; k++) t -= L[i * lda + k] * x[k];
    x[i] = t / L[i * lda + i];
  }
}
static void ltsolve(const double* L, int n, int lda, double* x) {
  for (int i = n - 1; i >= 0; i--) {
    double t = x[i];
    for (int k = i + 1; k < n; k++) t -= L[k * lda + i] * x[k];
    x[i] = t / L[i * lda + i];
  }
}

/* ------------------------------------------------------------------------------------------ */
/* condensed problem                                                                           */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
  int N, nu, ns, m;     /* nu = 2N decision inputs; m one-sided constraints */
  double A[9], B[6], C[3];
  double *G, *f;        /* Gamma (ns x nu), free response f (ns) */
  double *H, *g;        /* condensed Hessian (nu x nu), gradient (nu) */
  double *Cn, *b;       /* one-sided constraints Cn[j] . u >= b[j] (m x nu) */
  int* kind;            /* 0 box-lower, 1 box-upper, 2 gap (stage, h) */
  int* idx;             /* box: variable; gap: 2*stage + h */
} condensed;

static void condensed_free(condensed* c) {
  free(c->G); free(c->f); free(c->H); free(c->g); free(c->Cn); free(c->b); free(c->kind); free(c->idx);
}

static int build_condensed(const f110o_params* prm, const double x0[3], const double ulin[2],
                           const double* x_ref, const double* hs, int gap_active, condensed* c) {
  const int N = prm->horizon, nu = 2 * N, ns = 3 * (N + 1);
  c->N = N; c->nu = nu; c->ns = ns;
  f110o_linearize(x0[2], ulin[0], ulin[1], (double)prm->dt, c->A, c->B, c->C);
  c->G = (double*)calloc((size_t)ns * nu, sizeof(double));
  c->f = (double*)calloc(ns, sizeof(double));
  c->H = (double*)calloc((size_t)nu * nu, sizeof(double));
  c->g = (double*)calloc(nu, sizeof(double));
  int mg = gap_active ? 2 * N : 0;
  c->m = 2 * nu + mg;
  c->Cn = (double*)calloc((size_t)c->m * nu, sizeof(double));
  c->b = (double*)calloc(c->m, sizeof(double));
  c->kind = (int*)calloc(c->m, sizeof(int));
  c->idx = (int*)calloc(c->m, sizeof(int));
  /* x_i = A x_{i-1} + B u_{i-1} + C (the dynamics rows, mpc.cpp:244-248,299,305) */
  for (int r = 0; r < 3; r++) c->f[r] = x0[r];
  for (int i = 1; i <= N; i++) {
    for (int r = 0; r < 3; r++) {
      double s = c->C[r];
      for (int k = 0; k < 3; k++) s += c->A[r * 3 + k] * c->f[3 * (i - 1) + k];
      c->f[3 * i + r] = s;
      for (int j = 0; j < nu; j++) {
        double t = 0;
        for (int k = 0; k < 3; k++) t += c->A[r * 3 + k] * c->G[(size_t)(3 * (i - 1) + k) * nu + j];
        c->G[(size_t)(3 * i + r) * nu + j] = t;
      }
      c->G[(size_t)(3 * i + r) * nu + 2 * (i - 1) + 0] += c->B[r * 2 + 0];
      c->G[(size_t)(3 * i + r) * nu + 2 * (i - 1) + 1] += c->B[r * 2 + 1];
    }
  }
  /* H = sum_i G_i' Q G_i + blkdiag(R) ; g = sum_i G_i' Q (f_i - r_i) - R u_des (mpc.cpp:208-229) */
  for (int i = 0; i <= N; i++) {
    double r[3];
    ref_point(x_ref, N, i, r);
    for (int s = 0; s < 3; s++) {
      double qs = prm->q[s];
      if (qs == 0) continue;
      const double* Gi = c->G + (size_t)(3 * i + s) * nu;
      double e = c->f[3 * i + s] - r[s];
      for (int a = 0; a < nu; a++) {
        if (Gi[a] == 0) continue;
        c->g[a] += qs * Gi[a] * e;
        for (int bb = 0; bb < nu; bb++) c->H[a * nu + bb] += qs * Gi[a] * Gi[bb];
      }
    }
  }
  for (int k = 0; k < N; k++)
    for (int a = 0; a < 2; a++) {
      c->H[(2 * k + a) * nu + 2 * k + a] += prm->r[a];
      c->g[2 * k + a] -= prm->r[a] * prm->u_des[a];
    }
  /* one-sided constraints: input box (mpc.cpp:253,281,290), gap rows for stages 1..N */
  int j = 0;
  for (int k = 0; k < nu; k++) {
    c->Cn[(size_t)j * nu + k] = 1; c->b[j] = (double)prm->u_min[k % 2]; c->kind[j] = 0; c->idx[j] = k; j++;
    c->Cn[(size_t)j * nu + k] = -1; c->b[j] = -(double)prm->u_max[k % 2]; c->kind[j] = 1; c->idx[j] = k; j++;
  }
  if (gap_active) {
    for (int i = 1; i <= N; i++)
      for (int h = 0; h < 2; h++) {
        double a = hs[3 * h + 0], bb = hs[3 * h + 1], cc = hs[3 * h + 2];
        for (int t = 0; t < nu; t++)
          c->Cn[(size_t)j * nu + t] = a * c->G[(size_t)(3 * i) * nu + t] + bb * c->G[(size_t)(3 * i + 1) * nu + t];
        c->b[j] = -cc - a * c->f[3 * i] - bb * c->f[3 * i + 1];
        c->kind[j] = 2; c->idx[j] = 2 * i + h; j++;
      }
  }
  return 0;
}


int f110o_condense(const f110o_params* prm, const double x0[3], const double ulin[2],
                   const double* x_ref, double* H_out, double* g_out) {
  condensed c;
  build_condensed(prm, x0, ulin, x_ref, NULL, 0, &c);
  const int nu = c.nu;
  memcpy(H_out, c.H, (size_t)nu * nu * sizeof(double));
  memcpy(g_out, c.g, (size_t)nu * sizeof(double));
  condensed_free(&c);
  return 0;
}
/* ------------------------------------------------------------------------------------------ */
/* Goldfarb-Idnani dual active set, range-space form: maintains W = H^-1, the active normals'  */
/* W n_j and a Cholesky factor of S_A = N_A' W N_A. Exact (finite) for strictly convex QPs.    */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
  int n, m;
  const double *Cn, *b;
  double* W;     /* n x n */
  int q;         /* active count */
  int* act;      /* active constraint ids */
  double* mult;  /* multipliers (>= 0) */
  double* Wn;    /* q x n : W n_j */
  double* S;     /* q x q  (ld = n) */
  double* Ls;    /* q x q Cholesky */
} gi_state;

static void gi_refactor(gi_state* s) {
  const int n = s->n;
  for (int a = 0; a < s->q; a++)
    for (int c = 0; c < s->q; c++) s->Ls[a * n + c] = s->S[a * n + c];
  chol(s->Ls, s->q, n);
}

static void gi_drop(gi_state* s, int k) {
  const int n = s->n;
  for (int a = k; a < s->q - 1; a++) {
    s->act[a] = s->act[a + 1];
    s->mult[a] = s->mult[a + 1];
    memcpy(s->Wn + (size_t)a * n, s->Wn + (size_t)(a + 1) * n, n * sizeof(double));
  }
  /* S: remove row/col k */
  for (int a = 0; a < s->q; a++) {
    if (a == k) continue;
    int ra = a < k ? a : a - 1;
    for (int c = 0; c < s->q; c++) {
      if (c == k) continue;
      int rc = c < k ? c : c - 1;
      s->S[ra * n + rc] = s->S[a * n + c];
    }
  }
  s->q--;
  gi_refactor(s);
}

/* returns status; x is the primal solution (n) */
static int gi_solve(const double* H, const double* g, const double* Cn, const double* b, int n, int m,
                    double* x, int* act_out, double* mult_out, int* q_out) {
  gi_state s;
  s.n = n; s.m = m; s.Cn = Cn; s.b = b; s.q = 0;
  double* L = (double*)malloc((size_t)n * n * sizeof(double));
  s.W = (double*)malloc((size_t)n * n * sizeof(double));
  s.act = (int*)malloc(n * sizeof(int));
  s.mult = (double*)malloc((n + 1) * sizeof(double));
  s.Wn = (double*)malloc((size_t)n * n * sizeof(double));
  s.S = (double*)malloc((size_t)n * n * sizeof(double));
  s.Ls = (double*)malloc((size_t)n * n * sizeof(double));
  double* w = (double*)malloc(n * sizeof(double));
  double* v = (double*)malloc(n * sizeof(double));
  double* r = (double*)malloc(n * sizeof(double));
  double* z = (double*)malloc(n * sizeof(double));
  double* sl = (double*)malloc(m * sizeof(double));
  char* isact = (char*)calloc(m, 1);
  int status = F110O_MAX_ITER;
  memcpy(L, H, (size_t)n * n * sizeof(double));
  if (chol(L, n, n)) { status = -4; goto done; }
  for (int j = 0; j < n; j++) { /* W = H^-1 column by column */
    for (int i = 0; i < n; i++) w[i] = (i == j);
    lsolve(L, n, n, w);
    ltsolve(L, n, n, w);
    for (int i = 0; i < n; i++) s.W[i * n + j] = w[i];
  }
  for (int i = 0; i < n; i++) { double t = 0; for (int k = 0; k < n; k++) t -= s.W[i * n + k] * g[k]; x[i] = t; }
  double xscale = 0;
  for (int i = 0; i < n; i++) xscale = fmax(xscale, fabs(x[i]));
  const int max_iter = 20 * (n + m);
  int it = 0;
  for (;;) {
    /* step 1: most violated inactive constraint */
    int p = -1; double sp = 0;
    for (int j = 0; j < m; j++) {
      if (isact[j]) continue;
      double t = -b[j];
      const double* nj = Cn + (size_t)j * n;
      for (int k = 0; k < n; k++) t += nj[k] * x[k];
      double tol = 1e-11 * (1.0 + fabs(b[j]) + xscale);
      if (t < -tol && (p < 0 || t < sp)) { p = j; sp = t; }
    }
    if (p < 0) { status = F110O_SOLVED; break; }
    const double* np = Cn + (size_t)p * n;
    s.mult[s.q] = 0;
    for (;;) { /* step 2 */
      if (++it > max_iter) goto done;
      for (int i = 0; i < n; i++) { double t = 0; for (int k = 0; k < n; k++) t += s.W[i * n + k] * np[k]; w[i] = t; }
      double nw = 0;
      for (int k = 0; k < n; k++) nw += np[k] * w[k];
      for (int a = 0; a < s.q; a++) {
        const double* na = Cn + (size_t)s.act[a] * n;
        double t = 0;
        for (int k = 0; k < n; k++) t += na[k] * w[k];
        v[a] = t; r[a] = t;
      }
      lsolve(s.Ls, s.q, n, r); /* r = L^-1 v (new Cholesky row) */
      double ll = 0;
      for (int a = 0; a < s.q; a++) ll += r[a] * r[a];
      double lnew[256]; /* n <= 256 supported */
      for (int a = 0; a < s.q; a++) lnew[a] = r[a];
      ltsolve(s.Ls, s.q, n, r); /* r = S^-1 v  (dual step direction) */
      for (int i = 0; i < n; i++) {
        double t = w[i];
        for (int a = 0; a < s.q; a++) t -= r[a] * s.Wn[(size_t)a * n + i];
        z[i] = t;
      }
      double piv = nw - ll; /* = z' n_p */
      double t1 = INFINITY; int k = -1;
      for (int a = 0; a < s.q; a++)
        if (r[a] > 0) { double tt = s.mult[a] / r[a]; if (tt < t1) { t1 = tt; k = a; } }
      /* with n independent rows active the point is fixed: a further row is dependent (a pivot
         above the threshold there is rounding; adding it would overrun the n-slot state) */
      double t2 = (s.q < n && piv > 1e-12 * nw) ? -sp / piv : INFINITY;
      double t = t1 < t2 ? t1 : t2;
      if (!isfinite(t)) { status = F110O_PRIMAL_INFEASIBLE; goto done; }
      for (int a = 0; a < s.q; a++) s.mult[a] -= t * r[a];
      s.mult[s.q] += t;
      if (!isfinite(t2)) { /* dependent: pure dual step then drop */
        int kk = k; double keep = s.mult[s.q];
        isact[s.act[kk]] = 0; gi_drop(&s, kk); s.mult[s.q] = keep;
        continue;
      }
      for (int i = 0; i < n; i++) x[i] += t * z[i];
      sp += t * piv;
      if (t2 <= t1) { /* full step: add p */
        int q = s.q;
        s.act[q] = p; isact[p] = 1;
        memcpy(s.Wn + (size_t)q * n, w, n * sizeof(double));
        for (int a = 0; a < q; a++) { s.S[q * n + a] = v[a]; s.S[a * n + q] = v[a]; s.Ls[q * n + a] = lnew[a]; }
        s.S[q * n + q] = nw;
        s.Ls[q * n + q] = sqrt(piv);
        s.q++;
        break;
      } else { /* partial step: drop k, retry p */
        double keep = s.mult[s.q];
        isact[s.act[k]] = 0; gi_drop(&s, k); s.mult[s.q] = keep;
      }
    }
  }
done:
  if (act_out) memcpy(act_out, s.act, s.q * sizeof(int));
  if (mult_out) memcpy(mult_out, s.mult, s.q * sizeof(double));
  if (q_out) *q_out = s.q;
  free(L); free(s.W); free(s.act); free(s.mult); free(s.Wn); free(s.S); free(s.Ls);
  free(w); free(v); free(r); free(z); free(sl); free(isact);
  return status;
}

/* ------------------------------------------------------------------------------------------ */
/* full solve + OSQP-layout reconstruction                                                     */
/* ------------------------------------------------------------------------------------------ */
int f110o_solve(const f110o_params* prm, const double x0[3], const double ulin[2],
                const double* x_ref, const double* hs, int gap_active, double* u_out,
                double* x_out, double* z_out, double* y_out, double* obj_out, int* n_active) {
  const int N = prm->horizon, nu = 2 * N, ns = 3 * (N + 1), n = ns + nu;
  const int mt = f110o_num_constraints(N), gap0 = ns, inp0 = ns + 2 * (N + 1);
  condensed c;
  build_condensed(prm, x0, ulin, x_ref, hs, gap_active, &c);
  double* uu = (double*)malloc(nu * sizeof(double));
  int* act = (int*)malloc(nu * sizeof(int));
  double* mult = (double*)malloc((nu + 1) * sizeof(double));
  int q = 0, status;
  /* the stage-0 gap rows are constant (x0 lies on both lines, constraints.cpp:233-246): check */
  status = gi_solve(c.H, c.g, c.Cn, c.b, nu, c.m, uu, act, mult, &q);
  if (status == F110O_SOLVED) {
    /* self-check: every condensed row holds at the returned point. Near-infeasible gap wedges
       with u_des on a bound drive the active set to n rows; GI's steps there are rounding and
       have returned points 0.6 outside the box. Such a point is not a certificate. */
    double xs = 0;
    for (int k = 0; k < nu; k++) xs = fmax(xs, fabs(uu[k]));
    for (int j = 0; j < c.m; j++) {
      double t = -c.b[j];
      for (int k = 0; k < nu; k++) t += c.Cn[(size_t)j * nu + k] * uu[k];
      if (t < -1e-9 * (1.0 + fabs(c.b[j]) + xs)) { status = F110O_UNCERTIFIED; break; }
    }
  }
  if (gap_active && hs) {
    for (int h = 0; h < 2; h++)
      if (hs[3 * h] * x0[0] + hs[3 * h + 1] * x0[1] < -hs[3 * h + 2] - 1e-9) status = F110O_PRIMAL_INFEASIBLE;
  }
  double* z = (double*)malloc(n * sizeof(double));
  double* y = (double*)calloc(mt, sizeof(double));
  for (int i = 0; i <= N; i++)
    for (int r = 0; r < 3; r++) {
      double t = c.f[3 * i + r];
      for (int k = 0; k < nu; k++) t += c.G[(size_t)(3 * i + r) * nu + k] * uu[k];
      z[3 * i + r] = t;
    }
  for (int k = 0; k < nu; k++) z[ns + k] = uu[k];
  /* multipliers: OSQP sign convention y>0 upper active, y<0 lower active */
  for (int a = 0; a < q; a++) {
    int j = act[a];
    if (c.kind[j] == 0) y[inp0 + c.idx[j]] -= mult[a];
    else if (c.kind[j] == 1) y[inp0 + c.idx[j]] += mult[a];
    else y[gap0 + c.idx[j]] -= mult[a];
  }
  /* dynamics-row duals by the backward (costate) recursion from stationarity in x_i:
   *   -y_i + A' y_{i+1} + Gap_i' y_gap_i + Q x_i + q_i = 0 */
  double hz[6] = {0, 0, 0, 0, 0, 0};
  if (hs) memcpy(hz, hs, sizeof(hz));
  double ynext[3] = {0, 0, 0};
  for (int i = N; i >= 0; i--) {
    double r[3];
    ref_point(x_ref, N, i, r);
    for (int cc = 0; cc < 3; cc++) {
      double t = prm->q[cc] * z[3 * i + cc] - prm->q[cc] * r[cc];
      if (i < N) for (int rr = 0; rr < 3; rr++) t += c.A[rr * 3 + cc] * ynext[rr];
      for (int h = 0; h < 2; h++) {
        double coef = (i == 0 && !gap_active) ? 1.0 : (cc == 2 ? 0.0 : hz[3 * h + cc]);
        t += coef * y[gap0 + 2 * i + h];
      }
      y[3 * i + cc] = t;
    }
    for (int cc = 0; cc < 3; cc++) ynext[cc] = y[3 * i + cc];
  }
  if (u_out) memcpy(u_out, uu, nu * sizeof(double));
  if (x_out) memcpy(x_out, z, ns * sizeof(double));
  if (z_out) memcpy(z_out, z, n * sizeof(double));
  if (y_out) memcpy(y_out, y, mt * sizeof(double));
  if (obj_out) { /* OSQP objective 0.5 z'Pz + q'z */
    double o = 0;
    for (int i = 0; i <= N; i++) {
      double r[3];
      ref_point(x_ref, N, i, r);
      for (int cc = 0; cc < 3; cc++) o += 0.5 * prm->q[cc] * z[3 * i + cc] * z[3 * i + cc] - prm->q[cc] * r[cc] * z[3 * i + cc];
    }
    for (int k = 0; k < N; k++)
      for (int a = 0; a < 2; a++) o += 0.5 * prm->r[a] * uu[2 * k + a] * uu[2 * k + a] - prm->r[a] * prm->u_des[a] * uu[2 * k + a];
    *obj_out = o;
  }
  if (n_active) *n_active = q;
  if (status != F110O_SOLVED) {
    if (u_out) for (int k = 0; k < nu; k++) u_out[k] = NAN;
    if (x_out) for (int k = 0; k < ns; k++) x_out[k] = NAN;
  }
  free(uu); free(act); free(mult); free(z); free(y);
  condensed_free(&c);
  return status;
}

void f110o_kkt_residuals(const f110o_params* prm, const double x0[3], const double ulin[2],
                         const double* x_ref, const double* hs, int gap_active, const double* z,
                         const double* y, double res[3]) {
  const int N = prm->horizon, n = f110o_num_variables(N), m = f110o_num_constraints(N);
  int *Pc = (int*)malloc((n + 1) * sizeof(int)), *Pr = (int*)malloc(f110o_nnz_P(N) * sizeof(int));
  int *Ac = (int*)malloc((n + 1) * sizeof(int)), *Ar = (int*)malloc(f110o_nnz_A(N) * sizeof(int));
  double *Pv = (double*)malloc(f110o_nnz_P(N) * sizeof(double)), *Av = (double*)malloc(f110o_nnz_A(N) * sizeof(double));
  double *q = (double*)malloc(n * sizeof(double)), *l = (double*)malloc(m * sizeof(double)), *u = (double*)malloc(m * sizeof(double));
  double *r1 = (double*)calloc(n, sizeof(double)), *Az = (double*)calloc(m, sizeof(double));
  f110o_assemble(prm, x0, ulin, x_ref, hs, gap_active, Pc, Pr, Pv, q, Ac, Ar, Av, l, u);
  for (int j = 0; j < n; j++) {
    r1[j] += q[j];
    for (int p = Pc[j]; p < Pc[j + 1]; p++) r1[Pr[p]] += Pv[p] * z[j];
    for (int p = Ac[j]; p < Ac[j + 1]; p++) { r1[j] += Av[p] * y[Ar[p]]; Az[Ar[p]] += Av[p] * z[j]; }
  }
  double d = 0, pinf = 0, comp = 0;
  for (int j = 0; j < n; j++) d = fmax(d, fabs(r1[j]));
  for (int i = 0; i < m; i++) {
    double pr = Az[i] < l[i] ? l[i] - Az[i] : (Az[i] > u[i] ? Az[i] - u[i] : 0);
    pinf = fmax(pinf, pr);
    /* complementarity / dual sign: y>0 only at the upper bound, y<0 only at the lower bound */
    if (y[i] > 0) comp = fmax(comp, u[i] >= F110O_INFTY ? y[i] : fmin(y[i], fabs(u[i] - Az[i])));
    if (y[i] < 0) comp = fmax(comp, l[i] <= -F110O_INFTY ? -y[i] : fmin(-y[i], fabs(Az[i] - l[i])));
  }
  res[0] = d; res[1] = pinf; res[2] = comp;
  free(Pc); free(Pr); free(Ac); free(Ar); free(Pv); free(Av); free(q); free(l); free(u); free(r1); free(Az);
}

int f110o_solve_batch(const f110o_params* prm, int batch, const float* x0, const float* ulin,
                      const float* x_ref, const float* hs, int gap_active, double* u_out,
                      double* x_out, int* status, int num_threads) {
  return f110o_solve_batch_obj(prm, batch, x0, ulin, x_ref, hs, gap_active, u_out, x_out, status,
                               NULL, num_threads);
}

/* the same with OSQP's objective 0.5 z'Pz + q'z per QP (obj_out may be NULL) */
int f110o_solve_batch_obj(const f110o_params* prm, int batch, const float* x0, const float* ulin,
                          const float* x_ref, const float* hs, int gap_active, double* u_out,
                          double* x_out, int* status, double* obj_out, int num_threads) {
  const int N = prm->horizon;
  int nsolved = 0;
#ifdef _OPENMP
  if (num_threads > 0) omp_set_num_threads(num_threads);
#pragma omp parallel for schedule(dynamic, 16) reduction(+ : nsolved)
#endif
  for (int b = 0; b < batch; b++) {
    double xx[3], uu[2], hh[6];
    double* xr = (double*)malloc(3 * N * sizeof(double));
    for (int k = 0; k < 3; k++) xx[k] = x0[3 * b + k];
    for (int k = 0; k < 2; k++) uu[k] = ulin[2 * b + k];
    for (int k = 0; k < 3 * N; k++) xr[k] = x_ref[(size_t)b * 3 * N + k];
    if (hs) for (int k = 0; k < 6; k++) hh[k] = hs[6 * b + k];
    int st = f110o_solve(prm, xx, uu, xr, hs ? hh : NULL, gap_active,
                         u_out ? u_out + (size_t)b * 2 * N : NULL,
                         x_out ? x_out + (size_t)b * 3 * (N + 1) : NULL, NULL, NULL,
                         obj_out ? obj_out + b : NULL, NULL);
    if (status) status[b] = st;
    nsolved += (st == F110O_SOLVED);
    free(xr);
  }
  return nsolved;
}

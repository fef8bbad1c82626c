/*
 * osc_ref_port.c -- CPU restatement of the reference's per-tick OSC path, for the CPU baseline.
 *
 * TEST / BENCH INFRASTRUCTURE ONLY (the "port" cpu_baseline of bench.py, and a cross-check of
 * the oracle).  Nothing in the product links this file.
 *
 * What it restates (paths relative to /root/reference/operational-space-control):
 *   * update_optimization_data  (unitree_go2/operational_space_controller.h:457-481): the six
 *     CasADi functions H, f, Aeq, beq, Aineq, bineq in closed form (autogen.py:58-319), after
 *     the row->column-major copies of operational-space-control/utilities.h:17-38;
 *   * update_optimization       (operational_space_controller.h:483-529): A = [Aeq; Aineq; I],
 *     masked bounds, then OSQP's update_P_A / update_lin_cost / update_bounds;
 *   * solve_optimization        (operational_space_controller.h:531-536): osqp_solve with warm
 *     start from the previous tick; torque = x[nv : nv+nu] (:573).
 * OSQP 0.6.3 (MODULE.bazel:17-21; not vendored -- restated from its published algorithm):
 *   Ruiz equilibration (10 passes, cost scaling), rho vector (equality rows 1e3 rho, loose rows
 *   RHO_MIN), KKT [P + sigma I, A'; A, -diag(1/rho)] factorised by LDL^T, ADMM with
 *   relaxation alpha = 1.6, termination checked every 25 iterations on unscaled residuals with
 *   eps_abs = eps_rel = 1e-3, adaptive rho (tolerance 5), max_iter 4000, polish off.
 * Deliberate differences (stated in DESIGN.md): verbose printing off; adaptive-rho interval
 *   fixed at 25 iterations (OSQP's default 0 derives it from wall-clock setup time, which makes
 *   the reference non-deterministic); infeasibility detection omitted (the QP is always
 *   feasible); the LDL^T uses a dense array but visits only the symbolic nonzeros of a
 *   minimum-degree ordering (the work QDLDL + AMD do), not QDLDL's CSC data structure.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define OSQP_INFTY 1e30
#define MIN_SCALING 1e-4
#define MAX_SCALING 1e4
#define RHO_MIN 1e-6
#define RHO_MAX 1e6
#define RHO_EQ_OVER_RHO_INEQ 1e3
#define RHO_TOL 1e-4
#define DIV_TOL 1e-10

typedef struct {
  /* model */
  int nv, nu, nc, ns, n, m, N;
  double w_row[6 * 64], w_torque, w_reg, mu;
  double u_lb[32], u_ub[32];
  /* settings (OSQP 0.6.3 defaults via osqp-cpp OsqpSettings()) */
  double rho, sigma, alpha, eps_abs, eps_rel, ar_tol;
  int scaling, max_iter, check_term, ar_interval;
  /* problem data (unscaled copies + scaled working copies) */
  double *P0, *A0, *q0, *l0, *u0;       /* unscaled */
  double *P, *A, *q, *l, *u;            /* scaled */
  double *D, *E, c;                     /* scaling */
  double *rho_vec, *rho_inv;
  int *ctype;                           /* -1 loose, 0 ineq, 1 eq */
  /* iterates */
  double *x, *z, *y, *xt, *zt, *xp, *zp, *w1, *w2, *Ax, *Px, *Aty;
  /* KKT factor */
  int *perm, *iperm, *colptr, *rowidx;  /* symbolic: nonzero rows (> k) per column */
  double *K, *Dd, *rhs;
  unsigned char *pat;                   /* KKT structural pattern (N x N) */
  int initialized;
} osc_cpu;

static void* zalloc(size_t n) { return calloc(n, 1); }

/* ------------------------------ dense helpers ------------------------------ */
static double norm_inf(const double* v, int n) {
  double r = 0.0;
  for (int i = 0; i < n; ++i) r = fmax(r, fabs(v[i]));
  return r;
}

/* ------------------- symbolic: minimum degree + fill pattern ------------------- */
static void symbolic(osc_cpu* w) {
  const int N = w->N;
  unsigned char* g = (unsigned char*)zalloc((size_t)N * N);
  memcpy(g, w->pat, (size_t)N * N);
  unsigned char* done = (unsigned char*)zalloc(N);
  for (int step = 0; step < N; ++step) {          /* exact minimum degree */
    int best = -1, bestdeg = 1 << 30;
    for (int v = 0; v < N; ++v) {
      if (done[v]) continue;
      int deg = 0;
      for (int u = 0; u < N; ++u) deg += (!done[u] && u != v && g[v * N + u]);
      if (deg < bestdeg) { bestdeg = deg; best = v; }
    }
    w->perm[step] = best;
    done[best] = 1;
    for (int a = 0; a < N; ++a) {                 /* eliminate: clique on the neighbours */
      if (done[a] || !g[best * N + a]) continue;
      for (int b = 0; b < N; ++b)
        if (!done[b] && g[best * N + b]) { g[a * N + b] = 1; g[b * N + a] = 1; }
    }
  }
  for (int i = 0; i < N; ++i) w->iperm[w->perm[i]] = i;
  /* fill pattern in permuted order: symbolic elimination */
  unsigned char* f = (unsigned char*)zalloc((size_t)N * N);
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < N; ++j)
      if (w->pat[w->perm[i] * N + w->perm[j]]) f[i * N + j] = 1;
  int nnz = 0;
  for (int k = 0; k < N; ++k) {
    w->colptr[k] = nnz;
    for (int i = k + 1; i < N; ++i)
      if (f[i * N + k]) w->rowidx[nnz++] = i;
    for (int a = w->colptr[k]; a < nnz; ++a)
      for (int b = w->colptr[k]; b <= a; ++b) {
        int i = w->rowidx[a], j = w->rowidx[b];
        f[i * N + j] = f[j * N + i] = 1;
      }
  }
  w->colptr[N] = nnz;
  free(f);
  free(g);
  free(done);
}

/* KKT = [P + sigma I, A'; A, -diag(1/rho)] in permuted order, then LDL^T on the pattern */
static int factor(osc_cpu* w) {
  const int n = w->n, m = w->m, N = w->N;
  double* K = w->K;
  memset(K, 0, sizeof(double) * (size_t)N * N);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double v = w->P[i * n + j] + (i == j ? w->sigma : 0.0);
      if (v != 0.0 || i == j) K[w->iperm[i] * N + w->iperm[j]] = v;
    }
  for (int r = 0; r < m; ++r) {
    for (int j = 0; j < n; ++j) {
      double v = w->A[r * n + j];
      if (v != 0.0) {
        K[w->iperm[n + r] * N + w->iperm[j]] = v;
        K[w->iperm[j] * N + w->iperm[n + r]] = v;
      }
    }
    K[w->iperm[n + r] * N + w->iperm[n + r]] = -w->rho_inv[r];
  }
  for (int k = 0; k < N; ++k) {                   /* right-looking, pattern only */
    const double dk = K[k * N + k];
    if (dk == 0.0) return -1;
    w->Dd[k] = dk;
    const double inv = 1.0 / dk;
    for (int a = w->colptr[k]; a < w->colptr[k + 1]; ++a) {
      const int i = w->rowidx[a];
      const double lik = K[i * N + k] * inv;
      for (int b = w->colptr[k]; b <= a; ++b) {
        const int j = w->rowidx[b];
        K[i * N + j] -= lik * K[j * N + k];
      }
    }
    for (int a = w->colptr[k]; a < w->colptr[k + 1]; ++a) K[w->rowidx[a] * N + k] *= inv;
  }
  return 0;
}

static void kkt_solve(osc_cpu* w, double* b /* in: N (original order), out: solution */) {
  const int N = w->N;
  double* t = w->rhs;
  for (int i = 0; i < N; ++i) t[w->iperm[i]] = b[i];
  for (int k = 0; k < N; ++k)
    for (int a = w->colptr[k]; a < w->colptr[k + 1]; ++a) t[w->rowidx[a]] -= w->K[w->rowidx[a] * N + k] * t[k];
  for (int k = 0; k < N; ++k) t[k] /= w->Dd[k];
  for (int k = N - 1; k >= 0; --k)
    for (int a = w->colptr[k]; a < w->colptr[k + 1]; ++a) t[k] -= w->K[w->rowidx[a] * N + k] * t[w->rowidx[a]];
  for (int i = 0; i < N; ++i) b[i] = t[w->iperm[i]];
}

/* ----------------------------- scaling (Ruiz) ----------------------------- */
static void limit_scaling(double* v, int n) {
  for (int i = 0; i < n; ++i) {
    v[i] = v[i] < MIN_SCALING ? 1.0 : v[i];
    v[i] = v[i] > MAX_SCALING ? MAX_SCALING : v[i];
  }
}

static void scale_data(osc_cpu* w) {
  const int n = w->n, m = w->m;
  memcpy(w->P, w->P0, sizeof(double) * n * n);
  memcpy(w->A, w->A0, sizeof(double) * m * n);
  memcpy(w->q, w->q0, sizeof(double) * n);
  for (int i = 0; i < n; ++i) w->D[i] = 1.0;
  for (int i = 0; i < m; ++i) w->E[i] = 1.0;
  w->c = 1.0;
  double* Dt = w->w1;
  double* Et = w->w2;
  for (int it = 0; it < w->scaling; ++it) {
    for (int j = 0; j < n; ++j) {
      double v = 0.0;
      for (int i = 0; i < n; ++i) v = fmax(v, fabs(w->P[i * n + j]));
      for (int r = 0; r < m; ++r) v = fmax(v, fabs(w->A[r * n + j]));
      Dt[j] = v;
    }
    for (int r = 0; r < m; ++r) Et[r] = norm_inf(w->A + r * n, n);
    limit_scaling(Dt, n);
    limit_scaling(Et, m);
    for (int j = 0; j < n; ++j) Dt[j] = 1.0 / sqrt(Dt[j]);
    for (int r = 0; r < m; ++r) Et[r] = 1.0 / sqrt(Et[r]);
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) w->P[i * n + j] *= Dt[i] * Dt[j];
    for (int r = 0; r < m; ++r)
      for (int j = 0; j < n; ++j) w->A[r * n + j] *= Et[r] * Dt[j];
    for (int j = 0; j < n; ++j) w->q[j] *= Dt[j];
    for (int j = 0; j < n; ++j) w->D[j] *= Dt[j];
    for (int r = 0; r < m; ++r) w->E[r] *= Et[r];
    /* cost normalisation: mean column inf-norm of P vs ||q||_inf */
    double mean = 0.0;
    for (int j = 0; j < n; ++j) {
      double v = 0.0;
      for (int i = 0; i < n; ++i) v = fmax(v, fabs(w->P[i * n + j]));
      mean += v;
    }
    mean /= n;
    double nq = norm_inf(w->q, n);
    limit_scaling(&nq, 1);
    double ct = fmax(mean, nq);
    limit_scaling(&ct, 1);
    ct = 1.0 / ct;
    for (int i = 0; i < n * n; ++i) w->P[i] *= ct;
    for (int j = 0; j < n; ++j) w->q[j] *= ct;
    w->c *= ct;
  }
}

static void scale_bounds(osc_cpu* w) {
  for (int r = 0; r < w->m; ++r) {
    w->l[r] = w->E[r] * w->l0[r];
    w->u[r] = w->E[r] * w->u0[r];
  }
}

/* constraint types and rho vector; returns 1 if any type changed */
static int set_rho_vec(osc_cpu* w) {
  int changed = 0;
  for (int r = 0; r < w->m; ++r) {
    int t;
    if (w->l[r] < -OSQP_INFTY * MIN_SCALING && w->u[r] > OSQP_INFTY * MIN_SCALING) t = -1;
    else if (w->u[r] - w->l[r] < RHO_TOL) t = 1;
    else t = 0;
    if (t != w->ctype[r]) changed = 1;
    w->ctype[r] = t;
    w->rho_vec[r] = t == -1 ? RHO_MIN : (t == 1 ? RHO_EQ_OVER_RHO_INEQ * w->rho : w->rho);
    w->rho_inv[r] = 1.0 / w->rho_vec[r];
  }
  return changed;
}

/* ------------------------- assembly (CasADi-equivalent) ------------------------- */
static void assemble(osc_cpu* w, const double* M, const double* C, const double* J,
                     const double* b, const double* T, const double* mask) {
  const int nv = w->nv, nu = w->nu, nc = w->nc, ns = w->ns, n = w->n, m = w->m;
  const int s = 6 * ns, nz = 3 * nc;
  memset(w->P0, 0, sizeof(double) * n * n);
  memset(w->A0, 0, sizeof(double) * m * n);
  memset(w->q0, 0, sizeof(double) * n);
  double e[6 * 64];
  for (int r = 0; r < s; ++r) {                      /* e = b - t  (autogen.py:163-168) */
    const int half = r / (3 * ns), rr = r % (3 * ns);
    e[r] = b[r] - T[(rr / 3) * 6 + half * 3 + rr % 3];
  }
  for (int i = 0; i < nv; ++i) {                     /* H_dv = 2 J'WJ + 2 w_reg I, f = 2 J'W e */
    for (int j = 0; j < nv; ++j) {
      double acc = 0.0;
      for (int r = 0; r < s; ++r) acc += w->w_row[r] * J[r * nv + i] * J[r * nv + j];
      w->P0[i * n + j] = 2.0 * acc + (i == j ? 2.0 * w->w_reg : 0.0);
    }
    double acc = 0.0;
    for (int r = 0; r < s; ++r) acc += w->w_row[r] * J[r * nv + i] * e[r];
    w->q0[i] = 2.0 * acc;
  }
  for (int i = nv; i < nv + nu; ++i) w->P0[i * n + i] = 2.0 * (w->w_torque + w->w_reg);
  for (int i = nv + nu; i < n; ++i) w->P0[i * n + i] = 2.0 * w->w_reg;
  const int jc0 = 3 * (ns - nc);
  for (int i = 0; i < nv; ++i) {                     /* Aeq = [M, -B, -Jc]; beq = -C */
    for (int j = 0; j < nv; ++j) w->A0[i * n + j] = M[i * nv + j];
    if (i >= nv - nu) w->A0[i * n + nv + (i - (nv - nu))] = -1.0;
    for (int c = 0; c < nz; ++c) w->A0[i * n + nv + nu + c] = -J[(jc0 + c) * nv + i];
    w->l0[i] = w->u0[i] = -C[i];
  }
  static const double sx[4] = {1, -1, 1, -1}, sy[4] = {1, 1, -1, -1};
  for (int k = 0; k < nc; ++k)                       /* friction pyramid, bineq = 0 */
    for (int t = 0; t < 4; ++t) {
      const int r = nv + 4 * k + t;
      w->A0[r * n + nv + nu + 3 * k + 0] = sx[t];
      w->A0[r * n + nv + nu + 3 * k + 1] = sy[t];
      w->A0[r * n + nv + nu + 3 * k + 2] = -w->mu;
      w->l0[r] = -OSQP_INFTY;
      w->u0[r] = 0.0;
    }
  const int ob = nv + 4 * nc;
  for (int j = 0; j < n; ++j) w->A0[(ob + j) * n + j] = 1.0;
  for (int j = 0; j < nv; ++j) { w->l0[ob + j] = -OSQP_INFTY; w->u0[ob + j] = OSQP_INFTY; }
  for (int j = 0; j < nu; ++j) { w->l0[ob + nv + j] = w->u_lb[j]; w->u0[ob + nv + j] = w->u_ub[j]; }
  const float big_number = 1e4f;
  for (int k = 0; k < nc; ++k) {
    const double zl[3] = {-OSQP_INFTY, -OSQP_INFTY, 0.0}, zu[3] = {OSQP_INFTY, OSQP_INFTY, big_number};
    for (int t = 0; t < 3; ++t) {
      w->l0[ob + nv + nu + 3 * k + t] = zl[t] * mask[k];
      w->u0[ob + nv + nu + 3 * k + t] = zu[t] * mask[k];
    }
  }
}

/* -------------------------------- ADMM -------------------------------- */
static int admm(osc_cpu* w) {
  const int n = w->n, m = w->m;
  const double a = w->alpha;
  int iter;
  for (iter = 1; iter <= w->max_iter; ++iter) {
    memcpy(w->xp, w->x, sizeof(double) * n);
    memcpy(w->zp, w->z, sizeof(double) * m);
    /* x~, z~ from the KKT system */
    double* b = w->xt;   /* xt (n) and zt (m) are contiguous: one N-vector */
    for (int i = 0; i < n; ++i) b[i] = w->sigma * w->xp[i] - w->q[i];
    for (int r = 0; r < m; ++r) b[n + r] = w->zp[r] - w->rho_inv[r] * w->y[r];
    kkt_solve(w, b);
    for (int r = 0; r < m; ++r) w->zt[r] = w->zp[r] + w->rho_inv[r] * (w->zt[r] - w->y[r]);
    for (int i = 0; i < n; ++i) w->x[i] = a * w->xt[i] + (1.0 - a) * w->xp[i];
    for (int r = 0; r < m; ++r) {
      const double v = a * w->zt[r] + (1.0 - a) * w->zp[r];
      double zz = v + w->rho_inv[r] * w->y[r];
      zz = fmin(fmax(zz, w->l[r]), w->u[r]);
      w->z[r] = zz;
      w->y[r] += w->rho_vec[r] * (v - zz);
    }
    const int check = (iter % w->check_term) == 0;
    const int adapt = w->ar_interval > 0 && (iter % w->ar_interval) == 0;
    if (!check && !adapt) continue;
    /* residuals (unscaled for termination) */
    for (int r = 0; r < m; ++r) {
      double v = 0.0;
      for (int j = 0; j < n; ++j) v += w->A[r * n + j] * w->x[j];
      w->Ax[r] = v;
    }
    for (int i = 0; i < n; ++i) {
      double v = 0.0, t = 0.0;
      for (int j = 0; j < n; ++j) v += w->P[i * n + j] * w->x[j];
      for (int r = 0; r < m; ++r) t += w->A[r * n + i] * w->y[r];
      w->Px[i] = v;
      w->Aty[i] = t;
    }
    double pr = 0.0, nAx = 0.0, nz = 0.0, du = 0.0, nPx = 0.0, nAty = 0.0, nq = 0.0;
    for (int r = 0; r < m; ++r) {
      const double ei = 1.0 / w->E[r];
      pr = fmax(pr, fabs(ei * (w->Ax[r] - w->z[r])));
      nAx = fmax(nAx, fabs(ei * w->Ax[r]));
      nz = fmax(nz, fabs(ei * w->z[r]));
    }
    const double cinv = 1.0 / w->c;
    for (int i = 0; i < n; ++i) {
      const double di = 1.0 / w->D[i];
      du = fmax(du, fabs(cinv * di * (w->Px[i] + w->q[i] + w->Aty[i])));
      nPx = fmax(nPx, fabs(di * w->Px[i]));
      nAty = fmax(nAty, fabs(di * w->Aty[i]));
      nq = fmax(nq, fabs(di * w->q[i]));
    }
    if (check) {
      const double eps_p = w->eps_abs + w->eps_rel * fmax(nAx, nz);
      const double eps_d = w->eps_abs + w->eps_rel * cinv * fmax(nPx, fmax(nAty, nq));
      if (pr < eps_p && du < eps_d) return iter;
    }
    if (adapt) {   /* compute_rho_estimate on scaled residuals */
      double spr = 0.0, snz = 0.0, snAx = 0.0, sdu = 0.0, sq = 0.0, sAty = 0.0, sPx = 0.0;
      for (int r = 0; r < m; ++r) {
        spr = fmax(spr, fabs(w->Ax[r] - w->z[r]));
        snz = fmax(snz, fabs(w->z[r]));
        snAx = fmax(snAx, fabs(w->Ax[r]));
      }
      for (int i = 0; i < n; ++i) {
        sdu = fmax(sdu, fabs(w->Px[i] + w->q[i] + w->Aty[i]));
        sq = fmax(sq, fabs(w->q[i]));
        sAty = fmax(sAty, fabs(w->Aty[i]));
        sPx = fmax(sPx, fabs(w->Px[i]));
      }
      spr /= fmax(snz, snAx) + DIV_TOL;
      sdu /= fmax(sq, fmax(sAty, sPx)) + DIV_TOL;
      double rn = w->rho * sqrt(spr / (sdu + DIV_TOL));
      rn = fmin(fmax(rn, RHO_MIN), RHO_MAX);
      if (rn > w->rho * w->ar_tol || rn < w->rho / w->ar_tol) {
        w->rho = rn;
        set_rho_vec(w);
        factor(w);
      }
    }
  }
  return w->max_iter;
}

/* ------------------------------- public API ------------------------------- */
osc_cpu* osc_cpu_create(int nv, int nu, int nc, int ns, const double* w_row, double w_torque,
                        double w_reg, double mu, const double* u_lb, const double* u_ub,
                        int adaptive_rho_interval) {
  if (nv <= 0 || nu <= 0 || nu > 32 || ns <= 0 || ns > 64 || nc > ns) return NULL;
  osc_cpu* w = (osc_cpu*)zalloc(sizeof(osc_cpu));
  w->nv = nv; w->nu = nu; w->nc = nc; w->ns = ns;
  w->n = nv + nu + 3 * nc;
  w->m = nv + 4 * nc + w->n;
  w->N = w->n + w->m;
  memcpy(w->w_row, w_row, sizeof(double) * 6 * ns);
  w->w_torque = w_torque; w->w_reg = w_reg; w->mu = mu;
  memcpy(w->u_lb, u_lb, sizeof(double) * nu);
  memcpy(w->u_ub, u_ub, sizeof(double) * nu);
  w->rho = 0.1; w->sigma = 1e-6; w->alpha = 1.6; w->eps_abs = 1e-3; w->eps_rel = 1e-3;
  w->ar_tol = 5.0; w->scaling = 10; w->max_iter = 4000; w->check_term = 25;
  w->ar_interval = adaptive_rho_interval;
  const int n = w->n, m = w->m, N = w->N;
  w->P0 = zalloc(sizeof(double) * n * n); w->A0 = zalloc(sizeof(double) * m * n);
  w->q0 = zalloc(sizeof(double) * n); w->l0 = zalloc(sizeof(double) * m); w->u0 = zalloc(sizeof(double) * m);
  w->P = zalloc(sizeof(double) * n * n); w->A = zalloc(sizeof(double) * m * n);
  w->q = zalloc(sizeof(double) * n); w->l = zalloc(sizeof(double) * m); w->u = zalloc(sizeof(double) * m);
  w->D = zalloc(sizeof(double) * n); w->E = zalloc(sizeof(double) * m);
  w->rho_vec = zalloc(sizeof(double) * m); w->rho_inv = zalloc(sizeof(double) * m);
  w->ctype = zalloc(sizeof(int) * m);
  w->x = zalloc(sizeof(double) * n); w->z = zalloc(sizeof(double) * m); w->y = zalloc(sizeof(double) * m);
  w->xt = zalloc(sizeof(double) * N); w->zt = w->xt + n;
  w->xp = zalloc(sizeof(double) * n); w->zp = zalloc(sizeof(double) * m);
  w->w1 = zalloc(sizeof(double) * (n > m ? n : m)); w->w2 = zalloc(sizeof(double) * (n > m ? n : m));
  w->Ax = zalloc(sizeof(double) * m); w->Px = zalloc(sizeof(double) * n); w->Aty = zalloc(sizeof(double) * n);
  w->perm = zalloc(sizeof(int) * N); w->iperm = zalloc(sizeof(int) * N);
  w->colptr = zalloc(sizeof(int) * (N + 1)); w->rowidx = zalloc(sizeof(int) * (size_t)N * N);
  w->K = zalloc(sizeof(double) * (size_t)N * N); w->Dd = zalloc(sizeof(double) * N);
  w->rhs = zalloc(sizeof(double) * N); w->pat = zalloc((size_t)N * N);
  return w;
}

void osc_cpu_destroy(osc_cpu* w) {
  if (!w) return;
  void* p[] = {w->P0, w->A0, w->q0, w->l0, w->u0, w->P, w->A, w->q, w->l, w->u, w->D, w->E,
               w->rho_vec, w->rho_inv, w->ctype, w->x, w->z, w->y, w->xt, w->xp, w->zp, w->w1,
               w->w2, w->Ax, w->Px, w->Aty, w->perm, w->iperm, w->colptr, w->rowidx, w->K,
               w->Dd, w->rhs, w->pat};
  for (size_t i = 0; i < sizeof(p) / sizeof(p[0]); ++i) free(p[i]);
  free(w);
}

/* Structural pattern of the KKT matrix of the current data (sparseView() drops exact zeros). */
static int pattern_changed(osc_cpu* w) {
  const int n = w->n, m = w->m, N = w->N;
  int changed = 0;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      unsigned char v = (i == j) || w->P0[i * n + j] != 0.0;
      if (w->pat[i * N + j] != v) { w->pat[i * N + j] = v; changed = 1; }
    }
  for (int r = 0; r < m; ++r) {
    for (int j = 0; j < n; ++j) {
      unsigned char v = w->A0[r * n + j] != 0.0;
      if (w->pat[(n + r) * N + j] != v) {
        w->pat[(n + r) * N + j] = w->pat[j * N + n + r] = v;
        changed = 1;
      }
    }
    w->pat[(n + r) * N + n + r] = 1;
  }
  return changed;
}

/* One control tick: returns ADMM iterations (or -1 on a factorisation failure). */
int osc_cpu_step(osc_cpu* w, const double* M, const double* C, const double* J, const double* b,
                 const double* T, const double* mask, double* tau, double* x_out) {
  assemble(w, M, C, J, b, T, mask);
  const int first = !w->initialized;
  if (pattern_changed(w) || first) {
    /* osqp-cpp Init (osc.h:346) or the re-Init fallback of osc.h:513-526 */
    symbolic(w);
    if (first) {
      w->rho = 0.1;
      memset(w->x, 0, sizeof(double) * w->n);
      memset(w->z, 0, sizeof(double) * w->m);
      memset(w->y, 0, sizeof(double) * w->m);
      for (int r = 0; r < w->m; ++r) w->ctype[r] = 2;
    }
    w->initialized = 1;
  }
  /* UpdateObjectiveAndConstraintMatrices -> osqp_update_P_A (unscale, update, rescale) */
  scale_data(w);
  /* SetBounds -> osqp_update_bounds (rho vector follows the constraint types) */
  scale_bounds(w);
  set_rho_vec(w);
  if (factor(w) != 0) return -1;
  const int it = admm(w);
  for (int i = 0; i < w->nu; ++i) tau[i] = w->D[w->nv + i] * w->x[w->nv + i];
  if (x_out)
    for (int i = 0; i < w->n; ++i) x_out[i] = w->D[i] * w->x[i];
  return it;
}

/* Tighter settings for validating the restatement against the exact oracle (tests only). */
void osc_cpu_set_tolerances(osc_cpu* w, double eps_abs, double eps_rel, int max_iter) {
  w->eps_abs = eps_abs;
  w->eps_rel = eps_rel;
  w->max_iter = max_iter;
}

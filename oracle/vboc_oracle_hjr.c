/*
 * ORACLE - TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by or called from the product path
 * (vboc_amd/).  Only tests/ use it, and only as the checker.
 *
 * Plain-C FP64 restatement of the HJR one-step OCP, OCP<sys>.compute_problem(x0) of the reference's HJR
 * classes (HJR/triplependulum_hjr_class.py:7-134, HJR/doublependulum_hjr_class.py, HJR/pendulum_hjr_class.py):
 *  - N = 1, tf = 1e-2 (:66-69): x1 = RK4(x0, u0) with h = 1e-2, the same chain models as the VBOC classes
 *    (the pendulum of the HJR class is undamped, m 0.5, d 0.3, :14-36);
 *  - x0 fully fixed (constraints_set(0, lbx / ubx, x0), :121-122), u0 in the torque box (:94-96), x1 free;
 *  - terminal cost EXTERNAL = logit 0 of the classifier NeuralNetCLS(2nq, 100, 2) (my_nn.py:4-18) built by
 *    nn_decisionfunction (:135-152): (x - mean) / std, W0 . + b0, relu, W1 . + b1, relu, W2 . + b2, [0];
 *  - options (:98-108): SQP, EXACT Hessian with exact_hess_dyn = 0 (exact_hess_cost keeps its default 1:
 *    the network's Hessian, which is zero - ReLU layers are piecewise linear), MERIT_BACKTRACKING with
 *    alpha_reduction 0.3 / alpha_min 1e-2, levenberg_marquardt 1e-5 (pendulum 1e-2), max_iter 1000,
 *    qp_solver_iter_max 100; the tolerances keep the ACADOS defaults (nlp 1e-6, HPIPM 1e-8) - the HJR classes
 *    do not set the 1e-3 of the VBOC classes;
 *  - guess (:117-124): reset (u = 0, multipliers 0), x0 at stage 0, x1 = [q0 + v0 1e-2, 0.9 v0].
 * compute_problem returns 1 for status 0 (else 0); the HJR driver then labels the state by the sign of
 * get_cost() (HJR/triplependulum_hjr.py:21-40).
 * Algorithm: the SQP / L1-merit / Mehrotra-IPM of vboc_oracle.c specialised to one stage: decision variables
 * u0 (boxed) and x1 (free), the dynamics equality x1 = phi(x0, u0) with multiplier pi, the QP Hessian
 * levenberg_marquardt * I (+ the network's zero Hessian), x1 eliminated by the one-stage Riccati step.
 * Parity with ACADOS is unpinned (not importable); tests/test_hjr.py pins this restatement by KKT residuals
 * recomputed outside it and by scipy SLSQP on the same NLP.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "vboc_oracle.h"

#define HQ 3
#define HX 6
#define HMAX 128

typedef struct {
  int nx, h;
  const double *W0, *b0, *W1, *b1, *W2, *b2;
  double mean, std;
} hnn_t;

/* logit 0 of the network and its gradient (relu' = 1 for a positive argument, 0 otherwise) */
static double nn_eval(const hnn_t* n, const double* x, double* grad) {
  const int nx = n->nx, h = n->h;
  double z0[HX], h1[HMAX], h2[HMAX];
  int m1[HMAX], m2[HMAX];
  for (int i = 0; i < nx; ++i) z0[i] = (x[i] - n->mean) / n->std;
  for (int j = 0; j < h; ++j) {
    double t = 0.0;
    for (int i = 0; i < nx; ++i) t += n->W0[j * nx + i] * z0[i];
    t = n->b0[j] + t;
    m1[j] = t > 0.0;
    h1[j] = fmax(0.0, t);
  }
  for (int j = 0; j < h; ++j) {
    double t = 0.0;
    for (int i = 0; i < h; ++i) t += n->W1[j * h + i] * h1[i];
    t = n->b1[j] + t;
    m2[j] = t > 0.0;
    h2[j] = fmax(0.0, t);
  }
  double out = 0.0;
  for (int j = 0; j < h; ++j) out += n->W2[j] * h2[j];
  out = n->b2[0] + out;
  if (grad) {
    double v1[HMAX];
    for (int i = 0; i < h; ++i) {
      double t = 0.0;
      for (int j = 0; j < h; ++j) t += m2[j] ? n->W1[j * h + i] * n->W2[j] : 0.0;
      v1[i] = m1[i] ? t : 0.0;
    }
    for (int c = 0; c < nx; ++c) {
      double t = 0.0;
      for (int j = 0; j < h; ++j) t += n->W0[j * nx + c] * v1[j];
      grad[c] = t / n->std;
    }
  }
  return out;
}

/* the undamped pendulum of HJR/pendulum_hjr_class.py:14-36: theta'' = (m g d sin(theta) + F) / (d^2 m) */
static void pend_rhs(const double* x, const double* u, double* f, double* J /* 2 x 3 or NULL */) {
  const double m = 0.5, g = 9.81, d = 0.3;
  f[0] = x[1];
  f[1] = (m * g * d * sin(x[0]) + u[0]) / (d * d * m);
  if (J) {
    J[0] = 0.0; J[1] = 1.0; J[2] = 0.0;
    J[3] = m * g * d * cos(x[0]) / (d * d * m); J[4] = 0.0; J[5] = 1.0 / (d * d * m);
  }
}
/* one ERK4 step (h = 1e-2) with forward sensitivities, pendulum */
static void pend_rk4_sens(double h, const double* x, const double* u, double* x1, double* B /* 2 x 1 */) {
  double k[4][2], S[2][3] = {{1, 0, 0}, {0, 1, 0}}, dk[4][2][3];
  const double cc[4] = {0.0, 0.5, 0.5, 1.0};
  for (int st = 0; st < 4; ++st) {
    double xa[2], Sa[2][3], J[6];
    for (int i = 0; i < 2; ++i) {
      xa[i] = st ? x[i] + cc[st] * h * k[st - 1][i] : x[i];
      for (int c = 0; c < 3; ++c) Sa[i][c] = st ? S[i][c] + cc[st] * h * dk[st - 1][i][c] : S[i][c];
    }
    pend_rhs(xa, u, k[st], J);
    for (int i = 0; i < 2; ++i)
      for (int c = 0; c < 3; ++c) dk[st][i][c] = J[i * 3] * Sa[0][c] + J[i * 3 + 1] * Sa[1][c] + (c == 2 ? J[i * 3 + 2] : 0.0);
  }
  for (int i = 0; i < 2; ++i) {
    x1[i] = x[i] + h / 6.0 * (k[0][i] + 2.0 * k[1][i] + 2.0 * k[2][i] + k[3][i]);
    B[i] = h / 6.0 * (dk[0][i][2] + 2.0 * dk[1][i][2] + 2.0 * dk[2][i][2] + dk[3][i][2]);
  }
}

static void shoot(int nq, double h, const double* x, const double* u, double* x1, double* B) {
  if (nq == 1) { pend_rk4_sens(h, x, u, x1, B); return; }
  double A[HX * HX];
  vboc_oracle_rk4_sens(nq, h, x, u, x1, A, B);
}

static double wupd(double w, double lam) {
  const double a = fabs(lam), b = 0.5 * (w + a);
  return a > b ? a : b;
}

typedef struct { double n, d; } mr_t;
static void mr_add(mr_t* m, double t, double dt) {
  if (dt < 0.0 && t * m->d < m->n * (-dt)) { m->n = t; m->d = -dt; }
}

static int chol_n(int n, double* A) {
  for (int j = 0; j < n; ++j) {
    double s = A[j * n + j];
    for (int k = 0; k < j; ++k) s -= A[j * n + k] * A[j * n + k];
    if (!(s > 0.0)) return -1;
    const double d = sqrt(s);
    A[j * n + j] = d;
    for (int i = j + 1; i < n; ++i) {
      double t = A[i * n + j];
      for (int k = 0; k < j; ++k) t -= A[i * n + k] * A[j * n + k];
      A[i * n + j] = t / d;
    }
  }
  return 0;
}
static void chol_solve_n(int n, const double* L, double* b) {
  for (int i = 0; i < n; ++i) {
    double t = b[i];
    for (int k = 0; k < i; ++k) t -= L[i * n + k] * b[k];
    b[i] = t / L[i * n + i];
  }
  for (int i = n - 1; i >= 0; --i) {
    double t = b[i];
    for (int k = i + 1; k < n; ++k) t -= L[k * n + i] * b[k];
    b[i] = t / L[i * n + i];
  }
}

typedef struct {
  int nq, nx, nu;
  double h, rho;
  double x0[HX], lbu[HQ], ubu[HQ];
  double u[HQ], x1[HX], pi[HX], ll[HQ], lu[HQ], wpi[HX], wbnd;
  /* linearisation */
  double phi[HX], B[HX * HQ], b[HX], c, gnn[HX];
  /* QP */
  double du[HQ], dx[HX], ql[HQ], qu[HQ], L[HQ], U[HQ], e0[HX], qpi[HX];
  const hnn_t* nn;
  vboc_opts_t o;
} hprob_t;

/* one-stage Riccati solve of  min 1/2 d'Hd + g'd  s.t.  dx = B du + rs e0 :  x1 eliminated (P = diag(Hx),
   p = gx), du = -(Hu + B'PB)^-1 (gu + B'(P rs e0 + p)) */
static int newton(hprob_t* P, const double* Hu, const double* gu, const double* Hx, const double* gx, double rs,
                  double* du, double* dx) {
  const int nx = P->nx, nu = P->nu;
  double Ru[HQ * HQ], v[HX], r[HQ];
  for (int a = 0; a < nu; ++a)
    for (int c = 0; c < nu; ++c) {
      double t = (a == c) ? Hu[a] : 0.0;
      for (int i = 0; i < nx; ++i) t += P->B[i * nu + a] * Hx[i] * P->B[i * nu + c];
      Ru[a * nu + c] = t;
    }
  if (chol_n(nu, Ru)) return -1;
  for (int i = 0; i < nx; ++i) v[i] = Hx[i] * (rs * P->e0[i]) + gx[i];
  for (int a = 0; a < nu; ++a) {
    double t = gu[a];
    for (int i = 0; i < nx; ++i) t += P->B[i * nu + a] * v[i];
    r[a] = t;
  }
  chol_solve_n(nu, Ru, r);
  for (int a = 0; a < nu; ++a) du[a] = -r[a];
  for (int i = 0; i < nx; ++i) {
    double t = rs * P->e0[i];
    for (int a = 0; a < nu; ++a) t += P->B[i * nu + a] * du[a];
    dx[i] = t;
  }
  return 0;
}

/* the Mehrotra predictor-corrector IPM of vboc_oracle.c qp_solve on the one-stage QP; returns 0 converged,
   1 max-iter, -1 failure; the QP costate pi into qpi */
static int qp(hprob_t* P, int* iters) {
  const int nx = P->nx, nu = P->nu;
  const vboc_opts_t* o = &P->o;
  const double rho = P->rho;
  int nbox = 0;
  for (int a = 0; a < nu; ++a) {
    const double L = P->lbu[a] - P->u[a], U = P->ubu[a] - P->u[a], del = o->ipm_push * (U - L);
    double z0 = 0.0;
    if (z0 < L + del) z0 = L + del;
    if (z0 > U - del) z0 = U - del;
    P->L[a] = L; P->U[a] = U; P->du[a] = z0;
    P->ql[a] = o->mu0 / (z0 - L);
    P->qu[a] = o->mu0 / (U - z0);
    nbox += 2;
  }
  for (int i = 0; i < nx; ++i) P->dx[i] = 0.0;
  double e00 = 0.0, rd0 = 0.0;
  for (int i = 0; i < nx; ++i) {
    double t = P->b[i] - P->dx[i];
    for (int a = 0; a < nu; ++a) t += P->B[i * nu + a] * P->du[a];
    P->e0[i] = t;
    e00 = fmax(e00, fabs(t));
  }
  for (int a = 0; a < nu; ++a) rd0 = fmax(rd0, fabs(rho * P->du[a] - P->ql[a] + P->qu[a]));
  for (int i = 0; i < nx; ++i) rd0 = fmax(rd0, fabs(rho * P->dx[i] + P->gnn[i]));
  double rs = 1.0;
  int it, status = 1;
  double Hu[HQ], gu[HQ], Hx[HX], gx[HX], du[HQ], dx[HX], dua[HQ];
  for (it = 0; it < o->qp_max_iter; ++it) {
    double mu = 0.0;
    for (int a = 0; a < nu; ++a) mu += (P->du[a] - P->L[a]) * P->ql[a] + (P->U[a] - P->du[a]) * P->qu[a];
    mu /= (double)nbox;
    if (!isfinite(mu)) { status = -1; break; }
    if (mu < o->qp_tol_comp && rs * rd0 < o->qp_tol_stat && rs * e00 < o->qp_tol_eq) { status = 0; break; }
    /* predictor */
    for (int a = 0; a < nu; ++a) {
      const double tl = P->du[a] - P->L[a], tu = P->U[a] - P->du[a];
      Hu[a] = rho + P->ql[a] * (1.0 / tl) + P->qu[a] * (1.0 / tu);
      gu[a] = rho * P->du[a];
    }
    for (int i = 0; i < nx; ++i) { Hx[i] = rho; gx[i] = rho * P->dx[i] + P->gnn[i]; }
    if (newton(P, Hu, gu, Hx, gx, rs, du, dx)) { status = -1; break; }
    mr_t ma = {1.0, 1.0};
    for (int a = 0; a < nu; ++a) {
      const double tl = P->du[a] - P->L[a], tu = P->U[a] - P->du[a], itl = 1.0 / tl, itu = 1.0 / tu, d = du[a];
      const double dll = -P->ql[a] - P->ql[a] * d * itl, dlu = -P->qu[a] + P->qu[a] * d * itu;
      mr_add(&ma, tl, d);
      mr_add(&ma, tu, -d);
      mr_add(&ma, P->ql[a], dll);
      mr_add(&ma, P->qu[a], dlu);
      dua[a] = d;
    }
    const double aa = ma.n / ma.d;
    double muaff = 0.0;
    for (int a = 0; a < nu; ++a) {
      const double tl = P->du[a] - P->L[a], tu = P->U[a] - P->du[a], itl = 1.0 / tl, itu = 1.0 / tu, d = du[a];
      const double dll = -P->ql[a] - P->ql[a] * d * itl, dlu = -P->qu[a] + P->qu[a] * d * itu;
      muaff += (tl + aa * d) * (P->ql[a] + aa * dll) + (tu - aa * d) * (P->qu[a] + aa * dlu);
    }
    muaff /= (double)nbox;
    double sig = muaff / mu;
    sig = sig * sig * sig;
    if (sig > 1.0) sig = 1.0;
    const double smu = sig * mu;
    /* corrector */
    for (int a = 0; a < nu; ++a) {
      const double tl = P->du[a] - P->L[a], tu = P->U[a] - P->du[a], itl = 1.0 / tl, itu = 1.0 / tu, d = dua[a];
      const double dll = -P->ql[a] - P->ql[a] * d * itl, dlu = -P->qu[a] + P->qu[a] * d * itu;
      const double rl = smu - tl * P->ql[a] - d * dll, ru = smu - tu * P->qu[a] + d * dlu;
      gu[a] = rho * P->du[a] - P->ql[a] - rl * itl + P->qu[a] + ru * itu;
    }
    if (newton(P, Hu, gu, Hx, gx, rs, du, dx)) { status = -1; break; }
    mr_t mx = {1.0, o->ipm_tau};
    double dll[HQ], dlu[HQ];
    for (int a = 0; a < nu; ++a) {
      const double tl = P->du[a] - P->L[a], tu = P->U[a] - P->du[a], itl = 1.0 / tl, itu = 1.0 / tu;
      const double d = du[a], da = dua[a];
      const double dlla = -P->ql[a] - P->ql[a] * da * itl, dlua = -P->qu[a] + P->qu[a] * da * itu;
      const double rl = smu - tl * P->ql[a] - da * dlla, ru = smu - tu * P->qu[a] + da * dlua;
      dll[a] = (rl - P->ql[a] * d) * itl;
      dlu[a] = (ru + P->qu[a] * d) * itu;
      mr_add(&mx, tl, d);
      mr_add(&mx, tu, -d);
      mr_add(&mx, P->ql[a], dll[a]);
      mr_add(&mx, P->qu[a], dlu[a]);
    }
    const double alpha = fmin(1.0, o->ipm_tau * (mx.n / mx.d));
    for (int a = 0; a < nu; ++a) {
      P->ql[a] += alpha * dll[a];
      P->qu[a] += alpha * dlu[a];
      P->du[a] += alpha * du[a];
    }
    for (int i = 0; i < nx; ++i) P->dx[i] += alpha * dx[i];
    rs *= (1.0 - alpha);
  }
  *iters = it;
  if (status < 0) return -1;
  /* costate: stationarity of the QP in dx1 (x1 unboxed): pi = rho dx1 + grad NN */
  for (int i = 0; i < nx; ++i) P->qpi[i] = rho * P->dx[i] + P->gnn[i];
  for (int a = 0; a < nu; ++a)
    if (!isfinite(P->du[a]) || !isfinite(P->ql[a]) || !isfinite(P->qu[a])) return -1;
  return status;
}

/* L1 merit at (u + alpha du, x1 + alpha dx), the defect re-simulated */
static double merit(const hprob_t* P, double alpha) {
  const int nx = P->nx, nu = P->nu;
  double u[HQ], x1[HX], phi[HX], B[HX * HQ];
  double viol = 0.0;
  for (int a = 0; a < nu; ++a) {
    u[a] = P->u[a] + alpha * P->du[a];
    viol += fmax(0.0, P->lbu[a] - u[a]) + fmax(0.0, u[a] - P->ubu[a]);
  }
  for (int i = 0; i < nx; ++i) x1[i] = P->x1[i] + alpha * P->dx[i];
  double val = nn_eval(P->nn, x1, NULL) + P->wbnd * viol;
  shoot(P->nq, P->h, P->x0, u, phi, B);
  for (int i = 0; i < nx; ++i) val += P->wpi[i] * fabs(phi[i] - x1[i]);
  return val;
}

static void hjr_sqp(hprob_t* P, vboc_result_t* res) {
  const int nx = P->nx, nu = P->nu;
  const vboc_opts_t* o = &P->o;
  int status = 2, it, qp_total = 0;
  double rstat = 0, req = 0, rineq = 0, rcomp = 0;
  for (it = 0;; ++it) {
    shoot(P->nq, P->h, P->x0, P->u, P->phi, P->B);
    for (int i = 0; i < nx; ++i) P->b[i] = P->phi[i] - P->x1[i];
    P->c = nn_eval(P->nn, P->x1, P->gnn);
    double st = 0, eq = 0, in = 0, cp = 0;
    for (int i = 0; i < nx; ++i) eq = fmax(eq, fabs(P->b[i]));
    for (int a = 0; a < nu; ++a) {
      double gr = -P->ll[a] + P->lu[a];
      for (int r = 0; r < nx; ++r) gr += P->B[r * nu + a] * P->pi[r];
      st = fmax(st, fabs(gr));
      in = fmax(in, fmax(P->lbu[a] - P->u[a], P->u[a] - P->ubu[a]));
      cp = fmax(cp, fmax(fabs(P->ll[a] * (P->u[a] - P->lbu[a])), fabs(P->lu[a] * (P->ubu[a] - P->u[a]))));
    }
    for (int i = 0; i < nx; ++i) st = fmax(st, fabs(P->gnn[i] - P->pi[i]));
    rstat = st; req = eq; rineq = in; rcomp = cp;
    if (!isfinite(rstat) || !isfinite(req)) { status = 1; break; }
    if (rstat < o->tol_stat && req < o->tol_eq && rineq < o->tol_ineq && rcomp < o->tol_comp) { status = 0; break; }
    if (it >= o->max_iter) { status = 2; break; }
    int qit = 0;
    const int qs = qp(P, &qit);
    qp_total += qit;
    if (qs < 0) { status = 4; break; }
    double lmax = 0.0;
    for (int i = 0; i < nx; ++i) P->wpi[i] = wupd(P->wpi[i], P->qpi[i]);
    for (int a = 0; a < nu; ++a) lmax = fmax(lmax, fmax(P->ql[a], P->qu[a]));
    P->wbnd = wupd(P->wbnd, lmax);
    const double phi0 = merit(P, 0.0);
    double alpha = 1.0;
    for (;;) {
      const double pa = merit(P, alpha);
      if (pa < phi0) break;
      if (alpha * o->alpha_reduction < o->alpha_min) break;
      alpha *= o->alpha_reduction;
    }
    for (int a = 0; a < nu; ++a) {
      P->u[a] += alpha * P->du[a];
      P->ll[a] += alpha * (P->ql[a] - P->ll[a]);
      P->lu[a] += alpha * (P->qu[a] - P->lu[a]);
    }
    for (int i = 0; i < nx; ++i) {
      P->x1[i] += alpha * P->dx[i];
      P->pi[i] += alpha * (P->qpi[i] - P->pi[i]);
    }
  }
  res->status = status;
  res->sqp_iter = it;
  res->qp_iter = qp_total;
  res->cost = nn_eval(P->nn, P->x1, NULL);
  res->res_stat = rstat; res->res_eq = req; res->res_ineq = rineq; res->res_comp = rcomp;
}

void vboc_oracle_hjr_default_opts(int nq, vboc_opts_t* o) {
  vboc_oracle_default_opts(o);
  o->tol_stat = 1e-6;                  /* ACADOS defaults: the HJR classes set no tolerances */
  o->qp_tol_stat = 1e-8;
  o->lm = nq == 1 ? 1e-2 : 1e-5;       /* HJR/pendulum_hjr_class.py:97; triplependulum_hjr_class.py:108 */
}

int vboc_oracle_hjr_solve_batch(int nq, int B, const double* x0, int h, const double* W0, const double* b0,
                                const double* W1, const double* b1, const double* W2, const double* b2, double mean,
                                double std, double u_max, const vboc_opts_t* opts, int nthreads, double* u_out,
                                double* x1_out, double* mult_out, vboc_result_t* res) {
  if (nq < 1 || nq > 3 || h < 1 || h > HMAX || B < 0) return -1;
  const int nx = 2 * nq;
  hnn_t nn = {nx, h, W0, b0, W1, b1, W2, b2, mean, std};
#pragma omp parallel for schedule(dynamic, 4) num_threads(nthreads)
  for (int b = 0; b < B; ++b) {
    hprob_t P;
    memset(&P, 0, sizeof(P));
    P.nq = nq; P.nx = nx; P.nu = nq; P.h = 1e-2; P.rho = opts->lm; P.o = *opts; P.nn = &nn;
    const double* x = x0 + (size_t)b * nx;
    memcpy(P.x0, x, sizeof(double) * nx);
    for (int a = 0; a < nq; ++a) { P.lbu[a] = -u_max; P.ubu[a] = u_max; }
    /* compute_problem's guess: x1 = [q0 + v0 1e-2, 0.9 v0] (:119) */
    for (int j = 0; j < nq; ++j) { P.x1[j] = x[j] + x[nq + j] * 1e-2; P.x1[nq + j] = x[nq + j] * 0.9; }
    hjr_sqp(&P, res + b);
    memcpy(u_out + (size_t)b * nq, P.u, sizeof(double) * nq);
    memcpy(x1_out + (size_t)b * nx, P.x1, sizeof(double) * nx);
    if (mult_out) {   /* pi (nx), lam_l (nu), lam_u (nu) of the final iterate */
      double* m = mult_out + (size_t)b * (nx + 2 * nq);
      memcpy(m, P.pi, sizeof(double) * nx);
      memcpy(m + nx, P.ll, sizeof(double) * nq);
      memcpy(m + nx + nq, P.lu, sizeof(double) * nq);
    }
  }
  return 0;
}

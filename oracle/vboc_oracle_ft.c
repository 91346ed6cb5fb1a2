/*
 * ORACLE - TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by or called from the product
 * path (vboc_amd/).  Only tests/ use it, and only as the checker.
 *
 * Plain-C FP64 restatement of the FREE-TIME box OCP of the reference's OCP<sys> classes, i.e. what
 *   OCPpendulum.OCP_solve(x_guess, u_guess, cost_dir, q_lb, q_ub, q_init, q_fin)
 *   (VBOC/pendulum_class_vboc.py:107-130, model and options :8-103)
 * asks ACADOS to do.  Differences from the boundary OCP of vboc_oracle.c:
 *  - dt is a genuine state: x = [theta, dtheta, dt], f_expl = dt * [dtheta, acc, 0]
 *    (pendulum_class_vboc.py:23-40), bounded dt in [0, 1e-2] at every stage (:80-89); one ERK4 step
 *    of length 1 per interval (tf = N, :55-58) = RK4 with h = dt on the physics rhs, and the
 *    shooting map's Jacobian carries the d/d(dt) column;
 *  - cost EXTERNAL, linear: w1 * dtheta + wt * dt at stage 0, wt * dt at stages 1..N-1, none at N
 *    (:70-74, p = [cost_dir, 1] from OCP_solve :116);
 *  - no general constraint (ng = 0); stage 0 fixes the components with lbx_0 == ubx_0 (theta,
 *    :119-120), the terminal stage the components with lbx_e == ubx_e (theta and dtheta, :121-122).
 * Same SQP / merit / Mehrotra-IPM / Riccati algorithm and options as vboc_oracle.c (that file's
 * header lists them), generalised to:
 *  - stage-0 decision variables = the free components of x_0 plus u_0 (fixed ones are constants);
 *  - terminal equalities E x_N = x_fix on any subset of components (Schur complement in the
 *    backward sweep through Pi = E', exactly as the terminal-velocity equality of vboc_oracle.c);
 *  - per-stage linear cost gradients.
 * Path bounds must be proper boxes (lb < ub on every component); otherwise -2 (unsupported).
 *
 * The same solver also restates the Safe-MPC OCP of the reference (`OCPtriplependulumHardTerm`,
 * VBOC/Safe MPC/triplependulum_class_vboc.py:91-240; vboc_oracle_mpc_solve below):
 *  - model MODELtriplependulum (nx 6, nu 3, :8-78) on intervals of time_step: here the dt column of the
 *    free-time model pinned by the fixed x_0 (dt_{k+1} = dt_k, unbounded on the path), an exact reformulation;
 *  - LINEAR_LS cost 1/2 |[x; u] - yref|^2_W at stages 0..N-1 and 1/2 |x_N - yref_e|^2_{W_e} at N (:108-134) with the
 *    Gauss-Newton Hessian W (+ levenberg_marquardt), stage costs scaled by `cs` (ACADOS' cost_scaling: the time
 *    step in current releases, 1 in older ones - the version is unpinned);
 *  - x_0 fixed (OCP_solve's constraints_set(0, lbx / ubx, x0), :163-181), path and terminal boxes (:136-151);
 *  - the terminal nonlinear row 0 <= h(x_N) = NN(x_N) - max(|x_N[2:]|, 1e-3) <= 1e6 (HardTerm :197-240,
 *    nn_decisionfunction: NeuralNetDIR(6, hid, 1), positions (x - mean) / std, velocities / that norm - the
 *    reference's x[2:] includes theta_3, kept), handled like the Cartesian rows of vboc_oracle.c (two slacks,
 *    infeasible start, sigma c c' in the terminal Riccati block); no constraint Hessian (Gauss-Newton);
 *  - SQP_RTI (the Safe-MPC driver's option, hard_terminal_constraints/3dof_sym.py:96): one linearisation, one QP,
 *    the full step; status 0, or 4 if the QP fails.
 * and `OCPtriplependulumSoftTraj` (triplependulum_class_vboc.py:242-304; vboc_mpc_soft_t): the row scaled by the
 * safety margin, h(x) = NN(z(x)) (100 - m) / 100 - vn(x), on EVERY stage 0..N (con_h_expr and con_h_expr_e), each row
 * soft on its lower side (idxsh / idxsh_e) with a slack s_k >= 0 costing cs_k (zl_k s_k + Zl_k s_k^2 / 2), cs_k = cs
 * on stages 0..N-1 and 1 at N like the stage's least-squares cost (ACADOS' cost_scaling scales z / Z too; the drivers'
 * cost_set(k, "Zl", ...) per stage, soft_traj_constraints/3dof_sym.py:102-105, receiding_hard_constraints/
 * 3dof_sym.py:41-46); the upper side (uh = 1e6, zu = Zu = 0) is kept hard - it is never active.  In the QP the slack
 * is a variable of its own (absolute value, so an RTI QP does not depend on the previous slack iterate) with a
 * barrier on s >= 0; it is eliminated per stage in the Riccati recursion:
 *     W = Zl + Sl + Ss (Sl = ql / tl, Ss = qs / s),   sigma = Su + Sl (Zl + Ss) / W   (the row's c c' weight),
 *     gamma += Sl b / W with b = -(Zl s + zl - ql - qs) + rcl / tl + rcs / s - Sl rl  (the row's gradient term),
 *     ds = (b - Sl c'd) / W,  dtl = c'd + ds + rl,  dqs = (rcs - qs ds) / s.
 * In SQP mode the slacks are NLP variables (updated with the step, their cost and the soft rows' violation in the
 * merit); the drivers run SQP_RTI.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "vboc_oracle.h"

#define FQ 3
#define FX (2 * FQ + 1)
#define FU FQ
#define FZ (FX + FU)

typedef struct {
  double x[FX], u[FU];
  double pi[FX], ll[FZ], lu[FZ], wpi[FX];
  double A[FX * FX], B[FX * FU], F0[FX * FZ], b[FX];
  double Lb[FZ], Ub[FZ], dz[FZ], ql[FZ], qu[FZ], e0[FX];
  double H[FZ], g[FZ], d[FZ], daff[FZ];
  double K[FU * FX], kf[FU], Lr[FZ * FZ], M[FZ * FX], Y[FZ * FX], Pe[FX], qpi[FX];
  /* the Safe-MPC NN row of this stage (HardTerm: stage N only; SoftTraj: every stage): value, gradient, QP slacks /
     duals of both sides, their affine directions, residual starts, the NLP multipliers; the soft lower side's slack
     (QP value hs, dual hqs, affine directions), its NLP iterate sl / multiplier lsl and weights zl, Zl; hsig the
     row's c c' weight in the factorisation */
  double hv, hg[FX], hL, hU, htl, htu, hql, hqu, hr0l, hr0u, hatl, hatu, haql, haqu, hll, hlu;
  double hs, hqs, has, haqs, sl, lsl, zl, Zl, hsig, hb, hW;
  double hdtl, hdtu, hdql, hdqu, hds, hdqs;   /* the combined (corrector) directions of the iteration */
} fstage_t;

typedef struct {
  int nq, nx, nu, N;
  int nf0, f0[FX];              /* free stage-0 components */
  int ne, ei[FX];               /* fixed terminal components */
  double ev[FX];                /* their values */
  double c0[FX], cp[FX];        /* cost gradients: stage 0, stages 1..N-1 */
  double x0lb[FX], x0ub[FX], xlb[FX], xub[FX], xNlb[FX], xNub[FX], ulb[FU], uub[FU];
  int xNfix[FX];
  double tnu[FX], wnu[FX], wbnd, qnu[FX];   /* terminal multipliers, merit weights */
  double S[FX * FX], lin_e[FX], rs;
  fstage_t* st;
  vboc_opts_t o;
  /* Safe-MPC tracking cost and terminal row (vboc_oracle_mpc_solve; all zero / NULL for the free-time OCP) */
  int track, rti;
  double wq[FZ], yr[FZ], we[FX], yre[FX], cs;
  const vboc_mpc_nn_t* nn;
  int soft;        /* SoftTraj: rows on every stage, soft lower sides, the row scaled by sm / 100 */
  int qcf;         /* a QP stopped by qp_max_iter is a QP failure (status 4): the AL labelling OCP */
  double sm;       /* 100 - safety_margin */
} fprob_t;

/* stage k carries the NN row */
static int frow(const fprob_t* P, int k) { return P->nn && (P->soft || k == P->N); }

/* ------------------------------------------------------------------------------------------ */
/* the Safe-MPC terminal row h(x) = NN(z(x)) - vn(x) (nn_decisionfunction, :208-230) and grad    */
/* ------------------------------------------------------------------------------------------ */
static double nn_row(const vboc_mpc_nn_t* n, int nq, const double* x, double* grad, int soft, double sm) {
  const int nx = 2 * nq, H = n->hid;
  double ss = 0.0;
  for (int j = 2; j < nx; ++j) ss += x[j] * x[j];   /* norm_2(x[2:]) - theta_3 included, as the reference */
  const double nrm = sqrt(ss), vn = nrm > 1e-3 ? nrm : 1e-3;
  double z[2 * FQ];
  for (int j = 0; j < nq; ++j) z[j] = (x[j] - n->mean) / n->std;
  for (int j = nq; j < nx; ++j) z[j] = x[j] / vn;
  double* a1 = (double*)malloc(sizeof(double) * 2 * H);
  double* a2 = a1 + H;
  for (int i = 0; i < H; ++i) {
    double t = 0.0;
    for (int j = 0; j < nx; ++j) t += n->W0[i * nx + j] * z[j];
    t += n->b0[i];
    a1[i] = t > 0.0 ? t : 0.0;   /* fmax(0., out) */
  }
  double out = 0.0;
  for (int i = 0; i < H; ++i) {
    double t = 0.0;
    for (int j = 0; j < H; ++j) t += n->W1[i * H + j] * a1[j];
    t += n->b1[i];
    a2[i] = t;
    if (t > 0.0) out += n->W2[i] * t;
  }
  out += n->b2[0];
  if (soft) out = out * sm / 100.0;   /* nn_decisionfunction_conservative: out*(100-safety_margin)/100 (:301) */
  if (grad) {
    /* d out / d z by reverse mode through the two ReLUs (derivative 0 at a kink) */
    double* g1 = (double*)calloc((size_t)H, sizeof(double));
    for (int i = 0; i < H; ++i) {
      if (!(a2[i] > 0.0)) continue;
      const double w = n->W2[i];
      for (int j = 0; j < H; ++j) g1[j] += w * n->W1[i * H + j];
    }
    double gz[2 * FQ] = {0};
    for (int i = 0; i < H; ++i) {
      if (!(a1[i] > 0.0)) continue;
      for (int j = 0; j < nx; ++j) gz[j] += g1[i] * n->W0[i * nx + j];
    }
    free(g1);
    if (soft) for (int j = 0; j < nx; ++j) gz[j] = gz[j] * sm / 100.0;
    /* chain rule through z(x) and vn(x) = max(|x[2:]|, 1e-3) */
    double dvn[2 * FQ] = {0};
    if (nrm > 1e-3) for (int j = 2; j < nx; ++j) dvn[j] = x[j] / nrm;
    for (int j = 0; j < nx; ++j) {
      double t = j < nq ? gz[j] / n->std : gz[j] / vn;
      for (int q = nq; q < nx; ++q) t -= gz[q] * x[q] / (vn * vn) * dvn[j];
      grad[j] = t - dvn[j];
    }
  }
  free(a1);
  return out - vn;
}

/* ------------------------------------------------------------------------------------------ */
/* dynamics: physics rhs with analytic Jacobians (vboc_oracle_model), ERK4 with h = dt and the   */
/* exact derivative of the discrete map w.r.t. (theta, dtheta, dt, u)                           */
/* ------------------------------------------------------------------------------------------ */

/* k = f(X, u); dk[:, c] = J(X) T[:, c] + df/du e_{c - ncol_u}  for the given tangent columns */
static void rhs_t(int nq, const double* X, const double* u, const double* T, int nc, int cu0, double* k,
                  double* dk) {
  double acc[FQ], Jth[FQ * FQ], Jom[FQ * FQ], Ju[FQ * FQ];
  vboc_oracle_model(nq, X, X + nq, u, acc, Jth, Jom, Ju);
  for (int j = 0; j < nq; ++j) { k[j] = X[nq + j]; k[nq + j] = acc[j]; }
  for (int c = 0; c < nc; ++c) {
    for (int j = 0; j < nq; ++j) dk[j * nc + c] = T[(nq + j) * nc + c];
    for (int j = 0; j < nq; ++j) {
      double t = (c >= cu0 && c < cu0 + nq) ? Ju[j * nq + (c - cu0)] : 0.0;
      for (int q = 0; q < nq; ++q) t += Jth[j * nq + q] * T[q * nc + c] + Jom[j * nq + q] * T[(nq + q) * nc + c];
      dk[(nq + j) * nc + c] = t;
    }
  }
}

/* Phi(x, u) for x = [q, v, dt]; A = dPhi/dx (nx x nx, last column d/d(dt)), B = dPhi/du */
static void ft_rk4_sens(int nq, const double* x, const double* u, double* phi, double* A, double* B) {
  const int n2 = 2 * nq, nx = n2 + 1, nu = nq;
  const int nc = n2 + nu + 1, cu0 = n2, ch = n2 + nu; /* tangent columns: (q,v), u, h */
  const double h = x[n2];
  double X[2 * FQ], T[2 * FQ * (FX + FU)], k[2 * FQ], dk[2 * FQ * (FX + FU)];
  double ks[2 * FQ], Ts[2 * FQ * (FX + FU)], kp[2 * FQ], dkp[2 * FQ * (FX + FU)];
  static const double cst[4] = {0.0, 0.5, 0.5, 1.0}, wgt[4] = {1.0, 2.0, 2.0, 1.0};
  memset(ks, 0, sizeof(ks));
  memset(Ts, 0, sizeof(Ts));
  memset(kp, 0, sizeof(kp));
  memset(dkp, 0, sizeof(dkp));
  for (int s = 0; s < 4; ++s) {
    /* stage point X = x + c h k_prev, tangent d X / d(col) */
    for (int i = 0; i < n2; ++i) {
      X[i] = x[i] + cst[s] * h * kp[i];
      for (int c = 0; c < nc; ++c) {
        double t = cst[s] * h * dkp[i * nc + c];
        if (c == i) t += 1.0;
        if (c == ch) t += cst[s] * kp[i];
        T[i * nc + c] = t;
      }
    }
    rhs_t(nq, X, u, T, nc, cu0, k, dk);
    for (int i = 0; i < n2; ++i) {
      ks[i] += wgt[s] * k[i];
      for (int c = 0; c < nc; ++c) Ts[i * nc + c] += wgt[s] * dk[i * nc + c];
    }
    memcpy(kp, k, sizeof(kp));
    memcpy(dkp, dk, sizeof(dkp));
  }
  for (int i = 0; i < n2; ++i) {
    phi[i] = x[i] + h / 6.0 * ks[i];
    for (int c = 0; c < n2; ++c) A[i * nx + c] = (c == i ? 1.0 : 0.0) + h / 6.0 * Ts[i * nc + c];
    A[i * nx + n2] = ks[i] / 6.0 + h / 6.0 * Ts[i * nc + ch];
    for (int a = 0; a < nu; ++a) B[i * nu + a] = h / 6.0 * Ts[i * nc + cu0 + a];
  }
  phi[n2] = h;
  for (int c = 0; c < nx; ++c) A[n2 * nx + c] = (c == n2) ? 1.0 : 0.0;
  for (int a = 0; a < nu; ++a) B[n2 * nu + a] = 0.0;
}

static void ft_rk4(int nq, const double* x, const double* u, double* phi) {
  double A[FX * FX], B[FX * FU];
  ft_rk4_sens(nq, x, u, phi, A, B);
}

/* ------------------------------------------------------------------------------------------ */
/* stage variables                                                                             */
/* ------------------------------------------------------------------------------------------ */

static int fnz(const fprob_t* P, int k) {
  if (k == 0) return P->nf0 + P->nu;
  if (k == P->N) return P->nx;
  return P->nx + P->nu;
}

static void fcomp(const fprob_t* P, int k, int i, double* val, double* lb, double* ub, int* boxed) {
  const fstage_t* s = &P->st[k];
  const int nx = P->nx;
  *boxed = 1;
  if (k == 0) {
    if (i < P->nf0) { const int c = P->f0[i]; *val = s->x[c]; *lb = P->x0lb[c]; *ub = P->x0ub[c]; }
    else { *val = s->u[i - P->nf0]; *lb = P->ulb[i - P->nf0]; *ub = P->uub[i - P->nf0]; }
  } else if (k == P->N) {
    *val = s->x[i];
    if (P->xNfix[i]) { *lb = -INFINITY; *ub = INFINITY; *boxed = 0; }
    else { *lb = P->xNlb[i]; *ub = P->xNub[i]; }
  } else if (i < nx) { *val = s->x[i]; *lb = P->xlb[i]; *ub = P->xub[i]; }
  else { *val = s->u[i - nx]; *lb = P->ulb[i - nx]; *ub = P->uub[i - nx]; }
  if (isinf(*lb) && isinf(*ub)) *boxed = 0;   /* a free component (the Safe-MPC model's pinned dt) */
}

/* stage-variable index i of stage k -> index into the tracking weights [x (nx); u (nu)] (-1: none) */
static int fwidx(const fprob_t* P, int k, int i) {
  if (k == 0) return i < P->nf0 ? P->f0[i] : P->nx + (i - P->nf0);
  return i;
}
/* Gauss-Newton Hessian diagonal of the tracking cost (0 for the free-time OCP) */
static double fhq(const fprob_t* P, int k, int i) {
  if (!P->track) return 0.0;
  if (k == P->N) return P->we[i];
  return P->cs * P->wq[fwidx(P, k, i)];
}

static double fgrad(const fprob_t* P, int k, int i) {
  if (P->track) {   /* W ([x; u] - yref) at the current iterate */
    double v, lb, ub; int boxed;
    fcomp(P, k, i, &v, &lb, &ub, &boxed);
    if (k == P->N) return P->we[i] * (v - P->yre[i]);
    const int w = fwidx(P, k, i);
    return P->cs * P->wq[w] * (v - P->yr[w]);
  }
  if (k == 0) return i < P->nf0 ? P->c0[P->f0[i]] : 0.0;
  if (k == P->N) return 0.0;
  return i < P->nx ? P->cp[i] : 0.0;
}

/* the tracking cost of stage states (x, u) (u NULL at the terminal stage) */
static double ftrack(const fprob_t* P, int k, const double* x, const double* u) {
  double c = 0.0;
  if (k == P->N) {
    for (int i = 0; i < P->nx; ++i) { const double d = x[i] - P->yre[i]; c += P->we[i] * d * d; }
    return 0.5 * c;
  }
  for (int i = 0; i < P->nx; ++i) { const double d = x[i] - P->yr[i]; c += P->wq[i] * d * d; }
  for (int a = 0; a < P->nu; ++a) { const double d = u[a] - P->yr[P->nx + a]; c += P->wq[P->nx + a] * d * d; }
  return 0.5 * P->cs * c;
}

static double fcost(const fprob_t* P) {
  double c = 0.0;
  if (P->track) {
    for (int k = 0; k <= P->N; ++k) c += ftrack(P, k, P->st[k].x, k < P->N ? P->st[k].u : NULL);
    if (P->soft)   /* the slacks' penalties (ACADOS' get_cost includes them) */
      for (int k = 0; k <= P->N; ++k) c += P->st[k].zl * P->st[k].sl + 0.5 * P->st[k].Zl * P->st[k].sl * P->st[k].sl;
    return c;
  }
  for (int i = 0; i < P->nx; ++i) c += P->c0[i] * P->st[0].x[i];
  for (int k = 1; k < P->N; ++k)
    for (int i = 0; i < P->nx; ++i) c += P->cp[i] * P->st[k].x[i];
  return c;
}

/* ------------------------------------------------------------------------------------------ */
/* linearisation + NLP residuals                                                               */
/* ------------------------------------------------------------------------------------------ */

static void flinearize(fprob_t* P) {
  const int nx = P->nx, nu = P->nu, m0 = P->nf0 + nu;
  for (int k = 0; k < P->N; ++k) {
    fstage_t* s = &P->st[k];
    double phi[FX];
    ft_rk4_sens(P->nq, s->x, s->u, phi, s->A, s->B);
    for (int i = 0; i < nx; ++i) s->b[i] = phi[i] - P->st[k + 1].x[i];
  }
  fstage_t* s0 = &P->st[0];
  for (int i = 0; i < nx; ++i) {
    for (int j = 0; j < P->nf0; ++j) s0->F0[i * m0 + j] = s0->A[i * nx + P->f0[j]];
    for (int a = 0; a < nu; ++a) s0->F0[i * m0 + P->nf0 + a] = s0->B[i * nu + a];
  }
  for (int k = 0; k <= P->N; ++k) {   /* the rows: value and gradient (the pinned dt column has none) */
    if (!frow(P, k)) continue;
    fstage_t* s = &P->st[k];
    memset(s->hg, 0, sizeof(s->hg));
    s->hv = nn_row(P->nn, P->nq, s->x, s->hg, P->soft, P->sm);
  }
}

static void fresiduals(const fprob_t* P, double* rstat, double* req, double* rineq, double* rcomp) {
  const int nx = P->nx, nu = P->nu, N = P->N, m0 = P->nf0 + nu;
  double st = 0, eq = 0, in = 0, cp = 0;
  for (int k = 0; k < N; ++k)
    for (int i = 0; i < nx; ++i) eq = fmax(eq, fabs(P->st[k].b[i]));
  for (int j = 0; j < P->ne; ++j) eq = fmax(eq, fabs(P->st[N].x[P->ei[j]] - P->ev[j]));
  for (int k = 0; k <= N; ++k) {
    const fstage_t* s = &P->st[k];
    for (int i = 0; i < fnz(P, k); ++i) {
      double v, lb, ub; int boxed;
      fcomp(P, k, i, &v, &lb, &ub, &boxed);
      double gr = fgrad(P, k, i) - s->ll[i] + s->lu[i];
      if (k == 0) {
        for (int r = 0; r < nx; ++r) gr += s->F0[r * m0 + i] * s->pi[r];
      } else if (k < N) {
        if (i < nx) {
          for (int r = 0; r < nx; ++r) gr += s->A[r * nx + i] * s->pi[r];
          gr -= P->st[k - 1].pi[i];
        } else {
          for (int r = 0; r < nx; ++r) gr += s->B[r * nu + (i - nx)] * s->pi[r];
        }
      } else {
        gr -= P->st[N - 1].pi[i];
        for (int j = 0; j < P->ne; ++j) if (P->ei[j] == i) gr += P->tnu[j];
      }
      if (frow(P, k)) {   /* the row's term on the state components of the stage's variables */
        const int xi = k == 0 ? (i < P->nf0 ? P->f0[i] : -1) : (i < nx ? i : -1);
        if (xi >= 0) gr += s->hg[xi] * (s->hlu - s->hll);
      }
      st = fmax(st, fabs(gr));
      if (boxed) {
        in = fmax(in, fmax(lb - v, v - ub));
        cp = fmax(cp, fmax(fabs(s->ll[i] * (v - lb)), fabs(s->lu[i] * (ub - v))));
      }
    }
  }
  for (int k = 0; k <= N; ++k) {
    if (!frow(P, k)) continue;
    const fstage_t* s = &P->st[k];
    const double sl = P->soft ? s->sl : 0.0;
    in = fmax(in, fmax(P->nn->lh - (s->hv + sl), s->hv - P->nn->uh));
    cp = fmax(cp, fmax(fabs(s->hll * (s->hv + sl - P->nn->lh)), fabs(s->hlu * (P->nn->uh - s->hv))));
    if (P->soft) {   /* the slack: s >= 0, its stationarity Zl s + zl - lambda_row - lambda_s = 0 */
      in = fmax(in, -sl);
      cp = fmax(cp, fabs(s->lsl * sl));
      st = fmax(st, fabs(s->Zl * sl + s->zl - s->hll - s->lsl));
    }
  }
  *rstat = st; *req = eq; *rineq = in; *rcomp = cp;
}

/* ------------------------------------------------------------------------------------------ */
/* Riccati solve of the Newton system (see newton_solve in vboc_oracle.c; Pi = E' here)        */
/* ------------------------------------------------------------------------------------------ */

static int fchol(int n, double* A) {
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
    for (int i = 0; i < j; ++i) A[i * n + j] = 0.0;
  }
  return 0;
}

static void fchol_solve(int n, const double* L, double* b) {
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

static int fnewton(fprob_t* P, int factor, double* nu_new) {
  const int nx = P->nx, nu = P->nu, ne = P->ne, N = P->N, m0 = P->nf0 + nu;
  const double rs = P->rs;
  double Pm[FX * FX], p[FX], Pi[FX * FX], lin[FX];
  fstage_t* sN = &P->st[N];
  memset(Pm, 0, sizeof(Pm));
  for (int i = 0; i < nx; ++i) { Pm[i * nx + i] = sN->H[i]; p[i] = sN->g[i]; }
  if (frow(P, N)) {   /* the terminal row's barrier: sigma c c' */
    const double sig = sN->hsig;
    for (int i = 0; i < nx; ++i)
      for (int j = 0; j < nx; ++j) Pm[i * nx + j] += sig * sN->hg[i] * sN->hg[j];
  }
  memset(Pi, 0, sizeof(Pi));
  for (int j = 0; j < ne; ++j) Pi[P->ei[j] * ne + j] = 1.0;
  memset(lin, 0, sizeof(lin));
  if (factor) { memset(P->S, 0, sizeof(P->S)); memset(P->lin_e, 0, sizeof(P->lin_e)); }

  for (int k = N - 1; k >= 0; --k) {
    fstage_t* s = &P->st[k];
    const int mk = (k == 0) ? m0 : nu;
    const double* Bk = (k == 0) ? s->F0 : s->B;
    const int uoff = (k == 0) ? 0 : nx;
    double e[FX], v[FX], r[FZ];
    for (int i = 0; i < nx; ++i) e[i] = rs * s->e0[i];
    if (factor) {
      for (int i = 0; i < nx; ++i) {
        double t = 0; for (int j = 0; j < nx; ++j) t += Pm[i * nx + j] * e[j];
        s->Pe[i] = t;
      }
      for (int j = 0; j < ne; ++j) {
        double t = 0; for (int i = 0; i < nx; ++i) t += Pi[i * ne + j] * e[i];
        P->lin_e[j] += t;
      }
      double BP[FZ * FX], Ru[FZ * FZ];
      for (int a = 0; a < mk; ++a)
        for (int j = 0; j < nx; ++j) {
          double t = 0; for (int i = 0; i < nx; ++i) t += Bk[i * mk + a] * Pm[i * nx + j];
          BP[a * nx + j] = t;
        }
      for (int a = 0; a < mk; ++a)
        for (int c = 0; c < mk; ++c) {
          double t = (a == c) ? s->H[uoff + a] : 0.0;
          for (int i = 0; i < nx; ++i) t += BP[a * nx + i] * Bk[i * mk + c];
          Ru[a * mk + c] = t;
        }
      for (int a = 0; a < mk; ++a)
        for (int c = 0; c < a; ++c) { const double t = 0.5 * (Ru[a * mk + c] + Ru[c * mk + a]); Ru[a * mk + c] = Ru[c * mk + a] = t; }
      if (fchol(mk, Ru)) return -1;
      memcpy(s->Lr, Ru, sizeof(double) * mk * mk);
      for (int a = 0; a < mk; ++a)
        for (int j = 0; j < ne; ++j) {
          double t = 0; for (int i = 0; i < nx; ++i) t += Bk[i * mk + a] * Pi[i * ne + j];
          s->Y[a * ne + j] = t;
        }
      for (int j = 0; j < ne; ++j) {
        double col[FZ];
        for (int a = 0; a < mk; ++a) col[a] = s->Y[a * ne + j];
        fchol_solve(mk, s->Lr, col);
        for (int a = 0; a < mk; ++a) s->M[a * ne + j] = col[a];
      }
      for (int i = 0; i < ne; ++i)
        for (int j = 0; j < ne; ++j) {
          double t = 0; for (int a = 0; a < mk; ++a) t += s->Y[a * ne + i] * s->M[a * ne + j];
          P->S[i * ne + j] += t;
        }
      if (k > 0) {
        double Sux[FU * FX];
        for (int a = 0; a < nu; ++a)
          for (int j = 0; j < nx; ++j) {
            double t = 0; for (int i = 0; i < nx; ++i) t += BP[a * nx + i] * s->A[i * nx + j];
            Sux[a * nx + j] = t;
          }
        for (int j = 0; j < nx; ++j) {
          double col[FU];
          for (int a = 0; a < nu; ++a) col[a] = Sux[a * nx + j];
          fchol_solve(nu, s->Lr, col);
          for (int a = 0; a < nu; ++a) s->K[a * nx + j] = -col[a];
        }
        double AP[FX * FX], Pn[FX * FX], Acl[FX * FX], Pin[FX * FX];
        for (int i = 0; i < nx; ++i)
          for (int j = 0; j < nx; ++j) {
            double t = 0; for (int q = 0; q < nx; ++q) t += s->A[q * nx + i] * Pm[q * nx + j];
            AP[i * nx + j] = t;
          }
        const int rk = frow(P, k);
        for (int i = 0; i < nx; ++i)
          for (int j = 0; j < nx; ++j) {
            double t = (i == j) ? s->H[i] : 0.0;
            if (rk) t += s->hsig * s->hg[i] * s->hg[j];   /* a path row's barrier: sigma c c' */
            for (int q = 0; q < nx; ++q) t += AP[i * nx + q] * s->A[q * nx + j];
            for (int a = 0; a < nu; ++a) t += Sux[a * nx + i] * s->K[a * nx + j];
            Pn[i * nx + j] = t;
          }
        for (int i = 0; i < nx; ++i)
          for (int j = 0; j < i; ++j) { const double t = 0.5 * (Pn[i * nx + j] + Pn[j * nx + i]); Pn[i * nx + j] = Pn[j * nx + i] = t; }
        for (int i = 0; i < nx; ++i)
          for (int j = 0; j < nx; ++j) {
            double t = s->A[i * nx + j];
            for (int a = 0; a < nu; ++a) t += s->B[i * nu + a] * s->K[a * nx + j];
            Acl[i * nx + j] = t;
          }
        for (int i = 0; i < nx; ++i)
          for (int j = 0; j < ne; ++j) {
            double t = 0; for (int q = 0; q < nx; ++q) t += Acl[q * nx + i] * Pi[q * ne + j];
            Pin[i * ne + j] = t;
          }
        memcpy(Pm, Pn, sizeof(Pm));
        memcpy(Pi, Pin, sizeof(Pi));
      }
    }
    for (int i = 0; i < nx; ++i) v[i] = s->Pe[i] + p[i];
    for (int a = 0; a < mk; ++a) {
      double t = s->g[uoff + a];
      for (int i = 0; i < nx; ++i) t += Bk[i * mk + a] * v[i];
      r[a] = t;
    }
    double kf[FZ];
    for (int a = 0; a < mk; ++a) kf[a] = r[a];
    fchol_solve(mk, s->Lr, kf);
    for (int a = 0; a < mk; ++a) kf[a] = -kf[a];
    if (k > 0) {
      for (int a = 0; a < nu; ++a) s->kf[a] = kf[a];
      double pn[FX];
      for (int i = 0; i < nx; ++i) {
        double t = s->g[i];
        for (int q = 0; q < nx; ++q) t += s->A[q * nx + i] * v[q];
        for (int a = 0; a < nu; ++a) t += s->K[a * nx + i] * r[a];
        pn[i] = t;
      }
      memcpy(p, pn, sizeof(p));
    } else {
      for (int a = 0; a < mk; ++a) s->d[a] = kf[a];
    }
    for (int j = 0; j < ne; ++j) {
      double t = 0; for (int a = 0; a < mk; ++a) t += s->Y[a * ne + j] * kf[a];
      lin[j] += t;
    }
  }
  /* nu = S^-1 (E d_N^0 - e_N) */
  if (ne > 0) {
    double Sc[FX * FX], rhsn[FX];
    memcpy(Sc, P->S, sizeof(double) * ne * ne);
    if (fchol(ne, Sc)) return -1;
    for (int j = 0; j < ne; ++j) rhsn[j] = lin[j] + P->lin_e[j] - rs * P->st[N].e0[j];
    fchol_solve(ne, Sc, rhsn);
    for (int j = 0; j < ne; ++j) nu_new[j] = rhsn[j];
  }
  /* forward pass */
  {
    fstage_t* s0 = &P->st[0];
    double w[FZ], dx[FX];
    for (int a = 0; a < m0; ++a) {
      double t = s0->d[a];
      for (int j = 0; j < ne; ++j) t -= s0->M[a * ne + j] * nu_new[j];
      w[a] = t;
    }
    for (int a = 0; a < m0; ++a) s0->d[a] = w[a];
    for (int i = 0; i < nx; ++i) {
      double t = rs * s0->e0[i];
      for (int a = 0; a < m0; ++a) t += s0->F0[i * m0 + a] * w[a];
      dx[i] = t;
    }
    for (int k = 1; k < N; ++k) {
      fstage_t* s = &P->st[k];
      double du[FU], dn[FX];
      for (int a = 0; a < nu; ++a) {
        double t = s->kf[a];
        for (int i = 0; i < nx; ++i) t += s->K[a * nx + i] * dx[i];
        for (int j = 0; j < ne; ++j) t -= s->M[a * ne + j] * nu_new[j];
        du[a] = t;
      }
      for (int i = 0; i < nx; ++i) s->d[i] = dx[i];
      for (int a = 0; a < nu; ++a) s->d[nx + a] = du[a];
      for (int i = 0; i < nx; ++i) {
        double t = rs * s->e0[i];
        for (int q = 0; q < nx; ++q) t += s->A[i * nx + q] * dx[q];
        for (int a = 0; a < nu; ++a) t += s->B[i * nu + a] * du[a];
        dn[i] = t;
      }
      memcpy(dx, dn, sizeof(dx));
    }
    for (int i = 0; i < nx; ++i) P->st[N].d[i] = dx[i];
  }
  return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* interior-point QP (qp_solve of vboc_oracle.c over the generalised stage variables)           */
/* ------------------------------------------------------------------------------------------ */

typedef struct { double n, d; } fratio_t;
static void fr_add(fratio_t* m, double t, double dt) {
  if (dt < 0.0 && t * m->d < m->n * (-dt)) { m->n = t; m->d = -dt; }
}

/* the row's c'd over stage k's step d (its state components; stage 0: the free ones) */
static double frow_dot(const fprob_t* P, int k, const double* d) {
  const fstage_t* s = &P->st[k];
  double t = 0.0;
  if (k == 0) {
    for (int j = 0; j < P->nf0; ++j) t += s->hg[P->f0[j]] * d[j];
    return t;
  }
  for (int i = 0; i < P->nx; ++i) t += s->hg[i] * d[i];
  return t;
}
/* the row's term c * v on the gradient of stage k's variables */
static void frow_addgrad(const fprob_t* P, int k, double* g, double v) {
  const fstage_t* s = &P->st[k];
  if (k == 0) {
    for (int j = 0; j < P->nf0; ++j) g[j] += s->hg[P->f0[j]] * v;
    return;
  }
  for (int i = 0; i < P->nx; ++i) g[i] += s->hg[i] * v;
}
/* complementarity targets of the row's pairs: the predictor's (smu = 0, zero affine directions) or Mehrotra's */
static void frow_rc(const fstage_t* s, double smu, double* rcl, double* rcu, double* rcs) {
  *rcl = smu - s->htl * s->hql - s->hatl * s->haql;
  *rcu = smu - s->htu * s->hqu - s->hatu * s->haqu;
  *rcs = smu - s->hs * s->hqs - s->has * s->haqs;
}
/* the row's gradient term gamma for the targets rc (pred: the predictor's form), and (pred) its factorisation
   weight sigma; a soft row also keeps its slack elimination b, W (header) */
static double frow_gamma(const fprob_t* P, fstage_t* s, double rs, double rcl, double rcu, double rcs, int pred) {
  const double rl = rs * s->hr0l, ru = rs * s->hr0u;
  double gam;
  if (pred) gam = s->hql * rl / s->htl - s->hqu * ru / s->htu;
  else gam = -s->hql + s->hqu - (rcl - s->hql * rl) / s->htl + (rcu - s->hqu * ru) / s->htu;
  if (P->soft) {
    const double Sl = s->hql / s->htl, Ss = s->hqs / s->hs, W = s->Zl + Sl + Ss;
    const double b = -(s->Zl * s->hs + s->zl - s->hql - s->hqs) + rcl / s->htl + rcs / s->hs - Sl * rl;
    s->hW = W;
    s->hb = b;
    gam += Sl * b / W;
    if (pred) s->hsig = s->hqu / s->htu + Sl * (s->Zl + Ss) / W;
  } else if (pred) {
    s->hsig = s->hql / s->htl + s->hqu / s->htu;
  }
  return gam;
}
/* Newton directions of the row's slacks / duals (and a soft row's slack / dual) from cd = c'd */
static void frow_dirs(const fprob_t* P, const fstage_t* s, double cd, double rs, double rcl, double rcu, double rcs,
                      double* dtl, double* dtu, double* dql, double* dqu, double* ds, double* dqs) {
  const double rl = rs * s->hr0l, ru = rs * s->hr0u;
  *ds = 0.0;
  *dqs = 0.0;
  if (P->soft) {
    *ds = (s->hb - s->hql / s->htl * cd) / s->hW;
    *dtl = cd + *ds + rl;
  } else {
    *dtl = cd + rl;
  }
  *dtu = ru - cd;
  *dql = (rcl - s->hql * *dtl) / s->htl;
  *dqu = (rcu - s->hqu * *dtu) / s->htu;
  if (P->soft) *dqs = (rcs - s->hqs * *ds) / s->hs;
}

static int fqp(fprob_t* P, int* iters) {
  const int nx = P->nx, nu = P->nu, ne = P->ne, N = P->N, m0 = P->nf0 + nu;
  const vboc_opts_t* o = &P->o;
  const double rho = o->lm;
  int nbox = 0;
  for (int k = 0; k <= N; ++k) {
    fstage_t* s = &P->st[k];
    for (int i = 0; i < fnz(P, k); ++i) {
      double v, lb, ub; int boxed;
      fcomp(P, k, i, &v, &lb, &ub, &boxed);
      if (!boxed) { s->dz[i] = 0.0; s->ql[i] = s->qu[i] = 0.0; s->Lb[i] = -INFINITY; s->Ub[i] = INFINITY; continue; }
      const double L = lb - v, U = ub - v, del = o->ipm_push * (U - L);
      double z0 = 0.0;
      if (z0 < L + del) z0 = L + del;
      if (z0 > U - del) z0 = U - del;
      s->Lb[i] = L; s->Ub[i] = U; s->dz[i] = z0;
      s->ql[i] = o->mu0 / (z0 - L);
      s->qu[i] = o->mu0 / (U - z0);
      nbox += 2;
    }
  }
  for (int j = 0; j < ne; ++j) P->qnu[j] = 0.0;
  for (int k = 0; k <= N; ++k) {
    /* the rows: slacks from the initial c'dz, clipped to ipm_push (infeasible start); a soft row's slack starts at
       the row's violation + ipm_push, so its lower side starts feasible */
    if (!frow(P, k)) continue;
    fstage_t* s = &P->st[k];
    const double gd = frow_dot(P, k, s->dz);
    s->hL = P->nn->lh - s->hv;
    s->hU = P->nn->uh - s->hv;
    double gs = gd;
    s->hs = s->hqs = s->has = s->haqs = 0.0;
    if (P->soft) {
      s->hs = fmax(s->hL - gd, 0.0) + o->ipm_push;
      s->hqs = o->mu0 / s->hs;
      gs = gd + s->hs;
      nbox += 1;
    }
    s->htl = fmax(gs - s->hL, o->ipm_push);
    s->htu = fmax(s->hU - gd, o->ipm_push);
    s->hql = o->mu0 / s->htl;
    s->hqu = o->mu0 / s->htu;
    s->hr0l = gs - s->hL - s->htl;
    s->hr0u = s->hU - gd - s->htu;
    s->hatl = s->hatu = s->haql = s->haqu = 0.0;
    nbox += 2;
  }
  double e00 = 0.0, rd0 = 0.0;
  for (int k = 0; k < N; ++k) {
    fstage_t* s = &P->st[k];
    const fstage_t* s1 = &P->st[k + 1];
    for (int i = 0; i < nx; ++i) {
      double t = s->b[i] - s1->dz[i];
      if (k == 0) for (int a = 0; a < m0; ++a) t += s->F0[i * m0 + a] * s->dz[a];
      else {
        for (int q = 0; q < nx; ++q) t += s->A[i * nx + q] * s->dz[q];
        for (int a = 0; a < nu; ++a) t += s->B[i * nu + a] * s->dz[nx + a];
      }
      s->e0[i] = t;
      e00 = fmax(e00, fabs(t));
    }
  }
  for (int j = 0; j < ne; ++j) {
    const double t = P->ev[j] - P->st[N].x[P->ei[j]] - P->st[N].dz[P->ei[j]];
    P->st[N].e0[j] = t;
    e00 = fmax(e00, fabs(t));
  }
  for (int k = 0; k <= N; ++k)
    if (frow(P, k)) e00 = fmax(e00, fmax(fabs(P->st[k].hr0l), fabs(P->st[k].hr0u)));
  for (int k = 0; k <= N; ++k) {
    const fstage_t* s = &P->st[k];
    const int rk = frow(P, k);
    for (int i = 0; i < fnz(P, k); ++i) {
      const int xi = k == 0 ? (i < P->nf0 ? P->f0[i] : -1) : (i < nx ? i : -1);
      rd0 = fmax(rd0, fabs((rho + fhq(P, k, i)) * s->dz[i] + fgrad(P, k, i) - s->ql[i] + s->qu[i] +
                           ((rk && xi >= 0) ? s->hg[xi] * (s->hqu - s->hql) : 0.0)));
    }
    if (rk && P->soft) rd0 = fmax(rd0, fabs(s->Zl * s->hs + s->zl - s->hql - s->hqs));
  }
  P->rs = 1.0;
  int it, status = 1;
  double nu_new[FX] = {0};
  for (it = 0; it < o->qp_max_iter; ++it) {
    double mu = 0.0;
    for (int k = 0; k <= N; ++k) {
      const fstage_t* s = &P->st[k];
      for (int i = 0; i < fnz(P, k); ++i) {
        if (!isfinite(s->Lb[i])) continue;
        mu += (s->dz[i] - s->Lb[i]) * s->ql[i] + (s->Ub[i] - s->dz[i]) * s->qu[i];
      }
    }
    for (int k = 0; k <= N; ++k) {
      if (!frow(P, k)) continue;
      const fstage_t* s = &P->st[k];
      mu += s->htl * s->hql + s->htu * s->hqu;
      if (P->soft) mu += s->hs * s->hqs;
    }
    mu /= (double)nbox;
    if (!isfinite(mu)) { status = -1; break; }
    if (mu < o->qp_tol_comp && P->rs * rd0 < o->qp_tol_stat && P->rs * e00 < o->qp_tol_eq) { status = 0; break; }
    for (int k = 0; k <= N; ++k) {
      fstage_t* s = &P->st[k];
      for (int i = 0; i < fnz(P, k); ++i) {
        const double hq = rho + fhq(P, k, i);
        double H = hq;
        const double g = hq * s->dz[i] + fgrad(P, k, i);
        if (isfinite(s->Lb[i])) H += s->ql[i] / (s->dz[i] - s->Lb[i]) + s->qu[i] / (s->Ub[i] - s->dz[i]);
        s->H[i] = H; s->g[i] = g;
      }
    }
    for (int k = 0; k <= N; ++k) {   /* the rows' predictor terms c gamma in the stage gradients */
      if (!frow(P, k)) continue;
      fstage_t* s = &P->st[k];
      s->hatl = s->hatu = s->haql = s->haqu = s->has = s->haqs = 0.0;
      double rcl, rcu, rcs;
      frow_rc(s, 0.0, &rcl, &rcu, &rcs);
      frow_addgrad(P, k, s->g, frow_gamma(P, s, P->rs, rcl, rcu, rcs, 1));
    }
    if (fnewton(P, 1, nu_new)) { status = -1; break; }
    fratio_t ma = {1.0, 1.0};
    for (int k = 0; k <= N; ++k) {
      fstage_t* s = &P->st[k];
      for (int i = 0; i < fnz(P, k); ++i) {
        s->daff[i] = s->d[i];
        if (!isfinite(s->Lb[i])) continue;
        const double tl = s->dz[i] - s->Lb[i], tu = s->Ub[i] - s->dz[i], d = s->d[i];
        const double dll = -s->ql[i] - s->ql[i] * d / tl, dlu = -s->qu[i] + s->qu[i] * d / tu;
        fr_add(&ma, tl, d);
        fr_add(&ma, tu, -d);
        fr_add(&ma, s->ql[i], dll);
        fr_add(&ma, s->qu[i], dlu);
      }
    }
    for (int k = 0; k <= N; ++k) {
      if (!frow(P, k)) continue;
      fstage_t* s = &P->st[k];
      double rcl, rcu, rcs, dtl, dtu, dql, dqu, ds, dqs;
      frow_rc(s, 0.0, &rcl, &rcu, &rcs);
      frow_dirs(P, s, frow_dot(P, k, s->d), P->rs, rcl, rcu, rcs, &dtl, &dtu, &dql, &dqu, &ds, &dqs);
      s->hatl = dtl; s->hatu = dtu; s->haql = dql; s->haqu = dqu; s->has = ds; s->haqs = dqs;
      fr_add(&ma, s->htl, dtl);
      fr_add(&ma, s->htu, dtu);
      fr_add(&ma, s->hql, dql);
      fr_add(&ma, s->hqu, dqu);
      if (P->soft) {
        fr_add(&ma, s->hs, ds);
        fr_add(&ma, s->hqs, dqs);
      }
    }
    const double aa = ma.n / ma.d;
    double muaff = 0.0;
    for (int k = 0; k <= N; ++k) {
      const fstage_t* s = &P->st[k];
      for (int i = 0; i < fnz(P, k); ++i) {
        if (!isfinite(s->Lb[i])) continue;
        const double tl = s->dz[i] - s->Lb[i], tu = s->Ub[i] - s->dz[i], d = s->d[i];
        const double dll = -s->ql[i] - s->ql[i] * d / tl, dlu = -s->qu[i] + s->qu[i] * d / tu;
        muaff += (tl + aa * d) * (s->ql[i] + aa * dll) + (tu - aa * d) * (s->qu[i] + aa * dlu);
      }
    }
    for (int k = 0; k <= N; ++k) {
      if (!frow(P, k)) continue;
      const fstage_t* s = &P->st[k];
      muaff += (s->htl + aa * s->hatl) * (s->hql + aa * s->haql) + (s->htu + aa * s->hatu) * (s->hqu + aa * s->haqu);
      if (P->soft) muaff += (s->hs + aa * s->has) * (s->hqs + aa * s->haqs);
    }
    muaff /= (double)nbox;
    double sig = muaff / mu;
    sig = sig * sig * sig;
    if (sig > 1.0) sig = 1.0;
    const double smu = sig * mu;
    for (int k = 0; k <= N; ++k) {
      fstage_t* s = &P->st[k];
      for (int i = 0; i < fnz(P, k); ++i) {
        if (!isfinite(s->Lb[i])) continue;
        const double tl = s->dz[i] - s->Lb[i], tu = s->Ub[i] - s->dz[i], itl = 1.0 / tl, itu = 1.0 / tu, d = s->daff[i];
        const double dll = -s->ql[i] - s->ql[i] * d * itl, dlu = -s->qu[i] + s->qu[i] * d * itu;
        const double rl = smu - tl * s->ql[i] - d * dll, ru = smu - tu * s->qu[i] + d * dlu;
        s->g[i] = (rho + fhq(P, k, i)) * s->dz[i] + fgrad(P, k, i) - s->ql[i] - rl * itl + s->qu[i] + ru * itu;
      }
    }
    for (int k = 0; k <= N; ++k) {   /* the rows' Mehrotra-corrected terms */
      if (!frow(P, k)) continue;
      fstage_t* s = &P->st[k];
      double rcl, rcu, rcs;
      frow_rc(s, smu, &rcl, &rcu, &rcs);
      frow_addgrad(P, k, s->g, frow_gamma(P, s, P->rs, rcl, rcu, rcs, 0));
    }
    if (fnewton(P, 0, nu_new)) { status = -1; break; }
    fratio_t mx = {1.0, o->ipm_tau};
    for (int k = 0; k <= N; ++k) {
      const fstage_t* s = &P->st[k];
      for (int i = 0; i < fnz(P, k); ++i) {
        if (!isfinite(s->Lb[i])) continue;
        const double tl = s->dz[i] - s->Lb[i], tu = s->Ub[i] - s->dz[i], itl = 1.0 / tl, itu = 1.0 / tu;
        const double d = s->d[i], da = s->daff[i];
        const double dlla = -s->ql[i] - s->ql[i] * da * itl, dlua = -s->qu[i] + s->qu[i] * da * itu;
        const double rl = smu - tl * s->ql[i] - da * dlla, ru = smu - tu * s->qu[i] + da * dlua;
        const double dll = (rl - s->ql[i] * d) * itl, dlu = (ru + s->qu[i] * d) * itu;
        fr_add(&mx, tl, d);
        fr_add(&mx, tu, -d);
        fr_add(&mx, s->ql[i], dll);
        fr_add(&mx, s->qu[i], dlu);
      }
    }
    for (int k = 0; k <= N; ++k) {
      if (!frow(P, k)) continue;
      fstage_t* s = &P->st[k];
      double rcl, rcu, rcs;
      frow_rc(s, smu, &rcl, &rcu, &rcs);
      frow_dirs(P, s, frow_dot(P, k, s->d), P->rs, rcl, rcu, rcs, &s->hdtl, &s->hdtu, &s->hdql, &s->hdqu, &s->hds,
                &s->hdqs);
      fr_add(&mx, s->htl, s->hdtl);
      fr_add(&mx, s->htu, s->hdtu);
      fr_add(&mx, s->hql, s->hdql);
      fr_add(&mx, s->hqu, s->hdqu);
      if (P->soft) {
        fr_add(&mx, s->hs, s->hds);
        fr_add(&mx, s->hqs, s->hdqs);
      }
    }
    const double alpha = fmin(1.0, o->ipm_tau * (mx.n / mx.d));
    for (int k = 0; k <= N; ++k) {
      fstage_t* s = &P->st[k];
      for (int i = 0; i < fnz(P, k); ++i) {
        const double d = s->d[i];
        if (isfinite(s->Lb[i])) {
          const double tl = s->dz[i] - s->Lb[i], tu = s->Ub[i] - s->dz[i], itl = 1.0 / tl, itu = 1.0 / tu, da = s->daff[i];
          const double dlla = -s->ql[i] - s->ql[i] * da * itl, dlua = -s->qu[i] + s->qu[i] * da * itu;
          const double rl = smu - tl * s->ql[i] - da * dlla, ru = smu - tu * s->qu[i] + da * dlua;
          s->ql[i] += alpha * (rl - s->ql[i] * d) * itl;
          s->qu[i] += alpha * (ru + s->qu[i] * d) * itu;
        }
        s->dz[i] += alpha * d;
      }
    }
    for (int k = 0; k <= N; ++k) {
      if (!frow(P, k)) continue;
      fstage_t* s = &P->st[k];
      s->htl += alpha * s->hdtl; s->htu += alpha * s->hdtu;
      s->hql += alpha * s->hdql; s->hqu += alpha * s->hdqu;
      if (P->soft) {
        s->hs += alpha * s->hds;
        s->hqs += alpha * s->hdqs;
      }
    }
    for (int j = 0; j < ne; ++j) P->qnu[j] += alpha * (nu_new[j] - P->qnu[j]);
    P->rs *= (1.0 - alpha);
  }
  *iters = it;
  if (status < 0) return -1;
  /* costates by the backward adjoint from the final iterate */
  {
    double lam[FX];
    const fstage_t* sN = &P->st[N];
    for (int i = 0; i < nx; ++i) {
      lam[i] = (rho + fhq(P, N, i)) * sN->dz[i] + fgrad(P, N, i) - sN->ql[i] + sN->qu[i];
      if (frow(P, N)) lam[i] += sN->hg[i] * (sN->hqu - sN->hql);
    }
    for (int j = 0; j < ne; ++j) lam[P->ei[j]] += P->qnu[j];
    for (int k = N - 1; k >= 0; --k) {
      fstage_t* s = &P->st[k];
      memcpy(s->qpi, lam, sizeof(lam));
      if (k == 0) break;
      double ln[FX];
      for (int i = 0; i < nx; ++i) {
        double t = (rho + fhq(P, k, i)) * s->dz[i] + fgrad(P, k, i) - s->ql[i] + s->qu[i];
        if (frow(P, k)) t += s->hg[i] * (s->hqu - s->hql);   /* a path row's term */
        for (int q = 0; q < nx; ++q) t += s->A[q * nx + i] * lam[q];
        ln[i] = t;
      }
      memcpy(lam, ln, sizeof(lam));
    }
  }
  for (int k = 0; k <= N; ++k)
    for (int i = 0; i < fnz(P, k); ++i)
      if (!isfinite(P->st[k].dz[i]) || !isfinite(P->st[k].ql[i]) || !isfinite(P->st[k].qu[i])) return -1;
  return status;
}

/* ------------------------------------------------------------------------------------------ */
/* SQP with L1 merit backtracking                                                              */
/* ------------------------------------------------------------------------------------------ */

/* x_k + alpha dx_k of the stage state (stage 0: only the free components move) */
static void fstate_at(const fprob_t* P, int k, double alpha, double* x, double* u) {
  const fstage_t* s = &P->st[k];
  const int nx = P->nx, nu = P->nu;
  if (k == 0) {
    for (int i = 0; i < nx; ++i) x[i] = s->x[i];
    for (int j = 0; j < P->nf0; ++j) x[P->f0[j]] += alpha * s->dz[j];
    for (int a = 0; a < nu; ++a) u[a] = s->u[a] + alpha * s->dz[P->nf0 + a];
    return;
  }
  for (int i = 0; i < nx; ++i) x[i] = s->x[i] + alpha * s->dz[i];
  if (k < P->N) for (int a = 0; a < nu; ++a) u[a] = s->u[a] + alpha * s->dz[nx + a];
}

static double fmerit(const fprob_t* P, double alpha) {
  const int nx = P->nx, N = P->N;
  double xk[FX], uk[FU], xn[FX], un[FU], phi[FX];
  double val = 0.0, viol = 0.0;
  for (int k = 0; k <= N; ++k) {
    const fstage_t* st = &P->st[k];
    for (int i = 0; i < fnz(P, k); ++i) {
      double v, lb, ub; int boxed;
      fcomp(P, k, i, &v, &lb, &ub, &boxed);
      if (!boxed) continue;
      v += alpha * st->dz[i];
      viol += fmax(0.0, lb - v) + fmax(0.0, v - ub);
    }
  }
  val += P->wbnd * viol;
  fstate_at(P, 0, alpha, xk, uk);
  if (P->track) val += ftrack(P, 0, xk, uk);
  else for (int i = 0; i < nx; ++i) val += P->c0[i] * xk[i];
  for (int k = 0; k < N; ++k) {
    ft_rk4(P->nq, xk, uk, phi);
    fstate_at(P, k + 1, alpha, xn, un);
    for (int i = 0; i < nx; ++i) val += P->st[k].wpi[i] * fabs(phi[i] - xn[i]);
    if (P->track) val += ftrack(P, k + 1, xn, un);
    else if (k + 1 < N) for (int i = 0; i < nx; ++i) val += P->cp[i] * xn[i];
    memcpy(xk, xn, sizeof(xk));
    memcpy(uk, un, sizeof(uk));
  }
  for (int j = 0; j < P->ne; ++j) val += P->wnu[j] * fabs(xk[P->ei[j]] - P->ev[j]);
  for (int k = 0; k <= N; ++k) {
    /* the rows' violations at the trial states, weighted like the boxes; a soft row's trial slack, its cost and
       its bound s >= 0 */
    if (!frow(P, k)) continue;
    const fstage_t* st = &P->st[k];
    fstate_at(P, k, alpha, xn, un);
    const double hv = nn_row(P->nn, P->nq, xn, NULL, P->soft, P->sm);
    const double sa = P->soft ? st->sl + alpha * (st->hs - st->sl) : 0.0;
    double v = fmax(0.0, P->nn->lh - hv - sa) + fmax(0.0, hv - P->nn->uh);
    if (P->soft) {
      v += fmax(0.0, -sa);
      val += st->zl * sa + 0.5 * st->Zl * sa * sa;
    }
    val += P->wbnd * v;
  }
  return val;
}

static double fwupd(double w, double lam) {
  const double a = fabs(lam), b = 0.5 * (w + a);
  return a > b ? a : b;
}

static void fsqp(fprob_t* P, vboc_result_t* res) {
  const int nx = P->nx, nu = P->nu, N = P->N;
  const vboc_opts_t* o = &P->o;
  int status = 2, it, qp_total = 0;
  double rstat = 0, req = 0, rineq = 0, rcomp = 0;
  for (it = 0;; ++it) {
    flinearize(P);
    fresiduals(P, &rstat, &req, &rineq, &rcomp);
    if (!isfinite(rstat) || !isfinite(req)) { status = 1; break; }
    if (P->rti && it == 1) { status = 0; break; }   /* SQP_RTI: one QP and its full step */
    if (!P->rti && rstat < o->tol_stat && req < o->tol_eq && rineq < o->tol_ineq && rcomp < o->tol_comp) {
      status = 0;
      break;
    }
    if (it >= o->max_iter) { status = 2; break; }
    int qit = 0;
    const int qs = fqp(P, &qit);
    qp_total += qit;
    if (qs < 0 || (P->qcf && qs == 1)) { status = 4; break; }
    double lmax = 0.0;
    for (int k = 0; k <= N; ++k) {
      fstage_t* s = &P->st[k];
      if (k < N) for (int i = 0; i < nx; ++i) s->wpi[i] = fwupd(s->wpi[i], s->qpi[i]);
      for (int i = 0; i < fnz(P, k); ++i) lmax = fmax(lmax, fmax(s->ql[i], s->qu[i]));
    }
    for (int k = 0; k <= N; ++k) {
      if (!frow(P, k)) continue;
      const fstage_t* s = &P->st[k];
      lmax = fmax(lmax, fmax(s->hql, s->hqu));
      if (P->soft) lmax = fmax(lmax, s->hqs);
    }
    for (int j = 0; j < P->ne; ++j) P->wnu[j] = fwupd(P->wnu[j], P->qnu[j]);
    P->wbnd = fwupd(P->wbnd, lmax);
    double alpha = 1.0;
    if (!P->rti) {
      const double phi0 = fmerit(P, 0.0);
      for (;;) {
        const double pa = fmerit(P, alpha);
        if (pa < phi0) break;
        if (alpha * o->alpha_reduction < o->alpha_min) break;
        alpha *= o->alpha_reduction;
      }
    }
    for (int k = 0; k <= N; ++k) {
      fstage_t* s = &P->st[k];
      double x[FX], u[FU];
      fstate_at(P, k, alpha, x, u);
      memcpy(s->x, x, sizeof(double) * nx);
      if (k < N) memcpy(s->u, u, sizeof(double) * nu);
      for (int i = 0; i < fnz(P, k); ++i) {
        s->ll[i] += alpha * (s->ql[i] - s->ll[i]);
        s->lu[i] += alpha * (s->qu[i] - s->lu[i]);
      }
      if (k < N) for (int i = 0; i < nx; ++i) s->pi[i] += alpha * (s->qpi[i] - s->pi[i]);
    }
    for (int j = 0; j < P->ne; ++j) P->tnu[j] += alpha * (P->qnu[j] - P->tnu[j]);
    for (int k = 0; k <= N; ++k) {
      if (!frow(P, k)) continue;
      fstage_t* s = &P->st[k];
      s->hll += alpha * (s->hql - s->hll);
      s->hlu += alpha * (s->hqu - s->hlu);
      if (P->soft) {
        s->sl += alpha * (s->hs - s->sl);
        s->lsl += alpha * (s->hqs - s->lsl);
      }
    }
    if (!isfinite(P->st[0].x[nx - 1])) { status = 1; break; }
  }
  res->status = status;
  res->sqp_iter = it;
  res->qp_iter = qp_total;
  res->cost = fcost(P);
  res->res_stat = rstat; res->res_eq = req; res->res_ineq = rineq; res->res_comp = rcomp;
}

/* ------------------------------------------------------------------------------------------ */
/* public entry points                                                                         */
/* ------------------------------------------------------------------------------------------ */

void vboc_oracle_ft_rk4_sens(int nq, const double* x, const double* u, double* x1, double* A, double* B) {
  ft_rk4_sens(nq, x, u, x1, A, B);
}

/* Layout as vboc_oracle_solve (nx = 2 nq + 1 with the dt column, p = [w_1..w_nq, w_t]). */
int vboc_oracle_ft_solve(int nq, int N, const double* x_guess, const double* u_guess, const double* p,
                         const double* lbx, const double* ubx, const double* lbu, const double* ubu,
                         const double* lbx0, const double* ubx0, const double* lbxe, const double* ubxe,
                         const vboc_opts_t* opts, double* x_out, double* u_out, vboc_result_t* res) {
  if (nq < 1 || nq > FQ || N < 1) return -1;
  const int nx = 2 * nq + 1, nu = nq;
  for (int i = 0; i < nx; ++i) if (!(lbx[i] < ubx[i]) || !(lbx0[i] <= ubx0[i]) || !(lbxe[i] <= ubxe[i])) return -2;
  for (int a = 0; a < nu; ++a) if (!(lbu[a] < ubu[a])) return -2;
  fprob_t P;
  memset(&P, 0, sizeof(P));
  P.nq = nq; P.nx = nx; P.nu = nu; P.N = N; P.o = *opts;
  for (int i = 0; i < nx; ++i) {
    P.xlb[i] = lbx[i]; P.xub[i] = ubx[i]; P.x0lb[i] = lbx0[i]; P.x0ub[i] = ubx0[i];
    P.xNlb[i] = lbxe[i]; P.xNub[i] = ubxe[i];
    if (lbx0[i] < ubx0[i]) P.f0[P.nf0++] = i;
    if (lbxe[i] == ubxe[i]) { P.xNfix[i] = 1; P.ei[P.ne] = i; P.ev[P.ne] = lbxe[i]; P.ne++; }
  }
  for (int a = 0; a < nu; ++a) { P.ulb[a] = lbu[a]; P.uub[a] = ubu[a]; }
  for (int j = 0; j < nq; ++j) P.c0[nq + j] = p[j];
  P.c0[2 * nq] = p[nq];
  P.cp[2 * nq] = p[nq];
  P.st = (fstage_t*)calloc((size_t)N + 1, sizeof(fstage_t));
  if (!P.st) return -3;
  for (int k = 0; k <= N; ++k) {
    for (int i = 0; i < nx; ++i) P.st[k].x[i] = x_guess[k * nx + i];
    if (k < N) for (int a = 0; a < nu; ++a) P.st[k].u[a] = u_guess[k * nu + a];
  }
  for (int i = 0; i < nx; ++i) if (!(lbx0[i] < ubx0[i])) P.st[0].x[i] = lbx0[i];   /* fixed at stage 0 */
  fsqp(&P, res);
  for (int k = 0; k <= N; ++k) {
    for (int i = 0; i < nx; ++i) x_out[k * nx + i] = P.st[k].x[i];
    if (k < N) for (int a = 0; a < nu; ++a) u_out[k * nu + a] = P.st[k].u[a];
  }
  free(P.st);
  return 0;
}

int vboc_oracle_ft_solve_batch(int nq, int B, int Nmax, const int* N, const double* x_guess,
                               const double* u_guess, const double* p, const double* lbx, const double* ubx,
                               const double* lbu, const double* ubu, const double* lbx0, const double* ubx0,
                               const double* lbxe, const double* ubxe, const vboc_opts_t* opts, int nthreads,
                               double* x_out, double* u_out, vboc_result_t* res) {
  const int nxr = 2 * nq + 1, npr = nq + 1;
  int err = 0;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads) reduction(| : err)
  for (int b = 0; b < B; ++b) {
    const size_t xo = (size_t)b * (Nmax + 1) * nxr, uo = (size_t)b * Nmax * nq;
    const int r = vboc_oracle_ft_solve(nq, N[b], x_guess + xo, u_guess + uo, p + (size_t)b * npr,
                                       lbx + (size_t)b * nxr, ubx + (size_t)b * nxr, lbu + (size_t)b * nq,
                                       ubu + (size_t)b * nq, lbx0 + (size_t)b * nxr, ubx0 + (size_t)b * nxr,
                                       lbxe + (size_t)b * nxr, ubxe + (size_t)b * nxr, opts, x_out + xo,
                                       u_out + uo, res + b);
    if (r == -2) { res[b].status = 5; res[b].sqp_iter = 0; res[b].qp_iter = 0; res[b].cost = NAN; }
    else if (r) err |= 1;
  }
  return err ? -1 : 0;
}

/* Safe-MPC OCP_solve (HardTerm, :163-181): x_0 fixed, boxes, tracking cost, terminal NN row, SQP or SQP_RTI.
   x [N + 1][2 nq] and u [N][nq] without the dt column; hrow (may be NULL) gets h(x_N) of the result.
   soft (SoftTraj, :242-304; NULL = HardTerm): the margin-scaled row on every stage, soft lower sides with the
   per-stage weights zl / Zl [N + 1]. */
static int mpc_impl(int nq, int N, double h, const double* x0, const double* x_guess, const double* u_guess,
                    const double* xlb, const double* xub, const double* ulb, const double* uub, const double* xNlb,
                    const double* xNub, const double* W, const double* We, const double* yref, const double* yref_e,
                    double cs, const vboc_mpc_nn_t* nn, const vboc_mpc_soft_t* soft, int rti, int qcf,
                    const vboc_opts_t* opts, double* x_out, double* u_out, vboc_result_t* res, double* hrow) {
  if (nq < 1 || nq > FQ || N < 1) return -1;
  const int n2 = 2 * nq, nx = n2 + 1, nu = nq;
  /* path boxes proper; a terminal component with lb == ub is a terminal equality (AL's zero final velocity) */
  for (int i = 0; i < n2; ++i) if (!(xlb[i] < xub[i]) || !(xNlb[i] <= xNub[i])) return -2;
  for (int a = 0; a < nu; ++a) if (!(ulb[a] < uub[a])) return -2;
  if (nn && !(nn->lh <= nn->uh)) return -2;
  fprob_t P;
  memset(&P, 0, sizeof(P));
  P.nq = nq; P.nx = nx; P.nu = nu; P.N = N; P.o = *opts;
  for (int i = 0; i < n2; ++i) {
    P.xlb[i] = xlb[i]; P.xub[i] = xub[i]; P.xNlb[i] = xNlb[i]; P.xNub[i] = xNub[i];
    P.x0lb[i] = P.x0ub[i] = x0[i];
  }
  P.xlb[n2] = P.xNlb[n2] = -INFINITY; P.xub[n2] = P.xNub[n2] = INFINITY;   /* dt: pinned by x_0 and the dynamics */
  P.x0lb[n2] = P.x0ub[n2] = h;
  for (int a = 0; a < nu; ++a) { P.ulb[a] = ulb[a]; P.uub[a] = uub[a]; }
  for (int i = 0; i < n2; ++i)
    if (xNlb[i] == xNub[i]) { P.xNfix[i] = 1; P.ei[P.ne] = i; P.ev[P.ne] = xNlb[i]; P.ne++; }
  P.track = 1; P.rti = rti; P.cs = cs; P.nn = nn; P.qcf = qcf;
  if (soft && !nn) return -2;
  if (soft) { P.soft = 1; P.sm = 100.0 - soft->margin; }
  for (int i = 0; i < n2; ++i) { P.wq[i] = W[i]; P.yr[i] = yref[i]; P.we[i] = We[i]; P.yre[i] = yref_e[i]; }
  for (int a = 0; a < nu; ++a) { P.wq[nx + a] = W[n2 + a]; P.yr[nx + a] = yref[n2 + a]; }
  P.st = (fstage_t*)calloc((size_t)N + 1, sizeof(fstage_t));
  if (!P.st) return -3;
  for (int k = 0; k <= N; ++k) {
    for (int i = 0; i < n2; ++i) P.st[k].x[i] = x_guess[k * n2 + i];
    P.st[k].x[n2] = h;
    if (k < N) for (int a = 0; a < nu; ++a) P.st[k].u[a] = u_guess[k * nu + a];
  }
  for (int i = 0; i < n2; ++i) P.st[0].x[i] = x0[i];
  if (soft)   /* the slack weights scaled like their stage's cost (ACADOS cost_scaling: cs on 0..N-1, 1 at N) */
    for (int k = 0; k <= N; ++k) {
      const double sc = k < N ? cs : 1.0;
      P.st[k].zl = soft->zl ? sc * soft->zl[k] : 0.0;
      P.st[k].Zl = soft->Zl ? sc * soft->Zl[k] : 0.0;
    }
  fsqp(&P, res);
  for (int k = 0; k <= N; ++k) {
    for (int i = 0; i < n2; ++i) x_out[k * n2 + i] = P.st[k].x[i];
    if (k < N) for (int a = 0; a < nu; ++a) u_out[k * nu + a] = P.st[k].u[a];
  }
  if (hrow) *hrow = nn ? nn_row(nn, nq, P.st[N].x, NULL, P.soft, P.sm) : 0.0;
  free(P.st);
  return 0;
}

int vboc_oracle_mpc_solve_soft(int nq, int N, double h, const double* x0, const double* x_guess,
                               const double* u_guess, const double* xlb, const double* xub, const double* ulb,
                               const double* uub, const double* xNlb, const double* xNub, const double* W,
                               const double* We, const double* yref, const double* yref_e, double cs,
                               const vboc_mpc_nn_t* nn, const vboc_mpc_soft_t* soft, int rti, const vboc_opts_t* opts,
                               double* x_out, double* u_out, vboc_result_t* res, double* hrow) {
  return mpc_impl(nq, N, h, x0, x_guess, u_guess, xlb, xub, ulb, uub, xNlb, xNub, W, We, yref, yref_e, cs, nn, soft,
                  rti, 0, opts, x_out, u_out, res, hrow);
}

int vboc_oracle_mpc_solve(int nq, int N, double h, const double* x0, const double* x_guess, const double* u_guess,
                          const double* xlb, const double* xub, const double* ulb, const double* uub,
                          const double* xNlb, const double* xNub, const double* W, const double* We,
                          const double* yref, const double* yref_e, double cs, const vboc_mpc_nn_t* nn, int rti,
                          const vboc_opts_t* opts, double* x_out, double* u_out, vboc_result_t* res, double* hrow) {
  return vboc_oracle_mpc_solve_soft(nq, N, h, x0, x_guess, u_guess, xlb, xub, ulb, uub, xNlb, xNub, W, We, yref,
                                    yref_e, cs, nn, NULL, rti, opts, x_out, u_out, res, hrow);
}

/* SoftTraj batch: per problem its stage weights W [B][3 nq] / We [B][2 nq] (the receding driver's cost_set(i, "W")
   per initial state) and its slack weights zl / Zl [B][N + 1] */
int vboc_oracle_mpc_soft_solve_batch(int nq, int B, int N, double h, const double* x0, const double* x_guess,
                                     const double* u_guess, const double* xlb, const double* xub, const double* ulb,
                                     const double* uub, const double* xNlb, const double* xNub, const double* W,
                                     const double* We, const double* yref, const double* yref_e, double cs,
                                     const vboc_mpc_nn_t* nn, double margin, const double* zl, const double* Zl,
                                     int rti, const vboc_opts_t* opts, int nthreads, double* x_out, double* u_out,
                                     vboc_result_t* res, double* hrow) {
  const int n2 = 2 * nq;
  int err = 0;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads) reduction(| : err)
  for (int b = 0; b < B; ++b) {
    const size_t xo = (size_t)b * (N + 1) * n2, uo = (size_t)b * N * nq;
    vboc_mpc_soft_t sf;
    sf.margin = margin;
    sf.zl = zl + (size_t)b * (N + 1);
    sf.Zl = Zl + (size_t)b * (N + 1);
    const int r = vboc_oracle_mpc_solve_soft(nq, N, h, x0 + (size_t)b * n2, x_guess + xo, u_guess + uo, xlb, xub,
                                             ulb, uub, xNlb, xNub, W + (size_t)b * 3 * nq, We + (size_t)b * n2, yref,
                                             yref_e, cs, nn, &sf, rti, opts, x_out + xo, u_out + uo, res + b,
                                             hrow ? hrow + b : NULL);
    if (r == -2) { res[b].status = 5; res[b].sqp_iter = 0; res[b].qp_iter = 0; res[b].cost = NAN; }
    else if (r) err |= 1;
  }
  return err ? -1 : 0;
}

/* the SoftTraj row h(x) = NN(z(x)) (100 - margin) / 100 - vn(x) at B states x [B][2 nq] (nn_decisionfunction_
   conservative, :284-304; the receding driver evaluates it on the previous solution, receiding_hard_constraints/
   3dof_sym.py:32-35); margin < 0: the unscaled HardTerm row */
void vboc_oracle_mpc_row(int nq, int B, const double* x, const vboc_mpc_nn_t* nn, double margin, double* out) {
  for (int b = 0; b < B; ++b) {
    double xx[FX] = {0};
    for (int i = 0; i < 2 * nq; ++i) xx[i] = x[(size_t)b * 2 * nq + i];
    out[b] = nn_row(nn, nq, xx, NULL, margin >= 0.0, 100.0 - margin);
  }
}

int vboc_oracle_mpc_solve_batch(int nq, int B, int N, double h, const double* x0, const double* x_guess,
                                const double* u_guess, const double* xlb, const double* xub, const double* ulb,
                                const double* uub, const double* xNlb, const double* xNub, const double* W,
                                const double* We, const double* yref, const double* yref_e, double cs,
                                const vboc_mpc_nn_t* nn, int rti, const vboc_opts_t* opts, int nthreads,
                                double* x_out, double* u_out, vboc_result_t* res, double* hrow) {
  const int n2 = 2 * nq;
  int err = 0;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads) reduction(| : err)
  for (int b = 0; b < B; ++b) {
    const size_t xo = (size_t)b * (N + 1) * n2, uo = (size_t)b * N * nq;
    const int r = vboc_oracle_mpc_solve(nq, N, h, x0 + (size_t)b * n2, x_guess + xo, u_guess + uo, xlb, xub, ulb,
                                        uub, xNlb, xNub, W, We, yref, yref_e, cs, nn, rti, opts, x_out + xo,
                                        u_out + uo, res + b, hrow ? hrow + b : NULL);
    if (r == -2) { res[b].status = 5; res[b].sqp_iter = 0; res[b].qp_iter = 0; res[b].cost = NAN; }
    else if (r) err |= 1;
  }
  return err ? -1 : 0;
}

/* Active learning's labelling OCP, OCPtriplependulumINIT.compute_problem(q0, v0) (AL/triplependulum_class_al.py:
   148-169; the OCP :82-144, terminal rest :204-222): the tracking OCP above with yref = 0, no row, ACADOS' default
   SQP_RTI (one QP at the reset point, its full step), x_0 = (q0, v0) fixed, every stage's guess (q0, 0) (:157-160),
   u = 0 and zero multipliers (reset, :150) - or, x_guess [B][N+1][2 nq] given, compute_problem_nnguess's stage guesses
   (:171-201); a QP stopped by qp_max_iter is a QP failure (qcf: the label is the QP's
   feasibility answer).  label[b] = 1 / 0 / 2 for status 0 / 4 / other (:164-169). */
int vboc_oracle_al_solve_batch(int nq, int B, int N, double h, const double* x0, const double* x_guess,
                               const double* xlb, const double* xub, const double* ulb, const double* uub,
                               const double* xNlb, const double* xNub, const double* W, const double* We, double cs,
                               const vboc_opts_t* opts, int nthreads, double* x_out, double* u_out, vboc_result_t* res,
                               int* label) {
  if (nq < 1 || nq > FQ || N < 1) return -1;
  const int n2 = 2 * nq;
  const double zero[3 * FQ] = {0};
  int err = 0;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads) reduction(| : err)
  for (int b = 0; b < B; ++b) {
    double* xg = (double*)malloc(sizeof(double) * ((size_t)(N + 1) * n2 + (size_t)N * nq));
    if (!xg) { err |= 1; continue; }
    double* ug = xg + (size_t)(N + 1) * n2;
    for (int k = 0; k <= N; ++k)
      for (int i = 0; i < n2; ++i)
        xg[k * n2 + i] = x_guess ? x_guess[((size_t)b * (N + 1) + k) * n2 + i] : (i < nq ? x0[(size_t)b * n2 + i] : 0.0);
    for (int e = 0; e < N * nq; ++e) ug[e] = 0.0;
    const size_t xo = (size_t)b * (N + 1) * n2, uo = (size_t)b * N * nq;
    const int r = mpc_impl(nq, N, h, x0 + (size_t)b * n2, xg, ug, xlb, xub, ulb, uub, xNlb, xNub, W, We, zero, zero, cs,
                           NULL, NULL, 1, 1, opts, x_out + xo, u_out + uo, res + b, NULL);
    free(xg);
    if (r == -2) { res[b].status = 5; res[b].sqp_iter = 0; res[b].qp_iter = 0; res[b].cost = NAN; }
    else if (r) err |= 1;
    label[b] = res[b].status == 0 ? 1 : (res[b].status == 4 ? 0 : 2);
  }
  return err ? -1 : 0;
}

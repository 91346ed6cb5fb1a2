/*
 * ORACLE - TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by or called from the product
 * path (vboc_amd/).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it,
 * and only as the checker / CPU baseline.
 *
 * Plain-C FP64 restatement of the VBOC boundary OCP solve, i.e. of what
 *   OCPtriplependulumINIT.OCP_solve  (VBOC/triplependulum_class_vboc.py:155-191)
 * asks ACADOS to do with the options of VBOC/triplependulum_class_vboc.py:129-141
 * (same for the double pendulum :160-172 / :183-219 and the pendulum test set
 * pendulum_testdata.py:29-48 with VBOC/pendulum_class_vboc.py:91-103):
 *
 *   SQP, exact Hessian with exact_hess_dyn = exact_hess_constr = 0  => QP Hessian = LM * I
 *   (levenberg_marquardt = 1e-5); MERIT_BACKTRACKING (alpha_reduction 0.3, alpha_min 1e-2);
 *   nlp tol_stat 1e-3 (tol_eq/ineq/comp: ACADOS defaults 1e-6); nlp max_iter 1000;
 *   QP = HPIPM-style Riccati primal-dual interior point (Mehrotra predictor-corrector),
 *   qp iter_max 100, qp tol_stat 1e-3, other QP tolerances the HPIPM defaults (1e-8);
 *   ERK4, one step per shooting interval.
 *
 * ACADOS / HPIPM / BLASFEO / CasADi are un-vendored, un-pinned third-party dependencies absent
 * from /root/reference and from this image, so this file restates their published algorithms;
 * solver-level parity with ACADOS itself is unpinned (see DESIGN.md section "Oracle").  The
 * dynamics ARE pinned: tests/golden/dynamics_*.npz hold f, df/d(x,u) and RK4 steps evaluated
 * from the reference's own f_expl expressions.
 *
 * Exact reformulations (documented in DESIGN.md, each with its reference line):
 *  - dt is a state with zero derivative pinned to dt_sym by the driver bounds at every stage
 *    (VBOC/triplependulum_vboc.py:98-103) => eliminated; RK4 with h = dt on the physics rhs
 *    equals RK4 with h = 1 on dt*f (triplependulum_class_vboc.py:47, tf = N :74-76).
 *  - stage 0: positions fixed by lbx_0 == ubx_0 (:180-181) and the general constraint
 *    (I - d d^T) theta_dot_0 = 0 with d = p[:n] (:174-178) => theta_dot_0 = s * d, decision s.
 *  - stage N: velocities fixed by lbx_e == ubx_e (q_fin, :183-184) => equality E x_N = v_fin,
 *    handled exactly in the Riccati recursion through its multiplier nu.
 */
#include <complex.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "vboc_oracle.h"
#ifdef VBOC_TRACE
#include <stdio.h>
#endif

/* capacities: up to 4 joints (pendulum 1, double 2, triple 3, UR5 arm 4) */
#define NQ 4
#define NX 8
#define NU 4
#define NZ 12

/* ------------------------------------------------------------------------------------------ */
/* model                                                                                       */
/* ------------------------------------------------------------------------------------------ */

typedef struct {
  int nq, nx, nu, chain, ur5;
  double g, mu[NQ], l[NQ], a[NQ][NQ];
  double pm, pd, pb; /* damped pendulum: mass, rod length, damping */
} model_t;

/* VBOC/pendulum_class_vboc.py:14-17 ; VBOC/doublependulum_class_vboc.py:14-18 ;
   VBOC/triplependulum_class_vboc.py:15-21 */
static void model_init(model_t* m, int nq) {
  memset(m, 0, sizeof(*m));
  m->nq = nq; m->nx = 2 * nq; m->nu = nq;
  m->g = 9.81;
  if (nq == 4) {                 /* UR5 arm, VBOC/UR5/ur5reduced_class_fixedveldir.py:20-45 */
    m->chain = 0; m->ur5 = 1;
    return;
  }
  if (nq == 1) {
    m->chain = 0; m->pm = 0.5; m->pd = 0.3; m->pb = 0.01;
    return;
  }
  m->chain = 1;
  double mass[NQ] = {0.4, 0.4, 0.4, 0.0};
  for (int j = 0; j < nq; ++j) m->l[j] = 0.8;
  for (int j = 0; j < nq; ++j) {
    m->mu[j] = 0.0;
    for (int i = j; i < nq; ++i) m->mu[j] += mass[i];
  }
  for (int j = 0; j < nq; ++j)
    for (int k = 0; k < nq; ++k) m->a[j][k] = m->mu[j > k ? j : k] * m->l[j] * m->l[k];
}

/* Cholesky of an SPD n x n row-major matrix (lower factor in place). */
static int chol(int n, double* A) {
  for (int j = 0; j < n; ++j) {
    double s = A[j * n + j];
    for (int k = 0; k < j; ++k) s -= A[j * n + k] * A[j * n + k];
    if (!(s > 0.0)) return -1;
    double d = sqrt(s);
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

static void chol_solve(int n, const double* L, double* b) {
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

/* ------------------------------------------------------------------------------------------ */
/* UR5 arm (nq = 4): rigid-body chain of VBOC/UR5/ur5reduced_class_fixedveldir.py:20-45, whose  */
/* f_expl = [qdot; ABA(q, qdot, u)] comes from urdf2casadi (un-vendored, unpinned).  Parameters  */
/* (joint tree transforms, merged body inertias) are generated from VBOC/UR5/ur5.urdf by         */
/* tools/gen_ur5_model.py.  The oracle solves M(q) acc = u - RNEA(q, qdot, 0) with M from RNEA   */
/* columns and differentiates RNEA by the complex step (Im f(x + i h) / h, h = 1e-30: exact to   */
/* rounding, independent of the GPU's dual-number JVPs).                                        */
/* ------------------------------------------------------------------------------------------ */
#include "../vboc_amd/csrc/ur5_params.h"

typedef double complex cplx;

static void c_cross(const cplx* a, const cplx* b, cplx* o) {
  cplx t0 = a[1] * b[2] - a[2] * b[1], t1 = a[2] * b[0] - a[0] * b[2], t2 = a[0] * b[1] - a[1] * b[0];
  o[0] = t0; o[1] = t1; o[2] = t2;
}

/* tau = RNEA(q, qd, qdd) in body coordinates; grav = 0 drops gravity (mass-matrix columns).
 * Joint i: child frame = joint frame (UR5_R, UR5_P in the parent body) rotated by Rz(q_i);
 * motion transform E = Rz(q)^T R^T, r = P:  X(w, v) = (E w, E (v - r x w)). */
static void ur5_rnea(const cplx* q, const cplx* qd, const cplx* qdd, int grav, cplx* tau) {
  cplx E[4][9], w[4][3], v[4][3], aw[4][3], av[4][3], fn[4][3], ff[4][3];
  cplx wp[3] = {0, 0, 0}, vp[3] = {0, 0, 0}, awp[3] = {0, 0, 0}, avp[3] = {0, 0, grav ? 9.81 : 0.0};
  for (int i = 0; i < 4; ++i) {
    const double* R = UR5_R + 9 * i;
    const double* P = UR5_P + 3 * i;
    cplx c = ccos(q[i]), s = csin(q[i]);
    /* E = Rz(q)^T R^T: row a of Rz^T = (c, s, 0), (-s, c, 0), (0, 0, 1); R^T[b][k] = R[k][b] */
    for (int k = 0; k < 3; ++k) {
      E[i][0 * 3 + k] = c * R[k * 3 + 0] + s * R[k * 3 + 1];
      E[i][1 * 3 + k] = -s * R[k * 3 + 0] + c * R[k * 3 + 1];
      E[i][2 * 3 + k] = R[k * 3 + 2];
    }
    cplx r[3] = {P[0], P[1], P[2]}, t[3], t2[3], ew[3], ev[3], eaw[3], eav[3];
    c_cross(r, wp, t);
    for (int a = 0; a < 3; ++a) t[a] = vp[a] - t[a];
    c_cross(r, awp, t2);
    for (int a = 0; a < 3; ++a) t2[a] = avp[a] - t2[a];
    for (int a = 0; a < 3; ++a) {
      ew[a] = E[i][a * 3] * wp[0] + E[i][a * 3 + 1] * wp[1] + E[i][a * 3 + 2] * wp[2];
      ev[a] = E[i][a * 3] * t[0] + E[i][a * 3 + 1] * t[1] + E[i][a * 3 + 2] * t[2];
      eaw[a] = E[i][a * 3] * awp[0] + E[i][a * 3 + 1] * awp[1] + E[i][a * 3 + 2] * awp[2];
      eav[a] = E[i][a * 3] * t2[0] + E[i][a * 3 + 1] * t2[1] + E[i][a * 3 + 2] * t2[2];
    }
    /* v_i = X v_p + z qd ; a_i = X a_p + z qdd + v_i x_m (z qd) */
    for (int a = 0; a < 3; ++a) { w[i][a] = ew[a]; v[i][a] = ev[a]; }
    w[i][2] += qd[i];
    cplx zq[3] = {0, 0, qd[i]}, cw[3], cv[3];
    c_cross(w[i], zq, cw);
    c_cross(v[i], zq, cv);
    for (int a = 0; a < 3; ++a) { aw[i][a] = eaw[a] + cw[a]; av[i][a] = eav[a] + cv[a]; }
    aw[i][2] += qdd[i];
    /* f_i = I a_i + v_i x_f (I v_i);  I (w, v) = (Io w + mc x v, m v - mc x w) */
    const double* Io = UR5_IO + 9 * i;
    const double m = UR5_M[i];
    cplx mc[3] = {UR5_MC[3 * i], UR5_MC[3 * i + 1], UR5_MC[3 * i + 2]};
    cplx hA[3], hL[3], iaA[3], iaL[3], x1[3], x2[3];
    c_cross(mc, v[i], x1);
    c_cross(mc, w[i], x2);
    for (int a = 0; a < 3; ++a) {
      hA[a] = Io[a * 3] * w[i][0] + Io[a * 3 + 1] * w[i][1] + Io[a * 3 + 2] * w[i][2] + x1[a];
      hL[a] = m * v[i][a] - x2[a];
    }
    c_cross(mc, av[i], x1);
    c_cross(mc, aw[i], x2);
    for (int a = 0; a < 3; ++a) {
      iaA[a] = Io[a * 3] * aw[i][0] + Io[a * 3 + 1] * aw[i][1] + Io[a * 3 + 2] * aw[i][2] + x1[a];
      iaL[a] = m * av[i][a] - x2[a];
    }
    cplx y1[3], y2[3], y3[3];
    c_cross(w[i], hA, y1);
    c_cross(v[i], hL, y2);
    c_cross(w[i], hL, y3);
    for (int a = 0; a < 3; ++a) { fn[i][a] = iaA[a] + y1[a] + y2[a]; ff[i][a] = iaL[a] + y3[a]; }
    for (int a = 0; a < 3; ++a) { wp[a] = w[i][a]; vp[a] = v[i][a]; awp[a] = aw[i][a]; avp[a] = av[i][a]; }
  }
  /* backward: tau_i = z . n_i ; f_{i-1} += X_i^T f_i = (E^T n + r x E^T f, E^T f) */
  for (int i = 3; i >= 0; --i) {
    tau[i] = fn[i][2];
    if (i == 0) break;
    const double* P = UR5_P + 3 * i;
    cplx r[3] = {P[0], P[1], P[2]}, en[3], ef[3], x[3];
    for (int a = 0; a < 3; ++a) {
      en[a] = E[i][a] * fn[i][0] + E[i][3 + a] * fn[i][1] + E[i][6 + a] * fn[i][2];
      ef[a] = E[i][a] * ff[i][0] + E[i][3 + a] * ff[i][1] + E[i][6 + a] * ff[i][2];
    }
    c_cross(r, ef, x);
    for (int a = 0; a < 3; ++a) { fn[i - 1][a] += en[a] + x[a]; ff[i - 1][a] += ef[a]; }
  }
}

static void ur5_eval(const double* th, const double* om, const double* u, double* acc, double* Jth,
                     double* Jom, double* Ju) {
  cplx q[4], qd[4], qdd[4], tau[4];
  double M[16], L[16];
  for (int j = 0; j < 4; ++j) { q[j] = th[j]; qd[j] = om[j]; qdd[j] = 0.0; }
  /* M e_c = RNEA(q, 0, e_c) without gravity */
  cplx z4[4] = {0, 0, 0, 0};
  for (int c = 0; c < 4; ++c) {
    for (int j = 0; j < 4; ++j) qdd[j] = (j == c) ? 1.0 : 0.0;
    ur5_rnea(q, z4, qdd, 0, tau);
    for (int j = 0; j < 4; ++j) M[j * 4 + c] = creal(tau[j]);
  }
  for (int j = 0; j < 4; ++j) qdd[j] = 0.0;
  ur5_rnea(q, qd, qdd, 1, tau);
  for (int j = 0; j < 4; ++j) acc[j] = u[j] - creal(tau[j]);
  memcpy(L, M, sizeof(M));
  chol(4, L);
  chol_solve(4, L, acc);
  if (!Jth) return;
  const double hs = 1e-30;
  double col[4];
  for (int j = 0; j < 4; ++j) qdd[j] = acc[j];
  for (int c = 0; c < 8; ++c) {
    cplx qq[4], qv[4];
    for (int j = 0; j < 4; ++j) { qq[j] = th[j]; qv[j] = om[j]; }
    if (c < 4) qq[c] += I * hs; else qv[c - 4] += I * hs;
    ur5_rnea(qq, qv, qdd, 1, tau);
    for (int j = 0; j < 4; ++j) col[j] = -cimag(tau[j]) / hs;   /* d acc = -M^-1 d RNEA|acc */
    chol_solve(4, L, col);
    double* J = (c < 4) ? Jth : Jom;
    for (int j = 0; j < 4; ++j) J[j * 4 + (c & 3)] = col[j];
  }
  for (int c = 0; c < 4; ++c) {
    for (int j = 0; j < 4; ++j) col[j] = (j == c) ? 1.0 : 0.0;
    chol_solve(4, L, col);
    for (int j = 0; j < 4; ++j) Ju[j * 4 + c] = col[j];
  }
}

/* Accelerations and their Jacobians.  Point-mass chain (mass m_i at the tip of massless link
 * l_i, absolute angles from the downward vertical, generalised forces = C_i):
 *   M(th) acc = u - cor(th, om) - grav(th),   M_jk = a_jk cos(th_j - th_k),
 *   cor_j = sum_k a_jk sin(th_j - th_k) om_k^2,  grav_j = g mu_j l_j sin th_j.
 * This is the same function as f_expl of VBOC/doublependulum_class_vboc.py:40-91 and
 * VBOC/triplependulum_class_vboc.py:47-58 (pinned by tests/golden/dynamics_{2,3}.npz).
 * Pendulum: acc = (m g d sin th + F - b om) / (d^2 m)  (VBOC/pendulum_class_vboc.py:35-39). */
static void model_eval(const model_t* m, const double* th, const double* om, const double* u,
                       double* acc, double* Jth, double* Jom, double* Ju) {
  const int n = m->nq;
  if (m->ur5) {
    ur5_eval(th, om, u, acc, Jth, Jom, Ju);
    return;
  }
  if (!m->chain) {
    double inv = 1.0 / (m->pd * m->pd * m->pm);
    acc[0] = (m->pm * m->g * m->pd * sin(th[0]) + u[0] - m->pb * om[0]) * inv;
    if (Jth) {
      Jth[0] = m->pm * m->g * m->pd * cos(th[0]) * inv;
      Jom[0] = -m->pb * inv;
      Ju[0] = inv;
    }
    return;
  }
  double M[NQ * NQ], S[NQ][NQ], C[NQ][NQ], r[NQ];
  for (int j = 0; j < n; ++j)
    for (int k = 0; k < n; ++k) {
      S[j][k] = sin(th[j] - th[k]);
      C[j][k] = cos(th[j] - th[k]);
      M[j * n + k] = m->a[j][k] * C[j][k];
    }
  for (int j = 0; j < n; ++j) {
    double cor = 0.0;
    for (int k = 0; k < n; ++k) cor += m->a[j][k] * S[j][k] * om[k] * om[k];
    r[j] = u[j] - cor - m->g * m->mu[j] * m->l[j] * sin(th[j]);
  }
  chol(n, M);
  for (int j = 0; j < n; ++j) acc[j] = r[j];
  chol_solve(n, M, acc);
  if (!Jth) return;
  /* D = d r / d th - (dM/dth) acc ; Com = d(-cor)/d om */
  double D[NQ][NQ], Co[NQ][NQ];
  for (int j = 0; j < n; ++j) {
    double diag = 0.0;
    for (int k = 0; k < n; ++k) {
      if (k == j) continue;
      D[j][k] = m->a[j][k] * (C[j][k] * om[k] * om[k] - S[j][k] * acc[k]);
      diag += m->a[j][k] * (C[j][k] * om[k] * om[k] - S[j][k] * acc[k]);
    }
    D[j][j] = -diag - m->g * m->mu[j] * m->l[j] * cos(th[j]);
    for (int k = 0; k < n; ++k) Co[j][k] = -2.0 * m->a[j][k] * S[j][k] * om[k];
  }
  double col[NQ];
  for (int c = 0; c < n; ++c) {
    for (int j = 0; j < n; ++j) col[j] = D[j][c];
    chol_solve(n, M, col);
    for (int j = 0; j < n; ++j) Jth[j * n + c] = col[j];
    for (int j = 0; j < n; ++j) col[j] = Co[j][c];
    chol_solve(n, M, col);
    for (int j = 0; j < n; ++j) Jom[j * n + c] = col[j];
    for (int j = 0; j < n; ++j) col[j] = (j == c) ? 1.0 : 0.0;
    chol_solve(n, M, col);
    for (int j = 0; j < n; ++j) Ju[j * n + c] = col[j];
  }
}

/* ------------------------------------------------------------------------------------------ */
/* ERK4 (one step per shooting interval), with forward sensitivities = the exact derivative of */
/* the discrete map (ACADOS ERK forward VDE, num_stages 4, num_steps 1).                       */
/* ------------------------------------------------------------------------------------------ */

static void rhs(const model_t* m, const double* x, const double* u, double* k) {
  const int n = m->nq;
  for (int j = 0; j < n; ++j) k[j] = x[n + j];
  model_eval(m, x, x + n, u, k + n, NULL, NULL, NULL);
}

static void rk4(const model_t* m, double h, const double* x, const double* u, double* x1) {
  const int nx = m->nx;
  double k1[NX], k2[NX], k3[NX], k4[NX], X[NX] = {0};
  rhs(m, x, u, k1);
  for (int i = 0; i < nx; ++i) X[i] = x[i] + 0.5 * h * k1[i];
  rhs(m, X, u, k2);
  for (int i = 0; i < nx; ++i) X[i] = x[i] + 0.5 * h * k2[i];
  rhs(m, X, u, k3);
  for (int i = 0; i < nx; ++i) X[i] = x[i] + h * k3[i];
  rhs(m, X, u, k4);
  for (int i = 0; i < nx; ++i) x1[i] = x[i] + h / 6.0 * (k1[i] + 2.0 * k2[i] + 2.0 * k3[i] + k4[i]);
}

/* k = f(X,u), dk = df/dx(X) * SX + df/du(X) * [0 I]  (SX: nx x (nx+nu)) */
static void rhs_sens(const model_t* m, const double* X, const double* SX, const double* u,
                     double* k, double* dk) {
  const int n = m->nq, nx = m->nx, nz = nx + m->nu;
  double Jth[NQ * NQ], Jom[NQ * NQ], Ju[NQ * NQ];
  for (int j = 0; j < n; ++j) k[j] = X[n + j];
  model_eval(m, X, X + n, u, k + n, Jth, Jom, Ju);
  for (int j = 0; j < n; ++j)
    for (int c = 0; c < nz; ++c) dk[j * nz + c] = SX[(n + j) * nz + c];
  for (int j = 0; j < n; ++j)
    for (int c = 0; c < nz; ++c) {
      double t = (c >= nx) ? Ju[j * n + (c - nx)] : 0.0;
      for (int q = 0; q < n; ++q) t += Jth[j * n + q] * SX[q * nz + c] + Jom[j * n + q] * SX[(n + q) * nz + c];
      dk[(n + j) * nz + c] = t;
    }
}

static void rk4_sens(const model_t* m, double h, const double* x, const double* u, double* x1,
                     double* A, double* B) {
  const int nx = m->nx, nu = m->nu, nz = nx + nu;
  double S0[NX * NZ], S[NX * NZ], X[NX] = {0}, k[NX], dk[NX * NZ], ksum[NX], dsum[NX * NZ];
  memset(S0, 0, sizeof(S0));
  for (int i = 0; i < nx; ++i) S0[i * nz + i] = 1.0;
  /* stage 1 */
  rhs_sens(m, x, S0, u, k, dk);
  for (int i = 0; i < nx; ++i) ksum[i] = k[i];
  for (int i = 0; i < nx * nz; ++i) dsum[i] = dk[i];
  for (int i = 0; i < nx; ++i) X[i] = x[i] + 0.5 * h * k[i];
  for (int i = 0; i < nx * nz; ++i) S[i] = S0[i] + 0.5 * h * dk[i];
  /* stage 2 */
  rhs_sens(m, X, S, u, k, dk);
  for (int i = 0; i < nx; ++i) ksum[i] += 2.0 * k[i];
  for (int i = 0; i < nx * nz; ++i) dsum[i] += 2.0 * dk[i];
  for (int i = 0; i < nx; ++i) X[i] = x[i] + 0.5 * h * k[i];
  for (int i = 0; i < nx * nz; ++i) S[i] = S0[i] + 0.5 * h * dk[i];
  /* stage 3 */
  rhs_sens(m, X, S, u, k, dk);
  for (int i = 0; i < nx; ++i) ksum[i] += 2.0 * k[i];
  for (int i = 0; i < nx * nz; ++i) dsum[i] += 2.0 * dk[i];
  for (int i = 0; i < nx; ++i) X[i] = x[i] + h * k[i];
  for (int i = 0; i < nx * nz; ++i) S[i] = S0[i] + h * dk[i];
  /* stage 4 */
  rhs_sens(m, X, S, u, k, dk);
  for (int i = 0; i < nx; ++i) ksum[i] += k[i];
  for (int i = 0; i < nx * nz; ++i) dsum[i] += dk[i];
  for (int i = 0; i < nx; ++i) x1[i] = x[i] + h / 6.0 * ksum[i];
  for (int i = 0; i < nx; ++i)
    for (int c = 0; c < nz; ++c) {
      double v = S0[i * nz + c] + h / 6.0 * dsum[i * nz + c];
      if (c < nx) A[i * nx + c] = v; else B[i * nu + (c - nx)] = v;
    }
}

/* ------------------------------------------------------------------------------------------ */
/* problem / stage storage                                                                     */
/* ------------------------------------------------------------------------------------------ */

typedef struct {
  /* SQP iterate and NLP multipliers */
  double x[NX], u[NU];
  double pi[NX];               /* multiplier of x_{k+1} = phi_k(x_k,u_k), k = 0..N-1 */
  double ll[NZ], lu[NZ];       /* bound multipliers, stage layout z_k */
  double wpi[NX];              /* merit weights */
  /* linearisation */
  double A[NX * NX], B[NX * NU], F0[NX * (NU + 1)], b[NX];
  /* QP / IPM */
  double Lb[NZ], Ub[NZ];       /* box in step space */
  double dz[NZ], ql[NZ], qu[NZ];
  double e0[NX];               /* initial residual of the step dynamics */
  double H[NZ], g[NZ];
  double d[NZ], daff[NZ];
  double K[NU * NX], kf[NU], Lr[(NU + 1) * (NU + 1)], M[(NU + 1) * NQ], Y[(NU + 1) * NQ], Pe[NX];
  double qpi[NX];              /* QP costate (recovered) */
  /* Cartesian path constraint lh <= h(x_k) <= uh (stages 1..N-1, see hc_on) */
  double hv, hg[NQ];           /* h(x_k) and dh/dtheta at the iterate */
  double hll, hlu;             /* NLP multipliers */
  double hL, hU;               /* bounds of c'dz in step space */
  double htl, htu, hql, hqu;   /* QP slacks and their duals */
  double hr0l, hr0u;           /* slack residuals at the QP start (current = rs * r0) */
  double hatl, hatu, haql, haqu;  /* affine (predictor) directions of slacks and duals */
} stage_t;

typedef struct {
  model_t m;
  int N;
  double h;
  /* stage 0 parametrisation x0 = [q0 ; s d] */
  double q0[NQ], dir[NQ], s, slb, sub, cs, cost_const;
  double xlb[NX], xub[NX], ulb[NU], uub[NU];   /* path bounds */
  double qNlb[NQ], qNub[NQ], vfin[NQ];          /* terminal: position box, velocity target */
  double nu[NQ], wnu[NQ], wbnd;                 /* terminal multiplier, merit weights */
  double qnu[NQ];
  stage_t* st;                                  /* N+1 stages */
  vboc_opts_t o;
  /* QP bookkeeping */
  double S[NQ * NQ], lin_e[NQ];
  double rs;                                    /* residual scale prod(1 - alpha) */
  int hc;                                       /* Cartesian path constraint on (opts.hc) */
} prob_t;

/* number of step variables of stage k and their kind */
static int nz_of(const prob_t* P, int k) {
  if (k == 0) return 1 + P->m.nu;
  if (k == P->N) return P->m.nx;
  return P->m.nx + P->m.nu;
}

/* current value, bounds and "boxed" flag of component i of stage k */
static void comp(const prob_t* P, int k, int i, double* val, double* lb, double* ub, int* boxed) {
  const stage_t* s = &P->st[k];
  const int nx = P->m.nx, nq = P->m.nq;
  if (k == 0) {
    if (i == 0) { *val = P->s; *lb = P->slb; *ub = P->sub; }
    else { *val = s->u[i - 1]; *lb = P->ulb[i - 1]; *ub = P->uub[i - 1]; }
    *boxed = 1;
    return;
  }
  if (k == P->N) {
    *val = s->x[i];
    if (i < nq) { *lb = P->qNlb[i]; *ub = P->qNub[i]; *boxed = 1; }
    else { *lb = -INFINITY; *ub = INFINITY; *boxed = 0; }
    return;
  }
  if (i < nx) { *val = s->x[i]; *lb = P->xlb[i]; *ub = P->xub[i]; }
  else { *val = s->u[i - nx]; *lb = P->ulb[i - nx]; *ub = P->uub[i - nx]; }
  *boxed = 1;
}

static double cost_grad(const prob_t* P, int k, int i) { return (k == 0 && i == 0) ? P->cs : 0.0; }

/* Cartesian path constraint of VBOC/Cartesian constraints/doublependulum_class_fixedveldir.py:154-160:
 *   h(x) = (sum_j l_j sin th_j - x_c)^2 + (sum_j l_j cos th_j - y_c)^2,  lh <= h(x_k) <= uh
 * on the path stages (ACADOS con_h_expr).  Stage 0's positions are fixed, so there h is a constant:
 * it is checked once before the solve (vboc_oracle_solve), and the QP carries the constraint on
 * stages 1..N-1 as a general row c'dz in [lh - h, uh - h] with c = dh/dtheta (exact_hess_constr = 0:
 * no constraint curvature in the Hessian) and slack variables (HPIPM's general-constraint form). */
static int hc_on(const prob_t* P, int k) { return P->hc && k >= 1 && k < P->N; }
static double hc_eval(const prob_t* P, const double* x, double* grad) {
  const int nq = P->m.nq;
  double X = 0.0, Y = 0.0;
  for (int j = 0; j < nq; ++j) { X += P->m.l[j] * sin(x[j]); Y += P->m.l[j] * cos(x[j]); }
  const double dx = X - P->o.hc_xc, dy = Y - P->o.hc_yc;
  if (grad)
    for (int j = 0; j < nq; ++j) grad[j] = 2.0 * dx * (P->m.l[j] * cos(x[j])) - 2.0 * dy * (P->m.l[j] * sin(x[j]));
  return dx * dx + dy * dy;
}
static double hc_dot(const prob_t* P, const stage_t* s, const double* d) {
  double t = 0.0;
  for (int j = 0; j < P->m.nq; ++j) t += s->hg[j] * d[j];
  return t;
}

static void set_x0(prob_t* P) {
  const int nq = P->m.nq;
  for (int j = 0; j < nq; ++j) { P->st[0].x[j] = P->q0[j]; P->st[0].x[nq + j] = P->s * P->dir[j]; }
}

/* ------------------------------------------------------------------------------------------ */
/* linearisation + NLP residuals                                                               */
/* ------------------------------------------------------------------------------------------ */

static void linearize(prob_t* P) {
  const int nx = P->m.nx, nu = P->m.nu, nq = P->m.nq;
  set_x0(P);
  for (int k = 0; k < P->N; ++k) {
    stage_t* s = &P->st[k];
    double phi[NX];
    rk4_sens(&P->m, P->h, s->x, s->u, phi, s->A, s->B);
    for (int i = 0; i < nx; ++i) s->b[i] = phi[i] - P->st[k + 1].x[i];
    if (hc_on(P, k)) s->hv = hc_eval(P, s->x, s->hg);
  }
  /* F0 = [A0 g, B0], g = [0; dir] */
  stage_t* s0 = &P->st[0];
  for (int i = 0; i < nx; ++i) {
    double t = 0.0;
    for (int j = 0; j < nq; ++j) t += s0->A[i * nx + nq + j] * P->dir[j];
    s0->F0[i * (nu + 1)] = t;
    for (int j = 0; j < nu; ++j) s0->F0[i * (nu + 1) + 1 + j] = s0->B[i * nu + j];
  }
}

static void nlp_residuals(const prob_t* P, double* rstat, double* req, double* rineq, double* rcomp) {
  const int nx = P->m.nx, nu = P->m.nu, nq = P->m.nq, N = P->N;
  double st = 0, eq = 0, in = 0, cp = 0;
  for (int k = 0; k < N; ++k)
    for (int i = 0; i < nx; ++i) eq = fmax(eq, fabs(P->st[k].b[i]));
  for (int j = 0; j < nq; ++j) eq = fmax(eq, fabs(P->st[N].x[nq + j] - P->vfin[j]));
  for (int k = 0; k <= N; ++k) {
    const stage_t* s = &P->st[k];
    const int nz = nz_of(P, k);
    for (int i = 0; i < nz; ++i) {
      double v, lb, ub; int boxed;
      comp(P, k, i, &v, &lb, &ub, &boxed);
      double gr = cost_grad(P, k, i) - s->ll[i] + s->lu[i];
      if (k == 0) {
        const double* F = s->F0;
        for (int r = 0; r < nx; ++r) gr += F[r * (nu + 1) + i] * s->pi[r];
      } else if (k < N) {
        if (i < nx) {
          for (int r = 0; r < nx; ++r) gr += s->A[r * nx + i] * s->pi[r];
          gr -= P->st[k - 1].pi[i];
          if (hc_on(P, k) && i < nq) gr += s->hg[i] * (s->hlu - s->hll);
        } else {
          for (int r = 0; r < nx; ++r) gr += s->B[r * nu + (i - nx)] * s->pi[r];
        }
      } else {
        gr -= P->st[N - 1].pi[i];
        if (i >= nq) gr += P->nu[i - nq];
      }
      st = fmax(st, fabs(gr));
      if (boxed) {
        in = fmax(in, fmax(lb - v, v - ub));
        cp = fmax(cp, fmax(fabs(s->ll[i] * (v - lb)), fabs(s->lu[i] * (ub - v))));
      }
    }
    if (hc_on(P, k)) {
      in = fmax(in, fmax(P->o.hc_lh - s->hv, s->hv - P->o.hc_uh));
      cp = fmax(cp, fmax(fabs(s->hll * (s->hv - P->o.hc_lh)), fabs(s->hlu * (P->o.hc_uh - s->hv))));
    }
  }
  *rstat = st; *req = eq; *rineq = in; *rcomp = cp;
}

/* ------------------------------------------------------------------------------------------ */
/* Riccati solve of the Newton system                                                          */
/*   min sum 1/2 d'H d + g'd  s.t.  d_{k+1} = A d_x + B d_u + rs*e0_k,  E d_N = rs*e0_N        */
/* factor = 1: backward factorisation + vector pass; factor = 0: vector pass reusing factors.  */
/* ------------------------------------------------------------------------------------------ */

static int newton_solve(prob_t* P, int factor, double* nu_new) {
  const int nx = P->m.nx, nu = P->m.nu, nq = P->m.nq, N = P->N, m0 = nu + 1;
  const double rs = P->rs;
  double Pm[NX * NX], p[NX], Pi[NX * NQ], lin[NQ];
  stage_t* sN = &P->st[N];
  memset(Pm, 0, sizeof(Pm));
  for (int i = 0; i < nx; ++i) { Pm[i * nx + i] = sN->H[i]; p[i] = sN->g[i]; }
  memset(Pi, 0, sizeof(Pi));
  for (int j = 0; j < nq; ++j) Pi[(nq + j) * nq + j] = 1.0;
  memset(lin, 0, sizeof(lin));
  if (factor) { memset(P->S, 0, sizeof(P->S)); memset(P->lin_e, 0, sizeof(P->lin_e)); }

  for (int k = N - 1; k >= 0; --k) {
    stage_t* s = &P->st[k];
    const int mk = (k == 0) ? m0 : nu;          /* "control" block size */
    const double* Bk = (k == 0) ? s->F0 : s->B; /* nx x mk */
    double e[NX], v[NX], r[NU + 1];
    for (int i = 0; i < nx; ++i) e[i] = rs * s->e0[i];
    if (factor) {
      /* Pe = P e ; lin_e += Pi' e */
      for (int i = 0; i < nx; ++i) {
        double t = 0; for (int j = 0; j < nx; ++j) t += Pm[i * nx + j] * e[j];
        s->Pe[i] = t;
      }
      for (int j = 0; j < nq; ++j) {
        double t = 0; for (int i = 0; i < nx; ++i) t += Pi[i * nq + j] * e[i];
        P->lin_e[j] += t;
      }
      /* BP = Bk' P  (mk x nx) */
      double BP[(NU + 1) * NX], Ru[(NU + 1) * (NU + 1)];
      for (int a = 0; a < mk; ++a)
        for (int j = 0; j < nx; ++j) {
          double t = 0; for (int i = 0; i < nx; ++i) t += Bk[i * mk + a] * Pm[i * nx + j];
          BP[a * nx + j] = t;
        }
      const int uoff = (k == 0) ? 0 : nx; /* offset of the control block in z_k */
      for (int a = 0; a < mk; ++a)
        for (int c = 0; c < mk; ++c) {
          double t = (a == c) ? s->H[uoff + a] : 0.0;
          for (int i = 0; i < nx; ++i) t += BP[a * nx + i] * Bk[i * mk + c];
          Ru[a * mk + c] = t;
        }
      for (int a = 0; a < mk; ++a)
        for (int c = 0; c < a; ++c) { double t = 0.5 * (Ru[a * mk + c] + Ru[c * mk + a]); Ru[a * mk + c] = Ru[c * mk + a] = t; }
      if (chol(mk, Ru)) return -1;
      memcpy(s->Lr, Ru, sizeof(double) * mk * mk);
      /* Y = Bk' Pi (mk x nq) ; M = Ru^-1 Y ; S += Y' M */
      for (int a = 0; a < mk; ++a)
        for (int j = 0; j < nq; ++j) {
          double t = 0; for (int i = 0; i < nx; ++i) t += Bk[i * mk + a] * Pi[i * nq + j];
          s->Y[a * nq + j] = t;
        }
      for (int j = 0; j < nq; ++j) {
        double col[NU + 1];
        for (int a = 0; a < mk; ++a) col[a] = s->Y[a * nq + j];
        chol_solve(mk, s->Lr, col);
        for (int a = 0; a < mk; ++a) s->M[a * nq + j] = col[a];
      }
      for (int i = 0; i < nq; ++i)
        for (int j = 0; j < nq; ++j) {
          double t = 0; for (int a = 0; a < mk; ++a) t += s->Y[a * nq + i] * s->M[a * nq + j];
          P->S[i * nq + j] += t;
        }
      if (k > 0) {
        /* Sux = BP A (nu x nx) ; K = -Ru^-1 Sux */
        double Sux[NU * NX];
        for (int a = 0; a < nu; ++a)
          for (int j = 0; j < nx; ++j) {
            double t = 0; for (int i = 0; i < nx; ++i) t += BP[a * nx + i] * s->A[i * nx + j];
            Sux[a * nx + j] = t;
          }
        for (int j = 0; j < nx; ++j) {
          double col[NU];
          for (int a = 0; a < nu; ++a) col[a] = Sux[a * nx + j];
          chol_solve(nu, s->Lr, col);
          for (int a = 0; a < nu; ++a) s->K[a * nx + j] = -col[a];
        }
        /* Pnew = diag(Hx) + A' P A + Sux' K ; Pi_new = (A + B K)' Pi */
        double AP[NX * NX], Pn[NX * NX], Acl[NX * NX], Pin[NX * NQ];
        for (int i = 0; i < nx; ++i)
          for (int j = 0; j < nx; ++j) {
            double t = 0; for (int q = 0; q < nx; ++q) t += s->A[q * nx + i] * Pm[q * nx + j];
            AP[i * nx + j] = t;
          }
        for (int i = 0; i < nx; ++i)
          for (int j = 0; j < nx; ++j) {
            double t = (i == j) ? s->H[i] : 0.0;
            if (hc_on(P, k) && i < nq && j < nq) t += (s->hql / s->htl + s->hqu / s->htu) * s->hg[i] * s->hg[j];
            for (int q = 0; q < nx; ++q) t += AP[i * nx + q] * s->A[q * nx + j];
            for (int a = 0; a < nu; ++a) t += Sux[a * nx + i] * s->K[a * nx + j];
            Pn[i * nx + j] = t;
          }
        for (int i = 0; i < nx; ++i)
          for (int j = 0; j < i; ++j) { double t = 0.5 * (Pn[i * nx + j] + Pn[j * nx + i]); Pn[i * nx + j] = Pn[j * nx + i] = t; }
        for (int i = 0; i < nx; ++i)
          for (int j = 0; j < nx; ++j) {
            double t = s->A[i * nx + j];
            for (int a = 0; a < nu; ++a) t += s->B[i * nu + a] * s->K[a * nx + j];
            Acl[i * nx + j] = t;
          }
        for (int i = 0; i < nx; ++i)
          for (int j = 0; j < nq; ++j) {
            double t = 0; for (int q = 0; q < nx; ++q) t += Acl[q * nx + i] * Pi[q * nq + j];
            Pin[i * nq + j] = t;
          }
        /* vector part needs the OLD P (through Pe) - computed below from s->Pe */
        memcpy(Pm, Pn, sizeof(Pm));
        memcpy(Pi, Pin, sizeof(Pi));
      }
    }
    /* vector pass: v = P_{k+1} e + p_{k+1} ; r = g_u + Bk' v ; kf = -Ru^-1 r */
    for (int i = 0; i < nx; ++i) v[i] = s->Pe[i] + p[i];
    const int uoff = (k == 0) ? 0 : nx;
    for (int a = 0; a < mk; ++a) {
      double t = s->g[uoff + a];
      for (int i = 0; i < nx; ++i) t += Bk[i * mk + a] * v[i];
      r[a] = t;
    }
    double kf[NU + 1];
    for (int a = 0; a < mk; ++a) kf[a] = r[a];
    chol_solve(mk, s->Lr, kf);
    for (int a = 0; a < mk; ++a) kf[a] = -kf[a];
    if (k > 0) {
      for (int a = 0; a < nu; ++a) s->kf[a] = kf[a];
      /* p = g_x + A' v + K' r */
      double pn[NX];
      for (int i = 0; i < nx; ++i) {
        double t = s->g[i];
        for (int q = 0; q < nx; ++q) t += s->A[q * nx + i] * v[q];
        for (int a = 0; a < nu; ++a) t += s->K[a * nx + i] * r[a];
        pn[i] = t;
      }
      memcpy(p, pn, sizeof(p));
    } else {
      /* w0^0 kept in d (forward pass adds the nu part) */
      for (int a = 0; a < mk; ++a) s->d[a] = kf[a];
    }
    for (int j = 0; j < nq; ++j) {
      double t = 0; for (int a = 0; a < mk; ++a) t += s->Y[a * nq + j] * kf[a];
      lin[j] += t;
    }
  }
  /* nu = S^-1 (E d_N^0 - e_N) */
  double Sc[NQ * NQ], rhsn[NQ];
  memcpy(Sc, P->S, sizeof(Sc));
  if (chol(nq, Sc)) return -1;
  for (int j = 0; j < nq; ++j) rhsn[j] = lin[j] + P->lin_e[j] - rs * P->st[N].e0[j];
  chol_solve(nq, Sc, rhsn);
  for (int j = 0; j < nq; ++j) nu_new[j] = rhsn[j];

  /* forward pass */
  {
    stage_t* s0 = &P->st[0];
    double w[NU + 1], dx[NX];
    for (int a = 0; a < m0; ++a) {
      double t = s0->d[a];
      for (int j = 0; j < nq; ++j) t -= s0->M[a * nq + j] * nu_new[j];
      w[a] = t;
    }
    for (int a = 0; a < m0; ++a) s0->d[a] = w[a];
    for (int i = 0; i < nx; ++i) {
      double t = rs * s0->e0[i];
      for (int a = 0; a < m0; ++a) t += s0->F0[i * m0 + a] * w[a];
      dx[i] = t;
    }
    for (int k = 1; k < N; ++k) {
      stage_t* s = &P->st[k];
      double du[NU], dn[NX];
      for (int a = 0; a < nu; ++a) {
        double t = s->kf[a];
        for (int i = 0; i < nx; ++i) t += s->K[a * nx + i] * dx[i];
        for (int j = 0; j < nq; ++j) t -= s->M[a * nq + j] * nu_new[j];
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
/* interior-point QP                                                                           */
/* ------------------------------------------------------------------------------------------ */

/* fraction-to-boundary ratio test: running minimum of t / (-dt) over dt < 0, kept as n / d so
   that only the winning ratio is divided (the GPU kernel uses the same comparison) */
typedef struct { double n, d; } minratio_t;
static void mr_add(minratio_t* m, double t, double dt) {
  if (dt < 0.0 && t * m->d < m->n * (-dt)) { m->n = t; m->d = -dt; }
}

/* returns 0 converged, 1 max-iter (usable step), -1 failure */
/* Newton directions of the path constraint's slacks and duals from the step d of stage s (smu = 0 and
   zero affine directions give the predictor's) */
static void hc_dir(const prob_t* P, const stage_t* s, double smu, double* dtl, double* dtu, double* dql,
                   double* dqu) {
  const double cd = hc_dot(P, s, s->d), rl = P->rs * s->hr0l, ru = P->rs * s->hr0u;
  const double rcl = smu - s->htl * s->hql - s->hatl * s->haql, rcu = smu - s->htu * s->hqu - s->hatu * s->haqu;
  *dtl = cd + rl;
  *dtu = ru - cd;
  *dql = (rcl - s->hql * *dtl) / s->htl;
  *dqu = (rcu - s->hqu * *dtu) / s->htu;
}

static int qp_solve(prob_t* P, int* iters) {
  const int nx = P->m.nx, nu = P->m.nu, nq = P->m.nq, N = P->N;
  const vboc_opts_t* o = &P->o;
  const double rho = o->lm;
  int nbox = 0;
  /* init: box in step space, interior start, duals mu0 / t */
  for (int k = 0; k <= N; ++k) {
    stage_t* s = &P->st[k];
    const int nz = nz_of(P, k);
    for (int i = 0; i < nz; ++i) {
      double v, lb, ub; int boxed;
      comp(P, k, i, &v, &lb, &ub, &boxed);
      if (!boxed) { s->dz[i] = 0.0; s->ql[i] = s->qu[i] = 0.0; s->Lb[i] = -INFINITY; s->Ub[i] = INFINITY; continue; }
      double L = lb - v, U = ub - v, del = o->ipm_push * (U - L);
      double z0 = 0.0;
      if (z0 < L + del) z0 = L + del;
      if (z0 > U - del) z0 = U - del;
      s->Lb[i] = L; s->Ub[i] = U; s->dz[i] = z0;
      s->ql[i] = o->mu0 / (z0 - L);
      s->qu[i] = o->mu0 / (U - z0);
      nbox += 2;
    }
  }
  for (int j = 0; j < nq; ++j) P->qnu[j] = 0.0;
  /* path constraint rows: slacks from the initial c'dz, clipped to ipm_push (infeasible start,
     the residual r0 is driven out like the dynamics residual) */
  for (int k = 1; k < N; ++k) {
    if (!hc_on(P, k)) continue;
    stage_t* s = &P->st[k];
    const double gd = hc_dot(P, s, s->dz);
    s->hL = o->hc_lh - s->hv;
    s->hU = o->hc_uh - s->hv;
    s->htl = fmax(gd - s->hL, o->ipm_push);
    s->htu = fmax(s->hU - gd, o->ipm_push);
    s->hql = o->mu0 / s->htl;
    s->hqu = o->mu0 / s->htu;
    s->hr0l = gd - s->hL - s->htl;
    s->hr0u = s->hU - gd - s->htu;
    s->hatl = s->hatu = s->haql = s->haqu = 0.0;
    nbox += 2;
  }
  /* initial residuals: dynamics e0, terminal e0_N (stored in st[N].e0[0..nq)) */
  double e00 = 0.0, rd0 = 0.0;
  for (int k = 0; k < N; ++k) {
    stage_t* s = &P->st[k];
    stage_t* s1 = &P->st[k + 1];
    for (int i = 0; i < nx; ++i) {
      double t = s->b[i] - s1->dz[i];
      if (k == 0) for (int a = 0; a <= nu; ++a) t += s->F0[i * (nu + 1) + a] * s->dz[a];
      else {
        for (int q = 0; q < nx; ++q) t += s->A[i * nx + q] * s->dz[q];
        for (int a = 0; a < nu; ++a) t += s->B[i * nu + a] * s->dz[nx + a];
      }
      s->e0[i] = t;
      e00 = fmax(e00, fabs(t));
    }
  }
  for (int j = 0; j < nq; ++j) {
    double t = P->vfin[j] - P->st[N].x[nq + j] - P->st[N].dz[nq + j];
    P->st[N].e0[j] = t;
    e00 = fmax(e00, fabs(t));
  }
  for (int k = 0; k <= N; ++k) {
    const stage_t* s = &P->st[k];
    const int hk = hc_on(P, k);
    if (hk) e00 = fmax(e00, fmax(fabs(s->hr0l), fabs(s->hr0u)));
    for (int i = 0; i < nz_of(P, k); ++i)
      rd0 = fmax(rd0, fabs(rho * s->dz[i] + cost_grad(P, k, i) - s->ql[i] + s->qu[i] +
                           ((hk && i < nq) ? s->hg[i] * (s->hqu - s->hql) : 0.0)));
  }
  P->rs = 1.0;
  int it, status = 1;
  double nu_new[NQ];
  for (it = 0; it < o->qp_max_iter; ++it) {
    /* complementarity measure */
    double mu = 0.0;
    for (int k = 0; k <= N; ++k) {
      const stage_t* s = &P->st[k];
      for (int i = 0; i < nz_of(P, k); ++i) {
        if (!isfinite(s->Lb[i])) continue;
        mu += (s->dz[i] - s->Lb[i]) * s->ql[i] + (s->Ub[i] - s->dz[i]) * s->qu[i];
      }
      if (hc_on(P, k)) mu += s->htl * s->hql + s->htu * s->hqu;
    }
    mu /= (double)nbox;
    if (!isfinite(mu)) { status = -1; break; }
    if (mu < o->qp_tol_comp && P->rs * rd0 < o->qp_tol_stat && P->rs * e00 < o->qp_tol_eq) { status = 0; break; }
    /* predictor */
    for (int k = 0; k <= N; ++k) {
      stage_t* s = &P->st[k];
      for (int i = 0; i < nz_of(P, k); ++i) {
        double H = rho, g = rho * s->dz[i] + cost_grad(P, k, i);
        if (isfinite(s->Lb[i])) {
          double tl = s->dz[i] - s->Lb[i], tu = s->Ub[i] - s->dz[i], itl = 1.0 / tl, itu = 1.0 / tu;
          H += s->ql[i] * itl + s->qu[i] * itu;
        }
        s->H[i] = H; s->g[i] = g;
      }
      if (hc_on(P, k)) {
        s->hatl = s->hatu = s->haql = s->haqu = 0.0;
        const double gam = s->hql * (P->rs * s->hr0l) / s->htl - s->hqu * (P->rs * s->hr0u) / s->htu;
        for (int j = 0; j < nq; ++j) s->g[j] += s->hg[j] * gam;
      }
    }
    if (newton_solve(P, 1, nu_new)) { status = -1; break; }
    minratio_t ma = {1.0, 1.0};
    for (int k = 0; k <= N; ++k) {
      stage_t* s = &P->st[k];
      for (int i = 0; i < nz_of(P, k); ++i) {
        s->daff[i] = s->d[i];
        if (!isfinite(s->Lb[i])) continue;
        double tl = s->dz[i] - s->Lb[i], tu = s->Ub[i] - s->dz[i], itl = 1.0 / tl, itu = 1.0 / tu, d = s->d[i];
        double dll = -s->ql[i] - s->ql[i] * d * itl, dlu = -s->qu[i] + s->qu[i] * d * itu;
        mr_add(&ma, tl, d);
        mr_add(&ma, tu, -d);
        mr_add(&ma, s->ql[i], dll);
        mr_add(&ma, s->qu[i], dlu);
      }
      if (hc_on(P, k)) {
        double dtl, dtu, dql, dqu;
        hc_dir(P, s, 0.0, &dtl, &dtu, &dql, &dqu);
        s->hatl = dtl; s->hatu = dtu; s->haql = dql; s->haqu = dqu;
        mr_add(&ma, s->htl, dtl);
        mr_add(&ma, s->htu, dtu);
        mr_add(&ma, s->hql, dql);
        mr_add(&ma, s->hqu, dqu);
      }
    }
    const double aa = ma.n / ma.d;
    double muaff = 0.0;
    for (int k = 0; k <= N; ++k) {
      stage_t* s = &P->st[k];
      for (int i = 0; i < nz_of(P, k); ++i) {
        if (!isfinite(s->Lb[i])) continue;
        double tl = s->dz[i] - s->Lb[i], tu = s->Ub[i] - s->dz[i], itl = 1.0 / tl, itu = 1.0 / tu, d = s->d[i];
        double dll = -s->ql[i] - s->ql[i] * d * itl, dlu = -s->qu[i] + s->qu[i] * d * itu;
        muaff += (tl + aa * d) * (s->ql[i] + aa * dll) + (tu - aa * d) * (s->qu[i] + aa * dlu);
      }
      if (hc_on(P, k))
        muaff += (s->htl + aa * s->hatl) * (s->hql + aa * s->haql) + (s->htu + aa * s->hatu) * (s->hqu + aa * s->haqu);
    }
    muaff /= (double)nbox;
    double sig = muaff / mu;
    sig = sig * sig * sig;
    if (sig > 1.0) sig = 1.0;
    const double smu = sig * mu;
    /* corrector */
    for (int k = 0; k <= N; ++k) {
      stage_t* s = &P->st[k];
      for (int i = 0; i < nz_of(P, k); ++i) {
        if (!isfinite(s->Lb[i])) continue;
        double tl = s->dz[i] - s->Lb[i], tu = s->Ub[i] - s->dz[i], itl = 1.0 / tl, itu = 1.0 / tu, d = s->daff[i];
        double dll = -s->ql[i] - s->ql[i] * d * itl, dlu = -s->qu[i] + s->qu[i] * d * itu;
        double rl = smu - tl * s->ql[i] - d * dll;
        double ru = smu - tu * s->qu[i] + d * dlu;
        s->g[i] = rho * s->dz[i] + cost_grad(P, k, i) - s->ql[i] - rl * itl + s->qu[i] + ru * itu;
      }
      if (hc_on(P, k)) {
        const double rl = P->rs * s->hr0l, ru = P->rs * s->hr0u;
        const double rcl = smu - s->htl * s->hql - s->hatl * s->haql, rcu = smu - s->htu * s->hqu - s->hatu * s->haqu;
        const double gam = -s->hql + s->hqu - (rcl - s->hql * rl) / s->htl + (rcu - s->hqu * ru) / s->htu;
        for (int j = 0; j < nq; ++j) s->g[j] += s->hg[j] * gam;
      }
    }
    if (newton_solve(P, 0, nu_new)) { status = -1; break; }
    minratio_t mx = {1.0, o->ipm_tau};
    for (int k = 0; k <= N; ++k) {
      stage_t* s = &P->st[k];
      for (int i = 0; i < nz_of(P, k); ++i) {
        if (!isfinite(s->Lb[i])) continue;
        double tl = s->dz[i] - s->Lb[i], tu = s->Ub[i] - s->dz[i], itl = 1.0 / tl, itu = 1.0 / tu, d = s->d[i], da = s->daff[i];
        double dlla = -s->ql[i] - s->ql[i] * da * itl, dlua = -s->qu[i] + s->qu[i] * da * itu;
        double rl = smu - tl * s->ql[i] - da * dlla;
        double ru = smu - tu * s->qu[i] + da * dlua;
        double dll = (rl - s->ql[i] * d) * itl, dlu = (ru + s->qu[i] * d) * itu;
        mr_add(&mx, tl, d);
        mr_add(&mx, tu, -d);
        mr_add(&mx, s->ql[i], dll);
        mr_add(&mx, s->qu[i], dlu);
      }
      if (hc_on(P, k)) {
        double dtl, dtu, dql, dqu;
        hc_dir(P, s, smu, &dtl, &dtu, &dql, &dqu);
        mr_add(&mx, s->htl, dtl);
        mr_add(&mx, s->htu, dtu);
        mr_add(&mx, s->hql, dql);
        mr_add(&mx, s->hqu, dqu);
      }
    }
    const double amax = mx.n / mx.d;
    double alpha = fmin(1.0, o->ipm_tau * amax);
    for (int k = 0; k <= N; ++k) {
      stage_t* s = &P->st[k];
      for (int i = 0; i < nz_of(P, k); ++i) {
        double d = s->d[i];
        if (isfinite(s->Lb[i])) {
          double tl = s->dz[i] - s->Lb[i], tu = s->Ub[i] - s->dz[i], itl = 1.0 / tl, itu = 1.0 / tu, da = s->daff[i];
          double dlla = -s->ql[i] - s->ql[i] * da * itl, dlua = -s->qu[i] + s->qu[i] * da * itu;
          double rl = smu - tl * s->ql[i] - da * dlla;
          double ru = smu - tu * s->qu[i] + da * dlua;
          double dll = (rl - s->ql[i] * d) * itl, dlu = (ru + s->qu[i] * d) * itu;
          s->ql[i] += alpha * dll;
          s->qu[i] += alpha * dlu;
        }
        s->dz[i] += alpha * d;
      }
      if (hc_on(P, k)) {
        double dtl, dtu, dql, dqu;
        hc_dir(P, s, smu, &dtl, &dtu, &dql, &dqu);
        s->htl += alpha * dtl; s->htu += alpha * dtu;
        s->hql += alpha * dql; s->hqu += alpha * dqu;
      }
    }
    for (int j = 0; j < nq; ++j) P->qnu[j] += alpha * (nu_new[j] - P->qnu[j]);
    P->rs *= (1.0 - alpha);
  }
  *iters = it;
  if (status < 0) return -1;
  /* costate recovery from the final iterate: pi_{N-1} = H_N-part ..., backward adjoint */
  {
    double lam[NX];
    stage_t* sN = &P->st[N];
    for (int i = 0; i < nx; ++i) {
      double t = rho * sN->dz[i] - sN->ql[i] + sN->qu[i];
      if (i >= nq) t += P->qnu[i - nq];
      lam[i] = t;
    }
    for (int k = N - 1; k >= 0; --k) {
      stage_t* s = &P->st[k];
      memcpy(s->qpi, lam, sizeof(lam));
      if (k == 0) break;
      double ln[NX];
      for (int i = 0; i < nx; ++i) {
        double t = rho * s->dz[i] - s->ql[i] + s->qu[i];
        if (hc_on(P, k) && i < nq) t += s->hg[i] * (s->hqu - s->hql);
        for (int q = 0; q < nx; ++q) t += s->A[q * nx + i] * lam[q];
        ln[i] = t;
      }
      memcpy(lam, ln, sizeof(lam));
    }
  }
  for (int k = 0; k <= N; ++k)
    for (int i = 0; i < nz_of(P, k); ++i)
      if (!isfinite(P->st[k].dz[i]) || !isfinite(P->st[k].ql[i]) || !isfinite(P->st[k].qu[i])) return -1;
  return status;
}

/* ------------------------------------------------------------------------------------------ */
/* SQP with L1 merit backtracking                                                              */
/* ------------------------------------------------------------------------------------------ */

/* merit at z + alpha dz ; defects re-simulated */
static double merit(const prob_t* P, double alpha) {
  const int nx = P->m.nx, nu = P->m.nu, nq = P->m.nq, N = P->N;
  double xk[NX], uk[NX], xn[NX], phi[NX];
  double s = P->s + alpha * P->st[0].dz[0];
  double val = P->cs * s + P->cost_const;
  double viol = 0.0;
  for (int k = 0; k <= N; ++k) {
    const stage_t* st = &P->st[k];
    for (int i = 0; i < nz_of(P, k); ++i) {
      double v, lb, ub; int boxed;
      comp(P, k, i, &v, &lb, &ub, &boxed);
      if (!boxed) continue;
      v += alpha * st->dz[i];
      viol += fmax(0.0, lb - v) + fmax(0.0, v - ub);
    }
  }
  val += P->wbnd * viol;
  for (int j = 0; j < nq; ++j) { xk[j] = P->q0[j]; xk[nq + j] = s * P->dir[j]; }
  for (int a = 0; a < nu; ++a) uk[a] = P->st[0].u[a] + alpha * P->st[0].dz[1 + a];
  for (int k = 0; k < N; ++k) {
    const stage_t* s1 = &P->st[k + 1];
    rk4(&P->m, P->h, xk, uk, phi);
    for (int i = 0; i < nx; ++i) xn[i] = s1->x[i] + alpha * s1->dz[i];
    for (int i = 0; i < nx; ++i) val += P->st[k].wpi[i] * fabs(phi[i] - xn[i]);
    if (hc_on(P, k + 1)) {
      const double hv = hc_eval(P, xn, NULL);
      val += P->wbnd * (fmax(0.0, P->o.hc_lh - hv) + fmax(0.0, hv - P->o.hc_uh));
    }
    memcpy(xk, xn, sizeof(xk));
    if (k + 1 < N) for (int a = 0; a < nu; ++a) uk[a] = s1->u[a] + alpha * s1->dz[nx + a];
  }
  for (int j = 0; j < nq; ++j) val += P->wnu[j] * fabs(xk[nq + j] - P->vfin[j]);
  return val;
}

static double wupd(double w, double lam) {
  double a = fabs(lam);
  double b = 0.5 * (w + a);
  return a > b ? a : b;
}

static void sqp(prob_t* P, vboc_result_t* res) {
  const int nx = P->m.nx, nu = P->m.nu, nq = P->m.nq, N = P->N;
  const vboc_opts_t* o = &P->o;
  int status = 2, it, qp_total = 0;
  double rstat = 0, req = 0, rineq = 0, rcomp = 0;
  for (it = 0;; ++it) {
    linearize(P);
    nlp_residuals(P, &rstat, &req, &rineq, &rcomp);
    if (!isfinite(rstat) || !isfinite(req)) { status = 1; break; }
    if (rstat < o->tol_stat && req < o->tol_eq && rineq < o->tol_ineq && rcomp < o->tol_comp) { status = 0; break; }
    if (it >= o->max_iter) { status = 2; break; }
    int qit = 0;
    int qs = qp_solve(P, &qit);
    qp_total += qit;
    if (qs < 0) { status = 4; break; }
    /* merit weights (L1 exact penalty, weights from the QP multipliers) */
    double lmax = 0.0;
    for (int k = 0; k <= N; ++k) {
      stage_t* s = &P->st[k];
      if (k < N) for (int i = 0; i < nx; ++i) s->wpi[i] = wupd(s->wpi[i], s->qpi[i]);
      for (int i = 0; i < nz_of(P, k); ++i) lmax = fmax(lmax, fmax(s->ql[i], s->qu[i]));
      if (hc_on(P, k)) lmax = fmax(lmax, fmax(s->hql, s->hqu));
    }
    for (int j = 0; j < nq; ++j) P->wnu[j] = wupd(P->wnu[j], P->qnu[j]);
    P->wbnd = wupd(P->wbnd, lmax);
    double phi0 = merit(P, 0.0);
    double alpha = 1.0;
    double phia;
    for (;;) {
      phia = merit(P, alpha);
      if (phia < phi0) break;
      if (alpha * o->alpha_reduction < o->alpha_min) break;
      alpha *= o->alpha_reduction;
    }
#ifdef VBOC_TRACE
    { double dmax = 0; for (int k = 0; k <= N; ++k) for (int i = 0; i < nz_of(P, k); ++i) dmax = fmax(dmax, fabs(P->st[k].dz[i]));
      fprintf(stderr, "it %3d stat %.3e eq %.3e ineq %.3e comp %.3e | qp %d it %d | s %.6f ds %.3e |dz| %.3e phi0 %.6e phia %.6e a %.4f\n",
              it, rstat, req, rineq, rcomp, qs, qit, P->s, P->st[0].dz[0], dmax, phi0, phia, alpha); }
#endif
    /* update primal and dual iterates */
    P->s += alpha * P->st[0].dz[0];
    for (int a = 0; a < nu; ++a) P->st[0].u[a] += alpha * P->st[0].dz[1 + a];
    for (int k = 1; k <= N; ++k) {
      stage_t* s = &P->st[k];
      for (int i = 0; i < nx; ++i) s->x[i] += alpha * s->dz[i];
      if (k < N) for (int a = 0; a < nu; ++a) s->u[a] += alpha * s->dz[nx + a];
    }
    for (int k = 0; k <= N; ++k) {
      stage_t* s = &P->st[k];
      for (int i = 0; i < nz_of(P, k); ++i) {
        s->ll[i] += alpha * (s->ql[i] - s->ll[i]);
        s->lu[i] += alpha * (s->qu[i] - s->lu[i]);
      }
      if (hc_on(P, k)) {
        s->hll += alpha * (s->hql - s->hll);
        s->hlu += alpha * (s->hqu - s->hlu);
      }
      if (k < N) for (int i = 0; i < nx; ++i) s->pi[i] += alpha * (s->qpi[i] - s->pi[i]);
    }
    for (int j = 0; j < nq; ++j) P->nu[j] += alpha * (P->qnu[j] - P->nu[j]);
    if (!isfinite(P->s)) { status = 1; break; }
  }
  set_x0(P);
  res->status = status;
  res->sqp_iter = it;
  res->qp_iter = qp_total;
  res->cost = P->cs * P->s + P->cost_const;
  res->res_stat = rstat; res->res_eq = req; res->res_ineq = rineq; res->res_comp = rcomp;
}

/* ------------------------------------------------------------------------------------------ */
/* public entry points                                                                         */
/* ------------------------------------------------------------------------------------------ */

void vboc_oracle_default_opts(vboc_opts_t* o) {
  o->tol_stat = 1e-3; o->tol_eq = 1e-6; o->tol_ineq = 1e-6; o->tol_comp = 1e-6;
  o->max_iter = 1000; o->qp_max_iter = 100;
  o->alpha_min = 1e-2; o->alpha_reduction = 0.3; o->lm = 1e-5;
  o->mu0 = 1.0; o->ipm_push = 1e-2; o->ipm_tau = 0.995;
  /* QP: tol_stat from qp_solver_tol_stat = 1e-3 (triplependulum_class_vboc.py:135); the other
     HPIPM tolerances keep their library defaults (1e-8). */
  o->qp_tol_stat = 1e-3; o->qp_tol_eq = 1e-8; o->qp_tol_comp = 1e-8;
  o->hc = 0; o->hc_xc = o->hc_yc = o->hc_lh = o->hc_uh = 0.0;
}

void vboc_oracle_model(int nq, const double* th, const double* om, const double* u, double* acc,
                       double* Jth, double* Jom, double* Ju) {
  model_t m; model_init(&m, nq);
  model_eval(&m, th, om, u, acc, Jth, Jom, Ju);
}

void vboc_oracle_rk4(int nq, double h, const double* x, const double* u, double* x1) {
  model_t m; model_init(&m, nq);
  rk4(&m, h, x, u, x1);
}

void vboc_oracle_rk4_sens(int nq, double h, const double* x, const double* u, double* x1, double* A, double* B) {
  model_t m; model_init(&m, nq);
  rk4_sens(&m, h, x, u, x1, A, B);
}

/* Solve one OCP given in the reference's layout (nx_ref = 2 nq + 1 with the dt column):
 *   x_guess[(N+1) * nx_ref], u_guess[N * nq], p[nq + 1], lbx/ubx (path), lbu/ubu,
 *   lbx_0/ubx_0 (q_init), lbx_e/ubx_e (q_fin).  Outputs x_out[(N+1) nx_ref], u_out[N nq]. */
static int solve_impl(int nq, int N, const double* x_guess, const double* u_guess, const double* p,
                      const double* lbx, const double* ubx, const double* lbu, const double* ubu,
                      const double* lbx0, const double* ubx0, const double* lbxe, const double* ubxe,
                      const vboc_opts_t* opts, double* x_out, double* u_out, vboc_result_t* res, double* mult);

int vboc_oracle_solve(int nq, int N, const double* x_guess, const double* u_guess, const double* p,
                      const double* lbx, const double* ubx, const double* lbu, const double* ubu,
                      const double* lbx0, const double* ubx0, const double* lbxe, const double* ubxe,
                      const vboc_opts_t* opts, double* x_out, double* u_out, vboc_result_t* res) {
  return solve_impl(nq, N, x_guess, u_guess, p, lbx, ubx, lbu, ubu, lbx0, ubx0, lbxe, ubxe, opts, x_out, u_out,
                    res, NULL);
}

/* The same solve, also returning the NLP multipliers at the final iterate (for KKT checks recomputed outside
 * the oracle, tests/test_oracle_kkt.py): per stage k = 0..N a row of 3 (2 nq) + 2 (3 nq) doubles
 *   [pi_k (2nq; zero at k = N) | lam_l of z_k (3nq) | lam_u of z_k (3nq)]
 * with z_0 = (s, u_0), z_k = (x_k, u_k), z_N = x_N (unused entries zero), then nu (nq; the terminal
 * velocity multiplier) and s. */
int vboc_oracle_solve_mult(int nq, int N, const double* x_guess, const double* u_guess, const double* p,
                           const double* lbx, const double* ubx, const double* lbu, const double* ubu,
                           const double* lbx0, const double* ubx0, const double* lbxe, const double* ubxe,
                           const vboc_opts_t* opts, double* x_out, double* u_out, vboc_result_t* res, double* mult) {
  return solve_impl(nq, N, x_guess, u_guess, p, lbx, ubx, lbu, ubu, lbx0, ubx0, lbxe, ubxe, opts, x_out, u_out,
                    res, mult);
}

static int solve_impl(int nq, int N, const double* x_guess, const double* u_guess, const double* p,
                      const double* lbx, const double* ubx, const double* lbu, const double* ubu,
                      const double* lbx0, const double* ubx0, const double* lbxe, const double* ubxe,
                      const vboc_opts_t* opts, double* x_out, double* u_out, vboc_result_t* res, double* mult) {
  const int nxr = 2 * nq + 1;
  prob_t P;
  memset(&P, 0, sizeof(P));
  model_init(&P.m, nq);
  P.o = *opts;
  P.N = N;
  P.h = lbx[2 * nq];                      /* dt pinned by the path bounds */
  if (!(lbx[2 * nq] == ubx[2 * nq]) || !(lbx0[2 * nq] == ubx0[2 * nq]) || !(lbxe[2 * nq] == ubxe[2 * nq]))
    return -2;                            /* free time not supported */
  P.st = (stage_t*)calloc((size_t)N + 1, sizeof(stage_t));
  if (!P.st) return -3;
  /* direction d = p[:nq] (unit), stage-0 reparametrisation, s bounds from the velocity box */
  double nrm = 0.0;
  for (int j = 0; j < nq; ++j) nrm += p[j] * p[j];
  nrm = sqrt(nrm);
  P.slb = -INFINITY; P.sub = INFINITY; P.cs = 0.0;
  for (int j = 0; j < nq; ++j) {
    P.dir[j] = (nq == 1) ? 1.0 : p[j] / nrm;  /* pendulum: no C row, velocity free */
    P.q0[j] = lbx0[j];
    P.cs += p[j] * P.dir[j];
    double dj = P.dir[j], lo = lbx0[nq + j], hi = ubx0[nq + j];
    if (dj > 0) { P.slb = fmax(P.slb, lo / dj); P.sub = fmin(P.sub, hi / dj); }
    else if (dj < 0) { P.slb = fmax(P.slb, hi / dj); P.sub = fmin(P.sub, lo / dj); }
  }
  P.cost_const = p[nq] * P.h * (double)N;  /* wt * dt at stages 0..N-1 */
  for (int i = 0; i < 2 * nq; ++i) { P.xlb[i] = lbx[i]; P.xub[i] = ubx[i]; }
  for (int a = 0; a < nq; ++a) { P.ulb[a] = lbu[a]; P.uub[a] = ubu[a]; }
  for (int j = 0; j < nq; ++j) { P.qNlb[j] = lbxe[j]; P.qNub[j] = ubxe[j]; P.vfin[j] = lbxe[nq + j]; }
  /* guess */
  double s = 0.0;
  for (int j = 0; j < nq; ++j) s += P.dir[j] * x_guess[nq + j];
  P.s = s;
  for (int k = 0; k <= N; ++k) {
    for (int i = 0; i < 2 * nq; ++i) P.st[k].x[i] = x_guess[k * nxr + i];
    if (k < N) for (int a = 0; a < nq; ++a) P.st[k].u[a] = u_guess[k * nq + a];
  }
  P.hc = opts->hc != 0;
  if (P.hc && !P.m.chain) { free(P.st); return -2; }  /* the Cartesian constraint is the chains' tip */
  int infeasible0 = 0;
  if (P.hc) {
    /* stage 0: positions fixed, h constant - an initial state inside the keep-out region makes every
       QP infeasible; reported as a QP failure without iterating */
    const double h0 = hc_eval(&P, P.q0, NULL);
    infeasible0 = !(h0 >= opts->hc_lh && h0 <= opts->hc_uh);
  }
  if (infeasible0) {
    memset(res, 0, sizeof(*res));
    res->status = 4;
    res->cost = NAN;
    set_x0(&P);
  } else {
    sqp(&P, res);
  }
  for (int k = 0; k <= N; ++k) {
    for (int i = 0; i < 2 * nq; ++i) x_out[k * nxr + i] = P.st[k].x[i];
    x_out[k * nxr + 2 * nq] = P.h;
    if (k < N) for (int a = 0; a < nq; ++a) u_out[k * nq + a] = P.st[k].u[a];
  }
  if (mult) {
    const int nx = 2 * nq, nz = 3 * nq, row = nx + 2 * nz;
    for (int k = 0; k <= N; ++k) {
      double* m = mult + (size_t)k * row;
      for (int i = 0; i < row; ++i) m[i] = 0.0;
      if (k < N) for (int i = 0; i < nx; ++i) m[i] = P.st[k].pi[i];
      for (int i = 0; i < nz_of(&P, k); ++i) { m[nx + i] = P.st[k].ll[i]; m[nx + nz + i] = P.st[k].lu[i]; }
    }
    for (int j = 0; j < nq; ++j) mult[(size_t)(N + 1) * row + j] = P.nu[j];
    mult[(size_t)(N + 1) * row + nq] = P.s;
  }
  free(P.st);
  return 0;
}

/* Batched: problem-major arrays, horizon N[b] <= Nmax; OpenMP over problems (CPU baseline). */
int vboc_oracle_solve_batch(int nq, int B, int Nmax, const int* N, const double* x_guess,
                            const double* u_guess, const double* p, const double* lbx, const double* ubx,
                            const double* lbu, const double* ubu, const double* lbx0, const double* ubx0,
                            const double* lbxe, const double* ubxe, const vboc_opts_t* opts, int nthreads,
                            double* x_out, double* u_out, vboc_result_t* res) {
  const int nxr = 2 * nq + 1, npr = nq + 1;
  int err = 0;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads) reduction(| : err)
  for (int b = 0; b < B; ++b) {
    const size_t xo = (size_t)b * (Nmax + 1) * nxr, uo = (size_t)b * Nmax * nq;
    int r = vboc_oracle_solve(nq, N[b], x_guess + xo, u_guess + uo, p + (size_t)b * npr,
                              lbx + (size_t)b * nxr, ubx + (size_t)b * nxr, lbu + (size_t)b * nq,
                              ubu + (size_t)b * nq, lbx0 + (size_t)b * nxr, ubx0 + (size_t)b * nxr,
                              lbxe + (size_t)b * nxr, ubxe + (size_t)b * nxr, opts, x_out + xo, u_out + uo,
                              res + b);
    if (r) err |= 1;
  }
  return err ? -1 : 0;
}

/* ORACLE - TEST INFRASTRUCTURE ONLY.  Used by tests/ (checked against the reference's own function) and by
 * bench.py's cpu_baseline leg (the reference's CPU loop at full speed on the host cores).  The product path
 * (vboc_amd/) never links, loads or calls it.
 *
 * vboc_dg.c - plain-C restatement of the reference's per-problem data-generation state machine
 *   triple: data_generation(v), VBOC/triplependulum_vboc.py:19-370
 *   double: data_generation(v), VBOC/doublependulum_vboc.py:19-403 (3-tuple result, :399-402)
 * run the way the reference runs it: one problem per worker (Pool(30).map, VBOC/triplependulum_vboc.py:
 * 399-405) - here one problem per OpenMP thread, dynamic schedule, no rounds and no barriers - with the CPU
 * oracle (vboc_oracle.c) as its OCP solver (OCP_solve, :110) and twin integrator (SYM<sys>INIT, :346-353).
 *
 * Written from the reference's text, independently of the device loop (vboc_amd/csrc/dg.h) and of the
 * Python driver (vboc_amd/drivers.py).  Arithmetic follows the Python semantics the reference runs under
 * (built with -ffp-contract=off): every expression left to right with IEEE double rounding;
 * numpy.linalg.norm of a 2/3-vector is sqrt of numpy's dot, which OpenBLAS evaluates as the FMA chain
 * v0*v0, fma(v1, v1, .), fma(v2, v2, .); np.linspace(0, 1, n) is i * (1 / (n - 1)) with the last point 1.0;
 * math.sin is the C library's sin.  Randomness: random.random() / random.choice() are served from
 * Philox4x32-10 streams keyed by (seed, problem id) (vboc_amd/ics.py): stream 0 for the IC sampling, stream 2
 * for the restart perturbations, both in the reference's draw order.
 * Decisions shared with the rest of the repository: quirk A.1 fixed (N_start per
 * problem, as VBOC/vboc.py:28 does), quirk A.3 (the duplicated x_sol[f] sample) kept.
 * Pinned bit for bit against tests/golden/driver_{2,3}.json (the reference's own function on the oracle) and,
 * with the fixtures' failure injection (fail_mod, test-only) exercising the restart branches, against the
 * batched Python driver on the oracle (tests/test_oracle_dg.py). */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "vboc_oracle.h"

#define DNQ 3
#define DNX 6
#define DNXR 7

/* ---- Philox4x32-10 uniforms (vboc_amd/ics.py uniforms) ------------------------------------------- */
static void philox(const uint32_t in[4], uint32_t k0, uint32_t k1, uint32_t out[4]) {
  uint32_t c0 = in[0], c1 = in[1], c2 = in[2], c3 = in[3];
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0, hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c0 = hi1 ^ c1 ^ k0;
    c1 = lo1;
    c2 = hi0 ^ c3 ^ k1;
    c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

typedef struct {
  uint64_t id, seed;
  uint32_t stream;
  long pos;            /* next draw index */
} rng_t;

/* draw `idx` of (seed, id, stream): two 53-bit doubles per Philox block */
static double uniform_at(const rng_t* r, long idx) {
  const uint32_t ctr[4] = {(uint32_t)r->id, (uint32_t)(r->id >> 32), (uint32_t)(idx / 2), r->stream};
  uint32_t o[4];
  philox(ctr, (uint32_t)r->seed, (uint32_t)(r->seed >> 32) ^ 0x5BD1E995u, o);
  const uint32_t a = (idx & 1) ? o[2] : o[0], b = (idx & 1) ? o[3] : o[1];
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) / 9007199254740992.0;
}
static double rnd(rng_t* r) { return uniform_at(r, r->pos++); }
/* random.choice([-1, 1]) / ([0, 1]) / ([0, 1, 2]) */
static int choice_idx(rng_t* r, int n) {
  const double u = rnd(r);
  const long i = (long)(u * (double)n);
  return (int)(i < n - 1 ? i : n - 1);
}
static double choice_pm1(rng_t* r) { return choice_idx(r, 2) == 0 ? -1.0 : 1.0; }
/* `random.random() * random.choice([-1, 1]) * 0.01`, the two draws in that order (Python evaluates the left
   operand first; C leaves the order of two calls in one expression unspecified, so it is sequenced here) */
static double perturbation(rng_t* r) {
  const double u = rnd(r);
  const double s = choice_pm1(r);
  return u * s * 0.01;
}

/* numpy.linalg.norm of a 1-D vector (OpenBLAS ddot: FMA chain), n = 2 or 3 */
static double np_norm(const double* v, int n) {
  double s = v[0] * v[0];
  for (int i = 1; i < n; ++i) s = fma(v[i], v[i], s);
  return sqrt(s);
}

typedef struct {
  int nq;
  double q_min, q_max, v_max, tau_max, dt, tol, eps, g, l1, l2, m1, m2;
  int fail_mod;
  vboc_opts_t o;
} dg_cfg_t;

typedef struct {
  /* one OCP_solve request (the arguments of VBOC/triplependulum_class_vboc.py:155 OCP_solve) */
  int N, nrows;                    /* horizon; rows of the guess (N, or N + 1) */
  double *xg, *ug;                 /* [nrows][NXR], [nrows][NQ] */
  double p[DNQ + 1], lb0[DNXR], ub0[DNXR];
  /* the solution (ocp_solver.get / get_cost) */
  int status;
  double cost;
  double *xs, *us;                 /* [N + 1][NXR], [N][NQ] */
  /* scratch of the solve */
  double *xgs, *ugs;
  long long solves, rk4, sqp;
} dg_work_t;

static double grav_u(const dg_cfg_t* c, int j, const double* x) {
  /* ocp.g*ocp.l1*(ocp.m1+ocp.m2)*math.sin(x[0]), ocp.g*ocp.l2*ocp.m2*math.sin(x[1]) (doublependulum_vboc.py:84) */
  return j == 0 ? c->g * c->l1 * (c->m1 + c->m2) * sin(x[0]) : c->g * c->l2 * c->m2 * sin(x[1]);
}

/* ocp.OCP_solve(x_sol_guess, u_sol_guess, p, q_lb, q_ub, u_lb, u_ub, q_init_lb, q_init_ub, q_fin_lb, q_fin_ub):
 * stages i < N take guess row i, stage N the guess's last row (VBOC/triplependulum_class_vboc.py:163-186) */
static void ocp_solve(const dg_cfg_t* c, dg_work_t* w) {
  const int nq = c->nq, nxr = 2 * nq + 1, N = w->N;
  double lbx[DNXR], ubx[DNXR], lbu[DNQ], ubu[DNQ], lbxe[DNXR], ubxe[DNXR];
  for (int j = 0; j < nq; ++j) {
    lbx[j] = c->q_min; ubx[j] = c->q_max; lbx[nq + j] = -c->v_max; ubx[nq + j] = c->v_max;
    lbu[j] = -c->tau_max; ubu[j] = c->tau_max;
    lbxe[j] = c->q_min; ubxe[j] = c->q_max; lbxe[nq + j] = 0.0; ubxe[nq + j] = 0.0;
  }
  lbx[2 * nq] = ubx[2 * nq] = lbxe[2 * nq] = ubxe[2 * nq] = c->dt;
  for (int k = 0; k < N; ++k) {
    memcpy(w->xgs + (size_t)k * nxr, w->xg + (size_t)k * nxr, sizeof(double) * nxr);
    memcpy(w->ugs + (size_t)k * nq, w->ug + (size_t)k * nq, sizeof(double) * nq);
  }
  memcpy(w->xgs + (size_t)N * nxr, w->xg + (size_t)(w->nrows - 1) * nxr, sizeof(double) * nxr);
  vboc_result_t res;
  vboc_oracle_solve(nq, N, w->xgs, w->ugs, w->p, lbx, ubx, lbu, ubu, w->lb0, w->ub0, lbxe, ubxe, &c->o, w->xs,
                    w->us, &res);
  w->status = res.status;
  w->cost = res.cost;
  /* test-only failure injection (tests/oracle_backend.py forced_failure): the fixtures' restart branches */
  if (c->fail_mod > 0 && (long long)(fabs(w->lb0[0]) * 1e6) % c->fail_mod == 0) w->status = 4;
  w->solves += 1;
  w->sqp += res.sqp_iter;
}

/* straight-line guess over N rows (:85-93; double :64-70 with the gravity guess) */
static void straight_guess(const dg_cfg_t* c, dg_work_t* w, int N, const double* qpos, int joint_sel,
                           double q_init_sel, double q_fin_sel) {
  const int nq = c->nq, nxr = 2 * nq + 1;
  const double step = N > 1 ? 1.0 / (double)(N - 1) : 0.0;
  for (int i = 0; i < N; ++i) {
    const double tau = (N > 1 && i == N - 1) ? 1.0 : (double)i * step;
    double* x = w->xg + (size_t)i * nxr;
    for (int j = 0; j < nq; ++j) { x[j] = qpos[j]; x[nq + j] = 0.0; }
    x[2 * nq] = c->dt;
    x[joint_sel] = (1 - tau) * q_init_sel + tau * q_fin_sel;
    x[joint_sel + nq] = 2 * (1 - tau) * (q_fin_sel - q_init_sel);
    for (int a = 0; a < nq; ++a) w->ug[(size_t)i * nq + a] = nq == 2 ? grav_u(c, a, x) : 0.0;
  }
  w->N = N;
  w->nrows = N;
}

/* guess rows from the last solution (:123-130): N + 1 rows, u at N = 0 (double: gravity) */
static void guess_from_solution(const dg_cfg_t* c, dg_work_t* w, int N) {
  const int nq = c->nq, nxr = 2 * nq + 1;
  memcpy(w->xg, w->xs, sizeof(double) * (size_t)(N + 1) * nxr);
  memcpy(w->ug, w->us, sizeof(double) * (size_t)N * nq);
  for (int a = 0; a < nq; ++a) w->ug[(size_t)N * nq + a] = nq == 2 ? grav_u(c, a, w->xg + (size_t)N * nxr) : 0.0;
  w->nrows = N + 1;
}

/* one problem: returns the number of saved rows (-1: None); rows [cap][NX]; ic / ic_slot: the double's
 * OCP_store_ic and its tuple position (1 = (X, ic, None), 2 = (None, None, ic)) */
static int dg_problem(const dg_cfg_t* c, uint64_t pid, uint64_t seed, int N_start, dg_work_t* w, double* rows,
                      int cap, double* ic, int* ic_slot) {
  const int nq = c->nq, nx = 2 * nq, nxr = 2 * nq + 1;
  const double q_min = c->q_min, q_max = c->q_max, v_max = c->v_max, v_min = -c->v_max, eps = c->eps, tol = c->tol;
  rng_t r0 = {pid, seed, 0, 0}, r2 = {pid, seed, 2, 0};
  int N = N_start;
  /* ---- IC sampling (triple :32-83, double :33-60) ---- */
  const int joint_sel = choice_idx(&r0, nq);
  const int joint_oth = 1 - joint_sel;                  /* double */
  const double vel_sel = choice_pm1(&r0);
  const double q_init_sel = vel_sel == -1 ? q_min : q_max, q_fin_sel = vel_sel == -1 ? q_max : q_min;
  double ran[DNQ];
  ran[0] = vel_sel * rnd(&r0);
  for (int j = 1; j < nq; ++j) {
    const double sgn = choice_pm1(&r0);
    ran[j] = sgn * rnd(&r0);
  }
  double nw = np_norm(ran, nq);
  double p[DNQ + 1];
  /* joint_sel's component is ran1, the others ran2 (, ran3) in joint order (:49-54, double :45-50) */
  {
    int o = 1;
    for (int j = 0; j < nq; ++j) p[j] = (j == joint_sel) ? ran[0] / nw : ran[o++] / nw;
    p[nq] = 0.0;
  }
  double qpos[DNQ], q_init_oth = 0.0, store_ic[4] = {0, 0, 0, 0};
  if (nq == 2) {
    q_init_oth = q_min + rnd(&r0) * (q_max - q_min);
    if (q_init_oth > q_max - eps) q_init_oth = q_init_oth - eps;
    if (q_init_oth < q_min + eps) q_init_oth = q_init_oth + eps;
    store_ic[0] = vel_sel + 1 + joint_sel; store_ic[1] = ran[0]; store_ic[2] = ran[1]; store_ic[3] = q_init_oth;
    qpos[0] = qpos[1] = q_init_oth;
  } else {
    for (int j = 0; j < nq; ++j) {
      double q = q_min + rnd(&r0) * (q_max - q_min);
      if (q > q_max - eps) q = q - eps;
      if (q < q_min + eps) q = q + eps;
      qpos[j] = q;
    }
  }
  double lb0[DNXR], ub0[DNXR];
  for (int j = 0; j < nq; ++j) { lb0[j] = ub0[j] = qpos[j]; lb0[nq + j] = v_min; ub0[nq + j] = v_max; }
  lb0[nx] = ub0[nx] = c->dt;
  lb0[joint_sel] = ub0[joint_sel] = (q_init_sel == q_min) ? q_min + eps : q_max - eps;
  straight_guess(c, w, N, qpos, joint_sel, q_init_sel, q_fin_sel);
  /* ---- horizon extension (:105-174) ---- */
  double cost = 1e6;
  int all_ok = 0;
  for (int it = 0; it < 10; ++it) {
    w->N = N;
    memcpy(w->p, p, sizeof(p));
    memcpy(w->lb0, lb0, sizeof(lb0));
    memcpy(w->ub0, ub0, sizeof(ub0));
    ocp_solve(c, w);
    if (w->status == 0) {
      const double cost_new = w->cost;
      if (cost_new > cost - tol) { all_ok = 1; break; }
      cost = cost_new;
      guess_from_solution(c, w, N);
      N = N + 1;
    } else {
      if (nq == 2) {
        /* :137-157 */
        ran[0] = ran[0] + perturbation(&r2);
        ran[1] = ran[1] + perturbation(&r2);
        nw = np_norm(ran, 2);
        if (joint_sel == 0) { p[0] = ran[0] / nw; p[1] = ran[1] / nw; }
        else { p[0] = ran[1] / nw; p[1] = ran[0] / nw; }
        p[2] = 0.0;
        q_init_oth = q_init_oth + perturbation(&r2);
        if (q_init_oth > q_max - eps) q_init_oth = q_init_oth - eps;
        if (q_init_oth < q_min + eps) q_init_oth = q_init_oth + eps;
        lb0[joint_oth] = ub0[joint_oth] = q_init_oth;
        store_ic[0] = vel_sel + 1 + joint_sel; store_ic[1] = ran[0]; store_ic[2] = ran[1]; store_ic[3] = q_init_oth;
        qpos[0] = qpos[1] = q_init_oth;
      } else {
        /* :144-165 */
        double rr[DNQ];
        for (int k = 0; k < nq; ++k) rr[k] = p[k] + perturbation(&r2);
        nw = np_norm(rr, nq);
        for (int k = 0; k < nq; ++k) p[k] = rr[k] / nw;
        p[nq] = 0.0;
        const double dev = perturbation(&r2);
        for (int j = 0; j < nq; ++j) {
          if (j == joint_sel) continue;
          double val = lb0[j] + dev;
          if (val > q_max - eps) val = val - eps;
          if (val < q_min + eps) val = val + eps;
          lb0[j] = ub0[j] = val;
        }
        for (int j = 0; j < nq; ++j) qpos[j] = lb0[j];
      }
      straight_guess(c, w, N, qpos, joint_sel, q_init_sel, q_fin_sel);
      cost = 1e6;
    }
  }
  if (nq == 2) memcpy(ic, store_ic, sizeof(store_ic));
  if (!all_ok) {
    if (nq == 2) *ic_slot = 2;
    return -1;
  }
  if (nq == 2) *ic_slot = 1;
  /* ---- sweep along the optimal trajectory (:177-365) ---- */
  double* x_sol = (double*)malloc(sizeof(double) * (size_t)(N + 1) * nxr);
  double* u_sol = (double*)malloc(sizeof(double) * (size_t)N * nq);
  double* x_sym = (double*)malloc(sizeof(double) * (size_t)(N + 1) * nx);
  memcpy(x_sol, w->xs, sizeof(double) * (size_t)(N + 1) * nxr);
  memcpy(u_sol, w->us, sizeof(double) * (size_t)N * nq);
  int nr = 0;
#define SAVE(src) do { if (nr < cap) memcpy(rows + (size_t)nr * nx, (src), sizeof(double) * nx); ++nr; } while (0)
  SAVE(x_sol);
  double x_out[DNX];
  memcpy(x_out, x_sol, sizeof(double) * nx);
  for (int j = 0; j < nq; ++j) x_out[nq + j] = x_out[nq + j] - eps * p[j];
  int is_x_at_limit = 0;
  for (int j = 0; j < nq; ++j) if (x_out[nq + j] > v_max || x_out[nq + j] < v_min) is_x_at_limit = 1;
  if (!is_x_at_limit) memcpy(x_sym, x_out, sizeof(double) * nx);
  for (int f = 1; f < N; ++f) {
    const double* xf = x_sol + (size_t)f * nxr;
    if (is_x_at_limit) {
      memcpy(x_out, xf, sizeof(double) * nx);
      const double norm_vel = np_norm(x_out + nq, nq);
      for (int j = 0; j < nq; ++j) x_out[nq + j] = x_out[nq + j] + eps * x_out[nq + j] / norm_vel;
      int lim = 0, vo = 0, limp = 0;
      for (int j = 0; j < nq; ++j) {
        if (xf[j] > q_max - eps || xf[j] < q_min + eps) lim = 1;
        if (x_out[nq + j] > v_max || x_out[nq + j] < v_min) vo = 1;
        const double qp = x_sol[(size_t)(f - 1) * nxr + j];
        if (qp > q_max - eps || qp < q_min + eps) limp = 1;
      }
      if (lim || vo) {
        is_x_at_limit = 1;
      } else {
        is_x_at_limit = 0;
        if (limp) break;
        /* verification OCP from x_sol[f] (:232-339) */
        int N_test = N - f;
        double vf[DNQ] = {0, 0, 0};
        for (int j = 0; j < nq; ++j) vf[j] = xf[nq + j];
        const double nwv = np_norm(vf, nq);
        for (int j = 0; j < nq; ++j) p[j] = -xf[nq + j] / nwv;
        p[nq] = 0.0;
        for (int j = 0; j < nq; ++j) { lb0[j] = ub0[j] = xf[j]; lb0[nq + j] = v_min; ub0[nq + j] = v_max; }
        lb0[nx] = ub0[nx] = c->dt;
        for (int i = 0; i < N_test; ++i) {
          memcpy(w->xg + (size_t)i * nxr, x_sol + (size_t)(i + f) * nxr, sizeof(double) * nxr);
          memcpy(w->ug + (size_t)i * nq, u_sol + (size_t)(i + f) * nq, sizeof(double) * nq);
        }
        memcpy(w->xg + (size_t)N_test * nxr, x_sol + (size_t)N * nxr, sizeof(double) * nxr);
        for (int a = 0; a < nq; ++a)
          w->ug[(size_t)N_test * nq + a] = nq == 2 ? grav_u(c, a, x_sol + (size_t)N * nxr) : 0.0;
        w->nrows = N_test + 1;
        const double norm_old = np_norm(vf, nq);
        double norm_bef = 0, norm_new = 0;
        int ok_v = 0;
        for (int it = 0; it < 5; ++it) {
          w->N = N_test;
          memcpy(w->p, p, sizeof(p));
          memcpy(w->lb0, lb0, sizeof(lb0));
          memcpy(w->ub0, ub0, sizeof(ub0));
          ocp_solve(c, w);
          if (w->status == 0) {
            norm_new = np_norm(w->xs + nq, nq);
            if (norm_new < norm_bef + tol) { ok_v = 1; break; }
            norm_bef = norm_new;
            guess_from_solution(c, w, N_test);
            N_test = N_test + 1;
          } else {
            break;
          }
        }
        if (ok_v) {
          if (norm_new > norm_old + tol) {            /* the state is inside V (:304-316) */
            for (int i = 0; i < N - f; ++i) {
              memcpy(x_sol + (size_t)(i + f) * nxr, w->xs + (size_t)i * nxr, sizeof(double) * nxr);
              memcpy(u_sol + (size_t)(i + f) * nq, w->us + (size_t)i * nq, sizeof(double) * nq);
            }
            memcpy(x_out, xf, sizeof(double) * nx);
            for (int j = 0; j < nq; ++j) x_out[nq + j] = x_out[nq + j] + eps * x_out[nq + j] / norm_new;
            int vo2 = 0;
            for (int j = 0; j < nq; ++j) if (x_out[nq + j] > v_max || x_out[nq + j] < v_min) vo2 = 1;
            if (vo2) is_x_at_limit = 1;
            else { is_x_at_limit = 0; memcpy(x_sym + (size_t)f * nx, x_out, sizeof(double) * nx); }
          } else {                                     /* the state is on dV (:317-331) */
            is_x_at_limit = 0;
            memcpy(x_out, xf, sizeof(double) * nx);
            for (int j = 0; j < nq; ++j) x_out[nq + j] = x_out[nq + j] - eps * p[j];
            if (x_out[joint_sel + nq] > v_max) x_out[joint_sel + nq] = v_max;
            if (x_out[joint_sel + nq] < v_min) x_out[joint_sel + nq] = v_min;
            memcpy(x_sym + (size_t)f * nx, x_out, sizeof(double) * nx);
          }
        } else {
          /* unresolved: x_sol[f] once per later state at a velocity limit (quirk A.3, :333-337) */
          for (int rr = f; rr < N; ++rr) {
            int hit = 0;
            for (int j = 0; j < nq; ++j) if (fabs(x_sol[(size_t)rr * nxr + nq + j]) > v_max - eps) hit = 1;
            if (hit) SAVE(xf);
          }
          break;
        }
      }
    } else {
      /* one step of the unviable twin (:341-360) */
      vboc_oracle_rk4(nq, c->dt, x_sym + (size_t)(f - 1) * nx, u_sol + (size_t)(f - 1) * nq, x_sym + (size_t)f * nx);
      w->rk4 += 1;
      const double* xs = x_sym + (size_t)f * nx;
      int out = 0;
      for (int j = 0; j < nq; ++j) {
        if (xs[j] > q_max || xs[j] < q_min) out = 1;
        if (xs[nq + j] > v_max || xs[nq + j] < v_min) out = 1;
      }
      is_x_at_limit = out;
    }
    /* the save filter (:362-365) */
    int keep = 1;
    for (int j = 0; j < nq; ++j) {
      if (!(q_min + eps < xf[j] && xf[j] < q_max - eps)) keep = 0;
      if (!(fabs(xf[nq + j]) > tol)) keep = 0;
    }
    if (keep) SAVE(xf);
  }
#undef SAVE
  free(x_sol); free(u_sol); free(x_sym);
  return nr;
}

/* Batched: problems ids[0..B) (one per OpenMP thread, dynamic schedule).  rows [B][max_rows][2nq] with
 * row_cnt[b] rows (-1: None; > max_rows: overflow, rows truncated); ic [B][4] and ic_slot (double);
 * stats [B][3] = solves, twin steps, SQP iterations.  params: q_min, q_max, v_max, tau_max, dt, tol, eps,
 * g, l1, l2, m1, m2.  Returns 0, -1 on a bad argument. */
int vboc_oracle_data_generation(int nq, int B, const long long* ids, unsigned long long seed, int N_start,
                                const double* params, int fail_mod, int nthreads, int max_rows, double* rows,
                                int* row_cnt, double* ic, int* ic_slot, long long* stats) {
  if ((nq != 2 && nq != 3) || B < 0 || N_start < 2) return -1;
  dg_cfg_t c;
  c.nq = nq;
  c.q_min = params[0]; c.q_max = params[1]; c.v_max = params[2]; c.tau_max = params[3]; c.dt = params[4];
  c.tol = params[5]; c.eps = params[6]; c.g = params[7]; c.l1 = params[8]; c.l2 = params[9]; c.m1 = params[10];
  c.m2 = params[11];
  c.fail_mod = fail_mod;
  vboc_oracle_default_opts(&c.o);
  const int nmax = N_start + 16, nxr = 2 * nq + 1, nx = 2 * nq;
#pragma omp parallel num_threads(nthreads)
  {
    dg_work_t w;
    memset(&w, 0, sizeof(w));
    const size_t xr = (size_t)(nmax + 2) * nxr, ur = (size_t)(nmax + 2) * nq;
    w.xg = (double*)calloc(xr, sizeof(double)); w.ug = (double*)calloc(ur, sizeof(double));
    w.xs = (double*)calloc(xr, sizeof(double)); w.us = (double*)calloc(ur, sizeof(double));
    w.xgs = (double*)calloc(xr, sizeof(double)); w.ugs = (double*)calloc(ur, sizeof(double));
#pragma omp for schedule(dynamic, 1)
    for (int b = 0; b < B; ++b) {
      w.solves = w.rk4 = w.sqp = 0;
      int slot = 0;
      double icb[4] = {0, 0, 0, 0};
      row_cnt[b] = dg_problem(&c, (uint64_t)ids[b], (uint64_t)seed, N_start, &w, rows + (size_t)b * max_rows * nx,
                              max_rows, icb, &slot);
      if (ic) memcpy(ic + (size_t)b * 4, icb, sizeof(icb));
      if (ic_slot) ic_slot[b] = slot;
      stats[(size_t)b * 3] = w.solves; stats[(size_t)b * 3 + 1] = w.rk4; stats[(size_t)b * 3 + 2] = w.sqp;
    }
    free(w.xg); free(w.ug); free(w.xs); free(w.us); free(w.xgs); free(w.ugs);
  }
  return 0;
}

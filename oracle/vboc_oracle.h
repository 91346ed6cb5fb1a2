/* ORACLE - TEST INFRASTRUCTURE ONLY (see vboc_oracle.c header). */
#ifndef VBOC_ORACLE_H
#define VBOC_ORACLE_H
#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  double tol_stat, tol_eq, tol_ineq, tol_comp;
  int max_iter, qp_max_iter;
  double alpha_min, alpha_reduction, lm;
  double mu0, ipm_push, ipm_tau;
  double qp_tol_stat, qp_tol_eq, qp_tol_comp;
  /* Cartesian path constraint (VBOC/Cartesian constraints/doublependulum_class_fixedveldir.py:154-160):
     hc != 0 => hc_lh <= (sum_j l sin th_j - hc_xc)^2 + (sum_j l cos th_j - hc_yc)^2 <= hc_uh at
     stages 0..N-1 of the pendulum chains (nq 2, 3) */
  int hc;
  double hc_xc, hc_yc, hc_lh, hc_uh;
} vboc_opts_t;

typedef struct {
  int status, sqp_iter, qp_iter, pad;
  double cost, res_stat, res_eq, res_ineq, res_comp;
} vboc_result_t;

void vboc_oracle_default_opts(vboc_opts_t* o);
void vboc_oracle_model(int nq, const double* th, const double* om, const double* u, double* acc,
                       double* Jth, double* Jom, double* Ju);
void vboc_oracle_rk4(int nq, double h, const double* x, const double* u, double* x1);
void vboc_oracle_rk4_sens(int nq, double h, const double* x, const double* u, double* x1, double* A,
                          double* B);
int vboc_oracle_solve(int nq, int N, const double* x_guess, const double* u_guess, const double* p,
                      const double* lbx, const double* ubx, const double* lbu, const double* ubu,
                      const double* lbx0, const double* ubx0, const double* lbxe, const double* ubxe,
                      const vboc_opts_t* opts, double* x_out, double* u_out, vboc_result_t* res);
int vboc_oracle_solve_mult(int nq, int N, const double* x_guess, const double* u_guess, const double* p,
                           const double* lbx, const double* ubx, const double* lbu, const double* ubu,
                           const double* lbx0, const double* ubx0, const double* lbxe, const double* ubxe,
                           const vboc_opts_t* opts, double* x_out, double* u_out, vboc_result_t* res, double* mult);
int vboc_oracle_solve_batch(int nq, int B, int Nmax, const int* N, const double* x_guess,
                            const double* u_guess, const double* p, const double* lbx, const double* ubx,
                            const double* lbu, const double* ubu, const double* lbx0, const double* ubx0,
                            const double* lbxe, const double* ubxe, const vboc_opts_t* opts, int nthreads,
                            double* x_out, double* u_out, vboc_result_t* res);
/* free-time box OCP (vboc_oracle_ft.c): dt a state, terminal/stage-0 fixed components by lb == ub */
void vboc_oracle_ft_rk4_sens(int nq, const double* x, const double* u, double* x1, double* A, double* B);
int vboc_oracle_ft_solve(int nq, int N, const double* x_guess, const double* u_guess, const double* p,
                         const double* lbx, const double* ubx, const double* lbu, const double* ubu,
                         const double* lbx0, const double* ubx0, const double* lbxe, const double* ubxe,
                         const vboc_opts_t* opts, double* x_out, double* u_out, vboc_result_t* res);
int vboc_oracle_ft_solve_batch(int nq, int B, int Nmax, const int* N, const double* x_guess,
                               const double* u_guess, const double* p, const double* lbx, const double* ubx,
                               const double* lbu, const double* ubu, const double* lbx0, const double* ubx0,
                               const double* lbxe, const double* ubxe, const vboc_opts_t* opts, int nthreads,
                               double* x_out, double* u_out, vboc_result_t* res);
/* Safe-MPC tracking OCP with the terminal NN row (vboc_oracle_ft.c): NeuralNetDIR(2 nq, hid, 1) weights in
   float64 (row-major, torch's nn.Linear layout), the scalar position mean / std, the row's bounds */
typedef struct {
  int hid;
  const double *W0, *b0, *W1, *b1, *W2, *b2;
  double mean, std, lh, uh;
} vboc_mpc_nn_t;
/* x [N + 1][2 nq], u [N][nq]; W [3 nq] stage weights on [x; u], We [2 nq], yref [3 nq], yref_e [2 nq]; cs the
   stage-cost scale; nn NULL = no terminal row; rti 1 = SQP_RTI (one QP, full step) */
int vboc_oracle_mpc_solve(int nq, int N, double h, const double* x0, const double* x_guess, const double* u_guess,
                          const double* xlb, const double* xub, const double* ulb, const double* uub,
                          const double* xNlb, const double* xNub, const double* W, const double* We,
                          const double* yref, const double* yref_e, double cs, const vboc_mpc_nn_t* nn, int rti,
                          const vboc_opts_t* opts, double* x_out, double* u_out, vboc_result_t* res, double* hrow);
int vboc_oracle_mpc_solve_batch(int nq, int B, int N, double h, const double* x0, const double* x_guess,
                                const double* u_guess, const double* xlb, const double* xub, const double* ulb,
                                const double* uub, const double* xNlb, const double* xNub, const double* W,
                                const double* We, const double* yref, const double* yref_e, double cs,
                                const vboc_mpc_nn_t* nn, int rti, const vboc_opts_t* opts, int nthreads,
                                double* x_out, double* u_out, vboc_result_t* res, double* hrow);
/* OCPtriplependulumSoftTraj (vboc_oracle_ft.c header): the row scaled by (100 - margin) / 100 on every stage 0..N,
   soft lower sides with per-stage slack weights zl / Zl [N + 1] (zu = Zu = 0) */
typedef struct {
  double margin;
  const double *zl, *Zl;
} vboc_mpc_soft_t;
int vboc_oracle_mpc_solve_soft(int nq, int N, double h, const double* x0, const double* x_guess,
                               const double* u_guess, const double* xlb, const double* xub, const double* ulb,
                               const double* uub, const double* xNlb, const double* xNub, const double* W,
                               const double* We, const double* yref, const double* yref_e, double cs,
                               const vboc_mpc_nn_t* nn, const vboc_mpc_soft_t* soft, int rti, const vboc_opts_t* opts,
                               double* x_out, double* u_out, vboc_result_t* res, double* hrow);
int vboc_oracle_mpc_soft_solve_batch(int nq, int B, int N, double h, const double* x0, const double* x_guess,
                                     const double* u_guess, const double* xlb, const double* xub, const double* ulb,
                                     const double* uub, const double* xNlb, const double* xNub, const double* W,
                                     const double* We, const double* yref, const double* yref_e, double cs,
                                     const vboc_mpc_nn_t* nn, double margin, const double* zl, const double* Zl,
                                     int rti, const vboc_opts_t* opts, int nthreads, double* x_out, double* u_out,
                                     vboc_result_t* res, double* hrow);
void vboc_oracle_mpc_row(int nq, int B, const double* x, const vboc_mpc_nn_t* nn, double margin, double* out);
/* AL's compute_problem (vboc_oracle_ft.c): x0 [B][2 nq]; x_guess [B][N+1][2 nq] or NULL ((q0, 0)); boxes [2 nq] / [nq]; W [3 nq], We [2 nq]; label [B] 1/0/2 */
int vboc_oracle_al_solve_batch(int nq, int B, int N, double h, const double* x0, const double* x_guess,
                               const double* xlb, const double* xub, const double* ulb, const double* uub,
                               const double* xNlb, const double* xNub, const double* W, const double* We, double cs,
                               const vboc_opts_t* opts, int nthreads, double* x_out, double* u_out, vboc_result_t* res,
                               int* label);
/* HJR one-step OCP (vboc_oracle_hjr.c): x0 fixed, N = 1, terminal cost = logit 0 of NeuralNetCLS */
void vboc_oracle_hjr_default_opts(int nq, vboc_opts_t* o);
int vboc_oracle_hjr_solve_batch(int nq, int B, const double* x0, int h, const double* W0, const double* b0,
                                const double* W1, const double* b1, const double* W2, const double* b2, double mean,
                                double std, double u_max, const vboc_opts_t* opts, int nthreads, double* u_out,
                                double* x1_out, double* mult_out, vboc_result_t* res);
/* data_generation of the triple / double pendulum, one problem per OpenMP thread (vboc_dg.c) */
int vboc_oracle_data_generation(int nq, int B, const long long* ids, unsigned long long seed, int N_start,
                                const double* params, int fail_mod, int nthreads, int max_rows, double* rows,
                                int* row_cnt, double* ic, int* ic_slot, long long* stats);
#ifdef __cplusplus
}
#endif
#endif

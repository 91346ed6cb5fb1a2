/*
 * vboc.h - C ABI of the MI355X-native batched VBOC boundary-OCP solver (libvboc_amd.so).
 *
 * Plain pointers and sizes only (no torch / HIP types in the signatures; streams are passed as
 * void* = hipStream_t, NULL = default stream).  One handle <-> one device; not thread-safe.
 *
 * What each entry point replaces (the reference binds ACADOS's generated C solver through
 * acados_template's ctypes wrapper; every call below is a batched version of that path):
 *
 *   vboc_create            <- AcadosOcpSolver(self.ocp, json_file=...)
 *                             VBOC/triplependulum_class_vboc.py:153 (double :181, pendulum :105)
 *   vboc_set_option        <- ocp.solver_options.* (nlp_solver_tol_stat, qp_solver_iter_max,
 *                             levenberg_marquardt, alpha_min, alpha_reduction, nlp_solver_max_iter)
 *                             VBOC/triplependulum_class_vboc.py:129-141
 *   vboc_solve_batch       <- one OCPtriplependulumINIT.OCP_solve(...) per problem:
 *                             reset/set/constraints_set/solve, VBOC/triplependulum_class_vboc.py:155-191
 *                             (called from VBOC/triplependulum_vboc.py:110,262 and
 *                             triplependulum_testdata.py:44-75); results = ocp_solver.get(i,'x'|'u'),
 *                             get_cost(), solve() status (:115,126-129,189)
 *   vboc_rk4_batch         <- SYMtriplependulumINIT().acados_integrator set('x','u','T')/solve()/get('x')
 *                             VBOC/triplependulum_class_vboc.py:235-239, VBOC/triplependulum_vboc.py:346-353
 *   vboc_solve_batch_ft    <- one OCPpendulum.OCP_solve(...) per problem (free-time OCP, dt a state):
 *                             VBOC/pendulum_class_vboc.py:107-130, called from VBOC/pendulum_vboc.py:94,181
 *   vboc_data_generation   <- Pool(30).map(data_generation, range(P)): the whole per-problem boundary-sampling
 *                             state machine of VBOC/triplependulum_vboc.py:19-370 (fan-out :399-405) /
 *                             VBOC/doublependulum_vboc.py:19-403, with its OCP_solve calls (:110,262) and
 *                             twin-integrator steps (:346-353), run on the device
 *   vboc_mpc_solve_batch   <- one OCPtriplependulumHardTerm.OCP_solve(x0, x_sol_guess, u_sol_guess) per problem:
 *                             Safe MPC with the VBOC network as terminal constraint (VBOC/Safe MPC/
 *                             triplependulum_class_vboc.py:91-240; drivers hard_terminal_constraints/3dof_sym.py)
 *   vboc_mpc_soft_solve_batch <- one OCPtriplependulumSoftTraj.OCP_solve(...) per problem (:242-304; drivers
 *                             soft_traj_constraints/3dof_sym.py, receiding_hard_constraints/3dof_sym.py)
 *   vboc_al_solve_batch    <- one OCPtriplependulumINIT.compute_problem(q0, v0) per problem: the active-learning
 *                             labelling OCP (AL/triplependulum_class_al.py:148-169, fanned out by testing(s0) of
 *                             AL/triplependulum_al.py:24-42 at :133, :284)
 *   vboc_set_path_constraint <- model.con_h_expr + constraints.lh / uh of the Cartesian double pendulum
 *                             (VBOC/Cartesian constraints/doublependulum_class_fixedveldir.py:154-160)
 *   vboc_destroy           <- solver object destruction (acados_template __del__ -> free)
 *   vboc_last_error        <- Python exceptions raised by acados_template on bad fields
 *
 * Problem layout (problem-major, exactly the numpy arrays the reference passes, float64):
 *   nq = number of links (1 pendulum, 2 double, 3 triple) or 4 = the UR5 arm of
 *   VBOC/UR5/ur5reduced_class_fixedveldir.py (4 revolute joints of ur5.urdf, rigid-body dynamics);
 *   nx = 2*nq+1 (theta, dtheta, dt); nu = nq; np = nq+1 (w_1..w_nq, w_t).
 *   The UR5 OCP has no dt state (x = [q, qdot], p = w, tf = 1 over N = 100 intervals): its shooting
 *   interval (set_new_time_steps, dt_sym = 1e-2) travels in the dt column, and p[nq] = 0.  Its
 *   OCPUR5INIT.OCP_solve (:145-192) is otherwise the same boundary problem; levenberg_marquardt defaults
 *   to 1e-2 on an nq = 4 handle (:131).  nq = 4 runs on the wave solver (k_wave<4>,
 *   the default) or the lane-per-problem kernels (wave_all = 0); it has no free-time variant.
 *   N[b]                 horizon of problem b (<= nmax of the handle)
 *   x_guess[b][nmax+1][nx]  stage guesses; row N[b] is the stage-N guess (OCP_solve sets it from
 *                        x_sol_guess[-1], triplependulum_class_vboc.py:185)
 *   u_guess[b][nmax][nu]
 *   p[b][np]             cost parameters (stage-0 cost w.dtheta + wt.dt, :85-86)
 *   lbx/ubx[b][nx]       path state bounds q_lb/q_ub       (:165-166)
 *   lbu/ubu[b][nu]       control bounds u_lb/u_ub          (:167-168)
 *   lbx_0/ubx_0[b][nx]   stage-0 bounds q_init_lb/ub       (:180-181)
 *   lbx_e/ubx_e[b][nx]   terminal bounds q_fin_lb/ub       (:183-184)
 *   The stage-0 general constraint C = [0 | I - d d^T | 0], d = p[:nq], lg = ug = 0 (:174-178) is
 *   implied (as in OCP_solve).  Requirements, checked per problem: dt fixed (lb == ub on the dt
 *   column everywhere), stage-0 positions fixed, terminal velocities fixed, 1 <= N[b] <= nmax;
 *   a problem outside them gets status 5 and is not solved.
 * Outputs:
 *   status[b]            0 success, 1 NaN, 2 max iter, 4 QP failure (ACADOS codes),
 *                        5 unsupported problem structure
 *   x_out[b][nmax+1][nx], u_out[b][nmax][nu]  solution (rows beyond N[b] untouched)
 *   cost[b]              NLP cost at the solution (= get_cost())
 *   sqp_iter[b], qp_iter[b]  iteration counters (qp_iter summed over SQP iterations)
 *
 * Return value of every call: 0 on success, a negative VBOC_ERR_* code otherwise; the message is
 * available from vboc_last_error().
 */
#ifndef VBOC_H
#define VBOC_H

#ifdef __cplusplus
extern "C" {
#endif

#define VBOC_OK 0
#define VBOC_ERR_ARG (-1)
#define VBOC_ERR_HIP (-2)
#define VBOC_ERR_UNSUPPORTED (-3)
#define VBOC_ERR_NOMEM (-4)

typedef struct vboc_solver* vboc_handle;

typedef struct {
  int B;                 /* number of problems */
  int nmax;              /* leading horizon dimension of x_guess/u_guess/x_out/u_out */
  const int* N;
  const double* x_guess;
  const double* u_guess;
  const double* p;
  const double* lbx;
  const double* ubx;
  const double* lbu;
  const double* ubu;
  const double* lbx_0;
  const double* ubx_0;
  const double* lbx_e;
  const double* ubx_e;
  int* status;
  double* x_out;
  double* u_out;
  double* cost;
  int* sqp_iter;
  int* qp_iter;
} vboc_batch_t;

/* Create a solver for nq links (4 = UR5) with horizons up to nmax on HIP device `device`.  `slots` is the
 * number of concurrently resident problems (lanes) of the persistent kernel; 0 = default. */
int vboc_create(int nq, int nmax, int slots, int device, vboc_handle* out);
int vboc_destroy(vboc_handle h);

/* Solver options (names of AcadosOcpOptions): "nlp_solver_tol_stat", "nlp_solver_tol_eq",
 * "nlp_solver_tol_ineq", "nlp_solver_tol_comp", "nlp_solver_max_iter", "qp_solver_iter_max",
 * "qp_solver_tol_stat", "qp_solver_tol_eq", "qp_solver_tol_comp", "levenberg_marquardt",
 * "alpha_min", "alpha_reduction"; interior-point internals "ipm_mu0", "ipm_push", "ipm_tau";
 * scheduling: "wave_groups" (resident problems of the wave solver, 0 = automatic) and "mall_mib"
 * (automatic sizing: the resident problems' hot stage records fit this much Infinity Cache, default
 * 256); data-generation scheduling, none of which changes a result: "dg_park", "dg_park_window",
 * "dg_speculate", "dg_spec_window", "dg_spec_first" (default 2 = automatic: on for launches of fewer than 128
 * problems per resident wave), "dg_spec_crit" (INTEGRATION.md section 2).  Test-only: "dg_fail_mod" (> 0: vboc_data_generation reports status 4 for every solve whose
 * initial position q_0 has int(|q_0| 1e6) % dg_fail_mod == 0, exercising the restart branches). */
int vboc_set_option(vboc_handle h, const char* field, double value);
int vboc_get_option(vboc_handle h, const char* field, double* value);

/* Nonlinear path constraint of the OCP (an OCP-level definition, like ACADOS's con_h_expr / lh / uh):
 *   kind 1: end-effector keep-out circle of the pendulum chain (nq 2 or 3, link length 0.8),
 *           lh <= (sum_j l sin theta_j - x_c)^2 + (sum_j l cos theta_j - y_c)^2 <= uh
 *           on stages 0..N-1 (VBOC/Cartesian constraints/doublependulum_class_fixedveldir.py:154-160);
 *           at stage 0 the positions are fixed, so a problem whose initial position violates it gets
 *           status 4 (QP failure) without iterating;
 *   kind 0: no path constraint (the default).
 * Solves with the constraint run on the wave solver for nq = 2 (k_wave with the constraint rows; option
 * "hc_wave" = 0 or wave_all = 0: the lane-per-problem kernels) and on the lane kernels for nq = 3; the free-time solver and vboc_data_generation refuse a handle
 * that carries one (VBOC_ERR_UNSUPPORTED). */
int vboc_set_path_constraint(vboc_handle h, int kind, double x_c, double y_c, double lh, double uh);

/* Batched solve, every pointer a DEVICE pointer (inputs resident in HBM).  Kernels are enqueued on
 * `stream`; the call returns when every problem of the batch is finished (the SQP/IPM loops are
 * host-driven and poll a device counter on that stream). */
int vboc_solve_batch(vboc_handle h, const vboc_batch_t* batch, void* stream);
/* Same with HOST pointers: staged through the handle's device buffers; synchronous. */
int vboc_solve_batch_host(vboc_handle h, const vboc_batch_t* batch);

/* Free-time box OCP (OCP<sys>.OCP_solve with dt a decision state; the pendulum's
 * OCPpendulum.OCP_solve(x_guess, u_guess, cost_dir, q_lb, q_ub, q_init, q_fin),
 * VBOC/pendulum_class_vboc.py:107-130, called from VBOC/pendulum_vboc.py:94,181).  Same batch
 * layout; the semantics differ from vboc_solve_batch:
 *   x_k = [theta, dtheta, dt] with dt a state (dt_{k+1} = dt_k), RK4 with h = dt per interval;
 *   cost p[:nq] . dtheta_0 + p[nq] * sum_{k<N} dt_k  (EXTERNAL cost, :70-74);
 *   stage 0: components with lbx_0 == ubx_0 fixed, others boxed; stages 1..N-1: boxes lbx/ubx (every
 *   component must have lb < ub) and lbu/ubu; stage N: components with lbx_e == ubx_e are equality
 *   constraints, others boxed; no general constraint.  Anything else: status 5.
 * vboc_solve_batch_ft enqueues ONE kernel on `stream` and returns without waiting (device pointers);
 * the _host variant is synchronous. */
int vboc_solve_batch_ft(vboc_handle h, const vboc_batch_t* batch, void* stream);
int vboc_solve_batch_ft_host(vboc_handle h, const vboc_batch_t* batch);

/* Twin integrator: one ERK4 step of length T of the unscaled 2nq-state model for B states.
 * x[B][2nq], u[B][nq] -> x_out[B][2nq].  Device pointers (async) / host pointers (sync). */
int vboc_rk4_batch(int nq, int B, double T, const double* x, const double* u, double* x_out, void* stream);
int vboc_rk4_batch_host(int nq, int B, double T, const double* x, const double* u, double* x_out);
/* The solvers' linearisation, standalone: one ERK4 step of length T with its forward sensitivities
 * (ACADOS ERK forward VDE, the shooting Jacobians of every SQP iteration) for B states, host pointers:
 * x[B][2nq], u[B][nq] -> x_out[B][2nq], A[B][2nq][2nq] = dx_out/dx, Bm[B][2nq][nq] = dx_out/du. */
int vboc_rk4_sens_batch_host(int nq, int B, double T, const double* x, const double* u, double* x_out, double* A,
                             double* Bm);

/* Batched data generation ON THE DEVICE (nq = 2 or 3): for every problem id, the reference's
 * `data_generation(v)` - IC sampling (Philox4x32-10 keyed by (seed, id), streams 0 and 2 of
 * vboc_amd/ics.py), horizon extension (<= 10 solves, perturbed restarts), the sweep along the optimal
 * trajectory with the twin RK4 steps and the verification solves (<= 5 per exit of the state box),
 * the save filter.  One wave runs one problem's whole state machine with the wave solver in between
 * (dg.h).  Device pointers except rows_used; synchronous (returns when every problem finished).
 *   ids[B]              problem ids (int64)
 *   q_min .. m2         system constants (vboc_amd/systems.py; the double's gravity guess uses g, l, m)
 *   rows[rows_cap][2nq] saved samples, one contiguous block per problem (blocks in completion order)
 *   row_off[B], row_cnt[B]  block of problem b; row_cnt -1 = the reference returns None
 *   ic[B][4], ic_slot[B]    double pendulum store_ic and its tuple position (1 success, 2 failure);
 *                       may be NULL for the triple
 *   stats[B][13]        OCP solves, twin steps, SQP iterations, sum N*sqp_iter, sum N*qp_iter, start and
 *                       end time of the problem on its wave (device real-time clock, 100 MHz ticks), the
 *                       first solve's status and SQP iterations, and when a wave took the problem's last job
 *                       (its start, or its resume when its first solve was parked), and how many of its
 *                       solves were speculative restarts solved by other waves, the ticks it waited for them and
 *                       the sum over them of (job start - the chain's first failure)
 *   rows_used           OUT: rows written
 *   spec_solves, spec_used  OUT: speculative restarts (below)
 * Requires N_start + 12 <= nmax of the handle.
 * Speculative restarts (solver option "dg_speculate", default 1): when a horizon-extension solve fails, the
 * inputs of the problem's later attempts (perturbed restarts, up to 10 attempts) are known in advance, so
 * other waves solve them in parallel and the problem takes the results in order; results are identical to
 * the sequential chain.  Only solves the problem consumes count in stats.  They run on waves the problem queue
 * no longer feeds; solver option "dg_spec_early" = n (default 0) lets queued restart jobs go before new problems
 * once at most n problems are left (measured: no gain at n = 5 % of the queue, -10 % when always on).  Solver
 * option "dg_spec_window" = w (default 0 = off, 0..9): the w attempts after the one the problem is solving go before
 * every new or parked problem (a chain that succeeds early wastes at most w solves). */
typedef struct {
  int B;
  const long long* ids;
  unsigned long long seed;
  int N_start;
  double q_min, q_max, v_max, u_max, dt, tol, eps, g, l1, l2, m1, m2;
  double* rows;
  long long rows_cap;
  long long* row_off;
  int* row_cnt;
  double* ic;
  int* ic_slot;
  double* stats;
  long long rows_used;
  long long spec_solves;   /* OUT: speculative restart solves run by other waves */
  long long spec_used;     /* OUT: of them, taken by their problem (the rest is extra work, never counted) */
} vboc_dg_batch_t;
int vboc_data_generation(vboc_handle h, vboc_dg_batch_t* batch, void* stream);
/* The same launch, returning once it is queued on `stream` (the VBOC loop's streaming producer,
 * vboc_amd/pipeline.py): done_flag[B] (device ints, zeroed by the caller; may be NULL) gets 1 for each problem
 * once its rows, row_off, row_cnt, ic and stats are in memory - a system-scope release, so a copy or kernel on
 * another stream may read that problem's results while the launch runs; cancel (a device int, may be NULL),
 * set by the caller while the launch runs, makes the problems not yet started return at once with
 * row_cnt -3.  vboc_data_generation_wait ends the launch (synchronises `stream`, fills rows_used and the
 * speculation counts, reports pool overflow).  No other call may use the handle in between: the solve, testing,
 * data-generation, HJR and option entry points return VBOC_ERR_ARG on a handle with an un-waited launch, and
 * vboc_destroy synchronises the device before it frees the launch's buffers.
 * Replaces the reference's synchronous Pool(30).map per VBOC iteration (VBOC/triplependulum_vboc.py:493-506)
 * by one producer over every iteration's problems. */
int vboc_data_generation_async(vboc_handle h, vboc_dg_batch_t* batch, int* done_flag, const int* cancel,
                               void* stream);
int vboc_data_generation_wait(vboc_handle h, vboc_dg_batch_t* batch, void* stream);

/* The held-out set's testing(v) on the device (replaces Pool(...).map(testing, range(P)) over
 * triplependulum_testdata.py:9-125 / doublependulum_testdata.py:9-121, the a10 driver): one wave per problem runs the
 * draws (Philox stream 1, restarts stream 3), the horizon extension with the '{:.3f}' / '{:.4f}' rounded stop rule
 * and the perturbed restarts (at most max_restarts; the reference retries forever).  b: as vboc_data_generation,
 * with rows_cap >= B; row b of rows is problem b's x0[:2nq] (row_cnt[b] 1), or row_cnt[b] = -1 for None; ic,
 * ic_slot unused.  Synchronous on `stream`. */
int vboc_testing(vboc_handle h, vboc_dg_batch_t* b, int max_restarts, void* stream);

/* testing_test(v) on the device: the UR5 arm's (VBOC/UR5/vboc_multiprocessing_ur5.py:369-466, nq = 4) and the Cartesian
 * double pendulum's (VBOC/Cartesian constraints/vboc_multiprocessing.py:19-129, nq = 2 on a handle with the keep-out
 * circle) per-problem driver, the Pool(30).map fan-outs of their main blocks (:487-528; :557-585).  One wave per
 * problem: draws from Philox stream draw_stream (ids are the keys), p = r_j choice_j / norm, q0 = xlo + u (xhi - xlo),
 * then the horizon grows from N_start while the cost drops by more than tol; a failed solve gives None. */
typedef struct {
  int B;
  const long long* ids;     /* device, int64 [B] */
  unsigned long long seed;
  int N_start;
  int draw_stream;          /* vboc_amd.ics: UR5 5, Cartesian 6 */
  double tol, dt;           /* the stop rule's tol (nlp_solver_tol_stat), the pinned time step */
  double xlo[8], xhi[8];    /* state box [q, qdot] (2nq entries) */
  double ulim[4];           /* |u| <= ulim (nq entries) */
  double* rows;             /* device [B][2nq + 1]: x0 with the dt column (row_cnt 1) */
  int* row_cnt;             /* device [B]: 1, or -1 for None */
  double* stats;            /* device [B][13]: as vboc_dg_batch_t.stats */
} vboc_tt_batch_t;

int vboc_testing_test(vboc_handle h, vboc_tt_batch_t* b, void* stream);

/* The HJR one-step OCP, OCP<sys>.compute_problem(x0) of HJR/<sys>_hjr_class.py (triplependulum_hjr_class.py:
 * 117-134 with the model and options of :7-115), for every x0 of a batch, one problem per GPU lane (hjr.h):
 * x0 fixed, N = 1, h = 1e-2, u0 in [-u_max, u_max], terminal cost = logit 0 of NeuralNetCLS(2nq, hidden, 2)
 * ((x - mean) / std, Linear, ReLU, Linear, ReLU, Linear; my_nn.py:4-18, built by nn_decisionfunction :135-152),
 * the classes' SQP options (ACADOS default tolerances).  Device pointers; asynchronous on `stream`.
 *   x0[B][2nq]; W0[hidden][2nq], b0[hidden], W1[hidden][hidden], b1[hidden], W2[2][hidden], b2[2] (FP64 copies of
 *   model.parameters()); status[B] (compute_problem returns status == 0), cost[B] (get_cost: the network's
 *   logit 0 at x1), u[B][nq], x1[B][2nq], sqp_iter[B], qp_iter[B].  hidden must be 100 (the reference's). */
typedef struct {
  int B, hidden;
  const double* x0;
  const double *W0, *b0, *W1, *b1, *W2, *b2;
  double mean, std, u_max;
  int* status;
  double* cost;
  double* u;
  double* x1;
  int* sqp_iter;
  int* qp_iter;
} vboc_hjr_batch_t;
int vboc_hjr_solve_batch(vboc_handle h, const vboc_hjr_batch_t* batch, void* stream);

/* Safe MPC with the VBOC network as terminal constraint: OCPtriplependulumHardTerm.OCP_solve(x0, x_sol_guess,
 * u_sol_guess) (VBOC/Safe MPC/triplependulum_class_vboc.py:163-181; the OCP :91-161, the row :197-240) for every
 * x0 of a batch, one problem per wave (ft.h, the free-time solver with the tracking cost and the terminal row):
 * model MODELtriplependulum on N intervals of h = time_step; LINEAR_LS cost 1/2 |[x; u] - yref|^2_W (stages,
 * times cost_scale) + 1/2 |x_N - yref_e|^2_We, Gauss-Newton Hessian; x_0 fixed; path boxes lbx/ubx, lbu/ubu,
 * terminal box lbx_e/ubx_e; row lh <= NN(x_N) - max(|x_N[2:]|, 1e-3) <= uh with NeuralNetDIR(2nq, hidden, 1)
 * (hidden 0: no row); rti 1 = SQP_RTI (one QP, the full step; status 0 or 4), 0 = SQP with the handle's options.
 * Device pointers except the OCP's constant vectors W, We, yref, yref_e (host); asynchronous on `stream`.  The
 * handle: nq = 3, nmax >= N.
 *   x0[B][2nq], x_guess[B][N+1][2nq], u_guess[B][N][nq]; lbx..ubx_e [2nq] / [nq], W[3nq], We[2nq], yref[3nq],
 *   yref_e[2nq]; W0[hidden][2nq], b0[hidden], W1[hidden][hidden], b1[hidden], W2[hidden], b2[1] (FP64 copies of
 *   model.parameters()); outputs status[B], x_out[B][N+1][2nq], u_out[B][N][nq], cost[B], sqp_iter[B],
 *   qp_iter[B], h_out[B] (the row at the result's x_N; may be NULL).  hidden <= 512. */
typedef struct {
  int B, N, rti, hidden;
  double h, cost_scale;
  const double *x0, *x_guess, *u_guess;
  const double *lbx, *ubx, *lbu, *ubu, *lbx_e, *ubx_e;
  const double *W, *We, *yref, *yref_e;   /* host */
  const double *W0, *b0, *W1, *b1, *W2, *b2;
  double mean, std, lh, uh;
  int* status;
  double* x_out;
  double* u_out;
  double* cost;
  int* sqp_iter;
  int* qp_iter;
  double* h_out;
} vboc_mpc_batch_t;
int vboc_mpc_solve_batch(vboc_handle h, const vboc_mpc_batch_t* batch, void* stream);

/* The soft-constraint Safe MPC: OCPtriplependulumSoftTraj.OCP_solve(x0, x_sol_guess, u_sol_guess) (VBOC/Safe MPC/
 * triplependulum_class_vboc.py:242-304) for every x0 of a vboc_mpc_batch_t: the row
 * nn_decisionfunction_conservative = NN(x) (100 - safety_margin) / 100 - max(|x[2:]|, 1e-3) on EVERY stage 0..N
 * (con_h_expr and con_h_expr_e), each soft on its lower side (idxsh / idxsh_e) with a slack s_k >= 0 costing
 * c_k (zl_k s_k + Zl_k s_k^2 / 2), c_k = cost_scale on stages 0..N-1 and 1 at N (ACADOS' cost_scaling scales a
 * stage's slack weights with its least-squares weights) - zl / Zl the per-stage weights the drivers set with
 * ocp_solver.cost_set(i, "Zl", ...)
 * (soft_traj_constraints/3dof_sym.py:102-105, receiding_hard_constraints/3dof_sym.py:41-46); the upper side
 * (uh = 1e6, zu = Zu = 0) is never active and kept hard.  W_b / We_b: each problem's stage weights, the receding
 * driver's cost_set(i, "W", block_diag(Q, R)) / cost_set(N, "W", Q) (:36-40; NULL: the batch's host W / We).  Device
 * pointers: Zl [B][N+1] (required), zl [B][N+1] (NULL = 0), W_b [B][3nq], We_b [B][2nq].  hidden > 0 required. */
typedef struct {
  double safety_margin;
  const double* Zl;
  const double* zl;
  const double* W_b;
  const double* We_b;
} vboc_mpc_soft_t;
int vboc_mpc_soft_solve_batch(vboc_handle h, const vboc_mpc_batch_t* batch, const vboc_mpc_soft_t* soft,
                              void* stream);

/* Active learning's labelling OCP: OCPtriplependulumINIT.compute_problem(q0, v0) (AL/triplependulum_class_al.py:
 * 148-169; the OCP :82-144 with the terminal rest of :204-222) for every x0 = (q0, v0) of a batch, on the Safe-MPC
 * solver (ft.h) with ACADOS' default options (SQP_RTI, Gauss-Newton, levenberg_marquardt 0, qp_solver_iter_max 50
 * - the handle's options): reset (u = 0, multipliers 0), x_0 fixed, every stage's x guess (q0, 0), one QP and its
 * full step.  The QP is the feasibility question the label answers: a QP the interior-point solver does not finish
 * within qp_solver_iter_max (or a factorisation / NaN failure) is status 4.  label[b] = 1 (status 0), 0 (status 4)
 * or 2 (any other status), as compute_problem returns.  LINEAR_LS cost 1/2 |[x; u]|^2_W on stages 0..N-1 (times
 * cost_scale) + 1/2 |x_N|^2_We, yref = 0; path boxes lbx/ubx, lbu/ubu; terminal lbx_e/ubx_e (lb == ub: fixed, the
 * class's zero final velocity).  Device pointers except W [3nq] / We [2nq] (host); asynchronous on `stream`.
 * The handle: nq = 3, nmax >= N.  x0[B][2nq], x_guess (optional, see the struct); outputs label[B], status[B],
 * x_out[B][N+1][2nq] (get(i, "x")), u_out[B][N][nq], qp_iter[B]. */
typedef struct {
  int B, N;
  double h, cost_scale;
  const double* x0;
  const double* x_guess;  /* [B][N+1][2nq] or NULL: compute_problem's (q0, 0) at every stage; compute_problem_nnguess
                             (:171-201) passes the guess network's trajectory (stage 0 = x0) */
  const double *lbx, *ubx, *lbu, *ubu, *lbx_e, *ubx_e;
  const double *W, *We;   /* host */
  int* label;
  int* status;
  double* x_out;
  double* u_out;
  int* qp_iter;
} vboc_al_batch_t;
int vboc_al_solve_batch(vboc_handle h, const vboc_al_batch_t* batch, void* stream);

/* Device time of the last vboc_solve_batch* call's solver kernel in milliseconds (HIP events on
 * the call's stream) and the number of kernel launches it used. */
int vboc_last_kernel_ms(vboc_handle h, double* ms, int* launches);

/* Dominant-kernel accounting of the last solve (enable with vboc_set_option(h, "profile_kernels", 1)):
 * summed device time of the factorisation-sweep launches (HIP events recorded on the solve's
 * stream around every k_qp_factor launch), their number, and the algorithmic HBM bytes they had
 * to move (lane-stages factorised x bytes per stage; DESIGN.md "Roofline"). */
int vboc_kernel_stats(vboc_handle h, double* factor_ms, long long* factor_launches, double* factor_bytes);

/* Diagnostics: per-phase shader-clock cycles of the wave solver summed over all jobs since the last
 * call (then reset): [0] linearise [1] IPM init [2] H/g preparation [3] factorisation [4] vector
 * passes [5] forward sweeps [6] update [7] costate [8] line search + step, [9] SQP iterations,
 * [10] IPM iterations.  All zero unless the library was built with -DVBOC_COOP_PROF. */
int vboc_debug_counters(unsigned long long* out16);

const char* vboc_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* VBOC_H */

// dg.h - the VBOC data-generation loop ON THE DEVICE, fused with the wave solver.
//
// The reference runs `data_generation(v)` once per problem in a process pool
// (VBOC/triplependulum_vboc.py:19-370, fan-out :399-405; double pendulum VBOC/doublependulum_vboc.py:19-403).
// Each call is a sequential state machine: IC sampling, up to 10 horizon-extension OCP solves (with
// perturbed restarts), then a sweep f = 1..N-1 along the optimal trajectory that either advances the
// "unviable twin" by one RK4 step or, where the trajectory leaves the state box, runs up to 5
// verification OCPs.  Here ONE WAVE RUNS ONE PROBLEM'S WHOLE STATE MACHINE: k_dg pulls problem ids
// from a queue, and between the state machine's steps the same wave runs the wave solver (coop.h) on
// the request it just wrote.  No host round trip, no per-round batching and no per-round tail: a wave
// that finishes a problem pulls the next one, so the launch is bound by throughput plus ONE tail.
//
// The state machine is a restatement of vboc_amd/drivers.py::data_generation_problem (itself pinned bit
// for bit against the reference's own function, tests/test_drivers.py) with the same arithmetic:
//  * random draws: Philox4x32-10 keyed by (seed, problem id) - ics.uniforms stream 0 for the IC
//    sampling, stream 2 for the perturbations, drawn in the reference's call order;
//  * numpy.linalg.norm of a 2- or 3-vector = sqrt(x0*x0 (+) fma chain) (OpenBLAS ddot), reproduced
//    with explicit fma; np.linspace(0, 1, n) = i * (1 / (n - 1)) with the last point 1.0;
//  * every other expression is the Python scalar expression, evaluated left to right WITHOUT
//    contraction (`#pragma clang fp contract(off)` in every function here);
//  * the twin integrator is the same rk4<NQ> (model.h) as vboc_rk4_batch.
// The state lives in a per-workgroup scratch record in HBM (not in registers across the solve, which
// would push the wave kernel past its 256-VGPR budget); every lane executes the scalar logic
// redundantly (uniform control flow), row copies are lane-parallel.
#pragma once

namespace vboc {

struct DgJobs {
  const long long* ids;        // problem ids (Philox keys), one per job
  int count;
  int N_start, nmax;
  int fail_mod;                // test-only failure injection (solver option dg_fail_mod), 0 = off
  int max_restarts;            // testing (k_ts): restarts before a problem gives None (the reference: unbounded)
  double fmt_scale;            // testing (k_ts): 10^d of the stop rule's '{:.df}'.format(cost) (1e3 / 1e4)
  unsigned long long seed;
  // system constants (vboc_amd/systems.py; VBOC/triplependulum_vboc.py:381-393)
  double q_min, q_max, v_max, u_max, dt, tol, eps, g, l1, l2, m1, m2;
  // per-workgroup arrays (the solver's single-problem inputs / outputs are an Inputs batch of one
  // problem per workgroup, indexed by the workgroup: the kernel receives them as a kernel argument like
  // k_wave, so the solver's pointers stay rematerialisable kernarg loads)
  double* xs;                  // [groups][nmax + 1][nx]  x_sol
  double* us;                  // [groups][nmax + 1][nu]  u_sol
  double* vr;                  // [groups][vr_cap][2nq]   saved rows of the running problem
  double* st;                  // [groups][st_doubles]    DgState
  int vr_cap, st_doubles;
  double* rows;                // [rows_cap][2nq] saved samples, one block per problem
  long long rows_cap;
  long long* row_off;          // [count]
  int* row_cnt;                // [count]: number of rows, -1 = None, -2 = row pool overflow
  double* ic;                  // [count][4] double pendulum store_ic (nullptr for the triple)
  int* ic_slot;                // [count] 0: none, 1: tuple element 1 (success), 2: element 2 (failure)
  double* stats;               // [count][DG_NSTAT]
  unsigned* next;              // job counter
  unsigned long long* rows_next;
  unsigned* err;               // [0] pool overflow, [1] horizon > nmax
  unsigned* done;
  // streaming consumers (vboc_data_generation_async): done_flag[job] = 1 once the job's results (rows, row_off,
  // row_cnt, ic, stats) are in memory - a system-scope release store, so a host copy or a kernel on another
  // stream sees them while the launch runs; cancel: a host-written word, set = the jobs not yet started are
  // skipped (row_cnt -3).  Either may be nullptr.
  int* done_flag;
  const int* cancel;
  // speculative restarts (see "Speculative restarts" below); spec_events == 0 switches them off
  int spec_events, spec_stride;   // events in the pool, doubles per event
  int spec_early;                 // once at most this many problems are left unclaimed, queued restart jobs go first
  int spec_first;                 // 1: once the new problems run out, queued restart jobs go before parked resumes
  double* spec;                   // [spec_events][spec_stride]: snapshot header, then DG_SPEC_JOBS results
  int* spec_claim;                // [spec_events][DG_SPEC_JOBS + 1]: 0 free, 1 claimed
  int* spec_done;                 // [spec_events][DG_SPEC_JOBS + 1]: 1 = result written
  int* spec_cancel;               // [spec_events]: 1 = the owner no longer needs the event's results
  int* spec_q;                    // [spec_events * DG_SPEC_JOBS] queue of (event, job) + 1, 0 = not yet written
  unsigned* spec_ev_next;         // event allocator
  unsigned* spec_q_tail;          // queue: entries pushed / popped
  unsigned* spec_q_head;
  unsigned long long* spec_count; // [0] speculative solves run by other waves, [1] of them used
  // the eager window (see "Speculative restarts"): the next spec_window attempts of a chain also go to this queue,
  // which every wave serves before new or parked problems; 0 switches it off
  int spec_window;
  int spec_crit;                  // 1: critical-path rule (a chain's remaining attempts go eager when they would end
                                  //    after the job queues drain at the launch's rate so far)
  unsigned long long* t_launch;   // the launch's first job start (device real-time clock), set by the first wave
  int* spec_eq;                   // [spec_events * DG_SPEC_JOBS] like spec_q
  unsigned* spec_eq_tail;
  unsigned* spec_eq_head;
  // parked first solves (see "Parked first solves" below); park_res == nullptr switches parking off
  double* park_res;               // [count][park_stride]: status, cost, sqp, qp, t0, then x [N + 1][nx + 1], u [N][nu]
  int park_stride;
  int park_window;                // new problems go first while fewer than this many parked problems wait
  int park_hi_it;                 // first solves with >= this many SQP iterations resume first (queue 0)
  int* park_q;                    // [2][count]: queues 0 (high) and 1 of job + 1, 0 = not yet written
  // round gate of a streamed launch (pipeline.StreamedRounds, option dg_round; 0 off): jobs are the rounds' problems
  // in order, round_n per round; a parked resume or queued restart attempt of a round before the next new problem's
  // round goes before that new problem, so the rounds complete in order
  int round_n;
  unsigned* park_tail;            // [2] entries pushed
  unsigned* park_head;            // [2] entries taken
  // early events (the single and double pendulum's k_dg): > 0 - once the new problems have run out, a horizon-extension
  // solve still iterating after this many SQP iterations publishes its chain's later attempts (last, so that the other
  // fields keep their offsets in the triple's kernel)
  int spec_pause;
};

// a horizon extension gives up after 10 solves (VBOC/triplependulum_vboc.py:107): a failure at attempt a
// leaves at most 9 further attempts to speculate on
constexpr int DG_SPEC_JOBS = 9;
constexpr int DG_SPEC_HDR = 48;   // doubles of an event's snapshot header
constexpr int DG_SPEC_RH = 6;     // doubles of a job result's header: status, cost, sqp, qp, start, end (device clock)

// per-problem statistics: OCP solves, twin steps, SQP iterations, sum N*sqp_iter, sum N*qp_iter, and
// the wave's start / end time of the problem (s_memrealtime, 100 MHz constant clock)
// and the first solve's status and SQP iterations, and when a wave took the problem's last job (its start, or
// its resume when it was parked: the last of these over a launch is when the job queues drained), and how many of
// its solves were speculative restarts solved by other waves, the ticks its wave waited for them, and the sum over
// them of (job start - the chain's first failure)
enum : int { DG_SOLVES = 0, DG_RK4, DG_SQP, DG_NSQP, DG_NQP, DG_T0, DG_T1, DG_ST1, DG_IT1, DG_TQ, DG_TAKEN, DG_WAIT, DG_LAG,
             DG_NSTAT };

template <int NQ>
struct DgState {
  int phase, N, ext, joint_sel, vel_sel, f, at_limit, N_test, ver, nrows, rng_pos, solves, rk4s, fail, spec_ev,
      spec_base, resumed, taken, crit;
  double cost, q_init_sel, q_fin_sel, q_init_oth, norm_old, norm_bef, norm_new;
  double sqp, nsqp, nqp, t0, st1, it1, tq, wait, lag, tspec, treq;
  double ran[2], store_ic[4], xsym[2 * NQ];
};

// ------------------------------------------------------------------------------------------------
// Philox4x32-10 (Random123) and the 53-bit uniforms of vboc_amd/ics.py::uniforms
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void philox4x32_10(unsigned (&c)[4], unsigned k0, unsigned k1) {
  UNR for (int r = 0; r < 10; ++r) {
    const unsigned long long p0 = 0xD2511F53ull * c[0];
    const unsigned long long p1 = 0xCD9E8D57ull * c[2];
    const unsigned n0 = (unsigned)(p1 >> 32) ^ c[1] ^ k0;
    const unsigned n2 = (unsigned)(p0 >> 32) ^ c[3] ^ k1;
    c[1] = (unsigned)p1;
    c[3] = (unsigned)p0;
    c[0] = n0;
    c[2] = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}
// draw i of problem `id`'s stream (ics.uniforms(ids, n, seed, stream)[., i])
__device__ __forceinline__ double philox_uniform(long long id, int i, unsigned long long seed, unsigned stream) {
  unsigned c[4] = {(unsigned)(unsigned long long)id, (unsigned)((unsigned long long)id >> 32), (unsigned)(i >> 1),
                   stream};
  philox4x32_10(c, (unsigned)seed, (unsigned)(seed >> 32) ^ 0x5BD1E995u);
  const unsigned a = (i & 1) ? c[2] : c[0], b = (i & 1) ? c[3] : c[1];
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) / 9007199254740992.0;
}

// numpy.linalg.norm of a short float64 vector: sqrt(dot(x, x)), OpenBLAS ddot's FMA chain
template <int n>
__device__ __forceinline__ double np_norm(const double* v) {
  double s = v[0] * v[0];
  UNR for (int i = 1; i < n; ++i) s = fma(v[i], v[i], s);
  return sqrt(s);
}

// Cross-wave data of the speculative restarts (event snapshots, results, flags) is read and written with
// relaxed agent-scope atomics: on gfx950 these bypass the non-coherent per-XCD L2 state (sc1) and need no
// fence.  A release / acquire pair would instead write back / invalidate a whole XCD's L2 on every publish
// and on every poll of a waiting wave, which evicts the resident problems' stage records of every other
// wave on that XCD (measured: +16 s of queue time on the 400k-problem launch).  A writer orders its data
// before its flag with s_waitcnt vmcnt(0) (all of the wave's stores completed); a reader issues its data
// loads only after its flag load returned.
__device__ __forceinline__ void st_coh(double* p, double v) {
  __hip_atomic_store((unsigned long long*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_coh(const double* p) {
  return __longlong_as_double((long long)__hip_atomic_load((unsigned long long*)p, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_flag(int* p, int v) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ld_flag(const int* p) {
  return __hip_atomic_load((int*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Reader side, once per taken result / job (never per poll): a compiler-level barrier after the flag load
// has returned, so no data load of the published block can be scheduled above the poll loop.  The hardware
// side needs nothing more: the data loads are issued only after the flag value is in a register (the loop
// exit depends on it), and the sc1 loads bypass the stale per-XCD L2 state.  A real acquire fence
// (buffer_inv sc1) would invalidate the whole XCD L2 and evict every other wave's stage records there.
__device__ __forceinline__ void after_flag() { __atomic_signal_fence(__ATOMIC_SEQ_CST); }

template <int NQ>
struct Dg {
  static constexpr int NX = 2 * NQ, NXR = NX + 1, NU = NQ, NP = NQ + 1;
  static constexpr bool GRAV = NQ == 2;   // double pendulum: gravity-compensation guesses, 3-tuple result
  enum : int { START = 0, HEXT = 1, VERIF = 2, SWEEP = 3, DONE = 4 };

  const DgJobs& J;
  const Inputs& in;  // the solver's batch: one problem per workgroup, this one at index wg
  const int wg, t;
  DgState<NQ>* s;
  long long pid;
  int job;

  __device__ Dg(const DgJobs& J_, const Inputs& in_, int wg_, int t_) : J(J_), in(in_), wg(wg_), t(t_), pid(0), job(0) {
    s = (DgState<NQ>*)(J.st + (long long)wg * J.st_doubles);
  }

  __device__ __forceinline__ long long row(int r) const { return (long long)wg * (J.nmax + 1) + r; }
  __device__ __forceinline__ double* xg(int r) const { return (double*)in.xg + row(r) * NXR; }
  __device__ __forceinline__ double* ug(int r) const { return (double*)in.ug + ((long long)wg * J.nmax + r) * NU; }
  __device__ __forceinline__ const double* xo(int r) const { return in.xo + row(r) * NXR; }
  __device__ __forceinline__ const double* uo(int r) const { return in.uo + ((long long)wg * J.nmax + r) * NU; }
  __device__ __forceinline__ double* xs(int r) const { return J.xs + row(r) * NXR; }
  __device__ __forceinline__ double* us(int r) const { return J.us + row(r) * NU; }
  __device__ __forceinline__ double* pp() const { return (double*)in.p + (long long)wg * NP; }
  __device__ __forceinline__ double* qlb0() const { return (double*)in.lbx0 + (long long)wg * NXR; }
  __device__ __forceinline__ double* qub0() const { return (double*)in.ubx0 + (long long)wg * NXR; }
  __device__ __forceinline__ double* vr(int n) const { return J.vr + ((long long)wg * J.vr_cap + n) * NX; }
  __device__ __forceinline__ int status() const { return in.status[wg]; }
  __device__ __forceinline__ int nreq() const { return in.N[wg]; }

  // random.random() / random.choice([-1, 1]) of the problem's perturbation stream (ProblemRNG, stream 2)
  __device__ __forceinline__ double rng_random() {
    const int i = s->rng_pos;
    s->rng_pos = i + 1;
    return philox_uniform(pid, i, J.seed, 2u);
  }
  __device__ __forceinline__ static int choice_idx(double u, int n) {
#pragma clang fp contract(off)
    const int v = (int)(u * (double)n);
    return v < n - 1 ? v : n - 1;
  }
  __device__ __forceinline__ double rng_pm1() { return choice_idx(rng_random(), 2) == 0 ? -1.0 : 1.0; }

  // VBOC/doublependulum_vboc.py:84: u = [g l1 (m1 + m2) sin q1, g l2 m2 sin q2]
  __device__ __forceinline__ void grav_u(const double* x, double* u) const {
#pragma clang fp contract(off)
    if constexpr (GRAV) {
      u[0] = J.g * J.l1 * (J.m1 + J.m2) * sin(x[0]);
      u[1] = J.g * J.l2 * J.m2 * sin(x[1]);
    } else {
      UNR for (int a = 0; a < NU; ++a) u[a] = 0.0;
    }
  }
  __device__ __forceinline__ bool vel_out(const double* x) const {
    bool r = false;
    UNR for (int j = 0; j < NQ; ++j) r = r || x[NQ + j] > J.v_max || x[NQ + j] < -J.v_max;
    return r;
  }
  __device__ __forceinline__ bool pos_at_limit(const double* x) const {
#pragma clang fp contract(off)
    bool r = false;
    UNR for (int j = 0; j < NQ; ++j) r = r || x[j] > J.q_max - J.eps || x[j] < J.q_min + J.eps;
    return r;
  }

  // straight-line guess over Nc rows (VBOC/triplependulum_vboc.py:85-93; qpos: positions of the others)
  __device__ __forceinline__ void straight_guess(int Nc, const double* qpos) {
#pragma clang fp contract(off)
    const int js = s->joint_sel;
    const double qi = s->q_init_sel, qf = s->q_fin_sel;
    const double step = 1.0 / (double)(Nc - 1);
    double q[NQ];
    UNR for (int j = 0; j < NQ; ++j) q[j] = qpos[j];
    for (int r = t; r <= Nc; r += 64) {
      const int i = r < Nc ? r : Nc - 1;        // row Nc: the stage-N guess = the last row
      const double tau = (i == Nc - 1) ? 1.0 : (double)i * step;
      double x[NXR];
      UNR for (int j = 0; j < NQ; ++j) { x[j] = q[j]; x[NQ + j] = 0.0; }
      x[NX] = J.dt;
      UNR for (int j = 0; j < NQ; ++j)
        if (j == js) {
          x[j] = (1.0 - tau) * qi + tau * qf;
          x[NQ + j] = 2.0 * (1.0 - tau) * (qf - qi);
        }
      UNR for (int c = 0; c < NXR; ++c) xg(r)[c] = x[c];
      if (r < Nc) {
        double u[NU];
        grav_u(x, u);
        UNR for (int a = 0; a < NU; ++a) ug(r)[a] = u[a];
      }
    }
  }

  // x_guess[:n+1] = src_x[:n+1], u_guess[:n] = src_u[:n], u_guess[n] = gravity(x_guess[n]) | 0; then the
  // horizon grows by one and the stage-(n+1) guess is the last row (x_guess[n + 1] = x_guess[n])
  __device__ __forceinline__ void guess_from(const double* sx, const double* su, int n) {
#pragma clang fp contract(off)
    for (int r = t; r <= n + 1; r += 64) {
      const int rr = r <= n ? r : n;
      UNR for (int c = 0; c < NXR; ++c) xg(r)[c] = sx[(long long)rr * NXR + c];
      if (r < n) {
        UNR for (int a = 0; a < NU; ++a) ug(r)[a] = su[(long long)r * NU + a];
      } else if (r == n) {
        double u[NU];
        grav_u(sx + (long long)n * NXR, u);
        UNR for (int a = 0; a < NU; ++a) ug(r)[a] = u[a];
      }
    }
  }

  __device__ __forceinline__ void request(int N) {
    if (N > J.nmax) {   // cannot happen for N_start + 12 <= nmax (checked on the host)
      if (t == 0) atomicOr(J.err + 1, 1u);
      N = J.nmax;
    }
    ((int*)in.N)[wg] = N;
    s->solves += 1;
    s->treq = (double)__builtin_amdgcn_s_memrealtime();
  }

  // the critical-path rule: at a failed attempt of a chain, the rest of the chain run serially would take
  // (10 - ext) x the attempt's duration; the job queues will drain in about (jobs left) x (elapsed / jobs taken).  If
  // the chain would end after that, its remaining attempts go to the eager queue, once (waves take them before new or
  // parked problems) - the chains that would set the launch's end get help, the ones with time to spare run alone.
  __device__ __forceinline__ void crit_check(int ev) {
    if (!J.spec_crit || J.spec_window > 0 || s->crit || ev < 0) return;   // (the window's pushes are enough)
    const double now = (double)__builtin_amdgcn_s_memrealtime();
    const double dur = now - s->treq;
    int push = 0;
    if (t == 0) {
      const unsigned nx = __hip_atomic_load(J.next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned taken_new = nx < (unsigned)J.count ? nx : (unsigned)J.count;
      unsigned parked_wait = 0, resumed = 0;
      if (J.park_res) {
        UNR for (int q = 0; q < 2; ++q) {
          const unsigned tl = __hip_atomic_load(&J.park_tail[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const unsigned hd = __hip_atomic_load(&J.park_head[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          parked_wait += tl - hd;
          resumed += hd;
        }
      }
      const double left = (double)(J.count - taken_new) + (double)parked_wait;
      const double taken = (double)taken_new + (double)resumed;
      const double t0 = (double)__hip_atomic_load(J.t_launch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const double queue = taken > 0.0 ? left * (now - t0) / taken : 0.0;
      push = (10 - s->ext) * dur > queue ? 1 : 0;
    }
    push = __builtin_amdgcn_readfirstlane(__shfl(push, 0));
    if (!push) return;
    s->crit = 1;
    const int nj = 10 - s->spec_base;
    for (int j = (s->ext + 1) - s->spec_base + 1; j <= nj; ++j) push_eager(ev, j);
  }

  __device__ __forceinline__ void append(const double* x) {
    const int n = s->nrows;
    if (n < J.vr_cap) {
      double* d = vr(n);
      UNR for (int c = 0; c < NX; ++c) d[c] = x[c];
    }
    s->nrows = n + 1;
  }

  // ---- phase START: IC sampling (:32-83) and the first solve ----
  __device__ __forceinline__ bool start(int job_) {
#pragma clang fp contract(off)
    job = job_;
    pid = J.ids[job];
    s->t0 = (double)__builtin_amdgcn_s_memrealtime();
    s->tq = s->t0;
    const double q_min = J.q_min, q_max = J.q_max, v_max = J.v_max, v_min = -J.v_max, eps = J.eps;
    s->phase = HEXT; s->N = J.N_start; s->ext = 0; s->f = 0; s->at_limit = 0; s->N_test = 0; s->ver = 0;
    s->nrows = 0; s->rng_pos = 0; s->solves = 0; s->rk4s = 0; s->fail = 0; s->spec_ev = -1; s->spec_base = 0; s->taken = 0; s->wait = 0.0; s->lag = 0.0; s->crit = 0;
    s->resumed = 0;
    s->sqp = 0.0; s->nsqp = 0.0; s->nqp = 0.0; s->cost = 1e6;
    int di = 0;
    auto draw = [&]() { return philox_uniform(pid, di++, J.seed, 0u); };
    const int js = choice_idx(draw(), NQ);
    const int vs = choice_idx(draw(), 2) == 0 ? -1 : 1;
    s->joint_sel = js;
    s->vel_sel = vs;
    const double qis = vs == -1 ? q_min : q_max, qfs = vs == -1 ? q_max : q_min;
    s->q_init_sel = qis;
    s->q_fin_sel = qfs;
    double r[NQ];
    r[0] = (double)vs * draw();
    UNR for (int k = 1; k < NQ; ++k) {
      const double sg = choice_idx(draw(), 2) == 0 ? -1.0 : 1.0;
      r[k] = sg * draw();
    }
    const double nw = np_norm<NQ>(r);
    double p[NP];
    {
      int c = 1;
      UNR for (int j = 0; j < NQ; ++j) {
        if (j == js) p[j] = r[0] / nw;
        else { p[j] = r[c] / nw; ++c; }
      }
      p[NQ] = 0.0;
    }
    auto clamp_eps = [&](double v) {
      if (v > q_max - eps) v = v - eps;
      if (v < q_min + eps) v = v + eps;
      return v;
    };
    double qpos[NQ];
    if constexpr (GRAV) {
      const double qo = clamp_eps(q_min + draw() * (q_max - q_min));
      s->ran[0] = r[0]; s->ran[1] = r[1];
      s->q_init_oth = qo;
      s->store_ic[0] = (double)(vs + 1 + js); s->store_ic[1] = r[0]; s->store_ic[2] = r[1]; s->store_ic[3] = qo;
      UNR for (int j = 0; j < NQ; ++j) qpos[j] = qo;
    } else {
      UNR for (int j = 0; j < NQ; ++j) qpos[j] = clamp_eps(q_min + draw() * (q_max - q_min));
    }
    const double sel0 = qis == q_min ? q_min + eps : q_max - eps;
    double* P = pp();
    double *lb0 = qlb0(), *ub0 = qub0();
    UNR for (int j = 0; j < NP; ++j) P[j] = p[j];
    UNR for (int j = 0; j < NQ; ++j) {
      lb0[j] = j == js ? sel0 : qpos[j];
      ub0[j] = j == js ? sel0 : qpos[j];
      lb0[NQ + j] = v_min;
      ub0[NQ + j] = v_max;
    }
    lb0[NX] = J.dt; ub0[NX] = J.dt;
    set_bounds();
    straight_guess(J.N_start, qpos);
    request(J.N_start);
    return true;
  }

  // the solve just finished: account it and run the state machine to its next request
  __device__ __forceinline__ int feed(int job_) {
    job = job_;
    pid = J.ids[job];
    const int N = nreq();
    const int it = in.sqp_iter[wg], qit = in.qp_iter[wg];
    if (s->solves == 1) {
      s->st1 = (double)this->status();
      s->it1 = (double)it;
    }
    s->sqp += (double)it;
    s->nsqp += (double)N * (double)it;
    s->nqp += (double)N * (double)qit;
    if (J.fail_mod > 0) {   // tests: status 4 when int(|q_0| 1e6) % fail_mod == 0 (tests/oracle_backend.py)
      const long long q = (long long)(fabs(qlb0()[0]) * 1e6);
      if (q % J.fail_mod == 0) ((int*)in.status)[wg] = 4;
    }
    if (s->solves == 1 && !s->resumed && J.park_res && this->status() == 0 && park_open()) {
      park(it);
      return 3;
    }
    const int more = s->phase == HEXT ? on_hext() : (on_verif() ? 1 : 0);
    if (more) return more;
    return s->phase == SWEEP && sweep() ? 1 : 0;   // one inlined copy of the sweep (with its RK4)
  }

  // one perturbed restart of the horizon extension (:138-174): the cost direction p and the free initial
  // positions (the double: ran, q_init_oth and store_ic) move by <= 0.01, drawn from stream 2
  __device__ __forceinline__ void perturb() {
#pragma clang fp contract(off)
    const double q_min = J.q_min, q_max = J.q_max, eps = J.eps;
    double* P = pp();
    double *lb0 = qlb0(), *ub0 = qub0();
    const int js = s->joint_sel;
    if constexpr (GRAV) {
      double r0 = s->ran[0], r1 = s->ran[1];
      { const double a = rng_random(); const double c = rng_pm1(); r0 = r0 + a * c * 0.01; }
      { const double a = rng_random(); const double c = rng_pm1(); r1 = r1 + a * c * 0.01; }
      double rr[2] = {r0, r1};
      const double nw = np_norm<2>(rr);
      if (js == 0) { P[0] = r0 / nw; P[1] = r1 / nw; }
      else { P[0] = r1 / nw; P[1] = r0 / nw; }
      P[2] = 0.0;
      double qo = s->q_init_oth;
      { const double a = rng_random(); const double c = rng_pm1(); qo = qo + a * c * 0.01; }
      if (qo > q_max - eps) qo = qo - eps;
      if (qo < q_min + eps) qo = qo + eps;
      const int jo = 1 - js;
      lb0[jo] = qo; ub0[jo] = qo;
      s->ran[0] = r0; s->ran[1] = r1; s->q_init_oth = qo;
      s->store_ic[0] = (double)(s->vel_sel + 1 + js); s->store_ic[1] = r0; s->store_ic[2] = r1; s->store_ic[3] = qo;
    } else {
      double rans[NQ];
      UNR for (int k = 0; k < NQ; ++k) {
        const double a = rng_random();
        const double c = rng_pm1();
        rans[k] = P[k] + a * c * 0.01;
      }
      const double nw = np_norm<NQ>(rans);
      UNR for (int k = 0; k < NQ; ++k) P[k] = rans[k] / nw;
      P[NQ] = 0.0;
      const double a = rng_random();
      const double c = rng_pm1();
      const double dev = a * c * 0.01;
      UNR for (int j = 0; j < NQ; ++j) {
        if (j != js) {
          double val = lb0[j] + dev;
          if (val > q_max - eps) val = val - eps;
          if (val < q_min + eps) val = val + eps;
          lb0[j] = val;
          ub0[j] = val;
        }
      }
    }
  }

  // ---- Parked first solves ----
  // A launch ends with its slowest problems, and the slow ones are known after their first solve: in the measured
  // launches every problem longer than 5 s started with a first solve of >= 100 SQP iterations, and 97 % of the
  // 100 slowest with a FAILED first solve (max_iter, the chains of restarts).  So a problem whose first solve
  // succeeded is parked - its first-solve result goes to park_res[job] and the job to a queue - and the wave takes
  // the next new problem, while a failed first solve continues at once.  Once the new problems run out (or
  // park_window problems wait) waves resume parked problems, those with a first solve of >= park_hi_it SQP
  // iterations first: the long problems start early and the last ones to start are short.  Resuming re-runs the
  // deterministic IC sampling of start() and takes the parked result as the first solve, so every problem's
  // results are those of an unparked run (same inputs, same solver; tests/test_dg_device.py).
  __device__ __forceinline__ bool park_open() const {
    // parking only pays while new problems remain (else the wave would resume its own problem at once)
    return __hip_atomic_load(J.next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)J.count;
  }
  __device__ __forceinline__ void park(int it) {
    const int N = nreq();
    double* r = J.park_res + (long long)job * J.park_stride;
    for (int e = t; e < (N + 1) * NXR; e += 64) st_coh(r + 8 + e, xo(0)[e]);
    for (int e = t; e < N * NU; e += 64) st_coh(r + 8 + (N + 1) * NXR + e, uo(0)[e]);
    if (t == 0) {
      st_coh(r, (double)status()); st_coh(r + 1, in.cost[wg]);
      st_coh(r + 2, (double)in.sqp_iter[wg]); st_coh(r + 3, (double)in.qp_iter[wg]);
      st_coh(r + 4, s->t0);
      const int q = it >= J.park_hi_it ? 0 : 1;
      const unsigned pos = atomicAdd(&J.park_tail[q], 1u);
      st_flag(&J.park_q[(long long)q * J.count + pos], job + 1);   // waits for every lane's stores first
    }
    __syncthreads();
  }
  // a parked job: start()'s IC sampling and first request again, then the parked result as its solve
  __device__ __forceinline__ void resume(int job_) {
    start(job_);
    __syncthreads();
    const int N = nreq();
    const double* r = J.park_res + (long long)job * J.park_stride;
    for (int e = t; e < (N + 1) * NXR; e += 64) ((double*)in.xo)[row(0) * NXR + e] = ld_coh(r + 8 + e);
    for (int e = t; e < N * NU; e += 64)
      ((double*)in.uo)[((long long)wg * J.nmax) * NU + e] = ld_coh(r + 8 + (N + 1) * NXR + e);
    if (t == 0) {
      ((int*)in.status)[wg] = (int)ld_coh(r);
      ((double*)in.cost)[wg] = ld_coh(r + 1);
      ((int*)in.sqp_iter)[wg] = (int)ld_coh(r + 2);
      ((int*)in.qp_iter)[wg] = (int)ld_coh(r + 3);
    }
    s->t0 = ld_coh(r + 4);   // the problem's start: its first solve
    s->resumed = 1;
    __syncthreads();
  }

  // ---- Speculative restarts ----
  // A horizon-extension solve that fails (status != 0, in practice max_iter = 1000) is repeated with a
  // perturbed problem, up to 10 attempts in all; the perturbations depend only on the problem's random
  // stream, not on the failed solves, so the inputs of every later attempt - assuming the ones before it
  // fail too - are known as soon as the first failure is.  The slowest problems of a launch are exactly
  // such chains (10 x 1000 SQP iterations in a row on one wave, the launch tail).  At the first failure
  // the owner publishes an event (a snapshot of its restart state) and queues the later attempts as jobs
  // that idle or free waves solve in parallel; the owner walks the chain in order, taking a job's result
  // when another wave solved it and solving it itself otherwise, and cancels the event at the first
  // success.  Results are those of the sequential chain (same inputs, same deterministic solver); unused
  // speculative solves are counted apart (spec_count) and never in the solve statistics.
  enum : int { H_N = 0, H_JS, H_VS, H_QIS, H_QFS, H_RAN, H_QO = H_RAN + 2, H_IC, H_RNG = H_IC + 4, H_PID, H_NJOBS,
               H_TS, H_P, H_LB = H_P + NP, H_UB = H_LB + NXR, H_JOB = H_UB + NXR, H_END };
  static_assert(H_END <= DG_SPEC_HDR, "event header");
  __device__ __forceinline__ double* spec_hdr(int ev) const { return J.spec + (long long)ev * J.spec_stride; }
  __device__ __forceinline__ double* spec_res(int ev, int j) const {
    return spec_hdr(ev) + DG_SPEC_HDR + (long long)(j - 1) * (DG_SPEC_RH + (J.nmax + 1) * NXR + J.nmax * NU);
  }
  __device__ __forceinline__ bool claim(int ev, int j) const {
    int r = 0;
    if (t == 0) r = atomicCAS(&J.spec_claim[ev * (DG_SPEC_JOBS + 1) + j], 0, 1) == 0 ? 1 : 0;
    return __builtin_amdgcn_readfirstlane(__shfl(r, 0)) != 0;
  }
  // early event (spec_pause): the owner's horizon-extension attempt att = ext + 1 has run spec_pause SQP iterations
  // without converging.  Its later attempts depend only on the problem's random stream, so they are published now, as
  // its failure would publish them: spawn(att, N) with the running attempt's own restart state, job j = attempt att + j
  // (spec_prepare perturbs j times from it, as the owner's perturb() at the failure does once).  A success cancels the
  // event; a failure walks the chain from job 1.
  __device__ __forceinline__ bool pause_ok() const { return s->phase == HEXT && s->spec_ev < 0 && s->ext + 1 < 10; }
  __device__ __forceinline__ void early(int job_) {
    job = job_;
    pid = J.ids[job];
    spawn(s->ext + 1, nreq());
  }
  __device__ __forceinline__ void cancel_event() {
    const int ev = s->spec_ev;
    if (ev >= 0 && t == 0) __hip_atomic_store(&J.spec_cancel[ev], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s->spec_ev = -1;
  }
  // publish the restart state of attempt `att` (already perturbed into p / q_init) and queue attempts
  // att + 1 .. 10 as jobs 1 .. 10 - att
  __device__ __forceinline__ void spawn(int att, int N) {
    if (J.spec_events <= 0) return;
    unsigned e = 0;
    if (t == 0) e = atomicAdd(J.spec_ev_next, 1u);
    const int ev = __builtin_amdgcn_readfirstlane(__shfl((int)e, 0));
    if (ev >= J.spec_events) return;   // pool exhausted: this chain runs sequentially
    const int nj = 10 - att;
    double* h = spec_hdr(ev);
    const double *P = pp(), *lb0 = qlb0(), *ub0 = qub0();
    st_coh(h + H_N, N); st_coh(h + H_JS, s->joint_sel); st_coh(h + H_VS, s->vel_sel);
    st_coh(h + H_QIS, s->q_init_sel); st_coh(h + H_QFS, s->q_fin_sel);
    st_coh(h + H_RAN, s->ran[0]); st_coh(h + H_RAN + 1, s->ran[1]); st_coh(h + H_QO, s->q_init_oth);
    UNR for (int c = 0; c < 4; ++c) st_coh(h + H_IC + c, s->store_ic[c]);
    st_coh(h + H_RNG, s->rng_pos); st_coh(h + H_PID, (double)pid); st_coh(h + H_NJOBS, nj);
    st_coh(h + H_TS, (double)__builtin_amdgcn_s_memrealtime());
    st_coh(h + H_JOB, (double)job);
    UNR for (int c = 0; c < NP; ++c) st_coh(h + H_P + c, P[c]);
    UNR for (int c = 0; c < NXR; ++c) { st_coh(h + H_LB + c, lb0[c]); st_coh(h + H_UB + c, ub0[c]); }
    if (t == 0) {
      const unsigned q = atomicAdd(J.spec_q_tail, (unsigned)nj);
      for (int j = 1; j <= nj; ++j) st_flag(&J.spec_q[q + j - 1], ev * (DG_SPEC_JOBS + 1) + j + 1);
    }
    s->spec_ev = ev;
    s->spec_base = att;
    for (int j = 1; j <= J.spec_window && j <= nj; ++j) push_eager(ev, j);
  }
  // job j of event ev to the eager queue (lane 0; the header and the lazy queue entry are already published)
  __device__ __forceinline__ void push_eager(int ev, int j) const {
    if (t == 0) {
      const unsigned q = atomicAdd(J.spec_eq_tail, 1u);
      st_flag(&J.spec_eq[q], ev * (DG_SPEC_JOBS + 1) + j + 1);
    }
  }
  // the owner takes job j's result (solved by another wave) as its own solve of the current attempt
  __device__ __forceinline__ void take_result(int ev, int j, int N) {
    const int* dn = &J.spec_done[ev * (DG_SPEC_JOBS + 1) + j];
    const double tw = (double)__builtin_amdgcn_s_memrealtime();
    while (ld_flag(dn) == 0) __builtin_amdgcn_s_sleep(8);
    after_flag();
    const double* r = spec_res(ev, j);
    s->wait += (double)__builtin_amdgcn_s_memrealtime() - tw;
    s->lag += ld_coh(r + 4) - ld_coh(spec_hdr(ev) + H_TS);
    for (int e = t; e < (N + 1) * NXR; e += 64) ((double*)in.xo)[row(0) * NXR + e] = ld_coh(r + DG_SPEC_RH + e);
    for (int e = t; e < N * NU; e += 64)
      ((double*)in.uo)[((long long)wg * J.nmax) * NU + e] = ld_coh(r + DG_SPEC_RH + (J.nmax + 1) * NXR + e);
    ((int*)in.status)[wg] = (int)ld_coh(r);
    ((double*)in.cost)[wg] = ld_coh(r + 1);
    ((int*)in.sqp_iter)[wg] = (int)ld_coh(r + 2);
    ((int*)in.qp_iter)[wg] = (int)ld_coh(r + 3);
    request(N);
    s->taken += 1;
    if (t == 0) atomicAdd(&J.spec_count[1], 1ull);
    __syncthreads();
  }
  // a free wave runs job j of event ev: the owner's restart state plus j perturbations, straight guess
  __device__ __forceinline__ void spec_prepare(int ev, int j) {
    const double* h = spec_hdr(ev);
    s->tspec = (double)__builtin_amdgcn_s_memrealtime();
    const int N = (int)ld_coh(h + H_N);
    pid = (long long)ld_coh(h + H_PID);
    s->joint_sel = (int)ld_coh(h + H_JS); s->vel_sel = (int)ld_coh(h + H_VS);
    s->q_init_sel = ld_coh(h + H_QIS); s->q_fin_sel = ld_coh(h + H_QFS);
    s->ran[0] = ld_coh(h + H_RAN); s->ran[1] = ld_coh(h + H_RAN + 1); s->q_init_oth = ld_coh(h + H_QO);
    UNR for (int c = 0; c < 4; ++c) s->store_ic[c] = ld_coh(h + H_IC + c);
    s->rng_pos = (int)ld_coh(h + H_RNG);
    double *P = pp(), *lb0 = qlb0(), *ub0 = qub0();
    UNR for (int c = 0; c < NP; ++c) P[c] = ld_coh(h + H_P + c);
    UNR for (int c = 0; c < NXR; ++c) { lb0[c] = ld_coh(h + H_LB + c); ub0[c] = ld_coh(h + H_UB + c); }
    set_bounds();
    for (int k = 0; k < j; ++k) perturb();
    __syncthreads();
    straight_guess(N, qlb0());
    ((int*)in.N)[wg] = N;
  }
  __device__ __forceinline__ void spec_store(int ev, int j) {
    const int N = nreq();
    double* r = spec_res(ev, j);
    for (int e = t; e < (N + 1) * NXR; e += 64) st_coh(r + DG_SPEC_RH + e, xo(0)[e]);
    for (int e = t; e < N * NU; e += 64) st_coh(r + DG_SPEC_RH + (J.nmax + 1) * NXR + e, uo(0)[e]);
    st_coh(r, (double)status()); st_coh(r + 1, in.cost[wg]);
    st_coh(r + 2, (double)in.sqp_iter[wg]); st_coh(r + 3, (double)in.qp_iter[wg]);
    st_coh(r + 4, s->tspec); st_coh(r + 5, (double)__builtin_amdgcn_s_memrealtime());
    if (t == 0) {
      st_flag(&J.spec_done[ev * (DG_SPEC_JOBS + 1) + j], 1);
      atomicAdd(&J.spec_count[0], 1ull);
    }
  }

  // the bounds every OCP_solve of data_generation passes (:381-393)
  __device__ __forceinline__ void set_bounds() {
    const double q_min = J.q_min, q_max = J.q_max, v_max = J.v_max, v_min = -J.v_max;
    double* lbx = (double*)in.lbx + (long long)wg * NXR; double* ubx = (double*)in.ubx + (long long)wg * NXR;
    double* lbxe = (double*)in.lbxe + (long long)wg * NXR; double* ubxe = (double*)in.ubxe + (long long)wg * NXR;
    double* lbu = (double*)in.lbu + (long long)wg * NU; double* ubu = (double*)in.ubu + (long long)wg * NU;
    UNR for (int j = 0; j < NQ; ++j) {
      lbx[j] = q_min; ubx[j] = q_max; lbx[NQ + j] = v_min; ubx[NQ + j] = v_max;
      lbxe[j] = q_min; ubxe[j] = q_max; lbxe[NQ + j] = 0.0; ubxe[NQ + j] = 0.0;
      lbu[j] = -J.u_max; ubu[j] = J.u_max;
    }
    lbx[NX] = J.dt; ubx[NX] = J.dt; lbxe[NX] = J.dt; ubxe[NX] = J.dt;
  }

  // ---- horizon extension (:105-174) ----
  // returns 0: no solve pending (sweep or done), 1: solve the request, 2: the request's result is in place
  __device__ __forceinline__ int on_hext() {
#pragma clang fp contract(off)
    const int status = this->status();
    const double q_min = J.q_min, q_max = J.q_max, eps = J.eps;
    int N = s->N;
    s->ext += 1;
    if (status == 0) {
      cancel_event();   // a success ends the chain of failed attempts the event speculated on
      const double cost_new = in.cost[wg];
      if (cost_new > s->cost - J.tol) {
        sweep_init();
        return false;
      }
      s->cost = cost_new;
      guess_from(xo(0), uo(0), N);
      N = N + 1;
      s->N = N;
    } else {
      perturb();
      __syncthreads();
      s->cost = 1e6;
      if (s->ext < 10) {
        // the next attempt (ext + 1) repeats with perturbed p / q_init: speculate on the ones after it
        const int att = s->ext + 1;
        const int ev = s->spec_ev;
        const int j = att - s->spec_base;
        if (ev >= 0 && j >= 1 && j <= DG_SPEC_JOBS && j <= 10 - s->spec_base) {
          // the owner moves on to job j: the eager window moves with it
          if (J.spec_window > 0 && j + J.spec_window <= 10 - s->spec_base) push_eager(ev, j + J.spec_window);
          if (!claim(ev, j)) {            // another wave solves / solved this attempt: take its result
            take_result(ev, j, N);
            return 2;
          }
        } else if (ev < 0) {
          spawn(att, N);
        }
        crit_check(s->spec_ev);
      }
      straight_guess(N, qlb0());
    }
    if (s->ext >= 10) {     // all 10 solves used without an accepted horizon: None
      cancel_event();
      s->fail = 1;
      s->phase = DONE;
      return false;
    }
    request(N);
    return 1;
  }

  // ---- sweep along the optimal trajectory (:177-365) ----
  __device__ __forceinline__ void sweep_init() {
#pragma clang fp contract(off)
    const int N = s->N;
    for (int r = t; r <= N; r += 64) {
      UNR for (int c = 0; c < NXR; ++c) xs(r)[c] = xo(r)[c];
      if (r < N) UNR for (int a = 0; a < NU; ++a) us(r)[a] = uo(r)[a];
    }
    __syncthreads();
    append(xs(0));
    double x[NX];
    const double* P = pp();
    UNR for (int c = 0; c < NX; ++c) x[c] = xs(0)[c];
    UNR for (int j = 0; j < NQ; ++j) x[NQ + j] = x[NQ + j] - J.eps * P[j];
    const bool lim = vel_out(x);
    s->at_limit = lim ? 1 : 0;
    if (!lim) UNR for (int c = 0; c < NX; ++c) s->xsym[c] = x[c];
    s->f = 1;
    s->phase = SWEEP;
  }

  // save filter of the sweep's step f (:362-365)
  __device__ __forceinline__ void save_filter(int f) {
#pragma clang fp contract(off)
    const double* x = xs(f);
    bool ok = true;
    UNR for (int j = 0; j < NQ; ++j) ok = ok && (J.q_min + J.eps < x[j] && x[j] < J.q_max - J.eps);
    UNR for (int j = 0; j < NQ; ++j) ok = ok && fabs(x[NQ + j]) > J.tol;
    if (ok) append(x);
  }

  __device__ __forceinline__ bool sweep() {
#pragma clang fp contract(off)
    const int N = s->N;
    const double eps = J.eps;
    for (int f = s->f; f < N; ++f) {
      if (s->at_limit) {
        double x[NX];
        UNR for (int c = 0; c < NX; ++c) x[c] = xs(f)[c];
        const double nv = np_norm<NQ>(x + NQ);
        UNR for (int j = 0; j < NQ; ++j) x[NQ + j] = x[NQ + j] + eps * x[NQ + j] / nv;
        if (pos_at_limit(xs(f)) || vel_out(x)) {
          s->at_limit = 1;
        } else {
          s->at_limit = 0;
          if (pos_at_limit(xs(f - 1))) break;
          // verification OCP from x_sol[f] (:245-339)
          const int Nt = N - f;
          const double nw = np_norm<NQ>(xs(f) + NQ);
          double* P = pp();
          double *lb0 = qlb0(), *ub0 = qub0();
          UNR for (int j = 0; j < NQ; ++j) {
            P[j] = -xs(f)[NQ + j] / nw;
            lb0[j] = xs(f)[j]; ub0[j] = xs(f)[j];
          }
          P[NQ] = 0.0;
          for (int r = t; r <= Nt; r += 64) {
            const int src = r < Nt ? r + f : N;
            UNR for (int c = 0; c < NXR; ++c) xg(r)[c] = xs(src)[c];
            if (r < Nt) {
              UNR for (int a = 0; a < NU; ++a) ug(r)[a] = us(r + f)[a];
            } else {
              double u[NU];
              grav_u(xs(N), u);
              UNR for (int a = 0; a < NU; ++a) ug(r)[a] = u[a];
            }
          }
          s->norm_old = nw;
          s->norm_bef = 0.0;
          s->ver = 0;
          s->N_test = Nt;
          s->f = f;
          s->phase = VERIF;
          request(Nt);
          return true;
        }
      } else {
        double x1[NX], x0[NX], u0[NU];
        UNR for (int c = 0; c < NX; ++c) x0[c] = s->xsym[c];
        UNR for (int a = 0; a < NU; ++a) u0[a] = us(f - 1)[a];
        rk4<NQ>(J.dt, x0, u0, x1);
        s->rk4s += 1;
        UNR for (int c = 0; c < NX; ++c) s->xsym[c] = x1[c];
        bool lim = vel_out(x1);
        UNR for (int j = 0; j < NQ; ++j) lim = lim || x1[j] > J.q_max || x1[j] < J.q_min;
        s->at_limit = lim ? 1 : 0;
      }
      save_filter(f);
    }
    s->phase = DONE;
    return false;
  }

  // ---- a verification solve finished (:289-339) ----
  __device__ __forceinline__ bool on_verif() {
#pragma clang fp contract(off)
    const int status = this->status();
    const int N = s->N, f = s->f;
    const double eps = J.eps;
    s->ver += 1;
    bool ok_v = false;
    if (status == 0) {
      const double norm_new = np_norm<NQ>(xo(0) + NQ);
      s->norm_new = norm_new;
      if (norm_new < s->norm_bef + J.tol) {
        ok_v = true;
      } else {
        s->norm_bef = norm_new;
        const int Nt = s->N_test;
        guess_from(xo(0), uo(0), Nt);
        s->N_test = Nt + 1;
        if (s->ver < 5) {
          request(Nt + 1);
          return true;
        }
      }
    }
    if (!ok_v) {
      // unresolved: x_sol[f] appended once per later state at a velocity limit (quirk A.3, :333-337)
      for (int r = f; r < N; ++r) {
        bool hit = false;
        UNR for (int j = 0; j < NQ; ++j) hit = hit || fabs(xs(r)[NQ + j]) > J.v_max - eps;
        if (hit) append(xs(f));
      }
      s->phase = DONE;
      return false;
    }
    const double norm_new = s->norm_new;
    if (norm_new > s->norm_old + J.tol) {    // the state is inside V
      for (int r = t; r < N - f; r += 64) {
        UNR for (int c = 0; c < NXR; ++c) xs(r + f)[c] = xo(r)[c];
        UNR for (int a = 0; a < NU; ++a) us(r + f)[a] = uo(r)[a];
      }
      __syncthreads();
      double x[NX];
      UNR for (int c = 0; c < NX; ++c) x[c] = xs(f)[c];
      UNR for (int j = 0; j < NQ; ++j) x[NQ + j] = x[NQ + j] + eps * x[NQ + j] / norm_new;
      if (vel_out(x)) {
        s->at_limit = 1;
      } else {
        s->at_limit = 0;
        UNR for (int c = 0; c < NX; ++c) s->xsym[c] = x[c];
      }
    } else {                                  // the state is on dV
      s->at_limit = 0;
      double x[NX];
      const double* P = pp();
      UNR for (int c = 0; c < NX; ++c) x[c] = xs(f)[c];
      UNR for (int j = 0; j < NQ; ++j) x[NQ + j] = x[NQ + j] - eps * P[j];
      const int jv = s->joint_sel + NQ;
      UNR for (int c = NQ; c < NX; ++c)
        if (c == jv) {
          if (x[c] > J.v_max) x[c] = J.v_max;
          if (x[c] < -J.v_max) x[c] = -J.v_max;
        }
      UNR for (int c = 0; c < NX; ++c) s->xsym[c] = x[c];
    }
    save_filter(f);
    s->f = f + 1;
    s->phase = SWEEP;
    return false;
  }

  // ---- results: the problem's rows into the pool (reference order restored on the host) ----
  __device__ __forceinline__ void finish(int job_) {
    job = job_;
    __syncthreads();
    const int n = s->fail ? -1 : s->nrows;
    long long off = 0;
    int cnt = n;
    if (n > J.vr_cap) {
      cnt = -2;
      if (t == 0) atomicOr(J.err, 1u);
    } else if (n > 0) {
      unsigned long long o = 0;
      if (t == 0) o = atomicAdd(J.rows_next, (unsigned long long)n);
      o = ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(o >> 32)) << 32) |
          (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)o);
      if ((long long)o + n > J.rows_cap) {
        cnt = -2;
        if (t == 0) atomicOr(J.err, 1u);
      } else {
        off = (long long)o;
        const double* src = vr(0);
        for (int e = t; e < n * NX; e += 64) J.rows[off * NX + e] = src[e];
      }
    }
    if (t == 0) {
      J.row_off[job] = off;
      J.row_cnt[job] = cnt;
      if (J.ic) {
        UNR for (int c = 0; c < 4; ++c) J.ic[(long long)job * 4 + c] = GRAV ? s->store_ic[c] : 0.0;
        J.ic_slot[job] = GRAV ? (s->fail ? 2 : 1) : 0;
      }
      double* st = J.stats + (long long)job * DG_NSTAT;
      st[DG_SOLVES] = (double)s->solves;
      st[DG_RK4] = (double)s->rk4s;
      st[DG_SQP] = s->sqp;
      st[DG_NSQP] = s->nsqp;
      st[DG_NQP] = s->nqp;
      st[DG_T0] = s->t0;
      st[DG_T1] = (double)__builtin_amdgcn_s_memrealtime();
      st[DG_ST1] = s->st1;
      st[DG_IT1] = s->it1;
      st[DG_TQ] = s->tq;
      st[DG_TAKEN] = (double)s->taken;
      st[DG_WAIT] = s->wait;
      st[DG_LAG] = s->lag;
    }
    publish(job);
  }
  // a job skipped after the host cancelled the launch: no work, row_cnt -3
  __device__ __forceinline__ void skip(int job_) {
    job = job_;
    if (t == 0) {
      J.row_off[job] = 0;
      J.row_cnt[job] = -3;
      if (J.ic) J.ic_slot[job] = 0;
      double* st = J.stats + (long long)job * DG_NSTAT;
      for (int c = 0; c < DG_NSTAT; ++c) st[c] = 0.0;
    }
    publish(job);
  }
  // every lane's result stores complete (the barrier drains them into L2), then one system-scope release
  // store of the job's done flag (written back past the non-coherent per-XCD L2s), then the finished count
  __device__ __forceinline__ void publish(int job_) {
    __syncthreads();
    if (t == 0) {
      if (J.done_flag) __hip_atomic_store(&J.done_flag[job_], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      atomicAdd(J.done, 1u);
    }
  }
};

// The state machine's steps are inlined into the kernel.  Measured alternatives (hipcc -O3 resource
// usage of k_dg<3, true>, against k_wave<3, true>: 256 VGPRs, 12 B scratch): the steps as noinline calls
// 116-268 B of scratch with SGPR spills inside the solver's loops (a kernel with calls reserves SGPRs and
// must keep values across calls in callee-saved registers); the per-workgroup problem addressed through
// computed pointers instead of a kernel-argument Inputs batch 150-360 B.  Inlined with the kernarg batch:
// 76 B, spilled at the job boundaries, not in the IPM loop.
template <int NQ>
__device__ __forceinline__ bool dg_start(const DgJobs* J, const Inputs* in, int wg, int t, int job) {
  Dg<NQ> D(*J, *in, wg, t);
  return D.start(job);
}
template <int NQ>
__device__ __forceinline__ int dg_feed(const DgJobs* J, const Inputs* in, int wg, int t, int job) {
  Dg<NQ> D(*J, *in, wg, t);
  return D.feed(job);
}
template <int NQ>
__device__ __forceinline__ void dg_resume(const DgJobs* J, const Inputs* in, int wg, int t, int job) {
  Dg<NQ> D(*J, *in, wg, t);
  D.resume(job);
}
template <int NQ>
__device__ __forceinline__ void dg_finish(const DgJobs* J, const Inputs* in, int wg, int t, int job) {
  Dg<NQ> D(*J, *in, wg, t);
  D.finish(job);
}
template <int NQ>
__device__ __forceinline__ void dg_skip(const DgJobs* J, const Inputs* in, int wg, int t, int job) {
  Dg<NQ> D(*J, *in, wg, t);
  D.skip(job);
}
template <int NQ>
__device__ __forceinline__ bool dg_pause_ok(const DgJobs* J, const Inputs* in, int wg, int t) {
  Dg<NQ> D(*J, *in, wg, t);
  return D.pause_ok();
}
template <int NQ>
__device__ __forceinline__ void dg_early(const DgJobs* J, const Inputs* in, int wg, int t, int job) {
  Dg<NQ> D(*J, *in, wg, t);
  D.early(job);
}
template <int NQ>
__device__ __forceinline__ void dg_spec_prepare(const DgJobs* J, const Inputs* in, int wg, int t, int ev, int j) {
  Dg<NQ> D(*J, *in, wg, t);
  D.spec_prepare(ev, j);
}
template <int NQ>
__device__ __forceinline__ void dg_spec_store(const DgJobs* J, const Inputs* in, int wg, int t, int ev, int j) {
  Dg<NQ> D(*J, *in, wg, t);
  D.spec_store(ev, j);
}

// wave-uniform value of lane 0
__device__ __forceinline__ int dg_bcast(int v) { return __builtin_amdgcn_readfirstlane(__shfl(v, 0)); }

// lane 0: take a parked job (queue 0 first), -1 if none is waiting
__device__ __forceinline__ int dg_take_parked(const DgJobs* J) {
  for (int q = 0; q < 2; ++q) {
    unsigned h = __hip_atomic_load(&J->park_head[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (h < __hip_atomic_load(&J->park_tail[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
      if (__hip_atomic_compare_exchange_strong(&J->park_head[q], &h, h + 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)) {
        int e;
        while ((e = ld_flag(&J->park_q[(long long)q * J->count + h])) == 0) __builtin_amdgcn_s_sleep(2);
        after_flag();
        return e - 1;
      }
      // h now holds the current head: retry against it
    }
  }
  return -1;
}
// lane 0: parked jobs waiting (both queues)
__device__ __forceinline__ unsigned dg_parked_waiting(const DgJobs* J) {
  unsigned w = 0;
  for (int q = 0; q < 2; ++q)
    w += __hip_atomic_load(&J->park_tail[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) -
         __hip_atomic_load(&J->park_head[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return w;
}

// lane 0, round gate (J->round_n > 0): a parked job of a round before round r waits at the head of a park queue
__device__ __forceinline__ bool dg_parked_before(const DgJobs* J, unsigned r) {
  for (int q = 0; q < 2; ++q) {
    const unsigned h = __hip_atomic_load(&J->park_head[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (h >= __hip_atomic_load(&J->park_tail[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) continue;
    const int e = ld_flag(&J->park_q[(long long)q * J->count + h]);
    if (e > 0 && (unsigned)(e - 1) / (unsigned)J->round_n < r) return true;
  }
  return false;
}
// lane 0, round gate: the restart attempt at the head of the lazy queue belongs to a chain of a round before round r
template <int NQ>
__device__ __forceinline__ bool dg_restart_before(const DgJobs* J, unsigned r) {
  const unsigned h = __hip_atomic_load(J->spec_q_head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (h >= __hip_atomic_load(J->spec_q_tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return false;
  const int e = ld_flag(&J->spec_q[h]);
  if (e <= 0) return false;
  after_flag();
  const int ev = (e - 1) / (DG_SPEC_JOBS + 1);
  const double job = ld_coh(J->spec + (long long)ev * J->spec_stride + Dg<NQ>::H_JOB);
  return (unsigned)job / (unsigned)J->round_n < r;
}

// one workgroup = one wave: it owns one problem's whole data_generation at a time, or - once the problem
// queue is drained - runs one speculative restart solve for another problem's owner (they shorten the
// chains of failing solves that make the launch tail).  `in` is the Inputs batch of one problem per workgroup (the wave solver works on problem index wg
// of it, as k_wave on a pid), `inp` a device copy of it for the state machine.  A wave with nothing to do
// waits (s_sleep) while other waves' problems may still publish restart jobs, and leaves once every
// problem is finished - an exit every wave reaches.
template <int NQ, bool FM>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WavesPerEu<NQ>::v, WavesPerEu<NQ>::v)))
void k_dg(Work w, Opts o, Inputs in, const Inputs* inp, const DgJobs* J, WaveJobs jb) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int t = (int)threadIdx.x;
  const int wg = (int)blockIdx.x;
  Coop<NQ, FM> C(smem, gptr(jb.regions) + (long long)wg * jb.region_doubles, w, o, t);
  const int count = J->count;
  const bool spec = J->spec_events > 0;
  const bool park = J->park_res != nullptr;
  if (spec && J->spec_crit && t == 0) {
    unsigned long long z = 0;
    __hip_atomic_compare_exchange_strong(J->t_launch, &z, (unsigned long long)__builtin_amdgcn_s_memrealtime(),
                                         __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  for (;;) {
    int mode = 0, idx = 0, ev = 0, jj = 0, code = 0;
    // 0. the eager window: a queued attempt of a running chain that its owner reaches within spec_window attempts
    //    goes before every problem (the failing chains are the launch's critical paths; the window bounds the
    //    solves a chain that succeeds early wastes)
    if (spec && (J->spec_window > 0 || J->spec_crit)) {
      int got = -1;
      if (t == 0) {
        const unsigned h = __hip_atomic_load(J->spec_eq_head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned hh = h;
        if (h < __hip_atomic_load(J->spec_eq_tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) &&
            __hip_atomic_compare_exchange_strong(J->spec_eq_head, &hh, h + 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)) {
          int e;
          while ((e = ld_flag(&J->spec_eq[h])) == 0) __builtin_amdgcn_s_sleep(2);
          after_flag();
          const int ev_ = (e - 1) / (DG_SPEC_JOBS + 1), jj_ = (e - 1) % (DG_SPEC_JOBS + 1);
          if (ld_flag(&J->spec_cancel[ev_]) == 0 &&
              atomicCAS(&J->spec_claim[ev_ * (DG_SPEC_JOBS + 1) + jj_], 0, 1) == 0)
            got = e - 1;
        }
      }
      got = dg_bcast(got);
      if (got >= 0) {
        after_flag();
        ev = got / (DG_SPEC_JOBS + 1);
        jj = got % (DG_SPEC_JOBS + 1);
        dg_spec_prepare<NQ>(J, inp, wg, t, ev, jj);
        mode = 2;
        code = 1;
      }
    }
    // 0. near the end of the problem queue (spec_early), a queued restart job of a running chain goes before a new
    //    problem: the chains that make the launch tail start getting help before the last problems are handed out
    int pre = 0;
    //    With parked first solves (spec_first), the same once the new problems run out: the chains still open
    //    then are the launch's critical paths, and every parked resume after them is short work
    if (mode == 0 && spec && (J->spec_early > 0 || (park && J->spec_first))) {
      if (t == 0) {
        const unsigned nx = __hip_atomic_load(jb.next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool near = (J->spec_early > 0 && nx < (unsigned)count && nx + (unsigned)J->spec_early >= (unsigned)count) ||
                          (park && J->spec_first && nx >= (unsigned)count);
        if (near)
          pre = __hip_atomic_load(J->spec_q_head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
                __hip_atomic_load(J->spec_q_tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      pre = dg_bcast(pre);
    }
    //    Round gate (streamed launches): a restart attempt of an earlier round's chain goes before a later round's new
    //    problem
    if (mode == 0 && spec && !pre && J->round_n > 0) {
      if (t == 0) {
        const unsigned nx = __hip_atomic_load(jb.next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        pre = nx < (unsigned)count && dg_restart_before<NQ>(J, nx / (unsigned)J->round_n);
      }
      pre = dg_bcast(pre);
    }
    // 1. the next problem: a new one, or a parked one once the new ones run out or park_window parked ones wait
    if (mode == 0 && !pre) {
      int got = -1, res = 0;
      if (t == 0) {
        const unsigned nx = __hip_atomic_load(jb.next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool more = nx < (unsigned)count;
        if (park && (!more || dg_parked_waiting(J) >= (unsigned)J->park_window ||
                     (J->round_n > 0 && dg_parked_before(J, nx / (unsigned)J->round_n)))) {
          got = dg_take_parked(J);
          res = got >= 0;
        }
        if (got < 0 && more) {
          const unsigned i = atomicAdd(jb.next, 1u);
          if (i < (unsigned)count) got = (int)i;
        }
        if (got < 0 && park) {
          got = dg_take_parked(J);
          res = got >= 0;
        }
      }
      got = dg_bcast(got);
      res = dg_bcast(res);
      int cancelled = 0;
      if (got >= 0 && J->cancel && t == 0)
        cancelled = __hip_atomic_load(J->cancel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (got >= 0 && dg_bcast(cancelled)) {
        dg_skip<NQ>(J, inp, wg, t, got);
        continue;
      }
      if (got >= 0) {
        idx = got;
        mode = 1;
        if (res) {
          dg_resume<NQ>(J, inp, wg, t, idx);
          code = 2;   // the first solve's result is in place
        } else {
          code = dg_start<NQ>(J, inp, wg, t, idx) ? 1 : 0;
        }
      }
    }
    // 2. no problem left: a queued speculative restart of a chain that is still running (they only run
    //    on waves the problem queue no longer feeds, so they never take throughput from the bulk)
    if (mode == 0 && spec) {
      int got = -1;
      if (t == 0) {
        const unsigned h = __hip_atomic_load(J->spec_q_head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned tl = __hip_atomic_load(J->spec_q_tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned hh = h;
        if (h < tl && __hip_atomic_compare_exchange_strong(J->spec_q_head, &hh, h + 1, __ATOMIC_RELAXED,
                                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
          int e;
          while ((e = ld_flag(&J->spec_q[h])) == 0) __builtin_amdgcn_s_sleep(2);
          after_flag();
          got = e - 1;
        }
      }
      got = dg_bcast(got);
      if (got >= 0) {
        ev = got / (DG_SPEC_JOBS + 1);
        jj = got % (DG_SPEC_JOBS + 1);
        int ok = 0;
        if (t == 0 && ld_flag(&J->spec_cancel[ev]) == 0)
          ok = atomicCAS(&J->spec_claim[ev * (DG_SPEC_JOBS + 1) + jj], 0, 1) == 0 ? 1 : 0;
        if (!dg_bcast(ok)) continue;
        after_flag();
        dg_spec_prepare<NQ>(J, inp, wg, t, ev, jj);
        mode = 2;
        code = 1;
      }
    }
    // 3. nothing to do: leave once every problem is finished, else wait for restart jobs
    if (mode == 0 && pre) continue;   // the restart job went to another wave: back to the problem queue
    if (mode == 0) {
      int fin = 0;
      if (t == 0) fin = __hip_atomic_load(J->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (unsigned)count;
      // without speculation a wave leaves when it finds no work: every parked job was pushed by a wave that then
      // comes back here and takes it (or another one), so no parked job is left without a taker
      if (dg_bcast(fin) || !spec) break;
      __builtin_amdgcn_s_sleep(64);
      continue;
    }
    bool parked = false;
    while (code) {
      if (code == 1) {
        __syncthreads();
        int it = 0, qit = 0;
        Lane<NQ> chk(w, o, 0u);
        if (!chk.supported(in, wg)) {
          if (t == 0) {
            in.status[wg] = 5;
            in.sqp_iter[wg] = 0;
            in.qp_iter[wg] = 0;
          }
        } else {
          C.from_inputs(in, wg);
          // early events (spec_pause): a horizon-extension solve pauses after spec_pause SQP iterations and then every
          // 50; the event is published at the first pause after the new problems have run out (idle waves take its
          // jobs only then, and the event pool is not spent on the bulk's long solves)
          // (the single and double pendulum only: the triple's chains gained nothing from it, DESIGN.md section 14, and
          // its kernel keeps the code of the validated round-6 build)
          int status;
          if constexpr (NQ <= 2) {
            C.pause_at = (mode == 1 && spec && J->spec_pause > 0 && dg_pause_ok<NQ>(J, inp, wg, t)) ? J->spec_pause : -1;
            for (;;) {
              status = C.template run<true>(it, qit);
              if (status != -2) break;
              int drained = 0;
              if (t == 0) drained = __hip_atomic_load(jb.next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (unsigned)count;
              if (dg_bcast(drained)) {
                dg_early<NQ>(J, inp, wg, t, idx);
                C.pause_at = -1;
              } else {
                C.pause_at = it + 50;
              }
            }
          } else {
            status = C.run(it, qit);
          }
          C.store(in, wg, status, it, qit);
        }
        __syncthreads();
      }
      if (mode == 1) {
        code = dg_feed<NQ>(J, inp, wg, t, idx);
        if (code == 3) {   // the first solve succeeded and the problem was parked
          parked = true;
          code = 0;
        }
      } else {
        dg_spec_store<NQ>(J, inp, wg, t, ev, jj);
        code = 0;
      }
    }
    if (mode == 1 && !parked) dg_finish<NQ>(J, inp, wg, t, idx);
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------------
// The held-out set's `testing(v)` ON THE DEVICE (triplependulum_testdata.py:9-125, doublependulum_testdata.py:9-121;
// row a10): the same persistent job loop and wave solver as k_dg, with the testing state machine - a random cost
// direction and initial position, then extend the horizon while the cost still drops (by the stop rule's rounded
// threshold), restarting from a perturbed start on a failed solve.  A restatement of
// vboc_amd/drivers.py::testing_problem (pinned against the reference's own function, tests/test_drivers.py) with
// the same arithmetic: stream 1 for the first draws, stream 3 (TEST_STREAM) for the restarts, Python scalar
// expressions without contraction.  One row x0[:2nq] per problem (row_cnt 1), or None (row_cnt -1) once
// max_restarts restarts have failed.
// ------------------------------------------------------------------------------------------------
template <int NQ>
struct TsState {
  int N, restarts, rng_pos, solves, fail;
  double cost, sqp, nsqp, nqp, t0, st1, it1;
  double rans[NQ], qs[NQ];
};

// float('{:.df}'.format(v)) with scale = 10^d: v scaled exactly (a double-double product), rounded to the
// nearest integer with ties to even on the exact value (Python's correctly rounded formatting), divided back
// (the correctly rounded quotient is the double float() parses from the decimal string)
__device__ __forceinline__ double fmt_round(double v, double scale) {
#pragma clang fp contract(off)
  const double m = fabs(v);
  const double hi = m * scale;
  const double lo = fma(m, scale, -hi);    // m scale = hi + lo exactly
  const double k = floor(hi);
  const double a = hi - k;                 // exact (k <= hi < k + 1), a multiple of ulp(hi) > 2 |lo|
  double n;
  if (a > 0.5 || (a == 0.5 && lo > 0.0)) n = k + 1.0;
  else if (a < 0.5 || (a == 0.5 && lo < 0.0)) n = k;
  else n = fmod(k, 2.0) == 0.0 ? k : k + 1.0;   // an exact tie: to even
  const double r = n / scale;
  return v < 0.0 ? -r : r;
}

template <int NQ>
struct Ts {
  static constexpr int NX = 2 * NQ, NXR = NX + 1, NU = NQ, NP = NQ + 1;
  static constexpr bool GRAV = NQ == 2;   // double pendulum: gravity-compensation guesses
  const DgJobs& J;
  const Inputs& in;
  const int wg, t;
  TsState<NQ>* s;
  long long pid;
  int job;

  __device__ Ts(const DgJobs& J_, const Inputs& in_, int wg_, int t_) : J(J_), in(in_), wg(wg_), t(t_), pid(0), job(0) {
    s = (TsState<NQ>*)(J.st + (long long)wg * J.st_doubles);
  }
  __device__ __forceinline__ long long row(int r) const { return (long long)wg * (J.nmax + 1) + r; }
  __device__ __forceinline__ double* xg(int r) const { return (double*)in.xg + row(r) * NXR; }
  __device__ __forceinline__ double* ug(int r) const { return (double*)in.ug + ((long long)wg * J.nmax + r) * NU; }
  __device__ __forceinline__ const double* xo(int r) const { return in.xo + row(r) * NXR; }
  __device__ __forceinline__ const double* uo(int r) const { return in.uo + ((long long)wg * J.nmax + r) * NU; }
  __device__ __forceinline__ double* pp() const { return (double*)in.p + (long long)wg * NP; }
  __device__ __forceinline__ double* qlb0() const { return (double*)in.lbx0 + (long long)wg * NXR; }
  __device__ __forceinline__ double* qub0() const { return (double*)in.ubx0 + (long long)wg * NXR; }

  __device__ __forceinline__ void grav_u(const double* x, double* u) const {
#pragma clang fp contract(off)
    if constexpr (GRAV) {
      u[0] = J.g * J.l1 * (J.m1 + J.m2) * sin(x[0]);
      u[1] = J.g * J.l2 * J.m2 * sin(x[1]);
    } else {
      UNR for (int a = 0; a < NU; ++a) u[a] = 0.0;
    }
  }
  __device__ __forceinline__ double rng_random() {   // ProblemRNG(pid, stream=TEST_STREAM = 3).random()
    const int i = s->rng_pos;
    s->rng_pos = i + 1;
    return philox_uniform(pid, i, J.seed, 3u);
  }
  __device__ __forceinline__ double rng_pm1() { return Dg<NQ>::choice_idx(rng_random(), 2) == 0 ? -1.0 : 1.0; }

  __device__ __forceinline__ void request(int N) {
    if (N > J.nmax) {
      if (t == 0) atomicOr(J.err + 1, 1u);
      N = J.nmax;
    }
    ((int*)in.N)[wg] = N;
    s->solves += 1;
  }
  __device__ __forceinline__ void set_bounds() {
    const double q_min = J.q_min, q_max = J.q_max, v_max = J.v_max, v_min = -J.v_max;
    double* lbx = (double*)in.lbx + (long long)wg * NXR; double* ubx = (double*)in.ubx + (long long)wg * NXR;
    double* lbxe = (double*)in.lbxe + (long long)wg * NXR; double* ubxe = (double*)in.ubxe + (long long)wg * NXR;
    double* lbu = (double*)in.lbu + (long long)wg * NU; double* ubu = (double*)in.ubu + (long long)wg * NU;
    UNR for (int j = 0; j < NQ; ++j) {
      lbx[j] = q_min; ubx[j] = q_max; lbx[NQ + j] = v_min; ubx[NQ + j] = v_max;
      lbxe[j] = q_min; ubxe[j] = q_max; lbxe[NQ + j] = 0.0; ubxe[NQ + j] = 0.0;
      lbu[j] = -J.u_max; ubu[j] = J.u_max;
    }
    lbx[NX] = J.dt; ubx[NX] = J.dt; lbxe[NX] = J.dt; ubxe[NX] = J.dt;
  }
  // p = direction(rans) (:31-34); start(qs): the stage-0 box and the constant guess (:36-49)
  __device__ __forceinline__ void setup() {
#pragma clang fp contract(off)
    double r[NQ];
    UNR for (int j = 0; j < NQ; ++j) r[j] = s->rans[j];
    const double nw = np_norm<NQ>(r);
    double* P = pp();
    UNR for (int j = 0; j < NQ; ++j) P[j] = r[j] / nw;
    P[NQ] = 0.0;
    double q[NQ];
    UNR for (int j = 0; j < NQ; ++j) q[j] = s->qs[j];
    double *lb0 = qlb0(), *ub0 = qub0();
    UNR for (int j = 0; j < NQ; ++j) {
      lb0[j] = q[j]; ub0[j] = q[j];
      lb0[NQ + j] = -J.v_max; ub0[NQ + j] = J.v_max;
    }
    lb0[NX] = J.dt; ub0[NX] = J.dt;
    double x[NXR], u[NU];
    UNR for (int j = 0; j < NQ; ++j) { x[j] = q[j]; x[NQ + j] = 0.0; }
    x[NX] = J.dt;
    grav_u(x, u);
    const int N = J.N_start;
    for (int rr = t; rr <= N; rr += 64) {
      UNR for (int c = 0; c < NXR; ++c) xg(rr)[c] = x[c];
      if (rr < N) UNR for (int a = 0; a < NU; ++a) ug(rr)[a] = u[a];
    }
    s->N = N;
    s->cost = 1e6;
    request(N);
  }

  __device__ __forceinline__ bool start(int job_) {
#pragma clang fp contract(off)
    job = job_;
    pid = J.ids[job];
    s->t0 = (double)__builtin_amdgcn_s_memrealtime();
    s->restarts = 0; s->rng_pos = 0; s->solves = 0; s->fail = 0;
    s->sqp = 0.0; s->nsqp = 0.0; s->nqp = 0.0; s->st1 = 0.0; s->it1 = 0.0;
    int di = 0;
    auto draw = [&]() { return philox_uniform(pid, di++, J.seed, 1u); };
    UNR for (int j = 0; j < NQ; ++j) {
      const double c = Dg<NQ>::choice_idx(draw(), 2) == 0 ? -1.0 : 1.0;
      s->rans[j] = c * draw();
    }
    UNR for (int j = 0; j < NQ; ++j) s->qs[j] = J.q_min + draw() * (J.q_max - J.q_min);
    set_bounds();
    setup();
    return true;
  }

  // returns 1 when another solve is requested, 0 when the problem is done
  __device__ __forceinline__ int feed(int job_) {
#pragma clang fp contract(off)
    job = job_;
    pid = J.ids[job];
    const int N = in.N[wg];
    const int it = in.sqp_iter[wg], qit = in.qp_iter[wg];
    if (s->solves == 1) {
      s->st1 = (double)in.status[wg];
      s->it1 = (double)it;
    }
    s->sqp += (double)it;
    s->nsqp += (double)N * (double)it;
    s->nqp += (double)N * (double)qit;
    int status = in.status[wg];
    if (J.fail_mod > 0) {   // tests: status 4 when int(|q_0| 1e6) % fail_mod == 0 (tests/oracle_backend.py)
      const long long q = (long long)(fabs(qlb0()[0]) * 1e6);
      if (q % J.fail_mod == 0) status = 4;
    }
    if (status == 0) {
      const double cost_new = in.cost[wg];
      // `cost_new > float('{:.3f}'.format(cost)) - 1e-3` (triple :65-67; the double: 4 decimals and 1e-4, :80-82)
      if (cost_new > fmt_round(s->cost, J.fmt_scale) - (GRAV ? 1e-4 : 1e-3)) return 0;
      if (N + 1 > J.nmax) {   // the extension ran past the handle's horizon capacity: reported to the host
        if (t == 0) atomicOr(J.err + 1, 1u);
        s->fail = 1;
        return 0;
      }
      s->cost = cost_new;
      // the solution becomes the guess of horizon N + 1: rows 0..N, u rows < N, u[N] the gravity guess at x[N]
      for (int r = t; r <= N + 1; r += 64) {
        const int rr = r <= N ? r : N;
        UNR for (int c = 0; c < NXR; ++c) xg(r)[c] = xo(rr)[c];
        if (r < N) {
          UNR for (int a = 0; a < NU; ++a) ug(r)[a] = uo(r)[a];
        } else if (r == N) {
          double u[NU];
          grav_u(xo(N), u);
          UNR for (int a = 0; a < NU; ++a) ug(r)[a] = u[a];
        }
      }
      s->N = N + 1;
      request(N + 1);
      return 1;
    }
    s->restarts += 1;
    if (s->restarts > J.max_restarts) {
      s->fail = 1;
      return 0;
    }
    // a perturbed restart (:41-58): rans, then the initial positions, each by <= 0.01 (stream 3, random()
    // before choice() in `rans[j] + random.random() * random.choice([-1, 1]) * 0.01`)
    UNR for (int j = 0; j < NQ; ++j) {
      const double a = rng_random();
      const double b = rng_pm1();
      s->rans[j] = s->rans[j] + a * b * 0.01;
    }
    UNR for (int j = 0; j < NQ; ++j) {
      const double a = rng_random();
      const double b = rng_pm1();
      s->qs[j] = s->qs[j] + a * b * 0.01;
    }
    setup();
    return 1;
  }

  __device__ __forceinline__ void finish(int job_) {
    job = job_;
    __syncthreads();
    long long off = job;   // one row per problem, in problem order
    if (t == 0) {
      J.row_off[job] = off;
      J.row_cnt[job] = s->fail ? -1 : 1;
      double* st = J.stats + (long long)job * DG_NSTAT;
      st[DG_SOLVES] = (double)s->solves;
      st[DG_RK4] = 0.0;
      st[DG_SQP] = s->sqp;
      st[DG_NSQP] = s->nsqp;
      st[DG_NQP] = s->nqp;
      st[DG_T0] = s->t0;
      st[DG_T1] = (double)__builtin_amdgcn_s_memrealtime();
      st[DG_ST1] = s->st1;
      st[DG_IT1] = s->it1;
      st[DG_TQ] = s->t0;
      st[DG_TAKEN] = 0.0;
      st[DG_WAIT] = 0.0;
      st[DG_LAG] = 0.0;
    }
    if (!s->fail && t < NX) J.rows[off * NX + t] = xo(0)[t];
    __syncthreads();
    if (t == 0) {
      if (J.done_flag) __hip_atomic_store(&J.done_flag[job], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      atomicAdd(J.done, 1u);
    }
  }
};

template <int NQ>
__device__ __forceinline__ bool ts_start(const DgJobs* J, const Inputs* in, int wg, int t, int job) {
  Ts<NQ> T(*J, *in, wg, t);
  return T.start(job);
}
template <int NQ>
__device__ __forceinline__ int ts_feed(const DgJobs* J, const Inputs* in, int wg, int t, int job) {
  Ts<NQ> T(*J, *in, wg, t);
  return T.feed(job);
}
template <int NQ>
__device__ __forceinline__ void ts_finish(const DgJobs* J, const Inputs* in, int wg, int t, int job) {
  Ts<NQ> T(*J, *in, wg, t);
  T.finish(job);
}

// one workgroup = one wave = one held-out problem at a time (k_dg's loop without the speculation)
template <int NQ, bool FM>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WavesPerEu<NQ>::v, WavesPerEu<NQ>::v)))
void k_ts(Work w, Opts o, Inputs in, const Inputs* inp, const DgJobs* J, WaveJobs jb) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int t = (int)threadIdx.x;
  const int wg = (int)blockIdx.x;
  Coop<NQ, FM> C(smem, gptr(jb.regions) + (long long)wg * jb.region_doubles, w, o, t);
  const int count = J->count;
  for (;;) {
    int got = -1;
    if (t == 0 && __hip_atomic_load(jb.next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)count) {
      const unsigned i = atomicAdd(jb.next, 1u);
      if (i < (unsigned)count) got = (int)i;
    }
    got = dg_bcast(got);
    if (got < 0) break;
    int code = ts_start<NQ>(J, inp, wg, t, got) ? 1 : 0;
    while (code) {
      __syncthreads();
      int it = 0, qit = 0;
      Lane<NQ> chk(w, o, 0u);
      if (!chk.supported(in, wg)) {
        if (t == 0) {
          in.status[wg] = 5;
          in.sqp_iter[wg] = 0;
          in.qp_iter[wg] = 0;
        }
      } else {
        C.from_inputs(in, wg);
        const int status = C.run(it, qit);
        C.store(in, wg, status, it, qit);
      }
      __syncthreads();
      code = ts_feed<NQ>(J, inp, wg, t, got);
    }
    ts_finish<NQ>(J, inp, wg, t, got);
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------------
// `testing_test(v)` ON THE DEVICE: the training / test-set driver of the UR5 arm (VBOC/UR5/vboc_multiprocessing_ur5.py
// :369-466) and of the Cartesian double pendulum (VBOC/Cartesian constraints/vboc_multiprocessing.py:19-129; the
// handle carries the keep-out circle).  A random cost direction and initial position, then the horizon grows while
// the cost still drops by more than tol; a failed solve gives None (no restarts).  Restates
// vboc_amd/drivers.py::ur5_problem / cartesian_problem (pinned against the reference's own functions): draws from
// Philox stream `draw_stream` in the reference's order (random() before choice() in `random.random() *
// random.choice([-1, 1])`), p / norm(p), q0 = lo + random() (hi - lo).  Result: x0 incl. the dt column.
// ------------------------------------------------------------------------------------------------
struct TtJobs {
  const long long* ids;
  int count, N_start, nmax, draw_stream;
  int fail_mod;                     // test-only failure injection (solver option dg_fail_mod), 0 = off
  unsigned long long seed;
  double tol, dt;
  double xlo[8], xhi[8], ulim[4];   // state box [q, qdot] and torque limits (2nq / nq entries used)
  double* st;                       // [groups][st_doubles]
  int st_doubles;
  double* rows;                     // [count][2nq + 1]: x0 with the dt column
  int* row_cnt;                     // 1, or -1 for None
  double* stats;                    // [count][DG_NSTAT]
  unsigned* next;
  unsigned* done;
  unsigned* err;
};

template <int NQ>
struct TtState {
  int N, solves;
  double cost, sqp, nsqp, nqp, t0, st1, it1;
};

template <int NQ>
struct Tt {
  static constexpr int NX = 2 * NQ, NXR = NX + 1, NU = NQ, NP = NQ + 1;
  const TtJobs& J;
  const Inputs& in;
  const int wg, t;
  TtState<NQ>* s;

  __device__ Tt(const TtJobs& J_, const Inputs& in_, int wg_, int t_) : J(J_), in(in_), wg(wg_), t(t_) {
    s = (TtState<NQ>*)(J.st + (long long)wg * J.st_doubles);
  }
  __device__ __forceinline__ long long row(int r) const { return (long long)wg * (J.nmax + 1) + r; }
  __device__ __forceinline__ double* xg(int r) const { return (double*)in.xg + row(r) * NXR; }
  __device__ __forceinline__ double* ug(int r) const { return (double*)in.ug + ((long long)wg * J.nmax + r) * NU; }
  __device__ __forceinline__ const double* xo(int r) const { return in.xo + row(r) * NXR; }
  __device__ __forceinline__ const double* uo(int r) const { return in.uo + ((long long)wg * J.nmax + r) * NU; }

  __device__ __forceinline__ void request(int N) {
    ((int*)in.N)[wg] = N;
    s->solves += 1;
  }

  __device__ __forceinline__ bool start(int job) {
#pragma clang fp contract(off)
    const long long pid = J.ids[job];
    s->t0 = (double)__builtin_amdgcn_s_memrealtime();
    s->solves = 0; s->sqp = 0.0; s->nsqp = 0.0; s->nqp = 0.0; s->st1 = 0.0; s->it1 = 0.0;
    s->cost = 1e6;
    int di = 0;
    auto draw = [&]() { return philox_uniform(pid, di++, J.seed, (unsigned)J.draw_stream); };
    double p[NQ], q0[NQ];
    UNR for (int j = 0; j < NQ; ++j) {
      const double r = draw();
      const double c = Dg<(NQ < 4 ? NQ : 3)>::choice_idx(draw(), 2) == 0 ? -1.0 : 1.0;
      p[j] = r * c;
    }
    const double nw = np_norm<NQ>(p);
    UNR for (int j = 0; j < NQ; ++j) p[j] = p[j] / nw;
    UNR for (int j = 0; j < NQ; ++j) q0[j] = J.xlo[j] + draw() * (J.xhi[j] - J.xlo[j]);
    double* P = (double*)in.p + (long long)wg * NP;
    UNR for (int j = 0; j < NQ; ++j) P[j] = p[j];
    P[NQ] = 0.0;
    double* lbx = (double*)in.lbx + (long long)wg * NXR; double* ubx = (double*)in.ubx + (long long)wg * NXR;
    double* lbxe = (double*)in.lbxe + (long long)wg * NXR; double* ubxe = (double*)in.ubxe + (long long)wg * NXR;
    double* lb0 = (double*)in.lbx0 + (long long)wg * NXR; double* ub0 = (double*)in.ubx0 + (long long)wg * NXR;
    double* lbu = (double*)in.lbu + (long long)wg * NU; double* ubu = (double*)in.ubu + (long long)wg * NU;
    UNR for (int c = 0; c < NX; ++c) {
      lbx[c] = J.xlo[c]; ubx[c] = J.xhi[c];
      lbxe[c] = c < NQ ? J.xlo[c] : 0.0; ubxe[c] = c < NQ ? J.xhi[c] : 0.0;
      lb0[c] = c < NQ ? q0[c] : J.xlo[c]; ub0[c] = c < NQ ? q0[c] : J.xhi[c];
    }
    lbx[NX] = J.dt; ubx[NX] = J.dt; lbxe[NX] = J.dt; ubxe[NX] = J.dt; lb0[NX] = J.dt; ub0[NX] = J.dt;
    UNR for (int a = 0; a < NU; ++a) { lbu[a] = -J.ulim[a]; ubu[a] = J.ulim[a]; }
    const int N = J.N_start;
    for (int r = t; r <= N; r += 64) {
      UNR for (int c = 0; c < NXR; ++c) xg(r)[c] = c < NQ ? q0[c] : (c == NX ? J.dt : 0.0);
      if (r < N) UNR for (int a = 0; a < NU; ++a) ug(r)[a] = 0.0;
    }
    s->N = N;
    request(N);
    return true;
  }

  // 1: another solve is requested; 0: done (row written by finish)
  __device__ __forceinline__ int feed(int job, int& ok) {
#pragma clang fp contract(off)
    const int N = in.N[wg];
    const int it = in.sqp_iter[wg], qit = in.qp_iter[wg];
    if (s->solves == 1) {
      s->st1 = (double)in.status[wg];
      s->it1 = (double)it;
    }
    s->sqp += (double)it;
    s->nsqp += (double)N * (double)it;
    s->nqp += (double)N * (double)qit;
    int status = in.status[wg];
    if (J.fail_mod > 0) {   // tests: status 4 when int(|q_0| 1e6) % fail_mod == 0 (tests/oracle_backend.py)
      const long long q = (long long)(fabs(in.lbx0[(long long)wg * NXR]) * 1e6);
      if (q % J.fail_mod == 0) status = 4;
    }
    if (status != 0) { ok = 0; return 0; }
    const double cost = in.cost[wg];
    if (cost > s->cost - J.tol) { ok = 1; return 0; }
    if (N + 1 > J.nmax) {
      if (t == 0) atomicOr(J.err + 1, 1u);
      ok = 0;
      return 0;
    }
    s->cost = cost;
    for (int r = t; r <= N + 1; r += 64) {
      const int rr = r <= N ? r : N;
      UNR for (int c = 0; c < NXR; ++c) xg(r)[c] = xo(rr)[c];
      if (r < N) {
        UNR for (int a = 0; a < NU; ++a) ug(r)[a] = uo(r)[a];
      } else if (r == N) {
        UNR for (int a = 0; a < NU; ++a) ug(r)[a] = 0.0;
      }
    }
    s->N = N + 1;
    request(N + 1);
    return 1;
  }

  __device__ __forceinline__ void finish(int job, int ok) {
    __syncthreads();
    if (t == 0) {
      J.row_cnt[job] = ok ? 1 : -1;
      double* st = J.stats + (long long)job * DG_NSTAT;
      st[DG_SOLVES] = (double)s->solves;
      st[DG_RK4] = 0.0;
      st[DG_SQP] = s->sqp;
      st[DG_NSQP] = s->nsqp;
      st[DG_NQP] = s->nqp;
      st[DG_T0] = s->t0;
      st[DG_T1] = (double)__builtin_amdgcn_s_memrealtime();
      st[DG_ST1] = s->st1;
      st[DG_IT1] = s->it1;
      st[DG_TQ] = s->t0;
      st[DG_TAKEN] = 0.0;
      st[DG_WAIT] = 0.0;
      st[DG_LAG] = 0.0;
    }
    if (ok && t < NXR) J.rows[(long long)job * NXR + t] = xo(0)[t];
    __syncthreads();
    if (t == 0) atomicAdd(J.done, 1u);
  }
};

template <int NQ>
__device__ __forceinline__ bool tt_start(const TtJobs* J, const Inputs* in, int wg, int t, int job) {
  Tt<NQ> T(*J, *in, wg, t);
  return T.start(job);
}
template <int NQ>
__device__ __forceinline__ int tt_feed(const TtJobs* J, const Inputs* in, int wg, int t, int job, int& ok) {
  Tt<NQ> T(*J, *in, wg, t);
  return T.feed(job, ok);
}
template <int NQ>
__device__ __forceinline__ void tt_finish(const TtJobs* J, const Inputs* in, int wg, int t, int job, int ok) {
  Tt<NQ> T(*J, *in, wg, t);
  T.finish(job, ok);
}

// one workgroup = one wave = one testing_test problem at a time; HC: the Cartesian keep-out circle (a problem whose
// initial tip is inside it gets status 4 without iterating, as k_wave)
template <int NQ, bool FM, bool HC>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WavesPerEu<NQ>::v, WavesPerEu<NQ>::v)))
void k_tt(Work w, Opts o, Inputs in, const Inputs* inp, const TtJobs* J, WaveJobs jb) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int t = (int)threadIdx.x;
  const int wg = (int)blockIdx.x;
  Coop<NQ, FM, HC> C(smem, gptr(jb.regions) + (long long)wg * jb.region_doubles, w, o, t);
  if constexpr (HC) C.gh = gptr(jb.hc) + (long long)wg * jb.hc_doubles;
  const int count = J->count;
  for (;;) {
    int got = -1;
    if (t == 0 && __hip_atomic_load(jb.next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)count) {
      const unsigned i = atomicAdd(jb.next, 1u);
      if (i < (unsigned)count) got = (int)i;
    }
    got = dg_bcast(got);
    if (got < 0) break;
    int code = tt_start<NQ>(J, inp, wg, t, got) ? 1 : 0, ok = 0;
    while (code) {
      __syncthreads();
      int it = 0, qit = 0;
      Lane<NQ> chk(w, o, 0u);
      bool run = chk.supported(in, wg);
      if (!run) {
        if (t == 0) { in.status[wg] = 5; in.sqp_iter[wg] = 0; in.qp_iter[wg] = 0; }
      }
      if constexpr (HC) {
        if (run) {
          double q0[NQ];
          UNR for (int j = 0; j < NQ; ++j) q0[j] = in.lbx0[(long long)wg * (2 * NQ + 1) + j];
          const double h0 = C.hc_eval(q0, nullptr);
          if (!(h0 >= o.hlh && h0 <= o.huh)) {
            run = false;
            if (t == 0) { in.status[wg] = 4; in.sqp_iter[wg] = 0; in.qp_iter[wg] = 0; }
          }
        }
      }
      if (run) {
        C.from_inputs(in, wg);
        const int status = C.run(it, qit);
        C.store(in, wg, status, it, qit);
      }
      __syncthreads();
      code = tt_feed<NQ>(J, inp, wg, t, got, ok);
    }
    tt_finish<NQ>(J, inp, wg, t, got, ok);
    __syncthreads();
  }
}

}  // namespace vboc

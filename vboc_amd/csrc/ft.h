// ft.h - free-time box OCP solver: the reference's OCP<sys>.OCP_solve with dt a decision state
// (OCPpendulum.OCP_solve, VBOC/pendulum_class_vboc.py:107-130; model and options :8-103), batched.
//
// Problem (per batch entry, the vboc_batch_t layout of include/vboc.h, nx = 2 nq + 1):
//   x_k = [theta, dtheta, dt], x_{k+1} = Phi(x_k, u_k) = [RK4 with h = dt of the physics rhs ; dt]
//   (f_expl = dt * f, one ERK4 step of length 1 per interval, tf = N: :23-40, :55-58);
//   cost  w . dtheta_0 + wt * sum_{k<N} dt_k  (EXTERNAL cost :70-74, p = [w, wt]);
//   stage 0: components with lbx_0 == ubx_0 fixed, the others boxed; stages 1..N-1: boxes lbx/ubx
//   (lb < ub required) and lbu/ubu; stage N: components with lbx_e == ubx_e are terminal equalities,
//   the others boxed.  No general constraint.
// Algorithm: the SQP / L1-merit backtracking / Mehrotra interior-point QP / Riccati recursion of the
// boundary solver (coop.h, oracle/vboc_oracle.c), generalised to free stage-0 components and
// terminal equalities on any component subset (Schur complement through Pi = E'); restated on the
// CPU in oracle/vboc_oracle_ft.c (the checker).
//
// Execution: one problem per workgroup of one wave (64 lanes), persistent grid pulling problem ids
// from a global counter.  Stage records live in the workgroup's HBM region; stage-parallel passes
// (linearisation with the d/d(dt) sensitivity column, residuals, IPM set-up, barrier Hessians,
// step-length tests, updates, merit re-simulation) put stage k on lane k mod 64 and reduce with
// cross-lane shuffles; the Riccati recursions (factorisation + two vector/forward sweeps per IPM
// iteration) and the costate recursion run on lane 0, which issues each stage's loads as one
// independent batch.  The workload this serves is small (the pendulum's sequential VBOC sweep), so
// the kernel favours a direct mapping over the wave solver's LDS-ring machinery.
#pragma once
#include <hip/hip_runtime.h>

#include "model.h"

namespace vboc {

template <int NQ, bool MP = false>
struct FtL {
  static constexpr int NX = 2 * NQ + 1, NU = NQ, NZ = NX + NU, N2 = 2 * NQ;
  // stage record (doubles)
  static constexpr int X = 0, U = X + NX, PI = U + NU, LL = PI + NX, LU = LL + NZ, WPI = LU + NZ, A = WPI + NX,
                       B = A + NX * NX, BD = B + NX * NU, LB = BD + NX, UB = LB + NZ, DZ = UB + NZ, QL = DZ + NZ,
                       QU = QL + NZ, E0 = QU + NZ, H = E0 + NX, G = H + NZ, D = G + NZ, DAFF = D + NZ, K = DAFF + NZ,
                       KF = K + NU * NX, LR = KF + NU, M = LR + NZ * NZ, Y = M + NZ * NX, PE = Y + NZ * NX,
                       QPI = PE + NX, F0 = QPI + NX;
  // the Safe-MPC NN row of the stage (HardTerm: stage N; SoftTraj: every stage; the oracle's fstage_t row fields):
  // value, gradient, the QP slacks / duals of both sides, their affine directions, residual starts, the NLP
  // multipliers; a soft lower side's slack (QP value, dual, affine directions), its NLP iterate / multiplier and weights
  // zl, Zl; the factorisation weight sigma, the slack elimination b, W; the combined directions; lh - h, uh - h
  static constexpr int RV = F0 + NX * NZ, RG = RV + 1, RTL = RG + NX, RTU = RTL + 1, RQL = RTU + 1, RQU = RQL + 1,
                       RR0L = RQU + 1, RR0U = RR0L + 1, RATL = RR0U + 1, RATU = RATL + 1, RAQL = RATU + 1,
                       RAQU = RAQL + 1, RLL = RAQU + 1, RLU = RLL + 1, RS = RLU + 1, RQS = RS + 1, RAS = RQS + 1,
                       RAQS = RAS + 1, RSL = RAQS + 1, RLSL = RSL + 1, RZL = RLSL + 1, RZ2 = RZL + 1, RSIG = RZ2 + 1,
                       RB = RSIG + 1, RW = RB + 1, RDTL = RW + 1, RDTU = RDTL + 1, RDQL = RDTU + 1, RDQU = RDQL + 1,
                       RDS = RDQU + 1, RDQS = RDS + 1, RL = RDQS + 1, RU = RL + 1;
  // the free-time solver (MP false) never touches the row fields: its records end at F0's block
  static constexpr int REC = MP ? RU + 1 : F0 + NX * NZ;
  static constexpr long long region_doubles(int nmax) { return (long long)REC * (nmax + 1); }
};

// The Safe-MPC tracking OCP on this solver (vboc_mpc_solve_batch; VBOC/Safe MPC/triplependulum_class_vboc.py:91-240,
// restated in oracle/vboc_oracle_ft.c vboc_oracle_mpc_solve): LINEAR_LS cost with its Gauss-Newton Hessian
// (weights wq on [x; u], we at N, stage costs times cs), the dt column pinned by x_0, the terminal row
// lh <= NN(x_N) - max(|x_N[2:]|, 1e-3) <= uh (NeuralNetDIR(2 nq, hid, 1); W1T = W1 transposed, for coalesced loads),
// and SQP_RTI.  on == 0: the free-time OCP above, unchanged.
// soft == 1: OCPtriplependulumSoftTraj (triplependulum_class_vboc.py:242-304): the row scaled by sm / 100
// (sm = 100 - safety_margin) on every stage 0..N, soft lower sides with the per-problem per-stage slack weights zl / Zl
// [B][N + 1] (oracle/vboc_oracle_ft.c header: the slack eliminated per stage); Wb / Web [B][3 nq] / [B][2 nq]: per-problem
// stage weights (the receding driver's cost_set(i, "W")), nullptr = wq / we
constexpr int FT_NN_MAX = 512;
struct MpcArgs {
  int on, rti, hid, soft;
  int qcf;   // a QP stopped by qp_max_iter is a QP failure (status 4): the AL labelling OCP (vboc_al_solve_batch)
  double wq[10], yr[10], we[7], yre[7], cs, sm;
  const double *W0, *b0, *W1, *W1T, *b1, *W2, *b2;
  double mean, std, lh, uh;
  const double *zl, *Zl, *Wb, *Web;
  double* hrow;   // [B] h(x_N) of each result (nullptr: not written)
};

// MP: the Safe-MPC instantiation (k_ft<3, true>); the free-time pendulum solver carries no network buffers
template <int NQ, bool MP>
struct FtShared {
  static constexpr int NX = FtL<NQ, MP>::NX, NU = FtL<NQ, MP>::NU, NNB = MP ? FT_NN_MAX : 1;
  int N, nf0, ne, pid, bad;
  int f0[NX], ei[NX], fix[NX];
  double ev[NX], c0[NX], cp[NX], x0lb[NX], x0ub[NX], xlb[NX], xub[NX], xNlb[NX], xNub[NX], ulb[NU], uub[NU];
  double tnu[NX], wnu[NX], qnu[NX], nun[NX], S[NX * NX], lin_e[NX];
  double wbnd, rs;
  int qp_fail;
  double wq[NX + NU], we[NX];              // this problem's tracking weights (MpcArgs wq / we or Wb / Web)
  double nn1[NNB], nn2[NNB];               // hidden activations / backward weights of the row's network
};

__device__ __forceinline__ double ft_wmax(double v) {
  for (int o = 32; o >= 1; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ double ft_wsum(double v) {
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
// running minimum of t / (-dt) over dt < 0, kept as (n, d) (the oracle's fr_add comparison)
struct FtRatio {
  double n, d;
  __device__ void add(double t, double dt) {
    if (dt < 0.0 && t * d < n * (-dt)) { n = t; d = -dt; }
  }
  __device__ double reduce() {
    for (int o = 32; o >= 1; o >>= 1) {
      const double n2 = __shfl_xor(n, o), d2 = __shfl_xor(d, o);
      if (n2 * d < n * d2) { n = n2; d = d2; }
    }
    return n / d;
  }
};

// Phi(x, u) of the free-time model and its exact Jacobians A = dPhi/dx (last column d/d(dt)), B = dPhi/du
template <int NQ>
__device__ void ft_rk4_sens(const double* x, const double* u, double* phi, double* A, double* B) {
  constexpr int N2 = 2 * NQ, NX = N2 + 1, NU = NQ, NC = N2 + NU + 1, CU = N2, CH = N2 + NU;
  const double h = x[N2];
  double ks[N2], Ts[N2][NC], kp[N2], dkp[N2][NC];
  for (int i = 0; i < N2; ++i) {
    ks[i] = kp[i] = 0.0;
    for (int c = 0; c < NC; ++c) Ts[i][c] = dkp[i][c] = 0.0;
  }
#pragma unroll 1
  for (int s = 0; s < 4; ++s) {
    const double cs = (s == 0) ? 0.0 : (s == 3 ? 1.0 : 0.5), wg = (s == 0 || s == 3) ? 1.0 : 2.0;
    double X[N2], T[N2][NC];
    for (int i = 0; i < N2; ++i) {
      X[i] = x[i] + cs * h * kp[i];
      for (int c = 0; c < NC; ++c) {
        double t = cs * h * dkp[i][c];
        if (c == i) t += 1.0;
        if (c == CH) t += cs * kp[i];
        T[i][c] = t;
      }
    }
    double acc[NQ], Jth[NQ * NQ], Jom[NQ * NQ], Ju[NQ * NQ];
    model_eval<NQ, true>(X, X + NQ, u, acc, Jth, Jom, Ju);
    for (int j = 0; j < NQ; ++j) { kp[j] = X[NQ + j]; kp[NQ + j] = acc[j]; }
    for (int c = 0; c < NC; ++c) {
      for (int j = 0; j < NQ; ++j) dkp[j][c] = T[NQ + j][c];
      for (int j = 0; j < NQ; ++j) {
        double t = (c >= CU && c < CU + NQ) ? Ju[j * NQ + (c - CU)] : 0.0;
        for (int q = 0; q < NQ; ++q) t += Jth[j * NQ + q] * T[q][c] + Jom[j * NQ + q] * T[NQ + q][c];
        dkp[NQ + j][c] = t;
      }
    }
    for (int i = 0; i < N2; ++i) {
      ks[i] += wg * kp[i];
      for (int c = 0; c < NC; ++c) Ts[i][c] += wg * dkp[i][c];
    }
  }
  for (int i = 0; i < N2; ++i) {
    phi[i] = x[i] + h / 6.0 * ks[i];
    if (A) {
      for (int c = 0; c < N2; ++c) A[i * NX + c] = (c == i ? 1.0 : 0.0) + h / 6.0 * Ts[i][c];
      A[i * NX + N2] = ks[i] / 6.0 + h / 6.0 * Ts[i][CH];
      for (int a = 0; a < NU; ++a) B[i * NU + a] = h / 6.0 * Ts[i][CU + a];
    }
  }
  phi[N2] = h;
  if (A) {
    for (int c = 0; c < NX; ++c) A[N2 * NX + c] = (c == N2) ? 1.0 : 0.0;
    for (int a = 0; a < NU; ++a) B[N2 * NU + a] = 0.0;
  }
}

template <int n>
__device__ __forceinline__ bool ft_chol(double* A, int m) {   // m <= n used rows/cols, row stride m
  for (int j = 0; j < m; ++j) {
    double s = A[j * m + j];
    for (int k = 0; k < j; ++k) s -= A[j * m + k] * A[j * m + k];
    if (!(s > 0.0)) return false;
    const double d = sqrt(s);
    A[j * m + j] = d;
    for (int i = j + 1; i < m; ++i) {
      double t = A[i * m + j];
      for (int k = 0; k < j; ++k) t -= A[i * m + k] * A[j * m + k];
      A[i * m + j] = t / d;
    }
    for (int i = 0; i < j; ++i) A[i * m + j] = 0.0;
  }
  return true;
}
__device__ __forceinline__ void ft_chol_solve(const double* L, int m, double* b) {
  for (int i = 0; i < m; ++i) {
    double t = b[i];
    for (int k = 0; k < i; ++k) t -= L[i * m + k] * b[k];
    b[i] = t / L[i * m + i];
  }
  for (int i = m - 1; i >= 0; --i) {
    double t = b[i];
    for (int k = i + 1; k < m; ++k) t -= L[k * m + i] * b[k];
    b[i] = t / L[i * m + i];
  }
}

template <int NQ, bool MP = false>
struct Ft {
  using L = FtL<NQ, MP>;
  static constexpr int NX = L::NX, NU = L::NU, NZ = L::NZ, N2 = 2 * NQ;
  FtShared<NQ, MP>& sh;
  double* g;     // this workgroup's stage records
  const Opts& o;
  int t;
  const MpcArgs& mp;

  __device__ Ft(FtShared<NQ, MP>& s_, double* g_, const Opts& o_, int t_, const MpcArgs& mp_)
      : sh(s_), g(g_), o(o_), t(t_), mp(mp_) {}

  // ---- Safe-MPC terminal row (all lanes; x uniform): h(x) = NN(z(x)) - vn(x), grad (NX, uniform) if asked ----
  // Hidden unit i of a layer lives on lane i mod 64; layer 2 streams W1T row by row (64 consecutive doubles per
  // load across the wave), the backward pass W1 row by row.  The arithmetic is the oracle's (oracle/vboc_oracle_ft.c
  // nn_row) operation for operation: no contraction, every sum in the oracle's order - the two sums over hidden
  // units (the output and d out / d z) run serially over LDS on every lane (a few thousand cycles per evaluation,
  // once per SQP iteration and line-search trial), so the row and its gradient are bit-identical to the oracle's.
  __device__ double nn_row(const double* x, double* grad) {
#pragma clang fp contract(off)
    static_assert(MP, "the network row belongs to the Safe-MPC instantiation");
    const int H = mp.hid;
    double ss = 0.0;
    for (int j = 2; j < N2; ++j) ss += x[j] * x[j];    // norm_2(x[2:]): theta_3 included, as the reference
    const double nrm = sqrt(ss), vn = nrm > 1e-3 ? nrm : 1e-3;
    double z[N2];
    for (int j = 0; j < NQ; ++j) z[j] = (x[j] - mp.mean) / mp.std;
    for (int j = NQ; j < N2; ++j) z[j] = x[j] / vn;
    __syncthreads();   // the buffers may still be read by a previous evaluation
    for (int i = t; i < H; i += 64) {
      double a = 0.0;
      for (int j = 0; j < N2; ++j) a += mp.W0[i * N2 + j] * z[j];
      a += mp.b0[i];
      sh.nn1[i] = a > 0.0 ? a : 0.0;
    }
    __syncthreads();
    constexpr int MQ = FT_NN_MAX / 64;
    double acc[MQ];
    for (int m = 0; m < MQ; ++m) acc[m] = 0.0;
    for (int j = 0; j < H; ++j) {
      const double a1 = sh.nn1[j];
      const double* row = mp.W1T + (long long)j * H;
      for (int m = 0; m < MQ; ++m) {
        const int i = t + 64 * m;
        if (i < H) acc[m] += row[i] * a1;
      }
    }
    for (int m = 0; m < MQ; ++m) {
      const int i = t + 64 * m;
      if (i < H) sh.nn2[i] = acc[m] + mp.b1[i];   // layer-2 pre-activations
    }
    __syncthreads();
    double out = 0.0;
    for (int i = 0; i < H; ++i) {                 // the oracle's sequential sum (LDS / W2 reads broadcast)
      const double a2 = sh.nn2[i];
      if (a2 > 0.0) out += mp.W2[i] * a2;
    }
    out += mp.b2[0];
    if (mp.soft) out = out * mp.sm / 100.0;   // nn_decisionfunction_conservative: out*(100-safety_margin)/100 (:301)
    if (grad) {
      __syncthreads();
      for (int i = t; i < H; i += 64) sh.nn2[i] = sh.nn2[i] > 0.0 ? mp.W2[i] : 0.0;   // W2 [a2 > 0]
      __syncthreads();
      double g1[MQ];
      for (int m = 0; m < MQ; ++m) {   // g1[j] = sum_i W1[i][j] w_i (i ascending) for the lane's j
        const int j = t + 64 * m;
        g1[m] = 0.0;
        if (j >= H) continue;
        for (int i = 0; i < H; ++i) g1[m] += mp.W1[(long long)i * H + j] * sh.nn2[i];
      }
      __syncthreads();
      for (int m = 0; m < MQ; ++m) {
        const int j = t + 64 * m;
        if (j < H) sh.nn2[j] = g1[m];
      }
      __syncthreads();
      double gz[N2];
      for (int q = 0; q < N2; ++q) gz[q] = 0.0;
      for (int i = 0; i < H; ++i) {                // through layer 1, i ascending as the oracle
        if (!(sh.nn1[i] > 0.0)) continue;
        const double gi = sh.nn2[i];
        for (int q = 0; q < N2; ++q) gz[q] += gi * mp.W0[i * N2 + q];
      }
      if (mp.soft) for (int q = 0; q < N2; ++q) gz[q] = gz[q] * mp.sm / 100.0;
      double dvn[N2];
      for (int j = 0; j < N2; ++j) dvn[j] = (nrm > 1e-3 && j >= 2) ? x[j] / nrm : 0.0;
      for (int j = 0; j < N2; ++j) {
        double v = j < NQ ? gz[j] / mp.std : gz[j] / vn;
        for (int q = NQ; q < N2; ++q) v -= gz[q] * x[q] / (vn * vn) * dvn[j];
        grad[j] = v - dvn[j];
      }
      grad[N2] = 0.0;   // the pinned dt column
    }
    return out - vn;
  }
  __device__ __forceinline__ double hq(int k, int i) const {   // Gauss-Newton Hessian diagonal of the tracking cost
    if (!MP) return 0.0;
    if (k == sh.N) return sh.we[i];
    return mp.cs * sh.wq[k == 0 ? (i < sh.nf0 ? sh.f0[i] : NX + (i - sh.nf0)) : i];
  }
  __device__ __forceinline__ double track(int k, const double* x, const double* u) const {
    double c = 0.0;
    if (k == sh.N) {
      for (int i = 0; i < NX; ++i) { const double d = x[i] - mp.yre[i]; c += sh.we[i] * d * d; }
      return 0.5 * c;
    }
    for (int i = 0; i < NX; ++i) { const double d = x[i] - mp.yr[i]; c += sh.wq[i] * d * d; }
    for (int a = 0; a < NU; ++a) { const double d = u[a] - mp.yr[NX + a]; c += sh.wq[NX + a] * d * d; }
    return 0.5 * mp.cs * c;
  }
  // ---- the Safe-MPC rows (oracle/vboc_oracle_ft.c frow_*: the same expressions) ----------------------------
  __device__ __forceinline__ bool row_at(int k) const { return MP && mp.hid > 0 && (mp.soft || k == sh.N); }
  // c'd of stage k's row over the stage vector at record offset `off` (its state components; stage 0: the free ones)
  __device__ __forceinline__ double row_dot(const double* r, int k, int off) const {
    double v = 0.0;
    if (k == 0) {
      for (int j = 0; j < sh.nf0; ++j) v += r[L::RG + sh.f0[j]] * r[off + j];
      return v;
    }
    for (int i = 0; i < NX; ++i) v += r[L::RG + i] * r[off + i];
    return v;
  }
  __device__ __forceinline__ void row_addgrad(double* r, int k, double v) const {
    if (k == 0) {
      for (int j = 0; j < sh.nf0; ++j) r[L::G + j] += r[L::RG + sh.f0[j]] * v;
      return;
    }
    for (int i = 0; i < NX; ++i) r[L::G + i] += r[L::RG + i] * v;
  }
  __device__ __forceinline__ static void row_rc(const double* r, double smu, double& rcl, double& rcu, double& rcs) {
    rcl = smu - r[L::RTL] * r[L::RQL] - r[L::RATL] * r[L::RAQL];
    rcu = smu - r[L::RTU] * r[L::RQU] - r[L::RATU] * r[L::RAQU];
    rcs = smu - r[L::RS] * r[L::RQS] - r[L::RAS] * r[L::RAQS];
  }
  // the row's gradient term for the targets rc (pred: the predictor's form) and (pred) its factorisation weight
  __device__ __forceinline__ double row_gamma(double* r, double rs, double rcl, double rcu, double rcs, bool pred) const {
    const double rl = rs * r[L::RR0L], ru = rs * r[L::RR0U];
    const double tl = r[L::RTL], tu = r[L::RTU], ql = r[L::RQL], qu = r[L::RQU];
    double gam;
    if (pred) gam = ql * rl / tl - qu * ru / tu;
    else gam = -ql + qu - (rcl - ql * rl) / tl + (rcu - qu * ru) / tu;
    if (mp.soft) {
      const double sv = r[L::RS], qs = r[L::RQS], Z = r[L::RZ2];
      const double Sl = ql / tl, Ss = qs / sv, W = Z + Sl + Ss;
      const double b = -(Z * sv + r[L::RZL] - ql - qs) + rcl / tl + rcs / sv - Sl * rl;
      r[L::RW] = W;
      r[L::RB] = b;
      gam += Sl * b / W;
      if (pred) r[L::RSIG] = qu / tu + Sl * (Z + Ss) / W;
    } else if (pred) {
      r[L::RSIG] = ql / tl + qu / tu;
    }
    return gam;
  }
  __device__ __forceinline__ void row_dirs(const double* r, double cd, double rs, double rcl, double rcu, double rcs,
                                           double& dtl, double& dtu, double& dql, double& dqu, double& ds,
                                           double& dqs) const {
    const double rl = rs * r[L::RR0L], ru = rs * r[L::RR0U];
    ds = 0.0;
    dqs = 0.0;
    if (mp.soft) {
      ds = (r[L::RB] - r[L::RQL] / r[L::RTL] * cd) / r[L::RW];
      dtl = cd + ds + rl;
    } else {
      dtl = cd + rl;
    }
    dtu = ru - cd;
    dql = (rcl - r[L::RQL] * dtl) / r[L::RTL];
    dqu = (rcu - r[L::RQU] * dtu) / r[L::RTU];
    if (mp.soft) dqs = (rcs - r[L::RQS] * ds) / r[L::RS];
  }

  __device__ __forceinline__ double* rec(int k) const { return g + (long long)k * L::REC; }
  __device__ __forceinline__ int nz(int k) const { return k == 0 ? sh.nf0 + NU : (k == sh.N ? NX : NX + NU); }
  // value, bounds, boxed flag of stage variable i of stage k
  __device__ __forceinline__ bool comp(int k, int i, double& v, double& lb, double& ub) const {
    const double* r = rec(k);
    if (k == 0) {
      if (i < sh.nf0) { const int c = sh.f0[i]; v = r[L::X + c]; lb = sh.x0lb[c]; ub = sh.x0ub[c]; }
      else { v = r[L::U + i - sh.nf0]; lb = sh.ulb[i - sh.nf0]; ub = sh.uub[i - sh.nf0]; }
      return !(isinf(lb) && isinf(ub));
    }
    if (k == sh.N) {
      v = r[L::X + i];
      if (sh.fix[i]) { lb = -INFINITY; ub = INFINITY; return false; }
      lb = sh.xNlb[i]; ub = sh.xNub[i];
      return !(isinf(lb) && isinf(ub));
    }
    if (i < NX) { v = r[L::X + i]; lb = sh.xlb[i]; ub = sh.xub[i]; }
    else { v = r[L::U + i - NX]; lb = sh.ulb[i - NX]; ub = sh.uub[i - NX]; }
    // both sides infinite: a free component (the Safe-MPC model's pinned dt; any such input of the free-time OCP),
    // as the oracle's fcomp
    return !(isinf(lb) && isinf(ub));
  }
  __device__ __forceinline__ double grad(int k, int i) const {
    if (MP) {   // W ([x; u] - yref) at the current iterate
      double v, lb, ub;
      (void)comp(k, i, v, lb, ub);
      if (k == sh.N) return sh.we[i] * (v - mp.yre[i]);
      const int w = k == 0 ? (i < sh.nf0 ? sh.f0[i] : NX + (i - sh.nf0)) : i;
      return mp.cs * sh.wq[w] * (v - mp.yr[w]);
    }
    if (k == 0) return i < sh.nf0 ? sh.c0[sh.f0[i]] : 0.0;
    if (k == sh.N) return 0.0;
    return i < NX ? sh.cp[i] : 0.0;
  }

  // ---- set-up / output ------------------------------------------------------------------------
  __device__ void load(const Inputs& in, int pid) {
    constexpr int NP = NQ + 1;
    if (t == 0) {
      const int N = in.N[pid];
      sh.N = N; sh.pid = pid; sh.nf0 = 0; sh.ne = 0;
      const double* p = in.p + (long long)pid * NP;
      int bad = (N < 1 || N > in.nmax) ? 1 : 0;
      for (int i = 0; i < NX; ++i) {
        const long long o = (long long)pid * NX + i;
        sh.xlb[i] = in.lbx[o]; sh.xub[i] = in.ubx[o]; sh.x0lb[i] = in.lbx0[o]; sh.x0ub[i] = in.ubx0[o];
        sh.xNlb[i] = in.lbxe[o]; sh.xNub[i] = in.ubxe[o];
        if (!(sh.xlb[i] < sh.xub[i]) || !(sh.x0lb[i] <= sh.x0ub[i]) || !(sh.xNlb[i] <= sh.xNub[i])) bad = 1;
        if (sh.x0lb[i] < sh.x0ub[i]) sh.f0[sh.nf0++] = i;
        sh.fix[i] = (sh.xNlb[i] == sh.xNub[i]) ? 1 : 0;
        if (sh.fix[i]) { sh.ei[sh.ne] = i; sh.ev[sh.ne] = sh.xNlb[i]; sh.ne++; }
        sh.c0[i] = 0.0; sh.cp[i] = 0.0; sh.tnu[i] = 0.0; sh.wnu[i] = 0.0; sh.qnu[i] = 0.0; sh.nun[i] = 0.0;
      }
      for (int a = 0; a < NU; ++a) {
        sh.ulb[a] = in.lbu[(long long)pid * NU + a]; sh.uub[a] = in.ubu[(long long)pid * NU + a];
        if (!(sh.ulb[a] < sh.uub[a])) bad = 1;
      }
      // a stage-0 row acts on the free components of x_0, and the stage-0 Riccati block carries no sigma c c' term
      // for them: the soft rows are implemented for a fully pinned x_0 only (every Safe-MPC OCP_solve pins it)
      if (MP && mp.soft && sh.nf0 > 0) bad = 1;
      for (int j = 0; j < NQ; ++j) sh.c0[NQ + j] = p[j];
      sh.c0[2 * NQ] = p[NQ];
      sh.cp[2 * NQ] = p[NQ];
      sh.wbnd = 0.0;
      if (MP) {   // this problem's tracking weights
        for (int i = 0; i < NX + NU; ++i) sh.wq[i] = mp.wq[i];
        for (int i = 0; i < NX; ++i) sh.we[i] = mp.we[i];
        if (mp.Wb) {   // [3 nq]: x (2 nq, the pinned dt column carries none) then u
          for (int i = 0; i < N2; ++i) sh.wq[i] = mp.Wb[(long long)pid * (N2 + NU) + i];
          for (int a = 0; a < NU; ++a) sh.wq[NX + a] = mp.Wb[(long long)pid * (N2 + NU) + N2 + a];
        }
        if (mp.Web)
          for (int i = 0; i < N2; ++i) sh.we[i] = mp.Web[(long long)pid * N2 + i];
      }
      sh.bad = bad;
    }
    __syncthreads();
    if (sh.bad) return;
    const int N = sh.N;
    const double* xg = in.xg + (long long)pid * (in.nmax + 1) * NX;
    const double* ug = in.ug + (long long)pid * in.nmax * NU;
    for (int k = t; k <= N; k += 64) {
      double* r = rec(k);
      for (int i = 0; i < NX; ++i) r[L::X + i] = (k == 0 && !(sh.x0lb[i] < sh.x0ub[i])) ? sh.x0lb[i] : xg[(long long)k * NX + i];
      for (int i = 0; i < NZ; ++i) { r[L::LL + i] = 0.0; r[L::LU + i] = 0.0; }
      for (int i = 0; i < NX; ++i) { r[L::PI + i] = 0.0; r[L::WPI + i] = 0.0; }
      if (k < N)
        for (int a = 0; a < NU; ++a) r[L::U + a] = ug[(long long)k * NU + a];
      if (MP) {   // the rows' NLP multipliers and slacks start at 0 (ACADOS' nlp_out at creation); their weights,
        // scaled like the stage cost they belong to (ACADOS' cost_scaling multiplies a stage's z / Z with its
        // least-squares weights: cs on stages 0..N-1, 1 at N)
        const double sc = k < N ? mp.cs : 1.0;
        r[L::RLL] = r[L::RLU] = r[L::RSL] = r[L::RLSL] = 0.0;
        r[L::RZL] = (mp.soft && mp.zl) ? sc * mp.zl[(long long)pid * (N + 1) + k] : 0.0;
        r[L::RZ2] = (mp.soft && mp.Zl) ? sc * mp.Zl[(long long)pid * (N + 1) + k] : 0.0;
      }
    }
    __syncthreads();
  }

  __device__ double cost() const {
    double c = 0.0;
    if (MP) {
      for (int k = t; k <= sh.N; k += 64) c += track(k, rec(k) + L::X, rec(k) + L::U);
      c = ft_wsum(c);
      if (mp.soft) {   // the slacks' penalties (ACADOS' get_cost includes them), in stage order
        double sc = 0.0;
        for (int k = 0; k <= sh.N; ++k) {
          const double* r = rec(k);
          sc += r[L::RZL] * r[L::RSL] + 0.5 * r[L::RZ2] * r[L::RSL] * r[L::RSL];
        }
        c += sc;
      }
      return c;
    }
    for (int k = t; k < sh.N; k += 64) {
      const double* r = rec(k);
      for (int i = 0; i < NX; ++i) c += (k == 0 ? sh.c0[i] : sh.cp[i]) * r[L::X + i];
    }
    return ft_wsum(c);
  }

  __device__ void store(const Inputs& in, int status, int it, int qit) {
    const int N = sh.N, pid = sh.pid;
    double* xo = in.xo + (long long)pid * (in.nmax + 1) * NX;
    double* uo = in.uo + (long long)pid * in.nmax * NU;
    for (int k = t; k <= N; k += 64) {
      const double* r = rec(k);
      for (int i = 0; i < NX; ++i) xo[(long long)k * NX + i] = r[L::X + i];
      if (k < N)
        for (int a = 0; a < NU; ++a) uo[(long long)k * NU + a] = r[L::U + a];
    }
    const double c = cost();
    if constexpr (MP) {
      if (mp.hrow) {
        __syncthreads();
        double xN[NX];
        for (int i = 0; i < NX; ++i) xN[i] = rec(N)[L::X + i];
        const double hv = mp.hid > 0 ? nn_row(xN, nullptr) : 0.0;
        if (t == 0) mp.hrow[pid] = hv;
      }
    }
    if (t == 0) {
      in.status[pid] = status;
      in.cost[pid] = c;
      in.sqp_iter[pid] = it;
      in.qp_iter[pid] = qit;
    }
  }

  // ---- linearisation + NLP residuals ------------------------------------------------------------
  __device__ void linearize() {
    const int N = sh.N, m0 = sh.nf0 + NU;
    for (int k = t; k < N; k += 64) {
      double* r = rec(k);
      double phi[NX];
      ft_rk4_sens<NQ>(r + L::X, r + L::U, phi, r + L::A, r + L::B);
      const double* r1 = rec(k + 1);
      for (int i = 0; i < NX; ++i) r[L::BD + i] = phi[i] - r1[L::X + i];
      if (k == 0) {
        for (int i = 0; i < NX; ++i) {
          for (int j = 0; j < sh.nf0; ++j) r[L::F0 + i * m0 + j] = r[L::A + i * NX + sh.f0[j]];
          for (int a = 0; a < NU; ++a) r[L::F0 + i * m0 + sh.nf0 + a] = r[L::B + i * NU + a];
        }
      }
    }
    __syncthreads();
    if constexpr (MP) {
      if (mp.hid > 0) {   // the rows' values and gradients (HardTerm: x_N only; SoftTraj: every stage)
        for (int k = mp.soft ? 0 : N; k <= N; ++k) {
          double xk[NX], gr[NX];
          for (int i = 0; i < NX; ++i) xk[i] = rec(k)[L::X + i];
          const double hv = nn_row(xk, gr);
          if (t == 0) {
            rec(k)[L::RV] = hv;
            for (int i = 0; i < NX; ++i) rec(k)[L::RG + i] = gr[i];
          }
        }
        __syncthreads();
      }
    }
  }

  __device__ void residuals(double& rstat, double& req, double& rineq, double& rcomp) const {
    const int N = sh.N, m0 = sh.nf0 + NU;
    double st = 0.0, eq = 0.0, in = 0.0, cp = 0.0;
    for (int k = t; k <= N; k += 64) {
      const double* r = rec(k);
      if (k < N) for (int i = 0; i < NX; ++i) eq = fmax(eq, fabs(r[L::BD + i]));
      else for (int j = 0; j < sh.ne; ++j) eq = fmax(eq, fabs(r[L::X + sh.ei[j]] - sh.ev[j]));
      const double* rp = k > 0 ? rec(k - 1) : r;
      for (int i = 0; i < nz(k); ++i) {
        double v, lb, ub;
        const bool boxed = comp(k, i, v, lb, ub);
        double gr = grad(k, i) - r[L::LL + i] + r[L::LU + i];
        if (k == 0) {
          for (int q = 0; q < NX; ++q) gr += r[L::F0 + q * m0 + i] * r[L::PI + q];
        } else if (k < N) {
          if (i < NX) {
            for (int q = 0; q < NX; ++q) gr += r[L::A + q * NX + i] * r[L::PI + q];
            gr -= rp[L::PI + i];
          } else {
            for (int q = 0; q < NX; ++q) gr += r[L::B + q * NU + (i - NX)] * r[L::PI + q];
          }
        } else {
          gr -= rp[L::PI + i];
          for (int j = 0; j < sh.ne; ++j) if (sh.ei[j] == i) gr += sh.tnu[j];
        }
        if (row_at(k)) {   // the row's term on the state components of the stage's variables
          const int xi = k == 0 ? (i < sh.nf0 ? sh.f0[i] : -1) : (i < NX ? i : -1);
          if (xi >= 0) gr += r[L::RG + xi] * (r[L::RLU] - r[L::RLL]);
        }
        st = fmax(st, fabs(gr));
        if (boxed) {
          in = fmax(in, fmax(lb - v, v - ub));
          cp = fmax(cp, fmax(fabs(r[L::LL + i] * (v - lb)), fabs(r[L::LU + i] * (ub - v))));
        }
      }
    }
    for (int k = t; k <= N; k += 64) {
      if (!row_at(k)) continue;
      const double* r = rec(k);
      const double hv = r[L::RV], sl = mp.soft ? r[L::RSL] : 0.0;
      in = fmax(in, fmax(mp.lh - (hv + sl), hv - mp.uh));
      cp = fmax(cp, fmax(fabs(r[L::RLL] * (hv + sl - mp.lh)), fabs(r[L::RLU] * (mp.uh - hv))));
      if (mp.soft) {   // the slack: s >= 0, its stationarity Zl s + zl - lambda_row - lambda_s = 0
        in = fmax(in, -sl);
        cp = fmax(cp, fabs(r[L::RLSL] * sl));
        st = fmax(st, fabs(r[L::RZ2] * sl + r[L::RZL] - r[L::RLL] - r[L::RLSL]));
      }
    }
    rstat = ft_wmax(st); req = ft_wmax(eq); rineq = ft_wmax(in); rcomp = ft_wmax(cp);
  }

  // ---- Riccati solve (lane 0): factor = true -> factorisation + vector pass ----------------------
  __device__ bool newton(bool factor) {
    bool ok = true;
    if (t == 0) ok = newton_lane0(factor);
    __syncthreads();
    const int okw = __shfl(ok ? 1 : 0, 0);
    return okw != 0;
  }

  __device__ bool newton_lane0(bool factor) {
    const int N = sh.N, ne = sh.ne, m0 = sh.nf0 + NU;
    const double rs = sh.rs;
    double Pm[NX * NX], p[NX], Pi[NX * NX], lin[NX];
    const double* rN = rec(N);
    for (int i = 0; i < NX * NX; ++i) { Pm[i] = 0.0; Pi[i] = 0.0; }
    for (int i = 0; i < NX; ++i) { Pm[i * NX + i] = rN[L::H + i]; p[i] = rN[L::G + i]; lin[i] = 0.0; }
    if (row_at(N)) {   // the terminal row's barrier: sigma c c'
      const double sig = rN[L::RSIG];
      for (int i = 0; i < NX; ++i)
        for (int j = 0; j < NX; ++j) Pm[i * NX + j] += sig * rN[L::RG + i] * rN[L::RG + j];
    }
    for (int j = 0; j < ne; ++j) Pi[sh.ei[j] * ne + j] = 1.0;
    if (factor) {
      for (int i = 0; i < NX * NX; ++i) sh.S[i] = 0.0;
      for (int i = 0; i < NX; ++i) sh.lin_e[i] = 0.0;
    }
    for (int k = N - 1; k >= 0; --k) {
      double* r = rec(k);
      const int mk = (k == 0) ? m0 : NU;
      const double* Bk = (k == 0) ? r + L::F0 : r + L::B;
      const int uoff = (k == 0) ? 0 : NX;
      double e[NX], v[NX], rr[NZ];
      for (int i = 0; i < NX; ++i) e[i] = rs * r[L::E0 + i];
      if (factor) {
        for (int i = 0; i < NX; ++i) {
          double s = 0.0;
          for (int j = 0; j < NX; ++j) s += Pm[i * NX + j] * e[j];
          r[L::PE + i] = s;
        }
        for (int j = 0; j < ne; ++j) {
          double s = 0.0;
          for (int i = 0; i < NX; ++i) s += Pi[i * ne + j] * e[i];
          sh.lin_e[j] += s;
        }
        double BP[NZ * NX], Ru[NZ * NZ];
        for (int a = 0; a < mk; ++a)
          for (int j = 0; j < NX; ++j) {
            double s = 0.0;
            for (int i = 0; i < NX; ++i) s += Bk[i * mk + a] * Pm[i * NX + j];
            BP[a * NX + j] = s;
          }
        for (int a = 0; a < mk; ++a)
          for (int c = 0; c < mk; ++c) {
            double s = (a == c) ? r[L::H + uoff + a] : 0.0;
            for (int i = 0; i < NX; ++i) s += BP[a * NX + i] * Bk[i * mk + c];
            Ru[a * mk + c] = s;
          }
        for (int a = 0; a < mk; ++a)
          for (int c = 0; c < a; ++c) {
            const double s = 0.5 * (Ru[a * mk + c] + Ru[c * mk + a]);
            Ru[a * mk + c] = Ru[c * mk + a] = s;
          }
        if (!ft_chol<NZ>(Ru, mk)) return false;
        for (int e2 = 0; e2 < mk * mk; ++e2) r[L::LR + e2] = Ru[e2];
        for (int a = 0; a < mk; ++a)
          for (int j = 0; j < ne; ++j) {
            double s = 0.0;
            for (int i = 0; i < NX; ++i) s += Bk[i * mk + a] * Pi[i * ne + j];
            r[L::Y + a * ne + j] = s;
          }
        for (int j = 0; j < ne; ++j) {
          double col[NZ];
          for (int a = 0; a < mk; ++a) col[a] = r[L::Y + a * ne + j];
          ft_chol_solve(Ru, mk, col);
          for (int a = 0; a < mk; ++a) r[L::M + a * ne + j] = col[a];
        }
        for (int i = 0; i < ne; ++i)
          for (int j = 0; j < ne; ++j) {
            double s = 0.0;
            for (int a = 0; a < mk; ++a) s += r[L::Y + a * ne + i] * r[L::M + a * ne + j];
            sh.S[i * ne + j] += s;
          }
        if (k > 0) {
          double Sux[NU * NX];
          for (int a = 0; a < NU; ++a)
            for (int j = 0; j < NX; ++j) {
              double s = 0.0;
              for (int i = 0; i < NX; ++i) s += BP[a * NX + i] * r[L::A + i * NX + j];
              Sux[a * NX + j] = s;
            }
          for (int j = 0; j < NX; ++j) {
            double col[NU];
            for (int a = 0; a < NU; ++a) col[a] = Sux[a * NX + j];
            ft_chol_solve(Ru, NU, col);
            for (int a = 0; a < NU; ++a) r[L::K + a * NX + j] = -col[a];
          }
          double AP[NX * NX], Pn[NX * NX], Pin[NX * NX];
          for (int i = 0; i < NX; ++i)
            for (int j = 0; j < NX; ++j) {
              double s = 0.0;
              for (int q = 0; q < NX; ++q) s += r[L::A + q * NX + i] * Pm[q * NX + j];
              AP[i * NX + j] = s;
            }
          const bool rk = row_at(k);
          for (int i = 0; i < NX; ++i)
            for (int j = 0; j < NX; ++j) {
              double s = (i == j) ? r[L::H + i] : 0.0;
              if (rk) s += r[L::RSIG] * r[L::RG + i] * r[L::RG + j];   // a path row's barrier: sigma c c'
              for (int q = 0; q < NX; ++q) s += AP[i * NX + q] * r[L::A + q * NX + j];
              for (int a = 0; a < NU; ++a) s += Sux[a * NX + i] * r[L::K + a * NX + j];
              Pn[i * NX + j] = s;
            }
          for (int i = 0; i < NX; ++i)
            for (int j = 0; j < i; ++j) {
              const double s = 0.5 * (Pn[i * NX + j] + Pn[j * NX + i]);
              Pn[i * NX + j] = Pn[j * NX + i] = s;
            }
          for (int i = 0; i < NX; ++i)
            for (int j = 0; j < ne; ++j) {
              double s = 0.0;
              for (int q = 0; q < NX; ++q) {
                double acl = r[L::A + q * NX + i];
                for (int a = 0; a < NU; ++a) acl += r[L::B + q * NU + a] * r[L::K + a * NX + i];
                s += acl * Pi[q * ne + j];
              }
              Pin[i * ne + j] = s;
            }
          for (int i = 0; i < NX * NX; ++i) { Pm[i] = Pn[i]; Pi[i] = Pin[i]; }
        }
      }
      const double* Lr = r + L::LR;
      for (int i = 0; i < NX; ++i) v[i] = r[L::PE + i] + p[i];
      for (int a = 0; a < mk; ++a) {
        double s = r[L::G + uoff + a];
        for (int i = 0; i < NX; ++i) s += Bk[i * mk + a] * v[i];
        rr[a] = s;
      }
      double kf[NZ], Lc[NZ * NZ];
      for (int e2 = 0; e2 < mk * mk; ++e2) Lc[e2] = Lr[e2];
      for (int a = 0; a < mk; ++a) kf[a] = rr[a];
      ft_chol_solve(Lc, mk, kf);
      for (int a = 0; a < mk; ++a) kf[a] = -kf[a];
      if (k > 0) {
        for (int a = 0; a < NU; ++a) r[L::KF + a] = kf[a];
        double pn[NX];
        for (int i = 0; i < NX; ++i) {
          double s = r[L::G + i];
          for (int q = 0; q < NX; ++q) s += r[L::A + q * NX + i] * v[q];
          for (int a = 0; a < NU; ++a) s += r[L::K + a * NX + i] * rr[a];
          pn[i] = s;
        }
        for (int i = 0; i < NX; ++i) p[i] = pn[i];
      } else {
        for (int a = 0; a < mk; ++a) r[L::D + a] = kf[a];
      }
      for (int j = 0; j < ne; ++j) {
        double s = 0.0;
        for (int a = 0; a < mk; ++a) s += r[L::Y + a * ne + j] * kf[a];
        lin[j] += s;
      }
    }
    // terminal multiplier nu = S^-1 (E d_N^0 - e_N)
    if (ne > 0) {
      double Sc[NX * NX], rhs[NX];
      for (int e2 = 0; e2 < ne * ne; ++e2) Sc[e2] = sh.S[e2];
      if (!ft_chol<NX>(Sc, ne)) return false;
      for (int j = 0; j < ne; ++j) rhs[j] = lin[j] + sh.lin_e[j] - rs * rN[L::E0 + j];
      ft_chol_solve(Sc, ne, rhs);
      for (int j = 0; j < ne; ++j) sh.nun[j] = rhs[j];
    }
    // forward sweep
    double* r0 = rec(0);
    double w[NZ], dx[NX];
    for (int a = 0; a < m0; ++a) {
      double s = r0[L::D + a];
      for (int j = 0; j < ne; ++j) s -= r0[L::M + a * ne + j] * sh.nun[j];
      w[a] = s;
    }
    for (int a = 0; a < m0; ++a) r0[L::D + a] = w[a];
    for (int i = 0; i < NX; ++i) {
      double s = rs * r0[L::E0 + i];
      for (int a = 0; a < m0; ++a) s += r0[L::F0 + i * m0 + a] * w[a];
      dx[i] = s;
    }
    for (int k = 1; k < N; ++k) {
      double* r = rec(k);
      double du[NU], dn[NX];
      for (int a = 0; a < NU; ++a) {
        double s = r[L::KF + a];
        for (int i = 0; i < NX; ++i) s += r[L::K + a * NX + i] * dx[i];
        for (int j = 0; j < ne; ++j) s -= r[L::M + a * ne + j] * sh.nun[j];
        du[a] = s;
      }
      for (int i = 0; i < NX; ++i) r[L::D + i] = dx[i];
      for (int a = 0; a < NU; ++a) r[L::D + NX + a] = du[a];
      for (int i = 0; i < NX; ++i) {
        double s = rs * r[L::E0 + i];
        for (int q = 0; q < NX; ++q) s += r[L::A + i * NX + q] * dx[q];
        for (int a = 0; a < NU; ++a) s += r[L::B + i * NU + a] * du[a];
        dn[i] = s;
      }
      for (int i = 0; i < NX; ++i) dx[i] = dn[i];
    }
    double* rNw = rec(N);
    for (int i = 0; i < NX; ++i) rNw[L::D + i] = dx[i];
    return true;
  }

  // ---- interior-point QP ------------------------------------------------------------------------
  // returns 0 converged, 1 max-iter, -1 failure; iterations in qit
  __device__ int qp(int& qit) {
    const int N = sh.N, ne = sh.ne, m0 = sh.nf0 + NU;
    const double rho = o.lm;
    double nb = 0.0;
    for (int k = t; k <= N; k += 64) {
      double* r = rec(k);
      for (int i = 0; i < nz(k); ++i) {
        double v, lb, ub;
        if (!comp(k, i, v, lb, ub)) {
          r[L::DZ + i] = 0.0; r[L::QL + i] = 0.0; r[L::QU + i] = 0.0; r[L::LB + i] = -INFINITY; r[L::UB + i] = INFINITY;
          continue;
        }
        const double Lo = lb - v, Up = ub - v, del = o.push * (Up - Lo);
        double z0 = 0.0;
        if (z0 < Lo + del) z0 = Lo + del;
        if (z0 > Up - del) z0 = Up - del;
        r[L::LB + i] = Lo; r[L::UB + i] = Up; r[L::DZ + i] = z0;
        r[L::QL + i] = o.mu0 / (z0 - Lo);
        r[L::QU + i] = o.mu0 / (Up - z0);
        nb += 2.0;
      }
      if (row_at(k)) {
        // the row: slacks from the initial c'dz, clipped to ipm_push (infeasible start); a soft row's slack starts
        // at the row's violation + ipm_push, so its lower side starts feasible
        const double gd = row_dot(r, k, L::DZ);
        r[L::RL] = mp.lh - r[L::RV];
        r[L::RU] = mp.uh - r[L::RV];
        double gs = gd;
        r[L::RS] = r[L::RQS] = r[L::RAS] = r[L::RAQS] = 0.0;
        if (mp.soft) {
          r[L::RS] = fmax(r[L::RL] - gd, 0.0) + o.push;
          r[L::RQS] = o.mu0 / r[L::RS];
          gs = gd + r[L::RS];
          nb += 1.0;
        }
        r[L::RTL] = fmax(gs - r[L::RL], o.push);
        r[L::RTU] = fmax(r[L::RU] - gd, o.push);
        r[L::RQL] = o.mu0 / r[L::RTL];
        r[L::RQU] = o.mu0 / r[L::RTU];
        r[L::RR0L] = gs - r[L::RL] - r[L::RTL];
        r[L::RR0U] = r[L::RU] - gd - r[L::RTU];
        r[L::RATL] = r[L::RATU] = r[L::RAQL] = r[L::RAQU] = 0.0;
        nb += 2.0;
      }
    }
    const double nbox = ft_wsum(nb);
    __syncthreads();
    double e00 = 0.0, rd0 = 0.0;
    for (int k = t; k <= N; k += 64) {
      double* r = rec(k);
      if (k < N) {
        const double* r1 = rec(k + 1);
        for (int i = 0; i < NX; ++i) {
          double s = r[L::BD + i] - r1[L::DZ + i];
          if (k == 0) {
            for (int a = 0; a < m0; ++a) s += r[L::F0 + i * m0 + a] * r[L::DZ + a];
          } else {
            for (int q = 0; q < NX; ++q) s += r[L::A + i * NX + q] * r[L::DZ + q];
            for (int a = 0; a < NU; ++a) s += r[L::B + i * NU + a] * r[L::DZ + NX + a];
          }
          r[L::E0 + i] = s;
          e00 = fmax(e00, fabs(s));
        }
      } else {
        for (int j = 0; j < ne; ++j) {
          const double s = sh.ev[j] - r[L::X + sh.ei[j]] - r[L::DZ + sh.ei[j]];
          r[L::E0 + j] = s;
          e00 = fmax(e00, fabs(s));
        }
      }
      const bool rk = row_at(k);
      for (int i = 0; i < nz(k); ++i) {
        const int xi = k == 0 ? (i < sh.nf0 ? sh.f0[i] : -1) : (i < NX ? i : -1);
        rd0 = fmax(rd0, fabs((rho + hq(k, i)) * r[L::DZ + i] + grad(k, i) - r[L::QL + i] + r[L::QU + i] +
                             ((rk && xi >= 0) ? r[L::RG + xi] * (r[L::RQU] - r[L::RQL]) : 0.0)));
      }
      if (rk) {
        e00 = fmax(e00, fmax(fabs(r[L::RR0L]), fabs(r[L::RR0U])));
        if (mp.soft) rd0 = fmax(rd0, fabs(r[L::RZ2] * r[L::RS] + r[L::RZL] - r[L::RQL] - r[L::RQS]));
      }
    }
    e00 = ft_wmax(e00);
    rd0 = ft_wmax(rd0);
    if (t == 0) {
      sh.rs = 1.0;
      for (int j = 0; j < NX; ++j) sh.qnu[j] = 0.0;
    }
    __syncthreads();
    int it, status = 1;
    for (it = 0; it < o.qp_max_iter; ++it) {
      double mu = 0.0;
      for (int k = t; k <= N; k += 64) {
        const double* r = rec(k);
        for (int i = 0; i < nz(k); ++i) {
          if (!isfinite(r[L::LB + i])) continue;
          mu += (r[L::DZ + i] - r[L::LB + i]) * r[L::QL + i] + (r[L::UB + i] - r[L::DZ + i]) * r[L::QU + i];
        }
        if (row_at(k)) {
          mu += r[L::RTL] * r[L::RQL] + r[L::RTU] * r[L::RQU];
          if (mp.soft) mu += r[L::RS] * r[L::RQS];
        }
      }
      mu = ft_wsum(mu) / nbox;
      if (!isfinite(mu)) { status = -1; break; }
      const double rs = sh.rs;
      if (mu < o.qp_tol_comp && rs * rd0 < o.qp_tol_stat && rs * e00 < o.qp_tol_eq) { status = 0; break; }
      // predictor: barrier Hessian and gradient
      for (int k = t; k <= N; k += 64) {
        double* r = rec(k);
        for (int i = 0; i < nz(k); ++i) {
          const double hh = rho + hq(k, i);
          double Hh = hh;
          const double gg = hh * r[L::DZ + i] + grad(k, i);
          if (isfinite(r[L::LB + i]))
            Hh += r[L::QL + i] / (r[L::DZ + i] - r[L::LB + i]) + r[L::QU + i] / (r[L::UB + i] - r[L::DZ + i]);
          r[L::H + i] = Hh; r[L::G + i] = gg;
        }
        if (row_at(k)) {   // the row's predictor term c gamma in the stage gradient
          r[L::RATL] = r[L::RATU] = r[L::RAQL] = r[L::RAQU] = r[L::RAS] = r[L::RAQS] = 0.0;
          double rcl, rcu, rcs;
          row_rc(r, 0.0, rcl, rcu, rcs);
          row_addgrad(r, k, row_gamma(r, rs, rcl, rcu, rcs, true));
        }
      }
      __syncthreads();
      if (!newton(true)) { status = -1; break; }
      FtRatio ma{1.0, 1.0};
      for (int k = t; k <= N; k += 64) {
        double* r = rec(k);
        for (int i = 0; i < nz(k); ++i) {
          const double d = r[L::D + i];
          r[L::DAFF + i] = d;
          if (!isfinite(r[L::LB + i])) continue;
          const double tl = r[L::DZ + i] - r[L::LB + i], tu = r[L::UB + i] - r[L::DZ + i];
          const double ql = r[L::QL + i], qu = r[L::QU + i];
          const double dll = -ql - ql * d / tl, dlu = -qu + qu * d / tu;
          ma.add(tl, d); ma.add(tu, -d); ma.add(ql, dll); ma.add(qu, dlu);
        }
        if (row_at(k)) {
          double rcl, rcu, rcs, dtl, dtu, dql, dqu, ds, dqs;
          row_rc(r, 0.0, rcl, rcu, rcs);
          row_dirs(r, row_dot(r, k, L::D), rs, rcl, rcu, rcs, dtl, dtu, dql, dqu, ds, dqs);
          r[L::RATL] = dtl; r[L::RATU] = dtu; r[L::RAQL] = dql; r[L::RAQU] = dqu; r[L::RAS] = ds; r[L::RAQS] = dqs;
          ma.add(r[L::RTL], dtl); ma.add(r[L::RTU], dtu); ma.add(r[L::RQL], dql); ma.add(r[L::RQU], dqu);
          if (mp.soft) { ma.add(r[L::RS], ds); ma.add(r[L::RQS], dqs); }
        }
      }
      const double aa = ma.reduce();
      double muaff = 0.0;
      for (int k = t; k <= N; k += 64) {
        const double* r = rec(k);
        for (int i = 0; i < nz(k); ++i) {
          if (!isfinite(r[L::LB + i])) continue;
          const double d = r[L::D + i], tl = r[L::DZ + i] - r[L::LB + i], tu = r[L::UB + i] - r[L::DZ + i];
          const double ql = r[L::QL + i], qu = r[L::QU + i];
          const double dll = -ql - ql * d / tl, dlu = -qu + qu * d / tu;
          muaff += (tl + aa * d) * (ql + aa * dll) + (tu - aa * d) * (qu + aa * dlu);
        }
        if (row_at(k)) {
          muaff += (r[L::RTL] + aa * r[L::RATL]) * (r[L::RQL] + aa * r[L::RAQL]) +
                   (r[L::RTU] + aa * r[L::RATU]) * (r[L::RQU] + aa * r[L::RAQU]);
          if (mp.soft) muaff += (r[L::RS] + aa * r[L::RAS]) * (r[L::RQS] + aa * r[L::RAQS]);
        }
      }
      muaff = ft_wsum(muaff) / nbox;
      double sig = muaff / mu;
      sig = sig * sig * sig;
      if (sig > 1.0) sig = 1.0;
      const double smu = sig * mu;
      // corrector right-hand side
      for (int k = t; k <= N; k += 64) {
        double* r = rec(k);
        for (int i = 0; i < nz(k); ++i) {
          if (!isfinite(r[L::LB + i])) continue;
          const double tl = r[L::DZ + i] - r[L::LB + i], tu = r[L::UB + i] - r[L::DZ + i], itl = 1.0 / tl, itu = 1.0 / tu;
          const double d = r[L::DAFF + i], ql = r[L::QL + i], qu = r[L::QU + i];
          const double dll = -ql - ql * d * itl, dlu = -qu + qu * d * itu;
          const double rl = smu - tl * ql - d * dll, ru = smu - tu * qu + d * dlu;
          r[L::G + i] = (rho + hq(k, i)) * r[L::DZ + i] + grad(k, i) - ql - rl * itl + qu + ru * itu;
        }
        if (row_at(k)) {   // the row's Mehrotra-corrected term
          double rcl, rcu, rcs;
          row_rc(r, smu, rcl, rcu, rcs);
          row_addgrad(r, k, row_gamma(r, rs, rcl, rcu, rcs, false));
        }
      }
      __syncthreads();
      if (!newton(false)) { status = -1; break; }
      FtRatio mx{1.0, o.tau};
      for (int k = t; k <= N; k += 64) {
        const double* r = rec(k);
        for (int i = 0; i < nz(k); ++i) {
          if (!isfinite(r[L::LB + i])) continue;
          const double tl = r[L::DZ + i] - r[L::LB + i], tu = r[L::UB + i] - r[L::DZ + i], itl = 1.0 / tl, itu = 1.0 / tu;
          const double d = r[L::D + i], da = r[L::DAFF + i], ql = r[L::QL + i], qu = r[L::QU + i];
          const double dlla = -ql - ql * da * itl, dlua = -qu + qu * da * itu;
          const double rl = smu - tl * ql - da * dlla, ru = smu - tu * qu + da * dlua;
          const double dll = (rl - ql * d) * itl, dlu = (ru + qu * d) * itu;
          mx.add(tl, d); mx.add(tu, -d); mx.add(ql, dll); mx.add(qu, dlu);
        }
        if (row_at(k)) {
          double* rw = rec(k);
          double rcl, rcu, rcs;
          row_rc(rw, smu, rcl, rcu, rcs);
          row_dirs(rw, row_dot(rw, k, L::D), rs, rcl, rcu, rcs, rw[L::RDTL], rw[L::RDTU], rw[L::RDQL], rw[L::RDQU],
                   rw[L::RDS], rw[L::RDQS]);
          mx.add(rw[L::RTL], rw[L::RDTL]); mx.add(rw[L::RTU], rw[L::RDTU]);
          mx.add(rw[L::RQL], rw[L::RDQL]); mx.add(rw[L::RQU], rw[L::RDQU]);
          if (mp.soft) { mx.add(rw[L::RS], rw[L::RDS]); mx.add(rw[L::RQS], rw[L::RDQS]); }
        }
      }
      const double alpha = fmin(1.0, o.tau * mx.reduce());
      for (int k = t; k <= N; k += 64) {
        double* r = rec(k);
        for (int i = 0; i < nz(k); ++i) {
          const double d = r[L::D + i];
          if (isfinite(r[L::LB + i])) {
            const double tl = r[L::DZ + i] - r[L::LB + i], tu = r[L::UB + i] - r[L::DZ + i], itl = 1.0 / tl, itu = 1.0 / tu;
            const double da = r[L::DAFF + i], ql = r[L::QL + i], qu = r[L::QU + i];
            const double dlla = -ql - ql * da * itl, dlua = -qu + qu * da * itu;
            const double rl = smu - tl * ql - da * dlla, ru = smu - tu * qu + da * dlua;
            r[L::QL + i] = ql + alpha * (rl - ql * d) * itl;
            r[L::QU + i] = qu + alpha * (ru + qu * d) * itu;
          }
          r[L::DZ + i] += alpha * d;
        }
        if (row_at(k)) {
          r[L::RTL] += alpha * r[L::RDTL]; r[L::RTU] += alpha * r[L::RDTU];
          r[L::RQL] += alpha * r[L::RDQL]; r[L::RQU] += alpha * r[L::RDQU];
          if (mp.soft) {
            r[L::RS] += alpha * r[L::RDS];
            r[L::RQS] += alpha * r[L::RDQS];
          }
        }
      }
      if (t == 0) {
        for (int j = 0; j < ne; ++j) sh.qnu[j] += alpha * (sh.nun[j] - sh.qnu[j]);
        sh.rs = rs * (1.0 - alpha);
      }
      __syncthreads();
    }
    qit = it;
    if (status < 0) return -1;
    // costates by the backward adjoint from the final iterate (lane 0)
    if (t == 0) {
      double lam[NX];
      const double* rN = rec(N);
      for (int i = 0; i < NX; ++i) {
        lam[i] = (rho + hq(N, i)) * rN[L::DZ + i] + grad(N, i) - rN[L::QL + i] + rN[L::QU + i];
        if (row_at(N)) lam[i] += rN[L::RG + i] * (rN[L::RQU] - rN[L::RQL]);
      }
      for (int j = 0; j < ne; ++j) lam[sh.ei[j]] += sh.qnu[j];
      for (int k = N - 1; k >= 0; --k) {
        double* r = rec(k);
        for (int i = 0; i < NX; ++i) r[L::QPI + i] = lam[i];
        if (k == 0) break;
        double ln[NX];
        for (int i = 0; i < NX; ++i) {
          double s = (rho + hq(k, i)) * r[L::DZ + i] + grad(k, i) - r[L::QL + i] + r[L::QU + i];
          if (row_at(k)) s += r[L::RG + i] * (r[L::RQU] - r[L::RQL]);   // a path row's term
          for (int q = 0; q < NX; ++q) s += r[L::A + q * NX + i] * lam[q];
          ln[i] = s;
        }
        for (int i = 0; i < NX; ++i) lam[i] = ln[i];
      }
    }
    int bad = 0;
    for (int k = t; k <= N; k += 64) {
      const double* r = rec(k);
      for (int i = 0; i < nz(k); ++i)
        if (!isfinite(r[L::DZ + i]) || !isfinite(r[L::QL + i]) || !isfinite(r[L::QU + i])) bad = 1;
    }
    __syncthreads();
    if (ft_wmax(bad ? 1.0 : 0.0) > 0.0) return -1;
    return status;
  }

  // ---- merit line search + step ------------------------------------------------------------------
  __device__ void state_at(int k, double alpha, double* x, double* u) const {
    const double* r = rec(k);
    if (k == 0) {
      for (int i = 0; i < NX; ++i) x[i] = r[L::X + i];
      for (int j = 0; j < sh.nf0; ++j) x[sh.f0[j]] += alpha * r[L::DZ + j];
      for (int a = 0; a < NU; ++a) u[a] = r[L::U + a] + alpha * r[L::DZ + sh.nf0 + a];
      return;
    }
    for (int i = 0; i < NX; ++i) x[i] = r[L::X + i] + alpha * r[L::DZ + i];
    if (k < sh.N)
      for (int a = 0; a < NU; ++a) u[a] = r[L::U + a] + alpha * r[L::DZ + NX + a];
  }

  __device__ double merit(double alpha) {
    const int N = sh.N;
    double val = 0.0, viol = 0.0;
    for (int k = t; k <= N; k += 64) {
      const double* r = rec(k);
      for (int i = 0; i < nz(k); ++i) {
        double v, lb, ub;
        if (!comp(k, i, v, lb, ub)) continue;
        v += alpha * r[L::DZ + i];
        viol += fmax(0.0, lb - v) + fmax(0.0, v - ub);
      }
      double xk[NX], uk[NU], xn[NX], un[NU], phi[NX];
      if (k < N) {
        state_at(k, alpha, xk, uk);
        if (mp.on) val += track(k, xk, uk);
        else for (int i = 0; i < NX; ++i) val += (k == 0 ? sh.c0[i] : sh.cp[i]) * xk[i];
        ft_rk4_sens<NQ>(xk, uk, phi, nullptr, nullptr);
        state_at(k + 1, alpha, xn, un);
        for (int i = 0; i < NX; ++i) val += r[L::WPI + i] * fabs(phi[i] - xn[i]);
      } else {
        state_at(N, alpha, xn, un);
        if (mp.on) val += track(N, xn, un);
        for (int j = 0; j < sh.ne; ++j) val += sh.wnu[j] * fabs(xn[sh.ei[j]] - sh.ev[j]);
      }
    }
    double hviol = 0.0, hcost = 0.0;
    if constexpr (MP) {
      if (mp.hid > 0) {
        // the rows' violations at the trial states, weighted like the boxes (uniform: every lane evaluates); a soft
        // row's trial slack, its cost and its bound s >= 0
        for (int k = mp.soft ? 0 : N; k <= N; ++k) {
          double xk[NX], uk[NU];
          state_at(k, alpha, xk, uk);
          const double hv = nn_row(xk, nullptr);
          const double* r = rec(k);
          const double sa = mp.soft ? r[L::RSL] + alpha * (r[L::RS] - r[L::RSL]) : 0.0;
          double v = fmax(0.0, mp.lh - hv - sa) + fmax(0.0, hv - mp.uh);
          if (mp.soft) {
            v += fmax(0.0, -sa);
            hcost += r[L::RZL] * sa + 0.5 * r[L::RZ2] * sa * sa;
          }
          hviol += v;
        }
      }
    }
    return ft_wsum(val) + hcost + sh.wbnd * (ft_wsum(viol) + hviol);
  }

  __device__ void weights() {
    const int N = sh.N;
    double lmax = 0.0;
    for (int k = t; k <= N; k += 64) {
      double* r = rec(k);
      if (k < N)
        for (int i = 0; i < NX; ++i) {
          const double a = fabs(r[L::QPI + i]), b = 0.5 * (r[L::WPI + i] + a);
          r[L::WPI + i] = a > b ? a : b;
        }
      for (int i = 0; i < nz(k); ++i) lmax = fmax(lmax, fmax(r[L::QL + i], r[L::QU + i]));
      if (row_at(k)) {
        lmax = fmax(lmax, fmax(r[L::RQL], r[L::RQU]));
        if (mp.soft) lmax = fmax(lmax, r[L::RQS]);
      }
    }
    lmax = ft_wmax(lmax);
    if (t == 0) {
      for (int j = 0; j < sh.ne; ++j) {
        const double a = fabs(sh.qnu[j]), b = 0.5 * (sh.wnu[j] + a);
        sh.wnu[j] = a > b ? a : b;
      }
      const double b = 0.5 * (sh.wbnd + lmax);
      sh.wbnd = lmax > b ? lmax : b;
    }
    __syncthreads();
  }

  __device__ void apply(double alpha) {
    const int N = sh.N;
    for (int k = t; k <= N; k += 64) {
      double* r = rec(k);
      double x[NX], u[NU];
      state_at(k, alpha, x, u);
      for (int i = 0; i < NX; ++i) r[L::X + i] = x[i];
      if (k < N)
        for (int a = 0; a < NU; ++a) r[L::U + a] = u[a];
      for (int i = 0; i < nz(k); ++i) {
        r[L::LL + i] += alpha * (r[L::QL + i] - r[L::LL + i]);
        r[L::LU + i] += alpha * (r[L::QU + i] - r[L::LU + i]);
      }
      if (k < N)
        for (int i = 0; i < NX; ++i) r[L::PI + i] += alpha * (r[L::QPI + i] - r[L::PI + i]);
      if (row_at(k)) {
        r[L::RLL] += alpha * (r[L::RQL] - r[L::RLL]);
        r[L::RLU] += alpha * (r[L::RQU] - r[L::RLU]);
        if (mp.soft) {
          r[L::RSL] += alpha * (r[L::RS] - r[L::RSL]);
          r[L::RLSL] += alpha * (r[L::RQS] - r[L::RLSL]);
        }
      }
    }
    if (t == 0) {
      for (int j = 0; j < sh.ne; ++j) sh.tnu[j] += alpha * (sh.qnu[j] - sh.tnu[j]);
    }
    __syncthreads();
  }

  __device__ int run(int& it, int& qtot) {
    int status = 2;
    qtot = 0;
    for (it = 0;; ++it) {
      linearize();
      double rstat, req, rineq, rcomp;
      residuals(rstat, req, rineq, rcomp);
      if (!isfinite(rstat) || !isfinite(req)) { status = 1; break; }
      const bool rti = MP && mp.rti;
      if (rti && it == 1) { status = 0; break; }   // SQP_RTI: one QP and its full step
      if (!rti && rstat < o.tol_stat && req < o.tol_eq && rineq < o.tol_ineq && rcomp < o.tol_comp) { status = 0; break; }
      if (it >= o.max_iter) { status = 2; break; }
      int qit = 0;
      const int qs = qp(qit);
      qtot += qit;
      if (qs < 0 || (MP && mp.qcf && qs == 1)) { status = 4; break; }
      weights();
      double alpha = 1.0;
      if (!rti) {
        const double phi0 = merit(0.0);
        for (;;) {
          const double pa = merit(alpha);
          if (pa < phi0) break;
          if (alpha * o.alpha_red < o.alpha_min) break;
          alpha *= o.alpha_red;
        }
      }
      apply(alpha);
      if (!isfinite(rec(0)[L::X + NX - 1])) { status = 1; break; }
    }
    return status;
  }
};

// one workgroup = one wave = one problem at a time; workgroups pull problem ids until none are left
template <int NQ, bool MP>
__global__ __launch_bounds__(64) void k_ft(Opts o, Inputs in, double* regions, long long region_doubles,
                                           unsigned* head, MpcArgs mp) {
  __shared__ FtShared<NQ, MP> sh;
  __shared__ int job;
  const int t = (int)threadIdx.x;
  Ft<NQ, MP> F(sh, regions + (long long)blockIdx.x * region_doubles, o, t, mp);
  for (;;) {
    if (t == 0) job = (int)atomicAdd(head, 1u);
    __syncthreads();
    const int pid = job;
    __syncthreads();
    if (pid >= in.B) break;
    F.load(in, pid);
    if (sh.bad) {
      if (t == 0) {
        in.status[pid] = 5;
        in.cost[pid] = NAN;
        in.sqp_iter[pid] = 0;
        in.qp_iter[pid] = 0;
      }
      __syncthreads();
      continue;
    }
    int it = 0, qit = 0;
    const int status = F.run(it, qit);
    F.store(in, status, it, qit);
    __syncthreads();
  }
}

}  // namespace vboc

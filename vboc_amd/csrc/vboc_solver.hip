// vboc_solver.hip - MI355X-native batched boundary-OCP solver (the ACADOS SQP/HPIPM path of
// OCP<sys>INIT.OCP_solve, VBOC/triplependulum_class_vboc.py:155-191, run for a whole batch).
//
// Execution model (DESIGN.md "Kernels"):
//  * one OCP per LANE.  A wave carries 64 independent problems; every per-stage quantity is stored
//    slot-major SoA in HBM, [stage][field][slot], so the 64 lanes of a wave touch 512 contiguous
//    bytes per (stage, field) access - fully coalesced, no LDS needed, no cross-lane traffic.
//    Stage loops run over a wave-uniform stage index (bound = the wave's largest horizon, lanes
//    with a shorter horizon are predicated off), so every access is SGPR base + one per-lane VGPR
//    offset;
//  * a persistent kernel: each lane pulls problems from a global work queue (wave-aggregated
//    atomicAdd on one head word) and runs the SQP to termination, one synchronous SQP iteration at
//    a time for the whole wave, then pulls the next problem.  The SQP iteration count has a long
//    tail (median ~20, cap 1000), so the queue keeps lanes busy instead of idling behind the
//    slowest problem of a statically assigned wave;
//  * per SQP iteration: ERK4 + forward sensitivities (compute-heavy, registers only), then the
//    Riccati interior-point QP whose stage sweeps stream A_k, B_k, factors and iterates through HBM
//    (memory-bound), then merit line search (re-simulation) and the primal/dual update.
// Arithmetic is FP64 throughout (near-LP QPs with a 1e-5 Hessian need it).
//
// The algorithm is the one restated in oracle/vboc_oracle.c (the checker); see that file for the
// reference line of every option and reformulation.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/vboc.h"
#include "model.h"

#define UNR _Pragma("unroll")
#ifdef VBOC_WAVES
#define VBOC_WPE __attribute__((amdgpu_waves_per_eu(VBOC_WAVES, VBOC_WAVES)))
#else
#define VBOC_WPE
#endif

namespace vboc {

struct Opts {
  double tol_stat, tol_eq, tol_ineq, tol_comp;
  double qp_tol_stat, qp_tol_eq, qp_tol_comp;
  double alpha_min, alpha_red, lm, mu0, push, tau;
  int max_iter, qp_max_iter;
  // Cartesian path constraint hlh <= |tip(theta_k) - (hxc, hyc)|^2 <= huh on stages 0..N-1 (hc != 0;
  // vboc_set_path_constraint, VBOC/Cartesian constraints/doublependulum_class_fixedveldir.py:154-160)
  int hc;
  double hxc, hyc, hlh, huh;
};

// Slot-major workspace.  Field counts per stage are fixed by NQ.
struct Work {
  double *X, *U, *PI, *LL, *LU, *WPI;        // SQP iterate + NLP multipliers + merit weights
  double *A, *Bm, *BD;                        // linearisation (A_k, B_k, defect b_k)
  double *DZ, *QL, *QU, *E0;                  // IPM iterate (step, bound duals), initial residual
  double *K, *KF, *LR, *M, *Y, *PE, *D, *DAFF, *QPI;  // Riccati factors, directions, costate
  double *F0, *LR0, *M0, *Y0, *PE0, *PAR;     // stage-0 specials, problem parameters (per slot)
  double* HC;                                 // path-constraint rows (allocated with the constraint)
  long long S;                                // number of slots (lanes)
};

struct Inputs {
  int B, nmax;
  const int* N;
  const double *xg, *ug, *p, *lbx, *ubx, *lbu, *ubu, *lbx0, *ubx0, *lbxe, *ubxe;
  int* status;
  double *xo, *uo, *cost;
  int *sqp_iter, *qp_iter;
  unsigned int* head;   // work-queue head
};

// per-slot parameter fields
template <int NQ>
struct Par {
  static constexpr int NX = 2 * NQ, NU = NQ;
  enum : int {
    H = 0, Q0 = 1, DIR = Q0 + NQ, SLB = DIR + NQ, SUB, CS, CCONST, XLB, XUB = XLB + NX, ULB = XUB + NX,
    UUB = ULB + NU, QNLB = UUB + NU, QNUB = QNLB + NQ, VFIN = QNUB + NQ, S = VFIN + NQ, NU_ = S + 1,
    WNU = NU_ + NQ, WBND = WNU + NQ, E0N = WBND + 1, QNU = E0N + NQ,
    // interior-point scalars carried between the per-sweep kernels
    RS = QNU + NQ, RD0, E00, MU, NBOX, SMU, ALPHA, SC, LINE = SC + NQ * NQ, W0 = LINE + NQ, NUN = W0 + NQ + 1,
    COUNT = NUN + NQ
  };
};

// Force a wave-uniform pointer into SGPRs.  Opaque to loop strength reduction, so each access
// becomes `global_load ... vOFF, s[base]` with ONE shared per-lane offset register instead of a
// 64-bit per-field VGPR induction pointer.  Only for pointers that ARE uniform.
// Global-address-space double: loads/stores through it are `global_*` (never `flat_*`, which
// would be ordered against LDS/scratch and drained with vmcnt(0) lgkmcnt(0) one by one).
typedef __attribute__((address_space(1))) double gdouble;

__device__ __forceinline__ gdouble* gptr(double* p) { return (gdouble*)(unsigned long long)p; }

__device__ __forceinline__ gdouble* uptr(double* p) {
  const unsigned long long v = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return (gdouble*)(((unsigned long long)hi << 32) | lo);
}

__device__ __forceinline__ int wave_max(int v) {
  UNR for (int off = 32; off >= 1; off >>= 1) v = max(v, __shfl_xor(v, off));
  return __builtin_amdgcn_readfirstlane(v);
}

template <int NQ>
struct Lane {
  static constexpr int NX = 2 * NQ, NU = NQ, NZ = 3 * NQ, M0 = NQ + 1;
  static constexpr int FX = NX, FU = NU, FPI = NX, FZ = NZ, FA = NX * NX, FB = NX * NU, FK = NU * NX,
                       FLR = NU * NU, FM = NU * NQ;
  using PF = Par<NQ>;
  // per-stage fields of the Cartesian path-constraint row (w.HC; stages 1..N-1, see hc_on): h and
  // dh/dtheta at the iterate, NLP multipliers, QP slacks / duals, their residuals at the QP start and
  // their affine directions
  enum : int {
    HV = 0, HG = 1, HLL = 1 + NQ, HLU, HTL, HTU, HQL, HQU, HR0L, HR0U, HATL, HATU, HAQL, HAQU, FHC
  };

  const Work& w;
  const Opts& o;
  const unsigned slot;
  const int wv;   // wave index (wave-uniform, SGPR)
  const int ln;   // lane in wave
  int N;    // this lane's horizon
  int Nw;   // wave-uniform: largest horizon of the wave's active lanes (SGPR)
  // QP scalars (registers only while the QP runs)
  double rs, rd0, e00, mu, nbox;

  __device__ Lane(const Work& w_, const Opts& o_, unsigned slot_)
      : w(w_), o(o_), slot(slot_), wv(__builtin_amdgcn_readfirstlane((int)(slot_ >> 6))), ln((int)(slot_ & 63u)),
        N(0), Nw(0) {}

  // Wave-tiled, field-paired SoA: element (stage k, field f) of lane `ln` of wave `wv` lives at
  //   base[((k * SW + wv) * FP + f / 2) * 128 + ln * 2 + f % 2],  SW = S / 64, FP = ceil(F / 2).
  // A wave-instruction covering fields (2p, 2p+1) reads 64 x 16 B = 1 KiB contiguous
  // (global_load_dwordx4), and one base register per (array, stage) serves 8 fields through
  // immediate offsets.
  static constexpr int fp(int F) { return (F + 1) / 2; }
  __device__ __forceinline__ gdouble* stage_base(double* base, int F, int k) const {
    return gptr(base) + (((long long)k * (w.S >> 6) + wv) * fp(F)) * 128 + ln * 2;
  }
  __device__ __forceinline__ gdouble& at(double* base, int F, int k, int f) const {
    return stage_base(base, F, k)[(f >> 1) * 128 + (f & 1)];
  }
  // k per lane (the terminal stage N) - same formula, per-lane arithmetic
  __device__ __forceinline__ gdouble& atv(double* base, int F, int k, int f) const {
    return stage_base(base, F, k)[(f >> 1) * 128 + (f & 1)];
  }
  template <bool U>
  __device__ __forceinline__ gdouble& atk(double* base, int F, int k, int f) const {
    return stage_base(base, F, k)[(f >> 1) * 128 + (f & 1)];
  }
  // per-slot arrays (no stage index)
  __device__ __forceinline__ gdouble& at0(double* base, int F, int f) const {
    return (gptr(base) + ((long long)wv * fp(F)) * 128 + ln * 2)[(f >> 1) * 128 + (f & 1)];
  }
  __device__ __forceinline__ gdouble& par(int f) const { return at0(w.PAR, PF::COUNT, f); }

  // ---- Cartesian path constraint (oracle/vboc_oracle.c hc_*): the chain tip's squared distance to the
  // centre, a general row c'dz in [lh - h, uh - h] with c = dh/dtheta on stages 1..N-1 (stage 0's
  // positions are fixed: checked once in k_refill) ----
  __device__ __forceinline__ bool hc_on(int k) const { return o.hc && k >= 1 && k < N; }
  __device__ __forceinline__ gdouble& hcf(int k, int f) const { return at(w.HC, FHC, k, f); }
  __device__ __forceinline__ double hc_eval(const double* x, double* grad) const {
    constexpr double l = Chain<NQ>::l;
    double X = 0.0, Y = 0.0;
    UNR for (int j = 0; j < NQ; ++j) { X += l * sin(x[j]); Y += l * cos(x[j]); }
    const double dx = X - o.hxc, dy = Y - o.hyc;
    if (grad) {
      UNR for (int j = 0; j < NQ; ++j) grad[j] = 2.0 * dx * (l * cos(x[j])) - 2.0 * dy * (l * sin(x[j]));
    }
    return dx * dx + dy * dy;
  }
  // Newton directions of the row's slacks and duals from the stage step d (corrector right-hand sides
  // with the stored affine directions when CORR, the predictor's otherwise)
  template <bool CORR>
  __device__ __forceinline__ void hc_dir(int k, const double (&d)[NZ], double smu, double& dtl, double& dtu,
                                         double& dql, double& dqu) const {
    double cd = 0.0;
    UNR for (int j = 0; j < NQ; ++j) cd += hcf(k, HG + j) * d[j];
    const double htl = hcf(k, HTL), htu = hcf(k, HTU), hql = hcf(k, HQL), hqu = hcf(k, HQU);
    const double rl = rs * hcf(k, HR0L), ru = rs * hcf(k, HR0U);
    const double rcl = CORR ? smu - htl * hql - hcf(k, HATL) * hcf(k, HAQL) : -htl * hql;
    const double rcu = CORR ? smu - htu * hqu - hcf(k, HATU) * hcf(k, HAQU) : -htu * hqu;
    dtl = cd + rl;
    dtu = ru - cd;
    dql = (rcl - hql * dtl) / htl;
    dqu = (rcu - hqu * dtu) / htu;
  }

  // ---------------------------------------------------------------------------------------------
  // stage component view: value, bounds, boxed flag of the NZ step components of stage k
  // stage 0: (s, u_0); 0<k<N: (x_k, u_k); k == N: x_N with only the positions boxed.
  // ---------------------------------------------------------------------------------------------
  template <bool U = true>
  __device__ __forceinline__ void stage_box(int k, double (&z)[NZ], double (&lb)[NZ], double (&ub)[NZ],
                                            bool (&bx)[NZ]) const {
    if (k == 0) {
      z[0] = par(PF::S); lb[0] = par(PF::SLB); ub[0] = par(PF::SUB); bx[0] = true;
      UNR for (int a = 0; a < NU; ++a) {
        z[1 + a] = at(w.U, FU, 0, a); lb[1 + a] = par(PF::ULB + a); ub[1 + a] = par(PF::UUB + a); bx[1 + a] = true;
      }
      UNR for (int i = M0; i < NZ; ++i) { z[i] = 0; lb[i] = -1; ub[i] = 1; bx[i] = false; }
    } else if (k == N) {
      UNR for (int i = 0; i < NX; ++i) {
        z[i] = atk<U>(w.X, FX, k, i);
        const bool b = i < NQ;
        bx[i] = b;
        lb[i] = b ? par(PF::QNLB + (i < NQ ? i : 0)) : -1;
        ub[i] = b ? par(PF::QNUB + (i < NQ ? i : 0)) : 1;
      }
      UNR for (int i = NX; i < NZ; ++i) { z[i] = 0; lb[i] = -1; ub[i] = 1; bx[i] = false; }
    } else {
      UNR for (int i = 0; i < NX; ++i) {
        z[i] = atk<U>(w.X, FX, k, i); lb[i] = par(PF::XLB + i); ub[i] = par(PF::XUB + i); bx[i] = true;
      }
      UNR for (int a = 0; a < NU; ++a) {
        z[NX + a] = atk<U>(w.U, FU, k, a); lb[NX + a] = par(PF::ULB + a); ub[NX + a] = par(PF::UUB + a); bx[NX + a] = true;
      }
    }
  }

  // ---------------------------------------------------------------------------------------------
  // problem setup / output (per lane, divergent - once per problem)
  // ---------------------------------------------------------------------------------------------
  // Reads problem `pid` into this slot.  Returns false (nothing loaded) if its structure is
  // outside what the boundary-OCP solver implements: dt not pinned by the bounds, stage-0
  // positions not fixed, terminal velocities not fixed, horizon out of range.
  __device__ __forceinline__ bool supported(const Inputs& in, int pid) const {
    constexpr int NXR = NX + 1;
    const int n = in.N[pid];
    if (n < 1 || n > in.nmax) return false;
    const double* lbx = in.lbx + (long long)pid * NXR;
    const double* ubx = in.ubx + (long long)pid * NXR;
    const double* lbx0 = in.lbx0 + (long long)pid * NXR;
    const double* ubx0 = in.ubx0 + (long long)pid * NXR;
    const double* lbxe = in.lbxe + (long long)pid * NXR;
    const double* ubxe = in.ubxe + (long long)pid * NXR;
    bool ok = lbx[NX] == ubx[NX] && lbx0[NX] == lbx[NX] && ubx0[NX] == lbx[NX] && lbxe[NX] == lbx[NX] &&
              ubxe[NX] == lbx[NX] && lbx[NX] > 0.0;
    UNR for (int j = 0; j < NQ; ++j) ok = ok && lbx0[j] == ubx0[j] && lbxe[NQ + j] == ubxe[NQ + j];
    return ok;
  }

  __device__ void load(const Inputs& in, int pid) {
    constexpr int NXR = NX + 1, NP = NQ + 1;
    N = in.N[pid];
    const double* p = in.p + (long long)pid * NP;
    const double* lbx = in.lbx + (long long)pid * NXR;
    const double* ubx = in.ubx + (long long)pid * NXR;
    const double* lbx0 = in.lbx0 + (long long)pid * NXR;
    const double* ubx0 = in.ubx0 + (long long)pid * NXR;
    const double* lbxe = in.lbxe + (long long)pid * NXR;
    const double* ubxe = in.ubxe + (long long)pid * NXR;
    const double h = lbx[NX];
    par(PF::H) = h;
    double nrm = 0.0;
    UNR for (int j = 0; j < NQ; ++j) nrm += p[j] * p[j];
    nrm = sqrt(nrm);
    double slb = -INFINITY, sub = INFINITY, cs = 0.0, dir[NQ];
    UNR for (int j = 0; j < NQ; ++j) {
      dir[j] = (NQ == 1) ? 1.0 : p[j] / nrm;
      par(PF::DIR + j) = dir[j];
      par(PF::Q0 + j) = lbx0[j];
      cs += p[j] * dir[j];
      const double dj = dir[j], lo = lbx0[NQ + j], hi = ubx0[NQ + j];
      if (dj > 0) { slb = fmax(slb, lo / dj); sub = fmin(sub, hi / dj); }
      else if (dj < 0) { slb = fmax(slb, hi / dj); sub = fmin(sub, lo / dj); }
    }
    par(PF::SLB) = slb; par(PF::SUB) = sub; par(PF::CS) = cs;
    par(PF::CCONST) = p[NQ] * h * (double)N;
    UNR for (int i = 0; i < NX; ++i) { par(PF::XLB + i) = lbx[i]; par(PF::XUB + i) = ubx[i]; }
    UNR for (int a = 0; a < NU; ++a) {
      par(PF::ULB + a) = in.lbu[(long long)pid * NU + a];
      par(PF::UUB + a) = in.ubu[(long long)pid * NU + a];
    }
    UNR for (int j = 0; j < NQ; ++j) {
      par(PF::QNLB + j) = lbxe[j]; par(PF::QNUB + j) = ubxe[j]; par(PF::VFIN + j) = lbxe[NQ + j];
      par(PF::NU_ + j) = 0.0; par(PF::WNU + j) = 0.0;
    }
    par(PF::WBND) = 0.0;
    const double* xg = in.xg + (long long)pid * (in.nmax + 1) * NXR;
    const double* ug = in.ug + (long long)pid * in.nmax * NU;
    double s = 0.0;
    UNR for (int j = 0; j < NQ; ++j) s += dir[j] * xg[NQ + j];
    par(PF::S) = s;
    for (int k = 0; k <= N; ++k) {
      UNR for (int i = 0; i < NX; ++i) atv(w.X, FX, k, i) = xg[(long long)k * NXR + i];
      UNR for (int i = 0; i < NZ; ++i) { atv(w.LL, FZ, k, i) = 0.0; atv(w.LU, FZ, k, i) = 0.0; }
      if (o.hc && k >= 1 && k < N) { atv(w.HC, FHC, k, HLL) = 0.0; atv(w.HC, FHC, k, HLU) = 0.0; }
      if (k < N) {
        UNR for (int a = 0; a < NU; ++a) atv(w.U, FU, k, a) = ug[(long long)k * NU + a];
        UNR for (int i = 0; i < NX; ++i) { atv(w.PI, FPI, k, i) = 0.0; atv(w.WPI, FX, k, i) = 0.0; }
      }
    }
  }

  __device__ void store_result(const Inputs& in, int pid, int status, int sqp_it, int qp_tot) {
    constexpr int NXR = NX + 1;
    double* xo = in.xo + (long long)pid * (in.nmax + 1) * NXR;
    double* uo = in.uo + (long long)pid * in.nmax * NU;
    const double s = par(PF::S), h = par(PF::H);
    for (int k = 0; k <= N; ++k) {
      UNR for (int i = 0; i < NX; ++i) {
        const double v = (k == 0) ? (i < NQ ? par(PF::Q0 + i) : s * par(PF::DIR + (i - NQ + (i < NQ ? NQ : 0))))
                                  : (double)atv(w.X, FX, k, i);
        xo[(long long)k * NXR + i] = v;
      }
      xo[(long long)k * NXR + NX] = h;
      if (k < N) {
        UNR for (int a = 0; a < NU; ++a) uo[(long long)k * NU + a] = atv(w.U, FU, k, a);
      }
    }
    in.status[pid] = status;
    in.cost[pid] = par(PF::CS) * s + par(PF::CCONST);
    in.sqp_iter[pid] = sqp_it;
    in.qp_iter[pid] = qp_tot;
  }

  __device__ __forceinline__ void x0_of(double (&x)[NX], double sv) const {
    UNR for (int j = 0; j < NQ; ++j) { x[j] = par(PF::Q0 + j); x[NQ + j] = sv * par(PF::DIR + j); }
  }

  // ---------------------------------------------------------------------------------------------
  // linearisation: sweep 1 = ERK4 + sensitivities + defects, sweep 2 = NLP residuals
  // ---------------------------------------------------------------------------------------------
  __device__ void sens() {
    const double h = par(PF::H);
    {
      double xk[NX];
      x0_of(xk, par(PF::S));
      for (int k = 0; k < Nw; ++k) {
        if (k >= N) continue;
        double uk[NU], x1[NX];
        UNR for (int a = 0; a < NU; ++a) uk[a] = at(w.U, FU, k, a);
        rk4_sens<NQ>(h, xk, uk, x1, [&](int i, int c, double v) {
          // A (NX x NX) and B (NX x NU) are adjacent per stage in column-major-of-(i,c) order
          // through two field tables; c is wave-uniform so the select stays scalar.
          if (c < NX) at(w.A, FA, k, i * NX + c) = v;
          else at(w.Bm, FB, k, i * NU + (c - NX)) = v;
        });
        if (hc_on(k)) {
          double g[NQ];
          hcf(k, HV) = hc_eval(xk, g);
          UNR for (int j = 0; j < NQ; ++j) hcf(k, HG + j) = g[j];
        }
        UNR for (int i = 0; i < NX; ++i) {
          const double xn = at(w.X, FX, k + 1, i);
          const double b = x1[i] - xn;
          at(w.BD, FX, k, i) = b;
          xk[i] = xn;
        }
      }
    }
  }

  // sweep 2: NLP residuals with the current multipliers (defects from sweep 1)
  __device__ void residuals(double& rstat, double& req, double& rineq, double& rcomp) {
    double st = 0, eq = 0, in = 0, cp = 0;
    double pprev[NX];
    UNR for (int i = 0; i < NX; ++i) pprev[i] = 0.0;
    for (int k = 0; k < Nw; ++k) {
      if (k >= N) continue;
      double pik[NX];
      UNR for (int i = 0; i < NX; ++i) {
        pik[i] = at(w.PI, FPI, k, i);
        eq = fmax(eq, fabs((double)at(w.BD, FX, k, i)));
      }
      double z[NZ], lb[NZ], ub[NZ];
      bool bx[NZ];
      stage_box(k, z, lb, ub, bx);
      if (k == 0) {
        // F0 = [A0 g, B0] with g = [0; dir]
        UNR for (int i = 0; i < NX; ++i) {
          double t = 0.0;
          UNR for (int j = 0; j < NQ; ++j) t += at(w.A, FA, 0, i * NX + NQ + j) * par(PF::DIR + j);
          at0(w.F0, NX * M0, i * M0) = t;
          UNR for (int a = 0; a < NU; ++a) at0(w.F0, NX * M0, i * M0 + 1 + a) = at(w.Bm, FB, 0, i * NU + a);
        }
        UNR for (int c = 0; c < M0; ++c) {
          double gr = (c == 0 ? par(PF::CS) : 0.0) - at(w.LL, FZ, 0, c) + at(w.LU, FZ, 0, c);
          UNR for (int r = 0; r < NX; ++r) gr += at0(w.F0, NX * M0, r * M0 + c) * pik[r];
          st = fmax(st, fabs(gr));
        }
      } else {
        UNR for (int c = 0; c < NZ; ++c) {
          double gr = -at(w.LL, FZ, k, c) + at(w.LU, FZ, k, c);
          if (c < NX) {
            UNR for (int r = 0; r < NX; ++r) gr += at(w.A, FA, k, r * NX + c) * pik[r];
            gr -= pprev[c];
            if (c < NQ && hc_on(k)) gr += hcf(k, HG + c) * (hcf(k, HLU) - hcf(k, HLL));
          } else {
            UNR for (int r = 0; r < NX; ++r) gr += at(w.Bm, FB, k, r * NU + (c - NX)) * pik[r];
          }
          st = fmax(st, fabs(gr));
        }
      }
      UNR for (int c = 0; c < NZ; ++c) {
        if (!bx[c]) continue;
        const double ll = at(w.LL, FZ, k, c), lu = at(w.LU, FZ, k, c);
        in = fmax(in, fmax(lb[c] - z[c], z[c] - ub[c]));
        cp = fmax(cp, fmax(fabs(ll * (z[c] - lb[c])), fabs(lu * (ub[c] - z[c]))));
      }
      if (hc_on(k)) {
        const double hv = hcf(k, HV), hll = hcf(k, HLL), hlu = hcf(k, HLU);
        in = fmax(in, fmax(o.hlh - hv, hv - o.huh));
        cp = fmax(cp, fmax(fabs(hll * (hv - o.hlh)), fabs(hlu * (o.huh - hv))));
      }
      UNR for (int i = 0; i < NX; ++i) pprev[i] = pik[i];
    }
    // terminal stage (per-lane N)
    {
      double z[NZ], lb[NZ], ub[NZ];
      bool bx[NZ];
      stage_box<false>(N, z, lb, ub, bx);
      UNR for (int c = 0; c < NX; ++c) {
        double gr = -atv(w.LL, FZ, N, c) + atv(w.LU, FZ, N, c) - pprev[c];
        if (c >= NQ) {
          gr += par(PF::NU_ + c - NQ);
          eq = fmax(eq, fabs(z[c] - par(PF::VFIN + c - NQ)));
        }
        st = fmax(st, fabs(gr));
        if (bx[c]) {
          const double ll = atv(w.LL, FZ, N, c), lu = atv(w.LU, FZ, N, c);
          in = fmax(in, fmax(lb[c] - z[c], z[c] - ub[c]));
          cp = fmax(cp, fmax(fabs(ll * (z[c] - lb[c])), fabs(lu * (ub[c] - z[c]))));
        }
      }
    }
    rstat = st; req = eq; rineq = in; rcomp = cp;
  }

  // ---------------------------------------------------------------------------------------------
  // interior-point QP
  // ---------------------------------------------------------------------------------------------
  __device__ __forceinline__ double cgrad(int k, int i) const { return (k == 0 && i == 0) ? par(PF::CS) : 0.0; }

  // initial point, initial residuals
  __device__ void qp_init() {
    rd0 = 0.0; e00 = 0.0; nbox = 0.0;
    double musum = 0.0;
    double dprev[NZ];
    for (int k = 0; k <= Nw; ++k) {
      if (k > N) continue;
      double z[NZ], lb[NZ], ub[NZ];
      bool bx[NZ];
      stage_box(k, z, lb, ub, bx);
      double dz[NZ], qlv[NZ], quv[NZ];
      UNR for (int i = 0; i < NZ; ++i) {
        double ql = 0.0, qu = 0.0, d0 = 0.0;
        if (bx[i]) {
          const double L = lb[i] - z[i], U = ub[i] - z[i], del = o.push * (U - L);
          d0 = fmin(fmax(0.0, L + del), U - del);
          ql = o.mu0 / (d0 - L);
          qu = o.mu0 / (U - d0);
          musum += o.mu0 + o.mu0;
          nbox += 2.0;
        }
        dz[i] = d0;
        at(w.DZ, FZ, k, i) = d0;
        at(w.QL, FZ, k, i) = ql;
        at(w.QU, FZ, k, i) = qu;
        qlv[i] = ql;
        quv[i] = qu;
      }
      double hgam = 0.0, hg[NQ];
      const bool hk = hc_on(k);
      if (hk) {
        // slacks from the initial c'dz, clipped to ipm_push (infeasible start, residual r0 scaled by rs)
        double gd = 0.0;
        UNR for (int j = 0; j < NQ; ++j) { hg[j] = hcf(k, HG + j); gd += hg[j] * dz[j]; }
        const double hv = hcf(k, HV), L = o.hlh - hv, U = o.huh - hv;
        const double tl = fmax(gd - L, o.push), tu = fmax(U - gd, o.push);
        const double ql = o.mu0 / tl, qu = o.mu0 / tu;
        const double r0l = gd - L - tl, r0u = U - gd - tu;
        hcf(k, HTL) = tl; hcf(k, HTU) = tu; hcf(k, HQL) = ql; hcf(k, HQU) = qu;
        hcf(k, HR0L) = r0l; hcf(k, HR0U) = r0u;
        musum += tl * ql + tu * qu;
        nbox += 2.0;
        e00 = fmax(e00, fmax(fabs(r0l), fabs(r0u)));
        hgam = qu - ql;
      }
      UNR for (int i = 0; i < NZ; ++i)
        rd0 = fmax(rd0, fabs(o.lm * dz[i] + cgrad(k, i) - qlv[i] + quv[i] + ((hk && i < NQ) ? hg[i < NQ ? i : 0] * hgam : 0.0)));
      if (k > 0) {
        // residual of stage k-1 dynamics at the initial point
        const int kp = k - 1;
        UNR for (int i = 0; i < NX; ++i) {
          double t = at(w.BD, FX, kp, i) - dz[i];
          if (kp == 0) {
            UNR for (int a = 0; a < M0; ++a) t += at0(w.F0, NX * M0, i * M0 + a) * dprev[a];
          } else {
            UNR for (int q = 0; q < NX; ++q) t += at(w.A, FA, kp, i * NX + q) * dprev[q];
            UNR for (int a = 0; a < NU; ++a) t += at(w.Bm, FB, kp, i * NU + a) * dprev[NX + a];
          }
          at(w.E0, FX, kp, i) = t;
          e00 = fmax(e00, fabs(t));
        }
      }
      UNR for (int i = 0; i < NZ; ++i) dprev[i] = dz[i];
    }
    UNR for (int j = 0; j < NQ; ++j) {
      const double e = par(PF::VFIN + j) - atv(w.X, FX, N, NQ + j) - dprev[NQ + j];
      par(PF::E0N + j) = e;
      e00 = fmax(e00, fabs(e));
      par(PF::QNU + j) = 0.0;
    }
    mu = musum / nbox;
    rs = 1.0;
    qp_store_scalars();
  }

  struct CompState { double tl, tu, itl, itu, ql, qu, dz; bool bx; };

  // running minimum of t / (-dt) over dt < 0 without a division per candidate (value n / d, d > 0)
  struct MinRatio {
    double n, d;
    __device__ __forceinline__ void add(double t, double dt) {
      if (dt < 0.0 && t * d < n * (-dt)) { n = t; d = -dt; }
    }
    __device__ __forceinline__ double value() const { return n / d; }
  };

  template <bool U = true>
  __device__ __forceinline__ void comp_states(int k, CompState (&c)[NZ]) const {
    double z[NZ], lb[NZ], ub[NZ];
    bool bx[NZ];
    stage_box<U>(k, z, lb, ub, bx);
    UNR for (int i = 0; i < NZ; ++i) {
      const double dz = atk<U>(w.DZ, FZ, k, i);
      c[i].dz = dz;
      c[i].bx = bx[i];
      c[i].ql = atk<U>(w.QL, FZ, k, i);
      c[i].qu = atk<U>(w.QU, FZ, k, i);
      c[i].tl = dz - (lb[i] - z[i]);
      c[i].tu = (ub[i] - z[i]) - dz;
      c[i].itl = bx[i] ? 1.0 / c[i].tl : 0.0;
      c[i].itu = bx[i] ? 1.0 / c[i].tu : 0.0;
    }
  }

  // corrector complementarity right-hand sides from the affine direction da
  __device__ __forceinline__ static void corr_rhs(const CompState& c, double da, double smu, double& rl, double& ru) {
    const double dlla = -c.ql - c.ql * da * c.itl, dlua = -c.qu + c.qu * da * c.itu;
    rl = smu - c.tl * c.ql - da * dlla;
    ru = smu - c.tu * c.qu + da * dlua;
  }

  // H and g of stage k; corr: corrector RHS with the stored DAFF
  template <bool U = true>
  __device__ __forceinline__ void hess_grad(int k, bool corr, double smu, double (&H)[NZ], double (&g)[NZ]) const {
    CompState c[NZ];
    comp_states<U>(k, c);
    UNR for (int i = 0; i < NZ; ++i) {
      H[i] = o.lm;
      g[i] = o.lm * c[i].dz + cgrad(k, i);
      if (c[i].bx) {
        H[i] += c[i].ql * c[i].itl + c[i].qu * c[i].itu;
        if (corr) {
          double rl, ru;
          corr_rhs(c[i], atk<U>(w.DAFF, FZ, k, i), smu, rl, ru);
          g[i] += -c[i].ql - rl * c[i].itl + c[i].qu + ru * c[i].itu;
        }
      }
    }
    if (hc_on(k)) {
      const double htl = hcf(k, HTL), htu = hcf(k, HTU), hql = hcf(k, HQL), hqu = hcf(k, HQU);
      const double rl = rs * hcf(k, HR0L), ru = rs * hcf(k, HR0U);
      double gam;
      if (corr) {
        const double rcl = smu - htl * hql - hcf(k, HATL) * hcf(k, HAQL);
        const double rcu = smu - htu * hqu - hcf(k, HATU) * hcf(k, HAQU);
        gam = -hql + hqu - (rcl - hql * rl) / htl + (rcu - hqu * ru) / htu;
      } else {
        gam = hql * rl / htl - hqu * ru / htu;
      }
      UNR for (int j = 0; j < NQ; ++j) g[j] += hcf(k, HG + j) * gam;
    }
  }

  // backward Riccati sweep; FACTOR: full factorisation (stores K, LR, M, Y, PE) + vector pass;
  // otherwise vector pass only, reusing the factors.  Returns false on a failed Cholesky.  Leaves
  // the stage-0 open-loop step in w0 and the terminal multiplier in nun.
  template <bool FACTOR>
  __device__ bool backward(bool corr, double smu, double (&Sc)[NQ * NQ], double (&lin_e)[NQ], double (&w0)[M0],
                           double (&nun)[NQ]) {
    bool ok = true;
    double P[NX * NX], p[NX], Pi[NX * NQ], lin[NQ];
    {
      double H[NZ], g[NZ];
      hess_grad<false>(N, corr, smu, H, g);
      UNR for (int i = 0; i < NX; ++i) {
        UNR for (int j = 0; j < NX; ++j) P[i * NX + j] = (i == j) ? H[i] : 0.0;
        p[i] = g[i];
        UNR for (int j = 0; j < NQ; ++j) Pi[i * NQ + j] = (i == NQ + j) ? 1.0 : 0.0;
      }
    }
    UNR for (int j = 0; j < NQ; ++j) lin[j] = 0.0;
    if (FACTOR) {
      UNR for (int j = 0; j < NQ * NQ; ++j) Sc[j] = 0.0;
      UNR for (int j = 0; j < NQ; ++j) lin_e[j] = 0.0;
    }
    for (int k = Nw - 1; k >= 1; --k) {
      if (k >= N) continue;
      // load block: stage matrices first (independent of the recursion), then the IPM state
      double Ak[NX * NX], Bk[NX * NU], e[NX];
      UNR for (int i = 0; i < NX * NX; ++i) Ak[i] = at(w.A, FA, k, i);
      UNR for (int i = 0; i < NX * NU; ++i) Bk[i] = at(w.Bm, FB, k, i);
      if (FACTOR) {
        UNR for (int i = 0; i < NX; ++i) e[i] = rs * at(w.E0, FX, k, i);
      }
      double H[NZ], g[NZ];
      hess_grad(k, corr, smu, H, g);
      double Pe[NX], Lr[NU * NU], Yk[NU * NQ];
      double BP[NU * NX];
      if (FACTOR) {
        // Pe = P e ; lin_e += Pi' e
        UNR for (int i = 0; i < NX; ++i) {
          double t = 0.0;
          UNR for (int j = 0; j < NX; ++j) t += P[i * NX + j] * e[j];
          Pe[i] = t;
          at(w.PE, FX, k, i) = t;
        }
        UNR for (int j = 0; j < NQ; ++j) {
          double t = 0.0;
          UNR for (int i = 0; i < NX; ++i) t += Pi[i * NQ + j] * e[i];
          lin_e[j] += t;
        }
        // BP = B' P ; Ru = BP B + diag(Hu)
        UNR for (int a = 0; a < NU; ++a)
          UNR for (int j = 0; j < NX; ++j) {
            double t = 0.0;
            UNR for (int i = 0; i < NX; ++i) t += Bk[i * NU + a] * P[i * NX + j];
            BP[a * NX + j] = t;
          }
        UNR for (int a = 0; a < NU; ++a)
          UNR for (int c = 0; c <= a; ++c) {
            double t = (a == c) ? H[NX + a] : 0.0;
            UNR for (int i = 0; i < NX; ++i) t += BP[a * NX + i] * Bk[i * NU + c];
            Lr[a * NU + c] = t;
            Lr[c * NU + a] = t;
          }
        ok = ok && chol<NU>(Lr);
        UNR for (int i = 0; i < NU * NU; ++i) at(w.LR, FLR, k, i) = Lr[i];
        // Y = B' Pi ; M = Ru^-1 Y ; S += Y' M
        UNR for (int a = 0; a < NU; ++a)
          UNR for (int j = 0; j < NQ; ++j) {
            double t = 0.0;
            UNR for (int i = 0; i < NX; ++i) t += Bk[i * NU + a] * Pi[i * NQ + j];
            Yk[a * NQ + j] = t;
            at(w.Y, FM, k, a * NQ + j) = t;
          }
        UNR for (int j = 0; j < NQ; ++j) {
          double col[NU];
          UNR for (int a = 0; a < NU; ++a) col[a] = Yk[a * NQ + j];
          chol_solve<NU>(Lr, col);
          UNR for (int a = 0; a < NU; ++a) at(w.M, FM, k, a * NQ + j) = col[a];
          UNR for (int i = 0; i < NQ; ++i) {
            double t = 0.0;
            UNR for (int a = 0; a < NU; ++a) t += Yk[a * NQ + i] * col[a];
            Sc[i * NQ + j] += t;
          }
        }
      } else {
        UNR for (int i = 0; i < NX; ++i) Pe[i] = at(w.PE, FX, k, i);
        UNR for (int i = 0; i < NU * NU; ++i) Lr[i] = at(w.LR, FLR, k, i);
        UNR for (int i = 0; i < NU * NQ; ++i) Yk[i] = at(w.Y, FM, k, i);
      }
      // vector pass part 1: v = Pe + p ; r = g_u + B' v ; kf = -Ru^-1 r
      double v[NX], r[NU], kf[NU];
      UNR for (int i = 0; i < NX; ++i) v[i] = Pe[i] + p[i];
      UNR for (int a = 0; a < NU; ++a) {
        double t = g[NX + a];
        UNR for (int i = 0; i < NX; ++i) t += Bk[i * NU + a] * v[i];
        r[a] = t;
        kf[a] = t;
      }
      chol_solve<NU>(Lr, kf);
      UNR for (int a = 0; a < NU; ++a) {
        kf[a] = -kf[a];
        at(w.KF, FU, k, a) = kf[a];
      }
      UNR for (int j = 0; j < NQ; ++j) {
        double t = 0.0;
        UNR for (int a = 0; a < NU; ++a) t += Yk[a * NQ + j] * kf[a];
        lin[j] += t;
      }
      double Kk[NU * NX];
      if (FACTOR) {
        // W = L^-1 (BP A) ; K = -L^-T W
        double W[NU * NX];
        UNR for (int j = 0; j < NX; ++j) {
          double col[NU];
          UNR for (int a = 0; a < NU; ++a) {
            double t = 0.0;
            UNR for (int i = 0; i < NX; ++i) t += BP[a * NX + i] * Ak[i * NX + j];
            col[a] = t;
          }
          // forward substitution only (W), then back substitution (K)
          UNR for (int a = 0; a < NU; ++a) {
            double t = col[a];
            UNR for (int q = 0; q < a; ++q) t -= Lr[a * NU + q] * col[q];
            col[a] = t / Lr[a * NU + a];
          }
          UNR for (int a = 0; a < NU; ++a) W[a * NX + j] = col[a];
          UNR for (int a = NU - 1; a >= 0; --a) {
            double t = col[a];
            UNR for (int q = a + 1; q < NU; ++q) t -= Lr[q * NU + a] * col[q];
            col[a] = t / Lr[a * NU + a];
          }
          UNR for (int a = 0; a < NU; ++a) {
            Kk[a * NX + j] = -col[a];
            at(w.K, FK, k, a * NX + j) = -col[a];
          }
        }
        // Pn = diag(Hx) - W'W + A' P A   (A streamed column by column)
        double Pn[NX * NX], hsig = 0.0, hgk[NQ];
        const bool hk = hc_on(k);
        UNR for (int j = 0; j < NQ; ++j) hgk[j] = 0.0;
        if (hk) {
          hsig = hcf(k, HQL) / hcf(k, HTL) + hcf(k, HQU) / hcf(k, HTU);
          UNR for (int j = 0; j < NQ; ++j) hgk[j] = hcf(k, HG + j);
        }
        UNR for (int i = 0; i < NX; ++i)
          UNR for (int j = 0; j <= i; ++j) {
            double t = (i == j) ? H[i] : 0.0;
            if (hk && i < NQ && j < NQ) t += hsig * hgk[i < NQ ? i : 0] * hgk[j < NQ ? j : 0];
            UNR for (int a = 0; a < NU; ++a) t -= W[a * NX + i] * W[a * NX + j];
            Pn[i * NX + j] = t;
          }
        UNR for (int j = 0; j < NX; ++j) {
          double Aj[NX], t[NX];
          UNR for (int q = 0; q < NX; ++q) Aj[q] = Ak[q * NX + j];
          UNR for (int i = 0; i < NX; ++i) {
            double s = 0.0;
            UNR for (int q = 0; q < NX; ++q) s += P[i * NX + q] * Aj[q];
            t[i] = s;
          }
          UNR for (int i = j; i < NX; ++i) {
            double s = 0.0;
            UNR for (int q = 0; q < NX; ++q) s += Ak[q * NX + i] * t[q];
            Pn[i * NX + j] += s;
          }
        }
        // Pi <- A'Pi + K'Y
        double Pin[NX * NQ];
        UNR for (int i = 0; i < NX; ++i)
          UNR for (int j = 0; j < NQ; ++j) {
            double t = 0.0;
            UNR for (int q = 0; q < NX; ++q) t += Ak[q * NX + i] * Pi[q * NQ + j];
            UNR for (int a = 0; a < NU; ++a) t += Kk[a * NX + i] * Yk[a * NQ + j];
            Pin[i * NQ + j] = t;
          }
        UNR for (int i = 0; i < NX * NQ; ++i) Pi[i] = Pin[i];
        UNR for (int i = 0; i < NX; ++i)
          UNR for (int j = 0; j <= i; ++j) { P[i * NX + j] = Pn[i * NX + j]; P[j * NX + i] = Pn[i * NX + j]; }
      } else {
        UNR for (int i = 0; i < NU * NX; ++i) Kk[i] = at(w.K, FK, k, i);
      }
      // vector pass part 2: p = g_x + A' v + K' r
      UNR for (int i = 0; i < NX; ++i) {
        double t = g[i];
        UNR for (int q = 0; q < NX; ++q) t += Ak[q * NX + i] * v[q];
        UNR for (int a = 0; a < NU; ++a) t += Kk[a * NX + i] * r[a];
        p[i] = t;
      }
    }
    // stage 0: controls (s, u0), F0 = [A0 g, B0]
    {
      double H[NZ], g[NZ];
      hess_grad(0, corr, smu, H, g);
      double F[NX * M0], Pe[NX], Lr[M0 * M0], Yk[M0 * NQ];
      UNR for (int i = 0; i < NX * M0; ++i) F[i] = at0(w.F0, NX * M0, i);
      if (FACTOR) {
        UNR for (int i = 0; i < NX; ++i) {
          double t = 0.0;
          UNR for (int j = 0; j < NX; ++j) t += P[i * NX + j] * (rs * at(w.E0, FX, 0, j));
          Pe[i] = t;
          at0(w.PE0, NX, i) = t;
        }
        UNR for (int j = 0; j < NQ; ++j) {
          double t = 0.0;
          UNR for (int i = 0; i < NX; ++i) t += Pi[i * NQ + j] * (rs * at(w.E0, FX, 0, i));
          lin_e[j] += t;
        }
        double BP[M0 * NX];
        UNR for (int a = 0; a < M0; ++a)
          UNR for (int j = 0; j < NX; ++j) {
            double t = 0.0;
            UNR for (int i = 0; i < NX; ++i) t += F[i * M0 + a] * P[i * NX + j];
            BP[a * NX + j] = t;
          }
        UNR for (int a = 0; a < M0; ++a)
          UNR for (int c = 0; c <= a; ++c) {
            double t = (a == c) ? H[a] : 0.0;
            UNR for (int i = 0; i < NX; ++i) t += BP[a * NX + i] * F[i * M0 + c];
            Lr[a * M0 + c] = t;
            Lr[c * M0 + a] = t;
          }
        ok = ok && chol<M0>(Lr);
        UNR for (int i = 0; i < M0 * M0; ++i) at0(w.LR0, M0 * M0, i) = Lr[i];
        UNR for (int a = 0; a < M0; ++a)
          UNR for (int j = 0; j < NQ; ++j) {
            double t = 0.0;
            UNR for (int i = 0; i < NX; ++i) t += F[i * M0 + a] * Pi[i * NQ + j];
            Yk[a * NQ + j] = t;
            at0(w.Y0, M0 * NQ, a * NQ + j) = t;
          }
        UNR for (int j = 0; j < NQ; ++j) {
          double col[M0];
          UNR for (int a = 0; a < M0; ++a) col[a] = Yk[a * NQ + j];
          chol_solve<M0>(Lr, col);
          UNR for (int a = 0; a < M0; ++a) at0(w.M0, M0 * NQ, a * NQ + j) = col[a];
          UNR for (int i = 0; i < NQ; ++i) {
            double t = 0.0;
            UNR for (int a = 0; a < M0; ++a) t += Yk[a * NQ + i] * col[a];
            Sc[i * NQ + j] += t;
          }
        }
      } else {
        UNR for (int i = 0; i < NX; ++i) Pe[i] = at0(w.PE0, NX, i);
        UNR for (int i = 0; i < M0 * M0; ++i) Lr[i] = at0(w.LR0, M0 * M0, i);
        UNR for (int i = 0; i < M0 * NQ; ++i) Yk[i] = at0(w.Y0, M0 * NQ, i);
      }
      double v[NX];
      UNR for (int i = 0; i < NX; ++i) v[i] = Pe[i] + p[i];
      UNR for (int a = 0; a < M0; ++a) {
        double t = g[a];
        UNR for (int i = 0; i < NX; ++i) t += F[i * M0 + a] * v[i];
        w0[a] = t;
      }
      chol_solve<M0>(Lr, w0);
      UNR for (int a = 0; a < M0; ++a) w0[a] = -w0[a];
      UNR for (int j = 0; j < NQ; ++j) {
        double t = 0.0;
        UNR for (int a = 0; a < M0; ++a) t += Yk[a * NQ + j] * w0[a];
        lin[j] += t;
      }
    }
    // terminal multiplier: nu = S^-1 (E d_N^0 - e_N)
    {
      double Sl[NQ * NQ], rhs_[NQ];
      UNR for (int i = 0; i < NQ * NQ; ++i) Sl[i] = Sc[i];
      ok = ok && chol<NQ>(Sl);
      UNR for (int j = 0; j < NQ; ++j) rhs_[j] = lin[j] + lin_e[j] - rs * par(PF::E0N + j);
      chol_solve<NQ>(Sl, rhs_);
      UNR for (int j = 0; j < NQ; ++j) nun[j] = rhs_[j];
    }
    return ok;
  }

  // forward sweep.  CORR == false: stores DAFF, returns the affine step length and the mu_aff
  // polynomial; CORR == true: stores D, returns alpha_max of the combined step.
  template <bool CORR>
  __device__ void forward(double smu, const double (&w0in)[M0], const double (&nun)[NQ], double& amax, double& c0,
                          double& c1, double& c2) {
    MinRatio mr{CORR ? 1.0 : 1.0, CORR ? o.tau : 1.0};
    c0 = c1 = c2 = 0.0;
    double* dst = CORR ? w.D : w.DAFF;
    double dx[NX];
    for (int k = 0; k <= Nw; ++k) {
      if (k > N) continue;
      double d[NZ];
      if (k == 0) {
        double F[NX * M0], e[NX], Mk[M0 * NQ];
        UNR for (int i = 0; i < NX * M0; ++i) F[i] = at0(w.F0, NX * M0, i);
        UNR for (int i = 0; i < M0 * NQ; ++i) Mk[i] = at0(w.M0, M0 * NQ, i);
        UNR for (int i = 0; i < NX; ++i) e[i] = at(w.E0, FX, 0, i);
        double w0[M0];
        UNR for (int a = 0; a < M0; ++a) {
          double t = w0in[a];
          UNR for (int j = 0; j < NQ; ++j) t -= Mk[a * NQ + j] * nun[j];
          w0[a] = t;
        }
        UNR for (int i = 0; i < NZ; ++i) d[i] = i < M0 ? w0[i < M0 ? i : 0] : 0.0;
        UNR for (int i = 0; i < NX; ++i) {
          double t = rs * e[i];
          UNR for (int a = 0; a < M0; ++a) t += F[i * M0 + a] * w0[a];
          dx[i] = t;
        }
      } else if (k < N) {
        // load block: everything this stage needs, independent of the recursion
        double Kk[NU * NX], kf[NU], Mk[NU * NQ], Ak[NX * NX], Bk[NX * NU], e[NX];
        UNR for (int i = 0; i < NU * NX; ++i) Kk[i] = at(w.K, FK, k, i);
        UNR for (int a = 0; a < NU; ++a) kf[a] = at(w.KF, FU, k, a);
        UNR for (int i = 0; i < NU * NQ; ++i) Mk[i] = at(w.M, FM, k, i);
        UNR for (int i = 0; i < NX * NX; ++i) Ak[i] = at(w.A, FA, k, i);
        UNR for (int i = 0; i < NX * NU; ++i) Bk[i] = at(w.Bm, FB, k, i);
        UNR for (int i = 0; i < NX; ++i) e[i] = at(w.E0, FX, k, i);
        double du[NU];
        UNR for (int a = 0; a < NU; ++a) {
          double t = kf[a];
          UNR for (int i = 0; i < NX; ++i) t += Kk[a * NX + i] * dx[i];
          UNR for (int j = 0; j < NQ; ++j) t -= Mk[a * NQ + j] * nun[j];
          du[a] = t;
        }
        UNR for (int i = 0; i < NX; ++i) d[i] = dx[i];
        UNR for (int a = 0; a < NU; ++a) d[NX + a] = du[a];
        double dn[NX];
        UNR for (int i = 0; i < NX; ++i) {
          double t = rs * e[i];
          UNR for (int q = 0; q < NX; ++q) t += Ak[i * NX + q] * dx[q];
          UNR for (int a = 0; a < NU; ++a) t += Bk[i * NU + a] * du[a];
          dn[i] = t;
        }
        UNR for (int i = 0; i < NX; ++i) dx[i] = dn[i];
      } else {
        UNR for (int i = 0; i < NZ; ++i) d[i] = i < NX ? dx[i < NX ? i : 0] : 0.0;
      }
      CompState c[NZ];
      comp_states(k, c);
      double da[NZ];
      if (CORR) {
        UNR for (int i = 0; i < NZ; ++i) da[i] = at(w.DAFF, FZ, k, i);
      }
      UNR for (int i = 0; i < NZ; ++i) {
        at(dst, FZ, k, i) = d[i];
        if (!c[i].bx) continue;
        double dll, dlu;
        if (!CORR) {
          dll = -c[i].ql - c[i].ql * d[i] * c[i].itl;
          dlu = -c[i].qu + c[i].qu * d[i] * c[i].itu;
          c0 += c[i].tl * c[i].ql + c[i].tu * c[i].qu;
          c1 += c[i].tl * dll + d[i] * c[i].ql + c[i].tu * dlu - d[i] * c[i].qu;
          c2 += d[i] * dll - d[i] * dlu;
        } else {
          double rl, ru;
          corr_rhs(c[i], da[i], smu, rl, ru);
          dll = (rl - c[i].ql * d[i]) * c[i].itl;
          dlu = (ru + c[i].qu * d[i]) * c[i].itu;
        }
        mr.add(c[i].tl, d[i]);
        mr.add(c[i].tu, -d[i]);
        mr.add(c[i].ql, dll);
        mr.add(c[i].qu, dlu);
      }
      if (hc_on(k)) {
        double dtl, dtu, dql, dqu;
        hc_dir<CORR>(k, d, smu, dtl, dtu, dql, dqu);
        const double htl = hcf(k, HTL), htu = hcf(k, HTU), hql = hcf(k, HQL), hqu = hcf(k, HQU);
        if (!CORR) {
          hcf(k, HATL) = dtl; hcf(k, HATU) = dtu; hcf(k, HAQL) = dql; hcf(k, HAQU) = dqu;
          c0 += htl * hql + htu * hqu;
          c1 += htl * dql + dtl * hql + htu * dqu + dtu * hqu;
          c2 += dtl * dql + dtu * dqu;
        }
        mr.add(htl, dtl);
        mr.add(htu, dtu);
        mr.add(hql, dql);
        mr.add(hqu, dqu);
      }
    }
    amax = mr.value();
  }

  // apply the step; recompute mu of the new iterate
  __device__ void update_iterate(double alpha, double smu) {
    double musum = 0.0;
    for (int k = 0; k <= Nw; ++k) {
      if (k > N) continue;
      CompState c[NZ];
      comp_states(k, c);
      UNR for (int i = 0; i < NZ; ++i) {
        const double d = at(w.D, FZ, k, i);
        at(w.DZ, FZ, k, i) = c[i].dz + alpha * d;
        if (!c[i].bx) continue;
        double rl, ru;
        corr_rhs(c[i], at(w.DAFF, FZ, k, i), smu, rl, ru);
        const double dll = (rl - c[i].ql * d) * c[i].itl, dlu = (ru + c[i].qu * d) * c[i].itu;
        const double qln = c[i].ql + alpha * dll, qun = c[i].qu + alpha * dlu;
        at(w.QL, FZ, k, i) = qln;
        at(w.QU, FZ, k, i) = qun;
        musum += (c[i].tl + alpha * d) * qln + (c[i].tu - alpha * d) * qun;
      }
      if (hc_on(k)) {
        double dk[NZ], dtl, dtu, dql, dqu;
        UNR for (int i = 0; i < NZ; ++i) dk[i] = at(w.D, FZ, k, i);
        hc_dir<true>(k, dk, smu, dtl, dtu, dql, dqu);
        const double tl = hcf(k, HTL) + alpha * dtl, tu = hcf(k, HTU) + alpha * dtu;
        const double ql = hcf(k, HQL) + alpha * dql, qu = hcf(k, HQU) + alpha * dqu;
        hcf(k, HTL) = tl; hcf(k, HTU) = tu; hcf(k, HQL) = ql; hcf(k, HQU) = qu;
        musum += tl * ql + tu * qu;
      }
    }
    mu = musum / nbox;
  }

  // ---- interior-point iteration, one sweep per kernel (state in PAR between launches) ----------
  __device__ void qp_store_scalars() {
    par(PF::RS) = rs; par(PF::RD0) = rd0; par(PF::E00) = e00; par(PF::MU) = mu; par(PF::NBOX) = nbox;
  }
  __device__ void qp_load_scalars() {
    rs = par(PF::RS); rd0 = par(PF::RD0); e00 = par(PF::E00); mu = par(PF::MU); nbox = par(PF::NBOX);
  }
  // convergence test at the top of an iteration: 1 continue, 0 converged, -1 failure
  __device__ int qp_check() const {
    if (!isfinite(mu)) return -1;
    if (mu < o.qp_tol_comp && rs * rd0 < o.qp_tol_stat && rs * e00 < o.qp_tol_eq) return 0;
    return 1;
  }
  // predictor factorisation + vector pass; false on failure
  __device__ bool qp_factor() {
    double Sc[NQ * NQ], lin_e[NQ], w0[M0], nun[NQ];
    if (!backward<true>(false, 0.0, Sc, lin_e, w0, nun)) return false;
    UNR for (int i = 0; i < NQ * NQ; ++i) par(PF::SC + i) = Sc[i];
    UNR for (int j = 0; j < NQ; ++j) { par(PF::LINE + j) = lin_e[j]; par(PF::NUN + j) = nun[j]; }
    UNR for (int a = 0; a < M0; ++a) par(PF::W0 + a) = w0[a];
    return true;
  }
  __device__ void qp_fpred() {
    double w0[M0], nun[NQ], aa, c0, c1, c2;
    UNR for (int a = 0; a < M0; ++a) w0[a] = par(PF::W0 + a);
    UNR for (int j = 0; j < NQ; ++j) nun[j] = par(PF::NUN + j);
    forward<false>(0.0, w0, nun, aa, c0, c1, c2);
    const double muaff = (c0 + aa * (c1 + aa * c2)) / nbox;
    double sig = muaff / mu;
    sig = fmin(1.0, sig * sig * sig);
    par(PF::SMU) = sig * mu;
  }
  __device__ bool qp_bcorr() {
    double Sc[NQ * NQ], lin_e[NQ], w0[M0], nun[NQ];
    UNR for (int i = 0; i < NQ * NQ; ++i) Sc[i] = par(PF::SC + i);
    UNR for (int j = 0; j < NQ; ++j) lin_e[j] = par(PF::LINE + j);
    if (!backward<false>(true, par(PF::SMU), Sc, lin_e, w0, nun)) return false;
    UNR for (int j = 0; j < NQ; ++j) par(PF::NUN + j) = nun[j];
    UNR for (int a = 0; a < M0; ++a) par(PF::W0 + a) = w0[a];
    return true;
  }
  __device__ void qp_fcorr() {
    double w0[M0], nun[NQ], amax, c0, c1, c2;
    UNR for (int a = 0; a < M0; ++a) w0[a] = par(PF::W0 + a);
    UNR for (int j = 0; j < NQ; ++j) nun[j] = par(PF::NUN + j);
    forward<true>(par(PF::SMU), w0, nun, amax, c0, c1, c2);
    par(PF::ALPHA) = fmin(1.0, o.tau * amax);
  }
  __device__ void qp_update() {
    const double alpha = par(PF::ALPHA);
    update_iterate(alpha, par(PF::SMU));
    UNR for (int j = 0; j < NQ; ++j) par(PF::QNU + j) += alpha * (par(PF::NUN + j) - par(PF::QNU + j));
    rs *= (1.0 - alpha);
    par(PF::RS) = rs;
    par(PF::MU) = mu;
  }
  // costate recovery: pi_{N-1} = lm dz_N - ql + qu + E'nu ; pi_{k-1} = lm dz_k - ql + qu + A_k' pi_k
  __device__ bool qp_costate() {
    double lam[NX];
    bool fin = true;
    UNR for (int i = 0; i < NX; ++i) {
      const double dz = atv(w.DZ, FZ, N, i);
      lam[i] = o.lm * dz - atv(w.QL, FZ, N, i) + atv(w.QU, FZ, N, i) + (i >= NQ ? par(PF::QNU + (i >= NQ ? i - NQ : 0)) : 0.0);
      fin = fin && isfinite(dz);
    }
    for (int k = Nw - 1; k >= 0; --k) {
      if (k >= N) continue;
      UNR for (int i = 0; i < NX; ++i) at(w.QPI, FPI, k, i) = lam[i];
      if (k == 0) continue;
      double ln[NX];
      UNR for (int i = 0; i < NX; ++i) {
        const double dz = at(w.DZ, FZ, k, i);
        double t = o.lm * dz - at(w.QL, FZ, k, i) + at(w.QU, FZ, k, i);
        if (i < NQ && hc_on(k)) t += hcf(k, HG + (i < NQ ? i : 0)) * (hcf(k, HQU) - hcf(k, HQL));
        UNR for (int q = 0; q < NX; ++q) t += at(w.A, FA, k, q * NX + i) * lam[q];
        ln[i] = t;
      }
      UNR for (int i = 0; i < NX; ++i) lam[i] = ln[i];
    }
    return fin;
  }

  // ---------------------------------------------------------------------------------------------
  // merit line search + update
  // ---------------------------------------------------------------------------------------------
  __device__ __forceinline__ static double wupd(double wv, double lam) {
    const double a = fabs(lam), b = 0.5 * (wv + a);
    return a > b ? a : b;
  }

  // merit(alpha) = cost + sum w_pi |defect| + w_nu |v_N - v_fin| + w_bnd * bound violation
  __device__ double merit(double alpha) const {
    const double h = par(PF::H);
    const double sv = par(PF::S) + alpha * at(w.DZ, FZ, 0, 0);
    double val = par(PF::CS) * sv + par(PF::CCONST);
    double viol = 0.0;
    double xk[NX], uk[NU];
    x0_of(xk, sv);
    for (int k = 0; k <= Nw; ++k) {
      if (k > N) continue;
      double z[NZ], lb[NZ], ub[NZ];
      bool bx[NZ];
      stage_box(k, z, lb, ub, bx);
      double dzk[NZ];
      UNR for (int i = 0; i < NZ; ++i) {
        dzk[i] = at(w.DZ, FZ, k, i);
        if (!bx[i]) continue;
        const double v = z[i] + alpha * dzk[i];
        viol += fmax(0.0, lb[i] - v) + fmax(0.0, v - ub[i]);
      }
      if (k > 0) {
        double phi[NX];
        rk4<NQ>(h, xk, uk, phi);
        UNR for (int i = 0; i < NX; ++i) {
          const double xn = z[i] + alpha * dzk[i];
          val += at(w.WPI, FX, k - 1, i) * fabs(phi[i] - xn);
          xk[i] = xn;
        }
        if (hc_on(k)) {
          const double hv = hc_eval(xk, nullptr);
          val += par(PF::WBND) * (fmax(0.0, o.hlh - hv) + fmax(0.0, hv - o.huh));
        }
      }
      if (k < N) {
        if (k == 0) {
          UNR for (int a = 0; a < NU; ++a) uk[a] = z[1 + a] + alpha * dzk[1 + a];
        } else {
          UNR for (int a = 0; a < NU; ++a) uk[a] = z[NX + a] + alpha * dzk[NX + a];
        }
      }
    }
    UNR for (int j = 0; j < NQ; ++j) val += par(PF::WNU + j) * fabs(xk[NQ + j] - par(PF::VFIN + j));
    return val + par(PF::WBND) * viol;
  }

  __device__ void update_weights() {
    double lmax = 0.0;
    for (int k = 0; k <= Nw; ++k) {
      if (k > N) continue;
      if (k < N) {
        UNR for (int i = 0; i < NX; ++i) at(w.WPI, FX, k, i) = wupd(at(w.WPI, FX, k, i), at(w.QPI, FPI, k, i));
      }
      UNR for (int i = 0; i < NZ; ++i) lmax = fmax(lmax, fmax(at(w.QL, FZ, k, i), at(w.QU, FZ, k, i)));
      if (hc_on(k)) lmax = fmax(lmax, fmax((double)hcf(k, HQL), (double)hcf(k, HQU)));
    }
    UNR for (int j = 0; j < NQ; ++j) par(PF::WNU + j) = wupd(par(PF::WNU + j), par(PF::QNU + j));
    par(PF::WBND) = wupd(par(PF::WBND), lmax);
  }

  __device__ void apply_step(double alpha) {
    par(PF::S) += alpha * at(w.DZ, FZ, 0, 0);
    for (int k = 0; k <= Nw; ++k) {
      if (k > N) continue;
      if (k == 0) {
        UNR for (int a = 0; a < NU; ++a) at(w.U, FU, 0, a) += alpha * at(w.DZ, FZ, 0, 1 + a);
      } else {
        UNR for (int i = 0; i < NX; ++i) at(w.X, FX, k, i) += alpha * at(w.DZ, FZ, k, i);
        if (k < N) {
          UNR for (int a = 0; a < NU; ++a) at(w.U, FU, k, a) += alpha * at(w.DZ, FZ, k, NX + a);
        }
      }
      UNR for (int i = 0; i < NZ; ++i) {
        gdouble& ll = at(w.LL, FZ, k, i);
        gdouble& lu = at(w.LU, FZ, k, i);
        ll += alpha * (at(w.QL, FZ, k, i) - ll);
        lu += alpha * (at(w.QU, FZ, k, i) - lu);
      }
      if (hc_on(k)) {
        gdouble& hll = hcf(k, HLL);
        gdouble& hlu = hcf(k, HLU);
        hll += alpha * (hcf(k, HQL) - hll);
        hlu += alpha * (hcf(k, HQU) - hlu);
      }
      if (k < N) {
        UNR for (int i = 0; i < NX; ++i) {
          gdouble& pi = at(w.PI, FPI, k, i);
          pi += alpha * (at(w.QPI, FPI, k, i) - pi);
        }
      }
    }
    UNR for (int j = 0; j < NQ; ++j) par(PF::NU_ + j) += alpha * (par(PF::QNU + j) - par(PF::NU_ + j));
  }
};

// -------------------------------------------------------------------------------------------------
// phase kernels.  Each slot (lane) holds one problem at a time; per-slot integer state:
//   IS_PID  problem id (-1 free, -2 queue exhausted)   IS_IT   SQP iterations so far
//   IS_QIT  QP iterations so far                        IS_N    horizon
//   IS_PH   phase: 0 free, 1 linearise, 2 QP, 3 line search
// One SQP iteration = refill -> sens -> resid -> qp -> ls (host loop, vboc_solve_batch).
// -------------------------------------------------------------------------------------------------
enum { IS_PID = 0, IS_IT, IS_QIT, IS_N, IS_PH, IS_QST, IS_QCUR, IS_COUNT };

struct SlotState {
  int* ist;          // [IS_COUNT][S]
  unsigned* done;    // problems finished
  unsigned* qp_active;  // lanes whose QP is still iterating
  unsigned long long* work;  // [0] lane-stages swept by k_qp_factor (roofline accounting)
  long long S;
  __device__ __forceinline__ int& operator()(int f, unsigned slot) const { return ist[(long long)f * S + slot]; }
};

template <int NQ>
__device__ __forceinline__ void finish(Lane<NQ>& L, const Inputs& in, const SlotState& ss, int status) {
  const unsigned sl = L.slot;
  L.store_result(in, ss(IS_PID, sl), status, ss(IS_IT, sl), ss(IS_QIT, sl));
  ss(IS_PID, sl) = -1;
  ss(IS_PH, sl) = 0;
  atomicAdd(ss.done, 1u);
}

// lanes without a problem pull the next one (wave-aggregated atomicAdd on the queue head)
template <int NQ>
__global__ __launch_bounds__(256) void k_refill(Work w, Opts o, Inputs in, SlotState ss) {
  const unsigned slot = blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  int pid = ss(IS_PID, slot);
  const unsigned long long need = __ballot(pid == -1);
  if (!need) return;
  const int leader = __ffsll((unsigned long long)need) - 1;
  unsigned int base = 0;
  if (lane == leader) base = atomicAdd(in.head, (unsigned int)__popcll(need));
  base = __shfl(base, leader);
  if (pid != -1) return;
  const unsigned int cand = base + (unsigned)__popcll(need & ((1ull << lane) - 1ull));
  if (cand >= (unsigned int)in.B) {
    ss(IS_PID, slot) = -2;
    return;
  }
  Lane<NQ> L(w, o, slot);
  if (!L.supported(in, (int)cand)) {
    in.status[cand] = 5;
    in.cost[cand] = NAN;
    in.sqp_iter[cand] = 0;
    in.qp_iter[cand] = 0;
    atomicAdd(ss.done, 1u);
    ss(IS_PID, slot) = -1;   // pull another problem next round
    return;
  }
  if (o.hc) {
    // Cartesian constraint at stage 0: positions fixed, h constant - outside [lh, uh] every QP is
    // infeasible; reported as a QP failure without iterating (oracle/vboc_oracle.c, vboc_oracle_solve)
    constexpr int NXR = 2 * NQ + 1;
    double q0[NQ];
    UNR for (int j = 0; j < NQ; ++j) q0[j] = in.lbx0[(long long)cand * NXR + j];
    const double h0 = L.hc_eval(q0, nullptr);
    if (!(h0 >= o.hlh && h0 <= o.huh)) {
      in.status[cand] = 4;
      in.cost[cand] = NAN;
      in.sqp_iter[cand] = 0;
      in.qp_iter[cand] = 0;
      atomicAdd(ss.done, 1u);
      ss(IS_PID, slot) = -1;
      return;
    }
  }
  L.load(in, (int)cand);
  ss(IS_PID, slot) = (int)cand;
  ss(IS_IT, slot) = 0;
  ss(IS_QIT, slot) = 0;
  ss(IS_N, slot) = L.N;
  ss(IS_PH, slot) = 1;
}

// common prologue: horizon, wave-uniform sweep bound; false if this lane is not in phase `ph`
template <int NQ>
__device__ __forceinline__ bool prologue(Lane<NQ>& L, const SlotState& ss, int ph) {
  const bool act = ss(IS_PH, L.slot) == ph;
  L.N = act ? ss(IS_N, L.slot) : 0;
  L.Nw = wave_max(L.N);
  return act;
}

template <int NQ>
__global__ __launch_bounds__(256) VBOC_WPE void k_sens(Work w, Opts o, Inputs in, SlotState ss) {
  Lane<NQ> L(w, o, blockIdx.x * blockDim.x + threadIdx.x);
  if (!prologue(L, ss, 1)) return;
  L.sens();
}

template <int NQ>
__global__ __launch_bounds__(256) VBOC_WPE void k_resid(Work w, Opts o, Inputs in, SlotState ss) {
  Lane<NQ> L(w, o, blockIdx.x * blockDim.x + threadIdx.x);
  if (!prologue(L, ss, 1)) return;
  double rstat, req, rineq, rcomp;
  L.residuals(rstat, req, rineq, rcomp);
  int status = -1;
  if (!isfinite(rstat) || !isfinite(req)) status = 1;
  else if (rstat < o.tol_stat && req < o.tol_eq && rineq < o.tol_ineq && rcomp < o.tol_comp) status = 0;
  else if (ss(IS_IT, L.slot) >= o.max_iter) status = 2;
  if (status >= 0) finish(L, in, ss, status);
  else ss(IS_PH, L.slot) = 2;
}

// ---- interior-point sweeps: IS_QST = 1 running, 0 converged, 2 max iter, -1 failed ----------------
template <int NQ>
__device__ __forceinline__ bool qp_prologue(Lane<NQ>& L, const SlotState& ss) {
  const bool act = ss(IS_PH, L.slot) == 2 && ss(IS_QST, L.slot) == 1;
  L.N = act ? ss(IS_N, L.slot) : 0;
  L.Nw = wave_max(L.N);
  if (act) L.qp_load_scalars();
  return act;
}

template <int NQ>
__global__ __launch_bounds__(256) VBOC_WPE void k_qp_init(Work w, Opts o, Inputs in, SlotState ss) {
  Lane<NQ> L(w, o, blockIdx.x * blockDim.x + threadIdx.x);
  if (!prologue(L, ss, 2)) return;
  L.qp_init();
  ss(IS_QST, L.slot) = 1;
  ss(IS_QCUR, L.slot) = 0;
  atomicAdd(ss.qp_active, 1u);
}

template <int NQ>
__global__ __launch_bounds__(256) VBOC_WPE void k_qp_factor(Work w, Opts o, Inputs in, SlotState ss) {
  Lane<NQ> L(w, o, blockIdx.x * blockDim.x + threadIdx.x);
  const bool act = qp_prologue(L, ss);
  int st = 0;
  if (act) {
    st = L.qp_check();
    if (st == 1 && ss(IS_QCUR, L.slot) >= o.qp_max_iter) st = 2;
  }
  // roofline accounting: lane-stages factorised by this launch (all lanes still present here)
  unsigned long long n = (act && st == 1) ? (unsigned long long)(L.N - 1) : 0ull;  // middle stages
  UNR for (int off = 32; off >= 1; off >>= 1) n += __shfl_xor(n, off);
  if ((threadIdx.x & 63) == 0 && n) atomicAdd(ss.work, n);
  if (!act) return;
  if (st == 1 && !L.qp_factor()) st = -1;
  if (st != 1) {
    ss(IS_QST, L.slot) = st;
    atomicSub(ss.qp_active, 1u);
  }
}

template <int NQ>
__global__ __launch_bounds__(256) VBOC_WPE void k_qp_fpred(Work w, Opts o, Inputs in, SlotState ss) {
  Lane<NQ> L(w, o, blockIdx.x * blockDim.x + threadIdx.x);
  if (!qp_prologue(L, ss)) return;
  L.qp_fpred();
}

template <int NQ>
__global__ __launch_bounds__(256) VBOC_WPE void k_qp_bcorr(Work w, Opts o, Inputs in, SlotState ss) {
  Lane<NQ> L(w, o, blockIdx.x * blockDim.x + threadIdx.x);
  if (!qp_prologue(L, ss)) return;
  if (!L.qp_bcorr()) {
    ss(IS_QST, L.slot) = -1;
    atomicSub(ss.qp_active, 1u);
  }
}

template <int NQ>
__global__ __launch_bounds__(256) VBOC_WPE void k_qp_fcorr(Work w, Opts o, Inputs in, SlotState ss) {
  Lane<NQ> L(w, o, blockIdx.x * blockDim.x + threadIdx.x);
  if (!qp_prologue(L, ss)) return;
  L.qp_fcorr();
}

template <int NQ>
__global__ __launch_bounds__(256) VBOC_WPE void k_qp_update(Work w, Opts o, Inputs in, SlotState ss) {
  Lane<NQ> L(w, o, blockIdx.x * blockDim.x + threadIdx.x);
  if (!qp_prologue(L, ss)) return;
  L.qp_update();
  ss(IS_QCUR, L.slot) += 1;
}

template <int NQ>
__global__ __launch_bounds__(256) VBOC_WPE void k_qp_fin(Work w, Opts o, Inputs in, SlotState ss) {
  Lane<NQ> L(w, o, blockIdx.x * blockDim.x + threadIdx.x);
  if (!prologue(L, ss, 2)) return;
  ss(IS_QIT, L.slot) += ss(IS_QCUR, L.slot);
  const int qs = ss(IS_QST, L.slot);
  if (qs < 0 || !L.qp_costate()) finish(L, in, ss, 4);
  else ss(IS_PH, L.slot) = 3;
}

template <int NQ>
__global__ __launch_bounds__(256) VBOC_WPE void k_ls(Work w, Opts o, Inputs in, SlotState ss) {
  Lane<NQ> L(w, o, blockIdx.x * blockDim.x + threadIdx.x);
  if (!prologue(L, ss, 3)) return;
  L.update_weights();
  const double phi0 = L.merit(0.0);
  double alpha = 1.0;
  for (;;) {
    const double pa = L.merit(alpha);
    if (pa < phi0) break;
    if (alpha * o.alpha_red < o.alpha_min) break;
    alpha *= o.alpha_red;
  }
  L.apply_step(alpha);
  ss(IS_IT, L.slot) += 1;
  if (!isfinite((double)L.par(Par<NQ>::S))) finish(L, in, ss, 1);
  else ss(IS_PH, L.slot) = 1;
}

__global__ void k_slots_init(int* ist, long long S) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= S) return;
  ist[IS_PID * S + i] = -1;
  ist[IS_PH * S + i] = 0;
  ist[IS_N * S + i] = 0;
}

// -------------------------------------------------------------------------------------------------
// twin integrator (SYM<sys>INIT.acados_integrator): one RK4 step of length T per problem
// -------------------------------------------------------------------------------------------------
template <int NQ>
__global__ __launch_bounds__(256) void rk4_kernel(int B, double T, const double* __restrict__ x,
                                                  const double* __restrict__ u, double* __restrict__ xo) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  constexpr int NX = 2 * NQ;
  double xi[NX], ui[NQ], x1[NX];
  UNR for (int i = 0; i < NX; ++i) xi[i] = x[(long long)b * NX + i];
  UNR for (int a = 0; a < NQ; ++a) ui[a] = u[(long long)b * NQ + a];
  rk4<NQ>(T, xi, ui, x1);
  UNR for (int i = 0; i < NX; ++i) xo[(long long)b * NX + i] = x1[i];
}

// one ERK4 step with forward sensitivities per thread (the linearisation of the solvers, standalone)
template <int NQ>
__global__ __launch_bounds__(256) void rk4_sens_kernel(int B, double T, const double* __restrict__ x,
                                                       const double* __restrict__ u, double* __restrict__ xo,
                                                       double* __restrict__ A, double* __restrict__ Bm) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  constexpr int NX = 2 * NQ;
  double xi[NX], ui[NQ], x1[NX];
  UNR for (int i = 0; i < NX; ++i) xi[i] = x[(long long)b * NX + i];
  UNR for (int a = 0; a < NQ; ++a) ui[a] = u[(long long)b * NQ + a];
  rk4_sens<NQ>(T, xi, ui, x1, [&](int i, int c, double v) {
    if (c < NX) A[(long long)b * NX * NX + i * NX + c] = v;
    else Bm[(long long)b * NX * NQ + i * NQ + (c - NX)] = v;
  });
  UNR for (int i = 0; i < NX; ++i) xo[(long long)b * NX + i] = x1[i];
}

// Jobs of the persistent wave kernel: either the slots still iterating in lane mode (hand-off,
// list != nullptr) or problems [0, count) straight from the inputs.
struct WaveJobs {
  const int* list;
  int count;
  unsigned* next;          // job counter
  double* regions;         // one stage-record region per workgroup
  long long region_doubles;
  double* hc = nullptr;    // path-constraint rows, one region per workgroup (k_wave<NQ, false, true>)
  long long hc_doubles = 0;
};

}  // namespace vboc

#include "coop.h"
#include "ft.h"
#include "dg.h"
#include "hjr.h"

// =================================================================================================
// C ABI
// =================================================================================================
using namespace vboc;
static thread_local std::string g_err;
static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
#define HIPCHK(expr)                                                                          \
  do {                                                                                        \
    hipError_t e_ = (expr);                                                                   \
    if (e_ != hipSuccess) return fail(VBOC_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
  } while (0)

struct vboc_solver {
  int nq, nmax, device;
  long long slots;
  Opts o;
  Work w;
  void* pool = nullptr;
  size_t pool_bytes = 0;
  unsigned int* head = nullptr;     // [0] queue head, [1] problems finished
  int* ist = nullptr;               // per-slot integer state [IS_COUNT][slots]
  unsigned int* host_done = nullptr;  // pinned mirror of head[1]
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  int launches = 0;
  // optional per-launch timing of the dominant kernel (k_qp_factor) - HIP events on the launch stream
  bool profile = false;
  std::vector<hipEvent_t> pev;   // pairs
  int npev = 0;
  double fact_ms = 0.0;
  long long fact_calls = 0;
  unsigned long long fact_stages = 0;
  // host staging for vboc_solve_batch_host
  void* stage = nullptr;
  size_t stage_bytes = 0;
  // wave solver (coop.h): one problem per wave, stage records in per-workgroup HBM regions.
  // Used for the tail (queue drained and at most coop_threshold problems still iterating) or, with
  // wave_all, for every problem.
  int* list = nullptr;
  double coop_threshold = 8192;
  bool wave_all = true;
  bool factor_mfma = true;          // wave solver's Riccati factorisation on FP64 MFMA (nq <= 3)
  double* regions = nullptr;
  long long n_regions = 0, region_doubles = 0, group_cap = 0;
  double mall_mib = 256.0;          // MALL budget for the resident problems' hot stage fields (0: off)
  size_t wave_lds = 0;
  bool coop_ok = false;
  long long coop_count = 0;
  // free-time solver (ft.h): one problem per wave, per-workgroup stage-record regions
  double* ft_regions = nullptr;
  size_t ft_bytes = 0;
  // device data generation (dg.h): per-workgroup state-machine records
  double* dg_scratch = nullptr;
  size_t dg_bytes = 0;
  DgJobs* dg_jobs = nullptr;        // device copies of the job descriptor and of the per-workgroup batch
  Inputs* dg_in = nullptr;
  TtJobs* tt_jobs = nullptr;        // device copy of the testing_test job descriptor
  bool tt_attr[2] = {false, false};
  bool dg_attr[4] = {false, false, false, false};
  int dg_fail_mod = 0;              // test-only failure injection of the data-generation loop
  bool dg_speculate = true;         // speculative restarts of failed horizon-extension solves (dg.h)
  int dg_spec_early = 0;            // restart jobs before new problems once this few problems are left (0: only after)
  int dg_spec_pause = 300;          // early events after this many SQP iterations of a tail solve (0: at failures only;
                                    // the single and double pendulum's k_dg)
  // restart jobs before parked resumes once the new problems run out (dg.h): 0 off, 1 on, 2 (default) on for a short
  // launch - fewer than 128 problems per resident wave - where the restart chains found late set the launch's end
  // (round 4, same box: the 100k warmup launch -5.2 %, the 400k launch +1.4 % with it on)
  int dg_spec_first = 2;
  bool dg_spec_crit = false;        // critical-path rule for the eager restart queue (dg.h crit_check)
  int dg_spec_window = 0;           // eager window: a chain's next attempts that go before every problem (dg.h; off: measured slower)
  double* wave_hc = nullptr;        // path-constraint rows of the wave solver, one region per workgroup
  long long wave_hc_doubles = 0;
  bool hc_wave = true;              // constrained problems on the wave solver (k_wave<NQ, false, true>)
  void* dg_spec = nullptr;          // their pool (events, results, control words, queue)
  size_t dg_spec_bytes = 0;
  // Safe-MPC batches (vboc_mpc_solve_batch): the free-time solver's inputs with the dt column, W1 transposed
  void* mpc_buf = nullptr;
  size_t mpc_bytes = 0;
  void* al_buf = nullptr;           // the AL labelling batches' guesses (vboc_al_solve_batch)
  size_t al_bytes = 0;
  // parked first solves of the data-generation loop (dg.h): their results and the two resume queues
  bool dg_park = true;
  int dg_park_window = 0;           // 0: parked problems wait until the new ones run out
  int dg_park_hi = 100;             // first solves with >= this many SQP iterations resume first
  int dg_round = 0;                 // streamed launches: problems per round of the round gate (dg.h DgJobs::round_n)
  void* dg_park_buf = nullptr;
  size_t dg_park_bytes = 0;
  // a vboc_data_generation_async launch is running on this handle's buffers (dg_scratch, regions, head counters)
  // until vboc_data_generation_wait: every other entry point that would reuse them refuses (VBOC_ERR_ARG)
  bool dg_busy = false;
  long long last_groups = 0;        // resident problems (workgroups) of the last wave-solver / data-generation launch
};

static void default_opts(Opts& o) {
  o.tol_stat = 1e-3; o.tol_eq = 1e-6; o.tol_ineq = 1e-6; o.tol_comp = 1e-6;
  o.qp_tol_stat = 1e-3; o.qp_tol_eq = 1e-8; o.qp_tol_comp = 1e-8;
  o.alpha_min = 1e-2; o.alpha_red = 0.3; o.lm = 1e-5;
  o.mu0 = 1.0; o.push = 1e-2; o.tau = 0.995;
  o.max_iter = 1000; o.qp_max_iter = 100;
  o.hc = 0; o.hxc = o.hyc = o.hlh = o.huh = 0.0;
}

static int par_count(int nq) {
  return nq == 1 ? Par<1>::COUNT : (nq == 2 ? Par<2>::COUNT : (nq == 3 ? Par<3>::COUNT : Par<4>::COUNT));
}

static inline size_t ev(size_t f) { return (f + 1) & ~(size_t)1; }  // fields rounded up to pairs

static size_t work_doubles_per_slot(int nq, int nmax) {
  const size_t NX = 2 * nq, NU = nq, NZ = 3 * nq, M0 = nq + 1;
  const size_t per_stage = ev(NX) /*X*/ + ev(NU) + ev(NX) /*PI*/ + 2 * ev(NZ) + ev(NX) /*WPI*/ + ev(NX * NX) +
                           ev(NX * NU) + ev(NX) + 3 * ev(NZ) + ev(NX) /*E0*/ + ev(NU * NX) + ev(NU) + ev(NU * NU) +
                           2 * ev(NU * nq) + ev(NX) /*PE*/ + 2 * ev(NZ) + ev(NX);
  const size_t per_slot = ev(NX * M0) + ev(M0 * M0) + 2 * ev(M0 * nq) + ev(NX) + ev(par_count(nq));
  return per_stage * (size_t)(nmax + 1) + per_slot;
}

static hipError_t prof_flush(vboc_solver* h, hipStream_t st) {
  if (!h->npev) return hipSuccess;
  hipError_t e = hipStreamSynchronize(st);
  if (e != hipSuccess) return e;
  for (int i = 0; i < h->npev; ++i) {
    float f = 0.f;
    e = hipEventElapsedTime(&f, h->pev[2 * i], h->pev[2 * i + 1]);
    if (e != hipSuccess) return e;
    h->fact_ms += f;
  }
  h->fact_calls += h->npev;
  h->npev = 0;
  return hipSuccess;
}

// One SQP iteration of every resident problem: refill, linearise, QP (host-driven interior-point
// loop, one kernel per sweep, exits once no lane is iterating), line search + update.
template <int NQ>
static hipError_t launch_round(vboc_solver* h, dim3 grid, dim3 block, hipStream_t st, const Work& w, const Opts& o,
                               const Inputs& in, const SlotState& ss) {
  hipLaunchKernelGGL(k_refill<NQ>, grid, block, 0, st, w, o, in, ss);
  hipLaunchKernelGGL(k_sens<NQ>, grid, block, 0, st, w, o, in, ss);
  hipLaunchKernelGGL(k_resid<NQ>, grid, block, 0, st, w, o, in, ss);
  hipError_t e = hipMemsetAsync(ss.qp_active, 0, sizeof(unsigned), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_qp_init<NQ>, grid, block, 0, st, w, o, in, ss);
  h->launches += 5;
  for (int it = 0; it <= o.qp_max_iter; ++it) {
    if (h->profile) {
      if ((size_t)(2 * h->npev + 2) > h->pev.size()) {
        e = prof_flush(h, st);
        if (e != hipSuccess) return e;
      }
      e = hipEventRecord(h->pev[2 * h->npev], st);
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_qp_factor<NQ>, grid, block, 0, st, w, o, in, ss);
    if (h->profile) {
      e = hipEventRecord(h->pev[2 * h->npev + 1], st);
      if (e != hipSuccess) return e;
      ++h->npev;
    }
    ++h->launches;
    // poll the active-lane counter (one host sync) from the 6th iteration on, every other one
    if (it >= 6 && (it & 1) == 0) {
      e = hipMemcpyAsync(h->host_done + 1, ss.qp_active, sizeof(unsigned), hipMemcpyDeviceToHost, st);
      if (e == hipSuccess) e = hipStreamSynchronize(st);
      if (e != hipSuccess) return e;
      if (h->host_done[1] == 0) break;
    }
    if (it == o.qp_max_iter) break;
    hipLaunchKernelGGL(k_qp_fpred<NQ>, grid, block, 0, st, w, o, in, ss);
    hipLaunchKernelGGL(k_qp_bcorr<NQ>, grid, block, 0, st, w, o, in, ss);
    hipLaunchKernelGGL(k_qp_fcorr<NQ>, grid, block, 0, st, w, o, in, ss);
    hipLaunchKernelGGL(k_qp_update<NQ>, grid, block, 0, st, w, o, in, ss);
    h->launches += 4;
  }
  hipLaunchKernelGGL(k_qp_fin<NQ>, grid, block, 0, st, w, o, in, ss);
  hipLaunchKernelGGL(k_ls<NQ>, grid, block, 0, st, w, o, in, ss);
  h->launches += 2;
  return hipGetLastError();
}

// free-time solver: a persistent grid of one-wave workgroups, each with its own stage-record region
template <int NQ>
static int launch_ft(vboc_solver* h, const Inputs& in, hipStream_t st, const MpcArgs& mp = MpcArgs{}) {
  const long long rd = mp.on ? FtL<NQ, true>::region_doubles(in.nmax) : FtL<NQ, false>::region_doubles(in.nmax);
  long long groups = in.B < 1024 ? in.B : 1024;
  const size_t need = (size_t)groups * (size_t)rd * sizeof(double);
  if (need > h->ft_bytes) {
    if (h->ft_regions) (void)hipFree(h->ft_regions);
    h->ft_regions = nullptr;
    h->ft_bytes = 0;
    if (hipMalloc(&h->ft_regions, need) != hipSuccess) return -1;
    h->ft_bytes = need;
  }
  if constexpr (NQ == 3) {
    if (mp.on) {
      hipLaunchKernelGGL((k_ft<NQ, true>), dim3((unsigned)groups), dim3(64), 0, st, h->o, in, h->ft_regions, rd, h->head,
                         mp);
      return hipGetLastError() == hipSuccess ? 0 : -2;
    }
  }
  if (mp.on) return -2;   // the Safe-MPC OCP is the triple's
  hipLaunchKernelGGL((k_ft<NQ, false>), dim3((unsigned)groups), dim3(64), 0, st, h->o, in, h->ft_regions, rd, h->head,
                     mp);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// Resident wave-solver problems for a batch whose horizons are <= nmax: every IPM pass streams each
// problem's hot stage fields [0, OX) (170 KB for the triple at N = 100), so the set of resident problems
// is sized to stay inside the 256 MiB MALL (Infinity Cache) of MI355X - measured on the 100k triple
// batch (profiles/r01_wave_groups_sweep.log): 1024 groups 5434, 1408 groups 6212, 2048 groups 5504
// solves/s.  `wave_groups` overrides; `mall_mib` changes the budget.
static long long wave_group_budget(const vboc_solver* h, int nmax) {
  const long long hot = (long long)(h->nq == 1 ? WaveLayout<1>::OX
                                    : (h->nq == 2 ? WaveLayout<2>::OX : (h->nq == 3 ? WaveLayout<3>::OX : WaveLayout<4>::OX))) *
                        (long long)(nmax + 1) * (long long)sizeof(double);
  const long long g = (long long)(0.92 * h->mall_mib * 1024.0 * 1024.0) / (hot > 0 ? hot : 1);
  return g < 256 ? 256 : g;
}

static hipError_t launch_wave(vboc_solver* h, const WaveJobs& jb, long long jobs, hipStream_t st, const Work& w,
                              const Inputs& in, const SlotState& ss) {
  long long groups = jobs < h->n_regions ? jobs : h->n_regions;
  const long long cap = h->group_cap > 0 ? h->group_cap : (h->mall_mib > 0 ? wave_group_budget(h, in.nmax) : 0);
  if (cap > 0 && groups > cap) groups = cap;
  if (groups < 1) return hipSuccess;
  h->last_groups = groups;
  const dim3 grid((unsigned)groups), block(64);
  switch (h->nq) {
    case 1:
      if (h->factor_mfma) hipLaunchKernelGGL((k_wave<1, true>), grid, block, h->wave_lds, st, w, h->o, in, ss, jb);
      else hipLaunchKernelGGL((k_wave<1, false>), grid, block, h->wave_lds, st, w, h->o, in, ss, jb);
      break;
    case 2:
      if (h->o.hc) hipLaunchKernelGGL((k_wave<2, false, true>), grid, block, h->wave_lds, st, w, h->o, in, ss, jb);
      else if (h->factor_mfma) hipLaunchKernelGGL((k_wave<2, true>), grid, block, h->wave_lds, st, w, h->o, in, ss, jb);
      else hipLaunchKernelGGL((k_wave<2, false>), grid, block, h->wave_lds, st, w, h->o, in, ss, jb);
      break;
    case 3:
      if (h->factor_mfma) hipLaunchKernelGGL((k_wave<3, true>), grid, block, h->wave_lds, st, w, h->o, in, ss, jb);
      else hipLaunchKernelGGL((k_wave<3, false>), grid, block, h->wave_lds, st, w, h->o, in, ss, jb);
      break;
    default: hipLaunchKernelGGL((k_wave<4, false>), grid, block, h->wave_lds, st, w, h->o, in, ss, jb); break;
  }
  return hipGetLastError();
}

// the data-generation kernel (dg.h): one problem's whole state machine per wave, the wave solver inside
template <int NQ, bool FM>
static hipError_t launch_dg(vboc_solver* h, const DgJobs& J, const Inputs& in, long long groups, hipStream_t st,
                           bool testing = false) {
  const void* fn = testing ? (const void*)k_ts<NQ, FM> : (const void*)k_dg<NQ, FM>;
  bool& attr = h->dg_attr[(FM ? 1 : 0) + (testing ? 2 : 0)];
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->wave_lds);
    if (e != hipSuccess) return e;
    attr = true;
  }
  WaveJobs jb{nullptr, J.count, J.next, h->regions, h->region_doubles};
  hipError_t e = hipMemcpyAsync(h->dg_jobs, &J, sizeof(DgJobs), hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(h->dg_in, &in, sizeof(Inputs), hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);   // J and in live on the host stack
  if (e != hipSuccess) return e;
  if (testing)
    hipLaunchKernelGGL((k_ts<NQ, FM>), dim3((unsigned)groups), dim3(64), h->wave_lds, st, h->w, h->o, in,
                       (const Inputs*)h->dg_in, (const DgJobs*)h->dg_jobs, jb);
  else
    hipLaunchKernelGGL((k_dg<NQ, FM>), dim3((unsigned)groups), dim3(64), h->wave_lds, st, h->w, h->o, in,
                       (const Inputs*)h->dg_in, (const DgJobs*)h->dg_jobs, jb);
  return hipGetLastError();
}

template <int NQ, bool FM, bool HC>
static hipError_t launch_tt(vboc_solver* h, const TtJobs& J, const Inputs& in, long long groups, hipStream_t st) {
  const void* fn = (const void*)k_tt<NQ, FM, HC>;
  bool& attr = h->tt_attr[NQ == 4 ? 1 : 0];
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->wave_lds);
    if (e != hipSuccess) return e;
    attr = true;
  }
  WaveJobs jb{nullptr, J.count, J.next, h->regions, h->region_doubles, HC ? h->wave_hc : nullptr,
              HC ? h->wave_hc_doubles : 0};
  hipError_t e = hipMemcpyAsync(h->tt_jobs, &J, sizeof(TtJobs), hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(h->dg_in, &in, sizeof(Inputs), hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_tt<NQ, FM, HC>), dim3((unsigned)groups), dim3(64), h->wave_lds, st, h->w, h->o, in,
                     (const Inputs*)h->dg_in, (const TtJobs*)h->tt_jobs, jb);
  return hipGetLastError();
}

// an entry point that would reuse the handle's buffers while an async data-generation launch runs on them
static bool busy(const vboc_solver* h, const char* who) {
  if (!h || !h->dg_busy) return false;
  fail(VBOC_ERR_ARG, std::string(who) + ": a vboc_data_generation_async launch is still running on this handle "
                                        "(call vboc_data_generation_wait first)");
  return true;
}

extern "C" {

const char* vboc_last_error(void) { return g_err.c_str(); }

int vboc_create(int nq, int nmax, int slots, int device, vboc_handle* out) {
  if (!out) return fail(VBOC_ERR_ARG, "vboc_create: out is NULL");
  *out = nullptr;
  if (nq < 1 || nq > 4) return fail(VBOC_ERR_ARG, "vboc_create: nq must be 1, 2, 3 (pendulum chains) or 4 (UR5)");
  if (nmax < 1) return fail(VBOC_ERR_ARG, "vboc_create: nmax must be >= 1");
  HIPCHK(hipSetDevice(device));
  vboc_solver* h = new vboc_solver();
  h->nq = nq; h->nmax = nmax; h->device = device;
  h->factor_mfma = nq <= 3;
  default_opts(h->o);
  if (nq == 4) {
    h->o.lm = 1e-2;          // UR5 OCP: levenberg_marquardt = 1e-2 (VBOC/UR5/ur5reduced_class_fixedveldir.py:135)
    h->coop_threshold = 0;   // lane mode (wave_all = 0) for the arm runs without the wave tail
  }
  if (slots <= 0) slots = 64 * 1024;
  if (slots > (1 << 30)) return fail(VBOC_ERR_ARG, "vboc_create: too many slots");
  slots = ((slots + 255) / 256) * 256;
  h->slots = slots;
  const size_t per_slot = work_doubles_per_slot(nq, nmax);
  h->pool_bytes = per_slot * (size_t)slots * sizeof(double);
  hipError_t e = hipMalloc(&h->pool, h->pool_bytes);
  if (e != hipSuccess) {
    delete h;
    return fail(VBOC_ERR_NOMEM, std::string("vboc_create: hipMalloc workspace: ") + hipGetErrorString(e));
  }
  e = hipMalloc((void**)&h->head, 256);
  if (e == hipSuccess) e = hipMalloc((void**)&h->ist, sizeof(int) * IS_COUNT * (size_t)slots);
  if (e == hipSuccess) e = hipMalloc((void**)&h->list, sizeof(int) * (size_t)slots);
  if (e == hipSuccess) e = hipHostMalloc((void**)&h->host_done, 64);
  if (e != hipSuccess) {
    vboc_destroy(h);
    return fail(VBOC_ERR_NOMEM, "vboc_create: hipMalloc queue / slot state");
  }
  (void)hipEventCreate(&h->ev0);
  (void)hipEventCreate(&h->ev1);
  // wave solver: one region of stage records per resident workgroup (occupancy x CUs)
  {
    // occupancy of the VALU-factorisation instantiation; the MFMA one is held to the same register budget
    const void* fn = nq == 1 ? (const void*)k_wave<1, false>
                             : (nq == 2 ? (const void*)k_wave<2, false>
                                        : (nq == 3 ? (const void*)k_wave<3, false> : (const void*)k_wave<4, false>));
    h->wave_lds = nq == 1 ? WaveLayout<1>::lds_bytes(nmax)
                          : (nq == 2 ? WaveLayout<2>::lds_bytes(nmax)
                                     : (nq == 3 ? WaveLayout<3>::lds_bytes(nmax) : WaveLayout<4>::lds_bytes(nmax)));
    h->region_doubles = nq == 1 ? (long long)WaveLayout<1>::region_doubles(nmax)
                                : (nq == 2 ? (long long)WaveLayout<2>::region_doubles(nmax)
                                           : (nq == 3 ? (long long)WaveLayout<3>::region_doubles(nmax)
                                                      : (long long)WaveLayout<4>::region_doubles(nmax)));
    int per_cu = 0, cus = 0;
    hipDeviceProp_t prop;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 64, h->wave_lds) == hipSuccess &&
        hipGetDeviceProperties(&prop, device) == hipSuccess) {
      cus = prop.multiProcessorCount;
    }
    (void)hipGetLastError();
    if (per_cu < 1) per_cu = 1;
    if (cus < 1) cus = 256;
    h->n_regions = (long long)per_cu * cus;
    if (h->n_regions > 16384) h->n_regions = 16384;
    if (h->wave_lds > 160 * 1024) h->n_regions = 0;
    h->coop_ok = h->n_regions > 0 &&
                 hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->wave_lds) == hipSuccess &&
                 hipMalloc((void**)&h->regions, sizeof(double) * (size_t)h->region_doubles * (size_t)h->n_regions) ==
                     hipSuccess;
    (void)hipGetLastError();
  }
  // carve the workspace
  const int NX = 2 * nq, NU = nq, NZ = 3 * nq, M0 = nq + 1;
  const size_t st = (size_t)(nmax + 1) * slots;
  double* p = (double*)h->pool;
  auto take = [&](size_t fields_per_stage) { double* r = p; p += ev(fields_per_stage) * st; return r; };
  auto take0 = [&](size_t fields) { double* r = p; p += ev(fields) * (size_t)slots; return r; };
  Work& w = h->w;
  w.S = slots;
  w.HC = nullptr;
  w.X = take(NX); w.U = take(NU); w.PI = take(NX); w.LL = take(NZ); w.LU = take(NZ); w.WPI = take(NX);
  w.A = take(NX * NX); w.Bm = take(NX * NU); w.BD = take(NX);
  w.DZ = take(NZ); w.QL = take(NZ); w.QU = take(NZ); w.E0 = take(NX);
  w.K = take(NU * NX); w.KF = take(NU); w.LR = take(NU * NU); w.M = take(NU * nq); w.Y = take(NU * nq);
  w.PE = take(NX); w.D = take(NZ); w.DAFF = take(NZ); w.QPI = take(NX);
  w.F0 = take0(NX * M0); w.LR0 = take0(M0 * M0); w.M0 = take0(M0 * nq); w.Y0 = take0(M0 * nq); w.PE0 = take0(NX);
  w.PAR = take0(par_count(nq));
  if ((size_t)((char*)p - (char*)h->pool) != h->pool_bytes) {
    vboc_destroy(h);
    return fail(VBOC_ERR_ARG, "vboc_create: internal workspace size mismatch");
  }
  *out = h;
  return VBOC_OK;
}

int vboc_destroy(vboc_handle h) {
  if (!h) return VBOC_OK;
  (void)hipSetDevice(h->device);
  // an un-waited async launch still uses the buffers freed below: wait for it alone (ev1 is recorded behind it on its
  // stream), not for every stream of the device
  if (h->dg_busy && h->ev1) (void)hipEventSynchronize(h->ev1);
  if (h->pool) (void)hipFree(h->pool);
  if (h->head) (void)hipFree(h->head);
  if (h->ist) (void)hipFree(h->ist);
  if (h->w.HC) (void)hipFree(h->w.HC);
  if (h->wave_hc) (void)hipFree(h->wave_hc);
  if (h->list) (void)hipFree(h->list);
  if (h->regions) (void)hipFree(h->regions);
  if (h->host_done) (void)hipHostFree(h->host_done);
  if (h->stage) (void)hipFree(h->stage);
  if (h->ft_regions) (void)hipFree(h->ft_regions);
  if (h->dg_scratch) (void)hipFree(h->dg_scratch);
  if (h->dg_jobs) (void)hipFree(h->dg_jobs);
  if (h->dg_in) (void)hipFree(h->dg_in);
  if (h->tt_jobs) (void)hipFree(h->tt_jobs);
  if (h->dg_spec) (void)hipFree(h->dg_spec);
  if (h->dg_park_buf) (void)hipFree(h->dg_park_buf);
  if (h->mpc_buf) (void)hipFree(h->mpc_buf);
  if (h->al_buf) (void)hipFree(h->al_buf);
  if (h->ev0) (void)hipEventDestroy(h->ev0);
  if (h->ev1) (void)hipEventDestroy(h->ev1);
  for (auto ev : h->pev) (void)hipEventDestroy(ev);
  delete h;
  return VBOC_OK;
}

int vboc_set_option(vboc_handle h, const char* f, double v) {
  if (busy(h, "vboc_set_option")) return VBOC_ERR_ARG;
  if (!h || !f) return fail(VBOC_ERR_ARG, "vboc_set_option: NULL argument");
  Opts& o = h->o;
  const std::string s(f);
  if (s == "nlp_solver_tol_stat") o.tol_stat = v;
  else if (s == "nlp_solver_tol_eq") o.tol_eq = v;
  else if (s == "nlp_solver_tol_ineq") o.tol_ineq = v;
  else if (s == "nlp_solver_tol_comp") o.tol_comp = v;
  else if (s == "nlp_solver_max_iter") o.max_iter = (int)v;
  else if (s == "qp_solver_iter_max") o.qp_max_iter = (int)v;
  else if (s == "qp_solver_tol_stat") o.qp_tol_stat = v;
  else if (s == "qp_solver_tol_eq") o.qp_tol_eq = v;
  else if (s == "qp_solver_tol_comp") o.qp_tol_comp = v;
  else if (s == "levenberg_marquardt") o.lm = v;
  else if (s == "alpha_min") o.alpha_min = v;
  else if (s == "alpha_reduction") o.alpha_red = v;
  else if (s == "ipm_mu0") o.mu0 = v;
  else if (s == "ipm_push") o.push = v;
  else if (s == "ipm_tau") o.tau = v;
  else if (s == "coop_threshold") h->coop_threshold = v;
  else if (s == "wave_all") {
    h->wave_all = v != 0.0;
  }
  else if (s == "factor_mfma") h->factor_mfma = v != 0.0 && h->nq <= 3;
  else if (s == "wave_groups") h->group_cap = (long long)v;
  else if (s == "mall_mib") h->mall_mib = v;
  else if (s == "dg_fail_mod") h->dg_fail_mod = (int)v;
  else if (s == "dg_speculate") h->dg_speculate = v != 0.0;
  else if (s == "dg_spec_early") h->dg_spec_early = v > 0.0 ? (int)v : 0;
  else if (s == "dg_spec_pause") h->dg_spec_pause = v > 0.0 ? (int)v : 0;
  else if (s == "dg_spec_first") h->dg_spec_first = v >= 2.0 ? 2 : (v != 0.0 ? 1 : 0);
  else if (s == "dg_spec_crit") h->dg_spec_crit = v != 0.0;
  else if (s == "dg_spec_window") h->dg_spec_window = v > 0.0 ? (v < 9.0 ? (int)v : 9) : 0;
  else if (s == "dg_park") h->dg_park = v != 0.0;
  else if (s == "dg_park_window") h->dg_park_window = v > 0.0 ? (int)v : 0;
  else if (s == "dg_park_hi") h->dg_park_hi = v > 0.0 ? (int)v : 0;
  else if (s == "dg_round") h->dg_round = v > 0.0 ? (int)v : 0;
  else if (s == "hc_wave") h->hc_wave = v != 0.0;
  else if (s == "profile_kernels") {
    h->profile = v != 0.0;
    if (h->profile && h->pev.empty()) {
      h->pev.resize(2 * 4096);
      for (auto& ev : h->pev)
        if (hipEventCreate(&ev) != hipSuccess) return fail(VBOC_ERR_HIP, "vboc_set_option: hipEventCreate");
    }
  } else return fail(VBOC_ERR_ARG, "vboc_set_option: unknown field '" + s + "'");
  return VBOC_OK;
}

int vboc_get_option(vboc_handle h, const char* f, double* v) {
  if (!h || !f || !v) return fail(VBOC_ERR_ARG, "vboc_get_option: NULL argument");
  const Opts& o = h->o;
  const std::string s(f);
  if (s == "nlp_solver_tol_stat") *v = o.tol_stat;
  else if (s == "nlp_solver_tol_eq") *v = o.tol_eq;
  else if (s == "nlp_solver_tol_ineq") *v = o.tol_ineq;
  else if (s == "nlp_solver_tol_comp") *v = o.tol_comp;
  else if (s == "nlp_solver_max_iter") *v = o.max_iter;
  else if (s == "qp_solver_iter_max") *v = o.qp_max_iter;
  else if (s == "qp_solver_tol_stat") *v = o.qp_tol_stat;
  else if (s == "qp_solver_tol_eq") *v = o.qp_tol_eq;
  else if (s == "qp_solver_tol_comp") *v = o.qp_tol_comp;
  else if (s == "levenberg_marquardt") *v = o.lm;
  else if (s == "alpha_min") *v = o.alpha_min;
  else if (s == "alpha_reduction") *v = o.alpha_red;
  else if (s == "ipm_mu0") *v = o.mu0;
  else if (s == "ipm_push") *v = o.push;
  else if (s == "ipm_tau") *v = o.tau;
  else if (s == "coop_threshold") *v = h->coop_threshold;
  else if (s == "coop_available") *v = h->coop_ok ? 1.0 : 0.0;
  else if (s == "wave_all") *v = h->wave_all ? 1.0 : 0.0;
  else if (s == "dg_speculate") *v = h->dg_speculate ? 1.0 : 0.0;
  else if (s == "dg_spec_early") *v = (double)h->dg_spec_early;
  else if (s == "dg_spec_pause") *v = (double)h->dg_spec_pause;
  else if (s == "dg_spec_first") *v = (double)h->dg_spec_first;
  else if (s == "dg_spec_crit") *v = h->dg_spec_crit ? 1.0 : 0.0;
  else if (s == "dg_spec_window") *v = (double)h->dg_spec_window;
  else if (s == "dg_park") *v = h->dg_park ? 1.0 : 0.0;
  else if (s == "dg_park_window") *v = (double)h->dg_park_window;
  else if (s == "dg_park_hi") *v = (double)h->dg_park_hi;
  else if (s == "dg_round") *v = (double)h->dg_round;
  else if (s == "hc_wave") *v = h->hc_wave ? 1.0 : 0.0;
  else if (s == "factor_mfma") *v = h->factor_mfma ? 1.0 : 0.0;
  else if (s == "wave_groups") *v = (double)h->n_regions;
  else if (s == "last_groups") *v = (double)h->last_groups;
  else if (s == "dg_busy") *v = h->dg_busy ? 1.0 : 0.0;
  else if (s == "mall_mib") *v = h->mall_mib;
  else if (s == "coop_problems") *v = (double)h->coop_count;
  else if (s == "slots") *v = (double)h->slots;
  else if (s == "workspace_bytes") *v = (double)h->pool_bytes;
  else return fail(VBOC_ERR_ARG, "vboc_get_option: unknown field '" + s + "'");
  return VBOC_OK;
}

int vboc_set_path_constraint(vboc_handle h, int kind, double x_c, double y_c, double lh, double uh) {
  if (busy(h, "vboc_set_path_constraint")) return VBOC_ERR_ARG;
  if (!h) return fail(VBOC_ERR_ARG, "vboc_set_path_constraint: NULL handle");
  if (kind == 0) { h->o.hc = 0; return VBOC_OK; }
  if (kind != 1) return fail(VBOC_ERR_ARG, "vboc_set_path_constraint: unknown kind");
  if (h->nq != 2 && h->nq != 3)
    return fail(VBOC_ERR_UNSUPPORTED, "vboc_set_path_constraint: the keep-out circle needs a pendulum chain (nq 2 or 3)");
  if (!(lh <= uh)) return fail(VBOC_ERR_ARG, "vboc_set_path_constraint: lh > uh");
  if (!h->w.HC) {
    const size_t f = h->nq == 2 ? (size_t)Lane<2>::FHC : (size_t)Lane<3>::FHC;
    HIPCHK(hipSetDevice(h->device));
    const hipError_t e = hipMalloc((void**)&h->w.HC, sizeof(double) * ev(f) * (size_t)(h->nmax + 1) * (size_t)h->slots);
    if (e != hipSuccess) {
      h->w.HC = nullptr;
      return fail(VBOC_ERR_NOMEM, "vboc_set_path_constraint: hipMalloc constraint rows");
    }
  }
  // the wave solver carries the rows for the double pendulum (the reference's Cartesian system); the triple's
  // instantiation would spill (140 B of scratch), which the counted ring waits do not tolerate (DESIGN.md
  // section 5), so a constrained triple runs on the lane kernels
  if (!h->wave_hc && h->coop_ok && h->nq == 2) {
    const long long f = (long long)Lane<2>::FHC;
    h->wave_hc_doubles = f * (long long)(h->nmax + 1);
    if (hipMalloc((void**)&h->wave_hc, sizeof(double) * (size_t)h->wave_hc_doubles * (size_t)h->n_regions) != hipSuccess) {
      h->wave_hc = nullptr;
      (void)hipGetLastError();
    }
  }
  h->o.hc = 1; h->o.hxc = x_c; h->o.hyc = y_c; h->o.hlh = lh; h->o.huh = uh;
  return VBOC_OK;
}

int vboc_solve_batch(vboc_handle h, const vboc_batch_t* b, void* stream) {
  if (busy(h, "vboc_solve_batch")) return VBOC_ERR_ARG;
  if (!h || !b) return fail(VBOC_ERR_ARG, "vboc_solve_batch: NULL argument");
  if (b->B < 0) return fail(VBOC_ERR_ARG, "vboc_solve_batch: B < 0");
  if (b->nmax > h->nmax || b->nmax < 1)
    return fail(VBOC_ERR_ARG, "vboc_solve_batch: batch nmax exceeds the handle's nmax");
  if (b->B == 0) { h->launches = 0; return VBOC_OK; }
  const void* ptrs[] = {b->N, b->x_guess, b->u_guess, b->p, b->lbx, b->ubx, b->lbu, b->ubu, b->lbx_0, b->ubx_0,
                        b->lbx_e, b->ubx_e, b->status, b->x_out, b->u_out, b->cost, b->sqp_iter, b->qp_iter};
  for (const void* q : ptrs)
    if (!q) return fail(VBOC_ERR_ARG, "vboc_solve_batch: NULL array in batch");
  HIPCHK(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  Inputs in;
  in.B = b->B; in.nmax = b->nmax; in.N = b->N;
  in.xg = b->x_guess; in.ug = b->u_guess; in.p = b->p; in.lbx = b->lbx; in.ubx = b->ubx; in.lbu = b->lbu;
  in.ubu = b->ubu; in.lbx0 = b->lbx_0; in.ubx0 = b->ubx_0; in.lbxe = b->lbx_e; in.ubxe = b->ubx_e;
  in.status = b->status; in.xo = b->x_out; in.uo = b->u_out; in.cost = b->cost; in.sqp_iter = b->sqp_iter;
  in.qp_iter = b->qp_iter; in.head = h->head;
  HIPCHK(hipMemsetAsync(h->head, 0, 256, st));
  h->fact_ms = 0.0;
  h->fact_calls = 0;
  h->fact_stages = 0;
  h->npev = 0;
  h->coop_count = 0;
  // lanes: never more than the problems (rounded to whole workgroups), never more than the slots
  long long lanes = ((long long)b->B + 255) / 256 * 256;
  if (lanes > h->slots) lanes = h->slots;
  Work w = h->w;  // same carve, S = full slot stride
  SlotState ss{h->ist, h->head + 1, h->head + 2, (unsigned long long*)(h->head + 4), h->slots};
  const dim3 grid((unsigned)(lanes / 256)), block(256);
  HIPCHK(hipEventRecord(h->ev0, st));
  const bool hc_ok = !h->o.hc || (h->hc_wave && h->wave_hc);
  if (h->wave_all && h->coop_ok && hc_ok) {
    // every problem on its own wave, pulled from the input queue (head[0])
    WaveJobs jb{nullptr, b->B, h->head, h->regions, h->region_doubles, h->wave_hc, h->wave_hc_doubles};
    h->launches = 1;
    h->coop_count = b->B;
    HIPCHK(launch_wave(h, jb, (long long)b->B, st, w, in, ss));
    HIPCHK(hipEventRecord(h->ev1, st));
    HIPCHK(hipStreamSynchronize(st));
    HIPCHK(hipMemcpy(h->host_done, h->head + 1, sizeof(unsigned), hipMemcpyDeviceToHost));
    if (*h->host_done != (unsigned)b->B) return fail(VBOC_ERR_HIP, "vboc_solve_batch: wave solver did not finish");
    return VBOC_OK;
  }
  hipLaunchKernelGGL(k_slots_init, dim3((unsigned)((h->slots + 255) / 256)), block, 0, st, h->ist, h->slots);
  // One SQP iteration of every resident problem per round; finished slots refill from the queue.
  // The finished-problem counter is read back every `chunk` rounds (one host sync per chunk).
  const int chunk = 4;
  long long rounds = 0;
  h->launches = 1;
  const bool progress = getenv("VBOC_PROGRESS") != nullptr;
  auto t_start = std::chrono::steady_clock::now();
  unsigned last_print = 0;
  for (;;) {
    for (int r = 0; r < chunk; ++r) {
      hipError_t le;
      switch (h->nq) {
        case 1: le = launch_round<1>(h, grid, block, st, w, h->o, in, ss); break;
        case 2: le = launch_round<2>(h, grid, block, st, w, h->o, in, ss); break;
        case 3: le = launch_round<3>(h, grid, block, st, w, h->o, in, ss); break;
        default: le = launch_round<4>(h, grid, block, st, w, h->o, in, ss); break;
      }
      if (le != hipSuccess) return fail(VBOC_ERR_HIP, std::string("vboc_solve_batch: ") + hipGetErrorString(le));
    }
    rounds += chunk;
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(h->host_done + 4, h->head, 2 * sizeof(unsigned), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    h->host_done[0] = h->host_done[5];
    const unsigned pulled = h->host_done[4] < (unsigned)b->B ? h->host_done[4] : (unsigned)b->B;
    if (h->coop_ok && h->coop_threshold > 0 && !h->o.hc && h->host_done[4] >= (unsigned)b->B &&
        (double)(pulled - h->host_done[0]) <= h->coop_threshold && h->host_done[0] < (unsigned)b->B) {
      // queue drained, few problems left: finish each of them on one LDS-resident wave
      HIPCHK(hipMemsetAsync(h->head + 3, 0, sizeof(unsigned), st));
      hipLaunchKernelGGL(k_list, grid, block, 0, st, ss, h->list, h->head + 3);
      HIPCHK(hipMemcpyAsync(h->host_done + 2, h->head + 3, sizeof(unsigned), hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      const unsigned n = h->host_done[2];
      h->coop_count = n;
      if (n) {
        HIPCHK(hipMemsetAsync(h->head + 5, 0, sizeof(unsigned), st));
        WaveJobs jb{h->list, (int)n, h->head + 5, h->regions, h->region_doubles};
        HIPCHK(launch_wave(h, jb, (long long)n, st, w, in, ss));
        h->launches += 2;
      }
      HIPCHK(hipMemcpyAsync(h->host_done, h->head + 1, sizeof(unsigned), hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      if (progress) {
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
        fprintf(stderr, "[vboc] %.1f ms cooperative tail: %u problems, done %u / %d\n", ms, n, *h->host_done, b->B);
      }
      if (*h->host_done < (unsigned)b->B) return fail(VBOC_ERR_HIP, "vboc_solve_batch: cooperative tail did not finish");
    }
    if (progress && (*h->host_done - last_print >= (unsigned)b->B / 20 || *h->host_done >= (unsigned)b->B ||
                     rounds % 64 == 0)) {
      const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
      fprintf(stderr, "[vboc] %.1f ms rounds %lld done %u / %d\n", ms, rounds, *h->host_done, b->B);
      last_print = *h->host_done;
    }
    if (*h->host_done >= (unsigned)b->B) break;
    if (rounds > 4LL * (h->o.max_iter + 2) * ((b->B + lanes - 1) / lanes + 1))
      return fail(VBOC_ERR_HIP, "vboc_solve_batch: solver did not drain (internal error)");
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(h->ev1, st));
  if (h->profile) HIPCHK(prof_flush(h, st));
  HIPCHK(hipMemcpyAsync(&h->fact_stages, h->head + 4, sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return VBOC_OK;
}

int vboc_debug_counters(unsigned long long* out16) {
  if (!out16) return fail(VBOC_ERR_ARG, "vboc_debug_counters: NULL argument");
  HIPCHK(hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_wave_prof), 16 * sizeof(unsigned long long)));
  static const unsigned long long zero[16] = {0};
  HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_wave_prof), zero, sizeof(zero)));
  return VBOC_OK;
}

int vboc_last_kernel_ms(vboc_handle h, double* ms, int* launches) {
  if (!h || !ms) return fail(VBOC_ERR_ARG, "vboc_last_kernel_ms: NULL argument");
  float f = 0.0f;
  HIPCHK(hipEventSynchronize(h->ev1));
  HIPCHK(hipEventElapsedTime(&f, h->ev0, h->ev1));
  *ms = f;
  if (launches) *launches = h->launches;
  return VBOC_OK;
}

int vboc_kernel_stats(vboc_handle h, double* factor_ms, long long* factor_launches, double* factor_bytes) {
  if (!h || !factor_ms || !factor_launches || !factor_bytes) return fail(VBOC_ERR_ARG, "vboc_kernel_stats: NULL argument");
  const int nq = h->nq, NX = 2 * nq, NU = nq, NZ = 3 * nq;
  // algorithmic bytes of one middle stage of the factorisation sweep (k_qp_factor):
  //   reads  A, B, e, (dz, lambda_l, lambda_u), (x, u)   writes K, chol(Ru), M, Y, P e, k
  const double loads = NX * NX + NX * NU + NX + 3 * NZ + NZ;
  const double stores = NU * NX + NU * NU + 2 * NU * nq + NX + NU;
  *factor_ms = h->fact_ms;
  *factor_launches = h->fact_calls;
  *factor_bytes = (loads + stores) * 8.0 * (double)h->fact_stages;
  return VBOC_OK;
}

int vboc_solve_batch_ft(vboc_handle h, const vboc_batch_t* b, void* stream) {
  if (busy(h, "vboc_solve_batch_ft")) return VBOC_ERR_ARG;
  if (!h || !b) return fail(VBOC_ERR_ARG, "vboc_solve_batch_ft: NULL argument");
  if (h->o.hc) return fail(VBOC_ERR_UNSUPPORTED, "vboc_solve_batch_ft: no path constraint in the free-time OCP");
  if (b->B < 0) return fail(VBOC_ERR_ARG, "vboc_solve_batch_ft: B < 0");
  if (b->nmax > h->nmax || b->nmax < 1)
    return fail(VBOC_ERR_ARG, "vboc_solve_batch_ft: batch nmax exceeds the handle's nmax");
  if (b->B == 0) { h->launches = 0; return VBOC_OK; }
  const void* ptrs[] = {b->N, b->x_guess, b->u_guess, b->p, b->lbx, b->ubx, b->lbu, b->ubu, b->lbx_0, b->ubx_0,
                        b->lbx_e, b->ubx_e, b->status, b->x_out, b->u_out, b->cost, b->sqp_iter, b->qp_iter};
  for (const void* q : ptrs)
    if (!q) return fail(VBOC_ERR_ARG, "vboc_solve_batch_ft: NULL array in batch");
  HIPCHK(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  Inputs in;
  in.B = b->B; in.nmax = b->nmax; in.N = b->N;
  in.xg = b->x_guess; in.ug = b->u_guess; in.p = b->p; in.lbx = b->lbx; in.ubx = b->ubx; in.lbu = b->lbu;
  in.ubu = b->ubu; in.lbx0 = b->lbx_0; in.ubx0 = b->ubx_0; in.lbxe = b->lbx_e; in.ubxe = b->ubx_e;
  in.status = b->status; in.xo = b->x_out; in.uo = b->u_out; in.cost = b->cost; in.sqp_iter = b->sqp_iter;
  in.qp_iter = b->qp_iter; in.head = h->head;
  HIPCHK(hipMemsetAsync(h->head, 0, 256, st));
  HIPCHK(hipEventRecord(h->ev0, st));
  int rc;
  switch (h->nq) {
    case 1: rc = launch_ft<1>(h, in, st); break;
    case 2: rc = launch_ft<2>(h, in, st); break;
    case 3: rc = launch_ft<3>(h, in, st); break;
    default: return fail(VBOC_ERR_UNSUPPORTED, "vboc_solve_batch_ft: the free-time OCP is defined for the pendulum chains only");
  }
  if (rc == -1) return fail(VBOC_ERR_NOMEM, "vboc_solve_batch_ft: hipMalloc of the stage regions");
  if (rc) return fail(VBOC_ERR_HIP, std::string("vboc_solve_batch_ft: ") + hipGetErrorString(hipGetLastError()));
  HIPCHK(hipEventRecord(h->ev1, st));
  h->launches = 1;
  return VBOC_OK;
}

static int solve_host(vboc_handle h, const vboc_batch_t* b, bool ft) {
  if (!h || !b) return fail(VBOC_ERR_ARG, "vboc_solve_batch_host: NULL argument");
  if (b->B == 0) return VBOC_OK;
  HIPCHK(hipSetDevice(h->device));
  const int nq = h->nq, NXR = 2 * nq + 1, NU = nq, NP = nq + 1;
  const size_t B = b->B, Nn = b->nmax;
  const size_t sz_xg = B * (Nn + 1) * NXR, sz_ug = B * Nn * NU;
  const size_t dbl = sz_xg * 2 + sz_ug * 2 + B * NP + B * NXR * 6 + B * NU * 2 + B /*cost*/;
  const size_t ints = B * 4;
  const size_t need = dbl * sizeof(double) + ints * sizeof(int) + 256;
  if (need > h->stage_bytes) {
    if (h->stage) (void)hipFree(h->stage);
    h->stage = nullptr;
    h->stage_bytes = 0;
    hipError_t e = hipMalloc(&h->stage, need);
    if (e != hipSuccess) return fail(VBOC_ERR_NOMEM, "vboc_solve_batch_host: hipMalloc staging");
    h->stage_bytes = need;
  }
  double* d = (double*)h->stage;
  hipError_t cerr = hipSuccess;
  auto put = [&](const double* src, size_t n) -> double* {
    double* r = d;
    d += n;
    if (src && cerr == hipSuccess) cerr = hipMemcpy(r, src, n * sizeof(double), hipMemcpyHostToDevice);
    return r;
  };
  vboc_batch_t db = *b;
  db.x_guess = put(b->x_guess, sz_xg);
  db.u_guess = put(b->u_guess, sz_ug);
  db.p = put(b->p, B * NP);
  db.lbx = put(b->lbx, B * NXR); db.ubx = put(b->ubx, B * NXR);
  db.lbu = put(b->lbu, B * NU); db.ubu = put(b->ubu, B * NU);
  db.lbx_0 = put(b->lbx_0, B * NXR); db.ubx_0 = put(b->ubx_0, B * NXR);
  db.lbx_e = put(b->lbx_e, B * NXR); db.ubx_e = put(b->ubx_e, B * NXR);
  db.x_out = put(b->x_out, sz_xg);    // copy in so rows beyond N stay as the caller had them
  db.u_out = put(b->u_out, sz_ug);
  db.cost = put(nullptr, B);
  int* ip = (int*)d;
  db.N = ip; ip += B;
  db.status = ip; ip += B;
  db.sqp_iter = ip; ip += B;
  db.qp_iter = ip; ip += B;
  HIPCHK(cerr);
  HIPCHK(hipMemcpy((void*)db.N, b->N, B * sizeof(int), hipMemcpyHostToDevice));
  int rc = ft ? vboc_solve_batch_ft(h, &db, nullptr) : vboc_solve_batch(h, &db, nullptr);
  if (rc) return rc;
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(b->x_out, db.x_out, sz_xg * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(b->u_out, db.u_out, sz_ug * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(b->cost, db.cost, B * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(b->status, db.status, B * sizeof(int), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(b->sqp_iter, db.sqp_iter, B * sizeof(int), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(b->qp_iter, db.qp_iter, B * sizeof(int), hipMemcpyDeviceToHost));
  return VBOC_OK;
}

// a Safe-MPC batch as free-time inputs: x [q, v, h] (the dt column pinned by x_0), bounds with a free dt on the path
__global__ void k_mpc_prep(int B, int N, int nq, double hstep, const double* __restrict__ x0,
                           const double* __restrict__ xg6, const double* lbx, const double* ubx, const double* lbu,
                           const double* ubu, const double* lbxe, const double* ubxe, double* xg7, double* lbx7,
                           double* ubx7, double* lbu_b, double* ubu_b, double* lbx0, double* ubx0, double* lbxe7,
                           double* ubxe7, double* p, int* Nb) {
  const int n2 = 2 * nq, nx = n2 + 1;
  const long long tot = (long long)B * (N + 1);
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < tot; e += (long long)gridDim.x * blockDim.x) {
    const long long b = e / (N + 1);
    for (int i = 0; i < n2; ++i) xg7[e * nx + i] = xg6[e * n2 + i];
    xg7[e * nx + n2] = hstep;
    if (e % (N + 1) == 0) {
      Nb[b] = N;
      for (int i = 0; i < n2; ++i) {
        lbx7[b * nx + i] = lbx[i]; ubx7[b * nx + i] = ubx[i];
        lbxe7[b * nx + i] = lbxe[i]; ubxe7[b * nx + i] = ubxe[i];
        lbx0[b * nx + i] = ubx0[b * nx + i] = x0[b * n2 + i];
      }
      lbx7[b * nx + n2] = lbxe7[b * nx + n2] = -INFINITY;
      ubx7[b * nx + n2] = ubxe7[b * nx + n2] = INFINITY;
      lbx0[b * nx + n2] = ubx0[b * nx + n2] = hstep;
      for (int a = 0; a < nq; ++a) { lbu_b[b * nq + a] = lbu[a]; ubu_b[b * nq + a] = ubu[a]; }
      for (int a = 0; a <= nq; ++a) p[b * (nq + 1) + a] = 0.0;
    }
  }
}
__global__ void k_mpc_strip(long long tot, int nq, const double* __restrict__ xo7, double* __restrict__ xo6) {
  const int n2 = 2 * nq, nx = n2 + 1;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < tot; e += (long long)gridDim.x * blockDim.x)
    for (int i = 0; i < n2; ++i) xo6[e * n2 + i] = xo7[e * nx + i];
}
__global__ void k_transpose(int H, const double* __restrict__ a, double* __restrict__ at) {
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < (long long)H * H; e += (long long)gridDim.x * blockDim.x)
    at[(e % H) * H + e / H] = a[e];
}

static int mpc_solve(vboc_handle h, const vboc_mpc_batch_t* b, const vboc_mpc_soft_t* sf, void* stream,
                     const std::string& W, int qcf = 0);

int vboc_mpc_solve_batch(vboc_handle h, const vboc_mpc_batch_t* b, void* stream) {
  return mpc_solve(h, b, nullptr, stream, "vboc_mpc_solve_batch");
}

// AL compute_problem (AL/triplependulum_class_al.py:148-169): every stage's x guess (q0, 0) (:157-160), u = 0 (reset)
__global__ void k_al_guess(int B, int N, int nq, const double* __restrict__ x0, double* __restrict__ xg,
                           double* __restrict__ ug) {
  const int n2 = 2 * nq;
  const long long tot = (long long)B * (N + 1);
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < tot; e += (long long)gridDim.x * blockDim.x) {
    const long long b = e / (N + 1), k = e % (N + 1);
    for (int i = 0; i < n2; ++i) xg[e * n2 + i] = i < nq ? x0[b * n2 + i] : 0.0;
    if (k < N)
      for (int a = 0; a < nq; ++a) ug[(b * N + k) * nq + a] = 0.0;
  }
}
// compute_problem's return value: 1 (status 0), 0 (status 4), 2 (any other status) (:164-169)
__global__ void k_al_label(int B, const int* __restrict__ status, int* __restrict__ label) {
  for (int b = blockIdx.x * blockDim.x + threadIdx.x; b < B; b += gridDim.x * blockDim.x)
    label[b] = status[b] == 0 ? 1 : (status[b] == 4 ? 0 : 2);
}

int vboc_al_solve_batch(vboc_handle h, const vboc_al_batch_t* b, void* stream) {
  const std::string W = "vboc_al_solve_batch";
  if (!h || !b) return fail(VBOC_ERR_ARG, W + ": NULL argument");
  if (busy(h, W.c_str())) return VBOC_ERR_ARG;
  if (b->B < 0 || b->N < 1 || b->N > h->nmax) return fail(VBOC_ERR_ARG, W + ": needs B >= 0 and 1 <= N <= nmax");
  if (b->B == 0) { h->launches = 0; return VBOC_OK; }
  const void* ptrs[] = {b->x0, b->lbx, b->ubx, b->lbu, b->ubu, b->lbx_e, b->ubx_e, b->W, b->We, b->label,
                        b->status, b->x_out, b->u_out, b->qp_iter};
  for (const void* q : ptrs)
    if (!q) return fail(VBOC_ERR_ARG, W + ": NULL array in batch");
  if (h->nq != 3) return fail(VBOC_ERR_UNSUPPORTED, W + ": the AL labelling OCP is the triple pendulum's (nq = 3)");
  HIPCHK(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  constexpr int NQ = 3;
  const size_t B = (size_t)b->B, N = (size_t)b->N;
  // the guesses, the cost and the sqp counter the Safe-MPC call writes, in a buffer of their own (mpc_solve owns
  // mpc_buf)
  const size_t need = (B * (N + 1) * 2 * NQ + B * N * NQ + B) * sizeof(double) + B * sizeof(int) + 256;
  if (need > h->al_bytes) {
    if (h->al_buf) (void)hipFree(h->al_buf);
    h->al_buf = nullptr;
    h->al_bytes = 0;
    if (hipMalloc(&h->al_buf, need) != hipSuccess) return fail(VBOC_ERR_NOMEM, W + ": hipMalloc of the guesses");
    h->al_bytes = need;
  }
  double* xg = (double*)h->al_buf;
  double* ug = xg + B * (N + 1) * 2 * NQ;
  double* cost = ug + B * N * NQ;
  int* sqp = (int*)(cost + B);
  hipLaunchKernelGGL(k_al_guess, dim3(256), dim3(256), 0, st, b->B, b->N, NQ, b->x0, xg, ug);
  HIPCHK(hipGetLastError());
  static const double zero[3 * NQ] = {0.0};   // yref = yref_e = 0 (:114-115)
  vboc_mpc_batch_t m{};
  m.B = b->B; m.N = b->N; m.rti = 1; m.hidden = 0; m.h = b->h; m.cost_scale = b->cost_scale;
  m.x0 = b->x0; m.x_guess = b->x_guess ? b->x_guess : xg; m.u_guess = ug;   // u = 0 (reset) in both variants
  m.lbx = b->lbx; m.ubx = b->ubx; m.lbu = b->lbu; m.ubu = b->ubu; m.lbx_e = b->lbx_e; m.ubx_e = b->ubx_e;
  m.W = b->W; m.We = b->We; m.yref = zero; m.yref_e = zero;
  m.status = b->status; m.x_out = b->x_out; m.u_out = b->u_out; m.cost = cost; m.sqp_iter = sqp;
  m.qp_iter = b->qp_iter; m.h_out = nullptr;
  const int rc = mpc_solve(h, &m, nullptr, stream, W, 1);
  if (rc != VBOC_OK) return rc;
  hipLaunchKernelGGL(k_al_label, dim3(64), dim3(256), 0, st, b->B, b->status, b->label);
  HIPCHK(hipGetLastError());
  return VBOC_OK;
}

int vboc_mpc_soft_solve_batch(vboc_handle h, const vboc_mpc_batch_t* b, const vboc_mpc_soft_t* soft, void* stream) {
  const std::string W = "vboc_mpc_soft_solve_batch";
  if (!soft) return fail(VBOC_ERR_ARG, W + ": NULL soft-constraint description");
  if (b && b->B > 0 && !soft->Zl) return fail(VBOC_ERR_ARG, W + ": NULL Zl (the per-stage slack weights)");
  if (b && b->hidden <= 0) return fail(VBOC_ERR_ARG, W + ": the soft rows need the network (hidden > 0)");
  if (!(soft->safety_margin < 100.0)) return fail(VBOC_ERR_ARG, W + ": safety_margin must be < 100");
  return mpc_solve(h, b, soft, stream, W);
}

static int mpc_solve(vboc_handle h, const vboc_mpc_batch_t* b, const vboc_mpc_soft_t* sf, void* stream,
                     const std::string& W, int qcf) {
  if (busy(h, W.c_str())) return VBOC_ERR_ARG;
  if (!h || !b) return fail(VBOC_ERR_ARG, W + ": NULL argument");
  if (h->nq != 3) return fail(VBOC_ERR_UNSUPPORTED, W + ": the Safe-MPC OCP is the triple pendulum's (nq = 3)");
  if (h->o.hc) return fail(VBOC_ERR_UNSUPPORTED, W + ": no path constraint in the Safe-MPC OCP (clear it first)");
  if (b->B < 0 || b->N < 1 || b->N > h->nmax) return fail(VBOC_ERR_ARG, W + ": needs B >= 0 and 1 <= N <= nmax");
  if (b->hidden < 0 || b->hidden > FT_NN_MAX) return fail(VBOC_ERR_ARG, W + ": hidden must be in [0, 512]");
  if (!(b->h > 0.0)) return fail(VBOC_ERR_ARG, W + ": the time step must be positive");
  if (b->B == 0) { h->launches = 0; return VBOC_OK; }
  const void* ptrs[] = {b->x0, b->x_guess, b->u_guess, b->lbx, b->ubx, b->lbu, b->ubu, b->lbx_e, b->ubx_e, b->W,
                        b->We, b->yref, b->yref_e, b->status, b->x_out, b->u_out, b->cost, b->sqp_iter, b->qp_iter};
  for (const void* q : ptrs)
    if (!q) return fail(VBOC_ERR_ARG, W + ": NULL array in batch");
  if (b->hidden > 0 && (!b->W0 || !b->b0 || !b->W1 || !b->b1 || !b->W2 || !b->b2))
    return fail(VBOC_ERR_ARG, W + ": NULL network parameter");
  HIPCHK(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  constexpr int NQ = 3, NX = 2 * NQ + 1, NU = NQ;
  const size_t B = (size_t)b->B, N = (size_t)b->N, H = (size_t)b->hidden;
  const size_t dbl = B * (N + 1) * NX * 2 + B * NX * 6 + B * NU * 2 + B * (NQ + 1) + H * H;
  const size_t need = dbl * sizeof(double) + B * sizeof(int) + 512;
  if (need > h->mpc_bytes) {
    if (h->mpc_buf) (void)hipFree(h->mpc_buf);
    h->mpc_buf = nullptr;
    h->mpc_bytes = 0;
    if (hipMalloc(&h->mpc_buf, need) != hipSuccess) return fail(VBOC_ERR_NOMEM, W + ": hipMalloc of the batch inputs");
    h->mpc_bytes = need;
  }
  double* d = (double*)h->mpc_buf;
  auto take = [&](size_t n) { double* r = d; d += (n + 1) & ~(size_t)1; return r; };
  double* xg7 = take(B * (N + 1) * NX);
  double* xo7 = take(B * (N + 1) * NX);
  double *lbx7 = take(B * NX), *ubx7 = take(B * NX), *lbx0 = take(B * NX), *ubx0 = take(B * NX);
  double *lbxe7 = take(B * NX), *ubxe7 = take(B * NX), *lbu_b = take(B * NU), *ubu_b = take(B * NU);
  double* pp = take(B * (NQ + 1));
  double* w1t = take(H * H);
  int* Nb = (int*)d;
  hipLaunchKernelGGL(k_mpc_prep, dim3(256), dim3(256), 0, st, b->B, b->N, NQ, b->h, b->x0, b->x_guess, b->lbx, b->ubx,
                     b->lbu, b->ubu, b->lbx_e, b->ubx_e, xg7, lbx7, ubx7, lbu_b, ubu_b, lbx0, ubx0, lbxe7, ubxe7, pp,
                     Nb);
  MpcArgs mp{};
  mp.on = 1; mp.rti = b->rti ? 1 : 0; mp.hid = b->hidden; mp.cs = b->cost_scale; mp.qcf = qcf;
  const double *Wh = b->W, *Weh = b->We, *yr = b->yref, *yre = b->yref_e;   // host constants
  for (int i = 0; i < 2 * NQ; ++i) { mp.wq[i] = Wh[i]; mp.yr[i] = yr[i]; mp.we[i] = Weh[i]; mp.yre[i] = yre[i]; }
  mp.wq[2 * NQ] = mp.yr[2 * NQ] = mp.we[2 * NQ] = mp.yre[2 * NQ] = 0.0;   // the pinned dt column carries no cost
  for (int a = 0; a < NU; ++a) { mp.wq[NX + a] = Wh[2 * NQ + a]; mp.yr[NX + a] = yr[2 * NQ + a]; }
  if (b->hidden > 0) {
    hipLaunchKernelGGL(k_transpose, dim3(256), dim3(256), 0, st, b->hidden, b->W1, w1t);
    mp.W0 = b->W0; mp.b0 = b->b0; mp.W1 = b->W1; mp.W1T = w1t; mp.b1 = b->b1; mp.W2 = b->W2; mp.b2 = b->b2;
    mp.mean = b->mean; mp.std = b->std; mp.lh = b->lh; mp.uh = b->uh;
  }
  mp.hrow = b->h_out;
  mp.soft = 0; mp.sm = 100.0; mp.zl = mp.Zl = mp.Wb = mp.Web = nullptr;
  if (sf) {   // OCPtriplependulumSoftTraj: the margin-scaled row on every stage, soft lower sides
    mp.soft = 1; mp.sm = 100.0 - sf->safety_margin;
    mp.zl = sf->zl; mp.Zl = sf->Zl; mp.Wb = sf->W_b; mp.Web = sf->We_b;
  }
  Inputs in;
  in.B = b->B; in.nmax = b->N; in.N = Nb;
  in.xg = xg7; in.ug = b->u_guess; in.p = pp; in.lbx = lbx7; in.ubx = ubx7; in.lbu = lbu_b; in.ubu = ubu_b;
  in.lbx0 = lbx0; in.ubx0 = ubx0; in.lbxe = lbxe7; in.ubxe = ubxe7;
  in.status = b->status; in.xo = xo7; in.uo = b->u_out; in.cost = b->cost; in.sqp_iter = b->sqp_iter;
  in.qp_iter = b->qp_iter; in.head = h->head;
  HIPCHK(hipMemsetAsync(h->head, 0, 256, st));
  HIPCHK(hipEventRecord(h->ev0, st));
  const int rc = launch_ft<NQ>(h, in, st, mp);
  if (rc == -1) return fail(VBOC_ERR_NOMEM, W + ": hipMalloc of the stage regions");
  if (rc) return fail(VBOC_ERR_HIP, W + ": " + hipGetErrorString(hipGetLastError()));
  HIPCHK(hipEventRecord(h->ev1, st));
  hipLaunchKernelGGL(k_mpc_strip, dim3(256), dim3(256), 0, st, (long long)(B * (N + 1)), NQ, xo7, b->x_out);
  HIPCHK(hipGetLastError());
  h->launches = 1;
  return VBOC_OK;
}

int vboc_solve_batch_host(vboc_handle h, const vboc_batch_t* b) { return solve_host(h, b, false); }
int vboc_solve_batch_ft_host(vboc_handle h, const vboc_batch_t* b) { return solve_host(h, b, true); }

static int dg_wait(vboc_handle h, vboc_dg_batch_t* b, hipStream_t st);

int vboc_data_generation(vboc_handle h, vboc_dg_batch_t* b, void* stream) {
  const int rc = vboc_data_generation_async(h, b, nullptr, nullptr, stream);
  if (rc != VBOC_OK || !b || b->B == 0) return rc;
  return dg_wait(h, b, (hipStream_t)stream);
}

int vboc_data_generation_wait(vboc_handle h, vboc_dg_batch_t* b, void* stream) {
  if (!h || !b) return fail(VBOC_ERR_ARG, "vboc_data_generation_wait: NULL argument");
  if (b->B == 0) return VBOC_OK;
  return dg_wait(h, b, (hipStream_t)stream);
}

// the per-workgroup records, job descriptor and counters of a k_dg / k_ts launch (testing: the held-out set's
// state machine, no speculation, one row per problem)
static int dg_prepare(vboc_handle h, vboc_dg_batch_t* b, int* done_flag, const int* cancel, hipStream_t st,
                      bool testing, int max_restarts, const char* who) {
  const std::string W(who);
  if (busy(h, who)) return VBOC_ERR_ARG;
  if (h->nq != 2 && h->nq != 3)
    return fail(VBOC_ERR_UNSUPPORTED, W + ": defined for the double (nq = 2) and triple (nq = 3) pendulum");
  if (h->o.hc)
    return fail(VBOC_ERR_UNSUPPORTED, W + ": the boundary OCP of this driver has no path constraint (clear it first)");
  if (b->B < 0) return fail(VBOC_ERR_ARG, W + ": B < 0");
  b->rows_used = 0;
  if (b->B == 0) return VBOC_OK;
  if (b->N_start < 2 || b->N_start + 12 > h->nmax)
    return fail(VBOC_ERR_ARG, W + ": needs 2 <= N_start and N_start + 12 <= the handle's nmax "
                              "(horizon extension +9, verification horizons up to N - 1 + 4)");
  if (!b->ids || !b->rows || !b->row_off || !b->row_cnt || !b->stats ||
      (!testing && h->nq == 2 && (!b->ic || !b->ic_slot)))
    return fail(VBOC_ERR_ARG, W + ": NULL array");
  if (testing && b->rows_cap < b->B) return fail(VBOC_ERR_ARG, W + ": rows_cap < B (one row per problem)");
  if (testing && max_restarts < 0) return fail(VBOC_ERR_ARG, W + ": max_restarts < 0");
  if (!h->coop_ok) return fail(VBOC_ERR_HIP, W + ": wave solver unavailable on this device");
  HIPCHK(hipSetDevice(h->device));
  long long groups = b->B < h->n_regions ? b->B : h->n_regions;
  // resident problems: their hot stage records at the horizons data generation uses (N_start .. +12) fit the MALL
  const long long cap = h->group_cap > 0 ? h->group_cap
                                         : (h->mall_mib > 0 ? wave_group_budget(h, b->N_start + 10) : 0);
  if (cap > 0 && groups > cap) groups = cap;
  h->last_groups = groups;
  // per-workgroup arrays: the solver's one-problem batch (Inputs layout) + x_sol, u_sol, saved rows, state
  const int nq = h->nq, NXR = 2 * nq + 1, NU = nq, NP = nq + 1, NX = 2 * nq, nm = h->nmax;
  const int vr_cap = 2 * nm + 2;
  const size_t st_bytes = nq == 2 ? (sizeof(DgState<2>) > sizeof(TsState<2>) ? sizeof(DgState<2>) : sizeof(TsState<2>))
                                  : (sizeof(DgState<3>) > sizeof(TsState<3>) ? sizeof(DgState<3>) : sizeof(TsState<3>));
  const int st_d = (int)((st_bytes + 15) / 16 * 2);
  const size_t G = (size_t)groups;
  const size_t dbl = G * ((size_t)(nm + 1) * NXR * 3 + (size_t)nm * NU * 2 + (size_t)(nm + 1) * NU + NP + 6 * NXR +
                          2 * NU + 1 + (size_t)vr_cap * NX + st_d) + 64;
  const size_t need = dbl * sizeof(double) + 4 * G * sizeof(int) + 256;
  if (need > h->dg_bytes) {
    if (h->dg_scratch) (void)hipFree(h->dg_scratch);
    h->dg_scratch = nullptr;
    h->dg_bytes = 0;
    if (hipMalloc((void**)&h->dg_scratch, need) != hipSuccess)
      return fail(VBOC_ERR_NOMEM, W + ": hipMalloc of the state-machine records");
    h->dg_bytes = need;
  }
  if (!h->dg_jobs && hipMalloc((void**)&h->dg_jobs, sizeof(DgJobs)) != hipSuccess)
    return fail(VBOC_ERR_NOMEM, W + ": hipMalloc of the job descriptor");
  if (!h->dg_in && hipMalloc((void**)&h->dg_in, sizeof(Inputs)) != hipSuccess)
    return fail(VBOC_ERR_NOMEM, W + ": hipMalloc of the batch descriptor");
  double* d = h->dg_scratch;
  auto take = [&](size_t n) { double* r = d; d += (n + 1) & ~(size_t)1; return r; };
  Inputs in;
  in.B = (int)groups; in.nmax = nm; in.head = nullptr;
  double* xg = take(G * (nm + 1) * NXR); double* ug = take(G * nm * NU); double* pp = take(G * NP);
  double* lbx = take(G * NXR); double* ubx = take(G * NXR); double* lbu = take(G * NU); double* ubu = take(G * NU);
  double* lbx0 = take(G * NXR); double* ubx0 = take(G * NXR); double* lbxe = take(G * NXR); double* ubxe = take(G * NXR);
  in.xg = xg; in.ug = ug; in.p = pp; in.lbx = lbx; in.ubx = ubx; in.lbu = lbu; in.ubu = ubu;
  in.lbx0 = lbx0; in.ubx0 = ubx0; in.lbxe = lbxe; in.ubxe = ubxe;
  in.xo = take(G * (nm + 1) * NXR); in.uo = take(G * nm * NU); in.cost = take(G);
  DgJobs J;
  J.xs = take(G * (nm + 1) * NXR); J.us = take(G * (nm + 1) * NU); J.vr = take(G * vr_cap * NX);
  J.st = take(G * st_d);
  J.vr_cap = vr_cap; J.st_doubles = st_d;
  int* ip = (int*)d;
  in.N = ip; ip += G;
  in.status = ip; ip += G;
  in.sqp_iter = ip; ip += G;
  in.qp_iter = ip; ip += G;
  if ((size_t)((char*)ip - (char*)h->dg_scratch) > need) return fail(VBOC_ERR_ARG, W + ": internal size error");
  J.ids = b->ids; J.count = b->B; J.N_start = b->N_start; J.nmax = nm; J.seed = b->seed;
  J.fail_mod = h->dg_fail_mod;
  J.max_restarts = max_restarts;
  J.fmt_scale = nq == 2 ? 1e4 : 1e3;
  J.q_min = b->q_min; J.q_max = b->q_max; J.v_max = b->v_max; J.u_max = b->u_max; J.dt = b->dt; J.tol = b->tol;
  J.eps = b->eps; J.g = b->g; J.l1 = b->l1; J.l2 = b->l2; J.m1 = b->m1; J.m2 = b->m2;
  J.rows = b->rows; J.rows_cap = b->rows_cap; J.row_off = b->row_off; J.row_cnt = b->row_cnt;
  J.ic = (!testing && h->nq == 2) ? b->ic : nullptr; J.ic_slot = (!testing && h->nq == 2) ? b->ic_slot : nullptr;
  J.stats = b->stats;
  J.done_flag = done_flag; J.cancel = cancel;
  // counters: [0] job queue, [1] finished problems, [2..3] error flags, [4..5] rows used (u64),
  // [6] speculation events, [7] / [8] restart-job queue tail / head, [10..13] speculative solves run / used (u64),
  // [16..17] / [18..19] parked-job queue tails / heads, [20] / [21] eager restart-job queue tail / head,
  // [22..23] the launch's first job start (u64, the critical-path rule)
  J.next = h->head; J.done = h->head + 1; J.err = h->head + 2; J.rows_next = (unsigned long long*)(h->head + 4);
  J.spec_ev_next = h->head + 6; J.spec_q_tail = h->head + 7; J.spec_q_head = h->head + 8;
  J.spec_count = (unsigned long long*)(h->head + 10);
  // speculative restarts: one event per failed horizon-extension chain, at most min(B, 8192) per launch
  J.spec_events = 0; J.spec_stride = 0; J.spec = nullptr; J.spec_early = h->dg_spec_early; J.spec_pause = h->dg_spec_pause; J.spec_first = (h->dg_spec_first == 1 || (h->dg_spec_first == 2 && (long long)b->B < 128 * groups)) ? 1 : 0;
  J.spec_claim = J.spec_done = J.spec_cancel = J.spec_q = J.spec_eq = nullptr;
  J.spec_window = 0; J.spec_eq_tail = h->head + 20; J.spec_eq_head = h->head + 21;
  J.spec_crit = 0; J.t_launch = (unsigned long long*)(h->head + 22);   // [22..23]
  size_t spec_ctl = 0;
  if (h->dg_speculate && !testing) {
    const int E = b->B < 8192 ? b->B : 8192;
    const long long res = DG_SPEC_RH + (long long)(nm + 1) * NXR + (long long)nm * NU;
    const long long stride = DG_SPEC_HDR + DG_SPEC_JOBS * res;
    spec_ctl = sizeof(int) * ((size_t)E * (2 * (DG_SPEC_JOBS + 1) + 1 + 2 * DG_SPEC_JOBS));
    const size_t sneed = spec_ctl + sizeof(double) * (size_t)E * (size_t)stride + 256;
    if (sneed > h->dg_spec_bytes) {
      if (h->dg_spec) (void)hipFree(h->dg_spec);
      h->dg_spec = nullptr;
      h->dg_spec_bytes = 0;
      if (hipMalloc(&h->dg_spec, sneed) != hipSuccess)
        return fail(VBOC_ERR_NOMEM, W + ": hipMalloc of the speculation pool");
      h->dg_spec_bytes = sneed;
    }
    int* ci = (int*)h->dg_spec;
    J.spec_claim = ci; ci += (size_t)E * (DG_SPEC_JOBS + 1);
    J.spec_done = ci; ci += (size_t)E * (DG_SPEC_JOBS + 1);
    J.spec_cancel = ci; ci += E;
    J.spec_q = ci; ci += (size_t)E * DG_SPEC_JOBS;
    J.spec_eq = ci;
    J.spec_window = h->dg_spec_window;
    J.spec_crit = h->dg_spec_crit ? 1 : 0;
    J.spec = (double*)((char*)h->dg_spec + ((spec_ctl + 255) & ~(size_t)255));
    J.spec_events = E; J.spec_stride = (int)stride;
    HIPCHK(hipMemsetAsync(h->dg_spec, 0, spec_ctl, st));
  }
  // parked first solves (data generation only): one result record per job, two queues, counters head[16..19]
  J.park_res = nullptr; J.park_q = nullptr; J.park_stride = 0;
  J.park_window = 0; J.park_hi_it = h->dg_park_hi;
  J.round_n = done_flag ? h->dg_round : 0;   // the round gate belongs to streamed launches (done flags) only
  J.park_tail = h->head + 16; J.park_head = h->head + 18;
  if (h->dg_park && !testing) {
    const int stride = (8 + (b->N_start + 1) * NXR + b->N_start * NU + 1) & ~1;
    const size_t qbytes = ((sizeof(int) * 2 * (size_t)b->B) + 255) & ~(size_t)255;
    const size_t pneed = qbytes + sizeof(double) * (size_t)stride * (size_t)b->B;
    if (pneed > h->dg_park_bytes) {
      if (h->dg_park_buf) (void)hipFree(h->dg_park_buf);
      h->dg_park_buf = nullptr;
      h->dg_park_bytes = 0;
      if (hipMalloc(&h->dg_park_buf, pneed) != hipSuccess)
        return fail(VBOC_ERR_NOMEM, W + ": hipMalloc of the parked first solves");
      h->dg_park_bytes = pneed;
    }
    J.park_q = (int*)h->dg_park_buf;
    J.park_res = (double*)((char*)h->dg_park_buf + qbytes);
    J.park_stride = stride;
    // park window: by default parked problems wait until the new ones run out (one launch = one batch).  A streamed
    // launch (done flags: pipeline.StreamedRounds, many VBOC iterations' ids in order) releases its iterations as they
    // complete, so a parked problem must not wait for every later iteration's new problems: there the window
    // defaults to the resident waves, i.e. a parked problem resumes about one wave-generation after it was parked
    J.park_window = h->dg_park_window > 0 ? h->dg_park_window : (done_flag ? (int)(groups < b->B ? groups : b->B) : b->B);
    HIPCHK(hipMemsetAsync(h->dg_park_buf, 0, sizeof(int) * 2 * (size_t)b->B, st));
  }
  HIPCHK(hipMemsetAsync(h->head, 0, 256, st));
  HIPCHK(hipEventRecord(h->ev0, st));
  hipError_t e;
  if (h->nq == 2)
    e = h->factor_mfma ? launch_dg<2, true>(h, J, in, groups, st, testing) : launch_dg<2, false>(h, J, in, groups, st, testing);
  else
    e = h->factor_mfma ? launch_dg<3, true>(h, J, in, groups, st, testing) : launch_dg<3, false>(h, J, in, groups, st, testing);
  if (e != hipSuccess) return fail(VBOC_ERR_HIP, W + ": " + hipGetErrorString(e));
  HIPCHK(hipEventRecord(h->ev1, st));
  h->launches = 1;
  h->coop_count = b->B;
  return VBOC_OK;
}

int vboc_data_generation_async(vboc_handle h, vboc_dg_batch_t* b, int* done_flag, const int* cancel, void* stream) {
  if (!h || !b) return fail(VBOC_ERR_ARG, "vboc_data_generation: NULL argument");
  const int rc = dg_prepare(h, b, done_flag, cancel, (hipStream_t)stream, false, 0, "vboc_data_generation");
  if (rc == VBOC_OK && b->B > 0) h->dg_busy = true;
  return rc;
}

int vboc_testing(vboc_handle h, vboc_dg_batch_t* b, int max_restarts, void* stream) {
  if (!h || !b) return fail(VBOC_ERR_ARG, "vboc_testing: NULL argument");
  const int rc = dg_prepare(h, b, nullptr, nullptr, (hipStream_t)stream, true, max_restarts, "vboc_testing");
  if (rc != VBOC_OK || b->B == 0) return rc;
  return dg_wait(h, b, (hipStream_t)stream);
}

int vboc_testing_test(vboc_handle h, vboc_tt_batch_t* b, void* stream) {
  if (busy(h, "vboc_testing_test")) return VBOC_ERR_ARG;
  if (!h || !b) return fail(VBOC_ERR_ARG, "vboc_testing_test: NULL argument");
  const bool cart = h->nq == 2 && h->o.hc, arm = h->nq == 4;
  if (!cart && !arm)
    return fail(VBOC_ERR_UNSUPPORTED, "vboc_testing_test: defined for the UR5 arm (nq = 4) and the Cartesian double "
                                      "pendulum (nq = 2 with the path constraint set)");
  if (cart && !(h->hc_wave && h->wave_hc))
    return fail(VBOC_ERR_UNSUPPORTED, "vboc_testing_test: the Cartesian constraint needs the wave solver (hc_wave)");
  if (b->B < 0) return fail(VBOC_ERR_ARG, "vboc_testing_test: B < 0");
  if (b->B == 0) return VBOC_OK;
  if (b->N_start < 2 || b->N_start + 2 > h->nmax) return fail(VBOC_ERR_ARG, "vboc_testing_test: needs 2 <= N_start < nmax - 1");
  if (!b->ids || !b->rows || !b->row_cnt || !b->stats) return fail(VBOC_ERR_ARG, "vboc_testing_test: NULL array");
  if (!h->coop_ok) return fail(VBOC_ERR_HIP, "vboc_testing_test: wave solver unavailable on this device");
  HIPCHK(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  long long groups = b->B < h->n_regions ? b->B : h->n_regions;
  const long long cap = h->group_cap > 0 ? h->group_cap : (h->mall_mib > 0 ? wave_group_budget(h, b->N_start + 10) : 0);
  if (cap > 0 && groups > cap) groups = cap;
  h->last_groups = groups;
  const int nq = h->nq, NXR = 2 * nq + 1, NU = nq, NP = nq + 1, nm = h->nmax;
  const int st_d = (int)((sizeof(TtState<4>) + 15) / 16 * 2);
  const size_t G = (size_t)groups;
  const size_t dbl = G * ((size_t)(nm + 1) * NXR * 2 + (size_t)nm * NU * 2 + NP + 6 * NXR + 2 * NU + 1 + st_d) + 64;
  const size_t need = dbl * sizeof(double) + 4 * G * sizeof(int) + 256;
  if (need > h->dg_bytes) {
    if (h->dg_scratch) (void)hipFree(h->dg_scratch);
    h->dg_scratch = nullptr;
    h->dg_bytes = 0;
    if (hipMalloc((void**)&h->dg_scratch, need) != hipSuccess)
      return fail(VBOC_ERR_NOMEM, "vboc_testing_test: hipMalloc of the per-problem records");
    h->dg_bytes = need;
  }
  if (!h->tt_jobs && hipMalloc((void**)&h->tt_jobs, sizeof(TtJobs)) != hipSuccess)
    return fail(VBOC_ERR_NOMEM, "vboc_testing_test: hipMalloc of the job descriptor");
  if (!h->dg_in && hipMalloc((void**)&h->dg_in, sizeof(Inputs)) != hipSuccess)
    return fail(VBOC_ERR_NOMEM, "vboc_testing_test: hipMalloc of the batch descriptor");
  double* d = h->dg_scratch;
  auto take = [&](size_t n) { double* r = d; d += (n + 1) & ~(size_t)1; return r; };
  Inputs in;
  in.B = (int)groups; in.nmax = nm; in.head = nullptr;
  in.xg = take(G * (nm + 1) * NXR); in.ug = take(G * nm * NU); in.p = take(G * NP);
  in.lbx = take(G * NXR); in.ubx = take(G * NXR); in.lbu = take(G * NU); in.ubu = take(G * NU);
  in.lbx0 = take(G * NXR); in.ubx0 = take(G * NXR); in.lbxe = take(G * NXR); in.ubxe = take(G * NXR);
  in.xo = take(G * (nm + 1) * NXR); in.uo = take(G * nm * NU); in.cost = take(G);
  TtJobs J;
  J.st = take(G * st_d);
  J.st_doubles = st_d;
  int* ip = (int*)d;
  in.N = ip; ip += G;
  in.status = ip; ip += G;
  in.sqp_iter = ip; ip += G;
  in.qp_iter = ip; ip += G;
  if ((size_t)((char*)ip - (char*)h->dg_scratch) > need) return fail(VBOC_ERR_ARG, "vboc_testing_test: internal size error");
  J.ids = b->ids; J.count = b->B; J.N_start = b->N_start; J.nmax = nm; J.draw_stream = b->draw_stream;
  J.fail_mod = h->dg_fail_mod;
  J.seed = b->seed; J.tol = b->tol; J.dt = b->dt;
  for (int c = 0; c < 8; ++c) { J.xlo[c] = b->xlo[c]; J.xhi[c] = b->xhi[c]; }
  for (int c = 0; c < 4; ++c) J.ulim[c] = b->ulim[c];
  J.rows = b->rows; J.row_cnt = b->row_cnt; J.stats = b->stats;
  J.next = h->head; J.done = h->head + 1; J.err = h->head + 2;
  HIPCHK(hipMemsetAsync(h->head, 0, 256, st));
  HIPCHK(hipEventRecord(h->ev0, st));
  const hipError_t e = arm ? launch_tt<4, false, false>(h, J, in, groups, st) : launch_tt<2, false, true>(h, J, in, groups, st);
  if (e != hipSuccess) return fail(VBOC_ERR_HIP, std::string("vboc_testing_test: ") + hipGetErrorString(e));
  HIPCHK(hipEventRecord(h->ev1, st));
  h->launches = 1;
  h->coop_count = b->B;
  HIPCHK(hipMemcpyAsync(h->host_done, h->head, 14 * sizeof(unsigned), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  const unsigned* c = h->host_done;
  if (c[3]) return fail(VBOC_ERR_ARG, "vboc_testing_test: a horizon passed the handle's nmax");
  if (c[1] != (unsigned)b->B) return fail(VBOC_ERR_HIP, "vboc_testing_test: not every problem finished");
  return VBOC_OK;
}

// the end of a data-generation launch: its counters, the pool and horizon checks
static int dg_wait(vboc_handle h, vboc_dg_batch_t* b, hipStream_t st) {
  // the handle is released on every path: a failed copy / sync leaves the launch's outcome unknown (reported), but
  // must not lock the handle for good
  hipError_t e = hipSetDevice(h->device);
  if (e == hipSuccess) e = hipMemcpyAsync(h->host_done, h->head, 14 * sizeof(unsigned), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  h->dg_busy = false;   // the launch has ended: the handle's buffers are free again
  if (e != hipSuccess) return fail(VBOC_ERR_HIP, std::string("vboc_data_generation: waiting for the launch: ") + hipGetErrorString(e));
  const unsigned* c = h->host_done;
  b->rows_used = (long long)(((unsigned long long)c[5] << 32) | c[4]);
  b->spec_solves = (long long)(((unsigned long long)c[11] << 32) | c[10]);
  b->spec_used = (long long)(((unsigned long long)c[13] << 32) | c[12]);
  if (c[2]) return fail(VBOC_ERR_NOMEM, "vboc_data_generation: the row pool (rows_cap) overflowed");
  if (c[3]) return fail(VBOC_ERR_HIP, "vboc_data_generation: a horizon exceeded nmax (internal error)");
  if (c[1] != (unsigned)b->B) return fail(VBOC_ERR_HIP, "vboc_data_generation: not every problem finished");
  return VBOC_OK;
}

int vboc_hjr_solve_batch(vboc_handle h, const vboc_hjr_batch_t* b, void* stream) {
  if (busy(h, "vboc_hjr_solve_batch")) return VBOC_ERR_ARG;
  if (!h || !b) return fail(VBOC_ERR_ARG, "vboc_hjr_solve_batch: NULL argument");
  if (h->nq > 3) return fail(VBOC_ERR_UNSUPPORTED, "vboc_hjr_solve_batch: defined for the pendulum chains (nq 1-3)");
  if (b->B < 0) return fail(VBOC_ERR_ARG, "vboc_hjr_solve_batch: B < 0");
  if (b->B == 0) return VBOC_OK;
  if (b->hidden != 100)
    return fail(VBOC_ERR_UNSUPPORTED, "vboc_hjr_solve_batch: NeuralNetCLS hidden size 100 (the reference's) only");
  if (!b->x0 || !b->W0 || !b->b0 || !b->W1 || !b->b1 || !b->W2 || !b->b2 || !b->status || !b->cost || !b->u ||
      !b->x1 || !b->sqp_iter || !b->qp_iter)
    return fail(VBOC_ERR_ARG, "vboc_hjr_solve_batch: NULL array");
  if (!(b->std > 0.0) || !(b->u_max > 0.0)) return fail(VBOC_ERR_ARG, "vboc_hjr_solve_batch: std and u_max must be > 0");
  HIPCHK(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  // the HJR classes' options (HJR/triplependulum_hjr_class.py:98-108): the VBOC SQP / merit settings, the ACADOS
  // default tolerances (no tol_stat / qp_solver_tol_stat set), levenberg_marquardt 1e-5 (pendulum 1e-2)
  Opts o;
  default_opts(o);
  o.tol_stat = 1e-6;
  o.qp_tol_stat = 1e-8;
  o.lm = h->nq == 1 ? 1e-2 : 1e-5;
  HjrNet net{b->W0, b->b0, b->W1, b->b1, b->W2, b->b2, b->mean, b->std};
  HjrJobs J{b->B, b->x0, b->u_max, b->status, b->cost, b->u, b->x1, b->sqp_iter, b->qp_iter};
  const dim3 grid((unsigned)((b->B + 63) / 64)), block(64);
  HIPCHK(hipEventRecord(h->ev0, st));
  switch (h->nq) {
    case 1: hipLaunchKernelGGL((k_hjr<1, 100>), grid, block, 0, st, net, o, J); break;
    case 2: hipLaunchKernelGGL((k_hjr<2, 100>), grid, block, 0, st, net, o, J); break;
    default: hipLaunchKernelGGL((k_hjr<3, 100>), grid, block, 0, st, net, o, J); break;
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(h->ev1, st));
  h->launches = 1;
  return VBOC_OK;
}

int vboc_rk4_batch(int nq, int B, double T, const double* x, const double* u, double* x_out, void* stream) {
  if (nq < 1 || nq > 4 || B < 0) return fail(VBOC_ERR_ARG, "vboc_rk4_batch: bad nq/B");
  if (B == 0) return VBOC_OK;
  if (!x || !u || !x_out) return fail(VBOC_ERR_ARG, "vboc_rk4_batch: NULL array");
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((B + 255) / 256), block(256);
  switch (nq) {
    case 1: hipLaunchKernelGGL(rk4_kernel<1>, grid, block, 0, st, B, T, x, u, x_out); break;
    case 2: hipLaunchKernelGGL(rk4_kernel<2>, grid, block, 0, st, B, T, x, u, x_out); break;
    case 3: hipLaunchKernelGGL(rk4_kernel<3>, grid, block, 0, st, B, T, x, u, x_out); break;
    default: hipLaunchKernelGGL(rk4_kernel<4>, grid, block, 0, st, B, T, x, u, x_out); break;
  }
  HIPCHK(hipGetLastError());
  return VBOC_OK;
}

int vboc_rk4_sens_batch_host(int nq, int B, double T, const double* x, const double* u, double* x_out, double* A,
                             double* Bm) {
  if (nq < 1 || nq > 4 || B < 0) return fail(VBOC_ERR_ARG, "vboc_rk4_sens_batch_host: bad nq/B");
  if (B == 0) return VBOC_OK;
  const size_t nx = 2 * nq;
  double *dx, *du, *dxo, *dA, *dB;
  HIPCHK(hipMalloc(&dx, B * nx * sizeof(double)));
  HIPCHK(hipMalloc(&du, B * nq * sizeof(double)));
  HIPCHK(hipMalloc(&dxo, B * nx * sizeof(double)));
  HIPCHK(hipMalloc(&dA, B * nx * nx * sizeof(double)));
  HIPCHK(hipMalloc(&dB, B * nx * nq * sizeof(double)));
  HIPCHK(hipMemcpy(dx, x, B * nx * sizeof(double), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(du, u, B * nq * sizeof(double), hipMemcpyHostToDevice));
  const dim3 grid((B + 255) / 256), block(256);
  switch (nq) {
    case 1: hipLaunchKernelGGL(rk4_sens_kernel<1>, grid, block, 0, nullptr, B, T, dx, du, dxo, dA, dB); break;
    case 2: hipLaunchKernelGGL(rk4_sens_kernel<2>, grid, block, 0, nullptr, B, T, dx, du, dxo, dA, dB); break;
    case 3: hipLaunchKernelGGL(rk4_sens_kernel<3>, grid, block, 0, nullptr, B, T, dx, du, dxo, dA, dB); break;
    default: hipLaunchKernelGGL(rk4_sens_kernel<4>, grid, block, 0, nullptr, B, T, dx, du, dxo, dA, dB); break;
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(x_out, dxo, B * nx * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(A, dA, B * nx * nx * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(Bm, dB, B * nx * nq * sizeof(double), hipMemcpyDeviceToHost));
  (void)hipFree(dx); (void)hipFree(du); (void)hipFree(dxo); (void)hipFree(dA); (void)hipFree(dB);
  return VBOC_OK;
}

int vboc_rk4_batch_host(int nq, int B, double T, const double* x, const double* u, double* x_out) {
  if (nq < 1 || nq > 4 || B < 0) return fail(VBOC_ERR_ARG, "vboc_rk4_batch_host: bad nq/B");
  if (B == 0) return VBOC_OK;
  const size_t nx = 2 * nq;
  double *dx = nullptr, *du = nullptr, *dxo = nullptr;
  HIPCHK(hipMalloc(&dx, B * nx * sizeof(double)));
  HIPCHK(hipMalloc(&du, B * nq * sizeof(double)));
  HIPCHK(hipMalloc(&dxo, B * nx * sizeof(double)));
  HIPCHK(hipMemcpy(dx, x, B * nx * sizeof(double), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(du, u, B * nq * sizeof(double), hipMemcpyHostToDevice));
  int rc = vboc_rk4_batch(nq, B, T, dx, du, dxo, nullptr);
  if (rc == 0) {
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(x_out, dxo, B * nx * sizeof(double), hipMemcpyDeviceToHost));
  }
  (void)hipFree(dx);
  (void)hipFree(du);
  (void)hipFree(dxo);
  return rc;
}

}  // extern "C"

// hjr.h - the HJR one-step OCP on the GPU: OCP<sys>.compute_problem(x0) of the reference's HJR classes
// (HJR/triplependulum_hjr_class.py:7-134, HJR/doublependulum_hjr_class.py, HJR/pendulum_hjr_class.py), one problem
// per LANE.
//
// The problem (oracle/vboc_oracle_hjr.c states it with its reference lines): N = 1, h = 1e-2, x0 fixed, u0 in a
// torque box, x1 free, terminal cost = logit 0 of NeuralNetCLS(2nq, H, 2) at x1; SQP with the exact Hessian
// (levenberg_marquardt * I: the ReLU network's Hessian is zero), L1 merit backtracking, a Mehrotra IPM on the
// one-stage QP (x1 eliminated: a dense nq x nq Cholesky).  The state of a problem is a few dozen doubles, so a lane
// carries one problem through its whole SQP in registers; the network's weights are the same for every problem,
// so every weight load is wave-uniform (the scalar cache serves all 64 lanes) and a wave evaluates the network
// for 64 problems per instruction.  The hidden layer of the lane's own network evaluation lives in registers
// (H doubles); ReLU masks are kept as bit words.
// Arithmetic follows the oracle; summation orders differ at rounding level only where noted.
#pragma once

namespace vboc {

struct HjrNet {
  const double *W0, *b0, *W1, *b1, *W2, *b2;   // NeuralNetCLS parameters (model.parameters() order), FP64
  double mean, std;
};

// logit 0 of the network at x and (GRAD) its gradient; relu' = 1 on a positive argument
template <int NX, int H, bool GRAD>
__device__ __forceinline__ double hjr_nn(const HjrNet& n, const double* x, double* grad) {
  constexpr int MW = (H + 31) / 32;
  double z0[NX], h1[H];
  unsigned m1[MW], m2[MW];
  UNR for (int w = 0; w < MW; ++w) { m1[w] = 0u; m2[w] = 0u; }
  UNR for (int i = 0; i < NX; ++i) z0[i] = (x[i] - n.mean) / n.std;
  UNR for (int j = 0; j < H; ++j) {
    double t = 0.0;
    UNR for (int i = 0; i < NX; ++i) t += n.W0[j * NX + i] * z0[i];
    t = n.b0[j] + t;
    if (t > 0.0) m1[j >> 5] |= 1u << (j & 31);
    h1[j] = fmax(0.0, t);
  }
  double out = 0.0;
#pragma unroll 2
  for (int j = 0; j < H; ++j) {
    const double* w1 = n.W1 + j * H;
    double t = 0.0;
    UNR for (int i = 0; i < H; ++i) t += w1[i] * h1[i];
    t = n.b1[j] + t;
    if (t > 0.0) m2[j >> 5] |= 1u << (j & 31);
    out += n.W2[j] * fmax(0.0, t);
  }
  out = n.b2[0] + out;
  if constexpr (GRAD) {
    double g[NX];
    UNR for (int c = 0; c < NX; ++c) g[c] = 0.0;
#pragma unroll 1
    for (int i = 0; i < H; ++i) {
      double t = 0.0;
#pragma unroll 4
      for (int j = 0; j < H; ++j) t += ((m2[j >> 5] >> (j & 31)) & 1u) ? n.W1[j * H + i] * n.W2[j] : 0.0;
      const double v = ((m1[i >> 5] >> (i & 31)) & 1u) ? t : 0.0;
      UNR for (int c = 0; c < NX; ++c) g[c] += n.W0[i * NX + c] * v;
    }
    UNR for (int c = 0; c < NX; ++c) grad[c] = g[c] / n.std;
  }
  return out;
}

// x1 = RK4(x0, u) (h = 1e-2) and B = dx1/du: the chains' model (model.h); the pendulum of the HJR class is
// undamped (HJR/pendulum_hjr_class.py:14-36), written out here
template <int NQ>
__device__ __forceinline__ void hjr_shoot(double h, const double* x, const double* u, double* x1, double* B) {
  constexpr int NX = 2 * NQ;
  if constexpr (NQ == 1) {
    constexpr double m = 0.5, g = 9.81, d = 0.3;
    constexpr double cc[4] = {0.0, 0.5, 0.5, 1.0};
    double k[4][2], dk[4][2];   // dk: derivative along u
    UNR for (int st = 0; st < 4; ++st) {
      double xa[2], sa[2];
      UNR for (int i = 0; i < 2; ++i) {
        xa[i] = st ? x[i] + cc[st] * h * k[st - 1][i] : x[i];
        sa[i] = st ? cc[st] * h * dk[st - 1][i] : 0.0;
      }
      k[st][0] = xa[1];
      k[st][1] = (m * g * d * sin(xa[0]) + u[0]) / (d * d * m);
      dk[st][0] = sa[1];
      dk[st][1] = (m * g * d * cos(xa[0]) / (d * d * m)) * sa[0] + 1.0 / (d * d * m);
    }
    UNR for (int i = 0; i < 2; ++i) {
      x1[i] = x[i] + h / 6.0 * (k[0][i] + 2.0 * k[1][i] + 2.0 * k[2][i] + k[3][i]);
      B[i] = h / 6.0 * (dk[0][i] + 2.0 * dk[1][i] + 2.0 * dk[2][i] + dk[3][i]);
    }
  } else {
    rk4_sens<NQ>(h, x, u, x1, [&](int i, int c, double v) {
      if (c >= NX) B[i * NQ + (c - NX)] = v;
    });
  }
}

template <int NQ, int H>
struct Hjr {
  static constexpr int NX = 2 * NQ, NU = NQ;
  const HjrNet& n;
  const Opts& o;
  double x0[NX], lbu, ubu, rho;
  double u[NU], x1[NX], pi[NX], ll[NU], lu[NU], wpi[NX], wbnd;
  double Bm[NX * NU], b[NX], gnn[NX];
  double du[NU], dx[NX], ql[NU], qu[NU], L[NU], U[NU], e0[NX], qpi[NX];

  __device__ Hjr(const HjrNet& n_, const Opts& o_) : n(n_), o(o_) {}

  // one-stage Riccati step (vboc_oracle_hjr.c newton): Hx = rho on x1
  __device__ __forceinline__ bool newton(const double* Hu, const double* gu, const double* gx, double rs, double* d_u,
                                         double* d_x) const {
    double Ru[NU * NU], v[NX], r[NU];
    UNR for (int a = 0; a < NU; ++a)
      UNR for (int c = 0; c < NU; ++c) {
        double t = (a == c) ? Hu[a] : 0.0;
        UNR for (int i = 0; i < NX; ++i) t += Bm[i * NU + a] * rho * Bm[i * NU + c];
        Ru[a * NU + c] = t;
      }
    if (!chol<NU>(Ru)) return false;
    UNR for (int i = 0; i < NX; ++i) v[i] = rho * (rs * e0[i]) + gx[i];
    UNR for (int a = 0; a < NU; ++a) {
      double t = gu[a];
      UNR for (int i = 0; i < NX; ++i) t += Bm[i * NU + a] * v[i];
      r[a] = t;
    }
    chol_solve<NU>(Ru, r);
    UNR for (int a = 0; a < NU; ++a) d_u[a] = -r[a];
    UNR for (int i = 0; i < NX; ++i) {
      double t = rs * e0[i];
      UNR for (int a = 0; a < NU; ++a) t += Bm[i * NU + a] * d_u[a];
      d_x[i] = t;
    }
    return true;
  }

  struct MR { double n, d; };
  __device__ __forceinline__ static void mr_add(MR& m, double t, double dt) {
    if (dt < 0.0 && t * m.d < m.n * (-dt)) { m.n = t; m.d = -dt; }
  }

  // the Mehrotra IPM of the oracle's qp(): 0 converged, 1 max-iter, -1 failure
  __device__ __forceinline__ int qp(int& iters) {
    int nbox = 0;
    UNR for (int a = 0; a < NU; ++a) {
      const double Lo = lbu - u[a], Up = ubu - u[a], del = o.push * (Up - Lo);
      double z0 = 0.0;
      if (z0 < Lo + del) z0 = Lo + del;
      if (z0 > Up - del) z0 = Up - del;
      L[a] = Lo; U[a] = Up; du[a] = z0;
      ql[a] = o.mu0 / (z0 - Lo);
      qu[a] = o.mu0 / (Up - z0);
      nbox += 2;
    }
    UNR for (int i = 0; i < NX; ++i) dx[i] = 0.0;
    double e00 = 0.0, rd0 = 0.0;
    UNR for (int i = 0; i < NX; ++i) {
      double t = b[i] - dx[i];
      UNR for (int a = 0; a < NU; ++a) t += Bm[i * NU + a] * du[a];
      e0[i] = t;
      e00 = fmax(e00, fabs(t));
    }
    UNR for (int a = 0; a < NU; ++a) rd0 = fmax(rd0, fabs(rho * du[a] - ql[a] + qu[a]));
    UNR for (int i = 0; i < NX; ++i) rd0 = fmax(rd0, fabs(rho * dx[i] + gnn[i]));
    double rs = 1.0;
    int it, status = 1;
    double Hu[NU], gu[NU], gx[NX], d_u[NU], d_x[NX], dua[NU];
    for (it = 0; it < o.qp_max_iter; ++it) {
      double mu = 0.0;
      UNR for (int a = 0; a < NU; ++a) mu += (du[a] - L[a]) * ql[a] + (U[a] - du[a]) * qu[a];
      mu /= (double)nbox;
      if (!isfinite(mu)) { status = -1; break; }
      if (mu < o.qp_tol_comp && rs * rd0 < o.qp_tol_stat && rs * e00 < o.qp_tol_eq) { status = 0; break; }
      UNR for (int a = 0; a < NU; ++a) {
        const double tl = du[a] - L[a], tu = U[a] - du[a];
        Hu[a] = rho + ql[a] * (1.0 / tl) + qu[a] * (1.0 / tu);
        gu[a] = rho * du[a];
      }
      UNR for (int i = 0; i < NX; ++i) gx[i] = rho * dx[i] + gnn[i];
      if (!newton(Hu, gu, gx, rs, d_u, d_x)) { status = -1; break; }
      MR ma{1.0, 1.0};
      UNR for (int a = 0; a < NU; ++a) {
        const double tl = du[a] - L[a], tu = U[a] - du[a], itl = 1.0 / tl, itu = 1.0 / tu, d = d_u[a];
        const double dll = -ql[a] - ql[a] * d * itl, dlu = -qu[a] + qu[a] * d * itu;
        mr_add(ma, tl, d);
        mr_add(ma, tu, -d);
        mr_add(ma, ql[a], dll);
        mr_add(ma, qu[a], dlu);
        dua[a] = d;
      }
      const double aa = ma.n / ma.d;
      double muaff = 0.0;
      UNR for (int a = 0; a < NU; ++a) {
        const double tl = du[a] - L[a], tu = U[a] - du[a], itl = 1.0 / tl, itu = 1.0 / tu, d = d_u[a];
        const double dll = -ql[a] - ql[a] * d * itl, dlu = -qu[a] + qu[a] * d * itu;
        muaff += (tl + aa * d) * (ql[a] + aa * dll) + (tu - aa * d) * (qu[a] + aa * dlu);
      }
      muaff /= (double)nbox;
      double sig = muaff / mu;
      sig = sig * sig * sig;
      if (sig > 1.0) sig = 1.0;
      const double smu = sig * mu;
      UNR for (int a = 0; a < NU; ++a) {
        const double tl = du[a] - L[a], tu = U[a] - du[a], itl = 1.0 / tl, itu = 1.0 / tu, d = dua[a];
        const double dll = -ql[a] - ql[a] * d * itl, dlu = -qu[a] + qu[a] * d * itu;
        const double rl = smu - tl * ql[a] - d * dll, ru = smu - tu * qu[a] + d * dlu;
        gu[a] = rho * du[a] - ql[a] - rl * itl + qu[a] + ru * itu;
      }
      if (!newton(Hu, gu, gx, rs, d_u, d_x)) { status = -1; break; }
      MR mx{1.0, o.tau};
      double dll[NU], dlu[NU];
      UNR for (int a = 0; a < NU; ++a) {
        const double tl = du[a] - L[a], tu = U[a] - du[a], itl = 1.0 / tl, itu = 1.0 / tu;
        const double d = d_u[a], da = dua[a];
        const double dlla = -ql[a] - ql[a] * da * itl, dlua = -qu[a] + qu[a] * da * itu;
        const double rl = smu - tl * ql[a] - da * dlla, ru = smu - tu * qu[a] + da * dlua;
        dll[a] = (rl - ql[a] * d) * itl;
        dlu[a] = (ru + qu[a] * d) * itu;
        mr_add(mx, tl, d);
        mr_add(mx, tu, -d);
        mr_add(mx, ql[a], dll[a]);
        mr_add(mx, qu[a], dlu[a]);
      }
      const double alpha = fmin(1.0, o.tau * (mx.n / mx.d));
      UNR for (int a = 0; a < NU; ++a) {
        ql[a] += alpha * dll[a];
        qu[a] += alpha * dlu[a];
        du[a] += alpha * d_u[a];
      }
      UNR for (int i = 0; i < NX; ++i) dx[i] += alpha * d_x[i];
      rs *= (1.0 - alpha);
    }
    iters = it;
    if (status < 0) return -1;
    UNR for (int i = 0; i < NX; ++i) qpi[i] = rho * dx[i] + gnn[i];
    UNR for (int a = 0; a < NU; ++a)
      if (!isfinite(du[a]) || !isfinite(ql[a]) || !isfinite(qu[a])) return -1;
    return status;
  }

  __device__ __forceinline__ double merit(double alpha) const {
    double uu[NU], xx[NX], phi[NX], Bt[NX * NU];
    double viol = 0.0;
    UNR for (int a = 0; a < NU; ++a) {
      uu[a] = u[a] + alpha * du[a];
      viol += fmax(0.0, lbu - uu[a]) + fmax(0.0, uu[a] - ubu);
    }
    UNR for (int i = 0; i < NX; ++i) xx[i] = x1[i] + alpha * dx[i];
    double val = hjr_nn<NX, H, false>(n, xx, nullptr) + wbnd * viol;
    hjr_shoot<NQ>(1e-2, x0, uu, phi, Bt);
    UNR for (int i = 0; i < NX; ++i) val += wpi[i] * fabs(phi[i] - xx[i]);
    return val;
  }

  // the SQP of vboc_oracle_hjr.c hjr_sqp; returns the ACADOS status
  __device__ __forceinline__ int solve(int& it, int& qtot) {
    int status = 2;
    qtot = 0;
    for (it = 0;; ++it) {
      double phi[NX];
      hjr_shoot<NQ>(1e-2, x0, u, phi, Bm);
      UNR for (int i = 0; i < NX; ++i) b[i] = phi[i] - x1[i];
      hjr_nn<NX, H, true>(n, x1, gnn);
      double st = 0, eq = 0, in = 0, cp = 0;
      UNR for (int i = 0; i < NX; ++i) eq = fmax(eq, fabs(b[i]));
      UNR for (int a = 0; a < NU; ++a) {
        double gr = -ll[a] + lu[a];
        UNR for (int r = 0; r < NX; ++r) gr += Bm[r * NU + a] * pi[r];
        st = fmax(st, fabs(gr));
        in = fmax(in, fmax(lbu - u[a], u[a] - ubu));
        cp = fmax(cp, fmax(fabs(ll[a] * (u[a] - lbu)), fabs(lu[a] * (ubu - u[a]))));
      }
      UNR for (int i = 0; i < NX; ++i) st = fmax(st, fabs(gnn[i] - pi[i]));
      if (!isfinite(st) || !isfinite(eq)) { status = 1; break; }
      if (st < o.tol_stat && eq < o.tol_eq && in < o.tol_ineq && cp < o.tol_comp) { status = 0; break; }
      if (it >= o.max_iter) { status = 2; break; }
      int qit = 0;
      const int qs = qp(qit);
      qtot += qit;
      if (qs < 0) { status = 4; break; }
      double lmax = 0.0;
      UNR for (int i = 0; i < NX; ++i) {
        const double a = fabs(qpi[i]), bb = 0.5 * (wpi[i] + a);
        wpi[i] = a > bb ? a : bb;
      }
      UNR for (int a = 0; a < NU; ++a) lmax = fmax(lmax, fmax(ql[a], qu[a]));
      {
        const double a = fabs(lmax), bb = 0.5 * (wbnd + a);
        wbnd = a > bb ? a : bb;
      }
      const double phi0 = merit(0.0);
      double alpha = 1.0;
      for (;;) {
        const double pa = merit(alpha);
        if (pa < phi0) break;
        if (alpha * o.alpha_red < o.alpha_min) break;
        alpha *= o.alpha_red;
      }
      UNR for (int a = 0; a < NU; ++a) {
        u[a] += alpha * du[a];
        ll[a] += alpha * (ql[a] - ll[a]);
        lu[a] += alpha * (qu[a] - lu[a]);
      }
      UNR for (int i = 0; i < NX; ++i) {
        x1[i] += alpha * dx[i];
        pi[i] += alpha * (qpi[i] - pi[i]);
      }
    }
    return status;
  }
};

struct HjrJobs {
  int B;
  const double* x0;   // [B][2nq]
  double u_max;
  int* status;
  double *cost, *u, *x1;   // [B], [B][nq], [B][2nq]
  int *sqp_iter, *qp_iter;
};

// one lane = one problem; the lanes of a wave share the weight loads
template <int NQ, int H>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1)))
void k_hjr(HjrNet net, Opts o, HjrJobs J) {
  constexpr int NX = 2 * NQ;
  const int p = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (p >= J.B) return;
  Hjr<NQ, H> P(net, o);
  const double* x = J.x0 + (long long)p * NX;
  UNR for (int i = 0; i < NX; ++i) P.x0[i] = x[i];
  P.lbu = -J.u_max;
  P.ubu = J.u_max;
  P.rho = o.lm;
  UNR for (int a = 0; a < NQ; ++a) { P.u[a] = 0.0; P.ll[a] = 0.0; P.lu[a] = 0.0; }
  UNR for (int i = 0; i < NX; ++i) { P.pi[i] = 0.0; P.wpi[i] = 0.0; }
  P.wbnd = 0.0;
  // compute_problem's guess (HJR/triplependulum_hjr_class.py:119)
  UNR for (int j = 0; j < NQ; ++j) { P.x1[j] = x[j] + x[NQ + j] * 1e-2; P.x1[NQ + j] = x[NQ + j] * 0.9; }
  int it = 0, qit = 0;
  const int status = P.solve(it, qit);
  J.status[p] = status;
  J.cost[p] = hjr_nn<NX, H, false>(net, P.x1, nullptr);
  UNR for (int a = 0; a < NQ; ++a) J.u[(long long)p * NQ + a] = P.u[a];
  UNR for (int i = 0; i < NX; ++i) J.x1[(long long)p * NX + i] = P.x1[i];
  J.sqp_iter[p] = it;
  J.qp_iter[p] = qit;
}

}  // namespace vboc

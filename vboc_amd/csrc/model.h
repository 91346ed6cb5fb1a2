// model.h - N-link pendulum dynamics, analytic Jacobians and ERK4 (+ forward sensitivities) for
// gfx950.  Device-only; one lane evaluates one problem's stage, everything in registers.
//
// Physics (same function as the reference's CasADi f_expl, pinned by tests/golden/dynamics_*.npz):
//  * nq = 2, 3: point-mass chain, mass m_i = 0.4 at the tip of massless link l_i = 0.8, absolute
//    angles from the downward vertical, generalised forces C_i on the angles
//      M(th) acc = u - cor(th, om) - grav(th),  M_jk = a_jk cos(th_j - th_k),
//      cor_j = sum_k a_jk sin(th_j - th_k) om_k^2,  grav_j = g mu_j l_j sin th_j,
//      mu_j = sum_{i>=j} m_i,  a_jk = mu_max(j,k) l_j l_k
//    (VBOC/doublependulum_class_vboc.py:14-91, VBOC/triplependulum_class_vboc.py:15-58).
//  * nq = 1: damped pendulum acc = (m g d sin th + F - b om) / (d^2 m), m=0.5, d=0.3, b=0.01
//    (VBOC/pendulum_class_vboc.py:14-39).
//  * nq = 4: the UR5 arm of VBOC/UR5/ur5reduced_class_fixedveldir.py:20-45 (4 revolute joints of
//    VBOC/UR5/ur5.urdf between base_link and tool0; urdf2casadi's ABA in the reference).  Here
//    M(q) acc = u - RNEA(q, qd, 0): a body-frame recursive Newton-Euler pass over the generated
//    parameters of ur5_params.h (tools/gen_ur5_model.py), M from RNEA columns, and Jacobian-vector
//    products by ONE forward-mode (dual-number) RNEA pass per direction:
//      d acc = M^-1 (du - d RNEA(q, qd, acc)|acc fixed).
// The dt state of the reference (f = dt * f_phys, RK4 with h = 1, tf = N) is folded into the
// step length h = dt (exact: the dt state has zero derivative and is pinned by the bounds).  The UR5
// OCP has no dt state (tf = 1 s over N = 100 intervals, set_new_time_steps(dt_sym = 1e-2)); its time
// step travels in the same dt column of the C ABI.
#pragma once
#include <hip/hip_runtime.h>

#define UR5_CONST static constexpr
#include "ur5_params.h"


#ifndef VBOC_SENS_GROUP
#define VBOC_SENS_GROUP 1
#endif

namespace vboc {

template <int NQ>
struct Dim {
  static constexpr int NX = 2 * NQ, NU = NQ, NZ = 3 * NQ, M0 = NQ + 1;
};

template <int NQ>
struct Chain {
  static constexpr double g = 9.81, m = 0.4, l = 0.8;
  __device__ __forceinline__ static constexpr double mu(int j) { return m * (NQ - j); }
  __device__ __forceinline__ static constexpr double a(int j, int k) { return mu(j > k ? j : k) * l * l; }
};

// Cholesky of a small SPD matrix held in registers (row-major, lower factor in place).
// Returns false on a non-positive pivot.
template <int n>
__device__ __forceinline__ bool chol(double (&A)[n * n]) {
  bool ok = true;
#pragma unroll
  for (int j = 0; j < n; ++j) {
    double s = A[j * n + j];
#pragma unroll
    for (int k = 0; k < j; ++k) s -= A[j * n + k] * A[j * n + k];
    ok = ok && (s > 0.0);
    const double d = sqrt(s > 0.0 ? s : 1.0);
    const double inv = 1.0 / d;
    A[j * n + j] = d;
#pragma unroll
    for (int i = j + 1; i < n; ++i) {
      double t = A[i * n + j];
#pragma unroll
      for (int k = 0; k < j; ++k) t -= A[i * n + k] * A[j * n + k];
      A[i * n + j] = t * inv;
    }
  }
  return ok;
}

template <int n>
__device__ __forceinline__ void chol_solve(const double (&L)[n * n], double (&b)[n]) {
#pragma unroll
  for (int i = 0; i < n; ++i) {
    double t = b[i];
#pragma unroll
    for (int k = 0; k < i; ++k) t -= L[i * n + k] * b[k];
    b[i] = t / L[i * n + i];
  }
#pragma unroll
  for (int i = n - 1; i >= 0; --i) {
    double t = b[i];
#pragma unroll
    for (int k = i + 1; k < n; ++k) t -= L[k * n + i] * b[k];
    b[i] = t / L[i * n + i];
  }
}


// ---------------------------------------------------------------------------------------------
// UR5 (nq = 4) rigid-body dynamics: generic over double and a forward-mode dual number
// ---------------------------------------------------------------------------------------------
struct Dl {
  double v, d;
};
__device__ __forceinline__ Dl operator+(Dl a, Dl b) { return {a.v + b.v, a.d + b.d}; }
__device__ __forceinline__ Dl operator-(Dl a, Dl b) { return {a.v - b.v, a.d - b.d}; }
__device__ __forceinline__ Dl operator-(Dl a) { return {-a.v, -a.d}; }
__device__ __forceinline__ Dl operator*(Dl a, Dl b) { return {a.v * b.v, a.v * b.d + a.d * b.v}; }
__device__ __forceinline__ Dl operator*(double a, Dl b) { return {a * b.v, a * b.d}; }
__device__ __forceinline__ Dl operator*(Dl a, double b) { return {a.v * b, a.d * b}; }
__device__ __forceinline__ Dl operator+(Dl a, double b) { return {a.v + b, a.d}; }
__device__ __forceinline__ void tsincos(double x, double* s, double* c) { sincos(x, s, c); }
__device__ __forceinline__ void tsincos(Dl x, Dl* s, Dl* c) {
  double sv, cv;
  sincos(x.v, &sv, &cv);
  *s = {sv, cv * x.d};
  *c = {cv, -sv * x.d};
}
template <class T>
__device__ __forceinline__ T tzero() { return T{}; }
template <>
__device__ __forceinline__ double tzero<double>() { return 0.0; }
template <>
__device__ __forceinline__ Dl tzero<Dl>() { return Dl{0.0, 0.0}; }

template <class T, class U>
__device__ __forceinline__ void cross3(const T* a, const U* b, T* o) {
  const T t0 = a[1] * b[2] - a[2] * b[1], t1 = a[2] * b[0] - a[0] * b[2], t2 = a[0] * b[1] - a[1] * b[0];
  o[0] = t0; o[1] = t1; o[2] = t2;
}
template <class T>
__device__ __forceinline__ void cross3c(const double* a, const T* b, T* o) {   // constant x T
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}

// tau = RNEA(q, qd, qdd) in body coordinates (VEL: velocity terms, GRAV: gravity (0, 0, -9.81)).
// Joint i: child frame = joint frame (UR5_R, UR5_P in the parent body) rotated by Rz(q_i); motion
// transform E = Rz(q)^T R^T, r = P:  X (w, v) = (E w, E (v - r x w));  X^T (n, f) = (E^T n + r x E^T f, E^T f).
template <class T, bool VEL, bool GRAV>
__device__ __forceinline__ void ur5_rnea(const T* q, const T* qd, const double* qdd, T* tau) {
  T cs[4], sn[4], fn[4][3], ff[4][3];
  T w[3], v[3], aw[3], av[3];
  const T z = tzero<T>();
#pragma unroll
  for (int a = 0; a < 3; ++a) { w[a] = z; v[a] = z; aw[a] = z; av[a] = z; }
  if constexpr (GRAV) av[2] = av[2] + 9.81;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    tsincos(q[i], &sn[i], &cs[i]);
    T E[9];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      E[0 * 3 + k] = cs[i] * UR5_R[9 * i + k * 3 + 0] + sn[i] * UR5_R[9 * i + k * 3 + 1];
      E[1 * 3 + k] = cs[i] * UR5_R[9 * i + k * 3 + 1] - sn[i] * UR5_R[9 * i + k * 3 + 0];
      E[2 * 3 + k] = z + UR5_R[9 * i + k * 3 + 2];
    }
    const double r[3] = {UR5_P[3 * i], UR5_P[3 * i + 1], UR5_P[3 * i + 2]};
    T t[3], t2[3], nw[3], nv[3], naw[3], nav[3];
    if constexpr (VEL) {
      cross3c(r, w, t);
#pragma unroll
      for (int a = 0; a < 3; ++a) t[a] = v[a] - t[a];
    }
    cross3c(r, aw, t2);
#pragma unroll
    for (int a = 0; a < 3; ++a) t2[a] = av[a] - t2[a];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      if constexpr (VEL) {
        nw[a] = E[a * 3] * w[0] + E[a * 3 + 1] * w[1] + E[a * 3 + 2] * w[2];
        nv[a] = E[a * 3] * t[0] + E[a * 3 + 1] * t[1] + E[a * 3 + 2] * t[2];
      }
      naw[a] = E[a * 3] * aw[0] + E[a * 3 + 1] * aw[1] + E[a * 3 + 2] * aw[2];
      nav[a] = E[a * 3] * t2[0] + E[a * 3 + 1] * t2[1] + E[a * 3 + 2] * t2[2];
    }
    if constexpr (VEL) {
      // v_i = X v_p + z qd_i ; a_i = X a_p + z qdd_i + v_i x_m (z qd_i)
      nw[2] = nw[2] + qd[i];
      // (w x z qd, v x z qd) with z = e_3
      naw[0] = naw[0] + nw[1] * qd[i];
      naw[1] = naw[1] - nw[0] * qd[i];
      nav[0] = nav[0] + nv[1] * qd[i];
      nav[1] = nav[1] - nv[0] * qd[i];
    }
    naw[2] = naw[2] + qdd[i];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      if constexpr (VEL) { w[a] = nw[a]; v[a] = nv[a]; }
      aw[a] = naw[a]; av[a] = nav[a];
    }
    // f_i = I a_i + v_i x_f (I v_i);  I (w, v) = (Io w + mc x v, m v - mc x w)
    const double m = UR5_M[i];
    const double mc[3] = {UR5_MC[3 * i], UR5_MC[3 * i + 1], UR5_MC[3 * i + 2]};
    T x1[3], x2[3];
    cross3c(mc, av, x1);
    cross3c(mc, aw, x2);
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      fn[i][a] = UR5_IO[9 * i + a * 3] * aw[0] + UR5_IO[9 * i + a * 3 + 1] * aw[1] + UR5_IO[9 * i + a * 3 + 2] * aw[2] +
                 x1[a];
      ff[i][a] = m * av[a] - x2[a];
    }
    if constexpr (VEL) {
      T hA[3], hL[3], y1[3], y2[3], y3[3];
      cross3c(mc, v, x1);
      cross3c(mc, w, x2);
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        hA[a] = UR5_IO[9 * i + a * 3] * w[0] + UR5_IO[9 * i + a * 3 + 1] * w[1] + UR5_IO[9 * i + a * 3 + 2] * w[2] + x1[a];
        hL[a] = m * v[a] - x2[a];
      }
      cross3(w, hA, y1);
      cross3(v, hL, y2);
      cross3(w, hL, y3);
#pragma unroll
      for (int a = 0; a < 3; ++a) { fn[i][a] = fn[i][a] + y1[a] + y2[a]; ff[i][a] = ff[i][a] + y3[a]; }
    }
  }
#pragma unroll
  for (int i = 3; i >= 0; --i) {
    tau[i] = fn[i][2];
    if (i == 0) break;
    T E[9];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      E[0 * 3 + k] = cs[i] * UR5_R[9 * i + k * 3 + 0] + sn[i] * UR5_R[9 * i + k * 3 + 1];
      E[1 * 3 + k] = cs[i] * UR5_R[9 * i + k * 3 + 1] - sn[i] * UR5_R[9 * i + k * 3 + 0];
      E[2 * 3 + k] = z + UR5_R[9 * i + k * 3 + 2];
    }
    const double r[3] = {UR5_P[3 * i], UR5_P[3 * i + 1], UR5_P[3 * i + 2]};
    T en[3], ef[3], x[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      en[a] = E[a] * fn[i][0] + E[3 + a] * fn[i][1] + E[6 + a] * fn[i][2];
      ef[a] = E[a] * ff[i][0] + E[3 + a] * ff[i][1] + E[6 + a] * ff[i][2];
    }
    cross3c(r, ef, x);
#pragma unroll
    for (int a = 0; a < 3; ++a) { fn[i - 1][a] = fn[i - 1][a] + en[a] + x[a]; ff[i - 1][a] = ff[i - 1][a] + ef[a]; }
  }
}

// Cholesky factor of M(q) (columns M e_c = RNEA(q, 0, e_c) without gravity) and acc = M^-1 (u - RNEA(q, qd, 0))
__device__ __forceinline__ void ur5_point(const double* q, const double* qd, const double* u, double (&L)[16],
                                          double (&acc)[4]) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    double e[4] = {0.0, 0.0, 0.0, 0.0}, col[4];
    e[c] = 1.0;
    ur5_rnea<double, false, false>(q, q, e, col);
#pragma unroll
    for (int j = 0; j < 4; ++j) L[j * 4 + c] = col[j];
  }
  const double zq[4] = {0.0, 0.0, 0.0, 0.0};
  double b[4];
  ur5_rnea<double, true, true>(q, qd, zq, b);
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = u[j] - b[j];
  chol<4>(L);
  chol_solve<4>(L, acc);
}

// d acc along (dq, dqd, du) at a point with factor L and accelerations acc
__device__ __forceinline__ void ur5_jvp(const double* q, const double* qd, const double (&L)[16], const double* acc,
                                        const double* dq, const double* dqd, const double* du, double* dacc) {
  Dl Q[4], V[4], tau[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) { Q[j] = Dl{q[j], dq[j]}; V[j] = Dl{qd[j], dqd[j]}; }
  ur5_rnea<Dl, true, true>(Q, V, acc, tau);
  double r[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) r[j] = du[j] - tau[j].d;
  chol_solve<4>(L, r);
#pragma unroll
  for (int j = 0; j < 4; ++j) dacc[j] = r[j];
}

// acc = f(th, om, u); if JAC also Jth, Jom, Ju (row-major NQ x NQ).
template <int NQ, bool JAC>
__device__ __forceinline__ void model_eval(const double* th, const double* om, const double* u, double* acc,
                                           double* Jth, double* Jom, double* Ju) {
  if constexpr (NQ == 4) {
    double L[16], a[4];
    ur5_point(th, om, u, L, a);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = a[j];
    if constexpr (JAC) {
#pragma unroll
      for (int c = 0; c < 12; ++c) {
        double dq[4], dv[4], du[4], da[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) { dq[j] = (c == j) ? 1.0 : 0.0; dv[j] = (c == 4 + j) ? 1.0 : 0.0; du[j] = (c == 8 + j) ? 1.0 : 0.0; }
        ur5_jvp(th, om, L, a, dq, dv, du, da);
        double* J = c < 4 ? Jth : (c < 8 ? Jom : Ju);
#pragma unroll
        for (int j = 0; j < 4; ++j) J[j * 4 + (c & 3)] = da[j];
      }
    }
  } else if constexpr (NQ == 1) {
    constexpr double pm = 0.5, pd = 0.3, pb = 0.01, g = 9.81;
    constexpr double inv = 1.0 / (pd * pd * pm);
    double sn, cs;
    sincos(th[0], &sn, &cs);
    acc[0] = (pm * g * pd * sn + u[0] - pb * om[0]) * inv;
    if constexpr (JAC) {
      Jth[0] = pm * g * pd * cs * inv;
      Jom[0] = -pb * inv;
      Ju[0] = inv;
    }
  } else {
    using C = Chain<NQ>;
    double S[NQ][NQ], Cc[NQ][NQ], M[NQ * NQ], r[NQ], sth[NQ], cth[NQ];
#pragma unroll
    for (int j = 0; j < NQ; ++j) sincos(th[j], &sth[j], &cth[j]);
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      S[j][j] = 0.0;
      Cc[j][j] = 1.0;
#pragma unroll
      for (int k = 0; k < j; ++k) {
        // sin/cos of differences from the per-angle values (angle-difference identities)
        const double s = sth[j] * cth[k] - cth[j] * sth[k];
        const double c = cth[j] * cth[k] + sth[j] * sth[k];
        S[j][k] = s; S[k][j] = -s;
        Cc[j][k] = c; Cc[k][j] = c;
      }
    }
#pragma unroll
    for (int j = 0; j < NQ; ++j)
#pragma unroll
      for (int k = 0; k < NQ; ++k) M[j * NQ + k] = C::a(j, k) * Cc[j][k];
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      double cor = 0.0;
#pragma unroll
      for (int k = 0; k < NQ; ++k) cor += C::a(j, k) * S[j][k] * om[k] * om[k];
      r[j] = u[j] - cor - C::g * C::mu(j) * C::l * sth[j];
    }
    chol<NQ>(M);
    double a_[NQ];
#pragma unroll
    for (int j = 0; j < NQ; ++j) a_[j] = r[j];
    chol_solve<NQ>(M, a_);
#pragma unroll
    for (int j = 0; j < NQ; ++j) acc[j] = a_[j];
    if constexpr (JAC) {
#pragma unroll
      for (int c = 0; c < NQ; ++c) {
        double col[NQ], co[NQ], e[NQ];
#pragma unroll
        for (int j = 0; j < NQ; ++j) {
          if (j == c) {
            double diag = 0.0;
#pragma unroll
            for (int k = 0; k < NQ; ++k)
              if (k != j) diag += C::a(j, k) * (Cc[j][k] * om[k] * om[k] - S[j][k] * a_[k]);
            col[j] = -diag - C::g * C::mu(j) * C::l * cth[j];
          } else {
            col[j] = C::a(j, c) * (Cc[j][c] * om[c] * om[c] - S[j][c] * a_[c]);
          }
          co[j] = -2.0 * C::a(j, c) * S[j][c] * om[c];
          e[j] = (j == c) ? 1.0 : 0.0;
        }
        chol_solve<NQ>(M, col);
        chol_solve<NQ>(M, co);
        chol_solve<NQ>(M, e);
#pragma unroll
        for (int j = 0; j < NQ; ++j) {
          Jth[j * NQ + c] = col[j];
          Jom[j * NQ + c] = co[j];
          Ju[j * NQ + c] = e[j];
        }
      }
    }
  }
}

template <int NQ>
__device__ __forceinline__ void rhs(const double* x, const double* u, double* k) {
#pragma unroll
  for (int j = 0; j < NQ; ++j) k[j] = x[NQ + j];
  model_eval<NQ, false>(x, x + NQ, u, k + NQ, nullptr, nullptr, nullptr);
}

// One classical RK4 step of length h.
template <int NQ>
__device__ __forceinline__ void rk4(double h, const double* x, const double* u, double* x1) {
  constexpr int NX = 2 * NQ;
  double k[NX], X[NX], acc[NX];
  rhs<NQ>(x, u, k);
#pragma unroll
  for (int i = 0; i < NX; ++i) { acc[i] = k[i]; X[i] = x[i] + 0.5 * h * k[i]; }
  rhs<NQ>(X, u, k);
#pragma unroll
  for (int i = 0; i < NX; ++i) { acc[i] += 2.0 * k[i]; X[i] = x[i] + 0.5 * h * k[i]; }
  rhs<NQ>(X, u, k);
#pragma unroll
  for (int i = 0; i < NX; ++i) { acc[i] += 2.0 * k[i]; X[i] = x[i] + h * k[i]; }
  rhs<NQ>(X, u, k);
#pragma unroll
  for (int i = 0; i < NX; ++i) x1[i] = x[i] + h / 6.0 * (acc[i] + k[i]);
}

// Nominal model quantities at one point, reused by Jacobian-vector products (JVP) along
// tangent directions: the sensitivities never form the Jacobian (lower register pressure).
template <int NQ>
struct ModelPoint {
  double L[NQ * NQ];       // Cholesky factor of M(theta) (chain) / unused (pendulum)
  double sd[NQ][NQ];       // sin(th_j - th_k)
  double cd[NQ][NQ];       // cos(th_j - th_k)
  double cth[NQ];          // cos th_j
  double acc[NQ], om[NQ];
  double th[NQ];           // angles (UR5: the JVP re-runs RNEA at the point)
};

template <int NQ>
__device__ __forceinline__ void model_point(const double* th, const double* om, const double* u, ModelPoint<NQ>& mp) {
  if constexpr (NQ == 4) {
#pragma unroll
    for (int j = 0; j < 4; ++j) { mp.th[j] = th[j]; mp.om[j] = om[j]; }
    ur5_point(th, om, u, mp.L, mp.acc);
  } else if constexpr (NQ == 1) {
    constexpr double pm = 0.5, pd = 0.3, pb = 0.01, g = 9.81;
    constexpr double inv = 1.0 / (pd * pd * pm);
    double sn, cs;
    sincos(th[0], &sn, &cs);
    mp.cth[0] = cs;
    mp.om[0] = om[0];
    mp.acc[0] = (pm * g * pd * sn + u[0] - pb * om[0]) * inv;
  } else {
    using C = Chain<NQ>;
    double sth[NQ];
#pragma unroll
    for (int j = 0; j < NQ; ++j) { sincos(th[j], &sth[j], &mp.cth[j]); mp.om[j] = om[j]; }
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      mp.sd[j][j] = 0.0;
      mp.cd[j][j] = 1.0;
#pragma unroll
      for (int k = 0; k < j; ++k) {
        const double sv = sth[j] * mp.cth[k] - mp.cth[j] * sth[k];
        const double cv = mp.cth[j] * mp.cth[k] + sth[j] * sth[k];
        mp.sd[j][k] = sv; mp.sd[k][j] = -sv;
        mp.cd[j][k] = cv; mp.cd[k][j] = cv;
      }
    }
#pragma unroll
    for (int j = 0; j < NQ; ++j)
#pragma unroll
      for (int k = 0; k < NQ; ++k) mp.L[j * NQ + k] = C::a(j, k) * mp.cd[j][k];
    chol<NQ>(mp.L);
    double r[NQ];
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      double cor = 0.0;
#pragma unroll
      for (int k = 0; k < NQ; ++k) cor += C::a(j, k) * mp.sd[j][k] * om[k] * om[k];
      r[j] = u[j] - cor - C::g * C::mu(j) * C::l * sth[j];
    }
    chol_solve<NQ>(mp.L, r);
#pragma unroll
    for (int j = 0; j < NQ; ++j) mp.acc[j] = r[j];
  }
}

// d acc along (dth, dom, du):  M^-1 (du - dcor - dgrav - dM acc)
template <int NQ>
__device__ __forceinline__ void model_jvp(const ModelPoint<NQ>& mp, const double* dth, const double* dom,
                                          const double* du, double* dacc) {
  if constexpr (NQ == 4) {
    ur5_jvp(mp.th, mp.om, mp.L, mp.acc, dth, dom, du, dacc);
  } else if constexpr (NQ == 1) {
    constexpr double pm = 0.5, pd = 0.3, pb = 0.01, g = 9.81;
    constexpr double inv = 1.0 / (pd * pd * pm);
    dacc[0] = (pm * g * pd * mp.cth[0] * dth[0] + du[0] - pb * dom[0]) * inv;
  } else {
    using C = Chain<NQ>;
    double r[NQ];
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      double t = du[j] - C::g * C::mu(j) * C::l * mp.cth[j] * dth[j];
#pragma unroll
      for (int k = 0; k < NQ; ++k) {
        if (k == j) continue;
        const double dd = dth[j] - dth[k];
        t -= C::a(j, k) * (mp.cd[j][k] * dd * mp.om[k] * mp.om[k] + 2.0 * mp.sd[j][k] * mp.om[k] * dom[k]);
        t += C::a(j, k) * mp.sd[j][k] * dd * mp.acc[k];
      }
      r[j] = t;
    }
    chol_solve<NQ>(mp.L, r);
#pragma unroll
    for (int j = 0; j < NQ; ++j) dacc[j] = r[j];
  }
}

// RK4 step with forward sensitivities = exact derivative of the discrete map (ACADOS ERK
// forward VDE).  The NX + NU sensitivity columns are propagated as Jacobian-vector products in
// groups of G tangent directions; each group re-runs the nominal stages (more arithmetic, far
// fewer live registers - the sweep is latency-bound, not FLOP-bound).  Outputs x1 (NX);
// sensitivity entry (i, c), c < NX for A = dx1/dx, c >= NX for B = dx1/du -> store(i, c, v).
template <int NQ, int G, class Store>
__device__ __forceinline__ void rk4_sens_g(double h, const double* x, const double* u, double* x1, Store store) {
  constexpr int NX = 2 * NQ, NC = NX + NQ, NG = NC / G;
  static_assert(NC % G == 0, "group size must divide the column count");
#pragma unroll 1
  for (int grp = 0; grp < NG; ++grp) {
    const int c0 = grp * G;
    double T[NX][G], Ts[NX][G], X[NX], ks[NX];
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      X[i] = x[i];
      ks[i] = 0.0;
#pragma unroll
      for (int c = 0; c < G; ++c) {
        T[i][c] = (i == c0 + c) ? 1.0 : 0.0;
        Ts[i][c] = 0.0;
      }
    }
    // stages not unrolled: one ModelPoint live at a time (bounds register pressure; the
    // linearisation is ~1% of the solve)
#pragma unroll 1
    for (int st = 0; st < 4; ++st) {
      const double wgt = (st == 0 || st == 3) ? 1.0 : 2.0;
      const double cnext = (st < 2) ? 0.5 * h : h;
      ModelPoint<NQ> mp;
      model_point<NQ>(X, X + NQ, u, mp);
      double k[NX];
#pragma unroll
      for (int j = 0; j < NQ; ++j) { k[j] = X[NQ + j]; k[NQ + j] = mp.acc[j]; }
      double dk[NX][G];
#pragma unroll
      for (int c = 0; c < G; ++c) {
        double dth[NQ], dom[NQ], du[NQ], da[NQ];
#pragma unroll
        for (int j = 0; j < NQ; ++j) {
          dth[j] = T[j][c];
          dom[j] = T[NQ + j][c];
          du[j] = (c0 + c == NX + j) ? 1.0 : 0.0;
        }
        model_jvp<NQ>(mp, dth, dom, du, da);
#pragma unroll
        for (int j = 0; j < NQ; ++j) { dk[j][c] = dom[j]; dk[NQ + j][c] = da[j]; }
      }
#pragma unroll
      for (int i = 0; i < NX; ++i) {
        ks[i] += wgt * k[i];
#pragma unroll
        for (int c = 0; c < G; ++c) Ts[i][c] += wgt * dk[i][c];
      }
      if (st < 3) {
#pragma unroll
        for (int i = 0; i < NX; ++i) {
          X[i] = x[i] + cnext * k[i];
#pragma unroll
          for (int c = 0; c < G; ++c) T[i][c] = ((i == c0 + c) ? 1.0 : 0.0) + cnext * dk[i][c];
        }
      }
    }
    if (grp == 0) {
#pragma unroll
      for (int i = 0; i < NX; ++i) x1[i] = x[i] + h / 6.0 * ks[i];
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) {
#pragma unroll
      for (int c = 0; c < G; ++c) store(i, c0 + c, ((i == c0 + c) ? 1.0 : 0.0) + h / 6.0 * Ts[i][c]);
    }
  }
}

template <int NQ, class Store>
__device__ __forceinline__ void rk4_sens(double h, const double* x, const double* u, double* x1, Store store) {
  rk4_sens_g<NQ, VBOC_SENS_GROUP, Store>(h, x, u, x1, store);
}

}  // namespace vboc

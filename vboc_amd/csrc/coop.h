// coop.h - cooperative tail solver: ONE boundary OCP per wave, every stage array resident in LDS.
//
// Why: the lane-per-problem kernels (vboc_solver.hip) are bandwidth-efficient while tens of
// thousands of problems are resident, but the SQP iteration count has a long tail (a few percent of
// the problems take 300-1000 iterations).  Once only those remain, a lane-mode sweep is a serial
// chain of ~100 stage bodies of ~4k instructions each on an almost empty GPU, so one SQP iteration
// costs ~100 ms.  Here the 64 lanes of a wave cooperate on one problem instead:
//   * stage-parallel passes (linearisation + sensitivities, residuals, IPM initial point,
//     Hessian/gradient preparation, step-length tests, iterate update, merit re-simulation,
//     weights, step application): lane j owns stages j, j+64, ...;
//   * the Riccati factorisation recursion: per stage three "dot-product steps" in which every lane
//     computes one entry of P A, P B, A'PA, B'PB, B'PA, B'Pi, A'Pi+K'Y, ... from operands in LDS
//     (per-lane descriptor tables, so the 64 lanes run ONE instruction stream - no divergence),
//     plus one step where all lanes factorise Ru redundantly and lanes solve one column each;
//   * the vector, forward and costate recursions in closed-loop form, A_cl = A + B K, one short
//     dependent step per stage on NX lanes.
// The arithmetic is the algorithm of Lane<NQ> / oracle/vboc_oracle.c (same formulas, same
// decisions); only summation orders differ (rounding-level).
//
// LDS layout (doubles): stage record k at [k * REC, (k + 1) * REC), then a fixed region.
#pragma once

namespace vboc {

template <int NQ>
struct CoopLayout {
  static constexpr int NX = 2 * NQ, NU = NQ, NZ = 3 * NQ, M0 = NQ + 1;
  // stage record: A, B, z (current iterate), dz, lambda_l, lambda_u, e (defect -> initial residual),
  // K, k_f, chol(Ru), M, Y, P e, D (H / g_corr / corrector direction), DA (g_pred / affine
  // direction / costate), V (v = P e + p of the vector pass)
  static constexpr int OA = 0, OB = OA + NX * NX, OZ = OB + NX * NU, ODZ = OZ + NZ, OQL = ODZ + NZ, OQU = OQL + NZ,
                       OE = OQU + NZ, OK = OE + NX, OKF = OK + NU * NX, OLR = OKF + NU, OM = OLR + NU * NU,
                       OY = OM + NU * NQ, OPE = OY + NU * NQ, OD = OPE + NX, ODA = OD + NZ, OV = ODA + NZ,
                       REC = (OV + NX) | 1;
  // fixed region: stage-0 blocks, recursion scratch, constants, parameters
  static constexpr int F0 = 0, LR0 = F0 + NX * M0, MM0 = LR0 + M0 * M0, Y0 = MM0 + M0 * NQ, PE0 = Y0 + M0 * NQ,
                       P = PE0 + NX, PA = P + NX * NX, PB = PA + NX * NX, APA = PB + NX * NU, RU = APA + NX * NX,
                       S = RU + NU * NU, PI = S + NU * NX, PV = PI + NX * NQ, SC = PV + 2 * NX, LINE = SC + NQ * NQ,
                       ZERO = LINE + NQ, TRASH = ZERO + 16, PAR = TRASH + 64, FIXN = PAR + Par<NQ>::COUNT;
  static_assert(M0 * NX <= NX * NX, "stage-0 B'P reuses the PA scratch");
  static constexpr size_t lds_bytes(int nmax) { return ((size_t)REC * (nmax + 1) + FIXN) * sizeof(double); }
};

// one output of a recursion step:  out = s[ini] + sg * sum_q s[x1+q*sx1] s[y1+q*sy1]
//                                               +      sum_q s[x2+q*sx2] s[y2+q*sy2];  s[d1] = s[d2] = out
// `rel` marks operands inside the current stage record (offset by k * REC at run time).
struct Dsc {
  int x1, sx1, y1, sy1, x2, sx2, y2, sy2, ini, d1, d2;
  unsigned rel;
  double sg;
};
enum : unsigned { RX1 = 1, RY1 = 2, RX2 = 4, RY2 = 8, RINI = 16, RD1 = 32, RD2 = 64 };

__device__ __forceinline__ double uni(double v) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)b);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ double wsum(double v) {
  UNR for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
  return uni(v);
}
__device__ __forceinline__ double wmaxd(double v) {
  UNR for (int off = 32; off >= 1; off >>= 1) v = fmax(v, __shfl_xor(v, off));
  return uni(v);
}
__device__ __forceinline__ double wmind(double v) {
  UNR for (int off = 32; off >= 1; off >>= 1) v = fmin(v, __shfl_xor(v, off));
  return uni(v);
}
// Cholesky for the recursion's critical path: pivots from rsq + two Newton steps give both
// d = sqrt(s) and 1/d without a division; solves multiply by the inverse diagonal.  Same
// factorisation and failure test (s > 0) as chol<n> (model.h), rounding-level different.
template <int n>
__device__ __forceinline__ bool chol_inv(double (&A)[n * n], double (&id)[n]) {
  bool ok = true;
  UNR for (int j = 0; j < n; ++j) {
    double sj = A[j * n + j];
    UNR for (int k = 0; k < j; ++k) sj -= A[j * n + k] * A[j * n + k];
    ok = ok && (sj > 0.0);
    const double x = sj > 0.0 ? sj : 1.0;
    double r = __builtin_amdgcn_rsq(x);
    UNR for (int it = 0; it < 2; ++it) {
      const double e = fma(-(0.5 * x) * r, r, 0.5);
      r = fma(r, e, r);
    }
    A[j * n + j] = x * r;
    id[j] = r;
    UNR for (int i = j + 1; i < n; ++i) {
      double tt = A[i * n + j];
      UNR for (int k = 0; k < j; ++k) tt -= A[i * n + k] * A[j * n + k];
      A[i * n + j] = tt * r;
    }
  }
  return ok;
}
template <int n>
__device__ __forceinline__ void solve_inv(const double (&L)[n * n], const double (&id)[n], double (&b)[n]) {
  UNR for (int i = 0; i < n; ++i) {
    double tt = b[i];
    UNR for (int k = 0; k < i; ++k) tt -= L[i * n + k] * b[k];
    b[i] = tt * id[i];
  }
  UNR for (int i = n - 1; i >= 0; --i) {
    double tt = b[i];
    UNR for (int k = i + 1; k < n; ++k) tt -= L[k * n + i] * b[k];
    b[i] = tt * id[i];
  }
}

// lower-triangle enumeration u -> (i, j), j <= i
__device__ __forceinline__ void tri(int u, int& i, int& j) {
  i = 0;
  while ((i + 1) * (i + 2) / 2 <= u) ++i;
  j = u - i * (i + 1) / 2;
}

#ifdef VBOC_COOP_PROF
#define CPROF_DECL unsigned long long cp_[12] = {0}; unsigned long long cp_t = clock64();
#define CPROF(i) { __syncthreads(); const unsigned long long n_ = clock64(); cp_[i] += n_ - cp_t; cp_t = n_; }
#else
#define CPROF_DECL
#define CPROF(i)
#endif

template <int NQ>
struct Coop {
  using CL = CoopLayout<NQ>;
  using PF = Par<NQ>;
  static constexpr int NX = 2 * NQ, NU = NQ, NZ = 3 * NQ, M0 = NQ + 1, REC = CL::REC;
  static constexpr int OA = CL::OA, OB = CL::OB, OZ = CL::OZ, ODZ = CL::ODZ, OQL = CL::OQL, OQU = CL::OQU,
                       OE = CL::OE, OK = CL::OK, OKF = CL::OKF, OLR = CL::OLR, OM = CL::OM, OY = CL::OY,
                       OPE = CL::OPE, OD = CL::OD, ODA = CL::ODA, OV = CL::OV;

  double* s;      // LDS
  const int fx;   // fixed-region base
  const Work& w;
  const Opts& o;
  Lane<NQ> G;     // this problem's slot in the tiled global arrays (X, U, PI, LL, LU, WPI, PAR)
  const int t;    // lane
  int N;
  double rs, rd0, e00, mu, nbox;   // interior-point scalars (wave-uniform)

  __device__ Coop(double* s_, int fx_, const Work& w_, const Opts& o_, unsigned slot, int t_)
      : s(s_), fx(fx_), w(w_), o(o_), G(w_, o_, slot), t(t_), N(0) {}

  __device__ __forceinline__ double& st(int k, int off) const { return s[k * REC + off]; }
  __device__ __forceinline__ double& fv(int off) const { return s[fx + off]; }
  __device__ __forceinline__ double& par(int f) const { return s[fx + CL::PAR + f]; }

  // box of component i of stage k (the Lane::stage_box pattern)
  __device__ __forceinline__ bool box(int k, int i, double& lb, double& ub) const {
    lb = -1.0; ub = 1.0;
    if (k == 0) {
      if (i == 0) { lb = par(PF::SLB); ub = par(PF::SUB); return true; }
      if (i < M0) { lb = par(PF::ULB + i - 1); ub = par(PF::UUB + i - 1); return true; }
      return false;
    }
    if (k == N) {
      if (i < NQ) { lb = par(PF::QNLB + i); ub = par(PF::QNUB + i); return true; }
      return false;
    }
    if (i < NX) { lb = par(PF::XLB + i); ub = par(PF::XUB + i); }
    else { lb = par(PF::ULB + i - NX); ub = par(PF::UUB + i - NX); }
    return true;
  }
  __device__ __forceinline__ double dz_init(double lb, double ub, double z) const {
    const double L = lb - z, U = ub - z, del = o.push * (U - L);
    return fmin(fmax(0.0, L + del), U - del);
  }
  __device__ __forceinline__ double cgrad(int k, int i) const { return (k == 0 && i == 0) ? par(PF::CS) : 0.0; }

  struct CS { double tl, tu, itl, itu, ql, qu, dz; bool bx; };
  __device__ __forceinline__ CS comp(int k, int i) const {
    CS c;
    double lb, ub;
    c.bx = box(k, i, lb, ub);
    const double z = st(k, OZ + i);
    c.dz = st(k, ODZ + i); c.ql = st(k, OQL + i); c.qu = st(k, OQU + i);
    c.tl = c.dz - (lb - z); c.tu = (ub - z) - c.dz;
    c.itl = c.bx ? 1.0 / c.tl : 0.0;
    c.itu = c.bx ? 1.0 / c.tu : 0.0;
    return c;
  }
  __device__ __forceinline__ static void corr_rhs(const CS& c, double da, double smu, double& rl, double& ru) {
    const double dlla = -c.ql - c.ql * da * c.itl, dlua = -c.qu + c.qu * da * c.itu;
    rl = smu - c.tl * c.ql - da * dlla;
    ru = smu - c.tu * c.qu + da * dlua;
  }

  // ---------------------------------------------------------------------------------------------
  // recursion-step machinery
  // ---------------------------------------------------------------------------------------------
  __device__ __forceinline__ void dnull(Dsc& d) const {
    d.x1 = d.y1 = d.x2 = d.y2 = d.ini = fx + CL::ZERO;
    d.sx1 = d.sy1 = d.sx2 = d.sy2 = 0;
    d.d1 = d.d2 = fx + CL::TRASH + t;
    d.rel = 0;
    d.sg = 1.0;
  }
  template <int L1, int L2>
  __device__ __forceinline__ void dstep(const Dsc& d, int kb) const {
    auto ad = [&](int a, unsigned bit) { return a + ((d.rel & bit) ? kb : 0); };
    const int x1 = ad(d.x1, RX1), y1 = ad(d.y1, RY1), x2 = ad(d.x2, RX2), y2 = ad(d.y2, RY2);
    // every operand load issued before any arithmetic: one LDS round trip per step
    double a1[L1 > 0 ? L1 : 1], b1[L1 > 0 ? L1 : 1], a2[L2 > 0 ? L2 : 1], b2[L2 > 0 ? L2 : 1];
    UNR for (int q = 0; q < L1; ++q) { a1[q] = s[x1 + q * d.sx1]; b1[q] = s[y1 + q * d.sy1]; }
    UNR for (int q = 0; q < L2; ++q) { a2[q] = s[x2 + q * d.sx2]; b2[q] = s[y2 + q * d.sy2]; }
    const double r0 = s[ad(d.ini, RINI)];
    __builtin_amdgcn_sched_barrier(0);
    double s1 = 0.0, s2 = 0.0;
    UNR for (int q = 0; q < L1; ++q) s1 += a1[q] * b1[q];
    UNR for (int q = 0; q < L2; ++q) s2 += a2[q] * b2[q];
    const double r = r0 + d.sg * s1 + s2;
    __syncthreads();
    s[ad(d.d1, RD1)] = r;
    s[ad(d.d2, RD2)] = r;
    __syncthreads();
  }
  // all lanes: L = chol(s[ru..]); lane-specific column solve rhs -> sgn * Ru^-1 rhs; lane 0 stores L
  template <int n>
  __device__ __forceinline__ bool sstep(int ru, int ldst, int rb, int rstr, int db, int dstr, double sgn) const {
    double L[n * n], id[n], b[n];
    UNR for (int a = 0; a < n; ++a) b[a] = s[rb + a * rstr];
    UNR for (int e = 0; e < n * n; ++e) L[e] = s[ru + e];
    const bool ok = chol_inv<n>(L, id);
    solve_inv<n>(L, id, b);
    __syncthreads();
    UNR for (int a = 0; a < n; ++a) s[db + a * dstr] = sgn * b[a];
    if (t == 0) {
      UNR for (int e = 0; e < n * n; ++e) s[ldst + e] = L[e];
    }
    __syncthreads();
    return ok;
  }

  // descriptors of the middle-stage factorisation steps (rs enters through sg)
  __device__ void desc_mid(Dsc& d1, Dsc& d2, Dsc& d4) const {
    const int P = fx + CL::P, PA = fx + CL::PA, PB = fx + CL::PB, APA = fx + CL::APA, RU = fx + CL::RU,
              S = fx + CL::S, PI = fx + CL::PI, SC = fx + CL::SC, LINE = fx + CL::LINE;
    constexpr int TX = NX * (NX + 1) / 2, TU = NU * (NU + 1) / 2;
    dnull(d1); dnull(d2); dnull(d4);
    // step 1: PA = P A, PB = P B, P e (-> stage PE), lin_e += Pi' e
    int u = t;
    if (u < NX * NX) {
      const int i = u / NX, j = u % NX;
      d1.x1 = P + i * NX; d1.sx1 = 1; d1.y1 = OA + j; d1.sy1 = NX; d1.rel = RY1; d1.d1 = d1.d2 = PA + u;
    } else if ((u -= NX * NX) < NX * NU) {
      const int i = u / NU, a = u % NU;
      d1.x1 = P + i * NX; d1.sx1 = 1; d1.y1 = OB + a; d1.sy1 = NU; d1.rel = RY1; d1.d1 = d1.d2 = PB + u;
    } else if ((u -= NX * NU) < NX) {
      d1.x1 = P + u * NX; d1.sx1 = 1; d1.y1 = OE; d1.sy1 = 1; d1.sg = rs; d1.d1 = d1.d2 = OPE + u;
      d1.rel = RY1 | RD1 | RD2;
    } else if ((u -= NX) < NQ) {
      d1.x1 = PI + u; d1.sx1 = NQ; d1.y1 = OE; d1.sy1 = 1; d1.sg = rs; d1.ini = d1.d1 = d1.d2 = LINE + u; d1.rel = RY1;
    }
    // step 2: A'PA + diag(Hx), B'PB + diag(Hu), S = B'PA, Y = B'Pi
    u = t;
    if (u < TX) {
      int i, j;
      tri(u, i, j);
      d2.x1 = OA + i; d2.sx1 = NX; d2.y1 = PA + j; d2.sy1 = NX; d2.rel = RX1;
      if (i == j) { d2.ini = OD + i; d2.rel |= RINI; }
      d2.d1 = APA + i * NX + j; d2.d2 = APA + j * NX + i;
    } else if ((u -= TX) < TU) {
      int a, c;
      tri(u, a, c);
      d2.x1 = OB + a; d2.sx1 = NU; d2.y1 = PB + c; d2.sy1 = NU; d2.rel = RX1;
      if (a == c) { d2.ini = OD + NX + a; d2.rel |= RINI; }
      d2.d1 = RU + a * NU + c; d2.d2 = RU + c * NU + a;
    } else if ((u -= TU) < NU * NX) {
      const int a = u / NX, j = u % NX;
      d2.x1 = PB + a; d2.sx1 = NU; d2.y1 = OA + j; d2.sy1 = NX; d2.rel = RY1; d2.d1 = d2.d2 = S + u;
    } else if ((u -= NU * NX) < NU * NQ) {
      const int a = u / NQ, j = u % NQ;
      d2.x1 = OB + a; d2.sx1 = NU; d2.y1 = PI + j; d2.sy1 = NQ; d2.rel = RX1 | RD1 | RD2; d2.d1 = d2.d2 = OY + u;
    }
    // step 4: P <- A'PA + Hx + S'K, Pi <- A'Pi + K'Y, Sc += Y'M
    u = t;
    if (u < TX) {
      int i, j;
      tri(u, i, j);
      d4.x2 = S + i; d4.sx2 = NX; d4.y2 = OK + j; d4.sy2 = NX; d4.rel = RY2;
      d4.ini = APA + i * NX + j; d4.d1 = P + i * NX + j; d4.d2 = P + j * NX + i;
    } else if ((u -= TX) < NX * NQ) {
      const int i = u / NQ, j = u % NQ;
      d4.x1 = OA + i; d4.sx1 = NX; d4.y1 = PI + j; d4.sy1 = NQ;
      d4.x2 = OK + i; d4.sx2 = NX; d4.y2 = OY + j; d4.sy2 = NQ;
      d4.rel = RX1 | RX2 | RY2; d4.d1 = d4.d2 = PI + u;
    } else if ((u -= NX * NQ) < NQ * NQ) {
      const int i = u / NQ, j = u % NQ;
      d4.x2 = OY + i; d4.sx2 = NQ; d4.y2 = OM + j; d4.sy2 = NQ; d4.rel = RX2 | RY2;
      d4.ini = d4.d1 = d4.d2 = SC + u;
    }
  }
  // stage 0 (controls s, u_0; F0 = [A0 g, B0]); the stage-0 record starts at 0, so all absolute
  __device__ void desc_s0(Dsc& z1, Dsc& z2, Dsc& z4) const {
    const int P = fx + CL::P, BP = fx + CL::PA, PI = fx + CL::PI, F0 = fx + CL::F0, Y0 = fx + CL::Y0,
              PE0 = fx + CL::PE0, LINE = fx + CL::LINE, LR0 = fx + CL::LR0, MM0 = fx + CL::MM0, SC = fx + CL::SC;
    constexpr int TM = M0 * (M0 + 1) / 2;
    dnull(z1); dnull(z2); dnull(z4);
    int u = t;
    if (u < M0 * NX) {
      const int a = u / NX, j = u % NX;
      z1.x1 = F0 + a; z1.sx1 = M0; z1.y1 = P + j; z1.sy1 = NX; z1.d1 = z1.d2 = BP + u;
    } else if ((u -= M0 * NX) < M0 * NQ) {
      const int a = u / NQ, j = u % NQ;
      z1.x1 = F0 + a; z1.sx1 = M0; z1.y1 = PI + j; z1.sy1 = NQ; z1.d1 = z1.d2 = Y0 + u;
    } else if ((u -= M0 * NQ) < NX) {
      z1.x1 = P + u * NX; z1.sx1 = 1; z1.y1 = OE; z1.sy1 = 1; z1.sg = rs; z1.d1 = z1.d2 = PE0 + u;
    } else if ((u -= NX) < NQ) {
      z1.x1 = PI + u; z1.sx1 = NQ; z1.y1 = OE; z1.sy1 = 1; z1.sg = rs; z1.ini = z1.d1 = z1.d2 = LINE + u;
    }
    u = t;
    if (u < TM) {
      int a, c;
      tri(u, a, c);
      z2.x1 = BP + a * NX; z2.sx1 = 1; z2.y1 = F0 + c; z2.sy1 = M0;
      if (a == c) z2.ini = OD + a;
      z2.d1 = LR0 + a * M0 + c; z2.d2 = LR0 + c * M0 + a;
    }
    u = t;
    if (u < NQ * NQ) {
      const int i = u / NQ, j = u % NQ;
      z4.x2 = Y0 + i; z4.sx2 = NQ; z4.y2 = MM0 + j; z4.sy2 = NQ; z4.ini = z4.d1 = z4.d2 = SC + u;
    }
  }

  // ---------------------------------------------------------------------------------------------
  // linearisation (stage-parallel): ERK4 + sensitivities, defects, current z, NLP residuals
  // ---------------------------------------------------------------------------------------------
  __device__ void linearize(double& rstat, double& req, double& rineq, double& rcomp) {
    const double h = par(PF::H), sv = par(PF::S);
    double stt = 0.0, eq = 0.0, inq = 0.0, cp = 0.0;
    for (int k = t; k <= N; k += 64) {
      double* rec = &s[k * REC];
      if (k < N) {
        double xk[NX], uk[NU], x1[NX];
        if (k == 0) {
          UNR for (int j = 0; j < NQ; ++j) { xk[j] = par(PF::Q0 + j); xk[NQ + j] = sv * par(PF::DIR + j); }
        } else {
          UNR for (int i = 0; i < NX; ++i) xk[i] = G.atv(w.X, NX, k, i);
        }
        UNR for (int a = 0; a < NU; ++a) uk[a] = G.atv(w.U, NU, k, a);
        rk4_sens<NQ>(h, xk, uk, x1, [&](int i, int c, double v) {
          if (c < NX) rec[OA + i * NX + c] = v;
          else rec[OB + i * NU + (c - NX)] = v;
        });
        UNR for (int i = 0; i < NX; ++i) {
          const double b = x1[i] - G.atv(w.X, NX, k + 1, i);
          rec[OE + i] = b;
          eq = fmax(eq, fabs(b));
        }
        if (k == 0) {
          rec[OZ] = sv;
          UNR for (int a = 0; a < NU; ++a) rec[OZ + 1 + a] = uk[a];
          UNR for (int i = M0; i < NZ; ++i) rec[OZ + i] = 0.0;
        } else {
          UNR for (int i = 0; i < NX; ++i) rec[OZ + i] = xk[i];
          UNR for (int a = 0; a < NU; ++a) rec[OZ + NX + a] = uk[a];
        }
        double pik[NX];
        UNR for (int i = 0; i < NX; ++i) pik[i] = G.atv(w.PI, NX, k, i);
        if (k == 0) {
          double F[NX * M0];
          UNR for (int i = 0; i < NX; ++i) {
            double tt = 0.0;
            UNR for (int j = 0; j < NQ; ++j) tt += rec[OA + i * NX + NQ + j] * par(PF::DIR + j);
            F[i * M0] = tt;
            UNR for (int a = 0; a < NU; ++a) F[i * M0 + 1 + a] = rec[OB + i * NU + a];
          }
          UNR for (int e = 0; e < NX * M0; ++e) fv(CL::F0 + e) = F[e];
          UNR for (int c = 0; c < M0; ++c) {
            double gr = (c == 0 ? par(PF::CS) : 0.0) - G.atv(w.LL, NZ, 0, c) + G.atv(w.LU, NZ, 0, c);
            UNR for (int r = 0; r < NX; ++r) gr += F[r * M0 + c] * pik[r];
            stt = fmax(stt, fabs(gr));
          }
        } else {
          double pprev[NX];
          UNR for (int i = 0; i < NX; ++i) pprev[i] = G.atv(w.PI, NX, k - 1, i);
          UNR for (int c = 0; c < NZ; ++c) {
            double gr = -G.atv(w.LL, NZ, k, c) + G.atv(w.LU, NZ, k, c);
            if (c < NX) {
              UNR for (int r = 0; r < NX; ++r) gr += rec[OA + r * NX + c] * pik[r];
              gr -= pprev[c];
            } else {
              UNR for (int r = 0; r < NX; ++r) gr += rec[OB + r * NU + (c - NX)] * pik[r];
            }
            stt = fmax(stt, fabs(gr));
          }
        }
        UNR for (int c = 0; c < NZ; ++c) {
          double lb, ub;
          if (!box(k, c, lb, ub)) continue;
          const double z = rec[OZ + c], ll = G.atv(w.LL, NZ, k, c), lu = G.atv(w.LU, NZ, k, c);
          inq = fmax(inq, fmax(lb - z, z - ub));
          cp = fmax(cp, fmax(fabs(ll * (z - lb)), fabs(lu * (ub - z))));
        }
      } else {
        UNR for (int i = 0; i < NX; ++i) rec[OZ + i] = G.atv(w.X, NX, N, i);
        UNR for (int i = NX; i < NZ; ++i) rec[OZ + i] = 0.0;
        UNR for (int c = 0; c < NX; ++c) {
          const double z = rec[OZ + c];
          double gr = -G.atv(w.LL, NZ, N, c) + G.atv(w.LU, NZ, N, c) - G.atv(w.PI, NX, N - 1, c);
          if (c >= NQ) {
            gr += par(PF::NU_ + c - NQ);
            eq = fmax(eq, fabs(z - par(PF::VFIN + c - NQ)));
          }
          stt = fmax(stt, fabs(gr));
          if (c < NQ) {
            const double lb = par(PF::QNLB + c), ub = par(PF::QNUB + c);
            const double ll = G.atv(w.LL, NZ, N, c), lu = G.atv(w.LU, NZ, N, c);
            inq = fmax(inq, fmax(lb - z, z - ub));
            cp = fmax(cp, fmax(fabs(ll * (z - lb)), fabs(lu * (ub - z))));
          }
        }
      }
    }
    rstat = wmaxd(stt); req = wmaxd(eq); rineq = wmaxd(inq); rcomp = wmaxd(cp);
    __syncthreads();
  }

  // ---------------------------------------------------------------------------------------------
  // interior-point QP
  // ---------------------------------------------------------------------------------------------
  __device__ void qp_init() {
    double musum = 0.0, nb = 0.0, rd = 0.0, e0 = 0.0;
    for (int k = t; k <= N; k += 64) {
      double* rec = &s[k * REC];
      double dz[NZ];
      UNR for (int i = 0; i < NZ; ++i) {
        double lb, ub, ql = 0.0, qu = 0.0, d0 = 0.0;
        if (box(k, i, lb, ub)) {
          const double z = rec[OZ + i], L = lb - z, U = ub - z;
          d0 = dz_init(lb, ub, z);
          ql = o.mu0 / (d0 - L);
          qu = o.mu0 / (U - d0);
          musum += o.mu0 + o.mu0;
          nb += 2.0;
        }
        dz[i] = d0;
        rec[ODZ + i] = d0; rec[OQL + i] = ql; rec[OQU + i] = qu;
        rd = fmax(rd, fabs(o.lm * d0 + cgrad(k, i) - ql + qu));
      }
      if (k < N) {
        const double* rn = &s[(k + 1) * REC];
        UNR for (int i = 0; i < NX; ++i) {
          double lb, ub, dn = 0.0;
          if (box(k + 1, i, lb, ub)) dn = dz_init(lb, ub, rn[OZ + i]);
          double tt = rec[OE + i] - dn;
          if (k == 0) {
            UNR for (int a = 0; a < M0; ++a) tt += fv(CL::F0 + i * M0 + a) * dz[a];
          } else {
            UNR for (int q = 0; q < NX; ++q) tt += rec[OA + i * NX + q] * dz[q];
            UNR for (int a = 0; a < NU; ++a) tt += rec[OB + i * NU + a] * dz[NX + a];
          }
          rec[OE + i] = tt;
          e0 = fmax(e0, fabs(tt));
        }
      } else {
        UNR for (int j = 0; j < NQ; ++j) {
          const double e = par(PF::VFIN + j) - rec[OZ + NQ + j] - dz[NQ + j];
          par(PF::E0N + j) = e;
          e0 = fmax(e0, fabs(e));
          par(PF::QNU + j) = 0.0;
        }
      }
    }
    nbox = wsum(nb);
    mu = wsum(musum) / nbox;
    rd0 = wmaxd(rd);
    e00 = wmaxd(e0);
    rs = 1.0;
    __syncthreads();
  }

  __device__ int qp_check() const {
    if (!isfinite(mu)) return -1;
    if (mu < o.qp_tol_comp && rs * rd0 < o.qp_tol_stat && rs * e00 < o.qp_tol_eq) return 0;
    return 1;
  }

  // H -> D slot, predictor gradient -> DA slot
  __device__ void prep_pred() {
    for (int k = t; k <= N; k += 64) {
      UNR for (int i = 0; i < NZ; ++i) {
        const CS c = comp(k, i);
        st(k, OD + i) = o.lm + (c.bx ? c.ql * c.itl + c.qu * c.itu : 0.0);
        st(k, ODA + i) = o.lm * c.dz + cgrad(k, i);
      }
    }
    __syncthreads();
  }
  // corrector gradient (uses the affine direction in DA) -> D slot
  __device__ void prep_corr(double smu) {
    for (int k = t; k <= N; k += 64) {
      UNR for (int i = 0; i < NZ; ++i) {
        const CS c = comp(k, i);
        double g = o.lm * c.dz + cgrad(k, i);
        if (c.bx) {
          double rl, ru;
          corr_rhs(c, st(k, ODA + i), smu, rl, ru);
          g += -c.ql - rl * c.itl + c.qu + ru * c.itu;
        }
        st(k, OD + i) = g;
      }
    }
    __syncthreads();
  }

  // Riccati factorisation (matrix part) of stages N-1..0; the vector part is vec()
  __device__ bool factor() {
    for (int e = t; e < NX * NX; e += 64) {
      const int i = e / NX, j = e % NX;
      fv(CL::P + e) = (i == j) ? st(N, OD + i) : 0.0;
    }
    for (int e = t; e < NX * NQ; e += 64) {
      const int i = e / NQ, j = e % NQ;
      fv(CL::PI + e) = (i == NQ + j) ? 1.0 : 0.0;
    }
    for (int e = t; e < NQ * NQ; e += 64) fv(CL::SC + e) = 0.0;
    if (t < NQ) fv(CL::LINE + t) = 0.0;
    __syncthreads();
    bool ok = true;
    {
      Dsc d1, d2, d4;
      desc_mid(d1, d2, d4);
      const int Z = fx + CL::ZERO, TR = fx + CL::TRASH + t;
      for (int k = N - 1; k >= 1; --k) {
        const int kb = k * REC;
        dstep<NX, 0>(d1, kb);
        dstep<NX, 0>(d2, kb);
        int rb = Z, rstr = 0, db = TR, dstr = 0;
        double sgn = 1.0;
        if (t < NX) { rb = fx + CL::S + t; rstr = NX; db = kb + OK + t; dstr = NX; sgn = -1.0; }
        else if (t < NX + NQ) { rb = kb + OY + (t - NX); rstr = NQ; db = kb + OM + (t - NX); dstr = NQ; }
        const bool okk = sstep<NU>(fx + CL::RU, kb + OLR, rb, rstr, db, dstr, sgn);
        ok = ok && okk;
        dstep<NX, NU>(d4, kb);
      }
    }
    {
      Dsc z1, z2, z4;
      desc_s0(z1, z2, z4);
      dstep<NX, 0>(z1, 0);
      dstep<NX, 0>(z2, 0);
      int rb = fx + CL::ZERO, rstr = 0, db = fx + CL::TRASH + t, dstr = 0;
      if (t < NQ) { rb = fx + CL::Y0 + t; rstr = NQ; db = fx + CL::MM0 + t; dstr = NQ; }
      const bool ok0 = sstep<M0>(fx + CL::LR0, fx + CL::LR0, rb, rstr, db, dstr, 1.0);
      ok = ok && ok0;
      dstep<0, M0>(z4, 0);
    }
    return ok;
  }

  // vector pass with the gradient in slot OG; leaves the stage-0 open-loop step w0 and the
  // terminal multiplier nu (wave-uniform).  False if S = sum Y'M is not positive definite.
  __device__ bool vec(int OG, double (&w0)[M0], double (&nun)[NQ]) {
    // p_k = c_k + A_cl,k' (PE_k + p_{k+1}),  c_k = g_x + K'g_u,  A_cl = A + B K  (lane i: row i of p).
    // Software-pipelined: the stage-only terms of stage k-1 (closed-loop column, c + A_cl' PE) are
    // loaded and formed while stage k waits on p_{k+1}; PV is double-buffered (one barrier/stage).
    double pcur = 0.0;
    if (t < NX) {
      pcur = st(N, OG + t);
      fv(CL::PV + t) = pcur;
    }
    // raw stage operands of the closed-loop column (loaded as one block), then the arithmetic
    struct VT { double a[NX], b[NX * NU], k[NU], g, gu[NU], pe[NX], pei; };
    auto vload = [&](int k, VT& r) {
      const int i = t;
      UNR for (int q = 0; q < NX; ++q) r.a[q] = st(k, OA + q * NX + i);
      UNR for (int e = 0; e < NX * NU; ++e) r.b[e] = st(k, OB + e);
      UNR for (int b = 0; b < NU; ++b) { r.k[b] = st(k, OK + b * NX + i); r.gu[b] = st(k, OG + NX + b); }
      r.g = st(k, OG + i);
      UNR for (int q = 0; q < NX; ++q) r.pe[q] = st(k, OPE + q);
      r.pei = st(k, OPE + i);
    };
    auto vterms = [&](const VT& r, double (&acl)[NX], double& cc, double& pe) {
      double c = r.g;
      UNR for (int b = 0; b < NU; ++b) c += r.k[b] * r.gu[b];
      UNR for (int q = 0; q < NX; ++q) {
        double a = r.a[q];
        UNR for (int b = 0; b < NU; ++b) a += r.b[q * NU + b] * r.k[b];
        acl[q] = a;
      }
      UNR for (int q = 0; q < NX; ++q) c += acl[q] * r.pe[q];
      cc = c;
      pe = r.pei;
    };
    double acl[NX], cc = 0.0, pe = 0.0;
    if (t < NX) {
      VT r;
      vload(N - 1 >= 1 ? N - 1 : 1, r);
      vterms(r, acl, cc, pe);
    }
    __syncthreads();
    for (int k = N - 1; k >= 1; --k) {
      const int rb = fx + CL::PV + ((N - 1 - k) & 1) * NX, wb = fx + CL::PV + ((N - k) & 1) * NX;
      if (t < NX) {
        double pv[NX];
        UNR for (int q = 0; q < NX; ++q) pv[q] = s[rb + q];
        VT r;
        vload(k - 1 >= 1 ? k - 1 : 1, r);
        __builtin_amdgcn_sched_barrier(0);
        double p0 = cc, p1 = 0.0;
        UNR for (int q = 0; q < NX; q += 2) p0 += acl[q] * pv[q];
        UNR for (int q = 1; q < NX; q += 2) p1 += acl[q] * pv[q];
        st(k, OV + t) = pe + pcur;
        pcur = p0 + p1;
        s[wb + t] = pcur;
        vterms(r, acl, cc, pe);
      }
      __syncthreads();
    }
    if (t < NX) fv(CL::PV + t) = pcur;
    __syncthreads();
    // k_f = -Ru^-1 (g_u + B'v) per stage, lin = sum Y'k_f
    double lin[NQ];
    UNR for (int j = 0; j < NQ; ++j) lin[j] = 0.0;
    for (int k = 1 + t; k < N; k += 64) {
      double r[NU], L[NU * NU];
      UNR for (int a = 0; a < NU; ++a) {
        double x = st(k, OG + NX + a);
        UNR for (int i = 0; i < NX; ++i) x += st(k, OB + i * NU + a) * st(k, OV + i);
        r[a] = x;
      }
      UNR for (int e = 0; e < NU * NU; ++e) L[e] = st(k, OLR + e);
      chol_solve<NU>(L, r);
      UNR for (int a = 0; a < NU; ++a) {
        r[a] = -r[a];
        st(k, OKF + a) = r[a];
      }
      UNR for (int j = 0; j < NQ; ++j)
        UNR for (int a = 0; a < NU; ++a) lin[j] += st(k, OY + a * NQ + j) * r[a];
    }
    UNR for (int j = 0; j < NQ; ++j) lin[j] = wsum(lin[j]);
    // stage 0 (every lane, identical)
    {
      double v[NX], L[M0 * M0];
      UNR for (int i = 0; i < NX; ++i) v[i] = fv(CL::PE0 + i) + fv(CL::PV + i);
      UNR for (int a = 0; a < M0; ++a) {
        double x = st(0, OG + a);
        UNR for (int i = 0; i < NX; ++i) x += fv(CL::F0 + i * M0 + a) * v[i];
        w0[a] = x;
      }
      UNR for (int e = 0; e < M0 * M0; ++e) L[e] = fv(CL::LR0 + e);
      chol_solve<M0>(L, w0);
      UNR for (int a = 0; a < M0; ++a) w0[a] = -w0[a];
      UNR for (int j = 0; j < NQ; ++j)
        UNR for (int a = 0; a < M0; ++a) lin[j] += fv(CL::Y0 + a * NQ + j) * w0[a];
    }
    double Sl[NQ * NQ];
    UNR for (int e = 0; e < NQ * NQ; ++e) Sl[e] = fv(CL::SC + e);
    const bool ok = chol<NQ>(Sl);
    UNR for (int j = 0; j < NQ; ++j) nun[j] = lin[j] + fv(CL::LINE + j) - rs * par(PF::E0N + j);
    chol_solve<NQ>(Sl, nun);
    __syncthreads();
    return ok;
  }

  // forward sweep.  CORR == false: affine direction -> DA, returns the affine step and the mu_aff
  // polynomial; CORR == true: combined direction -> D, returns alpha_max.
  template <bool CORR>
  __device__ void fwd(const double (&w0in)[M0], const double (&nun)[NQ], double smu, double& amax, double& c0,
                      double& c1, double& c2) {
    constexpr int OT = CORR ? OD : ODA;
    {
      double w0[M0];
      UNR for (int a = 0; a < M0; ++a) {
        double x = w0in[a];
        UNR for (int j = 0; j < NQ; ++j) x -= fv(CL::MM0 + a * NQ + j) * nun[j];
        w0[a] = x;
      }
      if (t == 0) {
        UNR for (int i = 0; i < NZ; ++i) st(0, OT + i) = i < M0 ? w0[i < M0 ? i : 0] : 0.0;
      }
      if (t < NX) {
        double x = rs * st(0, OE + t);
        UNR for (int a = 0; a < M0; ++a) x += fv(CL::F0 + t * M0 + a) * w0[a];
        st(1, OT + t) = x;
      }
    }
    __syncthreads();
    // dx_{k+1} = c_k + A_cl,k dx_k, c_k = rs e_k + B_k (k_f - M nu); lane i: row i.  The stage-only
    // terms of stage k+1 are formed while stage k waits on dx_k.
    struct FT { double e, kf[NU], m[NU * NQ], b[NU], a[NX], k[NU * NX]; };
    auto fload = [&](int k, FT& r) {
      const int i = t;
      r.e = st(k, OE + i);
      UNR for (int a = 0; a < NU; ++a) { r.kf[a] = st(k, OKF + a); r.b[a] = st(k, OB + i * NU + a); }
      UNR for (int e = 0; e < NU * NQ; ++e) r.m[e] = st(k, OM + e);
      UNR for (int q = 0; q < NX; ++q) r.a[q] = st(k, OA + i * NX + q);
      UNR for (int e = 0; e < NU * NX; ++e) r.k[e] = st(k, OK + e);
    };
    auto fterms = [&](const FT& r, double (&acl)[NX], double& cc) {
      double c = rs * r.e;
      UNR for (int a = 0; a < NU; ++a) {
        double kfm = r.kf[a];
        UNR for (int j = 0; j < NQ; ++j) kfm -= r.m[a * NQ + j] * nun[j];
        c += r.b[a] * kfm;
      }
      UNR for (int q = 0; q < NX; ++q) {
        double a = r.a[q];
        UNR for (int b = 0; b < NU; ++b) a += r.b[b] * r.k[b * NX + q];
        acl[q] = a;
      }
      cc = c;
    };
    {
      double acl[NX], cc = 0.0;
      if (t < NX) {
        FT r;
        fload(1 < N ? 1 : N - 1 > 0 ? N - 1 : 1, r);
        fterms(r, acl, cc);
      }
      for (int k = 1; k < N; ++k) {
        if (t < NX) {
          double dx[NX];
          UNR for (int q = 0; q < NX; ++q) dx[q] = st(k, OT + q);
          FT r;
          fload(k + 1 < N ? k + 1 : k, r);
          __builtin_amdgcn_sched_barrier(0);
          double p0 = cc, p1 = 0.0;
          UNR for (int q = 0; q < NX; q += 2) p0 += acl[q] * dx[q];
          UNR for (int q = 1; q < NX; q += 2) p1 += acl[q] * dx[q];
          st(k + 1, OT + t) = p0 + p1;
          fterms(r, acl, cc);
        }
        __syncthreads();
      }
    }
    // controls of the middle stages, then the step-length tests (stage-parallel)
    typename Lane<NQ>::MinRatio mr{1.0, CORR ? o.tau : 1.0};
    double a0 = 0.0, a1 = 0.0, a2 = 0.0;
    for (int k = t; k <= N; k += 64) {
      if (k > 0) {
        UNR for (int a = 0; a < NU; ++a) {
          double x = 0.0;
          if (k < N) {
            x = st(k, OKF + a);
            UNR for (int j = 0; j < NQ; ++j) x -= st(k, OM + a * NQ + j) * nun[j];
            UNR for (int i = 0; i < NX; ++i) x += st(k, OK + a * NX + i) * st(k, OT + i);
          }
          st(k, OT + NX + a) = x;
        }
      }
      UNR for (int i = 0; i < NZ; ++i) {
        const CS c = comp(k, i);
        if (!c.bx) continue;
        const double d = st(k, OT + i);
        double dll, dlu;
        if (!CORR) {
          dll = -c.ql - c.ql * d * c.itl;
          dlu = -c.qu + c.qu * d * c.itu;
          a0 += c.tl * c.ql + c.tu * c.qu;
          a1 += c.tl * dll + d * c.ql + c.tu * dlu - d * c.qu;
          a2 += d * dll - d * dlu;
        } else {
          double rl, ru;
          corr_rhs(c, st(k, ODA + i), smu, rl, ru);
          dll = (rl - c.ql * d) * c.itl;
          dlu = (ru + c.qu * d) * c.itu;
        }
        mr.add(c.tl, d);
        mr.add(c.tu, -d);
        mr.add(c.ql, dll);
        mr.add(c.qu, dlu);
      }
    }
    amax = wmind(mr.value());
    c0 = wsum(a0); c1 = wsum(a1); c2 = wsum(a2);
    __syncthreads();
  }

  __device__ void update(double alpha, double smu) {
    double musum = 0.0;
    for (int k = t; k <= N; k += 64) {
      UNR for (int i = 0; i < NZ; ++i) {
        const CS c = comp(k, i);
        const double d = st(k, OD + i);
        st(k, ODZ + i) = c.dz + alpha * d;
        if (!c.bx) continue;
        double rl, ru;
        corr_rhs(c, st(k, ODA + i), smu, rl, ru);
        const double dll = (rl - c.ql * d) * c.itl, dlu = (ru + c.qu * d) * c.itu;
        const double qln = c.ql + alpha * dll, qun = c.qu + alpha * dlu;
        st(k, OQL + i) = qln;
        st(k, OQU + i) = qun;
        musum += (c.tl + alpha * d) * qln + (c.tu - alpha * d) * qun;
      }
    }
    mu = wsum(musum) / nbox;
    __syncthreads();
  }

  // costate recovery into the DA slot (x part) of stages 0..N-1
  __device__ bool costate() {
    bool fin = true;
    if (t < NX) {
      const int i = t;
      const double dz = st(N, ODZ + i);
      st(N - 1, ODA + i) = o.lm * dz - st(N, OQL + i) + st(N, OQU + i) +
                           (i >= NQ ? par(PF::QNU + (i >= NQ ? i - NQ : 0)) : 0.0);
      fin = isfinite(dz);
    }
    fin = __ballot(!fin) == 0ull;
    __syncthreads();
    {
      auto cterms = [&](int k, double (&ac)[NX], double& cc) {
        const int i = t;
        cc = o.lm * st(k, ODZ + i) - st(k, OQL + i) + st(k, OQU + i);
        UNR for (int q = 0; q < NX; ++q) ac[q] = st(k, OA + q * NX + i);
      };
      double ac[NX], cc = 0.0;
      if (t < NX) cterms(N - 1 >= 1 ? N - 1 : 1, ac, cc);
      for (int k = N - 1; k >= 1; --k) {
        if (t < NX) {
          double lam[NX], an[NX], cn;
          UNR for (int q = 0; q < NX; ++q) lam[q] = st(k, ODA + q);
          cterms(k - 1 >= 1 ? k - 1 : 1, an, cn);
          __builtin_amdgcn_sched_barrier(0);
          double p0 = cc, p1 = 0.0;
          UNR for (int q = 0; q < NX; q += 2) p0 += ac[q] * lam[q];
          UNR for (int q = 1; q < NX; q += 2) p1 += ac[q] * lam[q];
          st(k - 1, ODA + t) = p0 + p1;
          UNR for (int q = 0; q < NX; ++q) ac[q] = an[q];
          cc = cn;
        }
        __syncthreads();
      }
    }
    return fin;
  }

  // ---------------------------------------------------------------------------------------------
  // merit line search + update (stage-parallel)
  // ---------------------------------------------------------------------------------------------
  __device__ void update_weights() {
    double lmax = 0.0;
    for (int k = t; k <= N; k += 64) {
      if (k < N) {
        UNR for (int i = 0; i < NX; ++i) {
          gdouble& wp = G.atv(w.WPI, NX, k, i);
          wp = Lane<NQ>::wupd(wp, st(k, ODA + i));
        }
      }
      UNR for (int i = 0; i < NZ; ++i) lmax = fmax(lmax, fmax(st(k, OQL + i), st(k, OQU + i)));
    }
    lmax = wmaxd(lmax);
    if (t == 0) {
      UNR for (int j = 0; j < NQ; ++j) par(PF::WNU + j) = Lane<NQ>::wupd(par(PF::WNU + j), par(PF::QNU + j));
      par(PF::WBND) = Lane<NQ>::wupd(par(PF::WBND), lmax);
    }
    __syncthreads();
  }

  __device__ double merit(double alpha) const {
    const double h = par(PF::H);
    const double sv = par(PF::S) + alpha * st(0, ODZ);
    double val = 0.0, viol = 0.0;
    for (int k = t; k <= N; k += 64) {
      const double* rec = &s[k * REC];
      UNR for (int i = 0; i < NZ; ++i) {
        double lb, ub;
        if (!box(k, i, lb, ub)) continue;
        const double v = rec[OZ + i] + alpha * rec[ODZ + i];
        viol += fmax(0.0, lb - v) + fmax(0.0, v - ub);
      }
      if (k > 0) {
        const double* rp = &s[(k - 1) * REC];
        double xp[NX], up[NU], phi[NX];
        if (k == 1) {
          UNR for (int j = 0; j < NQ; ++j) { xp[j] = par(PF::Q0 + j); xp[NQ + j] = sv * par(PF::DIR + j); }
          UNR for (int a = 0; a < NU; ++a) up[a] = rp[OZ + 1 + a] + alpha * rp[ODZ + 1 + a];
        } else {
          UNR for (int i = 0; i < NX; ++i) xp[i] = rp[OZ + i] + alpha * rp[ODZ + i];
          UNR for (int a = 0; a < NU; ++a) up[a] = rp[OZ + NX + a] + alpha * rp[ODZ + NX + a];
        }
        rk4<NQ>(h, xp, up, phi);
        UNR for (int i = 0; i < NX; ++i) {
          const double xn = rec[OZ + i] + alpha * rec[ODZ + i];
          val += G.atv(w.WPI, NX, k - 1, i) * fabs(phi[i] - xn);
        }
        if (k == N) {
          UNR for (int j = 0; j < NQ; ++j)
            val += par(PF::WNU + j) * fabs(rec[OZ + NQ + j] + alpha * rec[ODZ + NQ + j] - par(PF::VFIN + j));
        }
      }
    }
    return par(PF::CS) * sv + par(PF::CCONST) + wsum(val) + par(PF::WBND) * wsum(viol);
  }

  __device__ void apply(double alpha) {
    for (int k = t; k <= N; k += 64) {
      if (k == 0) {
        UNR for (int a = 0; a < NU; ++a) G.atv(w.U, NU, 0, a) += alpha * st(0, ODZ + 1 + a);
      } else {
        UNR for (int i = 0; i < NX; ++i) G.atv(w.X, NX, k, i) += alpha * st(k, ODZ + i);
        if (k < N) {
          UNR for (int a = 0; a < NU; ++a) G.atv(w.U, NU, k, a) += alpha * st(k, ODZ + NX + a);
        }
      }
      UNR for (int i = 0; i < NZ; ++i) {
        gdouble& ll = G.atv(w.LL, NZ, k, i);
        gdouble& lu = G.atv(w.LU, NZ, k, i);
        ll += alpha * (st(k, OQL + i) - ll);
        lu += alpha * (st(k, OQU + i) - lu);
      }
      if (k < N) {
        UNR for (int i = 0; i < NX; ++i) {
          gdouble& pi = G.atv(w.PI, NX, k, i);
          pi += alpha * (st(k, ODA + i) - pi);
        }
      }
    }
    __syncthreads();
    if (t == 0) {
      par(PF::S) += alpha * st(0, ODZ);
      UNR for (int j = 0; j < NQ; ++j) par(PF::NU_ + j) += alpha * (par(PF::QNU + j) - par(PF::NU_ + j));
    }
    __syncthreads();
  }

  __device__ void store(const Inputs& in, int pid, int status, int it, int qit) const {
    constexpr int NXR = NX + 1;
    double* xo = in.xo + (long long)pid * (in.nmax + 1) * NXR;
    double* uo = in.uo + (long long)pid * in.nmax * NU;
    const double sv = par(PF::S), h = par(PF::H);
    for (int k = t; k <= N; k += 64) {
      UNR for (int i = 0; i < NX; ++i) {
        const double v = (k == 0) ? (i < NQ ? par(PF::Q0 + i) : sv * par(PF::DIR + (i - NQ + (i < NQ ? NQ : 0))))
                                  : (double)G.atv(w.X, NX, k, i);
        xo[(long long)k * NXR + i] = v;
      }
      xo[(long long)k * NXR + NX] = h;
      if (k < N) {
        UNR for (int a = 0; a < NU; ++a) uo[(long long)k * NU + a] = G.atv(w.U, NU, k, a);
      }
    }
    if (t == 0) {
      in.status[pid] = status;
      in.cost[pid] = par(PF::CS) * sv + par(PF::CCONST);
      in.sqp_iter[pid] = it;
      in.qp_iter[pid] = qit;
    }
  }

  // the remaining SQP of this slot's problem, to termination
  __device__ void run(const Inputs& in, const SlotState& ss) {
    const unsigned sl = G.slot;
    const int pid = ss(IS_PID, sl);
    N = ss(IS_N, sl);
    int it = ss(IS_IT, sl), qit = ss(IS_QIT, sl);
    for (int f = t; f < PF::COUNT; f += 64) par(f) = G.par(f);
    for (int e = t; e < 16; e += 64) fv(CL::ZERO + e) = 0.0;
    __syncthreads();
    int status = -1;
    CPROF_DECL
    for (;;) {
      double rstat, req, rineq, rcomp;
      linearize(rstat, req, rineq, rcomp);
      CPROF(0)
      if (!isfinite(rstat) || !isfinite(req)) status = 1;
      else if (rstat < o.tol_stat && req < o.tol_eq && rineq < o.tol_ineq && rcomp < o.tol_comp) status = 0;
      else if (it >= o.max_iter) status = 2;
      if (status >= 0) break;
      qp_init();
      CPROF(1)
      int qcur = 0, qst = 1;
      double w0[M0], nun[NQ];
      for (;;) {
        int q = qp_check();
        if (q == 1 && qcur >= o.qp_max_iter) q = 2;
        if (q != 1) { qst = q; break; }
        prep_pred();
        CPROF(2)
        const bool okf = factor();
        CPROF(3)
        const bool okv = vec(ODA, w0, nun);
        CPROF(4)
        if (!(okf && okv)) { qst = -1; break; }
        double aa, c0, c1, c2;
        fwd<false>(w0, nun, 0.0, aa, c0, c1, c2);
        CPROF(5)
        const double muaff = (c0 + aa * (c1 + aa * c2)) / nbox;
        double sig = muaff / mu;
        sig = fmin(1.0, sig * sig * sig);
        const double smu = sig * mu;
        prep_corr(smu);
        CPROF(2)
        if (!vec(OD, w0, nun)) { qst = -1; break; }
        CPROF(4)
        double amax;
        fwd<true>(w0, nun, smu, amax, c0, c1, c2);
        CPROF(5)
        const double alpha = fmin(1.0, o.tau * amax);
        update(alpha, smu);
        if (t == 0) {
          UNR for (int j = 0; j < NQ; ++j) par(PF::QNU + j) += alpha * (nun[j] - par(PF::QNU + j));
        }
        __syncthreads();
        rs *= (1.0 - alpha);
        ++qcur;
        CPROF(6)
      }
      qit += qcur;
      if (qst < 0 || !costate()) { status = 4; break; }
      CPROF(7)
      update_weights();
      const double phi0 = merit(0.0);
      double alpha = 1.0;
      for (;;) {
        const double pa = merit(alpha);
        if (pa < phi0) break;
        if (alpha * o.alpha_red < o.alpha_min) break;
        alpha *= o.alpha_red;
      }
      apply(alpha);
      CPROF(8)
      ++it;
      if (!isfinite(par(PF::S))) { status = 1; break; }
    }
#ifdef VBOC_COOP_PROF
    if (t == 0 && it - ss(IS_IT, sl) >= 300)
      printf("[coop] pid %d N %d sqp %d qp %d | cyc lin %llu qpinit %llu prep %llu factor %llu vec %llu fwd %llu upd %llu costate %llu ls %llu\n",
             pid, N, it, qit, cp_[0], cp_[1], cp_[2], cp_[3], cp_[4], cp_[5], cp_[6], cp_[7], cp_[8]);
#endif
    store(in, pid, status, it, qit);
    __syncthreads();
    if (t == 0) {
      ss(IS_PID, sl) = -1;
      ss(IS_PH, sl) = 0;
      atomicAdd(ss.done, 1u);
    }
  }
};

// one workgroup = one wave = one problem; list[] holds the slots still iterating
template <int NQ>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_coop(Work w, Opts o, Inputs in, SlotState ss, const int* list, int nmax) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const unsigned slot = (unsigned)__builtin_amdgcn_readfirstlane(list[blockIdx.x]);
  Coop<NQ> C(smem, CoopLayout<NQ>::REC * (nmax + 1), w, o, slot, (int)threadIdx.x);
  C.run(in, ss);
}

// compact the slots still iterating (phase 1 at a round boundary) into list[]
__global__ void k_list(SlotState ss, int* list, unsigned* cnt) {
  const unsigned slot = blockIdx.x * blockDim.x + threadIdx.x;
  if (ss(IS_PID, slot) >= 0 && ss(IS_PH, slot) == 1) list[atomicAdd(cnt, 1u)] = (int)slot;
}

}  // namespace vboc

// coop.h - wave solver: ONE boundary OCP per wave (64 lanes cooperate on one problem).
//
// Why: the lane-per-problem kernels (vboc_solver.hip) stream stage data at full HBM rate while every
// lane of a wave is iterating, but SQP/IPM iteration counts differ wildly between problems (SQP
// median ~20, a few percent at 300-1000; IPM 5-50 per SQP iteration), so lane-mode waves turn sparse
// (a masked wave still fetches whole lines and waits for its slowest lane).  Here a problem owns a
// wave and runs its own SQP/IPM loop to termination inside one persistent kernel:
//   * stage-parallel passes (linearisation + sensitivities, residuals, IPM initial point,
//     Hessian/gradient preparation, step-length tests, iterate update, merit re-simulation,
//     weights, step application): lane j owns stages j, j+64, ...;
//   * the Riccati factorisation recursion: per stage three "dot-product steps" in which every lane
//     computes one entry of P A, P B, A'PA, B'PB, B'PA, B'Pi, A'Pi+K'Y, ... from operands in LDS
//     (per-lane descriptor tables, so the 64 lanes run ONE instruction stream - no divergence),
//     plus one step where all lanes factorise Ru redundantly (rsq + Newton, no division) and lanes
//     solve one column each;
//   * the vector, forward and costate recursions in closed-loop form, A_cl = A + B K, one short
//     dependent step per stage on NX lanes.
// Storage: each problem's stage records live in a problem-major region in HBM (L2/MALL-resident
// while it is being solved); LDS holds only the recursion state, parameters, scratch and a 3-slot
// ring of stage windows that the recursions prefetch two stages ahead (16-B loads) and write back.
// LDS per problem is ~8 KB, so several problems share a CU (occupancy is set by registers).
// The arithmetic is the algorithm of Lane<NQ> / oracle/vboc_oracle.c (same formulas, same
// decisions); only summation orders differ (rounding-level).
// Sizes: NQ = 1-3 are the pendulum chains (one output per lane per recursion step, stage windows of
// one or two LDS-DMAs); NQ = 4 is the UR5 arm (NX = 8: two outputs per lane, windows of up to three DMAs).
#pragma once

// ring depths (slots / stages of prefetch) of the factorisation and of the vector / forward / costate
// recursions; build-time knobs for measurements
#ifndef VBOC_NSF
#define VBOC_NSF 4
#endif
#ifndef VBOC_DF
#define VBOC_DF 2
#endif
#ifndef VBOC_NSV
#define VBOC_NSV 8
#endif
#ifndef VBOC_DV
#define VBOC_DV 6
#endif

namespace vboc {

typedef double dbl2 __attribute__((ext_vector_type(2)));
typedef double dbl4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) dbl2 gdbl2;
typedef __attribute__((address_space(1))) void gvoid;
typedef __attribute__((address_space(3))) void lvoid;

__host__ __device__ constexpr int even_up(int v) { return (v + 1) & ~1; }
// stage-record stride: VBOC_REC_ALIGN doubles (2 = 16 B, the product; 16 = 128-B L2 lines: every stage record then
// starts on a line, measurement builds)
#ifndef VBOC_REC_ALIGN
#define VBOC_REC_ALIGN 2
#endif
__host__ __device__ constexpr int rec_up(int v) { return (v + VBOC_REC_ALIGN - 1) / VBOC_REC_ALIGN * VBOC_REC_ALIGN; }

template <int NQ>
struct WaveLayout {
  static constexpr int NX = 2 * NQ, NU = NQ, NZ = 3 * NQ, M0 = NQ + 1;
  // global stage record: A, B, e (defect -> initial residual), D (H / g_corr / corrector direction), DA (g_pred /
  // affine direction / costate), z (current iterate), dz, lambda_l, lambda_u, K, k_f, chol(Ru) (Ru^-1), M, Y, P e, C,
  // A_cl, then the SQP state x, u, pi, lam_l, lam_u, w_pi.  IN_FIRST (the pendulum chains, since round 6): the
  // factorisation's inputs A, B, e, D lead the record, so its window [0, W_FIN) carries nothing it does not read (the
  // triple: 70 doubles instead of the 114 before K); the arm (NQ = 4) keeps round 5's order A, B, z, dz, lambda, e, D, DA
  // (its k_wave<4> code is left as it was)
  static constexpr bool IN_FIRST = NQ <= 3;
  static constexpr int OA = 0, OB = OA + NX * NX, P0 = OB + NX * NU, OE = IN_FIRST ? P0 : P0 + 4 * NZ, OD = OE + NX,
                       ODA = OD + NZ, OZ = IN_FIRST ? ODA + NZ : P0, ODZ = OZ + NZ, OQL = ODZ + NZ, OQU = OQL + NZ,
                       OK = P0 + 6 * NZ + NX, OKF = OK + NU * NX,
                       OLR = IN_FIRST ? OKF + NU + NU * NQ : OKF + NU, OM = IN_FIRST ? OKF + NU : OLR + NU * NU,
                       OY = OKF + NU + NU * NU + NU * NQ, OPE = OY + NU * NQ, OC = OPE + NX,
                       OACL = OC + NX, OX = OACL + NX * NX, OU = OX + NX, OPI = OU + NU, OLL = OPI + NX,
                       OLU = OLL + NZ, OWPI = OLU + NZ, REC = rec_up(OWPI + NX);
  static_assert((IN_FIRST ? OQU : ODA) + NZ == OK, "the fields before K are A, B, e, D, DA, z, dz, lambda_l, lambda_u");
  // IN_FIRST also puts M before chol(Ru): the forward sweep's constant pass reads [k_f, M] and the vector pass's k_f
  // pass [chol(Ru), Y], each one contiguous range without the other's field
  static_assert(IN_FIRST ? (OM == OKF + NU && OLR == OM + NU * NQ && OY == OLR + NU * NU)
                         : (OLR == OKF + NU && OM == OLR + NU * NU && OY == OM + NU * NQ), "K, k_f, M / chol(Ru), Y");
  // OC: per-pass constant of the vector / forward recursion; OACL: closed-loop A + B K (row-major)
  // ring windows [lo, lo + W): factor [0, OC) (writes back [OK, OC)), or with FAC1 its inputs [0, W_FIN); vector pass
  // [OPE, OX); forward sweep [OC, OX); costate [0, W_COS): A (and B) to the end of lambda_u
  static constexpr int W_FAC = OC, W_FIN = even_up(ODA), LO_VEC = OPE, W_VEC = OX - OPE, LO_FWD = OC, W_FWD = OX - OC,
                       W_COS = even_up(OQU + NZ);
  // LDS-DMA rings (global_load_lds_dwordx4: one wave-instruction lands 64 lanes x 16 B = 128 doubles):
  // the factorisation streams its window two stages ahead through 4 slots of 2 KiB (two DMAs per
  // stage), the vector / forward / costate recursions six stages ahead through 8 slots of 1 KiB
  // DMAs per stage window (one DMA = 128 doubles); the slot sizes of the pendulum chains (NQ <= 3) are
  // kept as tuned, the UR5 arm (NQ = 4) gets slots of whole DMAs
  static constexpr int P_FAC = (W_FAC + 127) / 128, P_VEC = (W_VEC + 127) / 128, P_FWD = (W_FWD + 127) / 128,
                       P_COS = (W_COS + 127) / 128;
  static constexpr int P_VMAX = P_VEC > P_FWD ? (P_VEC > P_COS ? P_VEC : P_COS) : (P_FWD > P_COS ? P_FWD : P_COS);
  static constexpr int RSF = NQ <= 3 ? 256 : 128 * P_FAC, NSF = VBOC_NSF, DF = VBOC_DF,
                       RSV = NQ <= 3 ? 128 : 128 * P_VMAX, NSV = VBOC_NSV, DV = VBOC_DV;
  static constexpr int RING_D = NSF * RSF > NSV * RSV ? NSF * RSF : NSV * RSV;
  // Grouped recursions (pendulum chains): one LDS-DMA lands 64 chunks of 16 B, i.e. the windows of S
  // consecutive stages (lane l: chunk l % (W/2) of stage l / (W/2)), so the vector / forward sweeps issue one
  // DMA per S stages and walk a group's stages with compile-time slot offsets.  Groups may run past stage
  // N - 1 (the partial top group): the region carries SLACK stage records behind stage nmax for those loads.
  static constexpr int S_CAP = 4;
  static constexpr int S_VEC = NQ <= 3 ? (64 / (W_VEC / 2) < S_CAP ? 64 / (W_VEC / 2) : S_CAP) : 1,
                       S_FWD = NQ <= 3 ? (64 / (W_FWD / 2) < S_CAP ? 64 / (W_FWD / 2) : S_CAP) : 1, SLACK = S_CAP;
  static_assert(NQ > 3 || (S_VEC * W_VEC <= RSV && S_FWD * W_FWD <= RSV && (NSV & (NSV - 1)) == 0),
                "grouped windows fit one ring slot");
  static_assert(OB % 2 == 0 && OZ % 2 == 0 && OD % 2 == 0 && OK % 2 == 0 && OPE % 2 == 0 && OC % 2 == 0 &&
                    OACL % 2 == 0 && OX % 2 == 0,
                "16-byte aligned field ranges");
  static_assert(W_FAC <= RSF && W_VEC <= RSV && W_FWD <= RSV && W_COS <= RSV, "ring windows fit their slots");
  static_assert(NSF >= DF + 2 && NSV >= DV + 2, "a slot is refilled >= 2 stages after its last read");
  // LDS (doubles): ring, then the fixed region
  static constexpr int RING = 0, F0 = RING + RING_D, LR0 = F0 + NX * M0, MM0 = LR0 + M0 * M0, Y0 = MM0 + M0 * NQ,
                       PE0 = Y0 + M0 * NQ, P = PE0 + NX, PA = P + NX * NX, PB = PA + NX * NX, APA = PB + NX * NU,
                       RU = APA + NX * NX, S = RU + NU * NU, PI = S + NU * NX, PV = PI + NX * NQ, DXV = PV + 2 * NX,
                       SC = DXV + 2 * NX, LINE = SC + NQ * NQ, ZERO = LINE + NQ, TRASH = ZERO + 16, PAR = TRASH + 64,
                       XS = even_up(PAR + Par<NQ>::COUNT);
  // XS: per-stage staging rows [nmax + 1][NX] (v of the vector pass, dx of the forward sweep, the
  // costate) so that the recursions issue no global stores
  static_assert(M0 * NX <= NX * NX, "stage-0 B'P reuses the PA scratch");
  static constexpr size_t lds_bytes(int nmax) { return ((size_t)XS + (size_t)(nmax + 1) * NX) * sizeof(double); }
  static constexpr size_t region_doubles(int nmax) { return (size_t)REC * (nmax + 1 + SLACK); }
};

// one output of a recursion step:  out = s[ini] + sg * sum_q s[x1+q*sx1] s[y1+q*sy1]
//                                               +      sum_q s[x2+q*sx2] s[y2+q*sy2];  s[d1] = s[d2] = out
// `rel` marks operands inside the current stage window (offset by the ring slot base at run time).
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
// keep v in a VGPR (MFMA operands must not be folded to SGPRs / constants)
__device__ __forceinline__ void vreg(double& v) { asm volatile("" : "+v"(v)); }
// lane `lane` (wave-uniform constant) of v, as a uniform value
__device__ __forceinline__ double rdlane(double v, int lane) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, lane);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), lane);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
// Wave reductions: the butterfly `for (off = 32; off >= 1; off >>= 1) v = op(v, shfl_xor(v, off))` with the same
// association, but without the LDS crossbar (ds_bpermute: two per double per step, each a ~60-cycle round trip):
// off 32 / 16 by v_permlane32_swap / v_permlane16_swap (gfx950; each lane ends up with its own and its partner's
// value in the two outputs), off 8 by DPP row_ror:8 (= xor 8 inside a 16-lane row), off 4 by row_ror:4 (= xor 4
// once lanes i and i^8 hold equal values, which the off-8 step leaves), off 2 / 1 by quad_perm.  op is
// commutative (IEEE add / max / min), so every lane computes the bits of the shuffle butterfly.
__device__ __forceinline__ double dbl_of(unsigned hi, unsigned lo) {
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
template <bool P32>
__device__ __forceinline__ void wswap(double v, double& a, double& b) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  const unsigned l = (unsigned)u, h = (unsigned)(u >> 32);
  if constexpr (P32) {
    const auto lo = __builtin_amdgcn_permlane32_swap(l, l, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap(h, h, false, false);
    a = dbl_of(hi[0], lo[0]); b = dbl_of(hi[1], lo[1]);
  } else {
    const auto lo = __builtin_amdgcn_permlane16_swap(l, l, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap(h, h, false, false);
    a = dbl_of(hi[0], lo[0]); b = dbl_of(hi[1], lo[1]);
  }
}
template <int CTRL>
__device__ __forceinline__ double dppd(double v) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  const int l = __builtin_amdgcn_update_dpp(0, (int)(unsigned)u, CTRL, 0xF, 0xF, false);
  const int h = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), CTRL, 0xF, 0xF, false);
  return dbl_of((unsigned)h, (unsigned)l);
}
template <class OP>
__device__ __forceinline__ double wred(double v, OP op) {
  double a, b;
  wswap<true>(v, a, b);
  v = op(a, b);
  wswap<false>(v, a, b);
  v = op(a, b);
  v = op(v, dppd<0x128>(v));   // row_ror:8
  v = op(v, dppd<0x124>(v));   // row_ror:4
  v = op(v, dppd<0x4E>(v));    // quad_perm [2,3,0,1]
  v = op(v, dppd<0xB1>(v));    // quad_perm [1,0,3,2]
  return uni(v);
}
__device__ __forceinline__ double wsum(double v) {
  return wred(v, [](double x, double y) { return x + y; });
}
__device__ __forceinline__ double wmaxd(double v) {
  return wred(v, [](double x, double y) { return fmax(x, y); });
}
__device__ __forceinline__ double wmind(double v) {
  return wred(v, [](double x, double y) { return fmin(x, y); });
}

// Ordering point inside a recursion.  A k_wave workgroup is ONE wave and the LDS executes a wave's DS
// instructions in issue order, so lanes exchanging values through LDS only need the compiler not to
// move memory operations across this point.  Unlike __syncthreads() (a workgroup-scope fence, i.e.
// s_waitcnt vmcnt(0) lgkmcnt(0)) it leaves the ring prefetch loads and the per-stage global stores in
// flight.  Passes that exchange data through GLOBAL memory end with __syncthreads().
__device__ __forceinline__ void lsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
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

// Optional phase accounting (build with -DVBOC_COOP_PROF): shader-clock cycles per phase, summed over
// all jobs into g_wave_prof[0..9] ([9] = SQP iterations, [10] = IPM iterations), read with
// vboc_debug_counters().  Scalar counters (no arrays, no printf) keep the instrumented build's
// register allocation and schedule close to the product build.
__device__ unsigned long long g_wave_prof[16];
#ifdef VBOC_COOP_PROF
#define CPROF_DECL unsigned long long cp0 = 0, cp1 = 0, cp2 = 0, cp3 = 0, cp4 = 0, cp5 = 0, cp6 = 0, cp7 = 0, cp8 = 0; \
  unsigned long long cp_t = __builtin_amdgcn_s_memtime();
#define CPROF(i) { const unsigned long long n_ = __builtin_amdgcn_s_memtime(); cp##i += n_ - cp_t; cp_t = n_; }
#define CPROF_FLUSH(sq, ip) if (t == 0) { atomicAdd(&g_wave_prof[0], cp0); atomicAdd(&g_wave_prof[1], cp1); \
  atomicAdd(&g_wave_prof[2], cp2); atomicAdd(&g_wave_prof[3], cp3); atomicAdd(&g_wave_prof[4], cp4); \
  atomicAdd(&g_wave_prof[5], cp5); atomicAdd(&g_wave_prof[6], cp6); atomicAdd(&g_wave_prof[7], cp7); \
  atomicAdd(&g_wave_prof[8], cp8); atomicAdd(&g_wave_prof[9], (unsigned long long)(sq)); \
  atomicAdd(&g_wave_prof[10], (unsigned long long)(ip)); }
#else
#define CPROF_DECL
#define CPROF(i)
#define CPROF_FLUSH(sq, ip)
#endif
// Sub-step split of ONE pass (-DVBOC_COOP_PROF -DVBOC_PROF_SPLIT=1 factor / 2 vec / 3 fwd): cycles of up
// to five consecutive sections of that pass's stage loop into g_wave_prof[11..15]
#if defined(VBOC_COOP_PROF) && defined(VBOC_PROF_SPLIT)
#define SPROF_DECL(P) unsigned long long sp0 = 0, sp1 = 0, sp2 = 0, sp3 = 0, sp4 = 0, sp_t = 0; \
  constexpr bool sp_on = (VBOC_PROF_SPLIT == (P)); if (sp_on) sp_t = __builtin_amdgcn_s_memtime();
#define SPROF(i) if (sp_on) { const unsigned long long n_ = __builtin_amdgcn_s_memtime(); sp##i += n_ - sp_t; sp_t = n_; }
#define SPROF_FLUSH if (sp_on && t == 0) { atomicAdd(&g_wave_prof[11], sp0); atomicAdd(&g_wave_prof[12], sp1); \
  atomicAdd(&g_wave_prof[13], sp2); atomicAdd(&g_wave_prof[14], sp3); atomicAdd(&g_wave_prof[15], sp4); }
#else
#define SPROF_DECL(P)
#define SPROF(i)
#define SPROF_FLUSH
#endif
// Per-pass traffic / time split (-DVBOC_REPEAT=p, measurement builds only): pass p of the IPM iteration runs
// twice.  Every repeatable pass is idempotent (it recomputes its outputs from inputs it does not write), so
// results are unchanged and (bytes, time) of the build minus the product build's are those of pass p
// (tools/pass_split.py).  1 prep_pred, 2 factor, 3 acl, 4 vec (predictor), 5 fwd (predictor), 6 prep_corr,
// 7 vec (corrector), 8 fwd (corrector).
#ifndef VBOC_REPEAT
#define VBOC_REPEAT 0
#endif

#define VREP(id, stmt) do { stmt; if constexpr (VBOC_REPEAT == (id)) { stmt; } } while (0)

// Pass fusions of the IPM iteration (round 5; pendulum chains with the MFMA factorisation, no path constraint - the
// instantiations of the data-generation loop and the first solves).  Each removes stage-record traffic (a pass or
// part of a window); -DVBOC_FUSE=<mask> selects them for measurements (0: the round-4 passes).  1, 4 and 8 keep the
// arithmetic and its order (bit-identical); 2 re-associates at rounding level and is accepted under the tolerance
// parity rule of round 6.
//   1 FAC1   the factorisation's window is its inputs [A, W_FIN) - one LDS-DMA per stage instead of two ([K, C) was
//            loaded only to be overwritten by the stage's outputs before the write-back; since round 6 the record leads
//            with A, B, e, D, so the window holds only what the factorisation reads, 70 of 114 doubles);
//   2 PFUSE  the predictor preparation (D = H, DA = predictor gradient) is computed by the iterate update of the
//            previous IPM iteration from the values it has just written (prep_pred runs for the first only); the
//            compiler contracts the inlined copy differently (rounding level; round 5 dropped it on the digest);
//            with RINV below +2.1 % bulk rate, -3.2 % kernel time on 200k problems (same box, bracketed,
//            profiles/r06_probe_pfuse_rinv_ab.jsonl), parity suite green (profiles/r06_pytest_gpu_parity_pfuse_rinv.log);
//   4 CCORR  the corrector gradient pass also forms the corrector vector pass's constant c' (vec's stage-parallel
//            pre-pass re-read the gradient with K, A_cl, P e);
//   8 KFM    the forward sweep's constant pass stores k_f - M nu over k_f, and the step-length pass reads it instead
//            of re-reading M and chol(Ru) to recompute it.
#ifndef VBOC_FUSE
#define VBOC_FUSE 15
#endif

// HC: the Cartesian path-constraint rows (vboc_set_path_constraint; oracle/vboc_oracle.c hc_*, Lane::hc_*) on
// stages 1..N-1, pendulum chains with the VALU factorisation only.  No change of the stage-record layout: the
// rows' state lives in a per-workgroup region `gh` (Lane<NQ>::FHC fields per stage); the Hessian's position
// block diag(H_q) + sigma c c' travels to the factorisation in the K field of the record (free between
// prep_pred and the factorisation step that writes K), and the costate's c (lambda_u - lambda_l) term in the
// B field (free once the QP has finished).
template <int NQ, bool FM = false, bool HC = false>
struct Coop {
  using L = WaveLayout<NQ>;
  using HL = Lane<NQ>;
  static_assert(!HC || (!FM && NQ >= 2 && NQ <= 3), "path constraint: pendulum chains, VALU factorisation");
  using PF = Par<NQ>;
  static constexpr int NX = 2 * NQ, NU = NQ, NZ = 3 * NQ, M0 = NQ + 1, REC = L::REC;
  static constexpr bool FUSE_OK = FM && NQ <= 3 && !HC;
  static constexpr bool FAC1 = FUSE_OK && (VBOC_FUSE & 1), PFUSE = FUSE_OK && (VBOC_FUSE & 2),
                        CCORR = FUSE_OK && (VBOC_FUSE & 4), KFM = FUSE_OK && (VBOC_FUSE & 8);
  static constexpr int OA = L::OA, OB = L::OB, OZ = L::OZ, ODZ = L::ODZ, OQL = L::OQL, OQU = L::OQU,
                       OE = L::OE, OK = L::OK, OKF = L::OKF, OLR = L::OLR, OM = L::OM, OY = L::OY,
                       OPE = L::OPE, OD = L::OD, ODA = L::ODA, OC = L::OC, OACL = L::OACL, OX = L::OX, OU = L::OU,
                       OPI = L::OPI,
                       OLL = L::OLL, OLU = L::OLU, OWPI = L::OWPI;

  double* s;        // LDS (ring + fixed region)
  gdouble* g;       // this workgroup's stage records in HBM
  const Work& w;
  const Opts& o;
  int t;            // lane (re-made opaque at every pass entry, see fresh())
  int N;
  double rs, rd0, e00, mu, nbox;   // interior-point scalars (wave-uniform)

  unsigned lds0;    // LDS byte address of s[0] (wave-uniform), for the LDS-DMA's M0
  gdouble* gh = nullptr;   // HC: this workgroup's path-constraint rows, FHC doubles per stage
  int pause_at = -1;       // run<true>: return -2 at the top of SQP iteration pause_at (k_dg's early events)

  __device__ Coop(double* s_, gdouble* g_, const Work& w_, const Opts& o_, int t_)
      : s(s_), g(g_), w(w_), o(o_), t(t_), N(0),
        lds0((unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(size_t)(lvoid*)s_)) {}

  // The lane index as a fresh opaque value: lane-derived addresses and descriptors are then recomputed
  // in each pass instead of being hoisted to the kernel prologue and held live across the whole job
  // loop (that hoisting alone pushed the kernel past 256 registers, i.e. one wave per SIMD).
  __device__ __forceinline__ void fresh() { asm volatile("" : "+v"(t)); }

  __device__ __forceinline__ gdouble& st(int k, int off) const { return g[(long long)k * REC + off]; }
  __device__ __forceinline__ gdouble& hcr(int k, int f) const { return gh[(long long)k * HL::FHC + f]; }
  __device__ __forceinline__ bool hc_on(int k) const { return HC && k >= 1 && k < N; }
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
  // Newton directions of the row's slacks / duals from the stage step d (Lane::hc_dir)
  template <bool CORR>
  __device__ __forceinline__ void hc_dir(int k, const double* d, double smu, double& dtl, double& dtu, double& dql,
                                         double& dqu) const {
    double cd = 0.0;
    UNR for (int j = 0; j < NQ; ++j) cd += hcr(k, HL::HG + j) * d[j];
    const double htl = hcr(k, HL::HTL), htu = hcr(k, HL::HTU), hql = hcr(k, HL::HQL), hqu = hcr(k, HL::HQU);
    const double rl = rs * hcr(k, HL::HR0L), ru = rs * hcr(k, HL::HR0U);
    const double rcl = CORR ? smu - htl * hql - hcr(k, HL::HATL) * hcr(k, HL::HAQL) : -htl * hql;
    const double rcu = CORR ? smu - htu * hqu - hcr(k, HL::HATU) * hcr(k, HL::HAQU) : -htu * hqu;
    dtl = cd + rl;
    dtu = ru - cd;
    dql = (rcl - hql * dtl) / htl;
    dqu = (rcu - hqu * dtu) / htu;
  }
  __device__ __forceinline__ double& par(int f) const { return s[L::PAR + f]; }
  __device__ __forceinline__ static constexpr int fslot(int slot) { return L::RING + slot * L::RSF; }
  __device__ __forceinline__ static constexpr int vslot(int slot) { return L::RING + slot * L::RSV; }

  // ---- LDS-DMA rings of stage windows -----------------------------------------------------------------
  // One wave-instruction: lane t copies 16-B chunk (part*64 + t) of stage k's window [lo, lo + W) to LDS
  // doubles [dst + part*128 + 2t] (dst wave-uniform).  Chunk indices are clamped, never exec-masked, so
  // every call is exactly one VMEM op and the counted waits below stay exact.
  // Issued as inline asm: with the builtin, the compiler cannot tell the ring slots apart inside the one
  // dynamic LDS array and drains every in-flight DMA (vmcnt(0)) before each ds_read of the ring.  The asm
  // op is invisible to the compiler's own VMEM count, which can then only over-wait, never under-wait.
  // TAG: 1 factor, 2 vector pass, 4 forward sweep, 8 costate
  template <int TAG>
  __device__ __forceinline__ void dma(int k, int lo, int W, int dst, int part) const {
    const int nc = W / 2;
    const int c = part * 64 + t < nc ? part * 64 + t : nc - 1;
    // per-lane 64-bit addresses.  The SGPR-base form (dma_s) gives the pendulum chains the same bits, but
    // deterministically broke the UR5 instantiation (k_wave<4>: 24 % status agreement with the oracle,
    // profiles/r03z_ur5_sgpr_base_dma_bisect.log, r04_ur5_bisect.json) for a reason not found;
    // the grouped recursions (nq <= 3) keep dma_s
    const gdouble* src = g + (long long)k * REC + lo + 2 * c;
    const unsigned lds = lds0 + 8u * (unsigned)(dst + part * 128);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(lds)
                 : "memory");
  }
  // the same with a wave-uniform base (SGPR pair) and a per-lane byte offset: no per-lane 64-bit address
  // arithmetic in the recursions' loops (the lane offsets are computed once per pass)
  __device__ __forceinline__ void dma_s(const gdouble* base, unsigned voff, int dst) const {
    const unsigned lds = lds0 + 8u * (unsigned)dst;
    // the base as an SGPR pair (readfirstlane folds away where the compiler already holds it in SGPRs)
    const unsigned long long b = (unsigned long long)(size_t)base;
    const unsigned long long bs = ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(b >> 32)) << 32) |
                                  (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)b);
    // s_nop 4: an "s" operand fresh from readfirstlane / v_readlane, read by a VMEM instruction as its base, needs
    // 5 wait states that hipcc does not insert in front of inline asm (cdna_hip_programming.md, inline asm rules)
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 4\n\tglobal_load_lds_dwordx4 %1, %2\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(bs), "s"(lds)
                 : "memory");
  }
  // lane byte offset of a grouped window load: chunk l % (W/2) of stage l / (W/2) (lanes past S windows repeat
  // the last chunk of stage S - 1; they land in the slot's junk tail)
  template <int LO, int W, int S>
  __device__ __forceinline__ unsigned grp_off() const {
    constexpr int CH = W / 2;
    const int u = t / CH < S ? t / CH : S - 1;
    const int c = t - u * CH < CH ? t - u * CH : CH - 1;
    return 8u * (unsigned)(u * REC + LO + 2 * c);
  }
  // wait until at most N VMEM ops of this wave are outstanding (LDS-DMA landings are ordered for this
  // wave's own ds_reads by this wait alone)
  template <int N>
  __device__ __forceinline__ static void vmwait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
  }
  // retire every ordinary VMEM op in a way the compiler's waitcnt pass sees (the builtin, vmcnt(0)):
  // called before a ring's first DMA, so no loop-carried register is still "pending" in the pass's
  // bookkeeping - otherwise it re-waits vmcnt(0) inside the loop and drains the ring every stage
  __device__ __forceinline__ static void settle() {
    __builtin_amdgcn_s_waitcnt(0x0F70);
  }
  // write fields [LO, HI) of a factor slot back to stage k's record: exactly one VMEM op
  template <int LO, int HI>
  __device__ __forceinline__ void ring_wb(int slot, int k) const {
    static_assert((HI - LO) / 2 <= 64 && LO % 2 == 0, "one 16-B chunk per lane");
    const dbl2* src = (const dbl2*)(s + fslot(slot));
    gdbl2* dst = (gdbl2*)(g + (long long)k * REC);
    if constexpr (NQ <= 3) {
      // every lane stores (lanes past the field range repeat the last chunk: same bytes, same address), no exec
      // mask: 16k first solves 4 082 -> 3 949 ms on one box, same results (profiles/r03z_wb_ab.json).  The arm
      // keeps the masked store: its k_wave<4> lost parity with the unmasked one
      constexpr int NCH = (HI - LO) / 2;
      const int c = t < NCH ? t : NCH - 1;
      dst[LO / 2 + c] = src[LO / 2 + c];
      return;
    }
    if (t < (HI - LO) / 2) dst[LO / 2 + t] = src[LO / 2 + t];
  }


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
    const double Lo = lb - z, U = ub - z, del = o.push * (U - Lo);
    return fmin(fmax(0.0, Lo + del), U - del);
  }
  __device__ __forceinline__ double cgrad(int k, int i) const { return (k == 0 && i == 0) ? par(PF::CS) : 0.0; }

  // contiguous field range [LO, LO + 2*C) of stage k into registers (16-B loads, all issued at once)
  template <int LO, int C>
  __device__ __forceinline__ void ldr(int k, double (&d)[2 * C]) const {
    static_assert(LO % 2 == 0, "16-byte aligned range");
    const gdbl2* src = (const gdbl2*)(g + (long long)k * REC + LO);
    UNR for (int c = 0; c < C; ++c) {
      const dbl2 v = src[c];
      d[2 * c] = v.x;
      d[2 * c + 1] = v.y;
    }
  }
  // z, dz, lambda_l, lambda_u of a stage: the contiguous range [OZ, OZ + 4 NZ)
  static constexpr int NIP = (4 * NZ + 1) / 2;
  struct IP { double v[2 * NIP]; };
  __device__ __forceinline__ void ld_ip(int k, IP& r) const { ldr<OZ, NIP>(k, r.v); }
  // a part [LO, LO + CNT) of the D / DA slots in registers: element i is v[OFF + i].  The pendulum chains (IN_FIRST)
  // load its 16-B aligned cover only; the arm loads both slots [OD, OD + 2 NZ), as before round 6 (same k_wave<4> code)
  template <int LO, int CNT, bool WIDE = !L::IN_FIRST>
  struct Cov {
    static_assert(LO >= OD && LO + CNT <= OD + 2 * NZ, "a part of the D / DA slots");
    static constexpr int B = WIDE ? OD : (LO & ~1), OFF = LO - B, C = WIDE ? (2 * NZ + 1) / 2 : (OFF + CNT + 1) / 2;
    double v[2 * C];
  };
  template <int LO, int CNT>
  __device__ __forceinline__ void ldc(int k, Cov<LO, CNT>& c) const { ldr<Cov<LO, CNT>::B, Cov<LO, CNT>::C>(k, c.v); }

  struct CS { double tl, tu, itl, itu, ql, qu, dz; bool bx; };
  __device__ __forceinline__ CS comp_r(const IP& r, int k, int i) const {
    CS c;
    double lb, ub;
    c.bx = box(k, i, lb, ub);
    const double z = r.v[i];
    c.dz = r.v[NZ + i]; c.ql = r.v[2 * NZ + i]; c.qu = r.v[3 * NZ + i];
    c.tl = c.dz - (lb - z); c.tu = (ub - z) - c.dz;
    c.itl = c.bx ? 1.0 / c.tl : 0.0;
    c.itu = c.bx ? 1.0 / c.tu : 0.0;
    return c;
  }
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
  // recursion-step machinery (all operands in LDS)
  // ---------------------------------------------------------------------------------------------
  __device__ __forceinline__ void dnull(Dsc& d) const {
    d.x1 = d.y1 = d.x2 = d.y2 = d.ini = L::ZERO;
    d.sx1 = d.sy1 = d.sx2 = d.sy2 = 0;
    d.d1 = d.d2 = L::TRASH + t;
    d.rel = 0;
    d.sg = 1.0;
  }
  // outputs per lane of one recursion step: 1 for the pendulum chains, 2 for the UR5 arm (NX = 8)
  static constexpr int TXC = NX * (NX + 1) / 2, TUC = NU * (NU + 1) / 2, TMC = M0 * (M0 + 1) / 2;
  static constexpr int imax(int a, int b) { return a > b ? a : b; }
  static constexpr int OUTMAX =
      imax(imax(imax(NX * NX + NX * NU + NX + NQ, TXC + TUC + NU * NX + NU * NQ), imax(TXC + NX * NQ + NQ * NQ,
                                                                                      M0 * NX + M0 * NQ + NX + NQ)),
           imax(TMC, NQ * NQ));
  static constexpr int RD = (OUTMAX + 63) / 64;

  template <int L1, int L2, int R>
  __device__ __forceinline__ void dstep(const Dsc (&dd)[R], int kb) const {
    double res[R];
    UNR for (int rr = 0; rr < R; ++rr) {
      const Dsc& d = dd[rr];
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
      res[rr] = r0 + d.sg * s1 + s2;
    }
    lsync();
    UNR for (int rr = 0; rr < R; ++rr) {
      const Dsc& d = dd[rr];
      auto ad = [&](int a, unsigned bit) { return a + ((d.rel & bit) ? kb : 0); };
      s[ad(d.d1, RD1)] = res[rr];
      s[ad(d.d2, RD2)] = res[rr];
    }
    lsync();
  }
  // all lanes: L = chol(s[ru..]); lane-specific column solve rhs -> sgn * Ru^-1 rhs; lane 0 stores L
  template <int n>
  __device__ __forceinline__ bool sstep(int ru, int ldst, int rb, int rstr, int db, int dstr, double sgn) const {
    double Lm[n * n], id[n], b[n];
    UNR for (int a = 0; a < n; ++a) b[a] = s[rb + a * rstr];
    UNR for (int e = 0; e < n * n; ++e) Lm[e] = s[ru + e];
    const bool ok = chol_inv<n>(Lm, id);
    solve_inv<n>(Lm, id, b);
    lsync();
    UNR for (int a = 0; a < n; ++a) s[db + a * dstr] = sgn * b[a];
    if (t == 0) {
      UNR for (int e = 0; e < n * n; ++e) s[ldst + e] = Lm[e];
    }
    lsync();
    return ok;
  }

  // descriptors of the middle-stage factorisation steps (rs enters through sg)
  __device__ __forceinline__ void desc_mid(Dsc (&dd1)[RD], Dsc (&dd2)[RD], Dsc (&dd4)[RD]) const {
    UNR for (int rr = 0; rr < RD; ++rr) desc_mid1(dd1[rr], dd2[rr], dd4[rr], t + 64 * rr);
  }
  __device__ __forceinline__ void desc_mid1(Dsc& d1, Dsc& d2, Dsc& d4, const int lane) const {
    constexpr int P = L::P, PA = L::PA, PB = L::PB, APA = L::APA, RU = L::RU, S = L::S, PI = L::PI, SC = L::SC,
                  LINE = L::LINE;
    constexpr int TX = NX * (NX + 1) / 2, TU = NU * (NU + 1) / 2;
    dnull(d1); dnull(d2); dnull(d4);
    // step 1: PA = P A, PB = P B, P e (-> stage PE), lin_e += Pi' e
    int u = lane;
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
    u = lane;
    if (u < TX) {
      int i, j;
      tri(u, i, j);
      d2.x1 = OA + i; d2.sx1 = NX; d2.y1 = PA + j; d2.sy1 = NX; d2.rel = RX1;
      if (HC && i < NQ && j < NQ) { d2.ini = OK + i * NQ + j; d2.rel |= RINI; }   // diag(H_q) + sigma c c'
      else if (i == j) { d2.ini = OD + i; d2.rel |= RINI; }
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
    u = lane;
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
  // stage 0 (controls s, u_0; F0 = [A0 g, B0]): e and H of stage 0 come from its ring slot
  __device__ __forceinline__ void desc_s0(Dsc (&zz1)[RD], Dsc (&zz2)[RD], Dsc (&zz4)[RD]) const {
    UNR for (int rr = 0; rr < RD; ++rr) desc_s01(zz1[rr], zz2[rr], zz4[rr], t + 64 * rr);
  }
  __device__ __forceinline__ void desc_s01(Dsc& z1, Dsc& z2, Dsc& z4, const int lane) const {
    constexpr int P = L::P, BP = L::PA, PI = L::PI, F0 = L::F0, Y0 = L::Y0, PE0 = L::PE0, LINE = L::LINE,
                  LR0 = L::LR0, MM0 = L::MM0, SC = L::SC;
    constexpr int TM = M0 * (M0 + 1) / 2;
    dnull(z1); dnull(z2); dnull(z4);
    int u = lane;
    if (u < M0 * NX) {
      const int a = u / NX, j = u % NX;
      z1.x1 = F0 + a; z1.sx1 = M0; z1.y1 = P + j; z1.sy1 = NX; z1.d1 = z1.d2 = BP + u;
    } else if ((u -= M0 * NX) < M0 * NQ) {
      const int a = u / NQ, j = u % NQ;
      z1.x1 = F0 + a; z1.sx1 = M0; z1.y1 = PI + j; z1.sy1 = NQ; z1.d1 = z1.d2 = Y0 + u;
    } else if ((u -= M0 * NQ) < NX) {
      z1.x1 = P + u * NX; z1.sx1 = 1; z1.y1 = OE; z1.sy1 = 1; z1.sg = rs; z1.d1 = z1.d2 = PE0 + u; z1.rel = RY1;
    } else if ((u -= NX) < NQ) {
      z1.x1 = PI + u; z1.sx1 = NQ; z1.y1 = OE; z1.sy1 = 1; z1.sg = rs; z1.ini = z1.d1 = z1.d2 = LINE + u; z1.rel = RY1;
    }
    u = lane;
    if (u < TM) {
      int a, c;
      tri(u, a, c);
      z2.x1 = BP + a * NX; z2.sx1 = 1; z2.y1 = F0 + c; z2.sy1 = M0;
      if (a == c) { z2.ini = OD + a; z2.rel = RINI; }
      z2.d1 = LR0 + a * M0 + c; z2.d2 = LR0 + c * M0 + a;
    }
    u = lane;
    if (u < NQ * NQ) {
      const int i = u / NQ, j = u % NQ;
      z4.x2 = Y0 + i; z4.sx2 = NQ; z4.y2 = MM0 + j; z4.sy2 = NQ; z4.ini = z4.d1 = z4.d2 = SC + u;
    }
  }

  // ---------------------------------------------------------------------------------------------
  // problem set-up: from the inputs (wave mode) or from a lane-mode slot (hand-off)
  // ---------------------------------------------------------------------------------------------
  __device__ __forceinline__ void from_inputs(const Inputs& in, int pid) {
    fresh();
    constexpr int NXR = NX + 1, NP = NQ + 1;
    N = in.N[pid];
    const double* p = in.p + (long long)pid * NP;
    const double* lbx = in.lbx + (long long)pid * NXR;
    const double* ubx = in.ubx + (long long)pid * NXR;
    const double* lbx0 = in.lbx0 + (long long)pid * NXR;
    const double* ubx0 = in.ubx0 + (long long)pid * NXR;
    const double* lbxe = in.lbxe + (long long)pid * NXR;
    const double* ubxe = in.ubxe + (long long)pid * NXR;
    const double* xg = in.xg + (long long)pid * (in.nmax + 1) * NXR;
    const double* ug = in.ug + (long long)pid * in.nmax * NU;
    if (t == 0) {   // parameters: the Lane::load formulas
      const double h = lbx[NX];
      par(PF::H) = h;
      double nrm = 0.0;
      UNR for (int j = 0; j < NQ; ++j) nrm += p[j] * p[j];
      nrm = sqrt(nrm);
      double slb = -INFINITY, sub = INFINITY, cs = 0.0, sv = 0.0;
      UNR for (int j = 0; j < NQ; ++j) {
        const double dj = (NQ == 1) ? 1.0 : p[j] / nrm;
        par(PF::DIR + j) = dj;
        par(PF::Q0 + j) = lbx0[j];
        cs += p[j] * dj;
        const double lo = lbx0[NQ + j], hi = ubx0[NQ + j];
        if (dj > 0) { slb = fmax(slb, lo / dj); sub = fmin(sub, hi / dj); }
        else if (dj < 0) { slb = fmax(slb, hi / dj); sub = fmin(sub, lo / dj); }
        sv += dj * xg[NQ + j];
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
      par(PF::S) = sv;
    }
    for (int k = t; k <= N; k += 64) {
      UNR for (int i = 0; i < NX; ++i) st(k, OX + i) = xg[(long long)k * NXR + i];
      UNR for (int i = 0; i < NZ; ++i) { st(k, OLL + i) = 0.0; st(k, OLU + i) = 0.0; }
      if constexpr (HC) {
        hcr(k, HL::HLL) = 0.0;
        hcr(k, HL::HLU) = 0.0;
      }
      if (k < N) {
        UNR for (int a = 0; a < NU; ++a) st(k, OU + a) = ug[(long long)k * NU + a];
        UNR for (int i = 0; i < NX; ++i) { st(k, OPI + i) = 0.0; st(k, OWPI + i) = 0.0; }
      }
    }
    __syncthreads();
  }
  __device__ __forceinline__ void from_slot(const SlotState& ss, unsigned slot) {
    fresh();
    Lane<NQ> G(w, o, slot);
    N = ss(IS_N, slot);
    for (int f = t; f < PF::COUNT; f += 64) par(f) = G.par(f);
    for (int k = t; k <= N; k += 64) {
      UNR for (int i = 0; i < NX; ++i) st(k, OX + i) = G.atv(w.X, NX, k, i);
      UNR for (int i = 0; i < NZ; ++i) { st(k, OLL + i) = G.atv(w.LL, NZ, k, i); st(k, OLU + i) = G.atv(w.LU, NZ, k, i); }
      if (k < N) {
        UNR for (int a = 0; a < NU; ++a) st(k, OU + a) = G.atv(w.U, NU, k, a);
        UNR for (int i = 0; i < NX; ++i) { st(k, OPI + i) = G.atv(w.PI, NX, k, i); st(k, OWPI + i) = G.atv(w.WPI, NX, k, i); }
      }
    }
    __syncthreads();
  }

  // ---------------------------------------------------------------------------------------------
  // linearisation (stage-parallel): ERK4 + sensitivities, defects, current z, NLP residuals
  // ---------------------------------------------------------------------------------------------
  __device__ __forceinline__ void linearize(double& rstat, double& req, double& rineq, double& rcomp) {
    fresh();
    const double h = par(PF::H), sv = par(PF::S);
    double stt = 0.0, eq = 0.0, inq = 0.0, cp = 0.0;
    for (int k = t; k <= N; k += 64) {
      gdouble* rec = &g[(long long)k * REC];
      if (k < N) {
        double xk[NX], uk[NU], x1[NX];
        if (k == 0) {
          UNR for (int j = 0; j < NQ; ++j) { xk[j] = par(PF::Q0 + j); xk[NQ + j] = sv * par(PF::DIR + j); }
        } else {
          UNR for (int i = 0; i < NX; ++i) xk[i] = rec[OX + i];
        }
        UNR for (int a = 0; a < NU; ++a) uk[a] = rec[OU + a];
        rk4_sens<NQ>(h, xk, uk, x1, [&](int i, int c, double v) {
          if (c < NX) rec[OA + i * NX + c] = v;
          else rec[OB + i * NU + (c - NX)] = v;
        });
        UNR for (int i = 0; i < NX; ++i) {
          const double b = x1[i] - st(k + 1, OX + i);
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
        UNR for (int i = 0; i < NX; ++i) pik[i] = rec[OPI + i];
        if (k == 0) {
          double F[NX * M0];
          UNR for (int i = 0; i < NX; ++i) {
            double tt = 0.0;
            UNR for (int j = 0; j < NQ; ++j) tt += rec[OA + i * NX + NQ + j] * par(PF::DIR + j);
            F[i * M0] = tt;
            UNR for (int a = 0; a < NU; ++a) F[i * M0 + 1 + a] = rec[OB + i * NU + a];
          }
          UNR for (int e = 0; e < NX * M0; ++e) s[L::F0 + e] = F[e];
          UNR for (int c = 0; c < M0; ++c) {
            double gr = (c == 0 ? par(PF::CS) : 0.0) - rec[OLL + c] + rec[OLU + c];
            UNR for (int r = 0; r < NX; ++r) gr += F[r * M0 + c] * pik[r];
            stt = fmax(stt, fabs(gr));
          }
        } else {
          double pprev[NX];
          UNR for (int i = 0; i < NX; ++i) pprev[i] = st(k - 1, OPI + i);
          double hg[NQ], hmul = 0.0;
          if constexpr (HC) {
            const double hv = hc_eval(xk, hg);
            hcr(k, HL::HV) = hv;
            UNR for (int j = 0; j < NQ; ++j) hcr(k, HL::HG + j) = hg[j];
            const double hll = hcr(k, HL::HLL), hlu = hcr(k, HL::HLU);
            hmul = hlu - hll;
            inq = fmax(inq, fmax(o.hlh - hv, hv - o.huh));
            cp = fmax(cp, fmax(fabs(hll * (hv - o.hlh)), fabs(hlu * (o.huh - hv))));
          }
          UNR for (int c = 0; c < NZ; ++c) {
            double gr = -rec[OLL + c] + rec[OLU + c];
            if (c < NX) {
              UNR for (int r = 0; r < NX; ++r) gr += rec[OA + r * NX + c] * pik[r];
              gr -= pprev[c];
              if constexpr (HC) {
                if (c < NQ) gr += hg[c < NQ ? c : 0] * hmul;
              }
            } else {
              UNR for (int r = 0; r < NX; ++r) gr += rec[OB + r * NU + (c - NX)] * pik[r];
            }
            stt = fmax(stt, fabs(gr));
          }
        }
        UNR for (int c = 0; c < NZ; ++c) {
          double lb, ub;
          if (!box(k, c, lb, ub)) continue;
          const double z = rec[OZ + c], ll = rec[OLL + c], lu = rec[OLU + c];
          inq = fmax(inq, fmax(lb - z, z - ub));
          cp = fmax(cp, fmax(fabs(ll * (z - lb)), fabs(lu * (ub - z))));
        }
      } else {
        UNR for (int i = 0; i < NX; ++i) rec[OZ + i] = rec[OX + i];
        UNR for (int i = NX; i < NZ; ++i) rec[OZ + i] = 0.0;
        UNR for (int c = 0; c < NX; ++c) {
          const double z = rec[OX + c];
          double gr = -rec[OLL + c] + rec[OLU + c] - st(N - 1, OPI + c);
          if (c >= NQ) {
            gr += par(PF::NU_ + c - NQ);
            eq = fmax(eq, fabs(z - par(PF::VFIN + c - NQ)));
          }
          stt = fmax(stt, fabs(gr));
          if (c < NQ) {
            const double lb = par(PF::QNLB + c), ub = par(PF::QNUB + c);
            const double ll = rec[OLL + c], lu = rec[OLU + c];
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
  __device__ __forceinline__ void qp_init() {
    fresh();
    double musum = 0.0, nb = 0.0, rd = 0.0, e0 = 0.0;
    for (int k = t; k <= N; k += 64) {
      gdouble* rec = &g[(long long)k * REC];
      double dz[NZ];
      UNR for (int i = 0; i < NZ; ++i) {
        double lb, ub, ql = 0.0, qu = 0.0, d0 = 0.0;
        if (box(k, i, lb, ub)) {
          const double z = rec[OZ + i], Lo = lb - z, U = ub - z;
          d0 = dz_init(lb, ub, z);
          ql = o.mu0 / (d0 - Lo);
          qu = o.mu0 / (U - d0);
          musum += o.mu0 + o.mu0;
          nb += 2.0;
        }
        dz[i] = d0;
        rec[ODZ + i] = d0; rec[OQL + i] = ql; rec[OQU + i] = qu;
        if (!(HC && i < NQ && k >= 1 && k < N)) rd = fmax(rd, fabs(o.lm * d0 + cgrad(k, i) - ql + qu));
      }
      if constexpr (HC) {
        if (hc_on(k)) {
          // slacks from the initial c'dz, clipped to ipm_push (Lane::qp_init)
          double hg[NQ], gd = 0.0;
          UNR for (int j = 0; j < NQ; ++j) { hg[j] = hcr(k, HL::HG + j); gd += hg[j] * dz[j]; }
          const double hv = hcr(k, HL::HV), Lh = o.hlh - hv, Uh = o.huh - hv;
          const double tl = fmax(gd - Lh, o.push), tu = fmax(Uh - gd, o.push);
          const double ql = o.mu0 / tl, qu = o.mu0 / tu;
          const double r0l = gd - Lh - tl, r0u = Uh - gd - tu;
          hcr(k, HL::HTL) = tl; hcr(k, HL::HTU) = tu; hcr(k, HL::HQL) = ql; hcr(k, HL::HQU) = qu;
          hcr(k, HL::HR0L) = r0l; hcr(k, HL::HR0U) = r0u;
          musum += tl * ql + tu * qu;
          nb += 2.0;
          e0 = fmax(e0, fmax(fabs(r0l), fabs(r0u)));
          UNR for (int i = 0; i < NQ; ++i)
            rd = fmax(rd, fabs(o.lm * dz[i] + cgrad(k, i) - rec[OQL + i] + rec[OQU + i] + hg[i] * (qu - ql)));
        }
      }
      if (k < N) {
        const gdouble* rn = &g[(long long)(k + 1) * REC];
        UNR for (int i = 0; i < NX; ++i) {
          double lb, ub, dn = 0.0;
          if (box(k + 1, i, lb, ub)) dn = dz_init(lb, ub, rn[OZ + i]);
          double tt = rec[OE + i] - dn;
          if (k == 0) {
            UNR for (int a = 0; a < M0; ++a) tt += s[L::F0 + i * M0 + a] * dz[a];
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

  __device__ __forceinline__ int qp_check() const {
    if (!isfinite(mu)) return -1;
    if (mu < o.qp_tol_comp && rs * rd0 < o.qp_tol_stat && rs * e00 < o.qp_tol_eq) return 0;
    return 1;
  }

  // H -> D, predictor gradient -> DA of stage k from its iterate r (z, dz, lambda_l, lambda_u)
  __device__ __forceinline__ void prep_from(const IP& r, int k, gdouble* rec) const {
    UNR for (int i = 0; i < NZ; ++i) {
      const CS c = comp_r(r, k, i);
      rec[OD + i] = o.lm + (c.bx ? c.ql * c.itl + c.qu * c.itu : 0.0);
      rec[ODA + i] = o.lm * c.dz + cgrad(k, i);
    }
  }
  // H -> D slot, predictor gradient -> DA slot
  __device__ __forceinline__ void prep_pred() {
    fresh();
    for (int k = t; k <= N; k += 64) {
      IP r;
      ld_ip(k, r);
      __builtin_amdgcn_sched_barrier(0);
      gdouble* rec = &g[(long long)k * REC];
      prep_from(r, k, rec);
      if constexpr (HC) {
        if (hc_on(k)) {
          const double htl = hcr(k, HL::HTL), htu = hcr(k, HL::HTU), hql = hcr(k, HL::HQL), hqu = hcr(k, HL::HQU);
          const double sig = hql / htl + hqu / htu;
          const double gam = hql * (rs * hcr(k, HL::HR0L)) / htl - hqu * (rs * hcr(k, HL::HR0U)) / htu;
          double hg[NQ];
          UNR for (int j = 0; j < NQ; ++j) hg[j] = hcr(k, HL::HG + j);
          UNR for (int i = 0; i < NQ; ++i) {
            UNR for (int j = 0; j < NQ; ++j)
              rec[OK + i * NQ + j] = (i == j ? (double)rec[OD + i] : 0.0) + sig * hg[i] * hg[j];
            rec[ODA + i] += hg[i] * gam;
          }
        }
      }
    }
    __syncthreads();
  }
  // corrector gradient (uses the affine direction in DA) -> D slot
  __device__ __forceinline__ void prep_corr(double smu) {
    fresh();
    for (int k = t; k <= N; k += 64) {
      IP r;
      Cov<ODA, NZ> da;   // the affine direction (D is this pass's output)
      ld_ip(k, r);
      ldc(k, da);
      __builtin_amdgcn_sched_barrier(0);
      gdouble* rec = &g[(long long)k * REC];
      double gv[NZ];
      UNR for (int i = 0; i < NZ; ++i) {
        const CS c = comp_r(r, k, i);
        double gg = o.lm * c.dz + cgrad(k, i);
        if (c.bx) {
          double rl, ru;
          corr_rhs(c, da.v[da.OFF + i], smu, rl, ru);
          gg += -c.ql - rl * c.itl + c.qu + ru * c.itu;
        }
        rec[OD + i] = gg;
        gv[i] = gg;
      }
      if constexpr (CCORR) {
        // the corrector vector pass's constant c' = g_x + K' g_u + A_cl' P e (vec_const, the same arithmetic)
        if (k >= 1 && k < N) vec_const(k, gv);
      }
      if constexpr (HC) {
        if (hc_on(k)) {
          const double htl = hcr(k, HL::HTL), htu = hcr(k, HL::HTU), hql = hcr(k, HL::HQL), hqu = hcr(k, HL::HQU);
          const double rl = rs * hcr(k, HL::HR0L), ru = rs * hcr(k, HL::HR0U);
          const double rcl = smu - htl * hql - hcr(k, HL::HATL) * hcr(k, HL::HAQL);
          const double rcu = smu - htu * hqu - hcr(k, HL::HATU) * hcr(k, HL::HAQU);
          const double gam = -hql + hqu - (rcl - hql * rl) / htl + (rcu - hqu * ru) / htu;
          UNR for (int j = 0; j < NQ; ++j) rec[OD + j] += hcr(k, HL::HG + j) * gam;
        }
      }
    }
    __syncthreads();
  }

  // Riccati factorisation (matrix part) of stages N-1..0 through the LDS ring; the vector part is vec()
  __device__ __forceinline__ bool factor() {
    fresh();
    for (int e = t; e < NX * NX; e += 64) {
      const int i = e / NX, j = e % NX;
      s[L::P + e] = (i == j) ? (double)st(N, OD + i) : 0.0;
    }
    for (int e = t; e < NX * NQ; e += 64) {
      const int i = e / NQ, j = e % NQ;
      s[L::PI + e] = (i == NQ + j) ? 1.0 : 0.0;
    }
    for (int e = t; e < NQ * NQ; e += 64) s[L::SC + e] = 0.0;
    if (t < NQ) s[L::LINE + t] = 0.0;
    // stage windows through the 4-slot LDS-DMA ring, landing two stages ahead (sweep index j <-> stage
    // N-1-j, clamped at 0); P = DMAs per stage
    constexpr int P = L::P_FAC;
    auto fdma = [&](int j) {
      const int kk = N - 1 - j >= 0 ? N - 1 - j : 0;
      UNR for (int part = 0; part < P; ++part) dma<1>(kk, 0, L::W_FAC, fslot(j % L::NSF), part);
    };
    __syncthreads();   // before any DMA is in flight: this barrier's fence would drain them
    settle();
    fdma(0);
    fdma(1);
    bool ok = true;
    Dsc d1[RD], d2[RD], d4[RD];
    desc_mid(d1, d2, d4);
    SPROF_DECL(1)
    for (int j = 0; j < N; ++j) {
      const int k = N - 1 - j, kb = fslot(j % L::NSF);
      // outputs of the previous stage (k + 1) go out first (one store), then the DMA two stages ahead
      if (j >= 1) ring_wb<OK, OC>((j - 1) % L::NSF, k + 1);
      fdma(j + 2);
      SPROF(4)
      // stage k's DMAs have landed once at most the 2P DMAs issued after them are outstanding.  The wait
      // counts loads only: the ring_wb stores issued in between complete out of order with the loads, and
      // counting them (2P + 1 / 2P + 2, as before) let the wait pass with the last part of stage k's window
      // still in flight whenever they completed first
      vmwait<2 * P>();
      SPROF(3)
      if (k >= 1) {
        dstep<NX, 0>(d1, kb);
        SPROF(0)
        dstep<NX, 0>(d2, kb);
        SPROF(1)
        int rb = L::ZERO, rstr = 0, db = L::TRASH + t, dstr = 0;
        double sgn = 1.0;
        if (t < NX) { rb = L::S + t; rstr = NX; db = kb + OK + t; dstr = NX; sgn = -1.0; }
        else if (t < NX + NQ) { rb = kb + OY + (t - NX); rstr = NQ; db = kb + OM + (t - NX); dstr = NQ; }
        const bool okk = sstep<NU>(L::RU, kb + OLR, rb, rstr, db, dstr, sgn);
        ok = ok && okk;
        dstep<NX, NU>(d4, kb);
        SPROF(2)
      } else {
        Dsc z1[RD], z2[RD], z4[RD];
        desc_s0(z1, z2, z4);
        dstep<NX, 0>(z1, kb);
        dstep<NX, 0>(z2, kb);
        int rb = L::ZERO, rstr = 0, db = L::TRASH + t, dstr = 0;
        if (t < NQ) { rb = L::Y0 + t; rstr = NQ; db = L::MM0 + t; dstr = NQ; }
        const bool ok0 = sstep<M0>(L::LR0, L::LR0, rb, rstr, db, dstr, 1.0);
        ok = ok && ok0;
        dstep<0, M0>(z4, kb);
      }
      lsync();
      SPROF(4)
    }
    SPROF_FLUSH
    __syncthreads();   // write-back visible to the next sweep's ring loads
    return ok;
  }

  // The same factorisation of stages N-1..1 on FP64 MFMA (v_mfma_f64_16x16x4f64), pendulum chains only.
  // With G_k = [A_k | B_k | rs e_k] (NX x (NX + NU + 1), padded to 16 columns), every stage is
  //   PG = P G                                   (2 MFMAs: k = 0..7)
  //   H  = G' [PG | Pi] + diag(Hx, Hu) + carry   (2 MFMAs)   = [A'PA+Hx A'PB A'Pe A'Pi; B'PA B'PB+Hu . B'Pi; ..]
  //   Z  = L^-1 H_u, L = chol(Ru = H_uu)         (uniform 3x3 Cholesky, one column of Z per lane)
  //   D  = H - Z' Z                              (1 MFMA, k = 0..3)
  // so D holds P_k = A'PA + Hx - S'Ru^-1 S, Pi_k = A'Pi + K'Y, -Sc (Sc += Y'Ru^-1 Y) and LINE (+= rs e'Pi)
  // in the accumulator layout (lane l, reg r <-> row (l >> 4) + 4r, column l & 15).  Because P is
  // symmetric, accumulator register s of D is already the A operand of the next stage's P G for k-step s,
  // and the Pi columns are already its B operand: the recursion stays in registers, one LDS read of the
  // stage window per k-step, no LDS round trip between products.  K, M, chol(Ru), Y and P e go to the
  // ring slot (written back by ring_wb as in factor()).  Stage 0 (controls s, u_0) runs factor()'s
  // dot-product steps on P, Pi, Sc, LINE flushed to LDS.  Same algebra as factor(); the summation order
  // inside an MFMA differs (rounding-level).
  static constexpr int CE = NX + NU, CP = CE + 1;   // H row / G column of rs e; first Pi column
  // A_cl = A + B K of stages N-1..1 is formed inside factor_mfma (acl_slot) and written back with the
  // stage's outputs (ring_wb<OK, OX>: K .. Pe, C (dead until vec rebuilds it), A_cl): no acl_pass re-reading A, B
  // and K from the stage records.  Per chain (bit NQ of VBOC_ACL_FUSED_NQ): the triple only - the fusion makes the
  // triple's data-generation launch 2.4 % faster (profiles/r04_bytes_ab.json) but the double's 10k launches 4.3 %
  // (dg loop) / 10.2 % (first solves) slower (profiles/r05_double_acl_ab.json).
#ifndef VBOC_ACL_FUSED_NQ
#define VBOC_ACL_FUSED_NQ (1 << 3)
#endif
  static constexpr bool ACL_FUSED = FM && ((VBOC_ACL_FUSED_NQ >> NQ) & 1);
  // factor_mfma's junk target: lanes without an output write the slot's tail past the written-back fields
  static constexpr int FJUNK = L::OX;
  static constexpr bool MFMA_OK = (NX <= 8) && (CP + NQ <= 16) && (FJUNK + 2 * NX + 2 <= L::RSF);
  // H_u rows NX .. NX+NU-1 live in accumulator registers HR0, HR0 + 1; the LDS image keeps those two
  // registers of every lane group: image row (row & 3) + 4 * ((row >> 2) - HR0)
  static constexpr int HR0 = NX >> 2;
  // RINV: factor_mfma stores Ru^-1 in closed form instead of chol(Ru) for the triple, vec's k_f reads it as such
  // (the factorisation -4.9 % cycles, profiles/r05_factor_loop_experiments.json).  A rounding-level change (round 3 /
  // 5 kept it off because a digest or one tolerance decision moved, profiles/r03z_rinv_ab.json); on since round 6
  // under the tolerance parity rule, with PFUSE above.  -DVBOC_RINV=0: the Cholesky form.
#ifndef VBOC_RINV
#define VBOC_RINV 1
#endif
  static constexpr bool RINV = VBOC_RINV && FM && NU == 3;
  static_assert(((NX + NU - 1) >> 2) <= HR0 + 1, "H_u spans two accumulator registers");
  __device__ __forceinline__ static constexpr int hrow(int row) { return (row & 3) + 4 * ((row >> 2) - HR0); }
  // The loop body is written for a low VALU count (the wave solver is VALU-issue bound): loop-invariant
  // per-lane masks are FP64 0/1 multipliers (no lane-mask SGPRs to spill), H_u goes through an LDS image
  // (no readlane / bpermute), and outputs a lane does not own land in the slot's junk tail [W_FAC, RSF)
  // (never written back) instead of behind an exec mask.
  // A_cl = A + B K of the stage held in factor slot `sl` (its window and the K just computed), into the slot's
  // A_cl field: one entry per lane, acl_pass's arithmetic and order (same bits)
  __device__ __forceinline__ void acl_slot(int sl) {
    const int kb = fslot(sl);
    // branch-free (lanes past NX * NX repeat the last entry: the same value to the same word; the exec-masked
    // block cost 5 % of the factorisation, profiles/r05_factor_loop_experiments.json), all operand reads before
    // the FMAs (one LDS latency)
    const int tt = t < NX * NX ? t : NX * NX - 1;
    const int q = tt / NX, i = tt - q * NX;
    double av = s[kb + OA + q * NX + i], bv[NU], kv[NU];
    UNR for (int c = 0; c < NU; ++c) { bv[c] = s[kb + OB + q * NU + c]; kv[c] = s[kb + OK + c * NX + i]; }
    __builtin_amdgcn_sched_barrier(0);
    UNR for (int c = 0; c < NU; ++c) av += bv[c] * kv[c];
    s[kb + OACL + tt] = av;
  }

  __device__ __forceinline__ bool factor_mfma() {
    static_assert(MFMA_OK, "stage blocks fit one 16x16 FP64 MFMA tile");
    fresh();
    // -DVBOC_PROF_SPLIT=4: sections of the stage loop (top / products / Cholesky / outputs) + the tail; =5: the top
    // split (write-back / DMA issue / ring wait / the rest of the stage) + the tail
#if defined(VBOC_PROF_SPLIT) && VBOC_PROF_SPLIT == 5
    constexpr int FSPL = 5;
#else
    constexpr int FSPL = 4;
#endif
#define FS4(i) if constexpr (FSPL == 4) { SPROF(i) }
#define FS5(i) if constexpr (FSPL == 5) { SPROF(i) }
    SPROF_DECL(FSPL)
    const int c = t & 15, g = t >> 4;
    constexpr int HS = L::XS;   // H_u image [8][16] (rows g and 4 + g of every lane group); XS is free here
    // initial state: P_N = diag(D_N), Pi = E' (velocity selection), Sc = 0, LINE = 0
    dbl4 Dm;
    UNR for (int r = 0; r < 4; ++r) {
      const int row = g + 4 * r;
      double v = 0.0;
      if (row < NX && c == row) v = st(N, OD + row);
      if (row < NX && c >= CP && c < CP + NQ && row == NQ + (c - CP)) v = 1.0;
      Dm[r] = v;
    }
    // FAC1: the window is the stage's inputs [A, K) (A, B, z .. lambda_u, e, D, DA): the outputs [K, A_cl] are
    // written into the slot by this sweep before the write-back; k_f and C keep stale slot words, which the record
    // holds only until the vector passes rewrite them (neither is read before)
    constexpr int WF = FAC1 ? L::W_FIN : L::W_FAC, P = (WF + 127) / 128;
    static_assert(!FAC1 || P == 1, "the factorisation's inputs fit one LDS-DMA");
    auto fdma = [&](int j) {
      const int kk = N - 1 - j >= 0 ? N - 1 - j : 0;
      UNR for (int part = 0; part < P; ++part) dma<1>(kk, 0, WF, fslot(j % L::NSF), part);
    };
    // loop-invariant per-lane constants.  A lane without a G / H operand reads the zeroed LDS words (ZERO,
    // absolute: slot base multiplier 0), never the slot's tail: the tail holds whatever the record's next
    // fields or an earlier problem left there, and a stale NaN / Inf times a 0 mask is NaN (a problem that
    // failed with non-finite iterates used to poison the next problem solved on the same workgroup region)
    int goff[2], gb[2];
    double gm[2];
    UNR for (int q = 0; q < 2; ++q) {
      const int row = 4 * q + g;
      int off = L::ZERO, b = 0;
      double m = 0.0;
      if (row < NX) {
        if (c < NX) { off = OA + row * NX + c; m = 1.0; b = 1; }
        else if (c < CE) { off = OB + row * NU + (c - NX); m = 1.0; b = 1; }
        else if (c == CE) { off = OE + row; m = rs; b = 1; }
      }
      goff[q] = off;
      gb[q] = b;
      gm[q] = m;
    }
    const int hoff = c < CE ? OD + c : L::ZERO, hb = c < CE ? 1 : 0;
    double hm[4], cm[4];
    UNR for (int r = 0; r < 4; ++r) {
      const int row = g + 4 * r;
      hm[r] = (c < CE && row == c) ? 1.0 : 0.0;
      cm[r] = (c >= CP && c < CP + NQ && (row == CE || (row >= CP && row < CP + NQ))) ? 1.0 : 0.0;
    }
    const double pim = (c >= CP && c < CP + NQ) ? 1.0 : 0.0;
    const bool zc = c < NX || (c >= CP && c < CP + NQ);
    double zm[NU];
    UNR for (int a = 0; a < NU; ++a) zm[a] = (zc && g == a) ? 1.0 : 0.0;
    // output addresses (slot-relative; lanes without that output write the junk tail)
    const int kofs = (g == 0 && c < NX) ? OK + c : FJUNK;
    const int mofs = (g == 0 && c >= CP && c < CP + NQ) ? OM + (c - CP) : FJUNK;
    const int pofs = (c == CE) ? OPE + g : FJUNK;
    int yofs = FJUNK, ysrc = HS;
    if (t < NU * NQ) {
      const int a = t / NQ, jj = t % NQ, row = NX + a;
      yofs = OY + t;
      ysrc = HS + hrow(row) * 16 + CP + jj;
    }
    __syncthreads();   // before any DMA is in flight: this barrier's fence would drain them
    settle();
    fdma(0);
    fdma(1);
    bool ok = true;
    auto wb_prev = [&](int j, int k) {
      if constexpr (ACL_FUSED) {
        acl_slot((j - 1) % L::NSF);                   // LDS ops of this wave run in order: the write-back's
        ring_wb<OK, L::OX>((j - 1) % L::NSF, k + 1);  // reads of the slot see them
      } else {
        ring_wb<OK, OC>((j - 1) % L::NSF, k + 1);
      }
    };
    for (int j = 0; j < N - 1; ++j) {
      const int k = N - 1 - j, kb = fslot(j % L::NSF);
      if (j >= 1) wb_prev(j, k);
      FS5(0)
      fdma(j + 2);
      FS5(1)
      vmwait<2 * P>();   // loads only, as in factor()
      FS4(0)
      FS5(2)
      // the three operand reads issue back to back (one LDS latency, not three)
      const double r0 = s[kb * gb[0] + goff[0]], r1 = s[kb * gb[1] + goff[1]], hv = s[kb * hb + hoff];
      double g0 = r0 * gm[0], g1 = r1 * gm[1];
      vreg(g0);
      vreg(g1);
      // P G (rows / columns of D beyond the stage blocks only meet zero rows of G)
      double p0 = Dm[0], p1 = Dm[1];
      vreg(p0);
      vreg(p1);
      dbl4 pg = {0.0, 0.0, 0.0, 0.0};
      pg = __builtin_amdgcn_mfma_f64_16x16x4f64(p0, g0, pg, 0, 0, 0);
      pg = __builtin_amdgcn_mfma_f64_16x16x4f64(p1, g1, pg, 0, 0, 0);
      // H = G' [PG | Pi] + diag(Hx, Hu) + carried LINE / -Sc
      dbl4 h = {0.0, 0.0, 0.0, 0.0};   // (every entry set below; the initialiser only quiets -Wuninitialized)
      UNR for (int r = 0; r < 4; ++r) h[r] = fma(Dm[r], cm[r], hv * hm[r]);
      double b0 = fma(Dm[0], pim, pg[0]), b1 = fma(Dm[1], pim, pg[1]);
      vreg(b0);
      vreg(b1);
      h = __builtin_amdgcn_mfma_f64_16x16x4f64(g0, b0, h, 0, 0, 0);
      h = __builtin_amdgcn_mfma_f64_16x16x4f64(g1, b1, h, 0, 0, 0);
      FS4(1)
      // H rows 4..11 -> LDS image; Ru (uniform) and this lane's column of H_u back
      s[HS + g * 16 + c] = h[HR0];
      if (HR0 + 1 < 4) s[HS + (4 + g) * 16 + c] = h[HR0 + 1 < 4 ? HR0 + 1 : 3];
      double Lm[NU * NU], id[NU], hu[NU];
      UNR for (int a = 0; a < NU; ++a) {
        const int ia = hrow(NX + a);
        UNR for (int b = 0; b <= a; ++b) {
          const double v = s[HS + ia * 16 + NX + b];
          Lm[a * NU + b] = v;
          Lm[b * NU + a] = v;
        }
        hu[a] = s[HS + ia * 16 + c];
      }
      // Y's image word is read with the H_u image, not after the stage's output stores (the compiler cannot tell
      // that those do not alias it, and waited on the read at the end of the stage: 2 % of k_dg, same results)
      const double yv = s[ysrc];
      double w[NU];
      if constexpr (RINV) {
        // Ru^-1 in closed form (adjugate / determinant): a dependent chain of ~14 FP64 ops instead of the
        // Cholesky's ~35; positive definiteness by Sylvester's criterion (the Cholesky's pivot test in exact
        // arithmetic).  K = -Ru^-1 S and the Schur update S' Ru^-1 S = hu' w use the same w.
        const double a = Lm[0], b = Lm[1], c = Lm[2], d = Lm[4], e = Lm[5], f = Lm[8];
        const double c00 = d * f - e * e, c01 = c * e - b * f, c02 = b * e - c * d;
        const double c11 = a * f - c * c, c12 = b * c - a * e, c22 = a * d - b * b;
        const double det = a * c00 + b * c01 + c * c02;
        ok = ok && (a > 0.0) && (c22 > 0.0) && (det > 0.0);
        double r = __builtin_amdgcn_rcp(det);
        UNR for (int it = 0; it < 2; ++it) r = fma(r, fma(-det, r, 1.0), r);
        Lm[0] = c00 * r; Lm[1] = Lm[3] = c01 * r; Lm[2] = Lm[6] = c02 * r;
        Lm[4] = c11 * r; Lm[5] = Lm[7] = c12 * r; Lm[8] = c22 * r;
        UNR for (int i = 0; i < NU; ++i) w[i] = Lm[i * NU] * hu[0] + Lm[i * NU + 1] * hu[1] + Lm[i * NU + 2] * hu[2];
        double zs = 0.0, ws = 0.0;
        UNR for (int i = 0; i < NU; ++i) { zs = fma(hu[i], zm[i], zs); ws = fma(w[i], zm[i], ws); }
        double nz = -zs;
        vreg(ws);
        vreg(nz);
        Dm = __builtin_amdgcn_mfma_f64_16x16x4f64(nz, ws, h, 0, 0, 0);
      } else {
      const bool okk = chol_inv<NU>(Lm, id);
      ok = ok && okk;
      double z[NU], zs = 0.0;
      UNR for (int a = 0; a < NU; ++a) {
        double tt = hu[a];
        UNR for (int b = 0; b < a; ++b) tt -= Lm[a * NU + b] * z[b];
        z[a] = tt * id[a];
        zs = fma(z[a], zm[a], zs);
      }
      double nz = -zs;
      vreg(zs);
      vreg(nz);
      Dm = __builtin_amdgcn_mfma_f64_16x16x4f64(nz, zs, h, 0, 0, 0);
      UNR for (int a = NU - 1; a >= 0; --a) {
        double tt = z[a];
        UNR for (int b = a + 1; b < NU; ++b) tt -= Lm[b * NU + a] * w[b];
        w[a] = tt * id[a];
      }
      }
      // the recursion's state update issues before the stage's outputs (they are off the critical path):
      // the empty asm keeps the MFMA from being sunk to the loop latch
      asm volatile("" : "+v"(Dm));
      FS4(2)
      // outputs of stage k into its ring slot: K = -Ru^-1 S, M = Ru^-1 Y, chol(Ru) (RINV: Ru^-1), Y, P e
      UNR for (int a = 0; a < NU; ++a) {
        s[kb + kofs + a * NX] = -w[a];
        s[kb + mofs + a * NQ] = w[a];
      }
      UNR for (int e = 0; e < NU * NU; ++e) s[kb + OLR + e] = Lm[e];
      s[kb + yofs] = yv;
      s[kb + pofs] = pg[0];
      s[kb + pofs + 4] = pg[1];
      lsync();
      FS4(3)
      FS5(3)
    }
    // flush P, Pi, Sc, LINE for stage 0 (factor()'s dot-product steps)
    UNR for (int r = 0; r < 4; ++r) {
      const int row = g + 4 * r;
      if (row < NX && c < NX) s[L::P + row * NX + c] = Dm[r];
      if (row < NX && c >= CP && c < CP + NQ) s[L::PI + row * NQ + (c - CP)] = Dm[r];
      if (row >= CP && row < CP + NQ && c >= CP && c < CP + NQ) s[L::SC + (row - CP) * NQ + (c - CP)] = -Dm[r];
      if (row == CE && c >= CP && c < CP + NQ) s[L::LINE + (c - CP)] = Dm[r];
    }
    lsync();
    {
      const int j = N - 1, kb = fslot(j % L::NSF);
      if (j >= 1) {
        if constexpr (ACL_FUSED) {
          acl_slot((j - 1) % L::NSF);
          ring_wb<OK, L::OX>((j - 1) % L::NSF, 1);
        } else {
          ring_wb<OK, OC>((j - 1) % L::NSF, 1);
        }
      }
      // stage 0's window was issued two sweeps ago (and the clamped repeats after it): retire all
      vmwait<0>();
      Dsc z1[RD], z2[RD], z4[RD];
      desc_s0(z1, z2, z4);
      dstep<NX, 0>(z1, kb);
      dstep<NX, 0>(z2, kb);
      int rb = L::ZERO, rstr = 0, db = L::TRASH + t, dstr = 0;
      if (t < NQ) { rb = L::Y0 + t; rstr = NQ; db = L::MM0 + t; dstr = NQ; }
      const bool ok0 = sstep<M0>(L::LR0, L::LR0, rb, rstr, db, dstr, 1.0);
      ok = ok && ok0;
      dstep<0, M0>(z4, kb);
      lsync();
    }
    __syncthreads();   // write-back visible to the next sweep's ring loads
    SPROF(4)
    SPROF_FLUSH
#undef FS4
#undef FS5
    return ok;
  }

  // closed-loop matrices A_cl = A + B K of stages 1..N-1 (row-major, OACL): formed once per
  // factorisation, stage-parallel, and shared by both vector passes (columns) and both forward
  // sweeps (rows) of the interior-point iteration
  __device__ __forceinline__ void acl_pass() {
    fresh();
    constexpr int NAB = (NX * NX + NX * NU) / 2, NKK = (NU * NX) / 2;
    for (int k = 1 + t; k < N; k += 64) {
      double ab[2 * NAB], kk[2 * NKK];
      ldr<OA, NAB>(k, ab);
      ldr<OK, NKK>(k, kk);
      __builtin_amdgcn_sched_barrier(0);
      gdbl2* dst = (gdbl2*)(g + (long long)k * REC + OACL);
      UNR for (int e = 0; e < NX * NX; e += 2) {
        double v[2];
        UNR for (int h2 = 0; h2 < 2; ++h2) {
          const int q = (e + h2) / NX, i = (e + h2) % NX;
          double a = ab[q * NX + i];
          UNR for (int c = 0; c < NU; ++c) a += ab[NX * NX + q * NU + c] * kk[c * NX + i];
          v[h2] = a;
        }
        dbl2 vv;
        vv.x = v[0];
        vv.y = v[1];
        dst[e / 2] = vv;
      }
    }
    __syncthreads();
  }

  // vector pass with the gradient in slot OG; leaves the stage-0 open-loop step w0 and the
  // terminal multiplier nu (wave-uniform).  False if S = sum Y'M is not positive definite.
  // c'_k = g_x + K'g_u + A_cl' PE_k of stage k from its gradient gv (the vector pass's constant) -> OC
  __device__ __forceinline__ void vec_const(int k, const double* gv) const {
    constexpr int NKK = (NU * NX) / 2;
    double kk[2 * NKK], ac[NX * NX], pe[NX];
    ldr<OK, NKK>(k, kk);
    ldr<OACL, NX * NX / 2>(k, ac);
    ldr<OPE, NX / 2>(k, pe);
    gdbl2* dst = (gdbl2*)(g + (long long)k * REC + OC);
    double cv[NX];
    UNR for (int i = 0; i < NX; ++i) {
      double c = gv[i];
      UNR for (int q = 0; q < NU; ++q) c += kk[q * NX + i] * gv[NX + q];
      UNR for (int q = 0; q < NX; ++q) c += ac[q * NX + i] * pe[q];
      cv[i] = c;
    }
    UNR for (int i = 0; i < NX; i += 2) {
      dbl2 vv;
      vv.x = cv[i];
      vv.y = cv[i + 1];
      dst[i / 2] = vv;
    }
  }
  // PRE == false: the constants c' are already in OC (CCORR: prep_corr formed them)
  template <int OG, bool PRE = true>
  __device__ __forceinline__ bool vec(double (&w0)[M0], double (&nun)[NQ]) {
    fresh();
    // p_k = c'_k + A_cl,k' p_{k+1},  c'_k = g_x + K'g_u + A_cl' PE_k  (lane i: row i of p);
    // v_k = PE_k + p_{k+1} is kept for k_f.  c' is formed stage-parallel first (-> OC).
    SPROF_DECL(2)
    if constexpr (PRE) {
      constexpr int NKK = (NU * NX) / 2;
      for (int k = 1 + t; k < N; k += 64) {
        Cov<OG, NZ> gg;   // the gradient slot only
        double kk[2 * NKK], ac[NX * NX], pe[NX];
        ldc(k, gg);
        ldr<OK, NKK>(k, kk);
        ldr<OACL, NX * NX / 2>(k, ac);
        ldr<OPE, NX / 2>(k, pe);
        __builtin_amdgcn_sched_barrier(0);
        constexpr int go = Cov<OG, NZ>::OFF;
        gdbl2* dst = (gdbl2*)(g + (long long)k * REC + OC);
        double cv[NX];
        UNR for (int i = 0; i < NX; ++i) {
          double c = gg.v[go + i];
          UNR for (int q = 0; q < NU; ++q) c += kk[q * NX + i] * gg.v[go + NX + q];
          UNR for (int q = 0; q < NX; ++q) c += ac[q * NX + i] * pe[q];
          cv[i] = c;
        }
        UNR for (int i = 0; i < NX; i += 2) {
          dbl2 vv;
          vv.x = cv[i];
          vv.y = cv[i + 1];
          dst[i / 2] = vv;
        }
      }
      __syncthreads();
    }
    SPROF(0)
    double pcur = st(N, OG + (t < NX ? t : NX - 1));
    if (t < NX) s[L::PV + t] = pcur;
    const int cnt = N - 1;   // stages N-1 .. 1
    __syncthreads();
    if constexpr (L::S_VEC > 1) {
      // grouped sweep: group G = stages [1 + G S, 1 + G S + S), walked from the top group down (sweep index
      // j = ng - 1 - G selects the ring slot); one DMA lands a group's windows [PE | C | ACL], DV groups ahead
      constexpr int S = L::S_VEC, W = L::W_VEC;
      const int ng = (cnt + S - 1) / S;
      const unsigned voff = grp_off<L::LO_VEC, W, S>();
      auto gdma = [&](int j) {
        const int G = ng - 1 - j >= 0 ? ng - 1 - j : 0;
        dma_s(g + (long long)(1 + G * S) * REC, voff, vslot(j & (L::NSV - 1)));
      };
      const int i = t < NX ? t : NX - 1;
      // v rows land in XS (lanes past NX write their own TRASH word: no exec-masked store in the chain)
      const int xm = t < NX ? NX : 0, xb = t < NX ? L::XS + t : L::TRASH + t;
      double pv[NX];
      UNR for (int q = 0; q < NX; ++q) pv[q] = rdlane(pcur, q);
      settle();
      if (ng >= 1) {
        UNR for (int d = 0; d < L::DV; ++d) gdma(d);
      }
      for (int j = 0; j < ng; ++j) {
        const int G = ng - 1 - j;
        gdma(j + L::DV);
        double acl[S][NX], cc[S], pe[S];
        vmwait<L::DV>();   // group j has landed (the DV younger DMAs stay in flight)
        const int kb = vslot(j & (L::NSV - 1));
        UNR for (int u = 0; u < S; ++u) {
          UNR for (int q = 0; q < NX; ++q) acl[u][q] = s[kb + u * W + (OACL - OPE) + q * NX + i];
          cc[u] = s[kb + u * W + (OC - OPE) + i];
          pe[u] = s[kb + u * W + i];
        }
        __builtin_amdgcn_sched_barrier(0);
        UNR for (int u = S - 1; u >= 0; --u) {
          const int k = 1 + G * S + u;
          if (k > cnt) continue;   // stages past N - 1 in the top group (wave-uniform)
          double p0 = cc[u], p1 = 0.0;
          UNR for (int q = 0; q < NX; q += 2) p0 += acl[u][q] * pv[q];
          UNR for (int q = 1; q < NX; q += 2) p1 += acl[u][q] * pv[q];
          s[xb + k * xm] = pe[u] + pcur;
          pcur = p0 + p1;
          UNR for (int q = 0; q < NX; ++q) pv[q] = rdlane(pcur, q);
        }
      }
    } else {
    // stage windows [PE | C | ACL] through the 8-slot LDS-DMA ring, DV stages ahead (sweep index j <->
    // stage N-1-j, clamped at 1): one DMA per stage, so DV - 1 are younger than the one waited for
    constexpr int PV = L::P_VEC;
    auto vdma = [&](int j) {
      const int kk = N - 1 - j >= 1 ? N - 1 - j : 1;
      UNR for (int part = 0; part < PV; ++part) dma<2>(kk, L::LO_VEC, L::W_VEC, vslot(j % L::NSV), part);
    };
    auto vld = [&](int kb, double (&acl)[NX], double& cc, double& pe) {
      const int i = t < NX ? t : NX - 1;
      UNR for (int q = 0; q < NX; ++q) acl[q] = s[kb + (OACL - OPE) + q * NX + i];
      cc = s[kb + (OC - OPE) + i];
      pe = s[kb + i];
    };
    double acl[NX], cc = 0.0, pe = 0.0;
    settle();
    if (cnt >= 1) {
      UNR for (int d = 0; d < L::DV; ++d) vdma(d);
      vmwait<(L::DV - 1) * PV>();
      vld(vslot(0), acl, cc, pe);
    }
    // p_{k+1} reaches every lane by readlane (lane q holds component q): the recursion's dependent chain
    // carries no LDS round trip
    double pv[NX];
    UNR for (int q = 0; q < NX; ++q) pv[q] = rdlane(pcur, q);
    for (int j = 0; j < cnt; ++j) {
      const int k = N - 1 - j;
      vdma(j + L::DV);
      vmwait<(L::DV - 1) * PV>();   // stage of sweep index j + 1 has landed
      double an[NX], cn, pn;
      vld(vslot((j + 1) % L::NSV), an, cn, pn);
      __builtin_amdgcn_sched_barrier(0);
      double p0 = cc, p1 = 0.0;
      UNR for (int q = 0; q < NX; q += 2) p0 += acl[q] * pv[q];
      UNR for (int q = 1; q < NX; q += 2) p1 += acl[q] * pv[q];
      if (t < NX) s[L::XS + k * NX + t] = pe + pcur;
      pcur = p0 + p1;
      UNR for (int q = 0; q < NX; ++q) pv[q] = rdlane(pcur, q);
      UNR for (int q = 0; q < NX; ++q) acl[q] = an[q];
      cc = cn;
      pe = pn;
    }
    }
    if (t < NX) s[L::PV + t] = pcur;
    __syncthreads();
    SPROF(1)
    // k_f = -Ru^-1 (g_u + B'v) per stage, lin = sum Y'k_f  (stage-parallel)
    double lin[NQ];
    UNR for (int j = 0; j < NQ; ++j) lin[j] = 0.0;
    constexpr int NBB = (NX * NU + 1) / 2, NLY = (OPE - (OLR & ~1) + 1) / 2;   // B; chol(Ru) (.. M, with the old order), Y
    for (int k = 1 + t; k < N; k += 64) {
      double bb[2 * NBB], ly[2 * NLY];
      Cov<OG + NX, NU> gg;   // g_u of the gradient slot
      ldr<OB, NBB>(k, bb);
      ldr<(OLR & ~1), NLY>(k, ly);
      ldc(k, gg);
      __builtin_amdgcn_sched_barrier(0);
      constexpr int LR_ = OLR - (OLR & ~1), Y_ = OY - (OLR & ~1);
      double r[NU], Lm[NU * NU];
      UNR for (int a = 0; a < NU; ++a) {
        double x = gg.v[gg.OFF + a];
        UNR for (int i = 0; i < NX; ++i) x += bb[i * NU + a] * s[L::XS + k * NX + i];
        r[a] = x;
      }
      UNR for (int e = 0; e < NU * NU; ++e) Lm[e] = ly[LR_ + e];
      if constexpr (RINV) {
        double q[NU];
        UNR for (int a = 0; a < NU; ++a) {
          q[a] = 0.0;
          UNR for (int b = 0; b < NU; ++b) q[a] += Lm[a * NU + b] * r[b];
        }
        UNR for (int a = 0; a < NU; ++a) r[a] = q[a];
      } else {
        chol_solve<NU>(Lm, r);
      }
      UNR for (int a = 0; a < NU; ++a) {
        r[a] = -r[a];
        st(k, OKF + a) = r[a];
      }
      UNR for (int j = 0; j < NQ; ++j)
        UNR for (int a = 0; a < NU; ++a) lin[j] += ly[Y_ + a * NQ + j] * r[a];
    }
    UNR for (int j = 0; j < NQ; ++j) lin[j] = wsum(lin[j]);
    SPROF(2)
    // stage 0 (every lane, identical)
    {
      double v[NX], Lm[M0 * M0];
      UNR for (int i = 0; i < NX; ++i) v[i] = s[L::PE0 + i] + s[L::PV + i];
      UNR for (int a = 0; a < M0; ++a) {
        double x = st(0, OG + a);
        UNR for (int i = 0; i < NX; ++i) x += s[L::F0 + i * M0 + a] * v[i];
        w0[a] = x;
      }
      UNR for (int e = 0; e < M0 * M0; ++e) Lm[e] = s[L::LR0 + e];
      chol_solve<M0>(Lm, w0);
      UNR for (int a = 0; a < M0; ++a) w0[a] = -w0[a];
      UNR for (int j = 0; j < NQ; ++j)
        UNR for (int a = 0; a < M0; ++a) lin[j] += s[L::Y0 + a * NQ + j] * w0[a];
    }
    double Sl[NQ * NQ];
    UNR for (int e = 0; e < NQ * NQ; ++e) Sl[e] = s[L::SC + e];
    const bool ok = chol<NQ>(Sl);
    UNR for (int j = 0; j < NQ; ++j) nun[j] = lin[j] + s[L::LINE + j] - rs * par(PF::E0N + j);
    chol_solve<NQ>(Sl, nun);
    __syncthreads();
    SPROF(3)
    SPROF_FLUSH
    return ok;
  }

  // forward sweep.  CORR == false: affine direction -> DA, returns the affine step and the mu_aff
  // polynomial; CORR == true: combined direction -> D, returns alpha_max.
  template <bool CORR>
  __device__ __forceinline__ void fwd(const double (&w0in)[M0], const double (&nun)[NQ], double smu, double& amax, double& c0,
                      double& c1, double& c2) {
    fresh();
    constexpr int OT = CORR ? OD : ODA;
    // -DVBOC_PROF_SPLIT=3: [stage 0, constant pass, recursion, step-length pass]; =6: the step-length pass's trips
    // [load issue, controls + stores, component tests, reductions, everything before the pass]
#if defined(VBOC_PROF_SPLIT) && VBOC_PROF_SPLIT == 6
    constexpr int WSPL = 6;
#else
    constexpr int WSPL = 3;
#endif
#define W3(i) if constexpr (WSPL == 3) { SPROF(i) }
#define W6(i) if constexpr (WSPL == 6) { SPROF(i) }
    SPROF_DECL(WSPL)
    {
      double w0[M0];
      UNR for (int a = 0; a < M0; ++a) {
        double x = w0in[a];
        UNR for (int j = 0; j < NQ; ++j) x -= s[L::MM0 + a * NQ + j] * nun[j];
        w0[a] = x;
      }
      if (t == 0) {
        UNR for (int i = 0; i < NZ; ++i) st(0, OT + i) = i < M0 ? w0[i < M0 ? i : 0] : 0.0;

      }
      if (t < NX) {
        double x = rs * st(0, OE + t);
        UNR for (int a = 0; a < M0; ++a) x += s[L::F0 + t * M0 + a] * w0[a];
        s[L::XS + NX + t] = x;
        s[L::DXV + t] = x;
      }
    }
    W3(0)
    // dx_{k+1} = c_k + A_cl,k dx_k,  c_k = rs e_k + B_k (k_f - M_k nu)  (lane i: row i); c is formed
    // stage-parallel first (-> OC)
    {
      constexpr int NBB = (NX * NU + 1) / 2, NFM = (OM + NU * NQ - OKF + 1) / 2;   // B; k_f .. the end of M
      for (int k = 1 + t; k < N; k += 64) {
        double e[NX], bb[2 * NBB], fm[2 * NFM];
        ldr<OE, NX / 2>(k, e);
        ldr<OB, NBB>(k, bb);
        ldr<OKF, NFM>(k, fm);
        __builtin_amdgcn_sched_barrier(0);
        double kfm[NU];
        UNR for (int a = 0; a < NU; ++a) {
          double x = fm[a];
          UNR for (int j = 0; j < NQ; ++j) x -= fm[(OM - OKF) + a * NQ + j] * nun[j];
          kfm[a] = x;
        }
        if constexpr (KFM) {
          UNR for (int a = 0; a < NU; ++a) st(k, OKF + a) = kfm[a];   // read by the step-length pass below
        }
        gdbl2* dst = (gdbl2*)(g + (long long)k * REC + OC);
        UNR for (int i = 0; i < NX; i += 2) {
          double v[2];
          UNR for (int h2 = 0; h2 < 2; ++h2) {
            double c = rs * e[i + h2];
            UNR for (int a = 0; a < NU; ++a) c += bb[(i + h2) * NU + a] * kfm[a];
            v[h2] = c;
          }
          dbl2 vv;
          vv.x = v[0];
          vv.y = v[1];
          dst[i / 2] = vv;
        }
      }
      __syncthreads();
    }
    W3(1)
    const int cnt = N - 1;   // stages 1 .. N-1
    __syncthreads();
    if constexpr (L::S_FWD > 1) {
      // grouped sweep (see vec): group j = stages [1 + j S, 1 + j S + S), windows [C | ACL]
      constexpr int S = L::S_FWD, W = L::W_FWD;
      const int ng = (cnt + S - 1) / S;
      const unsigned voff = grp_off<L::LO_FWD, W, S>();
      auto gdma = [&](int j) {
        const int G = j < ng ? j : ng - 1;
        dma_s(g + (long long)(1 + G * S) * REC, voff, vslot(j & (L::NSV - 1)));
      };
      const int i = t < NX ? t : NX - 1;
      const int xm = t < NX ? NX : 0, xb = t < NX ? L::XS + NX + t : L::TRASH + t;
      double dx[NX];
      UNR for (int q = 0; q < NX; ++q) dx[q] = s[L::DXV + q];
      settle();
      if (ng >= 1) {
        UNR for (int d = 0; d < L::DV; ++d) gdma(d);
      }
      for (int j = 0; j < ng; ++j) {
        gdma(j + L::DV);
        double acl[S][NX], cc[S];
        vmwait<L::DV>();   // group j has landed
        const int kb = vslot(j & (L::NSV - 1));
        UNR for (int u = 0; u < S; ++u) {
          UNR for (int q = 0; q < NX; ++q) acl[u][q] = s[kb + u * W + (OACL - OC) + i * NX + q];
          cc[u] = s[kb + u * W + i];
        }
        __builtin_amdgcn_sched_barrier(0);
        UNR for (int u = 0; u < S; ++u) {
          const int k = 1 + j * S + u;
          if (k > cnt) break;   // stages past N - 1 in the top group (wave-uniform)
          double p0 = cc[u], p1 = 0.0;
          UNR for (int q = 0; q < NX; q += 2) p0 += acl[u][q] * dx[q];
          UNR for (int q = 1; q < NX; q += 2) p1 += acl[u][q] * dx[q];
          const double dn = p0 + p1;
          s[xb + k * xm] = dn;
          UNR for (int q = 0; q < NX; ++q) dx[q] = rdlane(dn, q);
        }
      }
    } else {
    // stage windows [C | ACL] through the 8-slot LDS-DMA ring, DV stages ahead (sweep index j <-> stage
    // 1 + j, clamped at N - 1)
    constexpr int PW = L::P_FWD;
    auto wdma = [&](int j) {
      const int kk = 1 + j < N ? 1 + j : N - 1;
      UNR for (int part = 0; part < PW; ++part) dma<4>(kk, L::LO_FWD, L::W_FWD, vslot(j % L::NSV), part);
    };
    auto fld = [&](int kb, double (&acl)[NX], double& cc) {
      const int i = t < NX ? t : NX - 1;
      UNR for (int q = 0; q < NX; ++q) acl[q] = s[kb + (OACL - OC) + i * NX + q];
      cc = s[kb + i];
    };
    {
      double acl[NX], cc = 0.0;
      settle();
      if (cnt >= 1) {
        UNR for (int d = 0; d < L::DV; ++d) wdma(d);
        vmwait<(L::DV - 1) * PW>();
        fld(vslot(0), acl, cc);
      }
      // dx_k reaches every lane by readlane (lane q holds component q): no LDS round trip in the chain
      double dx[NX];
      UNR for (int q = 0; q < NX; ++q) dx[q] = s[L::DXV + q];
      for (int j = 0; j < cnt; ++j) {
        const int k = 1 + j;
        wdma(j + L::DV);
        vmwait<(L::DV - 1) * PW>();
        double an[NX], cn;
        fld(vslot((j + 1) % L::NSV), an, cn);
        __builtin_amdgcn_sched_barrier(0);
        double p0 = cc, p1 = 0.0;
        UNR for (int q = 0; q < NX; q += 2) p0 += acl[q] * dx[q];
        UNR for (int q = 1; q < NX; q += 2) p1 += acl[q] * dx[q];
        const double dn = p0 + p1;
        if (t < NX) s[L::XS + (k + 1) * NX + t] = dn;
        UNR for (int q = 0; q < NX; ++q) dx[q] = rdlane(dn, q);
        UNR for (int q = 0; q < NX; ++q) acl[q] = an[q];
        cc = cn;
      }
    }
    }
    __syncthreads();   // dx rows (global) visible to the stage-parallel pass
    W3(2)
    W6(4)
    // controls of the middle stages, then the step-length tests (stage-parallel)
    typename Lane<NQ>::MinRatio mr{1.0, CORR ? o.tau : 1.0};
    double a0 = 0.0, a1 = 0.0, a2 = 0.0;
    // K, k_f, chol(Ru), M: the range [OK, OY); KFM: K and k_f - M nu, the range [OK, OKF + NU)
    constexpr int NKM = KFM ? (OKF + NU - OK + 1) / 2 : (OY - OK + 1) / 2;
    for (int k = t; k <= N; k += 64) {
      IP r;
      double km[2 * NKM];
      Cov<ODA, NZ> da;   // the affine direction
      const int kk = (k > 0 && k < N) ? k : 1 < N ? 1 : 0;
      ld_ip(k, r);
      ldr<OK, NKM>(kk, km);
      if (CORR) ldc(k, da);
      __builtin_amdgcn_sched_barrier(0);
      W6(0)
      gdouble* rec = &g[(long long)k * REC];
      double d[NZ];
      if (k == 0) {
        UNR for (int i = 0; i < NZ; ++i) d[i] = rec[OT + i];   // written by lane 0 before the sweep
      } else {
        UNR for (int i = 0; i < NX; ++i) d[i] = s[L::XS + k * NX + i];
        UNR for (int a = 0; a < NU; ++a) {
          double x = 0.0;
          if (k < N) {
            x = km[OKF - OK + a];
            if constexpr (!KFM) {
              UNR for (int j = 0; j < NQ; ++j) x -= km[OM - OK + a * NQ + j] * nun[j];
            }
            UNR for (int i = 0; i < NX; ++i) x += km[a * NX + i] * d[i];
          }
          d[NX + a] = x;
        }
        UNR for (int i = 0; i < NZ; ++i) rec[OT + i] = d[i];
      }
      W6(1)
      UNR for (int i = 0; i < NZ; ++i) {
        const CS c = comp_r(r, k, i);
        if (!c.bx) continue;
        double dll, dlu;
        if (!CORR) {
          dll = -c.ql - c.ql * d[i] * c.itl;
          dlu = -c.qu + c.qu * d[i] * c.itu;
          a0 += c.tl * c.ql + c.tu * c.qu;
          a1 += c.tl * dll + d[i] * c.ql + c.tu * dlu - d[i] * c.qu;
          a2 += d[i] * dll - d[i] * dlu;
        } else {
          double rl, ru;
          corr_rhs(c, da.v[da.OFF + i], smu, rl, ru);
          dll = (rl - c.ql * d[i]) * c.itl;
          dlu = (ru + c.qu * d[i]) * c.itu;
        }
        mr.add(c.tl, d[i]);
        mr.add(c.tu, -d[i]);
        mr.add(c.ql, dll);
        mr.add(c.qu, dlu);
      }
      if constexpr (HC) {
        if (hc_on(k)) {
          double dtl, dtu, dql, dqu;
          hc_dir<CORR>(k, d, smu, dtl, dtu, dql, dqu);
          const double htl = hcr(k, HL::HTL), htu = hcr(k, HL::HTU), hql = hcr(k, HL::HQL), hqu = hcr(k, HL::HQU);
          if (!CORR) {
            hcr(k, HL::HATL) = dtl; hcr(k, HL::HATU) = dtu; hcr(k, HL::HAQL) = dql; hcr(k, HL::HAQU) = dqu;
            a0 += htl * hql + htu * hqu;
            a1 += htl * dql + dtl * hql + htu * dqu + dtu * hqu;
            a2 += dtl * dql + dtu * dqu;
          }
          mr.add(htl, dtl);
          mr.add(htu, dtu);
          mr.add(hql, dql);
          mr.add(hqu, dqu);
        }
      }
      W6(2)
    }
    amax = wmind(mr.value());
    c0 = wsum(a0); c1 = wsum(a1); c2 = wsum(a2);
    __syncthreads();
    W3(3)
    W6(3)
    SPROF_FLUSH
#undef W3
#undef W6
  }

  __device__ __forceinline__ void update(double alpha, double smu) {
    fresh();
    double musum = 0.0;
    for (int k = t; k <= N; k += 64) {
      IP r;
      double dd[2 * ((2 * NZ + 1) / 2)];   // D then DA
      ld_ip(k, r);
      ldr<OD, (2 * NZ + 1) / 2>(k, dd);
      __builtin_amdgcn_sched_barrier(0);
      gdouble* rec = &g[(long long)k * REC];
      IP rn;   // PFUSE: the updated iterate, for the next IPM iteration's D / DA
      if constexpr (PFUSE) rn = r;
      UNR for (int i = 0; i < NZ; ++i) {
        const CS c = comp_r(r, k, i);
        const double d = dd[i];
        const double dzn = c.dz + alpha * d;
        rec[ODZ + i] = dzn;
        if constexpr (PFUSE) rn.v[NZ + i] = dzn;
        if (!c.bx) continue;
        double rl, ru;
        corr_rhs(c, dd[NZ + i], smu, rl, ru);
        const double dll = (rl - c.ql * d) * c.itl, dlu = (ru + c.qu * d) * c.itu;
        const double qln = c.ql + alpha * dll, qun = c.qu + alpha * dlu;
        rec[OQL + i] = qln;
        rec[OQU + i] = qun;
        if constexpr (PFUSE) { rn.v[2 * NZ + i] = qln; rn.v[3 * NZ + i] = qun; }
        musum += (c.tl + alpha * d) * qln + (c.tu - alpha * d) * qun;
      }
      if constexpr (PFUSE) prep_from(rn, k, rec);
      if constexpr (HC) {
        if (hc_on(k)) {
          double dtl, dtu, dql, dqu;
          hc_dir<true>(k, dd, smu, dtl, dtu, dql, dqu);
          const double tl = hcr(k, HL::HTL) + alpha * dtl, tu = hcr(k, HL::HTU) + alpha * dtu;
          const double ql = hcr(k, HL::HQL) + alpha * dql, qu = hcr(k, HL::HQU) + alpha * dqu;
          hcr(k, HL::HTL) = tl; hcr(k, HL::HTU) = tu; hcr(k, HL::HQL) = ql; hcr(k, HL::HQU) = qu;
          musum += tl * ql + tu * qu;
        }
      }
    }
    mu = wsum(musum) / nbox;
    __syncthreads();
  }

  // costate recovery into the DA slot (x part) of stages 0..N-1
  __device__ __forceinline__ bool costate() {
    fresh();
    if constexpr (HC) {
      // the rows' c (lambda_u - lambda_l) term of each stage's costate constant -> the B field (free now)
      for (int k = 1 + t; k < N; k += 64) {
        const double m = hcr(k, HL::HQU) - hcr(k, HL::HQL);
        UNR for (int j = 0; j < NQ; ++j) st(k, OB + j) = hcr(k, HL::HG + j) * m;
      }
      __syncthreads();
    }
    bool fin = true;
    if (t < NX) {
      const int i = t;
      const double dz = st(N, ODZ + i);
      const double lam = o.lm * dz - st(N, OQL + i) + st(N, OQU + i) +
                         (i >= NQ ? par(PF::QNU + (i >= NQ ? i - NQ : 0)) : 0.0);
      s[L::XS + (N - 1) * NX + i] = lam;
      s[L::DXV + i] = lam;
      fin = isfinite(dz);
    }
    fin = __ballot(!fin) == 0ull;
    const int cnt = N - 1;   // stages N-1 .. 1
    __syncthreads();
    // stage windows [A, e) through the 8-slot LDS-DMA ring (sweep index j <-> stage N-1-j, clamped at 1)
    constexpr int PC = L::P_COS;
    auto cdma = [&](int j) {
      const int kk = N - 1 - j >= 1 ? N - 1 - j : 1;
      UNR for (int part = 0; part < PC; ++part) dma<8>(kk, 0, L::W_COS, vslot(j % L::NSV), part);
    };
    auto cterms = [&](int kb, double (&ac)[NX], double& cc) {
      const int i = t < NX ? t : NX - 1;
      cc = o.lm * s[kb + ODZ + i] - s[kb + OQL + i] + s[kb + OQU + i];
      if constexpr (HC) cc += i < NQ ? s[kb + OB + (i < NQ ? i : 0)] : 0.0;
      UNR for (int q = 0; q < NX; ++q) ac[q] = s[kb + OA + q * NX + i];
    };
    double ac[NX], cc = 0.0;
    settle();
    if (cnt >= 1) {
      UNR for (int d = 0; d < L::DV; ++d) cdma(d);
      vmwait<(L::DV - 1) * PC>();
      cterms(vslot(0), ac, cc);
    }
    for (int j = 0; j < cnt; ++j) {
      const int k = N - 1 - j;
      const int rb = L::DXV + (j & 1) * NX, wb = L::DXV + ((j + 1) & 1) * NX;
      cdma(j + L::DV);
      vmwait<(L::DV - 1) * PC>();
      double lam[NX], an[NX], cn;
      UNR for (int q = 0; q < NX; ++q) lam[q] = s[rb + q];
      cterms(vslot((j + 1) % L::NSV), an, cn);
      __builtin_amdgcn_sched_barrier(0);
      double p0 = cc, p1 = 0.0;
      UNR for (int q = 0; q < NX; q += 2) p0 += ac[q] * lam[q];
      UNR for (int q = 1; q < NX; q += 2) p1 += ac[q] * lam[q];
      const double x = p0 + p1;
      if (t < NX) {
        s[wb + t] = x;
        s[L::XS + (k - 1) * NX + t] = x;
      }
      UNR for (int q = 0; q < NX; ++q) ac[q] = an[q];
      cc = cn;
      lsync();
    }
    __syncthreads();   // drains the clamped tail DMAs before the ring is reused
    for (int k = t; k < N; k += 64) {
      UNR for (int i = 0; i < NX; ++i) st(k, ODA + i) = s[L::XS + k * NX + i];
    }
    __syncthreads();
    return fin;
  }

  // ---------------------------------------------------------------------------------------------
  // merit line search + update (stage-parallel)
  // ---------------------------------------------------------------------------------------------
  __device__ __forceinline__ void update_weights() {
    fresh();
    double lmax = 0.0;
    for (int k = t; k <= N; k += 64) {
      if (k < N) {
        UNR for (int i = 0; i < NX; ++i) st(k, OWPI + i) = Lane<NQ>::wupd(st(k, OWPI + i), st(k, ODA + i));
      }
      UNR for (int i = 0; i < NZ; ++i) lmax = fmax(lmax, fmax((double)st(k, OQL + i), (double)st(k, OQU + i)));
      if constexpr (HC) {
        if (hc_on(k)) lmax = fmax(lmax, fmax((double)hcr(k, HL::HQL), (double)hcr(k, HL::HQU)));
      }
    }
    lmax = wmaxd(lmax);
    if (t == 0) {
      UNR for (int j = 0; j < NQ; ++j) par(PF::WNU + j) = Lane<NQ>::wupd(par(PF::WNU + j), par(PF::QNU + j));
      par(PF::WBND) = Lane<NQ>::wupd(par(PF::WBND), lmax);
    }
    __syncthreads();
  }

  // forced inline: as a call (the UR5 instantiation is large enough for the inliner to refuse), the
  // kernel's arguments and the Coop state had to live in scratch behind flat pointers
  __device__ __forceinline__ double merit(double alpha) {
    fresh();
    const double h = par(PF::H);
    const double sv = par(PF::S) + alpha * st(0, ODZ);
    double val = 0.0, viol = 0.0;
    // The arm (NQ = 4) runs the stage trips with a wave-uniform trip count: lanes past N evaluate stage N
    // and discard it by select (same additions in the same order for the live lanes).  With the usual
    // `k = t; k <= N; k += 64` loop the last trip runs the rigid-body RK4 (~430 registers, SGPRs spilled to
    // VGPR lanes, VGPRs to AGPRs) under a partial exec mask, and that build returned wrong merit values on a
    // few problems per batch: longer line searches than the oracle's, 3 % SQP-iteration agreement
    // (profiles/r02p_ur5_merit_bisect.log).
    constexpr bool UNI = NQ == 4;
    for (int k0 = UNI ? 0 : t; k0 <= N; k0 += 64) {
      const bool live = !UNI || k0 + t <= N;
      const int k = UNI ? (live ? k0 + t : N) : k0;
      auto acc = [live](double& a, double x) { a = live ? a + x : a; };
      const gdouble* rec = &g[(long long)k * REC];
      UNR for (int i = 0; i < NZ; ++i) {
        double lb, ub;
        if (!box(k, i, lb, ub)) continue;
        const double v = rec[OZ + i] + alpha * rec[ODZ + i];
        acc(viol, fmax(0.0, lb - v) + fmax(0.0, v - ub));
      }
      if constexpr (HC) {
        if (hc_on(k)) {
          double xq[NQ];
          UNR for (int j = 0; j < NQ; ++j) xq[j] = rec[OZ + j] + alpha * rec[ODZ + j];
          const double hv = hc_eval(xq, nullptr);
          acc(viol, fmax(0.0, o.hlh - hv) + fmax(0.0, hv - o.huh));
        }
      }
      if (k > 0) {
        const gdouble* rp = &g[(long long)(k - 1) * REC];
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
          acc(val, rp[OWPI + i] * fabs(phi[i] - xn));
        }
        if (k == N) {
          UNR for (int j = 0; j < NQ; ++j)
            acc(val, par(PF::WNU + j) * fabs(rec[OZ + NQ + j] + alpha * rec[ODZ + NQ + j] - par(PF::VFIN + j)));
        }
      }
    }
    return par(PF::CS) * sv + par(PF::CCONST) + wsum(val) + par(PF::WBND) * wsum(viol);
  }

  __device__ __forceinline__ void apply(double alpha) {
    fresh();
    for (int k = t; k <= N; k += 64) {
      gdouble* rec = &g[(long long)k * REC];
      if (k == 0) {
        UNR for (int a = 0; a < NU; ++a) rec[OU + a] += alpha * rec[ODZ + 1 + a];
      } else {
        UNR for (int i = 0; i < NX; ++i) rec[OX + i] += alpha * rec[ODZ + i];
        if (k < N) {
          UNR for (int a = 0; a < NU; ++a) rec[OU + a] += alpha * rec[ODZ + NX + a];
        }
      }
      UNR for (int i = 0; i < NZ; ++i) {
        rec[OLL + i] += alpha * (rec[OQL + i] - rec[OLL + i]);
        rec[OLU + i] += alpha * (rec[OQU + i] - rec[OLU + i]);
      }
      if constexpr (HC) {
        if (hc_on(k)) {
          hcr(k, HL::HLL) += alpha * (hcr(k, HL::HQL) - hcr(k, HL::HLL));
          hcr(k, HL::HLU) += alpha * (hcr(k, HL::HQU) - hcr(k, HL::HLU));
        }
      }
      if (k < N) {
        UNR for (int i = 0; i < NX; ++i) rec[OPI + i] += alpha * (rec[ODA + i] - rec[OPI + i]);
      }
    }
    __syncthreads();
    if (t == 0) {
      par(PF::S) += alpha * st(0, ODZ);
      UNR for (int j = 0; j < NQ; ++j) par(PF::NU_ + j) += alpha * (par(PF::QNU + j) - par(PF::NU_ + j));
    }
    __syncthreads();
  }

  __device__ __forceinline__ void store(const Inputs& in, int pid, int status, int it, int qit) {
    fresh();
    constexpr int NXR = NX + 1;
    double* xo = in.xo + (long long)pid * (in.nmax + 1) * NXR;
    double* uo = in.uo + (long long)pid * in.nmax * NU;
    const double sv = par(PF::S), h = par(PF::H);
    for (int k = t; k <= N; k += 64) {
      UNR for (int i = 0; i < NX; ++i) {
        const double v = (k == 0) ? (i < NQ ? par(PF::Q0 + i) : sv * par(PF::DIR + (i - NQ + (i < NQ ? NQ : 0))))
                                  : (double)st(k, OX + i);
        xo[(long long)k * NXR + i] = v;
      }
      xo[(long long)k * NXR + NX] = h;
      if (k < N) {
        UNR for (int a = 0; a < NU; ++a) uo[(long long)k * NU + a] = st(k, OU + a);
      }
    }
    if (t == 0) {
      in.status[pid] = status;
      in.cost[pid] = par(PF::CS) * sv + par(PF::CCONST);
      in.sqp_iter[pid] = it;
      in.qp_iter[pid] = qit;
    }
  }

  // the remaining SQP of the loaded problem, to termination; returns the ACADOS status
  // PAUSE: stop with status -2 before SQP iteration pause_at; a second call resumes (every SQP iteration starts from
  // the stage records and LDS alone, as the cooperative tail's resumption does)
  template <bool PAUSE = false>
  __device__ __forceinline__ int run(int& it, int& qit) {
    for (int e = t; e < 16; e += 64) s[L::ZERO + e] = 0.0;
    __syncthreads();
    int status = -1;
    CPROF_DECL
    const int it0 = it;
    int qtot = 0;
    for (;;) {
      if constexpr (PAUSE) {
        if (it == pause_at) { status = -2; break; }
      }
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
        if (!PFUSE || qcur == 0) VREP(1, prep_pred());   // PFUSE: update() prepared the later iterations
        CPROF(2)
        bool okf;
        if constexpr (FM) VREP(2, okf = factor_mfma());
        else VREP(2, okf = factor());
        if constexpr (!ACL_FUSED) VREP(3, acl_pass());
        CPROF(3)
        bool okv;
        VREP(4, okv = vec<ODA>(w0, nun));
        CPROF(4)
        if (!(okf && okv)) { qst = -1; break; }
        double aa, c0, c1, c2;
        VREP(5, fwd<false>(w0, nun, 0.0, aa, c0, c1, c2));
        CPROF(5)
        const double muaff = (c0 + aa * (c1 + aa * c2)) / nbox;
        double sig = muaff / mu;
        sig = fmin(1.0, sig * sig * sig);
        const double smu = sig * mu;
        VREP(6, prep_corr(smu));
        CPROF(2)
        bool okc;
        VREP(7, (okc = vec<OD, !CCORR>(w0, nun)));
        if (!okc) { qst = -1; break; }
        CPROF(4)
        double amax;
        VREP(8, fwd<true>(w0, nun, smu, amax, c0, c1, c2));
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
      qtot += qcur;
      if (qst < 0 || !costate()) { status = 4; break; }
      CPROF(7)
      update_weights();
      double alpha = 1.0;
      const double phi0 = merit(0.0);
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
    CPROF_FLUSH(it - it0, qtot)
    (void)it0;
    return status;
  }
};


// Register budget of the wave kernel.  The pendulum chains run two waves per SIMD (<= 256 registers,
// eight problems per CU); they fit without spills only because every pass re-derives its lane-dependent
// values (Coop::fresh()).  The UR5 arm's rigid-body model alone needs ~430 registers (rk4_kernel<4>), so
// its instantiation runs one wave per SIMD (256 VGPRs + 256 AGPRs, no scratch): squeezed into 256 it spilled
// ~2000 VGPRs to scratch and the -O2/-O3 builds then produced wrong QP steps.
template <int NQ>
struct WavesPerEu { static constexpr int v = NQ <= 3 ? 2 : 1; };

// one workgroup = one wave = one problem at a time; workgroups pull jobs until none are left
// FM: the Riccati factorisation on FP64 MFMA (factor_mfma, NQ <= 3) instead of VALU dot-product steps
template <int NQ, bool FM, bool HC = false>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WavesPerEu<NQ>::v, WavesPerEu<NQ>::v)))
void k_wave(Work w, Opts o, Inputs in, SlotState ss, WaveJobs jb) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int t = (int)threadIdx.x;
  Coop<NQ, FM, HC> C(smem, gptr(jb.regions) + (long long)blockIdx.x * jb.region_doubles, w, o, t);
  if constexpr (HC) C.gh = gptr(jb.hc) + (long long)blockIdx.x * jb.hc_doubles;
  for (;;) {
    unsigned idx = 0;
    if (t == 0) idx = atomicAdd(jb.next, 1u);
    idx = (unsigned)__builtin_amdgcn_readfirstlane((int)__shfl((int)idx, 0));
    if (idx >= (unsigned)jb.count) break;
    int pid, it = 0, qit = 0;
    unsigned slot = 0;
    if (jb.list) {
      slot = (unsigned)__builtin_amdgcn_readfirstlane(jb.list[idx]);
      pid = ss(IS_PID, slot);
      it = ss(IS_IT, slot);
      qit = ss(IS_QIT, slot);
      C.from_slot(ss, slot);
    } else {
      pid = (int)idx;
      Lane<NQ> chk(w, o, 0u);
      if (!chk.supported(in, pid)) {
        if (t == 0) {
          in.status[pid] = 5;
          in.cost[pid] = NAN;
          in.sqp_iter[pid] = 0;
          in.qp_iter[pid] = 0;
          atomicAdd(ss.done, 1u);
        }
        continue;
      }
      if constexpr (HC) {
        // stage 0: positions fixed, h constant - outside [lh, uh]: status 4 without iterating (k_refill)
        double q0[NQ];
        UNR for (int j = 0; j < NQ; ++j) q0[j] = in.lbx0[(long long)pid * (2 * NQ + 1) + j];
        const double h0 = C.hc_eval(q0, nullptr);
        if (!(h0 >= o.hlh && h0 <= o.huh)) {
          if (t == 0) {
            in.status[pid] = 4;
            in.cost[pid] = NAN;
            in.sqp_iter[pid] = 0;
            in.qp_iter[pid] = 0;
            atomicAdd(ss.done, 1u);
          }
          continue;
        }
      }
      C.from_inputs(in, pid);
    }
    const int status = C.run(it, qit);
    C.store(in, pid, status, it, qit);
    __syncthreads();
    if (t == 0) {
      if (jb.list) {
        ss(IS_PID, slot) = -1;
        ss(IS_PH, slot) = 0;
      }
      atomicAdd(ss.done, 1u);
    }
  }
}

// compact the slots still iterating (phase 1 at a round boundary) into list[]
__global__ void k_list(SlotState ss, int* list, unsigned* cnt) {
  const unsigned slot = blockIdx.x * blockDim.x + threadIdx.x;
  if (ss(IS_PID, slot) >= 0 && ss(IS_PH, slot) == 1) list[atomicAdd(cnt, 1u)] = (int)slot;
}

}  // namespace vboc

// Does a partitioned recursion shorten k_dg's forward sweep?  (verdict r05 item 3: "prototype a within-wave
// partitioned Riccati ... A/B it ... commit the measurement".)  The forward sweep of the IPM is the affine recursion
// dx_{k+1} = c_k + A_cl,k dx_k over the N - 1 middle stages (coop.h fwd(); the vector pass is its transpose).  Its
// cost is a dependent chain of N steps per wave.  This probe isolates that chain: one problem per one-wave workgroup,
// the stage windows [c | A_cl] (42 doubles, the product's forward window) already in LDS, and it times the chain
// with the shader clock (clock64) in four forms:
//   seq_rl    the product's form: lane i owns row i, dx reaches every lane by readlane (coop.h fwd(), ungrouped)
//   seq_dpp   the product's form with the readlanes replaced by DPP row_newbcast (lane q of each row of 16 to the
//             row: no SGPR round trip)
//   seq_mov64 the same with one 64-bit DPP move per component (v_mov_b64_dpp row_newbcast)
//   seq_fdpp  the broadcast folded into the FMA: v_fmac_f64_dpp src0 row_newbcast:q (the product's arithmetic, in
//             the same order: bit-identical dx)
//   seq_red   every lane computes the whole dx = c + A dx from broadcast LDS reads (no cross-lane exchange)
//   part<P>   P segments of L = ceil(N / P) stages on P lane groups of 16.  Pass A: lane (s, j < 6) carries column
//             j of the segment's transition matrix Phi_s = A_{end-1} ... A_{start}, lane (s, 6) the segment's
//             response y_s from dx = 0 (segment 0 from the true dx_0: its rows are final); every lane of a group
//             forms A v (+ c on the y lane) from broadcast LDS reads, so no cross-lane exchange either.  Boundary:
//             x_{s+1} = y_s + Phi_s x_s for s = 1 .. P - 1 (every lane, redundantly).  Pass B: segments 1 .. P - 1
//             re-run from their true starts.  The chain is 2 L + P steps instead of N, at 6 x the flops of pass A.
// Results are checked against a sequential host recursion (re-associated: max relative error printed).
// Cycles are the shader clock between the chain's ends on lane 0, per problem, averaged; the wall time of the whole
// launch (1 024 one-wave workgroups = one wave per SIMD, the product's 1.3) is printed beside it.
//
// build: hipcc --offload-arch=gfx950 -O3 tools/probes/sweep_partition.hip -o tools/probes/sweep_partition
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int NX = 6, W = 42, N = 100, G = 1024, REPS = 8;

__device__ __forceinline__ double rdlane(double v, int lane) {
  const unsigned long long b = __double_as_longlong(v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, lane), hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), lane);
  return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

template <int Q>
__device__ __forceinline__ double rowbcast(double v) {
  const unsigned long long b = __double_as_longlong(v);
  const unsigned lo = __builtin_amdgcn_update_dpp(0u, (unsigned)b, 0x150 + Q, 0xF, 0xF, false);
  const unsigned hi = __builtin_amdgcn_update_dpp(0u, (unsigned)(b >> 32), 0x150 + Q, 0xF, 0xF, false);
  return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

template <int Q>
__device__ __forceinline__ double bc64(double v) { return __builtin_amdgcn_update_dpp(0.0, v, 0x150 + Q, 0xF, 0xF, false); }
// acc += (lane Q of the row's v) * a.  The first use after v is written waits the VALU -> DPP read hazard (2 states).
template <int Q, bool FIRST>
__device__ __forceinline__ void fmac_bc(double& acc, double a, double v) {
  if constexpr (FIRST)
    asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %2, %1 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(acc) : "v"(a), "v"(v), "i"(Q));
  else
    asm volatile("v_fmac_f64_dpp %0, %2, %1 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(a), "v"(v), "i"(Q));
}

// LDS: windows [N][W], then the dx rows [N + 1][NX], then (part) Phi / y per segment and the segment starts
__device__ __forceinline__ void load(double* s, const double* win, const double* dx0, int t) {
  const double* src = win + (size_t)blockIdx.x * N * W;
  for (int e = t; e < N * W; e += 64) s[e] = src[e];
  if (t < NX) s[N * W + t] = dx0[blockIdx.x * NX + t];
  __syncthreads();
}
__device__ __forceinline__ void finish(const double* s, double* out, long long* cyc, long long c0, long long c1, int t) {
  __syncthreads();
  for (int e = t; e < (N + 1) * NX; e += 64) out[(size_t)blockIdx.x * (N + 1) * NX + e] = s[N * W + e];
  if (t == 0) cyc[blockIdx.x] = c1 - c0;
}

__global__ __launch_bounds__(64) void seq_rl(const double* win, const double* dx0, double* out, long long* cyc) {
  extern __shared__ double s[];
  const int t = threadIdx.x, i = t < NX ? t : NX - 1;
  load(s, win, dx0, t);
  double dx[NX];
  _Pragma("unroll") for (int q = 0; q < NX; ++q) dx[q] = s[N * W + q];
  double a[NX], c = s[i];
  _Pragma("unroll") for (int q = 0; q < NX; ++q) a[q] = s[NX + i * NX + q];
  const long long c0 = clock64();
  for (int k = 0; k < N; ++k) {
    const int kn = k + 1 < N ? k + 1 : k;
    double an[NX], cn = s[kn * W + i];
    _Pragma("unroll") for (int q = 0; q < NX; ++q) an[q] = s[kn * W + NX + i * NX + q];
    double p0 = c, p1 = 0.0;
    _Pragma("unroll") for (int q = 0; q < NX; q += 2) p0 += a[q] * dx[q];
    _Pragma("unroll") for (int q = 1; q < NX; q += 2) p1 += a[q] * dx[q];
    const double dn = p0 + p1;
    if (t < NX) s[N * W + (k + 1) * NX + t] = dn;
    _Pragma("unroll") for (int q = 0; q < NX; ++q) dx[q] = rdlane(dn, q);
    _Pragma("unroll") for (int q = 0; q < NX; ++q) a[q] = an[q];
    c = cn;
  }
  const long long c1 = clock64();
  finish(s, out, cyc, c0, c1, t);
}

__global__ __launch_bounds__(64) void seq_mov64(const double* win, const double* dx0, double* out, long long* cyc) {
  extern __shared__ double s[];
  const int t = threadIdx.x, i = t < NX ? t : NX - 1;
  load(s, win, dx0, t);
  double dx[NX];
  _Pragma("unroll") for (int q = 0; q < NX; ++q) dx[q] = s[N * W + q];
  double a[NX], c = s[i];
  _Pragma("unroll") for (int q = 0; q < NX; ++q) a[q] = s[NX + i * NX + q];
  const long long c0 = clock64();
  for (int k = 0; k < N; ++k) {
    const int kn = k + 1 < N ? k + 1 : k;
    double an[NX], cn = s[kn * W + i];
    _Pragma("unroll") for (int q = 0; q < NX; ++q) an[q] = s[kn * W + NX + i * NX + q];
    double p0 = c, p1 = 0.0;
    _Pragma("unroll") for (int q = 0; q < NX; q += 2) p0 += a[q] * dx[q];
    _Pragma("unroll") for (int q = 1; q < NX; q += 2) p1 += a[q] * dx[q];
    const double dn = p0 + p1;
    if (t < NX) s[N * W + (k + 1) * NX + t] = dn;
    dx[0] = bc64<0>(dn); dx[1] = bc64<1>(dn); dx[2] = bc64<2>(dn);
    dx[3] = bc64<3>(dn); dx[4] = bc64<4>(dn); dx[5] = bc64<5>(dn);
    _Pragma("unroll") for (int q = 0; q < NX; ++q) a[q] = an[q];
    c = cn;
  }
  const long long c1 = clock64();
  finish(s, out, cyc, c0, c1, t);
}

__global__ __launch_bounds__(64) void seq_fdpp(const double* win, const double* dx0, double* out, long long* cyc) {
  extern __shared__ double s[];
  const int t = threadIdx.x, i = t < NX ? t : NX - 1;
  load(s, win, dx0, t);
  double dn = s[N * W + (t < NX ? t : 0)];   // lane q holds component q (lanes 0..5 of row 0)
  double a[NX], c = s[i];
  _Pragma("unroll") for (int q = 0; q < NX; ++q) a[q] = s[NX + i * NX + q];
  const long long c0 = clock64();
  for (int k = 0; k < N; ++k) {
    const int kn = k + 1 < N ? k + 1 : k;
    double an[NX], cn = s[kn * W + i];
    _Pragma("unroll") for (int q = 0; q < NX; ++q) an[q] = s[kn * W + NX + i * NX + q];
    double p0 = c, p1 = 0.0;
    fmac_bc<0, true>(p0, a[0], dn);
    fmac_bc<1, false>(p1, a[1], dn);
    fmac_bc<2, false>(p0, a[2], dn);
    fmac_bc<3, false>(p1, a[3], dn);
    fmac_bc<4, false>(p0, a[4], dn);
    fmac_bc<5, false>(p1, a[5], dn);
    dn = p0 + p1;
    if (t < NX) s[N * W + (k + 1) * NX + t] = dn;
    _Pragma("unroll") for (int q = 0; q < NX; ++q) a[q] = an[q];
    c = cn;
  }
  const long long c1 = clock64();
  finish(s, out, cyc, c0, c1, t);
}

__global__ __launch_bounds__(64) void seq_dpp(const double* win, const double* dx0, double* out, long long* cyc) {
  extern __shared__ double s[];
  const int t = threadIdx.x, i = t < NX ? t : NX - 1;
  load(s, win, dx0, t);
  double dx[NX];
  _Pragma("unroll") for (int q = 0; q < NX; ++q) dx[q] = s[N * W + q];
  double a[NX], c = s[i];
  _Pragma("unroll") for (int q = 0; q < NX; ++q) a[q] = s[NX + i * NX + q];
  const long long c0 = clock64();
  for (int k = 0; k < N; ++k) {
    const int kn = k + 1 < N ? k + 1 : k;
    double an[NX], cn = s[kn * W + i];
    _Pragma("unroll") for (int q = 0; q < NX; ++q) an[q] = s[kn * W + NX + i * NX + q];
    double p0 = c, p1 = 0.0;
    _Pragma("unroll") for (int q = 0; q < NX; q += 2) p0 += a[q] * dx[q];
    _Pragma("unroll") for (int q = 1; q < NX; q += 2) p1 += a[q] * dx[q];
    const double dn = p0 + p1;
    if (t < NX) s[N * W + (k + 1) * NX + t] = dn;
    dx[0] = rowbcast<0>(dn); dx[1] = rowbcast<1>(dn); dx[2] = rowbcast<2>(dn);
    dx[3] = rowbcast<3>(dn); dx[4] = rowbcast<4>(dn); dx[5] = rowbcast<5>(dn);
    _Pragma("unroll") for (int q = 0; q < NX; ++q) a[q] = an[q];
    c = cn;
  }
  const long long c1 = clock64();
  finish(s, out, cyc, c0, c1, t);
}

// v <- A_k v (+ c_k): the whole 6-vector on one lane, A and c from broadcast LDS reads
__device__ __forceinline__ void step_full(const double* w, double (&v)[NX], bool affine) {
  double r[NX];
  _Pragma("unroll") for (int i = 0; i < NX; ++i) {
    double p0 = affine ? w[i] : 0.0, p1 = 0.0;
    _Pragma("unroll") for (int q = 0; q < NX; q += 2) p0 += w[NX + i * NX + q] * v[q];
    _Pragma("unroll") for (int q = 1; q < NX; q += 2) p1 += w[NX + i * NX + q] * v[q];
    r[i] = p0 + p1;
  }
  _Pragma("unroll") for (int i = 0; i < NX; ++i) v[i] = r[i];
}

__global__ __launch_bounds__(64) void seq_red(const double* win, const double* dx0, double* out, long long* cyc) {
  extern __shared__ double s[];
  const int t = threadIdx.x;
  load(s, win, dx0, t);
  double dx[NX];
  _Pragma("unroll") for (int q = 0; q < NX; ++q) dx[q] = s[N * W + q];
  const long long c0 = clock64();
  for (int k = 0; k < N; ++k) {
    step_full(s + k * W, dx, true);
    if (t == 0)
      _Pragma("unroll") for (int q = 0; q < NX; ++q) s[N * W + (k + 1) * NX + q] = dx[q];
  }
  const long long c1 = clock64();
  finish(s, out, cyc, c0, c1, t);
}

template <int P>
__global__ __launch_bounds__(64) void part(const double* win, const double* dx0, double* out, long long* cyc) {
  extern __shared__ double s[];
  constexpr int L = (N + P - 1) / P;
  const int t = threadIdx.x, sg = t / 16 < P ? t / 16 : P - 1, j = t % 16;
  double* phi = s + N * W + (N + 1) * NX;   // [P][NX + 1][NX]: Phi_s columns, then y_s
  double* xs = phi + P * (NX + 1) * NX;      // [P][NX] segment starts
  load(s, win, dx0, t);
  const bool ylane = j == NX;
  double v[NX];
  _Pragma("unroll") for (int q = 0; q < NX; ++q) v[q] = ylane ? (sg == 0 ? s[N * W + q] : 0.0) : (q == j ? 1.0 : 0.0);
  const long long c0 = clock64();
  // pass A: the segment's transition matrix (lanes j < 6) and response (lane 6)
  for (int u = 0; u < L; ++u) {
    const int k = sg * L + u;
    if (k < N) {
      step_full(s + k * W, v, ylane);
      if (ylane && sg == 0)
        _Pragma("unroll") for (int q = 0; q < NX; ++q) s[N * W + (k + 1) * NX + q] = v[q];
    }
  }
  if (j <= NX && t / 16 < P)
    _Pragma("unroll") for (int q = 0; q < NX; ++q) phi[(sg * (NX + 1) + j) * NX + q] = v[q];
  __syncthreads();
  // boundary: x_1 = y_0 (segment 0 ran from dx_0), x_{s+1} = y_s + Phi_s x_s
  double x[NX];
  _Pragma("unroll") for (int q = 0; q < NX; ++q) x[q] = phi[(0 * (NX + 1) + NX) * NX + q];
  if (t < NX) xs[1 * NX + t] = x[t];
  for (int b = 1; b + 1 < P; ++b) {
    double r[NX];
    _Pragma("unroll") for (int q = 0; q < NX; ++q) {
      double a = phi[(b * (NX + 1) + NX) * NX + q];
      _Pragma("unroll") for (int c = 0; c < NX; ++c) a += phi[(b * (NX + 1) + c) * NX + q] * x[c];
      r[q] = a;
    }
    _Pragma("unroll") for (int q = 0; q < NX; ++q) x[q] = r[q];
    if (t < NX) xs[(b + 1) * NX + t] = x[t];
  }
  __syncthreads();
  // pass B: segments 1 .. P - 1 from their true starts (lane 6 of each group)
  _Pragma("unroll") for (int q = 0; q < NX; ++q) v[q] = xs[sg * NX + q];
  for (int u = 0; u < L; ++u) {
    const int k = sg * L + u;
    if (sg > 0 && k < N) {
      step_full(s + k * W, v, true);
      if (ylane)
        _Pragma("unroll") for (int q = 0; q < NX; ++q) s[N * W + (k + 1) * NX + q] = v[q];
    }
  }
  const long long c1 = clock64();
  finish(s, out, cyc, c0, c1, t);
}

typedef void (*kern_t)(const double*, const double*, double*, long long*);

int main() {
  std::vector<double> win((size_t)G * N * W), dx0((size_t)G * NX), ref((size_t)G * (N + 1) * NX);
  srand(7);
  auto rnd = [] { return (double)rand() / RAND_MAX - 0.5; };
  for (int b = 0; b < G; ++b) {
    for (int k = 0; k < N; ++k) {
      double* w = &win[((size_t)b * N + k) * W];
      _Pragma("unroll") for (int i = 0; i < NX; ++i) w[i] = 0.1 * rnd();
      _Pragma("unroll") for (int i = 0; i < NX; ++i)
        _Pragma("unroll") for (int q = 0; q < NX; ++q) w[NX + i * NX + q] = (i == q ? 0.95 : 0.0) + 0.05 * rnd();   // A_cl ~ 0.95 I
    }
    _Pragma("unroll") for (int q = 0; q < NX; ++q) dx0[b * NX + q] = rnd();
    double* r = &ref[(size_t)b * (N + 1) * NX];
    _Pragma("unroll") for (int q = 0; q < NX; ++q) r[q] = dx0[b * NX + q];
    for (int k = 0; k < N; ++k) {
      const double* w = &win[((size_t)b * N + k) * W];
      _Pragma("unroll") for (int i = 0; i < NX; ++i) {
        double a = w[i];
        _Pragma("unroll") for (int q = 0; q < NX; ++q) a += w[NX + i * NX + q] * r[k * NX + q];
        r[(k + 1) * NX + i] = a;
      }
    }
  }
  double *dw, *dx, *dout;
  long long* dc;
  (void)hipMalloc(&dw, win.size() * 8);
  (void)hipMalloc(&dx, dx0.size() * 8);
  (void)hipMalloc(&dout, ref.size() * 8);
  (void)hipMalloc(&dc, G * sizeof(long long));
  (void)hipMemcpy(dw, win.data(), win.size() * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(dx, dx0.data(), dx0.size() * 8, hipMemcpyHostToDevice);
  const size_t lds = (size_t)(N * W + (N + 1) * NX + 4 * (NX + 1) * NX + 4 * NX) * 8;
  struct K { const char* name; kern_t f; int chain; } ks[] = {
      {"seq_rl (product form)", seq_rl, N},
      {"seq_dpp", seq_dpp, N},
      {"seq_mov64", seq_mov64, N},
      {"seq_fdpp", seq_fdpp, N},
      {"seq_red", seq_red, N},
      {"part<2>", part<2>, 2 * ((N + 1) / 2) + 2},
      {"part<4>", part<4>, 2 * ((N + 3) / 4) + 4}};
  std::vector<double> out(ref.size());
  std::vector<long long> cyc(G);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (const K& k : ks) {
    float ms_best = 1e30f;
    double cyc_best = 1e300;
    for (int rep = 0; rep < REPS; ++rep) {
      (void)hipMemset(dout, 0, ref.size() * 8);
      (void)hipEventRecord(e0, 0);
      hipLaunchKernelGGL(k.f, dim3(G), dim3(64), lds, 0, dw, dx, dout, dc);
      (void)hipEventRecord(e1, 0);
      if (hipEventSynchronize(e1) != hipSuccess) { printf("launch failed\n"); return 1; }
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      (void)hipMemcpy(cyc.data(), dc, G * sizeof(long long), hipMemcpyDeviceToHost);
      double m = 0;
      for (long long c : cyc) m += (double)c / G;
      if (m < cyc_best) { cyc_best = m; ms_best = ms; }
    }
    (void)hipMemcpy(out.data(), dout, ref.size() * 8, hipMemcpyDeviceToHost);
    double err = 0;
    for (size_t e = 0; e < ref.size(); ++e) err = fmax(err, fabs(out[e] - ref[e]) / (1.0 + fabs(ref[e])));
    printf("{\"kernel\": \"%s\", \"N\": %d, \"chain_steps\": %d, \"cycles_per_sweep\": %.0f, \"cycles_per_stage\": %.1f, "
           "\"launch_ms\": %.4f, \"max_rel_err\": %.3g}\n",
           k.name, N, k.chain, cyc_best, cyc_best / N, ms_best, err);
  }
  return 0;
}

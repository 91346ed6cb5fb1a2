// The VBOC loop's NN fit on the device: Adam/MSE training of NeuralNetDIR (Linear-ReLU-Linear-ReLU-Linear-ReLU)
// with the reference's minibatch sampling and stop rule, one step = four kernels, `poll` steps per HIP graph.
//
// Reference: VBOC/triplependulum_vboc.py:415-466 (first fit: random.sample(range(n), 4096), MSE, Adam(lr 1e-3),
// val = 0.95 val + 0.05 loss, `while val > 1e-3 and it < it_max`), :526-556 (refits: 2048 rows from the old
// rows + 2048 from the new ones), my_nn.py:20-34 (the model), the double / pendulum twins.  What PyTorch runs
// there as ~40 small kernels per step (plus a host sync on loss.item()) is here:
//
//   k_fwd_bwd   the step's gate (val > stop && it < it_max); one extra workgroup draws the NEXT step's
//               minibatch, a uniform k-subset of each row range (Philox draws with rejection of repeats:
//               random.sample's set method; k_sample draws a fit's first one); 16 minibatch rows per other
//               workgroup (gathered from the feature rows): H1 = relu(x W0' + b0),
//               H2 = relu(H1 W1' + b1) and
//               dH1 = (dH2 W1) * [H1 > 0] on v_mfma_f32_16x16x4_f32 (exact f32, as the f32 GEMMs of PyTorch),
//               the output layer, the MSE gradient, per-workgroup partial gradients of every small parameter
//   k_dw1       dW1 = dH2' H1 (split over minibatch rows), plus the EMA / counter update of the reference's loop
//   k_adam      the partial sums reduced in a fixed order, torch.optim.Adam's update (single-tensor path),
//               W1 rewritten as the packed MFMA fragments of the next step's two products
//
// Every operand streamed from L2 / MALL (W1 twice, H1 and dH2 for dW1) is stored fragment-packed (pk()): a wave's
// B (or A) fragment of one 16 x 16 block is 1 KB contiguous, so each load instruction moves whole 256-B lines.
//
// Every reduction has a fixed order, so a HIP-graph replay equals the eager launch sequence bit for bit; a step
// whose gate is 0 changes nothing, so running up to `poll - 1` steps past the stop is exact.  Parameters are kept
// in padded buffers (hidden rounded up to a multiple of 64; padding rows / columns stay exactly zero).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/vboc_fit.h"

namespace {

typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int R2 = 16;        // minibatch rows per k_fwd_bwd workgroup
constexpr int TBL = 8192;     // sampler hash slots (>= 2 x the largest sample of one range)
constexpr int MAXK = 4096;    // largest sample of one range
constexpr int ROUNDS = 128;   // rejection rounds before the (never expected) sequential completion

struct State {
  double val, stop, beta;
  long long it, it_lim, step_t;
  unsigned long long draws, seed;
  int gate, err, pad0, pad1;
};

struct Args {
  float* P;                   // parameters: [W0 (HP x NIN) | b0 | b1 | w2 (HP each) | b2 (4) | W1 (HP x HP)]
  float* M;                   // Adam exp_avg, same layout
  float* V;                   // Adam exp_avg_sq
  float* Wf;                  // W1 packed as the forward product's B fragments: pk(j, k, HP / 16)
  float* Wb;                  // W1 packed as the backward product's B fragments: element W1[j][c] at pk(c, j, HP / 16)
  int* idx;                   // this step's minibatch row indices [Bt]
  int* idx_next;              // the next step's, drawn by the forward kernel's extra workgroup
  float* H1p;                 // H1 packed as dW1's B fragments: element H1[r][c] at pk(c, r, Bt / 16)
  float* dH2p;                // dH2 packed as dW1's A fragments: element dH2[r][j] at pk(j, r, Bt / 16)
  float* part;                // per-workgroup partials [Bt / R2][REC]
  float* dW1p;                // split partials of dW1 [S][HP][HP]
  State* st;
  const float* F;             // feature rows [n][ldF]: NIN inputs then the target
  long long n, n_new;
  int ldF, Bt, S;
  float lr;
};

template <int NIN, int HP>
struct Lay {
  static constexpr int W0 = 0, B0 = HP * NIN, B1 = B0 + HP, W2 = B1 + HP, B2 = W2 + HP, SMALL = B2 + 4;
  static constexpr int W1 = SMALL, TOTAL = W1 + HP * HP, REC = SMALL + 4, LOSS = SMALL;
};

__device__ __forceinline__ f4 mfma(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Fragment-packed storage: the 16 x 16 block (RB, CB) of a matrix read as MFMA fragments "lane (lr, lq) takes
// [16 RB + lr][16 CB + 4 lq + s], s = 0..3" is 1 KB, lane-major: one wave-instruction loads it whole.
__host__ __device__ __forceinline__ size_t pk(int R, int C, int ncb) {
  return ((size_t)((R >> 4) * ncb + (C >> 4)) * 64 + (R & 15) + 16 * ((C & 15) >> 2)) * 4 + (C & 3);
}

__device__ __forceinline__ void philox(unsigned (&c)[4], unsigned k0, unsigned k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
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

__device__ __forceinline__ unsigned hslot(unsigned v) { return (v * 2654435761u) >> 19; }

// find-or-insert v (stored as v + 1) in the LDS table; returns its slot.  The table never holds more than
// MAXK = TBL / 2 values, so the probe ends.
__device__ __forceinline__ int tbl_insert(unsigned* keys, unsigned v) {
  int h = hslot(v);
  for (;;) {
    const unsigned old = atomicCAS(&keys[h], 0u, v + 1);
    if (old == 0u || old == v + 1) return h;
    h = (h + 1) & (TBL - 1);
  }
}

__device__ __forceinline__ bool tbl_has(const unsigned* keys, unsigned v) {
  int h = hslot(v);
  for (;;) {
    const unsigned k = keys[h];
    if (k == 0u) return false;
    if (k == v + 1) return true;
    h = (h + 1) & (TBL - 1);
  }
}

constexpr int SNT = 256;            // sampler threads (one workgroup of the forward kernel's shape)
constexpr int SL = MAXK / SNT;      // sample slots per thread

// 64 KB: the hash table, then the owners (reused for the sequential completion's values and, in the complement
// path, the marks and the compaction counts once the owners are no longer needed)
struct SampLds {
  unsigned keys[TBL];
  union {
    unsigned own[TBL];
    unsigned pendv[MAXK];
    struct {
      unsigned char mark[2 * MAXK];
      int cnt[SNT];
    } c;
  } u;
  int npend;
};

// kk <= n / 2 distinct values of [0, n); slot p < kk (thread p % SNT, register p / SNT) gets vals[p / SNT].
// Round r: every pending slot draws, inserts, and claims its value with key (r << 12 | p); the smallest key
// (earliest round, then lowest slot) owns the value and the other claimants draw again - the set of
// random.sample's "draw, redraw while already selected" loop.  With at most half of [0, n) taken a slot is
// pending after ROUNDS rounds with probability < 2^-128; such slots then take the smallest free values.
__device__ __forceinline__ void sample_set(SampLds& L, unsigned n, int kk, unsigned long long step,
                                           unsigned long long seed, unsigned range, unsigned (&vals)[SL]) {
  const int tid = threadIdx.x;
  for (int i = tid; i < TBL; i += SNT) {
    L.keys[i] = 0u;
    L.u.own[i] = 0xFFFFFFFFu;
  }
  if (tid == 0) L.npend = 0;
  __syncthreads();
  const unsigned thr = (0u - n) % n;
  unsigned pend = 0u;       // bit u: slot tid + SNT u still needs a value
  int slot[SL];
#pragma unroll
  for (int u = 0; u < SL; ++u) {
    if (tid + SNT * u < kk) pend |= 1u << u;
    vals[u] = 0u;
    slot[u] = 0;
  }
  int any = 1;
  const unsigned k0 = (unsigned)seed, k1 = (unsigned)(seed >> 32) ^ (0x2545F491u + range);
  for (unsigned r = 0; r < ROUNDS && any; ++r) {
    // one Philox block per four slots and round (Lemire: a word below thr is rejected and the slot simply
    // stays pending)
    unsigned drew = 0u;
#pragma unroll
    for (int q = 0; q < SL / 4; ++q) {
      if ((pend >> (4 * q)) & 15u) {
        unsigned c[4] = {(unsigned)step, (unsigned)(step >> 32), (unsigned)(tid + SNT * q), r};
        philox(c, k0, k1);
#pragma unroll
        for (int x = 0; x < 4; ++x) {
          const int u = 4 * q + x;
          if ((pend >> u) & 1u) {
            const unsigned long long m = (unsigned long long)c[x] * n;
            if ((unsigned)m >= thr) {
              vals[u] = (unsigned)(m >> 32);
              slot[u] = tbl_insert(L.keys, vals[u]);
              atomicMin(&L.u.own[slot[u]], (r << 12) | (unsigned)(tid + SNT * u));
              drew |= 1u << u;
            }
          }
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < SL; ++u)
      if (((drew >> u) & 1u) && L.u.own[slot[u]] == ((r << 12) | (unsigned)(tid + SNT * u))) pend &= ~(1u << u);
    any = __syncthreads_or(pend != 0u);
  }
  if (!any) return;
  // sequential completion: each still-pending slot gets a ticket (kept in slot[]), thread 0 hands out the
  // smallest free values in ticket order
#pragma unroll
  for (int u = 0; u < SL; ++u)
    if ((pend >> u) & 1u) slot[u] = atomicAdd(&L.npend, 1);
  __syncthreads();
  if (tid == 0) {
    unsigned v = 0;
    for (int i = 0; i < L.npend; ++i) {
      while (tbl_has(L.keys, v)) ++v;
      tbl_insert(L.keys, v);
      L.u.pendv[i] = v;
    }
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < SL; ++u)
    if ((pend >> u) & 1u) vals[u] = L.u.pendv[slot[u]];
  __syncthreads();
}

// indices of one range [lo, lo + n) into out[off, off + kk)
__device__ void sample_range(SampLds& L, const Args& a, int* out, long long lo, unsigned n, int kk, int off,
                             unsigned long long step, unsigned range) {
  const int tid = threadIdx.x;
  const unsigned long long seed = a.st->seed;
  unsigned vals[SL];
  if (2 * (long long)kk <= (long long)n) {
    sample_set(L, n, kk, step, seed, range, vals);
#pragma unroll
    for (int u = 0; u < SL; ++u) {
      const int p = tid + SNT * u;
      if (p < kk) out[off + p] = (int)(lo + vals[u]);
    }
    __syncthreads();
    return;
  }
  // kk > n / 2 (then n <= 2 MAXK): draw the n - kk rows left out, keep the others in increasing order
  const int nc = (int)n - kk;
  if (nc > 0) sample_set(L, n, nc, step, seed, range, vals);
  __syncthreads();
  for (int i = tid; i < (int)n; i += SNT) L.u.c.mark[i] = 0;
  __syncthreads();
  if (nc > 0) {
#pragma unroll
    for (int u = 0; u < SL; ++u)
      if (tid + SNT * u < nc) L.u.c.mark[vals[u]] = 1;
  }
  __syncthreads();
  // block compaction: thread t owns values [VT t, VT t + VT)
  constexpr int VT = 2 * MAXK / SNT;
  int c = 0;
  for (int q = 0; q < VT; ++q) {
    const int v = VT * tid + q;
    if (v < (int)n && !L.u.c.mark[v]) ++c;
  }
  L.u.c.cnt[tid] = c;
  __syncthreads();
  for (int d = 1; d < SNT; d <<= 1) {
    const int add = tid >= d ? L.u.c.cnt[tid - d] : 0;
    __syncthreads();
    L.u.c.cnt[tid] += add;
    __syncthreads();
  }
  int pos = L.u.c.cnt[tid] - c;
  for (int q = 0; q < VT; ++q) {
    const int v = VT * tid + q;
    if (v < (int)n && !L.u.c.mark[v]) out[off + pos++] = (int)(lo + v);
  }
  __syncthreads();
}

// one minibatch into `out`: draw number st->draws of the sampler's stream (then st->draws + 1)
__device__ __forceinline__ void sample_minibatch(SampLds& L, const Args& a, int* out) {
  State* st = a.st;
  const unsigned long long step = st->draws;
  __syncthreads();
  if (a.n_new == 0) {
    sample_range(L, a, out, 0, (unsigned)a.n, a.Bt, 0, step, 0u);
  } else {
    const long long n_old = a.n - a.n_new;
    sample_range(L, a, out, 0, (unsigned)n_old, a.Bt / 2, 0, step, 1u);
    sample_range(L, a, out, n_old, (unsigned)a.n_new, a.Bt / 2, a.Bt / 2, step, 2u);
  }
  if (threadIdx.x == 0) st->draws = step + 1;
}

// the first minibatch of a fit (and the test hook vboc_fit_sample), into a.idx
__global__ __launch_bounds__(SNT) void k_sample(Args a) {
  __shared__ SampLds L;
  sample_minibatch(L, a, a.idx);
}

// acc[u] += A[16 rows][HP] (LDS, row stride LD) x B' for the column tile 16 (w + 4u) .. +15, B [HP][HP] given
// fragment-packed (pk(j, k, HP / 16), row j = output column j).  MFMA step s of group t sums k = 16t + 4 lq + s.  Two register sets
// of B fragments alternate (group t + 1's loads are in flight while group t's MFMAs issue); no copies between
// them, so the compiler's waits stay one group behind the loads.
template <int NT, int LD>
__device__ __forceinline__ void mfma_group(const float* A, int t, int lr, int lq, const f4 (&bv)[NT],
                                           f4 (&acc)[NT]) {
  const f4 av = *(const f4*)&A[lr * LD + 16 * t + 4 * lq];
#pragma unroll
  for (int u = 0; u < NT; ++u) {
    acc[u] = mfma(av.x, bv[u].x, acc[u]);
    acc[u] = mfma(av.y, bv[u].y, acc[u]);
    acc[u] = mfma(av.z, bv[u].z, acc[u]);
    acc[u] = mfma(av.w, bv[u].w, acc[u]);
  }
}

template <int HP, int NT, int LD>
__device__ __forceinline__ void gemm_rows(const float* A, const float* B, int w, int lane, int lr, int lq,
                                          f4 (&acc)[NT]) {
  constexpr int TG = HP / 16;   // even for every instantiation (HP a multiple of 64)
  const float* bp[NT];
#pragma unroll
  for (int u = 0; u < NT; ++u) bp[u] = B + ((size_t)(w + 4 * u) * TG * 64 + lane) * 4;
  f4 b0[NT], b1[NT];
#pragma unroll
  for (int u = 0; u < NT; ++u) b0[u] = *(const f4*)bp[u];
  static_assert(TG % 2 == 0, "column groups come in pairs");
  for (int t = 0; t < TG; t += 2) {
#pragma unroll
    for (int u = 0; u < NT; ++u) b1[u] = *(const f4*)(bp[u] + 256 * (t + 1));
    mfma_group<NT, LD>(A, t, lr, lq, b0, acc);
    if (t + 2 < TG) {
#pragma unroll
      for (int u = 0; u < NT; ++u) b0[u] = *(const f4*)(bp[u] + 256 * (t + 2));
    }
    mfma_group<NT, LD>(A, t + 1, lr, lq, b1, acc);
  }
}

template <int NIN, int HP>
__global__ __launch_bounds__(256) void k_fwd_bwd(Args a) {
  using Ly = Lay<NIN, HP>;
  constexpr int NT = HP / 64;          // 16-column tiles per wave
  constexpr int LD = HP + 4;
  struct FwdLds {
    float H1[R2 * LD];
    float G2[R2 * LD];
    float xs[R2 * NIN], ys[R2], dout[R2], sq[R2], red[4][R2];
  };
  __shared__ __attribute__((aligned(16))) union {
    FwdLds f;
    SampLds s;
  } U;
  float* H1 = U.f.H1;
  float* G2 = U.f.G2;
  float* xs = U.f.xs;
  float* ys = U.f.ys;
  float* dout = U.f.dout;
  float* sq = U.f.sq;
  float (*red)[R2] = U.f.red;
  // the step's gate (the reference's `while val > stop and it < it_max`), from the state the previous step left;
  // block 0 publishes it for this step's dW1 / Adam kernels and the host's poll
  const State* sc = a.st;
  const int gate = (sc->val > sc->stop) && (sc->it < sc->it_lim);
  if (blockIdx.x == 0 && threadIdx.x == 0) a.st->gate = gate;
  if (!gate) return;
  // the last workgroup draws the next step's minibatch (it reads nothing this step writes)
  if ((int)blockIdx.x == a.Bt / R2) {
    sample_minibatch(U.s, a, a.idx_next);
    return;
  }
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, lr = lane & 15, lq = lane >> 4;
  const int row0 = blockIdx.x * R2;
  const float* P = a.P;
  // the workgroup's minibatch rows, gathered from the feature matrix
  if (tid < R2 * (NIN + 1)) {
    const int r = tid / (NIN + 1), i = tid % (NIN + 1);
    const float v = a.F[(size_t)a.idx[row0 + r] * a.ldF + i];
    if (i < NIN) xs[r * NIN + i] = v;
    else ys[r] = v;
  }
  __syncthreads();

  // H1 = relu(x W0' + b0), kept in LDS and written transposed for dW1
  for (int c = tid; c < HP; c += 256) {
    float wc[NIN];
#pragma unroll
    for (int i = 0; i < NIN; ++i) wc[i] = P[Ly::W0 + c * NIN + i];
    const float bc = P[Ly::B0 + c];
    float h[R2];
#pragma unroll
    for (int r = 0; r < R2; ++r) {
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < NIN; ++i) s = fmaf(xs[r * NIN + i], wc[i], s);
      h[r] = fmaxf(s + bc, 0.f);
      H1[r * LD + c] = h[r];
    }
    f4* dst = (f4*)(a.H1p + pk(c, row0, a.Bt / 16));
#pragma unroll
    for (int q = 0; q < 4; ++q) dst[16 * q] = f4{h[4 * q], h[4 * q + 1], h[4 * q + 2], h[4 * q + 3]};
  }
  __syncthreads();

  // A2 = H1 W1' on MFMA: wave w owns column tiles w, w + 4, ...; MFMA step s of group t sums k = 16t + 4 lq + s
  f4 acc[NT];
#pragma unroll
  for (int u = 0; u < NT; ++u) acc[u] = f4{0.f, 0.f, 0.f, 0.f};
  gemm_rows<HP, NT, LD>(H1, a.Wf, w, lane, lr, lq, acc);
  // acc[u][g] = A2[row 4 lq + g][col 16 (w + 4u) + lr]; H2 = relu(A2 + b1); output partial sums
  float op[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < NT; ++u) {
    const int j = 16 * (w + 4 * u) + lr;
    const float bj = P[Ly::B1 + j], wj = P[Ly::W2 + j];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float h = fmaxf(acc[u][g] + bj, 0.f);
      acc[u][g] = h;
      op[g] = fmaf(h, wj, op[g]);
    }
  }
#pragma unroll
  for (int g = 0; g < 4; ++g) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) op[g] += __shfl_xor(op[g], o);
  }
  if (lr == 0) {
#pragma unroll
    for (int g = 0; g < 4; ++g) red[w][4 * lq + g] = op[g];
  }
  __syncthreads();
  if (tid < R2) {
    const float s = ((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid];
    const float o = fmaxf(s + P[Ly::B2], 0.f);
    const float e = o - ys[tid];
    dout[tid] = o > 0.f ? e * (2.f / (float)a.Bt) : 0.f;     // d mean((o - y)^2) / d o, through the last ReLU
    sq[tid] = e * e;
  }
  __syncthreads();

  float* part = a.part + (size_t)blockIdx.x * Ly::REC;
  float dr[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) dr[g] = dout[4 * lq + g];
  // dH2 = dout w2 [H2 > 0]; db1 and dw2 partials; dH2 to LDS and transposed to global
#pragma unroll
  for (int u = 0; u < NT; ++u) {
    const int j = 16 * (w + 4 * u) + lr;
    const float wj = P[Ly::W2 + j];
    float gv[4], sb = 0.f, sw = 0.f;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float h = acc[u][g];
      gv[g] = h > 0.f ? dr[g] * wj : 0.f;
      sb += gv[g];
      sw = fmaf(dr[g], h, sw);
      G2[(4 * lq + g) * LD + j] = gv[g];
    }
    *(f4*)(a.dH2p + pk(j, row0 + 4 * lq, a.Bt / 16)) = f4{gv[0], gv[1], gv[2], gv[3]};
    sb += __shfl_xor(sb, 16);
    sb += __shfl_xor(sb, 32);
    sw += __shfl_xor(sw, 16);
    sw += __shfl_xor(sw, 32);
    if (lq == 0) {
      part[Ly::B1 + j] = sb;
      part[Ly::W2 + j] = sw;
    }
  }
  if (tid == 0) {
    float s = 0.f, l = 0.f;
    for (int r = 0; r < R2; ++r) {
      s += dout[r];
      l += sq[r];
    }
    part[Ly::B2] = s;
    part[Ly::B2 + 1] = 0.f;
    part[Ly::B2 + 2] = 0.f;
    part[Ly::B2 + 3] = 0.f;
    part[Ly::LOSS] = l;
  }
  __syncthreads();

  // dH1 = dH2 W1 [H1 > 0] on MFMA (B operand W1[j][c], packed in Wb); db0 and dW0 partials
#pragma unroll
  for (int u = 0; u < NT; ++u) acc[u] = f4{0.f, 0.f, 0.f, 0.f};
  gemm_rows<HP, NT, LD>(G2, a.Wb, w, lane, lr, lq, acc);
#pragma unroll
  for (int u = 0; u < NT; ++u) {
    const int c = 16 * (w + 4 * u) + lr;
    float sb = 0.f, sw[NIN];
#pragma unroll
    for (int i = 0; i < NIN; ++i) sw[i] = 0.f;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int r = 4 * lq + g;
      const float gg = H1[r * LD + c] > 0.f ? acc[u][g] : 0.f;
      sb += gg;
#pragma unroll
      for (int i = 0; i < NIN; ++i) sw[i] = fmaf(gg, xs[r * NIN + i], sw[i]);
    }
    sb += __shfl_xor(sb, 16);
    sb += __shfl_xor(sb, 32);
#pragma unroll
    for (int i = 0; i < NIN; ++i) {
      sw[i] += __shfl_xor(sw[i], 16);
      sw[i] += __shfl_xor(sw[i], 32);
    }
    if (lq == 0) {
      part[Ly::B0 + c] = sb;
#pragma unroll
      for (int i = 0; i < NIN; ++i) part[Ly::W0 + c * NIN + i] = sw[i];
    }
  }
}

// dW1 partials: workgroup = 64 x 64 output block x one of S row splits; wave = 32 x 32 (2 x 2 MFMA tiles).
// Block 0's first wave also applies the reference's loop update: val = beta val + (1 - beta) loss, it += 1.
template <int NIN, int HP>
__global__ __launch_bounds__(256) void k_dw1(Args a) {
  using Ly = Lay<NIN, HP>;
  State* st = a.st;
  if (!st->gate) return;
  constexpr int NB = HP / 64;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, lr = lane & 15, lq = lane >> 4;
  const int s = blockIdx.x / (NB * NB), b = blockIdx.x % (NB * NB);
  const int j0 = (b / NB) * 64 + (w >> 1) * 32, c0 = (b % NB) * 64 + (w & 1) * 32;
  const int KC = a.Bt / a.S, r0 = s * KC;
  f4 acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) acc[x][y] = f4{0.f, 0.f, 0.f, 0.f};
  const int RG = a.Bt / 16;
  const float* A0 = a.dH2p + ((size_t)((j0 >> 4) * RG + (r0 >> 4)) * 64 + lane) * 4;
  const float* A1 = A0 + (size_t)RG * 256;
  const float* B0 = a.H1p + ((size_t)((c0 >> 4) * RG + (r0 >> 4)) * 64 + lane) * 4;
  const float* B1 = B0 + (size_t)RG * 256;
  auto group = [&](const f4 (&av)[2], const f4 (&bv)[2]) {
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y) {
        acc[x][y] = mfma(av[x].x, bv[y].x, acc[x][y]);
        acc[x][y] = mfma(av[x].y, bv[y].y, acc[x][y]);
        acc[x][y] = mfma(av[x].z, bv[y].z, acc[x][y]);
        acc[x][y] = mfma(av[x].w, bv[y].w, acc[x][y]);
      }
  };
  // ping-pong register sets, as gemm_rows
  f4 a0[2] = {*(const f4*)A0, *(const f4*)A1}, b0[2] = {*(const f4*)B0, *(const f4*)B1};
  f4 a1[2], b1[2];
  const int T = KC / 16;
  for (int t = 0; t < T; t += 2) {
    const int o1 = 256 * (t + 1), o2 = 256 * (t + 2);
    const bool odd = t + 1 < T;
    if (odd) {
      a1[0] = *(const f4*)(A0 + o1);
      a1[1] = *(const f4*)(A1 + o1);
      b1[0] = *(const f4*)(B0 + o1);
      b1[1] = *(const f4*)(B1 + o1);
    }
    group(a0, b0);
    if (t + 2 < T) {
      a0[0] = *(const f4*)(A0 + o2);
      a0[1] = *(const f4*)(A1 + o2);
      b0[0] = *(const f4*)(B0 + o2);
      b0[1] = *(const f4*)(B1 + o2);
    }
    if (odd) group(a1, b1);
  }
  float* out = a.dW1p + (size_t)s * HP * HP;
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int g = 0; g < 4; ++g) out[(size_t)(j0 + 16 * x + 4 * lq + g) * HP + c0 + 16 * y + lr] = acc[x][y][g];
  if (blockIdx.x == 0 && w == 0) {
    const int nb = a.Bt / R2;
    float l = 0.f;
    for (int q = lane; q < nb; q += 64) l += a.part[(size_t)q * Ly::REC + Ly::LOSS];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) l += __shfl_xor(l, o);
    if (lane == 0) {
      const float loss = l / (float)a.Bt;
      st->val = st->beta * st->val + (1.0 - st->beta) * (double)loss;
      st->it += 1;
      st->step_t += 1;
    }
  }
}

// Adam (torch.optim.Adam, single-tensor path, betas (0.9, 0.999), eps 1e-8, no weight decay):
// exp_avg.lerp_(g, 1 - b1); exp_avg_sq.mul_(b2).addcmul_(g, g, value=1 - b2);
// p.addcdiv_(exp_avg, exp_avg_sq.sqrt() / sqrt(1 - b2^t) + eps, value=-lr / (1 - b1^t))
struct AdamC {
  float step, bc2s;
};
__device__ __forceinline__ void adam(float& p, float& m, float& v, float g, const AdamC& k) {
  m = m + 0.1f * (g - m);
  v = v * 0.999f + 0.001f * g * g;
  const float den = sqrtf(v) / k.bc2s + 1e-8f;
  p = p + k.step * (m / den);
}

template <int NIN, int HP>
__global__ __launch_bounds__(256) void k_adam(Args a) {
  using Ly = Lay<NIN, HP>;
  __shared__ float tile[32][33];
  __shared__ float red[16][17];
  const State* st = a.st;
  if (!st->gate) return;
  const double t = (double)st->step_t;
  AdamC k;
  k.step = (float)(-(double)a.lr / (1.0 - pow(0.9, t)));
  k.bc2s = (float)sqrt(1.0 - pow(0.999, t));
  constexpr int NW1 = (HP / 32) * (HP / 32);
  const int tid = threadIdx.x;
  if ((int)blockIdx.x < NW1) {
    const int tj = blockIdx.x / (HP / 32), tc = blockIdx.x % (HP / 32);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = tid + 256 * q, rj = e >> 5, rc = e & 31;
      const size_t o = (size_t)(tj * 32 + rj) * HP + tc * 32 + rc;
      float g = a.dW1p[o];
      for (int s = 1; s < a.S; ++s) g += a.dW1p[(size_t)s * HP * HP + o];
      float p = a.P[Ly::W1 + o], m = a.M[Ly::W1 + o], v = a.V[Ly::W1 + o];
      adam(p, m, v, g, k);
      a.P[Ly::W1 + o] = p;
      a.M[Ly::W1 + o] = m;
      a.V[Ly::W1 + o] = v;
      tile[rj][rc] = p;
    }
    __syncthreads();
    // the new W1 tile as the packed B fragments of both products: 4 blocks of 16 x 16 = 4 KB each, lane-major
    constexpr int TG = HP / 16;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = tid + 256 * q, bi = e >> 8, L = (e >> 2) & 63, sx = e & 3;
      const int b_r = bi >> 1, b_c = bi & 1, lr = L & 15, lq = L >> 4;
      // forward: rows j (output columns), k along the fragment
      a.Wf[(((size_t)(tj * 2 + b_r) * TG + tc * 2 + b_c) * 64 + L) * 4 + sx] = tile[16 * b_r + lr][16 * b_c + 4 * lq + sx];
      // backward: rows c, k = j along the fragment
      a.Wb[(((size_t)(tc * 2 + b_r) * TG + tj * 2 + b_c) * 64 + L) * 4 + sx] = tile[16 * b_c + 4 * lq + sx][16 * b_r + lr];
    }
    return;
  }
  // small parameters: 16 elements per workgroup, 16 partial-sum lanes each (fixed order)
  const int e = ((int)blockIdx.x - NW1) * 16 + (tid & 15), q = tid >> 4;
  const int nb = a.Bt / R2;
  float g = 0.f;
  if (e < Ly::SMALL)
    for (int wg = q; wg < nb; wg += 16) g += a.part[(size_t)wg * Ly::REC + e];
  red[q][tid & 15] = g;
  __syncthreads();
  if (q == 0 && e < Ly::SMALL) {
    float s = red[0][tid];
    for (int i = 1; i < 16; ++i) s += red[i][tid];
    float p = a.P[e], m = a.M[e], v = a.V[e];
    adam(p, m, v, s, k);
    a.P[e] = p;
    a.M[e] = m;
    a.V[e] = v;
  }
}

// torch layouts <-> padded buffers
template <int NIN, int HP>
__global__ void k_pack(float* P, float* Wf, float* Wb, float* W0, float* b0, float* W1, float* b1, float* W2,
                       float* b2, int H, int unpack) {
  using Ly = Lay<NIN, HP>;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < (long long)HP * HP) {
    const int j = (int)(i / HP), c = (int)(i % HP);
    if (unpack) {
      if (j < H && c < H) W1[j * H + c] = P[Ly::W1 + i];
    } else {
      const float v = (j < H && c < H) ? W1[j * H + c] : 0.f;
      P[Ly::W1 + i] = v;
      Wf[pk(j, c, HP / 16)] = v;
      Wb[pk(c, j, HP / 16)] = v;
    }
  }
  if (i < HP) {
    const int c = (int)i;
    if (unpack) {
      if (c < H) {
        for (int q = 0; q < NIN; ++q) W0[c * NIN + q] = P[Ly::W0 + c * NIN + q];
        b0[c] = P[Ly::B0 + c];
        b1[c] = P[Ly::B1 + c];
        W2[c] = P[Ly::W2 + c];
      }
      if (c == 0) b2[0] = P[Ly::B2];
    } else {
      for (int q = 0; q < NIN; ++q) P[Ly::W0 + c * NIN + q] = c < H ? W0[c * NIN + q] : 0.f;
      P[Ly::B0 + c] = c < H ? b0[c] : 0.f;
      P[Ly::B1 + c] = c < H ? b1[c] : 0.f;
      P[Ly::W2 + c] = c < H ? W2[c] : 0.f;
      if (c < 4) P[Ly::B2 + c] = c == 0 ? b2[0] : 0.f;
    }
  }
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
struct vboc_fit {
  int nin, hidden, hp, bt, S;
  int total, rec;
  float *P = nullptr, *M = nullptr, *V = nullptr, *Wf = nullptr, *Wb = nullptr;
  float *H1p = nullptr, *dH2p = nullptr, *part = nullptr, *dW1p = nullptr;
  int* idx[2] = {nullptr, nullptr};
  State* st = nullptr;
  State* st_host = nullptr;           // pinned
  hipStream_t stream = nullptr;
  hipEvent_t ev_in = nullptr, ev_out = nullptr, t0 = nullptr, t1 = nullptr;
  hipGraphExec_t exec = nullptr;
  Args key{};
  int key_poll = 0;
  double last_ms = 0.0;
  long long last_launched = 0;
};

static thread_local std::string g_fit_err;
static int ffail(int code, const std::string& m) {
  g_fit_err = m;
  return code;
}
#define FCHK(x)                                                                         \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) return ffail(VBOC_FIT_EHIP, std::string(#x ": ") + hipGetErrorString(e_)); \
  } while (0)

static void launch_sample(const vboc_fit*, const Args& a, hipStream_t s) {
  hipLaunchKernelGGL(k_sample, dim3(1), dim3(SNT), 0, s, a);
}

template <int NIN, int HP>
static void launch_train(const vboc_fit* h, const Args& a, hipStream_t s, bool fwd) {
  constexpr int NW1 = (HP / 32) * (HP / 32);
  const int nsmall = (Lay<NIN, HP>::SMALL + 15) / 16;
  if (fwd) {
    hipLaunchKernelGGL((k_fwd_bwd<NIN, HP>), dim3(h->bt / R2 + 1), dim3(256), 0, s, a);
  } else {
    hipLaunchKernelGGL((k_dw1<NIN, HP>), dim3((HP / 64) * (HP / 64) * h->S), dim3(256), 0, s, a);
    hipLaunchKernelGGL((k_adam<NIN, HP>), dim3(NW1 + nsmall), dim3(256), 0, s, a);
  }
}

static void train_part(const vboc_fit* h, const Args& a, hipStream_t s, bool fwd) {
  if (h->nin == 6 && h->hp == 512) launch_train<6, 512>(h, a, s, fwd);
  else if (h->nin == 4 && h->hp == 320) launch_train<4, 320>(h, a, s, fwd);
  else launch_train<2, 128>(h, a, s, fwd);
}

// Step i of a chunk uses the minibatch in idx[(parity + i) % 2], drawn by the previous step's forward kernel
// (or by the fit's first k_sample), and its forward kernel draws step i + 1's into the other buffer.
static void chunk(const vboc_fit* h, const Args& base, int steps, int parity, hipStream_t s) {
  for (int i = 0; i < steps; ++i) {
    Args a = base;
    a.idx = h->idx[(parity + i) & 1];
    a.idx_next = h->idx[(parity + i + 1) & 1];
    train_part(h, a, s, true);
    train_part(h, a, s, false);
  }
}

static bool supported(int nin, int hp) {
  return (nin == 6 && hp == 512) || (nin == 4 && hp == 320) || (nin == 2 && hp == 128);
}

template <int NIN, int HP>
static int total_of() { return Lay<NIN, HP>::TOTAL; }
template <int NIN, int HP>
static int rec_of() { return Lay<NIN, HP>::REC; }

static void pack(vboc_fit* h, float* W0, float* b0, float* W1, float* b1, float* W2, float* b2, int unpack,
                 float* src) {
  const int nthr = h->hp * h->hp;
  dim3 g((nthr + 255) / 256), b(256);
  if (h->nin == 6) hipLaunchKernelGGL((k_pack<6, 512>), g, b, 0, h->stream, src, h->Wf, h->Wb, W0, b0, W1, b1, W2, b2, h->hidden, unpack);
  else if (h->nin == 4) hipLaunchKernelGGL((k_pack<4, 320>), g, b, 0, h->stream, src, h->Wf, h->Wb, W0, b0, W1, b1, W2, b2, h->hidden, unpack);
  else hipLaunchKernelGGL((k_pack<2, 128>), g, b, 0, h->stream, src, h->Wf, h->Wb, W0, b0, W1, b1, W2, b2, h->hidden, unpack);
}

extern "C" {

const char* vboc_fit_last_error(void) { return g_fit_err.c_str(); }

int vboc_fit_create(int nin, int hidden, int minibatch, unsigned long long seed, vboc_fit_handle* out) {
  if (!out) return ffail(VBOC_FIT_EARG, "out is null");
  *out = nullptr;
  const int hp = (hidden + 63) / 64 * 64;
  if (!supported(nin, hp))
    return ffail(VBOC_FIT_EUNSUPPORTED, "native fit supports (inputs, hidden) = (6, 449..512), (4, 257..320), "
                                        "(2, 65..128)");
  if (minibatch < 32 || minibatch % 32 || minibatch > MAXK)
    return ffail(VBOC_FIT_EUNSUPPORTED, "minibatch must be a multiple of 32 in [32, 4096]");
  vboc_fit* h = new vboc_fit();
  h->nin = nin;
  h->hidden = hidden;
  h->hp = hp;
  h->bt = minibatch;
  // split of the dW1 rows: about 256 workgroups, each split a multiple of 32 rows
  const int blocks = (hp / 64) * (hp / 64);
  int S = 1;
  while (blocks * S * 2 <= 256 && (minibatch / (S * 2)) % 32 == 0) S *= 2;
  h->S = S;
  if (nin == 6) { h->total = total_of<6, 512>(); h->rec = rec_of<6, 512>(); }
  else if (nin == 4) { h->total = total_of<4, 320>(); h->rec = rec_of<4, 320>(); }
  else { h->total = total_of<2, 128>(); h->rec = rec_of<2, 128>(); }
  auto fail_free = [&](hipError_t e, const char* what) {
    vboc_fit_destroy(h);
    return ffail(VBOC_FIT_EHIP, std::string(what) + ": " + hipGetErrorString(e));
  };
  hipError_t e;
#define FALLOC(ptr, bytes) \
  if ((e = hipMalloc((void**)&(ptr), (bytes))) != hipSuccess) return fail_free(e, "hipMalloc " #ptr)
  FALLOC(h->P, sizeof(float) * h->total);
  FALLOC(h->M, sizeof(float) * h->total);
  FALLOC(h->V, sizeof(float) * h->total);
  FALLOC(h->Wf, sizeof(float) * hp * hp);
  FALLOC(h->Wb, sizeof(float) * hp * hp);
  FALLOC(h->idx[0], sizeof(int) * minibatch);
  FALLOC(h->idx[1], sizeof(int) * minibatch);
  FALLOC(h->H1p, sizeof(float) * (size_t)hp * minibatch);
  FALLOC(h->dH2p, sizeof(float) * (size_t)hp * minibatch);
  FALLOC(h->part, sizeof(float) * (size_t)(minibatch / R2) * h->rec);
  FALLOC(h->dW1p, sizeof(float) * (size_t)S * hp * hp);
  FALLOC(h->st, sizeof(State));
#undef FALLOC
  if ((e = hipHostMalloc((void**)&h->st_host, sizeof(State))) != hipSuccess) return fail_free(e, "hipHostMalloc");
  if ((e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking)) != hipSuccess) return fail_free(e, "stream");
  if ((e = hipEventCreateWithFlags(&h->ev_in, hipEventDisableTiming)) != hipSuccess) return fail_free(e, "event");
  if ((e = hipEventCreateWithFlags(&h->ev_out, hipEventDisableTiming)) != hipSuccess) return fail_free(e, "event");
  if ((e = hipEventCreate(&h->t0)) != hipSuccess) return fail_free(e, "event");
  if ((e = hipEventCreate(&h->t1)) != hipSuccess) return fail_free(e, "event");
  (void)hipMemsetAsync(h->P, 0, sizeof(float) * h->total, h->stream);
  (void)hipMemsetAsync(h->M, 0, sizeof(float) * h->total, h->stream);
  (void)hipMemsetAsync(h->V, 0, sizeof(float) * h->total, h->stream);
  (void)hipMemsetAsync(h->Wf, 0, sizeof(float) * hp * hp, h->stream);
  (void)hipMemsetAsync(h->Wb, 0, sizeof(float) * hp * hp, h->stream);
  State s{};
  s.seed = seed;
  *h->st_host = s;
  (void)hipMemcpyAsync(h->st, h->st_host, sizeof(State), hipMemcpyHostToDevice, h->stream);
  if ((e = hipStreamSynchronize(h->stream)) != hipSuccess) return fail_free(e, "init");
  *out = h;
  return 0;
}

int vboc_fit_destroy(vboc_fit_handle h) {
  if (!h) return 0;
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  if (h->exec) (void)hipGraphExecDestroy(h->exec);
  float* bufs[] = {h->P, h->M, h->V, h->Wf, h->Wb, h->H1p, h->dH2p, h->part, h->dW1p};
  for (float* b : bufs)
    if (b) (void)hipFree(b);
  for (int* b : h->idx)
    if (b) (void)hipFree(b);
  if (h->st) (void)hipFree(h->st);
  if (h->st_host) (void)hipHostFree(h->st_host);
  if (h->ev_in) (void)hipEventDestroy(h->ev_in);
  if (h->ev_out) (void)hipEventDestroy(h->ev_out);
  if (h->t0) (void)hipEventDestroy(h->t0);
  if (h->t1) (void)hipEventDestroy(h->t1);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
  return 0;
}

int vboc_fit_set_params(vboc_fit_handle h, const float* W0, const float* b0, const float* W1, const float* b1,
                        const float* W2, const float* b2, void* stream) {
  if (!h || !W0 || !b0 || !W1 || !b1 || !W2 || !b2) return ffail(VBOC_FIT_EARG, "null argument");
  FCHK(hipEventRecord(h->ev_in, (hipStream_t)stream));
  FCHK(hipStreamWaitEvent(h->stream, h->ev_in, 0));
  pack(h, const_cast<float*>(W0), const_cast<float*>(b0), const_cast<float*>(W1), const_cast<float*>(b1),
       const_cast<float*>(W2), const_cast<float*>(b2), 0, h->P);
  FCHK(hipGetLastError());
  FCHK(hipEventRecord(h->ev_out, h->stream));
  FCHK(hipStreamWaitEvent((hipStream_t)stream, h->ev_out, 0));
  return 0;
}

int vboc_fit_get_params(vboc_fit_handle h, int which, float* W0, float* b0, float* W1, float* b1, float* W2,
                        float* b2, void* stream) {
  if (!h || !W0 || !b0 || !W1 || !b1 || !W2 || !b2) return ffail(VBOC_FIT_EARG, "null argument");
  if (which < 0 || which > 2) return ffail(VBOC_FIT_EARG, "which: 0 parameters, 1 exp_avg, 2 exp_avg_sq");
  FCHK(hipEventRecord(h->ev_in, (hipStream_t)stream));
  FCHK(hipStreamWaitEvent(h->stream, h->ev_in, 0));
  pack(h, W0, b0, W1, b1, W2, b2, 1, which == 0 ? h->P : which == 1 ? h->M : h->V);
  FCHK(hipGetLastError());
  FCHK(hipEventRecord(h->ev_out, h->stream));
  FCHK(hipStreamWaitEvent((hipStream_t)stream, h->ev_out, 0));
  return 0;
}

int vboc_fit_train(vboc_fit_handle h, const vboc_fit_run_t* r, void* stream) {
  if (!h || !r || !r->F) return ffail(VBOC_FIT_EARG, "null argument");
  if (r->ld < h->nin + 1) return ffail(VBOC_FIT_EARG, "ld < inputs + 1");
  if (r->n_new == 0 && r->n < h->bt) return ffail(VBOC_FIT_EARG, "fewer rows than one minibatch");
  if (r->n_new != 0 && (r->n_new < h->bt / 2 || r->n - r->n_new < h->bt / 2 || r->n_new > r->n))
    return ffail(VBOC_FIT_EARG, "a refit needs at least minibatch/2 old and new rows");
  if (r->n >= (1ll << 31)) return ffail(VBOC_FIT_EARG, "more than 2^31 rows");
  if (r->it_max < 1) return ffail(VBOC_FIT_EARG, "it_max < 1");
  // a graph replays an even number of steps, so every replay starts on idx[0]
  const int poll = r->graphs ? (r->poll > 2 ? (r->poll + 1) / 2 * 2 : 2) : (r->poll > 0 ? r->poll : 1);
  Args a;
  memset(&a, 0, sizeof a);
  a.P = h->P; a.M = h->M; a.V = h->V; a.Wf = h->Wf; a.Wb = h->Wb; a.idx = nullptr;
  a.H1p = h->H1p; a.dH2p = h->dH2p; a.part = h->part; a.dW1p = h->dW1p; a.st = h->st;
  a.F = r->F; a.n = r->n; a.n_new = r->n_new; a.ldF = r->ld; a.Bt = h->bt; a.S = h->S; a.lr = (float)r->lr;
  // loop state of the reference: it = 1, val = max |qdot| of the training rows (given by the caller in f64)
  FCHK(hipStreamSynchronize(h->stream));
  State* s = h->st_host;
  FCHK(hipMemcpyAsync(s, h->st, sizeof(State), hipMemcpyDeviceToHost, h->stream));
  FCHK(hipStreamSynchronize(h->stream));
  s->val = r->val0;
  s->stop = r->stop_val;
  s->beta = r->beta;
  s->it = 1;
  s->it_lim = r->it_max;
  s->gate = 1;
  FCHK(hipEventRecord(h->ev_in, (hipStream_t)stream));
  FCHK(hipStreamWaitEvent(h->stream, h->ev_in, 0));
  FCHK(hipMemcpyAsync(h->st, s, sizeof(State), hipMemcpyHostToDevice, h->stream));
  const unsigned long long d0 = s->draws;
  // the first step's minibatch (draw d0); every later one is drawn beside the step before it
  Args a0 = a;
  a0.idx = h->idx[0];
  launch_sample(h, a0, h->stream);
  FCHK(hipGetLastError());
  const bool same = h->exec && h->key_poll == poll && memcmp(&h->key, &a, sizeof(Args)) == 0;
  if (r->graphs && !same) {
    if (h->exec) {
      (void)hipGraphExecDestroy(h->exec);
      h->exec = nullptr;
    }
    hipGraph_t g;
    FCHK(hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
    chunk(h, a, poll, 0, h->stream);
    FCHK(hipStreamEndCapture(h->stream, &g));
    hipError_t e = hipGraphInstantiate(&h->exec, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (e != hipSuccess) return ffail(VBOC_FIT_EHIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(e));
    h->key = a;
    h->key_poll = poll;
  }
  FCHK(hipEventRecord(h->t0, h->stream));
  long long launched = 0;
  for (;;) {
    if (r->graphs) FCHK(hipGraphLaunch(h->exec, h->stream));
    else chunk(h, a, poll, (int)(launched & 1), h->stream);
    FCHK(hipGetLastError());
    launched += poll;
    FCHK(hipMemcpyAsync(&s->gate, &h->st->gate, sizeof(int), hipMemcpyDeviceToHost, h->stream));
    FCHK(hipStreamSynchronize(h->stream));
    if (!s->gate) break;
    if (launched > r->it_max + poll) return ffail(VBOC_FIT_EHIP, "fit did not stop at it_max");
  }
  FCHK(hipEventRecord(h->t1, h->stream));
  FCHK(hipMemcpyAsync(s, h->st, sizeof(State), hipMemcpyDeviceToHost, h->stream));
  FCHK(hipStreamSynchronize(h->stream));
  // the sampler stream continues after the steps taken (the ones drawn past the stop are dropped), so the next
  // fit draws what a step-by-step loop would
  s->draws = d0 + (unsigned long long)(s->it - 1);
  FCHK(hipMemcpyAsync(&h->st->draws, &s->draws, sizeof(s->draws), hipMemcpyHostToDevice, h->stream));
  FCHK(hipStreamSynchronize(h->stream));
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, h->t0, h->t1);
  h->last_ms = ms;
  h->last_launched = launched;
  FCHK(hipEventRecord(h->ev_out, h->stream));
  FCHK(hipStreamWaitEvent((hipStream_t)stream, h->ev_out, 0));
  if (r->iterations) *r->iterations = s->it - 1;
  if (r->val) *r->val = s->val;
  if (r->launched) *r->launched = launched;
  if (r->kernel_ms) *r->kernel_ms = ms;
  return 0;
}

int vboc_fit_sample(vboc_fit_handle h, long long n, long long n_new, int steps, int* idx_out, void* stream) {
  if (!h || !idx_out || steps < 0) return ffail(VBOC_FIT_EARG, "bad argument");
  if (n_new == 0 && n < h->bt) return ffail(VBOC_FIT_EARG, "fewer rows than one minibatch");
  if (n_new != 0 && (n_new < h->bt / 2 || n - n_new < h->bt / 2 || n_new > n))
    return ffail(VBOC_FIT_EARG, "a refit needs at least minibatch/2 old and new rows");
  if (n >= (1ll << 31)) return ffail(VBOC_FIT_EARG, "more than 2^31 rows");
  FCHK(hipStreamSynchronize(h->stream));
  State* s = h->st_host;
  FCHK(hipMemcpyAsync(s, h->st, sizeof(State), hipMemcpyDeviceToHost, h->stream));
  FCHK(hipStreamSynchronize(h->stream));
  const State keep = *s;
  s->val = 1.0;
  s->stop = 0.0;
  s->it = 1;
  s->it_lim = 1ll << 62;
  FCHK(hipEventRecord(h->ev_in, (hipStream_t)stream));
  FCHK(hipStreamWaitEvent(h->stream, h->ev_in, 0));
  FCHK(hipMemcpyAsync(h->st, s, sizeof(State), hipMemcpyHostToDevice, h->stream));
  Args a;
  memset(&a, 0, sizeof a);
  a.idx = h->idx[0]; a.st = h->st;
  a.n = n; a.n_new = n_new; a.ldF = 0; a.Bt = h->bt; a.S = h->S;
  for (int i = 0; i < steps; ++i) {
    launch_sample(h, a, h->stream);
    FCHK(hipGetLastError());
    FCHK(hipMemcpyAsync(idx_out + (size_t)i * h->bt, h->idx[0], sizeof(int) * h->bt, hipMemcpyDeviceToDevice,
                        h->stream));
  }
  FCHK(hipMemcpyAsync(s, h->st, sizeof(State), hipMemcpyDeviceToHost, h->stream));
  FCHK(hipStreamSynchronize(h->stream));
  State back = keep;
  back.draws = s->draws;
  *s = back;
  FCHK(hipMemcpyAsync(h->st, s, sizeof(State), hipMemcpyHostToDevice, h->stream));
  FCHK(hipStreamSynchronize(h->stream));
  FCHK(hipEventRecord(h->ev_out, h->stream));
  FCHK(hipStreamWaitEvent((hipStream_t)stream, h->ev_out, 0));
  return 0;
}

int vboc_fit_info(vboc_fit_handle h, int* hidden_padded, int* splits, long long* adam_steps,
                  unsigned long long* draws) {
  if (!h) return ffail(VBOC_FIT_EARG, "null handle");
  FCHK(hipStreamSynchronize(h->stream));
  FCHK(hipMemcpyAsync(h->st_host, h->st, sizeof(State), hipMemcpyDeviceToHost, h->stream));
  FCHK(hipStreamSynchronize(h->stream));
  const State s = *h->st_host;
  if (hidden_padded) *hidden_padded = h->hp;
  if (splits) *splits = h->S;
  if (adam_steps) *adam_steps = s.step_t;
  if (draws) *draws = s.draws;
  return 0;
}

}  // extern "C"

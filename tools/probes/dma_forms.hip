// The two LDS-DMA forms of coop.h on the UR5 arm's stage windows (verdict r03 item 1, the k_wave<4> bisect):
//   VADDR  global_load_lds_dwordx4 v[addr:addr+1], off      (dma(): per-lane 64-bit address, the product)
//   SADDR  global_load_lds_dwordx4 v_off, s[base:base+1]    (dma_s(): wave-uniform base + per-lane 32-bit offset)
// Every window of every stage of WaveLayout<4> (REC = 392 doubles) - factor [0, 268) in 3 DMAs, vector [260, 340),
// forward [268, 340), costate [0, 144) in 2 - is landed by both forms into two LDS images and compared with the
// source doubles (lanes past the window repeat its last chunk, as in the product).  Prints the mismatch count per
// window and form; 0 everywhere means the two forms move the same bytes for these shapes.
//
// build: hipcc --offload-arch=gfx950 -O3 tools/probes/dma_forms.hip -o tools/probes/dma_forms
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int REC = 392, NST = 110, GROUPS = 512;

struct Win { int lo, w; };
__constant__ Win c_win[4] = {{0, 268}, {260, 80}, {268, 72}, {0, 144}};

__global__ __launch_bounds__(64) void k_forms(const double* __restrict__ g, unsigned* __restrict__ bad) {
  __shared__ __attribute__((aligned(16))) double la[384], lb[384];
  const int t = threadIdx.x;
  const double* base = g + (size_t)blockIdx.x * REC * (NST + 4);
  const unsigned a0 = (unsigned)(size_t)(__attribute__((address_space(3))) void*)&la[0];
  const unsigned b0 = (unsigned)(size_t)(__attribute__((address_space(3))) void*)&lb[0];
  for (int wi = 0; wi < 4; ++wi) {
    const int lo = c_win[wi].lo, W = c_win[wi].w, nc = W / 2, P = (nc + 63) / 64;
    for (int k = 0; k < NST; ++k) {
      const double* sb = base + (size_t)k * REC;
      for (int part = 0; part < P; ++part) {
        const int c = part * 64 + t < nc ? part * 64 + t : nc - 1;
        const double* src = sb + lo + 2 * c;
        const unsigned voff = 8u * (unsigned)(lo + 2 * c);
        const unsigned long long bb = (unsigned long long)(size_t)sb;
        const unsigned long long bs =
            ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(bb >> 32)) << 32) |
            (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)bb);
        const unsigned la_ = a0 + 8u * (unsigned)(part * 128), lb_ = b0 + 8u * (unsigned)(part * 128);
        unsigned keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(src), "s"(la_) : "memory");
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 4\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(voff), "s"(bs), "s"(lb_) : "memory");
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      for (int e = t; e < P * 128; e += 64) {
        const int ch = e / 2 < nc ? e / 2 : nc - 1;       // the chunk this LDS double came from
        const double want = sb[lo + 2 * ch + (e & 1)];
        const bool pa = __double_as_longlong(la[e]) == __double_as_longlong(want);
        const bool pb = __double_as_longlong(lb[e]) == __double_as_longlong(want);
        if (!pa) atomicAdd(&bad[wi * 2 + 0], 1u);
        if (!pb) atomicAdd(&bad[wi * 2 + 1], 1u);
      }
      __syncthreads();
    }
  }
}

int main() {
  const size_t n = (size_t)GROUPS * REC * (NST + 4);
  std::vector<double> h(n);
  for (size_t i = 0; i < n; ++i) h[i] = (double)i + 0.25;
  double* d;
  unsigned* bad;
  hipMalloc(&d, n * sizeof(double));
  hipMalloc(&bad, 8 * sizeof(unsigned));
  hipMemcpy(d, h.data(), n * sizeof(double), hipMemcpyHostToDevice);
  hipMemset(bad, 0, 8 * sizeof(unsigned));
  hipLaunchKernelGGL(k_forms, dim3(GROUPS), dim3(64), 0, 0, d, bad);
  unsigned hb[8];
  hipMemcpy(hb, bad, sizeof(hb), hipMemcpyDeviceToHost);
  const char* names[4] = {"factor [0,268) x3", "vector [260,340)", "forward [268,340)", "costate [0,144) x2"};
  for (int w = 0; w < 4; ++w)
    printf("{\"window\": \"%s\", \"vaddr_mismatches\": %u, \"saddr_mismatches\": %u}\n", names[w], hb[2 * w], hb[2 * w + 1]);
  hipFree(d);
  hipFree(bad);
  return 0;
}

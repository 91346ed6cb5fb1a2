// FETCH_SIZE calibration for the wave solver's stage-window loads (verdict r03, item 4: "check FETCH_SIZE on a
// probe that DMAs a known byte count with your own window / alignment pattern").
//
// Each one-wave workgroup owns a region of NST stage records of REC doubles (the WaveLayout<3> record, 250 doubles
// = 2 000 B, or the 128-B-line-aligned 256) and streams one field window [LO, LO + W) of every stage into LDS with
// the product's LDS-DMA form (coop.h dma() / dma_s(): global_load_lds_dwordx4, 64 lanes x 16 B per instruction,
// chunk indices clamped, never exec-masked; S stages per instruction for the grouped recursions).  The buffer is
// far larger than the 256 MiB MALL and every line is read by one wave once, so the memory-side request count of a
// launch is exactly the lines it touches.  rocprofv3 --pmc FETCH_SIZE per dispatch, compared with the bytes
// printed here (useful bytes, distinct 128-B lines x 128), calibrates the counter for these access shapes.
//
// build: hipcc --offload-arch=gfx950 -O3 tools/probes/fetch_calib.hip -o tools/probes/fetch_calib
// run:   rocprofv3 --pmc FETCH_SIZE --output-format csv -d <dir> -o run -- tools/probes/fetch_calib
#include <hip/hip_runtime.h>
#include <cstdio>
#include <set>
#include <vector>

constexpr int NST = 112;          // stage records per region (a triple problem at N <= 111)
constexpr int GROUPS = 8192;      // regions = workgroups

template <int REC, int LO, int W, int S>
__global__ __launch_bounds__(64) void k_win(const double* __restrict__ g, int dummy) {
  __shared__ double lds[4][128 * 2];
  const int t = threadIdx.x;
  const double* base = g + (size_t)blockIdx.x * REC * (NST + 4);
  const unsigned lds0 = (unsigned)(size_t)(__attribute__((address_space(3))) void*)&lds[0][0];
  constexpr int CH = W / 2;                 // 16-B chunks per stage window
  constexpr int P = (S * CH + 63) / 64;     // DMAs per group
  for (int k = 0; k + S <= NST; k += S) {
    for (int part = 0; part < P; ++part) {
      int idx = part * 64 + t;
      if (idx >= S * CH) idx = S * CH - 1;  // clamped (the product's lanes past the windows repeat the last chunk)
      const int u = idx / CH, c = idx - u * CH;
      const double* src = base + (size_t)(k + u) * REC + LO + 2 * c;
      const unsigned l = lds0 + 8u * (unsigned)(((k / S + part) & 3) * 256);
      unsigned keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep)
                   : "v"(src), "s"(l)
                   : "memory");
    }
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (dummy) ((double*)g)[0] = lds[0][t];
}

// plain streaming of the whole region with 16-B loads (the guide's calibrated case: FETCH_SIZE = bytes / 2)
template <int REC>
__global__ __launch_bounds__(64) void k_stream(const double* __restrict__ g, double* out) {
  typedef double d2 __attribute__((ext_vector_type(2)));
  const d2* base = (const d2*)(g + (size_t)blockIdx.x * REC * (NST + 4));
  const int n = REC * NST / 2;
  double acc = 0.0;
  for (int i = threadIdx.x; i < n; i += 64) {
    const d2 v = base[i];
    acc += v.x + v.y;
  }
  if (acc == 12345.678) out[0] = acc;
}

template <int REC, int LO, int W, int S>
static void report(const char* name, double* g) {
  std::set<long long> lines;
  long long useful = 0;
  constexpr int CH = W / 2, P = (S * CH + 63) / 64;
  for (int b = 0; b < GROUPS; ++b) {
    const long long base = (long long)b * REC * (NST + 4) * 8;
    for (int k = 0; k + S <= NST; k += S)
      for (int part = 0; part < P; ++part)
        for (int t = 0; t < 64; ++t) {
          int idx = part * 64 + t;
          if (idx >= S * CH) idx = S * CH - 1;
          const int u = idx / CH, c = idx - u * CH;
          const long long a = base + ((long long)(k + u) * REC + LO + 2 * c) * 8;
          lines.insert(a / 128);
          lines.insert((a + 15) / 128);
        }
    useful += (long long)(NST / S) * S * W * 8;
  }
  hipLaunchKernelGGL((k_win<REC, LO, W, S>), dim3(GROUPS), dim3(64), 0, 0, g, 0);
  (void)hipDeviceSynchronize();
  printf("{\"kernel\": \"k_win<%d, %d, %d, %d>\", \"case\": \"%s\", \"useful_bytes\": %lld, \"line_bytes\": %lld}\n", REC, LO,
         W, S, name, useful, (long long)lines.size() * 128);
}

int main() {
  const size_t n = (size_t)GROUPS * 256 * (NST + 4);   // 1.9 GB at REC 256: far past the MALL
  double* g = nullptr;
  double* out = nullptr;
  if (hipMalloc(&g, n * sizeof(double)) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  (void)hipMemset(g, 0, n * sizeof(double));
  (void)hipDeviceSynchronize();
  hipLaunchKernelGGL(k_stream<250>, dim3(GROUPS), dim3(64), 0, 0, g, out);
  (void)hipDeviceSynchronize();
  printf("{\"kernel\": \"k_stream<250>\", \"case\": \"stream\", \"useful_bytes\": %lld, \"line_bytes\": %lld}\n",
         (long long)GROUPS * 250 * NST * 8, (long long)GROUPS * ((250LL * NST * 8 + 127) / 128) * 128);
  // WaveLayout<3>: vector window [OPE, OX) = [162, 210), forward [OC, OX) = [168, 210), factor [0, OC) = [0, 168)
  report<250, 162, 48, 1>("vec window, 1 stage per DMA, REC 250", g);
  report<250, 162, 48, 2>("vec window, grouped 2 stages per DMA, REC 250 (product)", g);
  report<256, 162, 48, 2>("vec window, grouped 2, REC 256", g);
  report<250, 168, 42, 3>("fwd window, grouped 3 stages per DMA, REC 250 (product)", g);
  report<256, 168, 42, 3>("fwd window, grouped 3, REC 256", g);
  report<250, 0, 168, 1>("factor window [0, OC), 2 DMAs per stage, REC 250 (product)", g);
  report<256, 0, 168, 1>("factor window, REC 256", g);
  report<256, 160, 48, 2>("vec-size window at a 128-B-aligned offset, REC 256", g);
  (void)hipFree(g);
  (void)hipFree(out);
  return 0;
}

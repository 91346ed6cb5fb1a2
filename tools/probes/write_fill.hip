// Do partial-line stores fetch their lines?  (k_dg's memory side, DESIGN.md section 5 'Round 4': 13.1 KB per
// stage-IPM-iteration against ~6 KB of useful window bytes.)  Each one-wave workgroup owns NST stage records of REC
// doubles (the triple's WaveLayout<3> record, 250 doubles = 2 000 B) and only STORES one field range [LO, LO + W) of
// every stage, the shapes k_dg writes once per IPM pass: prep's D / DA [96, 114), the factorisation's write-back
// [114, 210) (one unmasked 16-B store per lane), the iterate update [54, 90) - plus a full-line control.  The buffer
// is far larger than the 256 MiB MALL.  rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE per dispatch against the bytes
// printed here tell whether the memory side fetches the lines that partial stores touch.
//
// build: hipcc --offload-arch=gfx950 -O3 tools/probes/write_fill.hip -o tools/probes/write_fill
#include <hip/hip_runtime.h>
#include <cstdio>
#include <set>

constexpr int NST = 112, GROUPS = 8192;

template <int REC, int LO, int W>
__global__ __launch_bounds__(64) void k_wpart(double* __restrict__ g) {
  const int t = threadIdx.x;
  double* base = g + (size_t)blockIdx.x * REC * (NST + 4);
  constexpr int CH = W / 2;                      // 16-B chunks of the range
  for (int k = 0; k < NST; ++k) {
    typedef double d2 __attribute__((ext_vector_type(2)));
    d2* dst = (d2*)(base + (size_t)k * REC + LO);
    for (int c = t; c < CH; c += 64) dst[c] = d2{(double)k, (double)c};
  }
}

template <int REC, int LO, int W>
void run(double* d, const char* name) {
  hipLaunchKernelGGL((k_wpart<REC, LO, W>), dim3(GROUPS), dim3(64), 0, 0, d);
  (void)hipDeviceSynchronize();
  std::set<size_t> lines;
  for (int k = 0; k < NST; ++k)
    for (int e = 0; e < W; ++e) lines.insert(((size_t)k * REC + LO + e) * 8 / 128);
  const double useful = (double)GROUPS * NST * W * 8, touched = (double)GROUPS * lines.size() * 128;
  printf("{\"kernel\": \"k_wpart<%d, %d, %d>\", \"case\": \"%s\", \"useful_bytes\": %.0f, \"line_bytes\": %.0f}\n", REC, LO, W,
         name, useful, touched);
}

int main() {
  const size_t n = (size_t)GROUPS * 256 * (NST + 4);
  double* d;
  if (hipMalloc(&d, n * sizeof(double)) != hipSuccess) return 1;
  (void)hipMemset(d, 0, n * sizeof(double));
  (void)hipDeviceSynchronize();
  run<250, 96, 18>(d, "prep D / DA [96, 114)");
  run<250, 114, 96>(d, "factor write-back [114, 210)");
  run<250, 54, 36>(d, "update z, dz, ql, qu [54, 90)");
  run<256, 0, 256>(d, "control: whole 128-B-aligned records");
  (void)hipFree(d);
  return 0;
}

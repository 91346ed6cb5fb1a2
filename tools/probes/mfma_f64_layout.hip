// Probe: operand / accumulator lane maps of v_mfma_f64_16x16x4f64 on gfx950 with exact integer data.
// Expected (cdna_hip_programming.md): A lane l = A[l&15][l>>4], B lane l = B[l>>4][l&15],
// D lane l reg r = D[(l>>4) + 4r][l&15].  Also checks that D reg s of a symmetric product is the
// next MFMA's A / B operand for k-step s (the map the wave solver's Riccati factorisation relies on).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double dbl4 __attribute__((ext_vector_type(4)));

__global__ void k(const double* A, const double* B, double* D, double* D2) {
  const int l = threadIdx.x, c = l & 15, g = l >> 4;
  dbl4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(A[c * 4 + g], B[g * 16 + c], acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[(g + 4 * r) * 16 + c] = acc[r];
  // second product X' X with X = acc (16x16): k-steps s = 0..3 take reg s as both operands
  dbl4 acc2 = {0, 0, 0, 0};
  for (int s = 0; s < 4; ++s) acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(acc[s], acc[s], acc2, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D2[(g + 4 * r) * 16 + c] = acc2[r];
}

int main() {
  double hA[64], hB[64], hD[256], hD2[256];
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 4; ++j) hA[i * 4 + j] = (double)((i * 7 + j * 3) % 11 - 5);
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 16; ++j) hB[i * 16 + j] = (double)((i * 5 + j * 2) % 9 - 4);
  double *dA, *dB, *dD, *dD2;
  hipMalloc(&dA, sizeof hA); hipMalloc(&dB, sizeof hB); hipMalloc(&dD, sizeof hD); hipMalloc(&dD2, sizeof hD2);
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD, dD2);
  hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
  hipMemcpy(hD2, dD2, sizeof hD2, hipMemcpyDeviceToHost);
  int bad = 0, bad2 = 0;
  double X[256];
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double s = 0;
      for (int q = 0; q < 4; ++q) s += hA[i * 4 + q] * hB[q * 16 + j];
      X[i * 16 + j] = s;
      bad += s != hD[i * 16 + j];
    }
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double s = 0;
      for (int q = 0; q < 16; ++q) s += X[q * 16 + i] * X[q * 16 + j];
      bad2 += s != hD2[i * 16 + j];
    }
  printf("mfma_f64_16x16x4 layout: product mismatches %d / 256, X'X via acc-as-operand mismatches %d / 256 -> %s\n",
         bad, bad2, (bad || bad2) ? "FAIL" : "OK");
  return bad || bad2;
}

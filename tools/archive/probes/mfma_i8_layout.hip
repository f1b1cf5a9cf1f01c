// Probe: the operand / result lane layout of v_mfma_i32_16x16x64_i8 on gfx950, against a host
// GEMM.  Candidate layout: lane l holds A[l&15][16(l>>4) + j] and B[16(l>>4) + j][l&15], j = 0..15,
// and C[4(l>>4) + i][l&15], i = 0..3.  Prints "layout ok" when the candidate reproduces the GEMM.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
typedef int i32x4 __attribute__((ext_vector_type(4)));
__global__ void k(const int8_t* A, const int8_t* B, int* C) {
  const int l = threadIdx.x, r = l & 15, h = l >> 4;
  int8_t a[16], b[16];
  for (int j = 0; j < 16; ++j) { a[j] = A[r * 64 + 16 * h + j]; b[j] = B[(16 * h + j) * 16 + r]; }
  i32x4 av = *(i32x4*)a, bv = *(i32x4*)b;
  i32x4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, c, 0, 0, 0);
  for (int i = 0; i < 4; ++i) C[(4 * h + i) * 16 + r] = c[i];
}
int main() {
  int8_t hA[16 * 64], hB[64 * 16];
  int ref[256], got[256];
  srand(1);
  for (int i = 0; i < 1024; ++i) { hA[i] = (int8_t)(rand() & 255); hB[i] = (int8_t)(rand() & 255); }
  for (int m = 0; m < 16; ++m)
    for (int n = 0; n < 16; ++n) {
      int s = 0;
      for (int q = 0; q < 64; ++q) s += hA[m * 64 + q] * hB[q * 16 + n];
      ref[m * 16 + n] = s;
    }
  int8_t *dA, *dB; int* dC;
  hipMalloc(&dA, 1024); hipMalloc(&dB, 1024); hipMalloc(&dC, 1024);
  hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  hipMemcpy(got, dC, 1024, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 256; ++i) bad += got[i] != ref[i];
  printf(bad ? "layout MISMATCH: %d of 256\n" : "layout ok (%d mismatches)\n", bad);
  return bad ? 1 : 0;
}

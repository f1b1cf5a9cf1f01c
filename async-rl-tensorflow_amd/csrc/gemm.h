#pragma once
#include "a3c_common.h"
#include "../../include/a3c_hip.h"



enum { EPI_STORE = 0, EPI_BIAS_RELU = 1, EPI_BIAS = 2, EPI_MASK = 3 };

// C[M][N] = epi( sum_k A(m,k) * B(k,n) )
//   A(m,k) = A[m*lda + k] when the template's A_KC (k-contiguous) else A[k*lda + m]
//   B(k,n) = B[k*ldb + n] when B_NC (n-contiguous) else B[n*ldb + k]
struct GemmArgs {
  const float* A; int64_t lda;
  const float* B; int64_t ldb;
  float* C; int64_t ldc;
  int M, N, K;
  int epi;
  const float* bias;          // EPI_BIAS*, indexed by n
  const float* mask; int64_t ldm;  // EPI_MASK: keep where mask[m*ldm+n] > 0
  float* slab;                // split-K partials [nsplit][M][N]
  int nsplit;                 // requested split (effective split may be smaller)
  int kchunk;                 // set by a3c_gemm
  float* colsum;              // optional [nsplit_eff][N] column sums of B over each K-chunk
};

int a3c_gemm(bool a_kcontig, bool b_ncontig, GemmArgs g, hipStream_t s);

// k-permuted fp32 MFMA step: in 16x16x4 step s of a 16-wide k block kb, lane (i16, j4) supplies
// A[row i16][kb + 4 j4 + s] and B[kb + 4 j4 + s][col i16] -- every k of the block exactly once,
// and each lane's four k are contiguous in memory for k-contiguous A rows and B^T rows, so both
// operands arrive as one 16-byte load per lane per four MFMAs (no LDS staging).
__device__ inline f32x4 mfma_k16(const f32x4 a, const f32x4 b, f32x4 c) {
#pragma unroll
  for (int s = 0; s < 4; ++s) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[s], c, 0, 0, 0);
  return c;
}
int a3c_gemm_plan_split(int M, int N, int K, int target_blocks);

inline int a3c_gemm_effective_split(int K, int nsplit) {
  int ktiles = (K + 15) / 16;
  if (nsplit < 1) nsplit = 1;
  int per = (ktiles + nsplit - 1) / nsplit;
  return (ktiles + per - 1) / per;
}

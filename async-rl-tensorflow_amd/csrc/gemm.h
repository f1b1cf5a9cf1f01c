#pragma once
#include "a3c_common.h"
#include "../../include/a3c_hip.h"



enum { EPI_STORE = 0, EPI_BIAS_RELU = 1, EPI_BIAS = 2, EPI_MASK = 3, EPI_MASKBITS = 4 };

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
  int defer_reduce;           // a3c_gemm: leave the split-K fold to the caller (a3c_gemm_reduce)
  // XCD-aware tile order (a3c_gemm): 0 = plain 3-D grid; 1 = the N-tiles of one (M-tile, K-chunk)
  // on one XCD (they share the A strip); 2 = the M-tiles of one (N-tile, K-chunk) on one XCD
  // (they share the B strip).  Speed only: every tile computes the same sums in the same order.
  int xcd;
  // a3c_gemm: at most this many workgroups (0 = one per tile), each looping over tiles id, id +
  // grid, ... -- fewer GEMM workgroups resident beside a concurrent kernel.  Speed only.
  int max_wgs;
  // a3c_gemm: 128x128 tiles (k_gemm_f32_big: a quarter of the workgroups, each four times the
  // work) -- fewer workgroups resident beside a concurrent kernel.  Speed only (bit-identical).
  int big;
  // a3c_gemm: 4 = split K over 4 groups of 4 waves inside each 64x64-tile workgroup
  // (k_gemm_f32_wks), folded in LDS -- nsplit is then 1 (no slab).  Not bit-identical to the
  // slab split (another summation grouping), deterministic.
  int wg_split;
  // EPI_MASKBITS: keep where bit n & 31 of maskbits[m*ldm + (n >> 5)] is set (ldm in 32-bit words):
  // the forward's ReLU mask as bits, 1/32 of the bytes of re-reading the activations
  const uint32_t* maskbits;
};

int a3c_gemm(bool a_kcontig, bool b_ncontig, GemmArgs g, hipStream_t s);
// three independent GEMMs in one launch: g0, g1 with (A k-strided, B n-contiguous), g2 with (A
// k-contiguous, B k-contiguous).  The split-K folds are left to the caller (a3c_gemm_reduce, with
// the arguments as updated here: effective split, K chunk)
int a3c_gemm3(GemmArgs& g0, GemmArgs& g1, GemmArgs& g2, hipStream_t s);
int a3c_gemm_reduce(const GemmArgs& g, hipStream_t s);
int a3c_gemm_plan_split(int M, int N, int K, int target_blocks);

inline int a3c_gemm_effective_split(int K, int nsplit) {
  int ktiles = (K + 15) / 16;
  if (nsplit < 1) nsplit = 1;
  int per = (ktiles + nsplit - 1) / nsplit;
  return (ktiles + per - 1) / per;
}

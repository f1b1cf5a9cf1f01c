// FP32 GEMM on gfx950 matrix cores (v_mfma_f32_32x32x2_f32: exact fp32 products, fp32
// accumulation) for the fully-connected layers of the trunk (ops.py:32-46 ``linear``):
//   forward  l3 = relu(l2 @ W + b)                       (agent.py:251)
//   backward dW = l2^T @ dl3, db = colsum(dl3), dl2 = (dl3 @ W^T) * (l2 > 0)
//   heads    dWh = l3^T @ dz, dbh = colsum(dz)
// Tile 64x64x16, 256 threads = 2x2 waves of 32x32, LDS-staged operands with a register
// prefetch of the next K-tile, optional split-K into fp32 slabs (reduced by k_reduce_slabs
// with the epilogue) and an optional fused column sum of the B operand (bias gradients).
#include <cstdlib>
#include "gemm.h"

#define BM 64
#define BN 64
#define BK 16
#define PAD 4

template <bool A_KC, bool B_NC>
__global__ void __launch_bounds__(256) k_gemm_f32(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) float As[BK][BM + PAD];
  __shared__ __attribute__((aligned(16))) float Bs[BK][BN + PAD];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int ks = blockIdx.z;
  const int kbeg = ks * g.kchunk;
  const int kend = min(g.K, kbeg + g.kchunk);
  const bool do_colsum = g.colsum != nullptr && blockIdx.y == 0;

  // per-thread load coordinates
  int a_r, a_c, b_r, b_c;
  if (A_KC) { a_r = tid >> 2; a_c = (tid & 3) * 4; }   // row m, k quad
  else      { a_r = tid >> 4; a_c = (tid & 15) * 4; }  // row k, m quad
  if (B_NC) { b_r = tid >> 4; b_c = (tid & 15) * 4; }  // row k, n quad
  else      { b_r = tid >> 2; b_c = (tid & 3) * 4; }   // row n, k quad

  auto load_a = [&](int k0) -> f32x4 {
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (A_KC) {
      int m = m0 + a_r, k = k0 + a_c;
      if (m < g.M && k < kend) v = *(const f32x4*)(g.A + (int64_t)m * g.lda + k);
    } else {
      int k = k0 + a_r, m = m0 + a_c;
      if (k < kend && m < g.M) v = *(const f32x4*)(g.A + (int64_t)k * g.lda + m);
    }
    return v;
  };
  auto load_b = [&](int k0) -> f32x4 {
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (B_NC) {
      int k = k0 + b_r, n = n0 + b_c;
      if (k < kend && n < g.N) v = *(const f32x4*)(g.B + (int64_t)k * g.ldb + n);
    } else {
      int n = n0 + b_r, k = k0 + b_c;
      if (n < g.N && k < kend) v = *(const f32x4*)(g.B + (int64_t)n * g.ldb + k);
    }
    return v;
  };
  auto store_a = [&](f32x4 v) {
    if (A_KC) { As[a_c][a_r] = v[0]; As[a_c + 1][a_r] = v[1]; As[a_c + 2][a_r] = v[2]; As[a_c + 3][a_r] = v[3]; }
    else      { *(f32x4*)&As[a_r][a_c] = v; }
  };
  auto store_b = [&](f32x4 v) {
    if (B_NC) { *(f32x4*)&Bs[b_r][b_c] = v; }
    else      { Bs[b_c][b_r] = v[0]; Bs[b_c + 1][b_r] = v[1]; Bs[b_c + 2][b_r] = v[2]; Bs[b_c + 3][b_r] = v[3]; }
  };

  f32x16 acc = {};
  float csum = 0.f;
  f32x4 ra = load_a(kbeg), rb = load_b(kbeg);
  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    __syncthreads();
    store_a(ra);
    store_b(rb);
    __syncthreads();
    if (k0 + BK < kend) { ra = load_a(k0 + BK); rb = load_b(k0 + BK); }
    if (do_colsum && tid < BN) {
#pragma unroll
      for (int k = 0; k < BK; ++k) csum += Bs[k][tid];
    }
    const int kh = lane >> 5, c = lane & 31;
#pragma unroll
    for (int kk = 0; kk < BK / 2; ++kk) {
      float a = As[2 * kk + kh][wm * 32 + c];
      float b = Bs[2 * kk + kh][wn * 32 + c];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
  }

  const int col = n0 + wn * 32 + (lane & 31);
  if (g.nsplit > 1) {
    float* out = g.slab + (int64_t)ks * g.M * g.N;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      int row = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (row < g.M && col < g.N) out[(int64_t)row * g.N + col] = acc[r];
    }
  } else {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      int row = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (row < g.M && col < g.N) {
        float v = acc[r];
        if (g.epi == EPI_BIAS_RELU) v = fmaxf(v + g.bias[col], 0.f);
        else if (g.epi == EPI_BIAS) v = v + g.bias[col];
        else if (g.epi == EPI_MASK) v = g.mask[(int64_t)row * g.ldm + col] > 0.f ? v : 0.f;
        g.C[(int64_t)row * g.ldc + col] = v;
      }
    }
  }
  if (do_colsum && tid < BN && n0 + tid < g.N) g.colsum[(int64_t)ks * g.N + n0 + tid] = csum;
}

// C[M][N] = epi(A B^T) with both operands k-contiguous ("NT": A[m*lda + k], B[n*ldb + k]), K % 16 == 0:
// the backward's dl2 = (dl3 W^T) * (l2 > 0).  256 threads = 2x2 waves of 32x32 (2x2 16x16 tiles),
// operands straight from global/L1 as 16-byte k-permuted loads (mfma_k16), two k blocks in flight,
// four independent accumulator chains.
__global__ void __launch_bounds__(256) k_gemm_nt(GemmArgs g) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int i16 = lane & 15, j4 = lane >> 4;
  const int m0 = blockIdx.y * 64 + (w >> 1) * 32, n0 = blockIdx.x * 64 + (w & 1) * 32;
  const float* pa[2];
  const float* pb[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    pa[t] = g.A + (int64_t)min(m0 + 16 * t + i16, g.M - 1) * g.lda + 4 * j4;
    pb[t] = g.B + (int64_t)min(n0 + 16 * t + i16, g.N - 1) * g.ldb + 4 * j4;
  }
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int nb = g.K / 16;
  f32x4 a0[2], b0[2], a1[2], b1[2];
  auto load = [&](int kb, f32x4 (&a)[2], f32x4 (&b)[2]) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      a[t] = *(const f32x4*)(pa[t] + 16 * kb);
      b[t] = *(const f32x4*)(pb[t] + 16 * kb);
    }
  };
  auto mma = [&](const f32x4 (&a)[2], const f32x4 (&b)[2]) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = mfma_k16(a[i], b[j], acc[i][j]);
  };
  load(0, a0, b0);
  for (int kb = 0; kb < nb; kb += 2) {
    if (kb + 1 < nb) load(kb + 1, a1, b1);
    mma(a0, b0);
    if (kb + 2 < nb) load(kb + 2, a0, b0);
    if (kb + 1 < nb) mma(a1, b1);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + 16 * j + i16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + 16 * i + 4 * j4 + r;
        if (row < g.M && col < g.N) {
          float v = acc[i][j][r];
          if (g.epi == EPI_BIAS_RELU) v = fmaxf(v + g.bias[col], 0.f);
          else if (g.epi == EPI_BIAS) v = v + g.bias[col];
          else if (g.epi == EPI_MASK) v = g.mask[(int64_t)row * g.ldm + col] > 0.f ? v : 0.f;
          g.C[(int64_t)row * g.ldc + col] = v;
        }
      }
    }
}

// C[M][N] = sum_k A[k*lda + m] B[k*ldb + n] -- the weight gradients X^T Y over the batch ("TN"),
// M % 4 == N % 4 == 0.  One wave per 64x64 tile: lane (i16, j4) loads the 16-byte A[k][m0 + 4 i16 ..]
// and B[k][n0 + 4 i16 ..] at k = k0 + j4, which feed the 4x4 16x16 tiles whose rows are
// m0 + 4 r + sa and columns n0 + 4 c + sb (a row / column permutation the stores undo): 16 MFMAs per
// two 16-byte loads, no LDS.  Split-K over blockIdx.z into slabs (k_reduce_slabs); optional column
// sums of B (bias gradients) from the m-tile-0 waves.
__global__ void __launch_bounds__(64) k_gemm_tn(GemmArgs g) {
  const int lane = threadIdx.x, i16 = lane & 15, j4 = lane >> 4;
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  const int ks = blockIdx.z;
  const int kbeg = ks * g.kchunk, kend = min(g.K, kbeg + g.kchunk);
  const bool mv = m0 + 4 * i16 < g.M, nv = n0 + 4 * i16 < g.N;
  const float* pa = g.A + m0 + 4 * i16;
  const float* pb = g.B + n0 + 4 * i16;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  f32x4 cs = {0.f, 0.f, 0.f, 0.f};
  const bool do_colsum = g.colsum != nullptr && blockIdx.y == 0;
  // one iteration = 16 k (4 MFMA k-steps); two iterations' operands in flight
  f32x4 a0[4], b0[4], a1[4], b1[4];
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
  auto load = [&](int k0, f32x4 (&a)[4], f32x4 (&b)[4]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = k0 + 4 * q + j4;
      const bool kv = k < kend;
      a[q] = kv && mv ? *(const f32x4*)(pa + (int64_t)k * g.lda) : z4;
      b[q] = kv && nv ? *(const f32x4*)(pb + (int64_t)k * g.ldb) : z4;
    }
  };
  auto mma = [&](const f32x4 (&a)[4], const f32x4 (&b)[4]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int sa = 0; sa < 4; ++sa)
#pragma unroll
        for (int sb = 0; sb < 4; ++sb)
          acc[sa][sb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q][sa], b[q][sb], acc[sa][sb], 0, 0, 0);
      if (do_colsum) cs += b[q];
    }
  };
  if (kbeg < kend) load(kbeg, a0, b0);
  for (int k0 = kbeg; k0 < kend; k0 += 32) {
    const bool has1 = k0 + 16 < kend;
    if (has1) load(k0 + 16, a1, b1);
    mma(a0, b0);
    if (k0 + 32 < kend) load(k0 + 32, a0, b0);
    if (has1) mma(a1, b1);
  }
  float* out = g.nsplit > 1 ? g.slab + (int64_t)ks * g.M * g.N : g.C;
  const int64_t ld = g.nsplit > 1 ? g.N : g.ldc;
  if (nv) {
#pragma unroll
    for (int sa = 0; sa < 4; ++sa)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int m = m0 + 16 * j4 + 4 * q + sa;    // tile row r = 4 j4 + q -> m0 + 4 r + sa
        if (m < g.M)
          *(f32x4*)(out + (int64_t)m * ld + n0 + 4 * i16) =
              (f32x4){acc[sa][0][q], acc[sa][1][q], acc[sa][2][q], acc[sa][3][q]};
      }
  }
  if (do_colsum) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      cs[s] += __shfl_xor(cs[s], 16, 64);
      cs[s] += __shfl_xor(cs[s], 32, 64);
    }
    if (j4 == 0 && nv) *(f32x4*)(g.colsum + (int64_t)ks * g.N + n0 + 4 * i16) = cs;
  }
}

// dst[row*ldc + col] = epi(scale * sum_s slab[s][row][col])
__global__ void k_reduce_slabs(const float* __restrict__ slab, int nsplit, int M, int N,
                               float* __restrict__ C, int64_t ldc, int epi,
                               const float* __restrict__ bias, const float* __restrict__ mask,
                               int64_t ldm) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t total = (int64_t)M * N;
  if (i >= total) return;
  float v = 0.f;
  for (int s = 0; s < nsplit; ++s) v += slab[(int64_t)s * total + i];
  int row = (int)(i / N), col = (int)(i - (int64_t)row * N);
  if (epi == EPI_BIAS_RELU) v = fmaxf(v + bias[col], 0.f);
  else if (epi == EPI_BIAS) v = v + bias[col];
  else if (epi == EPI_MASK) v = mask[(int64_t)row * ldm + col] > 0.f ? v : 0.f;
  C[(int64_t)row * ldc + col] = v;
}

int a3c_gemm_plan_split(int M, int N, int K, int target_blocks) {
  int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  int ktiles = (K + BK - 1) / BK;
  int split = target_blocks / (tiles > 0 ? tiles : 1);
  if (split < 1) split = 1;
  if (split > ktiles) split = ktiles;
  if (split > 32) split = 32;
  return split;
}

int a3c_gemm(bool a_kc, bool b_nc, GemmArgs g, hipStream_t s) {
  if (g.M <= 0 || g.N <= 0) return 0;
  if (((a_kc || !b_nc) && (g.K & 3)) || (g.lda & 3) || (g.ldb & 3) ||
      (((uintptr_t)g.A | (uintptr_t)g.B) & 15) || (a_kc ? 0 : (g.M & 3)) || (b_nc ? (g.N & 3) : 0))
    return a3c_set_error(A3C_ERR_INVALID, "a3c_gemm", "unaligned operands (need 16-B alignment, dims %4)");
  if (g.nsplit < 1) g.nsplit = 1;
  static const bool nt_off = getenv("A3C_GEMM_NT") && atoi(getenv("A3C_GEMM_NT")) == 0;
  if (a_kc && !b_nc && g.nsplit == 1 && g.K % 16 == 0 && g.K > 0 && !nt_off) {
    hipLaunchKernelGGL(k_gemm_nt, dim3((g.N + 63) / 64, (g.M + 63) / 64), dim3(256), 0, s, g);
    A3C_CHECK(hipGetLastError());
    return 0;
  }
  int ktiles = (g.K + BK - 1) / BK;
  int per = (ktiles + g.nsplit - 1) / g.nsplit;
  g.kchunk = per * BK;
  g.nsplit = (ktiles + per - 1) / per;
  if (g.nsplit > 1 && !g.slab) return a3c_set_error(A3C_ERR_INVALID, "a3c_gemm", "split-K needs a slab");
  static const bool tn_off = getenv("A3C_GEMM_TN") && atoi(getenv("A3C_GEMM_TN")) == 0;
  if (!a_kc && b_nc && g.epi == EPI_STORE && (g.M & 3) == 0 && (g.N & 3) == 0 && (g.ldc & 3) == 0 &&
      (((uintptr_t)g.C | (uintptr_t)(g.slab ? g.slab : g.C) | (uintptr_t)(g.colsum ? g.colsum : g.C)) & 15) == 0 &&
      !tn_off) {
    dim3 grid((g.N + 63) / 64, (g.M + 63) / 64, g.nsplit);
    hipLaunchKernelGGL(k_gemm_tn, grid, dim3(64), 0, s, g);
    A3C_CHECK(hipGetLastError());
    if (g.nsplit > 1) {
      int64_t total = (int64_t)g.M * g.N;
      hipLaunchKernelGGL(k_reduce_slabs, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                         g.slab, g.nsplit, g.M, g.N, g.C, g.ldc, g.epi, g.bias, g.mask, g.ldm);
      A3C_CHECK(hipGetLastError());
    }
    return 0;
  }
  dim3 grid((g.N + BN - 1) / BN, (g.M + BM - 1) / BM, g.nsplit);
  if (a_kc && b_nc) hipLaunchKernelGGL((k_gemm_f32<true, true>), grid, dim3(256), 0, s, g);
  else if (a_kc && !b_nc) hipLaunchKernelGGL((k_gemm_f32<true, false>), grid, dim3(256), 0, s, g);
  else if (!a_kc && b_nc) hipLaunchKernelGGL((k_gemm_f32<false, true>), grid, dim3(256), 0, s, g);
  else hipLaunchKernelGGL((k_gemm_f32<false, false>), grid, dim3(256), 0, s, g);
  A3C_CHECK(hipGetLastError());
  if (g.nsplit > 1) {
    int64_t total = (int64_t)g.M * g.N;
    hipLaunchKernelGGL(k_reduce_slabs, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                       g.slab, g.nsplit, g.M, g.N, g.C, g.ldc, g.epi, g.bias, g.mask, g.ldm);
    A3C_CHECK(hipGetLastError());
  }
  return 0;
}

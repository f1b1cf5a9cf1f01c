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

// one 64x64 output tile (bx, by) over K-chunk bz of C = A B (the block body of k_gemm_f32)
template <bool A_KC, bool B_NC>
__device__ inline void gemm_tile(const GemmArgs& g, int bx, int by, int bz, float (&As)[BK][BM + PAD],
                                 float (&Bs)[BK][BN + PAD]) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int m0 = by * BM, n0 = bx * BN;
  const int ks = bz;
  const int kbeg = ks * g.kchunk;
  const int kend = min(g.K, kbeg + g.kchunk);
  const bool do_colsum = g.colsum != nullptr && by == 0;

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
#ifndef A3C_NO_MASKBITS
      else if (g.epi == EPI_MASKBITS) v = (g.maskbits[(int64_t)row * g.ldm + (col >> 5)] >> (col & 31)) & 1u ? v : 0.f;
#endif
        g.C[(int64_t)row * g.ldc + col] = v;
      }
    }
  }
  if (do_colsum && tid < BN && n0 + tid < g.N) g.colsum[(int64_t)ks * g.N + n0 + tid] = csum;
}

// One 64x64 tile per workgroup with the K range split across KS groups of 4 waves inside the
// workgroup (256 KS threads): group q accumulates k-tiles [q T, (q+1) T) with its own LDS
// operand buffers, then the partial tiles are folded through LDS in the fixed order
// ((acc_0 + acc_1) + acc_2) + ... and group 0 stores C (and the column sums of B) once: split-K
// without slabs in HBM and without a separate fold kernel (the backward's fc weight GEMM,
// K = n E = 1280).  Deterministic; every group runs the same trip count (k-tiles past K load zeros,
// whose products add exact zeros).
template <bool A_KC, bool B_NC, int KS>
__global__ void __launch_bounds__(256 * KS) k_gemm_f32_wks(GemmArgs g) {
  WGLOG(5);
  __shared__ __attribute__((aligned(16))) float As[KS][BK][BM + PAD];
  __shared__ __attribute__((aligned(16))) float Bs[KS][BK][BN + PAD];
  const int grp = threadIdx.x >> 8, tid = threadIdx.x & 255, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  int bx = blockIdx.x, by = blockIdx.y;
  if (g.xcd == 1) {
    // 1-D grid, XCD-grouped (speed only): the N tiles of M tile t get ids with id % 8 == t % 8, so
    // under round-robin dispatch one XCD's L2 fetches the tile's A strip (the n E x 64 block of l2)
    // for all of them instead of each N tile's XCD fetching it again; ids past the last tile exit
    const int gx = (g.N + BN - 1) / BN, gy = (g.M + BM - 1) / BM;
    const int id = blockIdx.x, slot = id >> 3;
    by = 8 * (slot / gx) + (id & 7);
    bx = slot % gx;
    if (by >= gy) return;
  }
  const int m0 = by * BM, n0 = bx * BN;
  const int ktiles = (g.K + BK - 1) / BK, per = (ktiles + KS - 1) / KS;
  const int kbeg = grp * per * BK, kend = min(g.K, kbeg + per * BK);
  const bool do_colsum = g.colsum != nullptr && by == 0;
  int a_r, a_c, b_r, b_c;
  if (A_KC) { a_r = tid >> 2; a_c = (tid & 3) * 4; } else { a_r = tid >> 4; a_c = (tid & 15) * 4; }
  if (B_NC) { b_r = tid >> 4; b_c = (tid & 15) * 4; } else { b_r = tid >> 2; b_c = (tid & 3) * 4; }
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
  float (&as)[BK][BM + PAD] = As[grp];
  float (&bs)[BK][BN + PAD] = Bs[grp];
  f32x16 acc = {};
  float csum = 0.f;
  f32x4 ra = load_a(kbeg), rb = load_b(kbeg);
  for (int it = 0; it < per; ++it) {
    const int k0 = kbeg + it * BK;
    __syncthreads();
    if (A_KC) { as[a_c][a_r] = ra[0]; as[a_c + 1][a_r] = ra[1]; as[a_c + 2][a_r] = ra[2]; as[a_c + 3][a_r] = ra[3]; }
    else      { *(f32x4*)&as[a_r][a_c] = ra; }
    if (B_NC) { *(f32x4*)&bs[b_r][b_c] = rb; }
    else      { bs[b_c][b_r] = rb[0]; bs[b_c + 1][b_r] = rb[1]; bs[b_c + 2][b_r] = rb[2]; bs[b_c + 3][b_r] = rb[3]; }
    __syncthreads();
    if (it + 1 < per) { ra = load_a(k0 + BK); rb = load_b(k0 + BK); }
    if (do_colsum && tid < BN) {
#pragma unroll
      for (int k = 0; k < BK; ++k) csum += bs[k][tid];
    }
    const int kh = lane >> 5, c = lane & 31;
#pragma unroll
    for (int kk = 0; kk < BK / 2; ++kk)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(as[2 * kk + kh][wm * 32 + c], bs[2 * kk + kh][wn * 32 + c], acc, 0, 0, 0);
  }
  // fold the groups' partial tiles in order through LDS (the operand buffers, free now)
  static_assert(KS * BK * (BM + PAD) >= 16 * 256 + BN, "fold buffer");
  float* fold = &As[0][0][0];
  for (int q = 1; q < KS; ++q) {
    __syncthreads();
    if (grp == q) {
#pragma unroll
      for (int r = 0; r < 16; ++r) fold[r * 256 + tid] = acc[r];
      if (do_colsum && tid < BN) fold[16 * 256 + tid] = csum;
    }
    __syncthreads();
    if (grp == 0) {
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] += fold[r * 256 + tid];
      if (do_colsum && tid < BN) csum += fold[16 * 256 + tid];
    }
  }
  if (grp != 0) return;
  const int col = n0 + wn * 32 + (lane & 31);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (row < g.M && col < g.N) {
      float v = acc[r];
      if (g.epi == EPI_BIAS_RELU) v = fmaxf(v + g.bias[col], 0.f);
      else if (g.epi == EPI_BIAS) v = v + g.bias[col];
      else if (g.epi == EPI_MASK) v = g.mask[(int64_t)row * g.ldm + col] > 0.f ? v : 0.f;
#ifndef A3C_NO_MASKBITS
      else if (g.epi == EPI_MASKBITS) v = (g.maskbits[(int64_t)row * g.ldm + (col >> 5)] >> (col & 31)) & 1u ? v : 0.f;
#endif
      g.C[(int64_t)row * g.ldc + col] = v;
    }
  }
  if (do_colsum && tid < BN && n0 + tid < g.N) g.colsum[n0 + tid] = csum;
}

// 128x128 tile of C = A B over K-chunk blockIdx.z: 4 waves (2 x 2), each a 64x64 block as 2 x 2
// v_mfma_f32_32x32x2f32 tiles; operands LDS-staged BK = 16 deep with a register prefetch of the
// next K step, two f32x4 of A and two of B per thread; split-K partials to the slab and the
// optional column sums of B as k_gemm_f32.  The same products as k_gemm_f32 summed in the same K
// order per output, so the result is bit-identical.
template <bool A_KC, bool B_NC>
__global__ void __launch_bounds__(256) k_gemm_f32_big(GemmArgs g) {
  WGLOG(5);
  constexpr int TM = 128, TN = 128;
  __shared__ __attribute__((aligned(16))) float As[BK][TM + PAD];
  __shared__ __attribute__((aligned(16))) float Bs[BK][TN + PAD];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int m0 = blockIdx.y * TM, n0 = blockIdx.x * TN;
  const int ks = blockIdx.z;
  const int kbeg = ks * g.kchunk;
  const int kend = min(g.K, kbeg + g.kchunk);
  const bool do_colsum = g.colsum != nullptr && blockIdx.y == 0;
  // per-thread load coordinates of element u = 0, 1
  auto a_rc = [&](int u, int& r, int& c) {
    if (A_KC) { r = (tid >> 2) + 64 * u; c = (tid & 3) * 4; }   // row m, k quad
    else      { r = (tid >> 5) + 8 * u; c = (tid & 31) * 4; }   // row k, m quad
  };
  auto b_rc = [&](int u, int& r, int& c) {
    if (B_NC) { r = (tid >> 5) + 8 * u; c = (tid & 31) * 4; }   // row k, n quad
    else      { r = (tid >> 2) + 64 * u; c = (tid & 3) * 4; }   // row n, k quad
  };
  auto load_a = [&](int k0, int u) -> f32x4 {
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    int r, c;
    a_rc(u, r, c);
    if (A_KC) {
      const int m = m0 + r, k = k0 + c;
      if (m < g.M && k < kend) v = *(const f32x4*)(g.A + (int64_t)m * g.lda + k);
    } else {
      const int k = k0 + r, m = m0 + c;
      if (k < kend && m < g.M) v = *(const f32x4*)(g.A + (int64_t)k * g.lda + m);
    }
    return v;
  };
  auto load_b = [&](int k0, int u) -> f32x4 {
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    int r, c;
    b_rc(u, r, c);
    if (B_NC) {
      const int k = k0 + r, n = n0 + c;
      if (k < kend && n < g.N) v = *(const f32x4*)(g.B + (int64_t)k * g.ldb + n);
    } else {
      const int n = n0 + r, k = k0 + c;
      if (n < g.N && k < kend) v = *(const f32x4*)(g.B + (int64_t)n * g.ldb + k);
    }
    return v;
  };
  auto store_a = [&](f32x4 v, int u) {
    int r, c;
    a_rc(u, r, c);
    if (A_KC) { As[c][r] = v[0]; As[c + 1][r] = v[1]; As[c + 2][r] = v[2]; As[c + 3][r] = v[3]; }
    else      { *(f32x4*)&As[r][c] = v; }
  };
  auto store_b = [&](f32x4 v, int u) {
    int r, c;
    b_rc(u, r, c);
    if (B_NC) { *(f32x4*)&Bs[r][c] = v; }
    else      { Bs[c][r] = v[0]; Bs[c + 1][r] = v[1]; Bs[c + 2][r] = v[2]; Bs[c + 3][r] = v[3]; }
  };
  f32x16 acc[2][2] = {};
  float csum = 0.f;
  f32x4 ra0 = load_a(kbeg, 0), ra1 = load_a(kbeg, 1), rb0 = load_b(kbeg, 0), rb1 = load_b(kbeg, 1);
  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    __syncthreads();
    store_a(ra0, 0); store_a(ra1, 1);
    store_b(rb0, 0); store_b(rb1, 1);
    __syncthreads();
    if (k0 + BK < kend) {
      ra0 = load_a(k0 + BK, 0); ra1 = load_a(k0 + BK, 1);
      rb0 = load_b(k0 + BK, 0); rb1 = load_b(k0 + BK, 1);
    }
    if (do_colsum && tid < TN) {
#pragma unroll
      for (int k = 0; k < BK; ++k) csum += Bs[k][tid];
    }
    const int kh = lane >> 5, c = lane & 31;
#pragma unroll
    for (int kk = 0; kk < BK / 2; ++kk) {
      const float a0 = As[2 * kk + kh][wm * 64 + c], a1 = As[2 * kk + kh][wm * 64 + 32 + c];
      const float b0 = Bs[2 * kk + kh][wn * 64 + c], b1 = Bs[2 * kk + kh][wn * 64 + 32 + c];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn * 64 + 32 * j + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 64 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row >= g.M || col >= g.N) continue;
        float v = acc[i][j][r];
        if (g.nsplit > 1) {
          g.slab[(int64_t)ks * g.M * g.N + (int64_t)row * g.N + col] = v;
        } else {
          if (g.epi == EPI_BIAS_RELU) v = fmaxf(v + g.bias[col], 0.f);
          else if (g.epi == EPI_BIAS) v = v + g.bias[col];
          else if (g.epi == EPI_MASK) v = g.mask[(int64_t)row * g.ldm + col] > 0.f ? v : 0.f;
#ifndef A3C_NO_MASKBITS
      else if (g.epi == EPI_MASKBITS) v = (g.maskbits[(int64_t)row * g.ldm + (col >> 5)] >> (col & 31)) & 1u ? v : 0.f;
#endif
          g.C[(int64_t)row * g.ldc + col] = v;
        }
      }
    }
  if (do_colsum && tid < TN && n0 + tid < g.N) g.colsum[(int64_t)ks * g.N + n0 + tid] = csum;
}

// tile number id of g's (N tiles, M tiles, K-chunks) grid, N fastest (as k_gemm_f32's blockIdx)
template <bool A_KC, bool B_NC>
__device__ inline void gemm_tile_id(const GemmArgs& g, int id, float (&As)[BK][BM + PAD], float (&Bs)[BK][BN + PAD]) {
  const int gx = (g.N + BN - 1) / BN, gy = (g.M + BM - 1) / BM;
  gemm_tile<A_KC, B_NC>(g, id % gx, (id / gx) % gy, id / (gx * gy), As, Bs);
}

template <bool A_KC, bool B_NC>
__global__ void __launch_bounds__(256) k_gemm_f32(GemmArgs g) {
  WGLOG(5);
  __shared__ __attribute__((aligned(16))) float As[BK][BM + PAD];
  __shared__ __attribute__((aligned(16))) float Bs[BK][BN + PAD];
  gemm_tile<A_KC, B_NC>(g, blockIdx.x, blockIdx.y, blockIdx.z, As, Bs);
}

// The same tiles on a 1-D grid in XCD-grouped order: workgroup id goes to XCD id % 8 under the
// round-robin dispatch, so the J tiles of group g (which share one operand strip) all get ids
// with id % 8 == g % 8 and that strip is fetched from HBM by one XCD's L2 instead of several.
// Ids past the last group exit at once.
template <bool A_KC, bool B_NC>
__global__ void __launch_bounds__(256) k_gemm_f32_x(GemmArgs g, int G, int J) {
  WGLOG(5);
  __shared__ __attribute__((aligned(16))) float As[BK][BM + PAD];
  __shared__ __attribute__((aligned(16))) float Bs[BK][BN + PAD];
  const int id = blockIdx.x, slot = id >> 3;
  const int grp = 8 * (slot / J) + (id & 7), j = slot % J;
  if (grp >= G) return;
  const int gx = (g.N + BN - 1) / BN, gy = (g.M + BM - 1) / BM;
  if (g.xcd == 1) gemm_tile<A_KC, B_NC>(g, j, grp % gy, grp / gy, As, Bs);
  else gemm_tile<A_KC, B_NC>(g, grp % gx, j, grp / gx, As, Bs);
}

// the tiles of a 3-D k_gemm_f32 grid (nb of them) on a capped grid, each workgroup looping over
// tile ids blockIdx.x, + gridDim.x, ... (gemm_tile's leading barrier guards the LDS reuse)
template <bool A_KC, bool B_NC>
__global__ void __launch_bounds__(256) k_gemm_f32_p(GemmArgs g, int nb) {
  WGLOG(5);
  __shared__ __attribute__((aligned(16))) float As[BK][BM + PAD];
  __shared__ __attribute__((aligned(16))) float Bs[BK][BN + PAD];
  for (int id = blockIdx.x; id < nb; id += gridDim.x) gemm_tile_id<A_KC, B_NC>(g, id, As, Bs);
}

// k_gemm_f32_x on a capped grid (a multiple of 8, so every id a workgroup visits keeps its XCD)
template <bool A_KC, bool B_NC>
__global__ void __launch_bounds__(256) k_gemm_f32_xp(GemmArgs g, int G, int J, int nid) {
  WGLOG(5);
  __shared__ __attribute__((aligned(16))) float As[BK][BM + PAD];
  __shared__ __attribute__((aligned(16))) float Bs[BK][BN + PAD];
  const int gx = (g.N + BN - 1) / BN, gy = (g.M + BM - 1) / BM;
  for (int id = blockIdx.x; id < nid; id += gridDim.x) {
    const int slot = id >> 3;
    const int grp = 8 * (slot / J) + (id & 7), j = slot % J;
    if (grp >= G) continue;
    if (g.xcd == 1) gemm_tile<A_KC, B_NC>(g, j, grp % gy, grp / gy, As, Bs);
    else gemm_tile<A_KC, B_NC>(g, grp % gx, j, grp / gx, As, Bs);
  }
}

// Several independent GEMMs in one launch (the backward's dW_head, dW_fc and dl2 all need only
// dz / dl3): workgroup ids [0, nb[0]) are GEMM 0's tiles, then GEMM 1's, then GEMM 2's -- one
// kernel boundary instead of three and one fill/drain tail.  Flavours: (A k-contiguous, B
// n-contiguous) = (false, true), (false, true), (true, false).
__global__ void __launch_bounds__(256) k_gemm_multi(GemmArgs g0, GemmArgs g1, GemmArgs g2, int nb0, int nb1) {
  WGLOG(5);
  __shared__ __attribute__((aligned(16))) float As[BK][BM + PAD];
  __shared__ __attribute__((aligned(16))) float Bs[BK][BN + PAD];
  // (each branch names its own kernel argument: selecting a pointer to one would copy all three
  // to scratch)
  const int id = blockIdx.x;
  if (id < nb0) gemm_tile_id<false, true>(g0, id, As, Bs);
  else if (id < nb0 + nb1) gemm_tile_id<false, true>(g1, id - nb0, As, Bs);
  else gemm_tile_id<true, false>(g2, id - nb0 - nb1, As, Bs);
}

// dst[row*ldc + col] = epi(scale * sum_s slab[s][row][col])
__global__ void k_reduce_slabs(const float* __restrict__ slab, int nsplit, int M, int N,
                               float* __restrict__ C, int64_t ldc, int epi,
                               const float* __restrict__ bias, const float* __restrict__ mask,
                               int64_t ldm, const uint32_t* __restrict__ maskbits) {
  WGLOG(8);
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t total = (int64_t)M * N;
  if (i >= total) return;
  float v = sum_strided(slab + i, nsplit, total);
  int row = (int)(i / N), col = (int)(i - (int64_t)row * N);
  if (epi == EPI_BIAS_RELU) v = fmaxf(v + bias[col], 0.f);
  else if (epi == EPI_BIAS) v = v + bias[col];
  else if (epi == EPI_MASK) v = mask[(int64_t)row * ldm + col] > 0.f ? v : 0.f;
#ifndef A3C_NO_MASKBITS
  else if (epi == EPI_MASKBITS) v = (maskbits[(int64_t)row * ldm + (col >> 5)] >> (col & 31)) & 1u ? v : 0.f;
#endif
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

// shared by a3c_gemm and a3c_gemm3: alignment checks, effective split, K-chunk
static int gemm_setup(bool a_kc, bool b_nc, GemmArgs& g) {
  if (((a_kc || !b_nc) && (g.K & 3)) || (g.lda & 3) || (g.ldb & 3) ||
      (((uintptr_t)g.A | (uintptr_t)g.B) & 15) || (a_kc ? 0 : (g.M & 3)) || (b_nc ? (g.N & 3) : 0))
    return a3c_set_error(A3C_ERR_INVALID, "a3c_gemm", "unaligned operands (need 16-B alignment, dims %4)");
  if (g.nsplit < 1) g.nsplit = 1;
  const int ktiles = (g.K + BK - 1) / BK;
  const int per = (ktiles + g.nsplit - 1) / g.nsplit;
  g.kchunk = per * BK;
  g.nsplit = (ktiles + per - 1) / per;
  if (g.nsplit > 1 && !g.slab) return a3c_set_error(A3C_ERR_INVALID, "a3c_gemm", "split-K needs a slab");
  return 0;
}

static void gemm_reduce(const GemmArgs& g, hipStream_t s) {
  const int64_t total = (int64_t)g.M * g.N;
  hipLaunchKernelGGL(k_reduce_slabs, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                     g.slab, g.nsplit, g.M, g.N, g.C, g.ldc, g.epi, g.bias, g.mask, g.ldm, g.maskbits);
}

int a3c_gemm3(GemmArgs& g0, GemmArgs& g1, GemmArgs& g2, hipStream_t s) {
  if (g0.M <= 0 || g0.N <= 0 || g1.M <= 0 || g1.N <= 0 || g2.M <= 0 || g2.N <= 0)
    return a3c_set_error(A3C_ERR_INVALID, "a3c_gemm3", "empty GEMM");
  int rc = gemm_setup(false, true, g0);
  if (!rc) rc = gemm_setup(false, true, g1);
  if (!rc) rc = gemm_setup(true, false, g2);
  if (rc) return rc;
  auto blocks = [](const GemmArgs& g) {
    return ((g.N + BN - 1) / BN) * ((g.M + BM - 1) / BM) * g.nsplit;
  };
  const int nb0 = blocks(g0), nb1 = blocks(g1), nb2 = blocks(g2);
  hipLaunchKernelGGL(k_gemm_multi, dim3((unsigned)(nb0 + nb1 + nb2)), dim3(256), 0, s, g0, g1, g2, nb0, nb1);
  A3C_CHECK(hipGetLastError());
  return 0;
}

int a3c_gemm_reduce(const GemmArgs& g, hipStream_t s) {
  if (g.nsplit > 1) {
    gemm_reduce(g, s);
    A3C_CHECK(hipGetLastError());
  }
  return 0;
}

int a3c_gemm(bool a_kc, bool b_nc, GemmArgs g, hipStream_t s) {
  if (g.M <= 0 || g.N <= 0) return 0;
  if (g.wg_split == 4) {   // in-workgroup split-K (k_gemm_f32_wks): no slab, no fold kernel
    g.nsplit = 1;
    int rc = gemm_setup(a_kc, b_nc, g);
    if (rc) return rc;
    const int gx = (g.N + BN - 1) / BN, gy = (g.M + BM - 1) / BM;
    // g.xcd == 1: XCD-grouped 1-D grid (the kernel maps ids to tiles), else the plain 2-D grid
    const dim3 grid = g.xcd == 1 ? dim3((unsigned)(8 * ((gy + 7) / 8) * gx)) : dim3(gx, gy, 1);
    if (g.xcd != 0 && g.xcd != 1) return a3c_set_error(A3C_ERR_INVALID, "a3c_gemm", "wg_split: xcd 0 or 1");
    if (a_kc && b_nc) hipLaunchKernelGGL((k_gemm_f32_wks<true, true, 4>), grid, dim3(1024), 0, s, g);
    else if (a_kc && !b_nc) hipLaunchKernelGGL((k_gemm_f32_wks<true, false, 4>), grid, dim3(1024), 0, s, g);
    else if (!a_kc && b_nc) hipLaunchKernelGGL((k_gemm_f32_wks<false, true, 4>), grid, dim3(1024), 0, s, g);
    else hipLaunchKernelGGL((k_gemm_f32_wks<false, false, 4>), grid, dim3(1024), 0, s, g);
    A3C_CHECK(hipGetLastError());
    return 0;
  }
  if (g.wg_split > 1) return a3c_set_error(A3C_ERR_INVALID, "a3c_gemm", "wg_split: 4 only");
  int rc = gemm_setup(a_kc, b_nc, g);
  if (rc) return rc;
  dim3 grid((g.N + BN - 1) / BN, (g.M + BM - 1) / BM, g.nsplit);
  // XCD-grouped order where the caller asks for it (the overlapped backward when it bounds the
  // iteration): it halves the backward GEMMs' HBM bytes, 124 -> 73 MB per iteration (profile
  // r3v1), but beside a rollout that bounds the iteration it costs 4.56M -> 4.05M env-steps/s
  const int nb = (int)(grid.x * grid.y * grid.z);
  if (g.big) {
    const dim3 gb((g.N + 127) / 128, (g.M + 127) / 128, g.nsplit);
    if (a_kc && b_nc) hipLaunchKernelGGL((k_gemm_f32_big<true, true>), gb, dim3(256), 0, s, g);
    else if (a_kc && !b_nc) hipLaunchKernelGGL((k_gemm_f32_big<true, false>), gb, dim3(256), 0, s, g);
    else if (!a_kc && b_nc) hipLaunchKernelGGL((k_gemm_f32_big<false, true>), gb, dim3(256), 0, s, g);
    else hipLaunchKernelGGL((k_gemm_f32_big<false, false>), gb, dim3(256), 0, s, g);
    A3C_CHECK(hipGetLastError());
    return g.defer_reduce ? 0 : a3c_gemm_reduce(g, s);
  }
  if (g.xcd) {
    const int G = g.xcd == 1 ? (int)(grid.y * grid.z) : (int)(grid.x * grid.z);
    const int J = g.xcd == 1 ? (int)grid.x : (int)grid.y;
    const int nid = 8 * ((G + 7) / 8) * J;
    if (g.max_wgs > 0 && nid > g.max_wgs) {
      const dim3 gp((unsigned)(8 * ((g.max_wgs + 7) / 8)));
      if (a_kc && b_nc) hipLaunchKernelGGL((k_gemm_f32_xp<true, true>), gp, dim3(256), 0, s, g, G, J, nid);
      else if (a_kc && !b_nc) hipLaunchKernelGGL((k_gemm_f32_xp<true, false>), gp, dim3(256), 0, s, g, G, J, nid);
      else if (!a_kc && b_nc) hipLaunchKernelGGL((k_gemm_f32_xp<false, true>), gp, dim3(256), 0, s, g, G, J, nid);
      else hipLaunchKernelGGL((k_gemm_f32_xp<false, false>), gp, dim3(256), 0, s, g, G, J, nid);
      A3C_CHECK(hipGetLastError());
      return g.defer_reduce ? 0 : a3c_gemm_reduce(g, s);
    }
    const dim3 g1((unsigned)nid);
    if (a_kc && b_nc) hipLaunchKernelGGL((k_gemm_f32_x<true, true>), g1, dim3(256), 0, s, g, G, J);
    else if (a_kc && !b_nc) hipLaunchKernelGGL((k_gemm_f32_x<true, false>), g1, dim3(256), 0, s, g, G, J);
    else if (!a_kc && b_nc) hipLaunchKernelGGL((k_gemm_f32_x<false, true>), g1, dim3(256), 0, s, g, G, J);
    else hipLaunchKernelGGL((k_gemm_f32_x<false, false>), g1, dim3(256), 0, s, g, G, J);
    A3C_CHECK(hipGetLastError());
    return g.defer_reduce ? 0 : a3c_gemm_reduce(g, s);
  }
  if (g.max_wgs > 0 && nb > g.max_wgs) {
    const dim3 gp((unsigned)g.max_wgs);
    if (a_kc && b_nc) hipLaunchKernelGGL((k_gemm_f32_p<true, true>), gp, dim3(256), 0, s, g, nb);
    else if (a_kc && !b_nc) hipLaunchKernelGGL((k_gemm_f32_p<true, false>), gp, dim3(256), 0, s, g, nb);
    else if (!a_kc && b_nc) hipLaunchKernelGGL((k_gemm_f32_p<false, true>), gp, dim3(256), 0, s, g, nb);
    else hipLaunchKernelGGL((k_gemm_f32_p<false, false>), gp, dim3(256), 0, s, g, nb);
    A3C_CHECK(hipGetLastError());
    return g.defer_reduce ? 0 : a3c_gemm_reduce(g, s);
  }
  if (a_kc && b_nc) hipLaunchKernelGGL((k_gemm_f32<true, true>), grid, dim3(256), 0, s, g);
  else if (a_kc && !b_nc) hipLaunchKernelGGL((k_gemm_f32<true, false>), grid, dim3(256), 0, s, g);
  else if (!a_kc && b_nc) hipLaunchKernelGGL((k_gemm_f32<false, true>), grid, dim3(256), 0, s, g);
  else hipLaunchKernelGGL((k_gemm_f32<false, false>), grid, dim3(256), 0, s, g);
  A3C_CHECK(hipGetLastError());
  return g.defer_reduce ? 0 : a3c_gemm_reduce(g, s);
}

#ifdef A3C_WGLOG
WGLOG_BIND(a3c_wglog_bind_gemm)
#endif

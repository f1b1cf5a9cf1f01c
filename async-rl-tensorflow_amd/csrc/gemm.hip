// FP32 GEMM on gfx950 matrix cores (v_mfma_f32_32x32x2_f32: exact fp32 products, fp32
// accumulation) for the fully-connected layers of the trunk (ops.py:32-46 ``linear``):
//   forward  l3 = relu(l2 @ W + b)                       (agent.py:251)
//   backward dW = l2^T @ dl3, db = colsum(dl3), dl2 = (dl3 @ W^T) * (l2 > 0)
//   heads    dWh = l3^T @ dz, dbh = colsum(dz)
// Tile 64x64x16, 256 threads = 2x2 waves of 32x32, LDS-staged operands with a register
// prefetch of the next K-tile, optional split-K into fp32 slabs (reduced by k_reduce_slabs
// with the epilogue) and an optional fused column sum of the B operand (bias gradients).
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
  int ktiles = (g.K + BK - 1) / BK;
  int per = (ktiles + g.nsplit - 1) / g.nsplit;
  g.kchunk = per * BK;
  g.nsplit = (ktiles + per - 1) / per;
  if (g.nsplit > 1 && !g.slab) return a3c_set_error(A3C_ERR_INVALID, "a3c_gemm", "split-K needs a slab");
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

// ---------------------------------------------------------------------------------------
// fc-layer backward GEMMs (agent.py:317 compute_gradients of ops.py:32-46 ``linear``) on
// v_mfma_f32_32x32x2_f32 (exact fp32 products, fp32 accumulation).  A workgroup is 4 waves in
// 2x2 over a 64x64 output tile, each wave a 32x32 quarter.  Per 8-deep K chunk a lane holds
// k = 8c + 4h + j (h = lane >> 5, j = 0..3) of its A row and of its B column and issues 4 MFMAs
// (the same k permutation on both sides).  Loads run D chunks ahead of their MFMAs;
// sched_barrier keeps hipcc from sinking them to their use (it otherwise waits vmcnt(0) on
// every chunk).
//  k_gemm_nt_mask   C[m][n] = (sum_k A[m][k] B[n][k]) * (mask[m][n] > 0), full K per workgroup:
//                   dl2 = (dl3 W^T) * (l2 > 0).  A, B k-contiguous: one float4 per operand.
//  k_gemm_tn_splitk C[m][n] = sum_k A[k][m] B[k][n], K split over gridDim.y workgroups whose
//                   partial tiles the last one to finish folds in a fixed order (write-through
//                   sc1 stores, ticket, agent-scope acquire); colsum[s][n] = sum over split s
//                   of B[k][n] (bias gradient): dW = l2^T dl3, db.  A, B m/n-contiguous: four
//                   dwords per operand (two 128-B rows per instruction).
// ---------------------------------------------------------------------------------------
#define G32_D 8
__device__ inline void g32_store_tile(const f32x16& acc, float* C, int64_t ldc, int M, int N, int m0, int n0,
                                      int lane) {
  const int col = n0 + (lane & 31);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = m0 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (row < M && col < N) C[(int64_t)row * ldc + col] = acc[r];
  }
}

__global__ void __launch_bounds__(256) k_gemm_nt_mask(const float* __restrict__ A, int64_t lda,
                                                      const float* __restrict__ B, int64_t ldb,
                                                      float* __restrict__ C, int64_t ldc,
                                                      const float* __restrict__ mask, int64_t ldm, int M, int N,
                                                      int K, int ntm) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int i32 = lane & 31, h = lane >> 5;
  const int tm = blockIdx.x % ntm, tn = blockIdx.x / ntm;      // n-major: a W tile's workgroups adjacent
  const int m0 = 64 * tm + 32 * (wid >> 1), n0 = 64 * tn + 32 * (wid & 1);
  const float* a = A + (int64_t)min(m0 + i32, M - 1) * lda + 4 * h;
  const float* b = B + (int64_t)min(n0 + i32, N - 1) * ldb + 4 * h;
  const int nch = K / 8;
  f32x4 ra[G32_D], rb[G32_D];
  f32x16 acc = {};
#pragma unroll
  for (int d = 0; d < G32_D; ++d) {
    const int c = min(d, nch - 1);
    ra[d] = *(const f32x4*)(a + 8 * c);
    rb[d] = *(const f32x4*)(b + 8 * c);
  }
  // the epilogue's mask values, loaded up front (behind the first operands, off the critical path)
  float mk[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = min(m0 + (r & 3) + 8 * (r >> 2) + 4 * h, M - 1);
    mk[r] = mask[(int64_t)row * ldm + min(n0 + i32, N - 1)];
  }
  __builtin_amdgcn_sched_barrier(0);
  for (int c = 0; c < nch; c += G32_D) {
#pragma unroll
    for (int d = 0; d < G32_D; ++d) {
      const f32x4 av = c + d < nch ? ra[d] : (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 4; ++q) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[q], rb[d][q], acc, 0, 0, 0);
      const int cn = min(c + d + G32_D, nch - 1);               // refill (clamped: always issued)
      ra[d] = *(const f32x4*)(a + 8 * cn);
      rb[d] = *(const f32x4*)(b + 8 * cn);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = mk[r] > 0.f ? acc[r] : 0.f;
  g32_store_tile(acc, C, ldc, M, N, m0, n0, lane);
}

__global__ void __launch_bounds__(256) k_gemm_tn_splitk(const float* __restrict__ A, int64_t lda,
                                                        const float* __restrict__ B, int64_t ldb,
                                                        float* __restrict__ C, int64_t ldc, int M, int N, int K,
                                                        int ntm, int kper, float* __restrict__ slab,
                                                        uint32_t* __restrict__ cnt, float* __restrict__ colsum) {
  typedef __attribute__((address_space(1))) uint64_t gu64;
  typedef __attribute__((address_space(1))) uint32_t gu32;
  __shared__ uint32_t s_ticket;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int i32 = lane & 31, h = lane >> 5;
  const int tile = blockIdx.x, split = blockIdx.y, S = gridDim.y;
  const int tm = tile % ntm, tn = tile / ntm;
  const int m0 = 64 * tm + 32 * (wid >> 1), n0 = 64 * tn + 32 * (wid & 1);
  const int k0 = split * kper, k1 = min(K, k0 + kper);
  const float* a = A + min(m0 + i32, M - 1);
  const float* b = B + min(n0 + i32, N - 1);
  const int nch = (k1 - k0 + 7) / 8;
  // chunk c: rows k = k0 + 8c + 4h + j, clamped into [k0, k1) for the load; the rows past k1
  // are zeroed where they are consumed (a select right after the load would make hipcc wait for
  // it there and drain the ring)
  auto load = [&](int c, f32x4& va, f32x4& vb) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int kc = min(k0 + 8 * c + 4 * h + j, k1 - 1);
      va[j] = a[(int64_t)kc * lda];
      vb[j] = b[(int64_t)kc * ldb];
    }
  };
  f32x4 ra[G32_D], rb[G32_D];
  f32x16 acc = {};
  float cs = 0.f;                                   // this lane's share of B's column sum
#pragma unroll
  for (int d = 0; d < G32_D; ++d) load(min(d, nch - 1), ra[d], rb[d]);
  __builtin_amdgcn_sched_barrier(0);
  for (int c = 0; c < nch; c += G32_D) {
#pragma unroll
    for (int d = 0; d < G32_D; ++d) {
      f32x4 av, bv;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool kv = k0 + 8 * (c + d) + 4 * h + j < k1;   // also false for the ring's tail chunks
        av[j] = kv ? ra[d][j] : 0.f;
        bv[j] = kv ? rb[d][j] : 0.f;
      }
      cs += (bv[0] + bv[1]) + (bv[2] + bv[3]);
#pragma unroll
      for (int q = 0; q < 4; ++q) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[q], bv[q], acc, 0, 0, 0);
      load(min(c + d + G32_D, nch - 1), ra[d], rb[d]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // bias gradient of this split: the top row of waves of row tile 0 (every column once)
  if (colsum && tm == 0 && (wid >> 1) == 0) {
    cs += __shfl_xor(cs, 32, 64);
    if (h == 0 && n0 + i32 < N) colsum[(int64_t)split * N + n0 + i32] = cs;
  }
  if (S == 1) {
    g32_store_tile(acc, C, ldc, M, N, m0, n0, lane);
    return;
  }
  // publish the wave's quarter of the partial tile: [split][tile][wave][register pair][lane]
  gu64* mine = (gu64*)(slab + (((int64_t)split * gridDim.x + tile) * 4 + wid) * 1024) + lane;
#pragma unroll
  for (int r = 0; r < 16; r += 2) {
    const uint64_t v = (uint64_t)__float_as_uint(acc[r]) | ((uint64_t)__float_as_uint(acc[r + 1]) << 32);
    __hip_atomic_store(mine + 32 * r, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");           // every storing wave drains
  __syncthreads();
  if (threadIdx.x == 0)
    s_ticket = __hip_atomic_fetch_add((gu32*)(cnt + tile), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (s_ticket != (uint32_t)(S - 1)) return;                 // not the tile's last workgroup
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (threadIdx.x == 0) __hip_atomic_store((gu32*)(cnt + tile), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const float2* ps = (const float2*)(slab + ((int64_t)tile * 4 + wid) * 1024) + lane;
#pragma unroll
  for (int sp = 0; sp < S; ++sp)
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
      const float2 v = ps[(int64_t)sp * gridDim.x * 2048 + 32 * r];
      acc[r] = sp ? acc[r] + v.x : v.x;
      acc[r + 1] = sp ? acc[r + 1] + v.y : v.y;
    }
  g32_store_tile(acc, C, ldc, M, N, m0, n0, lane);
}

int a3c_gemm_nt_mask(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
                     const float* mask, int64_t ldm, int M, int N, int K, hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  if ((K & 7) || K <= 0 || (lda & 3) || (ldb & 3) || (((uintptr_t)A | (uintptr_t)B) & 15))
    return a3c_set_error(A3C_ERR_INVALID, "a3c_gemm_nt_mask", "K % 8, 16-B aligned rows needed");
  const int ntm = (M + 63) / 64, ntn = (N + 63) / 64;
  hipLaunchKernelGGL(k_gemm_nt_mask, dim3((unsigned)(ntm * ntn)), dim3(256), 0, s, A, lda, B, ldb, C, ldc, mask, ldm,
                     M, N, K, ntm);
  A3C_CHECK(hipGetLastError());
  return 0;
}

int a3c_gemm_tn_splitk(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc, int M, int N,
                       int K, int nsplit, float* slab, uint32_t* cnt, float* colsum, hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  if (K <= 0 || nsplit < 1 || (nsplit > 1 && (!slab || !cnt)))
    return a3c_set_error(A3C_ERR_INVALID, "a3c_gemm_tn_splitk", "bad argument");
  const int kper = ((K + nsplit - 1) / nsplit + 7) / 8 * 8;
  const int S = (K + kper - 1) / kper;
  const int ntm = (M + 63) / 64, ntn = (N + 63) / 64;
  hipLaunchKernelGGL(k_gemm_tn_splitk, dim3((unsigned)(ntm * ntn), (unsigned)S), dim3(256), 0, s, A, lda, B, ldb, C,
                     ldc, M, N, K, ntm, kper, slab, cnt, colsum);
  A3C_CHECK(hipGetLastError());
  return 0;
}

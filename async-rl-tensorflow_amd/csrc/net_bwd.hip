#include <algorithm>
#include <cstdlib>
// Loss + backward of the NIPS trunk on gfx950.
//
//  k_returns     n-step return per env in float64 (assets/a3c.png Algorithm S3).
//  k_td_target   agent.py:186-190 in float64.
//  k_head_bwd    one wave per sample: softmax/log-softmax/entropy, network.py:81-94 losses
//                (A11 fixes) or agent.py:310-314 MSE, dz, dl3 = (W_h dz) * (l3 > 0).
//  fc layer      gemm.hip: dW = l2^T dl3 (+colsum -> db), dl2 = (dl3 W^T) * (l2 > 0),
//                dW_h = l3^T dz (+colsum -> db_h).
//  k_conv_bwd    one workgroup per group of samples, three MFMA phases on LDS-resident tiles:
//                dW2 += patches(l1)^T dl2, dl1 = col2im(dl2 W2^T) * (l1 > 0) computed per
//                stride-2 parity class (4 waves = 4 classes, K = 2x2 taps x 32), and
//                dW1 += patches(x/255)^T dl1 (conv1 gets weight grads only) on the bf16
//                matrix cores: u8 pixels are exact in bf16 and dl1 is split into three bf16
//                terms, so every product is exact in the fp32 accumulator (5x fewer MFMA
//                cycles than fp32 16x16x4).  Per-workgroup partial slabs, reduced
//                deterministically by k_finalize.
#include "net.h"
#include "gemm.h"
#include "net_bwd.h"
#ifdef A3C_MARKERS
void a3c_mark(int id, hipStream_t s);
#endif

// ---------------------------------------------------------------------------------------
__global__ void k_returns(const float* __restrict__ rewards, const uint8_t* __restrict__ terms,
                          const float* __restrict__ boot, int64_t boot_stride, int n, int64_t E,
                          double gamma, float* __restrict__ R) {
#pragma clang fp contract(off)
  int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  double r = (double)boot[e * boot_stride];
  for (int i = n - 1; i >= 0; --i) {
    if (terms[i * E + e]) r = 0.0;
    r = (double)rewards[i * E + e] + gamma * r;
    R[i * E + e] = (float)r;
  }
}

// agent.py:186-190 (max_a Q'(s')), or with qsel the double-Q form agent.py:176-184: the target
// net's value at the online net's argmax (tf.argmax: the first maximum)
__global__ void k_td_target(const float* __restrict__ rewards, const uint8_t* __restrict__ terms,
                            const float* __restrict__ qn, int64_t B, int A, int zs, double discount,
                            float* __restrict__ target, const float* __restrict__ qsel) {
#pragma clang fp contract(off)
  int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float m = qn[b * zs];
  if (qsel) {
    float best = qsel[b * zs];
    int arg = 0;
    for (int j = 1; j < A; ++j) {
      const float v = qsel[b * zs + j];
      if (v > best) { best = v; arg = j; }
    }
    m = qn[b * zs + arg];
  } else {
    for (int j = 1; j < A; ++j) m = fmaxf(m, qn[b * zs + j]);
  }
  double t = terms[b] ? 1.0 : 0.0;
  double v = (1.0 - t) * discount * (double)m + (double)rewards[b];
  target[b] = (float)v;
}

// ---------------------------------------------------------------------------------------
// W: the head's input width (FC = 256, NIPS trunk; NT_FC = 512, nature trunk)
template <int W>
__global__ void __launch_bounds__(256) k_head_bwd(const float* __restrict__ z, int zs, int A, int algo,
                                                  const int32_t* __restrict__ actions,
                                                  const float* __restrict__ target,
                                                  const float* __restrict__ h3,
                                                  const float* __restrict__ Wp,
                                                  const float* __restrict__ Wv, float beta,
                                                  int literal, float invB, int64_t B,
                                                  float* __restrict__ dz, float* __restrict__ dh3,
                                                  float* __restrict__ terms, ReturnsArgs ra, int relu) {
  WGLOG(7);
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const float myz = lane < zs ? z[b * zs + lane] : 0.f;
  const int a = actions[b];
  float tgt;
  if (ra.rewards) {
    // n-step return of sample (t, e) (assets/a3c.png), float64 like k_returns
#pragma clang fp contract(off)
    const int64_t t = b / ra.E, e = b - t * ra.E;
    double r = (double)ra.boot[e * ra.boot_stride];
    for (int64_t i = ra.n - 1; i >= t; --i) {
      if (ra.terms[i * ra.E + e]) r = 0.0;
      r = (double)ra.rewards[i * ra.E + e] + ra.gamma * r;
    }
    tgt = (float)r;
    if (lane == 0) ra.R_out[b] = tgt;
  } else {
    tgt = target[b];
  }
  float mydz = 0.f, dV = 0.f;
  if (algo == A3C_ALGO_A3C) {
    float l = lane < A ? myz : -INFINITY;
    float m = wave_max(l);
    float ex = lane < A ? expf(myz - m) : 0.f;
    float s = wave_sum(ex);
    float pi = lane < A ? ex / s : 0.f;
    float logpi = lane < A ? (myz - m) - logf(s) : 0.f;
    float H = -wave_sum(lane < A ? pi * logpi : 0.f);
    float V = __shfl(myz, A, 64);
    float adv = tgt - V;
    float lpa = __shfl(logpi, a, 64);
    if (lane < A) mydz = -adv * ((lane == a ? 1.f : 0.f) - pi) + beta * pi * (logpi + H);
    dV = -adv + (literal ? lpa : 0.f);
    if (lane == A) mydz = dV;
    if (lane == 0) {
      float pl = -(lpa * adv) - beta * H;
      float vl = 0.5f * adv * adv;
      terms[b * 4 + 0] = pl;
      terms[b * 4 + 1] = vl;
      terms[b * 4 + 2] = H;
      terms[b * 4 + 3] = pl + vl;
    }
  } else {
    float qa = __shfl(myz, a, 64);
    float delta = tgt - qa;
    if (lane == a) mydz = -2.f * delta * invB;
    if (lane == 0) {
      terms[b * 4 + 0] = delta * delta * invB;
      terms[b * 4 + 1] = qa * invB;
      terms[b * 4 + 2] = 0.f;
      terms[b * 4 + 3] = 0.f;
    }
  }
  if (lane < zs) dz[b * zs + lane] = mydz;
  if constexpr (W == FC) {
    // dl3[k] = (sum_j W[k][j] dz_j) * (l3[k] > 0), k = 4*lane + i
    f32x4 g = {0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < A; ++j) {
      float dj = __shfl(mydz, j, 64);
#pragma unroll
      for (int i = 0; i < 4; ++i) g[i] += Wp[(int64_t)(4 * lane + i) * A + j] * dj;
    }
    if (Wv) {
      f32x4 wv = *(const f32x4*)(Wv + 4 * lane);
#pragma unroll
      for (int i = 0; i < 4; ++i) g[i] += wv[i] * dV;
    }
    if (relu) {    // feed-forward head: through the fc ReLU; LSTM head: dL/dh as is
      f32x4 h = *(const f32x4*)(h3 + b * FC + 4 * lane);
#pragma unroll
      for (int i = 0; i < 4; ++i) g[i] = h[i] > 0.f ? g[i] : 0.f;
    }
    *(f32x4*)(dh3 + b * FC + 4 * lane) = g;
  } else {
    // the same per feature k = 256 q + 4 lane + i, q < W / 256
    constexpr int NQ = W / 256;
    f32x4 g[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) g[q] = (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < A; ++j) {
      float dj = __shfl(mydz, j, 64);
#pragma unroll
      for (int q = 0; q < NQ; ++q)
#pragma unroll
        for (int i = 0; i < 4; ++i) g[q][i] += Wp[(int64_t)(256 * q + 4 * lane + i) * A + j] * dj;
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      if (Wv) {
        f32x4 wv = *(const f32x4*)(Wv + 256 * q + 4 * lane);
#pragma unroll
        for (int i = 0; i < 4; ++i) g[q][i] += wv[i] * dV;
      }
      if (relu) {
        f32x4 h = *(const f32x4*)(h3 + b * W + 256 * q + 4 * lane);
#pragma unroll
        for (int i = 0; i < 4; ++i) g[q][i] = h[i] > 0.f ? g[q][i] : 0.f;
      }
      *(f32x4*)(dh3 + b * W + 256 * q + 4 * lane) = g[q];
    }
  }
}

// ---------------------------------------------------------------------------------------
// fused conv backward
// ---------------------------------------------------------------------------------------
#define CB_X8 (HIST * PLANE)                 // 28224
// Two LDS layouts (template switch LX, see k_conv_bwd):
//  base (LX = 0): l1 [400][16] in rows of 20 floats, dl2 [81][32] in rows of 36;
//  lean (LX = 1): l1 rows of 24 floats, so phase (a)'s two 16-lane halves of a ds_read_b32
//    (positions 2 apart) fall on disjoint 16-bank halves of the 32 banks (rows of 20 overlap 8);
//    dl2 with the channels interleaved in pairs (co, co + 16) -- row q holds dl2[q][0],
//    dl2[q][16], dl2[q][1], dl2[q][17], ... -- so phase (a) reads its two B values with one
//    ds_read_b64; db2 summed by every wave over a row residue instead of one wave over all rows;
//    the dl1 term split writes a dword per term for two positions.  Measured (profile r3, PMC):
//    LDS-array cycles -20 %, bank-conflict cycles -34 %, conv backward alone 131 -> 122 us
//    (compact) and 82 -> 75 us (DMA).  Rows of 36 spread phase (b)'s ds_read_b128 rows over the
//    64 banks in both.
constexpr int cb_l1_ld(bool lx) { return lx ? 24 : 20; }
constexpr int cb_l1_bytes(bool lx) { return C1_P * cb_l1_ld(lx) * 4; }   // 32000 / 38400
#define CB_DL2_LD 36
#define CB_DL2 ((C2_Q + 1) * CB_DL2_LD * 4)  // 11808: row C2_Q stays zero (phase (b) off-grid taps)
__device__ inline int dl2_col(int co) { return 2 * (co & 15) + (co >> 4); }
#define CB_L1ST (C1_P * C1_N * 4)            // 25600: linear DMA staging of l1
#define CB_DL2ST (FLAT * 4)                  // 10368: linear DMA staging of dl2
#define CB_RED (8 * 64 * 4)
// dl1 as three bf16 terms, dlb[term][n][k] with k = 24 oy + ox (ox 20..23 padding, masked in
// the MFMA operand): rows of 60 16-byte slots (8 k each), slot G of row n stored at
// 4 (G >> 2) + ((G + ((n >> 1) & 2)) & 3) so that each 16-lane group of a ds_read_b128 in phase
// (c) covers the 64 banks once
#define CB_DLB_LD 480
#define CB_DLB (3 * C1_N * CB_DLB_LD * 2)    // 46080
__device__ inline int dlb_slot(int G, int n) { return 4 * (G >> 2) + ((G + ((n >> 1) & 2)) & 3); }
// Phase (c)'s schedule of the 60 position blocks G = 3 oy + blk (8 positions ox = 8 blk .. +7 of
// output row oy) over its 15 K-chunks x 4 lane groups j4 (round 4).  The x-plane reads are
// ds_read_b32 pairs serviced in lane groups {0-31} (j4 0, 1) and {32-63} (j4 2, 3), bank = dword
// mod 32; a lane's (cin, kernel row) offsets cover 16 banks, and the other j4 of its group covers
// the other 16 only if the two blocks sit 16 dwords apart mod 32: row oy's blocks 0 and 2, or block 1
// of rows 4 apart (the old G = 4 c + j4 paired blocks 8 or 4 dwords apart: every read 2-way
// conflicted).  28 of the 30 pairs are conflict-free (rows 16-19's block 1 pair up with Delta 20):
// the x reads' LDS cycles 480 -> 256 per wave and sample (tools/lds_bank_sim.py).  The dl1 terms
// of block G are stored at slot index cb_fmap(G) = 4 c + j4 of its place in this schedule, so the
// term reads (ds_read_b128, dlb_slot(4 c + j4, n)) keep their conflict-free pattern.
// Measured (profiles/round4_ab_cbsched.txt, 3 interleaved reps): slower -- conv backward alone
// 92.4 vs 90.8 us, M1 4.72M vs 4.74M, M2 5.56M vs 5.63M env-steps/s: the x reads are not what
// bounds phase (c), and the schedule's address math sits in its chain.  Kept behind
// -DCB_BANK_SCHED; the default is the round-3 schedule (cb_block / cb_fmap the identity).
__device__ inline void cb_block(int c, int j4, int& oy, int& blk) {
#ifndef CB_BANK_SCHED   // default: the round-3 schedule G = 4 c + j4 (measured faster, below)
  oy = (4 * c + j4) / 3; blk = 4 * c + j4 - 3 * oy; return;
#endif
  if (c < 10) {
    oy = 2 * c + (j4 >> 1);
    blk = 2 * (j4 & 1);
  } else {
    const int i = c - 10;
    oy = i < 4 ? 8 * (i >> 1) + 2 * (i & 1) + (j4 >> 1) + 4 * (j4 & 1) : 16 + 2 * (j4 >> 1) + (j4 & 1);
    blk = 1;
  }
}
__device__ inline int cb_fmap(int G) {      // the inverse of cb_block: 4 c + j4 of block G
#ifndef CB_BANK_SCHED
  return G;
#endif
  const int oy = G / 3, blk = G - 3 * oy;
  if (blk != 1) return 2 * oy + (blk >> 1);
  if (oy >= 16) return 56 + (oy - 16);
  const int local = oy & 7, rem = local & 3;
  return 4 * (10 + 2 * (oy >> 3) + (rem >> 1)) + 2 * (rem & 1) + ((local >> 2) & 1);
}
// l1s | dl2s | red, overlaid after phase (b) by dlb
constexpr int cb_tail(bool lx) {
  return cb_l1_bytes(lx) + CB_DL2 + CB_RED > CB_DLB ? cb_l1_bytes(lx) + CB_DL2 + CB_RED : CB_DLB;
}
// LDS: x8[2] | l1 stage | dl2 stage | tail
#define CB_SMEM_DMA (2 * CB_X8 + CB_L1ST + CB_DL2ST + cb_tail(true))                   // 144672
// compact variant (no prefetch): x8 | tail -- leaves LDS for co-resident rollout kernels when
// the backward overlaps the next rollout (engine overlap mode)
#define CB_SMEM_COMPACT (CB_X8 + cb_tail(false))                                        // 74304
#define CB_SMEM_COMPACT_LX (CB_X8 + cb_tail(true))                                      // 80480
// LDS the compact kernels reserve: more than half of the CU's 160 KB, so that two of their
// workgroups never share a CU -- such a CU has no room left for a rollout workgroup (79.6 KB),
// and the rollout step then runs a second round of workgroups -- and no more than 160 KB minus
// the rollout kernel's (A3C_CB_SOLO=0: the kernels' own sizes)
#define CB_SMEM_SOLO 82944
static_assert(2 * CB_SMEM_SOLO > 160 * 1024 && CB_SMEM_SOLO >= CB_SMEM_COMPACT_LX, "solo reservation");
static int cb_smem(int own) {
  static const bool solo = A3C_AB_KNOB("A3C_CB_SOLO", 1) != 0;
  return solo ? CB_SMEM_SOLO : own;
}

// the nw waves DMA `nbytes` (multiple of 16) from g to LDS dst in 1 KiB wave-instructions
__device__ inline void glds_copy(const uint8_t* g, uint8_t* dst, int nbytes, int wid, int lane, int nw) {
  for (int c = wid; c * 1024 < nbytes; c += nw) {
    const int off = c * 1024 + lane * 16;
    if (off < nbytes) glds16(g + off, dst + c * 1024);
  }
}

// workgroup barrier that keeps LDS-DMA loads in flight (retires LDS ops only)
__device__ inline void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Debug builds only (-DCB_PHASES, tools/cb_phases.py): wave 0 of every workgroup sums the
// s_memrealtime ticks of each phase over its samples -- staging, (a), (b), dl1 split, (c) -- and
// writes them as u64[6] (last: the whole workgroup) over its own consumed l1 rows.
#ifdef CB_PHASES
#define CB_PH_INIT() uint64_t cb_ph_[6] = {0, 0, 0, 0, 0, 0}; uint64_t cb_t_ = __builtin_amdgcn_s_memrealtime(); const uint64_t cb_t0_ = cb_t_
#define CB_PH(i) do { const uint64_t t_ = __builtin_amdgcn_s_memrealtime(); cb_ph_[i] += t_ - cb_t_; cb_t_ = t_; } while (0)
#define CB_PH_OUT(dst) do { if (threadIdx.x == 0) { cb_ph_[5] = __builtin_amdgcn_s_memrealtime() - cb_t0_; \
    for (int i_ = 0; i_ < 6; ++i_) ((uint64_t*)(dst))[i_] = cb_ph_[i_]; } } while (0)
#else
#define CB_PH_INIT() ((void)0)
#define CB_PH(i) ((void)0)
#define CB_PH_OUT(dst) ((void)0)
#endif

#ifdef CB_PHB_PERM
// Phase (b) (LX) position order within each M-tile: MFMA row m of tile mt is position 16 mt +
// nibble m of cb_phb_perm[mt] (tile 6, which holds positions 96..99 and the clamped duplicates,
// keeps the identity).  Found by a local search over the per-tile permutations for the fewest
// LDS-array cycles of the tile's ds_read_b128 operand reads and its epilogue's ReLU-mask reads
// over the four parity classes (tools/lds_bank_sim.py model): 2064 -> 1648 cycles per sample and
// wave for tiles 0-5.  Any order is valid: A row m and D row m name the same position.
__constant__ uint64_t cb_phb_perm[7] = {0x0c2af753d1b9864eull, 0xfa360b2795e48cd1ull, 0xfbe6c29783da1405ull, 0x3645eb1acd8f9072ull, 0xbe47851a63fc902dull, 0xa64893d57fe102bcull, 0xfedcba9876543210ull};
#endif

template <bool DMA, int NW, bool LX>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(2))) k_conv_bwd(StateAddr sa, int64_t B, int per_wg,
                                                  const float* __restrict__ act_l1,
                                                  const float* __restrict__ dl2,
                                                  const float* __restrict__ W2,
                                                  float* __restrict__ slab) {
  WGLOG(6);
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* x8buf = smem;                                             // [DMA ? 2 : 1][CB_X8]
  uint8_t* l1st = smem + (DMA ? 2 : 1) * CB_X8;
  uint8_t* dl2st = l1st + (DMA ? CB_L1ST : 0);
  float* l1s = (float*)(dl2st + (DMA ? CB_DL2ST : 0));
  // LX: the LDS-lean layout (above).  The 8-wave kernels always take it, the compact 4-wave one
  // that runs beside the rollout by default (a3c_lean_cbwd): with 183 workgroups it lost in mode M1
  // (4.45-4.48M vs 4.56M env-steps/s) and won in M2; with one workgroup per CU on all 256 CUs
  // (CB_SMEM_SOLO) it wins in both (M1 4.64M -> 4.67M)
  constexpr int L1LD = cb_l1_ld(LX);
  float* dl2s = (float*)((uint8_t*)l1s + cb_l1_bytes(LX));
  uint16_t* dlb = (uint16_t*)l1s;                                    // dl1 terms after phase (b)
  float* red = (float*)((uint8_t*)dl2s + CB_DL2);                    // [NW waves][64]
  constexpr int NT = 64 * NW;
  constexpr int T = 16 / NW;          // (kh,kw) tiles of dW2 and K1 tiles of dW1 per wave
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int i16 = lane & 15, j4 = lane >> 4;
  const int64_t tau0 = sa.tau_ptr ? *sa.tau_ptr : 0;
  const int64_t b0 = (int64_t)blockIdx.x * per_wg;
  const int64_t b1 = min(B, b0 + per_wg);
  WG_T0();
  unsigned long long* srec = span_rec(sa, tau0);
  span_begin(srec);

  // parity class of this wave for dl1: (py, px); with 8 waves two waves share a class and
  // split its 7 M-tiles (0-3 / 4-6)
  const int py = (wid & 3) >> 1, px = wid & 1;
  const int mt_lo = NW == 8 ? (wid >> 2) * 4 : 0, mt_hi = NW == 8 ? (wid >> 2 ? 7 : 4) : 7;
  // W2 taps for the class: w2c[(dy*2+dx)*8 + nb*4 + c4] = W2[py+2dy][px+2dx][ci=i16][16nb+4j4+c4]
  const float* w2lane = W2 + ((py * C2_K + px) * C1_N + i16) * C2_N + 4 * j4;
  float w2c[32];
#pragma unroll
  for (int dy = 0; dy < 2; ++dy)
#pragma unroll
    for (int dx = 0; dx < 2; ++dx)
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        const f32x4 w = *(const f32x4*)(w2lane + (2 * dy * C2_K + 2 * dx) * C1_N * C2_N + 16 * nb);
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) w2c[(dy * 2 + dx) * 8 + nb * 4 + c4] = w[c4];
      }

  f32x4 accW2[T][2];
  f32x4 accW1[4];
#pragma unroll
  for (int t = 0; t < T; ++t) accW2[t][0] = accW2[t][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 4; ++t) accW1[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // phase (c) tiles: wave w4 = wid & 3 owns the 4 M-tiles (kh = 4 (w4 >> 1) + (row >> 2),
  // kw = t + 4 (w4 & 1), cin = row & 3), t = 0..3; with 8 waves, waves w4 and w4 + 4 split the
  // K chunks (even / odd)
  const int w4 = wid & 3;
  const int c_first = NW == 8 ? wid >> 2 : 0, c_step = NW == 8 ? 2 : 1;
  const int xoff_c = (i16 & 3) * PLANE + (4 * (w4 >> 1) + (i16 >> 2)) * IMG + 4 * (w4 & 1);
  float db1acc = 0.f, db2acc = 0.f;
  float db2part = 0.f;                 // db2 of co = lane & 31 over rows q = 2 wid + (lane >> 5) (mod 2 NW)

  // Operands of sample b+1 (x planes, l1, dl2: 64 KB) are DMA'd global -> LDS while sample b
  // computes: x8 is double-buffered; l1 / dl2 land in linear staging buffers and are copied into
  // the padded (bank-spread) layouts at the top of the next sample.
  auto issue = [&](int64_t bb, uint8_t* x8dst) {
#pragma unroll
    for (int c = 0; c < HIST; ++c) glds_copy(state_plane(sa, bb, c, tau0), x8dst + c * PLANE, PLANE, wid, lane, NW);
    glds_copy((const uint8_t*)(act_l1 + bb * C1_P * C1_N), l1st, CB_L1ST, wid, lane, NW);
    glds_copy((const uint8_t*)(dl2 + bb * FLAT), dl2st, CB_DL2ST, wid, lane, NW);
  };
  if (DMA && b0 < b1) issue(b0, x8buf);
  CB_PH_INIT();

  for (int64_t b = b0; b < b1; ++b) {
    uint8_t* x8 = x8buf + (DMA ? ((b - b0) & 1) * CB_X8 : 0);
    if constexpr (DMA) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMA for sample b landed
      __syncthreads();                                    // ... and every wave's; sample b-1 done
      for (int i = tid; i < C1_P * 4; i += NT) {          // l1 [400][16] -> stride 20
        const int p = i >> 2, q4 = i & 3;
        *(f32x4*)(l1s + p * L1LD + 4 * q4) = ((const f32x4*)l1st)[i];
      }
      if constexpr (LX) {
        for (int i = tid; i < C2_Q * 4; i += NT) {        // dl2 [81][32] -> stride 36, pairs (co, co+16)
          const int q = i >> 2, j = i & 3;
          const f32x4 lo = ((const f32x4*)dl2st)[q * 8 + j], hi = ((const f32x4*)dl2st)[q * 8 + 4 + j];
          *(f32x4*)(dl2s + q * CB_DL2_LD + 8 * j) = (f32x4){lo[0], hi[0], lo[1], hi[1]};
          *(f32x4*)(dl2s + q * CB_DL2_LD + 8 * j + 4) = (f32x4){lo[2], hi[2], lo[3], hi[3]};
        }
      } else {
        for (int i = tid; i < C2_Q * 8; i += NT) {        // dl2 [81][32] -> stride 36
          const int q = i >> 3, q4 = i & 7;
          *(f32x4*)(dl2s + q * CB_DL2_LD + 4 * q4) = ((const f32x4*)dl2st)[i];
        }
      }
      if (tid < 8) *(f32x4*)(dl2s + C2_Q * CB_DL2_LD + 4 * tid) = (f32x4){0.f, 0.f, 0.f, 0.f};
      __syncthreads();                                    // staging buffers free again
      if (b + 1 < b1) issue(b + 1, x8buf + ((b + 1 - b0) & 1) * CB_X8);
    } else {
      // every load of the sample's l1 and dl2 rows in flight at once, then the LDS stores
      constexpr int NL1 = (C1_P * 4 + NT - 1) / NT, ND2 = (C2_Q * 8 + NT - 1) / NT;
      f32x4 rl1[NL1], rd2[ND2];
      const f32x4* gl1 = (const f32x4*)(act_l1 + b * C1_P * C1_N);
      const f32x4* gd2 = (const f32x4*)(dl2 + b * FLAT);
#pragma unroll
      for (int u = 0; u < NL1; ++u) rl1[u] = gl1[min(tid + NT * u, C1_P * 4 - 1)];
#pragma unroll
      for (int u = 0; u < ND2; ++u) rd2[u] = gd2[min(tid + NT * u, C2_Q * 8 - 1)];
      __syncthreads();                                    // previous sample done with LDS
#pragma unroll
      for (int u = 0; u < NL1; ++u) {
        const int i = tid + NT * u;
        if (i < C1_P * 4) *(f32x4*)(l1s + (i >> 2) * L1LD + 4 * (i & 3)) = rl1[u];
      }
#pragma unroll
      for (int u = 0; u < ND2; ++u) {                     // co 4 (i & 7) .. + 3 of row q -> 4 scattered columns
        const int i = tid + NT * u;
        if (i < C2_Q * 8) {
          if constexpr (LX) {
            float* d = dl2s + (i >> 3) * CB_DL2_LD + dl2_col(4 * (i & 7));
#pragma unroll
            for (int c = 0; c < 4; ++c) d[2 * c] = rd2[u][c];
          } else {
            *(f32x4*)(dl2s + (i >> 3) * CB_DL2_LD + 4 * (i & 7)) = rd2[u];
          }
        }
      }
      if (tid < 8) *(f32x4*)(dl2s + C2_Q * CB_DL2_LD + 4 * tid) = (f32x4){0.f, 0.f, 0.f, 0.f};
      __syncthreads();
      // the state planes are read in (c) only: DMA them global -> LDS now and let the copy run
      // under phases (a) and (b) (their barriers retire LDS ops only)
#pragma unroll
      for (int c = 0; c < HIST; ++c) glds_copy(state_plane(sa, b, c, tau0), x8 + c * PLANE, PLANE, wid, lane, NW);
    }
    CB_PH(0);

    // ---- (a) dW2[(kh,kw,ci)][n] += sum_q l1[2oy+kh][2ox+kw][ci] * dl2[q][n] ----
    for (int s = 0; s < (C2_Q + 3) / 4; ++s) {
      const int q = 4 * s + j4;
      const bool qv = q < C2_Q;
      const int qc = qv ? q : 0;
      const int oy = qc / C2_O, ox = qc - oy * C2_O;
      float bq0, bq1;
      if constexpr (LX) {
        const float2 bq = *(const float2*)(dl2s + qc * CB_DL2_LD + 2 * i16);   // (co, co + 16)
        bq0 = qv ? bq.x : 0.f;
        bq1 = qv ? bq.y : 0.f;
      } else {
        bq0 = qv ? dl2s[qc * CB_DL2_LD + i16] : 0.f;
        bq1 = qv ? dl2s[qc * CB_DL2_LD + 16 + i16] : 0.f;
      }
#pragma unroll
      for (int t = 0; t < T; ++t) {
        const int mt = T * wid + t;
        const int kh = mt >> 2, kw = mt & 3;
        const float av = qv ? l1s[((C2_S * oy + kh) * C1_O + C2_S * ox + kw) * L1LD + i16] : 0.f;
        accW2[t][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bq0, accW2[t][0], 0, 0, 0);
        accW2[t][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bq1, accW2[t][1], 0, 0, 0);
      }
    }

    lds_barrier();   // every wave done reading l1 in (a): (b) overwrites it with dl1
    CB_PH(1);

    // ---- (b) dl1 for parity class (py,px): 100 positions in 7 M-tiles of 16 ----
    constexpr int MTB = NW == 8 ? 4 : 7;
    // per-sample copies of the lane coordinates: keeps the compiler from hoisting every tile's
    // LDS addresses out of the sample loop (they would pin ~80 VGPRs)
    int bj4 = j4, bi16 = i16;
    asm volatile("" : "+v"(bj4), "+v"(bi16));
    // Two forms of (b), bit-identical.  The branch-free one below is faster alone (conv backward
    // 131 -> 122 us compact, 82 -> 77 us DMA) but its denser MFMA issue slows the co-resident
    // rollout more than it saves in overlap mode (4.45M vs 4.57M env-steps/s, tools/ab.sh): the
    // 8-wave sync kernel takes it (3.48M vs 3.45M), the compact overlap kernel keeps the old one.
    if constexpr (LX) {
    // One basic block per sample: the epilogue is branch-free, so the scheduler can run a tile's
    // address math, ReLU-mask reads and next operands under the previous tile's MFMAs.  Rows past
    // position 99 (tile 6) duplicate row 99: their A rows are row 99's (clamped), so their D rows
    // are bit-identical to it, the mask is read before any write of the tile, and all of them
    // store the same value into position 99's slot; only their db1 contribution is dropped.
    // (tile loop rolled: unrolled, the scheduler hoists every tile's addresses and spills)
#pragma unroll 1
    for (int u = 0; u < MTB; ++u) {
      const int mt = mt_lo + u;
      if (mt >= mt_hi) break;
#ifdef CB_PHB_PERM
      const uint64_t pm = cb_phb_perm[mt];
      const int pc = 16 * mt + (int)((pm >> (4 * bi16)) & 15);
#else
      const int pc = 16 * mt + bi16;
#endif
      const int pcc = pc < 100 ? pc : 99;
      const int ay = pcc / 10, cx = pcc - ay * 10;
      const int base = ay * C2_O + cx;
      int eo[4];
      float msk[4];
#ifdef CB_PHB_PERM
      bool rv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {          // D row 4 j4 + r: its position's slot (clamped at 99)
        const int pr = 16 * mt + (int)((pm >> (4 * (4 * bj4 + r))) & 15);
        const int prc = pr < 100 ? pr : 99;
        const int ayr = prc / 10, cxr = prc - ayr * 10;
        eo[r] = ((2 * ayr + py) * C1_O + 2 * cxr + px) * L1LD + bi16;
        rv[r] = pr < 100;
        msk[r] = l1s[eo[r]];                    // l1 (the ReLU mask), before any write of the tile
      }
#else
      // epilogue slots of rows r = 0..3: p = p0 + 2 rr + 20 [cx0 + rr >= 10], rr = min(r, 99 - prc0)
      const int pr0 = 16 * mt + 4 * bj4;
      const int prc0 = pr0 < 100 ? pr0 : 99;
      const int ay0 = prc0 / 10, cx0 = prc0 - ay0 * 10;
      const int p0 = (2 * ay0 + py) * C1_O + 2 * cx0 + px;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = min(r, 99 - prc0);
        eo[r] = (p0 + 2 * rr + (cx0 + rr >= 10 ? 20 : 0)) * L1LD + bi16;
        msk[r] = l1s[eo[r]];                    // l1 (the ReLU mask), before any write of the tile
      }
#endif
      int qo[4];
#pragma unroll
      for (int dy = 0; dy < 2; ++dy)
#pragma unroll
        for (int dx = 0; dx < 2; ++dx) {
          // dl2 position (ay - dy, cx - dx); off the 9x9 grid -> the zero row
          const bool v = (dy ? ay > 0 : ay < C2_O) && (dx ? cx > 0 : cx < C2_O);
          qo[dy * 2 + dx] = (v ? base - C2_O * dy - dx : C2_Q) * CB_DL2_LD + 8 * bj4;
        }
      f32x4 acc = {0.f, 0.f, 0.f, 0.f}, accb = {0.f, 0.f, 0.f, 0.f};   // two chains (nb)
      // operands of a tap: lo = (c4 0, nb 0), (0, 1), (1, 0), (1, 1); hi = the same for c4 2, 3
      f32x4 op[2][2];                          // two taps' operands in flight
      op[0][0] = *(const f32x4*)(dl2s + qo[0]);
      op[0][1] = *(const f32x4*)(dl2s + qo[0] + 4);
#pragma unroll
      for (int tp = 0; tp < 4; ++tp) {
        if (tp + 1 < 4) {
          op[(tp + 1) & 1][0] = *(const f32x4*)(dl2s + qo[tp + 1]);
          op[(tp + 1) & 1][1] = *(const f32x4*)(dl2s + qo[tp + 1] + 4);
        }
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) {
          const f32x4& o = op[tp & 1][c4 >> 1];
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(o[2 * (c4 & 1)], w2c[tp * 8 + c4], acc, 0, 0, 0);
          accb = __builtin_amdgcn_mfma_f32_16x16x4f32(o[2 * (c4 & 1) + 1], w2c[tp * 8 + 4 + c4], accb, 0, 0, 0);
        }
      }
      acc += accb;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float g = msk[r] > 0.f ? acc[r] : 0.f;
        l1s[eo[r]] = g;                          // dl1 in place over l1 (this lane's own slot)
#ifdef CB_PHB_PERM
        db1acc = rv[r] ? db1acc + g : db1acc;
#else
        db1acc = pr0 + r < 100 ? db1acc + g : db1acc;
#endif
      }
    }
    } else {
#pragma unroll
    for (int u = 0; u < MTB; ++u) {
      const int mt = mt_lo + u;
      if (mt >= mt_hi) break;
      const int pc = 16 * mt + bi16;
      const int pcc = pc < 100 ? pc : 99;
      const int ay = pcc / 10, cx = pcc - ay * 10;
      const int base = ay * C2_O + cx;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f}, accb = {0.f, 0.f, 0.f, 0.f};   // two chains (nb)
#pragma unroll
      for (int dy = 0; dy < 2; ++dy)
#pragma unroll
        for (int dx = 0; dx < 2; ++dx) {
          // dl2 position (ay - dy, cx - dx); off the 9x9 grid -> the zero row
          const bool v = (dy ? ay > 0 : ay < C2_O) && (dx ? cx > 0 : cx < C2_O);
          const int qq = v ? base - C2_O * dy - dx : C2_Q;
#pragma unroll
          for (int nb = 0; nb < 2; ++nb) {
            const f32x4 a = *(const f32x4*)(dl2s + qq * CB_DL2_LD + 16 * nb + 4 * bj4);
            f32x4& c = nb ? accb : acc;
#pragma unroll
            for (int c4 = 0; c4 < 4; ++c4)
              c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[c4], w2c[(dy * 2 + dx) * 8 + nb * 4 + c4], c, 0, 0, 0);
          }
        }
      acc += accb;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int pr = 16 * mt + 4 * bj4 + r;
        const int prc = pr < 100 ? pr : 99;
        const int p = (2 * (prc / 10) + py) * C1_O + 2 * (prc % 10) + px;
        if (pr < 100) {                          // dl1 in place over l1 (this lane's own slot)
          const float g = l1s[p * L1LD + bi16] > 0.f ? acc[r] : 0.f;
          l1s[p * L1LD + bi16] = g;
          db1acc += g;
        }
      }
    }
    }

    if constexpr (LX) {   // db2: this lane's channel over its row residue (dl2s intact until the split)
      const int co = lane & 31;
      float s2 = 0.f;
      for (int q = 2 * wid + (lane >> 5); q < C2_Q; q += 2 * NW) s2 += dl2s[q * CB_DL2_LD + dl2_col(co)];
      db2part += s2;
    } else if (tid < C2_N) {   // db2[n] += sum_q dl2[q][n]
      float s2 = 0.f;
      for (int q = 0; q < C2_Q; ++q) s2 += dl2s[q * CB_DL2_LD + tid];
      db2acc += s2;
    }
    lds_barrier();   // dl1 complete in l1s
    CB_PH(2);
    // dl1 -> three bf16 terms in dlb, which overlays l1s / dl2s: all reads first
    if constexpr (!LX) {
      constexpr int PER = (C1_P * C1_N + NT - 1) / NT;
      float v[PER];
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int e = min(tid + NT * i, C1_P * C1_N - 1);
        v[i] = l1s[(e >> 4) * L1LD + (e & 15)];
      }
      lds_barrier();   // (the DMA for b+1 stays in flight)
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int e = tid + NT * i;
        if (e < C1_P * C1_N) {
          // dl1 = hi + mid + lo (round-to-nearest bf16 terms, ~2^-24 relative)
          const int pos = e >> 4, n = e & 15;
          const int oy = pos / C1_O, k = pos + 4 * oy;           // k = 24 oy + ox
          const __bf16 h = (__bf16)v[i];
          const float r1 = v[i] - (float)h;
          const __bf16 m = (__bf16)r1;
          const __bf16 l = (__bf16)(r1 - (float)m);
          __bf16* d = (__bf16*)dlb + n * CB_DLB_LD + 8 * dlb_slot(cb_fmap(k >> 3), n) + (k & 7);
          d[0] = h;
          d[C1_N * CB_DLB_LD] = m;
          d[2 * C1_N * CB_DLB_LD] = l;
        }
      }
    } else
    // (LX) Task u = two
    // adjacent positions (ox even, ox + 1) of channel n = u & 15: one ds_write_b32 per term
    // instead of two ds_write_b16
    {
      constexpr int NTASK = C1_P / 2 * C1_N;                 // 3200
      constexpr int PER = (NTASK + NT - 1) / NT;
      float v[PER][2];
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int u = min(tid + NT * i, NTASK - 1);
        const int pos = 2 * (u >> 4), n = u & 15;
        v[i][0] = l1s[pos * L1LD + n];
        v[i][1] = l1s[(pos + 1) * L1LD + n];
      }
      lds_barrier();   // (the DMA for b+1 stays in flight)
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int u = tid + NT * i;
        if (u < NTASK) {
          const int pos = 2 * (u >> 4), n = u & 15;
          const int oy = pos / C1_O, k = pos + 4 * oy;           // k = 24 oy + ox, even
          // dl1 = hi + mid + lo (round-to-nearest bf16 terms, ~2^-24 relative)
          uint32_t hh[2], mm[2], ll[2];
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const __bf16 h = (__bf16)v[i][q];
            const float r1 = v[i][q] - (float)h;
            const __bf16 m = (__bf16)r1;
            const __bf16 l = (__bf16)(r1 - (float)m);
            hh[q] = __builtin_bit_cast(uint16_t, h);
            mm[q] = __builtin_bit_cast(uint16_t, m);
            ll[q] = __builtin_bit_cast(uint16_t, l);
          }
          uint32_t* d = (uint32_t*)(dlb + n * CB_DLB_LD + 8 * dlb_slot(cb_fmap(k >> 3), n) + (k & 7));
          d[0] = hh[0] | (hh[1] << 16);
          d[C1_N * CB_DLB_LD / 2] = mm[0] | (mm[1] << 16);
          d[C1_N * CB_DLB_LD] = ll[0] | (ll[1] << 16);
        }
      }
    }
    // zero padding k = 24 oy + 20..23 (slot 3 oy + 2, elements 4..7) of every term row
    for (int i = tid; i < 3 * C1_N * C1_O; i += NT) {
      const int row = i / C1_O, oy = i - row * C1_O;
      *(uint2*)(dlb + row * CB_DLB_LD + 8 * dlb_slot(cb_fmap(3 * oy + 2), row & 15) + 4) = make_uint2(0u, 0u);
    }
    if constexpr (!DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's x8 DMA landed
    lds_barrier();   // dl1 terms complete (and every wave's x8 DMA)
    CB_PH(3);

    // ---- (c) dW1[(kh,kw,cin)][n] += sum_p x[cin][4oy+kh][4ox+kw] * dl1[p][n]  (x unscaled) ----
    // v_mfma_f32_16x16x32_bf16: a u8 pixel is exact in bf16, dl1 = three bf16 terms, so every
    // product is exact in the fp32 accumulator.  K = 15 chunks of 32 padded positions: lane group
    // g takes 8 consecutive ox of block (oy, blk) = cb_block(chunk, g) (ox = 8 blk + j).
    // One dword of x holds the pixels of kw & 3 = 0..3 for one ox: 8 dwords feed the 4 tiles.
    // operands of chunk c: 8 x dwords and the 3 dl1-term fragments (next chunk's prefetched
    // while this one's MFMAs run)
    auto load_chunk = [&](int c, uint32_t (&d)[8], bf16x8 (&bv)[3]) {
      int oy, blk;
      cb_block(c, j4, oy, blk);                 // (the bank-spread schedule above)
      const uint32_t* xp = (const uint32_t*)(x8 + xoff_c + 4 * oy * IMG + 32 * blk);
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] = xp[j];
#pragma unroll
      for (int term = 0; term < 3; ++term)
        bv[term] = *(const bf16x8*)(dlb + (term * C1_N + i16) * CB_DLB_LD + 8 * dlb_slot(4 * c + j4, i16));
    };
    auto mma_chunk = [&](const uint32_t (&d)[8], const bf16x8 (&bt)[3]) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        uint32_t a[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const float f0 = (float)((d[2 * jj] >> (8 * t)) & 255u);
          const float f1 = (float)((d[2 * jj + 1] >> (8 * t)) & 255u);
          a[jj] = __builtin_amdgcn_perm(__float_as_uint(f1), __float_as_uint(f0), 0x07060302u);
        }
        const bf16x8 av = __builtin_bit_cast(bf16x8, make_uint4(a[0], a[1], a[2], a[3]));
        accW1[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bt[0], accW1[t], 0, 0, 0);
        accW1[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bt[1], accW1[t], 0, 0, 0);
        accW1[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bt[2], accW1[t], 0, 0, 0);
      }
    };
    // two operand sets in flight: chunk c + step loads while chunk c multiplies
    uint32_t d0[8], d1[8];
    bf16x8 b0[3], b1[3];
    load_chunk(c_first, d0, b0);
#pragma unroll 1
    for (int c = c_first; c < 15; c += 2 * c_step) {
      const bool has1 = c + c_step < 15;
      if (has1) load_chunk(c + c_step, d1, b1);
      mma_chunk(d0, b0);
      if (c + 2 * c_step < 15) load_chunk(c + 2 * c_step, d0, b0);
      if (has1) mma_chunk(d1, b1);
    }
    CB_PH(4);
  }

  // ---- write this workgroup's partial slab ----
  float* out = slab + (int64_t)blockIdx.x * CB_SLAB;
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const int mt = T * wid + t;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int krow = 16 * mt + 4 * j4 + r;     // dW2 row (kh,kw,ci)
      out[CB_OFF_W2 + krow * C2_N + i16] = accW2[t][0][r];
      out[CB_OFF_W2 + krow * C2_N + 16 + i16] = accW2[t][1][r];
    }
  }
  if constexpr (NW == 8) {                       // fold the odd-chunk half of dW1 (waves 4..7)
    __syncthreads();                             // LDS free: every wave past its last phase (c)
    f32x4* part = (f32x4*)smem;
    if (wid >= 4)
#pragma unroll
      for (int t = 0; t < 4; ++t) part[(w4 * 4 + t) * 64 + lane] = accW1[t];
    __syncthreads();
    if (wid < 4)
#pragma unroll
      for (int t = 0; t < 4; ++t) accW1[t] += part[(w4 * 4 + t) * 64 + lane];
  }
  if (wid < 4) {
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        // D row 4 j4 + r of tile t: kh = 4 (w4 >> 1) + j4, kw = t + 4 (w4 & 1), cin = r
        const int krow = ((4 * (w4 >> 1) + j4) * C1_K + t + 4 * (w4 & 1)) * HIST + r;
        out[CB_OFF_W1 + krow * C1_N + i16] = accW1[t][r];
      }
  }
  // db1: lanes with equal i16 (4 j4 groups) then the waves, in a fixed order
  db1acc += __shfl_xor(db1acc, 16, 64);
  db1acc += __shfl_xor(db1acc, 32, 64);
  __syncthreads();
  if (lane < 16) red[wid * 64 + lane] = db1acc;
  __syncthreads();
  if (tid < 16) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += red[w * 64 + tid];
    out[CB_OFF_B1 + tid] = v;
  }
  if constexpr (LX) {   // db2[co] = sum_q dl2[q][co]: the 2 NW row-residue partials in a fixed order
    __syncthreads();
    red[(2 * wid + (lane >> 5)) * 32 + (lane & 31)] = db2part;
    __syncthreads();
    if (tid < C2_N) {
      float v = 0.f;
#pragma unroll
      for (int g = 0; g < 2 * NW; ++g) v += red[g * 32 + tid];
      out[CB_OFF_B2 + tid] = v;
    }
  } else if (tid < C2_N) {
    out[CB_OFF_B2 + tid] = db2acc;
  }
  span_end(srec);
  CB_PH_OUT(act_l1 + b0 * C1_P * C1_N);
  WG_T1(act_l1 + b0 * C1_P * C1_N);   // debug: over this workgroup's own (consumed) l1 rows
}

// ---------------------------------------------------------------------------------------
// deterministic slab reductions into the flat gradient vector
// ---------------------------------------------------------------------------------------
// pass 1 of the conv-slab reduction: dst[g][i] = sum of slabs s in group g (fixed order)
__global__ void __launch_bounds__(256) k_slab_group(const float* __restrict__ src, int nsplit, int per,
                                                    int64_t len, float* __restrict__ dst) {
  WGLOG(8);
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= len) return;
  const int g = blockIdx.y;
  const int s0 = g * per, s1 = min(nsplit, s0 + per);
  dst[(int64_t)g * len + i] = sum_strided(src + (int64_t)s0 * len + i, s1 - s0, len);
}

__device__ void loss_reduce_block(const float* __restrict__ terms, int64_t B, float* __restrict__ out) {
  __shared__ double red[4][256];
  double s[4] = {0, 0, 0, 0};
  for (int64_t b = threadIdx.x; b < B; b += 256)
#pragma unroll
    for (int c = 0; c < 4; ++c) s[c] += (double)terms[b * 4 + c];
#pragma unroll
  for (int c = 0; c < 4; ++c) red[c][threadIdx.x] = s[c];
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o)
#pragma unroll
      for (int c = 0; c < 4; ++c) red[c][threadIdx.x] += red[c][threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x < 4) out[threadIdx.x] = (float)red[threadIdx.x][0];
}

// pass 2 + small segments: blocks [0, FIN_X n) = segment y = b / FIN_X, x = b % FIN_X (grid-stride
// within the segment; with fs.part, the block's fp64 sum of squares of what it wrote goes to
// part[slot + x]); block FIN_X n reduces the per-sample loss terms (and evaluates the schedule);
// the blocks after it sum the other tensors' chunks (fused per-tensor norms, FinalizeSegs)
__global__ void __launch_bounds__(256) k_finalize(FinalizeSegs fs, const float* __restrict__ terms, int64_t B,
                                                  float* __restrict__ loss_out) {
  WGLOG(8);
  const int b = blockIdx.x;
  if (b < FIN_X * fs.n) {
    const int y = b / FIN_X, x = b - y * FIN_X;
    const FinalizeSeg sg = fs.s[y];
    const int64_t n = (int64_t)sg.rows * sg.ncols;
    double ss = 0.0;
    for (int64_t i = (int64_t)x * 256 + threadIdx.x; i < n; i += (int64_t)FIN_X * 256) {
      const int r = (int)(i / sg.ncols), c = (int)(i - (int64_t)r * sg.ncols);
      const float* src = sg.src + (int64_t)r * sg.src_ld + sg.col0 + c;
      const float v = sum_strided(src, sg.nsplit, sg.split_stride) * sg.scale;
      fs.dst[sg.dst_off + (int64_t)r * sg.dst_ld + c] = v;
      ss += (double)v * v;
    }
    if (fs.part && sg.slot >= 0) {
      __shared__ double red[256];
      red[threadIdx.x] = ss;
      __syncthreads();
      for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
      }
      if (threadIdx.x == 0) fs.part[sg.slot + x] = red[0];
    }
    return;
  }
  if (!fs.no_tail && b == FIN_X * fs.n) {
    if (loss_out) loss_reduce_block(terms, B, loss_out);
    if (fs.part && threadIdx.x == 0) opt_schedule(fs.op);
    return;
  }
  const int k = b - FIN_X * fs.n - (fs.no_tail ? 0 : 1);
  int j = 0;
  while (j + 1 < fs.nsum && k >= fs.sum_c0[j + 1]) ++j;
  const int t = fs.sum_t[j], c = k - fs.sum_c0[j];
  sumsq_chunk(fs.dst, fs.tt, t, c, fs.part, fs.tt.pb_first[t] + c);
}

// host launchers shared with the nature trunk's backward (nature.hip)
int a3c_head_bwd_launch(int width, const NetLayout& L, const float* z, const int32_t* actions, const float* target,
                        const float* h, const float* Wp, const float* Wv, float beta, int literal, int64_t B,
                        float* dz, float* dh, float* terms, const ReturnsArgs& ra, int relu, hipStream_t s) {
  const dim3 grid((unsigned)((B + 3) / 4));
  if (width == FC)
    hipLaunchKernelGGL(k_head_bwd<FC>, grid, dim3(256), 0, s, z, L.zs, L.A, L.algo, actions, target, h, Wp, Wv, beta,
                       literal, 1.0f / (float)B, B, dz, dh, terms, ra, relu);
  else if (width == 512)
    hipLaunchKernelGGL(k_head_bwd<512>, grid, dim3(256), 0, s, z, L.zs, L.A, L.algo, actions, target, h, Wp, Wv, beta,
                       literal, 1.0f / (float)B, B, dz, dh, terms, ra, relu);
  else
    return a3c_set_error(A3C_ERR_INVALID, "a3c_head_bwd_launch", "head width");
  A3C_CHECK(hipGetLastError());
  return 0;
}
int a3c_slab_group_launch(const float* src, int nsplit, int groups, int64_t len, float* dst, hipStream_t s) {
  const int per = (nsplit + groups - 1) / groups;
  hipLaunchKernelGGL(k_slab_group, dim3((unsigned)((len + 255) / 256), (unsigned)groups), dim3(256), 0, s, src, nsplit,
                     per, len, dst);
  A3C_CHECK(hipGetLastError());
  return 0;
}
int a3c_finalize_launch(const FinalizeSegs& fs, int nsumblk, const float* terms, int64_t B, float* loss_out,
                        hipStream_t s) {
  hipLaunchKernelGGL(k_finalize, dim3((unsigned)(FIN_X * fs.n + (fs.no_tail ? 0 : 1) + nsumblk)), dim3(256), 0, s, fs,
                     terms, B, loss_out);
  A3C_CHECK(hipGetLastError());
  return 0;
}

// tensors whose gradient a k_finalize segment writes (a3c_backward_launch's seg() calls)
static bool finalize_tensor(const NetLayout& L, int t) {
  return t == T_L1W || t == T_L1B || t == T_L2W || t == T_L2B || t == T_FCB || t == T_HW || t == T_HB ||
         (L.algo == A3C_ALGO_A3C && (t == T_VW || t == T_VB));
}

int a3c_fused_tab(const NetLayout& L, TensorTab* tt) {
  if (L.nt <= 0 || L.nt > A3C_MAX_TENSORS) return -1;
  tt->n = L.nt;
  int nb = 0;
  for (int t = 0; t < L.nt; ++t) {
    tt->off[t] = L.off[t];
    tt->size[t] = L.size[t];
    tt->pb_first[t] = nb;
    tt->pb_count[t] = finalize_tensor(L, t) ? FIN_X : (int)((L.size[t] + SS_CHUNK - 1) / SS_CHUNK);
    nb += tt->pb_count[t];
  }
  if (nb > SS_MAX_BLOCKS) return -1;
  tt->nblocks = nb;
  tt->total = L.total;
  return 0;
}

// ---------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------
// The in-workgroup split-K fc weight GEMM (k_gemm_f32_wks) up to K = B = A3C_FC_WKS_MAXB samples
// (default 2560: M1 +1.1 %, 512 envs 5.38M vs 5.35M).  Its workgroups each walk a quarter of K per
// group, so at B = 5120 (1024 envs) it runs 176 us beside the rollout and the slab form wins
// (5.77M vs 5.64M env-steps/s); with the LSTM head the slab form wins too (3.19M vs 3.16M).
// A3C_FC_WKS=0 turns it off.
static bool fc_wks_on(int64_t B) {
  static const bool on = A3C_AB_KNOB("A3C_FC_WKS", 1) != 0;
  static const int64_t maxb = (int)A3C_AB_KNOB("A3C_FC_WKS_MAXB", 2560);
  return on && B <= maxb;
}

BwdPlan a3c_bwd_plan(const NetLayout& L, int64_t B, bool wks) {
  BwdPlan p;
  int64_t o = 0;
  auto take = [&](int64_t floats) { int64_t r = o; o += (floats + 63) & ~(int64_t)63; return r; };
  // conv-backward workgroups: one per CU when the backward owns the GPU (the 144 KB LDS-DMA
  // kernel fits once per CU); in overlap mode 224 compact (74 KB) workgroups, one per CU on 7/8
  // of the CUs, so that each CU keeps LDS for a concurrent rollout workgroup (conv12's 60 KB u8
  // variant, head_screen's 54 KB).  Measured on MI355X (Pong, 256 envs): 3.70M env-steps/s vs
  // 3.45M with 448 two-per-CU workgroups (those alone are faster, 92 vs 132 us, but leave no LDS
  // for the rollout).  Round 2, with the partial fc: 192 (-> 183 workgroups of 7 samples at
  // n*E = 1280) 4.37M env-steps/s vs 4.29M for 224 (214 x 6), 4.14M for 160 (160 x 8), 4.00M for 256.
  // The slab workspace is sized for the larger count, so the plan's offsets do not depend on the mode.
  static const int env_nwg = (int)A3C_AB_KNOB("A3C_CB_NWG", 0);
  // Round 3, with one compact workgroup per CU guaranteed (CB_SMEM_SOLO): 256 (5 samples each at
  // n*E = 1280) -- M2 5.36M -> 5.77M, M1 4.62M -> 4.66M against 183 x 7 (214 x 6: 5.71M / 4.65M)
  const int nwg_shared = env_nwg ? env_nwg : 256, nwg_own = env_nwg ? env_nwg : 256;
  auto count = [&](int nwg_max, int& per) {
    int nwg = (int)(B < nwg_max ? B : nwg_max);
    if (nwg < 1) nwg = 1;
    per = (int)((B + nwg - 1) / nwg);
    return (int)((B + per - 1) / per);
  };
  int per_alloc = 0;
  const int nwg_alloc = std::max(count(nwg_shared, per_alloc), count(nwg_own, per_alloc));
  p.nwg = count(a3c_shared_gpu() ? nwg_shared : nwg_own, p.per_wg);
  p.head_split = a3c_gemm_effective_split((int)B, a3c_gemm_plan_split(FC, L.zs, (int)B, 128));
  // wks: the fc weight GEMM (K = B) splits K inside its workgroups (k_gemm_f32_wks) -- no slab
  // round trip through HBM, no fold kernel; else split-K slabs + k_reduce_slabs.  The slab and column
  // sum buffers are sized for the slab form either way, so the offsets do not depend on it.
  const int fc_split_slab = a3c_gemm_effective_split((int)B, a3c_gemm_plan_split(FLAT, FC, (int)B, 512));
  p.fc_split = wks ? 1 : fc_split_slab;
  p.dz = take(B * L.zs);
  p.dh3 = take(B * FC);
  p.dl2 = take(B * FLAT);
  p.terms = take(B * 4);
  p.hgrad = take((int64_t)FC * L.zs);
  p.hcol = take((int64_t)p.head_split * L.zs);
  p.hslab = take(p.head_split > 1 ? (int64_t)p.head_split * FC * L.zs : 0);
  p.fccol = take((int64_t)fc_split_slab * FC);
  p.fcslab = take(fc_split_slab > 1 ? (int64_t)fc_split_slab * FLAT * FC : 0);
  p.cslab = take((int64_t)nwg_alloc * CB_SLAB);
  p.groups = p.nwg < 16 ? p.nwg : 16;
  p.cgroup = take((int64_t)16 * CB_SLAB);    // groups <= 16 in either mode
  p.total = o;
  return p;
}

// The split backward (SplitBwd): head and fc weight GEMMs with their folds right behind them, the
// dl2 GEMM, then [finalize of the fc / head segments + their norms + the schedule + the loss, the clip
// of grads[cut:], ev_head], then the conv backward, its slab folds + norms and the clip of
// grads[:cut].  Every fold, partial and clip value is the one-pass path's, so the gradients are
// bit-identical (tests/test_gpu_multirank.py).
static int backward_split(const NetLayout& L, const float* P, const StateAddr& sa, int64_t B, const float* act_l1,
                          float* ws, hipStream_t s, const BwdPlan& p, GemmArgs gh, GemmArgs gf, GemmArgs gd,
                          float* grads, const float* terms, float* loss_out, const SumsqFused* sf, const SplitBwd* sp) {
  const bool a3c = L.algo == A3C_ALGO_A3C;
  // the head weight GEMM's split-K partials are folded by the finalize segments (the same
  // sum_strided order as k_reduce_slabs: bit-identical, one kernel fewer)
  const float* hsrc = p.head_split > 1 ? ws + p.hslab : ws + p.hgrad;
  const int64_t hstride = (int64_t)FC * L.zs;
  gh.defer_reduce = 1;        // (the finalize folds the head slabs itself: hsrc below)
  gf.defer_reduce = 0;
  gh.big = gf.big = gd.big = 0;
  int rc = a3c_gemm(false, true, gh, s);
  if (!rc) rc = a3c_gemm(false, true, gf, s);
  if (!rc) rc = a3c_gemm(true, false, gd, s);
  if (rc) return rc;
  auto segs = [&](FinalizeSegs& fs) {
    fs.dst = grads;
    fs.part = sf->part;
    fs.tt = *sf->tt;
    fs.op = *sf->op;
    fs.sum_c0[0] = 0;
  };
  auto seg = [&](FinalizeSegs& fs, const float* src, int64_t stride, int nsplit, int rows, int src_ld, int col0,
                 int ncols, int tensor, int dst_ld, float scale) {
    FinalizeSeg& q = fs.s[fs.n++];
    q.src = src; q.split_stride = stride; q.nsplit = nsplit; q.rows = rows; q.src_ld = src_ld;
    q.col0 = col0; q.ncols = ncols; q.dst_off = L.off[tensor]; q.dst_ld = dst_ld; q.scale = scale;
    q.slot = sf->tt->pb_first[tensor];
  };
  // (1) fc / head tensors: segments, chunk sums of the tensors the GEMMs / BPTT wrote whole, the
  // loss and the schedule
  {
    FinalizeSegs fs = {};
    segs(fs);
    seg(fs, ws + p.fccol, FC, p.fc_split, 1, 0, 0, FC, T_FCB, 0, 1.0f);
    seg(fs, hsrc, hstride, p.head_split, FC, L.zs, 0, L.A, T_HW, L.A, 1.0f);
    seg(fs, ws + p.hcol, L.zs, p.head_split, 1, 0, 0, L.A, T_HB, 0, 1.0f);
    if (a3c) {
      seg(fs, hsrc, hstride, p.head_split, FC, L.zs, L.A, 1, T_VW, 1, 1.0f);
      seg(fs, ws + p.hcol, L.zs, p.head_split, 1, 0, L.A, 1, T_VB, 0, 1.0f);
    }
    for (int t = 0; t < L.nt; ++t) {
      if (finalize_tensor(L, t)) continue;
      if (L.off[t] < sp->cut || fs.nsum == 4)
        return a3c_set_error(A3C_ERR_INVALID, "a3c_loss_backward", "split backward: tensor layout");
      fs.sum_t[fs.nsum] = t;
      fs.sum_c0[fs.nsum + 1] = fs.sum_c0[fs.nsum] + fs.tt.pb_count[t];
      ++fs.nsum;
    }
    hipLaunchKernelGGL(k_finalize, dim3((unsigned)(FIN_X * fs.n + 1 + fs.sum_c0[fs.nsum])), dim3(256), 0, s, fs,
                       terms, B, loss_out);
    A3C_CHECK(hipGetLastError());
    OptParams op = sp->clip;
    op.q0 = sp->cut >> 2;
    op.q1 = L.total >> 2;
    rc = a3c_apply_launch(nullptr, nullptr, nullptr, grads, *sf->tt, op, sf->part, nullptr, s);
    if (rc) return rc;
    A3C_CHECK(hipEventRecord(sp->ev_head, s));
  }
  // (2) conv tensors
  rc = a3c_conv_bwd_launch(L, P, sa, B, act_l1, ws + p.dl2, ws, s);
  if (rc) return rc;
  const int per = (p.nwg + p.groups - 1) / p.groups;
  hipLaunchKernelGGL(k_slab_group, dim3((CB_SLAB + 255) / 256, p.groups), dim3(256), 0, s, ws + p.cslab, p.nwg, per,
                     (int64_t)CB_SLAB, ws + p.cgroup);
  A3C_CHECK(hipGetLastError());
  {
    FinalizeSegs fs = {};
    segs(fs);
    fs.no_tail = 1;
    const float* cs = ws + p.cgroup;
    seg(fs, cs + CB_OFF_W1, CB_SLAB, p.groups, 1, 0, 0, KC1 * C1_N, T_L1W, 0, 1.0f / 255.0f);
    seg(fs, cs + CB_OFF_B1, CB_SLAB, p.groups, 1, 0, 0, C1_N, T_L1B, 0, 1.0f);
    seg(fs, cs + CB_OFF_W2, CB_SLAB, p.groups, 1, 0, 0, KC2 * C2_N, T_L2W, 0, 1.0f);
    seg(fs, cs + CB_OFF_B2, CB_SLAB, p.groups, 1, 0, 0, C2_N, T_L2B, 0, 1.0f);
    hipLaunchKernelGGL(k_finalize, dim3((unsigned)(FIN_X * fs.n)), dim3(256), 0, s, fs, terms, B, loss_out);
    A3C_CHECK(hipGetLastError());
    OptParams op = sp->clip;
    op.q0 = 0;
    op.q1 = sp->cut >> 2;
    return a3c_apply_launch(nullptr, nullptr, nullptr, grads, *sf->tt, op, sf->part, sp->sumsq_out, s);
  }
}

static bool xcd_gemm();   // (below, beside the other mode knobs)
static bool dwfc_late_knob();
static bool bwd_bound_knob();
int a3c_backward_launch(const NetLayout& L, const float* params, const StateAddr& sa, int64_t B,
                        const float* act_l1, const float* act_l2, const float* act_l3,
                        const float* z, const int32_t* actions, const float* target, float beta,
                        int literal, float* grads, float* loss_out, float* ws, hipStream_t s,
                        const ReturnsArgs* ra_in, hipStream_t side, hipEvent_t ev_fork, hipEvent_t ev_join,
                        const LstmBwd* lb, const SumsqFused* sf, const SplitBwd* sp, const uint32_t* l2m) {
  ReturnsArgs ra = {};
  if (ra_in) ra = *ra_in;
  if (B <= 0) return a3c_set_error(A3C_ERR_INVALID, "a3c_loss_backward", "B must be > 0");
  // sync mode: the three GEMMs in one launch (3.32M -> 3.41M env-steps/s), and so where the
  // overlapped backward bounds the iteration (M2: 5.17-5.22M -> 5.38-5.39M); beside a rollout
  // that bounds it the 1,420-workgroup launch slows it more than it gains (M1: 4.62M -> 4.45M),
  // and so do the folds moved behind the conv backward alone (A3C_FOLD_LATE: 4.62M -> 4.45M)
  static const int env_multi = (int)A3C_AB_KNOB("A3C_GEMM_MULTI", -1);
  const bool multi0 = env_multi >= 0 ? env_multi != 0 : !a3c_shared_gpu() || bwd_bound_knob();
  // the in-workgroup split-K fc weight GEMM where its launch stands alone anyway (the M1 overlap
  // backward), not in the single three-GEMM launch.  The split backward (SplitBwd) takes the form
  // the one-phase backward of the same configuration takes (multi0 does not depend on sp), so the
  // two exchanges sum the fc weight gradient in one order and stay bit-identical
  // (test_gpu_multirank.py::test_split_exchange_equals_one_phase)
  const bool wks = fc_wks_on(B) && !L.lstm && !multi0;
  const BwdPlan p = a3c_bwd_plan(L, B, wks);
  const float* P = params;
  float* dz = ws + p.dz;
  float* dh3 = ws + p.dh3;
  float* dl2 = ws + p.dl2;
  float* terms = ws + p.terms;
  const bool a3c = L.algo == A3C_ALGO_A3C;

  if (L.lstm != (lb != nullptr) || (lb && !ra.terms))
    return a3c_set_error(A3C_ERR_INVALID, "a3c_loss_backward", "the LSTM head needs its rollout sequence");
  // head input: the fc ReLU output, or the LSTM's h (C5)
  const float* head_in = lb ? lb->h : act_l3;
  hipLaunchKernelGGL(k_head_bwd<FC>, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, s, z, L.zs, L.A, L.algo,
                     actions, target, head_in, P + L.off[T_HW], a3c ? P + L.off[T_VW] : nullptr, beta,
                     literal, 1.0f / (float)B, B, dz, lb ? lb->dh : dh3, terms, ra, lb ? 0 : 1);
  A3C_CHECK(hipGetLastError());
  if (lb) {
    // truncated BPTT: dL/dh_t -> dl3 (masked by the fc ReLU) + the gate-matrix gradients
    LstmSeq q = {act_l3, lb->hp, lb->cp, lb->gates, lb->c, ra.terms};
    int rc0 = a3c_lstm_bptt_launch(P + L.off[T_LW], lb->n, lb->E, q, lb->dh, dh3, grads + L.off[T_LW],
                                   grads + L.off[T_LB], lb->ws, s);
    if (rc0) return rc0;
  }

  // The weight-gradient GEMMs (head, fc) only need dz / dl3 from k_head_bwd: with a side stream
  // they run concurrently with the dl2 GEMM + conv backward (graph branches), joined before the
  // slab reductions.
  const bool fork = side && ev_fork && ev_join && !lb;
  hipStream_t ws_s = fork ? side : s;
  if (fork) {
    A3C_CHECK(hipEventRecord(ev_fork, s));
    A3C_CHECK(hipStreamWaitEvent(side, ev_fork, 0));
  }
  // head weights: dWh[256][zs] = l3^T dz ; dbh = colsum(dz)
  GemmArgs gh = {};
  gh.A = head_in; gh.lda = FC;       // A(m=feature, k=b) = l3[b][m]  (m contiguous)
  gh.B = dz; gh.ldb = L.zs;          // B(k=b, n=j) = dz[b][j]
  gh.C = ws + p.hgrad; gh.ldc = L.zs;
  gh.M = FC; gh.N = L.zs; gh.K = (int)B;
  gh.epi = EPI_STORE; gh.slab = ws + p.hslab; gh.nsplit = p.head_split; gh.colsum = ws + p.hcol;
  gh.defer_reduce = 1;                 // its split-K fold is the finalize's (segments over the slab)
  // fc weights: dW[2592][256] = l2^T dl3 -> grads directly ; db = colsum(dl3)
  GemmArgs gf = {};
  gf.A = act_l2; gf.lda = FLAT;
  gf.B = dh3; gf.ldb = FC;
  gf.C = grads + L.off[T_FCW]; gf.ldc = FC;
  gf.M = FLAT; gf.N = FC; gf.K = (int)B;
  gf.epi = EPI_STORE; gf.slab = ws + p.fcslab; gf.nsplit = p.fc_split; gf.colsum = ws + p.fccol;
  gf.wg_split = wks ? 4 : 0;
  gf.xcd = xcd_gemm() ? 1 : 0;          // the 4 column tiles of an l2 strip on one XCD
  // The in-workgroup split-K form in XCD-grouped order (its 4 N tiles share the 64-row strip of l2,
  // fetched once per XCD instead of once per N tile): HBM bytes per launch 58.5 -> 26.6 MB (PMC,
  // profiles/round5_ab/gemm_knobs.txt; the 8-XCD floor is 26.5: l2 13.3 + dl3 1.3 per XCD + dW
  // 2.65), M1 unchanged (4.884M vs 4.886M, 3 interleaved reps).  A3C_WKS_XCD=0 (A/B builds): plain grid
  if (wks) {
    static const int env_wx = (int)A3C_AB_KNOB("A3C_WKS_XCD", 1);
    gf.xcd = env_wx ? 1 : 0;
  }
  // dl2[B][2592] = (dl3 W^T) * (l2 > 0)
  GemmArgs gd = {};
  gd.A = dh3; gd.lda = FC;               // A(m=b, k) = dl3[b][k]
  gd.B = P + L.off[T_FCW]; gd.ldb = FC;  // B(k, n) = W[n][k]
  gd.C = dl2; gd.ldc = FLAT;
  gd.M = (int)B; gd.N = FLAT; gd.K = FC;
  gd.epi = EPI_MASK; gd.mask = act_l2; gd.ldm = FLAT; gd.nsplit = 1;
  if (l2m) {   // the forward's ReLU bits (engine): 415 KB instead of re-reading l2's 13.3 MB (E=256)
    gd.epi = EPI_MASKBITS; gd.maskbits = l2m; gd.mask = nullptr; gd.ldm = FLAT / 32;
  }
  gd.xcd = xcd_gemm() ? 2 : 0;          // the 20 row tiles of a W strip on one XCD
  {
    // overlap, A3C_GEMM_BIG=1: 128x128 tiles (210 workgroups instead of 820 beside the rollout;
    // bit-identical).  Off: +0.5 % on one box (4.79-4.81M -> 4.82-4.83M), -0.8 % on another
    // (4.80-4.83M -> 4.75-4.79M) -- the tile GEMM takes 62 us instead of ~35 and the caller
    // stream's loop (go -> backward -> apply -> hop) then bounds M1 again (tools/wglog.py)
    static const int env_big = (int)A3C_AB_KNOB("A3C_GEMM_BIG", 0);
    gd.big = a3c_shared_gpu() && env_big != 0;
    static const int env_bigf = (int)A3C_AB_KNOB("A3C_GEMM_BIG_FC", 0);
    gf.big = a3c_shared_gpu() && env_bigf != 0;
  }
  {
    static const int env_wgs = (int)A3C_AB_KNOB("A3C_GEMM_WGS", 0);
    if (a3c_shared_gpu()) gh.max_wgs = gf.max_wgs = gd.max_wgs = env_wgs;
  }
  int rc;
  if (sp) {
    if (!sf || fork) return a3c_set_error(A3C_ERR_INVALID, "a3c_loss_backward", "split backward: fused norms, no fork");
    return backward_split(L, P, sa, B, act_l1, ws, s, p, gh, gf, gd, grads, terms, loss_out, sf, sp);
  }
  static const int env_late = (int)A3C_AB_KNOB("A3C_FOLD_LATE", -1);
  // The head weight GEMM folds its own split-K slabs (k_reduce_slabs behind it) instead of the
  // finalize with the LSTM head (C5 3.19M vs 3.18M env-steps/s), not without it (M1 4.81M vs
  // 4.87M); A3C_HEAD_FOLD=0/1 overrides.  Separate-launch path below only.
  static const int env_hfold_knob = (int)A3C_AB_KNOB("A3C_HEAD_FOLD", -1);
  const bool env_hfold = env_hfold_knob >= 0 ? env_hfold_knob != 0 : lb != nullptr;
  bool hfold = false;
  const bool multi = multi0 && !wks;
  const bool late = env_late >= 0 ? env_late != 0 : multi;
  if (!fork && (multi || late)) {
    // the weight-gradient split-K folds go after the conv backward (only the clip / apply read
    // them), so nothing but dl2 stands between the head and the conv
    if (multi) {
      rc = a3c_gemm3(gh, gf, gd, s);
    } else {
      gh.defer_reduce = gf.defer_reduce = 1;
      rc = a3c_gemm(false, true, gh, s);
      if (!rc) rc = a3c_gemm(false, true, gf, s);
      if (!rc) rc = a3c_gemm(true, false, gd, s);
    }
    if (rc) return rc;
    rc = a3c_conv_bwd_launch(L, P, sa, B, act_l1, dl2, ws, s);
    if (rc) return rc;
    rc = a3c_gemm_reduce(gf, s);       // (gh: folded by the finalize)
    if (rc) return rc;
  } else {
#ifdef A3C_MARKERS
    static const bool abl_gemm = getenv("A3C_ABL_GEMM") != nullptr;   // measurement only: no fc/head GEMMs
#else
    constexpr bool abl_gemm = false;
#endif
    // dwfc_late: the fc weight GEMM (+ its fold) behind the conv backward -- only dl2 stands
    // between the head and the conv
    const bool dwfc_late = dwfc_late_knob() && !fork;
    hfold = env_hfold && p.head_split > 1;
    if (hfold) gh.defer_reduce = 0;
    rc = abl_gemm ? 0 : a3c_gemm(false, true, gh, ws_s);
    if (rc) return rc;
    if (!dwfc_late) {
      rc = abl_gemm ? 0 : a3c_gemm(false, true, gf, ws_s);
      if (rc) return rc;
    }
    if (fork) A3C_CHECK(hipEventRecord(ev_join, side));
    rc = abl_gemm ? 0 : a3c_gemm(true, false, gd, s);
    if (rc) return rc;
#ifdef A3C_MARKERS
    a3c_mark(4, s);
#endif
    rc = a3c_conv_bwd_launch(L, P, sa, B, act_l1, dl2, ws, s);
    if (rc) return rc;
#ifdef A3C_MARKERS
    a3c_mark(5, s);
#endif
    if (dwfc_late) {
      rc = abl_gemm ? 0 : a3c_gemm(false, true, gf, s);
      if (rc) return rc;
    }
  }

  FinalizeSegs fs = {};
  fs.dst = grads;
  auto seg = [&](const float* src, int64_t stride, int nsplit, int rows, int src_ld, int col0,
                 int ncols, int tensor, int dst_ld, float scale) {
    FinalizeSeg& q = fs.s[fs.n++];
    q.src = src; q.split_stride = stride; q.nsplit = nsplit; q.rows = rows; q.src_ld = src_ld;
    q.col0 = col0; q.ncols = ncols; q.dst_off = L.off[tensor]; q.dst_ld = dst_ld; q.scale = scale;
    q.slot = sf ? sf->tt->pb_first[tensor] : -1;
  };
  if (fork) A3C_CHECK(hipStreamWaitEvent(s, ev_join, 0));
  // conv slabs: nwg partials -> p.groups partials (pass 1), folded by k_finalize (pass 2)
  const int per = (p.nwg + p.groups - 1) / p.groups;
  hipLaunchKernelGGL(k_slab_group, dim3((CB_SLAB + 255) / 256, p.groups), dim3(256), 0, s, ws + p.cslab, p.nwg, per,
                     (int64_t)CB_SLAB, ws + p.cgroup);
  A3C_CHECK(hipGetLastError());
  const float* cs = ws + p.cgroup;
  seg(cs + CB_OFF_W1, CB_SLAB, p.groups, 1, 0, 0, KC1 * C1_N, T_L1W, 0, 1.0f / 255.0f);
  seg(cs + CB_OFF_B1, CB_SLAB, p.groups, 1, 0, 0, C1_N, T_L1B, 0, 1.0f);
  seg(cs + CB_OFF_W2, CB_SLAB, p.groups, 1, 0, 0, KC2 * C2_N, T_L2W, 0, 1.0f);
  seg(cs + CB_OFF_B2, CB_SLAB, p.groups, 1, 0, 0, C2_N, T_L2B, 0, 1.0f);
  seg(ws + p.fccol, FC, p.fc_split, 1, 0, 0, FC, T_FCB, 0, 1.0f);
  // the head weight GEMM's split-K partials folded here (gh.defer_reduce): one kernel fewer
  const float* hsrc = p.head_split > 1 && !hfold ? ws + p.hslab : ws + p.hgrad;
  const int64_t hstride = (int64_t)FC * L.zs;
  const int hsplit = hfold ? 1 : p.head_split;
  seg(hsrc, hstride, hsplit, FC, L.zs, 0, L.A, T_HW, L.A, 1.0f);
  seg(ws + p.hcol, L.zs, p.head_split, 1, 0, 0, L.A, T_HB, 0, 1.0f);
  if (a3c) {
    seg(hsrc, hstride, hsplit, FC, L.zs, L.A, 1, T_VW, 1, 1.0f);
    seg(ws + p.hcol, L.zs, p.head_split, 1, 0, L.A, 1, T_VB, 0, 1.0f);
  }
  int nsumblk = 0;
  if (sf) {   // every other tensor is final by now (fc weights: reduced above; LSTM: BPTT)
    fs.part = sf->part;
    fs.tt = *sf->tt;
    fs.op = *sf->op;
    fs.sum_c0[0] = 0;
    for (int t = 0; t < L.nt; ++t) {
      if (finalize_tensor(L, t)) continue;
      if (fs.nsum == 4) return a3c_set_error(A3C_ERR_INVALID, "a3c_loss_backward", "fused norms: too many tensors");
      fs.sum_t[fs.nsum] = t;
      fs.sum_c0[fs.nsum + 1] = fs.sum_c0[fs.nsum] + fs.tt.pb_count[t];
      ++fs.nsum;
    }
    nsumblk = fs.sum_c0[fs.nsum];
  }
  hipLaunchKernelGGL(k_finalize, dim3((unsigned)(FIN_X * fs.n + 1 + nsumblk)), dim3(256), 0, s, fs, terms, B,
                     loss_out);
  A3C_CHECK(hipGetLastError());
  return 0;
}

// Kernel variant choice: a3c_shared_gpu() is true while the engine enqueues work that will run
// concurrently with another stream (overlap mode) -- then the kernels take their smaller-footprint
// variants so both streams' workgroups co-reside on the CUs.  Thread-local switch set by the engine
// around its enqueue calls (captured into the graphs).
static thread_local bool t_shared_gpu = false;
bool a3c_shared_gpu() { return t_shared_gpu; }
void a3c_set_shared_gpu(bool v) { t_shared_gpu = v; }
// set by the engine where the backward stream, not the rollout, bounds the overlapped iteration
// (mode M2, several GPUs): there the three weight/input GEMMs run as one launch with their folds
// behind the conv backward (as in sync mode); A3C_CB_LEAN, A3C_GEMM_MULTI, A3C_GEMM_XCD and
// A3C_DWFC_LATE (0/1) override the choices
static thread_local bool t_bwd_bound = false;
static int env_knob(const char* name) { return (int)A3C_AB_KNOB(name, -1); }   // (A/B builds only)
bool a3c_lean_cbwd() {   // (every overlap mode since the 256-workgroup plan: M1 4.63M -> 4.66M)
  static const int env = env_knob("A3C_CB_LEAN");
  return env >= 0 ? env != 0 : true;
}
static bool xcd_gemm() {
  static const int env = env_knob("A3C_GEMM_XCD");
  return env >= 0 ? env != 0 : t_bwd_bound;
}
// the fc weight GEMM behind the conv backward (M2: 5.15-5.18M -> 5.20-5.22M; M1 neutral)
static bool dwfc_late_knob() {
  static const int env = env_knob("A3C_DWFC_LATE");
  return env >= 0 ? env != 0 : t_bwd_bound;
}
static bool bwd_bound_knob() { return t_bwd_bound; }
void a3c_set_bwd_bound(bool v) { t_bwd_bound = v; }

int a3c_conv_bwd_launch(const NetLayout& L, const float* P, const StateAddr& sa, int64_t B, const float* act_l1,
                        const float* dl2, float* ws, hipStream_t s) {
  const BwdPlan p = a3c_bwd_plan(L, B);
#ifdef A3C_MARKERS
  static const bool ablate = getenv("A3C_ABL_CBWD") != nullptr;   // measurement only: no conv backward
  if (ablate) return 0;
#endif
  // sync: the DMA-prefetching kernel at 8 waves (2 per SIMD) owns the GPU; overlap: the compact
  // 4-wave kernel leaves registers and LDS for the concurrent rollout (measured, tools/ab.sh)
  static const int env_nw = (int)A3C_AB_KNOB("A3C_CB_WAVES", 0);
  const int nw = env_nw ? env_nw : (a3c_shared_gpu() ? 4 : 8);
  if (a3c_shared_gpu() && nw == 4 && a3c_lean_cbwd())
    hipLaunchKernelGGL((k_conv_bwd<false, 4, true>), dim3((unsigned)p.nwg), dim3(256), cb_smem(CB_SMEM_COMPACT_LX), s, sa, B,
                       p.per_wg, act_l1, dl2, P + L.off[T_L2W], ws + p.cslab);
  else if (a3c_shared_gpu() && nw == 4)
    hipLaunchKernelGGL((k_conv_bwd<false, 4, false>), dim3((unsigned)p.nwg), dim3(256), cb_smem(CB_SMEM_COMPACT), s, sa, B,
                       p.per_wg, act_l1, dl2, P + L.off[T_L2W], ws + p.cslab);
  else if (a3c_shared_gpu())
    hipLaunchKernelGGL((k_conv_bwd<false, 8, true>), dim3((unsigned)p.nwg), dim3(512), cb_smem(CB_SMEM_COMPACT_LX), s, sa, B,
                       p.per_wg, act_l1, dl2, P + L.off[T_L2W], ws + p.cslab);
  else if (nw == 4)
    hipLaunchKernelGGL((k_conv_bwd<true, 4, false>), dim3((unsigned)p.nwg), dim3(256), CB_SMEM_DMA, s, sa, B, p.per_wg,
                       act_l1, dl2, P + L.off[T_L2W], ws + p.cslab);
  else
    hipLaunchKernelGGL((k_conv_bwd<true, 8, true>), dim3((unsigned)p.nwg), dim3(512), CB_SMEM_DMA, s, sa, B, p.per_wg,
                       act_l1, dl2, P + L.off[T_L2W], ws + p.cslab);
  A3C_CHECK(hipGetLastError());
  return 0;
}

int a3c_returns_launch(const float* rewards, const uint8_t* terms, const float* boot, int64_t boot_stride,
                       int n, int64_t E, double gamma, float* R, hipStream_t s) {
  if (E <= 0) return 0;
  hipLaunchKernelGGL(k_returns, dim3((unsigned)((E + 255) / 256)), dim3(256), 0, s, rewards, terms, boot,
                     boot_stride, n, E, gamma, R);
  A3C_CHECK(hipGetLastError());
  return 0;
}

int a3c_td_target_launch(const float* rewards, const uint8_t* terms, const float* qn, int64_t B, int A,
                         int zs, double discount, float* target, hipStream_t s, const float* qsel) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL(k_td_target, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, s, rewards, terms, qn,
                     B, A, zs, discount, target, qsel);
  A3C_CHECK(hipGetLastError());
  return 0;
}

void a3c_conv_bwd_set_smem() {
  const int a = hipFuncAttributeMaxDynamicSharedMemorySize;
  (void)hipFuncSetAttribute((const void*)k_conv_bwd<true, 4, false>, (hipFuncAttribute)a, CB_SMEM_DMA);
  (void)hipFuncSetAttribute((const void*)k_conv_bwd<true, 8, true>, (hipFuncAttribute)a, CB_SMEM_DMA);
  (void)hipFuncSetAttribute((const void*)k_conv_bwd<false, 4, false>, (hipFuncAttribute)a, cb_smem(CB_SMEM_COMPACT));
  (void)hipFuncSetAttribute((const void*)k_conv_bwd<false, 4, true>, (hipFuncAttribute)a, cb_smem(CB_SMEM_COMPACT_LX));
  (void)hipFuncSetAttribute((const void*)k_conv_bwd<false, 8, true>, (hipFuncAttribute)a, cb_smem(CB_SMEM_COMPACT_LX));
}

#ifdef A3C_WGLOG
WGLOG_BIND(a3c_wglog_bind_bwd)
#endif

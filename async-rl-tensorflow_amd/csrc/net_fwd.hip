#include <cstdlib>
// Forward of the NIPS trunk + heads on gfx950 matrix cores.
//
//  k_conv12_fwd : one workgroup per state.  The 4 u8 frame planes (28 KB) are staged in LDS;
//                 conv1 (8x8/4, 4->16, ops.py:22-28 VALID NHWC, weights [kh,kw,cin,cout]) runs as
//                 an implicit GEMM on v_mfma_f32_16x16x4_f32 (M = 400 positions in 25 tiles,
//                 N = 16, K = 256) with the whole W1 in 64 VGPRs per lane and the A operand
//                 converted u8 -> f32 in registers (the /255 of agent.py:226 is applied to the
//                 accumulator).  conv1 + relu goes to LDS (and HBM when the backward needs it);
//                 conv2 (4x4/2, 16->32, K = 256) reads it back as 16-byte fragments, W2 in
//                 registers, and writes the (h,w,c)-flattened l2 (agent.py:231-232).
//  fc layer     : gemm.hip (M = B, N = 256, K = 2592, split-K, bias+relu epilogue).
//  k_head_fwd   : one wave per state: logits/value (network.py:62,475) or q (agent.py:252),
//                 then the action draw (softmax sample / epsilon-greedy argmax).
#include "net.h"
#include "lstm.h"
#include "gemm.h"
#include "net_bwd.h"
#include "env_dev.h"
#include "screen_atari.h"
#include "net_head.h"

#define XB_BYTES (HIST * PLANE * 2)                  // 56448: state planes as bf16
#ifdef C2_FP32
#define L1S_BYTES (C1_P * L1S_LD * 4)                // 32000: conv1 out fp32, rows of 20 floats
#else
#define L1T_LD 56                                    // bf16 per position: 3 terms x 16 ch + pad
#define L1S_BYTES (C1_P * L1T_LD * 2)                // 44800: conv1 out as three bf16 terms
#endif
#define CONV12_SMEM (XB_BYTES + L1S_BYTES)           // 101248
#define CONV12_SMEM_U8 (HIST * PLANE + L1S_BYTES)    // 73024: u8 planes, converted per operand

// ---------------------------------------------------------------------------------------
// conv1 weights as three bf16 terms.  A u8 pixel is exact in bf16, so conv1 runs on the bf16
// matrix cores (16x16x32, 16x the fp32 MFMA rate) as x * (w_hi + w_mid + w_lo): the three
// round-to-nearest bf16 terms carry w to ~2^-24 relative and every product is exact in the
// fp32 accumulator -- fp32 accuracy for 3 MFMAs instead of 8 fp32 ones per 32-deep K step.
// The K = 256 reduction runs cin-major, so that the three older planes of a state can be
// reduced before its newest plane exists (the fused rollout kernel hides that part under the
// new frame's HBM load): K-step (cin c, half h2) covers kh = 4 h2 + 0..3, kw = 0..7.
// Fragment-ordered buffer w1s[f][lane][j] (bf16), f = (2 c + h2) * 3 + term: lane l = (j4 = l>>4,
// cout i = l&15) holds B[k = 8 j4 + j][i] = W1[kh = 4 h2 + j4][kw = j][cin = c][cout = i]
// (ops.py:21 layout).
// ---------------------------------------------------------------------------------------
// Forward weight preparation, once per parameter version (rollout start): the conv1 bf16
// terms above and the fc weights in MFMA fragment order, Wp[ct][c][lane][c4] =
// W[16c + 4(lane>>4) + c4][16ct + (lane&15)], so a lane's B operands for 4 MFMAs are one 16-byte load.
// conv2 weights as three bf16 terms in fragment order (w2f, at PREP_W2F_OFF):
// w2f[nt][ks][term][lane][j], lane = (j4 = lane>>4, i16 = lane&15), holds B[k][n] of K-step ks
// (taps kk = 2 ks + (j4>>1), cin = 8 (j4&1) + j) for cout n = 16 nt + i16.
__device__ inline void split3_bits(float w, uint32_t& h, uint32_t& m, uint32_t& l) {
#pragma clang fp contract(off)
  h = bf16_rn_bits(w);
  const float r1 = w - __uint_as_float(h << 16);
  m = bf16_rn_bits(r1);
  const float r2 = r1 - __uint_as_float(m << 16);
  l = bf16_rn_bits(r2);
}

__global__ void __launch_bounds__(256) k_prep_fwd(const float* __restrict__ W1, const float* __restrict__ Wfc,
                                                  const float* __restrict__ W2, uint8_t* __restrict__ prep,
                                                  const int64_t* __restrict__ tau_src, int64_t* __restrict__ tau_dst,
                                                  uint32_t* sig) {
#pragma clang fp contract(off)
  WGLOG(10);
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t == 0 && tau_dst) *tau_dst = *tau_src;
  // the engine's "previous rollout complete" sequence (it precedes this kernel on the stream), in
  // place of a stream write-value operation: one system-scope atomic, no extra kernel
  if (t == 0 && sig) (void)__hip_atomic_fetch_add(sig, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (t < C1_K * 64 * 8) {                                   // (kh, lane, j): conv1 split
    uint16_t* w1s = (uint16_t*)prep;
    const int ks = t >> 9, lane = (t >> 3) & 63, j = t & 7;     // ks = 2 cin + h2
    const int c = ks >> 1, kh = 4 * (ks & 1) + (lane >> 4), i = lane & 15;
    const float w = W1[((kh * C1_K + j) * HIST + c) * C1_N + i];
    uint32_t h, m, l;
    split3_bits(w, h, m, l);
    w1s[((ks * 3 + 0) * 64 + lane) * 8 + j] = (uint16_t)h;
    w1s[((ks * 3 + 1) * 64 + lane) * 8 + j] = (uint16_t)m;
    w1s[((ks * 3 + 2) * 64 + lane) * 8 + j] = (uint16_t)l;
    return;
  }
  const int q = t - C1_K * 64 * 8;                          // (ct, c, lane): one f32x4 of the fc pack
  if (q >= (FC / 16) * FC_CH * 64) {
    const int r = q - (FC / 16) * FC_CH * 64;               // (nt, ks, lane, j): conv2 split
    if (r >= W2F_ELEMS) return;
    const int nt = r >> 12, ks = (r >> 9) & 7, lane = (r >> 3) & 63, j = r & 7;
    const int j4 = lane >> 4, kk = 2 * ks + (j4 >> 1), ci = 8 * (j4 & 1) + j;
    uint32_t h, m, l;
    split3_bits(W2[(kk * C1_N + ci) * C2_N + 16 * nt + (lane & 15)], h, m, l);
    uint16_t* w2f = (uint16_t*)(prep + PREP_W2F_OFF) + ((nt * 8 + ks) * 3) * 512 + lane * 8 + j;
    w2f[0] = (uint16_t)h;
    w2f[512] = (uint16_t)m;
    w2f[1024] = (uint16_t)l;
    return;
  }
#ifndef FC_K32
  const int lane = q & 63, c = (q >> 6) % FC_CH, ct = (q >> 6) / FC_CH;
  const int j4 = lane >> 4, n = 16 * ct + (lane & 15);
  f32x4 v;
#pragma unroll
  for (int c4 = 0; c4 < 4; ++c4) v[c4] = Wfc[(int64_t)(16 * c + 4 * j4 + c4) * FC + n];
#else
  // 32-deep chunks: Wp[ct][c][lane][8] = W[32c + 8(lane>>4) + 0..7][16ct + (lane&15)], q = one f32x4
  const int half = q & 1, lane = (q >> 1) & 63, c = (q >> 7) % FC_CH32, ct = (q >> 7) / FC_CH32;
  const int j4 = lane >> 4, n = 16 * ct + (lane & 15);
  f32x4 v;
#pragma unroll
  for (int c4 = 0; c4 < 4; ++c4) v[c4] = Wfc[(int64_t)(32 * c + 8 * j4 + 4 * half + c4) * FC + n];
#endif
  ((f32x4*)(prep + PREP_W1S_BYTES))[q] = v;
}

int a3c_prep_fwd_launch(const NetLayout& L, const float* P, uint8_t* prep, hipStream_t s, const int64_t* tau_src,
                        int64_t* tau_dst, uint32_t* sig) {
  const int total = C1_K * 64 * 8 + (FC / 16) * FC_CH * 64 + W2F_ELEMS;
  hipLaunchKernelGGL(k_prep_fwd, dim3((total + 255) / 256), dim3(256), 0, s, P + L.off[T_L1W], P + L.off[T_FCW],
                     P + L.off[T_L2W], prep, tau_src, tau_src ? tau_dst : nullptr, sig);
  A3C_CHECK(hipGetLastError());
  return 0;
}

// 8 waves per state.  The 4 u8 planes are staged into LDS as bf16 (exact); conv1 = 25 M-tiles
// of 16 positions x K = 256 (8 steps of (kh; cin x kw 0..7)) on v_mfma_f32_16x16x32_bf16 with the
// three weight terms; conv1 + relu to LDS (and HBM when the backward needs it); conv2 (4x4/2,
// 16->32, K = 256) in fp32 MFMA from LDS, 12 (M-tile, N-tile) pairs over the 8 waves.
// 8 u8 pixels (two dwords, little-endian) -> 8 bf16 (integers 0..255 are exact in bf16: the
// upper half of the f32)
__device__ inline bf16x8 u8x8_to_bf16(uint32_t d0, uint32_t d1) {
  uint32_t o[4];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t d = h ? d1 : d0;
    const float f0 = (float)(d & 255u), f1 = (float)((d >> 8) & 255u);
    const float f2 = (float)((d >> 16) & 255u), f3 = (float)(d >> 24);
    o[2 * h] = __builtin_amdgcn_perm(__float_as_uint(f1), __float_as_uint(f0), 0x07060302u);
    o[2 * h + 1] = __builtin_amdgcn_perm(__float_as_uint(f3), __float_as_uint(f2), 0x07060302u);
  }
  return __builtin_bit_cast(bf16x8, make_uint4(o[0], o[1], o[2], o[3]));
}

// workgroup barrier that retires LDS operations only (vector-memory loads stay in flight)
__device__ inline void lds_only_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// conv1 of the state whose HIST planes are staged in LDS (x8 u8 when U8, else xb bf16) on the
// bf16 matrix cores: wave w owns the M-tiles m = w + 8 i (25 tiles of 16 positions), acc[i]
// accumulates the K-steps of input planes [CB, CE) in the fixed order (cin, h2, term), so a
// reduction split over two calls equals one call over all planes bit for bit.  wfrag(f) returns
// the lane's fragment f = (2 cin + h2) * 3 + term of the bf16-split weights (w1s layout).
#define C1_TILES 4
__device__ inline int conv1_ntiles(int wid) { return wid == 0 ? 4 : 3; }   // 25 = 4 + 7 * 3
template <bool U8, int CB, int CE, bool PIPE = true, typename WF>
__device__ inline void conv1_accum(const uint8_t* x8, const uint16_t* xb, f32x4 (&acc)[C1_TILES], WF wfrag) {
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int i16 = lane & 15, j4 = lane >> 4;
  const int nt = conv1_ntiles(wid);
  int off[C1_TILES];
#pragma unroll
  for (int i = 0; i < C1_TILES; ++i) {
    const int p = min(16 * (wid + 8 * i) + i16, C1_P - 1);
    const int oy = p / C1_O, ox = p - oy * C1_O;
    off[i] = (C1_S * oy + j4) * IMG + C1_S * ox;       // row 4 oy + 4 h2 + j4, columns 4 ox + 0..7
  }
  // one K-step's operands (3 weight fragments, the tiles' pixels) are all read before any is
  // used, and (PIPE) the next step's are read before this step's MFMAs, at +28 VGPRs
  constexpr int NS = (CE - CB) * 2;
  auto read_step = [&](int st, bf16x8 (&w)[3], uint32_t (&q)[C1_TILES][4]) {
    const int c = CB + (st >> 1), h2 = st & 1;
#pragma unroll
    for (int t = 0; t < 3; ++t) w[t] = wfrag((2 * c + h2) * 3 + t);
#pragma unroll
    for (int i = 0; i < C1_TILES; ++i) {
      if (i >= nt) break;
      const int o = c * PLANE + off[i] + 4 * h2 * IMG;
      if constexpr (U8) {
        const uint32_t* p = (const uint32_t*)(x8 + o);            // 4-byte aligned
        q[i][0] = p[0];
        q[i][1] = p[1];
      } else {
        const uint2* p = (const uint2*)(xb + o);                   // 8-byte aligned
        const uint2 lo = p[0], hi = p[1];
        q[i][0] = lo.x; q[i][1] = lo.y; q[i][2] = hi.x; q[i][3] = hi.y;
      }
    }
  };
  bf16x8 w[3];
  uint32_t q[C1_TILES][4];
  read_step(0, w, q);
#pragma unroll
  for (int st = 0; st < NS; ++st) {
    bf16x8 a[C1_TILES];
#pragma unroll
    for (int i = 0; i < C1_TILES; ++i) {
      if (i >= nt) break;
      if constexpr (U8) a[i] = u8x8_to_bf16(q[i][0], q[i][1]);
      else a[i] = __builtin_bit_cast(bf16x8, make_uint4(q[i][0], q[i][1], q[i][2], q[i][3]));
    }
    const bf16x8 w0 = w[0], w1 = w[1], w2 = w[2];
    if (PIPE && st + 1 < NS) read_step(st + 1, w, q);
#pragma unroll
    for (int i = 0; i < C1_TILES; ++i) {
      if (i >= nt) break;
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], w0, acc[i], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < C1_TILES; ++i) {
      if (i >= nt) break;
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], w1, acc[i], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < C1_TILES; ++i) {
      if (i >= nt) break;
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], w2, acc[i], 0, 0, 0);
    }
    if (!PIPE && st + 1 < NS) read_step(st + 1, w, q);
  }
}

// conv1 bias + relu of the accumulated tiles -> l1s as three bf16 terms (and act_l1), then conv2
// (bf16x6 MFMA) + relu -> act_l2 for state b.
// L2M: the epilogue can write the ReLU bits (when l2m is set); false compiles the ballot out --
// the fused rollout kernel runs measurably faster without it where the bits are not used
template <bool SAVE_L1, bool EW, bool L2M = true>
__device__ inline void conv12_finish(f32x4 (&acc)[C1_TILES], float* l1s, int64_t b,
                                     const uint16_t* __restrict__ w1s, const float* __restrict__ b1,
                                     const float* __restrict__ W2, float* __restrict__ act_l1,
                                     float* __restrict__ act_l2, float (&w2r)[64], float bias2,
                                     uint64_t* dbg, uint32_t* __restrict__ l2m = nullptr) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int i16 = lane & 15, j4 = lane >> 4;
  const int nt = wid & 1, grp = wid >> 1;          // conv2: M-tiles grp and grp + 4 (when < 6)
  const float bias1 = b1[i16];
  const int n1 = conv1_ntiles(__builtin_amdgcn_readfirstlane(wid));
#pragma unroll
  for (int i = 0; i < C1_TILES; ++i) {
    if (i >= n1) break;
    const int m = wid + 8 * i;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int pos = 16 * m + 4 * j4 + r;
      float v = fmaxf(acc[i][r] * (1.0f / 255.0f) + bias1, 0.f);
#ifdef C2_FP32
      l1s[pos * L1S_LD + i16] = v;
#else
      // l1 = h + m + l, three round-to-nearest bf16 terms (exact: 24 significant bits)
      uint32_t th, tm, tl;
      split3_bits(v, th, tm, tl);
      uint16_t* d = (uint16_t*)l1s + pos * L1T_LD + i16;
      d[0] = (uint16_t)th;
      d[16] = (uint16_t)tm;
      d[32] = (uint16_t)tl;
#endif
      if (SAVE_L1) st_act(act_l1 + (b * C1_P + pos) * C1_N + i16, v);
    }
  }

#ifdef C2_FP32
  if (!EW) {
#pragma unroll
    for (int kk = 0; kk < 16; ++kk)
#pragma unroll
      for (int c4 = 0; c4 < 4; ++c4) w2r[kk * 4 + c4] = W2[(kk * C1_N + 4 * j4 + c4) * C2_N + 16 * nt + i16];
  }
#else
  // conv2 B fragments: K-step 0's three terms now, each next step's under the current MFMAs
  const uint4* w2f = (const uint4*)((const uint8_t*)w1s + PREP_W2F_OFF) + nt * (8 * 3 * 64) + lane;
  uint4 bq[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) bq[t] = w2f[t * 64];
#endif
  if (dbg && threadIdx.x == 0) dbg[12] = __builtin_readcyclecounter();
  __syncthreads();
  if (dbg && threadIdx.x == 0) dbg[13] = __builtin_readcyclecounter();

  // ---- conv2: 6 M-tiles (81 rows padded to 96) x 2 N-tiles, K = 16 (kh,kw) x 16 cin ----
  const int nm = grp + 4 < 6 ? 2 : 1;
  int pos0[2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
    int q = 16 * (grp + 4 * mi) + i16;
    q = q < C2_Q ? q : C2_Q - 1;
    int oy = q / C2_O, ox = q - oy * C2_O;
    pos0[mi] = (C2_S * oy) * C1_O + C2_S * ox;
  }
  f32x4 acc2[2], acc2b[2];                         // two chains per tile
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) acc2[mi] = acc2b[mi] = (f32x4){0.f, 0.f, 0.f, 0.f};
#ifndef C2_FP32
  // bf16x6: l1 = a0+a1+a2 and W2 = b0+b1+b2 (bf16 terms); the six products with i + j <= 2 carry
  // each fp32 product to ~2^-24 relative (the dropped a1b2 + a2b1 + a2b2 are below 2^-24), every
  // product exact in the fp32 accumulator.  K-step ks = taps 2ks, 2ks+1 x 16 cin: 6 MFMAs of
  // 16x16x32 bf16 (96 cycles) for what took 8 fp32 16x16x4 ones (256 cycles).
  const uint16_t* l1t = (const uint16_t*)l1s;
#pragma unroll 2
  for (int ks = 0; ks < 8; ++ks) {
    uint4 bn[3];
    if (ks < 7) {
#pragma unroll
      for (int t = 0; t < 3; ++t) bn[t] = w2f[((ks + 1) * 3 + t) * 64];
    }
    const int kk = 2 * ks + (j4 >> 1), kh = kk >> 2, kw = kk & 3;
    const bf16x8 b0 = __builtin_bit_cast(bf16x8, bq[0]), bm = __builtin_bit_cast(bf16x8, bq[1]),
                 bl = __builtin_bit_cast(bf16x8, bq[2]);
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      if (mi >= nm) break;
      const uint16_t* ap = l1t + (pos0[mi] + kh * C1_O + kw) * L1T_LD + 8 * (j4 & 1);
      const bf16x8 a0 = *(const bf16x8*)ap, a1 = *(const bf16x8*)(ap + 16), a2 = *(const bf16x8*)(ap + 32);
      acc2[mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b0, acc2[mi], 0, 0, 0);
      acc2b[mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bm, acc2b[mi], 0, 0, 0);
      acc2[mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b0, acc2[mi], 0, 0, 0);
      acc2b[mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bl, acc2b[mi], 0, 0, 0);
      acc2[mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bm, acc2[mi], 0, 0, 0);
      acc2b[mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2, b0, acc2b[mi], 0, 0, 0);
    }
    if (ks < 7) {
#pragma unroll
      for (int t = 0; t < 3; ++t) bq[t] = bn[t];
    }
  }
#else
#pragma unroll
  for (int kh = 0; kh < C2_K; ++kh)
#pragma unroll
    for (int kw = 0; kw < C2_K; ++kw)
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) {
        if (mi >= nm) break;
        f32x4 a = *(const f32x4*)(l1s + (pos0[mi] + kh * C1_O + kw) * L1S_LD + 4 * j4);
        f32x4& c = (kw & 1) ? acc2b[mi] : acc2[mi];   // (alternating by c4 instead: measured no change)
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4)
          c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[c4], w2r[(kh * 4 + kw) * 4 + c4], c, 0, 0, 0);
      }
#endif
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) acc2[mi] += acc2b[mi];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
    if (mi >= nm) break;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = 16 * (grp + 4 * mi) + 4 * j4 + r;
      const float v = fmaxf(acc2[mi][r] + bias2, 0.f);
      if (q < C2_Q) st_act(act_l2 + b * FLAT + q * C2_N + 16 * nt + i16, v);
      if (L2M && l2m) {
        // the ReLU mask as bits for the backward's dl2 epilogue: position q's channels 16 nt ..
        // 16 nt + 15 are the 16 lanes of group j4, so one ballot gives its half word (flat index
        // q * 32 + c: word q of the row, bit c)
        const uint64_t bal = __ballot(v > 0.f);
        if (i16 == 0 && q < C2_Q)
          ((uint16_t*)l2m)[(b * C2_Q + q) * 2 + nt] = (uint16_t)(bal >> (16 * j4));
      }
    }
  }
}

// conv1 + conv2 of state b (planes staged by the caller, not yet synchronised).  The conv1 weight
// fragments (24 KB) are staged in the l1 region, which conv1's epilogue overwrites afterwards.
static_assert(W1S_ELEMS * 2 <= L1S_BYTES, "conv1 weights staged in the l1 region");
template <bool SAVE_L1, bool EW, bool U8>
__device__ inline void conv12_core(const uint8_t* x8, const uint16_t* xb, float* l1s, int64_t b,
                                   const uint16_t* __restrict__ w1s, const float* __restrict__ b1,
                                   const float* __restrict__ W2, float* __restrict__ act_l1,
                                   float* __restrict__ act_l2, float (&w2r)[64], float bias2,
                                   uint64_t* dbg = nullptr, uint32_t* __restrict__ l2m = nullptr) {
  const int lane = threadIdx.x & 63;
  uint4* wl = (uint4*)l1s;
  for (int i = threadIdx.x; i < W1S_ELEMS / 8; i += blockDim.x) wl[i] = ((const uint4*)w1s)[i];
  __syncthreads();
  if (dbg && threadIdx.x == 0) dbg[11] = __builtin_readcyclecounter();
  f32x4 acc[C1_TILES];
#pragma unroll
  for (int i = 0; i < C1_TILES; ++i) acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  conv1_accum<U8, 0, HIST>(x8, xb, acc, [&](int f) { return __builtin_bit_cast(bf16x8, wl[f * 64 + lane]); });
  lds_only_barrier();                                  // weights read: the l1 region is conv1's output
  conv12_finish<SAVE_L1, EW>(acc, l1s, b, w1s, b1, W2, act_l1, act_l2, w2r, bias2, dbg, l2m);
}


// U8: the planes stay u8 in LDS (28 KB instead of 56 KB) and each conv1 A operand is converted
// to bf16 in registers (8 pixels: 2 ds_read_b32 + 8 v_cvt_f32_ubyte + 4 v_perm) -- a 60 KB
// footprint, so a workgroup co-resides on a CU with the concurrent backward's (overlap mode).
template <bool SAVE_L1, bool EW, bool U8>
__global__ void __launch_bounds__(512) k_conv12_fwd(StateAddr sa, int64_t B,
                                                    const uint16_t* __restrict__ w1s,
                                                    const float* __restrict__ b1,
                                                    const float* __restrict__ W2,
                                                    const float* __restrict__ b2,
                                                    float* __restrict__ act_l1,
                                                    float* __restrict__ act_l2,
                                                    uint32_t* __restrict__ l2m) {
  WGLOG(3);
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint16_t* xb = (uint16_t*)smem;
  uint8_t* x8 = smem;
  float* l1s = (float*)(smem + (U8 ? HIST * PLANE : XB_BYTES));
  const int64_t b = blockIdx.x;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int i16 = lane & 15, j4 = lane >> 4;
  const int64_t tau0 = sa.tau_ptr ? *sa.tau_ptr : 0;
  WG_T0();

  // stage: u8 planes -> bf16 planes (integers 0..255 are exact in bf16).  EW: all of a thread's
  // loads issued before the first conversion; otherwise a load-convert loop (fewer live VGPRs)
  constexpr int NCH = HIST * (PLANE / 16);             // 1764 chunks of 16 pixels
  constexpr int PER = (NCH + 511) / 512;               // 4
  auto stage_chunk = [&](int i, const uint4 v) {
    if constexpr (U8) {                                // planes are contiguous: chunk i at 16 i
      ((uint4*)x8)[i] = v;
      return;
    }
    const int c = i / (PLANE / 16), j = i - c * (PLANE / 16);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t o[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float f0 = (float)(w[q] & 255u), f1 = (float)((w[q] >> 8) & 255u);
      const float f2 = (float)((w[q] >> 16) & 255u), f3 = (float)(w[q] >> 24);
      o[2 * q] = __builtin_amdgcn_perm(__float_as_uint(f1), __float_as_uint(f0), 0x07060302u);
      o[2 * q + 1] = __builtin_amdgcn_perm(__float_as_uint(f3), __float_as_uint(f2), 0x07060302u);
    }
    uint4* dst = (uint4*)(xb + c * PLANE + 16 * j);
    dst[0] = make_uint4(o[0], o[1], o[2], o[3]);
    dst[1] = make_uint4(o[4], o[5], o[6], o[7]);
  };
  auto chunk_src = [&](int i) -> uint4 {
    const int c = i / (PLANE / 16), j = i - c * (PLANE / 16);
    return ((const uint4*)state_plane(sa, b, c, tau0))[j];
  };
  uint4 sv[PER];
  if (EW) {
#pragma unroll
    for (int k = 0; k < PER; ++k) sv[k] = chunk_src(min((int)threadIdx.x + 512 * k, NCH - 1));
  } else {
    for (int i = threadIdx.x; i < NCH; i += 512) stage_chunk(i, chunk_src(i));
  }
  // conv2 weights for this wave's N tile (W2[kh][kw][4*j4 + c4][16*nt + i16]).  EW: issued here,
  // their latency hidden behind the staging and conv1 (+64 VGPRs live across conv1); otherwise
  // loaded after conv1 (the small-footprint variant for overlap mode)
  const int nt = wid & 1, grp = wid >> 1;          // M-tiles grp and grp + 4 (when < 6)
  float w2r[64];
#ifdef C2_FP32
  if (EW) {
#pragma unroll
    for (int kk = 0; kk < 16; ++kk)
#pragma unroll
      for (int c4 = 0; c4 < 4; ++c4) w2r[kk * 4 + c4] = W2[(kk * C1_N + 4 * j4 + c4) * C2_N + 16 * nt + i16];
  }
#endif
  const float bias2 = b2[16 * nt + i16];
  if (EW) {
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int i = threadIdx.x + 512 * k;
      if (i < NCH) stage_chunk(i, sv[k]);
    }
  }

  conv12_core<SAVE_L1, EW, U8>(x8, xb, l1s, b, w1s, b1, W2, act_l1, act_l2, w2r, bias2, nullptr, l2m);
  WG_T1(act_l2 + b * FLAT);
}

// head: one wave per state.  z[b][j] = h3[b] . W[:,j] + bias[j]
__global__ void __launch_bounds__(256) k_head_fwd(const float* __restrict__ h3, int64_t B,
                                                  const float* __restrict__ Wp, const float* __restrict__ bp,
                                                  const float* __restrict__ Wv, const float* __restrict__ bv,
                                                  int A, int zs, float* __restrict__ z, HeadSelect sel) {
  WGLOG(4);
  __shared__ __attribute__((aligned(16))) f32x4 l3s[4][64];
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  float myz;
  if (sel.fc_part) {
    // the fc as K-slice partials (k_fc_part): fold in slice order, + bias, ReLU, as the rollout
    // kernel's head does, then the head reads the row from LDS
    f32x4 fp[FC_NS];
#pragma unroll
    for (int w = 0; w < FC_NS; ++w) fp[w] = *(const f32x4*)(sel.fc_part + ((int64_t)w * B + b) * FC + 4 * lane);
    const f32x4 fb = *(const f32x4*)(sel.fc_bias + 4 * lane);
    f32x4 v = fp[0];
#pragma unroll
    for (int w = 1; w < FC_NS; ++w) v += fp[w];
#pragma unroll
    for (int c4 = 0; c4 < 4; ++c4) v[c4] = fmaxf(v[c4] + fb[c4], 0.f);
    l3s[threadIdx.x >> 6][lane] = v;
    if (sel.l3_out) *(f32x4*)(sel.l3_out + b * FC + 4 * lane) = v;
    myz = head_row((const float*)l3s[threadIdx.x >> 6], 0, Wp, bp, Wv, bv, A, lane);
  } else {
    myz = head_row(h3, b, Wp, bp, Wv, bv, A, lane);
  }
  if (lane < zs) z[b * zs + lane] = myz;   // padding columns are 0
  if (sel.mode >= 0) (void)head_act(myz, lane, A, sel, b);
  if (sel.adv_ptr && blockIdx.x == 0 && threadIdx.x == 0) *sel.adv_ptr += sel.adv_n;   // (reads no tau)
}

// engine rollout step tail, one workgroup per env: head + action draw (wave 0) while wave 1
// runs the env act up to the frame (env_act_pre: nothing but the frame depends on the action);
// returns the post-act frame (pool index) of env b
// (W: the width of the layer below the heads -- FC, or NT_FC for the nature trunk)
template <int W = FC>
__device__ inline int32_t head_act_env(const float* __restrict__ h3, const float* __restrict__ Wp,
                                       const float* __restrict__ bp, const float* __restrict__ Wv,
                                       const float* __restrict__ bv, int A, int zs, float* __restrict__ z,
                                       const HeadSelect& sel, int64_t b, int64_t tau, uint64_t* dbg,
                                       const float* hrow = nullptr) {
  __shared__ int32_t s_act;
  __shared__ uint32_t s_draw, s_term;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int e = (int)b;
  const int64_t nxt = ((tau + 1) & 1) * (int64_t)sel.par_E + e;
  if (wid == 0) {
    const float eps = sel_eps(sel, e, tau);
    u32x4 x;
    // the action draw does not depend on the head: computed under its load latency
    // (hrow: the layer-output row, already folded into LDS by the caller)
    float myz;
    if constexpr (W == FC) {
      myz = hrow ? head_row(hrow, 0, Wp, bp, Wv, bv, A, lane, [&]() { x = action_draw(sel, b, tau); })
                 : head_row(h3, b, Wp, bp, Wv, bv, A, lane, [&]() { x = action_draw(sel, b, tau); });
    } else {
      auto mid = [&]() { x = action_draw(sel, b, tau); };
      myz = hrow ? head_row<decltype(mid), W>(hrow, 0, Wp, bp, Wv, bv, A, lane, mid)
                 : head_row<decltype(mid), W>(h3, b, Wp, bp, Wv, bv, A, lane, mid);
    }
    if (dbg) {
      if (lane == 0) dbg[1] = __builtin_readcyclecounter() + (uint64_t)(myz * 0.f);
    } else if (lane < zs) {
      z[b * zs + lane] = myz;
    }
    const int32_t a = select_with(myz, lane, A, sel.mode, x, eps);
    if (lane == 0) {
      sel.actions[b] = a;
      s_act = a;
      if (dbg) dbg[2] = __builtin_readcyclecounter() + (uint64_t)a * 0;
    }
  } else if (wid == 1 && lane == 0 && sel.env_on) {
    const int64_t cur = (tau & 1) * (int64_t)sel.par_E + e;
    const uint32_t id = (uint32_t)(sel.env_id_base + e);
    EnvState s = env_load(sel.envb, cur);
    const uint32_t draw = env_act_pre(s, sel.envp, id, true);
    sel.rewards[e] = fmaxf(-1.0f, fminf(1.0f, s.reward));   // observe clip, agent.py:154
    if (sel.rewards_raw) sel.rewards_raw[e] = s.reward;
    sel.terms[e] = (uint8_t)s.terminal;
    s_draw = draw;
    s_term = s.terminal;
    if (s.terminal) {
      env_new_random_game(s, sel.envp, id);                  // agent.py:66-67
      env_store(sel.envb, nxt, s);
    } else {
      env_store(sel.envb, nxt, s, false);                    // frame: after the action draw
    }
    if (dbg) dbg[17] = __builtin_readcyclecounter();
  }
  __syncthreads();
  int32_t frame;
  if (sel.env_on) {
    frame = env_frame_of(s_draw + sel.frame_salt, (uint32_t)s_act, sel.envp);
#ifdef A3C_ABL_FRAME
    frame = e & 63;   // measurement only: every step reads from 64 L2-resident frames
#endif
    if (threadIdx.x == 0) {
      sel.frames_out[e] = frame;
      if (!s_term) sel.envb.frame[nxt] = frame;
    }
  } else {
    frame = sel.frames_out[b];                               // last frame (no env act)
  }
  if (dbg && threadIdx.x == 0) dbg[3] = __builtin_readcyclecounter();
  return frame;
}

// head + action draw + env act (head_act_env), then the whole workgroup computes
// Environment.screen (environment.py:49-53, bit-exact) of the post-act frame straight from the
// HBM pool into the env's frame-ring slot
template <int HS_THREADS, int W = FC>
__global__ void __launch_bounds__(HS_THREADS) k_head_screen(const float* __restrict__ h3,
                                                            const float* __restrict__ Wp,
                                                            const float* __restrict__ bp,
                                                            const float* __restrict__ Wv,
                                                            const float* __restrict__ bv, int A, int zs,
                                                            float* __restrict__ z, HeadSelect sel) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int64_t b = blockIdx.x;
  const int64_t tau = *sel.tau_ptr + sel.tau_add;
  WG_T0();
  uint64_t* dbg = nullptr;
#ifdef HS_TIMES
  dbg = blockIdx.x == HS_TIMES ? (uint64_t*)z : nullptr;
  if (dbg && threadIdx.x == 0) dbg[0] = __builtin_readcyclecounter();
#endif
  const int32_t frame = head_act_env<W>(h3, Wp, bp, Wv, bv, A, zs, z, sel, b, tau, dbg);
  uint8_t* slot = sel.ring + b * sel.R * PLANE + ((tau + 1) % sel.R) * PLANE;
  if (sel.frame84)
    atari::copy_frame84<HS_THREADS>(sel.pool + (int64_t)frame * PLANE, slot);
  else
    atari::screen_frame<HS_THREADS>(sel.pool + (int64_t)frame * (atari::IH * atari::IW * 3), slot, smem, dbg);
  WG_T1(z + b * zs);
}

// Rollout step t's tail fused with step t+1's head: head + act + Environment.screen of env b
// (as k_head_screen), then conv1 + conv2 of env b's next state s_{t+1} in the same workgroup --
// the next state is the 3 newest ring planes (prefetched into registers at kernel start, they
// are final) plus the screen just computed (kept in LDS).  One kernel boundary and the conv
// staging latency fewer per rollout step.  LDS: screen scratch (gray | tmpT, 51 KB, later
// overlaid by l1) | x8 (18 KB: the older planes' conv1 weight fragments, then the new plane as
// bf16 (14 KB) -- and in -DSCREEN_VALU builds the vertical-tap table behind it).
// A CU must hold one of it beside one compact conv backward workgroup (CB_SMEM_SOLO, 81 KB): the
// round-5 MFMA screen's first layout (78.8 KB, a 28 KB x8 region sized for u8 planes it no longer
// holds) left them no co-residency -- the conv backward then ran alone (90 us live) after the
// rollout, 4.10M vs 4.87M env-steps/s.  Hence the margin in the assert below.
#define HSC_X8_OFF (((SCREEN_FRAME_SMEM_NOKV) + 15) / 16 * 16)
#define HSC_X8_BYTES ((HIST - 1) * 2 * 3 * 64 * 16)              // 18432: the weight fragments
#define HSC_SMEM (HSC_X8_OFF + HSC_X8_BYTES)
#define HSC_KV_OFF (PLANE * 2)
static_assert(L1S_BYTES <= SCREEN_FRAME_SMEM_NOKV, "l1 overlays the screen scratch");
static_assert(HSC_KV_OFF % 16 == 0 && HSC_KV_OFF + SCREEN_KV_BYTES <= HSC_X8_BYTES, "tap table in the x8 region");
static_assert(HSC_SMEM + 16 + 4096 <= 160 * 1024 - 82944, "rollout workgroup beside a compact conv backward one");
// waves_per_eu(4) caps it at 128 VGPRs: with the concurrent k_conv_bwd<false,4> (254 VGPRs,
// one wave per SIMD) two of its waves per SIMD must fit in the remaining 258
template <bool SAVE_L1, bool L2M>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) k_head_screen_conv12(const float* __restrict__ h3,
                                                            const float* __restrict__ Wp,
                                                            const float* __restrict__ bp,
                                                            const float* __restrict__ Wv,
                                                            const float* __restrict__ bv, int A, int zs,
                                                            float* __restrict__ z, HeadSelect sel,
                                                            Conv12Next nx) {
  WGLOG(1);
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* x8 = smem + HSC_X8_OFF;
  const int64_t b = blockIdx.x;
  const int64_t tau = *sel.tau_ptr + sel.tau_add;
  const int64_t tau0 = *nx.sa.tau_ptr;
  WG_T0();
  unsigned long long* srec = span_rec(nx.sa, tau0);
  span_begin(srec);
  uint64_t* dbg = nullptr;
#ifdef HS_TIMES
  dbg = blockIdx.x == HS_TIMES ? (uint64_t*)z : nullptr;
  if (dbg && threadIdx.x == 0) dbg[0] = __builtin_readcyclecounter();
#endif
  // the next state's planes 0..2 (frames tau-1 .. tau+1 - 1): already in the ring.  Prefetched by
  // waves 2..7 only: in waves 0 (head) and 1 (env act) these loads would queue ahead of the head's
  // and the env state's (in-order vmcnt) -- measured +3k cycles on the head
  // ... and the conv1 weight fragments of those planes (18 KB).  LDS while the frame streams in:
  // scratch [0, 42 KB) = planes 0..2 as bf16 (converted once here, not per conv1 operand),
  // x8 region [0, 18 KB) = their weight fragments; after the screen the x8 region holds the new
  // plane as bf16 (written by the vertical pass) and the scratch becomes conv1's output.
  constexpr int NCH3 = (HIST - 1) * (PLANE / 16);        // 1323 chunks of 16 pixels
  constexpr int PT = 512 - 128;                          // prefetching threads
  constexpr int PER3 = (NCH3 + PT - 1) / PT;             // 4
  constexpr int NWF = (HIST - 1) * 2 * 3 * 64;           // 1152 16-byte fragment rows
  constexpr int PERW = NWF / PT;                         // 3
  static_assert(NWF % PT == 0 && NWF * 16 <= HSC_X8_BYTES, "old-plane conv1 weights in the x8 region");
  static_assert((HIST - 1) * PLANE * 2 <= 51 * 1024, "old planes as bf16 in the screen scratch");
  static_assert(PLANE * 2 <= HSC_X8_BYTES, "new plane as bf16 in the x8 region");
  // fc as K-slice partials (sel.fc_part), folded by wave 0 ahead of the head
  const int fwid = threadIdx.x >> 6, flane = threadIdx.x & 63;
  const bool fold = sel.fc_part != nullptr;
  f32x4 fbias = {0.f, 0.f, 0.f, 0.f};
  // wave 0 loads all FC_NS partial rows itself: no workgroup barrier before the head (each wave
  // loading one slice and meeting in LDS measured 4.10M vs 4.23M env-steps/s)
  f32x4 fpart[FC_NS];
  if (fold && fwid == 0) {
#pragma unroll
    for (int w = 0; w < FC_NS; ++w)
      fpart[w] = *(const f32x4*)(sel.fc_part + ((int64_t)w * gridDim.x + b) * FC + 4 * flane);
    fbias = *(const f32x4*)(sel.fc_bias + 4 * flane);
  }
  const int pt = (int)threadIdx.x - 128;
  uint4 pv[PER3];
  if (pt >= 0) {
#pragma unroll
    for (int k = 0; k < PER3; ++k) {
      const int i = min(pt + PT * k, NCH3 - 1);
      const int c = i / (PLANE / 16), j = i - c * (PLANE / 16);
      pv[k] = ((const uint4*)state_plane(nx.sa, b, c, tau0))[j];
    }
    // the weight fragments go global -> LDS (x8 region, free until the screen) by DMA: no VGPRs
    // (held in registers they spilled 48 B per lane to scratch); landed by the vmcnt(0) below
    const int wbase = (fwid - 2) * 64;
#pragma unroll
    for (int k = 0; k < PERW; ++k)
      glds16((const uint4*)nx.w1s + wbase + PT * k + flane, (uint4*)x8 + wbase + PT * k);
#ifdef HS_TIMES
    if (dbg && pt == 0) dbg[16] = __builtin_readcyclecounter() + (pv[0].x & 0);
#endif
  }
  const float* hrow = nullptr;
  if (fold) {
    // fold the FC_NS slices in slice order, + bias, ReLU; the row goes to LDS [0, 1 KB) (free
    // until head_act_env's barrier) for the head, and to l3_out for the backward
    f32x4* fl = (f32x4*)smem;
    if (fwid == 0) {
      f32x4 v = fpart[0];
#pragma unroll
      for (int w = 1; w < FC_NS; ++w) v += fpart[w];
#pragma unroll
      for (int c4 = 0; c4 < 4; ++c4) v[c4] = fmaxf(v[c4] + fbias[c4], 0.f);
      fl[flane] = v;
      *(f32x4*)(sel.l3_out + b * FC + 4 * flane) = v;
    }
    hrow = (const float*)fl;
  }
  const int32_t frame = head_act_env(h3, Wp, bp, Wv, bv, A, zs, z, sel, b, tau, dbg, hrow);
  uint16_t* xold = (uint16_t*)smem;                      // planes 0..2, bf16
  uint4* wlds = (uint4*)x8;
  if (pt >= 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // the planes and the weight DMA landed
#pragma unroll
    for (int k = 0; k < PER3; ++k) {
      const int i = pt + PT * k;                         // chunk i = pixels 16 i .. 16 i + 15
      if (i < NCH3) {
        uint4* d = (uint4*)(xold + 16 * i);
        const uint2 a0 = atari::u8x4_to_bf16x4(pv[k].x), a1 = atari::u8x4_to_bf16x4(pv[k].y);
        const uint2 a2 = atari::u8x4_to_bf16x4(pv[k].z), a3 = atari::u8x4_to_bf16x4(pv[k].w);
        d[0] = make_uint4(a0.x, a0.y, a1.x, a1.y);
        d[1] = make_uint4(a2.x, a2.y, a3.x, a3.y);
      }
    }
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  // conv1 over the 3 older planes while the new frame streams in from HBM (LDS operands only:
  // nothing here waits on the frame loads); the newest plane's K-steps follow the screen
  f32x4 acc[C1_TILES];
#pragma unroll
  for (int i = 0; i < C1_TILES; ++i) acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  auto conv1_old = [&]() {
    lds_only_barrier();                                  // planes 0..2 and their weights staged
    conv1_accum<false, 0, HIST - 1, false>(nullptr, xold, acc,   // (no pipelining: the frame holds 51 VGPRs)
                                           [&](int f) { return __builtin_bit_cast(bf16x8, wlds[f * 64 + lane]); });
    lds_only_barrier();                                  // operands read: scratch and x8 are the screen's
  };
  // plane 3 = the new screen: to the ring slot (tau + 1) % R and, as bf16, to the x8 region
  uint16_t* xnew = (uint16_t*)x8;
  uint8_t* slot = sel.ring + b * sel.R * PLANE + ((tau + 1) % sel.R) * PLANE;
  if (sel.frame84)
    atari::copy_frame84<512>(sel.pool + (int64_t)frame * PLANE, slot, xnew, conv1_old);
  else
    atari::screen_frame<512>(sel.pool + (int64_t)frame * (atari::IH * atari::IW * 3), slot, smem, dbg, xnew,
                             conv1_old, (int*)(x8 + HSC_KV_OFF));
  if (dbg && threadIdx.x == 0) dbg[9] = __builtin_readcyclecounter();
  uint4 wn[6];
#pragma unroll
  for (int f = 0; f < 6; ++f) wn[f] = ((const uint4*)nx.w1s)[((HIST - 1) * 6 + f) * 64 + lane];
  float w2r[64];
  const float bias2 = nx.b2[16 * (wid & 1) + (lane & 15)];
  __syncthreads();                                       // plane 3 complete in x8
  if (dbg && threadIdx.x == 0) dbg[11] = __builtin_readcyclecounter();
  conv1_accum<false, HIST - 1, HIST>(nullptr, xnew - (HIST - 1) * PLANE, acc, [&](int f) {
    return __builtin_bit_cast(bf16x8, wn[f - (HIST - 1) * 6]);
  });
  conv12_finish<SAVE_L1, false, L2M>(acc, (float*)smem, b, nx.w1s, nx.b1, nx.W2, SAVE_L1 ? nx.act_l1 : nullptr,
                                nx.act_l2, w2r, bias2, dbg, nx.l2m);
  span_end(srec);
  if (dbg) {
    __syncthreads();
    if (threadIdx.x == 0) dbg[10] = __builtin_readcyclecounter();
  }
  WG_T1(z + b * zs);
}

__global__ void __launch_bounds__(256) k_select(const float* __restrict__ z, int64_t B, int zs, int A,
                                                HeadSelect sel) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  float myz = lane < zs ? z[b * zs + lane] : 0.f;
  int32_t a = select_from_lanes(myz, lane, A, sel, b);
  if (lane == 0) sel.actions[b] = a;
}

int a3c_fc_fwd_launch(const float* A, const float* W, const float* bias, float* C, int64_t M, hipStream_t s,
                      const float* Wrows = nullptr);

// skip_conv12: conv1 + conv2 of these states already ran (fused into the previous step's
// k_head_screen_conv12); next: fuse the next states' conv1 + conv2 into this step's head + screen
// the nature trunk's rollout step tail with the fc's split-K fold in front: the workgroup folds
// env b's row of the nsplit K-slice partials (slice order, + bias, ReLU: k_reduce_slabs' order, so
// the row is bit-identical to the separate fold), keeps it in LDS for the head and writes it out for
// the backward -- one launch per step fewer
template <int HS_THREADS, int W>
__global__ void __launch_bounds__(HS_THREADS) k_head_screen_fold(const float* __restrict__ part, int nsplit,
                                                                 int64_t pstride, const float* __restrict__ fbias,
                                                                 float* __restrict__ hout,
                                                                 const float* __restrict__ Wp,
                                                                 const float* __restrict__ bp,
                                                                 const float* __restrict__ Wv,
                                                                 const float* __restrict__ bv, int A, int zs,
                                                                 float* __restrict__ z, HeadSelect sel) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  __shared__ __attribute__((aligned(16))) float hrow[W];
  const int64_t b = blockIdx.x;
  const int64_t tau = *sel.tau_ptr + sel.tau_add;
  for (int i = threadIdx.x; i < W; i += HS_THREADS) {
    const float v = fmaxf(sum_strided(part + b * W + i, nsplit, pstride) + fbias[i], 0.f);
    hrow[i] = v;
    hout[b * W + i] = v;
  }
  __syncthreads();
  const int32_t frame = head_act_env<W>(nullptr, Wp, bp, Wv, bv, A, zs, z, sel, b, tau, nullptr, hrow);
  uint8_t* slot = sel.ring + b * sel.R * PLANE + ((tau + 1) % sel.R) * PLANE;
  if (sel.frame84)
    atari::copy_frame84<HS_THREADS>(sel.pool + (int64_t)frame * PLANE, slot);
  else
    atari::screen_frame<HS_THREADS>(sel.pool + (int64_t)frame * (atari::IH * atari::IW * 3), slot, smem, nullptr);
}

int a3c_head_screen_fold_launch(const float* part, int nsplit, const float* fbias, float* l4, const float* Wp,
                                const float* bp, const float* Wv, const float* bv, int A, int zs, int64_t B, float* z,
                                const HeadSelect& sel, hipStream_t s) {
  static const int env_t = (int)A3C_AB_KNOB("A3C_HS_THREADS", 0);
  const int nt = env_t ? env_t : (a3c_shared_gpu() ? 512 : 1024);
  const int64_t ps = B * 512;
  if (nt == 1024)
    hipLaunchKernelGGL((k_head_screen_fold<1024, 512>), dim3((unsigned)B), dim3(1024), SCREEN_FRAME_SMEM, s, part,
                       nsplit, ps, fbias, l4, Wp, bp, Wv, bv, A, zs, z, sel);
  else
    hipLaunchKernelGGL((k_head_screen_fold<512, 512>), dim3((unsigned)B), dim3(512), SCREEN_FRAME_SMEM, s, part,
                       nsplit, ps, fbias, l4, Wp, bp, Wv, bv, A, zs, z, sel);
  A3C_CHECK(hipGetLastError());
  return 0;
}

// the same for the nature trunk's 512-wide fc output (nature.hip's rollout steps)
int a3c_head_screen_wide_launch(const float* l4, const float* Wp, const float* bp, const float* Wv, const float* bv,
                                int A, int zs, int64_t B, float* z, const HeadSelect& sel, hipStream_t s) {
  static const int env_t = (int)A3C_AB_KNOB("A3C_HS_THREADS", 0);
  const int nt = env_t ? env_t : (a3c_shared_gpu() ? 512 : 1024);
  if (nt == 1024)
    hipLaunchKernelGGL((k_head_screen<1024, 512>), dim3((unsigned)B), dim3(1024), SCREEN_FRAME_SMEM, s, l4, Wp, bp,
                       Wv, bv, A, zs, z, sel);
  else
    hipLaunchKernelGGL((k_head_screen<512, 512>), dim3((unsigned)B), dim3(512), SCREEN_FRAME_SMEM, s, l4, Wp, bp, Wv,
                       bv, A, zs, z, sel);
  A3C_CHECK(hipGetLastError());
  return 0;
}

int a3c_head_screen_conv12_launch(const NetLayout& L, const float* P, const float* act_l3, int64_t B, float* z,
                                  const HeadSelect& sel, const Conv12Next& nx, hipStream_t s);
int a3c_forward_launch(const NetLayout& L, const float* params, const uint8_t* prep, const StateAddr& sa,
                       int64_t B, float* act_l1, float* act_l2, float* act_l3, float* z, const HeadSelect& sel,
                       hipStream_t s, const LstmStep* ls, bool skip_conv12, const Conv12Next* next,
                       float* fc_part, uint32_t* l2m) {
  if (B <= 0) return 0;
  if (L.lstm != (ls != nullptr))
    return a3c_set_error(A3C_ERR_INVALID, "a3c_forward", "the LSTM head needs its recurrent state");
  const float* P = params;
  if (!skip_conv12) {
    int rc0 = a3c_conv12_launch(L, P, prep, sa, B, act_l1, act_l2, s, l2m);
    if (rc0) return rc0;
  }
  // fused overlap rollout: the fc as K-slice partials, folded by the head of k_head_screen_conv12
  // (and the bootstrap state's, folded by k_head_fwd)
  // C5: the LSTM cell folds the partials itself (k_lstm_fwd), on every step of a fused rollout
  const bool part_lstm = fc_part && ls != nullptr;
  const bool part = fc_part && (part_lstm || (next ? sel.mode >= 0 && sel.env_on && sel.ring : sel.mode < 0));
  // (with ls->fc_tick the fc's last K-slice workgroup per tile folds them instead: k_fc_part_fold)
  const bool fold_fc = part_lstm && ls->fc_tick;
  int rc = fold_fc ? a3c_fc_part_fold_launch(act_l2, (const float*)(prep + PREP_W1S_BYTES), fc_part, B, ls->fc_tick,
                                             P + L.off[T_FCB], act_l3, s)
         : part ? a3c_fc_part_launch(act_l2, (const float*)(prep + PREP_W1S_BYTES), fc_part, B, s)
                : a3c_fc_fwd_launch(act_l2, (const float*)(prep + PREP_W1S_BYTES), P + L.off[T_FCB], act_l3, B, s,
                                    P + L.off[T_FCW]);
  if (rc) return rc;
  const float* head_in = act_l3;
  if (ls) {   // C5: LSTM cell on the fc output, heads on its h
    LstmStep st = *ls;
    if (part_lstm && !fold_fc) {
      st.fc_part = fc_part;
      st.fc_bias = P + L.off[T_FCB];
      st.l3_out = act_l3;
    }
    rc = a3c_lstm_fwd_launch(P + L.off[T_LB], act_l3, st, B, s);
    if (rc) return rc;
    head_in = ls->h;
  }
  const float* Wv = L.algo == A3C_ALGO_A3C ? P + L.off[T_VW] : nullptr;
  const float* bv = L.algo == A3C_ALGO_A3C ? P + L.off[T_VB] : nullptr;
  if (sel.mode >= 0 && sel.env_on && sel.ring && next) {
    HeadSelect hs = sel;
    if (part && !part_lstm) {
      hs.fc_part = fc_part;
      hs.fc_bias = P + L.off[T_FCB];
      hs.l3_out = act_l3;
    }
    return a3c_head_screen_conv12_launch(L, P, head_in, B, z, hs, *next, s);
  }
  if (next) return a3c_set_error(A3C_ERR_INVALID, "a3c_forward", "conv fusion needs the fused env screen");
  if (sel.mode >= 0 && sel.env_on && sel.ring)
    return a3c_head_screen_launch(L, P, head_in, B, z, sel, s);
  else {
    HeadSelect hs = sel;
    if (part && !part_lstm) {
      hs.fc_part = fc_part;
      hs.fc_bias = P + L.off[T_FCB];
      hs.l3_out = act_l3;
    }
    hipLaunchKernelGGL(k_head_fwd, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, s, head_in, B,
                       P + L.off[T_HW], P + L.off[T_HB], Wv, bv, L.A, L.zs, z, hs);
  }
  A3C_CHECK(hipGetLastError());
  return 0;
}

// the fused head + env act + screen of one rollout step (profiling hook; see engine.hip)
int a3c_head_screen_launch(const NetLayout& L, const float* P, const float* act_l3, int64_t B, float* z,
                           const HeadSelect& sel, hipStream_t s) {
  const float* Wv = L.algo == A3C_ALGO_A3C ? P + L.off[T_VW] : nullptr;
  const float* bv = L.algo == A3C_ALGO_A3C ? P + L.off[T_VB] : nullptr;
  // 1024 threads when the step owns the GPU; 512 leave room for the concurrent backward
  static const int env_t = (int)A3C_AB_KNOB("A3C_HS_THREADS", 0);
  const int nt = env_t ? env_t : (a3c_shared_gpu() ? 512 : 1024);
  if (nt == 1024)
    hipLaunchKernelGGL(k_head_screen<1024>, dim3((unsigned)B), dim3(1024), SCREEN_FRAME_SMEM, s, act_l3,
                       P + L.off[T_HW], P + L.off[T_HB], Wv, bv, L.A, L.zs, z, sel);
  else
    hipLaunchKernelGGL(k_head_screen<512>, dim3((unsigned)B), dim3(512), SCREEN_FRAME_SMEM, s, act_l3,
                       P + L.off[T_HW], P + L.off[T_HB], Wv, bv, L.A, L.zs, z, sel);
  A3C_CHECK(hipGetLastError());
  return 0;
}

int a3c_head_screen_conv12_launch(const NetLayout& L, const float* P, const float* act_l3, int64_t B, float* z,
                                  const HeadSelect& sel, const Conv12Next& nx, hipStream_t s) {
  const float* Wv = L.algo == A3C_ALGO_A3C ? P + L.off[T_VW] : nullptr;
  const float* bv = L.algo == A3C_ALGO_A3C ? P + L.off[T_VB] : nullptr;
  if (!nx.sa.tau_ptr || !sel.tau_ptr)
    return a3c_set_error(A3C_ERR_INVALID, "a3c_head_screen_conv12", "device tau counters required");
#define HSC_GO(S, M) hipLaunchKernelGGL((k_head_screen_conv12<S, M>), dim3((unsigned)B), dim3(512), HSC_SMEM, s, act_l3, \
                                        P + L.off[T_HW], P + L.off[T_HB], Wv, bv, L.A, L.zs, z, sel, nx)
  if (nx.act_l1 && nx.l2m) HSC_GO(true, true);
  else if (nx.act_l1) HSC_GO(true, false);
  else if (nx.l2m) HSC_GO(false, true);
  else HSC_GO(false, false);
#undef HSC_GO
  A3C_CHECK(hipGetLastError());
  return 0;
}

int a3c_conv12_launch(const NetLayout& L, const float* P, const uint8_t* prep, const StateAddr& sa, int64_t B,
                      float* act_l1, float* act_l2, hipStream_t s, uint32_t* l2m) {
  if (!prep) return a3c_set_error(A3C_ERR_INVALID, "a3c_conv12_launch", "prepared forward weights missing");
  const uint16_t* w1s = (const uint16_t*)prep;
  const bool ew = !a3c_shared_gpu();
  // overlap mode: the 60 KB u8-plane variant (co-resides with the backward's workgroups)
  static const int env_u8 = (int)A3C_AB_KNOB("A3C_C12_U8", -1);
  const bool u8 = env_u8 >= 0 ? env_u8 != 0 : !ew;
#define CONV12_ARGS sa, B, w1s, P + L.off[T_L1B], P + L.off[T_L2W], P + L.off[T_L2B], act_l1, act_l2, l2m
#define CONV12_GO(S, E, U) \
  hipLaunchKernelGGL((k_conv12_fwd<S, E, U>), dim3((unsigned)B), dim3(512), U ? CONV12_SMEM_U8 : CONV12_SMEM, s, CONV12_ARGS)
  if (u8) {
    if (act_l1 && ew) CONV12_GO(true, true, true);
    else if (act_l1) CONV12_GO(true, false, true);
    else if (ew) CONV12_GO(false, true, true);
    else CONV12_GO(false, false, true);
  } else {
    if (act_l1 && ew) CONV12_GO(true, true, false);
    else if (act_l1) CONV12_GO(true, false, false);
    else if (ew) CONV12_GO(false, true, false);
    else CONV12_GO(false, false, false);
  }
#undef CONV12_GO
#undef CONV12_ARGS
  A3C_CHECK(hipGetLastError());
  return 0;
}

int a3c_select_launch(const float* z, int64_t B, int zs, int A, const HeadSelect& sel, hipStream_t s) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL(k_select, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, s, z, B, zs, A, sel);
  A3C_CHECK(hipGetLastError());
  return 0;
}

void a3c_conv12_set_smem() {
#define C12_SMEM(S, E, U)                                                                        \
  (void)hipFuncSetAttribute((const void*)k_conv12_fwd<S, E, U>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                            U ? CONV12_SMEM_U8 : CONV12_SMEM)
  C12_SMEM(true, true, false); C12_SMEM(true, false, false); C12_SMEM(false, true, false); C12_SMEM(false, false, false);
  C12_SMEM(true, true, true); C12_SMEM(true, false, true); C12_SMEM(false, true, true); C12_SMEM(false, false, true);
#undef C12_SMEM
  (void)hipFuncSetAttribute((const void*)k_head_screen_conv12<true, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            HSC_SMEM);
  (void)hipFuncSetAttribute((const void*)k_head_screen_conv12<true, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            HSC_SMEM);
  (void)hipFuncSetAttribute((const void*)k_head_screen_conv12<false, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            HSC_SMEM);
  (void)hipFuncSetAttribute((const void*)k_head_screen_conv12<false, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            HSC_SMEM);
  (void)hipFuncSetAttribute((const void*)k_head_screen<512>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            SCREEN_FRAME_SMEM);
  (void)hipFuncSetAttribute((const void*)k_head_screen<1024>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            SCREEN_FRAME_SMEM);
  (void)hipFuncSetAttribute((const void*)k_head_screen<512, 512>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            SCREEN_FRAME_SMEM);
  (void)hipFuncSetAttribute((const void*)k_head_screen<1024, 512>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            SCREEN_FRAME_SMEM);
  (void)hipFuncSetAttribute((const void*)k_head_screen_fold<512, 512>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            SCREEN_FRAME_SMEM);
  (void)hipFuncSetAttribute((const void*)k_head_screen_fold<1024, 512>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            SCREEN_FRAME_SMEM);
}

// ---------------------------------------------------------------------------------------
// fc layer of the rollout (agent.py:251 / network.py:51-52): l3 = relu(l2 @ W + b) for a
// skinny batch (M = E states, N = 256, K = 2592).  One workgroup per 16x16 output tile; the
// 4 waves split the 162 K-chunks of 16 and meet in LDS.  Per chunk a lane loads one 16-byte A
// fragment (4 consecutive k of its row) and one 16-byte B fragment from the fragment-packed
// weights (k_prep_fwd), feeding 4 v_mfma_f32_16x16x4_f32; a ring of D chunks keeps 2D loads in
// flight per wave.  blockIdx.x (column tile) is the fast grid index, so the 8 XCDs each stream
// 2 column tiles of W (L2-resident) and the l2 rows.
// ---------------------------------------------------------------------------------------
template <int NW>
__global__ void __launch_bounds__(64 * NW) k_fc_fwd(const float* __restrict__ A, const float* __restrict__ Wp,
                                                    const float* __restrict__ bias, float* __restrict__ C, int M,
                                                    int xcd_rows) {
  __shared__ f32x4 red[NW - 1][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int i16 = lane & 15, j4 = lane >> 4;
  // xcd_rows: 1-D grid, workgroup id -> XCD id % 8 gets a contiguous band of row tiles (all 16
  // column tiles each), so an XCD reads 1/8 of A and all of W (which is the same every step)
  int ct = blockIdx.x, mt = blockIdx.y;
  int m0, rstride = 1;                 // tile row i is row m0 + rstride * i
  if (xcd_rows == 2) {
    // rows of one XCD's envs: workgroup id -> XCD id % 8 = x takes rows x, x + 8, ... (the l2 rows
    // the rollout kernel's workgroups x + 8 k wrote on that XCD, and the l3 rows its next launch
    // reads there), all 16 column tiles; speed only, any placement is correct
    const int id = blockIdx.x, k = id >> 3;
    ct = k % (FC / 16);
    m0 = 128 * (k / (FC / 16)) + (id & 7);
    rstride = 8;
  } else {
    if (xcd_rows) {
      const int ntiles = gridDim.x, id = blockIdx.x;
      const int t = (id & 7) * (ntiles >> 3) + (id >> 3);
      ct = t % (FC / 16);
      mt = t / (FC / 16);
    }
    m0 = mt * 16;
  }
  const int n0 = ct * 16;
  const int m = min(m0 + rstride * i16, M - 1);
  WG_T0();
  // the waves' partial tiles meet in LDS (fixed order), bias + relu, store
  auto fc_epilogue = [&](f32x4 acc) {
    if (wid > 0) red[wid - 1][lane] = acc;
    __syncthreads();
    if (wid == 0) {
#pragma unroll
      for (int w = 0; w < NW - 1; ++w) acc += red[w][lane];
      const int n = n0 + i16;
      const float bb = bias[n];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + rstride * (4 * j4 + r);
        if (row < M) st_act(C + (int64_t)row * FC + n, fmaxf(acc[r] + bb, 0.f));
      }
    }
    WG_T1(C + (int64_t)m0 * FC + n0);   // debug: the tile's first 4 outputs
  };
#ifdef FC_K32   // A/B: faster alone (8.7 vs 9.2 us), slower overlapped (3.82M vs 4.00M)
  // 32-deep chunks [c0, c1) of this wave (81 split as evenly as possible): per chunk a lane loads
  // 8 consecutive k of its row (32 B: the row's 128-B line is read whole by the 4 lane groups)
  // and its 8 packed weights, for 8 MFMAs (k permuted within the chunk identically for A and B)
  {
    const int c0 = (wid * FC_CH32) / NW, c1 = ((wid + 1) * FC_CH32) / NW;
    constexpr int D = 4;
    const float* a = A + (int64_t)m * FLAT + 8 * j4;
    const f32x4* b = (const f32x4*)Wp + (int64_t)ct * FC_CH32 * 128 + 2 * lane;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    f32x4 ra[D][2], rb[D][2];
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int cc = min(c0 + d, c1 - 1);
      ra[d][0] = *(const f32x4*)(a + 32 * cc);
      ra[d][1] = *(const f32x4*)(a + 32 * cc + 4);
      rb[d][0] = b[(int64_t)cc * 128];
      rb[d][1] = b[(int64_t)cc * 128 + 1];
    }
    for (int c = c0; c < c1; c += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        if (c + d < c1) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[d][h][0], rb[d][h][0], acc, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[d][h][1], rb[d][h][1], acc1, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[d][h][2], rb[d][h][2], acc, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[d][h][3], rb[d][h][3], acc1, 0, 0, 0);
          }
          const int cn = c + d + D;
          if (cn < c1) {
            ra[d][0] = *(const f32x4*)(a + 32 * cn);
            ra[d][1] = *(const f32x4*)(a + 32 * cn + 4);
            rb[d][0] = b[(int64_t)cn * 128];
            rb[d][1] = b[(int64_t)cn * 128 + 1];
          }
        }
      }
    }
    fc_epilogue(acc + acc1);
    return;
  }
#endif
  // chunks [c0, c1) of this wave: the 162 chunks split as evenly as possible
  const int c0 = (wid * FC_CH) / NW, c1 = ((wid + 1) * FC_CH) / NW;
#ifndef FC_D
#define FC_D 8
#endif
  constexpr int D = FC_D;
  const float* a = A + (int64_t)m * FLAT + 4 * j4;
  const f32x4* b = (const f32x4*)Wp + (int64_t)ct * FC_CH * 64 + lane;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  f32x4 ra[D], rb[D];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    ra[d] = *(const f32x4*)(a + 16 * (c0 + d));
    rb[d] = b[(int64_t)(c0 + d) * 64];
  }
  for (int c = c0; c < c1; c += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      if (c + d < c1) {
        // two independent accumulation chains (MFMA dependent latency > issue interval)
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[d][0], rb[d][0], acc, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[d][1], rb[d][1], acc1, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[d][2], rb[d][2], acc, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[d][3], rb[d][3], acc1, 0, 0, 0);
        const int cn = c + d + D;                 // refill this slot with chunk cn
        if (cn < c1) {
          ra[d] = *(const f32x4*)(a + 16 * cn);
          rb[d] = b[(int64_t)cn * 64];
        }
      }
    }
  }
  fc_epilogue(acc + acc1);
}

// ---------------------------------------------------------------------------------------
// fc layer of the fused overlap rollout as K-slice partials (the consumer folds them): the
// k_fc_fwd tile above moves 332 KB per workgroup (a 16-row A strip and a 16-column W strip over
// all of K), which is what bounds it.  Here workgroup (x, rb, cb) multiplies the 32 rows of
// row block rb by the 64 columns of column block cb over K-slice x only (20-21 of the 162
// chunks of 16): 43 KB of A staged once in LDS and shared by the 4 waves (one 16-column tile
// each, both 16-row tiles), 21 KB of packed W per wave -- 129 KB per workgroup.  The partial
// sums go to part[x][row][256]; the head of the rollout kernel folds the FC_NS slices in a
// fixed order (+ bias, ReLU), so the layer output is deterministic.  blockIdx.x & 7 is the
// K-slice: under round-robin placement each XCD streams only its slice of W (332 KB), which
// stays L2-resident across the rollout's steps (speed only, any placement is correct).
// ---------------------------------------------------------------------------------------
#define FCP_RB 32                               // rows per row block
#define FCP_CB 64                               // columns per column block (4 waves x 16)
#define FCP_MAXCH ((FC_CH + FC_NS - 1) / FC_NS + 1)   // 21 chunks per slice at most
#define FCP_LD (FCP_MAXCH * 16 + 4)             // A row stride in LDS (floats), padded
#define FCP_SMEM (FCP_RB * FCP_LD * 4)          // 43520
__device__ inline int fcp_c0(int x) { return (FC_CH * x) / FC_NS; }

// KS > 1: each of the 4 column tiles is split over KS waves by K ranges (chunk ranges of equal
// length), so each wave's serial MFMA chain is KS times shorter; the waves of ranges 1..KS-1 hand
// their sums to range 0's wave through LDS, which adds them in range order and stores.  KS = 2:
// two waves per SIMD at 75 VGPRs, KS = 4: four at <= 64 VGPRs -- beside a compact conv backward
// workgroup either way.  Measured (M1 / M2 env-steps/s): KS 1 4.67M / 5.82M, KS 2 4.78M / 6.07M.
//
// FOLD (C5, the LSTM cell's input): the tile's K-slice workgroups hand their partials to the one
// whose ticket comes last, which folds the FC_NS slices in slice order (+ bias, ReLU: the cell
// kernel's fold, bit for bit) and writes the fc output rows -- once per tile instead of once per
// LSTM unit tile.  Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility, first row of the
// sc1 table): every partial is stored sc1 (write-through), every storing wave drains vmcnt before
// the workgroup barrier, lane 0 draws an agent-scope ticket, and the last arriver reads the
// partials with sc1 loads only.  tick[tile] is zeroed at engine creation and reset by the last
// arriver (every launch completes all FC_NS tickets of every tile).
template <int KS, bool FOLD>
__device__ __forceinline__ void fc_part_body(const float* __restrict__ A, const float* __restrict__ Wp,
                                             float* __restrict__ part, int M, int64_t* adv_ptr, int adv_n,
                                             unsigned* tick, const float* fbias, float* fout) {
  if (adv_ptr && blockIdx.x == 0 && threadIdx.x == 0) *adv_ptr += adv_n;   // (reads no tau)
  __shared__ __attribute__((aligned(16))) float as[FCP_RB * FCP_LD];
  constexpr int NT = 256 * KS;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int i16 = lane & 15, j4 = lane >> 4;
  const int id = blockIdx.x;
  const int x = id % FC_NS, k = id / FC_NS;
  const int rb = k / (FC / FCP_CB), cb = k % (FC / FCP_CB);
  const int c0 = fcp_c0(x), c1 = fcp_c0(x + 1), nch = c1 - c0;
  const int m0 = rb * FCP_RB, ct = cb * (FCP_CB / 16) + (wid & 3);
  // this wave's K range
  const int kr = wid >> 2;
  const int kc0 = (nch * kr) / KS, kc1 = (nch * (kr + 1)) / KS;
  const int kn = kc1 - kc0;
  // this wave's packed-W chunks (16-byte fragments, 4 MFMAs each), the first D in flight before
  // the A tile is staged.  D = 8 keeps the 4-wave kernel at 96 VGPRs: all 21 in flight (152
  // VGPRs) is faster alone (6.8 vs 7.4 us) and loses overlapped (3.83M vs 4.09M env-steps/s)
#ifndef FCP_D
#define FCP_D 8
#endif
#ifndef FCP_D4
#define FCP_D4 4
#endif
  constexpr int D = KS == 4 ? FCP_D4 : FCP_D;
  const f32x4* bp = (const f32x4*)Wp + ((int64_t)ct * FC_CH + c0 + kc0) * 64 + lane;
  f32x4 rb4[D];
#pragma unroll
  for (int d = 0; d < D; ++d) rb4[d] = bp[(int64_t)min(d, kn - 1) * 64];
  // A tile: 32 rows x nch chunks of 16 floats, f32x4 per thread-iteration, all loads issued first
  constexpr int NA = (FCP_RB * FCP_MAXCH * 4 + NT - 1) / NT;   // 11, 6, 3
  f32x4 ra[NA];
  const int q4 = nch * 4;                                    // f32x4 per row
#pragma unroll
  for (int u = 0; u < NA; ++u) {
    const int i = min((int)threadIdx.x + NT * u, FCP_RB * q4 - 1);
    const int r = i / q4, q = i - r * q4;
    ra[u] = *(const f32x4*)(A + (int64_t)min(m0 + r, M - 1) * FLAT + 16 * c0 + 4 * q);
  }
#pragma unroll
  for (int u = 0; u < NA; ++u) {
    const int i = (int)threadIdx.x + NT * u;
    if (i < FCP_RB * q4) {
      const int r = i / q4, q = i - r * q4;
      *(f32x4*)(as + r * FCP_LD + 4 * q) = ra[u];
    }
  }
  __syncthreads();
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};   // row tiles 0 / 1
  const float* a0 = as + i16 * FCP_LD + 4 * j4 + 16 * kc0;
  const float* a1 = a0 + 16 * FCP_LD;
  for (int c = 0; c < kn; c += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      if (c + d < kn) {
        const f32x4 x0 = *(const f32x4*)(a0 + 16 * (c + d));
        const f32x4 x1 = *(const f32x4*)(a1 + 16 * (c + d));
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) {
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x0[c4], rb4[d][c4], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(x1[c4], rb4[d][c4], acc1, 0, 0, 0);
        }
        const int cn = c + d + D;
        if (cn < kn) rb4[d] = bp[(int64_t)cn * 64];
      }
    }
  }
  if constexpr (KS > 1) {   // ranges 1.. -> LDS (the A tile is no longer read) -> range 0 adds in order
    __syncthreads();
    f32x4* xs = (f32x4*)as;
    if (kr) {
      xs[(((kr - 1) * 4 + (wid & 3)) * 2 + 0) * 64 + lane] = acc0;
      xs[(((kr - 1) * 4 + (wid & 3)) * 2 + 1) * 64 + lane] = acc1;
    }
    __syncthreads();
    if constexpr (!FOLD) {
      if (kr) return;
    }
    if (!kr) {
#pragma unroll
      for (int q = 0; q < KS - 1; ++q) {
        acc0 += xs[((q * 4 + (wid & 3)) * 2 + 0) * 64 + lane];
        acc1 += xs[((q * 4 + (wid & 3)) * 2 + 1) * 64 + lane];
      }
    }
  }
  // partial tile rows m0 + 16 rt + 4 j4 + r, column 16 ct + i16
  float* out = part + ((int64_t)x * M) * FC + 16 * ct + i16;
  if constexpr (!FOLD) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row0 = m0 + 4 * j4 + r, row1 = row0 + 16;
      if (row0 < M) out[(int64_t)row0 * FC] = acc0[r];
      if (row1 < M) out[(int64_t)row1 * FC] = acc1[r];
    }
  } else {
    if (kr == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row0 = m0 + 4 * j4 + r, row1 = row0 + 16;
        if (row0 < M) __hip_atomic_store(out + (int64_t)row0 * FC, acc0[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (row1 < M) __hip_atomic_store(out + (int64_t)row1 * FC, acc1[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");      // every storing wave drains its sc1 stores
    __syncthreads();
    unsigned* flag = (unsigned*)as + (FCP_RB * FCP_LD - 1);   // a pad word of the A tile's last row
    if (threadIdx.x == 0) {
      const unsigned t = __hip_atomic_fetch_add(tick + k, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (t == FC_NS - 1) __hip_atomic_store(tick + k, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = t;
    }
    __syncthreads();
    if (*flag != FC_NS - 1) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // (no instruction: keeps the loads below)
    // fold of the tile: 32 rows x 64 columns as 512 groups of 4, slices in order, + bias, ReLU
    for (int i = threadIdx.x; i < FCP_RB * FCP_CB / 4; i += 256 * KS) {
      const int row = m0 + i / (FCP_CB / 4), col = cb * FCP_CB + 4 * (i % (FCP_CB / 4));
      if (row >= M) continue;
      const float* pp = part + (int64_t)row * FC + col;
      f32x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = __hip_atomic_load(pp + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int xs2 = 1; xs2 < FC_NS; ++xs2) {
        const float* q = pp + (int64_t)xs2 * M * FC;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += __hip_atomic_load(q + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      const f32x4 fb = *(const f32x4*)(fbias + col);
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r] + fb[r], 0.f);
      *(f32x4*)(fout + (int64_t)row * FC + col) = v;
    }
  }
}

template <int KS>
__global__ void __launch_bounds__(256 * KS) __attribute__((amdgpu_waves_per_eu(KS == 4 ? 8 : 1)))
k_fc_part(const float* __restrict__ A, const float* __restrict__ Wp, float* __restrict__ part, int M,
          int64_t* adv_ptr, int adv_n) {
  WGLOG(2);
  fc_part_body<KS, false>(A, Wp, part, M, adv_ptr, adv_n, nullptr, nullptr, nullptr);
}

template <int KS>
__global__ void __launch_bounds__(256 * KS) __attribute__((amdgpu_waves_per_eu(KS == 4 ? 8 : 1)))
k_fc_part_fold(const float* __restrict__ A, const float* __restrict__ Wp, float* part, int M,
               unsigned* tick, const float* __restrict__ fbias, float* __restrict__ fout) {
  fc_part_body<KS, true>(A, Wp, part, M, nullptr, 0, tick, fbias, fout);
}

// K splits of the partial fc, set by the engine per frame mode (a3c_set_fcp_split; A3C_FCP_KS
// overrides): M1 4 (4.72-4.75M -> 4.76-4.81M env-steps/s against 2), M2 2 (6.02-6.03M vs 5.99-6.00M)
static thread_local int t_fcp_split = 2;
int a3c_fcp_split() { return t_fcp_split; }
void a3c_set_fcp_split(int ks) { t_fcp_split = ks; }

int a3c_fc_part_fold_launch(const float* A, const float* Wp, float* part, int64_t M, unsigned* tick,
                            const float* fbias, float* fout, hipStream_t s) {
  if (M <= 0) return 0;
  if (!tick || !fbias || !fout || (((uintptr_t)fbias | (uintptr_t)fout) & 15))
    return a3c_set_error(A3C_ERR_INVALID, "a3c_fc_part_fold", "bad argument");
  const int nrb = (int)((M + FCP_RB - 1) / FCP_RB);
  static const int env_ks = (int)A3C_AB_KNOB("A3C_FCP_KS", 0);
  const int ks = env_ks ? env_ks : a3c_fcp_split();
  const dim3 grid((unsigned)(FC_NS * nrb * (FC / FCP_CB)));
  if (ks == 4) hipLaunchKernelGGL(k_fc_part_fold<4>, grid, dim3(1024), 0, s, A, Wp, part, (int)M, tick, fbias, fout);
  else if (ks == 2) hipLaunchKernelGGL(k_fc_part_fold<2>, grid, dim3(512), 0, s, A, Wp, part, (int)M, tick, fbias, fout);
  else hipLaunchKernelGGL(k_fc_part_fold<1>, grid, dim3(256), 0, s, A, Wp, part, (int)M, tick, fbias, fout);
  A3C_CHECK(hipGetLastError());
  return 0;
}

int a3c_fc_part_launch(const float* A, const float* Wp, float* part, int64_t M, hipStream_t s, int64_t* adv_ptr,
                       int adv_n) {
  if (M <= 0) return 0;
#ifdef A3C_MARKERS
  static const bool ablate = getenv("A3C_ABL_FC") != nullptr;   // measurement only: no fc
  if (ablate && !adv_ptr) return 0;
#endif
  const int nrb = (int)((M + FCP_RB - 1) / FCP_RB);
  static const int env_ks = (int)A3C_AB_KNOB("A3C_FCP_KS", 0);
  const int ks = env_ks ? env_ks : a3c_fcp_split();
  const dim3 grid((unsigned)(FC_NS * nrb * (FC / FCP_CB)));
  if (ks == 4) hipLaunchKernelGGL(k_fc_part<4>, grid, dim3(1024), 0, s, A, Wp, part, (int)M, adv_ptr, adv_n);
  else if (ks == 2) hipLaunchKernelGGL(k_fc_part<2>, grid, dim3(512), 0, s, A, Wp, part, (int)M, adv_ptr, adv_n);
  else hipLaunchKernelGGL(k_fc_part<1>, grid, dim3(256), 0, s, A, Wp, part, (int)M, adv_ptr, adv_n);
  A3C_CHECK(hipGetLastError());
  return 0;
}

int a3c_head_fold_launch(const NetLayout& L, const float* P, const float* fc_part, int64_t B, float* z,
                         hipStream_t s) {
  if (B <= 0) return 0;
  HeadSelect hs = {};
  hs.mode = -1;
  hs.E = (int)B;
  hs.fc_part = fc_part;
  hs.fc_bias = P + L.off[T_FCB];
  const float* Wv = L.algo == A3C_ALGO_A3C ? P + L.off[T_VW] : nullptr;
  const float* bv = L.algo == A3C_ALGO_A3C ? P + L.off[T_VB] : nullptr;
  hipLaunchKernelGGL(k_head_fwd, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, s, nullptr, B, P + L.off[T_HW],
                     P + L.off[T_HB], Wv, bv, L.A, L.zs, z, hs);
  A3C_CHECK(hipGetLastError());
  return 0;
}

// row-major-weight variant (4 scalar B loads per chunk), kept for A/B measurement
__global__ void __launch_bounds__(256) k_fc_fwd_rows(const float* __restrict__ A, const float* __restrict__ W,
                                                const float* __restrict__ bias, float* __restrict__ C, int M) {
  __shared__ f32x4 red[3][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int i16 = lane & 15, j4 = lane >> 4;
  const int m0 = blockIdx.y * 16, n0 = blockIdx.x * 16;
  const int m = min(m0 + i16, M - 1);
  constexpr int KW = FLAT / 4;                    // 648 per wave
  constexpr int NCH = KW / 16;                    // 40 chunks of 16 (+ 8 left)
  constexpr int D = 8;                            // chunks in flight per wave (register ring)
  const float* a = A + (int64_t)m * FLAT + wid * KW + 4 * j4;
  const float* b = W + (int64_t)(wid * KW + 4 * j4) * FC + n0 + i16;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  f32x4 ra[D];
  float rb[D][4];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    ra[d] = *(const f32x4*)(a + 16 * d);
#pragma unroll
    for (int c4 = 0; c4 < 4; ++c4) rb[d][c4] = b[(int64_t)(16 * d + c4) * FC];
  }
  for (int c0 = 0; c0 < NCH; c0 += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
#pragma unroll
      for (int c4 = 0; c4 < 4; ++c4)
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[d][c4], rb[d][c4], acc, 0, 0, 0);
      const int cn = c0 + d + D;                  // refill this slot with chunk cn
      if (cn < NCH) {
        ra[d] = *(const f32x4*)(a + 16 * cn);
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) rb[d][c4] = b[(int64_t)(16 * cn + c4) * FC];
      }
    }
  }
  // tail: 8 = KW - 16*NCH values per wave -> lane groups j4 < 2 carry them, others add zeros
  {
    const bool live = j4 < 2;
    const float* at = A + (int64_t)m * FLAT + wid * KW + 16 * NCH + 4 * (j4 & 1);
    const float* bt = W + (int64_t)(wid * KW + 16 * NCH + 4 * (j4 & 1)) * FC + n0 + i16;
    f32x4 x = *(const f32x4*)at;
#pragma unroll
    for (int c4 = 0; c4 < 4; ++c4)
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(live ? x[c4] : 0.f, live ? bt[c4 * FC] : 0.f, acc, 0, 0, 0);
  }
  if (wid > 0) red[wid - 1][lane] = acc;
  __syncthreads();
  if (wid == 0) {
    acc += red[0][lane];
    acc += red[1][lane];
    acc += red[2][lane];
    const int n = n0 + i16;
    const float bb = bias[n];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + 4 * j4 + r;
      if (row < M) C[(int64_t)row * FC + n] = fmaxf(acc[r] + bb, 0.f);
    }
  }
}

int a3c_fc_fwd_launch(const float* A, const float* W, const float* bias, float* C, int64_t M, hipStream_t s,
                      const float* Wrows) {
  if (M <= 0) return 0;
#ifdef A3C_MARKERS
  static const bool ablate = getenv("A3C_ABL_FC") != nullptr;   // measurement only: no fc
  if (ablate) return 0;
#endif
  static const int env_nw = (int)A3C_AB_KNOB("A3C_FC_WAVES", -1);
  const int nw = env_nw >= 0 ? env_nw : (a3c_shared_gpu() ? 4 : 8);
  if (nw == 0 && Wrows)
    hipLaunchKernelGGL(k_fc_fwd_rows, dim3(FC / 16, (unsigned)((M + 15) / 16)), dim3(256), 0, s, A, Wrows, bias, C,
                       (int)M);
  else {
    static const int env_x = (int)A3C_AB_KNOB("A3C_FC_XCD", 0);
    const int mt = (int)((M + 15) / 16), ntiles = mt * (FC / 16);
    const int xr = env_x == 2 ? (M % 128 == 0 ? 2 : 0) : (env_x && ntiles % 8 == 0);
    const dim3 grid = xr ? dim3((unsigned)ntiles) : dim3(FC / 16, (unsigned)mt);
    if (nw == 4)
      hipLaunchKernelGGL(k_fc_fwd<4>, grid, dim3(256), 0, s, A, W, bias, C, (int)M, xr);
    else if (nw == 16)
      hipLaunchKernelGGL(k_fc_fwd<16>, grid, dim3(1024), 0, s, A, W, bias, C, (int)M, xr);
    else
      hipLaunchKernelGGL(k_fc_fwd<8>, grid, dim3(512), 0, s, A, W, bias, C, (int)M, xr);
  }
  A3C_CHECK(hipGetLastError());
  return 0;
}

#ifdef A3C_WGLOG
WGLOG_BIND(a3c_wglog_bind_fwd)
#endif

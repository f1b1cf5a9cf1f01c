// K1 specialised for the Atari geometry 210x160 RGB -> 84x84 (environment.py:49-53 with
// config.py:38-39): Pillow's BILINEAR coefficients are generated at compile time (constexpr
// restatement of precompute_coeffs/normalize_coeffs_8bpc, IEEE double, no contraction), every
// tap loop has a fixed length (zero weights past a row's count, reads clamped in bounds), and
// the luminance uses an exact integer form:
//   numpy's fp64  0.2126 R + 0.7152 G + 0.0722 B  truncated  ==  floor((2126R + 7152G + 722B) / 10^4)
// whenever the integer sum is not a multiple of 10^4 (the fp64 rounding error, < 1e-13, cannot
// cross an integer that lies >= 1e-4 away); multiples of 10^4 take the fp64 expression itself.
// Exhaustively checked over all 2^24 RGB values against the reference's table
// (tests/test_gpu_kernels.py::test_preprocess_full_luminance_table).
#pragma once
#include "preprocess_dev.h"

namespace atari {

constexpr int IH = 210, IW = 160, OH = 84, OW = 84;

template <int IN, int OUT>
struct Coef {
  static constexpr double scale = (double)(float)IN / (double)OUT;
  static constexpr double filterscale = scale < 1.0 ? 1.0 : scale;
  static constexpr double support = 1.0 * filterscale;
  static constexpr int K = ((int)support + ((double)(int)support < support ? 1 : 0)) * 2 + 1;
  int xmin[OUT];
  int cnt[OUT];
  int k[OUT][K];
  constexpr Coef() : xmin(), cnt(), k() {
    for (int xx = 0; xx < OUT; ++xx) {
      const double center = 0.0 + (xx + 0.5) * scale;
      const double ss = 1.0 / filterscale;
      int lo = (int)(center - support + 0.5);
      if (lo < 0) lo = 0;
      int hi = (int)(center + support + 0.5);
      if (hi > IN) hi = IN;
      const int n = hi - lo;
      double ww = 0.0;
      for (int x = 0; x < n; ++x) ww += tap(x, lo, center, ss);
      for (int x = 0; x < K; ++x) {
        double w = 0.0;
        if (x < n) {
          w = tap(x, lo, center, ss);
          if (ww != 0.0) w = w / ww;
        }
        const double v = w * (double)(1 << A3C_PRECISION_BITS);
        k[xx][x] = w < 0 ? (int)(-0.5 + v) : (int)(0.5 + v);
      }
      xmin[xx] = lo;
      cnt[xx] = n;
    }
  }
  static constexpr double tap(int x, int lo, double center, double ss) {
    double t = ((double)(x + lo) - center + 0.5) * ss;
    if (t < 0.0) t = -t;
    return t < 1.0 ? 1.0 - t : 0.0;
  }
};

constexpr Coef<IW, OW> kH{};
constexpr Coef<IH, OH> kV{};
constexpr int KH = Coef<IW, OW>::K;   // 5
constexpr int KV = Coef<IH, OH>::K;   // 7

// Bilinear taps are >= 0 and each output's sum stays below (2^30 - 2^21) / 255, so
// 2^21 + sum(v k) for 8-bit v never leaves [0, 256 * 2^22): Pillow's clip is a plain shift here
template <int IN, int OUT>
constexpr bool taps_shift_only(const Coef<IN, OUT>& c) {
  for (int xx = 0; xx < OUT; ++xx) {
    long sum = 0;
    for (int x = 0; x < Coef<IN, OUT>::K; ++x) {
      if (c.k[xx][x] < 0) return false;
      sum += c.k[xx][x];
    }
    if (255L * sum + (1L << (A3C_PRECISION_BITS - 1)) >= (256L << A3C_PRECISION_BITS)) return false;
  }
  return true;
}
static_assert(taps_shift_only(kH) && taps_shift_only(kV), "resampling taps need Pillow's clip");

__constant__ Coef<IW, OW> cH = kH;
__constant__ Coef<IH, OH> cV = kV;

// source rows [y0, y1) of output band [yy0, yy0 + rows)
constexpr int band_y0(int yy0) { return kV.xmin[yy0]; }
constexpr int band_y1(int yy0, int rows) { return kV.xmin[yy0 + rows - 1] + kV.cnt[yy0 + rows - 1]; }
template <int ROWS>
constexpr int max_src_rows() {
  int m = 0;
  for (int b = 0; b * ROWS < OH; ++b) {
    const int r = (b + 1) * ROWS <= OH ? ROWS : OH - b * ROWS;
    const int s = band_y1(b * ROWS, r) - band_y0(b * ROWS);
    m = s > m ? s : m;
  }
  return m;
}

// exact truncated fp64 luminance (see header)
__device__ inline uint32_t lum_exact(uint32_t r, uint32_t g, uint32_t b) {
  const uint32_t y = 2126u * r + 7152u * g + 722u * b;       // < 2^22
  const uint32_t q = (uint32_t)(((uint64_t)y * 3518437209ull) >> 45);   // y / 10000 (exact for y < 2^32/..)
  if (q * 10000u == y) return a3c_lum(r, g, b);               // exact multiple: fp64 decides
  return q;
}

// 4 pixels (3 dwords of RGB) -> 4 luminance bytes, the same exact integer form:
// y = 2126 R + 7152 G + 722 B from two v_dot4_u32_u8 over the weights' low / high bytes
// (2126 = 8*256 + 78, 7152 = 27*256 + 240, 722 = 2*256 + 210), floor(y / 10^4) by a
// multiply-high; a group with a multiple of 10^4 redoes its pixels with lum_exact.
__device__ inline uint32_t lum4(uint32_t d0, uint32_t d1, uint32_t d2) {
  constexpr uint32_t WLO = 78u | (240u << 8) | (210u << 16);
  constexpr uint32_t WHI = 8u | (27u << 8) | (2u << 16);
  const uint32_t px[4] = {d0, __builtin_amdgcn_alignbyte(d1, d0, 3), __builtin_amdgcn_alignbyte(d2, d1, 2), d2 >> 8};
  // stage by stage over the 4 pixels (independent chains interleave instead of each pixel's
  // dependent dot4 -> shift -> dot4 -> multiply sequence waiting on its own latency)
  uint32_t y[4], q[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) y[i] = __builtin_amdgcn_udot4(px[i], WHI, 0u, false) << 8;
#pragma unroll
  for (int i = 0; i < 4; ++i) y[i] = __builtin_amdgcn_udot4(px[i], WLO, y[i], false) & 0x3FFFFFu;
  // y <= 2,550,000 < 2^22, so floor(y / 10^4) = (y * 13743896) >> 37 (exhaustively checked over
  // [0, 2550000]) on the full-rate 24-bit multiplier (v_mul_hi_u32_u24), not the quarter-rate
  // 32-bit v_mul_hi_u32; the mask only tells the compiler the operand width
  // y is a multiple of 10^4 iff the product's low 37 bits are below 2^22 (multiples leave
  // q * 6528 <= 1,664,640 there, the others at least 13,743,896; exhaustively checked)
  bool mult = false;
  uint32_t out = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t hi = (uint32_t)(((uint64_t)y[i] * 13743896ull) >> 32);   // v_mul_hi_u32_u24
    const uint32_t lo = y[i] * 13743896u;                                   // v_mul_u32_u24
    q[i] = hi >> 5;
    mult |= (hi & 31u) == 0u && lo < (1u << 22);
    out |= q[i] << (8 * i);
  }
  if (mult) {
    out = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) out |= lum_exact(px[i] & 255u, (px[i] >> 8) & 255u, (px[i] >> 16) & 255u) << (8 * i);
  }
  return out;
}

// 16 pixels (48 bytes of RGB) -> 16 luminance bytes
__device__ inline uint4 lum16(const uint4 a, const uint4 b, const uint4 c) {
  const uint32_t w[12] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w};
  uint32_t o[4] = {0, 0, 0, 0};
#pragma unroll
  for (int p = 0; p < 16; ++p) {
    const int i0 = 3 * p, i1 = 3 * p + 1, i2 = 3 * p + 2;
    const uint32_t rr = (w[i0 >> 2] >> (8 * (i0 & 3))) & 255u;
    const uint32_t gg = (w[i1 >> 2] >> (8 * (i1 & 3))) & 255u;
    const uint32_t bb = (w[i2 >> 2] >> (8 * (i2 & 3))) & 255u;
    o[p >> 2] |= lum_exact(rr, gg, bb) << (8 * (p & 3));
  }
  return make_uint4(o[0], o[1], o[2], o[3]);
}

// Horizontal pass of output columns [X0, X1) of one gray row (segments 0..3 = [0,24), [24,44),
// [44,64), [64,84)): the 64-byte window from the 16-aligned byte below kH.xmin[X0] is read as
// four ds_read_b128 and every tap is a compile-time byte of it; outputs packed 4 per dword.
template <int SEG>
__device__ inline void hpass_seg(const uint8_t* __restrict__ grow, uint8_t* __restrict__ trow) {
  constexpr int X0 = SEG == 0 ? 0 : 4 + 20 * SEG, X1 = SEG == 0 ? 24 : X0 + 20;
  constexpr int BASE = kH.xmin[X0] & ~15;
  static_assert(kH.xmin[X1 - 1] + KH - 1 - BASE < 64, "horizontal window exceeds 64 bytes");
  uint32_t w[16];
  const uint4* src = (const uint4*)(grow + BASE);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint4 v = src[i];
    w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
  }
#pragma unroll
  for (int q = 0; q < (X1 - X0) / 4; ++q) {
    uint32_t packed = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int xx = X0 + 4 * q + u;
      int acc = 1 << (A3C_PRECISION_BITS - 1);
#pragma unroll
      for (int x = 0; x < KH; ++x) {
        const int bi = kH.xmin[xx] + x - BASE;
        acc += (int)((w[bi >> 2] >> (8 * (bi & 3))) & 255u) * kH.k[xx][x];
      }
      packed |= (uint32_t)(acc >> A3C_PRECISION_BITS) << (8 * u);   // clip-free (taps_shift_only)
    }
    *(uint32_t*)(trow + X0 + 4 * q) = packed;
  }
}

// 4 u8 pixels (one dword, little-endian) -> 4 bf16 (exact: integers 0..255 are the upper half of
// their f32)
__device__ inline uint2 u8x4_to_bf16x4(uint32_t d) {
  const float f0 = (float)(d & 255u), f1 = (float)((d >> 8) & 255u);
  const float f2 = (float)((d >> 16) & 255u), f3 = (float)(d >> 24);
  return make_uint2(__builtin_amdgcn_perm(__float_as_uint(f1), __float_as_uint(f0), 0x07060302u),
                    __builtin_amdgcn_perm(__float_as_uint(f3), __float_as_uint(f2), 0x07060302u));
}

// ---------------------------------------------------------------------------------------
// Both resampling passes on the int8 matrix cores (v_mfma_i32_16x16x64_i8), bit-exact.
// Pillow's pass is out = (2^21 + sum_t k_t v_t) >> 22 over 8-bit v and 22-bit taps k (every
// output's taps sum to 2^22 - delta, delta in {0, 1}; taps_shift_only: no clip).  As an integer
// GEMM on signed bytes:
//   v = x' + 128 with x' = v ^ 0x80 (a signed byte),  k = 65536 d2 + 256 d1 + d0 in balanced
//   base-256 digits d in [-128, 127] (k < 2^22: d2 <= 33),
//   acc = ((((2^21 >> 16) + S2) << 8) + S1) << 8) - 128 delta + S0,   S_j = sum_t d_j x'_t
// (three MFMAs chained by Horner shift-adds: the constants ride in the C input and the adds,
// every partial an exact i32) = 2^21 + sum k x' - 128 delta, and since sum k v = sum k x' +
// 128 (2^22 - delta):  2^21 + sum k v = acc + 2^29, so
//   out = 128 + (acc >> 22)   (arithmetic shift),  and the output byte is (acc >> 22) ^ 0x80.
// Horizontal: C[y][X] = sum_k gray[y][hbase + k] H[k][X] over 14 x 6 tiles of 16 rows x 16 outputs,
// the K = 64 window of each output tile starting at a 16-aligned source column; the result is
// written transposed, tmpT[X][y] (4 consecutive y per lane: one dword).  Vertical: C[x][yy] =
// sum_k tmpT[x][vbase + k] V[k][yy] over 6 x 6 tiles, 4 consecutive x per lane: one dword of the
// output row.  The B fragments (the tap digits) are compile-time tables in constant memory.
// Lane layout of 16x16x64 i8 (tools/archive/probes/mfma_i8_layout.hip): lane l holds A[l&15][16(l>>4)+j],
// B[16(l>>4)+j][l&15], j = 0..15, and C[4(l>>4)+i][l&15], i = 0..3.
// ---------------------------------------------------------------------------------------
typedef int i32x4 __attribute__((ext_vector_type(4)));
constexpr int MT_N = 6;                 // 16-wide tiles over the 84 outputs of a pass (+12 pad)
constexpr int TMPT_LD = 224;            // tmpT row: 210 source rows padded to a multiple of 16
constexpr int H_MT = 14;                // 16-row tiles over the 210 source rows

struct MfmaTab {
  int8_t hb[MT_N][3][64][16];           // horizontal B fragments [n-tile][digit 2, 1, 0][lane][j]
  int8_t vb[MT_N][3][64][16];           // vertical
  int hbase[MT_N], vbase[MT_N];         // 16-aligned K-window starts (source column / row)
  int hc0[MT_N * 16], vc0[MT_N * 16];   // -128 delta per output (0 in the pad)
  bool ok;                              // every window covers its taps, digits in range
  template <int IN, int OUT>
  constexpr void fill(const Coef<IN, OUT>& c, int8_t (&b)[MT_N][3][64][16], int (&base)[MT_N], int (&c0)[MT_N * 16]) {
    constexpr int K = Coef<IN, OUT>::K;
    for (int nt = 0; nt < MT_N; ++nt) {
      base[nt] = c.xmin[16 * nt] / 16 * 16;
      for (int n = 0; n < 16; ++n) {
        const int o = 16 * nt + n;
        long sum = 0;
        if (o < OUT) {
          for (int t = 0; t < K; ++t) sum += c.k[o][t];
          if (c.xmin[o] + K - 1 - base[nt] >= 64 && c.k[o][K - 1] != 0) ok = false;
          for (int t = 0; t < K; ++t)
            if (c.k[o][t] != 0 && c.xmin[o] + t - base[nt] >= 64) ok = false;
        }
        c0[o] = o < OUT ? -128 * (int)((1L << A3C_PRECISION_BITS) - sum) : 0;
        for (int k = 0; k < 64; ++k) {
          const int t = base[nt] + k - (o < OUT ? c.xmin[o] : 0);
          const int w = (o < OUT && t >= 0 && t < K) ? c.k[o][t] : 0;
          const int d0 = ((w + 128) & 255) - 128, w1 = (w - d0) / 256;
          const int d1 = ((w1 + 128) & 255) - 128, d2 = (w1 - d1) / 256;
          if (d2 < -128 || d2 > 127) ok = false;
          const int lane = n + 16 * (k >> 4), j = k & 15;
          b[nt][0][lane][j] = (int8_t)d2;
          b[nt][1][lane][j] = (int8_t)d1;
          b[nt][2][lane][j] = (int8_t)d0;
        }
      }
    }
  }
  constexpr MfmaTab() : hb(), vb(), hbase(), vbase(), hc0(), vc0(), ok(true) {
    fill(kH, hb, hbase, hc0);
    fill(kV, vb, vbase, vc0);
  }
};
constexpr MfmaTab kTab{};
static_assert(kTab.ok, "resampling tap windows / digits");
__constant__ MfmaTab cTab = kTab;

// A wave's B fragments of one pass (its n-tile's three digit planes) and the lane's output
// correction: loaded once per pass, issued right behind the frame loads (so the luminance pass's
// waits for the frame cover them too) -- per-tile loads of the constant tables each exposed an L2
// round trip (a first build: the fused kernel 25.9 vs 24.9 us alone).
struct TapFrag {
  i32x4 b2, b1, b0;
  int base, c0;
};
__device__ inline TapFrag load_frag(const int8_t (&b)[MT_N][3][64][16], const int (&base)[MT_N], const int (&c0)[MT_N * 16],
                                    int nt, int lane) {
  TapFrag f;
  f.b2 = *(const i32x4*)b[nt][0][lane];
  f.b1 = *(const i32x4*)b[nt][1][lane];
  f.b0 = *(const i32x4*)b[nt][2][lane];
  f.base = base[nt];
  f.c0 = c0[16 * nt + (lane & 15)];
  return f;
}
// wave -> (n-tile, m-tiles [m0, m1)) of a pass with `mt` m-tiles: waves 0-3 own n-tiles 0-3 whole,
// n-tiles 4 and 5 are split between waves 4/6 and 5/7 -- each SIMD (waves s, s + 4) gets 1.5
// n-tiles' work; waves 8+ (1024-thread kernels) take none
struct PassPlan {
  int nt, m0, m1;
};
__device__ inline PassPlan pass_plan(int wid, int mt) {
  if (wid < 4) return {wid, 0, mt};
  if (wid >= 8) return {0, 0, 0};
  const int half = (mt + 1) / 2;
  return {4 + (wid & 1), wid < 6 ? 0 : half, wid < 6 ? half : mt};
}

// one 16x16 output tile of a pass: A = 16 bytes of the lane's source row at `a_src` (LDS);
// returns the lane's 4 output bytes
__device__ inline uint32_t resample_tile(const uint8_t* a_src, const TapFrag& f) {
  i32x4 a = *(const i32x4*)a_src;
  a ^= (i32x4){(int)0x80808080, (int)0x80808080, (int)0x80808080, (int)0x80808080};
  i32x4 acc = {32, 32, 32, 32};                                     // 2^21 >> 16
  acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, f.b2, acc, 0, 0, 0);
  acc = acc << 8;
  acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, f.b1, acc, 0, 0, 0);
  acc = (acc << 8) + f.c0;
  acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, f.b0, acc, 0, 0, 0);
  uint32_t packed = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) packed |= (((uint32_t)acc[i] >> 22) & 255u) << (8 * i);
  return packed ^ 0x80808080u;
}

// two independent tiles interleaved: each tile's three MFMAs form a dependent chain (Horner), so
// one chain alone waits out every MFMA's latency; two chains fill each other's gaps
__device__ inline void resample_tile2(const uint8_t* s0, const uint8_t* s1, const TapFrag& f, uint32_t& v0, uint32_t& v1) {
  const i32x4 flip = {(int)0x80808080, (int)0x80808080, (int)0x80808080, (int)0x80808080};
  const i32x4 a0 = *(const i32x4*)s0 ^ flip, a1 = *(const i32x4*)s1 ^ flip;
  i32x4 c0 = {32, 32, 32, 32}, c1 = {32, 32, 32, 32};
  c0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, f.b2, c0, 0, 0, 0);
  c1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1, f.b2, c1, 0, 0, 0);
  c0 = c0 << 8;
  c1 = c1 << 8;
  c0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, f.b1, c0, 0, 0, 0);
  c1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1, f.b1, c1, 0, 0, 0);
  c0 = (c0 << 8) + f.c0;
  c1 = (c1 << 8) + f.c0;
  c0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, f.b0, c0, 0, 0, 0);
  c1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1, f.b0, c1, 0, 0, 0);
  uint32_t p0 = 0, p1 = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    p0 |= (((uint32_t)c0[i] >> 22) & 255u) << (8 * i);
    p1 |= (((uint32_t)c1[i] >> 22) & 255u) << (8 * i);
  }
  v0 = p0 ^ 0x80808080u;
  v1 = p1 ^ 0x80808080u;
}

// horizontal pass: gray [210][160] -> tmpT [84][TMPT_LD] (transposed), tiles in pairs
__device__ inline void hpass_mfma(const uint8_t* __restrict__ gray, uint8_t* __restrict__ tmpT, const TapFrag& f,
                                  const PassPlan& p) {
  const int lane = threadIdx.x & 63, n = lane & 15, h = lane >> 4;
  const int X = 16 * p.nt + n;
  uint8_t* t = tmpT + X * TMPT_LD + 4 * h;
  const uint8_t* g = gray + f.base + 16 * h;
  int mt = p.m0;
  for (; mt + 1 < p.m1; mt += 2) {
    uint32_t v0, v1;
    resample_tile2(g + min(16 * mt + n, IH - 1) * IW, g + min(16 * mt + 16 + n, IH - 1) * IW, f, v0, v1);
    if (X < OW) {
      *(uint32_t*)(t + 16 * mt) = v0;
      *(uint32_t*)(t + 16 * mt + 16) = v1;
    }
  }
  if (mt < p.m1) {
    const uint32_t v = resample_tile(g + min(16 * mt + n, IH - 1) * IW, f);
    if (X < OW) *(uint32_t*)(t + 16 * mt) = v;
  }
}

// vertical pass: tmpT -> the 84x84 screen (out, HBM ring slot) and, for the fused conv, the
// same plane as bf16 in LDS
__device__ inline void vpass_mfma(const uint8_t* __restrict__ tmpT, uint8_t* __restrict__ out, uint16_t* lds_bf16,
                                  const TapFrag& f, const PassPlan& p) {
  const int lane = threadIdx.x & 63, n = lane & 15, h = lane >> 4;
  const int yy = 16 * p.nt + n;                            // n-tile: output rows, m-tile: columns
  const uint8_t* t = tmpT + f.base + 16 * h;
  auto put = [&](int mt, uint32_t v) {
    const int x0 = 16 * mt + 4 * h;
    if (yy < OH && x0 < OW) {
      st_act((uint32_t*)(out + yy * OW + x0), v);
      if (lds_bf16) *(uint2*)(lds_bf16 + yy * OW + x0) = u8x4_to_bf16x4(v);   // (fused conv12)
    }
  };
  int mt = p.m0;
  for (; mt + 1 < p.m1; mt += 2) {
    uint32_t v0, v1;
    resample_tile2(t + min(16 * mt + n, OW - 1) * TMPT_LD, t + min(16 * mt + 16 + n, OW - 1) * TMPT_LD, f, v0, v1);
    put(mt, v0);
    put(mt + 1, v1);
  }
  if (mt < p.m1) put(mt, resample_tile(t + min(16 * mt + n, OW - 1) * TMPT_LD, f));
}

// Whole-frame Environment.screen by one workgroup of NT threads (gray 210x160 and the
// transposed horizontal-pass image tmpT in LDS, SCREEN_FRAME_SMEM bytes); the RGB frame streams
// from HBM straight into registers (all of a thread's loads issued before any use), the
// luminance runs on the vector ALUs, both resampling passes on the int8 matrix cores (above).
// -DSCREEN_VALU: the vector-ALU resampling passes of rounds 1-4 (A/B builds).
#define SCREEN_KV_BYTES (84 * 8 * 4)
#ifdef SCREEN_VALU
#define SCREEN_FRAME_SMEM_NOKV (210 * 160 + 210 * 84 + 96)   // the tap table elsewhere (kvs_at)
#define SCREEN_FRAME_SMEM (SCREEN_FRAME_SMEM_NOKV + SCREEN_KV_BYTES)
#else
// gray | slack | tmpT | slack: each pass's last K window reads up to 64 bytes from its 16-aligned
// start, past the end of the last source row (gray row 209, tmpT row 83); the slack keeps those
// reads inside the allocation and off the region other waves write (their taps are zero, so the
// bytes read there never reach a result)
constexpr int SCREEN_SLACK = 64;
static_assert(kTab.hbase[MT_N - 1] + 64 <= IW + SCREEN_SLACK, "horizontal K window past gray's slack");
static_assert(kTab.vbase[MT_N - 1] + 64 <= TMPT_LD + SCREEN_SLACK, "vertical K window past tmpT's slack");
#define SCREEN_FRAME_SMEM_NOKV (210 * 160 + 64 + 84 * 224 + 64)
#define SCREEN_FRAME_SMEM SCREEN_FRAME_SMEM_NOKV
#endif

struct NoScreenMid {
  __device__ void operator()() const {}
};

// mid(): work run by every thread while its frame loads are in flight, before the luminance
// pass writes the scratch (it may use the first 51 KB of smem; it must not wait on vector memory)
template <int NT, typename Mid = NoScreenMid>
__device__ __attribute__((always_inline)) inline void screen_frame(const uint8_t* __restrict__ rgb, uint8_t* __restrict__ out, uint8_t* smem,
                                    uint64_t* dbg = nullptr, uint16_t* lds_bf16 = nullptr, Mid mid = Mid(),
                                    int* kvs_at = nullptr) {
  uint8_t* gray = smem;
#ifdef SCREEN_VALU
  uint8_t* tmp = smem + IH * IW;
#else
  uint8_t* tmp = smem + IH * IW + SCREEN_SLACK;
#endif
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  constexpr int NWV = NT / 64;
  constexpr int NUNIT = IH * IW / 4;                   // 8400 units of 4 pixels (12 bytes)
  constexpr int PER = (NUNIT + NT - 1) / NT;
#ifdef SCREEN_VALU
  // [yy][8]: 7 taps, xmin -- after the scratch, or at kvs_at (written after mid())
  int* kvs = kvs_at ? kvs_at : (int*)(tmp + IH * OW + 96);
  // the vertical-tap table's loads are issued first and written after mid(): loads retire in
  // order (vmcnt), so waiting for one issued behind the frame would wait for the whole frame
  constexpr int NKV = OH * 8, PKV = (NKV + NT - 1) / NT;
  int kv[PKV];
#pragma unroll
  for (int j = 0; j < PKV; ++j) {
    const int i = min(tid + NT * j, NKV - 1);
    kv[j] = (i & 7) < KV ? cV.k[i >> 3][i & 7] : cV.xmin[i >> 3];
  }
#else
  (void)kvs_at;
#endif
  uint3 r[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const uint32_t* s = (const uint32_t*)(rgb + 12 * min(tid + NT * j, NUNIT - 1));
    r[j] = make_uint3(s[0], s[1], s[2]);
  }
  if (dbg && tid == 0) dbg[14] = __builtin_readcyclecounter();
  mid();
  if (dbg && tid == 0) dbg[15] = __builtin_readcyclecounter();
#ifdef SCREEN_VALU
#pragma unroll
  for (int j = 0; j < PKV; ++j)
    if (tid + NT * j < NKV) kvs[tid + NT * j] = kv[j];
#else
  // the wave's tap fragments of both passes, behind the frame loads (retire with them)
  const PassPlan hp = pass_plan(wid, H_MT), vp = pass_plan(wid, MT_N);
  const TapFrag hf = load_frag(cTab.hb, cTab.hbase, cTab.hc0, hp.nt, lane);
  const TapFrag vf = load_frag(cTab.vb, cTab.vbase, cTab.vc0, vp.nt, lane);
#endif
  if (dbg && tid == 0) dbg[4] = __builtin_readcyclecounter() + (r[0].x & 0);   // first unit landed
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int u = tid + NT * j;
    if (u < NUNIT) *(uint32_t*)(gray + 4 * u) = lum4(r[j].x, r[j].y, r[j].z);
  }
  if (dbg && tid == 0) dbg[5] = __builtin_readcyclecounter();
  __syncthreads();
  if (dbg && tid == 0) dbg[6] = __builtin_readcyclecounter();
#ifndef SCREEN_VALU
  hpass_mfma(gray, tmp, hf, hp);                       // tmp = tmpT [84][224]
  __syncthreads();
  if (dbg && tid == 0) dbg[7] = __builtin_readcyclecounter();
  vpass_mfma(tmp, out, lds_bf16, vf, vp);
#else
  for (int task = wid; task < 16; task += NWV) {
    const int seg = task & 3, rr = (task >> 2) * 64 + lane;
    if (rr < IH) {
      const uint8_t* g = gray + rr * IW;
      uint8_t* t = tmp + rr * OW;
      if (seg == 0) hpass_seg<0>(g, t);
      else if (seg == 1) hpass_seg<1>(g, t);
      else if (seg == 2) hpass_seg<2>(g, t);
      else hpass_seg<3>(g, t);
    }
  }
  __syncthreads();
  if (dbg && tid == 0) dbg[7] = __builtin_readcyclecounter();
  const int sub = lane / (OW / 4), cq = lane - sub * (OW / 4);
  for (int task = wid; task < OH / 3; task += NWV) {
    if (sub < 3) {
      const int yy = 3 * task + sub;
      const int* kc = kvs + yy * 8;
      const int b0 = kc[7];
      int acc[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] = 1 << (A3C_PRECISION_BITS - 1);
#pragma unroll
      for (int y = 0; y < KV; ++y) {
        const int ry = min(b0 + y, IH - 1);
        const uint32_t q = *(const uint32_t*)(tmp + ry * OW + 4 * cq);
        const int k = kc[y];
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[c] += (int)((q >> (8 * c)) & 255u) * k;
      }
      uint32_t packed = 0;
#pragma unroll
      for (int c = 0; c < 4; ++c) packed |= (uint32_t)(acc[c] >> A3C_PRECISION_BITS) << (8 * c);
      st_act((uint32_t*)(out + yy * OW + 4 * cq), packed);
      if (lds_bf16) *(uint2*)(lds_bf16 + yy * OW + 4 * cq) = u8x4_to_bf16x4(packed);   // (fused conv12)
    }
  }
#endif
  if (dbg) {
    __syncthreads();
    if (tid == 0) dbg[8] = __builtin_readcyclecounter();
  }
}

// Measurement mode M2 (a3c_engine_config.frame84): the pool frame is already an 84x84 u8 screen,
// so the "screen" is a copy into the ring slot (and, for the fused conv, the bf16 plane in LDS).
// mid() runs while the loads are in flight, as in screen_frame.
template <int NT, typename Mid = NoScreenMid>
__device__ inline void copy_frame84(const uint8_t* __restrict__ src, uint8_t* __restrict__ out,
                                    uint16_t* lds_bf16 = nullptr, Mid mid = Mid()) {
  constexpr int NCH = OH * OW / 16;                     // 441 chunks of 16 pixels
  constexpr int PER = (NCH + NT - 1) / NT;
  const int tid = threadIdx.x;
  uint4 v[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) v[j] = ((const uint4*)src)[min(tid + NT * j, NCH - 1)];
  mid();
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int i = tid + NT * j;
    if (i < NCH) {
      ((uint4*)out)[i] = v[j];
      if (lds_bf16) {
        uint4* d = (uint4*)(lds_bf16 + 16 * i);
        const uint2 a0 = u8x4_to_bf16x4(v[j].x), a1 = u8x4_to_bf16x4(v[j].y);
        const uint2 a2 = u8x4_to_bf16x4(v[j].z), a3 = u8x4_to_bf16x4(v[j].w);
        d[0] = make_uint4(a0.x, a0.y, a1.x, a1.y);
        d[1] = make_uint4(a2.x, a2.y, a3.x, a3.y);
      }
    }
  }
}

template <int ROWS>
struct Smem {
  static constexpr int SR = max_src_rows<ROWS>();
  static constexpr int RAW = SR * IW * 3;                      // multiple of 16 (IW*3 = 480)
  static constexpr int GRAY = SR * IW;                         // multiple of 16
  static constexpr int TMP = ((SR * OW + 15) / 16) * 16;
  static constexpr int BYTES = RAW + GRAY + TMP;
};

// One workgroup (256 threads) produces output rows [band*ROWS, band*ROWS + ROWS) of one frame.
template <int ROWS>
__device__ inline void screen_band(const uint8_t* __restrict__ rgb, uint8_t* __restrict__ out, int band,
                                   uint8_t* smem) {
  using S = Smem<ROWS>;
  const int tid = threadIdx.x;
  const int yy0 = band * ROWS;
  const int rows = (yy0 + ROWS <= OH) ? ROWS : OH - yy0;
  const int y0 = cV.xmin[yy0];
  const int y1 = cV.xmin[yy0 + rows - 1] + cV.cnt[yy0 + rows - 1];
  uint8_t* raw = smem;
  uint8_t* gray = smem + S::RAW;
  uint8_t* tmp = gray + S::GRAY;

  // ---- stage source rows [y0, y1): 16-byte coalesced loads, all issued before any store ----
  const uint4* s4 = (const uint4*)(rgb + y0 * IW * 3);
  const int n16 = (y1 - y0) * (IW * 3 / 16);
  constexpr int PER = (S::RAW / 16 + 255) / 256;
  uint4 r[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) r[j] = s4[min(tid + 256 * j, n16 - 1)];   // clamped: always a valid load
#pragma unroll
  for (int j = 0; j < PER; ++j)
    if (tid + 256 * j < n16) ((uint4*)raw)[tid + 256 * j] = r[j];
  __syncthreads();

  // ---- luminance, 16 pixels (48 B) per thread-iteration ----
  const int nunit = (y1 - y0) * (IW / 16);
  for (int u = tid; u < nunit; u += 256) {
    const uint4* r4 = (const uint4*)(raw + 48 * u);
    *(uint4*)(gray + 16 * u) = lum16(r4[0], r4[1], r4[2]);
  }
  __syncthreads();

  // ---- horizontal pass: thread -> (column, row phase); the column's taps stay in registers ----
  const int srows = y1 - y0;
  if (tid < 3 * OW) {
    const int xx = tid % OW, rp = tid / OW;
    const int x0 = cH.xmin[xx];
    int kk[KH], off[KH];
#pragma unroll
    for (int x = 0; x < KH; ++x) {
      kk[x] = cH.k[xx][x];
      off[x] = min(x0 + x, IW - 1);          // weight is 0 past the row's count
    }
    for (int rr = rp; rr < srows; rr += 3) {
      const uint8_t* s = gray + rr * IW;
      int acc = 1 << (A3C_PRECISION_BITS - 1);
#pragma unroll
      for (int x = 0; x < KH; ++x) acc += (int)s[off[x]] * kk[x];
      tmp[rr * OW + xx] = a3c_clip8(acc);
    }
  }
  __syncthreads();

  // ---- vertical pass for the band ----
  if (tid < 3 * OW) {
    const int xx = tid % OW, rp = tid / OW;
    for (int yy = rp; yy < rows; yy += 3) {
      const int Y = yy0 + yy;
      const int b0 = cV.xmin[Y] - y0;
      int acc = 1 << (A3C_PRECISION_BITS - 1);
#pragma unroll
      for (int y = 0; y < KV; ++y) {
        const int ry = min(b0 + y, srows - 1);
        acc += (int)tmp[ry * OW + xx] * cV.k[Y][y];
      }
      out[Y * OW + xx] = a3c_clip8(acc);
    }
  }
}

}  // namespace atari

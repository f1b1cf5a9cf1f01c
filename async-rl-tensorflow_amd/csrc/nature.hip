// The "nature" trunk of the reference's A3C Network (network.py:30-42: conv 8x8/4 32, conv 4x4/2
// 64, conv 3x3/1 64, fc 3136 -> 512, all ReLU; heads network.py:60-79) on gfx950 matrix cores.
//
//  k_nat_gemm<MODE, BN>  one implicit-GEMM tile kernel for every convolution pass, operands gathered
//                        straight from the NHWC activations (no im2col buffer in HBM), staged in LDS
//                        as 16-deep K slices with a register prefetch of the next slice, and reduced
//                        on v_mfma_f32_32x32x2f32 (exact fp32 products, fp32 accumulation: the
//                        reference computes in fp32).  4 waves, each a 32x32 block of a
//                        64x64 (BN = 64) or 128x32 (BN = 32: the 32-channel layers) tile.
//    NG_FWD1  conv1: rows = (sample, output pixel), K = (kh, kw, cin) in TF order, A read from the
//             u8 frame ring (the 4 history planes of the state, history.py:13-24), x / 255 applied to
//             the accumulator (agent.py:226 / network.py:46); + bias, ReLU
//    NG_FWD   conv2, conv3 from the fp32 NHWC output of the layer below; + bias, ReLU
//    NG_DX    dX = col2im(dY W^T) * (X > 0), one stride parity class (py, px) per grid z: the output
//             pixels y = S i + py, x = S j + px are reached only by taps kh = py + S th, kw = px + S tw,
//             so K = (th, tw, cout) holds only real taps (conv2: 2x2x64 instead of 4x4x64)
//    NG_DW    dW[k][cout] = sum over (sample, pixel) of patch(k) dY, the reduction split over grid z
//             into per-split slabs (+ the column sums of dY: the bias gradient), folded in a fixed
//             order by k_slab_group + k_finalize (net_bwd.hip) -- deterministic, no atomics
//    NG_DW1   the same for conv1 (patches from the u8 ring; the 1/255 is the finalize's scale)
//  fc 3136 -> 512 and its backward: gemm.hip (split-K slabs with the bias + ReLU epilogue; the
//  weight gradient in-workgroup split-K).  Head (k_nat_head): head_row<512> + the action draw and the
//  fused env act of net_head.h; head backward: k_head_bwd<512> (net_bwd.hip).
#include "nature.h"
#include "net_bwd.h"
#include "net_head.h"

enum { NG_FWD1 = 0, NG_FWD, NG_DX, NG_DW1, NG_DW };

// conv layer geometry (NHWC input H x W x C, TF weights [KH][KW][C][OC], VALID, stride S)
template <int LAYER> struct NG;
template <> struct NG<1> { static constexpr int H = IMG, W = IMG, C = HIST, KH = 8, KW = 8, S = 4, OH = NT1_O, OW = NT1_O, OC = NT1_N; };
template <> struct NG<2> { static constexpr int H = NT1_O, W = NT1_O, C = NT1_N, KH = 4, KW = 4, S = 2, OH = NT2_O, OW = NT2_O, OC = NT2_N; };
template <> struct NG<3> { static constexpr int H = NT2_O, W = NT2_O, C = NT2_N, KH = 3, KW = 3, S = 1, OH = NT3_O, OW = NT3_O, OC = NT3_N; };
// the fc 3136 -> 512 (network.py:41-42) as a 1x1 convolution of a 1x1 "image": the same tile
// kernels then run its forward, weight gradient (NG_DW) and input gradient with the l3 ReLU mask (NG_DX)
template <> struct NG<4> { static constexpr int H = 1, W = 1, C = NT_FLAT, KH = 1, KW = 1, S = 1, OH = 1, OW = 1, OC = NT_FC; };

struct NatGemm {
  StateAddr sa;        // NG_FWD1 / NG_DW1: the u8 state planes of sample b (b = t E + e)
  const float* X;      // fp32 NHWC input activation [B][H][W][C] (NG_FWD, NG_DW; NG_DX: its ReLU mask)
  const float* Wt;     // TF weights [KH][KW][C][OC]
  const float* bias;   // NG_FWD*: [OC]
  const float* dY;     // NG_DX, NG_DW*: [B][OH][OW][OC]
  float* Y;            // NG_FWD*: [B][OH][OW][OC]; NG_DX: dX [B][H][W][C]
  float* slab;         // NG_DW*: [nsplit][M][N]
  float* colsum;       // NG_DW*: [nsplit][N]
  int M, N, K;         // NG_DX: M per parity class; NG_DW*: M = KH KW C, N = OC, K = B OH OW (reduction)
  int kchunk;          // NG_DW*: reduction rows per split (a multiple of the K slice); NG_FWD: > 0 splits K
                       // over grid z into slab partials (the fold applies bias + ReLU)
  float scale;         // NG_FWD1: 1/255
  int xcd;             // NG_DW*, NG_DX: XCD-grouped tile order (nat_tile_of)
};

// The dispatcher deals workgroups round-robin over the 8 XCDs (linear id % 8), each with its own
// L2.  The workgroups that read the same operands -- the m-tiles of one reduction chunk (dW: the
// same dY rows and overlapping patches), the stride-parity classes of one m-tile (dX: the same dY
// rows) -- would land on 8 different XCDs and each fetch them from HBM; here a group of them takes
// consecutive ids of one XCD instead (grid x extent 1: id = y + Y z).
template <int MODE>
__device__ inline void nat_tile_of(int xcd, int& by, int& bz) {
  by = (int)blockIdx.y; bz = (int)blockIdx.z;
  if (!xcd || gridDim.x != 1 || MODE == NG_FWD1 || MODE == NG_FWD) return;
  constexpr bool DWM = MODE == NG_DW || MODE == NG_DW1;
  const int G = DWM ? (int)gridDim.z : (int)gridDim.y;     // groups sharing data
  const int S = DWM ? (int)gridDim.y : (int)gridDim.z;     // workgroups per group
  const int L = by + (int)gridDim.y * bz;
  const int full = G / 8 * 8;
  int g, m;
  if (L < full * S) {
    const int blk = L / (8 * S), rem = L - blk * 8 * S;
    m = rem / 8; g = blk * 8 + rem % 8;
  } else {
    const int cl = G - full, rem = L - full * S;
    m = rem / cl; g = full + rem % cl;
  }
  if (DWM) { bz = g; by = m; } else { by = g; bz = m; }
}

// the frame-ring planes of sample b = t E + e without 64-bit divisions: slot0 = the ring slot of
// plane 0 of t = 0, reduced once per launch
struct RingRows {
  const uint8_t* base;
  int64_t env_stride, plane_bytes;
  int E, R, slot0;
  uint64_t emagic;     // ceil(2^40 / E): t = b E^-1 by a multiply (b E < 2^40)
  __device__ void init(const StateAddr& sa, int64_t tau0) {
    base = sa.base; env_stride = sa.env_stride; plane_bytes = sa.plane_bytes; E = sa.E; R = sa.R;
    emagic = ((1ull << 40) + (uint64_t)E - 1) / (uint64_t)E;
    int64_t s0 = (tau0 + sa.tau_offset - (sa.L - 1)) % sa.R;
    slot0 = (int)(s0 < 0 ? s0 + sa.R : s0);
  }
  __device__ int step_of(int b) const { return (int)(((uint64_t)b * emagic) >> 40); }
  __device__ const uint8_t* plane(int e, int t, int c) const {
    int s = slot0 + t + c;
    while (s >= R) s -= R;
    return base + e * env_stride + s * plane_bytes;
  }
};

// One tile of an implicit GEMM on v_mfma_f32_32x32x2f32: 32-deep K slices, double-buffered in LDS
// (one barrier per slice), the next slice's operands loaded into registers under the current
// slice's 16 MFMAs per wave.  Geometry at compile time (every index division by a constant).
template <int MODE, int LAYER, int BN>
__global__ void __launch_bounds__(256) k_nat_gemm(NatGemm a) {
  using G = NG<LAYER>;
  constexpr int BM = 4096 / BN, BK = 32, LP = 4;
  constexpr int WN = BN / 32;                                   // waves along n
  constexpr bool A_KC = MODE == NG_FWD1 || MODE == NG_FWD || MODE == NG_DX;   // A quads along k
  constexpr bool B_NC = MODE != NG_DX;                           // B quads along n
  constexpr bool DW = MODE == NG_DW || MODE == NG_DW1;
  constexpr bool U8 = MODE == NG_FWD1 || MODE == NG_DW1;
  constexpr int AQ = BM * BK / 4 / 256;                          // A quads per thread (2 or 4)
  constexpr int BQ = BN * BK / 4 / 256;                          // B quads per thread (2 or 1)
  constexpr int P = G::OH * G::OW;
  constexpr int TW = G::KW / G::S;                               // NG_DX taps per class along x
  constexpr int NI = G::H / G::S, NJ = G::W / G::S;              // NG_DX class grid
  static_assert(MODE != NG_DX || (G::H % G::S == 0 && G::KH % G::S == 0), "parity classes");
  static_assert(!U8 || G::C == 4, "u8 planes: the 4 history frames");
  static_assert(P > BK, "one sample wrap per slice");
  __shared__ __attribute__((aligned(16))) float As[2][BK][BM + LP];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK][BN + LP];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  int by, bz;
  nat_tile_of<MODE>(a.xcd, by, bz);
  const int m0 = by * BM, n0 = blockIdx.x * BN;
  const bool split = DW || (MODE == NG_FWD && a.kchunk > 0);
  const int kbeg = split ? bz * a.kchunk : 0;
  const int kend = split ? min(a.K, kbeg + a.kchunk) : a.K;
  const int py = MODE == NG_DX ? bz / G::S : 0, px = MODE == NG_DX ? bz % G::S : 0;
  RingRows ring;
  if constexpr (U8) ring.init(a.sa, a.sa.tau_ptr ? *a.sa.tau_ptr : 0);

  // ---- per-thread operand coordinates ----
  int ar[AQ], ac[AQ];          // A_KC: row m (tile-local), k offset; else: reduction row, m offset
  bool aval[AQ];
  int64_t abase[AQ];           // NG_FWD: X offset of the patch origin; NG_DX: sample b
  int ai[AQ], aj[AQ];          // NG_DX: class grid position; NG_FWD1: pixel origin (y0, x0)
  const uint8_t* apl[AQ][4];   // NG_FWD1: the sample's 4 planes (ring slots wrap: no common stride)
  int mk[AQ][3];               // DW: (kh, kw, c0) of the thread's m quad
#pragma unroll
  for (int i = 0; i < AQ; ++i) {
    const int q = tid + 256 * i;
    if constexpr (A_KC) { ar[i] = q >> 3; ac[i] = (q & 7) * 4; }
    else { ar[i] = q / (BM / 4); ac[i] = (q % (BM / 4)) * 4; }
    abase[i] = 0; ai[i] = aj[i] = 0;
    if constexpr (A_KC) {
      const int m = m0 + ar[i];
      aval[i] = m < a.M;
      const int mm = aval[i] ? m : 0;
      if constexpr (MODE == NG_DX) {
        const int b = mm / (NI * NJ), r = mm - b * (NI * NJ);
        abase[i] = b; ai[i] = r / NJ; aj[i] = r - (r / NJ) * NJ;
      } else {
        const int b = mm / P, pos = mm - b * P, oy = pos / G::OW, ox = pos - oy * G::OW;
        if constexpr (MODE == NG_FWD1) {
          const int t = b / ring.E, e = b - t * ring.E;
#pragma unroll
          for (int cc = 0; cc < 4; ++cc) apl[i][cc] = ring.plane(e, t, cc);
          ai[i] = oy * G::S; aj[i] = ox * G::S;
        } else {
          abase[i] = (((int64_t)b * G::H + oy * G::S) * G::W + ox * G::S) * G::C;
        }
      }
    } else {
      const int m = m0 + ac[i];
      aval[i] = m < a.M;
      const int mm = aval[i] ? m : 0;
      if constexpr (U8) {                  // conv1: m = (cin, kh, kw), a quad = kw 4j..4j+3 of plane cin
        mk[i][0] = (mm >> 3) & 7; mk[i][1] = mm & 7; mk[i][2] = mm >> 6;
      } else {                             // TF order m = (kh KW + kw) C + c, a quad = 4 channels
        mk[i][0] = mm / (G::KW * G::C);
        mk[i][1] = (mm / G::C) % G::KW;
        mk[i][2] = mm % G::C;
      }
    }
  }
  int br[BQ], bc[BQ];          // B_NC: k row, n offset; else: n row, k offset
#pragma unroll
  for (int j = 0; j < BQ; ++j) {
    const int q = tid + 256 * j;
    if constexpr (B_NC) { br[j] = q / (BN / 4); bc[j] = (q % (BN / 4)) * 4; }
    else { br[j] = q >> 3; bc[j] = (q & 7) * 4; }
  }

  // A quad i of the slice at k0
  auto load_a = [&](int i, int k0) -> f32x4 {
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if constexpr (A_KC) {
      const int k = k0 + ac[i];
      if (!aval[i] || k >= kend) return v;
      if constexpr (MODE == NG_FWD1) {     // conv1's K order (cin, kh, kw): kw 4j..4j+3 of one plane, one dword
        const int cc = k >> 6, kh = (k >> 3) & 7, kw = k & 7;
        const uint32_t d = *(const uint32_t*)(apl[i][cc] + (ai[i] + kh) * IMG + aj[i] + kw);
        v[0] = (float)(d & 255u); v[1] = (float)((d >> 8) & 255u); v[2] = (float)((d >> 16) & 255u); v[3] = (float)(d >> 24);
      } else if constexpr (MODE == NG_FWD) {
        const int kh = k / (G::KW * G::C), rem = k - kh * (G::KW * G::C), kw = rem / G::C, c0 = rem - kw * G::C;
        v = *(const f32x4*)(a.X + abase[i] + (kh * G::W + kw) * G::C + c0);
      } else {                                                     // NG_DX: k = (th TW + tw) OC + oc
        const int th = k / (TW * G::OC), rem = k - th * (TW * G::OC), tw = rem / G::OC, oc0 = rem - tw * G::OC;
        const int oy = ai[i] - th, ox = aj[i] - tw;
        if (oy >= 0 && oy < G::OH && ox >= 0 && ox < G::OW)
          v = *(const f32x4*)(a.dY + ((abase[i] * G::OH + oy) * G::OW + ox) * G::OC + oc0);
      }
    } else {                                                       // DW: reduction row r, m quad
      const int r = k0 + ar[i];
      if (!aval[i] || r >= kend) return v;
      const int b = r / P, pos = r - b * P, oy = pos / G::OW, ox = pos - oy * G::OW;
      const int y = oy * G::S + mk[i][0], x = ox * G::S + mk[i][1];
      if constexpr (MODE == NG_DW1) {
        const int t = ring.step_of(b);
        const uint32_t d = *(const uint32_t*)(ring.plane(b - t * ring.E, t, mk[i][2]) + y * IMG + x);
        v[0] = (float)(d & 255u); v[1] = (float)((d >> 8) & 255u); v[2] = (float)((d >> 16) & 255u); v[3] = (float)(d >> 24);
      } else {
        v = *(const f32x4*)(a.X + (((int64_t)b * G::H + y) * G::W + x) * G::C + mk[i][2]);
      }
    }
    return v;
  };
  auto load_b = [&](int j, int k0) -> f32x4 {
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if constexpr (B_NC) {
      const int k = k0 + br[j], n = n0 + bc[j];
      if (k >= kend || n >= a.N) return v;
      const int row = MODE == NG_FWD1 ? ((((k >> 3) & 7) * 8 + (k & 7)) * 4 + (k >> 6)) : k;   // conv1: TF row of k
      v = DW ? *(const f32x4*)(a.dY + (int64_t)k * G::OC + n) : *(const f32x4*)(a.Wt + (int64_t)row * G::OC + n);
    } else {                                                       // NG_DX: B(k, c) = W[kh][kw][c][oc..]
      const int n = n0 + br[j], k = k0 + bc[j];
      if (n >= a.N || k >= kend) return v;
      const int th = k / (TW * G::OC), rem = k - th * (TW * G::OC), tw = rem / G::OC, oc0 = rem - tw * G::OC;
      const int kh = py + G::S * th, kw = px + G::S * tw;
      v = *(const f32x4*)(a.Wt + (((int64_t)kh * G::KW + kw) * G::C + n) * G::OC + oc0);
    }
    return v;
  };
  auto store = [&](int buf, const f32x4 (&ra)[AQ], const f32x4 (&rbv)[BQ]) {
#pragma unroll
    for (int i = 0; i < AQ; ++i) {
      if constexpr (A_KC) {
#pragma unroll
        for (int c = 0; c < 4; ++c) As[buf][ac[i] + c][ar[i]] = ra[i][c];
      } else {
        *(f32x4*)&As[buf][ar[i]][ac[i]] = ra[i];
      }
    }
#pragma unroll
    for (int j = 0; j < BQ; ++j) {
      if constexpr (B_NC) {
        *(f32x4*)&Bs[buf][br[j]][bc[j]] = rbv[j];
      } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) Bs[buf][bc[j] + c][br[j]] = rbv[j][c];
      }
    }
  };

  f32x16 acc = {};
  float csum = 0.f;
  const bool do_colsum = DW && a.colsum && by == 0 && tid < BN;
  const int kh = lane >> 5, c = lane & 31;
  auto load_all = [&](int k0, f32x4 (&ra)[AQ], f32x4 (&rbv)[BQ]) {
#if defined(NAT_ABL) && NAT_ABL == 2      // measurement only: no operand loads
    for (int i = 0; i < AQ; ++i) ra[i] = (f32x4){(float)k0, 1.f, 2.f, 3.f};
    for (int j = 0; j < BQ; ++j) rbv[j] = (f32x4){(float)k0, 1.f, 2.f, 3.f};
    return;
#endif
#pragma unroll
    for (int i = 0; i < AQ; ++i) ra[i] = load_a(i, k0);
#pragma unroll
    for (int j = 0; j < BQ; ++j) rbv[j] = load_b(j, k0);
  };
  auto compute = [&](int buf) {
    if (do_colsum) {
#pragma unroll
      for (int k = 0; k < BK; ++k) csum += Bs[buf][k][tid];
    }
#if defined(NAT_ABL) && NAT_ABL == 1      // measurement only: LDS operand reads, no MFMA
    for (int kk = 0; kk < BK / 2; ++kk) acc[kk] += As[buf][2 * kk + kh][wm * 32 + c] * Bs[buf][2 * kk + kh][wn * 32 + c];
    return;
#endif
#pragma unroll
    for (int kk = 0; kk < BK / 2; ++kk)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(As[buf][2 * kk + kh][wm * 32 + c], Bs[buf][2 * kk + kh][wn * 32 + c],
                                                 acc, 0, 0, 0);
  };
  if constexpr (DW) {
    // the weight-gradient passes (long reductions, ~110-120 VGPRs anyway): two register sets keep
    // two slices in flight beyond the one in LDS, slice s loading while slices s-2 and s-1 compute
    // (measured: conv1/2/3 dW 188/91/66 -> 175/87/63 us; the forward passes lose occupancy with it)
    f32x4 ra0[AQ], rb0[BQ], ra1[AQ], rb1[BQ];
    load_all(kbeg, ra0, rb0);
    store(0, ra0, rb0);
    if (kbeg + BK < kend) load_all(kbeg + BK, ra1, rb1);
    if (kbeg + 2 * BK < kend) load_all(kbeg + 2 * BK, ra0, rb0);
    __syncthreads();
    for (int k0 = kbeg; k0 < kend; k0 += 2 * BK) {
      // LDS buffer 0: slice k0; set 1: slice k0 + BK; set 0: slice k0 + 2 BK
      compute(0);
      if (k0 + BK < kend) {
        store(1, ra1, rb1);
        if (k0 + 3 * BK < kend) load_all(k0 + 3 * BK, ra1, rb1);
      }
      __syncthreads();
      if (k0 + BK >= kend) break;
      compute(1);
      if (k0 + 2 * BK < kend) {
        store(0, ra0, rb0);
        if (k0 + 4 * BK < kend) load_all(k0 + 4 * BK, ra0, rb0);
      }
      __syncthreads();
    }
  } else {
    // one register set: the next slice loads under this slice's MFMAs
    f32x4 ra[AQ], rbv[BQ];
    load_all(kbeg, ra, rbv);
    store(0, ra, rbv);
    __syncthreads();
    int buf = 0;
    for (int k0 = kbeg; k0 < kend; k0 += BK) {
      const bool more = k0 + BK < kend;
      if (more) load_all(k0 + BK, ra, rbv);
      compute(buf);
      if (more) store(buf ^ 1, ra, rbv);        // (the other buffer: last read before the previous barrier)
      __syncthreads();
      buf ^= 1;
    }
  }

  const int col = n0 + wn * 32 + (lane & 31);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (row >= a.M || col >= a.N) continue;
    float v = acc[r];
    if constexpr (MODE == NG_FWD1 || MODE == NG_FWD) {
      if (MODE == NG_FWD && split) {            // a K-split partial: the fold adds bias + ReLU
        a.slab[((int64_t)bz * a.M + row) * a.N + col] = v;
        continue;
      }
      v = fmaxf((MODE == NG_FWD1 ? v * a.scale : v) + a.bias[col], 0.f);
      a.Y[(int64_t)row * a.N + col] = v;
    } else if constexpr (MODE == NG_DX) {
      const int b = row / (NI * NJ), rr = row - b * (NI * NJ), i = rr / NJ, j = rr - (rr / NJ) * NJ;
      const int64_t o = (((int64_t)b * G::H + py + G::S * i) * G::W + px + G::S * j) * G::C + col;
      a.Y[o] = a.X[o] > 0.f ? v : 0.f;
    } else {
      // conv1's m = (cin, kh, kw) -> the TF row (kh 8 + kw) 4 + cin of dW1 [8][8][4][32]
      const int trow = MODE == NG_DW1 ? ((((row >> 3) & 7) * 8 + (row & 7)) * 4 + (row >> 6)) : row;
      a.slab[((int64_t)bz * a.M + trow) * a.N + col] = v;
    }
  }
  if (do_colsum && n0 + tid < a.N) a.colsum[(int64_t)bz * a.N + n0 + tid] = csum;
}

static int nat_xcd() {
  static const int v = (int)A3C_AB_KNOB("A3C_NAT_XCD", 1);   // A/B: 0 = the hardware tile order
  return v;
}
template <int MODE, int LAYER, int BN>
static int nat_go(NatGemm a, unsigned gz, hipStream_t s) {
  constexpr int BM = 4096 / BN;
  if (a.M <= 0 || a.N <= 0) return 0;
  a.xcd = nat_xcd();
  const dim3 grid((unsigned)((a.N + BN - 1) / BN), (unsigned)((a.M + BM - 1) / BM), gz);
  hipLaunchKernelGGL((k_nat_gemm<MODE, LAYER, BN>), grid, dim3(256), 0, s, a);
  A3C_CHECK(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------------------------------
// The same passes on the bf16 matrix cores (v_mfma_f32_32x32x16_bf16, 32 cycles per 32x32x16 vs 512
// for the 32x32x2f32 chain of the same depth).  Each fp32 operand is split at the LDS store into
// three round-to-nearest bf16 terms x = hi + mid + lo (v_cvt_pk_bf16_f32; exact to ~2^-24 relative)
// and the tile sums the six products hi.hi, hi.mid, mid.hi, mid.mid, hi.lo, lo.hi (the dropped
// ones are below 2^-24 of the product): fp32-class results, as the NIPS conv2 (net_fwd.hip).
// conv1's dW (TA = 1): a u8 pixel is exact in one bf16 term, three products.
// LDS holds the terms k-contiguous ([row][k], 40 bf16 a row) for the MFMA's 8-deep lane fragments;
// operands that arrive along rows (the dW passes' A and B, the forward's weights) are loaded as
// quad pairs at k and k + 1 and stored as packed (k, k + 1) dwords.
// ---------------------------------------------------------------------------------------
typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));

// NT terms (1 or 3) of the pair (x0, x1), each a packed bf16x2 dword
template <int NT>
__device__ inline void nat_split2(float x0, float x1, uint32_t (&o)[NT]) {
  const f32x2v v = {x0, x1};
  const bf16x2v h = __builtin_convertvector(v, bf16x2v);
  o[0] = __builtin_bit_cast(uint32_t, h);
  if constexpr (NT == 3) {
    const f32x2v r1 = v - __builtin_convertvector(h, f32x2v);
    const bf16x2v m = __builtin_convertvector(r1, bf16x2v);
    const f32x2v r2 = r1 - __builtin_convertvector(m, f32x2v);
    o[1] = __builtin_bit_cast(uint32_t, m);
    o[2] = __builtin_bit_cast(uint32_t, __builtin_convertvector(r2, bf16x2v));
  }
}

template <int MODE, int LAYER, int BN, int TA, int NBUF, int PF>
__global__ void __launch_bounds__(256) k_nat_gemm_bf(NatGemm a) {
  using G = NG<LAYER>;
  constexpr int BM = 4096 / BN, BK = 32, LD = 40;
  constexpr int WN = BN / 32;
  constexpr bool A_KC = MODE == NG_FWD || MODE == NG_DX;         // A quads along k (else pairs of row quads)
  constexpr bool B_NC = MODE != NG_DX;                           // B quads along n: pairs of row quads
  constexpr bool DW = MODE == NG_DW || MODE == NG_DW1;
  constexpr bool U8 = MODE == NG_DW1;
  static_assert(MODE != NG_FWD1, "conv1 forward: k_nat_conv1_bf");
  static_assert(TA == 3 || (TA == 1 && U8), "one A term only for the exact u8 pixels");
  constexpr int AQ = BM * BK / 4 / 256;                          // A quads per thread (2 or 4)
  constexpr int BQ0 = BN * BK / 4 / 256;
  constexpr int BQ = B_NC && BQ0 < 2 ? 2 : BQ0;                  // B quads per thread (pairs: >= 2)
  constexpr int BPAIRS = BN * BK / 8;                            // B_NC: quad pairs per slice
  constexpr int P = G::OH * G::OW;
  constexpr int TW = G::KW / G::S;
  constexpr int NI = G::H / G::S, NJ = G::W / G::S;
  static_assert(MODE != NG_DX || (G::H % G::S == 0 && G::KH % G::S == 0), "parity classes");
  static_assert(!U8 || G::C == 4, "u8 planes: the 4 history frames");
  static_assert((BM / 4) % 4 == 0 && (BN / 4) % 4 == 0, "pair mapping: 4 quads of a row per lane group");
  __shared__ __attribute__((aligned(16))) uint16_t As[NBUF][TA][BM][LD];   // NBUF 1: a third of the LDS,
  __shared__ __attribute__((aligned(16))) uint16_t Bs[NBUF][3][BN][LD];    // two barriers per slice
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  int by, bz;
  nat_tile_of<MODE>(a.xcd, by, bz);
  const int m0 = by * BM, n0 = blockIdx.x * BN;
  const bool split = DW || (MODE == NG_FWD && a.kchunk > 0);
  const int kbeg = split ? bz * a.kchunk : 0;
  const int kend = split ? min(a.K, kbeg + a.kchunk) : a.K;
  const int py = MODE == NG_DX ? bz / G::S : 0, px = MODE == NG_DX ? bz % G::S : 0;
  RingRows ring;
  if constexpr (U8) ring.init(a.sa, a.sa.tau_ptr ? *a.sa.tau_ptr : 0);
  // pair p of row quads: 4 lanes along the row's quads (64 contiguous bytes), then 16 k pairs
  auto pair_q = [](int p, int nrowq) { (void)nrowq; return ((p >> 2) / (BK / 2)) * 4 + (p & 3); };
  auto pair_k = [](int p) { return ((p >> 2) % (BK / 2)) * 2; };

  int ar[AQ], ac[AQ];          // A_KC: tile row m, k offset; else: reduction row, m offset
  bool aval[AQ];
  int64_t abase[AQ];
  int ai[AQ], aj[AQ];
  int mk[AQ][3];
#pragma unroll
  for (int i = 0; i < AQ; ++i) {
    if constexpr (A_KC) {
      const int q = tid + 256 * i;
      ar[i] = q >> 3; ac[i] = (q & 7) * 4;
    } else if constexpr (U8) {
      // conv1 dW: quads i = (half h = i >> 1, row i & 1) of one 8-pixel patch row: a lane loads
      // kw 0..7 of (cin, kh) as one 8-byte load per row; lanes run along the k pairs
      static_assert(AQ == 4 && BM == 128, "u8 octets: 16 octets x 16 k pairs");
      ar[i] = 2 * (tid % (BK / 2)) + (i & 1); ac[i] = ((tid / (BK / 2)) * 2 + (i >> 1)) * 4;
    } else {
      const int pp = tid + 256 * (i >> 1);
      ar[i] = pair_k(pp) + (i & 1); ac[i] = pair_q(pp, BM / 4) * 4;
    }
    abase[i] = 0; ai[i] = aj[i] = 0;
    if constexpr (A_KC) {
      const int m = m0 + ar[i];
      aval[i] = m < a.M;
      const int mm = aval[i] ? m : 0;
      if constexpr (MODE == NG_DX) {
        const int b = mm / (NI * NJ), r = mm - b * (NI * NJ);
        abase[i] = b; ai[i] = r / NJ; aj[i] = r - (r / NJ) * NJ;
      } else {
        const int b = mm / P, pos = mm - b * P, oy = pos / G::OW, ox = pos - oy * G::OW;
        abase[i] = (((int64_t)b * G::H + oy * G::S) * G::W + ox * G::S) * G::C;
      }
    } else {
      const int m = m0 + ac[i];
      aval[i] = m < a.M;
      const int mm = aval[i] ? m : 0;
      if constexpr (U8) {
        mk[i][0] = (mm >> 3) & 7; mk[i][1] = mm & 7; mk[i][2] = mm >> 6;
      } else {
        mk[i][0] = mm / (G::KW * G::C);
        mk[i][1] = (mm / G::C) % G::KW;
        mk[i][2] = mm % G::C;
      }
    }
  }
  int br[BQ], bc[BQ];          // B_NC: k row, n offset; else: n row, k offset
  bool bok[BQ];
#pragma unroll
  for (int j = 0; j < BQ; ++j) {
    if constexpr (B_NC) {
      const int pp = tid + 256 * (j >> 1);
      bok[j] = pp < BPAIRS;
      br[j] = pair_k(pp) + (j & 1); bc[j] = pair_q(pp, BN / 4) * 4;
    } else {
      const int q = tid + 256 * j;
      bok[j] = true;
      br[j] = q >> 3; bc[j] = (q & 7) * 4;
    }
  }

  auto load_a = [&](int i, int k0) -> f32x4 {
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if constexpr (A_KC) {
      const int k = k0 + ac[i];
      if (!aval[i] || k >= kend) return v;
      if constexpr (MODE == NG_FWD) {
        const int kh = k / (G::KW * G::C), rem = k - kh * (G::KW * G::C), kw = rem / G::C, c0 = rem - kw * G::C;
        v = *(const f32x4*)(a.X + abase[i] + (kh * G::W + kw) * G::C + c0);
      } else {
        const int th = k / (TW * G::OC), rem = k - th * (TW * G::OC), tw = rem / G::OC, oc0 = rem - tw * G::OC;
        const int oy = ai[i] - th, ox = aj[i] - tw;
        if (oy >= 0 && oy < G::OH && ox >= 0 && ox < G::OW)
          v = *(const f32x4*)(a.dY + ((abase[i] * G::OH + oy) * G::OW + ox) * G::OC + oc0);
      }
    } else {
      const int r = k0 + ar[i];
      if (!aval[i] || r >= kend) return v;
      const int b = r / P, pos = r - b * P, oy = pos / G::OW, ox = pos - oy * G::OW;
      const int y = oy * G::S + mk[i][0], x = ox * G::S + mk[i][1];
      if constexpr (U8) {
        const int t = ring.step_of(b);
        const uint32_t d = *(const uint32_t*)(ring.plane(b - t * ring.E, t, mk[i][2]) + y * IMG + x);
        v[0] = (float)(d & 255u); v[1] = (float)((d >> 8) & 255u); v[2] = (float)((d >> 16) & 255u); v[3] = (float)(d >> 24);
      } else {
        v = *(const f32x4*)(a.X + (((int64_t)b * G::H + y) * G::W + x) * G::C + mk[i][2]);
      }
    }
    return v;
  };
  auto load_b = [&](int j, int k0) -> f32x4 {
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (!bok[j]) return v;
    if constexpr (B_NC) {
      const int k = k0 + br[j], n = n0 + bc[j];
      if (k >= kend || n >= a.N) return v;
      v = DW ? *(const f32x4*)(a.dY + (int64_t)k * G::OC + n) : *(const f32x4*)(a.Wt + (int64_t)k * G::OC + n);
    } else {
      const int n = n0 + br[j], k = k0 + bc[j];
      if (n >= a.N || k >= kend) return v;
      const int th = k / (TW * G::OC), rem = k - th * (TW * G::OC), tw = rem / G::OC, oc0 = rem - tw * G::OC;
      const int kh = py + G::S * th, kw = px + G::S * tw;
      v = *(const f32x4*)(a.Wt + (((int64_t)kh * G::KW + kw) * G::C + n) * G::OC + oc0);
    }
    return v;
  };

  // bias gradient: column sums of dY from the B registers (before the split), one fixed order
  const bool do_colsum = DW && a.colsum && by == 0;
  constexpr int CSN = BQ / 2 > 0 ? BQ / 2 : 1;
  float cs[CSN][4];
#pragma unroll
  for (int jj = 0; jj < CSN; ++jj)
#pragma unroll
    for (int c = 0; c < 4; ++c) cs[jj][c] = 0.f;

  auto store = [&](int buf, const f32x4 (&ra)[AQ], const f32x4 (&rbv)[BQ]) {
    if constexpr (A_KC) {
#pragma unroll
      for (int i = 0; i < AQ; ++i) {
        uint32_t lo[TA], hi[TA];
        nat_split2<TA>(ra[i][0], ra[i][1], lo);
        nat_split2<TA>(ra[i][2], ra[i][3], hi);
#pragma unroll
        for (int t = 0; t < TA; ++t) *(uint2*)&As[buf][t][ar[i]][ac[i]] = make_uint2(lo[t], hi[t]);
      }
    } else {
#pragma unroll
      for (int i = 0; i < AQ; i += 2)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          uint32_t w[TA];
          nat_split2<TA>(ra[i][c], ra[i + 1][c], w);
#pragma unroll
          for (int t = 0; t < TA; ++t) *(uint32_t*)&As[buf][t][ac[i] + c][ar[i]] = w[t];
        }
    }
    if constexpr (B_NC) {
#pragma unroll
      for (int j = 0; j < BQ; j += 2) {
        if (!bok[j]) continue;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          uint32_t w[3];
          nat_split2<3>(rbv[j][c], rbv[j + 1][c], w);
#pragma unroll
          for (int t = 0; t < 3; ++t) *(uint32_t*)&Bs[buf][t][bc[j] + c][br[j]] = w[t];
          if (DW && do_colsum) cs[j / 2][c] += rbv[j][c] + rbv[j + 1][c];
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < BQ; ++j) {
        uint32_t lo[3], hi[3];
        nat_split2<3>(rbv[j][0], rbv[j][1], lo);
        nat_split2<3>(rbv[j][2], rbv[j][3], hi);
#pragma unroll
        for (int t = 0; t < 3; ++t) *(uint2*)&Bs[buf][t][br[j]][bc[j]] = make_uint2(lo[t], hi[t]);
      }
    }
  };

  f32x16 acc = {};
  const int r = lane & 31, h = lane >> 5;
  // conv1 dW: the 8 pixels kw 0..7 of quad i's (cin, kh) row -> quads i (kw 0..3) and i + 2 (kw 4..7)
  auto load_a8 = [&](int i, int k0, f32x4& lo, f32x4& hi) {
    const int r = k0 + ar[i];
    uint2 d = make_uint2(0u, 0u);
    if (aval[i] && r < kend) {
      const int b = r / P, pos = r - b * P, oy = pos / G::OW, ox = pos - oy * G::OW;
      const int y = oy * G::S + mk[i][0], x = ox * G::S;
      const int t = ring.step_of(b);
      const uint32_t* q = (const uint32_t*)(ring.plane(b - t * ring.E, t, mk[i][2]) + y * IMG + x);
      d.x = q[0];
      d.y = q[1];
    }
    lo = (f32x4){(float)(d.x & 255u), (float)((d.x >> 8) & 255u), (float)((d.x >> 16) & 255u), (float)(d.x >> 24)};
    hi = (f32x4){(float)(d.y & 255u), (float)((d.y >> 8) & 255u), (float)((d.y >> 16) & 255u), (float)(d.y >> 24)};
  };
  auto load_all = [&](int k0, f32x4 (&ra)[AQ], f32x4 (&rbv)[BQ]) {
    if constexpr (U8) {
      load_a8(0, k0, ra[0], ra[2]);
      load_a8(1, k0, ra[1], ra[3]);
    } else {
#pragma unroll
      for (int i = 0; i < AQ; ++i) ra[i] = load_a(i, k0);
    }
#pragma unroll
    for (int j = 0; j < BQ; ++j) rbv[j] = load_b(j, k0);
  };
  auto compute = [&](int buf) {
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      bf16x8 af[TA], bv[3];
#pragma unroll
      for (int t = 0; t < TA; ++t) af[t] = *(const bf16x8*)&As[buf][t][wm * 32 + r][16 * s + 8 * h];
#pragma unroll
      for (int t = 0; t < 3; ++t) bv[t] = *(const bf16x8*)&Bs[buf][t][wn * 32 + r][16 * s + 8 * h];
      if constexpr (TA == 1) {
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0], bv[2], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0], bv[1], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0], bv[0], acc, 0, 0, 0);
      } else {
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0], bv[2], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[2], bv[0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1], bv[1], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0], bv[1], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1], bv[0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0], bv[0], acc, 0, 0, 0);
      }
    }
  };
  if constexpr (PF == 2) {
    // two register sets: slice s + 2 loads while slice s computes (s + 1 waits in registers)
    f32x4 ra0[AQ], rb0[BQ], ra1[AQ], rb1[BQ];
    load_all(kbeg, ra0, rb0);
    store(0, ra0, rb0);
    if (kbeg + BK < kend) load_all(kbeg + BK, ra1, rb1);
    if (kbeg + 2 * BK < kend) load_all(kbeg + 2 * BK, ra0, rb0);
    __syncthreads();
    for (int k0 = kbeg; k0 < kend; k0 += 2 * BK) {
      compute(0);
      if constexpr (NBUF == 1) __syncthreads();
      if (k0 + BK < kend) {
        store(NBUF - 1, ra1, rb1);
        if (k0 + 3 * BK < kend) load_all(k0 + 3 * BK, ra1, rb1);
      }
      __syncthreads();
      if (k0 + BK >= kend) break;
      compute(NBUF - 1);
      if constexpr (NBUF == 1) __syncthreads();
      if (k0 + 2 * BK < kend) {
        store(0, ra0, rb0);
        if (k0 + 4 * BK < kend) load_all(k0 + 4 * BK, ra0, rb0);
      }
      __syncthreads();
    }
  } else if constexpr (NBUF == 1) {
    f32x4 ra[AQ], rbv[BQ];
    load_all(kbeg, ra, rbv);
    store(0, ra, rbv);
    __syncthreads();
    for (int k0 = kbeg; k0 < kend; k0 += BK) {
      const bool more = k0 + BK < kend;
      if (more) load_all(k0 + BK, ra, rbv);
      compute(0);
      __syncthreads();
      if (more) {
        store(0, ra, rbv);
        __syncthreads();
      }
    }
  } else {
    f32x4 ra[AQ], rbv[BQ];
    load_all(kbeg, ra, rbv);
    store(0, ra, rbv);
    __syncthreads();
    int buf = 0;
    for (int k0 = kbeg; k0 < kend; k0 += BK) {
      const bool more = k0 + BK < kend;
      if (more) load_all(k0 + BK, ra, rbv);
      compute(buf);
      if (more) store(buf ^ 1, ra, rbv);
      __syncthreads();
      buf ^= 1;
    }
  }

  const int col = n0 + wn * 32 + (lane & 31);
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int row = m0 + wm * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
    if (row >= a.M || col >= a.N) continue;
    float v = acc[q];
    if constexpr (MODE == NG_FWD) {
      if (split) {
        a.slab[((int64_t)bz * a.M + row) * a.N + col] = v;
        continue;
      }
      a.Y[(int64_t)row * a.N + col] = fmaxf(v + a.bias[col], 0.f);
    } else if constexpr (MODE == NG_DX) {
      const int b = row / (NI * NJ), rr = row - b * (NI * NJ), i = rr / NJ, j = rr - (rr / NJ) * NJ;
      const int64_t o = (((int64_t)b * G::H + py + G::S * i) * G::W + px + G::S * j) * G::C + col;
      a.Y[o] = a.X[o] > 0.f ? v : 0.f;
    } else {
      const int trow = MODE == NG_DW1 ? ((((row >> 3) & 7) * 8 + (row & 7)) * 4 + (row >> 6)) : row;
      a.slab[((int64_t)bz * a.M + trow) * a.N + col] = v;
    }
  }
  if constexpr (DW) {
    if (do_colsum) {      // (block-uniform) per-pair partials through LDS, summed over the k pairs in order
      float* red = (float*)&As[0][0][0][0];
#pragma unroll
      for (int j = 0; j < BQ; j += 2) {
        const int pp = tid + 256 * (j >> 1);
        if (pp < BPAIRS) *(f32x4*)&red[pp * 4] = (f32x4){cs[j / 2][0], cs[j / 2][1], cs[j / 2][2], cs[j / 2][3]};
      }
      __syncthreads();
      if (tid < BN && n0 + tid < a.N) {
        const int nq = tid >> 2, c = tid & 3;
        float sum = 0.f;
        for (int kp = 0; kp < BK / 2; ++kp) sum += red[((((nq >> 2) * (BK / 2) + kp) << 2) | (nq & 3)) * 4 + c];
        a.colsum[(int64_t)bz * a.N + n0 + tid] = sum;
      }
    }
  }
}

template <int MODE, int LAYER, int BN, int TA>
static int nat_go_bf(NatGemm a, unsigned gz, hipStream_t s, bool one_buf, bool pf2) {
  constexpr int BM = 4096 / BN;
  if (a.M <= 0 || a.N <= 0) return 0;
  a.xcd = nat_xcd();
  const dim3 grid((unsigned)((a.N + BN - 1) / BN), (unsigned)((a.M + BM - 1) / BM), gz);
  if (one_buf && pf2)
    hipLaunchKernelGGL((k_nat_gemm_bf<MODE, LAYER, BN, TA, 1, 2>), grid, dim3(256), 0, s, a);
  else if (one_buf)
    hipLaunchKernelGGL((k_nat_gemm_bf<MODE, LAYER, BN, TA, 1, 1>), grid, dim3(256), 0, s, a);
  else if (pf2)
    hipLaunchKernelGGL((k_nat_gemm_bf<MODE, LAYER, BN, TA, 2, 2>), grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((k_nat_gemm_bf<MODE, LAYER, BN, TA, 2, 1>), grid, dim3(256), 0, s, a);
  A3C_CHECK(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------------------------------
// conv1 forward on the bf16 matrix cores.  A u8 pixel is exact in bf16, and the fp32 weight is
// three round-to-nearest bf16 terms (w = hi + mid + lo to ~2^-24 relative, as the NIPS conv1,
// net_fwd.hip): acc += x hi + x mid + x lo, every product exact in the fp32 accumulator -- three
// v_mfma_f32_32x32x16_bf16 (32 cycles each) per 16-deep K step instead of eight 64-cycle fp32 ones.
// ---------------------------------------------------------------------------------------
#define W1T_ELEMS (3 * NT1_N * NT_K1)     // bf16: [term][cout][k'], k' = (cin, kh, kw)
#define C1B_LD 40                          // bf16 per LDS row: 32 + 8 (16-byte aligned, rows 80 B apart)

__device__ inline uint32_t nat_bf16_rn(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return u >> 16;
}

__device__ inline void nat_terms3(float w, uint16_t* dst, int64_t tstride) {
#pragma clang fp contract(off)
  const uint32_t h = nat_bf16_rn(w);
  const float r1 = w - __uint_as_float(h << 16);
  const uint32_t m = nat_bf16_rn(r1);
  const float r2 = r1 - __uint_as_float(m << 16);
  const uint32_t l = nat_bf16_rn(r2);
  dst[0] = (uint16_t)h;
  dst[tstride] = (uint16_t)m;
  dst[2 * tstride] = (uint16_t)l;
}

// the prepared block: conv1 [3][32][256] with k' = (cin, kh, kw); conv2 [3][64][512] and conv3
// [3][64][576] with k in TF order (kh, kw, cin) -- one thread per (cout, k)
__global__ void __launch_bounds__(256) k_nat_w_terms(const float* __restrict__ W1, const float* __restrict__ W2,
                                                     const float* __restrict__ W3, uint16_t* __restrict__ wt,
                                                     int all) {
  int i = blockIdx.x * 256 + threadIdx.x;
  if (i < NT1_N * NT_K1) {
    const int n = i / NT_K1, k = i - n * NT_K1;
    const int c = k >> 6, kh = (k >> 3) & 7, kw = k & 7;
    nat_terms3(W1[((kh * 8 + kw) * HIST + c) * NT1_N + n], wt + n * NT_K1 + k, NT1_N * NT_K1);
    return;
  }
  if (!all) return;
  i -= NT1_N * NT_K1;
  if (i < NT2_N * NT_K2) {
    const int n = i / NT_K2, k = i - n * NT_K2;
    nat_terms3(W2[k * NT2_N + n], wt + A3C_NAT_W2T_OFF / 2 + n * NT_K2 + k, NT2_N * NT_K2);
    return;
  }
  i -= NT2_N * NT_K2;
  if (i < NT3_N * NT_K3) {
    const int n = i / NT_K3, k = i - n * NT_K3;
    nat_terms3(W3[k * NT3_N + n], wt + A3C_NAT_W3T_OFF / 2 + n * NT_K3 + k, NT3_N * NT_K3);
    return;
  }
  i -= NT3_N * NT_K3;
  // dX forms: [term][cin][tap][cout] = W[tap][cin][cout] (TF [kh][kw][cin][cout]): a copy per term
  if (i < NT1_N * NT_X2) {
    const int c = i / NT_X2, r = i - c * NT_X2, tap = r >> 6, oc = r & 63;
    nat_terms3(W2[(tap * NT1_N + c) * NT2_N + oc], wt + A3C_NAT_W2X_OFF / 2 + i, NT1_N * NT_X2);
    return;
  }
  i -= NT1_N * NT_X2;
  if (i < NT2_N * NT_K3) {
    const int c = i / NT_K3, r = i - c * NT_K3, tap = r >> 6, oc = r & 63;
    nat_terms3(W3[(tap * NT2_N + c) * NT3_N + oc], wt + A3C_NAT_W3X_OFF / 2 + i, NT2_N * NT_K3);
  }
}

__device__ inline uint2 nat_u8x4_bf16(uint32_t d) {   // 4 pixels -> 4 bf16 (exact: the upper halves of their f32)
  const float f0 = (float)(d & 255u), f1 = (float)((d >> 8) & 255u);
  const float f2 = (float)((d >> 16) & 255u), f3 = (float)(d >> 24);
  return make_uint2(__builtin_amdgcn_perm(__float_as_uint(f1), __float_as_uint(f0), 0x07060302u),
                    __builtin_amdgcn_perm(__float_as_uint(f3), __float_as_uint(f2), 0x07060302u));
}

// tile: 128 rows (sample, pixel) x 32 channels, 4 waves of 32 rows; K = 256 in 8 slices of 32 (k' =
// (cin, kh, kw): a row's 32 k' of a slice are 4 kernel rows of 8 pixels of one plane), LDS double-buffered
template <int NBUF>
__global__ void __launch_bounds__(256) k_nat_conv1_bf(StateAddr sa, const uint16_t* __restrict__ w1t,
                                                      const float* __restrict__ bias, float* __restrict__ Y, int M,
                                                      float scale) {
  constexpr int BM = 128, BK = 32, P = NT1_P, OW = NT1_O;
  __shared__ __attribute__((aligned(16))) uint16_t As[NBUF][BM][C1B_LD];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[NBUF][3][NT1_N][C1B_LD];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int m0 = blockIdx.x * BM;
  RingRows ring;
  ring.init(sa, sa.tau_ptr ? *sa.tau_ptr : 0);
  // A: 2 octets per thread, an octet = kw 0..7 of one (cin, kh) patch row = one 8-byte load
  int ar[2], ac[2], ai[2], aj[2];
  bool aval[2];
  const uint8_t* apl[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = tid + 256 * i;
    ar[i] = q >> 2; ac[i] = (q & 3) * 8;
    const int m = m0 + ar[i];
    aval[i] = m < M;
    const int mm = aval[i] ? m : 0;
    const int b = mm / P, pos = mm - b * P, oy = pos / OW, ox = pos - oy * OW;
    const int t = ring.step_of(b), e = b - t * ring.E;
#pragma unroll
    for (int c = 0; c < 4; ++c) apl[i][c] = ring.plane(e, t, c);
    ai[i] = oy * 4; aj[i] = ox * 4;
  }
  auto load_a = [&](int i, int k0) -> uint2 {
    const int k = k0 + ac[i];
    if (!aval[i]) return make_uint2(0u, 0u);
    const int c = k >> 6, kh = (k >> 3) & 7;
    const uint32_t* q = (const uint32_t*)(apl[i][c] + (ai[i] + kh) * IMG + aj[i]);
    return make_uint2(q[0], q[1]);
  };
  // B: 3 terms x 32 couts x 32 k' per slice = 384 chunks of 8 bf16
  auto load_b = [&](int q, int k0) -> uint4 {
    const int term = q >> 7, n = (q >> 2) & 31, kc = (q & 3) * 8;
    return *(const uint4*)(w1t + (term * NT1_N + n) * NT_K1 + k0 + kc);
  };
  uint2 ra[2];
  uint4 rb0, rb1;
  const bool b2 = tid < 128;
  auto load_all = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) ra[i] = load_a(i, k0);
    rb0 = load_b(tid, k0);
    if (b2) rb1 = load_b(256 + tid, k0);
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const uint2 lo = nat_u8x4_bf16(ra[i].x), hi = nat_u8x4_bf16(ra[i].y);
      *(uint4*)&As[buf][ar[i]][ac[i]] = make_uint4(lo.x, lo.y, hi.x, hi.y);
    }
    {
      const int q = tid, term = q >> 7, n = (q >> 2) & 31, kc = (q & 3) * 8;
      *(uint4*)&Bs[buf][term][n][kc] = rb0;
    }
    if (b2) {
      const int q = 256 + tid, term = q >> 7, n = (q >> 2) & 31, kc = (q & 3) * 8;
      *(uint4*)&Bs[buf][term][n][kc] = rb1;
    }
  };
  f32x16 acc = {};
  const int r = lane & 31, h = lane >> 5;
  auto compute = [&](int buf) {
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      const bf16x8 a = *(const bf16x8*)&As[buf][wid * 32 + r][16 * s + 8 * h];
#pragma unroll
      for (int term = 0; term < 3; ++term) {
        const bf16x8 bv = *(const bf16x8*)&Bs[buf][term][r][16 * s + 8 * h];
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bv, acc, 0, 0, 0);
      }
    }
  };
  load_all(0);
  store(0);
  __syncthreads();
  int buf = 0;
  for (int k0 = 0; k0 < NT_K1; k0 += BK) {
    const bool more = k0 + BK < NT_K1;
    if (more) load_all(k0 + BK);
    compute(buf);
    if constexpr (NBUF == 1) {   // one buffer: the slice is stored after every wave has read it
      __syncthreads();
      if (more) store(0);
    } else {
      if (more) store(buf ^ 1);
    }
    __syncthreads();
    buf ^= NBUF - 1;
  }
  const int col = lane & 31;
  const float bc = bias[col];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int row = m0 + wid * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
    if (row < M) Y[(int64_t)row * NT1_N + col] = fmaxf(acc[q] * scale + bc, 0.f);
  }
}

// ---------------------------------------------------------------------------------------
// conv2 + conv3 forward fused, one workgroup per sample (the rollout's B = E states): the sample's
// l1 (20x20x32) is split into three bf16 terms into LDS once; conv2 (M = 81 pixels, N = 64,
// K = 16 taps x 32) and then conv3 (M = 49, N = 64, K = 9 taps x 64) run on
// v_mfma_f32_16x16x32_bf16 with the six products of the term split (as k_nat_gemm_bf); l2 goes
// out (the backward's operand) and, as terms, into the LDS the l1 terms held, for conv3.  Wave w
// owns output channels 16w..16w+15 of both layers, its weight fragments (the prepared terms,
// [term][cout][k]) streamed from L2 with a 3-tap register ring.  Replaces two K-chain-bound passes
// of 324 / 392 tiles and a fold with one 256-workgroup launch and no l2 re-read from HBM.
// ---------------------------------------------------------------------------------------
// l1 terms: [term][y 20][x parity 2][x / 2 10][32 bf16]: a 16-lane fragment read walks consecutive
// output pixels, which sit at x = 2 ox + kw -- parity-split rows put them one row apart.
// l2 terms: [term][81][72 bf16] over the same LDS after conv2.
#ifndef C23_R1          // (A/B builds: -DC23_R1=40, rows padded for the fragment reads' banks: 96 KB)
#define C23_R1 32          // unpadded: 77 KB, same time alone, room beside the backward (r6r32: 1.64M vs 1.59M)
#endif
#define C23_T1 (NT1_O * 2 * (NT1_O / 2) * C23_R1)   // bf16 per l1 term: 16000
#define C23_R2 72
#define C23_T2 (NT2_P * C23_R2)                     // 5832
static_assert(3 * C23_T2 <= 3 * C23_T1, "l2 terms overlay the l1 terms");

__device__ inline f32x4 c23_mfma6(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], acc, 0, 0, 0);
  return acc;
}

// C1: conv1 as well (k_nat_conv123): the sample's 4 u8 planes staged as bf16 rows, conv1 (M = 400
// pixels, N = 32, K = 256 in (cin, kh, kw) order, the u8 pixel exact: three products) on the same
// MFMA, its output (x/255 + bias, ReLU) written out for the backward and, as terms, into LDS.
#define C123_PR 88                                   // bf16 per staged plane row (84 + 4)
static_assert(HIST * IMG * C123_PR <= 3 * C23_T1, "planes fit the term LDS");
#ifndef C23_PD     // weight-fragment prefetch distance in K steps (the ring holds C23_PD + 1 steps)
#define C23_PD 2
#endif
#ifndef C23_BATCH  // 1: the plane staging issues all its loads before the first conversion
#define C23_BATCH 1
#endif
template <bool C1>
__global__ void __launch_bounds__(256) k_nat_conv23(const float* __restrict__ l1c, const uint16_t* __restrict__ w2t,
                                                    const float* __restrict__ b2, const uint16_t* __restrict__ w3t,
                                                    const float* __restrict__ b3, float* __restrict__ l2,
                                                    float* __restrict__ l3, StateAddr sa, const uint16_t* __restrict__ w1t,
                                                    const float* __restrict__ b1, float* __restrict__ l1, float scale) {
  __shared__ __attribute__((aligned(16))) uint16_t sm[3 * C23_T1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int i16 = lane & 15, g = lane >> 4;
  const int64_t b = blockIdx.x;
  // the engine's live launch span (a3c_engine_span_stats 1, bench.py's roofline)
  unsigned long long* srec = C1 ? span_rec(sa, sa.tau_ptr ? *sa.tau_ptr : 0) : nullptr;
  span_begin(srec);
  if constexpr (C1) {
    // ---- the 4 history planes of state b as bf16 [cin][84][88] ----
    RingRows ring;
    ring.init(sa, sa.tau_ptr ? *sa.tau_ptr : 0);
    const int st = ring.step_of((int)b), e = (int)b - st * ring.E;
#if C23_BATCH
    // every dword of the 4 planes in flight at once (28 per thread), then converted and stored
    constexpr int NQ = HIST * PLANE / 4, PQ = PLANE / 4, PER = (NQ + 255) / 256;
    const uint32_t* pl4[HIST];
#pragma unroll
    for (int c = 0; c < HIST; ++c) pl4[c] = (const uint32_t*)ring.plane(e, st, c);
    uint32_t pv[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int q = tid + 256 * i, c = q / PQ;
      pv[i] = q < NQ ? pl4[c < HIST ? c : 0][q - c * PQ] : 0u;
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int q = tid + 256 * i;
      if (q < NQ) {
        const int c = q / PQ, r = q - c * PQ, y = r / (IMG / 4), x4 = (r - y * (IMG / 4)) * 4;
        *(uint2*)&sm[(c * IMG + y) * C123_PR + x4] = nat_u8x4_bf16(pv[i]);
      }
    }
#else
#pragma unroll
    for (int c = 0; c < HIST; ++c) {
      const uint32_t* src = (const uint32_t*)ring.plane(e, st, c);
      for (int q = tid; q < PLANE / 4; q += 256) {
        const int y = q / (IMG / 4), x4 = (q - y * (IMG / 4)) * 4;
        *(uint2*)&sm[(c * IMG + y) * C123_PR + x4] = nat_u8x4_bf16(src[q]);
      }
    }
#endif
    __syncthreads();
    // ---- conv1: 25 m-tiles x 2 n-tiles of 16; wave w: n-tile w & 1, m-tiles (w >> 1) + 2 i ----
    const int n1 = 16 * (w & 1) + i16;
    const int mh = w >> 1;
    int base1[13];
    f32x4 acc1[13];
#pragma unroll
    for (int i = 0; i < 13; ++i) {
      const int m = min(16 * (mh + 2 * i) + i16, NT1_P - 1);
      const int oy = m / NT1_O, ox = m - oy * NT1_O;
      base1[i] = 4 * oy * C123_PR + 4 * ox;
      acc1[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
    }
    const uint16_t* wb1 = w1t + n1 * NT_K1 + 8 * g;
    bf16x8 q1[C23_PD + 1][3];
    auto ldb1 = [&](int ks, bf16x8 (&dst)[3]) {
#pragma unroll
      for (int t = 0; t < 3; ++t) dst[t] = *(const bf16x8*)(wb1 + t * NT1_N * NT_K1 + ks * 32);
    };
#pragma unroll
    for (int q = 0; q < C23_PD; ++q) ldb1(q, q1[q]);
#pragma unroll
    for (int ks = 0; ks < NT_K1 / 32; ++ks) {
      if (ks + C23_PD < NT_K1 / 32) ldb1(ks + C23_PD, q1[(ks + C23_PD) % (C23_PD + 1)]);
      const int cin = ks >> 1, kh = 4 * (ks & 1) + g;
      const uint16_t* rp = sm + (cin * IMG + kh) * C123_PR;
#pragma unroll
      for (int i = 0; i < 13; ++i) {
        if (mh + 2 * i >= NT1_P / 16) continue;          // (wave-uniform) the 25 tiles
        const uint2 u0 = *(const uint2*)(rp + base1[i]), u1 = *(const uint2*)(rp + base1[i] + 4);
        const bf16x8 a = __builtin_bit_cast(bf16x8, make_uint4(u0.x, u0.y, u1.x, u1.y));
        const bf16x8* bb = q1[ks % (C23_PD + 1)];
        acc1[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bb[2], acc1[i], 0, 0, 0);
        acc1[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bb[1], acc1[i], 0, 0, 0);
        acc1[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bb[0], acc1[i], 0, 0, 0);
      }
    }
    __syncthreads();   // the planes are no longer read: their LDS takes the l1 terms
    const float bn1 = b1[n1];
#pragma unroll
    for (int i = 0; i < 13; ++i) {
      if (mh + 2 * i >= NT1_P / 16) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 16 * (mh + 2 * i) + 4 * g + r;
        const float v = fmaxf(acc1[i][r] * scale + bn1, 0.f);
        l1[(b * NT1_P + m) * NT1_N + n1] = v;
        const int y = m / NT1_O, x = m - y * NT1_O;
        const int slot = (y * 2 + (x & 1)) * (NT1_O / 2) + (x >> 1);
        const float hf = __uint_as_float(nat_bf16_rn(v) << 16);
        const float r1 = v - hf;
        const float mf = __uint_as_float(nat_bf16_rn(r1) << 16);
        sm[0 * C23_T1 + slot * C23_R1 + n1] = (uint16_t)(__float_as_uint(hf) >> 16);
        sm[1 * C23_T1 + slot * C23_R1 + n1] = (uint16_t)(__float_as_uint(mf) >> 16);
        sm[2 * C23_T1 + slot * C23_R1 + n1] = (uint16_t)nat_bf16_rn(r1 - mf);
      }
    }
  } else {
    // ---- stage l1 of sample b as three bf16 terms (3200 float4 chunks, 12.5 per thread) ----
    const f32x4* src = (const f32x4*)(l1c + b * NT_A1);
    constexpr int NCH = NT_A1 / 4;
#pragma unroll 4
    for (int c = tid; c < NCH; c += 256) {
      const f32x4 v = src[c];
      const int px = c >> 3, c4 = (c & 7) * 4;          // pixel (y 20 x 20), channel quad
      const int y = px / NT1_O, x = px - y * NT1_O;
      const int slot = (y * 2 + (x & 1)) * (NT1_O / 2) + (x >> 1);
      uint32_t lo[3], hi[3];
      nat_split2<3>(v[0], v[1], lo);
      nat_split2<3>(v[2], v[3], hi);
#pragma unroll
      for (int t = 0; t < 3; ++t) *(uint2*)&sm[t * C23_T1 + slot * C23_R1 + c4] = make_uint2(lo[t], hi[t]);
    }
  }
  __syncthreads();
  // ---- conv2: 6 m-tiles of 16 pixels (81 valid) x this wave's 16 channels, 16 taps ----
  const int n = 16 * w + i16;
  int base2[6];
#pragma unroll
  for (int mt = 0; mt < 6; ++mt) {
    const int m = min(16 * mt + i16, NT2_P - 1);
    const int oy = m / NT2_O, ox = m - oy * NT2_O;
    base2[mt] = (oy * 2 * 2) * (NT1_O / 2) + ox;           // slot of (y = 2 oy, parity 0, x/2 = ox)
  }
  f32x4 acc2[6];
#pragma unroll
  for (int mt = 0; mt < 6; ++mt) acc2[mt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const uint16_t* wb2 = w2t + (int64_t)n * NT_K2 + 8 * g;
  bf16x8 bq[C23_PD + 1][3];
  auto ldb2 = [&](int tap, bf16x8 (&dst)[3]) {
#pragma unroll
    for (int t = 0; t < 3; ++t) dst[t] = *(const bf16x8*)(wb2 + (int64_t)t * NT2_N * NT_K2 + tap * 32);
  };
#pragma unroll
  for (int q = 0; q < C23_PD; ++q) ldb2(q, bq[q]);
#pragma unroll
  for (int tap = 0; tap < 16; ++tap) {
    if (tap + C23_PD < 16) ldb2(tap + C23_PD, bq[(tap + C23_PD) % (C23_PD + 1)]);
    const int kh = tap >> 2, kw = tap & 3;
    const int toff = (kh * 2 + (kw & 1)) * (NT1_O / 2) + (kw >> 1);
#pragma unroll
    for (int mt = 0; mt < 6; ++mt) {
      bf16x8 a[3];
      const uint16_t* ap = sm + (base2[mt] + toff) * C23_R1 + 8 * g;
#pragma unroll
      for (int t = 0; t < 3; ++t) a[t] = *(const bf16x8*)(ap + t * C23_T1);
      acc2[mt] = c23_mfma6(a, bq[tap % (C23_PD + 1)], acc2[mt]);
    }
  }
  __syncthreads();   // every wave is done reading the l1 terms
  // ---- conv2 epilogue: bias + ReLU, l2 out, l2 terms into LDS ----
  {
    const float bn = b2[n];
#pragma unroll
    for (int mt = 0; mt < 6; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 16 * mt + 4 * g + r;
        if (m < NT2_P) {
          const float v = fmaxf(acc2[mt][r] + bn, 0.f);
          l2[(b * NT2_P + m) * NT2_N + n] = v;
          const float hf = __uint_as_float(nat_bf16_rn(v) << 16);
          const float r1 = v - hf;
          const float mf = __uint_as_float(nat_bf16_rn(r1) << 16);
          const float r2 = r1 - mf;
          sm[0 * C23_T2 + m * C23_R2 + n] = (uint16_t)(__float_as_uint(hf) >> 16);
          sm[1 * C23_T2 + m * C23_R2 + n] = (uint16_t)(__float_as_uint(mf) >> 16);
          sm[2 * C23_T2 + m * C23_R2 + n] = (uint16_t)nat_bf16_rn(r2);
        }
      }
  }
  // weight ring of conv3 starts under the barrier
  const uint16_t* wb3 = w3t + (int64_t)n * NT_K3 + 8 * g;
  auto ldb3 = [&](int st, bf16x8 (&dst)[3]) {
#pragma unroll
    for (int t = 0; t < 3; ++t) dst[t] = *(const bf16x8*)(wb3 + (int64_t)t * NT3_N * NT_K3 + st * 32);
  };
#pragma unroll
  for (int q = 0; q < C23_PD; ++q) ldb3(q, bq[q]);
  __syncthreads();
  // ---- conv3: 4 m-tiles of 16 pixels (49 valid), 18 K steps (9 taps x 2 channel halves) ----
  int base3[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    const int m = min(16 * mt + i16, NT3_P - 1);
    const int oy = m / NT3_O, ox = m - oy * NT3_O;
    base3[mt] = oy * NT2_O + ox;
  }
  f32x4 acc3[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) acc3[mt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int st = 0; st < 18; ++st) {
    if (st + C23_PD < 18) ldb3(st + C23_PD, bq[(st + C23_PD) % (C23_PD + 1)]);
    const int tap = st >> 1, kh = tap / 3, kw = tap - kh * 3;
    const int off = (kh * NT2_O + kw) * C23_R2 + 32 * (st & 1) + 8 * g;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      bf16x8 a[3];
      const uint16_t* ap = sm + base3[mt] * C23_R2 + off;
#pragma unroll
      for (int t = 0; t < 3; ++t) a[t] = *(const bf16x8*)(ap + t * C23_T2);
      acc3[mt] = c23_mfma6(a, bq[st % (C23_PD + 1)], acc3[mt]);
    }
  }
  const float b3n = b3[n];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = 16 * mt + 4 * g + r;
      if (m < NT3_P) l3[(b * NT3_P + m) * NT3_N + n] = fmaxf(acc3[mt][r] + b3n, 0.f);
    }
  span_end(srec);
}

// ---------------------------------------------------------------------------------------
// conv3 dX and conv2 dX fused, one workgroup per sample (network.py's conv2 / conv3 backward):
//   dl2 = col2im(dl3 W3^T) * (l2 > 0)   M = 81 pixels, N = 64, K = 9 taps x 64 cout
//   dl1 = col2im(dl2 W2^T) * (l1 > 0)   per stride-2 parity class: M = 100, N = 32, K = 4 real taps x 64
// dl3 (already masked by l3 > 0) is staged as three bf16 terms on a zero-bordered 11 x 11 grid,
// so every tap reads a plain fragment (out-of-range sources are the zeros); dl2 goes out (conv2
// dW's operand) and, as terms on a 1-bordered 11 x 11 grid, into the same LDS for conv2 dX.
// The weights' dX forms ([term][cin][tap][cout], prepared per rollout) stream from L2.
// ---------------------------------------------------------------------------------------
#define DX_R 72                                   // bf16 per grid cell (64 + 8)
#define DX_G (11 * 11)
#define DX_T (DX_G * DX_R)                        // bf16 per term
__global__ void __launch_bounds__(256) k_nat_dx32(const float* __restrict__ dl3, const float* __restrict__ l2,
                                                  const float* __restrict__ l1, const uint16_t* __restrict__ w3x,
                                                  const uint16_t* __restrict__ w2x, float* __restrict__ dl2,
                                                  float* __restrict__ dl1) {
  __shared__ __attribute__((aligned(16))) uint16_t sm[3 * DX_T];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int i16 = lane & 15, g = lane >> 4;
  const int64_t b = blockIdx.x;
  auto zero_all = [&]() {
    for (int q = tid; q < 3 * DX_T / 8; q += 256) ((uint4*)sm)[q] = make_uint4(0u, 0u, 0u, 0u);
  };
  zero_all();
  __syncthreads();
  {   // dl3 [49][64] -> cells (y + 2, x + 2)
    const f32x4* src = (const f32x4*)(dl3 + b * NT_FLAT);
    for (int q = tid; q < NT_FLAT / 4; q += 256) {
      const f32x4 v = src[q];
      const int px = q >> 4, c4 = (q & 15) * 4, y = px / NT3_O, x = px - y * NT3_O;
      const int cell = (y + 2) * 11 + x + 2;
      uint32_t lo[3], hi[3];
      nat_split2<3>(v[0], v[1], lo);
      nat_split2<3>(v[2], v[3], hi);
#pragma unroll
      for (int t = 0; t < 3; ++t) *(uint2*)&sm[t * DX_T + cell * DX_R + c4] = make_uint2(lo[t], hi[t]);
    }
  }
  __syncthreads();
  // ---- conv3 dX: 6 m-tiles of the 81 l2 pixels x this wave's 16 cin, 18 K steps ----
  const int n3 = 16 * w + i16;
  int cell3[6];
#pragma unroll
  for (int mt = 0; mt < 6; ++mt) {
    const int m = min(16 * mt + i16, NT2_P - 1);
    const int y = m / NT2_O, x = m - y * NT2_O;
    cell3[mt] = (y + 2) * 11 + x + 2;
  }
  f32x4 acc3[6];
#pragma unroll
  for (int mt = 0; mt < 6; ++mt) acc3[mt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const uint16_t* wb3 = w3x + (int64_t)n3 * NT_K3 + 8 * g;
  bf16x8 bq[3][3];
  auto ldb3 = [&](int st, bf16x8 (&dst)[3]) {
#pragma unroll
    for (int t = 0; t < 3; ++t) dst[t] = *(const bf16x8*)(wb3 + (int64_t)t * NT2_N * NT_K3 + st * 32);
  };
  ldb3(0, bq[0]);
  ldb3(1, bq[1]);
#pragma unroll
  for (int st = 0; st < 18; ++st) {
    if (st + 2 < 18) ldb3(st + 2, bq[(st + 2) % 3]);
    const int tap = st >> 1, kh = tap / 3, kw = tap - kh * 3;
    const int off = -(kh * 11 + kw) * DX_R + 32 * (st & 1) + 8 * g;   // source dl3 pixel (y - kh, x - kw)
#pragma unroll
    for (int mt = 0; mt < 6; ++mt) {
      bf16x8 a[3];
      const uint16_t* ap = sm + cell3[mt] * DX_R + off;
#pragma unroll
      for (int t = 0; t < 3; ++t) a[t] = *(const bf16x8*)(ap + t * DX_T);
      acc3[mt] = c23_mfma6(a, bq[st % 3], acc3[mt]);
    }
  }
  __syncthreads();   // dl3 terms no longer read
  zero_all();
  __syncthreads();
  // dl2 = acc * (l2 > 0): out, and as terms into cells (y + 1, x + 1)
#pragma unroll
  for (int mt = 0; mt < 6; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = 16 * mt + 4 * g + r;
      if (m < NT2_P) {
        const int64_t o = (b * NT2_P + m) * NT2_N + n3;
        const float v = l2[o] > 0.f ? acc3[mt][r] : 0.f;
        dl2[o] = v;
        const int y = m / NT2_O, x = m - y * NT2_O, cell = (y + 1) * 11 + x + 1;
        const float hf = __uint_as_float(nat_bf16_rn(v) << 16);
        const float r1 = v - hf;
        const float mf = __uint_as_float(nat_bf16_rn(r1) << 16);
        sm[0 * DX_T + cell * DX_R + n3] = (uint16_t)(__float_as_uint(hf) >> 16);
        sm[1 * DX_T + cell * DX_R + n3] = (uint16_t)(__float_as_uint(mf) >> 16);
        sm[2 * DX_T + cell * DX_R + n3] = (uint16_t)nat_bf16_rn(r1 - mf);
      }
    }
  __syncthreads();
  // ---- conv2 dX: 4 parity classes x 7 m-tiles (100 pixels of the 10 x 10 class grid) x 2
  // n-tiles of 16 cin; wave w: n-tile w & 1, m-tiles (w >> 1) + 2 j of every class ----
  const int n2 = 16 * (w & 1) + i16;
  const int mh = w >> 1;
  const uint16_t* wb2 = w2x + (int64_t)n2 * NT_X2 + 8 * g;
#pragma unroll
  for (int cl = 0; cl < 4; ++cl) {
    const int py = cl >> 1, px = cl & 1;
    int cell2[4];
    f32x4 acc2[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = min(16 * (mh + 2 * j) + i16, 99);
      const int ci = m / 10, cj = m - ci * 10;
      cell2[j] = (ci + 1) * 11 + cj + 1;
      acc2[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    }
    // K step ks: real tap (th, tw) = ((ks >> 1) >> 1, (ks >> 1) & 1), kernel tap (py + 2 th, px + 2 tw)
    auto ldb2 = [&](int ks, bf16x8 (&dst)[3]) {
      const int tp = ks >> 1, th = tp >> 1, tw = tp & 1;
      const int tap = (py + 2 * th) * 4 + px + 2 * tw;
#pragma unroll
      for (int t = 0; t < 3; ++t)
        dst[t] = *(const bf16x8*)(wb2 + (int64_t)t * NT1_N * NT_X2 + tap * 64 + 32 * (ks & 1));
    };
    ldb2(0, bq[0]);
    ldb2(1, bq[1]);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      if (ks + 2 < 8) ldb2(ks + 2, bq[(ks + 2) % 3]);
      const int tp = ks >> 1, th = tp >> 1, tw = tp & 1;
      const int off = -(th * 11 + tw) * DX_R + 32 * (ks & 1) + 8 * g;   // dl2 pixel (i - th, j - tw)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (mh + 2 * j >= 7) continue;                  // (wave-uniform) the class's 7 tiles
        bf16x8 a[3];
        const uint16_t* ap = sm + cell2[j] * DX_R + off;
#pragma unroll
        for (int t = 0; t < 3; ++t) a[t] = *(const bf16x8*)(ap + t * DX_T);
        acc2[j] = c23_mfma6(a, bq[ks % 3], acc2[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (mh + 2 * j >= 7) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 16 * (mh + 2 * j) + 4 * g + r;
        if (m < 100) {
          const int ci = m / 10, cj = m - ci * 10;
          const int64_t o = (b * NT1_P + (2 * ci + py) * NT1_O + 2 * cj + px) * NT1_N + n2;
          dl1[o] = l1[o] > 0.f ? acc2[j][r] : 0.f;
        }
      }
    }
  }
}

// the policy / value head of B states (one wave each) on the 512-wide fc output, + the action
// draw and fused env act when sel.mode >= 0 (agent.py:59-62, network.py:72)
__global__ void __launch_bounds__(256) k_nat_head(const float* __restrict__ l4, int64_t B, const float* __restrict__ Wp,
                                                  const float* __restrict__ bp, const float* __restrict__ Wv,
                                                  const float* __restrict__ bv, int A, int zs, float* __restrict__ z,
                                                  HeadSelect sel) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const float myz = head_row<NoMid, NT_FC>(l4, b, Wp, bp, Wv, bv, A, lane);
  if (lane < zs) z[b * zs + lane] = myz;
  if (sel.mode >= 0) (void)head_act(myz, lane, A, sel, b);
  // the overlap rollout's bootstrap head (its last kernel) advances tau (no tau read here)
  if (sel.adv_ptr && blockIdx.x == 0 && threadIdx.x == 0) *sel.adv_ptr += sel.adv_n;
}

// ---------------------------------------------------------------------------------------
// passes (one launch each, timed individually by a3c_engine_time_kernel)
// ---------------------------------------------------------------------------------------
#define NAT_GROUPS 8
struct NatPlan {
  int head_split, ns1, ns2, ns3, kc1, kc2, kc3;
  int64_t dz, dl4, dl3, dl2, dl1, terms, hgrad, hcol, hslab, fccol, s1, s2, s3, c1, c2, c3, g1, g2, g3, wprep, total;
};
// the reduction split of a weight-gradient pass: ~target workgroups over its m tiles
static void dw_split(int64_t R, int mtiles, int target, int& ns, int& kc) {
  int want = target / mtiles;
  if (want < 1) want = 1;
  int64_t per = (R + want - 1) / want;
  per = (per + 31) / 32 * 32;               // whole K slices
  if (per < 32) per = 32;
  kc = (int)per;
  ns = (int)((R + per - 1) / per);
}
static NatPlan nat_plan(const NetLayout& L, int64_t B) {
  NatPlan p = {};
  int64_t o = 0;
  auto take = [&](int64_t floats) { int64_t r = o; o += (floats + 63) & ~(int64_t)63; return r; };
  p.head_split = a3c_gemm_effective_split((int)B, a3c_gemm_plan_split(NT_FC, L.zs, (int)B, 128));
  // workgroups per dW pass (the reduction's slab count): conv1 / conv2 / conv3 768 / 2048 / 768,
  // by whole-bench sweeps (r6dwg2-5, B = 1280): 1.717M against 1.653M for 1536 on all three (the
  // choice by times alone, r6dwg: 62 / 89 / 97 -> 51 / 74 / 81 us against 512); conv1's count is
  // the sensitive one (832: 1.65M, 1536: 1.65M, 640: 1.68M)
  static const int wgs = (int)A3C_AB_KNOB("A3C_NAT_DW_WGS", 0);   // > 0: one count for all three
  static const int wgs1 = (int)A3C_AB_KNOB("A3C_NAT_DW_WGS1", wgs > 0 ? wgs : 768);
  static const int wgs2 = (int)A3C_AB_KNOB("A3C_NAT_DW_WGS2", wgs > 0 ? wgs : 2048);
  static const int wgs3 = (int)A3C_AB_KNOB("A3C_NAT_DW_WGS3", wgs > 0 ? wgs : 768);
  dw_split(B * NT1_P, 2, wgs1, p.ns1, p.kc1);     // M = 256 in 128-row tiles
  dw_split(B * NT2_P, 8, wgs2, p.ns2, p.kc2);     // M = 512 in 64-row tiles
  dw_split(B * NT3_P, 9, wgs3, p.ns3, p.kc3);     // M = 576
  p.dz = take(B * L.zs);
  p.dl4 = take(B * NT_FC);
  p.dl3 = take(B * NT_FLAT);
  p.dl2 = take(B * NT_A2);
  p.dl1 = take(B * NT_A1);
  p.terms = take(B * 4);
  p.hgrad = take((int64_t)NT_FC * L.zs);
  p.hcol = take((int64_t)p.head_split * L.zs);
  p.hslab = take(p.head_split > 1 ? (int64_t)p.head_split * NT_FC * L.zs : 0);
  p.fccol = take(NT_FC);
  p.s1 = take((int64_t)p.ns1 * NT_K1 * NT1_N);
  p.s2 = take((int64_t)p.ns2 * NT_K2 * NT2_N);
  p.s3 = take((int64_t)p.ns3 * NT_K3 * NT3_N);
  p.c1 = take((int64_t)p.ns1 * NT1_N);
  p.c2 = take((int64_t)p.ns2 * NT2_N);
  p.c3 = take((int64_t)p.ns3 * NT3_N);
  p.g1 = take((int64_t)NAT_GROUPS * NT_K1 * NT1_N);
  p.g2 = take((int64_t)NAT_GROUPS * NT_K2 * NT2_N);
  p.g3 = take((int64_t)NAT_GROUPS * NT_K3 * NT3_N);
  p.wprep = take(A3C_NAT_PREP_BYTES / 4);   // the per-op path's weight terms (the engine's are in the slot)
  p.total = o;
  return p;
}

static int fc_split(int64_t B) {
  static const int v = (int)A3C_AB_KNOB("A3C_NAT_FC_SPLIT", 0);   // A/B: > 0 overrides the plan
  return a3c_gemm_effective_split(NT_FLAT, v > 0 ? v : a3c_gemm_plan_split((int)B, NT_FC, NT_FLAT, 512));
}
// conv2 / conv3 forward: few output tiles at the rollout's B = E (324 / 196 of 64 x 64 at 256
// envs), each a long K chain -- conv3 splits K in two so twice the workgroups run half the chain
// (measured, r6sp1: conv2 28.5 us unsplit vs 30.2 split in 2, conv3 25.3 vs 23.2; 4-way loses on both)
#define NAT_FWD_SPLIT(LAYER) ((LAYER) == 2 ? 1 : 2)
#define NAT_FWD_SPLIT_MAX 4
static int nat_fwd_split_n(int layer) {
  static const int v = (int)A3C_AB_KNOB("A3C_NAT_FWD_SPLIT", 0);   // A/B: 1..4 for both layers
  const int n = v > 0 ? v : NAT_FWD_SPLIT(layer);
  return n > NAT_FWD_SPLIT_MAX ? NAT_FWD_SPLIT_MAX : n;
}
// passes on the bf16 matrix cores / with one LDS buffer (bits NAT_*; measured per pass)
// (every pass on bf16 terms, with one LDS buffer (30 KB instead of 61: room for the other stream's
// workgroups); two slices in registers for conv1 dW.  Chosen by whole-bench A/B,
// tools/r6/nat_ab_bench.sh r6pf3 / r6pf4: 1.20M with two buffers on the dW passes although they time
// faster alone, 1.28M with one, 1.33M with conv3 fwd's one as well).  Bits NAT_FCF / NAT_FCW /
// NAT_FCX put the fc's forward and backward GEMMs on the same kernels: measured-and-rejected
// (r6fc1: 1.27M / 1.30M / 1.32M against 1.33M on gemm.hip), so they stay A/B-only)
#define NAT_BF_DEFAULT ((1 << NAT_C2F) | (1 << NAT_C3F) | (1 << NAT_C3W) | (1 << NAT_C3X) | (1 << NAT_C2W) | \
                        (1 << NAT_C2X) | (1 << NAT_C1W))
#define NAT_BF1_DEFAULT ((1 << NAT_C2F) | (1 << NAT_C3F) | (1 << NAT_C3W) | (1 << NAT_C3X) | (1 << NAT_C2W) | \
                         (1 << NAT_C2X))
#define NAT_PF2_DEFAULT (1 << NAT_C1W)

static int64_t nat_fwd_slab_floats(int64_t B) {
  const int sp = fc_split(B);
  const int64_t fc = sp > 1 ? (int64_t)sp * B * NT_FC : 0;
  const int64_t cv = (int64_t)NAT_FWD_SPLIT_MAX * B * (NT2_P * NT2_N > NT3_P * NT3_N ? NT2_P * NT2_N : NT3_P * NT3_N);
  return ((fc > cv ? fc : cv) + 63) / 64 * 64;
}
int64_t a3c_nat_fwd_ws_floats(int64_t B) { return nat_fwd_slab_floats(B) + A3C_NAT_PREP_BYTES / 4; }
// which passes run on the bf16 matrix cores (bit NAT_*) and which of those with one LDS buffer
static bool nat_bf(int pass) {
  static const long long v = A3C_AB_KNOB("A3C_NAT_BF", NAT_BF_DEFAULT);
  return (v >> pass) & 1;
}
static bool nat_bf1(int pass) {
  static const long long v = A3C_AB_KNOB("A3C_NAT_BF1", NAT_BF1_DEFAULT);
  return (v >> pass) & 1;
}
static bool nat_pf2(int pass) {     // two slices in flight in registers
  static const long long v = A3C_AB_KNOB("A3C_NAT_PF2", NAT_PF2_DEFAULT);
  return (v >> pass) & 1;
}
// A/B: 1 = the fc's split-K fold inside the head + screen kernel (one launch per step fewer);
// measured-and-rejected: 1.29M vs 1.33M (r6fh1) -- 256 workgroups each folding 16 slabs of one
// row are slower than the wide fold kernel
static int nat_fold_head() {
  static const int v = (int)A3C_AB_KNOB("A3C_NAT_FOLD_HEAD", 0);
  return v;
}
static int nat_fuse23() {
  static const int v = (int)A3C_AB_KNOB("A3C_NAT_FUSE23", 1);   // A/B: 0 = separate conv2 / conv3 passes
  return v;
}
static int nat_fuse123() {
  static const int v = (int)A3C_AB_KNOB("A3C_NAT_FUSE123", 1);   // A/B: 0 = conv1 its own launch
  return v;
}
// A/B: 1 = conv3 dX + conv2 dX as one per-sample launch (k_nat_dx32): 153 us alone against 85 + 107
// for the two passes, but the whole bench loses (r6fu: 1.51M vs 1.60M; r6dxp: 1.58M vs 1.64M) --
// two of its 52 KB workgroups on a CU keep the rollout's conv workgroup off it, and reserving LDS
// so that only one fits (1.37M) starves the pass itself; so it stays off
static int nat_fuse_dx() {
  static const int v = (int)A3C_AB_KNOB("A3C_NAT_FUSE_DX", 0);
  return v;
}
bool a3c_nat_dx_fused() { return nat_fuse_dx() != 0; }
bool a3c_nat_conv23_fused() { return nat_fuse23() != 0; }
bool a3c_nat_conv123_fused() { return nat_fuse23() && nat_fuse123(); }
static int nat_c1_bf() {
  static const int v = (int)A3C_AB_KNOB("A3C_NAT_C1_BF", 1);   // A/B: 0 = the fp32 MFMA conv1 forward
  return v;
}

// a split conv forward: partials into fws, then the fold with bias + ReLU into Y (gemm.hip)
template <int LAYER>
static int nat_fwd_split(NatGemm a, float* fws, hipStream_t s) {
  constexpr int pass = LAYER == 2 ? NAT_C2F : NAT_C3F;
  const int S = nat_fwd_split_n(LAYER);
  if (S == 1) {    // one K chain per tile: bias + ReLU in the tile's epilogue
    a.kchunk = 0;
    return nat_bf(pass) ? nat_go_bf<NG_FWD, LAYER, 64, 3>(a, 1, s, nat_bf1(pass), nat_pf2(pass)) : nat_go<NG_FWD, LAYER, 64>(a, 1, s);
  }
  a.kchunk = ((a.K + S - 1) / S + 31) / 32 * 32;
  const int ns = (a.K + a.kchunk - 1) / a.kchunk;
  a.slab = fws;
  int rc = nat_bf(pass) ? nat_go_bf<NG_FWD, LAYER, 64, 3>(a, (unsigned)ns, s, nat_bf1(pass), nat_pf2(pass))
                        : nat_go<NG_FWD, LAYER, 64>(a, (unsigned)ns, s);
  if (rc) return rc;
  GemmArgs g = {};
  g.slab = fws; g.nsplit = ns; g.M = a.M; g.N = a.N; g.C = a.Y; g.ldc = a.N; g.epi = EPI_BIAS_RELU; g.bias = a.bias;
  return a3c_gemm_reduce(g, s);
}
int64_t a3c_nat_bwd_ws_floats(const NetLayout& L, int64_t B) { return nat_plan(L, B).total; }

// one pass of the forward (B states) or of the backward (B samples, buffers of the plan in bws)
int a3c_nat_pass_launch(int pass, const NetLayout& L, const float* P, const StateAddr& sa, int64_t B, const float* l1,
                        const float* l2, const float* l3, const float* l4, const uint16_t* w1t, float* fws,
                        float* bws, hipStream_t s) {
  NatGemm a = {};
  switch (pass) {
    case NAT_C1F:
      if (w1t && nat_fuse23() && nat_fuse123()) return 0;   // inside NAT_C2F's launch
      if (w1t && nat_c1_bf()) {
        const int M = (int)(B * NT1_P);
        if (nat_bf1(NAT_C1F))
          hipLaunchKernelGGL(k_nat_conv1_bf<1>, dim3((unsigned)((M + 127) / 128)), dim3(256), 0, s, sa, w1t,
                             P + L.off[N_L1B], (float*)l1, M, 1.0f / 255.0f);
        else
          hipLaunchKernelGGL(k_nat_conv1_bf<2>, dim3((unsigned)((M + 127) / 128)), dim3(256), 0, s, sa, w1t,
                             P + L.off[N_L1B], (float*)l1, M, 1.0f / 255.0f);
        A3C_CHECK(hipGetLastError());
        return 0;
      }
      a.sa = sa;
      a.Wt = P + L.off[N_L1W]; a.bias = P + L.off[N_L1B]; a.Y = (float*)l1;
      a.M = (int)(B * NT1_P); a.N = NT1_N; a.K = NT_K1; a.scale = 1.0f / 255.0f;
      return nat_go<NG_FWD1, 1, 32>(a, 1, s);
    case NAT_C2F:
      if (w1t && nat_fuse23()) {   // conv2 + conv3 (+ conv1) in one launch; NAT_C3F (NAT_C1F) then empty
        if (nat_fuse123())
          hipLaunchKernelGGL(k_nat_conv23<true>, dim3((unsigned)B), dim3(256), 0, s, (const float*)nullptr,
                             w1t + A3C_NAT_W2T_OFF / 2, P + L.off[N_L2B], w1t + A3C_NAT_W3T_OFF / 2,
                             P + L.off[N_L3B], (float*)l2, (float*)l3, sa, w1t, P + L.off[N_L1B], (float*)l1,
                             1.0f / 255.0f);
        else
          hipLaunchKernelGGL(k_nat_conv23<false>, dim3((unsigned)B), dim3(256), 0, s, l1, w1t + A3C_NAT_W2T_OFF / 2,
                             P + L.off[N_L2B], w1t + A3C_NAT_W3T_OFF / 2, P + L.off[N_L3B], (float*)l2, (float*)l3,
                             sa, (const uint16_t*)nullptr, (const float*)nullptr, (float*)nullptr, 0.f);
        A3C_CHECK(hipGetLastError());
        return 0;
      }
      a.X = l1; a.Wt = P + L.off[N_L2W]; a.bias = P + L.off[N_L2B]; a.Y = (float*)l2;
      a.M = (int)(B * NT2_P); a.N = NT2_N; a.K = NT_K2;
      return nat_fwd_split<2>(a, fws, s);
    case NAT_C3F:
      if (w1t && nat_fuse23()) return 0;
      a.X = l2; a.Wt = P + L.off[N_L3W]; a.bias = P + L.off[N_L3B]; a.Y = (float*)l3;
      a.M = (int)(B * NT3_P); a.N = NT3_N; a.K = NT_K3;
      return nat_fwd_split<3>(a, fws, s);
    case NAT_FCF: {
      if (fws == nullptr) return a3c_set_error(A3C_ERR_INVALID, "a3c_nat_pass_launch", "fc: no slab workspace");
      if (nat_bf(NAT_FCF)) {   // bf16 terms: K split over grid z into fws slabs, fold with bias + ReLU
        a.X = l3; a.Wt = P + L.off[N_FCW]; a.bias = P + L.off[N_FCB]; a.Y = (float*)l4;
        a.M = (int)B; a.N = NT_FC; a.K = NT_FLAT;
        const int ns = fc_split(B);
        if (ns <= 1) return nat_go_bf<NG_FWD, 4, 64, 3>(a, 1, s, nat_bf1(NAT_FCF), nat_pf2(NAT_FCF));
        a.kchunk = ((a.K + ns - 1) / ns + 31) / 32 * 32;
        const int nz = (a.K + a.kchunk - 1) / a.kchunk;
        a.slab = fws;
        int rc = nat_go_bf<NG_FWD, 4, 64, 3>(a, (unsigned)nz, s, nat_bf1(NAT_FCF), nat_pf2(NAT_FCF));
        if (rc) return rc;
        GemmArgs g = {};
        g.slab = fws; g.nsplit = nz; g.M = a.M; g.N = a.N; g.C = a.Y; g.ldc = a.N; g.epi = EPI_BIAS_RELU; g.bias = a.bias;
        return a3c_gemm_reduce(g, s);
      }
      // l4 = relu(l3 W + b) (network.py:41-42, ops.py:41-44): split-K slabs, the fold applies the epilogue
      GemmArgs gf = {};
      gf.A = l3; gf.lda = NT_FLAT;
      gf.B = P + L.off[N_FCW]; gf.ldb = NT_FC;
      gf.C = (float*)l4; gf.ldc = NT_FC;
      gf.M = (int)B; gf.N = NT_FC; gf.K = NT_FLAT;
      gf.epi = EPI_BIAS_RELU; gf.bias = P + L.off[N_FCB];
      gf.nsplit = fc_split(B); gf.slab = fws;
      return a3c_gemm(true, true, gf, s);
    }
    default:
      break;
  }
  const NatPlan p = nat_plan(L, B);
  switch (pass) {
    case NAT_C3W:     // dW3 (+ db3) over the (sample, pixel) rows
      a.X = l2; a.dY = bws + p.dl3; a.slab = bws + p.s3; a.colsum = bws + p.c3;
      a.M = NT_K3; a.N = NT3_N; a.K = (int)(B * NT3_P); a.kchunk = p.kc3;
      return nat_bf(NAT_C3W) ? nat_go_bf<NG_DW, 3, 64, 3>(a, (unsigned)p.ns3, s, nat_bf1(NAT_C3W), nat_pf2(NAT_C3W))
                           : nat_go<NG_DW, 3, 64>(a, (unsigned)p.ns3, s);
    case NAT_C3X:     // dl2 = col2im(dl3 W3^T) * (l2 > 0)
      if (w1t && nat_fuse_dx()) {   // and dl1 in the same launch (k_nat_dx32); NAT_C2X then empty
        hipLaunchKernelGGL(k_nat_dx32, dim3((unsigned)B), dim3(256), 0, s, bws + p.dl3, l2, l1,
                           w1t + A3C_NAT_W3X_OFF / 2, w1t + A3C_NAT_W2X_OFF / 2, bws + p.dl2, bws + p.dl1);
        A3C_CHECK(hipGetLastError());
        return 0;
      }
      a.X = l2; a.dY = bws + p.dl3; a.Wt = P + L.off[N_L3W]; a.Y = bws + p.dl2;
      a.M = (int)(B * NT2_P); a.N = NT2_N; a.K = 3 * 3 * NT3_N;
      return nat_bf(NAT_C3X) ? nat_go_bf<NG_DX, 3, 64, 3>(a, 1, s, nat_bf1(NAT_C3X), nat_pf2(NAT_C3X))
                           : nat_go<NG_DX, 3, 64>(a, 1, s);
    case NAT_C2W:
      a.X = l1; a.dY = bws + p.dl2; a.slab = bws + p.s2; a.colsum = bws + p.c2;
      a.M = NT_K2; a.N = NT2_N; a.K = (int)(B * NT2_P); a.kchunk = p.kc2;
      return nat_bf(NAT_C2W) ? nat_go_bf<NG_DW, 2, 64, 3>(a, (unsigned)p.ns2, s, nat_bf1(NAT_C2W), nat_pf2(NAT_C2W))
                           : nat_go<NG_DW, 2, 64>(a, (unsigned)p.ns2, s);
    case NAT_C2X:     // dl1 = col2im(dl2 W2^T) * (l1 > 0), per stride-2 parity class
      if (w1t && nat_fuse_dx()) return 0;
      a.X = l1; a.dY = bws + p.dl2; a.Wt = P + L.off[N_L2W]; a.Y = bws + p.dl1;
      a.M = (int)(B * (NT1_O / 2) * (NT1_O / 2)); a.N = NT1_N; a.K = 2 * 2 * NT2_N;
      return nat_bf(NAT_C2X) ? nat_go_bf<NG_DX, 2, 32, 3>(a, 4, s, nat_bf1(NAT_C2X), nat_pf2(NAT_C2X))
                           : nat_go<NG_DX, 2, 32>(a, 4, s);
    case NAT_C1W:     // dW1 (+ db1) from the u8 planes (the input needs no gradient)
      a.sa = sa; a.dY = bws + p.dl1; a.slab = bws + p.s1; a.colsum = bws + p.c1;
      a.M = NT_K1; a.N = NT1_N; a.K = (int)(B * NT1_P); a.kchunk = p.kc1;
      return nat_bf(NAT_C1W) ? nat_go_bf<NG_DW1, 1, 32, 1>(a, (unsigned)p.ns1, s, nat_bf1(NAT_C1W), nat_pf2(NAT_C1W))
                           : nat_go<NG_DW1, 1, 32>(a, (unsigned)p.ns1, s);
    default:
      return a3c_set_error(A3C_ERR_INVALID, "a3c_nat_pass_launch", "unknown pass");
  }
}

// the rollout's tau snapshot and the backward's go (k_prep_fwd's duties, without the NIPS weight
// preparation)
__global__ void k_nat_prep(const int64_t* __restrict__ tau_src, int64_t* __restrict__ tau_dst, uint32_t* sig) {
  if (tau_dst) *tau_dst = *tau_src;
  if (sig) (void)__hip_atomic_fetch_add(sig, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
static int nat_w1_terms_launch(const NetLayout& L, const float* P, uint16_t* w1t, hipStream_t s) {
  // (the forward forms for k_nat_conv23, the dX forms only for k_nat_dx32)
  const int all = nat_fuse23() || nat_fuse_dx() ? 1 : 0;
  const int n = NT1_N * NT_K1 + (all ? NT2_N * NT_K2 + NT3_N * NT_K3 : 0) +
                (nat_fuse_dx() ? NT1_N * NT_X2 + NT2_N * NT_K3 : 0);
  hipLaunchKernelGGL(k_nat_w_terms, dim3((n + 255) / 256), dim3(256), 0, s, P + L.off[N_L1W], P + L.off[N_L2W],
                     P + L.off[N_L3W], w1t, all);
  A3C_CHECK(hipGetLastError());
  return 0;
}
int a3c_nat_prep_launch(const NetLayout& L, const float* P, uint16_t* w1t, const int64_t* tau_src, int64_t* tau_dst,
                        uint32_t* sig, hipStream_t s) {
  if (int rc = nat_w1_terms_launch(L, P, w1t, s)) return rc;
  hipLaunchKernelGGL(k_nat_prep, dim3(1), dim3(1), 0, s, tau_src, tau_src ? tau_dst : nullptr, sig);
  A3C_CHECK(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------------------
int a3c_nat_forward_launch(const NetLayout& L, const float* P, const StateAddr& sa, int64_t B, float* l1, float* l2,
                           float* l3, float* l4, float* z, const HeadSelect& sel, const uint16_t* w1t, float* ws,
                           hipStream_t s) {
  if (L.trunk != A3C_TRUNK_NATURE || B <= 0 || B * NT1_P > 0x7fffffffLL)
    return a3c_set_error(A3C_ERR_INVALID, "a3c_nat_forward", "nature trunk, 0 < B, B * 400 < 2^31");
  if (!w1t) {   // one-off forward: the weight terms into the workspace's tail first
    uint16_t* t = (uint16_t*)(ws + nat_fwd_slab_floats(B));
    if (int rc = nat_w1_terms_launch(L, P, t, s)) return rc;
    w1t = t;
  }
  const bool step_tail = sel.mode >= 0 && sel.env_on && sel.pool;   // the engine's rollout step
  const int fcs = fc_split(B);
  const bool fold_in_head = step_tail && fcs > 1 && !nat_bf(NAT_FCF) && nat_fold_head();
  for (int pass = NAT_C1F; pass <= (fold_in_head ? NAT_C3F : NAT_FCF); ++pass) {
    const int rc = a3c_nat_pass_launch(pass, L, P, sa, B, l1, l2, l3, l4, w1t, ws, nullptr, s);
    if (rc) return rc;
  }
  if (fold_in_head) {   // the fc's K-slice partials, folded by the head + act + screen kernel
    GemmArgs gf = {};
    gf.A = l3; gf.lda = NT_FLAT;
    gf.B = P + L.off[N_FCW]; gf.ldb = NT_FC;
    gf.C = l4; gf.ldc = NT_FC;
    gf.M = (int)B; gf.N = NT_FC; gf.K = NT_FLAT;
    gf.epi = EPI_BIAS_RELU; gf.bias = P + L.off[N_FCB];
    gf.nsplit = fcs; gf.slab = ws; gf.defer_reduce = 1;
    if (int rc = a3c_gemm(true, true, gf, s)) return rc;
    return a3c_head_screen_fold_launch(ws, fcs, P + L.off[N_FCB], l4, P + L.off[N_HW], P + L.off[N_HB],
                                       P + L.off[N_VW], P + L.off[N_VB], L.A, L.zs, B, z, sel, s);
  }
  if (step_tail)   // head + act + Environment.screen
    return a3c_head_screen_wide_launch(l4, P + L.off[N_HW], P + L.off[N_HB], P + L.off[N_VW], P + L.off[N_VB], L.A,
                                       L.zs, B, z, sel, s);
  hipLaunchKernelGGL(k_nat_head, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, s, l4, B, P + L.off[N_HW],
                     P + L.off[N_HB], P + L.off[N_VW], P + L.off[N_VB], L.A, L.zs, z, sel);
  A3C_CHECK(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------------------------------
// backward
// ---------------------------------------------------------------------------------------
// every tensor but the fc weights gets its gradient from a k_finalize segment
static bool nat_finalized(int t) { return t != N_FCW; }

int a3c_nat_fused_tab(const NetLayout& L, TensorTab* tt) {
  if (L.nt != N_NT) return -1;
  tt->n = L.nt;
  int nb = 0;
  for (int t = 0; t < L.nt; ++t) {
    tt->off[t] = L.off[t];
    tt->size[t] = L.size[t];
    tt->pb_first[t] = nb;
    tt->pb_count[t] = nat_finalized(t) ? FIN_X : (int)((L.size[t] + SS_CHUNK - 1) / SS_CHUNK);
    nb += tt->pb_count[t];
  }
  if (nb > SS_MAX_BLOCKS) return -1;
  tt->nblocks = nb;
  tt->total = L.total;
  return 0;
}

int a3c_nat_backward_launch(const NetLayout& L, const float* P, const StateAddr& sa, int64_t B, const float* l1,
                            const float* l2, const float* l3, const float* l4, const float* z,
                            const int32_t* actions, const float* target, float beta, int literal, float* grads,
                            float* loss_out, float* ws, hipStream_t s, const ReturnsArgs* ra_in, const SumsqFused* sf,
                            const uint16_t* wt) {
  if (L.trunk != A3C_TRUNK_NATURE || B <= 0 || B * NT1_P > 0x7fffffffLL)
    return a3c_set_error(A3C_ERR_INVALID, "a3c_nat_backward", "nature trunk, 0 < B, B * 400 < 2^31");
  ReturnsArgs ra = {};
  if (ra_in) ra = *ra_in;
  const NatPlan p = nat_plan(L, B);
  if (!wt) {   // one-off backward: the weight terms into the workspace first
    uint16_t* t = (uint16_t*)(ws + p.wprep);
    if (int rc = nat_w1_terms_launch(L, P, t, s)) return rc;
    wt = t;
  }
  float* dz = ws + p.dz;
  float* dl4 = ws + p.dl4;
  float* terms = ws + p.terms;
  // returns (fused), losses, dz, dl4 = (dz [W_p W_v]^T) * (l4 > 0)
  int rc = a3c_head_bwd_launch(NT_FC, L, z, actions, target, l4, P + L.off[N_HW], P + L.off[N_VW], beta, literal, B, dz,
                               dl4, terms, ra, 1, s);
  if (rc) return rc;
  // head weights: dW[512][zs] = l4^T dz (split-K folded by the finalize), db = colsum(dz)
  GemmArgs gh = {};
  gh.A = l4; gh.lda = NT_FC;
  gh.B = dz; gh.ldb = L.zs;
  gh.C = ws + p.hgrad; gh.ldc = L.zs;
  gh.M = NT_FC; gh.N = L.zs; gh.K = (int)B;
  gh.epi = EPI_STORE; gh.slab = ws + p.hslab; gh.nsplit = p.head_split; gh.colsum = ws + p.hcol;
  gh.defer_reduce = 1;
  rc = a3c_gemm(false, true, gh, s);
  if (rc) return rc;
  // fc weights: dW[3136][512] = l3^T dl4 straight into grads (split-K inside the workgroups), db = colsum
  if (nat_bf(NAT_FCW)) {   // bf16 terms, one reduction chain per tile straight into grads (+ db)
    NatGemm a = {};
    a.X = l3; a.dY = dl4; a.slab = grads + L.off[N_FCW]; a.colsum = ws + p.fccol;
    a.M = NT_FLAT; a.N = NT_FC; a.K = (int)B; a.kchunk = (int)B;
    rc = nat_go_bf<NG_DW, 4, 64, 3>(a, 1, s, nat_bf1(NAT_FCW), nat_pf2(NAT_FCW));
  } else {
  GemmArgs gf = {};
  gf.A = l3; gf.lda = NT_FLAT;
  gf.B = dl4; gf.ldb = NT_FC;
  gf.C = grads + L.off[N_FCW]; gf.ldc = NT_FC;
  gf.M = NT_FLAT; gf.N = NT_FC; gf.K = (int)B;
  gf.epi = EPI_STORE; gf.colsum = ws + p.fccol; gf.wg_split = 4; gf.xcd = 1;
  rc = a3c_gemm(false, true, gf, s);
  }
  if (rc) return rc;
  // dl3 = (dl4 W^T) * (l3 > 0)
  if (nat_bf(NAT_FCX)) {
    NatGemm a = {};
    a.X = l3; a.dY = dl4; a.Wt = P + L.off[N_FCW]; a.Y = ws + p.dl3;
    a.M = (int)B; a.N = NT_FLAT; a.K = NT_FC;
    rc = nat_go_bf<NG_DX, 4, 64, 3>(a, 1, s, nat_bf1(NAT_FCX), nat_pf2(NAT_FCX));
  } else {
  GemmArgs gd = {};
  gd.A = dl4; gd.lda = NT_FC;
  gd.B = P + L.off[N_FCW]; gd.ldb = NT_FC;
  gd.C = ws + p.dl3; gd.ldc = NT_FLAT;
  gd.M = (int)B; gd.N = NT_FLAT; gd.K = NT_FC;
  gd.epi = EPI_MASK; gd.mask = l3; gd.ldm = NT_FLAT; gd.nsplit = 1;
  rc = a3c_gemm(true, false, gd, s);
  }
  if (rc) return rc;
  for (int pass = NAT_C3W; pass <= NAT_C1W; ++pass) {
    rc = a3c_nat_pass_launch(pass, L, P, sa, B, l1, l2, l3, l4, wt, nullptr, ws, s);
    if (rc) return rc;
  }
  // the weight slabs in NAT_GROUPS fixed-order groups, then k_finalize: every segment, the loss
  // terms, the fused per-tensor norms and the lr schedule
  const int g1 = p.ns1 < NAT_GROUPS ? p.ns1 : NAT_GROUPS, g2 = p.ns2 < NAT_GROUPS ? p.ns2 : NAT_GROUPS,
            g3 = p.ns3 < NAT_GROUPS ? p.ns3 : NAT_GROUPS;
  rc = a3c_slab_group_launch(ws + p.s1, p.ns1, g1, (int64_t)NT_K1 * NT1_N, ws + p.g1, s);
  if (!rc) rc = a3c_slab_group_launch(ws + p.s2, p.ns2, g2, (int64_t)NT_K2 * NT2_N, ws + p.g2, s);
  if (!rc) rc = a3c_slab_group_launch(ws + p.s3, p.ns3, g3, (int64_t)NT_K3 * NT3_N, ws + p.g3, s);
  if (rc) return rc;
  FinalizeSegs fs = {};
  fs.dst = grads;
  auto seg = [&](const float* src, int64_t stride, int nsplit, int rows, int src_ld, int col0, int ncols, int tensor,
                 int dst_ld, float scale) {
    FinalizeSeg& q = fs.s[fs.n++];
    q.src = src; q.split_stride = stride; q.nsplit = nsplit; q.rows = rows; q.src_ld = src_ld;
    q.col0 = col0; q.ncols = ncols; q.dst_off = L.off[tensor]; q.dst_ld = dst_ld; q.scale = scale;
    q.slot = sf ? sf->tt->pb_first[tensor] : -1;
  };
  // the patch rows of conv1 are raw u8 pixels: dW1 takes the 1/255 of the input scaling here
  seg(ws + p.g1, (int64_t)NT_K1 * NT1_N, g1, 1, 0, 0, NT_K1 * NT1_N, N_L1W, 0, 1.0f / 255.0f);
  seg(ws + p.c1, NT1_N, p.ns1, 1, 0, 0, NT1_N, N_L1B, 0, 1.0f);
  seg(ws + p.g2, (int64_t)NT_K2 * NT2_N, g2, 1, 0, 0, NT_K2 * NT2_N, N_L2W, 0, 1.0f);
  seg(ws + p.c2, NT2_N, p.ns2, 1, 0, 0, NT2_N, N_L2B, 0, 1.0f);
  seg(ws + p.g3, (int64_t)NT_K3 * NT3_N, g3, 1, 0, 0, NT_K3 * NT3_N, N_L3W, 0, 1.0f);
  seg(ws + p.c3, NT3_N, p.ns3, 1, 0, 0, NT3_N, N_L3B, 0, 1.0f);
  seg(ws + p.fccol, NT_FC, 1, 1, 0, 0, NT_FC, N_FCB, 0, 1.0f);
  const float* hsrc = p.head_split > 1 ? ws + p.hslab : ws + p.hgrad;
  const int64_t hstride = (int64_t)NT_FC * L.zs;
  seg(hsrc, hstride, p.head_split, NT_FC, L.zs, 0, L.A, N_HW, L.A, 1.0f);
  seg(ws + p.hcol, L.zs, p.head_split, 1, 0, 0, L.A, N_HB, 0, 1.0f);
  seg(hsrc, hstride, p.head_split, NT_FC, L.zs, L.A, 1, N_VW, 1, 1.0f);
  seg(ws + p.hcol, L.zs, p.head_split, 1, 0, L.A, 1, N_VB, 0, 1.0f);
  int nsumblk = 0;
  if (sf) {
    fs.part = sf->part;
    fs.tt = *sf->tt;
    fs.op = *sf->op;
    fs.sum_c0[0] = 0;
    fs.sum_t[0] = N_FCW;
    fs.sum_c0[1] = fs.tt.pb_count[N_FCW];
    fs.nsum = 1;
    nsumblk = fs.sum_c0[1];
  }
  return a3c_finalize_launch(fs, nsumblk, terms, B, loss_out, s);
}

// ---------------------------------------------------------------------------------------
// C-ABI: the nature trunk as stateless per-op calls (include/a3c_hip.h), for src/network.py
// ---------------------------------------------------------------------------------------
static int nat_layout(const a3c_net_desc* net, NetLayout* L, const char* what) {
  if (a3c_make_layout(net, L) || L->trunk != A3C_TRUNK_NATURE)
    return a3c_set_error(A3C_ERR_INVALID, what, "a nature-trunk net description (a3c, no LSTM)");
  return 0;
}
static StateAddr nat_states(const uint8_t* states, int64_t B) {
  StateAddr sa;
  sa.base = states; sa.env_stride = (int64_t)HIST * PLANE; sa.plane_bytes = PLANE;
  sa.E = (int)B; sa.R = HIST; sa.L = HIST; sa.tau_offset = HIST - 1; sa.tau_ptr = nullptr;
  return sa;
}
static float* nat_align(void* ws) { return (float*)(((uintptr_t)ws + 255) & ~(uintptr_t)255); }

extern "C" int a3c_nature_workspace_bytes(const a3c_net_desc* net, int64_t B, int64_t* bytes) {
  NetLayout L;
  if (int rc = nat_layout(net, &L, "a3c_nature_workspace_bytes")) return rc;
  if (B < 1 || !bytes) return a3c_set_error(A3C_ERR_INVALID, "a3c_nature_workspace_bytes", "bad argument");
  const int64_t f = a3c_nat_fwd_ws_floats(B), b = a3c_nat_bwd_ws_floats(L, B);
  *bytes = (f > b ? f : b) * 4 + 256;
  return 0;
}

extern "C" int a3c_nature_forward(const a3c_net_desc* net, const float* params, const uint8_t* states, int64_t B,
                                  float* l1, float* l2, float* l3, float* l4, float* z, void* workspace,
                                  void* stream) {
  NetLayout L;
  if (int rc = nat_layout(net, &L, "a3c_nature_forward")) return rc;
  if (!params || !states || !l1 || !l2 || !l3 || !l4 || !z || !workspace || B < 0 || B * NT1_P > 0x7fffffffLL ||
      (((uintptr_t)params | (uintptr_t)l1 | (uintptr_t)l2 | (uintptr_t)l3 | (uintptr_t)l4) & 15))
    return a3c_set_error(A3C_ERR_INVALID, "a3c_nature_forward", "bad argument");
  if (B == 0) return 0;
  HeadSelect sel = {};
  sel.mode = -1;
  sel.E = 1;
  return a3c_nat_forward_launch(L, params, nat_states(states, B), B, l1, l2, l3, l4, z, sel, nullptr,
                                nat_align(workspace), (hipStream_t)stream);
}

extern "C" int a3c_nature_loss_backward(const a3c_net_desc* net, const float* params, const uint8_t* states,
                                        int64_t B, const float* l1, const float* l2, const float* l3, const float* l4,
                                        const float* z, const int32_t* actions, const float* target, float beta,
                                        int literal_adv, float* grads, float* loss_out, void* workspace,
                                        void* stream) {
  NetLayout L;
  if (int rc = nat_layout(net, &L, "a3c_nature_loss_backward")) return rc;
  if (!params || !states || !l1 || !l2 || !l3 || !l4 || !z || !actions || !target || !grads || !workspace ||
      B <= 0 || B * NT1_P > 0x7fffffffLL || (((uintptr_t)grads | (uintptr_t)l3 | (uintptr_t)l4) & 15))
    return a3c_set_error(A3C_ERR_INVALID, "a3c_nature_loss_backward", "bad argument");
  return a3c_nat_backward_launch(L, params, nat_states(states, B), B, l1, l2, l3, l4, z, actions, target, beta,
                                 literal_adv, grads, loss_out, nat_align(workspace), (hipStream_t)stream, nullptr,
                                 nullptr, nullptr);
}

// K1: Environment.screen (reference src/environment.py:95-99) as a block-cooperative
// device routine: fp64 luminance with u8 truncation, then Pillow's two-pass BILINEAR
// fixed-point resample (what scipy<1.3 imresize runs, environment.py:5-8,99).
// Bit-exact against tests/golden/screen_golden.npz (generated from the reference).
#pragma once
#include "a3c_common.h"

#define A3C_MAXK 16
#define A3C_PRECISION_BITS 22

struct PreGeom {
  int in_h, in_w, out_h, out_w;
  int kh, kv;          // horizontal / vertical ksize (host: ceil(support)*2+1)
};

// Pillow precompute_coeffs + normalize_coeffs_8bpc for ONE output index.  Evaluated in
// IEEE double with contraction off so every operation rounds exactly as the C code does.
__device__ inline void a3c_pillow_coeff(int in_size, int out_size, int ksize, int xx,
                                        int* bounds2, int* kk) {
#pragma clang fp contract(off)
  double scale = (double)(float)in_size / (double)out_size;
  double filterscale = scale < 1.0 ? 1.0 : scale;
  double support = 1.0 * filterscale;
  double center = 0.0 + (xx + 0.5) * scale;
  double ss = 1.0 / filterscale;
  int xmin = (int)(center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + support + 0.5);
  if (xmax > in_size) xmax = in_size;
  xmax -= xmin;
  double w[A3C_MAXK];
  double ww = 0.0;
  for (int x = 0; x < ksize; ++x) w[x] = 0.0;
  for (int x = 0; x < xmax && x < A3C_MAXK; ++x) {
    double t = ((double)(x + xmin) - center + 0.5) * ss;
    if (t < 0.0) t = -t;
    double f = t < 1.0 ? 1.0 - t : 0.0;
    w[x] = f;
    ww += f;
  }
  for (int x = 0; x < xmax && x < A3C_MAXK; ++x)
    if (ww != 0.0) w[x] = w[x] / ww;
  for (int x = 0; x < ksize; ++x) {
    double v = w[x] * (double)(1 << A3C_PRECISION_BITS);
    kk[x] = w[x] < 0 ? (int)(-0.5 + v) : (int)(0.5 + v);
  }
  bounds2[0] = xmin;
  bounds2[1] = xmax;
}

__device__ inline uint8_t a3c_clip8(int in) {
  if (in >= (1 << A3C_PRECISION_BITS << 8)) return 255;
  if (in <= 0) return 0;
  return (uint8_t)(in >> A3C_PRECISION_BITS);
}

// luminance of one pixel: numpy evaluates 0.2126*R + 0.7152*G + 0.0722*B in float64,
// left to right, no fused multiply-add; astype(uint8) truncates.
// (__dadd_rn/__dmul_rn are plain +/* in clang's HIP headers and get contracted to v_fmac_f64
// under hipcc's default -ffp-contract=fast: contraction must be switched off explicitly.)
__device__ inline uint32_t a3c_lum(uint32_t r, uint32_t g, uint32_t b) {
#pragma clang fp contract(off)
  double y = 0.2126 * (double)r + 0.7152 * (double)g + 0.0722 * (double)b;
  return (uint32_t)(int)y & 255u;
}

__host__ __device__ inline size_t a3c_pre_smem_bytes(const PreGeom& g) {
  size_t coef = (size_t)g.out_w * (2 + g.kh) * 4 + (size_t)g.out_h * (2 + g.kv) * 4;
  coef = (coef + 15) & ~(size_t)15;
  size_t gray = ((size_t)g.in_h * g.in_w + 15) & ~(size_t)15;
  size_t tmp = ((size_t)g.in_h * g.out_w + 15) & ~(size_t)15;
  return coef + gray + tmp;
}

// Whole block (blockDim.x threads) converts one RGB frame [in_h][in_w][3] into out[out_h][out_w].
__device__ inline void a3c_preprocess_block(const uint8_t* __restrict__ rgb, uint8_t* __restrict__ out,
                                            const PreGeom& g, uint8_t* smem) {
  const int tid = threadIdx.x, nt = blockDim.x;
  int* hb = (int*)smem;                       // [out_w][2]
  int* hk = hb + 2 * g.out_w;                 // [out_w][kh]
  int* vb = hk + g.kh * g.out_w;              // [out_h][2]
  int* vk = vb + 2 * g.out_h;                 // [out_h][kv]
  size_t coef = (size_t)g.out_w * (2 + g.kh) * 4 + (size_t)g.out_h * (2 + g.kv) * 4;
  coef = (coef + 15) & ~(size_t)15;
  uint8_t* gray = smem + coef;                                       // [in_h][in_w]
  uint8_t* tmp = gray + (((size_t)g.in_h * g.in_w + 15) & ~(size_t)15);  // [rows][out_w]

  for (int i = tid; i < g.out_w + g.out_h; i += nt) {
    if (i < g.out_w) a3c_pillow_coeff(g.in_w, g.out_w, g.kh, i, hb + 2 * i, hk + g.kh * i);
    else {
      int j = i - g.out_w;
      a3c_pillow_coeff(g.in_h, g.out_h, g.kv, j, vb + 2 * j, vk + g.kv * j);
    }
  }

  // ---- luminance (fp64, truncating) into LDS ----
  const int npix = g.in_h * g.in_w;
  if ((((uintptr_t)rgb) & 15) == 0 && (npix & 15) == 0) {
    const uint4* src = (const uint4*)rgb;
    for (int u = tid; u < npix / 16; u += nt) {
      uint4 a = src[3 * u], b = src[3 * u + 1], c = src[3 * u + 2];
      uint32_t w[12] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w};
      uint32_t o[4] = {0, 0, 0, 0};
#pragma unroll
      for (int p = 0; p < 16; ++p) {
        int i0 = 3 * p, i1 = 3 * p + 1, i2 = 3 * p + 2;
        uint32_t r = (w[i0 >> 2] >> (8 * (i0 & 3))) & 255u;
        uint32_t gg = (w[i1 >> 2] >> (8 * (i1 & 3))) & 255u;
        uint32_t bb = (w[i2 >> 2] >> (8 * (i2 & 3))) & 255u;
        o[p >> 2] |= a3c_lum(r, gg, bb) << (8 * (p & 3));
      }
      *(uint4*)(gray + 16 * u) = make_uint4(o[0], o[1], o[2], o[3]);
    }
  } else {
    for (int p = tid; p < npix; p += nt)
      gray[p] = (uint8_t)a3c_lum(rgb[3 * p], rgb[3 * p + 1], rgb[3 * p + 2]);
  }
  __syncthreads();

  // ---- horizontal pass: rows [y0, y1) of the source into tmp ----
  const int y0 = vb[0];
  const int y1 = vb[2 * (g.out_h - 1)] + vb[2 * (g.out_h - 1) + 1];
  const int rows = y1 - y0;
  for (int i = tid; i < rows * g.out_w; i += nt) {
    int r = i / g.out_w, xx = i - r * g.out_w;
    int xmin = hb[2 * xx], cnt = hb[2 * xx + 1];
    const uint8_t* src = gray + (size_t)(r + y0) * g.in_w + xmin;
    const int* k = hk + g.kh * xx;
    int ss = 1 << (A3C_PRECISION_BITS - 1);
    for (int x = 0; x < cnt; ++x) ss += (int)src[x] * k[x];
    tmp[(size_t)r * g.out_w + xx] = a3c_clip8(ss);
  }
  __syncthreads();

  // ---- vertical pass into the destination ----
  for (int i = tid; i < g.out_h * g.out_w; i += nt) {
    int yy = i / g.out_w, xx = i - yy * g.out_w;
    int ymin = vb[2 * yy] - y0, cnt = vb[2 * yy + 1];
    const int* k = vk + g.kv * yy;
    int ss = 1 << (A3C_PRECISION_BITS - 1);
    for (int y = 0; y < cnt; ++y) ss += (int)tmp[(size_t)(ymin + y) * g.out_w + xx] * k[y];
    out[i] = a3c_clip8(ss);
  }
}

// host-side ksize of Pillow's bilinear filter
inline int a3c_pillow_ksize(int in_size, int out_size) {
  double scale = (double)(float)in_size / (double)out_size;
  double filterscale = scale < 1.0 ? 1.0 : scale;
  double support = 1.0 * filterscale;
  int c = (int)support;
  if ((double)c < support) c += 1;
  return c * 2 + 1;
}

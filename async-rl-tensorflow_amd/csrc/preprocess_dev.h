// K1: Environment.screen (reference src/environment.py:49-53) as a block-cooperative
// device routine: fp64 luminance with u8 truncation, then Pillow's two-pass BILINEAR
// fixed-point resample (what scipy<1.3 imresize runs, environment.py:5-8,99).
// Bit-exact against tests/golden/screen_golden.npz (generated from the reference).
//
// Work split: a frame's output rows are cut into `parts` bands; one workgroup produces one
// band.  It stages the contiguous source-row range the band needs (RGB, 16-byte coalesced
// loads) in LDS, converts it to luminance, runs the horizontal pass over those rows only and
// the vertical pass for its band (Pillow's horizontal-first order, so results are identical to
// the whole-frame computation).
#pragma once
#include "a3c_common.h"

#define A3C_MAXK 16
#define A3C_PRECISION_BITS 22

struct PreGeom {
  int in_h, in_w, out_h, out_w;
  int kh, kv;          // horizontal / vertical ksize (host: ceil(support)*2+1)
  int parts;           // output-row bands per frame (= workgroups per frame)
  int rows_per;        // output rows per band
  int max_src;         // upper bound of source rows a band reads (LDS sizing)
};

__device__ inline double a3c_bilinear_tap(int x, int xmin, double center, double ss) {
#pragma clang fp contract(off)
  double t = ((double)(x + xmin) - center + 0.5) * ss;
  if (t < 0.0) t = -t;
  return t < 1.0 ? 1.0 - t : 0.0;
}

// bounds (xmin, count) of one output index: the integer half of precompute_coeffs
__device__ inline void a3c_pillow_bounds(int in_size, int out_size, int xx, int* xmin_out, int* cnt_out) {
#pragma clang fp contract(off)
  double scale = (double)(float)in_size / (double)out_size;
  double filterscale = scale < 1.0 ? 1.0 : scale;
  double support = 1.0 * filterscale;
  double center = 0.0 + (xx + 0.5) * scale;
  int xmin = (int)(center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + support + 0.5);
  if (xmax > in_size) xmax = in_size;
  *xmin_out = xmin;
  *cnt_out = xmax - xmin;
}

// Pillow precompute_coeffs + normalize_coeffs_8bpc for ONE output index, evaluated in IEEE
// double with contraction off so every operation rounds as the C code does (the weights are
// recomputed instead of stored: no per-thread scratch array).
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
  double ww = 0.0;
  for (int x = 0; x < xmax; ++x) ww += a3c_bilinear_tap(x, xmin, center, ss);
  for (int x = 0; x < ksize; ++x) {
    double w = 0.0;
    if (x < xmax) {
      w = a3c_bilinear_tap(x, xmin, center, ss);
      if (ww != 0.0) w = w / ww;
    }
    double v = w * (double)(1 << A3C_PRECISION_BITS);
    kk[x] = w < 0 ? (int)(-0.5 + v) : (int)(0.5 + v);
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

__host__ __device__ inline size_t a3c_align16(size_t x) { return (x + 15) & ~(size_t)15; }

__host__ __device__ inline size_t a3c_pre_coef_bytes(const PreGeom& g) {
  return a3c_align16((size_t)g.out_w * (2 + g.kh) * 4 + (size_t)g.rows_per * (2 + g.kv) * 4);
}

__host__ __device__ inline size_t a3c_pre_smem_bytes(const PreGeom& g) {
  const size_t px = (size_t)g.max_src * g.in_w;
  return a3c_pre_coef_bytes(g) + a3c_align16(px * 3) + a3c_align16(px) + a3c_align16((size_t)g.max_src * g.out_w);
}

// One workgroup produces output rows [part*rows_per, ...) of one frame.
__device__ inline void a3c_preprocess_part(const uint8_t* __restrict__ rgb, uint8_t* __restrict__ out,
                                           const PreGeom& g, int part, uint8_t* smem) {
  const int tid = threadIdx.x, nt = blockDim.x;
  const int yy0 = part * g.rows_per;
  const int nrows = min(g.out_h, yy0 + g.rows_per) - yy0;
  if (nrows <= 0) return;
  int* hb = (int*)smem;                       // [out_w][2]
  int* hk = hb + 2 * g.out_w;                 // [out_w][kh]
  int* vb = hk + g.kh * g.out_w;              // [rows_per][2]
  int* vk = vb + 2 * g.rows_per;              // [rows_per][kv]
  const size_t pxmax = (size_t)g.max_src * g.in_w;
  uint8_t* raw = smem + a3c_pre_coef_bytes(g);          // [src rows][in_w][3]
  uint8_t* gray = raw + a3c_align16(pxmax * 3);          // [src rows][in_w]
  uint8_t* tmp = gray + a3c_align16(pxmax);              // [src rows][out_w]

  // source rows of the band from the bounds alone (every thread, no barrier), so the RGB loads
  // can be in flight while the weights are computed
  int y0, c0, yl, cl;
  a3c_pillow_bounds(g.in_h, g.out_h, yy0, &y0, &c0);
  a3c_pillow_bounds(g.in_h, g.out_h, yy0 + nrows - 1, &yl, &cl);
  const int y1 = yl + cl;
  const int srows = y1 - y0;                 // <= max_src by construction of max_src
  const int npix = srows * g.in_w;
  const uint8_t* src = rgb + (size_t)y0 * g.in_w * 3;
  const int nbytes = npix * 3;
  const bool vec = ((((uintptr_t)src) | (uintptr_t)nbytes) & 15) == 0;
  const int n16 = nbytes >> 4;
  uint4 r0 = make_uint4(0, 0, 0, 0), r1 = r0, r2 = r0, r3 = r0;
  if (vec) {
    const uint4* s4 = (const uint4*)src;
    if (tid < n16) r0 = s4[tid];
    if (tid + nt < n16) r1 = s4[tid + nt];
    if (tid + 2 * nt < n16) r2 = s4[tid + 2 * nt];
    if (tid + 3 * nt < n16) r3 = s4[tid + 3 * nt];
  }
  for (int i = tid; i < g.out_w + nrows; i += nt) {
    if (i < g.out_w) a3c_pillow_coeff(g.in_w, g.out_w, g.kh, i, hb + 2 * i, hk + g.kh * i);
    else {
      const int j = i - g.out_w;
      a3c_pillow_coeff(g.in_h, g.out_h, g.kv, yy0 + j, vb + 2 * j, vk + g.kv * j);
    }
  }
  if (vec) {
    uint4* d4 = (uint4*)raw;
    const uint4* s4 = (const uint4*)src;
    if (tid < n16) d4[tid] = r0;
    if (tid + nt < n16) d4[tid + nt] = r1;
    if (tid + 2 * nt < n16) d4[tid + 2 * nt] = r2;
    if (tid + 3 * nt < n16) d4[tid + 3 * nt] = r3;
    for (int i = tid + 4 * nt; i < n16; i += nt) d4[i] = s4[i];
  } else {
    for (int i = tid; i < nbytes; i += nt) raw[i] = src[i];
  }
  __syncthreads();

  // ---- luminance (fp64, truncating): 16 pixels = 48 bytes per thread-iteration ----
  if ((npix & 15) == 0) {
    for (int u = tid; u < npix / 16; u += nt) {
      const uint4* r4 = (const uint4*)(raw + 48 * u);   // stride 48 B: conflict-free b128 reads
      uint4 a = r4[0], b = r4[1], c = r4[2];
      uint32_t w[12] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w};
      uint32_t o[4] = {0, 0, 0, 0};
#pragma unroll
      for (int p = 0; p < 16; ++p) {
        const int i0 = 3 * p, i1 = 3 * p + 1, i2 = 3 * p + 2;
        const uint32_t r = (w[i0 >> 2] >> (8 * (i0 & 3))) & 255u;
        const uint32_t gg = (w[i1 >> 2] >> (8 * (i1 & 3))) & 255u;
        const uint32_t bb = (w[i2 >> 2] >> (8 * (i2 & 3))) & 255u;
        o[p >> 2] |= a3c_lum(r, gg, bb) << (8 * (p & 3));
      }
      *(uint4*)(gray + 16 * u) = make_uint4(o[0], o[1], o[2], o[3]);
    }
  } else {
    for (int p = tid; p < npix; p += nt) gray[p] = (uint8_t)a3c_lum(raw[3 * p], raw[3 * p + 1], raw[3 * p + 2]);
  }
  __syncthreads();

  // ---- horizontal pass over the staged rows ----
  for (int i = tid; i < srows * g.out_w; i += nt) {
    const int r = i / g.out_w, xx = i - r * g.out_w;
    const int xmin = hb[2 * xx], cnt = hb[2 * xx + 1];
    const uint8_t* s = gray + (size_t)r * g.in_w + xmin;
    const int* k = hk + g.kh * xx;
    int acc = 1 << (A3C_PRECISION_BITS - 1);
    for (int x = 0; x < cnt; ++x) acc += (int)s[x] * k[x];
    tmp[(size_t)r * g.out_w + xx] = a3c_clip8(acc);
  }
  __syncthreads();

  // ---- vertical pass for this band ----
  uint8_t* o = out + (size_t)yy0 * g.out_w;
  for (int i = tid; i < nrows * g.out_w; i += nt) {
    const int yy = i / g.out_w, xx = i - yy * g.out_w;
    const int ymin = vb[2 * yy] - y0, cnt = vb[2 * yy + 1];
    const int* k = vk + g.kv * yy;
    int acc = 1 << (A3C_PRECISION_BITS - 1);
    for (int y = 0; y < cnt; ++y) acc += (int)tmp[(size_t)(ymin + y) * g.out_w + xx] * k[y];
    o[i] = a3c_clip8(acc);
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

// geometry with `parts` output bands per frame; max_src is a safe upper bound of the source
// rows one band touches: rows_per*scale + 2*ceil(support) + 2.
inline PreGeom a3c_make_geom_parts(int in_h, int in_w, int out_h, int out_w, int parts) {
  PreGeom g;
  g.in_h = in_h; g.in_w = in_w; g.out_h = out_h; g.out_w = out_w;
  g.kh = a3c_pillow_ksize(in_w, out_w);
  g.kv = a3c_pillow_ksize(in_h, out_h);
  if (parts < 1) parts = 1;
  if (parts > out_h) parts = out_h;
  g.parts = parts;
  g.rows_per = (out_h + parts - 1) / parts;
  double scale = (double)in_h / (double)out_h;
  int sup = (g.kv - 1) / 2;
  int m = (int)(g.rows_per * (scale > 1.0 ? scale : 1.0)) + 2 * sup + 2;
  g.max_src = m < in_h ? m : in_h;
  return g;
}

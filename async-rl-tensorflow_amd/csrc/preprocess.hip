// K1 Environment.screen + K2 History kernels and their C-ABI entry points.
#include <cstdlib>
#include "preprocess_dev.h"
#include "screen_atari.h"
#include "../../include/a3c_hip.h"

// grid (parts, n): workgroup (q, i) produces output band q of frame i
__global__ void __launch_bounds__(256) k_preprocess(const uint8_t* __restrict__ rgb,
                                                    const int32_t* __restrict__ frame_idx,
                                                    uint8_t* __restrict__ out, int64_t out_stride,
                                                    PreGeom g) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int64_t i = blockIdx.y;
  const int64_t fb = (int64_t)g.in_h * g.in_w * 3;
  const int64_t f = frame_idx ? (int64_t)frame_idx[i] : i;
  a3c_preprocess_part(rgb + f * fb, out + i * out_stride, g, blockIdx.x, smem);
}

// specialised Atari geometry: grid (84/ROWS bands, n)
template <int ROWS>
__global__ void __launch_bounds__(256) k_screen_atari(const uint8_t* __restrict__ rgb,
                                                      const int32_t* __restrict__ frame_idx,
                                                      uint8_t* __restrict__ out, int64_t out_stride) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int64_t i = blockIdx.y;
  const int64_t f = frame_idx ? (int64_t)frame_idx[i] : i;
  atari::screen_band<ROWS>(rgb + f * (atari::IH * atari::IW * 3), out + i * out_stride, blockIdx.x, smem);
}

template <int ROWS>
static void launch_atari(const uint8_t* rgb, const int32_t* idx, int64_t n, uint8_t* out, int64_t stride, hipStream_t s) {
  hipLaunchKernelGGL(k_screen_atari<ROWS>, dim3((atari::OH + ROWS - 1) / ROWS, (unsigned)n), dim3(256),
                     atari::Smem<ROWS>::BYTES, s, rgb, idx, out, stride);
}

// luminance step of Environment.screen alone (environment.py:51-52), the exact integer form the
// Atari kernel uses: out[i] = truncated fp64 0.2126 R + 0.7152 G + 0.0722 B of pixel i
// (groups of 4 pixels through atari::lum4 when the buffers are 4-byte aligned, else per pixel).
__global__ void k_luminance(const uint8_t* __restrict__ rgb, int64_t npix, uint8_t* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x, t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t done = 0;
  if ((((uintptr_t)rgb | (uintptr_t)out) & 3) == 0) {
    const int64_t ng = npix / 4;
    for (int64_t g = t0; g < ng; g += stride) {
      const uint32_t* s = (const uint32_t*)(rgb + 12 * g);
      ((uint32_t*)out)[g] = atari::lum4(s[0], s[1], s[2]);
    }
    done = 4 * ng;
  }
  for (int64_t p = done + t0; p < npix; p += stride)
    out[p] = (uint8_t)atari::lum_exact(rgb[3 * p], rgb[3 * p + 1], rgb[3 * p + 2]);
}

extern "C" int a3c_luminance_u8(const uint8_t* rgb, int64_t npix, uint8_t* out, void* stream) {
  if (!rgb || !out || npix < 0) return a3c_set_error(A3C_ERR_INVALID, "a3c_luminance_u8", "bad argument");
  if (npix == 0) return 0;
  hipLaunchKernelGGL(k_luminance, dim3(4096), dim3(256), 0, (hipStream_t)stream, rgb, npix, out);
  A3C_CHECK(hipGetLastError());
  return 0;
}

int a3c_screen_rows() {
  static int rows = [] {
    int r = (int)A3C_AB_KNOB("A3C_PRE_ROWS", 14);    // tuning knob (tools/microbench_preprocess.py)
    return (r == 7 || r == 12 || r == 14 || r == 21 || r == 28 || r == 42) ? r : 14;
  }();
  return rows;
}

int a3c_launch_screen_atari(const uint8_t* rgb, const int32_t* idx, int64_t n, uint8_t* out, int64_t stride,
                            hipStream_t s) {
  switch (a3c_screen_rows()) {
    case 7: launch_atari<7>(rgb, idx, n, out, stride, s); break;
    case 21: launch_atari<21>(rgb, idx, n, out, stride, s); break;
    case 28: launch_atari<28>(rgb, idx, n, out, stride, s); break;
    case 42: launch_atari<42>(rgb, idx, n, out, stride, s); break;
    case 12: launch_atari<12>(rgb, idx, n, out, stride, s); break;
    default: launch_atari<14>(rgb, idx, n, out, stride, s); break;
  }
  A3C_CHECK(hipGetLastError());
  return 0;
}

int a3c_launch_preprocess(const uint8_t* rgb, const int32_t* frame_idx, int64_t n, const PreGeom& g,
                          uint8_t* out, int64_t out_stride, hipStream_t s) {
  if (n <= 0) return 0;
  if (g.in_h == atari::IH && g.in_w == atari::IW && g.out_h == atari::OH && g.out_w == atari::OW &&
      (((uintptr_t)rgb) & 15) == 0 && n <= 65535)
    return a3c_launch_screen_atari(rgb, frame_idx, n, out, out_stride, s);
  size_t sm = a3c_pre_smem_bytes(g);
  if (sm > 160 * 1024) return a3c_set_error(A3C_ERR_INVALID, "a3c_preprocess_u8", "frame too large for LDS");
  if (n > 65535) {   // grid.y limit: chunk
    for (int64_t o = 0; o < n; o += 65535) {
      int64_t m = n - o < 65535 ? n - o : 65535;
      int rc = a3c_launch_preprocess(frame_idx ? rgb : rgb + o * (int64_t)g.in_h * g.in_w * 3,
                                     frame_idx ? frame_idx + o : nullptr, m, g, out + o * out_stride, out_stride, s);
      if (rc) return rc;
    }
    return 0;
  }
  hipLaunchKernelGGL(k_preprocess, dim3(g.parts, (unsigned)n), dim3(256), sm, s, rgb, frame_idx, out, out_stride, g);
  A3C_CHECK(hipGetLastError());
  return 0;
}

// output bands per frame for the standalone C-ABI path (A3C_PRE_PARTS overrides: tuning knob)
PreGeom a3c_make_geom(int in_h, int in_w, int out_h, int out_w) {
  static int parts = [] {
    int p = (int)A3C_AB_KNOB("A3C_PRE_PARTS", 8);
    return p > 0 ? p : 8;
  }();
  return a3c_make_geom_parts(in_h, in_w, out_h, out_w, parts);
}

extern "C" int a3c_preprocess_u8(const uint8_t* rgb, const int32_t* frame_idx, int64_t n, int in_h,
                                 int in_w, uint8_t* out, int64_t out_stride, int out_h, int out_w,
                                 void* stream) {
  if (!rgb || !out || in_h <= 0 || in_w <= 0 || out_h <= 0 || out_w <= 0 || n < 0)
    return a3c_set_error(A3C_ERR_INVALID, "a3c_preprocess_u8", "bad argument");
  PreGeom g = a3c_make_geom(in_h, in_w, out_h, out_w);
  if (g.kh > A3C_MAXK || g.kv > A3C_MAXK)
    return a3c_set_error(A3C_ERR_INVALID, "a3c_preprocess_u8", "downscale ratio too large");
  return a3c_launch_preprocess(rgb, frame_idx, n, g, out, out_stride, (hipStream_t)stream);
}

// ---- K2 History.add / reset (history.py:13-18) ------------------------------------------
// one block per history; planes moved with 16-byte accesses when aligned.
__global__ void __launch_bounds__(256) k_history_push(uint8_t* __restrict__ hist,
                                                      const uint8_t* __restrict__ screens,
                                                      const uint8_t* __restrict__ reset_mask,
                                                      int L, int64_t hw) {
  const int64_t i = blockIdx.x;
  uint8_t* h = hist + i * L * hw;
  const uint8_t* s = screens + i * hw;
  const bool reset = reset_mask && reset_mask[i];
  const bool vec = ((((uintptr_t)h) | ((uintptr_t)s)) & 15) == 0 && (hw & 15) == 0;
  if (vec) {
    const int64_t n16 = hw / 16;
    // each thread owns chunk j of every plane: shifting plane c+1 -> c in increasing c
    // reads every source before it is overwritten.
    for (int64_t j = threadIdx.x; j < n16; j += blockDim.x) {
      for (int c = 0; c + 1 < L; ++c) {
        uint4 v = reset ? make_uint4(0, 0, 0, 0) : ((const uint4*)(h + (c + 1) * hw))[j];
        ((uint4*)(h + c * hw))[j] = v;
      }
      ((uint4*)(h + (L - 1) * hw))[j] = ((const uint4*)s)[j];
    }
  } else {
    for (int64_t j = threadIdx.x; j < hw; j += blockDim.x) {
      for (int c = 0; c + 1 < L; ++c) h[c * hw + j] = reset ? 0 : h[(c + 1) * hw + j];
      h[(L - 1) * hw + j] = s[j];
    }
  }
}

extern "C" int a3c_history_push(uint8_t* hist, const uint8_t* screens, const uint8_t* reset_mask,
                                int64_t n, int L, int64_t hw, void* stream) {
  if (!hist || !screens || L <= 0 || hw <= 0 || n < 0)
    return a3c_set_error(A3C_ERR_INVALID, "a3c_history_push", "bad argument");
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_history_push, dim3((unsigned)n), dim3(256), 0, (hipStream_t)stream, hist,
                     screens, reset_mask, L, hw);
  A3C_CHECK(hipGetLastError());
  return 0;
}

// ---- History.get (history.py:20-24): float32, NHWC transpose or NCHW --------------------
__global__ void k_history_get(const uint8_t* __restrict__ hist, int64_t total, int L, int h, int w,
                              int nhwc, float* __restrict__ out) {
  int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int64_t hw = (int64_t)h * w;
  if (nhwc) {
    // out[i][y][x][c]
    int c = (int)(idx % L);
    int64_t p = idx / L;
    int64_t yx = p % hw, i = p / hw;
    out[idx] = (float)hist[(i * L + c) * hw + yx];
  } else {
    out[idx] = (float)hist[idx];
  }
}

extern "C" int a3c_history_get_f32(const uint8_t* hist, int64_t n, int L, int h, int w, int nhwc,
                                   float* out, void* stream) {
  if (!hist || !out || n < 0 || L <= 0 || h <= 0 || w <= 0)
    return a3c_set_error(A3C_ERR_INVALID, "a3c_history_get_f32", "bad argument");
  int64_t total = n * L * (int64_t)h * w;
  if (total == 0) return 0;
  hipLaunchKernelGGL(k_history_get, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, hist, total, L, h, w, nhwc, out);
  A3C_CHECK(hipGetLastError());
  return 0;
}

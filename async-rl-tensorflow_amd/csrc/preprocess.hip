// K1 Environment.screen + K2 History kernels and their C-ABI entry points.
#include "preprocess_dev.h"
#include "../../include/a3c_hip.h"

__global__ void __launch_bounds__(256) k_preprocess(const uint8_t* __restrict__ rgb,
                                                    const int32_t* __restrict__ frame_idx,
                                                    uint8_t* __restrict__ out, int64_t out_stride,
                                                    PreGeom g) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int64_t i = blockIdx.x;
  const int64_t fb = (int64_t)g.in_h * g.in_w * 3;
  const int64_t f = frame_idx ? (int64_t)frame_idx[i] : i;
  a3c_preprocess_block(rgb + f * fb, out + i * out_stride, g, smem);
}

int a3c_launch_preprocess(const uint8_t* rgb, const int32_t* frame_idx, int64_t n, const PreGeom& g,
                          uint8_t* out, int64_t out_stride, hipStream_t s) {
  if (n <= 0) return 0;
  size_t sm = a3c_pre_smem_bytes(g);
  if (sm > 160 * 1024) return a3c_set_error(A3C_ERR_INVALID, "a3c_preprocess_u8", "frame too large for LDS");
  hipLaunchKernelGGL(k_preprocess, dim3((unsigned)n), dim3(256), sm, s, rgb, frame_idx, out, out_stride, g);
  A3C_CHECK(hipGetLastError());
  return 0;
}

PreGeom a3c_make_geom(int in_h, int in_w, int out_h, int out_w) {
  PreGeom g;
  g.in_h = in_h; g.in_w = in_w; g.out_h = out_h; g.out_w = out_w;
  g.kh = a3c_pillow_ksize(in_w, out_w);
  g.kv = a3c_pillow_ksize(in_h, out_h);
  return g;
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

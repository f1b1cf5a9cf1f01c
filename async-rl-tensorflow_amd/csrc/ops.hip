// Generic layer ops for the ops.py drop-in (reference src/ops.py:4-46): VALID conv2d with TF's
// [kh,kw,cin,cout] weights in NHWC or NCHW (ops.py:13-28) and a strided fp32 matmul for
// ``linear`` (ops.py:32-46).  Off the hot path (the NIPS trunk uses the fused MFMA kernels);
// these serve arbitrary shapes (e.g. network.py's "nature" trunk) with autograd in the Python
// mirror.  Plain fp32 FMA loops, one thread per output element, fixed summation order.
#include "a3c_common.h"
#include "../../include/a3c_hip.h"

struct ConvShape { int N, H, W, C, KH, KW, SH, SW, OC, OH, OW, nhwc; };

__device__ inline int64_t x_index(const ConvShape& s, int n, int y, int x, int c) {
  return s.nhwc ? (((int64_t)n * s.H + y) * s.W + x) * s.C + c : (((int64_t)n * s.C + c) * s.H + y) * s.W + x;
}
__device__ inline int64_t y_index(const ConvShape& s, int n, int y, int x, int c) {
  return s.nhwc ? (((int64_t)n * s.OH + y) * s.OW + x) * s.OC + c : (((int64_t)n * s.OC + c) * s.OH + y) * s.OW + x;
}

__global__ void k_conv2d_fwd(ConvShape s, const float* __restrict__ x, const float* __restrict__ w,
                             const float* __restrict__ b, float* __restrict__ y, int relu) {
  const int64_t total = (int64_t)s.N * s.OH * s.OW * s.OC;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int oc = (int)(i % s.OC);
    int64_t r = i / s.OC;
    int ox = (int)(r % s.OW);
    r /= s.OW;
    int oy = (int)(r % s.OH);
    int n = (int)(r / s.OH);
    float acc = 0.f;
    for (int kh = 0; kh < s.KH; ++kh)
      for (int kw = 0; kw < s.KW; ++kw)
        for (int c = 0; c < s.C; ++c)
          acc += x[x_index(s, n, oy * s.SH + kh, ox * s.SW + kw, c)] * w[(((int64_t)kh * s.KW + kw) * s.C + c) * s.OC + oc];
    if (b) acc += b[oc];
    if (relu) acc = fmaxf(acc, 0.f);
    y[y_index(s, n, oy, ox, oc)] = acc;
  }
}

// dW[kh][kw][c][oc] = sum_{n,oy,ox} x[n][oy*SH+kh][ox*SW+kw][c] * dy[n][oy][ox][oc]; db[oc] = sum dy
__global__ void k_conv2d_dw(ConvShape s, const float* __restrict__ x, const float* __restrict__ dy,
                            float* __restrict__ dw, float* __restrict__ db) {
  const int64_t total = (int64_t)s.KH * s.KW * s.C * s.OC;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int oc = (int)(i % s.OC);
    int64_t r = i / s.OC;
    int c = (int)(r % s.C);
    r /= s.C;
    int kw = (int)(r % s.KW);
    int kh = (int)(r / s.KW);
    float acc = 0.f, accb = 0.f;
    for (int n = 0; n < s.N; ++n)
      for (int oy = 0; oy < s.OH; ++oy)
        for (int ox = 0; ox < s.OW; ++ox) {
          const float g = dy[y_index(s, n, oy, ox, oc)];
          acc += x[x_index(s, n, oy * s.SH + kh, ox * s.SW + kw, c)] * g;
          accb += g;
        }
    if (dw) dw[i] = acc;
    if (db && kh == 0 && kw == 0 && c == 0) db[oc] = accb;
  }
}

// dX[n][yy][xx][c] = sum over (kh,kw,oc) with yy = oy*SH+kh, xx = ox*SW+kw of dy * w
__global__ void k_conv2d_dx(ConvShape s, const float* __restrict__ w, const float* __restrict__ dy,
                            float* __restrict__ dx) {
  const int64_t total = (int64_t)s.N * s.H * s.W * s.C;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int c = (int)(i % s.C);
    int64_t r = i / s.C;
    int xx = (int)(r % s.W);
    r /= s.W;
    int yy = (int)(r % s.H);
    int n = (int)(r / s.H);
    float acc = 0.f;
    for (int kh = 0; kh < s.KH; ++kh) {
      const int ty = yy - kh;
      if (ty < 0 || ty % s.SH) continue;
      const int oy = ty / s.SH;
      if (oy >= s.OH) continue;
      for (int kw = 0; kw < s.KW; ++kw) {
        const int tx = xx - kw;
        if (tx < 0 || tx % s.SW) continue;
        const int ox = tx / s.SW;
        if (ox >= s.OW) continue;
        for (int oc = 0; oc < s.OC; ++oc)
          acc += dy[y_index(s, n, oy, ox, oc)] * w[(((int64_t)kh * s.KW + kw) * s.C + c) * s.OC + oc];
      }
    }
    dx[x_index(s, n, yy, xx, c)] = acc;
  }
}

static int conv_shape(int N, int H, int W, int C, int KH, int KW, int SH, int SW, int OC, int nhwc, ConvShape* s) {
  if (N < 0 || H < KH || W < KW || C < 1 || KH < 1 || KW < 1 || SH < 1 || SW < 1 || OC < 1) return -1;
  *s = ConvShape{N, H, W, C, KH, KW, SH, SW, OC, (H - KH) / SH + 1, (W - KW) / SW + 1, nhwc ? 1 : 0};
  return 0;
}

static unsigned grid_for(int64_t total) {
  int64_t g = (total + 255) / 256;
  return (unsigned)(g > 65535 ? 65535 : (g < 1 ? 1 : g));
}

extern "C" int a3c_conv2d_forward(const float* x, const float* w, const float* b, float* y, int N, int H, int W, int C,
                                  int KH, int KW, int SH, int SW, int OC, int nhwc, int relu, void* stream) {
  ConvShape s;
  if (!x || !w || !y || conv_shape(N, H, W, C, KH, KW, SH, SW, OC, nhwc, &s))
    return a3c_set_error(A3C_ERR_INVALID, "a3c_conv2d_forward", "bad argument");
  const int64_t total = (int64_t)s.N * s.OH * s.OW * s.OC;
  if (total == 0) return 0;
  hipLaunchKernelGGL(k_conv2d_fwd, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, s, x, w, b, y, relu);
  A3C_CHECK(hipGetLastError());
  return 0;
}

extern "C" int a3c_conv2d_backward(const float* x, const float* w, const float* dy, float* dx, float* dw, float* db,
                                   int N, int H, int W, int C, int KH, int KW, int SH, int SW, int OC, int nhwc,
                                   void* stream) {
  ConvShape s;
  if (!dy || conv_shape(N, H, W, C, KH, KW, SH, SW, OC, nhwc, &s) || ((dw || db) && !x) || (dx && !w))
    return a3c_set_error(A3C_ERR_INVALID, "a3c_conv2d_backward", "bad argument");
  hipStream_t st = (hipStream_t)stream;
  if (dw || db) {
    const int64_t t = (int64_t)KH * KW * C * OC;
    hipLaunchKernelGGL(k_conv2d_dw, dim3(grid_for(t)), dim3(256), 0, st, s, x, dy, dw, db);
    A3C_CHECK(hipGetLastError());
  }
  if (dx) {
    const int64_t t = (int64_t)N * H * W * C;
    if (t) hipLaunchKernelGGL(k_conv2d_dx, dim3(grid_for(t)), dim3(256), 0, st, s, w, dy, dx);
    A3C_CHECK(hipGetLastError());
  }
  return 0;
}

// C[m][n] (+)= sum_k A[m*sam + k*sak] * B[k*sbk + n*sbn]  (+ bias[n]) (relu)
__global__ void k_matmul(const float* __restrict__ A, int64_t sam, int64_t sak, const float* __restrict__ B,
                         int64_t sbk, int64_t sbn, float* __restrict__ C, int64_t ldc, int M, int N, int K,
                         const float* __restrict__ bias, int relu, int accumulate) {
  __shared__ float As[16][17], Bs[16][17];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int m = blockIdx.y * 16 + ty, n = blockIdx.x * 16 + tx;
  float acc = 0.f;
  for (int k0 = 0; k0 < K; k0 += 16) {
    const int ka = k0 + tx, kb = k0 + ty;
    As[ty][tx] = (m < M && ka < K) ? A[(int64_t)m * sam + (int64_t)ka * sak] : 0.f;
    Bs[ty][tx] = (kb < K && n < N) ? B[(int64_t)kb * sbk + (int64_t)n * sbn] : 0.f;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; ++k) acc += As[ty][k] * Bs[k][tx];
    __syncthreads();
  }
  if (m < M && n < N) {
    float v = acc + (bias ? bias[n] : 0.f);
    if (accumulate) v += C[(int64_t)m * ldc + n];
    if (relu) v = fmaxf(v, 0.f);
    C[(int64_t)m * ldc + n] = v;
  }
}

extern "C" int a3c_matmul(const float* A, int64_t sam, int64_t sak, const float* B, int64_t sbk, int64_t sbn, float* C,
                          int64_t ldc, int M, int N, int K, const float* bias, int relu, int accumulate, void* stream) {
  if (!A || !B || !C || M < 0 || N < 0 || K < 0) return a3c_set_error(A3C_ERR_INVALID, "a3c_matmul", "bad argument");
  if (!M || !N) return 0;
  dim3 grid((N + 15) / 16, (M + 15) / 16);
  if (grid.y > 65535) return a3c_set_error(A3C_ERR_INVALID, "a3c_matmul", "M too large");
  hipLaunchKernelGGL(k_matmul, grid, dim3(256), 0, (hipStream_t)stream, A, sam, sak, B, sbk, sbn, C, ldc, M, N, K, bias,
                     relu, accumulate);
  A3C_CHECK(hipGetLastError());
  return 0;
}

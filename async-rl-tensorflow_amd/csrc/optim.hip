// K10 per-tensor clip_by_norm (agent.py:316-319) + K11 TF ApplyRMSProp (main.py:63-65,
// agent.py:321) + K12 parameter copy (agent.py:342-344, network.py:96-107).
//
// Two launches: k_sumsq_partial (fixed-shape per-tensor partial sums of squares in fp64,
// deterministic order) then k_clip_apply (every block folds the partials into the per-tensor
// scales in LDS, then a grid-stride pass clips and/or applies RMSProp).  All element math is
// written with contraction off so it matches the numpy oracle bit for bit on equal grads.
#include "optim.h"

__global__ void __launch_bounds__(256) k_sumsq_partial(const float* __restrict__ g, TensorTab tt,
                                                       double* __restrict__ part) {
  __shared__ double red[256];
  const int t = blockIdx.y;
  const float* p = g + tt.off[t];
  const int64_t n = tt.size[t];
  double s = 0.0;
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < n; j += (int64_t)SS_BLOCKS * 256) {
    double v = (double)p[j];
    s += v * v;
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[t * SS_BLOCKS + blockIdx.x] = red[0];
}

__global__ void __launch_bounds__(256) k_clip_apply(float* __restrict__ w, float* __restrict__ ms,
                                                    float* __restrict__ mom, float* __restrict__ grads,
                                                    TensorTab tt, const double* __restrict__ part,
                                                    OptParams op, float* __restrict__ sumsq_out) {
#pragma clang fp contract(off)
  __shared__ float cm[A3C_MAX_TENSORS];
  __shared__ float s_lr;
  if (threadIdx.x < tt.n) {
    double ss = 0.0;
    for (int b = 0; b < SS_BLOCKS; ++b) ss += part[threadIdx.x * SS_BLOCKS + b];
    const float ssf = (float)ss;
    if (blockIdx.x == 0 && sumsq_out) sumsq_out[threadIdx.x] = ssf;
    float m = 1.0f;
    if (op.clip > 0.f) {
      const float inv = ssf > 0.f ? 1.0f / sqrtf(ssf) : INFINITY;
      m = fminf(inv, 1.0f / op.clip);
    }
    cm[threadIdx.x] = m;
  }
  if (threadIdx.x == 0) {
    float lr = op.lr;
    if (op.step_ptr) {
      const double step = (double)(*op.step_ptr + op.step_add);
      lr = (float)((double)(op.max_step - step + 1.0) / (double)op.max_step * op.lr0);
    }
    s_lr = lr;
  }
  __syncthreads();
  const float lr = s_lr;
  const float one_m_rho = 1.0f - op.rho;
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t gstride = (int64_t)gridDim.x * blockDim.x;
  for (int t = 0; t < tt.n; ++t) {
    const int64_t off = tt.off[t], n = tt.size[t];
    const float c = cm[t];
    for (int64_t j = gid; j < n; j += gstride) {
      float g = grads[off + j];
      if (op.clip > 0.f && (op.mode & OPT_CLIP)) g = (g * op.clip) * c;
      if (op.mode & OPT_APPLY) {
        float m2 = ms[off + j];
        m2 = m2 + (g * g - m2) * one_m_rho;
        float mo = mom[off + j] * op.momentum + (g * lr) / sqrtf(m2 + op.eps);
        ms[off + j] = m2;
        mom[off + j] = mo;
        w[off + j] = w[off + j] - mo;
      } else {
        grads[off + j] = g;
      }
    }
  }
}

__global__ void k_fill(float* __restrict__ p, int64_t n, float v) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

int a3c_optim_launch(float* w, float* ms, float* mom, float* grads, const TensorTab& tt, OptParams op,
                     double* part, float* sumsq_out, bool compute_sumsq, hipStream_t s) {
  if (tt.n <= 0 || tt.n > A3C_MAX_TENSORS) return a3c_set_error(A3C_ERR_INVALID, "optim", "bad tensor table");
  if (compute_sumsq) {
    hipLaunchKernelGGL(k_sumsq_partial, dim3(SS_BLOCKS, tt.n), dim3(256), 0, s, grads, tt, part);
    A3C_CHECK(hipGetLastError());
  }
  hipLaunchKernelGGL(k_clip_apply, dim3(256), dim3(256), 0, s, w, ms, mom, grads, tt, part, op, sumsq_out);
  A3C_CHECK(hipGetLastError());
  return 0;
}

int a3c_fill_launch(float* p, int64_t n, float v, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_fill, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, p, n, v);
  A3C_CHECK(hipGetLastError());
  return 0;
}

// --------------------------------------------------------------------------------------------
extern "C" int a3c_optim_workspace_bytes(int64_t total, int64_t* bytes) {
  (void)total;
  if (!bytes) return a3c_set_error(A3C_ERR_INVALID, "a3c_optim_workspace_bytes", "null");
  *bytes = (int64_t)A3C_MAX_TENSORS * SS_BLOCKS * sizeof(double);
  return 0;
}

static int make_tab(int n, const int64_t* off, const int64_t* size, TensorTab* tt) {
  if (n <= 0 || n > A3C_MAX_TENSORS || !off || !size) return -1;
  tt->n = n;
  for (int i = 0; i < n; ++i) { tt->off[i] = off[i]; tt->size[i] = size[i]; }
  return 0;
}

extern "C" int a3c_clip_grads(float* grads, int n_tensors, const int64_t* offsets, const int64_t* sizes,
                              float clip, float* sumsq_out, void* workspace, void* stream) {
  TensorTab tt;
  if (!grads || !workspace || make_tab(n_tensors, offsets, sizes, &tt))
    return a3c_set_error(A3C_ERR_INVALID, "a3c_clip_grads", "bad argument");
  OptParams op = {};
  op.mode = OPT_CLIP; op.clip = clip;
  return a3c_optim_launch(nullptr, nullptr, nullptr, grads, tt, op, (double*)workspace, sumsq_out, true,
                          (hipStream_t)stream);
}

extern "C" int a3c_clip_rmsprop_apply(float* params, float* ms, float* mom, float* grads, int n_tensors,
                                      const int64_t* offsets, const int64_t* sizes, float lr, float rho,
                                      float momentum, float eps, float clip, float* sumsq_out,
                                      void* workspace, void* stream) {
  TensorTab tt;
  if (!params || !ms || !mom || !grads || !workspace || make_tab(n_tensors, offsets, sizes, &tt))
    return a3c_set_error(A3C_ERR_INVALID, "a3c_clip_rmsprop_apply", "bad argument");
  OptParams op = {};
  op.mode = OPT_CLIP | OPT_APPLY; op.clip = clip; op.lr = lr; op.rho = rho; op.momentum = momentum; op.eps = eps;
  return a3c_optim_launch(params, ms, mom, grads, tt, op, (double*)workspace, sumsq_out, true,
                          (hipStream_t)stream);
}

extern "C" int a3c_copy_params(float* dst, const float* src, int64_t n, void* stream) {
  if (!dst || !src || n < 0) return a3c_set_error(A3C_ERR_INVALID, "a3c_copy_params", "bad argument");
  if (n == 0) return 0;
  A3C_CHECK(hipMemcpyAsync(dst, src, (size_t)n * sizeof(float), hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return 0;
}

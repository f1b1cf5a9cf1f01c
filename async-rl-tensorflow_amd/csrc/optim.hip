// K10 per-tensor clip_by_norm (agent.py:316-319) + K11 TF ApplyRMSProp (main.py:63-65,
// agent.py:321) + K12 parameter copy (agent.py:342-344, network.py:96-107).
//
// k_sumsq: one partial sum of squares (fp64, fixed order) per SS_CHUNK elements of each tensor,
//          blocks proportional to tensor size; block 0 also evaluates the lr schedule and the
//          target-sync decision from the device step counter.
// k_apply: every block folds the partials into the per-tensor clip scales in LDS, then one
//          float4 pass over the flat vector clips and/or applies RMSProp (and the target copy);
//          block 0 advances the engine counters at the end (nothing in this launch reads them).
// Element math is written with contraction off so it matches the numpy oracle bit for bit on
// equal gradients.
#include <cstring>
#include "optim.h"

int a3c_make_tab(int n, const int64_t* off, const int64_t* size, int64_t total, TensorTab* tt) {
  if (n <= 0 || n > A3C_MAX_TENSORS || !off || !size || (total & 3)) return -1;
  tt->n = n;
  int nb = 0;
  int64_t end = 0;
  for (int i = 0; i < n; ++i) {
    if ((off[i] & 3) || size[i] < 0 || off[i] < end) return -1;
    tt->off[i] = off[i];
    tt->size[i] = size[i];
    tt->pb_first[i] = nb;
    tt->pb_count[i] = (int)((size[i] + SS_CHUNK - 1) / SS_CHUNK);
    nb += tt->pb_count[i];
    end = off[i] + size[i];
  }
  if (nb > SS_MAX_BLOCKS || end > total) return -1;
  tt->nblocks = nb;
  tt->total = total;
  return 0;
}

__global__ void __launch_bounds__(256) k_sumsq(const float* __restrict__ g, TensorTab tt, OptParams op,
                                               double* __restrict__ part) {
  int t = 0;
  while (t + 1 < tt.n && (int)blockIdx.x >= tt.pb_first[t + 1]) ++t;
  sumsq_chunk(g, tt, t, blockIdx.x - tt.pb_first[t], part, blockIdx.x);
  if (blockIdx.x == 0 && threadIdx.x == 0) opt_schedule(op);
}

__global__ void __launch_bounds__(256) k_apply(float* __restrict__ w, float* __restrict__ ms,
                                               float* __restrict__ mom, float* __restrict__ grads,
                                               TensorTab tt, const double* __restrict__ part, OptParams op,
                                               float* __restrict__ sumsq_out) {
#pragma clang fp contract(off)
  WGLOG(9);
  __shared__ float cm[A3C_MAX_TENSORS];
  __shared__ float s_lr, s_copy;
  __shared__ double red[4][A3C_MAX_TENSORS];
  // per-tensor fold of the partials: wave w sums tensors t = w, w+4, ... with all 64 lanes
  {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int t = wv; t < tt.n; t += 4) {
      double v = 0.0;
      for (int b = lane; b < tt.pb_count[t]; b += 64) v += part[tt.pb_first[t] + b];
      v = wave_sum_d(v);
      if (lane == 0) red[0][t] = v;
    }
  }
  __syncthreads();
  if (threadIdx.x < tt.n) {
    const double ss = red[0][threadIdx.x];
    const float ssf = (float)ss;
    if (blockIdx.x == 0 && sumsq_out) sumsq_out[threadIdx.x] = ssf;
    float m = 1.0f;
    if (op.clip > 0.f && (op.mode & OPT_CLIP)) {
      const float inv = ssf > 0.f ? 1.0f / sqrtf(ssf) : INFINITY;
      m = fminf(inv, 1.0f / op.clip);      // tf.clip_by_norm: t * clip * min(rsqrt(ss), 1/clip)
    }
    cm[threadIdx.x] = m;
  }
  if (threadIdx.x == 0) {
    s_lr = op.sched ? op.sched[0] : op.lr;
    s_copy = (op.sched && op.target) ? op.sched[1] : 0.f;
  }
  __syncthreads();
  const float lr = s_lr;
  const bool copy = s_copy != 0.f;
  const bool clip = op.clip > 0.f && (op.mode & OPT_CLIP);
  const bool apply = op.mode & OPT_APPLY;
  const float one_m_rho = 1.0f - op.rho;
  const int64_t qe = op.q1 > 0 ? op.q1 : tt.total >> 2;
  for (int64_t q = (op.q1 > 0 ? op.q0 : 0) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < qe;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = 4 * q;
    int t = 0;
    while (t + 1 < tt.n && i >= tt.off[t + 1]) ++t;     // padding after tensor t has zero grads
    f32x4 g = *(const f32x4*)(grads + i);
    if (clip) {
      const float c = cm[t];
#pragma unroll
      for (int k = 0; k < 4; ++k) g[k] = (g[k] * op.clip) * c;
    }
    if (apply) {
      f32x4 m2 = *(const f32x4*)(ms + i);
      f32x4 mo = *(const f32x4*)(mom + i);
      f32x4 wv = *(const f32x4*)(w + i);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        m2[k] = m2[k] + (g[k] * g[k] - m2[k]) * one_m_rho;
        mo[k] = mo[k] * op.momentum + (g[k] * lr) / sqrtf(m2[k] + op.eps);
        wv[k] = wv[k] - mo[k];
      }
      *(f32x4*)(ms + i) = m2;
      *(f32x4*)(mom + i) = mo;
      *(f32x4*)(w + i) = wv;
      if (copy) *(f32x4*)(op.target + i) = wv;
      if (op.snap) *(f32x4*)(op.snap + i) = wv;
    } else {
      *(f32x4*)(grads + i) = g;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && op.counters && apply) {   // clip-only passes leave them
    if (op.dtau) op.counters[0] += op.dtau;   // overlap mode: the rollout owns tau
    op.counters[1] += op.step_add;
  }
}

// ---- partitioned parameter server (multi-GPU sequential exchange) ----------------------------
// The reference's PS applies every worker's clipped gradient as an RMSProp step of its own, in
// arrival order (one shared optimizer, main.py:63-65; each worker's apply_gradients, agent.py:321).
// Rank r owns [lo, lo + n) of params / ms / mom.  After the all-to-all it holds every rank's
// clipped gradient of that range (g + q*n, q = 0 .. nranks-1) and applies them one after the
// other in rank order: one legal arrival order of the reference PS, and deterministic.  The new
// weights go to w_out (the all-gather's input); ms / mom are updated in place (only the owner
// reads its range).  The element math is k_apply's, so one rank reproduces it bit for bit.
__global__ void __launch_bounds__(256) k_apply_seq(const float* __restrict__ w, float* __restrict__ ms,
                                                   float* __restrict__ mom, const float* __restrict__ g,
                                                   int nranks, int64_t n, const float* __restrict__ sched,
                                                   float rho, float momentum, float eps,
                                                   float* __restrict__ w_out) {
#pragma clang fp contract(off)
  const float lr = sched[0];
  const float one_m_rho = 1.0f - rho;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float wv = w[i], m2 = ms[i], mo = mom[i];
    for (int q = 0; q < nranks; ++q) {
      const float gi = g[(int64_t)q * n + i];
      m2 = m2 + (gi * gi - m2) * one_m_rho;
      mo = mo * momentum + (gi * lr) / sqrtf(m2 + eps);
      wv = wv - mo;
    }
    ms[i] = m2;
    mom[i] = mo;
    w_out[i] = wv;
  }
}

int a3c_apply_seq_launch(const float* w, float* ms, float* mom, const float* g, int nranks, int64_t n,
                         const float* sched, float rho, float momentum, float eps, float* w_out, hipStream_t s) {
  if (n <= 0) return 0;
  const int64_t blocks = (n + 255) / 256 < 1024 ? (n + 255) / 256 : 1024;
  hipLaunchKernelGGL(k_apply_seq, dim3((unsigned)blocks), dim3(256), 0, s, w, ms, mom, g, nranks, n, sched, rho,
                     momentum, eps, w_out);
  A3C_CHECK(hipGetLastError());
  return 0;
}

// The rest of an apply once the all-gather has assembled the new parameters in src: params (and
// the overlap pipeline's snapshot) <- src, target sync when the schedule flagged one (agent.py:
// 166-167, 342-344), and block 0 advances the counters.  n4 = float4 count.
__global__ void __launch_bounds__(256) k_commit(const float* __restrict__ src, int64_t n4, float* __restrict__ params,
                                                float* __restrict__ snap, float* __restrict__ target,
                                                const float* __restrict__ sched, int64_t* counters, int64_t dtau,
                                                int64_t dstep) {
  const bool tsync = target && sched[1] != 0.f;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += (int64_t)gridDim.x * blockDim.x) {
    const f32x4 v = ((const f32x4*)src)[q];
    if (src != params) ((f32x4*)params)[q] = v;
    if (snap) ((f32x4*)snap)[q] = v;
    if (tsync) ((f32x4*)target)[q] = v;
  }
  // tau only when this pass owns it: in overlap mode (dtau 0) the concurrent rollout stream advances
  // tau in its bootstrap head, and an unconditional `counters[0] += 0` here is a read-modify-write
  // that can overwrite that advance (round 3's w4-breakout-overlap divergence: the lost advance
  // shifted the rank's ring / Philox counters by n steps while the all-gather kept the ranks equal)
  if (blockIdx.x == 0 && threadIdx.x == 0 && counters) {
    if (dtau) counters[0] += dtau;
    counters[1] += dstep;
  }
}

int a3c_commit_launch(const float* src, int64_t total, float* params, float* snap, float* target, const float* sched,
                      int64_t* counters, int64_t dtau, int64_t dstep, hipStream_t s) {
  const int64_t n4 = total >> 2;
  int64_t blocks = (n4 + 255) / 256;
  blocks = blocks > 1024 ? 1024 : (blocks < 1 ? 1 : blocks);
  hipLaunchKernelGGL(k_commit, dim3((unsigned)blocks), dim3(256), 0, s, src, n4, params, snap, target, sched, counters,
                     dtau, dstep);
  A3C_CHECK(hipGetLastError());
  return 0;
}

__global__ void k_fill(float* __restrict__ p, int64_t n, float v) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

int a3c_sumsq_launch(const float* grads, const TensorTab& tt, const OptParams& op, double* part, hipStream_t s) {
  hipLaunchKernelGGL(k_sumsq, dim3(tt.nblocks), dim3(256), 0, s, grads, tt, op, part);
  A3C_CHECK(hipGetLastError());
  return 0;
}

int a3c_apply_launch(float* w, float* ms, float* mom, float* grads, const TensorTab& tt, const OptParams& op,
                     const double* part, float* sumsq_out, hipStream_t s) {
  const int64_t n4 = op.q1 > 0 ? op.q1 - op.q0 : tt.total >> 2;
  int blocks = (int)((n4 + 255) / 256);
  if (blocks > 1024) blocks = 1024;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(k_apply, dim3(blocks), dim3(256), 0, s, w, ms, mom, grads, tt, part, op, sumsq_out);
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
  *bytes = (int64_t)SS_MAX_BLOCKS * sizeof(double);
  return 0;
}

static int64_t tab_total(int n, const int64_t* off, const int64_t* size) {
  int64_t e = 0;
  for (int i = 0; i < n; ++i) e = off[i] + size[i] > e ? off[i] + size[i] : e;
  return (e + 3) & ~(int64_t)3;
}

extern "C" int a3c_clip_grads(float* grads, int n_tensors, const int64_t* offsets, const int64_t* sizes,
                              float clip, float* sumsq_out, void* workspace, void* stream) {
  TensorTab tt;
  if (!grads || !workspace || !offsets || !sizes || n_tensors <= 0 || n_tensors > A3C_MAX_TENSORS ||
      a3c_make_tab(n_tensors, offsets, sizes, tab_total(n_tensors, offsets, sizes), &tt))
    return a3c_set_error(A3C_ERR_INVALID, "a3c_clip_grads", "bad argument (offsets must be 4-aligned, ascending)");
  OptParams op = {};
  op.mode = OPT_CLIP; op.clip = clip;
  hipStream_t s = (hipStream_t)stream;
  int rc = a3c_sumsq_launch(grads, tt, op, (double*)workspace, s);
  if (rc) return rc;
  return a3c_apply_launch(nullptr, nullptr, nullptr, grads, tt, op, (double*)workspace, sumsq_out, s);
}

extern "C" int a3c_clip_rmsprop_apply(float* params, float* ms, float* mom, float* grads, int n_tensors,
                                      const int64_t* offsets, const int64_t* sizes, float lr, float rho,
                                      float momentum, float eps, float clip, float* sumsq_out,
                                      void* workspace, void* stream) {
  TensorTab tt;
  if (!params || !ms || !mom || !grads || !workspace || !offsets || !sizes || n_tensors <= 0 ||
      n_tensors > A3C_MAX_TENSORS || a3c_make_tab(n_tensors, offsets, sizes, tab_total(n_tensors, offsets, sizes), &tt))
    return a3c_set_error(A3C_ERR_INVALID, "a3c_clip_rmsprop_apply", "bad argument (offsets must be 4-aligned, ascending)");
  OptParams op = {};
  op.mode = OPT_CLIP | OPT_APPLY; op.clip = clip; op.lr = lr; op.rho = rho; op.momentum = momentum; op.eps = eps;
  hipStream_t s = (hipStream_t)stream;
  int rc = a3c_sumsq_launch(grads, tt, op, (double*)workspace, s);
  if (rc) return rc;
  return a3c_apply_launch(params, ms, mom, grads, tt, op, (double*)workspace, sumsq_out, s);
}

extern "C" int a3c_copy_params(float* dst, const float* src, int64_t n, void* stream) {
  if (!dst || !src || n < 0) return a3c_set_error(A3C_ERR_INVALID, "a3c_copy_params", "bad argument");
  if (n == 0) return 0;
  A3C_CHECK(hipMemcpyAsync(dst, src, (size_t)n * sizeof(float), hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return 0;
}

// ---- Hogwild shard apply ------------------------------------------------------------------
__global__ void k_rmsprop_range(float* __restrict__ w, float* __restrict__ ms, float* __restrict__ mom,
                                const float* __restrict__ g, int64_t n, const float* __restrict__ lr_dev, float lr,
                                float rho, float momentum, float eps) {
#pragma clang fp contract(off)
  const float l = lr_dev ? lr_dev[0] : lr;
  const float one_m_rho = 1.0f - rho;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float gi = g[i];
    const float m2 = ms[i] + (gi * gi - ms[i]) * one_m_rho;
    const float mo = mom[i] * momentum + (gi * l) / sqrtf(m2 + eps);
    ms[i] = m2;                // unlocked read-modify-write: concurrent workers may interleave
    mom[i] = mo;
    w[i] = w[i] - mo;
  }
}

extern "C" int a3c_rmsprop_range(float* w, float* ms, float* mom, const float* grads, int64_t n, const float* lr_dev,
                                 float lr, float rho, float momentum, float eps, void* stream) {
  if (!w || !ms || !mom || !grads || n < 0) return a3c_set_error(A3C_ERR_INVALID, "a3c_rmsprop_range", "bad argument");
  if (n == 0) return 0;
  const int64_t blocks = (n + 255) / 256 < 1024 ? (n + 255) / 256 : 1024;
  hipLaunchKernelGGL(k_rmsprop_range, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, w, ms, mom, grads, n,
                     lr_dev, lr, rho, momentum, eps);
  A3C_CHECK(hipGetLastError());
  return 0;
}

extern "C" int a3c_dev_alloc(int64_t bytes, void** out) {
  if (!out || bytes <= 0) return a3c_set_error(A3C_ERR_INVALID, "a3c_dev_alloc", "bad argument");
  A3C_CHECK(hipMalloc(out, (size_t)bytes));
  return 0;
}

// Hogwild shard memory (DESIGN §7 "memory model"): kind 0 coarse-grained (hipMalloc: coherent
// only at kernel boundaries), 1 fine-grained (coherent at instruction granularity across devices:
// a peer's RMW over xGMI and the owner's reads meet in memory, no stale L2 line on either side),
// 2 uncached (every access goes to memory).  All three are VRAM and IPC-exportable.
extern "C" int a3c_dev_alloc_kind(int64_t bytes, int kind, void** out) {
  if (!out || bytes <= 0 || kind < 0 || kind > 2) return a3c_set_error(A3C_ERR_INVALID, "a3c_dev_alloc_kind", "bad argument");
  if (kind == 0) {
    A3C_CHECK(hipMalloc(out, (size_t)bytes));
  } else {
    A3C_CHECK(hipExtMallocWithFlags(out, (size_t)bytes, kind == 1 ? hipDeviceMallocFinegrained : hipDeviceMallocUncached));
  }
  return 0;
}

extern "C" int a3c_dev_free(void* p) {
  if (p) A3C_CHECK(hipFree(p));
  return 0;
}

extern "C" int a3c_ipc_handle(void* base, void* handle64) {
  if (!base || !handle64) return a3c_set_error(A3C_ERR_INVALID, "a3c_ipc_handle", "bad argument");
  static_assert(sizeof(hipIpcMemHandle_t) <= 64, "ipc handle size");
  hipIpcMemHandle_t h;
  A3C_CHECK(hipIpcGetMemHandle(&h, base));
  memset(handle64, 0, 64);
  memcpy(handle64, &h, sizeof(h));
  return 0;
}

extern "C" int a3c_ipc_open(const void* handle64, void** out) {
  if (!handle64 || !out) return a3c_set_error(A3C_ERR_INVALID, "a3c_ipc_open", "bad argument");
  hipIpcMemHandle_t h;
  memcpy(&h, handle64, sizeof(h));
  A3C_CHECK(hipIpcOpenMemHandle(out, h, hipIpcMemLazyEnablePeerAccess));
  return 0;
}

extern "C" int a3c_ipc_close(void* p) {
  if (p) A3C_CHECK(hipIpcCloseMemHandle(p));
  return 0;
}

#ifdef A3C_WGLOG
WGLOG_BIND(a3c_wglog_bind_optim)
#endif

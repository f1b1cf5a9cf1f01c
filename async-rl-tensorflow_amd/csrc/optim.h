#pragma once
#include "a3c_common.h"
#include "../../include/a3c_hip.h"

#define SS_CHUNK 4096          // elements per sum-of-squares partial block
#ifndef SS_MAX_BLOCKS
#define SS_MAX_BLOCKS 1024     // partial slots (>= sum over tensors of ceil(size / SS_CHUNK))
#endif
enum { OPT_CLIP = 1, OPT_APPLY = 2 };

struct TensorTab {
  int n;
  int64_t off[A3C_MAX_TENSORS];
  int64_t size[A3C_MAX_TENSORS];
  int pb_first[A3C_MAX_TENSORS];   // first partial block of tensor t
  int pb_count[A3C_MAX_TENSORS];   // partial blocks of tensor t
  int nblocks;
  int64_t total;                   // padded flat length (multiple of 4): the apply pass covers [0, total)
};

struct OptParams {
  int mode;              // OPT_CLIP | OPT_APPLY
  float clip;            // <= 0: no clipping
  float lr;              // used when sched == nullptr
  // schedule (engine): the sum-of-squares kernel computes
  //   sched[0] = lr = (max_step - step + 1)/max_step * lr0              (agent.py:393-395)
  //   sched[1] = 1 if a target sync falls in (T, T + step_add]          (agent.py:165-167)
  // where T = *step_ptr is the global step (the reference's step_op, every worker's env steps) and
  // `step` is the worker's own loop counter (agent.py:55: `for self.step in xrange(T0, max_step)`)
  // at the update: with wstep_ptr, step = *wstep_ptr + (*tau_ptr - tau0) + n_step - 1 -- the base
  // the workers started from, plus the env steps before the rollout, plus the rollout's last step
  // (batch_update runs inside that step's observe, agent.py:162-163); without it, T + step_add.
  float* sched;
  const int64_t* step_ptr;
  int64_t step_add;
  const int64_t* wstep_ptr;
  const int64_t* tau_ptr;
  int64_t tau0, n_step;
  double lr0;
  int64_t max_step;
  int64_t target_period;  // 0: no target network
  float* target;          // apply: params also written here when sched[1] != 0
  float* snap;            // apply (nullable): the new params also written here (overlap snapshot)
  int64_t* counters;      // apply: block 0 advances counters[0] += dtau, counters[1] += step_add
  int64_t dtau;
  float rho, momentum, eps;
  // apply / clip pass over float4 indices [q0, q1) only (q1 == 0: the whole flat vector) -- the
  // split exchange clips the fc / head tensors before the conv backward, the conv tensors after
  int64_t q0, q1;
};

int a3c_make_tab(int n, const int64_t* off, const int64_t* size, int64_t total, TensorTab* tt);

// the lr schedule and target-sync decision from the device step counter (one thread; k_sumsq's
// block 0, or the backward's finalize when it produces the partials itself)
__device__ inline void opt_schedule(const OptParams& op) {
  if (!op.sched || !op.step_ptr) return;
  const int64_t g0 = *op.step_ptr;
  const double step = op.wstep_ptr ? (double)(*op.wstep_ptr + (*op.tau_ptr - op.tau0) + op.n_step - 1)
                                   : (double)(g0 + op.step_add);
  // agent.py:393-395; the reference never trains past max_step (agent.py:46,55-57), so the
  // schedule is clamped at 0 there instead of turning negative (RMSProp would ascend)
  const double lr = (double)(op.max_step - step + 1.0) / (double)op.max_step * op.lr0;
  op.sched[0] = (float)(lr > 0.0 ? lr : 0.0);
  int copy = 0;
  if (op.target_period > 0) copy = (g0 + op.step_add + 1) / op.target_period != (g0 + 1) / op.target_period;
  op.sched[1] = copy ? 1.0f : 0.0f;
}

// fp64 sum of squares of chunk c (SS_CHUNK elements) of tensor t, by one 256-thread block into
// part[slot]: float4 body + scalar tail, then a fixed-order tree
__device__ inline void sumsq_chunk(const float* __restrict__ g, const TensorTab& tt, int t, int64_t c,
                                   double* __restrict__ part, int slot) {
  __shared__ double red[256];
  const int64_t beg = c * SS_CHUNK;
  const int64_t end = min(tt.size[t], beg + (int64_t)SS_CHUNK);
  const float* p = g + tt.off[t];
  double s = 0.0;
  // tensor offsets are 4-aligned, chunk starts are 4096-aligned
  const int64_t end4 = beg + ((end - beg) & ~(int64_t)3);
  for (int64_t j = beg + 4 * threadIdx.x; j < end4; j += 4 * 256) {
    f32x4 v = *(const f32x4*)(p + j);
    s += (double)v[0] * v[0] + (double)v[1] * v[1] + (double)v[2] * v[2] + (double)v[3] * v[3];
  }
  for (int64_t j = end4 + threadIdx.x; j < end; j += 256) s += (double)p[j] * p[j];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[slot] = red[0];
}
int a3c_sumsq_launch(const float* grads, const TensorTab& tt, const OptParams& op, double* part, hipStream_t s);
int a3c_apply_launch(float* w, float* ms, float* mom, float* grads, const TensorTab& tt, const OptParams& op,
                     const double* part, float* sumsq_out, hipStream_t s);
int a3c_fill_launch(float* p, int64_t n, float v, hipStream_t s);
// partitioned PS: nranks sequential RMSProp steps of the owned range (lr = sched[0]) -> w_out
int a3c_apply_seq_launch(const float* w, float* ms, float* mom, const float* g, int nranks, int64_t n,
                         const float* sched, float rho, float momentum, float eps, float* w_out, hipStream_t s);
// params / snapshot / target (if sched[1]) <- src, counters += (dtau, dstep)
int a3c_commit_launch(const float* src, int64_t total, float* params, float* snap, float* target, const float* sched,
                      int64_t* counters, int64_t dtau, int64_t dstep, hipStream_t s);

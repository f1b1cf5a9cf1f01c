// Action draw and policy / value head rows shared by the NIPS rollout kernels (net_fwd.hip) and
// the nature trunk's head (nature.hip): network.py:62-79 heads, network.py:72 batch_sample /
// agent.py:141-151 epsilon-greedy, the fused env act of agent.py:59-62.
#pragma once
#include "net.h"
#include "env_dev.h"

// ---------------------------------------------------------------------------------------
// action selection from a head row held one-value-per-lane (lane j holds z[j])
// ---------------------------------------------------------------------------------------
// the action draw's counter-based random words for state b at step tau
__device__ inline u32x4 action_draw(const HeadSelect& sel, int64_t b, int64_t tau) {
  const int e = (int)(b % sel.E);
  const uint32_t env = sel.env_ids ? (uint32_t)sel.env_ids[b] : (uint32_t)(sel.env_id_base + e);
  return philox4x32((uint32_t)tau, (uint32_t)((uint64_t)tau >> 32), env, P_ACTION, sel.k0, sel.k1);
}

// x = action_draw(sel, b, tau); eps = the env's exploration rate (Q mode)
__device__ inline int32_t select_with(float myz, int lane, int A, int mode, u32x4 x, float eps) {
  if (A <= 8) {
    // the logits to every lane via v_readlane (wave-uniform values, no cross-lane round trips)
    float zv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) zv[j] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(myz), j));
    if (mode == 0) {
      float m = zv[0];
#pragma unroll
      for (int j = 1; j < 8; ++j) m = j < A ? fmaxf(m, zv[j]) : m;
      // lane j: exp and probability of action j (one expf / divide per lane, in parallel)
      const float ex = lane < A ? expf(myz - m) : 0.f;
      float ssum = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) ssum += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ex), j));
      const float pi = ex / ssum;
      const float u = u01(x.x);
      float cdf = 0.f;
      int32_t act = A - 1;
      bool found = false;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (j < A) {
          cdf += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pi), j));
          if (!found && cdf > u) { act = j; found = true; }
        }
      }
      return act;
    }
    if (u01(x.x) < eps) return (int32_t)(x.y % (uint32_t)A);
    float best = zv[0];
    int32_t arg = 0;
#pragma unroll
    for (int j = 1; j < 8; ++j)
      if (j < A && zv[j] > best) { best = zv[j]; arg = j; }
    return arg;
  }
  if (mode == 0) {
    float l = lane < A ? myz : -INFINITY;
    float m = wave_max(l);
    float ex = lane < A ? expf(myz - m) : 0.f;
    float ssum = wave_sum(ex);
    float pi = ex / ssum;
    float u = u01(x.x);
    float cdf = 0.f;
    int32_t act = A - 1;
    for (int j = 0; j < A; ++j) {
      cdf += __shfl(pi, j, 64);
      if (cdf > u) { act = j; break; }
    }
    return act;
  } else {
    if (u01(x.x) < eps) return (int32_t)(x.y % (uint32_t)A);
    float best = __shfl(myz, 0, 64);
    int32_t arg = 0;
    for (int j = 1; j < A; ++j) {
      float v = __shfl(myz, j, 64);
      if (v > best) { best = v; arg = j; }
    }
    return arg;
  }
}

// the exploration rate of env e at step tau (Q mode): the linear schedule of agent.py:142-144 at
// the worker's own step (agent.py:55 loop counter) when sel.ep_end is set, else sel.eps[e]
__device__ inline float sel_eps(const HeadSelect& sel, int e, int64_t tau) {
  if (sel.mode == 0) return 0.f;
  if (sel.ep_end) {
    const double step = (double)(sel.tau_ptr[2] + tau - (HIST - 1));
    const double ee = sel.ep_end[e];
    const double d = (double)sel.ep_end_t - fmax(0.0, step - (double)sel.learn_start);
    return (float)(ee + fmax(0.0, ((double)sel.ep_start - ee) * d / (double)sel.ep_end_t));
  }
  return sel.eps ? sel.eps[e] : 0.f;
}

__device__ inline int32_t select_from_lanes(float myz, int lane, int A, const HeadSelect& sel, int64_t b) {
  const int64_t tau = (sel.tau_ptr ? *sel.tau_ptr : 0) + sel.tau_add;
  const float eps = sel_eps(sel, (int)(b % sel.E), tau);
  return select_with(myz, lane, A, sel.mode, action_draw(sel, b, tau), eps);
}

struct NoMid {
  __device__ void operator()() const {}
};

// mid(): work to overlap with the head's load latency (runs after the loads are issued)
// W: the layer width (FC = 256 for the NIPS trunk, NT_FC = 512 for the nature trunk)
template <typename Mid = NoMid, int W = FC>
__device__ inline float head_row(const float* __restrict__ h3, int64_t b, const float* __restrict__ Wp,
                                 const float* __restrict__ bp, const float* __restrict__ Wv,
                                 const float* __restrict__ bv, int A, int lane, Mid mid = Mid()) {
  static_assert(W % 256 == 0, "head width");
  float myz = 0.f;
  const int nout = A + (Wv ? 1 : 0);
  if (nout <= 8) {
    // lane = (output o = lane & 7, chunk c = lane >> 3 of W/8 features): 8 outputs at once,
    // then a 3-step butterfly over the 8 chunks; W/256 passes of 32 features per lane
    const int o = lane & 7, c = lane >> 3;
    constexpr int PER = W / 8;
    const float* hp = h3 + b * W + PER * c;
    const bool val = Wv && o == A;                 // (lanes o >= nout read column 0, result dropped)
    const int oc = o < nout ? o : 0;
    const float* w = val ? Wv + PER * c : Wp + (int64_t)(PER * c) * A + oc;
    const int st = val ? 1 : A;
    float hv[32], wv[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      hv[k] = hp[k];
      wv[k] = w[k * st];
    }
    const float bias = lane < A ? bp[lane] : (Wv && lane == A ? bv[0] : 0.f);
    mid();
    float p = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k) p += hv[k] * wv[k];
#pragma unroll
    for (int pass = 1; pass < W / 256; ++pass) {   // (W > 256: the chunk's next 32 features)
#pragma unroll
      for (int k = 0; k < 32; ++k) {
        hv[k] = hp[32 * pass + k];
        wv[k] = w[(32 * pass + k) * st];
      }
#pragma unroll
      for (int k = 0; k < 32; ++k) p += hv[k] * wv[k];
    }
    if (o >= nout) p = 0.f;
    p += __shfl_xor(p, 8, 64);
    p += __shfl_xor(p, 16, 64);
    p += __shfl_xor(p, 32, 64);
    const float zj = __shfl(p, lane & 7, 64);
    if (lane < A || (Wv && lane == A)) myz = zj + bias;
  } else if constexpr (W == FC) {
    mid();
    f32x4 h = *(const f32x4*)(h3 + b * FC + 4 * lane);
    for (int j = 0; j < A; ++j) {
      const float* w = Wp + (int64_t)(4 * lane) * A + j;
      float p = h[0] * w[0] + h[1] * w[A] + h[2] * w[2 * A] + h[3] * w[3 * A];
      p = wave_sum(p);
      if (lane == j) myz = p + bp[j];
    }
    if (Wv) {
      f32x4 w = *(const f32x4*)(Wv + 4 * lane);
      float p = wave_sum(h[0] * w[0] + h[1] * w[1] + h[2] * w[2] + h[3] * w[3]);
      if (lane == A) myz = p + bv[0];
    }
  } else {
    mid();
    for (int j = 0; j < A; ++j) {
      float p = 0.f;
#pragma unroll
      for (int pass = 0; pass < W / 256; ++pass) {
        const f32x4 h = *(const f32x4*)(h3 + b * W + 256 * pass + 4 * lane);
        const float* w = Wp + (int64_t)(256 * pass + 4 * lane) * A + j;
        p += h[0] * w[0] + h[1] * w[A] + h[2] * w[2 * A] + h[3] * w[3 * A];
      }
      p = wave_sum(p);
      if (lane == j) myz = p + bp[j];
    }
    if (Wv) {
      float p = 0.f;
#pragma unroll
      for (int pass = 0; pass < W / 256; ++pass) {
        const f32x4 h = *(const f32x4*)(h3 + b * W + 256 * pass + 4 * lane);
        const f32x4 w = *(const f32x4*)(Wv + 256 * pass + 4 * lane);
        p += h[0] * w[0] + h[1] * w[1] + h[2] * w[2] + h[3] * w[3];
      }
      p = wave_sum(p);
      if (lane == A) myz = p + bv[0];
    }
  }
  return myz;
}

// action draw for row b (all lanes) and, in lane 0, the fused env act (agent.py:59-62).
// Returns the post-act frame index in lane 0 when the env is stepped, else -1.
__device__ inline int32_t head_act(float myz, int lane, int A, const HeadSelect& sel, int64_t b) {
  int32_t frame = -1;
  const int32_t a = select_from_lanes(myz, lane, A, sel, b);
  if (lane == 0) {
    sel.actions[b] = a;
    if (sel.env_on) {
      const int64_t tau = *sel.tau_ptr + sel.tau_add;
      const int e = (int)b;
      const int64_t cur = (tau & 1) * (int64_t)sel.par_E + e, nxt = ((tau + 1) & 1) * (int64_t)sel.par_E + e;
      const uint32_t id = (uint32_t)(sel.env_id_base + e);
      EnvState s = env_load(sel.envb, cur);
      env_act(s, sel.envp, id, (uint32_t)a, true);
      sel.rewards[e] = fmaxf(-1.0f, fminf(1.0f, s.reward));   // observe clip, agent.py:154
      if (sel.rewards_raw) sel.rewards_raw[e] = s.reward;
      sel.terms[e] = (uint8_t)s.terminal;
      sel.frames_out[e] = s.frame;
      frame = s.frame;
      if (s.terminal) env_new_random_game(s, sel.envp, id);    // agent.py:66-67
      env_store(sel.envb, nxt, s);
    }
  }
  return frame;
}


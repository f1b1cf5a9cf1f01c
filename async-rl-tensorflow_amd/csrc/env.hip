// Batched synthetic Atari stand-in on device (gym/ALE is absent; SURVEY §2 OUT OF SCOPE) with the
// reference's interface semantics, bit-identical to oracle/synthetic_env.py:
//   new_game          environment.py:74-79
//   new_random_game   environment.py:81-86
//   act               environment.py:124-142 (action repeat, life-loss terminal when training)
//   observe clip      agent.py:154
// k_env_step fuses one env step with K1 (Environment.screen) and the K2 history push: the new
// 84x84 screen is written straight into the env's frame-ring slot, so the "shift" of
// history.py:13-15 costs nothing (states are read through StateAddr).
#include "env.h"
#include "preprocess_dev.h"

#define GOLDEN_MULT 2654435761u

struct EnvCtx {
  const EnvParams& p;
  const EnvBufs& s;
  int e;
  uint32_t id;
};

__device__ inline void env_reset(const EnvCtx& c) {
  uint32_t ep = c.s.episode[c.e] + 1u;
  c.s.episode[c.e] = ep;
  c.s.ep_step[c.e] = 0;
  c.s.lives[c.e] = c.p.L0;
  u32x4 x = philox4x32(ep, c.id, P_RESET, 0u, c.p.k0, c.p.k1);
  c.s.ep_len[c.e] = 200u + x.x % 1801u;
  c.s.frame[c.e] = (int32_t)(x.y % (uint32_t)c.p.P);
}

__device__ inline void env_step_raw(const EnvCtx& c, uint32_t action) {
  const uint32_t st = c.s.ep_step[c.e] + 1u;
  c.s.ep_step[c.e] = st;
  u32x4 x = philox4x32(st, c.id, c.s.episode[c.e], P_STEP, c.p.k0, c.p.k1);
  const uint32_t mix = x.x + action * GOLDEN_MULT;
  c.s.frame[c.e] = (int32_t)(mix % (uint32_t)c.p.P);
  const float u = u01(x.y);
  const float rp = 0.02f;
  c.s.reward[c.e] = u < rp ? 1.0f : (u >= 1.0f - rp ? -1.0f : 0.0f);
  int32_t lives = c.s.lives[c.e];
  if (u01(x.z) < (1.0f / 256.0f) && lives > 0) lives -= 1;
  const bool over = st >= c.s.ep_len[c.e];
  if (over) lives = 0;
  c.s.lives[c.e] = lives;
  c.s.terminal[c.e] = (over || (c.p.L0 > 0 && lives == 0)) ? 1 : 0;
}

__device__ inline void env_new_random_game(const EnvCtx& c) {
  if (c.s.lives[c.e] == 0) env_reset(c);
  env_step_raw(c, 0u);
  u32x4 x = philox4x32(c.s.ep_step[c.e], c.id, c.s.episode[c.e], P_NOOP, c.p.k0, c.p.k1);
  const uint32_t k = x.x % (uint32_t)c.p.random_start;
  for (uint32_t i = 0; i < k; ++i) env_step_raw(c, 0u);
}

__device__ inline void env_act(const EnvCtx& c, uint32_t action, bool training) {
  float cum = 0.f;
  const int32_t start_lives = c.s.lives[c.e];
  for (int r = 0; r < c.p.action_repeat; ++r) {
    env_step_raw(c, action);
    cum = cum + c.s.reward[c.e];
    if (training && start_lives > c.s.lives[c.e]) {
      cum -= 1.0f;
      c.s.terminal[c.e] = 1;
    }
    if (c.s.terminal[c.e]) break;
  }
  c.s.reward[c.e] = cum;
}

// ---------------------------------------------------------------------------------------------
__global__ void k_pool_fill(uint8_t* __restrict__ pool, int64_t chunks_per_frame, int64_t total_chunks,
                            uint32_t k0, uint32_t k1) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total_chunks;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t f = (uint32_t)(i / chunks_per_frame), j = (uint32_t)(i - (int64_t)f * chunks_per_frame);
    u32x4 x = philox4x32(j, f, P_POOL, 0u, k0, k1);
    ((uint4*)pool)[i] = make_uint4(x.x, x.y, x.z, x.w);
  }
}

// reset every env (state zeroed, lives = 0 so new_game resets), new_random_game, and fill the
// history with HIST copies of the first screen (agent.py:35-38).  tau := HIST-1.
__global__ void __launch_bounds__(256) k_env_init(EnvParams p, EnvBufs s, int E, const uint8_t* __restrict__ pool,
                                                  uint8_t* __restrict__ ring, int R, PreGeom g,
                                                  int64_t* __restrict__ counters) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  int32_t& s_frame = *(int32_t*)(smem + a3c_pre_smem_bytes(g));   // kept in the dynamic region
  const int e = blockIdx.x;
  if (threadIdx.x == 0) {
    s.episode[e] = 0; s.ep_step[e] = 0; s.ep_len[e] = 0; s.lives[e] = 0; s.frame[e] = 0;
    s.reward[e] = 0.f; s.terminal[e] = 0;
    EnvCtx c{p, s, e, (uint32_t)(p.env_id_base + e)};
    env_new_random_game(c);
    s_frame = s.frame[e];
    if (e == 0) { counters[0] = HIST - 1; counters[1] = 0; }
  }
  __syncthreads();
  uint8_t* base = ring + (int64_t)e * R * PLANE;
  const int64_t fb = (int64_t)g.in_h * g.in_w * 3;
  a3c_preprocess_block(pool + (int64_t)s_frame * fb, base, g, smem);
  __syncthreads();
  for (int c = 1; c < HIST; ++c)
    for (int i = threadIdx.x; i < PLANE / 16; i += blockDim.x)
      ((uint4*)(base + (int64_t)(c % R) * PLANE))[i] = ((const uint4*)base)[i];
}

// one env step of env e at rollout step t: act, observe-clip, (terminal -> new_random_game),
// screen of the post-act frame -> ring slot (tau + t + 1) mod R.
__global__ void __launch_bounds__(256) k_env_step(EnvParams p, EnvBufs s, int E, const int32_t* __restrict__ actions,
                                                  float* __restrict__ rewards, uint8_t* __restrict__ terms,
                                                  float min_r, float max_r, const uint8_t* __restrict__ pool,
                                                  uint8_t* __restrict__ ring, int R, PreGeom g,
                                                  const int64_t* __restrict__ counters, int t) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  int32_t& s_frame = *(int32_t*)(smem + a3c_pre_smem_bytes(g));
  const int e = blockIdx.x;
  if (threadIdx.x == 0) {
    EnvCtx c{p, s, e, (uint32_t)(p.env_id_base + e)};
    env_act(c, (uint32_t)actions[e], true);
    const float r = s.reward[e];
    rewards[e] = fmaxf(min_r, fminf(max_r, r));
    const uint8_t term = s.terminal[e];
    terms[e] = term;
    s_frame = s.frame[e];
    if (term) env_new_random_game(c);
  }
  __syncthreads();
  const int64_t tau = counters[0] + t + 1;
  uint8_t* dst = ring + (int64_t)e * R * PLANE + (tau % R) * PLANE;
  const int64_t fb = (int64_t)g.in_h * g.in_w * 3;
  a3c_preprocess_block(pool + (int64_t)s_frame * fb, dst, g, smem);
}

int a3c_pool_fill_launch(uint8_t* pool, int P, uint32_t k0, uint32_t k1, hipStream_t s) {
  const int64_t cpf = (int64_t)SCREEN_H * SCREEN_W * 3 / 16;
  const int64_t total = cpf * P;
  hipLaunchKernelGGL(k_pool_fill, dim3(4096), dim3(256), 0, s, pool, cpf, total, k0, k1);
  A3C_CHECK(hipGetLastError());
  return 0;
}

int a3c_env_init_launch(const EnvParams& p, const EnvBufs& b, int E, const uint8_t* pool, uint8_t* ring,
                        int R, int64_t* counters, hipStream_t s) {
  PreGeom g = a3c_make_geom(SCREEN_H, SCREEN_W, IMG_OUT, IMG_OUT);
  hipLaunchKernelGGL(k_env_init, dim3(E), dim3(256), a3c_pre_smem_bytes(g) + 16, s, p, b, E, pool, ring, R, g,
                     counters);
  A3C_CHECK(hipGetLastError());
  return 0;
}

int a3c_env_step_launch(const EnvParams& p, const EnvBufs& b, int E, const int32_t* actions, float* rewards,
                        uint8_t* terms, float min_r, float max_r, const uint8_t* pool, uint8_t* ring, int R,
                        const int64_t* counters, int t, hipStream_t s) {
  PreGeom g = a3c_make_geom(SCREEN_H, SCREEN_W, IMG_OUT, IMG_OUT);
  hipLaunchKernelGGL(k_env_step, dim3(E), dim3(256), a3c_pre_smem_bytes(g) + 16, s, p, b, E, actions, rewards, terms,
                     min_r, max_r, pool, ring, R, g, counters, t);
  A3C_CHECK(hipGetLastError());
  return 0;
}

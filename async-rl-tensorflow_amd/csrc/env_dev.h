// Synthetic Atari stand-in (device side), bit-identical to oracle/synthetic_env.py, with the
// reference's interface semantics: new_game environment.py:28-33, new_random_game :35-40,
// act :78-96 (action repeat, life-loss terminal when training).
#pragma once
#include "env.h"

#define GOLDEN_MULT 2654435761u

struct EnvState {
  uint32_t episode, ep_step, ep_len;
  int32_t lives, frame;
  float reward;
  uint32_t terminal;
};

__device__ inline EnvState env_load(const EnvBufs& b, int64_t i) {
  EnvState s;
  s.episode = b.episode[i]; s.ep_step = b.ep_step[i]; s.ep_len = b.ep_len[i];
  s.lives = b.lives[i]; s.frame = b.frame[i]; s.reward = b.reward[i]; s.terminal = b.terminal[i];
  return s;
}

__device__ inline void env_store(const EnvBufs& b, int64_t i, const EnvState& s, bool frame = true) {
  b.episode[i] = s.episode; b.ep_step[i] = s.ep_step; b.ep_len[i] = s.ep_len;
  b.lives[i] = s.lives; b.reward[i] = s.reward; b.terminal[i] = (uint8_t)s.terminal;
  if (frame) b.frame[i] = s.frame;
}

// self.env.reset() (environment.py:30)
__host__ __device__ inline void env_reset(EnvState& s, const EnvParams& p, uint32_t id) {
  s.episode += 1u;
  s.ep_step = 0;
  s.lives = p.L0;
  u32x4 x = philox4x32(s.episode, id, P_RESET, 0u, p.k0, p.k1);
  s.ep_len = 200u + x.x % 1801u;
  s.frame = (int32_t)(x.y % (uint32_t)p.P);
}

// frame index of a step whose draw was x.x, for `action`
__host__ __device__ inline int32_t env_frame_of(uint32_t xx, uint32_t action, const EnvParams& p) {
  return (int32_t)((xx + action * GOLDEN_MULT) % (uint32_t)p.P);
}

// self.env.step(action) (environment.py:42-43) without the frame: nothing here depends on the
// action, which only picks the frame (env_frame_of(returned x.x, action))
__host__ __device__ inline uint32_t env_step_core(EnvState& s, const EnvParams& p, uint32_t id) {
  const uint32_t st = s.ep_step + 1u;
  s.ep_step = st;
  u32x4 x = philox4x32(st, id, s.episode, P_STEP, p.k0, p.k1);
  const float u = u01(x.y);
  const float rp = 0.02f;
  s.reward = u < rp ? 1.0f : (u >= 1.0f - rp ? -1.0f : 0.0f);
  int32_t lives = s.lives;
  if (u01(x.z) < (1.0f / 256.0f) && lives > 0) lives -= 1;
  const bool over = st >= s.ep_len;
  if (over) lives = 0;
  s.lives = lives;
  s.terminal = (over || (p.L0 > 0 && lives == 0)) ? 1u : 0u;
  return x.x;
}

// self.env.step(action) (environment.py:42-43)
__host__ __device__ inline void env_step_raw(EnvState& s, const EnvParams& p, uint32_t id, uint32_t action) {
  s.frame = env_frame_of(env_step_core(s, p, id), action, p);
}

// Environment.new_random_game (environment.py:35-40) via new_game (:28-33)
__host__ __device__ inline void env_new_random_game(EnvState& s, const EnvParams& p, uint32_t id) {
  if (s.lives == 0) env_reset(s, p, id);
  env_step_raw(s, p, id, 0u);
  u32x4 x = philox4x32(s.ep_step, id, s.episode, P_NOOP, p.k0, p.k1);
  const uint32_t k = x.x % (uint32_t)p.random_start;
  for (uint32_t i = 0; i < k; ++i) env_step_raw(s, p, id, 0u);
}

// GymEnvironment.act (environment.py:78-96) up to the frame: the repeats' rewards, lives
// and terminal do not depend on the action; returns the last executed step's draw, whose
// frame is env_frame_of(draw, action) (so the act can run before the action is drawn)
__host__ __device__ inline uint32_t env_act_pre(EnvState& s, const EnvParams& p, uint32_t id, bool training) {
  float cum = 0.f;
  const int32_t start_lives = s.lives;
  uint32_t xx = 0;
  for (int r = 0; r < p.action_repeat; ++r) {
    xx = env_step_core(s, p, id);
    cum = cum + s.reward;
    if (training && start_lives > s.lives) {
      cum -= 1.0f;
      s.terminal = 1u;
    }
    if (s.terminal) break;
  }
  s.reward = cum;
  return xx;
}

// GymEnvironment.act (environment.py:78-96)
__host__ __device__ inline void env_act(EnvState& s, const EnvParams& p, uint32_t id, uint32_t action, bool training) {
  s.frame = env_frame_of(env_act_pre(s, p, id, training), action, p);
}


// Synthetic Atari stand-in (device side), bit-identical to oracle/synthetic_env.py, with the
// reference's interface semantics: new_game environment.py:74-79, new_random_game :81-86,
// act :124-142 (action repeat, life-loss terminal when training).
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

__device__ inline void env_store(const EnvBufs& b, int64_t i, const EnvState& s) {
  b.episode[i] = s.episode; b.ep_step[i] = s.ep_step; b.ep_len[i] = s.ep_len;
  b.lives[i] = s.lives; b.frame[i] = s.frame; b.reward[i] = s.reward; b.terminal[i] = (uint8_t)s.terminal;
}

// self.env.reset() (environment.py:76)
__device__ inline void env_reset(EnvState& s, const EnvParams& p, uint32_t id) {
  s.episode += 1u;
  s.ep_step = 0;
  s.lives = p.L0;
  u32x4 x = philox4x32(s.episode, id, P_RESET, 0u, p.k0, p.k1);
  s.ep_len = 200u + x.x % 1801u;
  s.frame = (int32_t)(x.y % (uint32_t)p.P);
}

// self.env.step(action) (environment.py:88-89)
__device__ inline void env_step_raw(EnvState& s, const EnvParams& p, uint32_t id, uint32_t action) {
  const uint32_t st = s.ep_step + 1u;
  s.ep_step = st;
  u32x4 x = philox4x32(st, id, s.episode, P_STEP, p.k0, p.k1);
  const uint32_t mix = x.x + action * GOLDEN_MULT;
  s.frame = (int32_t)(mix % (uint32_t)p.P);
  const float u = u01(x.y);
  const float rp = 0.02f;
  s.reward = u < rp ? 1.0f : (u >= 1.0f - rp ? -1.0f : 0.0f);
  int32_t lives = s.lives;
  if (u01(x.z) < (1.0f / 256.0f) && lives > 0) lives -= 1;
  const bool over = st >= s.ep_len;
  if (over) lives = 0;
  s.lives = lives;
  s.terminal = (over || (p.L0 > 0 && lives == 0)) ? 1u : 0u;
}

// Environment.new_random_game (environment.py:81-86) via new_game (:74-79)
__device__ inline void env_new_random_game(EnvState& s, const EnvParams& p, uint32_t id) {
  if (s.lives == 0) env_reset(s, p, id);
  env_step_raw(s, p, id, 0u);
  u32x4 x = philox4x32(s.ep_step, id, s.episode, P_NOOP, p.k0, p.k1);
  const uint32_t k = x.x % (uint32_t)p.random_start;
  for (uint32_t i = 0; i < k; ++i) env_step_raw(s, p, id, 0u);
}

// GymEnvironment.act (environment.py:124-142)
__device__ inline void env_act(EnvState& s, const EnvParams& p, uint32_t id, uint32_t action, bool training) {
  float cum = 0.f;
  const int32_t start_lives = s.lives;
  for (int r = 0; r < p.action_repeat; ++r) {
    env_step_raw(s, p, id, action);
    cum = cum + s.reward;
    if (training && start_lives > s.lives) {
      cum -= 1.0f;
      s.terminal = 1u;
    }
    if (s.terminal) break;
  }
  s.reward = cum;
}


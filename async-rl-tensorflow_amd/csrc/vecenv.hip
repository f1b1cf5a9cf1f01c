// Standalone batched synthetic env (C-ABI a3c_env_*): the reference's Environment /
// GymEnvironment interface (environment.py:14-106) for E envs on device, used by the Python
// mirror src/environment.py.  Dynamics are env_dev.h (bit-identical to oracle/synthetic_env.py);
// screens go through the Atari Environment.screen kernel.
#include <new>
#include "env_dev.h"

int a3c_pool_fill_launch(uint8_t* pool, int P, uint32_t k0, uint32_t k1, hipStream_t s, int frame_bytes);
int a3c_launch_screen_atari(const uint8_t* rgb, const int32_t* idx, int64_t n, uint8_t* out, int64_t stride,
                            hipStream_t s);

struct a3c_env {
  EnvParams p;
  EnvBufs b;      // single-buffered: these kernels update state in place, one thread per env
  int E;
  uint8_t* pool;
  void* mem;
};

__global__ void k_venv_zero(EnvBufs b, int E) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  EnvState s = {0u, 0u, 0u, 0, 0, 0.f, 0u};
  env_store(b, e, s);
}

// op 0: new_game (environment.py:28-33), 1: new_random_game (:35-40)
__global__ void k_venv_new(EnvParams p, EnvBufs b, int E, const uint8_t* __restrict__ mask, int random) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E || (mask && !mask[e])) return;
  const uint32_t id = (uint32_t)(p.env_id_base + e);
  EnvState s = env_load(b, e);
  if (random) {
    env_new_random_game(s, p, id);
  } else {
    if (s.lives == 0) env_reset(s, p, id);
    env_step_raw(s, p, id, 0u);
  }
  env_store(b, e, s);
}

// GymEnvironment.act (environment.py:78-96) / SimpleGymEnvironment.act (:102-106 with simple=1)
__global__ void k_venv_act(EnvParams p, EnvBufs b, int E, const int32_t* __restrict__ actions, int training,
                           int simple, float* __restrict__ rewards, uint8_t* __restrict__ terms,
                           int32_t* __restrict__ frames) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const uint32_t id = (uint32_t)(p.env_id_base + e);
  EnvState s = env_load(b, e);
  if (simple) env_step_raw(s, p, id, (uint32_t)actions[e]);
  else env_act(s, p, id, (uint32_t)actions[e], training != 0);
  env_store(b, e, s);
  if (rewards) rewards[e] = s.reward;
  if (terms) terms[e] = (uint8_t)s.terminal;
  if (frames) frames[e] = s.frame;
}

extern "C" int a3c_env_create(int num_envs, int action_size, int start_lives, int random_start, int action_repeat,
                              int num_frames, uint64_t seed, int env_id_base, a3c_env** out) {
  if (!out || num_envs < 1 || action_size < 1 || random_start < 1 || action_repeat < 1 || num_frames < 1 ||
      start_lives < 0)
    return a3c_set_error(A3C_ERR_INVALID, "a3c_env_create", "bad argument");
  a3c_env* v = new (std::nothrow) a3c_env();
  if (!v) return a3c_set_error(A3C_ERR_INVALID, "a3c_env_create", "oom");
  const int64_t E = num_envs;
  const size_t state = 64 * ((E * 4 * 6 + E + 63) / 64) + 256;
  const size_t pool = (size_t)num_frames * SCREEN_H * SCREEN_W * 3;
  if (hipMalloc(&v->mem, state + pool) != hipSuccess) {
    delete v;
    return a3c_set_error(A3C_ERR_INVALID, "a3c_env_create", "hipMalloc");
  }
  uint8_t* m = (uint8_t*)v->mem;
  v->b.episode = (uint32_t*)m;
  v->b.ep_step = (uint32_t*)(m + 4 * E);
  v->b.ep_len = (uint32_t*)(m + 8 * E);
  v->b.lives = (int32_t*)(m + 12 * E);
  v->b.frame = (int32_t*)(m + 16 * E);
  v->b.reward = (float*)(m + 20 * E);
  v->b.terminal = m + 24 * E;
  v->pool = m + state;
  v->E = num_envs;
  v->p.k0 = (uint32_t)seed;
  v->p.k1 = (uint32_t)(seed >> 32);
  v->p.P = num_frames;
  v->p.A = action_size;
  v->p.L0 = start_lives;
  v->p.random_start = random_start;
  v->p.action_repeat = action_repeat;
  v->p.env_id_base = env_id_base;
  int rc = a3c_pool_fill_launch(v->pool, num_frames, v->p.k0, v->p.k1, nullptr, SCREEN_H * SCREEN_W * 3);
  if (!rc) {
    hipLaunchKernelGGL(k_venv_zero, dim3((num_envs + 63) / 64), dim3(64), 0, nullptr, v->b, num_envs);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess)
      rc = a3c_set_error(A3C_ERR_INVALID, "a3c_env_create", "init kernels failed");
  }
  if (rc) {
    (void)hipFree(v->mem);
    delete v;
    return rc;
  }
  *out = v;
  return 0;
}

extern "C" int a3c_env_destroy(a3c_env* v) {
  if (!v) return 0;
  (void)hipFree(v->mem);
  delete v;
  return 0;
}

extern "C" int a3c_env_new_game(a3c_env* v, const uint8_t* mask, int random, void* stream) {
  if (!v) return a3c_set_error(A3C_ERR_INVALID, "a3c_env_new_game", "null");
  hipLaunchKernelGGL(k_venv_new, dim3((v->E + 63) / 64), dim3(64), 0, (hipStream_t)stream, v->p, v->b, v->E, mask,
                     random);
  A3C_CHECK(hipGetLastError());
  return 0;
}

extern "C" int a3c_env_act(a3c_env* v, const int32_t* actions, int is_training, int simple, float* rewards,
                           uint8_t* terminals, int32_t* frames, void* stream) {
  if (!v || !actions) return a3c_set_error(A3C_ERR_INVALID, "a3c_env_act", "null");
  hipLaunchKernelGGL(k_venv_act, dim3((v->E + 63) / 64), dim3(64), 0, (hipStream_t)stream, v->p, v->b, v->E, actions,
                     is_training, simple, rewards, terminals, frames);
  A3C_CHECK(hipGetLastError());
  return 0;
}

extern "C" int a3c_env_screen(a3c_env* v, uint8_t* out, int64_t out_stride, void* stream) {
  if (!v || !out) return a3c_set_error(A3C_ERR_INVALID, "a3c_env_screen", "null");
  return a3c_launch_screen_atari(v->pool, v->b.frame, v->E, out, out_stride, (hipStream_t)stream);
}

extern "C" int a3c_env_buffers(a3c_env* v, uint8_t** pool, int32_t** frame, int32_t** lives, uint32_t** episode,
                               uint32_t** ep_step, float** reward, uint8_t** terminal) {
  if (!v) return a3c_set_error(A3C_ERR_INVALID, "a3c_env_buffers", "null");
  if (pool) *pool = v->pool;
  if (frame) *frame = v->b.frame;
  if (lives) *lives = v->b.lives;
  if (episode) *episode = v->b.episode;
  if (ep_step) *ep_step = v->b.ep_step;
  if (reward) *reward = v->b.reward;
  if (terminal) *terminal = v->b.terminal;
  return 0;
}

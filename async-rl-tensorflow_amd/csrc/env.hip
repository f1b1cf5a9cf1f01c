// Batched synthetic Atari stand-in on device (gym/ALE is absent; SURVEY §2 OUT OF SCOPE) with the
// reference's interface semantics, bit-identical to oracle/synthetic_env.py:
//   new_game          environment.py:28-33
//   new_random_game   environment.py:35-40
//   act               environment.py:78-96 (action repeat, life-loss terminal when training)
//   observe clip      agent.py:154
// k_env_step fuses one env step with K1 (Environment.screen) and the K2 history push: the new
// 84x84 screen is written straight into the env's frame-ring slot, so the "shift" of
// history.py:13-15 costs nothing (states are read through StateAddr).
#include "env_dev.h"
#include "preprocess_dev.h"
#include "screen_atari.h"

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
// history with HIST copies of the first screen (agent.py:35-38).  tau := HIST-1; the env
// state lives at parity (tau & 1) of the double-buffered state arrays.
__global__ void k_env_init_state(EnvParams p, EnvBufs b, int E, int64_t* __restrict__ counters) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e == 0) { counters[0] = HIST - 1; counters[1] = 0; counters[2] = 0; }   // tau, global, worker step
  if (e >= E) return;
  EnvState s = {0u, 0u, 0u, 0, 0, 0.f, 0u};
  env_new_random_game(s, p, (uint32_t)(p.env_id_base + e));
  env_store(b, (int64_t)((HIST - 1) & 1) * E + e, s);
}

// screen of each env's current frame into all HIST ring slots (grid (parts, E))
__global__ void __launch_bounds__(256) k_env_init_screens(EnvBufs b, int E, const uint8_t* __restrict__ pool,
                                                          uint8_t* __restrict__ ring, int R, PreGeom g) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int e = blockIdx.y;
  const int32_t f = b.frame[(int64_t)((HIST - 1) & 1) * E + e];
  uint8_t* base = ring + (int64_t)e * R * PLANE;
  const int64_t fb = (int64_t)g.in_h * g.in_w * 3;
  for (int c = 0; c < HIST; ++c) {
    a3c_preprocess_part(pool + (int64_t)f * fb, base + (int64_t)(c % R) * PLANE, g, blockIdx.x, smem);
    __syncthreads();
  }
}

// screen of env e's post-act frame (written by the fused head+act kernel) into ring slot
// (tau + t + 1) mod R: Environment.screen (environment.py:49-53) + History.add (history.py:13-15).
// grid (bands, E): one output band per workgroup.
template <int ROWS>
__global__ void __launch_bounds__(256) k_env_screen(int E, const int32_t* __restrict__ frames,
                                                    const uint8_t* __restrict__ pool, uint8_t* __restrict__ ring,
                                                    int R, const int64_t* __restrict__ counters, int t) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int e = blockIdx.y;
  const int64_t tau = counters[0] + t;
  atari::screen_band<ROWS>(pool + (int64_t)frames[e] * (atari::IH * atari::IW * 3),
                           ring + (int64_t)e * R * PLANE + ((tau + 1) % R) * PLANE, blockIdx.x, smem);
}

// mode M2 (pre-sized frames): frame f of the pool copied into all HIST ring slots of env e (grid E)
__global__ void __launch_bounds__(256) k_env_init_copy84(EnvBufs b, int E, const uint8_t* __restrict__ pool,
                                                         uint8_t* __restrict__ ring, int R) {
  const int e = blockIdx.x;
  const int32_t f = b.frame[(int64_t)((HIST - 1) & 1) * E + e];
  const uint4* src = (const uint4*)(pool + (int64_t)f * PLANE);
  uint8_t* base = ring + (int64_t)e * R * PLANE;
  for (int i = threadIdx.x; i < PLANE / 16; i += blockDim.x) {
    const uint4 v = src[i];
    for (int c = 0; c < HIST; ++c) ((uint4*)(base + (int64_t)(c % R) * PLANE))[i] = v;
  }
}

// frame f, 16-byte chunk j = philox(j, f, P_POOL, 0): frame_bytes = 210*160*3 (RGB frames) or
// 84*84 (mode M2 -- the first 441 chunks of the same hash)
int a3c_pool_fill_launch(uint8_t* pool, int P, uint32_t k0, uint32_t k1, hipStream_t s, int frame_bytes) {
  const int64_t cpf = frame_bytes / 16;
  const int64_t total = cpf * P;
  hipLaunchKernelGGL(k_pool_fill, dim3(4096), dim3(256), 0, s, pool, cpf, total, k0, k1);
  A3C_CHECK(hipGetLastError());
  return 0;
}

int a3c_env_init_launch(const EnvParams& p, const EnvBufs& b, int E, const uint8_t* pool, uint8_t* ring,
                        int R, int64_t* counters, hipStream_t s, int frame84) {
  PreGeom g = a3c_make_geom(SCREEN_H, SCREEN_W, IMG_OUT, IMG_OUT);
  hipLaunchKernelGGL(k_env_init_state, dim3((E + 63) / 64), dim3(64), 0, s, p, b, E, counters);
  A3C_CHECK(hipGetLastError());
  if (frame84) {
    hipLaunchKernelGGL(k_env_init_copy84, dim3(E), dim3(256), 0, s, b, E, pool, ring, R);
    A3C_CHECK(hipGetLastError());
    return 0;
  }
  hipLaunchKernelGGL(k_env_init_screens, dim3(g.parts, E), dim3(256), a3c_pre_smem_bytes(g), s, b, E, pool, ring, R, g);
  A3C_CHECK(hipGetLastError());
  return 0;
}

int a3c_env_init_screens_launch(const EnvBufs& b, int E, const uint8_t* pool, uint8_t* ring, int R, hipStream_t s) {
  PreGeom g = a3c_make_geom(SCREEN_H, SCREEN_W, IMG_OUT, IMG_OUT);
  hipLaunchKernelGGL(k_env_init_screens, dim3(g.parts, E), dim3(256), a3c_pre_smem_bytes(g), s, b, E, pool, ring, R, g);
  A3C_CHECK(hipGetLastError());
  return 0;
}

int a3c_screen_rows();

template <int ROWS>
static void launch_env_screen(int E, const int32_t* frames, const uint8_t* pool, uint8_t* ring, int R,
                              const int64_t* counters, int t, hipStream_t s) {
  hipLaunchKernelGGL(k_env_screen<ROWS>, dim3((atari::OH + ROWS - 1) / ROWS, E), dim3(256),
                     atari::Smem<ROWS>::BYTES, s, E, frames, pool, ring, R, counters, t);
}

int a3c_env_screen_launch(int E, const int32_t* frames, const uint8_t* pool, uint8_t* ring, int R,
                          const int64_t* counters, int t, hipStream_t s) {
  switch (a3c_screen_rows()) {
    case 7: launch_env_screen<7>(E, frames, pool, ring, R, counters, t, s); break;
    case 21: launch_env_screen<21>(E, frames, pool, ring, R, counters, t, s); break;
    case 28: launch_env_screen<28>(E, frames, pool, ring, R, counters, t, s); break;
    case 42: launch_env_screen<42>(E, frames, pool, ring, R, counters, t, s); break;
    case 12: launch_env_screen<12>(E, frames, pool, ring, R, counters, t, s); break;
    default: launch_env_screen<14>(E, frames, pool, ring, R, counters, t, s); break;
  }
  A3C_CHECK(hipGetLastError());
  return 0;
}

#pragma once
#include "net.h"

#define SCREEN_H 210
#define SCREEN_W 160
#define IMG_OUT IMG

struct EnvParams {
  uint32_t k0, k1;
  int P, A, L0, random_start, action_repeat, env_id_base;
};

struct EnvBufs {
  uint32_t* episode;
  uint32_t* ep_step;
  uint32_t* ep_len;
  int32_t* lives;
  int32_t* frame;
  float* reward;
  uint8_t* terminal;
};

struct PreGeom;
PreGeom a3c_make_geom(int in_h, int in_w, int out_h, int out_w);
int a3c_pool_fill_launch(uint8_t* pool, int P, uint32_t k0, uint32_t k1, hipStream_t s);
int a3c_env_init_launch(const EnvParams& p, const EnvBufs& b, int E, const uint8_t* pool, uint8_t* ring,
                        int R, int64_t* counters, hipStream_t s);
int a3c_env_step_launch(const EnvParams& p, const EnvBufs& b, int E, const int32_t* actions, float* rewards,
                        uint8_t* terms, float min_r, float max_r, const uint8_t* pool, uint8_t* ring, int R,
                        const int64_t* counters, int t, hipStream_t s);

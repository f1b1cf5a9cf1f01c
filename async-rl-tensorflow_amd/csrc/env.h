#pragma once
#include "net.h"

#define SCREEN_H 210
#define SCREEN_W 160
#define IMG_OUT IMG

struct PreGeom;
PreGeom a3c_make_geom(int in_h, int in_w, int out_h, int out_w);
int a3c_pool_fill_launch(uint8_t* pool, int P, uint32_t k0, uint32_t k1, hipStream_t s,
                         int frame_bytes = SCREEN_H * SCREEN_W * 3);
int a3c_env_init_launch(const EnvParams& p, const EnvBufs& b, int E, const uint8_t* pool, uint8_t* ring,
                        int R, int64_t* counters, hipStream_t s, int frame84 = 0);
// screen of frame env.frame[(HIST-1)&1][e] of the pool into all HIST ring slots of env e
int a3c_env_init_screens_launch(const EnvBufs& b, int E, const uint8_t* pool, uint8_t* ring, int R, hipStream_t s);
int a3c_env_screen_launch(int E, const int32_t* frames, const uint8_t* pool, uint8_t* ring, int R,
                          const int64_t* counters, int t, hipStream_t s);

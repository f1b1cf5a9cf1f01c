#pragma once
#include "a3c_common.h"
#include "../../include/a3c_hip.h"

#define SS_BLOCKS 64
enum { OPT_CLIP = 1, OPT_APPLY = 2 };

struct TensorTab {
  int n;
  int64_t off[A3C_MAX_TENSORS];
  int64_t size[A3C_MAX_TENSORS];
};

struct OptParams {
  int mode;              // OPT_CLIP | OPT_APPLY
  float clip;            // <= 0: no clipping
  float lr;              // used when step_ptr == nullptr
  const int64_t* step_ptr;  // device global step: lr = (max_step - step + 1)/max_step * lr0 (agent.py:393-395)
  int64_t step_add;
  double lr0;
  int64_t max_step;
  float rho, momentum, eps;
};

int a3c_optim_launch(float* w, float* ms, float* mom, float* grads, const TensorTab& tt, OptParams op,
                     double* part, float* sumsq_out, bool compute_sumsq, hipStream_t s);
int a3c_fill_launch(float* p, int64_t n, float v, hipStream_t s);

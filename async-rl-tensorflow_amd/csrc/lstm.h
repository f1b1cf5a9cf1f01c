// C5 LSTM policy head (BASELINE config 5).  Build-defined: the reference has no recurrent code
// (SURVEY §8(f) rank 4).  Cell = TF1 BasicLSTMCell (gate columns i, j, f, o; forget_bias 1.0)
// on the fc ReLU output; the policy / value heads read h.  Oracle: oracle/ref_cpu.py lstm_*.
#pragma once
#include "net.h"

// one step of the cell for B envs.  h_src / c_src: the previous step's raw outputs, zeroed
// where prev_terms[e] (the previous transition was terminal).  hp / cp / gates nullable.
struct LstmStep {
  const float* wt;          // gate matrix transposed, [1024][512] (a3c_lstm_transpose_launch)
  const float* h_src;
  const float* c_src;
  const uint8_t* prev_terms;
  float *hp, *cp, *gates, *h, *c;
  // the cell's input as the fc layer's FC_NS K-slice partials (a3c_fc_part_launch), folded by the
  // cell kernel in slice order + fc bias + ReLU (as the feed-forward head folds them); the folded
  // rows go to l3_out (the backward's act_l3).  nullptr: x is the finished fc output
  const float* fc_part = nullptr;
  const float* fc_bias = nullptr;
  float* l3_out = nullptr;
  // with fc_part set by the caller: the fc launch folds its own partials (k_fc_part_fold, one
  // ticket word per fc tile) and the cell reads the finished rows
  unsigned* fc_tick = nullptr;
};

int a3c_lstm_fwd_launch(const float* bias, const float* x, const LstmStep& st, int64_t B, hipStream_t s);
// Wt[1024][512] = W[512][1024]^T (once per parameter version: the rollout's forward operand)
int a3c_lstm_transpose_launch(const float* W, float* Wt, hipStream_t s);

// truncated BPTT over n steps of E envs (see include/a3c_hip.h a3c_lstm_bptt)
struct LstmSeq {
  const float *x, *hp, *cp, *gates, *c;   // [n][E][...]
  const uint8_t* terms;                   // [n][E]
};
int64_t a3c_lstm_ws_floats(int n, int64_t E);
int a3c_lstm_bptt_launch(const float* W, int n, int64_t E, const LstmSeq& q, const float* dh, float* dx,
                         float* dw, float* db, float* ws, hipStream_t s);

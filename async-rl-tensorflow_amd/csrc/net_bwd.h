#pragma once
#include "net.h"
#include "lstm.h"
#include "optim.h"

// per-workgroup partial slab of k_conv_bwd: dW1 [256][16] (unscaled by 1/255), dW2 [256][32],
// db1 [16], db2 [32]
#define CB_OFF_W1 0
#define CB_OFF_W2 (KC1 * C1_N)                    // 4096
#define CB_OFF_B1 (CB_OFF_W2 + KC2 * C2_N)         // 12288
#define CB_OFF_B2 (CB_OFF_B1 + C1_N)               // 12304
#define CB_SLAB (CB_OFF_B2 + C2_N)                 // 12336

struct FinalizeSeg {
  const float* src;       // element (r, c) of split s: src[s*split_stride + r*src_ld + col0 + c]
  int64_t split_stride;
  int nsplit, rows, src_ld, col0, ncols;
  int64_t dst_off;        // dst[dst_off + r*dst_ld + c] = scale * sum_s
  int dst_ld;
  float scale;
  int slot;               // >= 0: block x of the segment writes its fp64 sum of squares to part[slot + x]
};
#ifndef FIN_X
#define FIN_X 32          // k_finalize blocks per segment
#endif
struct FinalizeSegs {
  FinalizeSeg s[12];
  int n;
  float* dst;
  // fused per-tensor norms (engine): the segments' partials as above, then one block per
  // SS_CHUNK of the tensors the segments do not write (already final: fc weights, LSTM) and the
  // lr / target-sync schedule -- what k_sumsq would compute, without its launch
  double* part;           // nullptr: none of this
  TensorTab tt;           // partial layout (a3c_fused_tab)
  int nsum;               // tensors summed by chunk blocks
  int sum_t[4];           // their indices
  int sum_c0[5];          // prefix sums of their chunk counts
  OptParams op;
  int no_tail;            // 1: no loss / schedule block (the split backward's second finalize)
};

// engine form of the per-tensor norms: k_finalize produces the partials (layout tt) and the schedule
struct SumsqFused {
  double* part;
  const TensorTab* tt;
  const OptParams* op;
};
// the partial layout SumsqFused expects: FIN_X slots for each tensor a finalize segment writes,
// SS_CHUNK chunks for the others
int a3c_fused_tab(const NetLayout& L, TensorTab* tt);

// Split exchange (multi-GPU): the fc / head gradients -- 99 % of the bytes -- are final
// before the conv backward starts, so the backward finalizes, norms and clips them first, records
// ev_head (the exchange of that range starts on a comm stream under the conv backward), then the
// conv tensors.  Bit-identical to the one-pass clip: the same partials, the same clip math.
struct SplitBwd {
  hipEvent_t ev_head;     // recorded on the backward's stream once grads[cut:] are clipped
  OptParams clip;         // the per-worker clip (mode OPT_CLIP), its range set per pass
  float* sumsq_out;       // per-tensor squared norms (written by the second pass, all tensors)
  int64_t cut;            // float offset of the fc weights: conv tensors [0, cut), the rest [cut, total)
};

struct BwdPlan {
  int nwg, per_wg, head_split, fc_split, groups;
  int64_t dz, dh3, dl2, terms, hgrad, hcol, hslab, fccol, fcslab, cslab, cgroup, total;  // float offsets
};

// optional fused n-step returns in the head backward (engine a3c path)
struct ReturnsArgs {
  const float* rewards;      // [n][E] (nullptr: use the explicit target array)
  const uint8_t* terms;      // [n][E]
  const float* boot;         // V(s_{t+n}) at boot[e * boot_stride]
  int64_t boot_stride;
  int n;
  int64_t E;
  double gamma;
  float* R_out;              // [n*E] the returns (inspection)
};

// C5 LSTM head: the rollout's sequence buffers (engine slot) for the truncated BPTT; the
// terminals come from ReturnsArgs.terms
struct LstmBwd {
  int n;
  int64_t E;
  const float *h, *c, *hp, *cp, *gates;   // [n][E][...]
  float* dh;                              // [n*E][U] scratch: dL/dh_t from the heads
  float* ws;                              // a3c_lstm_ws_floats(n, E) floats
};

BwdPlan a3c_bwd_plan(const NetLayout& L, int64_t B, bool wks = false);
int a3c_backward_launch(const NetLayout& L, const float* params, const StateAddr& sa, int64_t B,
                        const float* act_l1, const float* act_l2, const float* act_l3,
                        const float* z, const int32_t* actions, const float* target, float beta,
                        int literal, float* grads, float* loss_out, float* ws, hipStream_t s,
                        const ReturnsArgs* ra = nullptr,
                        hipStream_t side = nullptr, hipEvent_t ev_fork = nullptr, hipEvent_t ev_join = nullptr,
                        const LstmBwd* lb = nullptr, const SumsqFused* sf = nullptr,
                        const SplitBwd* sp = nullptr, const uint32_t* l2m = nullptr);
int a3c_returns_launch(const float* rewards, const uint8_t* terms, const float* boot, int64_t boot_stride,
                       int n, int64_t E, double gamma, float* R, hipStream_t s);
// qsel != nullptr: double Q-learning -- the value of qn's row at qsel's row argmax (agent.py:176-184)
int a3c_td_target_launch(const float* rewards, const uint8_t* terms, const float* qn, int64_t B, int A,
                         int zs, double discount, float* target, hipStream_t s, const float* qsel = nullptr);
int a3c_select_launch(const float* z, int64_t B, int zs, int A, const HeadSelect& sel, hipStream_t s);
void a3c_conv12_set_smem();
void a3c_conv_bwd_set_smem();
int a3c_head_screen_fold_launch(const float* part, int nsplit, const float* fbias, float* l4, const float* Wp,
                                const float* bp, const float* Wv, const float* bv, int A, int zs, int64_t B, float* z,
                                const HeadSelect& sel, hipStream_t s);
int a3c_head_screen_wide_launch(const float* l4, const float* Wp, const float* bp, const float* Wv, const float* bv,
                                int A, int zs, int64_t B, float* z, const HeadSelect& sel, hipStream_t s);
int a3c_head_screen_launch(const NetLayout& L, const float* P, const float* act_l3, int64_t B, float* z,
                           const HeadSelect& sel, hipStream_t s);
int a3c_head_screen_conv12_launch(const NetLayout& L, const float* P, const float* act_l3, int64_t B, float* z,
                                  const HeadSelect& sel, const Conv12Next& nx, hipStream_t s);
int a3c_conv12_launch(const NetLayout& L, const float* P, const uint8_t* prep, const StateAddr& sa, int64_t B,
                      float* act_l1, float* act_l2, hipStream_t s, uint32_t* l2m = nullptr);
int a3c_conv_bwd_launch(const NetLayout& L, const float* P, const StateAddr& sa, int64_t B, const float* act_l1,
                        const float* dl2, float* ws, hipStream_t s);

// shared with the nature trunk (nature.hip): the head backward at width 256 (FC) or 512, the
// deterministic slab grouping, and k_finalize (segments + loss terms + fused norms / schedule)
int a3c_head_bwd_launch(int width, const NetLayout& L, const float* z, const int32_t* actions, const float* target,
                        const float* h, const float* Wp, const float* Wv, float beta, int literal, int64_t B,
                        float* dz, float* dh, float* terms, const ReturnsArgs& ra, int relu, hipStream_t s);
int a3c_slab_group_launch(const float* src, int nsplit, int groups, int64_t len, float* dst, hipStream_t s);
int a3c_finalize_launch(const FinalizeSegs& fs, int nsumblk, const float* terms, int64_t B, float* loss_out,
                        hipStream_t s);

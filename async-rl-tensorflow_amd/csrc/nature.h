// The "nature" trunk of the reference's A3C Network (network.py:30-42, DQN_type='nature'):
// 84x84x4 -> conv 8x8/4 32 -> conv 4x4/2 64 -> conv 3x3/1 64 -> fc 3136 -> 512 -> policy / value
// heads (network.py:60-79).  Kernels in nature.hip; the engine runs it with cfg.net.trunk =
// A3C_TRUNK_NATURE (A3C heads, feed-forward: the reference pairs it with no Q-net or LSTM).
#pragma once
#include "net.h"
#include "gemm.h"
#include "optim.h"

#define NT1_N 32                 // conv1 channels
#define NT1_O 20
#define NT1_P (NT1_O * NT1_O)    // 400
#define NT2_N 64
#define NT2_O 9
#define NT2_P (NT2_O * NT2_O)    // 81
#define NT3_N 64
#define NT3_O 7
#define NT3_P (NT3_O * NT3_O)    // 49
#define NT_K1 (8 * 8 * HIST)     // 256
#define NT_K2 (4 * 4 * NT1_N)    // 512
#define NT_K3 (3 * 3 * NT2_N)    // 576
#define NT_FLAT (NT3_P * NT3_N)  // 3136
#define NT_FC 512
#define NT_A1 (NT1_P * NT1_N)    // 12800 floats of conv1 output per sample ([20][20][32], NHWC)
#define NT_A2 (NT2_P * NT2_N)    // 5184  ([9][9][64])
// flat tensor order (TF variable order, network.py:33-42, 62-79)
enum { N_L1W = 0, N_L1B, N_L2W, N_L2B, N_L3W, N_L3B, N_FCW, N_FCB, N_HW, N_HB, N_VW, N_VB, N_NT };

// per-sample floats of the saved activations: l1 | l2 | l3 | l4
inline int64_t nat_act_floats() { return (int64_t)NT_A1 + NT_A2 + NT_FLAT + NT_FC; }

// forward of B states s_{tau0 + b / E} (sa) with parameters P.  Activations [B][...] NHWC:
// l1 [B][12800], l2 [B][5184], l3 [B][3136] (the (h,w,c) flatten of network.py's linear), l4 [B][512];
// z [B][zs] (logits, value); sel.mode >= 0: action draw + fused env act (as the NIPS head kernels).
// ws: a3c_nat_fwd_ws_floats(B) floats (split-K slabs; with w1t null, also the prepared weight
// terms, made there first).  w1t: the prepared block a3c_nat_prep_launch made from P (the engine's
// rollouts: conv1's terms at its start, then the conv2 / conv3 forms, A3C_NAT_*_OFF).
int64_t a3c_nat_fwd_ws_floats(int64_t B);
int a3c_nat_forward_launch(const NetLayout& L, const float* P, const StateAddr& sa, int64_t B, float* l1, float* l2,
                           float* l3, float* l4, float* z, const HeadSelect& sel, const uint16_t* w1t, float* ws,
                           hipStream_t s);

struct ReturnsArgs;
struct SumsqFused;
// loss + backward over B samples (network.py:81-94 with the SURVEY A11 fixes, as the NIPS path):
// gradients of every tensor into grads (TF order), loss terms summed into loss_out[4]; with sf, the
// per-tensor squared-norm partials (layout a3c_nat_fused_tab) and the lr schedule as well.
int64_t a3c_nat_bwd_ws_floats(const NetLayout& L, int64_t B);
// wt: the prepared weight terms of P (a3c_nat_prep_launch), or null: prepared into ws first
int a3c_nat_backward_launch(const NetLayout& L, const float* P, const StateAddr& sa, int64_t B, const float* l1,
                            const float* l2, const float* l3, const float* l4, const float* z,
                            const int32_t* actions, const float* target, float beta, int literal, float* grads,
                            float* loss_out, float* ws, hipStream_t s, const ReturnsArgs* ra, const SumsqFused* sf,
                            const uint16_t* wt);
int a3c_nat_fused_tab(const NetLayout& L, TensorTab* tt);
// the single launches behind both (a3c_engine_time_kernel): forward passes over B states
// (fws: the fc's split-K slabs), backward passes over B samples on the plan's buffers in bws
// (valid after a backward of the same B has filled them); w1t: the prepared block (null: the
// per-layer forms of the passes that need none)
enum { NAT_C1F = 0, NAT_C2F, NAT_C3F, NAT_FCF, NAT_C3W, NAT_C3X, NAT_C2W, NAT_C2X, NAT_C1W };
enum { NAT_FCW = NAT_C1W + 1, NAT_FCX };
// conv2 + conv3 forward run as one launch (k_nat_conv23, under NAT_C2F; NAT_C3F launches nothing)
bool a3c_nat_conv23_fused();
bool a3c_nat_conv123_fused();   // conv1 as well (NAT_C1F launches nothing)
bool a3c_nat_dx_fused();        // conv3 dX + conv2 dX as one launch under NAT_C3X (NAT_C2X launches nothing)   // (variant-selection bits of the fc backward GEMMs, nature.hip)
int a3c_nat_pass_launch(int pass, const NetLayout& L, const float* P, const StateAddr& sa, int64_t B, const float* l1,
                        const float* l2, const float* l3, const float* l4, const uint16_t* w1t, float* fws,
                        float* bws, hipStream_t s);
// the rollout start on the nature trunk: the bf16 weight terms of P into w1t (the prepared block,
// A3C_NAT_PREP_BYTES: conv1's [3][32][256] in (cin, kh, kw) order, then conv2's [3][64][512] and
// conv3's [3][64][576], each [term][cout][k] in TF k order), tau snapshot (overlap) and the
// backward's go
#define A3C_NAT_W1T_BYTES (3 * NT1_N * NT_K1 * 2)
#define A3C_NAT_W2T_OFF A3C_NAT_W1T_BYTES
#define A3C_NAT_W3T_OFF (A3C_NAT_W2T_OFF + 3 * NT2_N * NT_K2 * 2)
#define A3C_NAT_W2X_OFF (A3C_NAT_W3T_OFF + 3 * NT3_N * NT_K3 * 2)
#define NT_X2 (4 * 4 * NT2_N)     // conv2's dX form: a cin row of 16 taps x 64 cout (1024)
#define A3C_NAT_W3X_OFF (A3C_NAT_W2X_OFF + 3 * NT1_N * NT_X2 * 2)
// (+ the dX forms: conv2's [3][32 cin][16 taps x 64 cout], conv3's [3][64 cin][9 taps x 64 cout])
#define A3C_NAT_PREP_BYTES (A3C_NAT_W3X_OFF + 3 * NT2_N * NT_K3 * 2)
int a3c_nat_prep_launch(const NetLayout& L, const float* P, uint16_t* w1t, const int64_t* tau_src, int64_t* tau_dst,
                        uint32_t* sig, hipStream_t s);

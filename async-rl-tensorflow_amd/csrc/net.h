// NIPS trunk geometry (agent.py:226-252, network.py:43-52) and the flat parameter layout.
#pragma once
#include "a3c_common.h"
#include "../../include/a3c_hip.h"

// round-to-nearest-even bf16 bits of a finite float
__device__ inline uint32_t bf16_rn_bits(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return u >> 16;
}

// fixed trunk geometry: 84x84x4 -> conv 8x8/4 16 -> conv 4x4/2 32 -> fc 256
#define IMG 84
#define PLANE (IMG * IMG)      // 7056 bytes per u8 frame plane
#define C1_K 8
#define C1_S 4
#define C1_O 20                 // conv1 output side
#define C1_N 16                 // conv1 channels
#define C1_P (C1_O * C1_O)      // 400 positions
#define C2_K 4
#define C2_S 2
#define C2_O 9
#define C2_N 32
#define C2_Q (C2_O * C2_O)      // 81 positions
#define FLAT (C2_Q * C2_N)      // 2592
#define FC 256
#define HIST 4
#define KC1 (C1_K * C1_K * HIST) // 256 = conv1 reduction length
#define KC2 (C2_K * C2_K * C1_N) // 256 = conv2 reduction length
#define L1S_LD 20               // LDS row stride (floats) of the conv1 output tile

enum { T_L1W = 0, T_L1B, T_L2W, T_L2B, T_FCW, T_FCB, T_HW, T_HB, T_VW, T_VB, T_LW, T_LB };
#define LSTM_U 256              // C5 LSTM head width (A3C_LSTM_UNITS)
#define LSTM_K (FC + LSTM_U)    // 512 = [x, h] rows of the gate matrix
#define LSTM_G (4 * LSTM_U)     // 1024 gate columns (i, j, f, o)

struct NetLayout {
  int algo, A, zs;
  int trunk;                // A3C_TRUNK_NIPS (tensor order T_*), A3C_TRUNK_NATURE (nature.h N_*)
  int lstm;                 // 1: LSTM head (tensors T_LW, T_LB; heads read the LSTM's h)
  int nt;
  int64_t off[A3C_MAX_TENSORS], size[A3C_MAX_TENSORS];
  int64_t total;
};

inline int a3c_zs(int algo, int A) {
  int w = algo == A3C_ALGO_A3C ? A + 1 : A;
  return (w + 3) & ~3;
}

inline int a3c_make_layout(const a3c_net_desc* d, NetLayout* L) {
  if (!d) return -1;
  // the nature trunk (network.py:30-42) belongs to the A3C Network only: feed-forward policy /
  // value heads (the reference's Q-net, agent.py:226-252, is NIPS-only, and has no LSTM)
  const bool nature = d->trunk == A3C_TRUNK_NATURE;
  if ((d->trunk != A3C_TRUNK_NIPS && !nature) || d->history_length != HIST || d->screen_h != IMG ||
      d->screen_w != IMG || d->action_size < 1 || d->action_size > 31 ||
      (d->algo != A3C_ALGO_A3C && d->algo != A3C_ALGO_Q) ||
      (d->lstm_units != 0 && (d->lstm_units != LSTM_U || d->algo != A3C_ALGO_A3C)) ||
      (nature && (d->algo != A3C_ALGO_A3C || d->lstm_units != 0)))
    return -1;
  const int A = d->action_size;
  L->algo = d->algo;
  L->A = A;
  L->zs = a3c_zs(d->algo, A);
  L->trunk = d->trunk;
  L->lstm = d->lstm_units != 0;
  if (nature) {   // l1..l3 conv [kh,kw,cin,cout] + bias, l4 [3136,512] + bias, p [512,A] + bias, q [512,1] + bias
    const int64_t ns[12] = {8 * 8 * HIST * 32, 32, 4 * 4 * 32 * 64, 64, 3 * 3 * 64 * 64, 64, 3136LL * 512, 512,
                            512LL * A, A, 512, 1};
    L->nt = 12;
    int64_t o = 0;
    for (int i = 0; i < L->nt; ++i) {
      L->off[i] = o;
      L->size[i] = ns[i];
      o += (ns[i] + 63) & ~(int64_t)63;
    }
    L->total = o;
    return 0;
  }
  int64_t sizes[12] = {(int64_t)KC1 * C1_N, C1_N, (int64_t)KC2 * C2_N, C2_N, (int64_t)FLAT * FC, FC,
                       (int64_t)FC * A, A, FC, 1, (int64_t)LSTM_K * LSTM_G, LSTM_G};
  L->nt = d->algo == A3C_ALGO_A3C ? (L->lstm ? 12 : 10) : 8;
  int64_t o = 0;
  for (int i = 0; i < L->nt; ++i) {
    L->off[i] = o;
    L->size[i] = sizes[i];
    o += (sizes[i] + 63) & ~(int64_t)63;
  }
  L->total = o;
  return 0;
}

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

struct HeadSelect {
  int mode;                 // -1 none, 0 categorical (a3c), 1 epsilon-greedy argmax (q)
  uint32_t k0, k1;          // philox key (seed)
  const int64_t* tau_ptr;   // device tau (nullable)
  int64_t tau_add;          // tau = *tau_ptr + tau_add
  const int32_t* env_ids;   // nullable: env id = env_id_base + (b % E)
  int env_id_base;
  int E;
  const float* eps;         // mode 1: per env (index b % E)
  // mode 1, when set: the head computes the env's epsilon at the worker's own step instead of
  // reading eps (agent.py:142-144, step = tau_ptr[2] + tau - (HIST-1); one launch fewer per
  // rollout step than a separate schedule kernel: Q sync 3.447M -> 3.547M env-steps/s)
  const float* ep_end;      // per env final epsilon (index b % E)
  float ep_start;
  int64_t ep_end_t, learn_start;
  int32_t* actions;         // [B]
  // fused env step (engine rollout): act() on the drawn action right after predict, as the
  // reference worker does (agent.py:59-62); env state double-buffered by (tau & 1)
  int env_on;
  int par_E;                // env-state parity stride (all envs of the engine); envb is
                            // pre-offset to this launch's first env
  EnvParams envp;
  EnvBufs envb;
  float* rewards;           // [E] observe-clipped reward (agent.py:154)
  float* rewards_raw;       // [E] nullable: the unclipped act() reward (train_with_summary's sums)
  uint8_t* terms;           // [E]
  int32_t* frames_out;      // [E] post-act frame index (the screen the history gets)
  // fused Environment.screen of the post-act frame into the frame ring (engine rollout):
  // ring slot (tau + 1) % R of env e <- screen(pool[frame]); null ring -> separate kernel
  const uint8_t* pool;
  uint8_t* ring;
  int R;
  int frame84;              // 1: pool frames are pre-sized 84x84 screens (mode M2): a copy
  // measurement only (a3c_engine_time_kernel): offsets the post-act frame index so that every
  // timed launch streams a different set of frames from HBM, as the live rollout does; 0 in
  // every product launch
  uint32_t frame_salt;
  // k_head_fwd only (the overlap rollout's bootstrap head, its last kernel): *adv_ptr += adv_n
  // once the launch's heads are written (the rollout's tau advance, no kernel of its own)
  int64_t* adv_ptr;
  int64_t adv_n;
  // k_head_screen_conv12 only (fused overlap rollout): the fc layer arrives as FC_NS K-slice
  // partials fc_part[x][b][FC] (k_fc_part); the head folds them in slice order, + fc_bias, ReLU,
  // and writes the layer output row to l3_out[b] (the backward's activation)
  const float* fc_part;
  const float* fc_bias;
  float* l3_out;
};
#define FC_NS 8                 // K-slices of the partial fc (= waves of k_head_screen_conv12)

// forward of B states; returns 0 or error
// prep: the forward's prepared weights of `params` (a3c_prep_fwd_launch, PREP_BYTES):
// conv1 split into bf16 terms (W1S_ELEMS u16) then the fc weights in MFMA fragment order
#define W1S_ELEMS (C1_K * 3 * 64 * 8)   // 12288 bf16
#define PREP_W1S_BYTES (W1S_ELEMS * 2)  // 24576
#define FC_CH (FLAT / 16)               // 162 K-chunks of 16
#define FC_CH32 (FLAT / 32)             // 81 K-chunks of 32
#define PREP_W2F_OFF (PREP_W1S_BYTES + FLAT * FC * 4)
#define W2F_ELEMS (2 * 8 * 64 * 8)      // conv2 weights (16x16x32), as three bf16 terms each
#define PREP_BYTES (PREP_W2F_OFF + W2F_ELEMS * 3 * 2)
struct LstmStep;
// the next state's conv1 + conv2, fused into rollout step t's head + screen kernel
// (k_head_screen_conv12): s_{t+1} addressing, conv weights (prep'd W1 terms) and outputs
struct Conv12Next {
  StateAddr sa;
  const uint16_t* w1s;
  const float* b1;
  const float* W2;
  const float* b2;
  float* act_l1;            // nullable: the bootstrap state keeps no l1
  float* act_l2;
  uint32_t* l2m;            // nullable: act_l2's ReLU mask as bits [b][81] (the backward's dl2 epilogue)
};
// ls (LSTM head, C5): the cell step runs on act_l3 and the heads read ls->h
int a3c_forward_launch(const NetLayout& L, const float* params, const uint8_t* prep, const StateAddr& sa,
                       int64_t B, float* act_l1, float* act_l2, float* act_l3, float* z, const HeadSelect& sel,
                       hipStream_t s, const LstmStep* ls = nullptr, bool skip_conv12 = false,
                       const Conv12Next* next = nullptr, float* fc_part = nullptr, uint32_t* l2m = nullptr);
// fc layer as FC_NS K-slice partials part[x][M][FC] (folded by k_head_screen_conv12's head)
// adv_ptr: the launch also advances the device tau counter by adv_n (thread 0 of block 0; the fc
// reads no tau) -- the rollout's last kernel when the bootstrap head runs on the backward stream
int a3c_fc_part_launch(const float* A, const float* Wp, float* part, int64_t M, hipStream_t s,
                       int64_t* adv_ptr = nullptr, int adv_n = 0);
// the policy / value head of B states from the fc's K-slice partials (fold + bias + ReLU + head,
// k_head_fwd): z rows, no action draw
// the same with the fold in the launch (C5): each tile's last K-slice workgroup folds the FC_NS
// partials in slice order + fbias + ReLU into fout[M][FC]; tick: one zeroed word per 32 x 64 tile,
// (ceil(M / 32) * 4), left zeroed by the launch
int a3c_fc_part_fold_launch(const float* A, const float* Wp, float* part, int64_t M, unsigned* tick,
                            const float* fbias, float* fout, hipStream_t s);
int a3c_head_fold_launch(const NetLayout& L, const float* P, const float* fc_part, int64_t B, float* z,
                         hipStream_t s);
int a3c_fcp_split();
void a3c_set_fcp_split(int ks);
// tau_src / tau_dst (nullable): *tau_dst = *tau_src as well (the overlap rollout's tau snapshot);
// sig (nullable): *sig += 1 (a system-scope atomic: the engine's rollout sequence)
int a3c_prep_fwd_launch(const NetLayout& L, const float* P, uint8_t* prep, hipStream_t s,
                        const int64_t* tau_src = nullptr, int64_t* tau_dst = nullptr,
                        uint32_t* sig = nullptr);
// true while enqueuing work that runs concurrently with another stream (engine overlap mode)
bool a3c_shared_gpu();
void a3c_set_shared_gpu(bool v);
bool a3c_lean_cbwd();
void a3c_set_bwd_bound(bool v);

// stage the HIST u8 planes of state b into LDS (HIST x 441 uint4)
__device__ inline void stage_state(const StateAddr& sa, int64_t b, int64_t tau0, uint8_t* x8) {
  for (int i = threadIdx.x; i < HIST * (PLANE / 16); i += blockDim.x) {
    int c = i / (PLANE / 16), j = i - c * (PLANE / 16);
    const uint4* src = (const uint4*)state_plane(sa, b, c, tau0);
    ((uint4*)(x8 + c * PLANE))[j] = src[j];
  }
}

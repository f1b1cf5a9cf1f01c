/*
 * a3c_hip.h -- C-ABI of liba3c_hip.so, the MI355X (gfx950) rollout + gradient path of
 * datavizweb/async-rl-tensorflow re-built as hand-written HIP kernels.
 *
 * The reference has no FFI: its boundary is the Python object API.
 * Each entry point below names the reference interface (file:line under the reference
 * root) whose arithmetic it replaces; the Python mirror in
 * async-rl-tensorflow_amd/src/ binds them through ctypes.
 *
 * Conventions
 *  - extern "C", plain pointers and sizes; every pointer is a CALLER-OWNED device buffer
 *    unless stated.  Nothing here allocates on the hot path; a3c_engine_create is the only
 *    allocating call (one-time workspace).
 *  - every call enqueues on the caller's stream (`stream` is a hipStream_t; NULL = legacy
 *    default stream) and returns an int status: 0 = ok, otherwise a hipError_t value or one
 *    of the A3C_ERR_* codes; a3c_last_error() gives the message.  No C++ exception crosses
 *    the ABI.  The Python side raises ValueError / RuntimeError (network.py:21,28,54).
 *  - no call is re-entrant on the same engine handle.
 */
#ifndef A3C_HIP_H
#define A3C_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define A3C_OK 0
#define A3C_ERR_INVALID 10001   /* bad argument / unsupported shape            */
#define A3C_ERR_STATE 10002     /* engine used in the wrong order               */

#define A3C_ALGO_A3C 0          /* policy + value heads (src/network.py:60-94) */
#define A3C_ALGO_Q 1            /* one-step Q-learning head (src/agent.py:251-254) */

#define A3C_TRUNK_NIPS 0        /* 16/32/256 trunk: agent.py:226-251, network.py:43-52 */
#define A3C_TRUNK_NATURE 1      /* 32/64/64/512 trunk: network.py:30-42 (A3C heads only)   */
#define A3C_LSTM_UNITS 256      /* C5 LSTM head width (build-defined: the reference has no
                                   recurrent code)                 */

const char* a3c_version(void);
const char* a3c_last_error(void);
/* 1 when a gfx950 device is visible (no compute). */
int a3c_device_ok(void);

/* ----------------------------------------------------------------------------
 * Network description and flat parameter layout.
 * Flat fp32 vector in TF variable order (ops.py:21,24,36,38; agent.py:226-252 /
 * network.py:47-79); each tensor starts at a 64-float (256 B) aligned offset,
 * padding floats are zero and stay zero.
 *  a3c : l1_w[8,8,4,16] l1_b l2_w[4,4,16,32] l2_b l4_w[2592,256] l4_b p_w[256,A] p_b q_w[256,1] q_b
 *  q   : l1_w l1_b l2_w l2_b l3_w[2592,256] l3_b q_w[256,A] q_b
 *  a3c, nature trunk: l1_w[8,8,4,32] l1_b l2_w[4,4,32,64] l2_b l3_w[3,3,64,64] l3_b
 *        l4_w[3136,512] l4_b p_w[512,A] p_b q_w[512,1] q_b   (network.py:30-42, 62-79)
 *  a3c + LSTM head (lstm_units = 256, BASELINE config 5): the a3c list, then
 *        lstm_w[256+U, 4U] lstm_b[4U]   (TF1 BasicLSTMCell "Matrix"/"Bias", gate columns
 *        i, j, f, o, forget_bias 1.0); the policy / value heads read the LSTM's h.
 * -------------------------------------------------------------------------- */
typedef struct a3c_net_desc {
  int algo;            /* A3C_ALGO_*                                       */
  int trunk;           /* A3C_TRUNK_NIPS, or A3C_TRUNK_NATURE (algo A3C, no LSTM: the
                          engine only; the per-op a3c_forward / a3c_loss_backward are NIPS) */
  int action_size;     /* A (<= 31)                                        */
  int history_length;  /* 4 (config.py:22)                                 */
  int screen_h;        /* 84                                               */
  int screen_w;        /* 84                                               */
  int lstm_units;      /* 0: feed-forward head; A3C_LSTM_UNITS: LSTM head (a3c only).  The
                          batch-independent a3c_forward / a3c_loss_backward reject it (a
                          recurrent head needs the sequence: a3c_lstm_step / a3c_lstm_bptt
                          or the engine). */
} a3c_net_desc;

#define A3C_MAX_TENSORS 16
/* n_tensors, offsets[i], sizes[i] (floats), total padded length. */
int a3c_param_layout(const a3c_net_desc* net, int* n_tensors, int64_t* offsets, int64_t* sizes,
                     int64_t* total);
/* bytes of scratch a3c_forward / a3c_loss_backward need for batch B */
int a3c_workspace_bytes(const a3c_net_desc* net, int64_t B, int64_t* bytes);

/* ----------------------------------------------------------------------------
 * The nature trunk (network.py:30-42, Network(DQN_type='nature')): net->trunk =
 * A3C_TRUNK_NATURE, algo A3C, history_length 4.  Stateless forward / loss + backward over B
 * states (u8 planes [B][4][84][84], 16-B aligned), implicit-GEMM kernels of nature.hip:
 *   l1 [B][20][20][32], l2 [B][9][9][64], l3 [B][3136] (conv3 out, (h,w,c) flatten),
 *   l4 [B][512] (fc out), z [B][zs] (logits, value).  The backward (network.py:81-94 with the
 *   A11 fixes) reads the forward's activations; grads [total] in the flat layout, loss_out[4].
 * Replace network.py:30-42 + 81-94 (the TF graph of the nature trunk, its compute_gradients).
 * -------------------------------------------------------------------------- */
int a3c_nature_workspace_bytes(const a3c_net_desc* net, int64_t B, int64_t* bytes);
int a3c_nature_forward(const a3c_net_desc* net, const float* params, const uint8_t* states, int64_t B,
                       float* l1, float* l2, float* l3, float* l4, float* z, void* workspace, void* stream);
int a3c_nature_loss_backward(const a3c_net_desc* net, const float* params, const uint8_t* states, int64_t B,
                             const float* l1, const float* l2, const float* l3, const float* l4, const float* z,
                             const int32_t* actions, const float* target, float beta, int literal_adv,
                             float* grads, float* loss_out, void* workspace, void* stream);

/* ----------------------------------------------------------------------------
 * K1  Environment.screen (environment.py:49-53): fp64 luminance truncated to u8, then
 *     Pillow BILINEAR fixed-point resample (scipy.misc.imresize, environment.py:5-8).
 *     rgb frames [*, in_h, in_w, 3] u8; frame i reads rgb + (frame_idx ? frame_idx[i] : i)
 *     * in_h*in_w*3 and writes out + i*out_stride ([out_h][out_w] u8).  Bit-exact.
 * -------------------------------------------------------------------------- */
int a3c_preprocess_u8(const uint8_t* rgb, const int32_t* frame_idx, int64_t n, int in_h, int in_w,
                      uint8_t* out, int64_t out_stride, int out_h, int out_w, void* stream);

/* luminance step alone (environment.py:51-52): out[i] = uint8(fp64 0.2126R+0.7152G+0.0722B)
 * for npix RGB pixels, in the exact integer form the Atari screen kernel uses. */
int a3c_luminance_u8(const uint8_t* rgb, int64_t npix, uint8_t* out, void* stream);

/* ----------------------------------------------------------------------------
 * K2  History (history.py:3-27).  hist is [n][L][h*w] u8 (oldest plane first);
 *     push: if reset_mask && reset_mask[i]: zero (History.reset, :17-18); then shift one
 *     plane and append screens[i] (History.add, :13-15).
 *     get: float32 copy, NHWC [n][h][w][L] when nhwc else [n][L][h][w] (History.get, :20-24).
 * -------------------------------------------------------------------------- */
int a3c_history_push(uint8_t* hist, const uint8_t* screens, const uint8_t* reset_mask, int64_t n,
                     int L, int64_t hw, void* stream);
int a3c_history_get_f32(const uint8_t* hist, int64_t n, int L, int h, int w, int nhwc, float* out,
                        void* stream);

/* ----------------------------------------------------------------------------
 * Forward (agent.py:217-254 q-net / network.py:43-79 a3c net, ops.py:4-46).
 *  states  [B][L][84][84] u8 (frame values; the /255 of agent.py:226 is applied inside)
 *  act_l1  [B][400][16]  f32 conv1 out (nullable: only needed for a3c_loss_backward)
 *  act_l2  [B][2592]     f32 conv2 out, (h,w,c) flatten order (agent.py:231-232)
 *  act_l3  [B][256]      f32 fc out
 *  z       [B][zs]       f32 head: a3c -> A logits then V at column A; q -> A q-values.
 *                         zs = a3c_z_stride(net).
 * -------------------------------------------------------------------------- */
int a3c_z_stride(const a3c_net_desc* net);
int a3c_forward(const a3c_net_desc* net, const float* params, const uint8_t* states, int64_t B,
                float* act_l1, float* act_l2, float* act_l3, float* z, void* workspace,
                void* stream);

/* ----------------------------------------------------------------------------
 * K6  action selection.
 *  mode 0 (a3c, network.py:65-72 softmax + batch_sample): categorical draw
 *        u = philox(seed; tau, env_ids[i], P_ACTION); first j with fp32 cumsum(pi)[j] > u.
 *  mode 1 (q, agent.py:141-151): if u01(x0) < eps[i]: x1 % A  else argmax_j q[j]
 *        (first maximum, tf.argmax agent.py:254).
 *  env_ids nullable (= i).  eps nullable in mode 0.
 * -------------------------------------------------------------------------- */
int a3c_select_action(int mode, const float* z, int64_t B, int zs, int A, const float* eps,
                      uint64_t seed, int64_t tau, const int32_t* env_ids, int32_t* actions,
                      void* stream);

/* ----------------------------------------------------------------------------
 * K7  n-step returns (assets/a3c.png Algorithm S3) over [n][E] in float64:
 *     R = bootstrap[e] (0 if terminals[n-1]); R <- r_i + gamma*R, reset at terminals.
 *     TD target (agent.py:186-190): (1-term)*discount*max_a q_next[i][a] + reward[i] (fp64).
 * -------------------------------------------------------------------------- */
int a3c_returns(const float* rewards, const uint8_t* terminals, const float* bootstrap, int n,
                int64_t E, double gamma, float* R, void* stream);
int a3c_td_target(const float* rewards, const uint8_t* terminals, const float* q_next, int64_t B,
                  int A, int zs, double discount, float* target, void* stream);

/* ----------------------------------------------------------------------------
 * K8+K9  loss + backward (network.py:81-94 with the SURVEY §8 A11 fixes / agent.py:306-317).
 *  target: a3c -> R (n-step return); q -> TD target.
 *  a3c loss per sample  -log pi(a)*stopgrad(R-V) - beta*H + (R-V)^2/2, summed over B
 *      (literal_adv != 0: no stop-gradient, network.py:83-84 literal form);
 *  q   loss mean((target - Q[a])^2) over B (agent.py:313-314).
 *  grads: flat fp32 (layout of a3c_param_layout), OVERWRITTEN.
 *  loss_out (device, 4 floats): a3c {policy_sum, value_sum, entropy_sum, total_sum};
 *                               q {loss, mean_q_acted, 0, 0}.
 * -------------------------------------------------------------------------- */
int a3c_loss_backward(const a3c_net_desc* net, const float* params, const uint8_t* states,
                      int64_t B, const float* act_l1, const float* act_l2, const float* act_l3,
                      const float* z, const int32_t* actions, const float* target, float beta,
                      int literal_adv, float* grads, float* loss_out, void* workspace,
                      void* stream);

/* ----------------------------------------------------------------------------
 * K10+K11  per-tensor clip_by_norm (agent.py:316-319) + TF ApplyRMSProp
 *  (main.py:63-65, agent.py:321): ms += (g^2-ms)(1-rho); mom = mom*momentum +
 *  lr*g/sqrt(ms+eps); w -= mom.  ms must be initialised to 1.0, mom to 0 (TF1 slots).
 *  clip <= 0 disables clipping.  sumsq_out (nullable, device, n_tensors floats) receives
 *  the pre-clip squared norms.  workspace >= a3c_optim_workspace_bytes().
 *  a3c_clip_grads only clips in place (multi-GPU: clip per worker, then all-reduce).
 * -------------------------------------------------------------------------- */
int a3c_optim_workspace_bytes(int64_t total, int64_t* bytes);
int a3c_clip_grads(float* grads, int n_tensors, const int64_t* offsets, const int64_t* sizes,
                   float clip, float* sumsq_out, void* workspace, void* stream);
int a3c_clip_rmsprop_apply(float* params, float* ms, float* mom, float* grads, int n_tensors,
                           const int64_t* offsets, const int64_t* sizes, float lr, float rho,
                           float momentum, float eps, float clip, float* sumsq_out,
                           void* workspace, void* stream);

/* ----------------------------------------------------------------------------
 * Generic layer ops (ops.py:4-46 drop-ins, any shape; off the hot path).
 *  conv2d VALID, weights [kh,kw,cin,cout] (ops.py:16-21), x NHWC [N,H,W,C] or NCHW [N,C,H,W]
 *  (nhwc flag), y likewise; bias nullable; relu = activation_fn tf.nn.relu (ops.py:27-28).
 *  backward: dx (nullable) / dw, db (nullable) -- OVERWRITTEN.
 *  matmul: C[m][n] (+)= sum_k A[m*sam+k*sak] * B[k*sbk+n*sbn] (+bias[n]) (relu) -- linear
 *  (ops.py:41-46) and its gradients through the strides.
 * -------------------------------------------------------------------------- */
int a3c_conv2d_forward(const float* x, const float* w, const float* b, float* y, int N, int H, int W, int C,
                       int KH, int KW, int SH, int SW, int OC, int nhwc, int relu, void* stream);
int a3c_conv2d_backward(const float* x, const float* w, const float* dy, float* dx, float* dw, float* db, int N,
                        int H, int W, int C, int KH, int KW, int SH, int SW, int OC, int nhwc, void* stream);
int a3c_matmul(const float* A, int64_t sam, int64_t sak, const float* B, int64_t sbk, int64_t sbn, float* C,
               int64_t ldc, int M, int N, int K, const float* bias, int relu, int accumulate, void* stream);

/* ----------------------------------------------------------------------------
 * C5  LSTM head (BASELINE config 5; no reference code -- build-defined after TF1
 *     BasicLSTMCell, forget_bias 1.0, and the A3C-LSTM of assets/a3c.png's paper).
 *  a3c_lstm_transpose: w_t [4U][256+U] = w^T, the forward's operand layout (once per
 *    parameter version).
 *  a3c_lstm_step: one cell step for B envs on w_t.  x [B][256] (fc ReLU output), h_src/c_src [B][U]
 *    the previous step's outputs; prev_terms [B] (nullable): state zeroed where the previous
 *    transition was terminal.  Writes h/c [B][U]; hp/cp (the masked inputs it used) and gates
 *    ([B][4U], activated i, j, f, o) are nullable (only the backward needs them).
 *  a3c_lstm_bptt: truncated BPTT over n steps of E envs (b = t*E + e), given dh [n*E][U] =
 *    dL/dh_t from the heads.  dx [n*E][256] = dL/dx_t masked by x > 0 (the fc ReLU: ready for
 *    the fc backward); dw [256+U][4U], db [4U] OVERWRITTEN.  terms [n][E] (transition t
 *    terminal -> no gradient flows from step t+1 into step t's state).
 * -------------------------------------------------------------------------- */
int a3c_lstm_transpose(const float* w, float* w_t, void* stream);
int a3c_lstm_step(const float* w_t, const float* b, const float* x, const float* h_src, const float* c_src,
                  const uint8_t* prev_terms, int64_t B, float* hp, float* cp, float* gates, float* h,
                  float* c, void* stream);
int a3c_lstm_workspace_bytes(int n, int64_t E, int64_t* bytes);
int a3c_lstm_bptt(const float* w, int n, int64_t E, const float* x, const float* hp, const float* cp,
                  const float* gates, const float* c, const uint8_t* terms, const float* dh, float* dx,
                  float* dw, float* db, void* workspace, void* stream);

/* K12  target sync (agent.py:342-344) / theta' <- theta (network.py:96-107). */
int a3c_copy_params(float* dst, const float* src, int64_t n, void* stream);

/* ----------------------------------------------------------------------------
 * Hogwild parameter server across GPUs (main.py:58-66 ps with unlocked RMSProp,
 * SURVEY §8(e) "async"): every GPU owns a byte-range shard of params / ms / mom in
 * its HBM, exported over IPC; workers push clipped gradients straight into every
 * shard with an unlocked elementwise RMSProp over xGMI and pull the parameters back
 * at rollout start (theta' <- theta, network.py:96-107).
 *  a3c_dev_alloc/free: plain hipMalloc'd device memory (IPC-exportable base pointer).
 *  a3c_dev_alloc_kind: the same with kind 0 coarse-grained (= a3c_dev_alloc), 1 fine-grained
 *                      (hipDeviceMallocFinegrained: peer writes coherent at instruction
 *                      granularity, the Hogwild shards' default), 2 uncached; free with a3c_dev_free.
 *  a3c_ipc_handle:     64-byte hipIpcMemHandle of such a base pointer.
 *  a3c_ipc_open/close: map a peer's handle (lazy peer access) into this process.
 *  a3c_rmsprop_range:  TF ApplyRMSProp on n elements (w, ms, mom may live on a peer
 *                      GPU); lr read from lr_dev[0] when lr_dev != NULL.
 * -------------------------------------------------------------------------- */
int a3c_dev_alloc(int64_t bytes, void** out);
int a3c_dev_alloc_kind(int64_t bytes, int kind, void** out);
int a3c_dev_free(void* p);
int a3c_ipc_handle(void* base, void* handle64);
int a3c_ipc_open(const void* handle64, void** out);
int a3c_ipc_close(void* p);
int a3c_rmsprop_range(float* w, float* ms, float* mom, const float* grads, int64_t n, const float* lr_dev,
                      float lr, float rho, float momentum, float eps, void* stream);

/* ----------------------------------------------------------------------------
 * Batched synthetic Atari env (gym/ALE is absent): the Environment / GymEnvironment interface
 * of environment.py:14-106 for E envs on device (dynamics: oracle/synthetic_env.py).
 *  new_game(random=0): environment.py:28-33; random=1: new_random_game :35-40 (mask nullable)
 *  act: GymEnvironment.act :78-96 (simple=1: SimpleGymEnvironment.act :102-106); outputs
 *       reward / terminal / frame index per env (each nullable), state updated in place
 *  screen: Environment.screen :49-53 of every env's current frame -> out + e*out_stride
 * -------------------------------------------------------------------------- */
typedef struct a3c_env a3c_env;
int a3c_env_create(int num_envs, int action_size, int start_lives, int random_start, int action_repeat,
                   int num_frames, uint64_t seed, int env_id_base, a3c_env** out);
int a3c_env_destroy(a3c_env* env);
int a3c_env_new_game(a3c_env* env, const uint8_t* mask, int random, void* stream);
int a3c_env_act(a3c_env* env, const int32_t* actions, int is_training, int simple, float* rewards,
                uint8_t* terminals, int32_t* frames, void* stream);
int a3c_env_screen(a3c_env* env, uint8_t* out, int64_t out_stride, void* stream);
int a3c_env_buffers(a3c_env* env, uint8_t** pool, int32_t** frame, int32_t** lives, uint32_t** episode,
                    uint32_t** ep_step, float** reward, uint8_t** terminal);

/* ----------------------------------------------------------------------------
 * Batched actor-learner engine: E envs per GPU stepped in lock-step on device
 * (synthetic ALE stand-in, oracle/synthetic_env.py semantics), n-step rollout,
 * backward, per-tensor clip, RMSProp.  One process per GPU; the multi-GPU gradient
 * exchange happens between a3c_engine_rollout_grad and a3c_engine_apply (RCCL from the
 * host, on the same stream).
 * -------------------------------------------------------------------------- */
typedef struct a3c_engine a3c_engine;

typedef struct a3c_engine_config {
  a3c_net_desc net;
  int num_envs;          /* E per GPU                                              */
  int n_step;            /* rollout length n (a3c 5; q: train_frequency 32)          */
  int env_id_base;       /* global id of this GPU's env 0 (rank * E)                 */
  int world_size;        /* GPUs taking part (lr schedule counts their env-steps)    */
  int start_lives;       /* 0 Pong, 5 Breakout, 3 SpaceInvaders                      */
  int random_start;      /* config.py:7 (30)                                          */
  int action_repeat;     /* config.py:50 (1)                                          */
  int num_frames;        /* synthetic frame pool size (HBM resident RGB frames)       */
  int use_graph;         /* 1: capture the rollout / backward into hipGraphs; default 0
                            (eager launches: faster on MI355X)          */
  uint64_t seed;         /* main.py:35 random_seed (123)                             */
  double gamma;          /* config.py:9 discount 0.99                                 */
  float beta;            /* config.py:16 entropy weight 0.01                          */
  float learning_rate;   /* config.py:11 7e-4                                          */
  int64_t max_step;      /* config.py:5 8e7                                           */
  float decay, momentum, epsilon;   /* main.py:64-65: 0.99, 0, 0.1                    */
  float clip_norm;       /* agent.py:319: 40                                          */
  int literal_adv;       /* 1: network.py literal un-stopped advantage gradient       */
  /* q-learning only */
  float ep_start, ep_end; int64_t ep_end_t, learn_start;  /* config.py:18-25         */
  int64_t target_q_update_step;   /* config.py:10 (4e4)                               */
  double discount;                /* config.py:9                                      */
  int overlap;        /* 1 (a3c, q; not with host envs): rollout k runs on an engine stream while the backward +
                        apply of rollout k-1 run on the caller's stream; rollout k uses the
                        parameters after update k-2 (A3C stale-parameter asynchrony, fixed
                        staleness 1).  0: synchronous rollout -> grad -> apply.          */
  int external_env;   /* 1: the envs are stepped by the host (real ALE / gym workers,
                        SURVEY §8(f)1): a3c_engine_ext_* below feed their RGB frames,
                        rewards and terminals each step; no synthetic env, no frame pool
                        (num_frames ignored).  Synchronous engines only.                 */
  int frame84;        /* 1: measurement mode M2: the pool holds pre-sized 84x84
                        grey frames (the north star's synthetic 84x84x4 states), so the env
                        step's Environment.screen becomes a 7 KB copy into the history ring.
                        0 (default, M1): raw 210x160x3 RGB frames, screen computed on device. */
  int split_exchange; /* 1 (world_size > 1, eager launches): the backward clips the fc / head
                        gradients (99 % of the bytes) before the conv backward and records an
                        event there, so the partitioned-PS exchange of that range runs on a comm
                        stream under the conv backward (a3c_engine_wait_grad_head); only the
                        conv tensors' exchange waits for the whole backward.  Gradients are
                        bit-identical either way.  Default 1.                                 */
  int double_q;       /* q only: double Q-learning (agent.py:176-184) -- the TD target of transition
                        t takes the target net's q of s_{t+1} at the online net's argmax action
                        (the rollout's own q rows, plus one online forward of the bootstrap state
                        s_n) instead of the target net's max.  Default 0.                     */
} a3c_engine_config;

void a3c_engine_config_default(a3c_engine_config* cfg);
int a3c_engine_create(const a3c_engine_config* cfg, a3c_engine** out);
int a3c_engine_destroy(a3c_engine* eng);
/* fill the frame pool, reset the envs (new_random_game, environment.py:35-40), fill each
 * history with 4 copies of the first screen (agent.py:37-38) and initialise params
 * from host memory (nullable -> keep), rms slot = 1, mom = 0. */
int a3c_engine_reset(a3c_engine* eng, const float* host_params, void* stream);
/* n rollout steps + bootstrap + loss + backward + per-tensor clip -> grads */
int a3c_engine_rollout_grad(a3c_engine* eng, void* stream);
/* RMSProp apply of grads (lr from the device worker step, agent.py:393-395) and advance counters.
 * overlap: a no-op until the pipeline holds a gradient (first call after reset). */
int a3c_engine_apply(a3c_engine* eng, void* stream);
/* a3c_engine_rollout_grad + a3c_engine_apply as one enqueue (single GPU, device envs only: no
 * gradient exchange between them), the apply captured into the same hipGraphs.  Same results
 * bit for bit; a3c_engine_grad_ready reports as after a3c_engine_rollout_grad, and a following
 * a3c_engine_apply is a no-op (the gradient is applied already). */
int a3c_engine_iterate(a3c_engine* eng, void* stream);
/* 1 if the last a3c_engine_rollout_grad produced a gradient (always, unless overlap and it
 * was the first call after reset) -- exchange / apply only then. */
int a3c_engine_grad_ready(a3c_engine* eng);
/* advance tau / global step as a3c_engine_apply does, without touching the parameters
 * (Hogwild: the gradient went to the shared shards instead) */
int a3c_engine_advance(a3c_engine* eng, void* stream);

/* Partitioned parameter server: the multi-GPU form of the reference's PS (main.py:58-66), where
 * every worker's per-worker-clipped gradient (agent.py:316-319) is its own RMSProp step on the
 * shared variables (agent.py:321), applied in arrival order.  Rank r of W owns the flat range
 * [lo, lo + n) of params / ms / mom.  Per iteration, after a3c_engine_rollout_grad (world_size > 1:
 * grads hold this worker's clipped gradient):
 *   host: all-to-all of grads -> grads_by_rank [W][n] (rank q's gradient of this range);
 *   a3c_engine_apply_shard: the W RMSProp steps of the range, in rank order q = 0..W-1 (lr from the
 *     device schedule), new weights -> w_out [n];
 *   host: all-gather of every rank's w_out -> the full parameter vector;
 *   a3c_engine_apply_commit: params <- params_src (nullable: already there), overlap snapshot,
 *     target sync (q), counters -- the rest of a3c_engine_apply.
 * Both are no-ops when no gradient is pending (overlap pipeline filling). */
int a3c_engine_apply_shard(a3c_engine* eng, const float* grads_by_rank, int nranks, int64_t lo, int64_t n,
                           float* w_out, void* stream);
int a3c_engine_apply_commit(a3c_engine* eng, const float* params_src, void* stream);
/* Split exchange (cfg.split_exchange, world_size > 1): the backward clips grads[cut:] (fc + heads,
 * 99 % of the bytes) before the conv backward and marks it; the exchange of that range (all-to-all,
 * a3c_engine_apply_shard of its part of each owned range, all-gather) then runs on a comm stream
 * under the conv backward, and only grads[:cut] (the conv tensors, ~50 KB) wait for the whole
 * backward (src/distributed.py PartitionedPS).  The same apply_shard / apply_commit calls, on the
 * sub-ranges; results bit-identical to the one-phase exchange.
 *   a3c_engine_exchange_split: *cut (0: the engine does not split);
 *   a3c_engine_wait_grad_head: `stream` waits for grads[cut:] of the last rollout_grad. */
int a3c_engine_exchange_split(a3c_engine* eng, int64_t* cut);
int a3c_engine_wait_grad_head(a3c_engine* eng, void* stream);

/* ----------------------------------------------------------------------------
 * Summaries: the aggregates train_with_summary logs every test_step
 * (agent.py:69-139), kept on device over every env of this GPU.
 *  stats_accumulate: adds the rollout whose gradient the last rollout_grad / iterate computed
 *                    (enqueue after it on the same stream; a no-op while no gradient is ready).
 *  stats_read:       waits for `stream`, copies the A3C_STATS_N doubles; reset = 1 starts a new
 *                    interval (each env's running episode reward carries on).
 * out: [0] sum of act() rewards (unclipped, every env-step; agent.py:101), [1] sum, [2] max,
 *      [3] min of finished episodes' rewards (the terminal step's reward excluded, agent.py:91-98;
 *      max -inf / min +inf when none), [4] games, [5] sum over updates of the per-sample loss
 *      (q: the MSE, agent.py:196; a3c: total / (n*E)), [6] sum over updates of the batch mean
 *      Q(s) (q: over actions, agent.py:200; a3c: V(s)), [7] updates, [8] env-steps, [9..11] sums
 *      of per-sample policy loss, value loss, entropy (a3c). */
#define A3C_STATS_N 16
int a3c_engine_stats_accumulate(a3c_engine* eng, void* stream);
int a3c_engine_stats_read(a3c_engine* eng, double* out, int reset, void* stream);

/* ----------------------------------------------------------------------------
 * Checkpoint / resume.  Replaces the Supervisor's Saver (main.py:74-90, which saves
 * the prediction weights + `step` every 600 s, agent.py:29) and its restore at managed_session.
 *  set_step:    resume from parameters + step only (what the reference's Saver keeps; the caller
 *               writes params / target / RMSProp slots through a3c_engine_get_buffers): the global
 *               step T (agent.py:165) and the workers' loop counter (agent.py:34,46,55: the lr and
 *               epsilon schedules run on it) restart at the given values.  After a3c_engine_reset.
 *  state_*:     the whole engine state -- parameters, target, RMSProp slots, counters, env state,
 *               frame ring, LSTM carry and, in overlap mode, the rollout in flight -- so a restored
 *               engine of the same configuration continues the run bit for bit.  state_save / load
 *               wait for the engine's streams; load needs a3c_engine_reset first (frame pool).
 *               Engines with host-stepped envs (external_env) refuse: the host envs cannot be
 *               snapshotted, they resume with set_step. */
int a3c_engine_set_step(a3c_engine* eng, int64_t global_step, int64_t worker_step, void* stream);
int a3c_engine_state_bytes(a3c_engine* eng, int64_t* bytes);
int a3c_engine_state_save(a3c_engine* eng, void* host, int64_t bytes, void* stream);
int a3c_engine_state_load(a3c_engine* eng, const void* host, int64_t bytes, void* stream);

/* ----------------------------------------------------------------------------
 * External (host-stepped) environments, cfg.external_env = 1.  Per rollout:
 *   for t in 0..n-1:  a3c_engine_ext_act -> sync -> host steps every env with its action
 *                     (GymEnvironment.act, environment.py:78-96; new_random_game on a
 *                     terminal, agent.py:66-67) -> a3c_engine_ext_observe
 *   a3c_engine_rollout_grad (bootstrap + loss + backward) -> [exchange] -> a3c_engine_apply.
 * Host pointers should be pinned (hipHostMalloc / torch pin_memory) for async copies; device
 * pointers work too (hipMemcpyDefault).
 *  ext_begin:   rgb [E][210][160][3] u8 first frames of each env (after new_random_game):
 *               every history slot <- its screen (agent.py:33-38), tau / step counters reset.
 *  ext_act:     predict of step t (agent.py:141-151 / network.py:65-72 draw); actions [E] i32.
 *  ext_observe: post-act frames rgb, rewards [E] f32 (clipped here, agent.py:154), terminals
 *               [E] u8 -> Environment.screen (environment.py:49-53) + History.add.
 * -------------------------------------------------------------------------- */
int a3c_engine_ext_begin(a3c_engine* eng, const uint8_t* rgb, void* stream);
int a3c_engine_ext_act(a3c_engine* eng, int32_t* actions, void* stream);
int a3c_engine_ext_observe(a3c_engine* eng, const uint8_t* rgb, const float* rewards, const uint8_t* terminals,
                           void* stream);
/* part of observe (same step, before it): frames of envs [env_lo, env_hi) only, so the copy of
 * one range overlaps the host stepping of the next; observe is then called with rgb = NULL, which
 * fails with A3C_ERR_STATE unless the step's ranges covered every env in [0, E) */
int a3c_engine_ext_upload(a3c_engine* eng, const uint8_t* rgb, int env_lo, int env_hi, void* stream);

/* Host-side batched synthetic env (the device env's emulator, bit-identical dynamics, stepped by
 * `threads` CPU threads): raw RGB frames into caller host buffers -- a stand-in for real ALE
 * worker processes when driving / measuring the external-env path.  No GPU work.
 *  begin: new_random_game of every env; first frames -> rgb [E][210][160][3] u8
 *  step:  GymEnvironment.act (environment.py:78-96) of every env, post-act frames -> rgb,
 *         rewards [E] f32 (unclipped), terminals [E] u8; new_random_game where terminal
 *         (agent.py:66-67). */
typedef struct a3c_hostenv a3c_hostenv;
int a3c_hostenv_create(int num_envs, int action_size, int start_lives, int random_start, int action_repeat,
                       int num_frames, uint64_t seed, int env_id_base, int threads, a3c_hostenv** out);
int a3c_hostenv_destroy(a3c_hostenv* env);
int a3c_hostenv_begin(a3c_hostenv* env, uint8_t* rgb);
int a3c_hostenv_step(a3c_hostenv* env, const int32_t* actions, int is_training, uint8_t* rgb, float* rewards,
                     uint8_t* terminals);
/* step of envs [env_lo, env_hi) only (buffers stay full-size, indexed by env) */
int a3c_hostenv_step_range(a3c_hostenv* env, const int32_t* actions, int is_training, uint8_t* rgb,
                           float* rewards, uint8_t* terminals, int env_lo, int env_hi);

/* device pointers owned by the engine (valid until destroy) */
typedef struct a3c_engine_buffers {
  float* params; float* target_params; float* ms; float* mom; float* grads;
  int64_t n_params;
  uint8_t* frame_ring;     /* [E][R][84*84] u8                                */
  int ring_slots;
  int64_t* tau;            /* device: current frame index tau; tau[2] = the workers' base step
                              (worker step of rollout step t = tau[2] + tau - 3 + t)  */
  int64_t* global_step;    /* device: env-steps taken by all GPUs (= tau + 1)  */
  int32_t* actions;        /* [n][E]                                           */
  float* rewards;          /* [n][E]                                           */
  uint8_t* terminals;      /* [n][E]                                           */
  float* z;                /* [(n+1)][E][zs] (row n = bootstrap forward)       */
  float* returns;          /* [n][E] R or TD target                            */
  float* loss;             /* [4]                                              */
  float* sumsq;            /* [n_tensors] pre-clip squared norms               */
  float* act_l1; float* act_l2; float* act_l3;  /* [n*E][...]                  */
  uint8_t* frame_pool;     /* [num_frames][210][160][3]                        */
  int32_t* env_frame; int32_t* env_lives; uint32_t* env_episode; uint32_t* env_step;
  uint32_t* env_len;
  int zs; int n_tensors; int64_t offsets[A3C_MAX_TENSORS]; int64_t sizes[A3C_MAX_TENSORS];
  float* sched;            /* device: [0] learning rate of the last gradient (agent.py:393-395) */
  /* LSTM head (net.lstm_units > 0), per rollout step t: h_t, c_t [n][E][U]; the masked state
   * inputs hp, cp [n][E][U]; activated gates [n][E][4U].  NULL without the LSTM head. */
  float* lstm_h; float* lstm_c; float* lstm_hp; float* lstm_cp; float* lstm_gates;
  int lstm_units;
  /* nature trunk (net.trunk = A3C_TRUNK_NATURE): act_l1 [n*E][20][20][32], act_l2 [n*E][9][9][64],
   * act_l3 [n*E][3136] (the conv3 output, (h,w,c)-flattened), act_l4 [n*E][512] (fc out);
   * NIPS: act_l4 NULL */
  float* act_l4;
  int trunk;
} a3c_engine_buffers;
int a3c_engine_get_buffers(a3c_engine* eng, a3c_engine_buffers* out);
/* same, with the rollout buffers (actions .. act_l3) of slot 0 or 1 (overlap: rollout k
 * writes slot k & 1); get_buffers == slot 0 */
int a3c_engine_slot_buffers(a3c_engine* eng, int slot, a3c_engine_buffers* out);

/* profiling hook: average device time (ms) of `iters` back-to-back launches of one engine
 * kernel on its live buffers, bracketed by HIP events on `stream` (idempotent: each
 * relaunch recomputes the same outputs). */
#define A3C_KER_CONV12_FWD 0   /* conv1+conv2 forward, B = E (saves conv1 out)          */
#define A3C_KER_FC_FWD 1       /* fc 2592->256 forward GEMM (+split-K reduce), B = E     */
#define A3C_KER_ENV_STEP 2     /* Environment.screen of the post-act frames into the ring */
#define A3C_KER_CONV_BWD 3     /* fused conv backward over B = n*E                       */
#define A3C_KER_HEAD_SCREEN 4  /* fused head + action draw + Environment.screen, B = E    */
#define A3C_KER_HEAD_SCREEN_CONV12 5  /* ... + conv1+conv2 of the next states (overlap mode) */
#define A3C_KER_FC_PART 6      /* fc as K-slice partials (overlap mode; the head folds them)  */
/* nature trunk engines (nature.hip k_nat_gemm passes): forward over E states of the live
 * parameters, backward passes over the n*E samples of the last back-propagated rollout */
/* The release build runs the three forward convolutions of a state as ONE launch (the per-state
 * kernel k_nat_conv23, nature.hip) under A3C_KER_NAT_C2F; A3C_KER_NAT_C1F and _C3F then have no
 * launch of their own and a3c_engine_time_kernel returns A3C_ERR_INVALID for them (likewise
 * _C2X in builds that fuse the two dX passes under _C3X). */
#define A3C_KER_NAT_C1F 7      /* conv1 8x8/4 4->32 forward (u8 ring -> l1), B = E         */
#define A3C_KER_NAT_C2F 8      /* conv2 4x4/2 32->64 forward (release: conv1+conv2+conv3)  */
#define A3C_KER_NAT_C3F 9      /* conv3 3x3/1 64->64 forward                               */
#define A3C_KER_NAT_FCF 10     /* fc 3136->512 forward (split-K GEMM + bias/ReLU fold)      */
#define A3C_KER_NAT_C3W 11     /* conv3 weight gradient (slabs), B = n*E                  */
#define A3C_KER_NAT_C3X 12     /* conv3 input gradient dl2                                 */
#define A3C_KER_NAT_C2W 13     /* conv2 weight gradient                                    */
#define A3C_KER_NAT_C2X 14     /* conv2 input gradient dl1 (4 stride-parity classes)       */
#define A3C_KER_NAT_C1W 15     /* conv1 weight gradient from the u8 planes                 */
/* Live launch spans, recorded by the kernels themselves inside the engine's graphs (which 0:
 * k_conv_bwd, 1: k_head_screen_conv12): per launch, last workgroup end - first workgroup start
 * (s_memrealtime).  reset = 1 clears the records (before a timed region); otherwise returns the
 * average and max span in microseconds and the number of launches recorded (at most 1024). */
int a3c_engine_span_stats(a3c_engine* eng, int which, int reset, double* avg_us, double* max_us,
                          int64_t* launches);
/* The same records of k_head_screen_conv12 (which = 1) split by rollout step: avg_us[t] is the
 * average live span of the launch that runs step t's head (t = 0..n-1; the last one also runs the
 * bootstrap state's conv1+conv2), launches[t] how many were recorded.  Call synchronised, after a
 * timed region with no a3c_engine_set_step/reset since the records were cleared. */
int a3c_engine_span_steps(a3c_engine* eng, double* avg_us, int64_t* launches);
/* The raw records behind both (measurement): out[2 r], out[2 r + 1] = first workgroup start and
 * last workgroup end (s_memrealtime ticks, 100 MHz; 0 = not recorded) of record r < 1024 of
 * `which`, and the live tau counter (records are keyed by tau, see a3c_engine_span_steps). */
int a3c_engine_span_raw(a3c_engine* eng, int which, unsigned long long* out, int64_t* tau_now);
int a3c_engine_time_kernel(a3c_engine* eng, int kernel, int iters, void* stream, float* avg_ms);

#ifdef __cplusplus
}
#endif
#endif /* A3C_HIP_H */

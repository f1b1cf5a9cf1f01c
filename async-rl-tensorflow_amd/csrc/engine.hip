// Batched actor-learner engine (one per GPU): E envs stepped in lock-step on device, n-step
// rollout with the forward of every step, bootstrap forward, returns, loss + backward, per-tensor
// clip, then (after the host's optional RCCL all-reduce of the clipped gradients) RMSProp apply.
//
// Reference loop it replaces (per worker): agent.py:52-67 train -> predict (:141-151) ->
// env.act (environment.py:78-96) -> observe (agent.py:153-167) -> batch_update (agent.py:169-207) with the
// shared RMSProp apply on the parameter server (main.py:60-66).  A3C (network.py + assets/a3c.png)
// uses n-step returns instead of the TD target; algo Q keeps agent.py's target network.
//
// All per-iteration varying quantities (tau = frame counter, global env-step count, epsilon)
// live in device memory, so the whole rollout+backward sequence is captured once into a hipGraph
// and replayed (no host work per kernel).
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>
#include "env.h"
#include "net_bwd.h"
#include "optim.h"
#include "gemm.h"
#include "nature.h"

void a3c_init_once();
int a3c_fc_fwd_launch(const float* A, const float* W, const float* bias, float* C, int64_t M, hipStream_t s,
                      const float* Wrows = nullptr);

// Per-rollout buffers.  Sync mode has one slot whose params are the live parameters and whose
// tau is the live frame counter.  Overlap mode (cfg.overlap = 1) has two: rollout k fills slot
// k & 1 with its own parameter snapshot and tau while the backward + apply of rollout k-1 (slot
// (k-1) & 1) runs on the caller's stream -- A3C's stale-parameter asynchrony at a fixed
// staleness of one update.
struct Slot {
  float* P;                // params the rollout (and its backward) use
  int64_t* tau;            // tau at rollout start (sync: the live counter)
  int32_t* actions;        // [n][E]
  int32_t* frames;         // [n][E] post-act frame index per step
  float* rewards;          // [n][E] observe-clipped (agent.py:154)
  float* rewards_raw;      // [n][E] unclipped act() rewards (the summaries' sums, agent.py:91-100)
  uint8_t* terms;          // [n][E]
  float* z;                // [(n+1)][E][zs]
  float* R_buf;            // [n][E] returns / TD targets
  float *act_l1, *act_l2, *act_l3;
  float* act_l4;           // nature trunk: the fc output [n*E][512] (act_l1..3: its conv outputs)
  float* nscr;             // nature trunk: the bootstrap state's activations [E][l1 | l2 | l3 | l4]
  uint32_t* l2m;           // act_l2's ReLU mask as bits [n*E][81], written by the forward's conv2
  float *scr_l2, *scr_l3;  // bootstrap / target forward scratch
  float* fcboot;           // boot_bwd: the bootstrap state's fc partials, read by the slot's backward
  uint8_t* prep;           // forward weights of P prepared for the kernels (k_prep_fwd)
  // C5 LSTM head: per step h_t, c_t, masked inputs hp, cp [n][E][U], gates [n][E][4U];
  // bootstrap-step h, c [E][U]
  float *lh, *lc, *lhp, *lcp, *lg, *lhb, *lcb;
  float* lwt;              // LSTM gate matrix of P, transposed for the forward (rollout start)
};

// graphs: 0 sync rollout+grad; 1, 2 rollout of slot 0, 1; 3, 4 grad of slot 0, 1; and with the
// apply fused (a3c_engine_iterate, world_size 1): 5 sync rollout+grad+apply; 6, 7 grad+apply
// (+ the parameter snapshot) of slot 0, 1
#define NGRAPH 8
struct a3c_engine {
  a3c_engine_config cfg;
  NetLayout L;
  int E, n, R;
  int64_t nE;
  uint32_t k0, k1;
  std::vector<void*> allocs;
  float *params, *tparams, *ms, *mom, *grads;
  uint8_t *ring, *pool;
  int64_t* counters;  // [0] tau, [1] global step
  EnvBufs env;
  EnvParams envp;
  int overlap, nslot;
  int fused_screen;        // 1: screen kernel fused into the head (k_head_screen)
  int frame84;             // cfg.frame84: pre-sized 84x84 pool frames (measurement mode M2)
  int fuse_conv;           // 1: step t+1's conv1 + conv2 fused into step t's head + screen
  unsigned long long* spans;  // [2][SPAN_RECS][2]: live launch spans of k_conv_bwd, k_head_screen_conv12
  Slot slot[2];
  float* loss;
  float* sumsq;
  float* zt;               // q: target-net q values [nE][zs]
  uint8_t* prep_t;         // q: prepared forward weights of the target network
  float* ep_end;           // q: per env final epsilon
  float* ws;               // backward workspace
  float* fcpart;           // fused overlap rollout: the fc as FC_NS K-slice partials [FC_NS][E][FC]
  unsigned* fctick;        // C5 with lstm_fcfold: k_fc_part_fold's ticket word per 32 x 64 fc tile (zeroed)
  int lstm_fcfold;         // C5: the fc launch folds its partials (k_fc_part_fold), not every cell workgroup
  int fc_split;            // 1: the fused rollout's fc runs as k_fc_part + the head's fold
  int nat;                 // the nature trunk (cfg.net.trunk = A3C_TRUNK_NATURE, nature.hip)
  float* nat_fws;          // nature trunk: the rollout forward's fc split-K slabs
  float* lws;              // LSTM BPTT workspace (a3c_lstm_ws_floats)
  float* ldh;              // LSTM: dL/dh_t from the heads [nE][U]
  double* opt_part;
  float* sched;            // [0] lr, [1] target-sync flag (device)
  double* stats;           // [A3C_STATS_N] train_with_summary aggregates since the last read
  double* ep_acc;          // [E] running episode reward per env (agent.py:91-98)
  TensorTab tt;
  TensorTab tt_f;             // partial layout of the norms the backward's finalize produces (a3c_fused_tab)
  // sync: one graph (rollout + grad); overlap: rollout and grad graphs per slot
  hipGraph_t graph[NGRAPH];
  hipGraphExec_t gexec[NGRAPH];
  bool captured[NGRAPH];
  // overlap pipeline
  hipStream_t rs;          // rollout stream
  hipStream_t gs;          // backward side stream (weight-gradient GEMMs beside the conv backward)
  hipEvent_t ev_gfork, ev_gjoin;
  hipEvent_t ev_start, ev_roll[2];
  // split exchange (several GPUs, cfg.split_exchange): ev_head marks the fc / head gradients
  // clipped, mid-backward; a comm stream waits on it (a3c_engine_wait_grad_head)
  int split;
  hipEvent_t ev_head;
  int l2bits;              // the forward writes act_l2's ReLU bits and the dl2 epilogue reads them
  // cross-stream ordering by stream memory operations (hipStreamWriteValue32 / WaitValue32 on
  // monotonic counters in device memory) instead of events: measured 3.6 us per hop against
  // 12-40 us for hipEventRecord + hipStreamWaitEvent (tools/waitvalue_probe.py)
  int wait_value;
  uint32_t* xflags;        // [0]: caller-stream sequence, [1]: rollout-stream sequence
  uint32_t s_seq, r_seq, roll_seq[2];
  // external (host) envs: the host steps the envs between ext_act and ext_observe
  int ext;                 // cfg.external_env
  int ext_t;               // next rollout step (0..n; n: ready for rollout_grad)
  bool ext_begun;          // a3c_engine_ext_begin done since reset
  int32_t* ext_idx;        // [E] identity frame index into the staging buffer (pool)
  std::vector<uint8_t> ext_sent;   // [E] env frame sent by a3c_engine_ext_upload this step
  int ext_nsent;                   // envs marked in ext_sent
  bool ext_acted;                  // ext_act of step ext_t issued, its ext_observe not yet
  int64_t iter;            // rollouts issued since reset
  int64_t step0_g, step0_w;   // global / worker step the counters start from (a3c_engine_set_step)
  bool grad_ready;         // the last rollout_grad call computed a gradient
  bool grad_applied;       // ... and a3c_engine_iterate already applied it (apply is then a no-op)
  bool reset_done;
};

// k_fc_part_fold's ticket words: one per 32-row x 64-column tile of the E-row fc
static size_t fctick_bytes(int64_t E) { return (size_t)((E + 31) / 32) * (FC / 64) * sizeof(unsigned); }

static int dalloc(a3c_engine* e, void** p, size_t bytes) {
  bytes = (bytes + 255) & ~(size_t)255;
  if (bytes == 0) bytes = 256;
  hipError_t st = hipMalloc(p, bytes);
  if (st != hipSuccess) return a3c_set_error((int)st, "a3c_engine_create", "hipMalloc failed");
  e->allocs.push_back(*p);
  return 0;
}

extern "C" void a3c_engine_config_default(a3c_engine_config* c) {
  memset(c, 0, sizeof(*c));
  c->net.algo = A3C_ALGO_A3C;
  c->net.trunk = A3C_TRUNK_NIPS;
  c->net.action_size = 6;
  c->net.history_length = 4;
  c->net.screen_h = 84;
  c->net.screen_w = 84;
  c->num_envs = 256;
  c->n_step = 5;
  c->overlap = 0;
  c->env_id_base = 0;
  c->world_size = 1;
  c->start_lives = 0;
  c->random_start = 30;
  c->action_repeat = 1;
  c->num_frames = 1024;
  // eager by default: measured on MI355X (ROCm 7), each hipGraph launch ends ~13 us before the next
  // packet on its stream starts, and the overlap pipeline puts one graph end per stream on the
  // critical path of every iteration; eager dispatch from a host thread that runs ahead costs
  // less (Pong 256 envs: overlap 4.56M vs 4.44M env-steps/s, sync 3.45M vs 3.43M)
  c->use_graph = 0;
  c->seed = 123;
  c->gamma = 0.99;
  c->beta = 0.01f;
  c->learning_rate = 0.0007f;
  c->max_step = 80000000LL;
  c->decay = 0.99f;
  c->momentum = 0.0f;
  c->epsilon = 0.1f;
  c->clip_norm = 40.0f;
  c->literal_adv = 0;
  c->ep_start = 1.0f;
  c->ep_end = 0.1f;
  c->ep_end_t = 4000000LL;
  c->learn_start = 32;
  c->target_q_update_step = 40000LL;
  c->discount = 0.99;
  c->split_exchange = 1;   // several GPUs: the fc / head exchange under the conv backward
}

extern "C" int a3c_engine_destroy(a3c_engine* e) {
  if (!e) return 0;
  if (e->rs) (void)hipStreamSynchronize(e->rs);
  for (int i = 0; i < NGRAPH; ++i)
    if (e->captured[i]) {
      (void)hipGraphExecDestroy(e->gexec[i]);
      (void)hipGraphDestroy(e->graph[i]);
    }
  if (e->rs) (void)hipStreamDestroy(e->rs);
  if (e->gs) (void)hipStreamDestroy(e->gs);
  if (e->ev_gfork) (void)hipEventDestroy(e->ev_gfork);
  if (e->ev_gjoin) (void)hipEventDestroy(e->ev_gjoin);
  if (e->ev_start) (void)hipEventDestroy(e->ev_start);
  if (e->ev_head) (void)hipEventDestroy(e->ev_head);
  for (int k = 0; k < 2; ++k) {
    if (e->ev_roll[k]) (void)hipEventDestroy(e->ev_roll[k]);
  }
  for (void* p : e->allocs) (void)hipFree(p);
  delete e;
  return 0;
}

static int frame_bytes(const a3c_engine* e) { return e->frame84 ? PLANE : SCREEN_H * SCREEN_W * 3; }

static bool boot_bwd(const a3c_engine* e);
static int l2bits_choice(const a3c_engine* e);
extern "C" int a3c_engine_create(const a3c_engine_config* cfg, a3c_engine** out) {
  if (!cfg || !out) return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_create", "null");
  *out = nullptr;
  a3c_engine* e = new (std::nothrow) a3c_engine();
  if (!e) return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_create", "oom");
  e->cfg = *cfg;
  if (a3c_make_layout(&cfg->net, &e->L) || cfg->num_envs < 1 || cfg->n_step < 1 || cfg->n_step > 64 ||
      cfg->num_frames < 1 || cfg->random_start < 1 || cfg->action_repeat < 1 || cfg->world_size < 1 ||
      (cfg->overlap && cfg->external_env) || (cfg->overlap && cfg->net.lstm_units && cfg->net.algo != A3C_ALGO_A3C) ||
      (cfg->net.lstm_units && !cfg->overlap && cfg->n_step < 2)) {   // sync n=1 would read and
                                                                       // write one state buffer
    delete e;
    return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_create", "bad config");
  }
  if (cfg->double_q && cfg->net.algo != A3C_ALGO_Q) {
    delete e;
    return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_create", "double_q is a Q-learning option (agent.py:176-184)");
  }
  a3c_init_once();
  const NetLayout& L = e->L;
  e->E = cfg->num_envs;
  e->n = cfg->n_step;
  e->overlap = cfg->overlap ? 1 : 0;
  e->ext = cfg->external_env ? 1 : 0;
  if (e->ext) e->cfg.num_frames = cfg->num_envs;   // the pool is the host frames' staging buffer
  e->fused_screen = 1;
  e->fused_screen = A3C_KNOB("A3C_FUSED_SCREEN", e->fused_screen) != 0;
  // overlap mode only: measured on MI355X (Pong, 256 envs) 3.65M -> 3.84M env-steps/s overlapped,
  // but 3.25M -> 3.08M in sync mode, where the unfused kernels run their bigger variants
  // (1024-thread screen, early-W2 conv12) with the GPU to themselves
  e->fuse_conv = e->overlap;
  e->fuse_conv = A3C_KNOB("A3C_FUSE_CONV", e->fuse_conv) != 0;
  e->fc_split = 1;
  e->fc_split = A3C_KNOB("A3C_FC_SPLIT", e->fc_split) != 0;
  e->frame84 = cfg->frame84 ? 1 : 0;
  e->lstm_fcfold = 0;
  e->lstm_fcfold = A3C_KNOB("A3C_LSTM_FCFOLD", e->lstm_fcfold) != 0;
  // the nature trunk (network.py:30-42) runs its own passes (nature.hip): of the NIPS fusions only
  // the head + act + screen kernel (its 512-wide form), the exchange one-phase
  e->nat = L.trunk == A3C_TRUNK_NATURE ? 1 : 0;
  if (e->nat) {
    e->fuse_conv = 0;
    e->fc_split = 0;
    if (e->ext) {
      delete e;
      return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_create", "the nature trunk runs with device envs");
    }
  }
  if (e->frame84 && (e->ext || !e->fused_screen)) {   // the copy lives in the fused head kernels
    delete e;
    return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_create", "frame84 needs device envs and the fused screen");
  }
  e->nslot = e->overlap ? 2 : 1;
  // ring: the states of one rollout (frames tau-3 .. tau+n); overlap keeps two rollouts' frames
  e->R = (e->overlap ? 2 * e->n : e->n) + HIST + (cfg->net.algo == A3C_ALGO_Q ? 1 : 0);
  e->nE = (int64_t)e->n * e->E;
  e->k0 = (uint32_t)cfg->seed;
  e->k1 = (uint32_t)(cfg->seed >> 32);
  const int64_t nE = e->nE, E = e->E;
  const int zs = L.zs;
  int rc = 0;
#define ALLOC(ptr, bytes) do { void* _p; if ((rc = dalloc(e, &_p, (size_t)(bytes)))) { a3c_engine_destroy(e); return rc; } ptr = (decltype(ptr))_p; } while (0)
  ALLOC(e->params, L.total * 4);
  ALLOC(e->tparams, L.total * 4);
  ALLOC(e->ms, L.total * 4);
  ALLOC(e->mom, L.total * 4);
  ALLOC(e->grads, L.total * 4);
  ALLOC(e->ring, (int64_t)E * e->R * PLANE);
  ALLOC(e->pool, (int64_t)e->cfg.num_frames * frame_bytes(e));
  ALLOC(e->ext_idx, E * 4);
  ALLOC(e->counters, 64);
  ALLOC(e->xflags, 64);
  ALLOC(e->env.episode, 2 * E * 4);
  ALLOC(e->env.ep_step, 2 * E * 4);
  ALLOC(e->env.ep_len, 2 * E * 4);
  ALLOC(e->env.lives, 2 * E * 4);
  ALLOC(e->env.frame, 2 * E * 4);
  ALLOC(e->env.reward, 2 * E * 4);
  ALLOC(e->env.terminal, 2 * E);
  ALLOC(e->loss, 64);
  ALLOC(e->sumsq, A3C_MAX_TENSORS * 4);
  const int64_t scrB = cfg->net.algo == A3C_ALGO_Q ? nE : E;
  for (int k = 0; k < e->nslot; ++k) {
    Slot& sl = e->slot[k];
    if (e->overlap) {
      ALLOC(sl.P, L.total * 4);
      ALLOC(sl.tau, 64);
    } else {
      sl.P = e->params;
      sl.tau = e->counters;
    }
    ALLOC(sl.actions, nE * 4);
    ALLOC(sl.frames, nE * 4);
    ALLOC(sl.rewards, nE * 4);
    ALLOC(sl.rewards_raw, nE * 4);
    ALLOC(sl.terms, nE);
    ALLOC(sl.z, (nE + E) * zs * 4);
    ALLOC(sl.R_buf, nE * 4);
    if (e->nat) {
      ALLOC(sl.act_l1, nE * NT_A1 * 4);
      ALLOC(sl.act_l2, nE * NT_A2 * 4);
      ALLOC(sl.act_l3, nE * NT_FLAT * 4);
      ALLOC(sl.act_l4, nE * NT_FC * 4);
      ALLOC(sl.nscr, E * nat_act_floats() * 4);
    } else {
      ALLOC(sl.act_l1, nE * C1_P * C1_N * 4);
      ALLOC(sl.act_l2, nE * FLAT * 4);
      ALLOC(sl.act_l3, nE * FC * 4);
    }
    ALLOC(sl.scr_l2, scrB * FLAT * 4);
    ALLOC(sl.scr_l3, scrB * FC * 4);
    ALLOC(sl.prep, PREP_BYTES);
    if (boot_bwd(e)) ALLOC(sl.fcboot, (int64_t)FC_NS * E * FC * 4);   // (only the A/B knob's form reads it)
    if (L.lstm) {
      ALLOC(sl.lh, nE * LSTM_U * 4);
      ALLOC(sl.lc, nE * LSTM_U * 4);
      ALLOC(sl.lhp, nE * LSTM_U * 4);
      ALLOC(sl.lcp, nE * LSTM_U * 4);
      ALLOC(sl.lg, nE * LSTM_G * 4);
      ALLOC(sl.lhb, E * LSTM_U * 4);
      ALLOC(sl.lcb, E * LSTM_U * 4);
      ALLOC(sl.lwt, (int64_t)LSTM_K * LSTM_G * 4);
    }
  }
  if (L.lstm) {
    ALLOC(e->lws, a3c_lstm_ws_floats(e->n, E) * 4);
    ALLOC(e->ldh, nE * LSTM_U * 4);
  }
  ALLOC(e->prep_t, PREP_BYTES);
  ALLOC(e->spans, 2 * (size_t)SPAN_RECS * SPAN_WGS * 2 * sizeof(unsigned long long));
  ALLOC(e->zt, scrB * zs * 4);
  ALLOC(e->ep_end, E * 4);
  if (e->nat) {
    ALLOC(e->ws, a3c_nat_bwd_ws_floats(L, nE) * 4);
    ALLOC(e->nat_fws, (a3c_nat_fwd_ws_floats(E) > 0 ? a3c_nat_fwd_ws_floats(E) : 1) * 4);
  } else {
    BwdPlan bp = a3c_bwd_plan(L, nE);
    ALLOC(e->ws, bp.total * 4);
  }
  ALLOC(e->fcpart, (int64_t)FC_NS * E * FC * 4);
  ALLOC(e->opt_part, (int64_t)SS_MAX_BLOCKS * 8);
  ALLOC(e->sched, 64);
  ALLOC(e->stats, A3C_STATS_N * 8);
  ALLOC(e->ep_acc, E * 8);
  // last: the other buffers keep the placement they had before the ReLU bits existed
  for (int k = 0; k < e->nslot; ++k) ALLOC(e->slot[k].l2m, nE * C2_Q * 4);
  ALLOC(e->fctick, fctick_bytes(E));
  if (hipError_t st = hipMemset(e->fctick, 0, fctick_bytes(E))) {
    a3c_engine_destroy(e);
    return a3c_set_error((int)st, "a3c_engine_create", "hipMemset failed");
  }
#undef ALLOC
  if (a3c_make_tab(L.nt, L.off, L.size, L.total, &e->tt) ||
      (e->nat ? a3c_nat_fused_tab(L, &e->tt_f) : a3c_fused_tab(L, &e->tt_f))) {
    a3c_engine_destroy(e);
    return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_create", "tensor table");
  }
  {
    bool ok = hipStreamCreateWithFlags(&e->gs, hipStreamNonBlocking) == hipSuccess &&
              hipEventCreateWithFlags(&e->ev_gfork, hipEventDisableTiming) == hipSuccess &&
              hipEventCreateWithFlags(&e->ev_gjoin, hipEventDisableTiming) == hipSuccess;
    if (!ok) {
      a3c_engine_destroy(e);
      return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_create", "stream/event creation failed");
    }
  }
  // the split exchange needs eager launches (its event is recorded mid-backward) and a peer
  e->split = cfg->split_exchange && cfg->world_size > 1 && !cfg->use_graph && !e->nat;
  e->l2bits = e->nat ? 0 : l2bits_choice(e);
  if (e->split && hipEventCreateWithFlags(&e->ev_head, hipEventDisableTiming) != hipSuccess) {
    a3c_engine_destroy(e);
    return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_create", "event creation failed");
  }
  if (e->overlap) {
    // the rollout is a serial chain of small kernels: give its stream the higher priority so
    // its workgroups are dispatched first when the concurrent backward frees CU resources
    int lo_prio = 0, hi_prio = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo_prio, &hi_prio);
    int prio = hi_prio;
    if (!A3C_AB_KNOB("A3C_ROLLOUT_PRIO", 1)) prio = lo_prio;
    // the cross-stream events order two streams of this device and the host never inspects
    // them: no system-scope fence (measured: 4.54M vs 4.47M env-steps/s with events, on par with
    // the wait-value hop; A3C_DEVICE_EVENTS=0 restores the default events)
    unsigned evf = hipEventDisableTiming | hipEventDisableSystemFence;
    if (!A3C_AB_KNOB("A3C_DEVICE_EVENTS", 1)) evf = hipEventDisableTiming;
    bool ok = hipStreamCreateWithPriority(&e->rs, hipStreamNonBlocking, prio) == hipSuccess &&
              hipEventCreateWithFlags(&e->ev_start, evf) == hipSuccess;
    for (int k = 0; k < 2 && ok; ++k)
      ok = hipEventCreateWithFlags(&e->ev_roll[k], evf) == hipSuccess;
    // (one GPU: with an exchange the collectives' own stream synchronisation sits between the
    // graphs, a combination the pool has not run on several GPUs -- events there)
    e->wait_value = e->cfg.world_size == 1;
    e->wait_value = A3C_KNOB("A3C_WAIT_VALUE", e->wait_value) != 0;

    if (!ok) {
      a3c_engine_destroy(e);
      return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_create", "stream/event creation failed");
    }
  }
  e->envp.k0 = e->k0; e->envp.k1 = e->k1;
  e->envp.P = e->cfg.num_frames;
  e->envp.A = L.A;
  e->envp.L0 = cfg->start_lives;
  e->envp.random_start = cfg->random_start;
  e->envp.action_repeat = cfg->action_repeat;
  e->envp.env_id_base = cfg->env_id_base;
  // per-env final epsilon (main.py:68 samples ep_end per worker from {0.1, 0.01, 0.5})
  std::vector<int32_t> idx(E);
  for (int64_t i = 0; i < E; ++i) idx[i] = (int32_t)i;
  if (hipMemcpy(e->ext_idx, idx.data(), E * 4, hipMemcpyHostToDevice) != hipSuccess) {
    a3c_engine_destroy(e);
    return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_create", "hipMemcpy");
  }
  std::vector<float> ee(E);
  static const float choices[3] = {0.1f, 0.01f, 0.5f};
  for (int64_t i = 0; i < E; ++i) {
    u32x4 x = philox4x32((uint32_t)(cfg->env_id_base + i), 0u, 0u, 11u, e->k0, e->k1);
    ee[i] = choices[x.x % 3u];
  }
  if (hipMemcpy(e->ep_end, ee.data(), E * 4, hipMemcpyHostToDevice) != hipSuccess) {
    a3c_engine_destroy(e);
    return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_create", "hipMemcpy");
  }
  *out = e;
  return 0;
}

// ---- small device kernels -------------------------------------------------------------------
// ---- train_with_summary aggregates (agent.py:69-139) ----------------------------------------
// stats: [0] sum of act() rewards over env-steps, [1] sum / [2] max / [3] min of finished episodes'
// rewards, [4] games, [5] sum of per-update loss (per sample), [6] sum of per-update mean Q(s) (q:
// over actions; a3c: V(s)), [7] updates, [8] env-steps, [9..11] sums of per-sample policy / value
// loss and entropy (a3c)
__global__ void k_stats_reset(double* st) {
  const int i = threadIdx.x;
  if (i < A3C_STATS_N) st[i] = i == 2 ? -INFINITY : (i == 3 ? INFINITY : 0.0);
}

// one update's rollout (n steps of E envs), in the reference chief's order per env: the episode
// reward excludes the terminal step's reward and restarts after it (agent.py:91-98); total reward
// includes every step (agent.py:101).  One workgroup, fixed-order tree reductions: deterministic.
__global__ void __launch_bounds__(256) k_stats(const float* __restrict__ rraw, const uint8_t* __restrict__ terms,
                                               const float* __restrict__ z, int zs, int A, int q, int n, int E,
                                               const float* __restrict__ loss, double* __restrict__ ep_acc,
                                               double* __restrict__ st) {
  __shared__ double red[6][256];
  double tr = 0.0, es = 0.0, emax = -INFINITY, emin = INFINITY, games = 0.0, qs = 0.0;
  for (int e = threadIdx.x; e < E; e += 256) {
    double acc = ep_acc[e];
    for (int t = 0; t < n; ++t) {
      const int64_t b = (int64_t)t * E + e;
      const double r = rraw[b];
      tr += r;
      if (terms[b]) {
        games += 1.0; es += acc; emax = fmax(emax, acc); emin = fmin(emin, acc);
        acc = 0.0;
      } else {
        acc += r;
      }
      const float* zr = z + b * zs;
      if (q) {
        double m = 0.0;
        for (int a = 0; a < A; ++a) m += zr[a];
        qs += m / A;
      } else {
        qs += zr[A];
      }
    }
    ep_acc[e] = acc;
  }
  const int i = threadIdx.x;
  red[0][i] = tr; red[1][i] = es; red[2][i] = emax; red[3][i] = emin; red[4][i] = games; red[5][i] = qs;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (i < o) {
      red[0][i] += red[0][i + o]; red[1][i] += red[1][i + o];
      red[2][i] = fmax(red[2][i], red[2][i + o]); red[3][i] = fmin(red[3][i], red[3][i + o]);
      red[4][i] += red[4][i + o]; red[5][i] += red[5][i + o];
    }
    __syncthreads();
  }
  if (i == 0) {
    const double B = (double)n * E;
    st[0] += red[0][0]; st[1] += red[1][0];
    st[2] = fmax(st[2], red[2][0]); st[3] = fmin(st[3], red[3][0]);
    st[4] += red[4][0];
    st[5] += q ? (double)loss[0] : (double)loss[3] / B;
    st[6] += red[5][0] / B;
    st[7] += 1.0;
    st[8] += B;
    if (!q) { st[9] += (double)loss[0] / B; st[10] += (double)loss[1] / B; st[11] += (double)loss[2] / B; }
  }
}

// the epsilon schedule of agent.py:142-144 at the worker's own step, evaluated by the head kernel
// (sel_eps in net_fwd.hip): the workers' base step counters[2] plus the env steps taken so far
// (tau - (HIST-1)).  A separate per-step schedule kernel cost Q sync 3% (round-5 bisect).
static void set_eps_schedule(const a3c_engine* e, HeadSelect& sel) {
  sel.ep_end = e->ep_end;
  sel.ep_start = e->cfg.ep_start;
  sel.ep_end_t = e->cfg.ep_end_t;
  sel.learn_start = e->cfg.learn_start;
}

static StateAddr ring_addr(const a3c_engine* e, int tau_offset, const int64_t* tau_ptr) {
  StateAddr sa;
  sa.base = e->ring;
  sa.env_stride = (int64_t)e->R * PLANE;
  sa.plane_bytes = PLANE;
  sa.E = e->E;
  sa.R = e->R;
  sa.L = HIST;
  sa.tau_offset = tau_offset;
  sa.tau_ptr = tau_ptr;
  return sa;
}

// live launch-span stamps in k_conv_bwd / k_head_screen_conv12 (A3C_SPANS=0 turns them off)
static bool spans_on() {
  static const bool on = A3C_KNOB("A3C_SPANS", 1) != 0;
  return on;
}
// the nature trunk's rollout states s_{tau + t}: its per-state conv kernel records its live launch
// span in spans[1] (the nips engine's k_head_screen_conv12 slot, unused on this trunk)
static StateAddr nat_step_addr(const a3c_engine* e, int t) {
  StateAddr sa = ring_addr(e, t, e->counters);
  sa.span = spans_on() ? e->spans + (size_t)SPAN_RECS * SPAN_WGS * 2 : nullptr;
  return sa;
}
// conv fusion (k_head_screen_conv12) runs with the device envs and the fused screen
static bool conv_fused(const a3c_engine* e) { return e->fuse_conv && !e->ext && e->fused_screen; }
// the fused rollout's fc as K-slice partials folded by the head (feed-forward head only)
// (the LSTM head: the cell kernel folds them, k_lstm_fwd)
static bool fc_split(const a3c_engine* e) { return conv_fused(e) && e->fc_split; }
// Overlap, A3C feed-forward head: the bootstrap state's head (the fold of its fc partials, V(s_n))
// runs as the first kernel of the slot's backward on the caller's stream instead of as the
// rollout's last kernel; the rollout ends with the fc of s_n (into the slot's own partial buffer,
// which the next rollout does not touch), which also advances tau.
static bool boot_bwd(const a3c_engine* e) {
  static const int env = (int)A3C_AB_KNOB("A3C_BOOT_BWD", 0);
  return env != 0 && e->overlap && fc_split(e) && !e->L.lstm && e->L.algo == A3C_ALGO_A3C;
}

__global__ void k_advance_tau(int64_t* counters, int n) { counters[0] += n; }

// optimizer parameters of the update of the rollout in slot sl (its tau gives the worker step of
// the lr schedule, OptParams)
static OptParams opt_params(const a3c_engine* e, const Slot& sl) {
  const a3c_engine_config& c = e->cfg;
  OptParams op = {};
  op.clip = c.clip_norm;
  op.sched = e->sched;
  op.step_ptr = e->counters + 1;
  op.step_add = e->nE * c.world_size;
  op.wstep_ptr = e->counters + 2;
  op.tau_ptr = sl.tau;
  op.tau0 = HIST - 1;
  op.n_step = e->n;
  op.lr0 = c.learning_rate;
  op.max_step = c.max_step;
  op.target_period = e->L.algo == A3C_ALGO_Q ? c.target_q_update_step : 0;
  op.target = e->L.algo == A3C_ALGO_Q ? e->tparams : nullptr;
  op.counters = e->counters;
  op.dtau = e->overlap ? 0 : e->n;   // overlap: the rollout advances tau itself
  op.rho = c.decay;
  op.momentum = c.momentum;
  op.eps = c.epsilon;
  return op;
}

// n env steps of every env (forward + action draw + env act fused into the head, then the
// Environment.screen of the new frames into the ring) and the bootstrap forward.
static int enqueue_rollout_impl(a3c_engine* e, const Slot& sl, hipStream_t s);
static int enqueue_rollout(a3c_engine* e, const Slot& sl, hipStream_t s) {
  a3c_set_shared_gpu(e->overlap != 0);
  a3c_set_fcp_split(e->frame84 ? 2 : 4);
  int rc = enqueue_rollout_impl(e, sl, s);
  a3c_set_shared_gpu(false);
  a3c_set_fcp_split(2);
  return rc;
}

// the slot holding the rollout before sl's (its last LSTM state is sl's carry-in)
static const Slot& prev_slot(const a3c_engine* e, const Slot& sl) {
  return e->nslot == 2 ? e->slot[&sl == &e->slot[0] ? 1 : 0] : sl;
}

// "rollout k done", the go of its backward (rollout_grad): on one GPU at the start of rollout
// k+1, behind its wait for the apply it needs -- the backward of k then starts with rollout k+1
// instead of ~10 us ahead of it, where its GEMMs slowed rollout k+1's first steps (DESIGN §6;
// M1 4.42-4.53M -> 4.56-4.57M), and rollout k+1's prep kernel bumps the sequence itself
// (kernel_go: no write-value operation on the rollout stream); with an exchange, right behind
// rollout k on the rollout stream
static bool bwd_bound(const a3c_engine* e);
static bool late_go(const a3c_engine* e) {
  static const int env = (int)A3C_AB_KNOB("A3C_LATE_GO", -1);   // A/B override
  // one GPU: M1 and M2 (M2 5.77M -> 5.83M since the conv backward runs one workgroup per CU);
  // with an exchange the caller stream carries it behind the backward: right behind the rollout
  return env >= 0 ? env != 0 : e->cfg.world_size == 1;
}
static bool kernel_go(const a3c_engine* e) {
  static const int env = (int)A3C_AB_KNOB("A3C_KERNEL_GO", 1);   // A/B override
  return e->overlap && e->wait_value && late_go(e) && env != 0;
}

// rollout start: forward weights of the rollout's parameters (+ q: the epsilon schedule)
static int enqueue_rollout_begin(a3c_engine* e, const Slot& sl, hipStream_t s) {
  const a3c_engine_config& c = e->cfg;
  if (e->nat)   // (prepared: conv1's bf16 weight terms; the other passes read the fp32 parameters)
    return a3c_nat_prep_launch(e->L, sl.P, (uint16_t*)sl.prep, e->overlap ? e->counters : nullptr,
                               e->overlap ? sl.tau : nullptr, kernel_go(e) ? e->xflags + 1 : nullptr, s);
  // params are fixed for the rollout; overlap: the prep kernel also snapshots tau for the slot's
  // backward (sync: the slot's tau is the live counter)
  int rc = a3c_prep_fwd_launch(e->L, sl.P, sl.prep, s, e->overlap ? e->counters : nullptr,
                           e->overlap ? sl.tau : nullptr, kernel_go(e) ? e->xflags + 1 : nullptr);
  if (rc) return rc;
  if (e->L.lstm) {
    rc = a3c_lstm_transpose_launch(sl.P + e->L.off[T_LW], sl.lwt, s);
    if (rc) return rc;
  }
  return 0;
}

// rollout step t: forward of s_{tau+t}, action draw (agent.py:141-151 / network.py:65-72) and,
// with the device env, act + observe clip + Environment.screen of the new frame into the ring
// (external envs: the host steps them between a3c_engine_ext_act and a3c_engine_ext_observe).
static bool l2bits_on(const a3c_engine* e);
static int l2bits_choice(const a3c_engine* e);
static int enqueue_step(a3c_engine* e, const Slot& sl, int t, hipStream_t s) {
  const a3c_engine_config& c = e->cfg;
  const NetLayout& L = e->L;
  const int E = e->E, n = e->n, zs = L.zs;
  const bool q = L.algo == A3C_ALGO_Q;
  const bool dev_env = !e->ext;
  HeadSelect sel = {};
  sel.mode = q ? 1 : 0;
  sel.k0 = e->k0; sel.k1 = e->k1;
  sel.tau_ptr = e->counters; sel.tau_add = t;
  sel.env_ids = nullptr; sel.env_id_base = c.env_id_base; sel.E = E;
  if (q) set_eps_schedule(e, sel);   // epsilon of this step, in the head (q engines are synchronous)
  const int64_t o = (int64_t)t * E;
  sel.actions = sl.actions + o;
  sel.env_on = dev_env ? 1 : 0;
  if (dev_env) {
    sel.par_E = E;
    sel.envp = e->envp;
    sel.envb = e->env;
    sel.rewards = sl.rewards + o;
    sel.rewards_raw = sl.rewards_raw + o;
    sel.terms = sl.terms + o;
    sel.frames_out = sl.frames + o;
    if (e->fused_screen) {      // Environment.screen of the new frame inside the head kernel
      sel.pool = e->pool;
      sel.ring = e->ring;
      sel.R = e->R;
      sel.frame84 = e->frame84;
    }
  }
  LstmStep ls = {};
  if (L.lstm) {   // carry-in: step t-1 of this rollout, or the last step of the previous one
    const Slot& src = t > 0 ? sl : prev_slot(e, sl);
    const int64_t so = t > 0 ? o - E : (int64_t)(n - 1) * E;
    ls.wt = sl.lwt;
    ls.h_src = src.lh + so * LSTM_U; ls.c_src = src.lc + so * LSTM_U; ls.prev_terms = src.terms + so;
    ls.hp = sl.lhp + o * LSTM_U; ls.cp = sl.lcp + o * LSTM_U; ls.gates = sl.lg + o * LSTM_G;
    ls.h = sl.lh + o * LSTM_U; ls.c = sl.lc + o * LSTM_U;
    if (e->lstm_fcfold) ls.fc_tick = e->fctick;
  }
  // conv fusion: step t > 0's conv1 + conv2 ran inside step t-1's head + screen kernel, and this
  // step's head + screen runs step t+1's (the bootstrap state's after the last step, a3c)
  const bool fuse = conv_fused(e);
  Conv12Next nx = {};
  const bool has_next = fuse && (t + 1 < n || !q);
  if (has_next) {
    nx.sa = ring_addr(e, t + 1, e->counters);
    nx.sa.span = spans_on() ? e->spans + (size_t)SPAN_RECS * SPAN_WGS * 2 : nullptr;   // per launch
    nx.w1s = (const uint16_t*)sl.prep;
    nx.b1 = sl.P + L.off[T_L1B];
    nx.W2 = sl.P + L.off[T_L2W];
    nx.b2 = sl.P + L.off[T_L2B];
    nx.act_l1 = t + 1 < n ? sl.act_l1 + (o + E) * C1_P * C1_N : nullptr;
#ifdef A3C_ABL_NOL1
    nx.act_l1 = nullptr;   // measurement only: the fused rollout kernel saves no conv1 output
#endif
    nx.act_l2 = t + 1 < n ? sl.act_l2 + (o + E) * FLAT : sl.scr_l2;
    nx.l2m = t + 1 < n && l2bits_on(e) ? sl.l2m + (o + E) * C2_Q : nullptr;
  }
  int rc;
  if (e->nat)
    rc = a3c_nat_forward_launch(L, sl.P, nat_step_addr(e, t), E, sl.act_l1 + o * NT_A1,
                                sl.act_l2 + o * NT_A2, sl.act_l3 + o * NT_FLAT, sl.act_l4 + o * NT_FC, sl.z + o * zs, sel,
                                (const uint16_t*)sl.prep, e->nat_fws, s);
  else
    rc = a3c_forward_launch(L, sl.P, sl.prep, ring_addr(e, t, e->counters), E, sl.act_l1 + o * C1_P * C1_N,
                              sl.act_l2 + o * FLAT, sl.act_l3 + o * FC, sl.z + o * zs, sel, s,
                              L.lstm ? &ls : nullptr, fuse && t > 0, has_next ? &nx : nullptr,
                              fc_split(e) ? e->fcpart : nullptr, l2bits_on(e) ? sl.l2m + o * C2_Q : nullptr);
  if (rc) return rc;
  if (dev_env && !e->fused_screen) {
    rc = a3c_env_screen_launch(E, sl.frames + o, e->pool, e->ring, e->R, e->counters, t, s);
    if (rc) return rc;
  }
  return 0;
}

// rollout end: bootstrap V(s_{t+n}) with the same parameters (assets/a3c.png)
static int enqueue_rollout_end(a3c_engine* e, const Slot& sl, hipStream_t s) {
  const NetLayout& L = e->L;
  const int E = e->E, n = e->n;
  if (boot_bwd(e))      // the fc of s_n (conv ran in the last step's kernel) + the tau advance
    return a3c_fc_part_launch(sl.scr_l2, (const float*)(sl.prep + PREP_W1S_BYTES), sl.fcboot, E, s, e->counters, n);
  if (L.algo != A3C_ALGO_Q) {
    const int64_t lastE = (int64_t)(n - 1) * E;
    HeadSelect none = {};
    none.mode = -1;
    none.E = E;
    if (e->overlap) {          // the rollout advances tau: in its last kernel, the bootstrap head
      none.adv_ptr = e->counters;
      none.adv_n = n;
    }
    LstmStep ls = {};
    if (L.lstm) {
      ls.wt = sl.lwt;
      ls.h_src = sl.lh + lastE * LSTM_U; ls.c_src = sl.lc + lastE * LSTM_U; ls.prev_terms = sl.terms + lastE;
      ls.h = sl.lhb; ls.c = sl.lcb;
      if (e->lstm_fcfold) ls.fc_tick = e->fctick;
    }
    if (e->nat) {
      float* x = sl.nscr;
      // (no span record: s_n is the next rollout's s_0, whose step-0 launch keys the same record)
      return a3c_nat_forward_launch(L, sl.P, ring_addr(e, n, e->counters), E, x, x + E * NT_A1,
                                    x + E * (NT_A1 + NT_A2), x + E * (NT_A1 + NT_A2 + NT_FLAT), sl.z + e->nE * L.zs,
                                    none, (const uint16_t*)sl.prep, e->nat_fws, s);
    }
    int rc = a3c_forward_launch(L, sl.P, sl.prep, ring_addr(e, n, e->counters), E, nullptr, sl.scr_l2,
                                sl.scr_l3, sl.z + e->nE * L.zs, none, s, L.lstm ? &ls : nullptr,
                                conv_fused(e),   // s_n's convs ran in the last step's kernel
                                nullptr, fc_split(e) ? e->fcpart : nullptr);
    return rc;
  }
  if (e->overlap) {
    hipLaunchKernelGGL(k_advance_tau, dim3(1), dim3(1), 0, s, e->counters, n);
    A3C_CHECK(hipGetLastError());
  }
  return 0;
}

// Debug builds only (-DA3C_MARKERS, tools/markers.py): one-lane marker kernels captured at the
// edges of the rollout and backward graphs record (id, s_memrealtime) in a device log, so the
// unprofiled timeline of the two streams (and the cross-stream hops between them) can be read.
#ifdef A3C_MARKERS
#define MARK_CAP 8192
__device__ unsigned long long g_marks[2 + 2 * MARK_CAP];
__global__ void k_mark(int id) {
  const unsigned long long i = atomicAdd(&g_marks[0], 1ull);
  if (i < MARK_CAP) {
    g_marks[2 + 2 * i] = (unsigned long long)id;
    g_marks[3 + 2 * i] = __builtin_amdgcn_s_memrealtime();
  }
}
static void mark(int id, hipStream_t s) { hipLaunchKernelGGL(k_mark, dim3(1), dim3(1), 0, s, id); }
void a3c_mark(int id, hipStream_t s) { mark(id, s); }   // (net_bwd.hip: 4 = conv backward start, 5 = its end)
extern "C" int a3c_debug_marks(unsigned long long* host, int reset) {
  A3C_CHECK(hipDeviceSynchronize());
  A3C_CHECK(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_marks), sizeof(g_marks)));
  if (reset) {
    unsigned long long z = 0;
    A3C_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_marks), &z, sizeof(z)));
  }
  return MARK_CAP;
}
#else
static void mark(int, hipStream_t) {}
#endif

#ifdef A3C_WGLOG
void a3c_wglog_bind_fwd(WglBuf*);
void a3c_wglog_bind_bwd(WglBuf*);
void a3c_wglog_bind_gemm(WglBuf*);
void a3c_wglog_bind_optim(WglBuf*);
// Debug builds only (tools/wglog.py): on >= 0 switches logging, reset clears the log; the whole
// WglBuf is copied to host when host != nullptr (after a device sync); returns its size in bytes
extern "C" int64_t a3c_debug_wglog(void* host, int on, int reset) {
  static WglBuf* buf = nullptr;
  if (!buf) {
    A3C_CHECK(hipMalloc(&buf, sizeof(WglBuf)));
    A3C_CHECK(hipMemset(buf, 0, sizeof(WglBuf)));
    a3c_wglog_bind_fwd(buf); a3c_wglog_bind_bwd(buf); a3c_wglog_bind_gemm(buf); a3c_wglog_bind_optim(buf);
  }
  A3C_CHECK(hipDeviceSynchronize());
  if (host) A3C_CHECK(hipMemcpy(host, buf, sizeof(WglBuf), hipMemcpyDeviceToHost));
  if (reset) A3C_CHECK(hipMemset(buf, 0, sizeof(WglBuf)));
  if (on >= 0) {
    const unsigned v = (unsigned)on;
    A3C_CHECK(hipMemcpy(buf, &v, 4, hipMemcpyHostToDevice));
  }
  A3C_CHECK(hipDeviceSynchronize());
  return (int64_t)sizeof(WglBuf);
}
#endif

static int enqueue_rollout_impl(a3c_engine* e, const Slot& sl, hipStream_t s) {
  mark(0, s);
  int rc = enqueue_rollout_begin(e, sl, s);
  for (int t = 0; t < e->n && !rc; ++t) rc = enqueue_step(e, sl, t, s);
  rc = rc ? rc : enqueue_rollout_end(e, sl, s);
  mark(1, s);
  return rc;
}

// returns / TD target, loss + backward over the slot's n*E samples, per-tensor norms (+ the
// per-worker clip when gradients are exchanged across GPUs).
static int enqueue_grad_impl(a3c_engine* e, const Slot& sl, hipStream_t s);
// Overlapped runs where the backward stream, not the rollout, bounds the iteration: mode M2 (a
// shorter rollout) and several GPUs (the exchange -- all-to-all, sharded apply, all-gather -- runs on
// the backward's stream).  There the three backward GEMMs run as one launch with their folds
// behind the conv backward (M2 5.17-5.22M -> 5.36-5.40M env-steps/s); in mode M1 the rollout
// co-bounds it and the single 1,420-workgroup launch costs the rollout more than it saves
// (net_bwd.hip's knobs).
static bool bwd_bound(const a3c_engine* e) {
  static const int env = (int)A3C_AB_KNOB("A3C_BWD_BOUND", -1);   // A/B override
  if (env >= 0) return e->overlap && env != 0;
  return e->overlap && (e->frame84 || e->cfg.world_size > 1);
}
static int enqueue_grad(a3c_engine* e, const Slot& sl, hipStream_t s) {
  // overlap: the backward shares CUs with the next rollout -> small-footprint kernel variants
  a3c_set_shared_gpu(e->overlap != 0);
  a3c_set_bwd_bound(bwd_bound(e));
  mark(2, s);
  int rc = enqueue_grad_impl(e, sl, s);
  a3c_set_shared_gpu(false);
  a3c_set_bwd_bound(false);
  return rc;
}

#ifdef A3C_HOG
// Measurement only (-DA3C_HOG): in place of the backward, a synthetic kernel with the conv
// backward's footprint (183 workgroups x 4 waves, 74 KB LDS, one wave per SIMD) that keeps one
// resource busy for A3C_HOG_ITERS loop trips, so the rollout's sensitivity to each kind of
// co-resident work can be read from its launch spans (tools/span_timeline.py).
// type: 0 fp32 16x16x4 MFMA, 1 fp32 32x32x2 MFMA, 2 bf16 16x16x32 MFMA, 3 VALU fma, 4 LDS b128
// reads, 5 s_sleep (occupancy only), 6 HBM stream reads
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) k_hog(int type, int iters,
                                                                                    const float* src, float* out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int lane = threadIdx.x & 63;
  f32x4 a4 = {0.f, 0.f, 0.f, 0.f}, b4 = a4;
  f32x16 a16 = {}, b16 = {};
  float x = (float)lane * 1e-3f, y = x + 1.f, z = 0.f;
  if (type == 0) {
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        a4 = __builtin_amdgcn_mfma_f32_16x16x4f32(x, y, a4, 0, 0, 0);
        b4 = __builtin_amdgcn_mfma_f32_16x16x4f32(y, x, b4, 0, 0, 0);
      }
    }
  } else if (type == 1) {
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        a16 = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, a16, 0, 0, 0);
        b16 = __builtin_amdgcn_mfma_f32_32x32x2f32(y, x, b16, 0, 0, 0);
      }
    }
  } else if (type == 2) {
    bf16x8 av = __builtin_bit_cast(bf16x8, make_uint4(lane, lane + 1, lane + 2, lane + 3));
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        a4 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, av, a4, 0, 0, 0);
        b4 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, av, b4, 0, 0, 0);
      }
    }
  } else if (type == 3) {
    float p = x, q = y, r = x + y, t = x - y;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        p = fmaf(p, 0.999f, 1e-3f); q = fmaf(q, 0.999f, 1e-3f);
        r = fmaf(r, 0.999f, 1e-3f); t = fmaf(t, 0.999f, 1e-3f);
      }
    }
    z = p + q + r + t;
  } else if (type == 4) {
    const uint4* l = (const uint4*)smem;
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint4 v = l[(lane + 64 * k + 7 * i) & 1023];
        acc.x ^= v.x; acc.y += v.y; acc.z ^= v.z; acc.w += v.w;
      }
    }
    z = (float)(acc.x + acc.y + acc.z + acc.w);
  } else if (type == 5) {
    for (int i = 0; i < iters; ++i) __builtin_amdgcn_s_sleep(10);
  } else {
    const f32x4* g = (const f32x4*)src + (size_t)blockIdx.x * 8192;
    for (int i = 0; i < iters; ++i) {
      const f32x4 v = g[(threadIdx.x + 256 * (i & 31)) & 8191];
      z += v[0] + v[1] + v[2] + v[3];
    }
  }
  float sum = z + a4[0] + b4[1] + a16[0] + b16[3];
  if (sum == 1234.5f) out[blockIdx.x * 256 + threadIdx.x] = sum;   // (keeps the work alive)
}
#endif

// The ReLU bits of act_l2 (the forward's conv2 epilogue ballots them, the backward's dl2 GEMM
// epilogue reads 1/32 of the bytes of re-reading l2) where the backward bounds the overlapped
// iteration (bwd_bound: M2, several GPUs): M2 6.03M vs 6.00M env-steps/s.  Where the rollout bounds
// it (M1, C5 LSTM, 1024 envs) the ballot costs the rollout more than the bytes save the backward
// (M1 4.85M vs 4.86M, and the rollout kernel without the ballot compiled in: C5 +0.9 %).
// A3C_L2BITS=0/1 overrides.
static bool l2bits_on(const a3c_engine* e) { return e->l2bits != 0; }
static int l2bits_choice(const a3c_engine* e) {   // at create (a test compares the two forms)
  return A3C_KNOB("A3C_L2BITS", bwd_bound(e) ? 1 : 0) != 0;
}

static int enqueue_grad_impl(a3c_engine* e, const Slot& sl, hipStream_t s) {
  const a3c_engine_config& c = e->cfg;
#ifdef A3C_HOG
  {
    static const int hog_type = getenv("A3C_HOG_TYPE") ? atoi(getenv("A3C_HOG_TYPE")) : -1;
    static const int hog_iters = getenv("A3C_HOG_ITERS") ? atoi(getenv("A3C_HOG_ITERS")) : 1000;
    if (hog_type >= 0) {
      static bool attr = false;
      if (!attr) {
        (void)hipFuncSetAttribute((const void*)k_hog, hipFuncAttributeMaxDynamicSharedMemorySize, 74304);
        attr = true;
      }
      hipLaunchKernelGGL(k_hog, dim3(183), dim3(256), 74304, s, hog_type, hog_iters, (const float*)e->pool,
                         e->ws);
      A3C_CHECK(hipGetLastError());
      OptParams op = opt_params(e, sl);
      return a3c_sumsq_launch(e->grads, e->tt_f, op, e->opt_part, s);   // (F tensors read as 0: measurement only)
    }
  }
#endif
  const NetLayout& L = e->L;
  const int E = e->E, n = e->n, zs = L.zs;
  const bool q = L.algo == A3C_ALGO_Q;
  int rc;
  if (q) {
    // target network on s_{t+1} for every transition (agent.py:186)
    HeadSelect none = {};
    none.mode = -1;
    none.E = E;
    const float* qsel = nullptr;
    if (c.double_q) {
      // double Q (agent.py:176-184): the online net's q of s_{t+1} -- rows t+1 of the rollout's own
      // q (the slot's parameters, those the loss is taken at), and for t = n-1 one forward of s_n
      // with them into the slot's bootstrap row block
      rc = a3c_forward_launch(L, sl.P, sl.prep, ring_addr(e, n, sl.tau), E, nullptr, sl.scr_l2, sl.scr_l3,
                              sl.z + e->nE * zs, none, s);
      if (rc) return rc;
      qsel = sl.z + (int64_t)E * zs;
    }
    rc = a3c_prep_fwd_launch(L, e->tparams, e->prep_t, s);
    if (rc) return rc;
    rc = a3c_forward_launch(L, e->tparams, e->prep_t, ring_addr(e, 1, sl.tau), e->nE, nullptr, sl.scr_l2,
                            sl.scr_l3, e->zt, none, s);
    if (rc) return rc;
    rc = a3c_td_target_launch(sl.rewards, sl.terms, e->zt, e->nE, L.A, zs, c.discount, sl.R_buf, s, qsel);
    if (rc) return rc;
  }
  if (boot_bwd(e)) {   // V(s_n) of the slot (its fc partials: the rollout's last kernel)
    rc = a3c_head_fold_launch(L, sl.P, sl.fcboot, E, sl.z + e->nE * zs, s);
    if (rc) return rc;
  }
  ReturnsArgs ra = {};
  if (!q) {   // n-step returns computed inside the head backward (assets/a3c.png)
    ra.rewards = sl.rewards; ra.terms = sl.terms; ra.boot = sl.z + e->nE * zs + L.A; ra.boot_stride = zs;
    ra.n = n; ra.E = E; ra.gamma = c.gamma; ra.R_out = sl.R_buf;
  }
  static const bool fork_env = A3C_AB_KNOB("A3C_BWD_FORK", 0) != 0;  // measured slower
  const bool fork = fork_env && !L.lstm;
  LstmBwd lb = {};
  if (L.lstm) {
    lb.n = n; lb.E = E;
    lb.h = sl.lh; lb.c = sl.lc; lb.hp = sl.lhp; lb.cp = sl.lcp; lb.gates = sl.lg;
    lb.dh = e->ldh; lb.ws = e->lws;
  }
  StateAddr bsa = ring_addr(e, 0, sl.tau);
  bsa.span = spans_on() ? e->spans : nullptr;   // one record per backward (tau advances by n)
  bsa.span_div = n;
  // the per-tensor squared norms (+ lr / target-sync schedule from the device step counter) come
  // out of the backward's last kernel (k_finalize): no separate k_sumsq launch (round 3)
  OptParams op = opt_params(e, sl);
  const SumsqFused sf = {e->opt_part, &e->tt_f, &op};
  // split exchange: the backward clips the fc / head range first and records ev_head (SplitBwd)
  SplitBwd sp = {};
  if (e->split) {
    sp.ev_head = e->ev_head;
    sp.clip = op;
    sp.clip.mode = OPT_CLIP;
    sp.sumsq_out = e->sumsq;
    sp.cut = L.off[T_FCW];
  }
  if (e->nat)
    rc = a3c_nat_backward_launch(L, sl.P, bsa, e->nE, sl.act_l1, sl.act_l2, sl.act_l3, sl.act_l4, sl.z, sl.actions,
                                 sl.R_buf, c.beta, c.literal_adv, e->grads, e->loss, e->ws, s, &ra, &sf,
                                 (const uint16_t*)sl.prep);
  else
  rc = a3c_backward_launch(L, sl.P, bsa, e->nE, sl.act_l1, sl.act_l2, sl.act_l3, sl.z,
                           sl.actions, sl.R_buf, c.beta, c.literal_adv, e->grads, e->loss, e->ws, s, &ra,
                           fork && !e->split ? e->gs : nullptr, fork && !e->split ? e->ev_gfork : nullptr,
                           fork && !e->split ? e->ev_gjoin : nullptr, L.lstm ? &lb : nullptr, &sf,
                           e->split ? &sp : nullptr, l2bits_on(e) ? sl.l2m : nullptr);
  if (rc) return rc;
  if (c.world_size > 1 && !e->split) {
    // multi-GPU: clip this worker's gradient (agent.py:319) before the cross-GPU exchange
    op.mode = OPT_CLIP;
    return a3c_apply_launch(nullptr, nullptr, nullptr, e->grads, e->tt_f, op, e->opt_part, e->sumsq, s);
  }
  return 0;
}

static int enqueue_rollout_grad(a3c_engine* e, hipStream_t s) {
  int rc = enqueue_rollout(e, e->slot[0], s);
  return rc ? rc : enqueue_grad(e, e->slot[0], s);
}

// RMSProp apply (lr from the schedule computed on device), target sync (q) and the counter
// advance in one launch; world_size == 1: the per-tensor clip as well.  Overlap: then the
// parameter snapshot of the rollout that will use slot `snap` (the slot just back-propagated).
static int enqueue_apply(a3c_engine* e, int snap, hipStream_t s) {
  OptParams op = opt_params(e, e->slot[snap]);    // (the schedule was evaluated by the backward)
  op.mode = e->cfg.world_size > 1 ? OPT_APPLY : (OPT_CLIP | OPT_APPLY);
  // overlap: the same pass writes the parameter snapshot of the rollout that will use slot `snap`
  if (e->overlap) op.snap = e->slot[snap].P;
  int rc = a3c_apply_launch(e->params, e->ms, e->mom, e->grads, e->tt_f, op, e->opt_part,
                            e->cfg.world_size > 1 ? nullptr : e->sumsq, s);
  mark(3, s);
  return rc;
}

// Graph gi (see NGRAPH) is captured on first use (what: 0 rollout+grad, 1 rollout, 2 grad,
// 3 grad+apply, 4 rollout+grad+apply) and launched on s.
static int run_graph(a3c_engine* e, int gi, int what, int slot, hipStream_t s) {
  if (gi < 0 || gi >= NGRAPH) return a3c_set_error(A3C_ERR_INVALID, "run_graph", "graph index");
  auto enqueue = [&](hipStream_t cs) -> int {
    int rc;
    switch (what) {
      case 0: return enqueue_rollout_grad(e, cs);
      case 1: return enqueue_rollout(e, e->slot[slot], cs);
      case 2: return enqueue_grad(e, e->slot[slot], cs);
      case 3:
        rc = enqueue_grad(e, e->slot[slot], cs);
        return rc ? rc : enqueue_apply(e, slot, cs);
      default:
        rc = enqueue_rollout_grad(e, cs);
        return rc ? rc : enqueue_apply(e, 0, cs);
    }
  };
  if (!e->cfg.use_graph) return enqueue(s);
  if (!e->captured[gi]) {
    hipStream_t cs;
    A3C_CHECK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    A3C_CHECK(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
    int rc = enqueue(cs);
    hipGraph_t g;
    hipError_t st = hipStreamEndCapture(cs, &g);
    (void)hipStreamDestroy(cs);
    if (rc) return rc;
    if (st != hipSuccess) return a3c_set_error((int)st, "a3c_engine_rollout_grad", "capture failed");
    st = hipGraphInstantiate(&e->gexec[gi], g, nullptr, nullptr, 0);
    if (st != hipSuccess) {
      (void)hipGraphDestroy(g);
      return a3c_set_error((int)st, "a3c_engine_rollout_grad", "instantiate failed");
    }
    e->graph[gi] = g;
    e->captured[gi] = true;
  }
  A3C_CHECK(hipGraphLaunch(e->gexec[gi], s));
  return 0;
}

extern "C" int a3c_engine_reset(a3c_engine* e, const float* host_params, void* stream) {
  if (!e) return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_reset", "null");
  hipStream_t s = (hipStream_t)stream;
  const NetLayout& L = e->L;
  if (host_params) {
    A3C_CHECK(hipMemcpyAsync(e->params, host_params, L.total * 4, hipMemcpyHostToDevice, s));
    A3C_CHECK(hipStreamSynchronize(s));
  }
  A3C_CHECK(hipMemcpyAsync(e->tparams, e->params, L.total * 4, hipMemcpyDeviceToDevice, s));
  int rc = a3c_fill_launch(e->ms, L.total, 1.0f, s);   // TF1 RMSProp rms slot init = 1
  if (rc) return rc;
  A3C_CHECK(hipMemsetAsync(e->mom, 0, L.total * 4, s));
  A3C_CHECK(hipMemsetAsync(e->grads, 0, L.total * 4, s));
  A3C_CHECK(hipMemsetAsync(e->loss, 0, 64, s));
  A3C_CHECK(hipMemsetAsync(e->ring, 0, (size_t)e->E * e->R * PLANE, s));
  if (!e->ext) {
    rc = a3c_pool_fill_launch(e->pool, e->cfg.num_frames, e->k0, e->k1, s, frame_bytes(e));
    if (rc) return rc;
    rc = a3c_env_init_launch(e->envp, e->env, e->E, e->pool, e->ring, e->R, e->counters, s, e->frame84);
    if (rc) return rc;
  }
  if (e->overlap)
    for (int k = 0; k < 2; ++k)
      A3C_CHECK(hipMemcpyAsync(e->slot[k].P, e->params, L.total * 4, hipMemcpyDeviceToDevice, s));
  if (L.lstm)   // zero LSTM state (the first rollout's carry-in) and terminals
    for (int k = 0; k < e->nslot; ++k) {
      A3C_CHECK(hipMemsetAsync(e->slot[k].lh, 0, (size_t)e->nE * LSTM_U * 4, s));
      A3C_CHECK(hipMemsetAsync(e->slot[k].lc, 0, (size_t)e->nE * LSTM_U * 4, s));
      A3C_CHECK(hipMemsetAsync(e->slot[k].terms, 0, (size_t)e->nE, s));
    }
  A3C_CHECK(hipMemsetAsync(e->xflags, 0, 64, s));
  if (e->ext) A3C_CHECK(hipMemsetAsync(e->counters, 0, 64, s));   // ext_begin sets them
  A3C_CHECK(hipMemsetAsync(e->ep_acc, 0, (size_t)e->E * 8, s));
  hipLaunchKernelGGL(k_stats_reset, dim3(1), dim3(A3C_STATS_N), 0, s, e->stats);
  A3C_CHECK(hipGetLastError());
  A3C_CHECK(hipStreamSynchronize(s));
  e->step0_g = e->step0_w = 0;
  e->s_seq = e->r_seq = 0;
  e->roll_seq[0] = e->roll_seq[1] = 0;
  e->iter = 0;
  e->grad_ready = false;
  e->grad_applied = false;
  e->reset_done = true;
  e->ext_t = 0;
  e->ext_begun = false;
  e->ext_acted = false;
  return 0;
}

// rollout + gradient (fused = 0), or rollout + gradient + apply (fused = 1: world_size 1, the
// apply captured in the same graphs -- a3c_engine_iterate)
static int rollout_grad(a3c_engine* e, hipStream_t s, bool fused) {
  if (e->ext) {
    // external envs: the n steps were driven by ext_act / ext_observe; bootstrap + grad here
    if (e->ext_t != e->n)
      return a3c_set_error(A3C_ERR_STATE, "a3c_engine_rollout_grad", "external envs: n ext_act/ext_observe first");
    int rc = enqueue_rollout_end(e, e->slot[0], s);
    if (!rc) rc = run_graph(e, 3, 2, 0, s);
    e->grad_ready = rc == 0;
    e->grad_applied = false;
    e->ext_t = 0;
    return rc;
  }
  if (!e->overlap) {
    int rc = fused ? run_graph(e, 5, 4, 0, s) : run_graph(e, 0, 0, 0, s);
    e->grad_ready = rc == 0;
    e->grad_applied = fused;
    return rc;
  }
  // overlap: rollout k (slot p) on the engine's rollout stream, after everything the caller
  // enqueued so far -- in steady state the apply of rollout k-2, which also left the parameter
  // snapshot of rollout k in slot p (enqueue_apply); the backward of rollout k-1 (slot p^1) on
  // the caller's stream once that rollout is complete.
  const int p = (int)(e->iter & 1);
  const Slot& sl = e->slot[p];
  if (e->wait_value) {
    A3C_CHECK(hipStreamWriteValue32(s, e->xflags, ++e->s_seq, 0));
    A3C_CHECK(hipStreamWaitValue32(e->rs, e->xflags, e->s_seq, hipStreamWaitValueGte, 0xffffffffu));
  } else {
    A3C_CHECK(hipEventRecord(e->ev_start, s));
    A3C_CHECK(hipStreamWaitEvent(e->rs, e->ev_start, 0));
  }
  // the go of the backward of rollout k-1 (late_go); in rs order rollout k-1 is complete
  const bool late = late_go(e);
  auto signal_rollout = [&](int q) -> int {
    if (e->wait_value) {
      A3C_CHECK(hipStreamWriteValue32(e->rs, e->xflags + 1, ++e->r_seq, 0));
      e->roll_seq[q] = e->r_seq;
    } else {
      A3C_CHECK(hipEventRecord(e->ev_roll[q], e->rs));
    }
    return 0;
  };
  int rc = 0;
  if (kernel_go(e)) {            // the rollout's prep kernel bumps xflags[1] (every rollout)
    e->roll_seq[p ^ 1] = ++e->r_seq;
  } else if (late && e->iter >= 1) {
    rc = signal_rollout(p ^ 1);
  }
  if (rc) return rc;
  rc = run_graph(e, 1 + p, 1, p, e->rs);   // (its prep kernel snapshots tau into sl.tau)
  if (rc) return rc;
  rc = late ? 0 : signal_rollout(p);
  if (rc) return rc;
  e->grad_ready = false;
#ifdef A3C_MARKERS
  static const bool abl_bwd = getenv("A3C_ABL_BWD") != nullptr;   // measurement only: rollouts alone
  if (abl_bwd && e->iter >= 4) {
    e->iter += 1;
    return 0;
  }
#endif
  if (e->iter >= 1) {
    if (e->wait_value)
      A3C_CHECK(hipStreamWaitValue32(s, e->xflags + 1, e->roll_seq[p ^ 1], hipStreamWaitValueGte, 0xffffffffu));
    else
      A3C_CHECK(hipStreamWaitEvent(s, e->ev_roll[p ^ 1], 0));
    rc = fused ? run_graph(e, 6 + (p ^ 1), 3, p ^ 1, s) : run_graph(e, 3 + (p ^ 1), 2, p ^ 1, s);
    if (rc) return rc;
    e->grad_ready = true;
    e->grad_applied = fused;
  }
  e->iter += 1;
  return 0;
}

extern "C" int a3c_engine_rollout_grad(a3c_engine* e, void* stream) {
  if (!e) return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_rollout_grad", "null");
  if (!e->reset_done) return a3c_set_error(A3C_ERR_STATE, "a3c_engine_rollout_grad", "call a3c_engine_reset first");
  return rollout_grad(e, (hipStream_t)stream, false);
}

// One whole iteration (rollout_grad + apply) for a single-GPU engine, the apply captured into the
// same hipGraphs (no host-launched kernel between the graph and the apply).  Bit-identical to
// a3c_engine_rollout_grad followed by a3c_engine_apply.
extern "C" int a3c_engine_iterate(a3c_engine* e, void* stream) {
  if (!e) return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_iterate", "null");
  if (!e->reset_done) return a3c_set_error(A3C_ERR_STATE, "a3c_engine_iterate", "call a3c_engine_reset first");
  if (e->ext || e->cfg.world_size != 1)
    return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_iterate",
                         "single-GPU device-env engines only (else rollout_grad, exchange, apply)");
  return rollout_grad(e, (hipStream_t)stream, true);
}

extern "C" int a3c_engine_grad_ready(a3c_engine* e) { return e && e->grad_ready ? 1 : 0; }

// Split exchange: *cut = the float offset where the fc / head range starts (its gradients are
// clipped before the conv backward runs), 0 when the engine does not split.
extern "C" int a3c_engine_exchange_split(a3c_engine* e, int64_t* cut) {
  if (!e || !cut) return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_exchange_split", "null");
  *cut = e->split ? e->L.off[T_FCW] : 0;
  return 0;
}

// `stream` waits until the last rollout_grad's backward has clipped grads[cut:] (ev_head): the
// exchange of that range can start there, under the conv backward.
extern "C" int a3c_engine_wait_grad_head(a3c_engine* e, void* stream) {
  if (!e) return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_wait_grad_head", "null");
  if (!e->split) return a3c_set_error(A3C_ERR_STATE, "a3c_engine_wait_grad_head", "the engine does not split its exchange");
  if (!e->grad_ready) return a3c_set_error(A3C_ERR_STATE, "a3c_engine_wait_grad_head", "no gradient computed yet");
  A3C_CHECK(hipStreamWaitEvent((hipStream_t)stream, e->ev_head, 0));
  return 0;
}

// RMSProp apply (lr from the schedule computed on device), target sync (q) and the counter
// advance, all in one launch.  world_size == 1: the per-tensor clip is applied here as well.
extern "C" int a3c_engine_apply(a3c_engine* e, void* stream) {
  if (!e) return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_apply", "null");
  // overlap pipeline still filling (no gradient yet), or a3c_engine_iterate applied it already
  if (!e->grad_ready || e->grad_applied) return 0;
  // overlap: the snapshot is for the next rollout (iter), whose slot's previous rollout (iter - 2)
  // has just been back-propagated on this stream
  int rc = enqueue_apply(e, (int)(e->iter & 1), (hipStream_t)stream);
  e->grad_applied = rc == 0;
  return rc;
}

// Partitioned parameter server, step 1 (after the all-to-all of the clipped gradients): the
// nranks sequential RMSProp steps of this rank's range [lo, lo + n); new weights -> w_out.
extern "C" int a3c_engine_apply_shard(a3c_engine* e, const float* grads_by_rank, int nranks, int64_t lo, int64_t n,
                                      float* w_out, void* stream) {
  if (!e) return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_apply_shard", "null");
  if (nranks < 1 || lo < 0 || n < 0 || lo + n > e->L.total || (n > 0 && (!grads_by_rank || !w_out)))
    return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_apply_shard", "bad shard");
  if (!e->grad_ready || e->grad_applied) return 0;
  if (e->cfg.world_size == 1)   // one rank: the per-worker clip has not run (a3c_engine_apply fuses it)
    return a3c_set_error(A3C_ERR_STATE, "a3c_engine_apply_shard", "world_size 1 engines use a3c_engine_apply");
  const a3c_engine_config& c = e->cfg;
  return a3c_apply_seq_launch(e->params + lo, e->ms + lo, e->mom + lo, grads_by_rank, nranks, n, e->sched, c.decay,
                              c.momentum, c.epsilon, w_out, (hipStream_t)stream);
}

// Partitioned parameter server, step 2 (after the all-gather assembled every rank's range in
// params_src, nullable = already in params): params / overlap snapshot / target sync, counters.
extern "C" int a3c_engine_apply_commit(a3c_engine* e, const float* params_src, void* stream) {
  if (!e) return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_apply_commit", "null");
  if (!e->grad_ready || e->grad_applied) return 0;
  const OptParams op = opt_params(e, e->slot[0]);
  float* snap = e->overlap ? e->slot[(int)(e->iter & 1)].P : nullptr;
  int rc = a3c_commit_launch(params_src ? params_src : e->params, e->L.total, e->params, snap, op.target, e->sched,
                             e->counters, op.dtau, op.step_add, (hipStream_t)stream);
  e->grad_applied = rc == 0;
  return rc;
}

// ---- external (host) environments (env workers feeding host RGB buffers) ----
__global__ void k_ext_init(int64_t* counters, int32_t* frame1, int E, int64_t step0_g, int64_t step0_w) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e == 0) { counters[0] = HIST - 1; counters[1] = step0_g; counters[2] = step0_w; }
  if (e < E) frame1[e] = e;      // env state parity (HIST-1)&1 = 1: frame e of the staging buffer
}

__global__ void k_ext_clip(const float* raw, float* r, int E) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < E) r[e] = fmaxf(-1.0f, fminf(1.0f, raw[e]));   // observe clip, agent.py:154
}

static int ext_check(a3c_engine* e, const char* what) {
  if (!e) return a3c_set_error(A3C_ERR_INVALID, what, "null");
  if (!e->ext) return a3c_set_error(A3C_ERR_INVALID, what, "engine was not created with external_env = 1");
  if (!e->reset_done) return a3c_set_error(A3C_ERR_STATE, what, "call a3c_engine_reset first");
  return 0;
}

// first screens of the new (random) games -> every history slot (agent.py:33-38 before_train)
extern "C" int a3c_engine_ext_begin(a3c_engine* e, const uint8_t* rgb, void* stream) {
  if (int rc = ext_check(e, "a3c_engine_ext_begin")) return rc;
  if (!rgb) return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_ext_begin", "null frames");
  hipStream_t s = (hipStream_t)stream;
  const int E = e->E;
  A3C_CHECK(hipMemcpyAsync(e->pool, rgb, (size_t)E * SCREEN_H * SCREEN_W * 3, hipMemcpyDefault, s));
  hipLaunchKernelGGL(k_ext_init, dim3((E + 255) / 256), dim3(256), 0, s, e->counters, e->env.frame + E, E,
                     e->step0_g, e->step0_w);
  A3C_CHECK(hipGetLastError());
  int rc = a3c_env_init_screens_launch(e->env, E, e->pool, e->ring, e->R, s);
  if (rc) return rc;
  e->ext_begun = true;
  e->ext_t = 0;
  e->ext_acted = false;
  return 0;
}

// predict of rollout step t for every env (forward + action draw); actions -> `actions`
// (host, pinned for a true async copy, or device), valid once the stream reaches this point
extern "C" int a3c_engine_ext_act(a3c_engine* e, int32_t* actions, void* stream) {
  if (int rc = ext_check(e, "a3c_engine_ext_act")) return rc;
  if (!e->ext_begun || e->ext_t >= e->n || e->ext_acted || !actions)
    return a3c_set_error(A3C_ERR_STATE, "a3c_engine_ext_act",
                         "ext_begin first; one ext_observe per ext_act; at most n steps per rollout");
  hipStream_t s = (hipStream_t)stream;
  const Slot& sl = e->slot[0];
  if (e->ext_t == 0) {
    int rc = enqueue_rollout_begin(e, sl, s);
    if (rc) return rc;
  }
  int rc = enqueue_step(e, sl, e->ext_t, s);
  if (rc) return rc;
  A3C_CHECK(hipMemcpyAsync(actions, sl.actions + (int64_t)e->ext_t * e->E, (size_t)e->E * 4, hipMemcpyDefault, s));
  e->ext_sent.assign(e->E, 0);          // the step's uploads start empty
  e->ext_nsent = 0;
  e->ext_acted = true;
  return 0;
}

// part of observe: the post-act frames of envs [env_lo, env_hi) (rgb indexed by env, full
// [E][210][160][3] buffer) -> device, so the H2D copy of one range overlaps the host stepping of
// the next; a3c_engine_ext_observe(rgb = NULL, ...) then completes the step
extern "C" int a3c_engine_ext_upload(a3c_engine* e, const uint8_t* rgb, int env_lo, int env_hi, void* stream) {
  if (int rc = ext_check(e, "a3c_engine_ext_upload")) return rc;
  if (!e->ext_begun || !e->ext_acted || !rgb)
    return a3c_set_error(A3C_ERR_STATE, "a3c_engine_ext_upload", "ext_act of this step first");
  if (env_lo < 0 || env_hi > e->E || env_lo > env_hi)
    return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_ext_upload", "env range outside [0, num_envs]");
  const int64_t fb = (int64_t)SCREEN_H * SCREEN_W * 3;
  if (env_hi > env_lo)
    A3C_CHECK(hipMemcpyAsync(e->pool + env_lo * fb, rgb + env_lo * fb, (size_t)(env_hi - env_lo) * fb,
                             hipMemcpyDefault, (hipStream_t)stream));
  for (int i = env_lo; i < env_hi; ++i) {
    e->ext_nsent += !e->ext_sent[i];
    e->ext_sent[i] = 1;
  }
  return 0;
}

// observe of rollout step t: the post-act RGB frames [E][210][160][3] u8, rewards [E] f32 and
// terminals [E] u8 of every env (GymEnvironment.act, environment.py:78-96, done on the host) ->
// reward clip (agent.py:154), Environment.screen + History.add into the frame ring
// rgb == NULL: the frames of every env were already sent by a3c_engine_ext_upload this step
// (checked: the step's uploaded ranges must cover [0, E), else the screen would read stale frames).
extern "C" int a3c_engine_ext_observe(a3c_engine* e, const uint8_t* rgb, const float* rewards,
                                      const uint8_t* terminals, void* stream) {
  if (int rc = ext_check(e, "a3c_engine_ext_observe")) return rc;
  if (!e->ext_begun || !e->ext_acted || !rewards || !terminals)
    return a3c_set_error(A3C_ERR_STATE, "a3c_engine_ext_observe", "ext_act of this step first");
  if (!rgb && e->ext_nsent != e->E)
    return a3c_set_error(A3C_ERR_STATE, "a3c_engine_ext_observe",
                         "rgb == NULL but ext_upload did not send every env's frame this step");
  hipStream_t s = (hipStream_t)stream;
  const Slot& sl = e->slot[0];
  const int E = e->E, t = e->ext_t;
  const int64_t o = (int64_t)t * E;
  if (rgb) A3C_CHECK(hipMemcpyAsync(e->pool, rgb, (size_t)E * SCREEN_H * SCREEN_W * 3, hipMemcpyDefault, s));
  A3C_CHECK(hipMemcpyAsync(sl.rewards_raw + o, rewards, (size_t)E * 4, hipMemcpyDefault, s));
  A3C_CHECK(hipMemcpyAsync(sl.terms + o, terminals, (size_t)E, hipMemcpyDefault, s));
  hipLaunchKernelGGL(k_ext_clip, dim3((E + 255) / 256), dim3(256), 0, s, sl.rewards_raw + o, sl.rewards + o, E);
  A3C_CHECK(hipGetLastError());
  int rc = a3c_env_screen_launch(E, e->ext_idx, e->pool, e->ring, e->R, e->counters, t, s);
  if (rc) return rc;
  e->ext_t = t + 1;
  e->ext_acted = false;
  return 0;
}

// ---- summaries (agent.py:69-139 train_with_summary) ------------------------------------------
// Adds the rollout whose gradient the last rollout_grad / iterate computed to the aggregates, on
// `stream` after that call's backward (overlap: the rollout of the previous call).
extern "C" int a3c_engine_stats_accumulate(a3c_engine* e, void* stream) {
  if (!e) return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_stats_accumulate", "null");
  if (!e->reset_done) return a3c_set_error(A3C_ERR_STATE, "a3c_engine_stats_accumulate", "call a3c_engine_reset first");
  if (!e->grad_ready) return 0;
  const Slot& sl = e->slot[e->overlap ? (int)(e->iter & 1) : 0];
  hipLaunchKernelGGL(k_stats, dim3(1), dim3(256), 0, (hipStream_t)stream, sl.rewards_raw, sl.terms, sl.z, e->L.zs,
                     e->L.A, e->L.algo == A3C_ALGO_Q ? 1 : 0, e->n, e->E, e->loss, e->ep_acc, e->stats);
  A3C_CHECK(hipGetLastError());
  return 0;
}

// Waits for `stream`, copies the A3C_STATS_N aggregates to out; reset = 1 starts a new interval
// (the per-env running episode rewards carry on).
extern "C" int a3c_engine_stats_read(a3c_engine* e, double* out, int reset, void* stream) {
  if (!e || !out) return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_stats_read", "null");
  if (!e->reset_done) return a3c_set_error(A3C_ERR_STATE, "a3c_engine_stats_read", "call a3c_engine_reset first");
  hipStream_t s = (hipStream_t)stream;
  A3C_CHECK(hipStreamSynchronize(s));
  A3C_CHECK(hipMemcpy(out, e->stats, A3C_STATS_N * 8, hipMemcpyDeviceToHost));
  if (reset) {
    hipLaunchKernelGGL(k_stats_reset, dim3(1), dim3(A3C_STATS_N), 0, s, e->stats);
    A3C_CHECK(hipGetLastError());
  }
  return 0;
}

// ---- checkpoint / resume (the Supervisor's Saver, main.py:74-90, agent.py:29) ----
__global__ void k_set_step(int64_t* counters, int64_t g, int64_t w) {
  counters[1] = g;
  counters[2] = w;
}

// Resume from a checkpoint of parameters + step only (the reference's Saver keeps no more): the
// global step T and the workers' loop counter restart at the restored step (agent.py:34,46).
extern "C" int a3c_engine_set_step(a3c_engine* e, int64_t global_step, int64_t worker_step, void* stream) {
  if (!e || global_step < 0 || worker_step < 0) return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_set_step", "bad argument");
  if (!e->reset_done) return a3c_set_error(A3C_ERR_STATE, "a3c_engine_set_step", "call a3c_engine_reset first");
  e->step0_g = global_step;
  e->step0_w = worker_step;
  if (!e->ext || e->ext_begun) {
    hipLaunchKernelGGL(k_set_step, dim3(1), dim3(1), 0, (hipStream_t)stream, e->counters, global_step, worker_step);
    A3C_CHECK(hipGetLastError());
  }
  return 0;
}

namespace {
struct StateRegion { void* p; size_t bytes; };
struct StateHeader {
  uint32_t magic, version;
  int32_t E, n, R, algo, A, lstm, overlap, world, frame84, env_id_base;
  int64_t total, bytes, iter;
  uint64_t seed;
  int32_t grad_ready, grad_applied;
  int32_t l2bits;        // whether the rollout in flight wrote the l2 ReLU bits its backward reads
  int32_t boot_bwd;      // whether the pending backward folds V(s_n) from the slot's fc partials
};
constexpr uint32_t STATE_MAGIC = 0x53433341u;   // "A3CS"
}

// every device buffer whose contents carry from one iteration to the next: parameters, target,
// RMSProp slots, counters, env state, frame ring, the LSTM carry, and in overlap mode the rollout
// in flight (its parameter snapshot, tau, transitions and saved activations)
static std::vector<StateRegion> state_regions(const a3c_engine* e) {
  std::vector<StateRegion> r;
  const int64_t T = e->L.total, E = e->E, nE = e->nE, zs = e->L.zs;
  auto add = [&](const void* p, int64_t b) { r.push_back({const_cast<void*>(p), (size_t)b}); };
  add(e->params, T * 4); add(e->tparams, T * 4); add(e->ms, T * 4); add(e->mom, T * 4);
  add(e->counters, 64); add(e->loss, 64); add(e->stats, A3C_STATS_N * 8); add(e->ep_acc, E * 8);
  add(e->ring, E * e->R * PLANE);
  add(e->env.episode, 2 * E * 4); add(e->env.ep_step, 2 * E * 4); add(e->env.ep_len, 2 * E * 4);
  add(e->env.lives, 2 * E * 4); add(e->env.frame, 2 * E * 4); add(e->env.reward, 2 * E * 4);
  add(e->env.terminal, 2 * E);
  for (int k = 0; k < e->nslot; ++k) {
    const Slot& sl = e->slot[k];
    if (e->overlap) {
      add(sl.P, T * 4); add(sl.tau, 64);
      add(sl.actions, nE * 4); add(sl.frames, nE * 4); add(sl.rewards, nE * 4); add(sl.rewards_raw, nE * 4);
      add(sl.terms, nE);
      add(sl.z, (nE + E) * zs * 4); add(sl.R_buf, nE * 4);
      if (e->nat) {
        add(sl.act_l1, nE * NT_A1 * 4); add(sl.act_l2, nE * NT_A2 * 4); add(sl.act_l3, nE * NT_FLAT * 4);
        add(sl.act_l4, nE * NT_FC * 4);
      } else {
        add(sl.act_l1, nE * C1_P * C1_N * 4); add(sl.act_l2, nE * FLAT * 4); add(sl.act_l3, nE * FC * 4);
      }
      add(sl.l2m, nE * C2_Q * 4);     // (the pending backward's dl2 mask)
      if (boot_bwd(e)) add(sl.fcboot, (int64_t)FC_NS * E * FC * 4);   // (the pending backward's V(s_n) partials)
    }
    if (e->L.lstm) {
      add(sl.lh, nE * LSTM_U * 4); add(sl.lc, nE * LSTM_U * 4);
      if (!e->overlap) add(sl.terms, nE);
      else {
        add(sl.lhp, nE * LSTM_U * 4); add(sl.lcp, nE * LSTM_U * 4); add(sl.lg, nE * LSTM_G * 4);
        add(sl.lhb, E * LSTM_U * 4); add(sl.lcb, E * LSTM_U * 4);
      }
    }
  }
  return r;
}

static StateHeader state_header(const a3c_engine* e) {
  StateHeader h = {};
  // 2: + the l2 ReLU bits of the rollout in flight; 3: + l2bits; 4: + boot_bwd, fcboot only with it
  h.magic = STATE_MAGIC; h.version = 4;
  h.E = e->E; h.n = e->n; h.R = e->R; h.algo = e->L.algo; h.A = e->L.A; h.lstm = e->L.lstm ? 1 : 0;
  h.overlap = e->overlap; h.world = e->cfg.world_size; h.frame84 = e->frame84;
  h.env_id_base = e->cfg.env_id_base; h.seed = e->cfg.seed;   // the env shard and its random streams
  h.total = e->L.total;
  h.l2bits = l2bits_on(e) ? 1 : 0;
  h.boot_bwd = boot_bwd(e) ? 1 : 0;
  int64_t b = sizeof(StateHeader);
  for (const StateRegion& x : state_regions(e)) b += (int64_t)x.bytes;
  h.bytes = b;
  return h;
}

static int state_check(const a3c_engine* e, const char* what) {
  if (!e) return a3c_set_error(A3C_ERR_INVALID, what, "null");
  if (e->ext)
    return a3c_set_error(A3C_ERR_INVALID, what, "host-stepped envs cannot be snapshotted: resume from params + "
                         "RMSProp slots + a3c_engine_set_step");
  if (!e->reset_done) return a3c_set_error(A3C_ERR_STATE, what, "call a3c_engine_reset first");
  return 0;
}

extern "C" int a3c_engine_state_bytes(a3c_engine* e, int64_t* bytes) {
  if (int rc = state_check(e, "a3c_engine_state_bytes")) return rc;
  if (!bytes) return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_state_bytes", "null");
  *bytes = state_header(e).bytes;
  return 0;
}

// Waits for the engine's work on `stream` and its rollout stream, then copies the state to host.
extern "C" int a3c_engine_state_save(a3c_engine* e, void* host, int64_t bytes, void* stream) {
  if (int rc = state_check(e, "a3c_engine_state_save")) return rc;
  StateHeader h = state_header(e);
  if (!host || bytes != h.bytes) return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_state_save", "buffer size");
  A3C_CHECK(hipStreamSynchronize((hipStream_t)stream));
  if (e->rs) A3C_CHECK(hipStreamSynchronize(e->rs));
  h.iter = e->iter;
  h.grad_ready = e->grad_ready;
  h.grad_applied = e->grad_applied;
  uint8_t* o = (uint8_t*)host;
  memcpy(o, &h, sizeof(h));
  o += sizeof(h);
  for (const StateRegion& x : state_regions(e)) {
    A3C_CHECK(hipMemcpy(o, x.p, x.bytes, hipMemcpyDeviceToHost));
    o += x.bytes;
  }
  return 0;
}

// Restores a state written by a3c_engine_state_save into an engine of the same configuration
// (after a3c_engine_reset: the frame pool is regenerated there); the next iteration continues
// the saved run bit for bit.
extern "C" int a3c_engine_state_load(a3c_engine* e, const void* host, int64_t bytes, void* stream) {
  if (int rc = state_check(e, "a3c_engine_state_load")) return rc;
  const StateHeader want = state_header(e);
  StateHeader h;
  if (!host || bytes < (int64_t)sizeof(h)) return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_state_load", "short buffer");
  memcpy(&h, host, sizeof(h));
  if (h.magic != STATE_MAGIC || h.version != want.version)
    return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_state_load", "not an engine state");
  if (h.E != want.E || h.n != want.n || h.R != want.R || h.algo != want.algo || h.A != want.A ||
      h.lstm != want.lstm || h.overlap != want.overlap || h.world != want.world || h.frame84 != want.frame84 ||
      h.env_id_base != want.env_id_base || h.seed != want.seed || h.total != want.total || h.bytes != want.bytes ||
      h.l2bits != want.l2bits || h.boot_bwd != want.boot_bwd || bytes != want.bytes)
    return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_state_load", "state of a different engine configuration");
  hipStream_t s = (hipStream_t)stream;
  A3C_CHECK(hipStreamSynchronize(s));
  if (e->rs) A3C_CHECK(hipStreamSynchronize(e->rs));
  const uint8_t* o = (const uint8_t*)host + sizeof(h);
  for (const StateRegion& x : state_regions(e)) {
    A3C_CHECK(hipMemcpy(x.p, o, x.bytes, hipMemcpyHostToDevice));
    o += x.bytes;
  }
  A3C_CHECK(hipMemset(e->xflags, 0, 64));       // fresh cross-stream sequence numbers
  A3C_CHECK(hipDeviceSynchronize());
  e->s_seq = e->r_seq = 0;
  e->roll_seq[0] = e->roll_seq[1] = 0;
  e->iter = h.iter;
  e->grad_ready = h.grad_ready != 0;
  e->grad_applied = h.grad_applied != 0;
  return 0;
}

extern "C" int a3c_engine_slot_buffers(a3c_engine* e, int slot, a3c_engine_buffers* b) {
  if (!e || !b || slot < 0 || slot >= e->nslot)
    return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_slot_buffers", "bad argument");
  const Slot& sl = e->slot[slot];
  memset(b, 0, sizeof(*b));
  b->params = e->params; b->target_params = e->tparams; b->ms = e->ms; b->mom = e->mom; b->grads = e->grads;
  b->n_params = e->L.total;
  b->frame_ring = e->ring; b->ring_slots = e->R;
  b->tau = e->counters; b->global_step = e->counters + 1;
  b->actions = sl.actions; b->rewards = sl.rewards; b->terminals = sl.terms;
  b->z = sl.z; b->returns = sl.R_buf; b->loss = e->loss; b->sumsq = e->sumsq;
  b->act_l1 = sl.act_l1; b->act_l2 = sl.act_l2; b->act_l3 = sl.act_l3; b->act_l4 = sl.act_l4;
  b->trunk = e->L.trunk;
  b->frame_pool = e->pool;
  b->env_frame = e->env.frame; b->env_lives = e->env.lives; b->env_episode = e->env.episode;
  b->env_step = e->env.ep_step; b->env_len = e->env.ep_len;
  b->zs = e->L.zs; b->n_tensors = e->L.nt;
  for (int i = 0; i < e->L.nt; ++i) { b->offsets[i] = e->L.off[i]; b->sizes[i] = e->L.size[i]; }
  b->sched = e->sched;
  if (e->L.lstm) {
    b->lstm_h = sl.lh; b->lstm_c = sl.lc; b->lstm_hp = sl.lhp; b->lstm_cp = sl.lcp; b->lstm_gates = sl.lg;
    b->lstm_units = LSTM_U;
  }
  return 0;
}

__global__ void k_advance(int64_t* counters, int64_t dtau, int64_t dstep) {
  counters[0] += dtau;
  counters[1] += dstep;
}

extern "C" int a3c_engine_advance(a3c_engine* e, void* stream) {
  if (!e || e->overlap) return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_advance", "sync engines only");
  if (!e->grad_ready) return 0;
  hipLaunchKernelGGL(k_advance, dim3(1), dim3(1), 0, (hipStream_t)stream, e->counters, (int64_t)e->n,
                     e->nE * e->cfg.world_size);
  A3C_CHECK(hipGetLastError());
  return 0;
}

extern "C" int a3c_engine_get_buffers(a3c_engine* e, a3c_engine_buffers* b) {
  return a3c_engine_slot_buffers(e, 0, b);
}

// ---- profiling hook: average duration of one engine kernel, HIP events on the caller's stream ----
extern "C" int a3c_engine_time_kernel(a3c_engine* e, int kernel, int iters, void* stream, float* avg_ms) {
  if (!e || !avg_ms || iters < 1 || !e->reset_done)
    return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_time_kernel", "bad argument");
  hipStream_t s = (hipStream_t)stream;
  const NetLayout& L = e->L;
  const int E = e->E;
  const Slot& sl = e->slot[0];
  if (e->rs) A3C_CHECK(hipStreamSynchronize(e->rs));
  a3c_set_shared_gpu(e->overlap != 0);      // time the variants the engine runs
  a3c_set_bwd_bound(bwd_bound(e));
  a3c_set_fcp_split(e->frame84 ? 2 : 4);
  struct ResetShared {
    ~ResetShared() { a3c_set_shared_gpu(false); a3c_set_bwd_bound(false); a3c_set_fcp_split(2); }
  } reset_shared;
  if (e->nat != (kernel >= A3C_KER_NAT_C1F))
    return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_time_kernel", "kernel id of another trunk");
  if (e->nat) {   // one pass of the nature trunk: forward over E states, backward passes over n*E samples
    const int pass = kernel - A3C_KER_NAT_C1F;
    const bool fwd = pass <= NAT_FCF;
    if ((pass == NAT_C3F && a3c_nat_conv23_fused()) || (pass == NAT_C1F && a3c_nat_conv123_fused()) ||
        (pass == NAT_C2X && a3c_nat_dx_fused()))
      return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_time_kernel",
                           "this pass runs inside another pass's launch (k_nat_conv23 under A3C_KER_NAT_C2F, k_nat_dx32 under A3C_KER_NAT_C3X)");
    if (!fwd && !e->grad_ready)
      return a3c_set_error(A3C_ERR_STATE, "a3c_engine_time_kernel", "backward passes: run an iteration first");
    const Slot& bs = e->slot[e->nslot == 2 ? (int)((e->iter - 2) & 1) : 0];   // the last back-propagated rollout
    const StateAddr sa = fwd ? ring_addr(e, 0, e->counters) : ring_addr(e, 0, bs.tau);
    auto go = [&]() -> int {
      return fwd ? a3c_nat_pass_launch(pass, L, e->params, sa, E, sl.act_l1, sl.act_l2, sl.act_l3, sl.act_l4,
                                       (const uint16_t*)sl.prep, e->nat_fws, nullptr, s)
                 : a3c_nat_pass_launch(pass, L, bs.P, sa, e->nE, bs.act_l1, bs.act_l2, bs.act_l3, bs.act_l4,
                                       (const uint16_t*)bs.prep, nullptr, e->ws, s);
    };
    int rc = go();
    if (rc) return rc;
    hipEvent_t a, b;
    A3C_CHECK(hipEventCreate(&a));
    A3C_CHECK(hipEventCreate(&b));
    A3C_CHECK(hipEventRecord(a, s));
    for (int i = 0; i < iters && !rc; ++i) rc = go();
    A3C_CHECK(hipEventRecord(b, s));
    A3C_CHECK(hipEventSynchronize(b));
    float ms = 0.f;
    A3C_CHECK(hipEventElapsedTime(&ms, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    if (rc) return rc;
    *avg_ms = ms / (float)iters;
    return 0;
  }
  if (kernel == A3C_KER_CONV12_FWD || kernel == A3C_KER_FC_FWD || kernel == A3C_KER_HEAD_SCREEN_CONV12) {
    int rc0 = a3c_prep_fwd_launch(L, e->params, sl.prep, s);
    if (rc0) return rc0;
  }
  // head_screen: each launch shifts the frame indices (frame_salt) so it streams frames that are
  // not cache-resident, like the live rollout (re-reading one frame set would time MALL hits)
  uint32_t salt = 0;
  auto launch = [&]() -> int {
    salt += 4099u;
    switch (kernel) {
      case A3C_KER_CONV12_FWD:
        return a3c_conv12_launch(L, e->params, sl.prep, ring_addr(e, 0, e->counters), E, sl.act_l1, sl.act_l2, s);
      case A3C_KER_FC_FWD:
        return a3c_fc_fwd_launch(sl.act_l2, (const float*)(sl.prep + PREP_W1S_BYTES), e->params + L.off[T_FCB],
                                 sl.act_l3, E, s, e->params + L.off[T_FCW]);
      case A3C_KER_FC_PART:
        return a3c_fc_part_launch(sl.act_l2, (const float*)(sl.prep + PREP_W1S_BYTES), e->fcpart, E, s);
      case A3C_KER_ENV_STEP:
        if (e->frame84) return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_time_kernel", "no screen kernel in frame84 mode");
        return a3c_env_screen_launch(E, sl.frames, e->pool, e->ring, e->R, e->counters, 0, s);
      case A3C_KER_HEAD_SCREEN:
      case A3C_KER_HEAD_SCREEN_CONV12: {
        // head + action draw + env act + Environment.screen as in rollout step 0 (idempotent:
        // the env state is read from the tau-parity half and written to the other one)
        HeadSelect sel = {};
        sel.mode = L.algo == A3C_ALGO_Q ? 1 : 0;
        sel.k0 = e->k0; sel.k1 = e->k1;
        sel.tau_ptr = e->counters; sel.tau_add = 0;
        sel.env_id_base = e->cfg.env_id_base; sel.E = E; sel.par_E = E;
        if (sel.mode) set_eps_schedule(e, sel);
        sel.actions = sl.actions;
        sel.env_on = 1;
        sel.envp = e->envp; sel.envb = e->env;
        sel.rewards = sl.rewards; sel.terms = sl.terms;
        sel.frames_out = sl.frames;
        sel.pool = e->pool; sel.ring = e->ring; sel.R = e->R;
        sel.frame84 = e->frame84;
        sel.frame_salt = salt;
        if (kernel == A3C_KER_HEAD_SCREEN)
          return a3c_head_screen_launch(L, e->params, L.lstm ? sl.lh : sl.act_l3, E, sl.z, sel, s);
        // + conv1 + conv2 of the next states into step 1's activation rows (as rollout step 0)
        Conv12Next nx = {};
        nx.sa = ring_addr(e, 1, e->counters);
        nx.w1s = (const uint16_t*)sl.prep;
        nx.b1 = e->params + L.off[T_L1B]; nx.W2 = e->params + L.off[T_L2W]; nx.b2 = e->params + L.off[T_L2B];
        nx.act_l1 = sl.act_l1 + (int64_t)E * C1_P * C1_N;
        nx.act_l2 = sl.act_l2 + (int64_t)E * FLAT;
        if (fc_split(e)) {       // the head folds the fc partials, as in the rollout
          sel.fc_part = e->fcpart;
          sel.fc_bias = e->params + L.off[T_FCB];
          sel.l3_out = sl.act_l3;
        }
        return a3c_head_screen_conv12_launch(L, e->params, L.lstm ? sl.lh : sl.act_l3, E, sl.z, sel, nx, s);
      }
      case A3C_KER_CONV_BWD: {
        const BwdPlan p = a3c_bwd_plan(L, e->nE);
        return a3c_conv_bwd_launch(L, e->params, ring_addr(e, 0, e->counters), e->nE, sl.act_l1, e->ws + p.dl2, e->ws, s);
      }
      default:
        return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_time_kernel", "unknown kernel id");
    }
  };
  int rc = launch();   // warm
  if (rc) return rc;
  hipEvent_t a, b;
  A3C_CHECK(hipEventCreate(&a));
  A3C_CHECK(hipEventCreate(&b));
  A3C_CHECK(hipEventRecord(a, s));
  for (int i = 0; i < iters && !rc; ++i) rc = launch();
  A3C_CHECK(hipEventRecord(b, s));
  A3C_CHECK(hipEventSynchronize(b));
  float ms = 0.f;
  A3C_CHECK(hipEventElapsedTime(&ms, a, b));
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  if (rc) return rc;
  *avg_ms = ms / (float)iters;
  return 0;
}

// Live launch spans of the engine's dominant kernels (which 0: k_conv_bwd, 1:
// k_head_screen_conv12), recorded by the kernels themselves inside the replayed graphs: per
// launch, last workgroup end - first workgroup start (s_memrealtime, 100 MHz).  reset = 1 clears
// the records (call it synchronised, before a timed region); otherwise the average / max span
// in microseconds over the launches recorded since.
extern "C" int a3c_engine_span_stats(a3c_engine* e, int which, int reset, double* avg_us, double* max_us,
                                     int64_t* launches) {
  if (!e || which < 0 || which > 1) return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_span_stats", "bad argument");
  const size_t per = (size_t)SPAN_RECS * SPAN_WGS * 2;
  unsigned long long* d = e->spans + (size_t)which * per;
  std::vector<unsigned long long> h(per);
  if (reset) {                            // start stamps ~0, end stamps 0 = not written
    for (size_t i = 0; i < per; i += 2) { h[i] = ~0ull; h[i + 1] = 0ull; }
    A3C_CHECK(hipDeviceSynchronize());
    A3C_CHECK(hipMemcpy(d, h.data(), per * sizeof(unsigned long long), hipMemcpyHostToDevice));
    return 0;
  }
  A3C_CHECK(hipDeviceSynchronize());
  A3C_CHECK(hipMemcpy(h.data(), d, per * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  double sum = 0.0, mx = 0.0;
  int64_t n = 0;
  for (int r = 0; r < SPAN_RECS; ++r) {
    unsigned long long lo = ~0ull, hi = 0ull;
    for (int w = 0; w < SPAN_WGS; ++w) {
      const unsigned long long a = h[2 * ((size_t)r * SPAN_WGS + w)], b = h[2 * ((size_t)r * SPAN_WGS + w) + 1];
      if (a == ~0ull || b == 0ull) continue;
      lo = a < lo ? a : lo;
      hi = b > hi ? b : hi;
    }
    if (hi == 0ull || lo == ~0ull || hi < lo) continue;
    const double us = (double)(hi - lo) * 0.01;
    sum += us;
    mx = us > mx ? us : mx;
    ++n;
  }
  if (avg_us) *avg_us = n ? sum / (double)n : 0.0;
  if (max_us) *max_us = mx;
  if (launches) *launches = n;
  return 0;
}

// Raw records (measurement): out[2 r] / out[2 r + 1] = first workgroup start / last workgroup end
// (s_memrealtime, 0 when not recorded) of record r of `which`; *tau_now = the live tau counter.
extern "C" int a3c_engine_span_raw(a3c_engine* e, int which, unsigned long long* out, int64_t* tau_now) {
  if (!e || which < 0 || which > 1 || !out || !tau_now)
    return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_span_raw", "bad argument");
  const size_t per = (size_t)SPAN_RECS * SPAN_WGS * 2;
  std::vector<unsigned long long> h(per);
  A3C_CHECK(hipDeviceSynchronize());
  A3C_CHECK(hipMemcpy(h.data(), e->spans + (size_t)which * per, per * sizeof(unsigned long long),
                      hipMemcpyDeviceToHost));
  A3C_CHECK(hipMemcpy(tau_now, e->counters, sizeof(int64_t), hipMemcpyDeviceToHost));
  for (int r = 0; r < SPAN_RECS; ++r) {
    unsigned long long lo = ~0ull, hi = 0ull;
    for (int w = 0; w < SPAN_WGS; ++w) {
      const unsigned long long a = h[2 * ((size_t)r * SPAN_WGS + w)], b = h[2 * ((size_t)r * SPAN_WGS + w) + 1];
      if (a == ~0ull || b == 0ull) continue;
      lo = a < lo ? a : lo;
      hi = b > hi ? b : hi;
    }
    const bool ok = hi != 0ull && lo != ~0ull && hi >= lo;
    out[2 * r] = ok ? lo : 0ull;
    out[2 * r + 1] = ok ? hi : 0ull;
  }
  return 0;
}

// Per-step split of the k_head_screen_conv12 records.  Step t of the rollout at tau writes record
// (tau + t + 1) % SPAN_RECS (its Conv12Next reads state tau + t + 1), and every rollout's tau is
// congruent to the live counter modulo n, so record r belongs to the most recent value
// v = tau + t + 1 <= tau_now + n with v = r (mod SPAN_RECS), and t = (v - 1 - tau_now) mod n.
extern "C" int a3c_engine_span_steps(a3c_engine* e, double* avg_us, int64_t* launches) {
  if (!e || !avg_us || !launches) return a3c_set_error(A3C_ERR_INVALID, "a3c_engine_span_steps", "bad argument");
  const int n = e->n;
  const size_t per = (size_t)SPAN_RECS * SPAN_WGS * 2;
  std::vector<unsigned long long> h(per);
  int64_t tau_now = 0;
  A3C_CHECK(hipDeviceSynchronize());
  A3C_CHECK(hipMemcpy(h.data(), e->spans + per, per * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  A3C_CHECK(hipMemcpy(&tau_now, e->counters, sizeof(int64_t), hipMemcpyDeviceToHost));
  std::vector<double> sum(n, 0.0);
  for (int t = 0; t < n; ++t) launches[t] = 0;
  for (int r = 0; r < SPAN_RECS; ++r) {
    unsigned long long lo = ~0ull, hi = 0ull;
    for (int w = 0; w < SPAN_WGS; ++w) {
      const unsigned long long a = h[2 * ((size_t)r * SPAN_WGS + w)], b = h[2 * ((size_t)r * SPAN_WGS + w) + 1];
      if (a == ~0ull || b == 0ull) continue;
      lo = a < lo ? a : lo;
      hi = b > hi ? b : hi;
    }
    if (hi == 0ull || lo == ~0ull || hi < lo) continue;
    const int64_t top = tau_now + n;
    const int64_t v = top - (((top - r) % SPAN_RECS) + SPAN_RECS) % SPAN_RECS;
    const int t = (int)((((v - 1 - tau_now) % n) + n) % n);
    sum[t] += (double)(hi - lo) * 0.01;
    launches[t] += 1;
  }
  for (int t = 0; t < n; ++t) avg_us[t] = launches[t] ? sum[t] / (double)launches[t] : 0.0;
  return 0;
}

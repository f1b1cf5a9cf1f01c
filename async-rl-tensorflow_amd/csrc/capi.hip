// C-ABI entry points of liba3c_hip.so (include/a3c_hip.h): error channel, layout queries and the
// stateless network ops.  Everything enqueues on the caller's stream; nothing allocates.
#include <cstdio>
#include <cstring>
#include <mutex>
#include "net_bwd.h"
#include "optim.h"

static thread_local char g_err[512] = "";

extern "C" int a3c_set_error(int code, const char* what, const char* detail) {
  snprintf(g_err, sizeof(g_err), "%s: %s (code %d)", what ? what : "?", detail ? detail : "", code);
  return code ? code : A3C_ERR_INVALID;
}

extern "C" const char* a3c_last_error(void) { return g_err; }
extern "C" const char* a3c_version(void) { return "a3c_hip 0.1.0 gfx950"; }

extern "C" int a3c_device_ok(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return 0;
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 0;
  return strncmp(p.gcnArchName, "gfx950", 6) == 0 ? 1 : 0;
}

void a3c_init_once() {
  static std::once_flag f;
  std::call_once(f, [] {
    a3c_conv12_set_smem();
    a3c_conv_bwd_set_smem();
  });
}

extern "C" int a3c_param_layout(const a3c_net_desc* net, int* n_tensors, int64_t* offsets, int64_t* sizes,
                                int64_t* total) {
  NetLayout L;
  if (a3c_make_layout(net, &L)) return a3c_set_error(A3C_ERR_INVALID, "a3c_param_layout", "unsupported net");
  if (n_tensors) *n_tensors = L.nt;
  for (int i = 0; i < L.nt; ++i) {
    if (offsets) offsets[i] = L.off[i];
    if (sizes) sizes[i] = L.size[i];
  }
  if (total) *total = L.total;
  return 0;
}

extern "C" int a3c_z_stride(const a3c_net_desc* net) {
  NetLayout L;
  if (a3c_make_layout(net, &L)) return -1;
  return L.zs;
}

extern "C" int a3c_workspace_bytes(const a3c_net_desc* net, int64_t B, int64_t* bytes) {
  NetLayout L;
  if (a3c_make_layout(net, &L) || L.trunk != A3C_TRUNK_NIPS || B < 0 || !bytes)
    return a3c_set_error(A3C_ERR_INVALID, "a3c_workspace_bytes", "bad argument (per-op ops: NIPS trunk)");
  // forward: the bf16-split conv1 weights; backward: its plan (they never run at once)
  BwdPlan p = a3c_bwd_plan(L, B > 0 ? B : 1);
  int64_t m = p.total > PREP_BYTES / 4 ? p.total : PREP_BYTES / 4;
  *bytes = m * (int64_t)sizeof(float) + 256;
  return 0;
}

static StateAddr contiguous_states(const uint8_t* states, int64_t B) {
  StateAddr sa;
  sa.base = states;
  sa.env_stride = (int64_t)HIST * PLANE;
  sa.plane_bytes = PLANE;
  sa.E = (int)B;
  sa.R = HIST;
  sa.L = HIST;
  sa.tau_offset = HIST - 1;
  sa.tau_ptr = nullptr;
  return sa;
}

static float* align_ws(void* ws) { return (float*)(((uintptr_t)ws + 255) & ~(uintptr_t)255); }

extern "C" int a3c_forward(const a3c_net_desc* net, const float* params, const uint8_t* states, int64_t B,
                           float* act_l1, float* act_l2, float* act_l3, float* z, void* workspace,
                           void* stream) {
  NetLayout L;
  if (a3c_make_layout(net, &L) || L.lstm || L.trunk != A3C_TRUNK_NIPS || !params || !states || !act_l2 || !act_l3 || !z || B < 0 ||
      B > 0x7fffffff || (((uintptr_t)states) & 15))
    return a3c_set_error(A3C_ERR_INVALID, "a3c_forward", "bad argument");
  if (B == 0) return 0;
  a3c_init_once();
  if (!workspace) return a3c_set_error(A3C_ERR_INVALID, "a3c_forward", "workspace required");
  HeadSelect sel = {};
  sel.mode = -1;
  sel.E = 1;
  uint8_t* prep = (uint8_t*)align_ws(workspace);
  int rc = a3c_prep_fwd_launch(L, params, prep, (hipStream_t)stream);
  if (rc) return rc;
  return a3c_forward_launch(L, params, prep, contiguous_states(states, B), B, act_l1, act_l2, act_l3, z, sel,
                            (hipStream_t)stream);
}

extern "C" int a3c_select_action(int mode, const float* z, int64_t B, int zs, int A, const float* eps,
                                 uint64_t seed, int64_t tau, const int32_t* env_ids, int32_t* actions,
                                 void* stream) {
  if (!z || !actions || B < 0 || A < 1 || A > 31 || zs < A || zs > 64 || (mode != 0 && mode != 1) ||
      (mode == 1 && !eps))
    return a3c_set_error(A3C_ERR_INVALID, "a3c_select_action", "bad argument");
  HeadSelect sel = {};
  sel.mode = mode;
  sel.k0 = (uint32_t)seed;
  sel.k1 = (uint32_t)(seed >> 32);
  sel.tau_ptr = nullptr;
  sel.tau_add = tau;
  sel.env_ids = env_ids;
  sel.env_id_base = 0;
  sel.E = (int)(B > 0 ? B : 1);
  sel.eps = eps;
  sel.actions = actions;
  return a3c_select_launch(z, B, zs, A, sel, (hipStream_t)stream);
}

extern "C" int a3c_returns(const float* rewards, const uint8_t* terminals, const float* bootstrap, int n,
                           int64_t E, double gamma, float* R, void* stream) {
  if (!rewards || !terminals || !bootstrap || !R || n <= 0 || E < 0)
    return a3c_set_error(A3C_ERR_INVALID, "a3c_returns", "bad argument");
  return a3c_returns_launch(rewards, terminals, bootstrap, 1, n, E, gamma, R, (hipStream_t)stream);
}

extern "C" int a3c_td_target(const float* rewards, const uint8_t* terminals, const float* q_next, int64_t B,
                             int A, int zs, double discount, float* target, void* stream) {
  if (!rewards || !terminals || !q_next || !target || B < 0 || A < 1 || zs < A)
    return a3c_set_error(A3C_ERR_INVALID, "a3c_td_target", "bad argument");
  return a3c_td_target_launch(rewards, terminals, q_next, B, A, zs, discount, target, (hipStream_t)stream);
}

extern "C" int a3c_loss_backward(const a3c_net_desc* net, const float* params, const uint8_t* states, int64_t B,
                                 const float* act_l1, const float* act_l2, const float* act_l3, const float* z,
                                 const int32_t* actions, const float* target, float beta, int literal_adv,
                                 float* grads, float* loss_out, void* workspace, void* stream) {
  NetLayout L;
  if (a3c_make_layout(net, &L) || L.lstm || L.trunk != A3C_TRUNK_NIPS || !params || !states || !act_l1 || !act_l2 || !act_l3 || !z || !actions ||
      !target || !grads || !workspace || B <= 0 || B > 0x7fffffff || (((uintptr_t)states) & 15))
    return a3c_set_error(A3C_ERR_INVALID, "a3c_loss_backward", "bad argument");
  a3c_init_once();
  return a3c_backward_launch(L, params, contiguous_states(states, B), B, act_l1, act_l2, act_l3, z, actions,
                             target, beta, literal_adv, grads, loss_out, align_ws(workspace),
                             (hipStream_t)stream);
}

// C5 LSTM policy head for gfx950 (BASELINE config 5; build-defined, the reference has no
// recurrent code).  TF1 BasicLSTMCell semantics, oracle/ref_cpu.py lstm_cell / lstm_*_seq:
//   a = [x, h_prev] @ W + b  (W [512][1024], gate columns i, j, f, o)
//   c = c_prev * sigmoid(f + 1) + sigmoid(i) * tanh(j);  h = tanh(c) * sigmoid(o)
// with the carried state zeroed after a terminal transition.
//
//  k_lstm_fwd       one workgroup per (16 envs x 16 units): the [x, h_prev] rows are staged in
//                   LDS (masked), wave g runs gate g's 16x16 tile over K = 512 on
//                   v_mfma_f32_16x16x4_f32 (two independent accumulator chains), the four
//                   gate tiles meet in LDS and the cell update is fused into the epilogue.
//  k_lstm_cell_bwd  elementwise cell backward of step t; also finishes step t+1's input
//                   gradient (dx masked by the fc ReLU, dh into the recurrence).
//  BPTT GEMMs       dxh_t = da_t W^T per step, dW = [x, hp]^T da over all n*E rows (+ colsum
//                   -> db) on the fp32 MFMA GEMM of gemm.hip.
#include "lstm.h"
#include "gemm.h"

#define LT 16                    // envs / units per workgroup tile
#define LA_LD (LSTM_K + 4)       // LDS row stride of the staged [x, h] rows

__device__ inline float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

__global__ void __launch_bounds__(256) k_lstm_fwd(const float* __restrict__ X, const float* __restrict__ W,
                                                  const float* __restrict__ bias, LstmStep st, int64_t B) {
  __shared__ __attribute__((aligned(16))) float As[LT][LA_LD];
  __shared__ float Gs[4][LT][LT + 1];
  const int tid = threadIdx.x, lane = tid & 63, g = tid >> 6;
  const int64_t e0 = (int64_t)blockIdx.x * LT;
  const int u0 = blockIdx.y * LT;
  // stage rows e0..e0+15 of [x | h_prev * keep] (16 x 512 floats, float4 per thread-step)
  for (int i = tid; i < LT * (LSTM_K / 4); i += 256) {
    const int r = i / (LSTM_K / 4), q = i - r * (LSTM_K / 4);
    const int64_t e = e0 + r;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (e < B) {
      if (q < FC / 4) {
        v = *(const f32x4*)(X + e * FC + 4 * q);
      } else if (!(st.prev_terms && st.prev_terms[e])) {
        v = *(const f32x4*)(st.h_src + e * LSTM_U + 4 * (q - FC / 4));
      }
    }
    *(f32x4*)&As[r][4 * q] = v;
  }
  __syncthreads();
  // wave g: gate g, columns g*256 + u0 .. +15; A[row = lane&15][k = lane>>4], B[k][col = lane&15]
  const int col = g * LSTM_U + u0 + (lane & 15);
  const int kr = lane >> 4;
  const float* wp = W + (int64_t)kr * LSTM_G + col;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int k0 = 0; k0 < LSTM_K; k0 += 8) {
    const float a0 = As[lane & 15][k0 + kr];
    const float a1 = As[lane & 15][k0 + 4 + kr];
    const float b0 = wp[(int64_t)k0 * LSTM_G];
    const float b1 = wp[(int64_t)(k0 + 4) * LSTM_G];
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc1, 0, 0, 0);
  }
  const float bc = bias[col];
#pragma unroll
  for (int i = 0; i < 4; ++i) Gs[g][4 * kr + i][lane & 15] = acc0[i] + acc1[i] + bc;
  __syncthreads();
  // cell update of (env r, unit c)
  const int r = tid >> 4, c = tid & 15;
  const int64_t e = e0 + r;
  if (e >= B) return;
  const int u = u0 + c;
  const int64_t o = e * LSTM_U + u;
  const bool keep = !(st.prev_terms && st.prev_terms[e]);
  const float cprev = keep ? st.c_src[o] : 0.f;
  const float ig = sigmoidf_(Gs[0][r][c]);
  const float jg = tanhf(Gs[1][r][c]);
  const float fg = sigmoidf_(Gs[2][r][c] + 1.0f);     // forget_bias = 1.0
  const float og = sigmoidf_(Gs[3][r][c]);
  const float cn = cprev * fg + ig * jg;
  const float hn = tanhf(cn) * og;
  if (st.hp) st.hp[o] = keep ? st.h_src[o] : 0.f;
  if (st.cp) st.cp[o] = cprev;
  if (st.gates) {
    float* gp = st.gates + e * LSTM_G + u;
    gp[0] = ig;
    gp[LSTM_U] = jg;
    gp[2 * LSTM_U] = fg;
    gp[3 * LSTM_U] = og;
  }
  st.c[o] = cn;
  st.h[o] = hn;
}

int a3c_lstm_fwd_launch(const float* W, const float* bias, const float* x, const LstmStep& st, int64_t B,
                        hipStream_t s) {
  if (B <= 0) return 0;
  if (!W || !bias || !x || !st.h_src || !st.c_src || !st.h || !st.c ||
      (((uintptr_t)x | (uintptr_t)st.h_src) & 15))
    return a3c_set_error(A3C_ERR_INVALID, "a3c_lstm_step", "bad argument");
  hipLaunchKernelGGL(k_lstm_fwd, dim3((unsigned)((B + LT - 1) / LT), LSTM_U / LT), dim3(256), 0, s, x, W, bias,
                     st, B);
  A3C_CHECK(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------------------------------
// backward of step t (one thread per (env, unit)); dxh holds d[x, hp] of step t+1 when has_next
__global__ void __launch_bounds__(256) k_lstm_cell_bwd(int64_t E, int has_next, const float* __restrict__ G,
                                                       const float* __restrict__ C, const float* __restrict__ CP,
                                                       const float* __restrict__ dH,
                                                       const uint8_t* __restrict__ terms_t,
                                                       const float* __restrict__ dxh, float* __restrict__ dcp,
                                                       const float* __restrict__ x_next, float* __restrict__ dx_next,
                                                       float* __restrict__ DA) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= E * LSTM_U) return;
  const int64_t e = i / LSTM_U;
  const int u = (int)(i - e * LSTM_U);
  float dh = dH[i];
  float dcn = 0.f;
  if (has_next) {
    const float keep = terms_t[e] ? 0.f : 1.f;     // the carry into step t+1 was zeroed
    dh += keep * dxh[e * LSTM_K + FC + u];
    dcn = keep * dcp[i];
    const int64_t xi = e * FC + u;                 // FC == LSTM_U: x and h share the index
    dx_next[xi] = x_next[xi] > 0.f ? dxh[e * LSTM_K + u] : 0.f;
  }
  const float* gp = G + e * LSTM_G + u;
  const float ig = gp[0], jg = gp[LSTM_U], fg = gp[2 * LSTM_U], og = gp[3 * LSTM_U];
  const float tc = tanhf(C[i]);
  const float dc = dcn + dh * og * (1.f - tc * tc);
  float* da = DA + e * LSTM_G + u;
  da[0] = dc * jg * ig * (1.f - ig);
  da[LSTM_U] = dc * ig * (1.f - jg * jg);
  da[2 * LSTM_U] = dc * CP[i] * fg * (1.f - fg);
  da[3 * LSTM_U] = dh * tc * og * (1.f - og);
  dcp[i] = dc * fg;
}

__global__ void k_lstm_colsum(const float* __restrict__ part, int nsplit, float* __restrict__ db) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= LSTM_G) return;
  float v = 0.f;
  for (int s = 0; s < nsplit; ++s) v += part[(int64_t)s * LSTM_G + j];
  db[j] = v;
}

struct LstmWs {
  int64_t da, dxh, dcp, slab, col, total;
  int split_dx, split_dw;
};

static LstmWs lstm_ws(int n, int64_t E) {
  LstmWs w;
  const int64_t nE = (int64_t)n * E;
  w.split_dx = a3c_gemm_effective_split(LSTM_G, a3c_gemm_plan_split((int)E, LSTM_K, LSTM_G, 256));
  w.split_dw = a3c_gemm_effective_split((int)nE, a3c_gemm_plan_split(FC, LSTM_G, (int)nE, 256));
  int64_t o = 0;
  auto take = [&](int64_t floats) { int64_t r = o; o += (floats + 63) & ~(int64_t)63; return r; };
  w.da = take(nE * LSTM_G);
  w.dxh = take(E * LSTM_K);
  w.dcp = take(E * LSTM_U);
  const int64_t s1 = w.split_dx > 1 ? (int64_t)w.split_dx * E * LSTM_K : 0;
  const int64_t s2 = w.split_dw > 1 ? (int64_t)w.split_dw * FC * LSTM_G : 0;
  w.slab = take(s1 > s2 ? s1 : s2);
  w.col = take((int64_t)w.split_dw * LSTM_G);
  w.total = o;
  return w;
}

int64_t a3c_lstm_ws_floats(int n, int64_t E) { return lstm_ws(n, E).total; }

int a3c_lstm_bptt_launch(const float* W, int n, int64_t E, const LstmSeq& q, const float* dh, float* dx,
                         float* dw, float* db, float* ws, hipStream_t s) {
  if (n < 1 || E < 1 || E > 0x7fffffff / 8) return a3c_set_error(A3C_ERR_INVALID, "a3c_lstm_bptt", "bad shape");
  const LstmWs w = lstm_ws(n, E);
  float* DA = ws + w.da;
  float* dxh = ws + w.dxh;
  float* dcp = ws + w.dcp;
  const int64_t EU = E * LSTM_U;
  const unsigned nb = (unsigned)((EU + 255) / 256);
  for (int t = n - 1; t >= 0; --t) {
    const int64_t ot = (int64_t)t * E;
    const bool nx = t < n - 1;
    hipLaunchKernelGGL(k_lstm_cell_bwd, dim3(nb), dim3(256), 0, s, E, nx ? 1 : 0, q.gates + ot * LSTM_G,
                       q.c + ot * LSTM_U, q.cp + ot * LSTM_U, dh + ot * LSTM_U, q.terms + ot, dxh, dcp,
                       nx ? q.x + (ot + E) * FC : nullptr, nx ? dx + (ot + E) * FC : nullptr,
                       DA + ot * LSTM_G);
    A3C_CHECK(hipGetLastError());
    // d[x, hp]_t = da_t W^T   (B(k = gate col, n = row of W) = W[n][k])
    GemmArgs g = {};
    g.A = DA + ot * LSTM_G; g.lda = LSTM_G;
    g.B = W; g.ldb = LSTM_G;
    g.M = (int)E; g.K = LSTM_G;
    g.slab = ws + w.slab; g.nsplit = w.split_dx;
    if (t > 0) {
      g.C = dxh; g.ldc = LSTM_K; g.N = LSTM_K; g.epi = EPI_STORE;
    } else {   // step 0: only dx (truncated BPTT), masked by the fc ReLU straight into dx[0]
      g.C = dx; g.ldc = FC; g.N = FC; g.epi = EPI_MASK; g.mask = q.x; g.ldm = FC;
    }
    int rc = a3c_gemm(true, false, g, s);
    if (rc) return rc;
  }
  // dW[0:256] = x^T da (+ colsum -> db), dW[256:512] = hp^T da over all n*E rows
  const int64_t nE = (int64_t)n * E;
  for (int part = 0; part < 2; ++part) {
    GemmArgs g = {};
    g.A = part == 0 ? q.x : q.hp; g.lda = part == 0 ? FC : LSTM_U;   // A(m = feature, k = b)
    g.B = DA; g.ldb = LSTM_G;
    g.C = dw + (int64_t)part * FC * LSTM_G; g.ldc = LSTM_G;
    g.M = part == 0 ? FC : LSTM_U; g.N = LSTM_G; g.K = (int)nE;
    g.epi = EPI_STORE; g.slab = ws + w.slab; g.nsplit = w.split_dw;
    g.colsum = part == 0 ? ws + w.col : nullptr;
    int rc = a3c_gemm(false, true, g, s);
    if (rc) return rc;
  }
  hipLaunchKernelGGL(k_lstm_colsum, dim3((LSTM_G + 255) / 256), dim3(256), 0, s, ws + w.col, w.split_dw, db);
  A3C_CHECK(hipGetLastError());
  return 0;
}

// ---- C-ABI ------------------------------------------------------------------------------
extern "C" int a3c_lstm_step(const float* w, const float* b, const float* x, const float* h_src,
                             const float* c_src, const uint8_t* prev_terms, int64_t B, float* hp, float* cp,
                             float* gates, float* h, float* c, void* stream) {
  if (B < 0) return a3c_set_error(A3C_ERR_INVALID, "a3c_lstm_step", "B < 0");
  LstmStep st = {h_src, c_src, prev_terms, hp, cp, gates, h, c};
  return a3c_lstm_fwd_launch(w, b, x, st, B, (hipStream_t)stream);
}

extern "C" int a3c_lstm_workspace_bytes(int n, int64_t E, int64_t* bytes) {
  if (n < 1 || E < 1 || !bytes) return a3c_set_error(A3C_ERR_INVALID, "a3c_lstm_workspace_bytes", "bad argument");
  *bytes = a3c_lstm_ws_floats(n, E) * (int64_t)sizeof(float) + 256;
  return 0;
}

extern "C" int a3c_lstm_bptt(const float* w, int n, int64_t E, const float* x, const float* hp, const float* cp,
                             const float* gates, const float* c, const uint8_t* terms, const float* dh, float* dx,
                             float* dw, float* db, void* workspace, void* stream) {
  if (!w || !x || !hp || !cp || !gates || !c || !terms || !dh || !dx || !dw || !db || !workspace)
    return a3c_set_error(A3C_ERR_INVALID, "a3c_lstm_bptt", "null argument");
  float* ws = (float*)(((uintptr_t)workspace + 255) & ~(uintptr_t)255);
  LstmSeq q = {x, hp, cp, gates, c, terms};
  return a3c_lstm_bptt_launch(w, n, E, q, dh, dx, dw, db, ws, (hipStream_t)stream);
}

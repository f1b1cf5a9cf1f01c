// C5 LSTM policy head for gfx950 (BASELINE config 5; build-defined, the reference has no
// recurrent code).  TF1 BasicLSTMCell semantics, oracle/ref_cpu.py lstm_cell / lstm_*_seq:
//   a = [x, h_prev] @ W + b  (W [512][1024], gate columns i, j, f, o)
//   c = c_prev * sigmoid(f + 1) + sigmoid(i) * tanh(j);  h = tanh(c) * sigmoid(o)
// with the carried state zeroed after a terminal transition.
//
//  k_lstm_fwd        one workgroup per (16 envs x 16 units), 8 waves = 4 gates x 2 K halves
//                    (x / h_prev) on v_mfma_f32_16x16x4_f32 with k-permuted 16-byte operand loads
//                    (W pre-transposed once per parameter version, k_lstm_transpose); the gate
//                    tiles meet in LDS and the cell update is fused into the epilogue.
//  k_lstm_bptt_step  d[x, hp]_{t+1} = da_{t+1} W^T, fused with dx_{t+1} (fc ReLU mask) and the
//                    cell backward of step t, which is elementwise once dh_t is complete: one
//                    launch per step.
//  dW GEMMs          dW = [x, hp]^T da over all n*E rows (+ colsum -> db) on gemm.hip.
#include "lstm.h"
#include "gemm.h"

#define LT 16                    // envs per workgroup tile

__device__ inline float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

// Wt[c][k] = W[k][c]: W [512][1024] -> Wt [1024][512]; 32x32 tiles through LDS
__global__ void __launch_bounds__(256) k_lstm_transpose(const float* __restrict__ W, float* __restrict__ Wt) {
  __shared__ float tile[32][33];
  const int c0 = blockIdx.x * 32, k0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int r = ty; r < 32; r += 8) tile[r][tx] = W[(int64_t)(k0 + r) * LSTM_G + c0 + tx];
  __syncthreads();
  for (int r = ty; r < 32; r += 8) Wt[(int64_t)(c0 + r) * LSTM_K + k0 + tx] = tile[tx][r];
}

int a3c_lstm_transpose_launch(const float* W, float* Wt, hipStream_t s) {
  hipLaunchKernelGGL(k_lstm_transpose, dim3(LSTM_G / 32, LSTM_K / 32), dim3(256), 0, s, W, Wt);
  A3C_CHECK(hipGetLastError());
  return 0;
}

// k-permuted fp32 MFMA step: in 16x16x4 step s of a 16-wide k block kb, lane (i16, j4) supplies
// A[row i16][kb + 4 j4 + s] and B[kb + 4 j4 + s][col i16] -- every k of the block exactly once,
// and each lane's four k are contiguous in memory for row-major A and for B given as B^T rows,
// so both operands arrive as one 16-byte load per lane per four MFMAs.
__device__ inline f32x4 mfma_k16(const f32x4 a, const f32x4 b, f32x4 c) {
#pragma unroll
  for (int s = 0; s < 4; ++s) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[s], c, 0, 0, 0);
  return c;
}

// cell step: workgroup = 16 envs x 16 units x 4 gates, 8 waves = (gate g, K half kh): kh 0 runs
// x @ W[0:256], kh 1 runs h_prev @ W[256:512] (rows of terminal-masked envs zeroed afterwards:
// (keep h) W = keep (h W)).  The tile's 16 rows of [x, h_prev] (32 KB) are staged in LDS once and
// shared by the 4 gate waves of each half (each wave loaded them itself before round 5: 4x the
// operand traffic); with st.fc_part the x rows are folded there from the fc's K-slice partials
// (slice order + bias + ReLU, the feed-forward head's fold) and written to st.l3_out by the
// workgroups of unit tile 0, so the fc needs no separate finishing pass.  The W rows of the
// wave's 16 units (16 KB) go straight to registers, issued first.
#define LSTM_LD (FC + 4)            // LDS row of the [x, h] tile: 260 floats (row r starts 4 r banks on)
__global__ void __launch_bounds__(512) k_lstm_fwd(const float* __restrict__ X, const float* __restrict__ bias,
                                                  LstmStep st, int64_t B) {
  __shared__ __attribute__((aligned(16))) float As[2][LT][LSTM_LD];
  __shared__ float Gs[2][4][LT][LT + 1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = w & 3, kh = w >> 2, i16 = lane & 15, j4 = lane >> 4;
  const int64_t e0 = (int64_t)blockIdx.x * LT;
  const int u0 = blockIdx.y * LT;
  const float* pw = st.wt + (int64_t)(g * LSTM_U + u0 + i16) * LSTM_K + kh * FC + 4 * j4;
  f32x4 b[FC / 16];
#pragma unroll
  for (int it = 0; it < FC / 16; ++it) b[it] = *(const f32x4*)(pw + 16 * it);
  // stage [x, h_prev] of the tile's 16 envs: 2 x 16 x 64 chunks of 4 floats, 4 per thread
  // (chunks 0..1023 the x half: thread tid's q = 0, 1; 1024..2047 the h half: q = 2, 3)
  constexpr int NCH = 2 * LT * (FC / 4);
  static_assert(NCH == 4 * 512 && LSTM_U == FC, "tile staging");
  f32x4 xin[2], hin[2];
  if (st.fc_part) {
    f32x4 p[2][FC_NS];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int c = tid + 512 * q, row = c >> 6, c4 = c & 63;
      const int64_t e = min(e0 + row, B - 1);
#pragma unroll
      for (int x = 0; x < FC_NS; ++x) p[q][x] = *(const f32x4*)(st.fc_part + ((int64_t)x * B + e) * FC + 4 * c4);
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int c = tid + 512 * q, row = c >> 6, c4 = c & 63;
      const int64_t e = min(e0 + row, B - 1);
      hin[q] = *(const f32x4*)(st.h_src + e * FC + 4 * c4);
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int c = tid + 512 * q, row = c >> 6, c4 = c & 63;
      const f32x4 fb = *(const f32x4*)(st.fc_bias + 4 * c4);
      f32x4 v = p[q][0];
#pragma unroll
      for (int x = 1; x < FC_NS; ++x) v += p[q][x];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r] + fb[r], 0.f);
      xin[q] = v;
      if (blockIdx.y == 0 && e0 + row < B) *(f32x4*)(st.l3_out + (e0 + row) * FC + 4 * c4) = v;
    }
  } else {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int c = tid + 512 * q, row = c >> 6, c4 = c & 63;
      const int64_t e = min(e0 + row, B - 1);
      xin[q] = *(const f32x4*)(X + e * FC + 4 * c4);
      hin[q] = *(const f32x4*)(st.h_src + e * FC + 4 * c4);
    }
  }
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int c = tid + 512 * q, row = c >> 6, c4 = c & 63;
    *(f32x4*)&As[0][row][4 * c4] = xin[q];
    *(f32x4*)&As[1][row][4 * c4] = hin[q];
  }
  __syncthreads();
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  const float* ar = &As[kh][i16][4 * j4];
#pragma unroll
  for (int it = 0; it < FC / 16; it += 2) {
    acc0 = mfma_k16(*(const f32x4*)(ar + 16 * it), b[it], acc0);
    acc1 = mfma_k16(*(const f32x4*)(ar + 16 * it + 16), b[it + 1], acc1);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float v = acc0[r] + acc1[r];
    if (kh) {
      const int64_t e = e0 + 4 * j4 + r;
      if (e >= B || (st.prev_terms && st.prev_terms[e])) v = 0.f;
    }
    Gs[kh][g][4 * j4 + r][i16] = v;
  }
  __syncthreads();
  if (tid >= LT * LT) return;
  // cell update of (env r, unit c)
  const int r = tid >> 4, c = tid & 15;
  const int64_t e = e0 + r;
  if (e >= B) return;
  const int u = u0 + c;
  const int64_t o = e * LSTM_U + u;
  const bool keep = !(st.prev_terms && st.prev_terms[e]);
  const float cprev = keep ? st.c_src[o] : 0.f;
  float pre[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) pre[q] = Gs[0][q][r][c] + Gs[1][q][r][c] + bias[q * LSTM_U + u];
  const float ig = sigmoidf_(pre[0]);
  const float jg = tanhf(pre[1]);
  const float fg = sigmoidf_(pre[2] + 1.0f);     // forget_bias = 1.0
  const float og = sigmoidf_(pre[3]);
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

int a3c_lstm_fwd_launch(const float* bias, const float* x, const LstmStep& st, int64_t B, hipStream_t s) {
  if (B <= 0) return 0;
  if (!st.wt || !bias || !st.h_src || !st.c_src || !st.h || !st.c || (!x && !st.fc_part) ||
      (st.fc_part && (!st.fc_bias || !st.l3_out)) ||
      (((uintptr_t)x | (uintptr_t)st.h_src | (uintptr_t)st.wt | (uintptr_t)st.fc_part) & 15))
    return a3c_set_error(A3C_ERR_INVALID, "a3c_lstm_step", "bad argument");
  hipLaunchKernelGGL(k_lstm_fwd, dim3((unsigned)((B + LT - 1) / LT), LSTM_U / LT), dim3(512), 0, s, x, bias, st, B);
  A3C_CHECK(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------------------------------
// cell backward of step t at (e, u) given dh (heads + recurrence) and the carried dc
__device__ inline void lstm_cell_bwd(int64_t e, int u, float dh, float dcn, const float* __restrict__ G,
                                     const float* __restrict__ C, const float* __restrict__ CP,
                                     float* __restrict__ dcp, float* __restrict__ DA) {
  const int64_t i = e * LSTM_U + u;
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

// last step (t = n-1): nothing flows in from the future
__global__ void __launch_bounds__(256) k_lstm_cell_bwd_last(int64_t E, const float* __restrict__ G,
                                                            const float* __restrict__ C, const float* __restrict__ CP,
                                                            const float* __restrict__ dH, float* __restrict__ dcp,
                                                            float* __restrict__ DA) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= E * LSTM_U) return;
  const int64_t e = i / LSTM_U;
  lstm_cell_bwd(e, (int)(i - e * LSTM_U), dH[i], 0.f, G, C, CP, dcp, DA);
}

struct BpttStep {
  const float* DAn;       // da of step t+1 [E][1024]
  const float* xn;        // x of step t+1 [E][256] (fc ReLU output: the dx mask)
  float* dxn;             // dx of step t+1 [E][256]
  int cell;               // 1: run the cell backward of step t in the h-half epilogue
  const float *G, *C, *CP, *dH;   // step t
  const uint8_t* terms;   // terms[t] [E]
  float* dcp;             // [E][U] carried dc (in: step t+1's dc*f, out: step t's)
  float* DA;              // da of step t [E][1024]
};

// d[x, hp]_{t+1} = da_{t+1} W^T for a tile of 16 envs x 32 of the 512 columns, 8 waves = (16-col
// half ct, K quarter kq); the epilogue writes dx_{t+1} (x half, fc ReLU mask) or, for the hp half,
// runs the cell backward of step t on the finished dh (elementwise in (e, u)).
__global__ void __launch_bounds__(512) k_lstm_bptt_step(int64_t E, const float* __restrict__ W, BpttStep q) {
  __shared__ float Ps[4][2][LT][LT + 1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int ct = w & 1, kq = w >> 1, i16 = lane & 15, j4 = lane >> 4;
  const int64_t e0 = (int64_t)blockIdx.x * LT;
  const int n0 = blockIdx.y * 32;
  const int64_t er = min(e0 + i16, E - 1);
  constexpr int KQ = LSTM_G / 4;                 // 256
  const float* pa = q.DAn + er * LSTM_G + kq * KQ + 4 * j4;
  const float* pb = W + (int64_t)(n0 + 16 * ct + i16) * LSTM_G + kq * KQ + 4 * j4;   // B^T rows = W rows
  f32x4 a[KQ / 16], b[KQ / 16];
#pragma unroll
  for (int it = 0; it < KQ / 16; ++it) {
    a[it] = *(const f32x4*)(pa + 16 * it);
    b[it] = *(const f32x4*)(pb + 16 * it);
  }
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int it = 0; it < KQ / 16; it += 2) {
    acc0 = mfma_k16(a[it], b[it], acc0);
    acc1 = mfma_k16(a[it + 1], b[it + 1], acc1);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) Ps[kq][ct][4 * j4 + r][i16] = acc0[r] + acc1[r];
  __syncthreads();
  const int r = tid >> 5, c = tid & 31;
  const int64_t e = e0 + r;
  if (e >= E) return;
  const float v = (Ps[0][c >> 4][r][c & 15] + Ps[1][c >> 4][r][c & 15]) +
                  (Ps[2][c >> 4][r][c & 15] + Ps[3][c >> 4][r][c & 15]);
  const int col = n0 + c;
  if (col < FC) {
    const int64_t xi = e * FC + col;
    q.dxn[xi] = q.xn[xi] > 0.f ? v : 0.f;
  } else if (q.cell) {
    const int u = col - FC;
    const float keep = q.terms[e] ? 0.f : 1.f;     // the carry into step t+1 was zeroed
    const int64_t i = e * LSTM_U + u;
    lstm_cell_bwd(e, u, q.dH[i] + keep * v, keep * q.dcp[i], q.G, q.C, q.CP, q.dcp, q.DA);
  }
}

__global__ void k_lstm_colsum(const float* __restrict__ part, int nsplit, float* __restrict__ db) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= LSTM_G) return;
  float v = 0.f;
  for (int s = 0; s < nsplit; ++s) v += part[(int64_t)s * LSTM_G + j];
  db[j] = v;
}

struct LstmWs {
  int64_t da, dcp, slab, col, total;
  int split_dw;
};

static LstmWs lstm_ws(int n, int64_t E) {
  LstmWs w;
  const int64_t nE = (int64_t)n * E;
  w.split_dw = a3c_gemm_effective_split((int)nE, a3c_gemm_plan_split(FC, LSTM_G, (int)nE, 256));
  int64_t o = 0;
  auto take = [&](int64_t floats) { int64_t r = o; o += (floats + 63) & ~(int64_t)63; return r; };
  w.da = take(nE * LSTM_G);
  w.dcp = take(E * LSTM_U);
  w.slab = take(w.split_dw > 1 ? (int64_t)w.split_dw * FC * LSTM_G : 0);
  w.col = take((int64_t)w.split_dw * LSTM_G);
  w.total = o;
  return w;
}

int64_t a3c_lstm_ws_floats(int n, int64_t E) { return lstm_ws(n, E).total; }

// truncated BPTT: cell backward of step n-1, then per step one fused launch (d[x, hp]_{t+1} GEMM
// + dx_{t+1} + cell backward of step t), then dx_0, then the gate-matrix gradients over n*E rows
int a3c_lstm_bptt_launch(const float* W, int n, int64_t E, const LstmSeq& q, const float* dh, float* dx,
                         float* dw, float* db, float* ws, hipStream_t s) {
  if (n < 1 || E < 1 || E > 0x7fffffff / 8) return a3c_set_error(A3C_ERR_INVALID, "a3c_lstm_bptt", "bad shape");
  const LstmWs w = lstm_ws(n, E);
  float* DA = ws + w.da;
  float* dcp = ws + w.dcp;
  const int64_t EU = E * LSTM_U;
  const int64_t last = (int64_t)(n - 1) * E;
  hipLaunchKernelGGL(k_lstm_cell_bwd_last, dim3((unsigned)((EU + 255) / 256)), dim3(256), 0, s, E,
                     q.gates + last * LSTM_G, q.c + last * LSTM_U, q.cp + last * LSTM_U, dh + last * LSTM_U, dcp,
                     DA + last * LSTM_G);
  A3C_CHECK(hipGetLastError());
  const unsigned etiles = (unsigned)((E + LT - 1) / LT);
  for (int t = n - 2; t >= -1; --t) {
    const int64_t on = (int64_t)(t + 1) * E, ot = (int64_t)(t < 0 ? 0 : t) * E;
    BpttStep b = {};
    b.DAn = DA + on * LSTM_G;
    b.xn = q.x + on * FC;
    b.dxn = dx + on * FC;
    b.cell = t >= 0;
    b.G = q.gates + ot * LSTM_G; b.C = q.c + ot * LSTM_U; b.CP = q.cp + ot * LSTM_U; b.dH = dh + ot * LSTM_U;
    b.terms = q.terms + ot;
    b.dcp = dcp;
    b.DA = DA + ot * LSTM_G;
    // t = -1: dx_0 only (x half of the columns)
    hipLaunchKernelGGL(k_lstm_bptt_step, dim3(etiles, (t >= 0 ? LSTM_K : FC) / 32), dim3(512), 0, s, E, W, b);
    A3C_CHECK(hipGetLastError());
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
extern "C" int a3c_lstm_transpose(const float* w, float* w_t, void* stream) {
  if (!w || !w_t) return a3c_set_error(A3C_ERR_INVALID, "a3c_lstm_transpose", "null");
  return a3c_lstm_transpose_launch(w, w_t, (hipStream_t)stream);
}

extern "C" int a3c_lstm_step(const float* w_t, const float* b, const float* x, const float* h_src,
                             const float* c_src, const uint8_t* prev_terms, int64_t B, float* hp, float* cp,
                             float* gates, float* h, float* c, void* stream) {
  if (B < 0) return a3c_set_error(A3C_ERR_INVALID, "a3c_lstm_step", "B < 0");
  LstmStep st = {w_t, h_src, c_src, prev_terms, hp, cp, gates, h, c};
  return a3c_lstm_fwd_launch(b, x, st, B, (hipStream_t)stream);
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

// Shared device helpers for the MI355X (gfx950) A3C rollout + gradient path.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define A3C_WAVE 64

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#define A3C_CHECK(expr)                                                       \
  do {                                                                        \
    hipError_t _e = (expr);                                                   \
    if (_e != hipSuccess) return a3c_set_error((int)_e, #expr, hipGetErrorString(_e)); \
  } while (0)

// Error reporting (defined in capi.cpp).
extern "C" int a3c_set_error(int code, const char* what, const char* detail);

// Environment switches.  A release build reads only the documented, tested ones (A3C_KNOB:
// A3C_WAIT_VALUE, A3C_L2BITS, A3C_FC_SPLIT, A3C_FUSE_CONV, A3C_FUSED_SCREEN, A3C_SPANS, A3C_LSTM_FCFOLD; bench.py
// records every A3C_* variable that is set).  The A/B knobs of measured-and-rejected variants
// (A3C_AB_KNOB) compile to their defaults unless the library is built with -DA3C_KNOBS
// (tools/build_variant.sh), so a stray variable cannot change a release run's summation order.
#include <cstdlib>
inline long long a3c_env_ll(const char* name, long long dflt) {
  const char* v = getenv(name);
  return v ? atoll(v) : dflt;
}
#define A3C_KNOB(name, dflt) a3c_env_ll(name, dflt)
#ifdef A3C_KNOBS
#define A3C_AB_KNOB(name, dflt) a3c_env_ll(name, dflt)
#else
#define A3C_AB_KNOB(name, dflt) ((void)(name), (long long)(dflt))
#endif

// ---------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al. 2011) -- bit-identical to oracle/philox.py.
// ---------------------------------------------------------------------------
enum : uint32_t { P_ACTION = 1u, P_STEP = 3u, P_RESET = 6u, P_NOOP = 7u, P_POOL = 9u };

struct u32x4 { uint32_t x, y, z, w; };

__host__ __device__ inline u32x4 philox4x32(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                            uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return {c0, c1, c2, c3};
}

// top 24 bits * 2^-24 : exact in fp32, identical to oracle philox.u01
__host__ __device__ inline float u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }

// ---------------------------------------------------------------------------
// wave reductions (64 lanes)
// ---------------------------------------------------------------------------
__device__ inline float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ inline float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ inline double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---------------------------------------------------------------------------
// Addressing of stacked frame states.
//
// Frames (84x84 u8 planes) live in a per-env ring of R slots; the state s_tau of env e is
// the L planes of frames tau-L+1 .. tau (oldest first == history.py:13-15 order, channel c
// of the NHWC view history.py:20-22).  A contiguous [B][L][H][W] tensor is the special case
// R = L, E = B, tau = L-1.
// sample b -> (t = b / E, e = b % E); frame tau = (*tau_ptr) + t + tau_offset.
// ---------------------------------------------------------------------------
struct StateAddr {
  const uint8_t* base;   // ring base
  int64_t env_stride;    // bytes between envs
  int64_t plane_bytes;   // bytes per plane (H*W)
  int E;                 // envs per rollout step
  int R;                 // ring slots
  int L;                 // history length
  int tau_offset;        // added to tau (+1 for next states)
  const int64_t* tau_ptr;  // device counter (nullable -> 0)
  // launch-span record (engine measurement, a3c_engine_span_stats): a kernel reading these
  // states stores its workgroups' start and end s_memrealtime stamps (plain stores, one slot per
  // workgroup: no same-address atomics) into launch record (tau + tau_offset) / span_div % SPAN_RECS
  unsigned long long* span = nullptr;
  int span_div = 1;
};
#define SPAN_RECS 1024
#define SPAN_WGS 512              // workgroup slots per launch record
__device__ inline unsigned long long* span_rec(const StateAddr& a, int64_t tau0) {
  if (!a.span || blockIdx.x >= SPAN_WGS) return nullptr;
  return a.span + 2 * ((((tau0 + a.tau_offset) / a.span_div) % SPAN_RECS) * SPAN_WGS + blockIdx.x);
}
// the workgroup's start stamp (thread 0, at its start)
__device__ inline void span_begin(unsigned long long* r) {
  if (r && threadIdx.x == 0) r[0] = (unsigned long long)__builtin_amdgcn_s_memrealtime();
}
// its end stamp (after a workgroup barrier, once all of the workgroup's work is issued)
__device__ inline void span_end(unsigned long long* r) {
  if (!r) return;
  __syncthreads();
  if (threadIdx.x == 0) r[1] = (unsigned long long)__builtin_amdgcn_s_memrealtime();
}

__device__ inline const uint8_t* state_plane(const StateAddr& a, int64_t b, int c, int64_t tau0) {
  int64_t t = b / a.E, e = b - t * a.E;
  int64_t tau = tau0 + t + a.tau_offset - (a.L - 1) + c;
  int64_t slot = tau % a.R;
  if (slot < 0) slot += a.R;
  return a.base + e * a.env_stride + slot * a.plane_bytes;
}

// Debug builds only (-DA3C_WG_TIMES, tools/wg_times.py): every workgroup writes its start and
// end s_memrealtime stamps (100 MHz, one clock for the whole chip) as two u64 at `dst`, a
// location of the kernel's own output that the caller then reads back -- the dispatch skew and
// the per-workgroup duration of one launch.
#ifdef A3C_WG_TIMES
#define WG_T0() const uint64_t wg_t0_ = __builtin_amdgcn_s_memrealtime()
#define WG_T1(dst)                                                    \
  do {                                                                \
    __syncthreads();                                                  \
    if (threadIdx.x == 0) {                                           \
      ((uint64_t*)(dst))[0] = wg_t0_;                                 \
      ((uint64_t*)(dst))[1] = __builtin_amdgcn_s_memrealtime();       \
    }                                                                 \
  } while (0)
#else
#define WG_T0() ((void)0)
#define WG_T1(dst) ((void)0)
#endif

// Debug builds only (-DA3C_WGLOG, tools/wglog.py): every workgroup of the instrumented kernels
// appends (start, end, kind | xcc | workgroup | HW_ID) to a device log, so which workgroups shared
// a CU, and when, can be read back (a3c_debug_wglog).  Thread 0 logs at its own exit.
#ifdef A3C_WGLOG
// no atomics (a single log counter serialised the chip): workgroup b of kind k keeps its own
// launch counter cnt[k][b] (launches of one kernel are ordered on their stream, and kernel
// boundaries make the previous launch's store visible) and writes slot e[k][b][cnt % WGL_RING]
#define WGL_KINDS 16
#define WGL_MAXWG 4096
#define WGL_RING 16
struct WglBuf {
  unsigned int on, pad[3];
  unsigned int cnt[WGL_KINDS][WGL_MAXWG];
  unsigned long long e[WGL_KINDS][WGL_MAXWG][WGL_RING][3];   // start, end, xcc << 32 | HW_ID
};
static __device__ WglBuf* g_wgl;   // one per translation unit, bound by its a3c_wglog_bind_* hook
struct WgLog {
  unsigned long long t0;
  unsigned kind, c;
  WglBuf* b;
  __device__ explicit WgLog(unsigned k) : t0(__builtin_amdgcn_s_memrealtime()), kind(k), c(0), b(nullptr) {
    WglBuf* g = g_wgl;
    if (threadIdx.x == 0 && g && g->on && blockIdx.x < WGL_MAXWG) {
      b = g;
      c = g->cnt[k][blockIdx.x];   // (used at the end: the load retires meanwhile)
    }
  }
  __device__ ~WgLog() {
    if (!b) return;
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    unsigned long long* e = b->e[kind][blockIdx.x][c % WGL_RING];
    e[0] = t0;
    e[1] = __builtin_amdgcn_s_memrealtime();
    e[2] = ((unsigned long long)(xcc & 15) << 32) | hw;
    b->cnt[kind][blockIdx.x] = c + 1;
  }
};
#define WGLOG(kind) WgLog wgl_(kind)
#define WGLOG_BIND(name) \
  void name(WglBuf* p) { (void)hipMemcpyToSymbol(HIP_SYMBOL(g_wgl), &p, sizeof(p)); }
#else
#define WGLOG(kind) ((void)0)
#endif

// Stores of activations that the next kernel reads on other XCDs (l1, l2, l3, the frame ring):
// non-temporal with A3C_NT_STORE (bypass the writing XCD's L2, so the end-of-kernel release has
// fewer dirty lines to write back) -- an A/B switch.
template <typename T>
__device__ inline void st_act(T* p, T v) {
#ifdef A3C_NT_STORE
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}

// one 16-byte-per-lane global -> LDS DMA wave-instruction: lane l's 16 bytes land at
// lds_base + 16 l (lds_base wave-uniform), no VGPR destination
__device__ inline void glds16(const void* g, void* lds_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

// sum_{s < n} p[s * stride], accumulated in s order (bit-identical to the plain loop) with 8 loads in
// flight: the deterministic slab folds would otherwise wait one full load latency per term
__device__ inline float sum_strided(const float* __restrict__ p, int n, int64_t stride) {
  float v = 0.f;
  int s = 0;
  for (; s + 8 <= n; s += 8) {
    float t[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) t[j] = p[(int64_t)(s + j) * stride];
#pragma unroll
    for (int j = 0; j < 8; ++j) v += t[j];
  }
  for (; s < n; ++s) v += p[(int64_t)s * stride];
  return v;
}

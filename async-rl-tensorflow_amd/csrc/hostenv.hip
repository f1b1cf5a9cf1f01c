// Host-side batched synthetic Atari env (a3c_hostenv_*): the same emulator as the device env
// (env_dev.h, bit-identical dynamics) stepped by CPU threads, writing RAW RGB frames into a
// caller (pinned) host buffer -- the stand-in for real ALE worker processes feeding the
// external-env engine (a3c_engine_ext_*) when measuring the PCIe-inclusive host
// path.  Semantics: new_random_game environment.py:35-40, act :78-96 with life-loss terminal,
// new_random_game after a terminal (agent.py:66-67).  Host code only; no GPU work.
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <new>
#include <thread>
#include <vector>
#include "env_dev.h"

// Persistent workers: a step is 16-64 us of work per thread, so spawning and joining threads
// per call (tens of us each) would dominate it.  The caller runs slice 0 itself.
struct WorkerPool {
  int T = 1;
  std::vector<std::thread> th;
  std::mutex m;
  std::condition_variable go, done;
  uint64_t gen = 0;
  int pending = 0;
  bool quit = false;
  std::function<void(int, int)> job;
  int lo = 0, hi = 0;

  void start(int threads) {
    T = threads < 1 ? 1 : threads;
    for (int t = 1; t < T; ++t) th.emplace_back([this, t]() { loop(t); });
  }
  void slice(int t, int& a, int& b) const {
    const int64_t n = hi - lo;
    a = lo + (int)(n * t / T);
    b = lo + (int)(n * (t + 1) / T);
  }
  void loop(int t) {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(m);
        go.wait(lk, [&] { return quit || gen != seen; });
        if (quit) return;
        seen = gen;
      }
      int a, b;
      slice(t, a, b);
      if (a < b) job(a, b);
      std::lock_guard<std::mutex> lk(m);
      if (--pending == 0) done.notify_one();
    }
  }
  void run(int a0, int b0, std::function<void(int, int)> f) {
    if (T <= 1 || b0 - a0 < 2) {
      if (a0 < b0) f(a0, b0);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(m);
      job = std::move(f);
      lo = a0;
      hi = b0;
      pending = T - 1;
      ++gen;
    }
    go.notify_all();
    int a, b;
    slice(0, a, b);
    if (a < b) job(a, b);
    std::unique_lock<std::mutex> lk(m);
    done.wait(lk, [&] { return pending == 0; });
  }
  ~WorkerPool() {
    {
      std::lock_guard<std::mutex> lk(m);
      quit = true;
    }
    go.notify_all();
    for (auto& x : th) x.join();
  }
};

struct a3c_hostenv {
  int E, threads;
  EnvParams p;
  std::vector<EnvState> st;
  std::vector<uint8_t> pool;      // [P][210][160][3] host frame pool (same frames as the device pool)
  WorkerPool workers;
};

static const int64_t FRAME_BYTES = (int64_t)SCREEN_H * SCREEN_W * 3;

template <typename F>
static void parallel_envs(const a3c_hostenv* h, F f) {
  const int T = h->threads < h->E ? h->threads : h->E;
  if (T <= 1) {
    f(0, h->E);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(T);
  for (int t = 0; t < T; ++t) {
    const int lo = (int)((int64_t)h->E * t / T), hi = (int)((int64_t)h->E * (t + 1) / T);
    th.emplace_back([=]() { f(lo, hi); });
  }
  for (auto& x : th) x.join();
}

extern "C" int a3c_hostenv_create(int num_envs, int action_size, int start_lives, int random_start,
                                  int action_repeat, int num_frames, uint64_t seed, int env_id_base, int threads,
                                  a3c_hostenv** out) {
  if (!out || num_envs < 1 || action_size < 1 || random_start < 1 || action_repeat < 1 || num_frames < 1 ||
      threads < 1)
    return a3c_set_error(A3C_ERR_INVALID, "a3c_hostenv_create", "bad argument");
  a3c_hostenv* h = new (std::nothrow) a3c_hostenv();
  if (!h) return a3c_set_error(A3C_ERR_INVALID, "a3c_hostenv_create", "oom");
  h->E = num_envs;
  h->threads = threads;
  h->p.k0 = (uint32_t)seed;
  h->p.k1 = (uint32_t)(seed >> 32);
  h->p.P = num_frames;
  h->p.A = action_size;
  h->p.L0 = start_lives;
  h->p.random_start = random_start;
  h->p.action_repeat = action_repeat;
  h->p.env_id_base = env_id_base;
  h->st.assign(num_envs, EnvState{0u, 0u, 0u, 0, 0, 0.f, 0u});
  try {
    h->pool.resize((size_t)num_frames * FRAME_BYTES);
  } catch (...) {
    delete h;
    return a3c_set_error(A3C_ERR_INVALID, "a3c_hostenv_create", "frame pool allocation failed");
  }
  // frame f, 16-byte chunk j = philox(j, f, P_POOL, 0) (k_pool_fill)
  const int64_t cpf = FRAME_BYTES / 16;
  a3c_hostenv tmp_view;   // thread split over frames
  tmp_view.E = num_frames;
  tmp_view.threads = threads;
  uint8_t* pool = h->pool.data();
  const uint32_t k0 = h->p.k0, k1 = h->p.k1;
  parallel_envs(&tmp_view, [=](int lo, int hi) {
    for (int f = lo; f < hi; ++f)
      for (int64_t j = 0; j < cpf; ++j) {
        u32x4 x = philox4x32((uint32_t)j, (uint32_t)f, P_POOL, 0u, k0, k1);
        uint32_t w[4] = {x.x, x.y, x.z, x.w};
        memcpy(pool + f * FRAME_BYTES + j * 16, w, 16);
      }
  });
  try {
    h->workers.start(threads < num_envs ? threads : num_envs);
  } catch (...) {       // no exception crosses the C ABI
    delete h;
    return a3c_set_error(A3C_ERR_INVALID, "a3c_hostenv_create", "could not start worker threads");
  }
  *out = h;
  return 0;
}

extern "C" int a3c_hostenv_destroy(a3c_hostenv* h) {
  delete h;
  return 0;
}

// new_random_game of every env (agent.py:33-35); first frames -> rgb [E][210][160][3]
extern "C" int a3c_hostenv_begin(a3c_hostenv* h, uint8_t* rgb) {
  if (!h || !rgb) return a3c_set_error(A3C_ERR_INVALID, "a3c_hostenv_begin", "null");
  h->workers.run(0, h->E, [=](int lo, int hi) {
    for (int e = lo; e < hi; ++e) {
      EnvState& s = h->st[e];
      s = EnvState{0u, 0u, 0u, 0, 0, 0.f, 0u};
      env_new_random_game(s, h->p, (uint32_t)(h->p.env_id_base + e));
      memcpy(rgb + (int64_t)e * FRAME_BYTES, h->pool.data() + (int64_t)s.frame * FRAME_BYTES, FRAME_BYTES);
    }
  });
  return 0;
}

// act of envs [env_lo, env_hi) (agent.py:59-62), post-act frames -> rgb, rewards, terminals
// (indexed by env, full-size buffers); then new_random_game where terminal (agent.py:66-67).
// Stepping the envs in ranges lets the caller start the H2D copy of one range while the next
// is being stepped (Engine.iterate_host).
extern "C" int a3c_hostenv_step_range(a3c_hostenv* h, const int32_t* actions, int is_training, uint8_t* rgb,
                                      float* rewards, uint8_t* terminals, int env_lo, int env_hi) {
  if (!h || !actions || !rgb || !rewards || !terminals)
    return a3c_set_error(A3C_ERR_INVALID, "a3c_hostenv_step", "null");
  if (env_lo < 0 || env_hi > h->E || env_lo > env_hi)
    return a3c_set_error(A3C_ERR_INVALID, "a3c_hostenv_step", "env range outside [0, num_envs]");
  h->workers.run(env_lo, env_hi, [=](int lo, int hi) {
    for (int e = lo; e < hi; ++e) {
      EnvState& s = h->st[e];
      const uint32_t id = (uint32_t)(h->p.env_id_base + e);
      env_act(s, h->p, id, (uint32_t)actions[e], is_training != 0);
      memcpy(rgb + (int64_t)e * FRAME_BYTES, h->pool.data() + (int64_t)s.frame * FRAME_BYTES, FRAME_BYTES);
      rewards[e] = s.reward;
      terminals[e] = (uint8_t)s.terminal;
      if (s.terminal) env_new_random_game(s, h->p, id);
    }
  });
  return 0;
}

// act of every env
extern "C" int a3c_hostenv_step(a3c_hostenv* h, const int32_t* actions, int is_training, uint8_t* rgb,
                                float* rewards, uint8_t* terminals) {
  if (!h) return a3c_set_error(A3C_ERR_INVALID, "a3c_hostenv_step", "null");
  return a3c_hostenv_step_range(h, actions, is_training, rgb, rewards, terminals, 0, h->E);
}

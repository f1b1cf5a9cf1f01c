"""Host-stepped environments feeding the engine (real ALE env workers feeding
pinned host RGB buffers).

``AtariEnv`` wraps one emulator behind gym's API (``reset()``, ``step(a)``, ``ale.lives()``,
``action_space.n``) with the reference's Environment / GymEnvironment semantics
(environment.py:28-96) but returns the RAW RGB frame: Environment.screen (environment.py:49-53)
runs on the GPU, inside the engine, instead of on the host.

``HostEnvPool`` steps E such envs and writes their post-act frames, rewards and terminals into
pinned host buffers; ``Engine(external_env=True).iterate_host(pool)`` moves them to the GPU
(a3c_engine_ext_observe) once per rollout step, after the GPU drew the actions
(a3c_engine_ext_act).  gym/ALE is not installed in this image: any object with the same methods
drives it (tests use the synthetic emulator).
"""
import random as _random
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

SCREEN_SHAPE = (210, 160, 3)


class AtariEnv(object):
  """One game with environment.py:14-96 semantics on raw frames (u8 [210,160,3])."""

  def __init__(self, gym_env, action_repeat=1, random_start=30, rng=None, seed=None):
    self.env = gym_env
    self.action_repeat = int(action_repeat)
    self.random_start = int(random_start)
    self.rng = rng if rng is not None else _random     # environment.py:37 uses module `random`
    # emulator seed: gym < 0.26 has env.seed(s); newer gym seeds through the first reset(seed=s)
    self._reset_seed = None
    if seed is not None:
      if callable(getattr(gym_env, 'seed', None)):
        gym_env.seed(int(seed))
      else:
        self._reset_seed = int(seed)
    self._screen = None
    self.reward = 0
    self.terminal = True

  @property
  def lives(self):                                     # environment.py:59-61
    ale = getattr(self.env, 'ale', None) or getattr(getattr(self.env, 'unwrapped', None), 'ale', None)
    return int(ale.lives())

  @property
  def action_size(self):                               # environment.py:55-57
    return int(self.env.action_space.n)

  def _step(self, action):                             # environment.py:42-43
    out = self.env.step(action)
    if len(out) == 5:                                  # gym >= 0.26: terminated, truncated
      obs, r, term, trunc, _ = out
      term = term or trunc
    else:
      obs, r, term, _ = out
    self._screen, self.reward, self.terminal = obs, r, bool(term)

  def new_game(self, from_random_game=False):          # environment.py:28-33
    if self.lives == 0:
      if self._reset_seed is not None:
        out = self.env.reset(seed=self._reset_seed)
        self._reset_seed = None
      else:
        out = self.env.reset()
      self._screen = out[0] if isinstance(out, tuple) else out
    self._step(0)
    return self._screen, 0, 0, self.terminal

  def new_random_game(self):                           # environment.py:35-40
    self.new_game(True)
    for _ in range(self.rng.randint(0, self.random_start - 1)):
      self._step(0)
    return self._screen, 0, 0, self.terminal

  def act(self, action, is_training=True):             # environment.py:78-96
    cumulated_reward = 0
    start_lives = self.lives
    for _ in range(self.action_repeat):
      self._step(action)
      cumulated_reward = cumulated_reward + self.reward
      if is_training and start_lives > self.lives:
        cumulated_reward -= 1
        self.terminal = True
      if self.terminal:
        break
    self.reward = cumulated_reward
    return self._screen, self.reward, self.terminal


class HostEnvPool(object):
  """E host envs (objects with ``new_random_game()`` -> (rgb, ...) and ``act(a, is_training)`` ->
  (rgb, reward, terminal)) writing into pinned buffers: rgb [E,210,160,3] u8, rewards [E] f32,
  terminals [E] u8.  ``threads`` > 1 steps env chunks concurrently (emulators that release the
  GIL, like ALE's C++ core, then run in parallel)."""

  def __init__(self, envs, threads=1, is_training=True):
    self.envs = list(envs)
    self.E = len(self.envs)
    if self.E < 1:
      raise ValueError('HostEnvPool needs at least one env')
    pin = torch.cuda.is_available()
    mk = lambda shape, dt: torch.zeros(shape, dtype=dt).pin_memory() if pin else torch.zeros(shape, dtype=dt)  # noqa: E731
    self.rgb = mk((self.E,) + SCREEN_SHAPE, torch.uint8)
    self.rewards = mk((self.E,), torch.float32)
    self.terminals = mk((self.E,), torch.uint8)
    self._rgb = self.rgb.numpy()
    self._rew = self.rewards.numpy()
    self._term = self.terminals.numpy()
    self.is_training = is_training
    self.threads = max(1, int(threads))
    self._ex = ThreadPoolExecutor(self.threads) if self.threads > 1 else None
    self._chunks = np.array_split(np.arange(self.E), self.threads)

  def _run(self, fn):
    if self._ex is None:
      fn(range(self.E))
    else:
      list(self._ex.map(fn, self._chunks))

  def begin(self):
    """new_random_game of every env (agent.py:33-35); their first frames in ``rgb``."""
    def f(idx):
      for e in idx:
        self._rgb[e] = self.envs[e].new_random_game()[0]
    self._run(f)
    return self.rgb

  def step(self, actions):
    """act of every env (agent.py:59-62), then new_random_game where terminal (agent.py:66-67);
    the post-act frames (what observe gets) are in ``rgb``."""
    actions = np.asarray(actions)

    def f(idx):
      for e in idx:
        env = self.envs[e]
        scr, r, term = env.act(int(actions[e]), is_training=self.is_training)
        self._rgb[e] = scr
        self._rew[e] = r
        self._term[e] = 1 if term else 0
        if term:
          env.new_random_game()
    self._run(f)
    return self.rgb, self.rewards, self.terminals

  def close(self):
    if self._ex is not None:
      self._ex.shutdown()
      self._ex = None


class SyntheticHostEnvPool(object):
  """The synthetic emulator (bit-identical to the device env) stepped on host threads by the
  C-ABI (a3c_hostenv_*), with HostEnvPool's interface: a stand-in for E real ALE workers when
  driving or measuring the external-env path (PCIe-inclusive).  Buffers are pinned."""

  def __init__(self, num_envs, action_size, start_lives=0, num_frames=1024, seed=123, env_id_base=0,
               random_start=30, action_repeat=1, threads=8, is_training=True, upload_chunks=2):
    import ctypes
    from . import _lib
    self._lib = _lib
    self.E = int(num_envs)
    h = ctypes.c_void_p()
    _lib.check(_lib.lib().a3c_hostenv_create(self.E, int(action_size), int(start_lives), int(random_start),
                                             int(action_repeat), int(num_frames), int(seed), int(env_id_base),
                                             int(threads), ctypes.byref(h)), 'a3c_hostenv_create')
    self._h = h
    pin = torch.cuda.is_available()
    mk = lambda shape, dt: torch.zeros(shape, dtype=dt).pin_memory() if pin else torch.zeros(shape, dtype=dt)  # noqa: E731
    self.rgb = mk((self.E,) + SCREEN_SHAPE, torch.uint8)
    self.rewards = mk((self.E,), torch.float32)
    self.terminals = mk((self.E,), torch.uint8)
    self._acts = mk((self.E,), torch.int32)
    self.is_training = is_training
    self.upload_chunks = int(upload_chunks)   # Engine.iterate_host: ranges per step (H2D overlap)

  def begin(self):
    self._lib.check(self._lib.lib().a3c_hostenv_begin(self._h, self._lib.ptr(self.rgb)), 'a3c_hostenv_begin')
    return self.rgb

  def step(self, actions):
    a = torch.as_tensor(np.asarray(actions, np.int32))
    self._acts.copy_(a)
    L, p = self._lib.lib(), self._lib.ptr
    self._lib.check(L.a3c_hostenv_step(self._h, p(self._acts), 1 if self.is_training else 0, p(self.rgb),
                                       p(self.rewards), p(self.terminals)), 'a3c_hostenv_step')
    return self.rgb, self.rewards, self.terminals

  def step_range(self, actions, env_lo, env_hi):
    """step of envs [env_lo, env_hi) only; actions is the full [E] array."""
    self._acts.copy_(torch.as_tensor(np.asarray(actions, np.int32)))
    L, p = self._lib.lib(), self._lib.ptr
    self._lib.check(L.a3c_hostenv_step_range(self._h, p(self._acts), 1 if self.is_training else 0, p(self.rgb),
                                             p(self.rewards), p(self.terminals), int(env_lo), int(env_hi)),
                    'a3c_hostenv_step_range')

  def close(self):
    if getattr(self, '_h', None):
      self._lib.lib().a3c_hostenv_destroy(self._h)
      self._h = None

  def __del__(self):
    try:
      self.close()
    except Exception:
      pass

"""Environment / GymEnvironment / SimpleGymEnvironment (environment.py:14-106) on device.

``gym``/ALE is absent from this image, so the emulator behind these classes is the batched
synthetic Atari env of the C-ABI (a3c_env_*; dynamics restated in oracle/synthetic_env.py):
ALE-like lives, episode ends, rewards in {-1,0,1}, RGB 210x160x3 frames from an HBM frame
pool.  The reference's interface semantics are kept exactly: ``new_game`` resets only when
``lives == 0`` then takes one no-op step (:28-33), ``new_random_game`` adds 0..random_start-1
no-ops (:35-40), ``act`` repeats the action, turns a lost life into reward -1 + terminal when
training and stops at a terminal (:78-96), ``screen`` is the fp64-luminance + Pillow
BILINEAR 84x84 image (:49-53, bit-exact).  Screens are u8 [84,84] device tensors.

``BatchedEnvironment`` is the same for E envs at once (the MI355X-native form).
"""
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import check, lib

GAMES = {  # ALE minimal action sets and starting lives
    'Pong-v0': (6, 0),
    'Breakout-v0': (4, 5),
    'SpaceInvaders-v0': (6, 3),
}


def game_spec(env_name):
  if env_name not in GAMES:
    raise ValueError('unknown env_name %r (synthetic env knows %s)' % (env_name, sorted(GAMES)))
  return GAMES[env_name]


class BatchedEnvironment(object):
  """E synthetic Atari envs on device."""

  def __init__(self, config, num_envs=1, env_id_base=0, seed=None, num_frames=None):
    _lib.require_device()
    self.action_size_, self.start_lives = game_spec(config.env_name)
    self.E = int(num_envs)
    self.dims = (config.screen_width, config.screen_height)
    if tuple(self.dims) != (84, 84):
      raise ValueError('the HIP screen kernel is specialised for 84x84 (config.py:38-39)')
    self.random_start = int(config.random_start)
    self.action_repeat = int(getattr(config, 'action_repeat', 1))
    self.display = getattr(config, 'display', False)
    seed = int(getattr(config, 'random_seed', 123) if seed is None else seed)
    nf = int(num_frames if num_frames is not None else min(getattr(config, 'num_frames', 1024), 4096))
    h = ctypes.c_void_p()
    check(lib().a3c_env_create(self.E, self.action_size_, self.start_lives, self.random_start, self.action_repeat,
                               nf, seed, int(env_id_base), ctypes.byref(h)), 'a3c_env_create')
    self._h = h
    ptrs = [ctypes.c_void_p() for _ in range(7)]
    check(lib().a3c_env_buffers(h, *[ctypes.byref(p) for p in ptrs]), 'a3c_env_buffers')
    from .engine import _view
    self._frame = _view(ptrs[1].value, (self.E,), torch.int32)
    self._lives = _view(ptrs[2].value, (self.E,), torch.int32)
    self._reward = _view(ptrs[5].value, (self.E,), torch.float32)
    self._terminal = _view(ptrs[6].value, (self.E,), torch.uint8)
    self.frame_pool = _view(ptrs[0].value, (nf, 210, 160, 3), torch.uint8)
    self._screens = torch.empty((self.E, 84, 84), dtype=torch.uint8, device='cuda')
    self._act = torch.zeros(self.E, dtype=torch.int32, device='cuda')

  def __del__(self):
    try:
      if getattr(self, '_h', None):
        lib().a3c_env_destroy(self._h)
        self._h = None
    except Exception:
      pass

  # -- reference interface, vectorised -------------------------------------------------
  def new_game(self, mask=None):
    check(lib().a3c_env_new_game(self._h, _lib.ptr(mask), 0, _lib.stream_handle()), 'a3c_env_new_game')
    return self.screens(), 0, 0, self.terminals

  def new_random_game(self, mask=None):
    check(lib().a3c_env_new_game(self._h, _lib.ptr(mask), 1, _lib.stream_handle()), 'a3c_env_new_game')
    return self.screens(), 0, 0, self.terminals

  def act(self, actions, is_training=True, simple=False):
    a = torch.as_tensor(actions, dtype=torch.int32).to('cuda').reshape(self.E).contiguous()
    check(lib().a3c_env_act(self._h, _lib.ptr(a), 1 if is_training else 0, 1 if simple else 0, None, None, None,
                            _lib.stream_handle()), 'a3c_env_act')
    return self.screens(), self.rewards, self.terminals

  def screens(self):
    check(lib().a3c_env_screen(self._h, _lib.ptr(self._screens), 84 * 84, _lib.stream_handle()), 'a3c_env_screen')
    return self._screens

  @property
  def rewards(self):
    return self._reward

  @property
  def terminals(self):
    return self._terminal

  @property
  def lives_all(self):
    return self._lives

  @property
  def action_size(self):
    return self.action_size_


class Environment(object):
  """environment.py:14-72 for one env (the synthetic emulator, E = 1)."""

  def __init__(self, config):
    self.env = BatchedEnvironment(config, 1)

    screen_width, screen_height, self.action_repeat, self.random_start = \
        config.screen_width, config.screen_height, config.action_repeat, config.random_start

    self.display = config.display
    self.dims = (screen_width, screen_height)

    self._screen = None
    self.reward = 0
    self.terminal = True

  def new_game(self, from_random_game=False):
    self.env.new_game()
    self._sync()
    self.render()
    return self.screen, 0, 0, self.terminal

  def new_random_game(self):
    self.env.new_random_game()
    self._sync()
    self.render()
    return self.screen, 0, 0, self.terminal

  def _sync(self):
    self.reward = float(self.env.rewards[0].item())
    self.terminal = bool(self.env.terminals[0].item())

  @property
  def screen(self):
    return self.env.screens()[0]

  @property
  def action_size(self):
    return self.env.action_size

  @property
  def lives(self):
    return int(self.env.lives_all[0].item())

  @property
  def state(self):
    return self.screen, self.reward, self.terminal

  def render(self):
    if self.display:
      pass   # no display in this runtime

  def after_act(self, action):
    self.render()


class GymEnvironment(Environment):
  def __init__(self, config):
    super(GymEnvironment, self).__init__(config)

  def act(self, action, is_training=True):       # environment.py:78-96
    self.env.act([int(action)], is_training=is_training)
    self._sync()
    self.after_act(action)
    return self.state


class SimpleGymEnvironment(Environment):
  def __init__(self, config):
    super(SimpleGymEnvironment, self).__init__(config)

  def act(self, action, is_training=True):       # environment.py:102-106
    self.env.act([int(action)], is_training=is_training, simple=True)
    self._sync()
    self.after_act(action)
    return self.state

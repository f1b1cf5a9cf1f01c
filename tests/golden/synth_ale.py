"""gym/ALE stand-in whose emulator primitives are the build's synthetic Atari (test data generator).

The engine's device env (csrc/env_dev.h), the C++ host workers (a3c_hostenv_*) and
oracle/synthetic_env.py all implement the same emulator *and* the reference's interface rules
on top of it (new_game / new_random_game / act, environment.py:28-96).  To pin those rules to
the reference itself, this module exposes ONLY the emulator primitives -- ``reset()`` (a new
episode), ``step(a)`` (one emulator frame: frame id, reward, lives, game over) and
``ale.lives()`` -- in gym's interface, so the reference's own ``GymEnvironment`` can drive them
(make_env_goldens.py).  The rules then come from the reference's code, not from the build.

The one substitution: the reference draws its no-op count with ``random.randint(0,
random_start - 1)`` (environment.py:37).  Python's stream cannot be reproduced on the GPU, so the
build draws it from Philox keyed by the emulator state after ``new_game`` (ep_step, env id,
episode).  ``PhiloxRandom`` is a ``random`` module stand-in with that ``randint``; the
reference's loop around it is unchanged.
"""
import numpy as np

from oracle import philox as px
from oracle.synthetic_env import SyntheticAtari


class _Ale:
    def __init__(self, env):
        self._env = env

    def lives(self):
        return int(self._env.emu.lives[0])


class _Space:
    def __init__(self, n):
        self.n = n


class SynthALE:
    """One synthetic emulator (env id ``env_id``) behind gym's reset / step / ale.lives."""

    def __init__(self, seed, env_id, num_frames, action_size, start_lives):
        self.emu = SyntheticAtari(seed, 1, num_frames, action_size, start_lives, env_id_base=env_id)
        self.ale = _Ale(self)
        self.action_space = _Space(action_size)
        self._all = np.ones(1, bool)
        self.resets = 0
        self.steps = 0

    def _obs(self):
        # the trace reads the frame id; the RGB frame itself is pool_frame(seed, id)
        return np.full((1, 1, 3), int(self.emu.frame[0]), np.int64)

    def reset(self):
        self.resets += 1
        self.emu._reset(self._all)
        return self._obs()

    def step(self, a):
        self.steps += 1
        self.emu._step(int(a), self._all)
        return self._obs(), float(self.emu.reward[0]), bool(self.emu.terminal[0]), {}


class PhiloxRandom:
    """``random`` stand-in for environment.py:37: randint(0, k-1) = Philox(ep_step, env id,
    episode, P_NOOP).x % k of the emulator the reference env is driving."""

    def __init__(self):
        self.ale = None

    def randint(self, lo, hi):
        assert lo == 0 and self.ale is not None
        e = self.ale.emu
        x0 = px.philox4x32(e.ep_step, e.ids, e.episode, px.P_NOOP, e.k0, e.k1)[0]
        return int(x0[0] % np.uint32(hi + 1))

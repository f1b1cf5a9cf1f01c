"""Scripted gym/ALE stand-in for env-semantics goldens (test data generator, not an emulator of
any game): ``reset()`` / ``step(a)`` -> (obs, reward, done, info) / ``ale.lives()`` /
``action_space.n`` with a seeded, action-dependent script.  Observations are tiny RGB frames
whose pixels encode a running frame id, so a trace records which frame a call returned."""
import numpy as np


class _Ale:
    def __init__(self, env):
        self._env = env

    def lives(self):
        return self._env.lives_


class _Space:
    def __init__(self, n):
        self.n = n


class ScriptedALE:
    def __init__(self, seed, start_lives=3, max_len=40, n_actions=6, frame_shape=(6, 5, 3)):
        self.rng = np.random.default_rng(seed)
        self.L0 = start_lives
        self.max_len = max_len
        self.ale = _Ale(self)
        self.action_space = _Space(n_actions)
        self.lives_ = 0
        self.t = 0
        self.fid = 0
        self.resets = 0
        self.steps = 0
        self.frame_shape = frame_shape

    def _obs(self):
        self.fid += 1
        v = self.fid % 251
        return np.full(self.frame_shape, v, np.uint8)

    def reset(self):
        self.resets += 1
        self.lives_ = self.L0 if self.L0 > 0 else 1
        self.t = 0
        return self._obs()

    def step(self, a):
        self.steps += 1
        self.t += 1
        u = self.rng.random(3)
        r = 1.0 if u[0] < 0.15 + 0.02 * (int(a) % 3) else (-1.0 if u[0] > 0.9 else 0.0)
        if u[1] < 0.12 and self.lives_ > 0:
            self.lives_ -= 1
        done = self.lives_ == 0 or self.t >= self.max_len
        if self.t >= self.max_len:
            self.lives_ = 0
        return self._obs(), r, done, {}

"""Synthetic Atari stand-in, numpy restatement (TEST INFRASTRUCTURE ONLY).

gym/ALE is absent from the image (SURVEY.md §2 "OUT OF SCOPE | gym/ALE emulation"),
so the build defines a deterministic emulator with the same *interface semantics*
the reference relies on:

* ``Environment.new_game``       environment.py:28-33   (reset only when lives == 0, then one no-op step)
* ``Environment.new_random_game`` environment.py:35-40  (0..random_start-1 extra no-op steps)
* ``GymEnvironment.act``          environment.py:78-96 (action repeat, life-loss -> reward-1 & terminal
                                                          when training, break on terminal)
* ``Environment.lives``           environment.py:59-61

Emulator state per env (all integers): episode, ep_step, ep_len, lives, frame.
Screens are RGB u8 [210,160,3] frames drawn from a hashed pool of ``num_frames`` frames.
The HIP engine (csrc/env.hip) implements exactly this function; tests replay it.
"""
import numpy as np

from . import philox as px

SCREEN_H, SCREEN_W = 210, 160
FRAME_BYTES = SCREEN_H * SCREEN_W * 3
GOLDEN_MULT = 2654435761  # action mixing constant

# ALE minimal action sets / starting lives for the configs of BASELINE.json
GAMES = {
    'Pong-v0': dict(action_size=6, start_lives=0),
    'Breakout-v0': dict(action_size=4, start_lives=5),
    'SpaceInvaders-v0': dict(action_size=6, start_lives=3),
}

REWARD_P = np.float32(0.02)      # P(+1) = P(-1) = 0.02
LIFE_LOSS_P = np.float32(1.0 / 256.0)
EP_LEN_MIN, EP_LEN_SPAN = 200, 1801  # episode length in [200, 2000]


def pool_frame(seed, f):
    """Frame ``f`` of the hashed pool: byte i of 16-byte chunk j comes from
    philox(ctr=(j, f, P_POOL, 0)).  Returns u8 [210,160,3]."""
    k0, k1 = px.seed_key(seed)
    nchunk = FRAME_BYTES // 16
    j = np.arange(nchunk, dtype=np.uint32)
    w = px.philox4x32(j, np.uint32(f), px.P_POOL, 0, k0, k1)
    words = np.stack(w, axis=1).astype('<u4')           # [nchunk, 4]
    return words.view(np.uint8).reshape(SCREEN_H, SCREEN_W, 3)


def pool_frame84(seed, f):
    """Frame ``f`` of the pre-sized pool (measurement mode M2): the same hash as
    pool_frame over the 441 chunks of one 84x84 u8 plane.  Returns u8 [84, 84]."""
    k0, k1 = px.seed_key(seed)
    j = np.arange(84 * 84 // 16, dtype=np.uint32)
    w = px.philox4x32(j, np.uint32(f), px.P_POOL, 0, k0, k1)
    return np.stack(w, axis=1).astype('<u4').view(np.uint8).reshape(84, 84)


class SyntheticAtari:
    """Vectorised over E envs with global ids ``env_ids``."""

    def __init__(self, seed, num_envs, num_frames, action_size, start_lives,
                 random_start=30, action_repeat=1, env_id_base=0):
        self.seed = int(seed)
        self.k0, self.k1 = px.seed_key(seed)
        self.E = num_envs
        self.P = int(num_frames)
        self.A = int(action_size)
        self.L0 = int(start_lives)
        self.random_start = int(random_start)
        self.action_repeat = int(action_repeat)
        self.ids = np.arange(env_id_base, env_id_base + num_envs, dtype=np.uint32)
        self.episode = np.zeros(num_envs, np.uint32)
        self.ep_step = np.zeros(num_envs, np.uint32)
        self.ep_len = np.zeros(num_envs, np.uint32)
        self.lives = np.zeros(num_envs, np.int32)
        self.frame = np.zeros(num_envs, np.uint32)
        self.reward = np.zeros(num_envs, np.float32)
        self.terminal = np.zeros(num_envs, bool)

    # -- emulator primitives --------------------------------------------------
    def _reset(self, m):
        """``self.env.reset()`` (environment.py:30) for envs in mask m."""
        self.episode[m] += 1
        self.ep_step[m] = 0
        self.lives[m] = self.L0
        x0, x1, _, _ = px.philox4x32(self.episode, self.ids, px.P_RESET, 0, self.k0, self.k1)
        self.ep_len[m] = (EP_LEN_MIN + x0 % EP_LEN_SPAN)[m]
        self.frame[m] = (x1 % self.P)[m]

    def _step(self, action, m):
        """``self.env.step(action)`` (environment.py:42-43) for envs in mask m."""
        action = np.broadcast_to(np.asarray(action, np.uint32), (self.E,))
        self.ep_step[m] += 1
        x0, x1, x2, _ = px.philox4x32(self.ep_step, self.ids, self.episode, px.P_STEP,
                                      self.k0, self.k1)
        mix = (x0.astype(np.uint64) + action.astype(np.uint64) * GOLDEN_MULT) & 0xFFFFFFFF
        frame = (mix % self.P).astype(np.uint32)
        u = px.u01(x1)
        r = np.where(u < REWARD_P, 1.0, np.where(u >= np.float32(1.0) - REWARD_P, -1.0, 0.0))
        lose = (px.u01(x2) < LIFE_LOSS_P) & (self.lives > 0)
        over = self.ep_step >= self.ep_len
        self.frame[m] = frame[m]
        self.reward[m] = r.astype(np.float32)[m]
        lives = np.where(lose, self.lives - 1, self.lives)
        lives = np.where(over, 0, lives)
        self.lives[m] = lives[m]
        term = over | ((self.L0 > 0) & (self.lives == 0))
        self.terminal[m] = term[m]

    # -- reference interface semantics ----------------------------------------
    def new_game(self, m=None):
        """environment.py:28-33."""
        m = np.ones(self.E, bool) if m is None else m
        self._reset(m & (self.lives == 0))
        self._step(0, m)

    def new_random_game(self, m=None):
        """environment.py:35-40."""
        m = np.ones(self.E, bool) if m is None else m
        self.new_game(m)
        x0, _, _, _ = px.philox4x32(self.ep_step, self.ids, self.episode, px.P_NOOP,
                                    self.k0, self.k1)
        k = np.where(m, x0 % np.uint32(self.random_start), 0).astype(np.int64)
        for i in range(int(k.max(initial=0))):
            self._step(0, m & (k > i))

    def act(self, action, is_training=True):
        """GymEnvironment.act, environment.py:78-96.  Returns (frame_idx, reward, terminal)."""
        cum = np.zeros(self.E, np.float32)
        start_lives = self.lives.copy()
        active = np.ones(self.E, bool)
        for _ in range(self.action_repeat):
            self._step(action, active)
            cum = np.where(active, cum + self.reward, cum)
            if is_training:
                lost = active & (start_lives > self.lives)
                cum = np.where(lost, cum - 1, cum)
                self.terminal[lost] = True
            active = active & ~self.terminal
            if not active.any():
                break
        self.reward = cum.astype(np.float32)
        return self.frame.copy(), self.reward.copy(), self.terminal.copy()

    def simple_act(self, action):
        """SimpleGymEnvironment.act, environment.py:102-106 (one raw step, no life-loss handling)."""
        self._step(action, np.ones(self.E, bool))
        return self.frame.copy(), self.reward.copy(), self.terminal.copy()

    def screens_rgb(self, frames=None):
        frames = self.frame if frames is None else frames
        return np.stack([pool_frame(self.seed, int(f)) for f in frames])

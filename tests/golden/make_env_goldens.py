"""Golden traces of the reference's OWN Environment / GymEnvironment semantics
(environment.py:28-96: new_game resets only when lives == 0, new_random_game's 0..random_start-1
no-ops, act's action repeat, life loss -> reward - 1 and terminal when training, break on
terminal, and agent.py:66-67's new_random_game after a terminal), written by driving the
reference's code itself:

* env_act_golden.npz   over the scripted emulator of fake_ale.py, with Python ``random`` no-op
                       draws -- pins the host env adapter src/host_env.AtariEnv;
* synth_env_golden.npz over synth_ale.SynthALE, whose reset / step / lives are the build's
                       synthetic emulator primitives and whose no-op draw is the build's Philox
                       draw -- pins the rules that oracle/synthetic_env.py, the device env
                       (a3c_env_*, the engine) and the C++ host workers (a3c_hostenv_*) implement
                       on top of that emulator (tests/test_host_env.py, tests/test_gpu_dropin.py).

Run in the build container only (the reference never travels to the GPU box):

    python tests/golden/make_env_goldens.py
"""
import os
import random

import numpy as np

from fake_ale import ScriptedALE
from make_goldens import _import_reference

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = [  # (emulator seed, start lives, action_repeat, random_start, is_training, python random seed)
    (1, 3, 1, 30, True, 11), (2, 5, 4, 30, True, 12), (3, 0, 1, 30, True, 13),
    (4, 3, 2, 5, False, 14), (5, 1, 3, 8, True, 15),
]
STEPS = 120


def trace(env, emu, actions, is_training):
    """per call: kind (0 new_random_game, 1 act), frame id, reward, terminal, lives, emulator
    steps and resets so far."""
    rows = []

    def rec(kind, r, term):
        rows.append((kind, int(env._screen[0, 0, 0]), float(r), int(bool(term)), emu.lives_, emu.steps,
                     emu.resets))

    _, r, _, term = env.new_random_game()
    rec(0, r, term)
    for a in actions:
        _, r, term = env.act(int(a), is_training=is_training)
        rec(1, r, term)
        if term:
            _, r, _, t2 = env.new_random_game()
            rec(0, r, t2)
    return np.array(rows, np.float64)


# (game, emulator seed, env id, pool frames, action_repeat, random_start, is_training, steps)
SYNTH_GAMES = {'Pong-v0': (6, 0), 'Breakout-v0': (4, 5), 'SpaceInvaders-v0': (6, 3)}
SYNTH_CASES = [
    ('Pong-v0', 123, 0, 64, 1, 30, True, 2500), ('Breakout-v0', 7, 5, 32, 1, 30, True, 2000),
    ('SpaceInvaders-v0', 9, 300, 48, 3, 30, True, 1500), ('Breakout-v0', 11, 17, 40, 2, 8, False, 1500),
    ('Breakout-v0', 13, 1, 16, 4, 30, True, 1500), ('SpaceInvaders-v0', 99, 4095, 64, 1, 1, True, 1500),
]


def synth_trace(env, emu, actions, is_training):
    """per call: kind (0 new_random_game, 1 act), frame id, reward, terminal, lives, and the
    emulator's ep_step and episode after the call (pins reset / no-op / repeat counts)."""
    rows = []

    def rec(kind, r, term):
        rows.append((kind, int(emu.emu.frame[0]), float(r), int(bool(term)), int(emu.emu.lives[0]),
                     int(emu.emu.ep_step[0]), int(emu.emu.episode[0])))

    _, r, _, term = env.new_random_game()
    rec(0, r, term)
    for a in actions:
        _, r, term = env.act(int(a), is_training=is_training)
        rec(1, r, term)
        if term:                                     # agent.py:66-67
            _, r, _, t2 = env.new_random_game()
            rec(0, r, t2)
    return np.array(rows, np.float64)


def synth_main(ref_env):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))      # repo root: oracle/
    from synth_ale import PhiloxRandom, SynthALE
    shim = PhiloxRandom()
    saved = ref_env.random
    ref_env.random = shim                            # environment.py:37's no-op draw source
    out = {}
    try:
        for i, (game, seed, env_id, P, rep, rs, training, steps) in enumerate(SYNTH_CASES):
            A, L0 = SYNTH_GAMES[game]
            emu = SynthALE(seed, env_id, P, A, L0)
            shim.ale = emu
            env = object.__new__(ref_env.GymEnvironment)
            env.env = emu
            env.action_repeat, env.random_start, env.display = rep, rs, False
            env.dims = (84, 84)
            env._screen, env.reward, env.terminal = None, 0, True
            acts = np.random.default_rng(200 + i).integers(0, A, steps)
            out[f'trace{i}'] = synth_trace(env, emu, acts, training)
            out[f'actions{i}'] = acts
    finally:
        ref_env.random = saved
    out['games'] = np.array([c[0] for c in SYNTH_CASES])
    out['cases'] = np.array([c[1:] for c in SYNTH_CASES], np.int64)
    np.savez_compressed(os.path.join(HERE, 'synth_env_golden.npz'), **out)
    print('wrote synth_env_golden.npz:', {k: v.shape for k, v in out.items() if k.startswith('trace')})
    for i in range(len(SYNTH_CASES)):
        t = out[f'trace{i}']
        print(i, 'terminals', int(t[:, 3].sum()), 'resets(episodes)', int(t[-1, 6]), 'life values',
              sorted(set(t[:, 4].astype(int))), 'rewards', sorted(set(t[:, 2])))


def main():
    ref_env, _ = _import_reference()
    synth_main(ref_env)
    out = {}
    for i, (seed, lives, rep, rs, training, pyseed) in enumerate(CASES):
        emu = ScriptedALE(seed, start_lives=lives)
        env = object.__new__(ref_env.GymEnvironment)
        env.env = emu
        env.action_repeat, env.random_start, env.display = rep, rs, False
        env.dims = (84, 84)
        env._screen, env.reward, env.terminal = None, 0, True
        acts = np.random.default_rng(100 + i).integers(0, 6, STEPS)
        random.seed(pyseed)
        out[f'trace{i}'] = trace(env, emu, acts, training)
        out[f'actions{i}'] = acts
    out['cases'] = np.array(CASES, np.float64)
    np.savez_compressed(os.path.join(HERE, 'env_act_golden.npz'), **out)
    print('wrote env_act_golden.npz:', {k: v.shape for k, v in out.items() if k.startswith('trace')})


if __name__ == '__main__':
    main()

"""Golden traces of the reference's OWN Environment / GymEnvironment semantics
(environment.py:28-96: new_game resets only when lives == 0, new_random_game's 0..random_start-1
no-ops from Python ``random``, act's action repeat, life loss -> reward - 1 and terminal when
training, break on terminal) over the scripted emulator of fake_ale.py.  Pins the host env
adapter src/host_env.AtariEnv (tests/test_host_env.py).  Run in the build container only:

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


def main():
    ref_env, _ = _import_reference()
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

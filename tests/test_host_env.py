"""Host env adapter (src/host_env.py) against golden traces of the reference's own
Environment / GymEnvironment code (tests/golden/make_env_goldens.py, environment.py:28-96) on a
scripted emulator: same frames, rewards, terminals, lives, emulator step and reset counts."""
import random

import pytest

import numpy as np

from fake_ale import ScriptedALE
from src.host_env import AtariEnv, HostEnvPool


def _trace(env, emu, actions, is_training):
    rows = []

    def rec(kind, r, term):
        rows.append((kind, int(env._screen[0, 0, 0]), float(r), int(bool(term)), emu.lives_, emu.steps, emu.resets))

    _, r, _, term = env.new_random_game()
    rec(0, r, term)
    for a in actions:
        _, r, term = env.act(int(a), is_training=is_training)
        rec(1, r, term)
        if term:
            _, r, _, t2 = env.new_random_game()
            rec(0, r, t2)
    return np.array(rows, np.float64)


def test_atari_env_matches_reference_traces(golden_dir):
    g = np.load(f'{golden_dir}/env_act_golden.npz')
    for i, (seed, lives, rep, rs, training, pyseed) in enumerate(g['cases']):
        emu = ScriptedALE(int(seed), start_lives=int(lives))
        env = AtariEnv(emu, action_repeat=int(rep), random_start=int(rs), rng=random.Random(int(pyseed)))
        got = _trace(env, emu, g[f'actions{i}'], bool(training))
        assert np.array_equal(got, g[f'trace{i}']), i


def test_host_env_pool_steps_and_resets():
    envs = [AtariEnv(ScriptedALE(s, start_lives=2, max_len=7, frame_shape=(210, 160, 3)), random_start=3, rng=random.Random(s)) for s in range(5)]
    pool = HostEnvPool(envs, threads=2)
    rgb = pool.begin()
    assert tuple(rgb.shape) == (5, 210, 160, 3)
    seen_term = False
    for _ in range(20):
        pool.step(np.arange(5) % 6)
        t = pool.terminals.numpy()
        seen_term |= bool(t.any())
        assert set(np.unique(pool.rewards.numpy())) <= {-2.0, -1.0, 0.0, 1.0}
    assert seen_term
    pool.close()


def test_cpp_host_env_matches_oracle():
    """a3c_hostenv_* (C++ threads, no GPU) == oracle/synthetic_env.py: frames, rewards, terminals,
    resets after terminals (agent.py:66-67)."""
    from oracle.synthetic_env import SyntheticAtari, pool_frame
    from src.host_env import SyntheticHostEnvPool
    E, P, A, L = 5, 40, 6, 3
    pool = SyntheticHostEnvPool(E, A, L, num_frames=P, seed=77, threads=3)
    ref = SyntheticAtari(77, E, P, A, L)
    rgb = pool.begin().numpy()
    ref.new_random_game()
    assert all(np.array_equal(rgb[e], pool_frame(77, int(ref.frame[e]))) for e in range(E))
    rng = np.random.default_rng(0)
    terms = 0
    for it in range(250):
        a = rng.integers(0, A, E).astype(np.int32)
        pool.step(a)
        f, r, t = ref.act(a, True)
        assert np.array_equal(pool.rewards.numpy(), r), it
        assert np.array_equal(pool.terminals.numpy(), t.astype(np.uint8)), it
        assert all(np.array_equal(pool.rgb.numpy()[e], pool_frame(77, int(f[e]))) for e in range(E)), it
        terms += int(t.sum())
        if t.any():
            ref.new_random_game(t.astype(bool))
    assert terms > 0
    pool.close()


def test_cpp_host_env_ranges_equal_full_step():
    """a3c_hostenv_step_range over ragged env ranges (Engine.iterate_host's upload chunks) ==
    a3c_hostenv_step of every env at once, and bad ranges raise."""
    from src.host_env import SyntheticHostEnvPool
    E, P, A, L = 11, 40, 6, 3
    full = SyntheticHostEnvPool(E, A, L, num_frames=P, seed=5, threads=4)
    part = SyntheticHostEnvPool(E, A, L, num_frames=P, seed=5, threads=3)
    assert np.array_equal(full.begin().numpy(), part.begin().numpy())
    rng = np.random.default_rng(1)
    for it in range(120):
        a = rng.integers(0, A, E).astype(np.int32)
        full.step(a)
        cuts = sorted(set([0, E] + list(rng.integers(0, E + 1, 3))))
        for lo, hi in zip(cuts[:-1], cuts[1:]):
            part.step_range(a, lo, hi)
        part.step_range(a, 4, 4)            # empty range: no env steps
        assert np.array_equal(full.rgb.numpy(), part.rgb.numpy()), it
        assert np.array_equal(full.rewards.numpy(), part.rewards.numpy()), it
        assert np.array_equal(full.terminals.numpy(), part.terminals.numpy()), it
    with pytest.raises(RuntimeError):
        part.step_range(a, 3, E + 1)
    with pytest.raises(RuntimeError):
        part.step_range(a, 5, 2)
    full.close()
    part.close()

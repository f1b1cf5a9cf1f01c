"""Env rules against golden traces of the reference's own Environment / GymEnvironment code
(tests/golden/make_env_goldens.py, environment.py:28-96 + agent.py:66-67):
* the host env adapter (src/host_env.AtariEnv) on a scripted emulator: same
  frames, rewards, terminals, lives, emulator step and reset counts (env_act_golden.npz);
* the synthetic env the engine runs -- oracle/synthetic_env.py and the C++ host workers
  (a3c_hostenv_*) -- against the reference's GymEnvironment driving the synthetic emulator's own
  primitives (synth_env_golden.npz): new_game's reset rule, the no-op start count, action repeat,
  life-loss reward and terminal.  The device env (a3c_env_*) is checked against the same file in
  tests/test_gpu_dropin.py."""
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


def _synth_cases(golden_dir):
    g = np.load(f'{golden_dir}/synth_env_golden.npz')
    games = {'Pong-v0': (6, 0), 'Breakout-v0': (4, 5), 'SpaceInvaders-v0': (6, 3)}
    for i, (game, c) in enumerate(zip(g['games'], g['cases'])):
        seed, env_id, P, rep, rs, training, _ = (int(x) for x in c)
        A, L0 = games[str(game)]
        yield dict(seed=seed, env_id=env_id, P=P, rep=rep, rs=rs, training=bool(training), A=A, L0=L0,
                   actions=g[f'actions{i}'], trace=g[f'trace{i}'])


def test_synthetic_env_matches_reference_act_rule(golden_dir):
    """oracle/synthetic_env.py's new_random_game / act == the reference's GymEnvironment over the
    same emulator primitives, call for call."""
    from oracle.synthetic_env import SyntheticAtari
    n = 0
    for c in _synth_cases(golden_dir):
        env = SyntheticAtari(c['seed'], 1, c['P'], c['A'], c['L0'], c['rs'], c['rep'], c['env_id'])
        rows = []

        def rec(kind, r, t):
            rows.append((kind, int(env.frame[0]), float(r), int(bool(t)), int(env.lives[0]), int(env.ep_step[0]),
                         int(env.episode[0])))
        env.new_random_game()
        rec(0, 0, env.terminal[0])
        for a in c['actions']:
            _, r, t = env.act(np.array([a]), is_training=c['training'])
            rec(1, r[0], t[0])
            if t[0]:
                env.new_random_game()
                rec(0, 0, env.terminal[0])
        got = np.array(rows, np.float64)
        assert got.shape == c['trace'].shape
        bad = np.nonzero((got != c['trace']).any(1))[0]
        assert bad.size == 0, (c['seed'], bad[:3], got[bad[:3]], c['trace'][bad[:3]])
        n += int(c['trace'][:, 3].sum())
    assert n > 50       # terminals (life losses and game overs) were exercised


def test_cpp_host_env_matches_reference_act_rule(golden_dir):
    """The C++ host workers (a3c_hostenv_*, the --envs_on host stand-in for ALE processes) follow
    the reference's rules: per act the post-act frame, reward and terminal of the golden trace,
    with new_random_game after a terminal done inside step (agent.py:66-67)."""
    from oracle.synthetic_env import pool_frame
    from src.host_env import SyntheticHostEnvPool
    for c in _synth_cases(golden_dir):
        tr = c['trace']
        pool = SyntheticHostEnvPool(1, c['A'], c['L0'], num_frames=c['P'], seed=c['seed'], env_id_base=c['env_id'],
                                    random_start=c['rs'], action_repeat=c['rep'], threads=1,
                                    is_training=c['training'])
        frames = {f: pool_frame(c['seed'], f) for f in range(c['P'])}
        rgb = pool.begin().numpy()
        assert np.array_equal(rgb[0], frames[int(tr[0, 1])])
        acts = tr[tr[:, 0] == 1]
        assert len(acts) == len(c['actions'])
        for a, row in zip(c['actions'], acts):
            pool.step(np.array([a], np.int32))
            assert pool.rewards.numpy()[0] == row[2] and pool.terminals.numpy()[0] == row[3], (c['seed'], row)
            assert np.array_equal(pool.rgb.numpy()[0], frames[int(row[1])]), (c['seed'], row)
        pool.close()


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

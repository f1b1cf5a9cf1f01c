"""Checkpoint / resume and summaries of the batched engine.

* Resume (the Supervisor's Saver + managed_session restore, main.py:74-90, agent.py:29,34,46): k
  iterations, save, restore into a FRESH engine, m more iterations == k + m uninterrupted
  iterations, bit for bit (parameters, RMSProp slots, frame ring, counters, losses), in every
  engine mode.  The file is keyed by the TF variable names.
* The reference-style resume from parameters + step only (what the reference's Saver keeps):
  parameters and slots restored, global step and worker step restart at the saved step.
* main.py --mode engine: a run of 2K iterations == a run of K, then a second run of K that
  restores the first's checkpoint.
* Summaries: the device aggregates equal a hand replay of train_with_summary's bookkeeping
  (agent.py:91-131) over the oracle's unclipped rewards and terminals."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')

from _engine_parity import build  # noqa: E402

STATE_NAMES = ('params', 'target_params', 'ms', 'mom', 'frame_ring', 'counters', 'loss')

MODES = [dict(algo='a3c', A=6, lives=0), dict(algo='a3c', A=6, lives=0, overlap=True),
         dict(algo='q', A=6, lives=3, n=8), dict(algo='a3c', A=4, lives=5, overlap=True, frame84=1),
         dict(algo='a3c', A=6, lives=3, lstm=True), dict(algo='a3c', A=6, lives=3, lstm=True, overlap=True),
         dict(algo='a3c', A=6, lives=0, dqn_type='nature'), dict(algo='a3c', A=4, lives=5, overlap=True, dqn_type='nature')]
IDS = ['sync', 'overlap', 'q', 'overlap-m2-breakout', 'lstm-sync', 'lstm-overlap', 'nature-sync', 'nature-overlap']


def _make(mode, seed=61):
    m = dict(mode)
    algo, A, lives, n = m.pop('algo'), m.pop('A'), m.pop('lives'), m.pop('n', 5)
    lstm = m.pop('lstm', False)
    if lstm:
        from src.engine import Engine
        from src.initializers import flatten_host, init_params
        from src.kernels import param_names_shapes
        eng = Engine(num_envs=12, n_step=n, action_size=A, algo=algo, start_lives=lives, num_frames=64, seed=seed,
                     lstm=True, learning_rate=3e-3, **m)
        ns = param_names_shapes(A, algo, lstm=True)
        eng.reset(flatten_host(ns, eng.offsets, eng.params.numel(), init_params(ns, seed=seed, stddev=0.06)))
        return eng, ns
    eng, _, ns = build(algo, A, 12, n, lives, seed, frames=64, learning_rate=3e-3, target_q_update_step=200, **m)
    return eng, ns


@pytest.mark.parametrize('mode', MODES, ids=IDS)
def test_resume_is_bit_continuous(mode, tmp_path):
    from src import checkpoint as C
    k, m = 3, 4
    a, ns = _make(mode)
    for _ in range(k + m):
        a.iterate()
    torch.cuda.synchronize()
    b, _ = _make(mode)
    for _ in range(k):
        b.iterate()
    saver = C.Saver(str(tmp_path), max_to_keep=2)
    step = C.save_engine(saver, b, ns)
    assert saver.latest().endswith('model.ckpt-%d.npz' % step)
    arrays = C.load(saver.latest())
    dqn = mode.get('dqn_type', 'nips')          # nature: the Nature_DQN/ scope of network.py:31
    want = ['step'] + [C.tf_name(nm, b.algo, dqn) for nm, _ in ns] + \
        [C.slot_names(C.tf_name(nm, b.algo, dqn))[1] for nm, _ in ns]
    if dqn == 'nature':
        assert 'Nature_DQN/l3_conv/w' in arrays and 'policy/linear/Matrix' in arrays
    assert all(w in arrays for w in want), [w for w in want if w not in arrays]
    del b
    with pytest.raises(RuntimeError):           # the state is tied to its env shard and seed
        _make(mode, seed=999)[0].load_state(arrays['__engine_state__'])
    c, _ = _make(mode)                           # a fresh engine of the same configuration
    assert C.restore_engine(saver, c, ns) == step
    for _ in range(m):
        c.iterate()
    torch.cuda.synchronize()
    for name in STATE_NAMES:
        assert torch.equal(getattr(a, name), getattr(c, name)), name


def test_resume_from_params_and_step(tmp_path):
    """Without the engine state (e.g. a checkpoint converted from another run): parameters, target
    and RMSProp slots come back, and the global step restarts at `step`; the workers' step at the
    saved worker step, or at `step` for a file without one (agent.py:34,46: before_train reads
    step_op into self.T and self.step)."""
    from src import checkpoint as C
    a, ns = _make(MODES[2])                        # q: has a target network
    for _ in range(3):
        a.iterate()
    arrays = C.engine_arrays(a, ns, with_state=False)
    assert 'prediction/l1/w' in arrays and 'target/target_q/bias' in arrays and 'prediction/q/Matrix/RMSProp' in arrays
    step = int(arrays['step'])
    saver = C.Saver(str(tmp_path))
    saver.save(arrays, step)
    c, _ = _make(MODES[2], seed=5)
    assert C.restore_engine(saver, c, ns) == step
    torch.cuda.synchronize()
    for name in ('params', 'target_params', 'ms', 'mom'):       # every tensor (not the alignment padding)
        for off, sz in zip(a.offsets, a.sizes):
            assert torch.equal(getattr(a, name)[off:off + sz], getattr(c, name)[off:off + sz]), name
    # the file keeps the worker step too (host-env resumes continue at it)
    assert int(c.counters[1].item()) == step and c.worker_step == a.worker_step
    del arrays[C.WSTEP_KEY]                        # a file with only `step`: the reference's rule
    saver2 = C.Saver(str(tmp_path / 'ref'))
    saver2.save(arrays, step)
    d, _ = _make(MODES[2], seed=5)
    assert C.restore_engine(saver2, d, ns) == step
    assert int(d.counters[1].item()) == step and d.worker_step == step


def test_state_load_rejects_other_configuration():
    a, _ = _make(MODES[0])
    blob = a.save_state()
    b, _ = _make(MODES[1])
    with pytest.raises(RuntimeError):
        b.load_state(blob)
    with pytest.raises(RuntimeError):
        a.load_state(blob[:100])


def test_main_engine_resumes_bit_for_bit(tmp_path):
    import main
    common = ['--mode', 'engine', '--env_name', 'Breakout-v0', '--num_envs', '8', '--num_frames', '64',
              '--log_every', '2', '--random_seed', '3', '--update', 'overlap']
    one = main.main(common + ['--iterations', '8', '--logdir', str(tmp_path / 'one')])
    torch.cuda.synchronize()
    ref = {k: getattr(one, k).clone() for k in STATE_NAMES}
    del one
    main.main(common + ['--iterations', '4', '--logdir', str(tmp_path / 'two')])
    two = main.main(common + ['--iterations', '4', '--logdir', str(tmp_path / 'two')])
    torch.cuda.synchronize()
    for k in STATE_NAMES:
        assert torch.equal(ref[k], getattr(two, k)), k
    import json
    recs = [json.loads(x) for x in open(tmp_path / 'two' / 'engine.jsonl')]
    assert recs and all(k in recs[-1] for k in ('avg_reward', 'avg_loss', 'avg_q', 'avg_ep_reward', 'max_ep_reward',
                                                'min_ep_reward', 'num_game', 'learning_rate'))


def test_main_engine_host_envs_resume_shortens_the_run(tmp_path):
    """Host-stepped envs resume from parameters + step (no engine state): the resumed run trains
    only the worker steps left to max_step (agent.py:46 `xrange(self.step, self.max_step)`), and a
    fresh run takes exactly ceil(max_step / n) rollouts (the step was read before the
    host engine had written its counters)."""
    import main
    common = ['--mode', 'engine', '--env_name', 'Pong-v0', '--num_envs', '8', '--num_frames', '64', '--envs_on',
              'host', '--host_threads', '2', '--update', 'sync', '--random_seed', '3', '--max_step', '40']
    one = main.main(common + ['--iterations', '3', '--logdir', str(tmp_path / 'a')])
    torch.cuda.synchronize()
    assert one.worker_step == 15
    del one
    two = main.main(common + ['--iterations', '100', '--logdir', str(tmp_path / 'a')])
    torch.cuda.synchronize()
    assert two.worker_step == 40                 # 5 more rollouts, not max_step / n + 1 again
    del two
    fresh = main.main(common + ['--iterations', '100', '--logdir', str(tmp_path / 'b')])
    torch.cuda.synchronize()
    assert fresh.worker_step == 40


@pytest.mark.parametrize('algo,A,lives,n', [('a3c', 6, 3, 5), ('q', 4, 5, 8)])
def test_summaries_match_reference_bookkeeping(algo, A, lives, n):
    """train_with_summary (agent.py:91-131) per env, replayed by hand on the oracle's unclipped
    rewards and terminals: total reward over every step; at a terminal the running episode
    reward (terminal step excluded) is recorded and restarts; loss and q averaged per update."""
    E, iters = 16, 30
    eng, ref, _ = build(algo, A, E, n, lives, seed=71, frames=64, scale=1.0, learning_rate=1e-3,
                        target_q_update_step=100)
    acc = np.zeros(E)
    tot, eps_done, losses, qs = 0.0, [], [], []
    for it in range(iters):
        eng.rollout_grad()
        eng.stats_accumulate()
        torch.cuda.synchronize()
        out = ref.iterate(forced_actions=eng.actions.cpu().numpy())
        assert np.array_equal(eng.terminals.cpu().numpy(), out['terminals'])
        r, t = out['rewards_raw'].astype(np.float64), out['terminals']
        for s in range(n):
            tot += r[s].sum()
            for e in range(E):
                if t[s, e]:
                    eps_done.append(acc[e])
                    acc[e] = 0.0
                else:
                    acc[e] += r[s, e]
        loss = eng.loss.cpu().numpy().astype(np.float64)
        z = eng.z.cpu().numpy()[:n].reshape(n * E, -1).astype(np.float64)
        losses.append(loss[0] if algo == 'q' else loss[3] / (n * E))
        qs.append(z[:, :A].mean() if algo == 'q' else z[:, A].mean())
        eng.apply()
        ref.apply(out['clipped'])          # (advances the oracle's tau / counters with the engine's)
    st = eng.read_stats(reset=True)
    assert eps_done, 'no episode finished: lengthen the run'
    assert st['num_game'] == len(eps_done) and st['env_steps'] == iters * n * E and st['updates'] == iters
    assert st['avg_reward'] == pytest.approx(tot / (iters * n * E), rel=1e-12, abs=1e-15)
    assert st['avg_ep_reward'] == pytest.approx(np.mean(eps_done), rel=1e-12)
    assert st['max_ep_reward'] == max(eps_done) and st['min_ep_reward'] == min(eps_done)
    assert st['avg_loss'] == pytest.approx(np.mean(losses), rel=1e-6)
    assert st['avg_q'] == pytest.approx(np.mean(qs), rel=1e-5, abs=1e-7)
    st2 = eng.read_stats(reset=True)                 # a new interval starts empty
    assert st2['num_game'] == 0 and st2['updates'] == 0

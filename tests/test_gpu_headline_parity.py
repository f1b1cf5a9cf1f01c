"""Oracle parity at the configurations bench.py measures (BASELINE.json configs 2-5, per GPU).

The small-shape tests of test_gpu_engine.py reach only the small-grid kernel variants.  These run
the engine at the exact shapes the bench times, so the variants it actually launches are checked
against oracle/engine_ref.py:
  * C2 headline: Pong, 256 envs, n=5, mode M1 (raw RGB + Environment.screen on device), overlap
    pipeline: k_head_screen_conv12 (fused step t head + screen + step t+1 conv1/conv2), k_fc_part
    over 256 rows with the wave-0 fold, k_conv_bwd<false,4> on 256 workgroups of 5 samples (one per
    CU, the CB_SMEM_SOLO reservation);
    and the synchronous update (k_head_screen, k_conv12_fwd, k_fc_fwd, k_conv_bwd<true,8>);
  * C3 per-GPU shard: Breakout (A=4, 5 lives), 256 envs;
  * C4 per-GPU shard: Pong, 512 envs, sync, overlap and Hogwild at world 1;
  * C5 per-GPU shard: SpaceInvaders LSTM head, 256 envs (build-defined head, oracle restated);
  * async one-step Q-learning at bench.py's Q shape (256 envs, train_frequency 32), plain and
    double-Q, with an epsilon schedule that crosses the greedy / random split inside the run.
Initial weights are the reference's init (stddev 0.02, agent.py:214 / ops.py:36-37) and the
optimizer constants the reference's (config.py:11-16, main.py:64-65), so the shapes, weights and
update rule are the headline's.  Tolerances: see tests/_engine_parity.py."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')

from _engine_parity import (assert_draws_explained, check_hogwild1_vs_oracle, check_overlap_vs_oracle,  # noqa: E402
                            check_sync_vs_oracle)


FRAMES = 512     # pool frames: more than the envs, so every env reads its own frames


@pytest.mark.timeout(900)
def test_c2_headline_overlap_m1_matches_oracle():
    """The bench's default line: Pong, E=256, n=5, M1, overlap (stale-1), reference init/lr."""
    check_overlap_vs_oracle(6, 256, 5, 0, rollouts=5, seed=123, frames=FRAMES, scale=1.0)


@pytest.mark.timeout(900)
def test_c2_headline_overlap_m1_large_lr_matches_oracle():
    """Same shape with larger weights and step size, so parameter drift and ReLU-mask changes
    between iterations are visible in the 1e-5 parameter check."""
    check_overlap_vs_oracle(6, 256, 5, 0, rollouts=3, seed=5, frames=FRAMES, scale=4.0, learning_rate=3e-3)


@pytest.mark.timeout(900)
def test_c2_headline_sync_m1_matches_oracle():
    check_sync_vs_oracle('a3c', 6, 256, 5, 0, iters=3, seed=123, frames=FRAMES, scale=1.0)


@pytest.mark.timeout(900)
def test_c2_headline_overlap_m2_matches_oracle():
    """Measurement mode M2 (pre-sized 84x84 frames) at the headline shape."""
    check_overlap_vs_oracle(6, 256, 5, 0, rollouts=3, seed=124, frames=FRAMES, scale=1.0, frame84=1)


@pytest.mark.timeout(900)
@pytest.mark.parametrize('overlap', [True, False])
def test_c3_breakout_shard_matches_oracle(overlap):
    """C3 per GPU: Breakout-v0 (A=4, 5 lives: life-loss terminals inside the rollout), 256 envs."""
    if overlap:
        check_overlap_vs_oracle(4, 256, 5, 5, rollouts=3, seed=33, frames=FRAMES, scale=4.0, learning_rate=2e-3)
    else:
        check_sync_vs_oracle('a3c', 4, 256, 5, 5, iters=2, seed=33, frames=FRAMES, scale=4.0, learning_rate=2e-3)


@pytest.mark.timeout(900)
@pytest.mark.parametrize('mode', ['overlap', 'sync', 'hogwild', 'hogwild-sync'])
def test_c4_512_env_shard_matches_oracle(mode):
    """C4 per GPU: Pong, 512 envs, in the update modes (Hogwild at world 1: one worker's clip +
    unlocked push + pull equals the oracle's clip + RMSProp -- overlapped with the next rollout at
    staleness 1, bench.py's default, or after each rollout)."""
    kw = dict(seed=44, frames=1024, scale=4.0, learning_rate=2e-3)
    if mode == 'overlap':
        check_overlap_vs_oracle(6, 512, 5, 0, rollouts=3, **kw)
    elif mode == 'sync':
        check_sync_vs_oracle('a3c', 6, 512, 5, 0, iters=2, **kw)
    elif mode == 'hogwild':
        check_overlap_vs_oracle(6, 512, 5, 0, rollouts=3, hogwild=True, **kw)
    else:
        check_hogwild1_vs_oracle(6, 512, 5, 0, iters=2, **kw)


@pytest.mark.timeout(900)
def test_c5_lstm_shard_matches_oracle():
    """C5 per GPU: SpaceInvaders (A=6, 3 lives), LSTM head, 256 envs, n=5, synchronous engine,
    against the restated oracle (the reference has no recurrent code: parity unpinned against
    a reference execution)."""
    from test_gpu_lstm import build, same_act_grads, unflat, rel_l2
    from oracle import ref_cpu as Rc
    A, E, n = 6, 256, 5
    eng, ref, ns = build(A, E, n, 3, seed=55, frames=FRAMES, scale=2.0, learning_rate=2e-3)
    for it in range(2):
        Pk = unflat(eng, ns, eng.params)
        eng.rollout_grad()
        torch.cuda.synchronize()
        acts = eng.actions.cpu().numpy()
        out = ref.iterate(forced_actions=acts)
        planes = np.concatenate([np.transpose(ref.states(ref.tau + t), (0, 3, 1, 2)) for t in range(n)])
        assert_draws_explained(acts, out, 'a3c', A, it, z_eng=eng.z.cpu().numpy()[:n])
        assert np.array_equal(eng.rewards.cpu().numpy(), out['rewards'])
        terms = eng.terminals.cpu().numpy()
        assert np.array_equal(terms, out['terminals'])
        np.testing.assert_allclose(eng.lstm_h.cpu().numpy(), out['lstm']['H'], rtol=1e-4, atol=2e-5)
        tgt = eng.returns.cpu().numpy()
        np.testing.assert_allclose(tgt, out['target'], rtol=1e-4, atol=2e-5)
        losses, g_same = same_act_grads(eng.slot(0), planes, Pk, A, n, E, tgt, terms)
        loss = eng.loss.cpu().numpy()
        for i, key in enumerate(('policy', 'value', 'entropy', 'total')):
            assert abs(loss[i] - losses[key]) <= 1e-4 * max(1.0, abs(losses[key])), (it, key)
            # independent: the oracle's own fp64 lstm_a3c_forward and its bootstrap targets
            ind = out['losses'][key]
            assert abs(loss[i] - ind) <= 1e-4 * max(1.0, abs(ind)), ('independent', it, key, loss[i], ind)
        G = unflat(eng, ns, eng.grads)
        for name, _ in ns:
            assert rel_l2(G[name], g_same[name]) < 1e-4, (it, name, rel_l2(G[name], g_same[name]))
        eng.apply()
        ref.apply({k: Rc.clip_by_norm(v, 40.0) for k, v in g_same.items()})
        torch.cuda.synchronize()
        P = unflat(eng, ns, eng.params)
        for name, _ in ns:
            d = np.abs(P[name] - ref.params[name]).max()
            assert d <= 1e-5 * max(1.0, np.abs(ref.params[name]).max()), (it, name, d)


@pytest.mark.timeout(900)
@pytest.mark.parametrize('double_q', [False, True])
def test_q_bench_shape_matches_oracle(double_q):
    """bench.py --algo q --n-step 32 --update sync: 256 envs, 32 steps per update, the target copy
    every 40 updates' worth of steps.  The epsilon schedule (agent.py:142-144, evaluated per env and
    step inside the head kernel) starts at 0.5 and decays over 2,000 steps toward each env's own
    final epsilon (0.1 / 0.01 / 0.5, main.py:68), so both the greedy argmax and the random draw run."""
    check_sync_vs_oracle('q', 6, 256, 32, 0, iters=2, seed=66, frames=FRAMES, scale=4.0, learning_rate=2e-3,
                         ep_start=0.5, ep_end_t=2000, learn_start=0, double_q=double_q)


@pytest.mark.timeout(900)
def test_q_overlap_bench_shape_matches_oracle():
    """bench.py --algo q --n-step 32 (the overlapped pipeline): 256 envs, stale-1 acting, the TD
    targets of rollout k-1 formed by its backward with the target network as it stands then, a
    target sync inside the run (target_q_update_step 16,384 = two updates of 8,192 env-steps)."""
    check_overlap_vs_oracle(6, 256, 32, 0, rollouts=4, seed=67, frames=FRAMES, scale=4.0, learning_rate=2e-3,
                            algo='q', target_q_update_step=16384, ep_start=0.5, ep_end_t=2000, learn_start=0)


@pytest.mark.timeout(900)
def test_1024_env_overlap_matches_oracle():
    """bench.py --envs 1024 (overlap): 32 row blocks in the partial fc, the fc weight GEMM's
    in-workgroup split-K form (B = 5,120 > 2,560: the slab form), the conv backward over 5,120
    samples -- the variants the 1,024-env line launches, against the oracle."""
    check_overlap_vs_oracle(6, 1024, 5, 0, rollouts=3, seed=88, frames=2048, scale=4.0, learning_rate=2e-3)

"""The nature trunk in the engine (network.py:30-42, DQN_type='nature': conv 8x8/4 32, conv 4x4/2 64,
conv 3x3/1 64, fc 3136 -> 512 under the A3C policy / value heads), against the CPU oracle
(oracle/engine_ref.py with dqn_type='nature', ref_cpu.forward / backward of the same trunk).

Same bars as the NIPS engine (tests/_engine_parity.py): env dynamics, rewards, terminals and the
frame ring bit-exact; zero unexplained action-draw mismatches; the rollout's head rows against the
oracle's independent fp64 forward at rtol 1e-4; n-step returns 1e-5; losses 1e-4 of max(1, |loss|)
against both the oracle backward on the engine's own activations and the independent forward;
gradients 1e-4 relative-L2 (same activations) and 2e-2 (independent, ReLU flips allowed);
parameters after clip + RMSProp within 1e-5 over the iterations.  The nature trunk exists only in
the reference's (unused, unimportable) A3C Network, so parity is against the restated oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')

from _engine_parity import check_overlap_vs_oracle, check_sync_vs_oracle  # noqa: E402

NAT = dict(dqn_type='nature')


@pytest.mark.timeout(600)
@pytest.mark.parametrize('A,E,n,lives', [(6, 8, 3, 0), (4, 13, 5, 5)])
def test_nature_sync_matches_oracle(A, E, n, lives):
    check_sync_vs_oracle('a3c', A, E, n, lives, iters=3, seed=500 + E, frames=48, scale=2.0, learning_rate=2e-3, **NAT)


@pytest.mark.timeout(600)
def test_nature_overlap_matches_oracle():
    check_overlap_vs_oracle(6, 16, 5, 3, rollouts=4, seed=520, frames=48, scale=2.0, learning_rate=2e-3, **NAT)


@pytest.mark.timeout(600)
@pytest.mark.parametrize('overlap', [False, True])
def test_nature_frame84_mode_matches_oracle(overlap):
    """Mode M2 (pre-sized 84x84 frames, copied by the fused head + screen kernel) on the nature trunk."""
    if overlap:
        check_overlap_vs_oracle(6, 16, 5, 0, rollouts=4, seed=540, frames=48, scale=2.0, learning_rate=2e-3,
                                frame84=1, **NAT)
    else:
        check_sync_vs_oracle('a3c', 6, 8, 4, 0, iters=3, seed=541, frames=48, scale=2.0, learning_rate=2e-3,
                             frame84=1, **NAT)


@pytest.mark.timeout(900)
def test_nature_bench_shape_sync_matches_oracle():
    """bench.py --dqn-type nature --update sync: Pong, 256 envs, n = 5, reference init."""
    check_sync_vs_oracle('a3c', 6, 256, 5, 0, iters=2, seed=530, frames=512, scale=1.0, **NAT)


@pytest.mark.timeout(900)
def test_nature_bench_shape_overlap_matches_oracle():
    """bench.py --dqn-type nature (the overlapped pipeline): Pong, 256 envs, n = 5."""
    check_overlap_vs_oracle(6, 256, 5, 0, rollouts=3, seed=531, frames=512, scale=2.0, learning_rate=2e-3, **NAT)


def test_nature_graph_equals_eager_and_deterministic():
    from _engine_parity import build
    a, _, _ = build('a3c', 6, 32, 5, 0, seed=9, frames=64, use_graph=True, overlap=True, **NAT)
    b, _, _ = build('a3c', 6, 32, 5, 0, seed=9, frames=64, use_graph=False, overlap=True, **NAT)
    for _ in range(3):
        a.iterate()
        b.iterate()
    torch.cuda.synchronize()
    assert torch.isfinite(a.params).all()
    assert torch.equal(a.params, b.params) and torch.equal(a.loss, b.loss)


def test_nature_rejects_what_the_reference_lacks():
    from src.engine import Engine
    with pytest.raises(ValueError):
        Engine(num_envs=4, n_step=2, algo='q', dqn_type='nature')        # the Q-net is NIPS only (agent.py:226)
    with pytest.raises(ValueError):
        Engine(num_envs=4, n_step=2, lstm=True, dqn_type='nature')
    with pytest.raises(ValueError):
        Engine(num_envs=4, n_step=2, dqn_type='wide')                     # network.py:54


def test_nature_pass_timing_hook():
    """a3c_engine_time_kernel's nature ids time the single passes (bench.py's roofline)."""
    from _engine_parity import build
    from src import _lib
    eng, _, _ = build('a3c', 6, 64, 5, 0, seed=3, frames=64, **NAT)
    eng.iterate()
    torch.cuda.synchronize()
    for name, k in _lib.KER_NAT.items():
        if name in ('conv1_fwd', 'conv3_fwd', 'conv2_dx'):   # inside a fused launch: none of their own
            try:
                ms = eng.time_kernel(k, 3)
            except _lib.A3CError as e:
                assert 'k_nat_' in str(e)
                continue
        else:
            ms = eng.time_kernel(k, 3)
        assert 0.0 < ms < 100.0, (name, ms)
    with pytest.raises(RuntimeError):
        eng.time_kernel(_lib.KER_CONV12_FWD, 1)                            # a NIPS kernel id

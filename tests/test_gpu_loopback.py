"""The partitioned-PS exchange on the device, one process (src/distributed.py LoopbackPS): W
virtual ranks that hold the engine's own per-worker-clipped gradient, the collectives as
device-to-device copies on the exchange's streams -- no host staging, no process group.  This runs
the multi-GPU exchange path the RCCL bench takes (two-phase: phase A on the comm stream behind
wait_grad_head, under the conv backward; phase B after the whole backward; the join; the commit)
on a one-GPU box, where RCCL refuses two ranks on one device.  Unmeasured on RCCL / xGMI.

Checks: the two-phase and one-phase forms train bit for bit alike (sync and overlap), and the
update equals the reference PS rule for W workers that pushed the same clipped gradient -- W
sequential RMSProp steps (main.py:63-65, agent.py:316-321) -- on the CPU oracle within 1e-5."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')

W = 4


def _engine(split, overlap, E=32, seed=31, **kw):
    from _engine_parity import build
    eng, ref, ns = build('a3c', 6, E, 5, 0, seed=seed, frames=128, scale=4.0, overlap=overlap,
                         world_size=W, split_exchange=split, learning_rate=3e-3, **kw)
    return eng, ref, ns


@pytest.mark.timeout(600)
@pytest.mark.parametrize('overlap', [False, True], ids=['sync', 'overlap'])
def test_loopback_two_phase_equals_one_phase(overlap):
    from src.distributed import LoopbackPS
    runs = []
    for split in (1, 0):
        eng, _, _ = _engine(split, overlap)
        assert (eng.split_point > 0) == bool(split)
        ps = LoopbackPS(eng.params.numel(), W, split=bool(split))
        for _ in range(5):
            eng.iterate(exchange=ps)
        torch.cuda.synchronize()
        runs.append(eng)
    a, b = runs
    for name in ('params', 'ms', 'mom', 'grads', 'counters', 'loss', 'frame_ring'):
        assert torch.equal(getattr(a, name), getattr(b, name)), name


@pytest.mark.timeout(600)
def test_loopback_split_exchange_matches_oracle():
    """Sync engine at world W with the two-phase loopback exchange: every iteration the oracle
    takes its clipped gradient (on the engine's own activations) as W rank-ordered RMSProp
    steps; parameters within 1e-5, the global step advanced by n E W."""
    from src.distributed import LoopbackPS
    from oracle import ref_cpu as Rc
    from oracle.engine_ref import EngineRef
    from _engine_parity import same_act_grads, rollout_planes, unflat, rel_l2, assert_params
    from src.initializers import init_params
    eng, ref0, ns = _engine(1, False)
    ref = EngineRef(init_params(ns, seed=31, stddev=0.08), 32, 5, 6, 'a3c', 0, 128, 31, world_size=W,
                    learning_rate=3e-3)
    ref.reset()
    ps = LoopbackPS(eng.params.numel(), W, split=True)
    for it in range(3):
        Pk = unflat(eng, ns, eng.params)
        eng.rollout_grad()
        torch.cuda.synchronize()
        out = ref.iterate(forced_actions=eng.actions.cpu().numpy(), grads=False)
        planes = rollout_planes(ref, 5)
        tgt = eng.returns.cpu().numpy()
        np.testing.assert_allclose(tgt, out['target'], rtol=1e-5, atol=1e-5)
        _, g = same_act_grads(eng, planes, Pk, 'a3c', 6, 5, 32, tgt)
        clipped = {k: Rc.clip_by_norm(v, 40.0) for k, v in g.items()}
        G = unflat(eng, ns, eng.grads)             # world > 1: clipped per worker by the backward
        for name, _ in ns:
            assert rel_l2(G[name], clipped[name]) < 1e-4, (it, name)
        ps.apply(eng)
        torch.cuda.synchronize()
        ref.apply_sequence([clipped] * W)
        assert_params(eng, ns, ref, it)
        assert int(eng.counters[1].item()) == ref.global_step == (it + 1) * 5 * 32 * W

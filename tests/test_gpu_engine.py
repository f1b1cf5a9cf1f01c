"""End-to-end parity of the batched actor-learner engine (graph-captured HIP path) against the
CPU replay oracle/engine_ref.py on fixed seeds: env dynamics and frames bit-exact, action draws
consistent, returns / losses within 1e-5 relative (north star bar: 1e-3), gradients within 1e-4,
parameters after RMSProp within 1e-5 over several iterations."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')

from oracle import ref_cpu as Rc  # noqa: E402
from oracle.engine_ref import EngineRef  # noqa: E402


def rel_l2(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def build(algo, A, E, n, lives, seed, frames=48, use_graph=False, scale=4.0, **kw):
    from src.engine import Engine
    from src.initializers import init_params, flatten_host
    from src.kernels import param_names_shapes
    eng = Engine(num_envs=E, n_step=n, action_size=A, algo=algo, start_lives=lives, num_frames=frames, seed=seed,
                 use_graph=use_graph, **kw)
    ns = param_names_shapes(A, algo)
    p = init_params(ns, seed=seed, stddev=0.02 * scale)
    eng.reset(flatten_host(ns, eng.offsets, eng.params.numel(), p))
    ref = EngineRef(p, E, n, A, algo, lives, frames, seed, **{k: v for k, v in kw.items() if k in
                                                              ('target_q_update_step', 'learning_rate', 'frame84')})
    ref.reset()
    return eng, ref, ns


def gpu_act_grads(eng, ref, algo, A, n, E, ns, tgt):
    """oracle backward over the iteration's batch using the engine's saved activations."""
    B = n * E
    planes = np.concatenate([np.transpose(ref.states(ref.tau + t), (0, 3, 1, 2)) for t in range(n)])  # before apply
    l1 = eng.act_l1.cpu().numpy().astype(np.float64).reshape(B, 20, 20, 16)
    l2 = eng.act_l2.cpu().numpy().astype(np.float64)
    zw = A + 1 if algo == 'a3c' else A
    z = eng.z.cpu().numpy()[:n].reshape(B, -1)[:, :zw].astype(np.float64)
    fwd = dict(z=z, h3=eng.act_l3.cpu().numpy().astype(np.float64), flat=l2,
               acts=[Rc.states_nhwc(planes).astype(np.float64) / 255.0, l1, l2.reshape(B, 9, 9, 32)])
    acts = eng.actions.cpu().numpy().reshape(-1)
    P = unflat(eng, ns, eng.params)
    if algo == 'a3c':
        _, dz = Rc.a3c_loss_and_dz(z, acts, tgt.reshape(-1).astype(np.float64), 0.01)
    else:
        _, dz = Rc.q_loss_and_dz(z, acts, tgt.reshape(-1).astype(np.float64))
    g = Rc.backward(P, fwd, dz, algo)
    return {k: np.asarray(v, np.float32).reshape(P[k].shape) for k, v in g.items()}


def unflat(eng, ns, flat):
    out = {}
    f = flat.cpu().numpy()
    for (name, shp), off, sz in zip(ns, eng.offsets, eng.sizes):
        out[name] = f[off:off + sz].reshape(shp)
    return out


@pytest.mark.parametrize('algo,A,E,n,lives', [('a3c', 6, 8, 5, 0), ('a3c', 4, 6, 3, 5), ('q', 6, 4, 8, 3),
                                               ('a3c', 6, 1, 5, 0), ('a3c', 6, 37, 2, 3)])
def test_engine_matches_oracle(algo, A, E, n, lives):
    check_engine_vs_oracle(algo, A, E, n, lives)


@pytest.mark.parametrize('algo,A,E,n,lives', [('a3c', 6, 8, 5, 0), ('q', 6, 4, 8, 3)])
def test_frame84_mode_matches_oracle(algo, A, E, n, lives):
    """Measurement mode M2: pre-sized 84x84 pool frames copied into the history
    ring instead of Environment.screen of RGB frames; the same parity bar as the RGB mode."""
    check_engine_vs_oracle(algo, A, E, n, lives, frame84=1)


def check_engine_vs_oracle(algo, A, E, n, lives, **kw):
    eng, ref, ns = build(algo, A, E, n, lives, seed=123 + E, target_q_update_step=40, **kw)
    torch.cuda.synchronize()
    # initial env state and history ring
    assert np.array_equal(eng.env_frame.cpu().numpy(), ref.env.frame.astype(np.int32))
    R = eng.ring_slots
    ring = eng.frame_ring.cpu().numpy()
    for c in range(4):
        assert np.array_equal(ring[:, c % R], ref.ring[:, c % R])
    for it in range(3):
        eng.rollout_grad()
        torch.cuda.synchronize()
        acts = eng.actions.cpu().numpy()
        out = ref.iterate(forced_actions=acts)
        # the GPU's own draws agree with the oracle's policy except at fp cdf boundaries
        agree = (acts == out['sampled']).mean()
        assert agree >= 0.98, agree
        assert np.array_equal(eng.rewards.cpu().numpy(), out['rewards'])
        assert np.array_equal(eng.terminals.cpu().numpy(), out['terminals'])
        gr = eng.frame_ring.cpu().numpy()
        bad = [(e, sl, int((gr[e, sl] != ref.ring[e, sl]).sum())) for e in range(E) for sl in range(R)
               if not np.array_equal(gr[e, sl], ref.ring[e, sl])]
        assert not bad, (it, ref.tau, bad, out['terminals'].T.tolist())
        tgt = eng.returns.cpu().numpy()
        np.testing.assert_allclose(tgt, out['target'], rtol=1e-5, atol=1e-5)
        loss = eng.loss.cpu().numpy()
        if algo == 'a3c':
            ref_l = out['losses']
            for i, k in enumerate(('policy', 'value', 'entropy', 'total')):
                # sums of +- per-sample terms: 1e-4 of max(1, |sum|) (north star 1e-3)
                assert abs(loss[i] - ref_l[k]) <= 1e-4 * max(1.0, abs(ref_l[k])), (k, loss[i], ref_l[k])
        else:
            assert abs(loss[0] - out['losses']['loss']) <= 1e-4 * max(1.0, abs(out['losses']['loss']))
        ss = eng.sumsq.cpu().numpy()
        G = unflat(eng, ns, eng.grads)
        # single GPU: the per-tensor clip is fused into apply, so after rollout_grad the buffer
        # holds the raw gradient and sumsq its squared norms
        # backward arithmetic on the GPU's own activations (same ReLU masks): 1e-4
        g_same = gpu_act_grads(eng, ref, algo, A, n, E, ns, tgt)
        for i, (name, _) in enumerate(ns):
            assert rel_l2(G[name], g_same[name]) < 1e-4, (it, name)
            # fully independent fp64 oracle: ReLU-mask flips allowed
            assert rel_l2(G[name], out['grads'][name]) < 2e-2, (it, name)
        eng.apply()
        torch.cuda.synchronize()
        ss = eng.sumsq.cpu().numpy()
        for i, (name, _) in enumerate(ns):
            assert np.isclose(ss[i], np.sum(G[name].astype(np.float64) ** 2), rtol=1e-5), (it, name)
        # the oracle optimizer consumes the same-mask gradients so the two parameter
        # trajectories stay comparable at 1e-5 over iterations
        ref.apply({k: Rc.clip_by_norm(v, 40.0) for k, v in g_same.items()})
        torch.cuda.synchronize()
        P = unflat(eng, ns, eng.params)
        for name, _ in ns:
            d = np.abs(P[name] - ref.params[name]).max()
            assert d <= 1e-5 * max(1.0, np.abs(ref.params[name]).max()), (it, name, d)
        cnt = eng.counters.cpu().numpy()
        assert cnt[0] == ref.tau and cnt[1] == ref.global_step
        for f, ref_v in (('frame', ref.env.frame), ('lives', ref.env.lives), ('episode', ref.env.episode),
                         ('ep_step', ref.env.ep_step), ('ep_len', ref.env.ep_len)):
            assert np.array_equal(eng.env_field(f).cpu().numpy(), ref_v.astype(np.int32)), f
        if algo == 'q':
            T = unflat(eng, ns, eng.target_params)
            for name, _ in ns:
                np.testing.assert_allclose(T[name], ref.tparams[name], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize('overlap', [False, True])
def test_engine_deterministic_and_graph_equals_eager(overlap):
    a, _, ns = build('a3c', 6, 16, 5, 0, seed=7, use_graph=True, overlap=overlap)
    b, _, _ = build('a3c', 6, 16, 5, 0, seed=7, use_graph=False, overlap=overlap)
    for _ in range(4):
        a.iterate()
        b.iterate()
    torch.cuda.synchronize()
    assert torch.equal(a.params, b.params)
    assert torch.equal(a.frame_ring, b.frame_ring)
    assert torch.equal(a.loss, b.loss)


@pytest.mark.parametrize('overlap', [False, True])
def test_fused_iterate_equals_rollout_grad_then_apply(overlap):
    """a3c_engine_iterate (apply captured into the graphs) == a3c_engine_rollout_grad +
    a3c_engine_apply, bit for bit (params, RMSProp slots, frames, losses, counters)."""
    a, _, _ = build('a3c', 6, 16, 5, 0, seed=11, overlap=overlap)
    b, _, _ = build('a3c', 6, 16, 5, 0, seed=11, overlap=overlap)
    for _ in range(5):
        a.iterate()                       # fused path
        b.rollout_grad()                  # split path
        assert a.grad_ready == b.grad_ready
        if b.grad_ready:
            b.apply()
        a.apply()                         # no-op: the fused iterate applied already
    torch.cuda.synchronize()
    for name in ('params', 'ms', 'mom', 'frame_ring', 'loss', 'counters'):
        assert torch.equal(getattr(a, name), getattr(b, name)), name


@pytest.mark.parametrize('overlap', [False, True])
def test_conv_fusion_is_bit_exact(overlap, monkeypatch):
    """k_head_screen_conv12 (step t+1's conv1 + conv2 inside step t's head + screen kernel) gives
    the same rollouts, activations and updates as the separate kernels, bit for bit."""
    engs = []
    monkeypatch.setenv('A3C_FC_SPLIT', '0')     # the same fc kernel in both (see the next test)
    for fuse in ('0', '1'):
        monkeypatch.setenv('A3C_FUSE_CONV', fuse)
        engs.append(build('a3c', 6, 16, 5, 0, seed=13, overlap=overlap)[0])
    a, b = engs
    for _ in range(4):
        a.iterate()
        b.iterate()
    torch.cuda.synchronize()
    for name in ('params', 'ms', 'mom', 'frame_ring', 'loss', 'counters', 'actions', 'act_l1', 'act_l2', 'z'):
        assert torch.equal(getattr(a, name), getattr(b, name)), name


@pytest.mark.parametrize('E', [16, 256])
def test_fc_split_matches_monolithic_fc(E, monkeypatch):
    """Fused overlap rollout: the fc as K-slice partials (k_fc_part) folded by the head of
    k_head_screen_conv12 equals the single-pass fc kernel up to fp32 summation order -- same
    rollouts (actions, frames, rewards), layer outputs and updates to 1e-5."""
    engs = []
    for split in ('0', '1'):
        monkeypatch.setenv('A3C_FC_SPLIT', split)
        engs.append(build('a3c', 6, E, 5, 0, seed=21, overlap=True, frames=512)[0])
    a, b = engs
    for _ in range(4):
        a.iterate()
        b.iterate()
    torch.cuda.synchronize()
    for name in ('actions', 'frame_ring', 'counters'):
        assert torch.equal(getattr(a, name), getattr(b, name)), name
    for name in ('act_l3', 'z', 'params', 'ms', 'mom', 'loss'):
        x, y = getattr(a, name).double(), getattr(b, name).double()
        err = (x - y).norm() / max(y.norm().item(), 1e-30)
        assert err < 1e-5, (name, float(err))


def test_engine_bench_shape_runs():
    """The bench configuration (Pong, 256 envs, n=5) runs and stays finite."""
    eng, _, ns = build('a3c', 6, 256, 5, 0, seed=123, frames=256, scale=1.0)
    for _ in range(3):
        eng.iterate()
    torch.cuda.synchronize()
    assert torch.isfinite(eng.params).all()
    assert torch.isfinite(eng.loss).all()
    acts = eng.actions.cpu().numpy()
    assert acts.min() >= 0 and acts.max() < 6


# ------------------------------------------------------------------ overlap (stale-1) pipeline
def _same_act_grads(slot, planes, P, algo, A, n, E, tgt):
    """oracle backward of one rollout on the engine's saved activations of that rollout's slot."""
    B = n * E
    l1 = slot['act_l1'].cpu().numpy().astype(np.float64).reshape(B, 20, 20, 16)
    l2 = slot['act_l2'].cpu().numpy().astype(np.float64)
    zw = A + 1 if algo == 'a3c' else A
    z = slot['z'].cpu().numpy()[:n].reshape(B, -1)[:, :zw].astype(np.float64)
    fwd = dict(z=z, h3=slot['act_l3'].cpu().numpy().astype(np.float64), flat=l2,
               acts=[Rc.states_nhwc(planes).astype(np.float64) / 255.0, l1, l2.reshape(B, 9, 9, 32)])
    acts = slot['actions'].cpu().numpy().reshape(-1)
    losses, dz = Rc.a3c_loss_and_dz(z, acts, tgt.reshape(-1).astype(np.float64), 0.01)
    g = Rc.backward(P, fwd, dz, algo)
    return losses, {k: np.asarray(v, np.float32).reshape(P[k].shape) for k, v in g.items()}


def test_overlap_with_zero_lr_equals_sync():
    """With learning_rate 0 staleness is invisible: the pipelined engine must reproduce the
    synchronous engine's rollouts exactly (actions, rewards) one call later, and its returns,
    losses and gradients to fp32 summation order (the two modes run different-footprint kernel
    variants, see a3c_shared_gpu)."""
    s, _, _ = build('a3c', 6, 16, 5, 0, seed=31, learning_rate=0.0)
    o, _, _ = build('a3c', 6, 16, 5, 0, seed=31, learning_rate=0.0, overlap=True)
    assert o.ring_slots == 2 * 5 + 4 and s.ring_slots == 5 + 4
    o.iterate()
    torch.cuda.synchronize()
    assert not o.grad_ready
    for k in range(1, 5):
        s.iterate()
        o.iterate()
        torch.cuda.synchronize()
        assert o.grad_ready
        prev = o.slot((k - 1) & 1)
        assert torch.equal(prev['actions'], s.actions), k
        assert torch.equal(prev['rewards'], s.rewards), k
        torch.testing.assert_close(prev['returns'], s.returns, rtol=1e-5, atol=1e-6)
        # the loss terms are sums over n*E samples with cancellation (policy term): fp32
        # summation-order differences between the modes' kernel variants show at ~2e-5 relative
        torch.testing.assert_close(o.loss, s.loss, rtol=1e-4, atol=1e-4)
        # (the conv backward partitions the samples differently per mode: 256 vs 224 workgroup
        # slabs, so dW1's cancelling sums differ in fp32 order, ~1e-5 relative-L2)
        assert rel_l2(o.grads.cpu().numpy(), s.grads.cpu().numpy()) < 5e-5, k
        assert torch.equal(o.params, s.params), k          # lr = 0: parameters never move
    assert int(o.counters[0].item()) == int(s.counters[0].item()) + 5     # one rollout ahead
    assert int(o.counters[1].item()) == int(s.counters[1].item())


@pytest.mark.parametrize('E,frame84', [(8, 0), (8, 1), (1, 0), (37, 0)])
def test_overlap_stale_semantics_match_oracle(E, frame84):
    """Rollout k uses the parameters after update k-2 (staleness 1): replay that order on the
    oracle with the engine's own actions and activations; parameters agree at 1e-5 (RGB frames,
    and the pre-sized 84x84 frames of measurement mode M2; one env, and a ragged 37 that leaves
    partial row blocks in the partial fc, the bootstrap head and the conv backward's groups)."""
    A, n = 6, 5
    eng, ref, ns = build('a3c', A, E, n, 0, seed=77, overlap=True, learning_rate=3e-3, frame84=frame84)
    hist = []                  # per rollout: (oracle params used, planes, oracle out)
    for k in range(5):
        eng.iterate()
        torch.cuda.synchronize()
        sl = eng.slot(k & 1)
        Pk = {kk: v.copy() for kk, v in ref.params.items()}
        out = ref.iterate(forced_actions=sl['actions'].cpu().numpy())
        planes = np.concatenate([np.transpose(ref.states(ref.tau + t), (0, 3, 1, 2)) for t in range(n)])
        ref.tau += n                                    # the rollout owns tau in overlap mode
        assert np.array_equal(sl['rewards'].cpu().numpy(), out['rewards']), k
        assert np.array_equal(sl['terminals'].cpu().numpy(), out['terminals']), k
        ring = eng.frame_ring.cpu().numpy()            # the rollout's new screens, bit-exact
        for t in range(n):
            tt = ref.tau - n + t + 1
            assert np.array_equal(ring[:, tt % eng.ring_slots], ref.ring[:, tt % ref.R]), (k, t)
        agree = (sl['actions'].cpu().numpy() == out['sampled']).mean()
        assert agree >= 0.98, (k, agree)
        hist.append((Pk, planes, out))
        if k == 0:
            assert not eng.grad_ready
            continue
        Pp, planes_p, out_p = hist[k - 1]
        slp = eng.slot((k - 1) & 1)
        tgt = slp['returns'].cpu().numpy()
        np.testing.assert_allclose(tgt, out_p['target'], rtol=1e-5, atol=1e-5)
        losses, g_same = _same_act_grads(slp, planes_p, Pp, 'a3c', A, n, E, tgt)
        loss = eng.loss.cpu().numpy()
        for i, key in enumerate(('policy', 'value', 'entropy', 'total')):
            assert abs(loss[i] - losses[key]) <= 1e-4 * max(1.0, abs(losses[key])), (k, key)
        ref.apply({kk: Rc.clip_by_norm(v, 40.0) for kk, v in g_same.items()}, advance_tau=False)
        P = unflat(eng, ns, eng.params)
        for name, _ in ns:
            d = np.abs(P[name] - ref.params[name]).max()
            assert d <= 1e-5 * max(1.0, np.abs(ref.params[name]).max()), (k, name, d)
        assert int(eng.counters[1].item()) == ref.global_step

def test_stream_ordering_modes_are_bit_identical(monkeypatch):
    """Overlap pipeline: ordering the rollout and backward streams by stream wait-value operations
    on device counters (default) or by HIP events gives the same training, bit for bit."""
    engs = []
    for wv in ('0', '1'):
        monkeypatch.setenv('A3C_WAIT_VALUE', wv)
        engs.append(build('a3c', 6, 32, 5, 0, seed=17, overlap=True, frames=256)[0])
    a, b = engs
    for _ in range(6):
        a.iterate()
        b.iterate()
    torch.cuda.synchronize()
    for name in ('params', 'ms', 'mom', 'frame_ring', 'loss', 'counters', 'actions', 'z'):
        assert torch.equal(getattr(a, name), getattr(b, name)), name


@pytest.mark.parametrize('overlap,frame84', [(False, 0), (True, 0), (True, 1)])
def test_bench_shape_is_deterministic(overlap, frame84):
    """At the bench configuration (Pong, 256 envs, n=5) two engines from the same seed train bit for
    bit alike: every reduction is fixed-order (slab folds, sum of squares), no atomics."""
    engs = [build('a3c', 6, 256, 5, 0, seed=29, frames=512, scale=1.0, overlap=overlap, frame84=frame84)[0]
            for _ in range(2)]
    for _ in range(4):
        for e in engs:
            e.iterate()
    torch.cuda.synchronize()
    a, b = engs
    for name in ('params', 'ms', 'mom', 'frame_ring', 'loss', 'counters', 'actions', 'z', 'act_l3'):
        assert torch.equal(getattr(a, name), getattr(b, name)), name
    assert torch.isfinite(a.params).all() and torch.isfinite(a.loss).all()

"""C5 LSTM policy head (BASELINE config 5, SpaceInvaders-v0 LSTM): HIP kernels and the engine's
recurrent path against the CPU oracle (oracle/ref_cpu.py lstm_*, oracle/engine_ref.py lstm=True).
The reference has no recurrent code, so the oracle is a build-defined restatement of TF1
BasicLSTMCell, pinned by torch autograd (tests/test_oracle_autograd.py) -- parity unpinned
against a reference execution.  Tolerances: cell outputs 1e-5 relative (fp32 MFMA vs fp64),
BPTT gradients 1e-4 relative-L2, engine losses 1e-4 (north star 1e-3)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')

from oracle import ref_cpu as Rc  # noqa: E402
from oracle.engine_ref import EngineRef  # noqa: E402
from _engine_parity import assert_draws_explained  # noqa: E402

U = 256


def rel_l2(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def _lstm_params(seed, scale=0.06):
    rng = np.random.default_rng(seed)
    w = (rng.standard_normal((512, 1024)) * scale).astype(np.float32)
    b = (rng.standard_normal(1024) * 0.1).astype(np.float32)
    return w, b


@pytest.mark.parametrize('B', [1, 16, 37, 256])
def test_lstm_step_matches_oracle(B):
    from src import kernels as K
    rng = np.random.default_rng(B)
    w, b = _lstm_params(B)
    x = np.maximum(rng.standard_normal((B, 256)), 0).astype(np.float32)
    h = (rng.standard_normal((B, U)) * 0.5).astype(np.float32)
    c = (rng.standard_normal((B, U)) * 0.5).astype(np.float32)
    terms = (rng.random(B) < 0.3).astype(np.uint8)
    dev = lambda a: torch.as_tensor(a).cuda()  # noqa: E731
    out = K.lstm_step(dev(w), dev(b), dev(x), dev(h), dev(c), dev(terms))
    torch.cuda.synchronize()
    keep = (1 - terms.astype(np.float64))[:, None]
    hr, cr, gr = Rc.lstm_cell(x.astype(np.float64), h * keep, c * keep, w.astype(np.float64), b.astype(np.float64))
    # fp32 MFMA accumulation over K = 512 of O(1) terms: ~1e-6 absolute on the preactivations
    np.testing.assert_allclose(out['h'].cpu().numpy(), hr, rtol=1e-5, atol=5e-6)
    np.testing.assert_allclose(out['c'].cpu().numpy(), cr, rtol=1e-5, atol=5e-6)
    np.testing.assert_allclose(out['gates'].cpu().numpy(), gr, rtol=1e-5, atol=5e-6)
    assert np.array_equal(out['hp'].cpu().numpy(), (h * keep).astype(np.float32))
    assert np.array_equal(out['cp'].cpu().numpy(), (c * keep).astype(np.float32))
    # no mask / no saved tensors
    out2 = K.lstm_step(dev(w), dev(b), dev(x), dev(h), dev(c), None, save=False)
    hr2, _, _ = Rc.lstm_cell(x.astype(np.float64), h.astype(np.float64), c.astype(np.float64), w.astype(np.float64),
                             b.astype(np.float64))
    np.testing.assert_allclose(out2['h'].cpu().numpy(), hr2, rtol=1e-5, atol=5e-6)


@pytest.mark.parametrize('n,E', [(5, 37), (1, 16), (5, 256)])
def test_lstm_bptt_matches_oracle(n, E):
    from src import kernels as K
    rng = np.random.default_rng(100 + E)
    w, b = _lstm_params(E)
    P = {'lstm_w': w, 'lstm_b': b}
    x = np.maximum(rng.standard_normal((n, E, 256)) - 0.3, 0).astype(np.float32)
    terms = (rng.random((n, E)) < 0.2).astype(np.uint8)
    h0 = (rng.standard_normal((E, U)) * 0.3).astype(np.float32)
    c0 = (rng.standard_normal((E, U)) * 0.3).astype(np.float32)
    seq = Rc.lstm_forward_seq(P, x.astype(np.float64), h0.astype(np.float64), c0.astype(np.float64), terms)
    seq32 = {k: seq[k].astype(np.float32) for k in ('HP', 'CP', 'G', 'C')}
    dH = rng.standard_normal((n, E, U)).astype(np.float32)
    dev = lambda a: torch.as_tensor(np.ascontiguousarray(a)).cuda()  # noqa: E731
    dx, dw, db = K.lstm_bptt(dev(w), dev(x), dev(seq32['HP']), dev(seq32['CP']), dev(seq32['G']), dev(seq32['C']),
                             dev(terms), dev(dH))
    torch.cuda.synchronize()
    s64 = {k: v.astype(np.float64) for k, v in seq32.items()}
    dX, dW, dB = Rc.lstm_backward_seq(P, s64, x.astype(np.float64), dH.astype(np.float64), terms)
    dX = dX * (x > 0)
    assert rel_l2(dx.cpu().numpy(), dX) < 1e-5
    assert rel_l2(dw.cpu().numpy(), dW) < 1e-5
    assert rel_l2(db.cpu().numpy(), dB) < 1e-5


# ------------------------------------------------------------------ engine (C5)
def build(A, E, n, lives, seed, frames=48, scale=4.0, **kw):
    from src.engine import Engine
    from src.initializers import init_params, flatten_host
    from src.kernels import param_names_shapes
    eng = Engine(num_envs=E, n_step=n, action_size=A, algo='a3c', start_lives=lives, num_frames=frames, seed=seed,
                 lstm=True, **kw)
    ns = param_names_shapes(A, 'a3c', lstm=True)
    p = init_params(ns, seed=seed, stddev=0.02 * scale)
    eng.reset(flatten_host(ns, eng.offsets, eng.params.numel(), p))
    ref = EngineRef(p, E, n, A, 'a3c', lives, frames, seed, lstm=True,
                    **{k: v for k, v in kw.items() if k in ('learning_rate',)})
    ref.reset()
    return eng, ref, ns


def unflat(eng, ns, flat):
    f = flat.cpu().numpy()
    return {name: f[off:off + sz].reshape(shp) for (name, shp), off, sz in zip(ns, eng.offsets, eng.sizes)}


def same_act_grads(slot, planes, P, A, n, E, tgt, terms):
    """oracle backward (heads, BPTT, trunk) on the engine's own saved activations and LSTM sequence."""
    B = n * E
    l1 = slot['act_l1'].cpu().numpy().astype(np.float64).reshape(B, 20, 20, 16)
    l2 = slot['act_l2'].cpu().numpy().astype(np.float64)
    z = slot['z'].cpu().numpy()[:n].reshape(B, -1)[:, :A + 1].astype(np.float64)
    h3 = slot['act_l3'].cpu().numpy().astype(np.float64)
    seq = {'H': slot['lstm_h'], 'C': slot['lstm_c'], 'HP': slot['lstm_hp'], 'CP': slot['lstm_cp'],
           'G': slot['lstm_gates']}
    seq = {k: v.cpu().numpy().astype(np.float64) for k, v in seq.items()}
    fwd = dict(z=z, h3=h3, flat=l2, lstm=seq, x_seq=h3.reshape(n, E, -1),
               acts=[Rc.states_nhwc(planes).astype(np.float64) / 255.0, l1, l2.reshape(B, 9, 9, 32)])
    acts = slot['actions'].cpu().numpy().reshape(-1)
    losses, dz = Rc.a3c_loss_and_dz(z, acts, tgt.reshape(-1).astype(np.float64), 0.01)
    g = Rc.lstm_a3c_backward(P, fwd, dz, terms)
    return losses, {k: np.asarray(v, np.float32).reshape(P[k].shape) for k, v in g.items()}


@pytest.mark.parametrize('A,E,n,lives', [(6, 8, 5, 3), (4, 20, 3, 5)])
def test_engine_lstm_matches_oracle(A, E, n, lives):
    eng, ref, ns = build(A, E, n, lives, seed=300 + E, learning_rate=2e-3)
    for it in range(4):
        Pk = unflat(eng, ns, eng.params)
        eng.rollout_grad()
        torch.cuda.synchronize()
        acts = eng.actions.cpu().numpy()
        h0 = ref.hc[0].copy()
        # the rollout's carry-in state = the oracle's carry (computed on its own fp64 forward)
        np.testing.assert_allclose(eng.lstm_hp.cpu().numpy()[0], h0, rtol=1e-4, atol=2e-5)
        out = ref.iterate(forced_actions=acts)
        assert_draws_explained(acts, out, 'a3c', A, it, z_eng=eng.z.cpu().numpy()[:n])
        assert np.array_equal(eng.rewards.cpu().numpy(), out['rewards'])
        terms = eng.terminals.cpu().numpy()
        assert np.array_equal(terms, out['terminals'])
        # per-step policy/value outputs of the recurrent forward
        z = eng.z.cpu().numpy()[:n, :, :A + 1]
        np.testing.assert_allclose(z, out['z'][:, :, :A + 1], rtol=1e-4, atol=2e-5)
        np.testing.assert_allclose(eng.lstm_h.cpu().numpy(), out['lstm']['H'], rtol=1e-4, atol=2e-5)
        tgt = eng.returns.cpu().numpy()
        np.testing.assert_allclose(tgt, out['target'], rtol=1e-4, atol=2e-5)
        planes = np.concatenate([np.transpose(ref.states(ref.tau + t), (0, 3, 1, 2)) for t in range(n)])
        losses, g_same = same_act_grads(eng.slot(0), planes, Pk, A, n, E, tgt, terms)
        loss = eng.loss.cpu().numpy()
        for i, key in enumerate(('policy', 'value', 'entropy', 'total')):
            assert abs(loss[i] - losses[key]) <= 1e-4 * max(1.0, abs(losses[key])), (it, key, loss[i], losses[key])
            assert abs(loss[i] - out['losses'][key]) <= 1e-4 * max(1.0, abs(out['losses'][key])), (it, key)
        G = unflat(eng, ns, eng.grads)
        for name, _ in ns:
            assert rel_l2(G[name], g_same[name]) < 1e-4, (it, name, rel_l2(G[name], g_same[name]))
            assert rel_l2(G[name], out['grads'][name]) < 2e-2, (it, name)
        eng.apply()
        ref.apply({k: Rc.clip_by_norm(v, 40.0) for k, v in g_same.items()})
        torch.cuda.synchronize()
        P = unflat(eng, ns, eng.params)
        for name, _ in ns:
            d = np.abs(P[name] - ref.params[name]).max()
            assert d <= 1e-5 * max(1.0, np.abs(ref.params[name]).max()), (it, name, d)


def test_engine_lstm_overlap_zero_lr_equals_sync():
    """The pipelined engine carries the LSTM state across its two slots exactly as the synchronous
    one does: with lr 0 its rollouts reproduce sync's one call later."""
    s, _, _ = build(6, 16, 5, 3, seed=41, learning_rate=0.0)
    o, _, _ = build(6, 16, 5, 3, seed=41, learning_rate=0.0, overlap=True)
    o.iterate()
    for k in range(1, 5):
        s.iterate()
        o.iterate()
        torch.cuda.synchronize()
        prev = o.slot((k - 1) & 1)
        assert torch.equal(prev['actions'], s.actions), k
        assert torch.equal(prev['terminals'], s.terminals), k
        torch.testing.assert_close(prev['lstm_h'], s.lstm_h, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(o.loss, s.loss, rtol=1e-5, atol=1e-5)
        assert rel_l2(o.grads.cpu().numpy(), s.grads.cpu().numpy()) < 1e-5, k


def test_engine_lstm_bench_shape_runs():
    """BASELINE config 5 per GPU (SpaceInvaders, 256 envs, n=5, LSTM head): runs, finite, graph
    replay equals eager."""
    a, _, _ = build(6, 256, 5, 3, seed=5, frames=256, scale=1.0, overlap=True, use_graph=True)
    b, _, _ = build(6, 256, 5, 3, seed=5, frames=256, scale=1.0, overlap=True, use_graph=False)
    for _ in range(3):
        a.iterate()
        b.iterate()
    torch.cuda.synchronize()
    assert torch.isfinite(a.params).all() and torch.isfinite(a.loss).all()
    assert torch.equal(a.params, b.params)


@pytest.mark.parametrize('E', [40, 256])
def test_engine_lstm_fc_fold_forms_identical(E, monkeypatch):
    """C5's fc fold in either place -- by every cell workgroup (k_lstm_fwd) or once per fc tile by
    the tile's last K-slice workgroup (k_fc_part_fold, an in-launch hand-off through sc1 stores and
    an agent-scope ticket) -- sums the same partials in the same order: bit-identical rollouts and
    updates, overlapped with the backward (uneven load), E = 40 a ragged last tile of both kernels."""
    runs = {}
    for fold in ('0', '1'):
        monkeypatch.setenv('A3C_LSTM_FCFOLD', fold)
        runs[fold], _, _ = build(6, E, 5, 3, seed=77, frames=256, scale=2.0, learning_rate=2e-3, overlap=True,
                                 use_graph=True)
    a, b = runs['0'], runs['1']
    for k in range(6):
        a.iterate()
        b.iterate()
        torch.cuda.synchronize()
        sa, sb = a.slot(k & 1), b.slot(k & 1)
        for key in ('actions', 'z', 'lstm_h', 'lstm_c', 'lstm_gates', 'act_l3'):
            if key in sa:
                assert torch.equal(sa[key], sb[key]), (k, key)
        assert torch.equal(a.loss, b.loss), k
        assert torch.equal(a.params, b.params), k


def test_lstm_rejected_where_unsupported():
    from src import _lib
    from src.kernels import Net  # noqa: F401
    desc = _lib.net_desc(6, 'q', lstm=True)
    with pytest.raises(RuntimeError):
        _lib.param_layout(desc)


@pytest.mark.parametrize('E,frames', [(16, 48), (256, 512)])
def test_engine_lstm_overlap_matches_oracle(E, frames):
    """The pipelined C5 engine (bench.py --lstm: rollout k on the parameters after update k-2) against
    the oracle replayed in that order with the engine's own actions: per-step outputs, returns,
    losses, gradients on the engine's own saved activations and LSTM sequence, and parameters.  The
    fc arrives at the cell as K-slice partials folded by k_lstm_fwd (act_l3 written there)."""
    from _engine_parity import rollout_planes
    A, n = 6, 5
    eng, ref, ns = build(A, E, n, 3, seed=60 + E, frames=frames, scale=2.0, learning_rate=2e-3, overlap=True)
    hist = []
    for k in range(4):
        eng.iterate()
        torch.cuda.synchronize()
        sl = eng.slot(k & 1)
        Pk = {kk: v.copy() for kk, v in ref.params.items()}
        out = ref.iterate(forced_actions=sl['actions'].cpu().numpy(), grads='losses')
        planes = rollout_planes(ref, n)
        ref.tau += n
        assert np.array_equal(sl['rewards'].cpu().numpy(), out['rewards']), k
        assert np.array_equal(sl['terminals'].cpu().numpy(), out['terminals']), k
        assert_draws_explained(sl['actions'].cpu().numpy(), out, 'a3c', A, k,
                               z_eng=sl['z'].cpu().numpy()[:n].reshape(n, E, -1))
        z = sl['z'].cpu().numpy()[:n].reshape(n, E, -1)[:, :, :A + 1]
        np.testing.assert_allclose(z, out['z'][:, :, :A + 1], rtol=1e-4, atol=2e-5)
        hist.append((Pk, planes, out))
        if k == 0:
            continue
        Pp, planes_p, out_p = hist[k - 1]
        slp = eng.slot((k - 1) & 1)
        tgt = slp['returns'].cpu().numpy()
        np.testing.assert_allclose(tgt, out_p['target'], rtol=1e-4, atol=2e-5)
        terms = slp['terminals'].cpu().numpy()
        losses, g_same = same_act_grads(slp, planes_p, Pp, A, n, E, tgt, terms)
        loss = eng.loss.cpu().numpy()
        for i, key in enumerate(('policy', 'value', 'entropy', 'total')):
            assert abs(loss[i] - losses[key]) <= 1e-4 * max(1.0, abs(losses[key])), (k, key, loss[i], losses[key])
            # independent: the oracle's own fp64 lstm_a3c_forward of rollout k-1 and its targets
            ind = out_p['losses'][key]
            assert abs(loss[i] - ind) <= 1e-4 * max(1.0, abs(ind)), ('independent', k, key, loss[i], ind)
        G = unflat(eng, ns, eng.grads)
        for name, _ in ns:
            assert rel_l2(G[name], g_same[name]) < 1e-4, (k, name, rel_l2(G[name], g_same[name]))
        ref.apply({kk: Rc.clip_by_norm(v, 40.0) for kk, v in g_same.items()}, advance_tau=False, tau=out_p['tau'])
        P = unflat(eng, ns, eng.params)
        for name, _ in ns:
            d = np.abs(P[name] - ref.params[name]).max()
            assert d <= 1e-5 * max(1.0, np.abs(ref.params[name]).max()), (k, name, d)

"""Shared checks of the batched engine against the CPU replay oracle (oracle/engine_ref.py).

Test infrastructure only (imported by tests/test_gpu_*.py).  Each check drives the HIP engine
through src/engine.py (the C-ABI) and replays the same iteration on the oracle with the engine's
own action draws, then asserts:
  * env dynamics, rewards, terminals and the frame ring (Environment.screen + History) bit-exact;
  * the engine's draws agree with the oracle's policy except at fp32 cdf boundaries;
  * n-step returns / TD targets within 1e-5;
  * losses within 1e-4 of max(1, |loss|) (north star: 1e-3);
  * gradients within 1e-4 relative-L2 of the fp64 oracle backward on the engine's own saved
    activations (same ReLU masks), and within 2e-2 of the fully independent fp64 forward+backward;
  * parameters after clip + RMSProp within 1e-5 over the iterations.
Reference: agent.py:141-207 (act / observe / batch_update), agent.py:306-321 (loss, clip, apply),
network.py:60-94 + assets/a3c.png (A3C losses, n-step returns), main.py:63-65 (RMSProp)."""
import numpy as np
import torch

from oracle import ref_cpu as Rc
from oracle.engine_ref import EngineRef


def rel_l2(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


REF_KEYS = ('target_q_update_step', 'learning_rate', 'frame84', 'double_q', 'ep_start', 'ep_end_t', 'learn_start',
            'dqn_type')


def build(algo, A, E, n, lives, seed, frames=48, use_graph=False, scale=4.0, **kw):
    """An engine and an oracle from the same seed and initial parameters (stddev 0.02*scale).
    external_env=True: the engine's frames come from host-stepped envs (no device frame pool)."""
    from src.engine import Engine
    from src.initializers import init_params, flatten_host
    from src.kernels import param_names_shapes
    eng_frames = 1 if kw.get('external_env') else frames
    eng = Engine(num_envs=E, n_step=n, action_size=A, algo=algo, start_lives=lives, num_frames=eng_frames, seed=seed,
                 use_graph=use_graph, **kw)
    ns = param_names_shapes(A, algo, dqn_type=kw.get('dqn_type', 'nips'))
    p = init_params(ns, seed=seed, stddev=0.02 * scale)
    eng.reset(flatten_host(ns, eng.offsets, eng.params.numel(), p))
    ref = EngineRef(p, E, n, A, algo, lives, frames, seed, **{k: v for k, v in kw.items() if k in REF_KEYS})
    ref.reset()
    return eng, ref, ns


def unflat(eng, ns, flat):
    f = flat.cpu().numpy()
    return {name: f[off:off + sz].reshape(shp) for (name, shp), off, sz in zip(ns, eng.offsets, eng.sizes)}


def same_act_grads(slot, planes, P, algo, A, n, E, tgt):
    """oracle loss + backward of one rollout on the engine's saved activations of that rollout
    (slot: Engine.slot(k), or the engine itself in sync mode)."""
    g = (lambda k: slot[k]) if isinstance(slot, dict) else (lambda k: getattr(slot, k))
    nature = ('act_l4' in slot) if isinstance(slot, dict) else getattr(slot, 'dqn_type', 'nips') == 'nature'
    B = n * E
    zw = A + 1 if algo == 'a3c' else A
    z = g('z').cpu().numpy()[:n].reshape(B, -1)[:, :zw].astype(np.float64)
    x0 = Rc.states_nhwc(planes).astype(np.float64) / 255.0
    if nature:      # network.py:30-42: conv 32 / 64 / 64 (NHWC), flat 3136, fc 512
        l1 = g('act_l1').cpu().numpy().astype(np.float64).reshape(B, 20, 20, 32)
        l2 = g('act_l2').cpu().numpy().astype(np.float64).reshape(B, 9, 9, 64)
        l3 = g('act_l3').cpu().numpy().astype(np.float64)
        fwd = dict(z=z, h3=g('act_l4').cpu().numpy().astype(np.float64), flat=l3,
                   acts=[x0, l1, l2, l3.reshape(B, 7, 7, 64)])
    else:
        l1 = g('act_l1').cpu().numpy().astype(np.float64).reshape(B, 20, 20, 16)
        l2 = g('act_l2').cpu().numpy().astype(np.float64)
        fwd = dict(z=z, h3=g('act_l3').cpu().numpy().astype(np.float64), flat=l2,
                   acts=[x0, l1, l2.reshape(B, 9, 9, 32)])
    acts = g('actions').cpu().numpy().reshape(-1)
    if algo == 'a3c':
        losses, dz = Rc.a3c_loss_and_dz(z, acts, tgt.reshape(-1).astype(np.float64), 0.01)
    else:
        loss, dz = Rc.q_loss_and_dz(z, acts, tgt.reshape(-1).astype(np.float64))
        losses = dict(loss=loss)
    gr = Rc.backward(P, fwd, dz, algo, 'nature' if nature else 'nips')
    return losses, {k: np.asarray(v, np.float32).reshape(P[k].shape) for k, v in gr.items()}


def rollout_planes(ref, n):
    """[n*E,4,84,84] u8 states of the oracle's current rollout (b = t*E + e); call after
    ref.iterate() (the states hold the frames the rollout produced) and before tau advances."""
    return np.concatenate([np.transpose(ref.states(ref.tau + t), (0, 3, 1, 2)) for t in range(n)])


def _boundary_distance(z, a, u):
    """How far u lies outside action a's interval [cdf[a-1], cdf[a]) of softmax(z) in fp64 (the
    draw rule of ref_cpu.sample_categorical: the first j with cdf[j] > u, else A-1); 0 inside."""
    z = np.asarray(z, np.float64)
    e = np.exp(z - z.max())
    cdf = np.cumsum(e / e.sum())
    lo = cdf[a - 1] if a > 0 else 0.0
    hi = cdf[a] if a < len(z) - 1 else np.inf
    return max(lo - float(u), float(u) - hi, 0.0)


def assert_draws_explained(acts, out, algo, A, tag, z_eng=None, tol=1e-5, tol_self=1e-6):
    """Zero unexplained action mismatches (agent.py:141-151 epsilon-greedy, network.py:72
    categorical draw).  Every engine action equals the oracle's draw on the same Philox word u,
    except where the two fp32 evaluations may legitimately disagree:
      * a3c: u lies within `tol` of the boundary of the engine's action's interval in the oracle's
        own fp64 CDF (its independent forward's logits);
      * q: u >= eps for both (the random branch is exact), and the engine's greedy action's q is
        within `tol` (relative to max(1, |q|)) of the oracle's top value -- a near-tie.
    z_eng [n, E, >= A]: the engine's own saved head rows; the sampler restated on them must put
    every engine action inside its interval to `tol_self` (ulp-level: the fused sampler's expf
    against numpy's exp), which pins the fused head kernel's draw itself."""
    acts = np.asarray(acts).reshape(out['sampled'].shape)
    bad = []
    for t, e in np.argwhere(acts != out['sampled']):
        a, b = int(acts[t, e]), int(out['sampled'][t, e])
        z = out['z'][t][e, :A]
        if algo == 'a3c':
            d = _boundary_distance(z, a, out['u'][t, e])
            why = d <= tol
        else:
            u, eps = float(out['u'][t, e]), float(out['eps'][t, e])
            gap = float(np.max(z) - z[a])
            d = gap / max(1.0, float(np.abs(z).max()))
            why = (u >= eps or abs(u - eps) <= tol) and d <= tol
        if not why:
            bad.append((int(t), int(e), a, b, d))
    assert not bad, (tag, 'unexplained draw mismatches (t, e, engine, oracle, distance)', len(bad), bad[:8])
    if z_eng is not None and algo == 'a3c':
        ze = np.asarray(z_eng, np.float64).reshape(acts.shape + (-1,))[..., :A]
        off = [(int(t), int(e), int(acts[t, e])) for t in range(acts.shape[0]) for e in range(acts.shape[1])
               if _boundary_distance(ze[t, e], acts[t, e], out['u'][t, e]) > tol_self]
        assert not off, (tag, 'engine draw outside its own CDF interval (t, e, action)', len(off), off[:8])
    return len(np.argwhere(acts != out['sampled']))


def assert_z(z_eng, z_ref, A_or_zw, tag, rtol=1e-4):
    """The rollout's saved head rows [n, E, zs] against the oracle's independent fp64 forward."""
    ze = np.asarray(z_eng, np.float64)[..., :A_or_zw]
    zr = np.asarray(z_ref, np.float64)[..., :A_or_zw]
    np.testing.assert_allclose(ze, zr, rtol=rtol, atol=rtol * max(1.0, float(np.abs(zr).max())), err_msg=str(tag))


def assert_losses(loss, ref_losses, algo, tag):
    keys = ('policy', 'value', 'entropy', 'total') if algo == 'a3c' else ('loss',)
    for i, k in enumerate(keys):
        # sums of +- per-sample terms: 1e-4 of max(1, |sum|) (north star 1e-3)
        assert abs(loss[i] - ref_losses[k]) <= 1e-4 * max(1.0, abs(ref_losses[k])), (tag, k, loss[i], ref_losses[k])


def assert_params(eng, ns, ref, tag):
    P = unflat(eng, ns, eng.params)
    for name, _ in ns:
        d = np.abs(P[name] - ref.params[name]).max()
        assert d <= 1e-5 * max(1.0, np.abs(ref.params[name]).max()), (tag, name, d)


def assert_env_state(eng, ref, tag):
    for f, ref_v in (('frame', ref.env.frame), ('lives', ref.env.lives), ('episode', ref.env.episode),
                     ('ep_step', ref.env.ep_step), ('ep_len', ref.env.ep_len)):
        assert np.array_equal(eng.env_field(f).cpu().numpy(), ref_v.astype(np.int32)), (tag, f)


def check_sync_vs_oracle(algo, A, E, n, lives, iters=3, seed=None, frames=48, scale=4.0, independent=True,
                         host_pool=None, **kw):
    """Synchronous engine (rollout_grad + apply): every iteration against the oracle.
    host_pool(seed): a host env pool factory -- the engine then runs with external_env and its
    n env steps are driven by Engine.rollout_host."""
    seed = 123 + E if seed is None else seed
    kw.setdefault('target_q_update_step', 40)
    pool = None
    if host_pool is not None:
        kw['external_env'] = True
    eng, ref, ns = build(algo, A, E, n, lives, seed=seed, frames=frames, scale=scale, **kw)
    if host_pool is not None:
        pool = host_pool(seed)
        eng.begin_host(pool)
    torch.cuda.synchronize()
    if pool is None:
        assert np.array_equal(eng.env_frame.cpu().numpy(), ref.env.frame.astype(np.int32))
    R = eng.ring_slots
    ring = eng.frame_ring.cpu().numpy()
    for c in range(4):
        assert np.array_equal(ring[:, c % R], ref.ring[:, c % R])
    for it in range(iters):
        Pk = unflat(eng, ns, eng.params)          # the parameters this rollout runs with
        if pool is not None:
            eng.rollout_host(pool)
        eng.rollout_grad()
        torch.cuda.synchronize()
        acts = eng.actions.cpu().numpy()
        out = ref.iterate(forced_actions=acts)
        planes = rollout_planes(ref, n)           # after: the rollout's own frames are in the ring
        zw = A + 1 if algo == 'a3c' else A
        z_eng = eng.z.cpu().numpy()[:n].reshape(n, E, -1)
        assert_draws_explained(acts, out, algo, A, it, z_eng=z_eng)
        assert_z(z_eng, out['z'], zw, it)
        assert np.array_equal(eng.rewards.cpu().numpy(), out['rewards']), it
        assert np.array_equal(eng.terminals.cpu().numpy(), out['terminals']), it
        gr = eng.frame_ring.cpu().numpy()
        bad = [(e, sl) for e in range(E) for sl in range(R) if not np.array_equal(gr[e, sl], ref.ring[e, sl])]
        assert not bad, (it, ref.tau, bad[:8])
        tgt = eng.returns.cpu().numpy()
        np.testing.assert_allclose(tgt, out['target'], rtol=1e-5, atol=1e-5)
        assert_losses(eng.loss.cpu().numpy(), out['losses'], algo, it)
        G = unflat(eng, ns, eng.grads)
        # single GPU: the per-tensor clip is fused into apply, so after rollout_grad the buffer
        # holds the raw gradient
        _, g_same = same_act_grads(eng, planes, Pk, algo, A, n, E, tgt)
        for name, _ in ns:
            assert rel_l2(G[name], g_same[name]) < 1e-4, (it, name, rel_l2(G[name], g_same[name]))
            if independent:     # fully independent fp64 oracle: ReLU-mask flips allowed
                assert rel_l2(G[name], out['grads'][name]) < 2e-2, (it, name)
        eng.apply()
        torch.cuda.synchronize()
        ss = eng.sumsq.cpu().numpy()
        for i, (name, _) in enumerate(ns):
            assert np.isclose(ss[i], np.sum(G[name].astype(np.float64) ** 2), rtol=1e-5), (it, name)
        # the oracle optimizer consumes the same-mask gradients so the two parameter
        # trajectories stay comparable at 1e-5 over iterations
        ref.apply({k: Rc.clip_by_norm(v, 40.0) for k, v in g_same.items()})
        assert_params(eng, ns, ref, it)
        cnt = eng.counters.cpu().numpy()
        assert cnt[0] == ref.tau and cnt[1] == ref.global_step
        if pool is None:
            assert_env_state(eng, ref, it)
        if algo == 'q':
            T = unflat(eng, ns, eng.target_params)
            for name, _ in ns:
                np.testing.assert_allclose(T[name], ref.tparams[name], rtol=1e-5, atol=1e-6)
    if pool is not None:
        pool.close()
    return eng, ref


def check_overlap_vs_oracle(A, E, n, lives, rollouts=5, seed=77, frames=48, scale=4.0, algo='a3c', hogwild=False,
                            grads=True, **kw):
    """Overlap (stale-1) pipeline: rollout k uses the parameters after update k-2.  The oracle is
    replayed in that order with the engine's own actions and activations.  algo='q': the TD targets
    of rollout k-1 are formed by its backward, after rollout k, with the target network as it
    stands then (synced by apply k-2 at the latest), so the replay recomputes them from the
    rollout's next-state planes with the oracle's target parameters at that point.
    hogwild=True: the engine runs Engine.iterate_hogwild on a one-shard HogwildPS (the clipped
    gradient of rollout k-1 pushed and the shard pulled under rollout k): the same stale-1 replay."""
    if algo == 'q':
        kw.setdefault('target_q_update_step', 40)
    eng, ref, ns = build(algo, A, E, n, lives, seed=seed, frames=frames, scale=scale, overlap=True, **kw)
    ps = None
    if hogwild:
        from src.hogwild import HogwildPS
        ps = HogwildPS(eng.params)
    hist = []                  # per rollout: (oracle params used, planes, oracle out)
    for k in range(rollouts):
        if ps is not None:
            eng.iterate_hogwild(ps)
        else:
            eng.iterate()
        torch.cuda.synchronize()
        sl = eng.slot(k & 1)
        Pk = {kk: v.copy() for kk, v in ref.params.items()}
        out = ref.iterate(forced_actions=sl['actions'].cpu().numpy(), grads=grads)
        planes = rollout_planes(ref, n)
        if algo == 'q':                                 # s_{t+1} of every step, for the late TD target
            out['next_states'] = np.concatenate([ref.states(ref.tau + t + 1) for t in range(n)])
        ref.tau += n                                    # the rollout owns tau in overlap mode
        assert np.array_equal(sl['rewards'].cpu().numpy(), out['rewards']), k
        assert np.array_equal(sl['terminals'].cpu().numpy(), out['terminals']), k
        ring = eng.frame_ring.cpu().numpy()            # the rollout's new screens, bit-exact
        for t in range(n):
            tt = ref.tau - n + t + 1
            assert np.array_equal(ring[:, tt % eng.ring_slots], ref.ring[:, tt % ref.R]), (k, t)
        zw = A + 1 if algo == 'a3c' else A
        z_eng = sl['z'].cpu().numpy()[:n].reshape(n, E, -1)
        assert_draws_explained(sl['actions'].cpu().numpy(), out, algo, A, k, z_eng=z_eng)
        assert_z(z_eng, out['z'], zw, k)       # the rollout's head rows vs the independent fp64 forward
        hist.append((Pk, planes, out))
        if k == 0:
            assert not eng.grad_ready
            continue
        Pp, planes_p, out_p = hist[k - 1]
        slp = eng.slot((k - 1) & 1)
        tgt = slp['returns'].cpu().numpy()
        want = out_p['target']
        if algo == 'q':
            qn = Rc.forward(ref.tparams, out_p['next_states'], 'q', keep=False)['z']
            if kw.get('double_q'):     # the argmax of the online net the rollout ran (its q rows)
                qo = Rc.forward(Pp, out_p['next_states'], 'q', keep=False)['z']
                want = Rc.td_target_double(out_p['rewards'].reshape(-1), out_p['terminals'].reshape(-1),
                                           qn.astype(np.float32), qo[:, :A].astype(np.float32),
                                           ref.h['discount']).astype(np.float32).reshape(n, E)
            else:
                want = Rc.td_target(out_p['rewards'].reshape(-1), out_p['terminals'].reshape(-1),
                                    qn.astype(np.float32), ref.h['discount']).astype(np.float32).reshape(n, E)
        np.testing.assert_allclose(tgt, want, rtol=1e-5, atol=1e-5)
        losses, g_same = same_act_grads(slp, planes_p, Pp, algo, A, n, E, tgt)
        assert_losses(eng.loss.cpu().numpy(), losses, algo, k)
        if algo == 'a3c':
            # independent: the oracle's own fp64 batch forward of rollout k-1 (its logits, values
            # and bootstrap targets), not the engine's saved activations
            assert_losses(eng.loss.cpu().numpy(), out_p['losses'], algo, ('independent', k))
            assert_z(slp['z'].cpu().numpy()[:n].reshape(n * E, -1), out_p['z_batch'], A + 1, ('z_batch', k))
        G = unflat(eng, ns, eng.grads)
        if ps is not None:     # (hogwild clips the buffer in place before its push)
            g_same_c = {kk: Rc.clip_by_norm(v, 40.0) for kk, v in g_same.items()}
        for name, _ in ns:
            want_g = g_same_c[name] if ps is not None else g_same[name]
            assert rel_l2(G[name], want_g) < 1e-4, (k, name, rel_l2(G[name], want_g))
            if algo == 'a3c' and ps is None:    # (q: the rollout-time oracle targets are not the late ones)
                assert rel_l2(G[name], out_p['grads'][name]) < 2e-2, (k, name)
        ref.apply({kk: Rc.clip_by_norm(v, 40.0) for kk, v in g_same.items()}, advance_tau=False, tau=out_p['tau'])
        assert_params(eng, ns, ref, k)
        if ps is not None:
            assert torch.equal(ps.gather(), eng.params)
        assert int(eng.counters[1].item()) == ref.global_step
        if algo == 'q':
            T = unflat(eng, ns, eng.target_params)
            for name, _ in ns:
                np.testing.assert_allclose(T[name], ref.tparams[name], rtol=1e-5, atol=1e-6)
    if ps is not None:
        ps.close()
    return eng, ref


def check_hogwild1_vs_oracle(A, E, n, lives, iters=3, seed=91, frames=48, scale=4.0, **kw):
    """Hogwild with one worker (src/hogwild.py at world 1): rollout + gradient, per-worker clip,
    unlocked RMSProp push into the sharded PS, pull.  With one worker the push order is fixed, so
    it must equal the oracle's clip + RMSProp step for step."""
    from src.hogwild import HogwildPS
    algo = 'a3c'
    eng, ref, ns = build(algo, A, E, n, lives, seed=seed, frames=frames, scale=scale, **kw)
    ps = HogwildPS(eng.params)
    try:
        for it in range(iters):
            Pk = unflat(eng, ns, eng.params)
            eng.iterate_hogwild(ps)
            torch.cuda.synchronize()
            out = ref.iterate(forced_actions=eng.actions.cpu().numpy())
            planes = rollout_planes(ref, n)
            assert np.array_equal(eng.rewards.cpu().numpy(), out['rewards']), it
            assert np.array_equal(eng.terminals.cpu().numpy(), out['terminals']), it
            tgt = eng.returns.cpu().numpy()
            np.testing.assert_allclose(tgt, out['target'], rtol=1e-5, atol=1e-5)
            losses, g_same = same_act_grads(eng, planes, Pk, algo, A, n, E, tgt)
            assert_losses(eng.loss.cpu().numpy(), losses, algo, it)
            clipped = {k: Rc.clip_by_norm(v, 40.0) for k, v in g_same.items()}
            G = unflat(eng, ns, eng.grads)        # the engine's buffer holds the clipped gradient
            for name, _ in ns:
                assert rel_l2(G[name], clipped[name]) < 1e-4, (it, name)
            ref.apply(clipped)
            assert_params(eng, ns, ref, it)
            assert torch.equal(ps.gather(), eng.params)
            cnt = eng.counters.cpu().numpy()
            assert cnt[0] == ref.tau and cnt[1] == ref.global_step
    finally:
        ps.close()
    return eng, ref

"""Multi-rank engine path on one GPU: 2 or 4 processes (gloo process group over GPU tensors) each
run an engine on their own env shard (env ids rank*E ..), clip per worker, exchange and apply --
the bench.py / main.py N>1 path with RCCL swapped for gloo so it runs on a 1-GPU box (RCCL refuses
two ranks on one device).

Three layers of checks (reference: main.py:58-66 PS, agent.py:316-321 clip + apply):
* the replicas stay bit-identical;
* every rank's per-iteration record (tau, global step, per-tensor hashes of its parameters and of
  its own clipped gradient, the q target net) equals ONE process driving every shard's engine with
  the same exchange done by hand -- a mismatch names the first iteration, field and tensor;
* that hand-driven replay is checked against the CPU oracle (oracle/engine_ref.py): every rank's
  rollout (rewards, terminals, draws, returns / TD targets, losses) and its clipped gradient on
  its own saved activations, and the parameters after EVERY rank's clipped gradient was applied
  as its own RMSProp step in rank order (the reference PS rule) within 1e-5, with the q target
  copy at the same global step (agent.py:166-167) on every rank."""
import hashlib
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


E, N, A, ITERS = 64, 5, 6, 4
TQ = 2000       # q target period: with 64 envs x 5 steps x 4 ranks (1,280 per update) it fires at updates 1 and 3


def _cfg(cfg):
    c = dict(A=A, lives=0, lstm=False, algo='a3c', E=E, n=N, tq=TQ, split=1, ov=False, dqn='nips')
    c.update(cfg or {})
    return c


def _make(rank, world, overlap, cfg=None):
    """Rank `rank`'s engine on env ids rank*E.. (cfg: A, lives, lstm, algo -- Pong A3C by default;
    Breakout A=4 with 5 lives is BASELINE config 3, the LSTM head config 5, algo 'q' the
    reference's own async one-step Q-learning)."""
    from src.engine import Engine
    from src.initializers import init_params, flatten_host
    from src.kernels import param_names_shapes
    c = _cfg(cfg)
    kw = dict(target_q_update_step=c['tq']) if c['algo'] == 'q' else {}
    kw['split_exchange'] = c['split']      # (several ranks: the two-phase exchange, PartitionedPS)
    eng = Engine(num_envs=c['E'], n_step=c['n'], action_size=c['A'], algo=c['algo'], num_frames=64, seed=11,
                 env_id_base=rank * c['E'], world_size=world, overlap=overlap, start_lives=c['lives'],
                 lstm=c['lstm'], dqn_type=c['dqn'], **kw)
    ns = param_names_shapes(c['A'], c['algo'], lstm=c['lstm'], dqn_type=c['dqn'])
    eng.reset(flatten_host(ns, eng.offsets, eng.params.numel(), _init(ns)))
    return eng


def _init(ns):
    from src.initializers import init_params
    return init_params(ns, seed=4, stddev=0.05)


def _sha(t, offsets, sizes):
    """per-tensor hashes of a flat device buffer"""
    a = t.cpu().numpy()
    return [hashlib.sha1(a[o:o + s].tobytes()).hexdigest()[:16] for o, s in zip(offsets, sizes)]


def _record(eng, q):
    c = eng.counters.cpu().numpy()
    rec = dict(tau=int(c[0]), step=int(c[1]), params=_sha(eng.params, eng.offsets, eng.sizes),
               grads=_sha(eng.grads, eng.offsets, eng.sizes))
    if q:
        rec['target'] = _sha(eng.target_params, eng.offsets, eng.sizes)
    return rec


def _first_divergence(ranks, replay, names):
    """(iteration, field, tensor) of the first difference between a rank's records and the
    replay's, or None."""
    for it, (a, b) in enumerate(zip(ranks, replay)):
        for f in ('tau', 'step', 'grads', 'params', 'target'):
            if f not in a:
                continue
            if isinstance(a[f], list):
                for i, (x, y) in enumerate(zip(a[f], b[f])):
                    if x != y:
                        return it, f, names[i]
            elif a[f] != b[f]:
                return it, f, (a[f], b[f])
    if len(ranks) != len(replay):
        return min(len(ranks), len(replay)), 'length', None
    return None


def _worker_env(rank, world, port):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, 'async-rl-tensorflow_amd')]
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK='0')


def _run_ranks(target, world, args):
    import torch.multiprocessing as mp
    ctx = mp.get_context('spawn')
    with ctx.Manager() as m:
        out = m.dict()
        port = _free_port()
        procs = [ctx.Process(target=target, args=(r, world, port, out) + args) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(500)
            assert p.exitcode == 0
        return dict(out)


def _worker(rank, world, port, out, overlap):
    _worker_env(rank, world, port)
    import torch.distributed as dist
    from src.distributed import GradExchange
    dist.init_process_group('gloo')
    eng = _make(rank, world, overlap, dict(E=16))
    xch = GradExchange()
    for _ in range(ITERS):
        eng.iterate(exchange=xch)
    torch.cuda.synchronize()
    out[rank] = dict(params=eng.params.cpu().numpy(), step=int(eng.counters[1].item()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize('overlap', [False, True])
def test_two_ranks_sum_exchange_match_manual_exchange(overlap):
    """--exchange sum (the plain data-parallel rule, kept as a baseline) at world 2."""
    world, e = 2, 16
    res = _run_ranks(_worker, world, (overlap,))
    assert np.array_equal(res[0]['params'], res[1]['params'])
    assert res[0]['step'] == res[1]['step'] == ITERS * N * e * world - (N * e * world if overlap else 0)
    engs = [_make(r, world, overlap, dict(E=e)) for r in range(world)]
    for _ in range(ITERS):
        for x in engs:
            x.rollout_grad()
        if not engs[0].grad_ready:
            continue
        total = engs[0].grads + engs[1].grads
        for x in engs:
            x.grads.copy_(total)
            x.apply()
    torch.cuda.synchronize()
    assert torch.equal(engs[0].params, engs[1].params)
    np.testing.assert_array_equal(engs[0].params.cpu().numpy(), res[0]['params'])


# ------------------------------------------------------- partitioned PS (default multi-GPU exchange)
def _pps_worker(rank, world, port, out, overlap, cfg):
    _worker_env(rank, world, port)
    import torch.distributed as dist
    from src.distributed import PartitionedPS
    dist.init_process_group('gloo')
    eng = _make(rank, world, overlap, cfg)
    q = _cfg(cfg)['algo'] == 'q'
    assert (eng.split_point > 0) == bool(_cfg(cfg)['split'])
    ps = PartitionedPS(eng.params.numel(), split=True)     # two phases on host-staged gloo too
    recs = []
    for _ in range(ITERS):
        eng.iterate(exchange=ps)
        torch.cuda.synchronize()
        recs.append(_record(eng, q))
    out[rank] = dict(params=eng.params.cpu().numpy(), step=int(eng.counters[1].item()), recs=recs)
    dist.barrier()
    dist.destroy_process_group()


class _Oracle:
    """The CPU oracle of a `world`-rank run: one EngineRef per rank shard (the same seeds and env
    ids as the engines), stepped with each engine's own draws; each update applies every rank's
    clipped gradient (oracle backward on that engine's saved activations of the rollout, so the
    ReLU masks are the engine's) as its own RMSProp step, in rank order, to every replica."""

    def __init__(self, world, cfg, ns):
        from oracle.engine_ref import EngineRef
        c = _cfg(cfg)
        self.c, self.ns, self.world = c, ns, world
        kw = dict(target_q_update_step=c['tq']) if c['algo'] == 'q' else {}
        self.refs = [EngineRef(_init(ns), c['E'], c['n'], c['A'], c['algo'], c['lives'], 64, 11,
                               env_id_base=r * c['E'], world_size=world, dqn_type=c['dqn'], **kw)
                     for r in range(world)]
        for ref in self.refs:
            ref.reset()
        self.hist = [[] for _ in range(world)]

    def rollout(self, k, engs, overlap):
        """The oracle's rollout k of every rank, checked against the engines' (call after
        rollout_grad k); returns the rollout's parameters."""
        from tests._engine_parity import rollout_planes
        c = self.c
        Pk = {kk: v.copy() for kk, v in self.refs[0].params.items()}
        for r, (eng, ref) in enumerate(zip(engs, self.refs)):
            sl = eng.slot(k & 1) if overlap else {kk: getattr(eng, kk) for kk in ('actions', 'rewards', 'terminals')}
            acts = sl['actions'].cpu().numpy()
            out = ref.iterate(forced_actions=acts, grads=False)
            planes = rollout_planes(ref, c['n'])
            if overlap and c['algo'] == 'q':      # s_{t+1} planes for the backward-time TD targets
                out['next_states'] = np.concatenate([ref.states(ref.tau + t + 1) for t in range(c['n'])])
            if overlap:
                ref.tau += c['n']                 # the rollout owns tau in overlap mode
            assert np.array_equal(sl['rewards'].cpu().numpy(), out['rewards']), (k, r)
            assert np.array_equal(sl['terminals'].cpu().numpy(), out['terminals']), (k, r)
            from tests._engine_parity import assert_draws_explained
            z_eng = (sl['z'] if overlap else eng.z).cpu().numpy()[:c['n']].reshape(c['n'], c['E'], -1)
            assert_draws_explained(acts, out, c['algo'], c['A'], (k, r), z_eng=z_eng)
            self.hist[r].append((Pk, planes, out))
        return Pk

    def gradients(self, j, engs, overlap):
        """Every rank's clipped gradient of rollout j against the engine's (grads buffer)."""
        from oracle import ref_cpu as Rc
        from tests._engine_parity import same_act_grads, assert_losses, unflat, rel_l2
        c, out_c = self.c, []
        for r, eng in enumerate(engs):
            Pj, planes, out = self.hist[r][j]
            sl = eng.slot(j & 1) if overlap else eng
            ret = (sl['returns'] if overlap else sl.returns).cpu().numpy()
            want = out['target']
            if 'next_states' in out:              # q overlap: the target net of backward time
                qn = Rc.forward(self.refs[r].tparams, out['next_states'], 'q', keep=False)['z']
                want = Rc.td_target(out['rewards'].reshape(-1), out['terminals'].reshape(-1), qn.astype(np.float32),
                                    self.refs[r].h['discount']).astype(np.float32).reshape(c['n'], c['E'])
            np.testing.assert_allclose(ret, want, rtol=1e-5, atol=1e-5)
            losses, g = same_act_grads(sl, planes, Pj, c['algo'], c['A'], c['n'], c['E'], ret)
            assert_losses(eng.loss.cpu().numpy(), losses, c['algo'], (j, r))
            clipped = {kk: Rc.clip_by_norm(v, 40.0) for kk, v in g.items()}
            G = unflat(eng, self.ns, eng.grads)             # world > 1: the engine clipped per worker
            for name, _ in self.ns:
                err = rel_l2(G[name], clipped[name])
                assert err < 1e-4, (j, r, name, err)
            out_c.append(clipped)
        return out_c

    def update(self, j, clipped, engs, overlap):
        from tests._engine_parity import assert_params, unflat
        tau = self.hist[0][j][2]['tau']
        for ref in self.refs:
            ref.apply_sequence(clipped, advance_tau=not overlap, tau=tau)
        for r, eng in enumerate(engs):
            assert_params(eng, self.ns, self.refs[r], (j, r))
            cnt = eng.counters.cpu().numpy()
            assert cnt[1] == self.refs[r].global_step, (j, r)
            if not overlap:
                assert cnt[0] == self.refs[r].tau, (j, r)
            if self.c['algo'] == 'q':
                T = unflat(eng, self.ns, eng.target_params)
                for name, _ in self.ns:
                    np.testing.assert_allclose(T[name], self.refs[r].tparams[name], rtol=1e-5, atol=1e-6)


@pytest.mark.timeout(900)
@pytest.mark.parametrize('world,overlap,cfg,oracle', [
    (2, False, {}, False), (2, True, {}, False), (4, False, {}, True), (4, True, {}, False),
    (4, True, dict(A=4, lives=5), True), (4, False, dict(A=6, lives=3, lstm=True, E=16), False),
    (4, False, dict(algo='q', A=6, lives=3), True), (2, False, dict(algo='q', A=4, lives=5, n=8), False),
    (4, True, dict(split=0), False), (2, False, dict(split=0), False),
    (2, True, dict(algo='q', A=6, lives=3, tq=700), True), (4, True, dict(algo='q', A=4, lives=5, tq=700), False),
    (2, False, dict(dqn='nature', split=0, E=24), True), (2, True, dict(dqn='nature', split=0, E=24, A=4, lives=5), True)],
    ids=['w2-sync', 'w2-overlap', 'w4-sync', 'w4-overlap', 'w4-breakout-overlap', 'w4-lstm-sync', 'w4-q-sync',
         'w2-q-breakout-sync', 'w4-overlap-onephase', 'w2-sync-onephase', 'w2-q-overlap', 'w4-q-breakout-overlap',
         'w2-nature-sync', 'w2-nature-breakout-overlap'])
def test_partitioned_ps_ranks(world, overlap, cfg, oracle):
    """`world` ranks on one GPU (gloo, host-staged collectives) run the default multi-GPU exchange:
    all-to-all of the clipped gradients, each rank's W sequential RMSProp steps on its range,
    all-gather -- by default in two phases (the fc / head range on a comm stream under the conv
    backward, then the conv prefix: `split`), `onephase` ids after the whole backward.  Replicas stay identical; every rank's per-iteration record equals one process
    driving every shard through the same C-ABI by hand (first divergence named); in sync mode that
    also equals applying every rank's clipped gradient, in rank order, to full copies with
    a3c_rmsprop_range (the reference PS rule, main.py:60-65); `oracle`: the replay against the CPU
    oracle (module docstring)."""
    import ctypes
    from src._lib import lib, ptr, stream_handle
    from src.distributed import shard_ranges
    from src.kernels import param_names_shapes
    c = _cfg(cfg)
    q = c['algo'] == 'q'
    res = _run_ranks(_pps_worker, world, (overlap, cfg))
    per_update = c['n'] * c['E'] * world
    for r in range(1, world):
        assert np.array_equal(res[0]['params'], res[r]['params']), r
        assert res[0]['step'] == res[r]['step'] == ITERS * per_update - (per_update if overlap else 0)
    ns = param_names_shapes(c['A'], c['algo'], lstm=c['lstm'], dqn_type=c['dqn'])
    names = [nm for nm, _ in ns]
    engs = [_make(r, world, overlap, cfg) for r in range(world)]
    orc = _Oracle(world, cfg, ns) if oracle else None
    total = engs[0].params.numel()
    shard, lo, n = shard_ranges(total, world)
    w_out = [torch.zeros(shard, device='cuda') for _ in range(world)]
    if not overlap:
        w = engs[0].params.clone()
        ms, mom = torch.ones_like(w), torch.zeros_like(w)
    recs = [[] for _ in range(world)]
    for k in range(ITERS):
        for e in engs:
            e.rollout_grad()
        torch.cuda.synchronize()
        if orc:
            orc.rollout(k, engs, overlap)
        if engs[0].grad_ready:
            j = k - 1 if overlap else k                     # the rollout whose gradient is exchanged
            clipped = orc.gradients(j, engs, overlap) if orc else None
            if not overlap:
                for e in engs:
                    lib().a3c_rmsprop_range(ptr(w), ptr(ms), ptr(mom), ptr(e.grads), total,
                                            ctypes.c_void_p(e.sched_ptr), 0.0, 0.99, 0.0, 0.1, stream_handle())
            for r, e in enumerate(engs):
                recv = torch.cat([engs[x].grads[lo[r]:lo[r] + n[r]] for x in range(world)])
                e.apply_shard(recv, world, lo[r], n[r], w_out[r])
            gathered = torch.cat(w_out)
            for e in engs:
                e.apply_commit(gathered)
            torch.cuda.synchronize()
            if orc:
                orc.update(j, clipped, engs, overlap)
        for r, e in enumerate(engs):
            recs[r].append(_record(e, q))
    torch.cuda.synchronize()
    for r in range(world):
        d = _first_divergence(res[r]['recs'], recs[r], names)
        assert d is None, f'rank {r} diverges from the by-hand replay at (iteration, field, tensor) {d}'
    for e in engs[1:]:
        assert torch.equal(engs[0].params, e.params)
    np.testing.assert_array_equal(engs[0].params.cpu().numpy(), res[0]['params'])
    if not overlap:
        np.testing.assert_array_equal(w.cpu().numpy(), res[0]['params'])
    if q:   # the target copy fired (at the same global step on every rank: the records are equal)
        assert any(a['target'] != b['target'] for a, b in zip(recs[0], recs[0][1:]))


@pytest.mark.timeout(600)
@pytest.mark.parametrize('overlap', [False, True], ids=['sync', 'overlap'])
def test_split_exchange_equals_one_phase(overlap):
    """The two-phase exchange (fc / head range under the conv backward, then the conv prefix) and
    the one-phase exchange after the whole backward, from one seed at world 2: the backward of
    either sums every gradient in the same order (the split backward takes the fc weight GEMM form
    of the one-phase backward of the same configuration, net_bwd.hip), so the parameters, counters
    and per-iteration records are bit-identical."""
    two = _run_ranks(_pps_worker, 2, (overlap, dict(split=1)))
    one = _run_ranks(_pps_worker, 2, (overlap, dict(split=0)))
    for r in range(2):
        np.testing.assert_array_equal(two[r]['params'], one[r]['params'])
        assert two[r]['step'] == one[r]['step']
        assert two[r]['recs'] == one[r]['recs'], r


# ------------------------------------------------------------------ Hogwild (SURVEY §8(e) async)
def _hog_worker(rank, world, port, out, lockstep, cfg):
    _worker_env(rank, world, port)
    import torch.distributed as dist
    from src.hogwild import HogwildPS
    dist.init_process_group('gloo')
    ov = _cfg(cfg)['ov']
    eng = _make(rank, world, ov, cfg)
    ps = HogwildPS(eng.params)
    for it in range(ITERS):
        if lockstep:                      # deterministic order for the check: rank 0, then rank 1, ...
            # the production call in each rank's turn: rollout k (overlap: and the backward of k-1),
            # the push of the clipped gradient, the pull into the next rollout's snapshot, the commit
            for turn in range(world):
                dist.barrier()
                if turn == rank:
                    eng.iterate_hogwild(ps)
                    torch.cuda.synchronize()
            dist.barrier()
        else:
            eng.iterate_hogwild(ps)
    torch.cuda.synchronize()
    dist.barrier()
    out[rank] = dict(shared=ps.gather().cpu().numpy(), params=eng.params.cpu().numpy(),
                     target=eng.target_params.cpu().numpy(), step=int(eng.counters[1].item()),
                     finite=bool(torch.isfinite(eng.params).all().item()))
    ps.close()
    dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize('world,lockstep,cfg', [(2, True, {}), (2, False, {}), (4, True, {}), (4, False, {}),
                                                (2, True, dict(algo='q', tq=300)), (4, True, dict(algo='q', A=4, lives=5, tq=300)),
                                                (2, True, dict(ov=True)), (4, False, dict(ov=True)),
                                                (2, True, dict(algo='q', tq=300, ov=True)),
                                                (2, True, dict(dqn='nature', split=0)),
                                                (2, True, dict(dqn='nature', split=0, ov=True))],
                         ids=['w2-lockstep', 'w2-free', 'w4-lockstep', 'w4-free', 'w2-q-lockstep',
                              'w4-q-breakout-lockstep', 'w2-overlap-lockstep', 'w4-overlap-free',
                              'w2-q-overlap-lockstep', 'w2-nature-lockstep', 'w2-nature-overlap-lockstep'])
def test_hogwild_sharded_ps(world, lockstep, cfg):
    """`world` ranks on one GPU push into each other's IPC-mapped shards.  Lock-step: each rank runs
    the production Engine.iterate_hogwild in its turn (rollout, push, pull, commit), which must
    equal a single process applying every rank's clipped gradient in rank order, each rank pulling
    right after its own push (q: and copying the target net at the same global step); free-running
    (the real unlocked mode) must stay finite with every rank seeing the same shared params."""
    c = _cfg(dict(cfg, E=16))
    cfg = dict(cfg, E=16)
    res = _run_ranks(_hog_worker, world, (lockstep, cfg))
    for r in range(1, world):
        np.testing.assert_array_equal(res[0]['shared'], res[r]['shared'])
    assert all(res[r]['finite'] for r in range(world))
    if not lockstep:
        return
    # replay: the engines, one shared RMSProp state applied in the same order
    import ctypes
    from src._lib import lib, ptr, stream_handle
    engs = [_make(r, world, c['ov'], cfg) for r in range(world)]
    w = engs[0].params.clone()
    ms, mom = torch.ones_like(w), torch.zeros_like(w)
    for it in range(ITERS):
        for e in engs:          # rank order: each rank's push lands before the next rank's turn
            e.rollout_grad()
            if not e.grad_ready:                # (overlap: the pipeline's first rollout)
                continue
            lib().a3c_rmsprop_range(ptr(w), ptr(ms), ptr(mom), ptr(e.grads), w.numel(), ctypes.c_void_p(e.sched_ptr),
                                    0.0, 0.99, 0.0, 0.1, stream_handle())
            e.params.copy_(w)   # its pull sees every push so far
            e.apply_commit(None)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(w.cpu().numpy(), res[0]['shared'])
    for r in range(world):
        np.testing.assert_array_equal(engs[r].params.cpu().numpy(), res[r]['params'])
        np.testing.assert_array_equal(engs[r].target_params.cpu().numpy(), res[r]['target'])
        assert res[r]['step'] == (ITERS - (1 if c['ov'] else 0)) * c['n'] * c['E'] * world
    if c['algo'] == 'q':    # the target copy fired (tq 300: at updates 1 and 3 at world 2, every update at 4)
        assert not np.array_equal(res[0]['target'], _make(0, world, False, cfg).target_params.cpu().numpy())

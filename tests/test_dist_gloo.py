"""CPU (gloo) tests at world sizes 2, 4 and 8 of the multi-GPU update paths (src/distributed.py).

Each rank runs the oracle iteration on its own env shard (env ids rank*E..) and clips per tensor
(agent.py:319).  Then:
* PartitionedPS (the default exchange): the real all-to-all / all-gather protocol drives a
  CPU stand-in of the engine's shard apply (oracle RMSProp on flat arrays).  The replicas must
  stay bit-identical and equal ONE process applying every rank's clipped gradient, in rank order,
  as W RMSProp steps (EngineRef.apply_sequence) -- the reference PS's rule (main.py:63-65,
  agent.py:321) in rank order.
* GradExchange (``--exchange sum``): SUM all-reduce, one step of the sum, for comparison.
And, without processes: the summed single step is NOT the reference's W steps."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup_paths():
    import sys
    for p in (ROOT, os.path.join(ROOT, 'async-rl-tensorflow_amd')):
        if p not in sys.path:
            sys.path.insert(0, p)


def aligned_layout(ns, align=64):
    """The engine's flat layout (include/a3c_hip.h a3c_param_layout): TF variable order, every
    tensor 64-float aligned, total rounded up to 64 -- so the shard ranges below are the ones the
    real engine exchanges (678,144 floats for Pong, 677,632 for Breakout, 1,203,456 with LSTM)."""
    offs, off = [], 0
    for _, shp in ns:
        offs.append(off)
        off = -(-(off + int(np.prod(shp))) // align) * align
    return offs, off


class _CpuShardEngine:
    """The engine's partitioned-PS interface (apply_shard / apply_commit) over an EngineRef:
    flat float32 params / ms / mom in the engine's aligned layout, RMSProp from oracle/ref_cpu."""

    def __init__(self, ref, ns, split=False):
        self.ref, self.ns = ref, ns
        self.offs, self.total = aligned_layout(ns)
        # the engine's split exchange: the fc / head range (from the fc weights on) first
        self.split_point = self.offs[4] if split else 0
        self.ms, self.mom = self.flat(ref.ms, 1.0), self.flat(ref.mom)
        self.grads = None

    def flat(self, d, pad=0.0):
        out = np.full(self.total, pad, np.float32)
        for (name, _), off in zip(self.ns, self.offs):
            v = np.asarray(d[name], np.float32).reshape(-1)
            out[off:off + v.size] = v
        return out

    def set_grads(self, clipped):
        self.grads = torch.as_tensor(self.flat(clipped))

    def apply_shard(self, recv, nranks, lo, n, w_out):
        from oracle import ref_cpu as R
        h = self.ref.h
        lr = self.ref.next_lr()
        w = self.flat(self.ref.params)[lo:lo + n].copy()
        g = recv.numpy()[:nranks * n].reshape(nranks, n)
        for q in range(nranks):                     # rank order: one arrival order of the PS
            R.rmsprop_apply(w, self.ms[lo:lo + n], self.mom[lo:lo + n], g[q], lr, h['decay'], h['momentum'],
                            h['epsilon'])
        w_out[:n] = torch.as_tensor(w)

    def apply_commit(self, gathered):
        flat = gathered.numpy()[:self.total]
        for (name, shp), off in zip(self.ns, self.offs):
            self.ref.params[name] = flat[off:off + int(np.prod(shp))].reshape(shp).astype(np.float32).copy()
        self.ref.finish_update()


def _init(rank, world, port):
    _setup_paths()
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from src.distributed import init_from_env
    r, w, _ = init_from_env(backend='gloo')
    assert (r, w) == (rank, world)


def _shared_start(rank, A=6, lstm=False, algo='a3c'):
    """Every rank starts from rank 0's parameters (broadcast, as main.py / bench.py do)."""
    from src.distributed import broadcast_params
    from src.initializers import init_params
    from src.kernels import param_names_shapes
    ns = param_names_shapes(A, algo, lstm=lstm)
    p = init_params(ns, seed=5 + rank, stddev=0.08)       # different on purpose: broadcast fixes it
    names = [n for n, _ in ns]
    flat = torch.cat([torch.as_tensor(p[n]).reshape(-1) for n in names])
    broadcast_params(flat, src=0)
    sizes = [int(np.prod(s)) for _, s in ns]
    parts = torch.split(flat, sizes)
    return {n: parts[i].reshape(s).numpy().copy() for i, (n, s) in enumerate(ns)}, ns


def _ref(p, rank, world, cfg):
    from oracle.engine_ref import EngineRef
    E = cfg.get('E', 3)
    algo = cfg.get('algo', 'a3c')
    kw = dict(target_q_update_step=cfg['tq']) if 'tq' in cfg else {}
    ref = EngineRef(p, E, 2, cfg.get('A', 6), algo, cfg.get('lives', 0), 16, seed=9, env_id_base=rank * E,
                    world_size=world, lstm=cfg.get('lstm', False), **kw)
    ref.reset()
    return ref


def _worker_partitioned(rank, world, port, out, cfg):
    _init(rank, world, port)
    from src.distributed import PartitionedPS
    p, ns = _shared_start(rank, cfg.get('A', 6), cfg.get('lstm', False), cfg.get('algo', 'a3c'))
    ref = _ref(p, rank, world, cfg)
    eng = _CpuShardEngine(ref, ns, split=cfg.get('split', False))
    ps = PartitionedPS(eng.total, device='cpu')
    mine = []
    for it in range(cfg.get('iters', 3)):
        o = ref.iterate()
        eng.set_grads(o['clipped'])
        mine.append(eng.grads.numpy().copy())
        ps.apply(eng)
    out[rank] = dict(params=eng.flat(ref.params), grads=mine, ms=eng.ms.copy(), lo=ps.lo, n=ps.n,
                     step=ref.global_step, target=eng.flat(ref.tparams))
    dist.barrier()
    dist.destroy_process_group()


def _worker_sum(rank, world, port, out, cfg):
    _init(rank, world, port)
    from src.distributed import GradExchange
    p, ns = _shared_start(rank)
    names = [n for n, _ in ns]
    ref = _ref(p, rank, world, cfg)
    xch = GradExchange()
    for it in range(2):
        o = ref.iterate()
        g = torch.cat([torch.as_tensor(o['clipped'][n]).reshape(-1) for n in names])
        xch(g)                                             # SUM over ranks
        gs = torch.split(g, [ref.params[n].size for n in names])
        ref.apply({n: gs[i].reshape(ref.params[n].shape).numpy().copy() for i, n in enumerate(names)})
    out[rank] = dict(params=np.concatenate([ref.params[n].reshape(-1) for n in names]))
    dist.barrier()
    dist.destroy_process_group()


def _spawn(fn, world=2, cfg=None):
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(fn, args=(world, port, out, dict(cfg or {})), nprocs=world, join=True)
        return dict(out)


def _replay(world, iters, combine, cfg=None):
    """Single process: every shard's EngineRef from rank 0's parameters, combine(refs, outs)."""
    _setup_paths()
    from src.initializers import init_params
    from src.kernels import param_names_shapes
    cfg = dict(cfg or {})
    ns = param_names_shapes(cfg.get('A', 6), cfg.get('algo', 'a3c'), lstm=cfg.get('lstm', False))
    names = [n for n, _ in ns]
    p = init_params(ns, seed=5, stddev=0.08)               # rank 0's params (broadcast source)
    refs = [_ref(p, r, world, cfg) for r in range(world)]
    for _ in range(iters):
        combine(refs, [r.iterate() for r in refs], names)
    return refs[0], ns


def _check_partitioned(world, cfg):
    res = _spawn(_worker_partitioned, world, cfg)
    for r in range(1, world):
        assert np.array_equal(res[0]['params'], res[r]['params']), r           # replicas identical
    assert not np.allclose(res[0]['grads'][0], res[1]['grads'][0])             # different shards, grads
    lo, n = res[0]['lo'], res[0]['n']
    total = res[0]['params'].size
    assert sum(n) == total and all(lo[r + 1] == lo[r] + n[r] for r in range(world - 1))
    assert all(x % 64 == 0 for x in lo)

    def sequential(refs, outs, names):
        for r in refs:
            r.apply_sequence([o['clipped'] for o in outs])             # rank 0's step, then rank 1's, ...
    ref0, ns = _replay(world, cfg.get('iters', 3), sequential, cfg)
    np.testing.assert_array_equal(res[0]['params'], _CpuShardEngine(ref0, ns).flat(ref0.params))
    assert res[0]['step'] == ref0.global_step
    for r in range(world):      # q: every rank copied its target net at the same global step
        np.testing.assert_array_equal(res[r]['target'], _CpuShardEngine(ref0, ns).flat(ref0.tparams))
    return res


@pytest.mark.timeout(300)
def test_gloo_two_rank_partitioned_ps_is_the_reference_ps_rule():
    _check_partitioned(2, {})


@pytest.mark.timeout(600)
@pytest.mark.parametrize('world', [2, 4])
def test_gloo_split_exchange_is_the_reference_ps_rule(world):
    """The two-phase exchange (fc / head range first, then the conv prefix -- held by rank 0's range)
    gives the same replicas as the one-phase exchange: W sequential oracle RMSProp steps."""
    _check_partitioned(world, dict(A=6, split=True))


@pytest.mark.timeout(600)
@pytest.mark.parametrize('cfg', [dict(A=6), dict(A=4, lives=5), dict(A=4, lives=5, split=True)],
                         ids=['pong', 'breakout', 'breakout-split'])
def test_gloo_eight_rank_partitioned_ps_is_the_reference_ps_rule(cfg):
    """BASELINE configs 3/4 are 8-GPU runs: 8 ranks, 8 sequential RMSProp steps per range, and
    the last 64-aligned range ragged (Pong: 7 x 84,800 + 84,544 of 678,144 floats; Breakout:
    7 x 84,736 + 84,480 of 677,632)."""
    res = _check_partitioned(8, dict(cfg, iters=2))
    n = res[0]['n']
    assert n[-1] < n[0] and len(set(n[:-1])) == 1


@pytest.mark.timeout(600)
def test_gloo_four_rank_partitioned_ps_lstm_head():
    """C5 (LSTM head, 1,203,456 floats) through the same exchange at world 4."""
    _check_partitioned(4, dict(A=6, lives=3, lstm=True, iters=2))


@pytest.mark.timeout(600)
@pytest.mark.parametrize('world', [2, 4])
def test_gloo_partitioned_ps_async_q_learning(world):
    """The reference's own running path, async one-step Q-learning (agent.py:153-207, main.py:60-66),
    through the partitioned PS: every rank's clipped TD-loss gradient is its own RMSProp step in
    rank order, and the target net (agent.py:166-167, 342-344) is copied at the same global step T
    on every rank (tq 30 with 2 steps x 3 envs x world per update: at update 1 and later)."""
    cfg = dict(algo='q', A=4, lives=5, tq=30, iters=3)
    res = _check_partitioned(world, cfg)
    p0, ns = _shared_start_host(cfg)
    assert not np.array_equal(res[0]['target'], p0)    # the copy happened


def _shared_start_host(cfg):
    _setup_paths()
    from src.initializers import init_params
    from src.kernels import param_names_shapes
    ns = param_names_shapes(cfg.get('A', 6), cfg.get('algo', 'a3c'))
    p = init_params(ns, seed=5, stddev=0.08)
    offs, total = aligned_layout(ns)
    flat = np.zeros(total, np.float32)
    for (name, _), off in zip(ns, offs):
        flat[off:off + p[name].size] = p[name].reshape(-1)
    return flat, ns


@pytest.mark.timeout(300)
def test_gloo_two_rank_sum_exchange():
    world = 2
    res = _spawn(_worker_sum, world)
    assert np.array_equal(res[0]['params'], res[1]['params'])

    def summed(refs, outs, names):
        s = {n: sum(o['clipped'][n] for o in outs).astype(np.float32) for n in names}
        for r in refs:
            r.apply(s)
    ref0, ns = _replay(world, 2, summed)
    flat = np.concatenate([ref0.params[n].reshape(-1) for n, _ in ns])
    np.testing.assert_allclose(res[0]['params'], flat, rtol=1e-6, atol=1e-9)


def test_summed_step_is_not_the_reference_ps_rule():
    """Once the rms slot has adapted, one RMSProp step of the sum of W equal gradients moves
    about lr*sign(g) per iteration, while the reference's W separate pushes move about
    W*lr*sign(g): the summed rule learns up to W times slower."""
    _setup_paths()
    from oracle import ref_cpu as R
    W, lr, iters = 8, 7e-4, 1000
    g = np.full(64, 0.5, np.float32)

    def run(steps_per_iter, grad):
        v, ms, mom = np.zeros(64, np.float32), np.ones(64, np.float32), np.zeros(64, np.float32)
        for _ in range(iters):
            before = float(v[0])
            for _ in range(steps_per_iter):
                R.rmsprop_apply(v, ms, mom, grad, lr)
        return before - float(v[0])                                    # last iteration's move
    seq = run(W, g)                                                    # the reference PS
    summed = run(1, (W * g).astype(np.float32))                        # all-reduce + one step
    assert seq > 0.0 and summed > 0.0
    assert seq / summed > 0.75 * W

"""World-size-2 CPU (gloo) test of the multi-GPU gradient exchange semantics used by bench.py:
each rank runs the oracle iteration on its own env shard (env ids rank*E..), clips per tensor
(agent.py:319), GradExchange SUM-all-reduces, every rank applies RMSProp; the replicas must stay
bit-identical and equal a single-process application of the summed clipped gradients."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, 'async-rl-tensorflow_amd')]
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from src.distributed import GradExchange, broadcast_params, init_from_env
    from src.initializers import init_params
    from src.kernels import param_names_shapes
    from oracle.engine_ref import EngineRef
    from oracle import ref_cpu as R
    r, w, _ = init_from_env(backend='gloo')
    assert (r, w) == (rank, world)
    ns = param_names_shapes(6, 'a3c')
    p = init_params(ns, seed=5 + rank, stddev=0.08)       # different on purpose: broadcast fixes it
    names = [n for n, _ in ns]
    flat = torch.cat([torch.as_tensor(p[n]).reshape(-1) for n in names])
    broadcast_params(flat, src=0)
    sizes = [int(np.prod(s)) for _, s in ns]
    parts = torch.split(flat, sizes)
    p = {n: parts[i].reshape(s).numpy().copy() for i, (n, s) in enumerate(ns)}
    ref = EngineRef(p, 3, 2, 6, 'a3c', 0, 16, seed=9, env_id_base=rank * 3, world_size=world)
    ref.reset()
    xch = GradExchange()
    history = []
    for it in range(2):
        o = ref.iterate()
        g = torch.cat([torch.as_tensor(o['clipped'][n]).reshape(-1) for n in names])
        mine = g.clone()
        xch(g)                                             # SUM over ranks
        gs = torch.split(g, sizes)
        summed = {n: gs[i].reshape(ref.params[n].shape).numpy().copy() for i, n in enumerate(names)}
        ref.apply(summed)
        history.append(mine.numpy())
    flat_p = np.concatenate([ref.params[n].reshape(-1) for n in names])
    out[rank] = dict(params=flat_p, grads=history)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gloo_two_rank_sync_exchange():
    world = 2
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
        res = dict(out)
    # replicas identical
    assert np.array_equal(res[0]['params'], res[1]['params'])
    # the two shards saw different envs -> different local gradients
    assert not np.allclose(res[0]['grads'][0], res[1]['grads'][0])
    # single-process restatement: both shards' clipped grads summed, one RMSProp step each iteration
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, 'async-rl-tensorflow_amd')]
    from src.initializers import init_params
    from src.kernels import param_names_shapes
    from oracle.engine_ref import EngineRef
    ns = param_names_shapes(6, 'a3c')
    names = [n for n, _ in ns]
    p = init_params(ns, seed=5, stddev=0.08)               # rank 0's params (broadcast source)
    refs = [EngineRef(p, 3, 2, 6, 'a3c', 0, 16, seed=9, env_id_base=r * 3, world_size=world) for r in range(world)]
    for r in refs:
        r.reset()
    for it in range(2):
        outs = [r.iterate() for r in refs]
        summed = {n: sum(o['clipped'][n] for o in outs).astype(np.float32) for n in names}
        for r in refs:
            r.apply(summed)
    flat = np.concatenate([refs[0].params[n].reshape(-1) for n in names])
    np.testing.assert_allclose(res[0]['params'], flat, rtol=1e-6, atol=1e-9)

"""Multi-rank engine path on one GPU: two processes (gloo process group over GPU tensors) each
run an engine on their own env shard (env ids rank*E ..), clip per worker, SUM-exchange and apply
-- the bench.py / main.py N>1 path with RCCL swapped for gloo so it runs on a 1-GPU box.  The
replicas must stay bit-identical and equal one process driving both shards' engines with the
same exchange done by hand."""
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


E, N, A, ITERS = 16, 5, 6, 4


def _make(rank, world, overlap):
    from src.engine import Engine
    from src.initializers import init_params, flatten_host
    from src.kernels import param_names_shapes
    eng = Engine(num_envs=E, n_step=N, action_size=A, num_frames=64, seed=11, env_id_base=rank * E,
                 world_size=world, overlap=overlap)
    ns = param_names_shapes(A, 'a3c')
    eng.reset(flatten_host(ns, eng.offsets, eng.params.numel(), init_params(ns, seed=4, stddev=0.05)))
    return eng


def _worker(rank, world, port, overlap, out):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, 'async-rl-tensorflow_amd')]
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK='0')
    import torch.distributed as dist
    from src.distributed import GradExchange
    dist.init_process_group('gloo')
    eng = _make(rank, world, overlap)
    xch = GradExchange()
    for _ in range(ITERS):
        eng.iterate(exchange=xch)
    torch.cuda.synchronize()
    out[rank] = dict(params=eng.params.cpu().numpy(), loss=eng.loss.cpu().numpy(),
                     step=int(eng.counters[1].item()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize('overlap', [False, True])
def test_two_ranks_stay_identical_and_match_manual_exchange(overlap):
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context('spawn')
    with ctx.Manager() as m:
        out = m.dict()
        port = _free_port()
        procs = [ctx.Process(target=_worker, args=(r, world, port, overlap, out)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(500)
            assert p.exitcode == 0
        res = dict(out)
    assert np.array_equal(res[0]['params'], res[1]['params'])
    assert res[0]['step'] == res[1]['step'] == ITERS * N * E * world - (N * E * world if overlap else 0)
    # one process, both shards, exchange by hand
    engs = [_make(r, world, overlap) for r in range(world)]
    for _ in range(ITERS):
        for e in engs:
            e.rollout_grad()
        if not engs[0].grad_ready:
            continue
        total = engs[0].grads + engs[1].grads
        for e in engs:
            e.grads.copy_(total)
            e.apply()
    torch.cuda.synchronize()
    assert torch.equal(engs[0].params, engs[1].params)
    np.testing.assert_array_equal(engs[0].params.cpu().numpy(), res[0]['params'])

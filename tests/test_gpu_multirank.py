"""Multi-rank engine path on one GPU: 2 or 4 processes (gloo process group over GPU tensors) each
run an engine on their own env shard (env ids rank*E ..), clip per worker, exchange and apply --
the bench.py / main.py N>1 path with RCCL swapped for gloo so it runs on a 1-GPU box (RCCL refuses
two ranks on one device).  The replicas must stay bit-identical and equal one process driving
every shard's engine with the same exchange done by hand."""
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


def _make(rank, world, overlap, cfg=None):
    """Rank `rank`'s engine on env ids rank*E.. (cfg: A, lives, lstm -- Pong by default; Breakout
    A=4 with 5 lives is BASELINE config 3, the LSTM head config 5)."""
    from src.engine import Engine
    from src.initializers import init_params, flatten_host
    from src.kernels import param_names_shapes
    cfg = cfg or {}
    a, lstm = cfg.get('A', A), cfg.get('lstm', False)
    eng = Engine(num_envs=E, n_step=N, action_size=a, num_frames=64, seed=11, env_id_base=rank * E,
                 world_size=world, overlap=overlap, start_lives=cfg.get('lives', 0), lstm=lstm)
    ns = param_names_shapes(a, 'a3c', lstm=lstm)
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


# ------------------------------------------------------- partitioned PS (default multi-GPU exchange)
def _pps_worker(rank, world, port, overlap, out, cfg):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, 'async-rl-tensorflow_amd')]
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK='0')
    import torch.distributed as dist
    from src.distributed import PartitionedPS
    dist.init_process_group('gloo')
    eng = _make(rank, world, overlap, cfg)
    ps = PartitionedPS(eng.params.numel())
    for _ in range(ITERS):
        eng.iterate(exchange=ps)
    torch.cuda.synchronize()
    out[rank] = dict(params=eng.params.cpu().numpy(), step=int(eng.counters[1].item()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize('world,overlap,cfg', [
    (2, False, {}), (2, True, {}), (4, False, {}), (4, True, {}),
    (4, True, dict(A=4, lives=5)), (4, False, dict(A=6, lives=3, lstm=True))],
    ids=['w2-sync', 'w2-overlap', 'w4-sync', 'w4-overlap', 'w4-breakout-overlap', 'w4-lstm-sync'])
def test_partitioned_ps_ranks(world, overlap, cfg):
    """`world` ranks on one GPU (gloo, host-staged collectives) run the default multi-GPU exchange:
    all-to-all of the clipped gradients, each rank's W sequential RMSProp steps on its range,
    all-gather.  Replicas stay identical and equal one process driving every shard through the
    same C-ABI by hand; in sync mode that also equals applying every rank's clipped gradient, in
    rank order, to full copies with a3c_rmsprop_range (the reference PS rule, main.py:60-65)."""
    import ctypes
    import torch.multiprocessing as mp
    from src._lib import lib, ptr, stream_handle
    from src.distributed import shard_ranges
    ctx = mp.get_context('spawn')
    with ctx.Manager() as m:
        out = m.dict()
        port = _free_port()
        procs = [ctx.Process(target=_pps_worker, args=(r, world, port, overlap, out, cfg)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(500)
            assert p.exitcode == 0
        res = dict(out)
    for r in range(1, world):
        assert np.array_equal(res[0]['params'], res[r]['params']), r
        assert res[0]['step'] == res[r]['step'] == ITERS * N * E * world - (N * E * world if overlap else 0)
    engs = [_make(r, world, overlap, cfg) for r in range(world)]
    total = engs[0].params.numel()
    shard, lo, n = shard_ranges(total, world)
    w_out = [torch.zeros(shard, device='cuda') for _ in range(world)]
    if not overlap:
        w = engs[0].params.clone()
        ms, mom = torch.ones_like(w), torch.zeros_like(w)
    for _ in range(ITERS):
        for e in engs:
            e.rollout_grad()
        if not engs[0].grad_ready:
            continue
        if not overlap:
            for e in engs:
                lib().a3c_rmsprop_range(ptr(w), ptr(ms), ptr(mom), ptr(e.grads), total, ctypes.c_void_p(e.sched_ptr),
                                        0.0, 0.99, 0.0, 0.1, stream_handle())
        for r, e in enumerate(engs):
            recv = torch.cat([engs[q].grads[lo[r]:lo[r] + n[r]] for q in range(world)])
            e.apply_shard(recv, world, lo[r], n[r], w_out[r])
        gathered = torch.cat(w_out)
        for e in engs:
            e.apply_commit(gathered)
    torch.cuda.synchronize()
    for e in engs[1:]:
        assert torch.equal(engs[0].params, e.params)
    np.testing.assert_array_equal(engs[0].params.cpu().numpy(), res[0]['params'])
    if not overlap:
        np.testing.assert_array_equal(w.cpu().numpy(), res[0]['params'])


# ------------------------------------------------------------------ Hogwild (SURVEY §8(e) async)
def _hog_worker(rank, world, port, out, lockstep):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, 'async-rl-tensorflow_amd')]
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK='0')
    import torch.distributed as dist
    from src.hogwild import HogwildPS
    dist.init_process_group('gloo')
    eng = _make(rank, world, False)
    ps = HogwildPS(eng.params)
    grads = []
    for it in range(ITERS):
        if lockstep:                      # deterministic order for the check: rank 0 then rank 1
            for turn in range(world):
                dist.barrier()
                if turn == rank:
                    eng.rollout_grad()
                    grads.append(eng.grads.clone())
                    ps.push(eng.grads, lr_dev=eng.sched_ptr)
                    eng.advance()
                    torch.cuda.synchronize()
            dist.barrier()
            ps.pull(eng.params)
            torch.cuda.synchronize()
        else:
            eng.iterate_hogwild(ps)
    torch.cuda.synchronize()
    dist.barrier()
    out[rank] = dict(shared=ps.gather().cpu().numpy(), params=eng.params.cpu().numpy(),
                     finite=bool(torch.isfinite(eng.params).all().item()))
    ps.close()
    dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize('world,lockstep', [(2, True), (2, False), (4, True), (4, False)])
def test_hogwild_sharded_ps(world, lockstep):
    """`world` ranks on one GPU push into each other's IPC-mapped shards.  Lock-step order must
    equal a single process applying every rank's clipped gradient in rank order each iteration;
    free-running (the real unlocked mode) must stay finite with every rank seeing the same shared
    params."""
    import torch.multiprocessing as mp
    ctx = mp.get_context('spawn')
    with ctx.Manager() as m:
        out = m.dict()
        port = _free_port()
        procs = [ctx.Process(target=_hog_worker, args=(r, world, port, out, lockstep)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(500)
            assert p.exitcode == 0
        res = dict(out)
    for r in range(1, world):
        np.testing.assert_array_equal(res[0]['shared'], res[r]['shared'])
    assert all(res[r]['finite'] for r in range(world))
    if not lockstep:
        return
    # replay: two engines, one shared RMSProp state applied in the same order
    from oracle import ref_cpu as Rc
    engs = [_make(r, world, False) for r in range(world)]
    w = engs[0].params.clone()
    ms, mom = torch.ones_like(w), torch.zeros_like(w)
    from src._lib import lib, ptr, stream_handle
    for it in range(ITERS):
        for e in engs:
            e.params.copy_(w)
        for e in engs:
            e.rollout_grad()
            e.advance()
            lib().a3c_rmsprop_range(ptr(w), ptr(ms), ptr(mom), ptr(e.grads), w.numel(),
                                    __import__('ctypes').c_void_p(e.sched_ptr), 0.0, 0.99, 0.0, 0.1, stream_handle())
            # the next engine of the same iteration still uses the start-of-iteration params
    torch.cuda.synchronize()
    np.testing.assert_array_equal(w.cpu().numpy(), res[0]['shared'])

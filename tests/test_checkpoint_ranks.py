"""CPU (gloo) tests of the multi-rank checkpoint paths (src/checkpoint.py, src/distributed.py):

* restore_engine: rank 0 picks the checkpoint and the path and every rank follows it -- a rank
  whose own state file is missing sends EVERY rank to the parameters + step path, a rank that
  cannot read the checkpoint fails every rank together (no rank left waiting in a collective);
* the index stores names relative to its directory, so a run resumed from another working
  directory finds its checkpoints;
* PartitionedPS.sync_slots gathers every rank's owned range of the RMSProp slots, so rank 0's
  checkpoint holds the true slots of every range (the reference Saver's slot variables)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _paths():
    import sys
    for p in (ROOT, os.path.join(ROOT, 'async-rl-tensorflow_amd')):
        if p not in sys.path:
            sys.path.insert(0, p)


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


NS = [('l1_w', (8, 8, 4, 16)), ('l1_b', (16,)), ('l2_w', (4, 4, 16, 32)), ('l2_b', (32,)),
      ('l4_w', (2592, 256)), ('l4_b', (256,)), ('p_w', (256, 6)), ('p_b', (6,)), ('q_w', (256, 1)), ('q_b', (1,))]


class FakeEngine:
    """The restore interface of src/engine.Engine over CPU tensors: state blobs of this rank load,
    others raise RuntimeError (as a3c_engine_state_load rejects another shard's state)."""

    def __init__(self, rank, fault=False):
        self.rank, self.algo, self.external_env, self.overlap = rank, 'a3c', False, False
        self.fault = fault
        self.offsets, self.sizes, off = [], [], 0
        for _, shp in NS:
            self.offsets.append(off)
            self.sizes.append(int(np.prod(shp)))
            off = -(-(off + self.sizes[-1]) // 64) * 64
        self.params = torch.zeros(off)
        self.target_params, self.ms, self.mom = torch.zeros(off), torch.ones(off), torch.zeros(off)
        self.counters = torch.zeros(3, dtype=torch.int64)
        self.loaded = None

    def reset(self, host_params=None):
        if host_params is not None:
            self.params.copy_(torch.as_tensor(host_params))
        self.ms.fill_(1.0)
        self.mom.zero_()

    def save_state(self):
        return np.array([self.rank, 7], np.uint8)

    def load_state(self, buf):
        from src._lib import A3CError, ERR_INVALID
        if self.fault:              # a HIP failure inside the load (hipErrorLaunchFailure)
            raise A3CError('a3c_engine_state_load failed (719): unspecified launch failure', 719)
        if int(buf[0]) != self.rank:
            raise A3CError('a3c_engine_state_load failed (10001): state of another env shard', ERR_INVALID)
        self.loaded = 'exact'

    def set_step(self, g, w=None):
        self.counters[1] = g
        self.loaded = 'params'


def _init(rank, world, port):
    _paths()
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group('gloo', rank=rank, world_size=world)


def _restore_worker(rank, world, port, out, ckdir, case):
    _init(rank, world, port)
    from src import checkpoint as C
    eng = FakeEngine(rank)
    eng.params.copy_(torch.arange(eng.params.numel(), dtype=torch.float32) * 1e-3)
    eng.counters[1] = 4321
    saver = C.Saver(ckdir, max_to_keep=3)
    if case != 'fresh':
        C.save_engine(saver, eng, NS, rank, world, barrier=dist.barrier)
        dist.barrier()
        if case == 'rank_file_missing' and rank == 0:
            os.remove(saver.path(4321, 1))
        if case == 'unreadable' and rank == 0:
            with open(saver.path(4321), 'wb') as f:
                f.write(b'not a checkpoint')
        dist.barrier()
    eng2 = FakeEngine(rank, fault=case == 'device_fault' and rank == 1)
    try:
        step = C.restore_engine(saver, eng2, NS, rank, world)
        res = dict(step=step, how=eng2.loaded, params=eng2.params.numpy().copy())
    except RuntimeError as e:
        res = dict(error=str(e))
    out[rank] = res
    dist.barrier()
    dist.destroy_process_group()


def _spawn(fn, world, *args):
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(fn, args=(world, port, out) + args, nprocs=world, join=True)
        return dict(out)


@pytest.mark.timeout(300)
@pytest.mark.parametrize('case', ['exact', 'rank_file_missing', 'unreadable', 'fresh', 'device_fault'])
def test_ranks_restore_alike(case, tmp_path):
    """Every rank takes the same path: exact states, parameters + step when a state is unusable
    (logged), or one agreed error -- an unreadable file, or a device fault inside a state load on
    any rank, which must not silently fall back."""
    res = _spawn(_restore_worker, 2, str(tmp_path / 'ck'), case)
    if case == 'device_fault':
        assert all('restoring the engine state' in res[r].get('error', '') for r in range(2)), res
        return
    if case == 'unreadable':
        assert all('cannot read' in res[r].get('error', '') for r in range(2)), res
        return
    if case == 'fresh':
        assert res[0]['step'] is None and res[1]['step'] is None
        return
    want = 'exact' if case == 'exact' else 'params'
    for r in range(2):
        assert res[r]['step'] == 4321 and res[r]['how'] == want, (r, res[r])
    if case != 'exact':
        assert np.array_equal(res[0]['params'], res[1]['params'])


def test_index_paths_are_relative_to_the_index(tmp_path):
    _paths()
    from src import checkpoint as C
    d = tmp_path / 'logs' / 'model'
    cwd = os.getcwd()
    try:
        os.chdir(tmp_path)
        saver = C.Saver(os.path.join('logs', 'model'), max_to_keep=2)      # relative, as main.py's default
        for step in (10, 20, 30):
            saver.save({'step': np.array(step)}, step)
        import json
        idx = json.load(open(d / 'checkpoint'))
        assert idx['all_model_checkpoint_paths'] == ['model.ckpt-20.npz', 'model.ckpt-30.npz']
        os.chdir(d)                                                          # resume from elsewhere
        assert C.Saver(str(d), max_to_keep=2).latest() == str(d / 'model.ckpt-30.npz')
        assert not os.path.exists(d / 'model.ckpt-10.npz')                   # pruned by max_to_keep
    finally:
        os.chdir(cwd)


def _slots_worker(rank, world, port, out):
    _init(rank, world, port)
    from src.distributed import PartitionedPS

    class E:
        pass
    total = 1000
    eng = E()
    ps = PartitionedPS(total, device='cpu')
    eng.ms = torch.full((total,), -1.0)
    eng.mom = torch.full((total,), -2.0)
    lo, n = ps.lo[rank], ps.n[rank]
    eng.ms[lo:lo + n] = float(rank)                  # only the owned range is this rank's truth
    eng.mom[lo:lo + n] = 10.0 + rank
    ps.sync_slots(eng)
    out[rank] = dict(ms=eng.ms.numpy().copy(), mom=eng.mom.numpy().copy(), lo=ps.lo, n=ps.n)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_partitioned_ps_sync_slots_gathers_owned_ranges():
    world = 4
    res = _spawn(_slots_worker, world)
    lo, n = res[0]['lo'], res[0]['n']
    want_ms = np.concatenate([np.full(n[r], float(r), np.float32) for r in range(world)])
    want_mom = np.concatenate([np.full(n[r], 10.0 + r, np.float32) for r in range(world)])
    for r in range(world):
        np.testing.assert_array_equal(res[r]['ms'], want_ms)
        np.testing.assert_array_equal(res[r]['mom'], want_mom)

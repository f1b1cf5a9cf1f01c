"""Hogwild parameter server across GPUs: SURVEY §8(e) "async", BASELINE config 4.

It replaces the reference's parameter server (main.py:58-66). There, every worker pushes its
per-worker-clipped gradient (agent.py:316-319) into a shared RMSProp that applies it unlocked,
and pulls the current weights for its next rollout.

MI355X form, one process per GPU:
* each rank owns a contiguous byte-range shard of the flat params / ms / mom in its own HBM.
  It is exported over IPC (a3c_ipc_handle); every rank maps every shard (a3c_ipc_open, lazy
  peer access over xGMI).
* push: for every shard, one unlocked elementwise RMSProp kernel (a3c_rmsprop_range) writes
  straight into the owner's memory. Concurrent pushes from other ranks interleave, like the
  reference's lock-free PS.
* pull: the shards are copied back into the rank's local parameter buffer before its next
  rollout (theta' <- theta, network.py:96-107).
No collective runs on the data path. The only collectives are the handle exchange at setup and
the barrier at teardown.

Memory model: the shards are allocated FINE-GRAINED by default
(``memory='fine'``, hipDeviceMallocFinegrained).  Plain hipMalloc memory is coarse-grained: it is
coherent only at kernel boundaries, and a peer GPU's read-modify-writes over xGMI and the owner's
L2-cached reads of the same lines are ordered by nothing but those boundaries.  Fine-grained
memory is coherent at instruction granularity across devices, so every push lands in the owner's
memory and every pull reads it from there: what remains unordered is exactly Hogwild's element
interleaving of concurrent unlocked RMWs (the reference's ``use_locking=False`` PS apply,
main.py:63-65).  ``memory='coarse'`` and ``'uncached'`` remain selectable for measurement.
"""
import ctypes

import torch
import torch.distributed as dist

from . import _lib
from ._lib import check, lib, stream_handle


class HogwildPS:
    MEMORY_KINDS = {'coarse': 0, 'fine': 1, 'uncached': 2}

    def __init__(self, local_params, decay=0.99, momentum=0.0, epsilon=0.1, group=None, memory='fine',
                 ms=None, mom=None):
        """local_params (and ms / mom: full RMSProp slots to start from, e.g. restored from a
        checkpoint; default the TF1 init 1 / 0): this rank's shard is initialised from its range."""
        if memory not in self.MEMORY_KINDS:
            raise ValueError(f'memory must be one of {sorted(self.MEMORY_KINDS)}')
        self.memory = memory
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.decay, self.momentum, self.epsilon = float(decay), float(momentum), float(epsilon)
        total = int(local_params.numel())
        shard = -(-total // self.world)
        shard = (shard + 63) // 64 * 64
        self.total, self.shard = total, shard
        self.lo = [min(total, r * shard) for r in range(self.world)]
        self.n = [max(0, min(total, (r + 1) * shard) - self.lo[r]) for r in range(self.world)]
        base = ctypes.c_void_p()
        check(lib().a3c_dev_alloc_kind(3 * shard * 4, self.MEMORY_KINDS[memory], ctypes.byref(base)),
              'a3c_dev_alloc_kind')
        self._own = base.value
        from .engine import _view
        own = _view(self._own, (3, shard), torch.float32)
        own.zero_()
        r = self.rank
        sl = slice(self.lo[r], self.lo[r] + self.n[r])
        own[0, :self.n[r]].copy_(local_params[sl])
        own[1].fill_(1.0)                              # TF1 rms slot init
        if ms is not None:
            own[1, :self.n[r]].copy_(ms[sl])
        if mom is not None:
            own[2, :self.n[r]].copy_(mom[sl])
        self.own = own
        h = (ctypes.c_char * 64)()
        check(lib().a3c_ipc_handle(ctypes.c_void_p(self._own), h), 'a3c_ipc_handle')
        mine = bytes(h)
        if self.world > 1:
            handles = [None] * self.world
            dist.all_gather_object(handles, mine, group=group)
        else:
            handles = [mine]
        self.base = []
        self._opened = []
        for q in range(self.world):
            if q == r:
                self.base.append(self._own)
                continue
            p = ctypes.c_void_p()
            hb = (ctypes.c_char * 64).from_buffer_copy(handles[q])
            check(lib().a3c_ipc_open(hb, ctypes.byref(p)), 'a3c_ipc_open')
            self.base.append(p.value)
            self._opened.append(p.value)
        torch.cuda.synchronize()
        if self.world > 1:
            dist.barrier(group=group)                  # every shard initialised before any push

    def _ptrs(self, q):
        b = self.base[q]
        return b, b + 4 * self.shard, b + 8 * self.shard

    def push(self, grads, lr_dev=None, lr=0.0):
        """Unlocked RMSProp of this worker's (already clipped) gradient into every shard,
        starting with this rank's own shard and walking the ring (spreads the xGMI links)."""
        gp = grads.data_ptr()
        for k in range(self.world):
            q = (self.rank + k) % self.world
            if self.n[q] == 0:
                continue
            w, ms, mom = self._ptrs(q)
            check(lib().a3c_rmsprop_range(ctypes.c_void_p(w), ctypes.c_void_p(ms), ctypes.c_void_p(mom),
                                          ctypes.c_void_p(gp + 4 * self.lo[q]), self.n[q],
                                          ctypes.c_void_p(lr_dev) if lr_dev else None, float(lr), self.decay,
                                          self.momentum, self.epsilon, stream_handle()), 'a3c_rmsprop_range')

    def pull(self, params):
        """theta' <- theta: copy every shard into the local parameter buffer."""
        pp = params.data_ptr()
        for k in range(self.world):
            q = (self.rank + k) % self.world
            if self.n[q] == 0:
                continue
            check(lib().a3c_copy_params(ctypes.c_void_p(pp + 4 * self.lo[q]), ctypes.c_void_p(self.base[q]),
                                        self.n[q], stream_handle()), 'a3c_copy_params')

    def params_view(self):
        """world 1: the single shard's parameters (the whole flat vector) as a device tensor."""
        assert self.world == 1
        return self.own[0, :self.total]

    def sync_slots(self, eng):
        """The shared RMSProp slots (every shard's ms / mom) into the engine's full ms / mom
        buffers, which Hogwild does not otherwise use: checkpoints then hold the true slots."""
        for k, dst in ((1, eng.ms), (2, eng.mom)):
            base = dst.data_ptr()
            for q in range(self.world):
                if self.n[q]:
                    check(lib().a3c_copy_params(ctypes.c_void_p(base + 4 * self.lo[q]),
                                                ctypes.c_void_p(self.base[q] + 4 * k * self.shard), self.n[q],
                                                stream_handle()), 'a3c_copy_params')

    def gather(self):
        """Current shared parameters as one device tensor (for checks)."""
        out = torch.empty(self.total, dtype=torch.float32, device='cuda')
        self.pull(out)
        return out

    def close(self):
        if getattr(self, '_own', None) is None:
            return
        torch.cuda.synchronize()
        if self.world > 1 and dist.is_initialized():
            dist.barrier(group=self.group)             # nobody writes into our shard any more
        for p in self._opened:
            lib().a3c_ipc_close(ctypes.c_void_p(p))
        self._opened = []
        lib().a3c_dev_free(ctypes.c_void_p(self._own))
        self._own = None

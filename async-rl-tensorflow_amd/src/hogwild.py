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
"""
import ctypes

import torch
import torch.distributed as dist

from . import _lib
from ._lib import check, lib, stream_handle


class HogwildPS:
    def __init__(self, local_params, decay=0.99, momentum=0.0, epsilon=0.1, group=None):
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
        check(lib().a3c_dev_alloc(3 * shard * 4, ctypes.byref(base)), 'a3c_dev_alloc')
        self._own = base.value
        from .engine import _view
        own = _view(self._own, (3, shard), torch.float32)
        own.zero_()
        r = self.rank
        own[0, :self.n[r]].copy_(local_params[self.lo[r]:self.lo[r] + self.n[r]])
        own[1].fill_(1.0)                              # TF1 rms slot init
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

"""Multi-GPU gradient exchange that replaces the TF parameter server (main.py:50-66).

The reference runs W worker processes that push per-worker-clipped gradients (agent.py:316-319)
to a PS which applies shared RMSProp unlocked and asynchronously (main.py:64-65,
``replica_device_setter`` main.py:60-62).  Here every GPU is one process (torch.distributed,
backend "nccl" = RCCL over xGMI); each GPU clips its own gradient per tensor, the clipped
gradients are SUMMED with one all-reduce of the flat fp32 vector (2.71 MB for Pong), and every
GPU applies the identical RMSProp step to its replica of the parameters and slots.

Semantics vs the reference: the sum of W clipped gradients is applied as ONE RMSProp step,
where the reference applies W steps in arrival order; first-order equivalent, and
deterministic (no lock-free races).  DESIGN.md "Multi-GPU".
"""
import os

import torch
import torch.distributed as dist


def init_from_env(backend=None):
    """Initialise torch.distributed from the torchrun environment (MASTER_ADDR/PORT, RANK,
    WORLD_SIZE, LOCAL_RANK).  Returns (rank, world, local_rank)."""
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = 'nccl' if torch.cuda.is_available() else 'gloo'
        kw = {}
        if backend == 'nccl':
            torch.cuda.set_device(local)
            kw['device_id'] = torch.device('cuda', local)
        dist.init_process_group(backend, **kw)
    return rank, world, local


class GradExchange:
    """Callable handed to ``Engine.iterate(exchange=...)``: sum-all-reduce of the clipped grads."""

    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1

    def __call__(self, grads):
        if self.world > 1:
            dist.all_reduce(grads, op=dist.ReduceOp.SUM, group=self.group)
        return grads


def broadcast_params(t, src=0, group=None):
    """Start every replica from rank ``src``'s parameters (the PS's initial values)."""
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(t, src=src, group=group)
    return t

"""Multi-GPU update paths that replace the TF parameter server (main.py:50-66).

The reference runs W worker processes.  Each clips its own gradient per tensor
(agent.py:316-319) and pushes it to the PS, whose shared RMSProp (main.py:63-65, rms slot
initialised to 1) applies every push as an update of its own, unlocked, in arrival order
(``replica_device_setter`` main.py:60-62, ``apply_gradients`` agent.py:321).  Here every GPU is
one process (torch.distributed, backend "nccl" = RCCL over xGMI) and two exchanges exist:

``PartitionedPS`` (default, ``--exchange sequential``): the PS partitioned across the GPUs.
  Rank r owns a 1/W byte range of params / ms / mom.  Per iteration:
    1. all-to-all of the clipped gradients: rank r receives every rank's gradient of its range;
    2. ``a3c_engine_apply_shard``: the W RMSProp steps of the range, one per rank, in rank order;
    3. all-gather of the updated ranges into every replica;
    4. ``a3c_engine_apply_commit``: snapshot / target sync / counters.
  That is the reference PS's update rule, W separate steps, in one fixed arrival order (rank
  order), so it is deterministic and every replica is bit-identical.  Traffic per GPU equals a
  ring all-reduce's: (W-1)/W of the 2.71 MB gradient out and in, twice.

``GradExchange`` (``--exchange sum``): one SUM all-reduce, then every GPU applies ONE RMSProp
  step of the summed gradient.  That is NOT the reference's rule: RMSProp divides by
  sqrt(ms), and ms tracks the square of the gradient it is given, so once ms has warmed up a
  summed step moves about lr*sign(g) where the reference's W steps move about W*lr*sign(g).
  It learns up to W times slower per env-step and is kept only as the plain data-parallel
  baseline (tests/test_dist_gloo.py shows the two rules differ).

``sequential_apply`` is the agent-mode (one env per process) form of the PS rule: all-gather
the clipped gradients, apply them in rank order.
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


def _world(group):
    return dist.get_world_size(group) if dist.is_initialized() else 1


def _rank(group):
    return dist.get_rank(group) if dist.is_initialized() else 0


def _host_staged(t, group):
    """gloo moves CPU tensors only: device tensors are staged through host memory."""
    return t.is_cuda and dist.is_initialized() and dist.get_backend(group) == 'gloo'


def shard_ranges(total, world, align=64):
    """(lo, n) of every rank: contiguous ranges of ceil(total / world) floats rounded up to
    `align` (tensor offsets are 64-float aligned, so are the ranges); the last may be short."""
    shard = -(-int(total) // int(world))
    shard = -(-shard // align) * align
    lo = [min(total, r * shard) for r in range(world)]
    n = [min(total, (r + 1) * shard) - lo[r] for r in range(world)]
    return shard, lo, n


class PartitionedPS:
    """Partitioned parameter server over ``torch.distributed`` (module docstring).  Handed to
    ``Engine.iterate(exchange=...)``; performs the apply itself (``owns_apply``)."""

    owns_apply = True

    def __init__(self, total, group=None, device='cuda', split=None):
        """split: run the two-phase exchange when the engine offers a split point (True), never
        (False), or (None) only where the collectives run on the device -- host-staged gloo
        collectives block the host at every staging copy, so two phases there only add stalls."""
        self.group = group
        self.split = split
        self.world, self.rank = _world(group), _rank(group)
        self.total = int(total)
        self.shard, self.lo, self.n = shard_ranges(self.total, self.world)
        r = self.rank
        self.recv = torch.zeros(max(1, self.world * self.n[r]), dtype=torch.float32, device=device)
        self.w_out = torch.zeros(self.shard, dtype=torch.float32, device=device)
        self.gathered = torch.zeros(self.world * self.shard, dtype=torch.float32, device=device)

    def all_to_all(self, grads):
        """recv[q*n_r : (q+1)*n_r] <- rank q's gradient of this rank's range."""
        r = self.rank
        if self.world == 1:
            self.recv[:self.n[0]].copy_(grads[:self.n[0]])
            return self.recv
        out_splits, in_splits = [self.n[r]] * self.world, list(self.n)
        if _host_staged(grads, self.group):
            out = torch.empty(self.recv.numel(), dtype=torch.float32)
            dist.all_to_all_single(out, grads.cpu(), out_splits, in_splits, group=self.group)
            self.recv.copy_(out)
        else:
            dist.all_to_all_single(self.recv[:self.world * self.n[r]], grads, out_splits, in_splits, group=self.group)
        return self.recv

    def all_gather(self):
        """gathered[q*shard : q*shard + n_q] <- rank q's updated range."""
        if self.world == 1:
            self.gathered.copy_(self.w_out)
        elif _host_staged(self.w_out, self.group):
            out = torch.empty(self.gathered.numel(), dtype=torch.float32)
            dist.all_gather_into_tensor(out, self.w_out.cpu(), group=self.group)
            self.gathered.copy_(out)
        else:
            dist.all_gather_into_tensor(self.gathered, self.w_out, group=self.group)
        return self.gathered

    def sync_slots(self, eng):
        """Every rank owns (updates) only its range of the RMSProp slots: gather the owned ranges
        of ms and mom into every replica's full buffers, so that a checkpoint (rank 0 writes the
        slots under TF1's slot names) holds the true slots of every range.  A collective: every
        rank calls it at the same point, between iterations."""
        r = self.rank
        lo, n = self.lo[r], self.n[r]
        for t in (eng.ms, eng.mom):
            self.w_out.zero_()
            self.w_out[:n].copy_(t[lo:lo + n])
            self.all_gather()
            t.copy_(self.gathered[:self.total])

    def apply(self, eng):
        cut = eng.split_point if self.world > 1 else 0
        if cut and self.split is None:
            cut = 0 if _host_staged(eng.grads, self.group) else cut
        if cut and self.split is not False:
            return self._apply_split(eng, cut)
        r = self.rank
        self.all_to_all(eng.grads)
        eng.apply_shard(self.recv, self.world, self.lo[r], self.n[r], self.w_out)
        self.all_gather()
        eng.apply_commit(self.gathered)

    # -------------------------------------------------------------------- split exchange
    def _split_plan(self, cut):
        """Each owned range [lo_q, lo_q + n_q) splits at `cut` into its conv part (a prefix of the
        range: the conv tensors come first in the flat layout) and its fc / head part."""
        if getattr(self, '_cut', None) != cut:
            W, lo, n = self.world, self.lo, self.n
            self._cut = cut
            self.conv_n = [max(0, min(lo[q] + n[q], cut) - lo[q]) for q in range(W)]
            self.fc_n = [n[q] - self.conv_n[q] for q in range(W)]
            self.cmax = max(1, max(self.conv_n))
            dev = self.recv.device
            r = self.rank
            self.recv_fc = torch.zeros(max(1, W * self.fc_n[r]), dtype=torch.float32, device=dev)
            self.recv_conv = torch.zeros(max(1, W * self.conv_n[r]), dtype=torch.float32, device=dev)
            self.w_conv = torch.zeros(self.cmax, dtype=torch.float32, device=dev)
            self.g_conv = torch.zeros(W * self.cmax, dtype=torch.float32, device=dev)
            self.comm = torch.cuda.Stream(device=dev) if dev.type == 'cuda' else None

    def _a2a(self, out, src, splits_out, splits_in):
        if _host_staged(src, self.group):
            h = torch.empty(out.numel(), dtype=torch.float32)
            dist.all_to_all_single(h, src.cpu(), splits_out, splits_in, group=self.group)
            out.copy_(h)
        else:
            dist.all_to_all_single(out, src, splits_out, splits_in, group=self.group)

    def _ag(self, out, src):
        if _host_staged(src, self.group):
            h = torch.empty(out.numel(), dtype=torch.float32)
            dist.all_gather_into_tensor(h, src.cpu(), group=self.group)
            out.copy_(h)
        else:
            dist.all_gather_into_tensor(out, src, group=self.group)

    def _apply_split(self, eng, cut):
        """The exchange in two phases (comm on its own stream).  Phase A, on a comm
        stream that waits only for the backward's clip of grads[cut:] (fc + heads, 99 % of the
        bytes): all-to-all of that range, the W rank-ordered RMSProp steps of each owned range's fc
        part, all-gather -- concurrent with the conv backward on the caller's stream.  Phase B, on
        the caller's stream behind the whole backward: the same for the conv prefix (~50 KB, held by
        rank 0's range at W <= 8), then the caller joins the comm stream and commits.  The same
        element math on the same values as the one-phase exchange: bit-identical replicas."""
        import contextlib
        self._split_plan(cut)
        r, W = self.rank, self.world
        g = eng.grads
        total = self.total
        lo_fc = self.lo[r] + self.conv_n[r]
        ctx = torch.cuda.stream(self.comm) if self.comm is not None else contextlib.nullcontext()
        with ctx:
            if self.comm is not None:
                eng.wait_grad_head()
            # phase A: fc / head range
            self._a2a(self.recv_fc[:W * self.fc_n[r]], g[cut:total], [self.fc_n[r]] * W, list(self.fc_n))
            eng.apply_shard(self.recv_fc, W, lo_fc, self.fc_n[r], self.w_out[self.conv_n[r]:])
            self._ag(self.gathered, self.w_out)
        # phase B: conv prefix (caller's stream, after the whole backward)
        self._a2a(self.recv_conv[:W * self.conv_n[r]], g[:cut], [self.conv_n[r]] * W, list(self.conv_n))
        if self.conv_n[r]:
            eng.apply_shard(self.recv_conv, W, self.lo[r], self.conv_n[r], self.w_conv)
        self._ag(self.g_conv, self.w_conv)
        if self.comm is not None:
            torch.cuda.current_stream().wait_stream(self.comm)
        for q in range(W):
            if self.conv_n[q]:
                self.gathered[q * self.shard:q * self.shard + self.conv_n[q]].copy_(
                    self.g_conv[q * self.cmax:q * self.cmax + self.conv_n[q]])
        eng.apply_commit(self.gathered)


class LoopbackPS(PartitionedPS):
    """The partitioned PS of ``world`` virtual ranks inside ONE process on one GPU: every virtual
    rank holds this engine's (per-worker clipped) gradient, so the all-to-all and all-gather become
    device-to-device copies on the exchange's own streams, with no host staging and no process
    group.  It drives the exchange code path of a real multi-GPU run -- the two-phase form with
    phase A on the comm stream behind ``wait_grad_head`` (under the conv backward), phase B on the
    caller's stream, the join and the commit; the one-phase form after the whole backward -- on a
    one-GPU box, where RCCL refuses two ranks.  The update it applies is the reference PS rule for
    W workers that pushed the same gradient: W rank-ordered RMSProp steps of every range
    (main.py:63-65).  Test and rehearsal infrastructure: the engine must be created with
    ``world_size=world`` (per-worker clip, split backward, global-step accounting)."""

    def __init__(self, total, world, device='cuda', split=True):
        self.group = None
        self.split = split
        self.world, self.rank = int(world), 0
        self.total = int(total)
        self.shard, self.lo, self.n = shard_ranges(self.total, self.world)
        self.recv = torch.zeros(max(1, self.world * max(self.n)), dtype=torch.float32, device=device)
        self.recv_a = torch.zeros_like(self.recv)      # phase A's staging (the comm stream's own)
        self.w_out = torch.zeros(self.shard, dtype=torch.float32, device=device)
        self.gathered = torch.zeros(self.world * self.shard, dtype=torch.float32, device=device)

    def _steps(self, eng, g, a, b, recv, out):
        """the W rank-ordered steps of [a, b): every virtual rank's gradient is g[a:b]"""
        n = b - a
        if n <= 0:
            return
        for q in range(self.world):
            recv[q * n:(q + 1) * n].copy_(g[a:b])
        eng.apply_shard(recv, self.world, a, n, out)

    def apply(self, eng):
        cut = eng.split_point
        g = eng.grads
        if cut and self.split:
            return self._apply_split_loopback(eng, cut)
        for q in range(self.world):               # one phase: every range after the whole backward
            a = self.lo[q]
            self._steps(eng, g, a, a + self.n[q], self.recv, self.w_out)
            self.gathered[q * self.shard:q * self.shard + self.n[q]].copy_(self.w_out[:self.n[q]])
        eng.apply_commit(self.gathered)

    def _apply_split_loopback(self, eng, cut):
        """PartitionedPS._apply_split with the collectives as copies: phase A (the fc / head part
        of every range) on the comm stream after ``wait_grad_head``, phase B (the conv prefix) on
        the caller's stream after the whole backward, then the join and the commit."""
        self._split_plan(cut)
        g = eng.grads
        # (the event it waits for is recorded on the caller's stream behind the previous commit,
        # so the comm stream's buffers are free again when it fires)
        with torch.cuda.stream(self.comm):
            eng.wait_grad_head()
            for q in range(self.world):
                a = self.lo[q] + self.conv_n[q]
                self._steps(eng, g, a, self.lo[q] + self.n[q], self.recv_a, self.w_out[self.conv_n[q]:])
                self.gathered[q * self.shard + self.conv_n[q]:q * self.shard + self.n[q]].copy_(
                    self.w_out[self.conv_n[q]:self.n[q]])
        for q in range(self.world):
            if self.conv_n[q]:
                self._steps(eng, g, self.lo[q], self.lo[q] + self.conv_n[q], self.recv, self.w_conv)
                self.g_conv[q * self.cmax:q * self.cmax + self.conv_n[q]].copy_(self.w_conv[:self.conv_n[q]])
        torch.cuda.current_stream().wait_stream(self.comm)
        for q in range(self.world):
            if self.conv_n[q]:
                self.gathered[q * self.shard:q * self.shard + self.conv_n[q]].copy_(
                    self.g_conv[q * self.cmax:q * self.cmax + self.conv_n[q]])
        eng.apply_commit(self.gathered)


class GradExchange:
    """Callable handed to ``Engine.iterate(exchange=...)``: SUM all-reduce of the clipped grads
    (the plain data-parallel rule, NOT the reference PS's: module docstring)."""

    def __init__(self, group=None):
        self.group = group
        self.world = _world(group)

    def __call__(self, grads):
        if self.world > 1:
            if _host_staged(grads, self.group):
                h = grads.cpu()
                dist.all_reduce(h, op=dist.ReduceOp.SUM, group=self.group)
                grads.copy_(h)
            else:
                dist.all_reduce(grads, op=dist.ReduceOp.SUM, group=self.group)
        return grads


def gather_grads(grads, group=None):
    """Every rank's flat gradient, in rank order (agent mode: one env per process)."""
    world = _world(group)
    if world == 1:
        return [grads]
    staged = _host_staged(grads, group)
    src = grads.cpu() if staged else grads
    out = [torch.empty_like(src) for _ in range(world)]
    dist.all_gather(out, src, group=group)
    return [o.to(grads.device) for o in out] if staged else out


def broadcast_params(t, src=0, group=None):
    """Start every replica from rank ``src``'s parameters (the PS's initial values)."""
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        if _host_staged(t, group):
            h = t.cpu()
            dist.broadcast(h, src=src, group=group)
            t.copy_(h)
        else:
            dist.broadcast(t, src=src, group=group)
    return t

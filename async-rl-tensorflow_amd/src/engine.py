"""Batched A3C / Q-learning actor-learner engine (one per GPU) over the C-ABI.

``Engine.iterate()`` is one pass of the rollout + gradient path for E envs: n env steps
(forward, action draw, env step, Atari preprocessing into the frame ring), bootstrap /
target-net forward, returns, loss + backward, per-tensor clip, then the optional multi-GPU
gradient exchange (``exchange`` callback, e.g. an RCCL all-reduce) and the RMSProp apply.
It replaces the per-worker loop of agent.py:52-67 (+ observe/batch_update :153-207) and the
parameter-server apply of main.py:60-66.

``overlap=True`` pipelines the engine: rollout k runs on an engine-owned stream with the
parameters after update k-2 while the backward, exchange and apply of rollout k-1 run on the
caller's stream (A3C's stale-parameter asynchrony at a fixed staleness of one update).  Rollout
k's buffers are ``slot(k & 1)``.  With ``algo='q'`` rollout k-1's TD targets are formed by its
backward, with the target network as it stands then (agent.py:169-190 at the same staleness).

Kernels are launched eagerly by default; ``use_graph=True`` captures each engine call into
hipGraphs and replays them (bit-identical, measured slower on MI355X: DESIGN.md §6).
``frame84=1`` (an engine option) feeds pre-sized 84x84 frames instead of raw RGB (measurement
mode M2).
"""
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import check, lib

GAMES = {  # ALE minimal action sets / starting lives
    'Pong-v0': (6, 0),
    'Breakout-v0': (4, 5),
    'SpaceInvaders-v0': (6, 3),
}


class _DevArray:
    """Zero-copy view of engine-owned device memory for torch.as_tensor."""

    def __init__(self, ptr, shape, typestr):
        self.__cuda_array_interface__ = {'data': (int(ptr), False), 'shape': tuple(int(s) for s in shape),
                                         'typestr': typestr, 'version': 2, 'strides': None}


def _view(ptr, shape, dtype):
    typestr = {torch.float32: '<f4', torch.int32: '<i4', torch.uint8: '|u1', torch.int64: '<i8',
               torch.uint32: '<u4'}[dtype]
    return torch.as_tensor(_DevArray(ptr, shape, typestr), device='cuda')


class Engine:
    def __init__(self, num_envs=256, n_step=5, action_size=6, algo='a3c', start_lives=0, num_frames=1024,
                 seed=123, env_id_base=0, world_size=1, use_graph=False, overlap=False, lstm=False,
                 external_env=False, dqn_type='nips', **overrides):
        _lib.require_device()
        if lstm and algo != 'a3c':
            raise ValueError('the LSTM head is an a3c head')
        self.dqn_type = str(dqn_type).lower()
        if self.dqn_type == 'nature' and (algo != 'a3c' or lstm or external_env):
            raise ValueError('the nature trunk (network.py:30-42) runs A3C heads, feed-forward, on device envs')
        cfg = _lib.EngineConfig()
        lib().a3c_engine_config_default(ctypes.byref(cfg))
        cfg.net = _lib.net_desc(action_size, algo, lstm, self.dqn_type)
        self.lstm = bool(lstm)
        cfg.num_envs = int(num_envs)
        cfg.n_step = int(n_step)
        cfg.start_lives = int(start_lives)
        cfg.num_frames = int(num_frames)
        cfg.seed = int(seed)
        cfg.env_id_base = int(env_id_base)
        cfg.world_size = int(world_size)
        cfg.use_graph = 1 if use_graph else 0
        cfg.overlap = 1 if overlap else 0
        cfg.external_env = 1 if external_env else 0
        self.overlap = bool(overlap)
        self.external_env = bool(external_env)
        for k, v in overrides.items():
            if not hasattr(cfg, k):
                raise ValueError(f'unknown engine option {k}')
            setattr(cfg, k, v)
        self.cfg = cfg
        self.algo = algo
        self.A = int(action_size)
        self.E, self.n = int(num_envs), int(n_step)
        h = ctypes.c_void_p()
        check(lib().a3c_engine_create(ctypes.byref(cfg), ctypes.byref(h)), 'a3c_engine_create')
        self._h = h
        b = _lib.EngineBuffers()
        check(lib().a3c_engine_get_buffers(h, ctypes.byref(b)), 'a3c_engine_get_buffers')
        self._b = b
        self.zs = int(b.zs)
        self.offsets = [int(b.offsets[i]) for i in range(b.n_tensors)]
        self.sizes = [int(b.sizes[i]) for i in range(b.n_tensors)]
        P, E, n = int(b.n_params), self.E, self.n
        self.params = _view(b.params, (P,), torch.float32)
        self.target_params = _view(b.target_params, (P,), torch.float32)
        self.ms = _view(b.ms, (P,), torch.float32)
        self.mom = _view(b.mom, (P,), torch.float32)
        self.grads = _view(b.grads, (P,), torch.float32)
        self.frame_ring = _view(b.frame_ring, (E, b.ring_slots, 84, 84), torch.uint8)
        self.ring_slots = int(b.ring_slots)
        # [0] tau, [1] global step T (agent.py:165), [2] the workers' base step (agent.py:34,55)
        self.counters = _view(b.tau, (3,), torch.int64)
        self.loss = _view(b.loss, (4,), torch.float32)
        self.sched_ptr = int(b.sched)             # device [0] = lr of the last gradient
        self.sumsq = _view(b.sumsq, (b.n_tensors,), torch.float32)
        self._slots = [self._slot_views(k) for k in range(2 if self.overlap else 1)]
        for k, v in self._slots[0].items():
            setattr(self, k, v)
        self.frame84 = bool(cfg.frame84)
        self.frame_pool = _view(b.frame_pool, (int(cfg.num_frames),) + ((84, 84) if self.frame84 else (210, 160, 3)),
                                torch.uint8)
        # env state is double-buffered by step parity: the current state lives at tau & 1
        self._env = {'frame': _view(b.env_frame, (2, E), torch.int32),
                     'lives': _view(b.env_lives, (2, E), torch.int32),
                     'episode': _view(b.env_episode, (2, E), torch.int32),
                     'ep_step': _view(b.env_step, (2, E), torch.int32),
                     'ep_len': _view(b.env_len, (2, E), torch.int32)}

    def _slot_views(self, k):
        b = _lib.EngineBuffers()
        check(lib().a3c_engine_slot_buffers(self._h, k, ctypes.byref(b)), 'a3c_engine_slot_buffers')
        E, n = self.E, self.n
        lstm = {}
        if self.lstm:
            U = int(b.lstm_units)
            lstm = dict(lstm_h=_view(b.lstm_h, (n, E, U), torch.float32),
                        lstm_c=_view(b.lstm_c, (n, E, U), torch.float32),
                        lstm_hp=_view(b.lstm_hp, (n, E, U), torch.float32),
                        lstm_cp=_view(b.lstm_cp, (n, E, U), torch.float32),
                        lstm_gates=_view(b.lstm_gates, (n, E, 4 * U), torch.float32))
        if self.dqn_type == 'nature':     # conv outputs NHWC [20,20,32] / [9,9,64] / [7,7,64], fc out 512
            acts = dict(act_l1=_view(b.act_l1, (n * E, 12800), torch.float32),
                        act_l2=_view(b.act_l2, (n * E, 5184), torch.float32),
                        act_l3=_view(b.act_l3, (n * E, 3136), torch.float32),
                        act_l4=_view(b.act_l4, (n * E, 512), torch.float32))
        else:
            acts = dict(act_l1=_view(b.act_l1, (n * E, 6400), torch.float32),
                        act_l2=_view(b.act_l2, (n * E, 2592), torch.float32),
                        act_l3=_view(b.act_l3, (n * E, 256), torch.float32))
        return dict(**lstm, **acts, actions=_view(b.actions, (n, E), torch.int32),
                    rewards=_view(b.rewards, (n, E), torch.float32),
                    terminals=_view(b.terminals, (n, E), torch.uint8),
                    z=_view(b.z, (n + 1, E, self.zs), torch.float32),
                    returns=_view(b.returns, (n, E), torch.float32))

    def slot(self, k):
        """Rollout buffers of slot k (overlap: rollout i lives in slot i & 1)."""
        return self._slots[k]

    def env_field(self, name):
        """Current synthetic-env state field [E] (frame, lives, episode, ep_step, ep_len)."""
        tau = int(self.counters[0].item())
        return self._env[name][tau & 1]

    @property
    def env_frame(self):
        return self.env_field('frame')

    def close(self):
        if getattr(self, '_h', None):
            lib().a3c_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------------------------------
    def reset(self, host_params=None):
        """host_params: flat float32 numpy array of the engine layout (None keeps params)."""
        arg = None
        if host_params is not None:
            hp = np.ascontiguousarray(np.asarray(host_params, dtype=np.float32))
            if hp.size != self.params.numel():
                raise ValueError('host_params has the wrong length')
            self._hp = hp
            arg = hp.ctypes.data_as(ctypes.c_void_p)
        check(lib().a3c_engine_reset(self._h, arg, _lib.stream_handle()), 'a3c_engine_reset')
        self._ext_began = False
        self._step0_w = 0

    def rollout_grad(self):
        check(lib().a3c_engine_rollout_grad(self._h, _lib.stream_handle()), 'a3c_engine_rollout_grad')

    def apply(self):
        check(lib().a3c_engine_apply(self._h, _lib.stream_handle()), 'a3c_engine_apply')

    @property
    def grad_ready(self):
        return bool(lib().a3c_engine_grad_ready(self._h))

    @property
    def split_point(self):
        """Split exchange (several GPUs): the float offset where the fc / head gradients start --
        clipped before the conv backward, so their exchange can run under it; 0: no split."""
        if not hasattr(lib(), 'a3c_engine_exchange_split'):
            return 0          # (an older build selected by A3C_LIB: the one-phase exchange, named on load)
        cut = _lib.c_i64()
        check(lib().a3c_engine_exchange_split(self._h, ctypes.byref(cut)), 'a3c_engine_exchange_split')
        return int(cut.value)

    def wait_grad_head(self):
        """The current stream waits until the last rollout_grad's grads[split_point:] are clipped."""
        check(lib().a3c_engine_wait_grad_head(self._h, _lib.stream_handle()), 'a3c_engine_wait_grad_head')

    def apply_shard(self, grads_by_rank, nranks, lo, n, w_out):
        """Partitioned PS step 1: nranks sequential RMSProp steps of [lo, lo+n) -> w_out."""
        check(lib().a3c_engine_apply_shard(self._h, _lib.ptr(grads_by_rank), int(nranks), int(lo), int(n),
                                           _lib.ptr(w_out), _lib.stream_handle()), 'a3c_engine_apply_shard')

    def apply_commit(self, params_src=None):
        """Partitioned PS step 2: params <- params_src, snapshot / target sync, counters."""
        check(lib().a3c_engine_apply_commit(self._h, _lib.ptr(params_src), _lib.stream_handle()),
              'a3c_engine_apply_commit')

    def iterate(self, exchange=None):
        """One iteration: rollout + gradient, [exchange(grads)], apply.  Single-GPU device-env
        engines without an exchange take the fused path (a3c_engine_iterate: the apply enqueued with
        the backward, bit-identical to rollout_grad() + apply()).  An exchange with
        ``owns_apply`` (src.distributed.PartitionedPS) performs the apply itself."""
        if exchange is None and self.cfg.world_size == 1 and not self.external_env:
            check(lib().a3c_engine_iterate(self._h, _lib.stream_handle()), 'a3c_engine_iterate')
            return
        self.rollout_grad()
        if not self.grad_ready:          # overlap pipeline filling: no gradient yet
            return
        if getattr(exchange, 'owns_apply', False):
            exchange.apply(self)
            return
        if exchange is not None:
            exchange(self.grads)
        self.apply()

    # ---------------------------------------------------------------- summaries (agent.py:69-139)
    STATS = ('reward_sum', 'ep_reward_sum', 'ep_reward_max', 'ep_reward_min', 'games', 'loss_sum', 'q_sum',
             'updates', 'env_steps', 'policy_loss_sum', 'value_loss_sum', 'entropy_sum')

    def stats_accumulate(self):
        """Add the rollout whose gradient the last iterate() computed to the device aggregates."""
        check(lib().a3c_engine_stats_accumulate(self._h, _lib.stream_handle()), 'a3c_engine_stats_accumulate')

    def read_stats(self, reset=True):
        """train_with_summary's aggregates since the last read (agent.py:104-131) over this GPU's
        envs: avg reward per env-step, avg loss / q per update, episode max / min / avg reward,
        number of games."""
        out = (ctypes.c_double * 16)()
        check(lib().a3c_engine_stats_read(self._h, out, 1 if reset else 0, _lib.stream_handle()),
              'a3c_engine_stats_read')
        raw = dict(zip(self.STATS, list(out)[:len(self.STATS)]))
        games, upd, steps = raw['games'], raw['updates'], raw['env_steps']
        res = {'avg_reward': raw['reward_sum'] / steps if steps else 0.0,
               'avg_loss': raw['loss_sum'] / upd if upd else 0.0,
               'avg_q': raw['q_sum'] / upd if upd else 0.0,
               # agent.py:110-115: 0 when no episode finished in the interval
               'avg_ep_reward': raw['ep_reward_sum'] / games if games else 0.0,
               'max_ep_reward': raw['ep_reward_max'] if games else 0.0,
               'min_ep_reward': raw['ep_reward_min'] if games else 0.0,
               'num_game': int(games), 'updates': int(upd), 'env_steps': int(steps)}
        if self.algo == 'a3c' and upd:
            res.update(avg_policy_loss=raw['policy_loss_sum'] / upd, avg_value_loss=raw['value_loss_sum'] / upd,
                       avg_entropy=raw['entropy_sum'] / upd)
        return res

    # ---------------------------------------------------------------- checkpoint / resume
    @property
    def worker_step(self):
        """agent.py:55's loop counter (the lr / epsilon schedules' step) at the next rollout.
        Host-stepped engines before their first rollout: the device counters are written by
        ext_begin, so the step is the one set_step restored (0 on a fresh run)."""
        if self.external_env and not getattr(self, '_ext_began', False):
            return int(getattr(self, '_step0_w', 0))
        c = self.counters.cpu()
        return int(c[2]) + int(c[0]) - 3

    def set_step(self, global_step, worker_step=None):
        """Resume from parameters + step (the reference's Saver, agent.py:29): the global step and
        the workers' loop counter restart there (agent.py:34,46)."""
        w = global_step if worker_step is None else worker_step
        self._step0_w = int(w)
        check(lib().a3c_engine_set_step(self._h, int(global_step), int(w), _lib.stream_handle()),
              'a3c_engine_set_step')

    def save_state(self):
        """The whole engine state as a host u8 array (parameters, RMSProp slots, counters, envs,
        frame ring, LSTM carry, the overlap pipeline's rollout in flight)."""
        nb = _lib.c_i64()
        check(lib().a3c_engine_state_bytes(self._h, ctypes.byref(nb)), 'a3c_engine_state_bytes')
        buf = np.empty(int(nb.value), np.uint8)
        check(lib().a3c_engine_state_save(self._h, buf.ctypes.data_as(ctypes.c_void_p), buf.size,
                                          _lib.stream_handle()), 'a3c_engine_state_save')
        return buf

    def load_state(self, buf):
        """Restore save_state()'s array into this (reset) engine of the same configuration; the
        next iteration continues the saved run bit for bit."""
        buf = np.ascontiguousarray(np.asarray(buf, np.uint8))
        check(lib().a3c_engine_state_load(self._h, buf.ctypes.data_as(ctypes.c_void_p), buf.size,
                                          _lib.stream_handle()), 'a3c_engine_state_load')

    def advance(self):
        check(lib().a3c_engine_advance(self._h, _lib.stream_handle()), 'a3c_engine_advance')

    def iterate_hogwild(self, ps):
        """Rollout + gradient, unlocked push of the (per-worker clipped) gradient into the
        sharded Hogwild parameter server, pull of the shared parameters (src/hogwild.py).

        Overlap engine (the default of bench.py / main.py --update hogwild): rollout k runs on the
        engine's rollout stream while the caller's stream back-propagates rollout k-1, pushes its
        clipped gradient into every shard and pulls the shards into the parameter snapshot of
        rollout k+1 -- the push and pull overlap the next rollout, at staleness 1 like the overlap
        mode (the reference's workers keep acting while the PS applies, main.py:60-65).  Rollout
        k+1 is enqueued behind that pull (the engine orders its rollout stream after the caller's)."""
        self.rollout_grad()
        if not self.grad_ready:
            return                      # overlap pipeline filling: no gradient yet
        if self.cfg.world_size == 1:
            # one worker: the engine fuses its clip into apply, which hogwild bypasses
            if not hasattr(self, '_clip_ws'):
                b = _lib.c_i64()
                check(lib().a3c_optim_workspace_bytes(self.params.numel(), ctypes.byref(b)), 'ws')
                self._clip_ws = torch.empty(int(b.value), dtype=torch.uint8, device='cuda')
            check(lib().a3c_clip_grads(_lib.ptr(self.grads), len(self.offsets), _lib.i64_array(self.offsets),
                                       _lib.i64_array(self.sizes), float(self.cfg.clip_norm), None,
                                       _lib.ptr(self._clip_ws), _lib.stream_handle()), 'a3c_clip_grads')
        ps.push(self.grads, lr_dev=self.sched_ptr)
        # counters, the overlap snapshot, and for q the target copy of the pulled (global) weights
        # when the global step crossed a multiple of target_q_update_step (agent.py:166-167, 342-344)
        if ps.world == 1:
            self.apply_commit(ps.params_view())     # the one shard is the whole vector: pull = commit
        else:
            ps.pull(self.params)
            self.apply_commit(None)

    # ---------------------------------------------------------------- host-stepped envs
    def ext_begin(self, rgb):
        """external_env: first frames [E,210,160,3] u8 (pinned host or device) -> every history slot."""
        self._ext_check(rgb, torch.uint8, (self.E, 210, 160, 3), 'rgb')
        check(lib().a3c_engine_ext_begin(self._h, _lib.ptr(rgb), _lib.stream_handle()), 'a3c_engine_ext_begin')

    def ext_act(self, actions_out):
        """external_env: forward + draw of the next rollout step; actions -> actions_out [E] int32
        (pinned host: valid after the stream synchronises)."""
        self._ext_check(actions_out, torch.int32, (self.E,), 'actions_out')
        check(lib().a3c_engine_ext_act(self._h, _lib.ptr(actions_out), _lib.stream_handle()), 'a3c_engine_ext_act')

    def ext_upload(self, rgb, env_lo, env_hi):
        """external_env: the post-act frames of envs [env_lo, env_hi) only (rgb stays the full
        [E,210,160,3] buffer); finish the step with ext_observe(None, rewards, terminals)."""
        self._ext_check(rgb, torch.uint8, (self.E, 210, 160, 3), 'rgb')
        check(lib().a3c_engine_ext_upload(self._h, _lib.ptr(rgb), int(env_lo), int(env_hi), _lib.stream_handle()),
              'a3c_engine_ext_upload')

    def ext_observe(self, rgb, rewards, terminals):
        """external_env: the step's post-act frames (None: sent by ext_upload), rewards and
        terminals of every env."""
        if rgb is not None:
            self._ext_check(rgb, torch.uint8, (self.E, 210, 160, 3), 'rgb')
        self._ext_check(rewards, torch.float32, (self.E,), 'rewards')
        self._ext_check(terminals, torch.uint8, (self.E,), 'terminals')
        check(lib().a3c_engine_ext_observe(self._h, _lib.ptr(rgb), _lib.ptr(rewards), _lib.ptr(terminals),
                                           _lib.stream_handle()), 'a3c_engine_ext_observe')

    def _ext_check(self, t, dtype, shape, name):
        if not self.external_env:
            raise ValueError('engine was not created with external_env=True')
        if not isinstance(t, torch.Tensor) or t.dtype != dtype or tuple(t.shape) != shape or not t.is_contiguous():
            raise ValueError(f'{name} must be a contiguous {dtype} tensor of shape {shape}')
        if not t.is_cuda and not t.is_pinned():
            raise ValueError(f'{name}: host buffers must be pinned (async copies)')

    def begin_host(self, pool):
        """New random games of every host env; their first screens fill the history (ext_begin)."""
        self.ext_begin(pool.begin())
        self._ext_began = True
        self._ext_actions = torch.zeros(self.E, dtype=torch.int32).pin_memory()

    def rollout_host(self, pool):
        """The n env steps of one iteration with host-stepped envs (src/host_env.HostEnvPool): per
        rollout step the GPU draws the actions, the host steps every env, the post-act frames go
        back to the GPU for Environment.screen + History.add.  Finish with rollout_grad()."""
        if not getattr(self, '_ext_began', False):
            self.begin_host(pool)
        stream = torch.cuda.current_stream()
        # pools that step env ranges (SyntheticHostEnvPool) are stepped in `upload_chunks` ranges:
        # the H2D copy of one range runs while the host steps the next
        chunks = max(1, min(int(getattr(pool, 'upload_chunks', 1)), self.E)) if hasattr(pool, 'step_range') else 1
        bounds = [self.E * c // chunks for c in range(chunks + 1)]
        for _ in range(self.n):
            self.ext_act(self._ext_actions)
            stream.synchronize()            # actions on the host; the previous H2D copies are done
            acts = self._ext_actions.numpy()
            if chunks == 1:
                pool.step(acts)
                self.ext_observe(pool.rgb, pool.rewards, pool.terminals)
                continue
            for lo, hi in zip(bounds[:-1], bounds[1:]):
                pool.step_range(acts, lo, hi)
                self.ext_upload(pool.rgb, lo, hi)
            self.ext_observe(None, pool.rewards, pool.terminals)

    def iterate_host(self, pool, exchange=None):
        """One iteration with host-stepped envs: rollout_host, then loss, backward, exchange, apply."""
        self.rollout_host(pool)
        self.rollout_grad()
        if getattr(exchange, 'owns_apply', False):
            exchange.apply(self)
            return
        if exchange is not None:
            exchange(self.grads)
        self.apply()

    def span_stats(self, which, reset=False):
        """Live launch spans recorded by the kernels themselves (which 0: k_conv_bwd, 1:
        k_head_screen_conv12): reset=True clears; else (avg_us, max_us, launches)."""
        avg, mx, cnt = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
        check(lib().a3c_engine_span_stats(self._h, int(which), 1 if reset else 0, ctypes.byref(avg),
                                          ctypes.byref(mx), ctypes.byref(cnt)), 'a3c_engine_span_stats')
        return float(avg.value), float(mx.value), int(cnt.value)

    def span_steps(self):
        """k_head_screen_conv12's live spans split by rollout step: ([avg_us] * n, [launches] * n)."""
        avg = (ctypes.c_double * self.n)()
        cnt = (ctypes.c_int64 * self.n)()
        check(lib().a3c_engine_span_steps(self._h, avg, cnt), 'a3c_engine_span_steps')
        return [round(float(a), 2) for a in avg], [int(c) for c in cnt]

    def time_kernel(self, kernel, iters=20):
        """Average device ms of one engine kernel (HIP events on the current stream)."""
        out = ctypes.c_float()
        check(lib().a3c_engine_time_kernel(self._h, int(kernel), int(iters), _lib.stream_handle(),
                                           ctypes.byref(out)), 'a3c_engine_time_kernel')
        return float(out.value)

    @property
    def env_steps_per_iteration(self):
        return self.E * self.n

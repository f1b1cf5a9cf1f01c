"""Checkpoints keyed by TensorFlow variable names.

The reference checkpoints with a Saver over the prediction weights plus the global ``step``
(agent.py:29, ``tf.train.Saver(self.w.values() + [self.step_op], max_to_keep=30)``), written by the
Supervisor every 600 s (main.py:74-80) into ``./logs/<model_dir>`` and restored by
``managed_session`` (main.py:90); training resumes at the restored step (agent.py:34,46).

Here a checkpoint is ``<dir>/model.ckpt-<step>.npz`` (numpy, loaded with allow_pickle=False) whose
keys are the TF variable names the reference's graph would give each tensor:

* Q-learning agent (agent.py:218-252, ``prediction`` scope, ops.py ``w``/``biases``/``Matrix``/
  ``bias``): ``prediction/l1/w``, ``prediction/l1/biases``, ``prediction/l2/w``, ...,
  ``prediction/l3/Matrix``, ``prediction/l3/bias``, ``prediction/q/Matrix``, ``prediction/q/bias``;
  the target network (agent.py:257-296) ``target/target_l1/w`` ...;
* A3C network (network.py:43-79): ``l1_conv/w``, ``l1_conv/biases``, ``l2_conv/...``,
  ``l4_linear/Matrix``, ``l4_linear/bias``, ``policy/linear/Matrix``, ``policy/linear/bias``,
  ``value/linear/Matrix``, ``value/linear/bias`` (the nature trunk under ``Nature_DQN/``);
* C5 LSTM head (build-defined, TF1 BasicLSTMCell naming): ``lstm/basic_lstm_cell/weights``,
  ``lstm/basic_lstm_cell/biases``;
* ``step``: the global step (the reference's ``step`` variable).

Beyond what the reference's Saver keeps, the file also holds the RMSProp slots under TF1's slot
names (``<var>/RMSProp`` = ms, ``<var>/RMSProp_1`` = momentum) and, for the batched engine, the
whole engine state (``__engine_state__``: counters, env state, frame ring, LSTM carry, the overlap
pipeline's rollout in flight), so that a resumed run continues bit for bit.  With several GPUs each
rank writes its own env shard's state to ``model.ckpt-<step>.rank<r>.npz``.  A ``checkpoint``
index file (JSON) lists the kept checkpoints, newest last; ``max_to_keep`` (30) bounds it.  The
``world`` key records how many ranks wrote the checkpoint: the engine states are only taken back by
a run of the same size (each rank's env shard); any other run resumes from parameters + step.
"""
import glob
import json
import os
import sys
import zipfile

import numpy as np

STEP_KEY = 'step'
STATE_KEY = '__engine_state__'
WSTEP_KEY = '__worker_step__'

_Q = {'l1_w': 'l1/w', 'l1_b': 'l1/biases', 'l2_w': 'l2/w', 'l2_b': 'l2/biases',
      'l3_w': 'l3/Matrix', 'l3_b': 'l3/bias', 'q_w': 'q/Matrix', 'q_b': 'q/bias',
      # dueling (agent.py:234-249)
      'l3_val_w': 'value_hid/Matrix', 'l3_val_b': 'value_hid/bias', 'l3_adv_w': 'adv_hid/Matrix',
      'l3_adv_b': 'adv_hid/bias', 'val_w_out': 'value_out/Matrix', 'val_w_b': 'value_out/bias',
      'adv_w_out': 'adv_out/Matrix', 'adv_w_b': 'adv_out/bias'}
_A3C_NIPS = {'l1_w': 'l1_conv/w', 'l1_b': 'l1_conv/biases', 'l2_w': 'l2_conv/w', 'l2_b': 'l2_conv/biases',
             'l4_w': 'l4_linear/Matrix', 'l4_b': 'l4_linear/bias',
             'p_w': 'policy/linear/Matrix', 'p_b': 'policy/linear/bias',
             'q_w': 'value/linear/Matrix', 'q_b': 'value/linear/bias',
             'lstm_w': 'lstm/basic_lstm_cell/weights', 'lstm_b': 'lstm/basic_lstm_cell/biases'}


def tf_name(name, algo='a3c', dqn_type='nips'):
    """TF variable name of flat tensor ``name`` (the python dict keys of agent.py / network.py)."""
    if algo == 'q':
        return 'prediction/' + _Q[name]
    if dqn_type.lower() == 'nature':
        m = dict(_A3C_NIPS, l3_w='l3_conv/w', l3_b='l3_conv/biases')
        n = m[name]
        return n if n.split('/')[0] in ('policy', 'value', 'lstm') else 'Nature_DQN/' + n
    return _A3C_NIPS[name]


def tf_target_name(name):
    """agent.py:257-296: the target network's layers are ``target_<layer>`` under ``target``."""
    layer, var = _Q[name].split('/')
    return 'target/target_%s/%s' % (layer, var)


def slot_names(var):
    """TF1 RMSPropOptimizer slot variables of ``var``: (rms, momentum)."""
    return var + '/RMSProp', var + '/RMSProp_1'


class Saver(object):
    """tf.train.Saver stand-in: ``save(arrays, step)`` -> ``<dir>/model.ckpt-<step>.npz`` and the
    index; ``latest()`` -> newest kept path (tf.train.latest_checkpoint)."""

    def __init__(self, directory, max_to_keep=30, basename='model.ckpt'):
        self.dir, self.max_to_keep, self.basename = directory, int(max_to_keep), basename

    @property
    def index_path(self):
        return os.path.join(self.dir, 'checkpoint')

    def path(self, step, rank=0):
        p = os.path.join(self.dir, '%s-%d' % (self.basename, int(step)))
        return p + ('.rank%d.npz' % rank if rank else '.npz')

    def _resolve(self, p):
        """Index entries are file names relative to the index's directory (as tf.train writes
        them), so a run resumed from another working directory finds them; older indices held
        paths as built from checkpoint_dir: every checkpoint lives in self.dir, so the base name
        resolves both."""
        return os.path.join(self.dir, os.path.basename(p))

    def kept(self):
        try:
            with open(self.index_path) as f:
                return [self._resolve(p) for p in json.load(f)['all_model_checkpoint_paths']]
        except (OSError, ValueError, KeyError, TypeError):
            return []

    def latest(self):
        k = self.kept()
        for p in reversed(k):
            if os.path.exists(p):
                return p
        return None

    def write(self, arrays, step, rank=0):
        """Write one file (every rank its own); the index is updated by ``commit``."""
        os.makedirs(self.dir, exist_ok=True)
        path = self.path(step, rank)
        tmp = path[:-4] + '.tmp.npz'
        np.savez(tmp, **arrays)
        os.replace(tmp, path)
        return path

    def commit(self, step):
        """Rank 0, after every rank wrote: add the checkpoint to the index, drop the oldest beyond
        max_to_keep (with their rank files)."""
        path = self.path(step)
        kept = [p for p in self.kept() if p != path] + [path]
        while self.max_to_keep > 0 and len(kept) > self.max_to_keep:
            old = kept.pop(0)
            for f in [old] + glob.glob(old[:-4] + '.rank*.npz'):
                try:
                    os.remove(f)
                except OSError:
                    pass
        tmp = self.index_path + '.tmp'
        with open(tmp, 'w') as f:
            json.dump({'model_checkpoint_path': os.path.basename(path),
                       'all_model_checkpoint_paths': [os.path.basename(p) for p in kept]}, f)
        os.replace(tmp, self.index_path)
        return path

    def save(self, arrays, step):
        self.write(arrays, step)
        return self.commit(step)


def load(path):
    with np.load(path, allow_pickle=False) as f:
        return {k: f[k] for k in f.files}


# ------------------------------------------------------------------------------ batched engine
def engine_arrays(eng, names_shapes, with_state=True):
    """The engine's parameters (+ target for q, RMSProp slots, step) keyed by TF names, and its
    whole state blob."""
    algo, dqn = eng.algo, getattr(eng, 'dqn_type', 'nips')
    state = eng.save_state() if with_state else None     # (first: waits for every engine stream)

    def tensors(flat):
        f = flat.detach().cpu().numpy()
        return {name: f[off:off + sz].reshape(shp).copy()
                for (name, shp), off, sz in zip(names_shapes, eng.offsets, eng.sizes)}
    P, MS, MOM = tensors(eng.params), tensors(eng.ms), tensors(eng.mom)
    out = {}
    for name, _ in names_shapes:
        tn = tf_name(name, algo, dqn)
        out[tn] = P[name]
        rms, mom = slot_names(tn)
        out[rms], out[mom] = MS[name], MOM[name]
    if algo == 'q':
        T = tensors(eng.target_params)
        for name, _ in names_shapes:
            out[tf_target_name(name)] = T[name]
    out[STEP_KEY] = np.array(int(eng.counters[1].item()), np.int64)
    if hasattr(eng, 'worker_step'):
        # the workers' own loop counter (agent.py:55); the reference's Saver keeps only `step` and
        # resumes every worker at it (agent.py:34,46) -- kept so that a resume without the engine
        # state (host-stepped envs) continues at the worker step it left
        out[WSTEP_KEY] = np.array(int(eng.worker_step), np.int64)
    if state is not None:
        out[STATE_KEY] = state
    return out


def engine_restore(eng, names_shapes, arrays, state=None):
    """Restore into a created engine.  With a state blob of the same configuration: the exact
    state (bit-continuous).  Otherwise the reference's resume: parameters (and whatever of the
    target / RMSProp slots the file has) on freshly reset envs, global and worker step at the
    restored ``step`` (agent.py:34,46) -- the worker step at the saved ``__worker_step__`` when the
    file has one.  Returns the global step."""
    import torch
    algo, dqn = eng.algo, getattr(eng, 'dqn_type', 'nips')
    step = int(arrays[STEP_KEY])
    if state is not None and not eng.external_env:
        eng.reset()
        try:
            eng.load_state(state)
            return step
        except RuntimeError:
            pass        # another engine configuration: fall back to params + step

    def flat(get, default=None):
        out = np.zeros(eng.params.numel(), np.float32)
        for (name, shp), off, sz in zip(names_shapes, eng.offsets, eng.sizes):
            v = get(name)
            if v is None:
                if default is None:
                    return None
                v = default[off:off + sz]
            out[off:off + sz] = np.asarray(v, np.float32).reshape(-1)
        return out
    P = flat(lambda n: arrays.get(tf_name(n, algo, dqn)))
    if P is None:
        missing = [tf_name(n, algo, dqn) for n, _ in names_shapes if tf_name(n, algo, dqn) not in arrays]
        raise ValueError('checkpoint lacks %s' % missing)
    eng.reset(P)
    if algo == 'q':
        T = flat(lambda n: arrays.get(tf_target_name(n)), P)
        eng.target_params.copy_(torch.as_tensor(T))
    ms = flat(lambda n: arrays.get(slot_names(tf_name(n, algo, dqn))[0]))
    mom = flat(lambda n: arrays.get(slot_names(tf_name(n, algo, dqn))[1]))
    if ms is not None and mom is not None:
        eng.ms.copy_(torch.as_tensor(ms))
        eng.mom.copy_(torch.as_tensor(mom))
    eng.set_step(step, int(arrays.get(WSTEP_KEY, step)))
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    return step


def save_engine(saver, eng, names_shapes, rank=0, world=1, barrier=None):
    """Every rank writes its file (rank 0: parameters + its state; rank r: its state), then rank 0
    commits the index once all are on disk (``barrier``: a callable, e.g. dist.barrier)."""
    step = int(eng.counters[1].item())
    if rank == 0:
        arrays = engine_arrays(eng, names_shapes, with_state=not eng.external_env)
        arrays['world'] = np.array(world)
        saver.write(arrays, step)
    elif not eng.external_env:
        saver.write({STATE_KEY: eng.save_state(), 'world': np.array(world)}, step, rank)
    if barrier is not None and world > 1:
        barrier()
    if rank == 0:
        saver.commit(step)
    return step


def _collectives(world):
    """(broadcast_object from rank 0, all-ranks AND of a flag) over torch.distributed, or the
    one-rank identities."""
    import torch.distributed as dist
    if world == 1 or not dist.is_initialized():
        return (lambda obj: obj), (lambda ok: bool(ok))

    def bcast(obj):
        box = [obj]
        dist.broadcast_object_list(box, src=0)
        return box[0]

    def all_ok(ok):
        box = [None] * dist.get_world_size()
        dist.all_gather_object(box, bool(ok))
        return all(box)
    return bcast, all_ok


def restore_engine(saver, eng, names_shapes, rank=0, world=1):
    """Restore the newest checkpoint of ``saver`` (None if there is none) on every rank alike.

    Rank 0 picks the checkpoint and the path -- none, the exact engine states (written by as many
    ranks: each rank takes its own env shard's state), or parameters + step like the reference --
    and broadcasts it; every rank then checks that it can follow, and the ranks agree on the
    outcome: a rank that cannot read the parameter file fails every rank together; a rank whose
    state file is missing or does not load sends every rank to the parameters + step path (the
    ranks then verify they restored rank 0's parameters bit for bit).  So the ranks never take different paths and their
    collectives keep matching (the exact path restores the overlap pipeline in flight)."""
    bcast, all_ok = _collectives(world)
    plan = None
    if rank == 0:
        path = saver.latest()
        if path is not None:
            try:
                w = int(load(path).get('world', -1))
            except Exception:      # (a truncated zip raises BadZipFile, a short read EOFError, ...)
                w = -2
            plan = (os.path.basename(path), 'exact' if w == world and not eng.external_env else 'params')
    plan = bcast(plan)
    if plan is None:
        return None
    path = os.path.join(saver.dir, plan[0])
    try:
        arrays = load(path)
        err = None
    except Exception as e:         # any failure goes through the agreed all_ok path below
        arrays, err = None, e
    if not all_ok(arrays is not None):
        raise RuntimeError('restore_engine: a rank cannot read %s (%s)' % (path, err or 'another rank'))
    if plan[1] == 'exact':
        from . import _lib
        ok, unusable, fatal = False, None, None
        try:
            state = arrays.get(STATE_KEY) if rank == 0 else load(path[:-4] + '.rank%d.npz' % rank).get(STATE_KEY)
            if state is not None:
                eng.reset()
                eng.load_state(state)
                ok = True
            else:
                unusable = 'no engine state in the file'
        except _lib.A3CError as e:
            # a state of another engine configuration / format version is unusable (fall back to
            # parameters + step); a HIP failure is a device fault and must not be papered over
            if e.device_fault:
                fatal = e
            else:
                unusable = e
        except (OSError, EOFError, KeyError, ValueError, zipfile.BadZipFile) as e:    # missing / damaged file
            unusable = e
        except Exception as e:             # programming errors are not a reason to fall back either
            fatal = e
        # every rank reaches both agreements, so a failure on one rank never strands the others
        if not all_ok(fatal is None):
            raise RuntimeError('restore_engine: rank %d: restoring the engine state from %s failed (%s)'
                               % (rank, path, fatal if fatal is not None else 'on another rank')) from fatal
        if unusable is not None:
            print('[rank %d] restore_engine: the engine state of %s is unusable (%s); resuming from parameters '
                  '+ step' % (rank, path, unusable), file=sys.stderr, flush=True)
        if all_ok(ok):
            return int(arrays[STEP_KEY])
    step = engine_restore(eng, names_shapes, arrays, None)
    if world > 1:   # every rank read rank 0's file: the replicas must hold rank 0's parameters exactly
        import hashlib
        digest = hashlib.sha1(eng.params.detach().cpu().numpy().tobytes()).hexdigest()
        if not all_ok(digest == bcast(digest)):
            raise RuntimeError('restore_engine: the ranks restored different parameters from %s' % path)
    return step

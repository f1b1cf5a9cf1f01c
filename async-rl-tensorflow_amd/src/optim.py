"""RMSPropOptimizer with TF1 semantics (main.py:63-65 ``tf.train.RMSPropOptimizer(lr_op,
decay=0.99, momentum=0, epsilon=0.1)``): rms slot initialised to 1.0, momentum slot to 0,
ms += (g^2 - ms)(1 - decay); mom = mom*momentum + lr*g/sqrt(ms + epsilon); w -= mom, with the
per-tensor clip_by_norm of agent.py:316-319 fused in (a3c_clip_rmsprop_apply).  Works on a flat
fp32 parameter buffer + the tensor table of the C-ABI layout."""
import ctypes

import torch

from . import _lib
from ._lib import check, lib, ptr, stream_handle


class RMSPropOptimizer(object):
  def __init__(self, learning_rate, decay=0.9, momentum=0.0, epsilon=1e-10, clip_norm=40.0):
    self.learning_rate = learning_rate      # float, or a callable returning the current lr (lr_op)
    self.decay, self.momentum, self.epsilon = float(decay), float(momentum), float(epsilon)
    self.clip_norm = float(clip_norm)
    self._slots = {}

  def slots(self, flat):
    key = flat.data_ptr()
    if key not in self._slots:
      self._slots[key] = (torch.ones_like(flat), torch.zeros_like(flat))
    return self._slots[key]

  def lr(self):
    return float(self.learning_rate() if callable(self.learning_rate) else self.learning_rate)

  def _ws(self, like):
    b = _lib.c_i64()
    check(lib().a3c_optim_workspace_bytes(int(like.numel()), ctypes.byref(b)), 'a3c_optim_workspace_bytes')
    return torch.empty(int(b.value), dtype=torch.uint8, device=like.device)

  def clip_only(self, flat_grads, offsets, sizes, sumsq=None):
    """Per-tensor clip_by_norm in place (each worker before the multi-GPU SUM all-reduce)."""
    check(lib().a3c_clip_grads(ptr(flat_grads), len(offsets), _lib.i64_array(offsets), _lib.i64_array(sizes),
                               self.clip_norm, ptr(sumsq), ptr(self._ws(flat_grads)), stream_handle()),
          'a3c_clip_grads')

  def apply_gradients(self, flat_params, flat_grads, offsets, sizes, lr=None, sumsq=None, clip=True):
    """clip (unless clip=False: already clipped per worker) + RMSProp apply."""
    ms, mom = self.slots(flat_params)
    ws = self._ws(flat_params)
    check(lib().a3c_clip_rmsprop_apply(ptr(flat_params), ptr(ms), ptr(mom), ptr(flat_grads), len(offsets),
                                       _lib.i64_array(offsets), _lib.i64_array(sizes),
                                       float(self.lr() if lr is None else lr), self.decay, self.momentum,
                                       self.epsilon, self.clip_norm if clip else 0.0, ptr(sumsq), ptr(ws), stream_handle()),
          'a3c_clip_rmsprop_apply')

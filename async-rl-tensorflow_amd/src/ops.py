"""ops.py:1-46 drop-ins: ``conv2d`` and ``linear`` build their variables and return
``(out, w, b)`` like the reference, computing on device with the generic HIP kernels
(a3c_conv2d_forward/backward, a3c_matmul); gradients flow through torch.autograd into the same
kernels.  Variables use TF's layouts: conv ``w`` [kh,kw,cin,cout] + ``biases`` (ops.py:16-24),
linear ``Matrix`` [in,out] + ``bias`` (ops.py:36-39).

Initialisers mirror the TF ones the reference passes (agent.py:214, network.py:10, ops.py:8,37).
"""
import math

import numpy as np
import torch

from . import _lib
from ._lib import check, lib, ptr, stream_handle


# ---- initialisers (TF names) ---------------------------------------------------------
def truncated_normal_initializer(mean=0.0, stddev=1.0, seed=None):
  rng = np.random.default_rng(seed)

  def init(shape):
    v = rng.standard_normal(shape)
    bad = np.abs(v) > 2.0
    while bad.any():
      v[bad] = rng.standard_normal(int(bad.sum()))
      bad = np.abs(v) > 2.0
    return (mean + stddev * v).astype(np.float32)
  return init


def random_normal_initializer(mean=0.0, stddev=1.0, seed=None):
  rng = np.random.default_rng(seed)
  return lambda shape: (mean + stddev * rng.standard_normal(shape)).astype(np.float32)


def constant_initializer(value=0.0):
  return lambda shape: np.full(shape, value, np.float32)


def xavier_initializer(uniform=True, seed=None):
  """tf.contrib.layers.xavier_initializer (ops.py:8 default): fan_in/fan_out of a conv kernel
  are receptive field * channels."""
  rng = np.random.default_rng(seed)

  def init(shape):
    rf = int(np.prod(shape[:-2])) if len(shape) > 2 else 1
    fan_in, fan_out = shape[-2] * rf, shape[-1] * rf
    if uniform:
      lim = math.sqrt(6.0 / (fan_in + fan_out))
      return rng.uniform(-lim, lim, shape).astype(np.float32)
    std = math.sqrt(2.0 / (fan_in + fan_out))
    return truncated_normal_initializer(0.0, std, int(rng.integers(1 << 31)))(shape)
  return init


def relu(x):
  """tf.nn.relu; recognised by conv2d/linear and fused into the kernel epilogue."""
  return torch.relu(x)


def _is_relu(fn):
  return fn is relu or fn is torch.relu or fn is torch.nn.functional.relu or fn == 'relu'


# ---- autograd functions over the HIP kernels -------------------------------------------
class _Conv2d(torch.autograd.Function):
  @staticmethod
  def forward(ctx, x, w, b, stride, nhwc, fuse_relu):
    x = x.contiguous()
    w = w.contiguous()
    if nhwc:
      N, H, W, C = x.shape
    else:
      N, C, H, W = x.shape
    KH, KW, C2, OC = w.shape
    if C2 != C:
      raise ValueError('conv2d: input has %d channels, kernel expects %d' % (C, C2))
    SH, SW = stride
    OH, OW = (H - KH) // SH + 1, (W - KW) // SW + 1
    y = torch.empty((N, OH, OW, OC) if nhwc else (N, OC, OH, OW), dtype=torch.float32, device=x.device)
    check(lib().a3c_conv2d_forward(ptr(x), ptr(w), ptr(b), ptr(y), N, H, W, C, KH, KW, SH, SW, OC, int(nhwc),
                                   int(fuse_relu), stream_handle()), 'a3c_conv2d_forward')
    ctx.save_for_backward(x, w, y)
    ctx.meta = (N, H, W, C, KH, KW, SH, SW, OC, int(nhwc), fuse_relu, b is not None)
    return y

  @staticmethod
  def backward(ctx, gy):
    x, w, y = ctx.saved_tensors
    N, H, W, C, KH, KW, SH, SW, OC, nhwc, fuse_relu, has_b = ctx.meta
    gy = gy.contiguous()
    if fuse_relu:
      gy = torch.where(y > 0, gy, torch.zeros_like(gy))
    dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
    dw = torch.empty_like(w) if ctx.needs_input_grad[1] else None
    db = torch.empty(OC, dtype=torch.float32, device=x.device) if (has_b and ctx.needs_input_grad[2]) else None
    check(lib().a3c_conv2d_backward(ptr(x), ptr(w), ptr(gy), ptr(dx), ptr(dw), ptr(db), N, H, W, C, KH, KW, SH, SW,
                                    OC, nhwc, stream_handle()), 'a3c_conv2d_backward')
    return dx, dw, db, None, None, None


def _matmul(A, B, bias=None, fuse_relu=False, transA=False, transB=False):
  """C = op(A) @ op(B) (+ bias) (relu) on the HIP strided matmul."""
  M = A.shape[1] if transA else A.shape[0]
  K = A.shape[0] if transA else A.shape[1]
  N = B.shape[0] if transB else B.shape[1]
  A = A.contiguous()
  B = B.contiguous()
  C = torch.empty((M, N), dtype=torch.float32, device=A.device)
  sam, sak = (1, A.shape[1]) if transA else (A.shape[1], 1)
  sbk, sbn = (1, B.shape[1]) if transB else (B.shape[1], 1)
  check(lib().a3c_matmul(ptr(A), sam, sak, ptr(B), sbk, sbn, ptr(C), N, M, N, K, ptr(bias), int(fuse_relu), 0,
                         stream_handle()), 'a3c_matmul')
  return C


class _Linear(torch.autograd.Function):
  @staticmethod
  def forward(ctx, x, w, b, fuse_relu):
    y = _matmul(x, w, b, fuse_relu)
    ctx.save_for_backward(x, w, y)
    ctx.fuse_relu = fuse_relu
    ctx.has_b = b is not None
    return y

  @staticmethod
  def backward(ctx, gy):
    x, w, y = ctx.saved_tensors
    gy = gy.contiguous()
    if ctx.fuse_relu:
      gy = torch.where(y > 0, gy, torch.zeros_like(gy))
    dx = _matmul(gy, w, transB=True) if ctx.needs_input_grad[0] else None
    dw = _matmul(x, gy, transA=True) if ctx.needs_input_grad[1] else None
    db = None
    if ctx.has_b and ctx.needs_input_grad[2]:
      ones = torch.ones((gy.shape[0], 1), dtype=torch.float32, device=gy.device)
      db = _matmul(ones, gy, transA=True).reshape(-1)
    return dx, dw, db, None


def _param(value, device):
  return torch.nn.Parameter(torch.as_tensor(value, dtype=torch.float32, device=device))


def conv2d(x, output_dim, kernel_size, stride, initializer=None, activation_fn=relu, data_format='NHWC',
           padding='VALID', name='conv2d', w=None, b=None):
  """ops.py:4-30.  Returns (out, w, b).  ``w``/``b`` may be passed to reuse variables
  (the reference shares them through tf variable scopes)."""
  if data_format not in ('NHWC', 'NCHW'):
    raise ValueError('unknown data_format : %s' % data_format)
  if padding != 'VALID':
    raise ValueError('only VALID padding is used by the reference (ops.py:11)')
  cin = x.shape[-1] if data_format == 'NHWC' else x.shape[1]
  kernel_shape = [kernel_size[0], kernel_size[1], int(cin), output_dim]
  init = initializer if initializer is not None else xavier_initializer()
  if w is None:
    w = _param(init(kernel_shape), x.device)
  if b is None:
    b = _param(np.zeros(output_dim, np.float32), x.device)
  fuse = _is_relu(activation_fn)
  out = _Conv2d.apply(x.float(), w, b, tuple(stride), data_format == 'NHWC', fuse)
  if activation_fn is not None and not fuse:
    out = activation_fn(out)
  return out, w, b


def linear(input_, output_size, stddev=0.02, bias_start=0.0, activation_fn=None, name='linear', w=None, b=None):
  """ops.py:32-46.  Returns (out, w, b); w ``Matrix`` [in,out] ~ N(0, stddev), b = bias_start."""
  shape = list(input_.shape)
  x = input_.reshape(shape[0], -1).float()
  if w is None:
    w = _param(random_normal_initializer(stddev=stddev)([x.shape[1], output_size]), x.device)
  if b is None:
    b = _param(np.full(output_size, bias_start, np.float32), x.device)
  fuse = _is_relu(activation_fn)
  out = _Linear.apply(x, w, b, fuse)
  if activation_fn is not None and not fuse:
    out = activation_fn(out)
  return out, w, b

"""Network (network.py:6-127): the A3C policy/value net with the reference constructor.

* ``DQN_type='nips'`` (network.py:43-52: conv 16/32 + fc 256) runs on the fused HIP kernels of
  the batched engine (a3c_forward / a3c_loss_backward, include/a3c_hip.h) over one flat fp32
  parameter buffer in the C-ABI layout.
* ``DQN_type='nature'`` (network.py:30-42: conv 32/64/64 + fc 512) runs on the nature trunk's
  implicit-GEMM MFMA kernels (a3c_nature_forward / a3c_nature_loss_backward, nature.hip) with
  history_length 4 and NHWC (main.py:45); other history lengths and NCHW (whose fc weights follow
  the (c,h,w) flatten) take the generic HIP conv2d/matmul kernels (src/ops.py) with torch.autograd.

The loss follows network.py:81-94 with the SURVEY §8 A11 fixes: V squeezed to [B], log pi(a)
gathered from log_softmax (no placeholder), advantage stop-gradient unless ``literal_adv``.
``copy_from_global`` (network.py:96-107), ``save_model`` / ``load_model`` (:109-127) keep their
signatures; the TF Session/Saver arguments are accepted and ignored.
"""
import glob
import os

import numpy as np
import torch

from . import _lib
from . import kernels as K
from . import ops
from . import checkpoint as C
from .base import copy_named, load_checkpoint, save_checkpoint


def _align(n, a=64):
  return (n + a - 1) // a * a


def nature_names_shapes(history_length, action_size):
  """network.py:30-42 + heads :60,79 (TF variable shapes)."""
  A = int(action_size)
  return [('l1_w', (8, 8, history_length, 32)), ('l1_b', (32,)), ('l2_w', (4, 4, 32, 64)), ('l2_b', (64,)),
          ('l3_w', (3, 3, 64, 64)), ('l3_b', (64,)), ('l4_w', (7 * 7 * 64, 512)), ('l4_b', (512,)),
          ('p_w', (512, A)), ('p_b', (A,)), ('q_w', (512, 1)), ('q_b', (1,))]


class Network(object):
  def __init__(self, sess, data_format, history_length,
               screen_height, screen_width,
               action_size, activation_fn=ops.relu,
               initializer=ops.truncated_normal_initializer(0, 0.02),
               gamma=0.01, beta=0.0, global_network=None, global_optim=None, DQN_type='',
               literal_adv=False, device='cuda', seed=None):
    self.sess = sess
    if data_format not in ('NHWC', 'NCHW'):
      raise ValueError("unknown data_format : %s" % data_format)       # network.py:21
    self.data_format = data_format
    self.dqn_type = DQN_type.lower()
    if self.dqn_type not in ('nature', 'nips'):
      raise ValueError('Wrong DQN type: %s' % DQN_type)                # network.py:54
    if not ops._is_relu(activation_fn):
      raise ValueError('the HIP kernels fuse relu; activation_fn must be relu (network.py:9)')
    if (screen_height, screen_width) != (84, 84):
      raise ValueError('the HIP kernels are specialised for 84x84 screens (config.py:38-39)')
    if self.dqn_type == 'nips' and history_length != 4:
      raise ValueError('the fused nips kernels take history_length 4 (config.py:21)')
    _lib.require_device()
    self.history_length = int(history_length)
    self.action_size = int(action_size)
    self.gamma, self.beta, self.literal_adv = gamma, float(beta), bool(literal_adv)
    self.global_network, self.global_optim = global_network, global_optim
    self.device = device

    self._ws = {}
    self.nat = None
    if self.dqn_type == 'nips':
      self.net = K.Net(self.action_size, 'a3c')
      self.names_shapes = self.net.names_shapes
      self.offsets, self.sizes, total = self.net.offsets, self.net.sizes, self.net.total
    elif self.history_length == 4 and data_format == 'NHWC':   # the nature trunk's kernels (nature.hip):
      # their fc reads the (h,w,c) flatten of NHWC (agent.py:231-232); NCHW flattens (c,h,w)
      self.net = None
      self.nat = K.NatureNet(self.action_size)
      self.names_shapes = self.nat.names_shapes
      self.offsets, self.sizes, total = self.nat.offsets, self.nat.sizes, self.nat.total
    else:
      self.net = None
      self.names_shapes = nature_names_shapes(self.history_length, self.action_size)
      self.offsets, self.sizes, off = [], [], 0
      for _, shp in self.names_shapes:
        n = int(np.prod(shp))
        self.offsets.append(off)
        self.sizes.append(n)
        off = _align(off + n)
      total = off
    self.flat = torch.zeros(total, dtype=torch.float32, device=device)
    if seed is not None and initializer is Network.__init__.__defaults__[1]:
      initializer = ops.truncated_normal_initializer(0, 0.02, seed=seed)
    lin_init = ops.random_normal_initializer(stddev=0.02, seed=None if seed is None else seed + 1)
    for (name, shp), o, n in zip(self.names_shapes, self.offsets, self.sizes):
      if name.endswith('_b'):
        continue
      init = initializer if len(shp) == 4 else lin_init   # ops.py:37
      self.flat[o:o + n] = torch.as_tensor(init(list(shp))).reshape(-1).to(device)
    self.w = {name: self.flat[o:o + n].view(shp)
              for (name, shp), o, n in zip(self.names_shapes, self.offsets, self.sizes)}

  # ---------------------------------------------------------------------------------
  def _planes(self, s_t):
    """s_t -> u8 [B,L,84,84] planes (the fused kernels' layout).  Accepts u8 planes directly,
    or the reference's float placeholder layout (NHWC [B,84,84,L] / NCHW [B,L,84,84])."""
    if s_t.dtype == torch.uint8 and s_t.dim() == 4 and s_t.shape[1] == self.history_length:
      return s_t.to(self.device).contiguous()
    s = torch.as_tensor(s_t, device=self.device)
    if s.dim() == 3:
      s = s.unsqueeze(0)
    if self.data_format == 'NHWC':
      s = s.permute(0, 3, 1, 2)
    return s.round().clamp(0, 255).to(torch.uint8).contiguous()

  def _workspace(self, B):
    if B not in self._ws:
      self._ws[B] = (self.net or self.nat).workspace(B, self.device)
    return self._ws[B]

  def _nature_z(self, flat, planes):
    w = {name: flat[o:o + n].view(shp) for (name, shp), o, n in zip(self.names_shapes, self.offsets, self.sizes)}
    x = planes.float() / 255.                                    # network.py:34
    nchw = self.data_format == 'NCHW'
    if not nchw:
      x = x.permute(0, 2, 3, 1).contiguous()
    fmt = self.data_format
    l1, _, _ = ops.conv2d(x, 32, [8, 8], [4, 4], data_format=fmt, w=w['l1_w'], b=w['l1_b'])
    l2, _, _ = ops.conv2d(l1, 64, [4, 4], [2, 2], data_format=fmt, w=w['l2_w'], b=w['l2_b'])
    l3, _, _ = ops.conv2d(l2, 64, [3, 3], [1, 1], data_format=fmt, w=w['l3_w'], b=w['l3_b'])
    l4, _, _ = ops.linear(l3, 512, activation_fn=ops.relu, w=w['l4_w'], b=w['l4_b'])
    logits, _, _ = ops.linear(l4, self.action_size, w=w['p_w'], b=w['p_b'])
    value, _, _ = ops.linear(l4, 1, w=w['q_w'], b=w['q_b'])
    return logits, value[:, 0]

  def forward(self, s_t):
    """network.py:60-79 evaluated: policy_logits, policy, log_policy, policy_entropy, value."""
    planes = self._planes(s_t)
    if self.net is not None or self.nat is not None:
      z = self.z(planes)
      logits, value = z[:, :self.action_size], z[:, self.action_size]
    else:
      with torch.no_grad():
        logits, value = self._nature_z(self.flat, planes)
    log_policy = torch.log_softmax(logits.double(), dim=1)
    policy = log_policy.exp()
    return dict(policy_logits=logits, policy=policy.float(), log_policy=log_policy.float(),
                policy_entropy=(-(policy * log_policy).sum(1)).float(), value=value)

  def z(self, s_t):
    """[B, zs] logits | V rows, the layout a3c_select_action reads."""
    planes = self._planes(s_t)
    if self.net is not None:
      return self.net.forward(self.flat, planes, save_l1=False, workspace=self._workspace(int(planes.shape[0])))['z']
    if self.nat is not None:
      return self.nat.forward(self.flat, planes, workspace=self._workspace(int(planes.shape[0])))['z']
    with torch.no_grad():
      logits, value = self._nature_z(self.flat, planes)
    zs = (self.action_size + 1 + 3) // 4 * 4
    z = torch.zeros((planes.shape[0], zs), dtype=torch.float32, device=self.device)
    z[:, :self.action_size] = logits
    z[:, self.action_size] = value
    return z

  def sample_action(self, s_t, seed=123, step=0, env_ids=None):
    """batch_sample (network.py:72): categorical draw from pi, Philox-keyed by (seed, step, env)."""
    return K.select_action(0, self.z(s_t), self.action_size, seed, step, env_ids=env_ids)

  def loss_backward(self, s_t, actions, R):
    """Gradients of sum_b total_loss (network.py:86-94, A11 fixes) w.r.t. the flat parameters.
    Returns (grads [P] fp32, losses [4] = policy, value, entropy, total sums; a3c_hip.h order)."""
    planes = self._planes(s_t)
    B = int(planes.shape[0])
    a = torch.as_tensor(actions, dtype=torch.int32, device=self.device).reshape(B).contiguous()
    R = torch.as_tensor(R, dtype=torch.float32, device=self.device).reshape(B).contiguous()
    if self.net is not None or self.nat is not None:
      net, ws = self.net or self.nat, self._workspace(B)
      fwd = self.net.forward(self.flat, planes, save_l1=True, workspace=ws) if self.net is not None else \
          self.nat.forward(self.flat, planes, workspace=ws)
      self.last_forward = fwd       # (the activations the gradients were taken at: tests)
      return net.loss_backward(self.flat, planes, fwd, a, R, beta=self.beta, literal_adv=self.literal_adv,
                               workspace=ws)
    flat = self.flat.detach().requires_grad_(True)
    logits, V = self._nature_z(flat, planes)
    logp = torch.log_softmax(logits, dim=1)
    H = -(logp.exp() * logp).sum(1)
    adv = R - V
    lp_a = logp.gather(1, a.long()[:, None])[:, 0]
    pol = -(lp_a * (adv if self.literal_adv else adv.detach())) - self.beta * H
    val = 0.5 * adv * adv
    total = (pol + val).sum()
    total.backward()
    losses = torch.stack([(-(lp_a * adv) - self.beta * H).sum(), val.sum(), H.sum(), total]).detach()
    return flat.grad.detach(), losses

  def apply_gradients(self, grads, lr=None):
    """Clip per tensor + RMSProp apply of this worker's gradients onto the global network's
    parameters (the A3C shared-parameter update, main.py:63-65)."""
    target = self.global_network if self.global_network is not None else self
    opt = self.global_optim
    if opt is None:
      raise ValueError('apply_gradients needs global_optim')
    opt.apply_gradients(target.flat, grads, self.offsets, self.sizes, lr=lr)

  # ---------------------------------------------------------------------------------
  def copy_from_global(self):
    """theta' <- theta (network.py:96-107) on device (a3c_copy_params)."""
    if self.global_network is None:
      raise ValueError('copy_from_global needs global_network')
    K.copy_params(self.flat, self.global_network.flat)

  def save_model(self, saver, checkpoint_dir, step=None):
    print(" [*] Saving checkpoints...")
    os.makedirs(checkpoint_dir, exist_ok=True)
    name = type(self).__name__ + ('-%d' % step if step is not None else '')
    named = {C.tf_name(k, 'a3c', self.dqn_type): v for k, v in self.w.items()}     # network.py scopes
    return save_checkpoint(os.path.join(checkpoint_dir, name), named, step or 0)

  def load_model(self, saver, checkpoint_dir):
    files = sorted(glob.glob(os.path.join(checkpoint_dir, type(self).__name__ + '*.npz')), key=os.path.getmtime)
    if not files:
      print(" [!] Load FAILED: %s" % checkpoint_dir)
      return False
    arrays, step = load_checkpoint(files[-1])
    # TF variable names; round-1/2 files used the raw dict names
    copy_named(arrays, {name: (w, [C.tf_name(name, 'a3c', self.dqn_type), name]) for name, w in self.w.items()},
               files[-1])
    print(" [*] Load SUCCESS: %s" % files[-1])
    return True

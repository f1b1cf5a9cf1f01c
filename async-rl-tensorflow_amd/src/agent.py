"""Agent (agent.py:14-396): the reference's Q-learning actor-learner, one env per process.

Same constructor, attributes and loop as the reference.  The compute is on device:
* online / target Q nets (agent.py:209-296): the fused nips kernels (a3c_forward /
  a3c_loss_backward with algo 'q') over flat parameter buffers ``params`` / ``target_params``;
  the dueling variant (agent.py:234-249, off by default) runs on the generic HIP conv/matmul
  ops with autograd;
* TD target (agent.py:176-190): a3c_td_target (fp64 arithmetic, as numpy does);
* clip_by_norm(40) per tensor + RMSProp apply (agent.py:316-321, main.py:63-65):
  a3c_clip_rmsprop_apply; with several worker processes every worker's clipped gradient is
  applied as its own step, in rank order (src/distributed.py replaces the parameter server);
* history (agent.py:18, history.py): device u8 frame stack.
Exploration uses Python's ``random`` exactly like agent.py:141-151.  ``sv`` is any object with
``request_stop()`` and ``summary_computed(step, dict)`` (see ``Supervisor`` below).
"""
import json
import os
import random
import time

import numpy as np
import torch

from . import kernels as K
from . import ops
from . import checkpoint as C
from .base import BaseModel, copy_named, load_checkpoint, save_checkpoint
from .distributed import GradExchange, gather_grads
from .history import History
from .utils import get_time

try:
  from tqdm import tqdm
except ImportError:    # pragma: no cover
  tqdm = None


class Supervisor(object):
  """Stand-in for tf.train.Supervisor (main.py:77-83): stop flag, JSONL summaries, periodic
  checkpoint of the agent (save_model_secs)."""

  def __init__(self, is_chief=True, logdir=None, save_model_secs=600, agent=None):
    self.is_chief, self.logdir, self.save_model_secs, self.agent = is_chief, logdir, save_model_secs, agent
    self._stop = False
    self._last_save = time.time()
    if logdir and is_chief:
      os.makedirs(logdir, exist_ok=True)

  def request_stop(self):
    self._stop = True

  def should_stop(self):
    return self._stop

  def summary_computed(self, step, values):
    if self.logdir and self.is_chief:
      rec = {'step': int(step)}
      for k, v in values.items():
        rec[k] = [float(x) for x in v] if isinstance(v, (list, tuple, np.ndarray)) else float(v)
      with open(os.path.join(self.logdir, 'summary.jsonl'), 'a') as f:
        f.write(json.dumps(rec) + '\n')
    if self.agent is not None and self.is_chief and self.logdir and \
        time.time() - self._last_save >= self.save_model_secs:
      self.agent.save(os.path.join(self.logdir, 'model'))
      self._last_save = time.time()


class _DuelingQ(object):
  """agent.py:234-249 on the generic HIP ops (flat params, torch.autograd over the kernels)."""

  def __init__(self, A, fmt):
    self.A, self.fmt = A, fmt
    self.names_shapes = [('l1_w', (8, 8, 4, 16)), ('l1_b', (16,)), ('l2_w', (4, 4, 16, 32)), ('l2_b', (32,)),
                         ('l3_val_w', (2592, 256)), ('l3_val_b', (256,)), ('l3_adv_w', (2592, 256)),
                         ('l3_adv_b', (256,)), ('val_w_out', (256, 1)), ('val_w_b', (1,)),
                         ('adv_w_out', (256, A)), ('adv_w_b', (A,))]
    self.offsets, self.sizes, off = [], [], 0
    for _, s in self.names_shapes:
      n = int(np.prod(s))
      self.offsets.append(off)
      self.sizes.append(n)
      off = (off + n + 63) // 64 * 64
    self.total = off

  def q(self, flat, planes):
    w = {n: flat[o:o + k].view(s) for (n, s), o, k in zip(self.names_shapes, self.offsets, self.sizes)}
    x = planes.float() / 255.
    if self.fmt == 'NHWC':
      x = x.permute(0, 2, 3, 1).contiguous()
    l1, _, _ = ops.conv2d(x, 16, [8, 8], [4, 4], data_format=self.fmt, w=w['l1_w'], b=w['l1_b'])
    l2, _, _ = ops.conv2d(l1, 32, [4, 4], [2, 2], data_format=self.fmt, w=w['l2_w'], b=w['l2_b'])
    vh, _, _ = ops.linear(l2, 256, activation_fn=ops.relu, w=w['l3_val_w'], b=w['l3_val_b'])
    ah, _, _ = ops.linear(l2, 256, activation_fn=ops.relu, w=w['l3_adv_w'], b=w['l3_adv_b'])
    v, _, _ = ops.linear(vh, 1, w=w['val_w_out'], b=w['val_w_b'])
    adv, _, _ = ops.linear(ah, self.A, w=w['adv_w_out'], b=w['adv_w_b'])
    return v + (adv - adv.mean(1, keepdim=True))


class Agent(BaseModel):
  def __init__(self, config, environment, optimizer, lr_op=None, device='cuda', verbose=False):
    super(Agent, self).__init__(config, verbose=verbose)
    self.weight_dir = 'weights'
    self.device = device

    self.env = environment
    self.history = History(self.config, device=device)

    self.lr_op = lr_op
    self.optimizer = optimizer
    self.exchange = GradExchange()

    self.step_op = 0          # global step (tf.Variable 'step', agent.py:24)
    self.build_dqn()
    self.saver = None
    self.init_op = None

  # -- graph (agent.py:209-344) -----------------------------------------------------------
  def build_dqn(self):
    A = self.env.action_size
    self.A = A
    fmt = 'NHWC' if self.cnn_format == 'NHWC' else 'NCHW'
    if self.dueling:
      self.qnet = _DuelingQ(A, fmt)
      names_shapes, offsets, sizes, total = (self.qnet.names_shapes, self.qnet.offsets, self.qnet.sizes,
                                             self.qnet.total)
      self.net = None
    else:
      self.net = K.Net(A, 'q')
      names_shapes, offsets, sizes, total = self.net.names_shapes, self.net.offsets, self.net.sizes, self.net.total
    self.names_shapes, self.offsets, self.sizes = names_shapes, offsets, sizes
    init = ops.truncated_normal_initializer(0, 0.02, seed=getattr(self, 'random_seed', 123))   # agent.py:214
    lin = ops.random_normal_initializer(stddev=0.02, seed=getattr(self, 'random_seed', 123) + 1)
    self.params = torch.zeros(total, dtype=torch.float32, device=self.device)
    for (name, shp), o, n in zip(names_shapes, offsets, sizes):
      if len(shp) == 1:
        continue
      v = init(list(shp)) if len(shp) == 4 else lin(list(shp))
      self.params[o:o + n] = torch.as_tensor(v).reshape(-1).to(self.device)
    self.target_params = self.params.clone()
    self.w = {n: self.params[o:o + k].view(s) for (n, s), o, k in zip(names_shapes, offsets, sizes)}
    self.t_w = {n: self.target_params[o:o + k].view(s) for (n, s), o, k in zip(names_shapes, offsets, sizes)}
    self._ws = {}

  def _workspace(self, B):
    if B not in self._ws:
      self._ws[B] = self.net.workspace(B, self.device)
    return self._ws[B]

  def q_values(self, planes, target=False):
    """[B,A] Q (or target Q) for u8 planes [B,4,84,84]."""
    p = self.target_params if target else self.params
    if self.net is None:
      with torch.no_grad():
        return self.qnet.q(p, planes)
    return self.net.forward(p, planes, save_l1=False, workspace=self._workspace(int(planes.shape[0])))['z'][:, :self.A]

  def update_target_q_network(self):
    """agent.py:342-344 (t_w <- w) as one device copy."""
    K.copy_params(self.target_params, self.params)

  # -- acting (agent.py:141-167) ------------------------------------------------------------
  def predict(self, s_t, test_ep=None):
    ep = test_ep or (self.ep_end +
        max(0., (self.ep_start - self.ep_end)
          * (self.ep_end_t - max(0., self.step - self.learn_start)) / self.ep_end_t))

    if random.random() < ep:
      action = random.randrange(self.env.action_size)
    else:
      planes = s_t if isinstance(s_t, torch.Tensor) and s_t.dtype == torch.uint8 else self.history.planes()
      action = int(torch.argmax(self.q_values(planes.reshape(1, 4, 84, 84))[0]).item())
    return action

  def observe(self, screen, reward, action, terminal, is_chief=False):
    reward = max(self.min_reward, min(self.max_reward, reward))

    self.history.add(screen)
    self.batch_s_t.append(self.history.planes().clone())
    self.batch_action.append(action)
    self.batch_reward.append(reward)
    self.batch_terminal.append(terminal)

    if self.step % self.train_frequency == 0:
      self.batch_update(is_chief)

    prev = self.T
    self.T = self.step_op = self.step_op + self.exchange.world       # step_inc_op, all workers
    t = self.target_q_update_step
    if (self.T + 1) // t != (prev + 1) // t:                         # T % t == t - 1 crossed
      self.update_target_q_network()

  def batch_update(self, is_chief):
    """agent.py:169-207: TD target from the target net, MSE loss, clip + RMSProp apply."""
    states = torch.stack(self.batch_s_t)                             # [B+1,4,84,84] u8
    s_t, s_t_plus_1 = states[:-1].contiguous(), states[1:].contiguous()
    B = int(s_t.shape[0])
    action = torch.as_tensor(self.batch_action, dtype=torch.int32, device=self.device)
    reward = torch.as_tensor(self.batch_reward, dtype=torch.float32, device=self.device)
    terminal = torch.as_tensor([1 if t else 0 for t in self.batch_terminal], dtype=torch.uint8, device=self.device)

    q_next = self.q_values(s_t_plus_1, target=True).contiguous()
    if self.double_q:
      pred_action = torch.argmax(self.q_values(s_t_plus_1), dim=1)
      q_sel = q_next.gather(1, pred_action[:, None]).contiguous()     # gather_nd, agent.py:176-182
      target_q_t = K.td_target(reward, terminal, q_sel, 1, self.discount)
    else:
      target_q_t = K.td_target(reward, terminal, q_next, self.A, self.discount)

    if self.net is not None:
      ws = self._workspace(B)
      fwd = self.net.forward(self.params, s_t, save_l1=True, workspace=ws)
      grads, loss = self.net.loss_backward(self.params, s_t, fwd, action, target_q_t, workspace=ws)
      q_t = fwd['z'][:, :self.A]
      loss = loss[0]                     # q: {loss, mean q_acted, 0, 0}
    else:
      flat = self.params.detach().requires_grad_(True)
      q = self.qnet.q(flat, s_t)
      q_acted = q.gather(1, action.long()[:, None])[:, 0]
      loss = ((target_q_t - q_acted) ** 2).mean()
      loss.backward()
      grads, q_t = flat.grad.detach(), q.detach()
      loss = loss.detach()
    if self.exchange.world > 1:
      # the PS applies every worker's clipped push as an RMSProp step of its own (main.py:63-65,
      # agent.py:321): gather all workers' clipped gradients and apply them in rank order
      self.optimizer.clip_only(grads, self.offsets, self.sizes)
      for g in gather_grads(grads):
        self.optimizer.apply_gradients(self.params, g, self.offsets, self.sizes, lr=self.lr, clip=False)
    else:
      self.optimizer.apply_gradients(self.params, grads, self.offsets, self.sizes, lr=self.lr)

    if is_chief:
      self.total_loss += float(loss.item())
      self.total_q += float(q_t.mean().item())
      self.update_count += 1

    self.batch_s_t = [self.history.planes().clone()]
    self.batch_reward = []
    self.batch_action = []
    self.batch_terminal = []

  # -- loops (agent.py:33-139, 351-391) ------------------------------------------------------
  def before_train(self, is_chief):
    self.T = self.step = self.step_op
    screen, reward, action, terminal = self.env.new_random_game()

    for _ in range(self.history_length):
      self.history.add(screen)

    self.batch_s_t = [self.history.planes().clone()]
    self.batch_reward = []
    self.batch_action = []
    self.batch_terminal = []
    self.total_loss, self.total_q, self.update_count = 0., 0., 0

    rng = range(self.step, self.max_step)
    iterator = tqdm(rng, ncols=70, initial=self.step) if (is_chief and tqdm is not None) else rng
    return screen, reward, action, terminal, iterator

  def train(self, sv, is_chief):
    screen, reward, action, terminal, iterator = self.before_train(is_chief)

    for self.step in iterator:
      if self.step >= self.max_step or sv.should_stop():
        sv.request_stop()
        break
      action = self.predict(self.history.planes())
      screen, reward, terminal = self.env.act(action, is_training=True)
      self.observe(screen, reward, action, terminal)

      if terminal:
        screen, reward, action, terminal = self.env.new_random_game()

  def train_with_summary(self, sv, is_chief):
    screen, reward, action, terminal, iterator = self.before_train(is_chief)

    num_game, self.update_count, ep_reward = 0, 0, 0.
    total_reward, self.total_loss, self.total_q = 0., 0., 0.
    ep_rewards, actions = [], []

    for self.step in iterator:
      if self.step >= self.max_step or sv.should_stop():
        sv.request_stop()
        break

      if self.step == self.learn_start:
        num_game, self.update_count, ep_reward = 0, 0, 0.
        total_reward, self.total_loss, self.total_q = 0., 0., 0.
        ep_rewards, actions = [], []

      action = self.predict(self.history.planes())
      screen, reward, terminal = self.env.act(action, is_training=True)
      self.observe(screen, reward, action, terminal, is_chief=True)

      if terminal:
        screen, reward, action, terminal = self.env.new_random_game()
        num_game += 1
        ep_rewards.append(ep_reward)
        ep_reward = 0.
      else:
        ep_reward += reward

      actions.append(action)
      total_reward += reward

      if self.step % self.test_step == self.test_step - 1:
        avg_reward = total_reward / self.test_step
        avg_loss = self.total_loss / max(self.update_count, 1)
        avg_q = self.total_q / max(self.update_count, 1)
        if ep_rewards:
          max_ep_reward, min_ep_reward, avg_ep_reward = np.max(ep_rewards), np.min(ep_rewards), np.mean(ep_rewards)
        else:
          max_ep_reward, min_ep_reward, avg_ep_reward = 0, 0, 0

        print('\navg_r: %.4f, avg_l: %.6f, avg_q: %3.6f, avg_ep_r: %.4f, max_ep_r: %.4f, min_ep_r: %.4f, # game: %d'
              % (avg_reward, avg_loss, avg_q, avg_ep_reward, max_ep_reward, min_ep_reward, num_game))

        if self.step > 180:
          self.inject_summary(sv, {
              'average.reward': avg_reward,
              'average.loss': avg_loss,
              'average.q': avg_q,
              'episode.max reward': max_ep_reward,
              'episode.min reward': min_ep_reward,
              'episode.avg reward': avg_ep_reward,
              'episode.num of game': num_game,
              'episode.rewards': ep_rewards,
              'episode.actions': actions,
              'training.learning_rate': self.lr,
          }, self.T)

        num_game = 0
        total_reward = 0.
        self.total_loss = 0.
        self.total_q = 0.
        self.update_count = 0
        ep_rewards = []
        actions = []

  def inject_summary(self, sv, tag_dict, step):
    sv.summary_computed(step, tag_dict)

  def play(self, sv, is_chief, n_step=10000, n_episode=100, test_ep=None, render=False):
    if test_ep is None:
      test_ep = self.ep_end

    test_history = History(self.config, device=self.device)
    best_reward, best_idx = 0, 0
    self.step = self.step_op
    for idx in range(n_episode):
      screen, reward, action, terminal = self.env.new_random_game()
      current_reward = 0

      for _ in range(self.history_length):
        test_history.add(screen)

      for t in range(n_step):
        action = self.predict(test_history.planes(), test_ep)
        screen, reward, terminal = self.env.act(action, is_training=False)
        test_history.add(screen)

        current_reward += reward
        if terminal:
          break

      if current_reward > best_reward:
        best_reward = current_reward
        best_idx = idx

      print("=" * 30)
      print(" [%d] Best reward : %d" % (best_idx, best_reward))
      print("=" * 30)
    return best_reward

  @property
  def lr(self):
    return (self.max_step - self.step + 1.) / self.max_step * self.learning_rate

  # -- checkpoints (Saver, agent.py:29) ------------------------------------------------------
  def save(self, path):
    """Saver of agent.py:29 (prediction weights + step) keyed by the TF variable names, plus the
    target network (agent.py:257-296 names)."""
    named = {C.tf_name(k, 'q'): v for k, v in self.w.items()}
    named.update({C.tf_target_name(k): v for k, v in self.t_w.items()})
    return save_checkpoint(path, named, self.step_op)

  def load(self, path):
    arrays, step = load_checkpoint(path)
    # TF variable names; round-1/2 files used the raw dict names and 'target/<k>'
    dst = {'w/' + k: (v, [C.tf_name(k, 'q'), k]) for k, v in self.w.items()}
    dst.update({'t_w/' + k: (v, [C.tf_target_name(k), 'target/' + k]) for k, v in self.t_w.items()})
    copy_named(arrays, dst, path)
    self.step_op = step
    return step

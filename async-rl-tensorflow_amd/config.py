"""Hyper-parameters, same classes, names and defaults as the reference's config.py:1-66.

Additions for the batched MI355X engine are grouped in ``EngineConfig`` (n_step, num_envs,
algo, dqn_type, num_frames, literal_adv, clip_norm) and mixed into M1.
"""


class AgentConfig(object):
  scale = 10000
  display = False

  max_step = 8000 * scale

  random_start = 30
  cnn_format = 'NCHW'
  discount = 0.99
  target_q_update_step = 4 * scale
  learning_rate = 0.0007

  decay = 0.99
  epsilon = 0.1
  momentum = 0.0
  beta = 0.01

  ep_end = 0.1
  ep_start = 1.
  ep_end_t = 400 * scale

  history_length = 4
  batch_size = 32
  train_frequency = batch_size
  learn_start = batch_size

  min_delta = -1
  max_delta = 1

  double_q = False
  dueling = False

  _test_step = 0.5 * scale


class EnvironmentConfig(object):
  env_name = 'Breakout-v0'

  screen_width = 84
  screen_height = 84
  max_reward = 1.
  min_reward = -1.


class EngineConfig(object):
  """MI355X engine knobs (no reference counterpart)."""
  algo = 'a3c'            # 'a3c' (network.py + assets/a3c.png) or 'q' (agent.py)
  dqn_type = 'nips'       # network.py:26,39
  n_step = 5              # A3C rollout length (BASELINE.json config 2)
  num_envs = 256          # envs per GPU
  num_frames = 16384      # synthetic HBM frame pool
  clip_norm = 40.0        # agent.py:319
  literal_adv = False     # network.py's un-stopped advantage gradient


class DQNConfig(AgentConfig, EnvironmentConfig, EngineConfig):
  model = ''
  pass


class M1(DQNConfig):
  backend = 'tf'
  env_type = 'detail'
  action_repeat = 1


def _flags_dict(FLAGS):
  try:
    return dict(FLAGS.__dict__['__flags'])        # tf.app.flags (config.py:56)
  except (KeyError, AttributeError, TypeError):
    return dict(vars(FLAGS))                      # argparse.Namespace / plain object


def get_config(FLAGS):
  """config.py:52-66.  (The reference raises UnboundLocalError for any model but 'm1'; here
  that is a ValueError.)"""
  if FLAGS.model == 'm1':
    config = M1
  else:
    raise ValueError('unknown model: %s' % FLAGS.model)

  for k, v in _flags_dict(FLAGS).items():
    if k == 'gpu':
      if v == False:
        config.cnn_format = 'NHWC'
      else:
        config.cnn_format = 'NCHW'

    if hasattr(config, k) and v is not None:     # unset optional flags keep the config default
      setattr(config, k, v)

  return config

"""Hyper-parameters: the reference's config classes (config.py:1-50) with the same names,
attribute names and defaults, plus ``get_config`` (config.py:52-66).

The values live in per-class tables below, each entry citing the reference line it mirrors;
the classes are built from them so that ``M1.learning_rate`` etc. read exactly as in the
reference.  ``EngineConfig`` holds the knobs of the batched MI355X engine (no reference
counterpart) and is mixed into ``DQNConfig``.
"""

_SCALE = 10000                                   # config.py:2

_AGENT = {                                       # config.py:1-33
    'scale': _SCALE,
    'display': False,
    'max_step': 8000 * _SCALE,                   # :5
    'random_start': 30,                          # :7
    'cnn_format': 'NCHW',                        # :8 (main.py:45 forces NHWC)
    'discount': 0.99,                            # :9
    'target_q_update_step': 4 * _SCALE,          # :10
    'learning_rate': 0.0007,                     # :11
    'decay': 0.99,                               # :13 (main.py:64-65 hard-codes the optimizer)
    'epsilon': 0.1,                              # :14
    'momentum': 0.0,                             # :15
    'beta': 0.01,                                # :16 entropy weight
    'ep_end': 0.1,                               # :18
    'ep_start': 1.,                              # :19
    'ep_end_t': 400 * _SCALE,                    # :20
    'history_length': 4,                         # :22
    'batch_size': 32,                            # :23
    'train_frequency': 32,                       # :24 (= batch_size)
    'learn_start': 32,                           # :25 (= batch_size)
    'min_delta': -1,                             # :27
    'max_delta': 1,                              # :28
    'double_q': False,                           # :30
    'dueling': False,                            # :31
    '_test_step': 0.5 * _SCALE,                  # :33
}

_ENVIRONMENT = {                                 # config.py:35-41
    'env_name': 'Breakout-v0',
    'screen_width': 84,
    'screen_height': 84,
    'max_reward': 1.,
    'min_reward': -1.,
}

_ENGINE = {                                      # MI355X engine knobs (no reference counterpart)
    'algo': 'a3c',            # 'a3c' (network.py + assets/a3c.png) or 'q' (agent.py)
    'dqn_type': 'nips',       # network.py:26,39
    'n_step': 5,              # A3C rollout length (BASELINE.json config 2)
    'num_envs': 256,          # envs per GPU
    'num_frames': 16384,      # synthetic HBM frame pool
    'clip_norm': 40.0,        # agent.py:319
    'literal_adv': False,     # network.py's un-stopped advantage gradient
}

AgentConfig = type('AgentConfig', (object,), dict(_AGENT))
EnvironmentConfig = type('EnvironmentConfig', (object,), dict(_ENVIRONMENT))
EngineConfig = type('EngineConfig', (object,), dict(_ENGINE, __doc__='MI355X engine knobs.'))
DQNConfig = type('DQNConfig', (AgentConfig, EnvironmentConfig, EngineConfig), {'model': ''})   # :43-45
M1 = type('M1', (DQNConfig,), {'backend': 'tf', 'env_type': 'detail', 'action_repeat': 1})    # :47-50

_MODELS = {'m1': M1}


def _flag_items(FLAGS):
  """(name, value) pairs of tf.app.flags (config.py:56) or of an argparse namespace."""
  stored = getattr(FLAGS, '__dict__', {})
  if isinstance(stored, dict) and isinstance(stored.get('__flags'), dict):
    return list(stored['__flags'].items())
  return list(vars(FLAGS).items())


def get_config(FLAGS):
  """config.py:52-66: the model's config class with every matching flag written onto it.
  ``gpu`` picks the conv layout.  (An unknown model is an UnboundLocalError in the
  reference; here a ValueError.)"""
  base = _MODELS.get(FLAGS.model)
  if base is None:
    raise ValueError('unknown model: %s' % FLAGS.model)
  # the flags go onto a per-call subclass: the reference writes them onto the model class itself,
  # which in one process (several main() calls, the tests) would carry one run's flags into the next
  config = type(base.__name__, (base,), {})
  for name, value in _flag_items(FLAGS):
    if name == 'gpu':
      config.cnn_format = 'NCHW' if value else 'NHWC'
    if value is not None and hasattr(config, name):   # unset optional flags keep the default
      setattr(config, name, value)
  return config

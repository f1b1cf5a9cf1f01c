"""BaseModel (base.py:13-41): copies the config's attributes onto the model (``_x`` -> ``x``),
``model_dir`` / ``checkpoint_dir`` strings.  Checkpoints (the Saver of agent.py:29 /
main.py:74-80) are written as ``.npz`` keyed by the TF variable names plus the step."""
import inspect
import os
import pprint

import numpy as np

pp = pprint.PrettyPrinter().pprint


def class_vars(obj):
  return {k: v for k, v in inspect.getmembers(obj)
          if not k.startswith('__') and not callable(k)}


class BaseModel(object):
  """Abstract object representing an Reader model."""
  def __init__(self, config, verbose=True):
    self.config = config

    try:
      self._attrs = config.__dict__['__flags']
    except (KeyError, AttributeError, TypeError):
      self._attrs = class_vars(config)
    if verbose:
      pp(self._attrs)

    self.config = config

    for attr in self._attrs:
      name = attr if not attr.startswith('_') else attr[1:]
      setattr(self, name, getattr(self.config, attr))

  @property
  def checkpoint_dir(self):
    return os.path.join('checkpoints', self.model_dir)

  @property
  def model_dir(self):
    model_dir = self.config.env_name
    for k, v in self._attrs.items():
      if not k.startswith('_') and k not in ['display']:
        model_dir += "/%s-%s" % (k, ",".join([str(i) for i in v])
            if type(v) == list else v)
    return model_dir + '/'


def save_checkpoint(path, named_tensors, step):
  """{tf variable name: tensor} + global step -> path.npz (max_to_keep handled by callers)."""
  d = os.path.dirname(path)
  if d:
    os.makedirs(d, exist_ok=True)
  arrays = {k: (v.detach().cpu().numpy() if hasattr(v, 'detach') else np.asarray(v)) for k, v in named_tensors.items()}
  np.savez(path, __step__=np.array(int(step), np.int64), **arrays)
  return path if path.endswith('.npz') else path + '.npz'


def load_checkpoint(path):
  with np.load(path, allow_pickle=False) as f:
    step = int(f['__step__'])
    return {k: f[k] for k in f.files if k != '__step__'}, step

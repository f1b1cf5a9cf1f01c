"""BaseModel (reference src/base.py:13-41) and the checkpoint format.

The model copies every public attribute of its config onto itself (a leading underscore is
dropped: ``_test_step`` -> ``test_step``), and derives ``model_dir`` from the config values
(everything but ``display``), which the reference uses as the run / checkpoint directory.
Checkpoints (the Saver of agent.py:29 / main.py:74-80) are ``.npz`` files keyed by the TF
variable names (src/checkpoint.py) plus the global step ``step``.
"""
import inspect
import os
import pprint

import numpy as np

pp = pprint.PrettyPrinter().pprint


def class_vars(obj):
  """Public (non-dunder) members of a config class or object, as a dict."""
  out = {}
  for name, value in inspect.getmembers(obj):
    if name.startswith('__') or callable(name):
      continue
    out[name] = value
  return out


def _config_attrs(config):
  # tf.app.flags objects keep their values in __dict__['__flags']; plain classes do not
  flags = getattr(config, '__dict__', {})
  if isinstance(flags, dict) and '__flags' in flags:
    return flags['__flags']
  return class_vars(config)


def _fmt(value):
  return ','.join(str(v) for v in value) if isinstance(value, list) else value


class BaseModel(object):
  """Abstract object representing an Reader model."""

  def __init__(self, config, verbose=True):
    self.config = config
    self._attrs = _config_attrs(config)
    if verbose:
      pp(self._attrs)
    for key in self._attrs:
      setattr(self, key[1:] if key.startswith('_') else key, getattr(config, key))

  @property
  def checkpoint_dir(self):
    return os.path.join('checkpoints', self.model_dir)

  @property
  def model_dir(self):
    parts = [self.config.env_name]
    parts += ['%s-%s' % (k, _fmt(v)) for k, v in self._attrs.items()
              if not k.startswith('_') and k != 'display']
    return '/'.join(parts) + '/'


def save_checkpoint(path, named_tensors, step):
  """{tf variable name: tensor} + the global step (TF variable ``step``, agent.py:25) -> path.npz
  (max_to_keep handled by callers; src/checkpoint.py has the names and the Saver)."""
  d = os.path.dirname(path)
  if d:
    os.makedirs(d, exist_ok=True)
  arrays = {k: (v.detach().cpu().numpy() if hasattr(v, 'detach') else np.asarray(v)) for k, v in named_tensors.items()}
  np.savez(path, step=np.array(int(step), np.int64), **arrays)
  return path if path.endswith('.npz') else path + '.npz'


def copy_named(arrays, targets, what):
  """Copy checkpoint arrays into tensors.  targets: {destination tensor name: (tensor, [keys, ...])},
  the keys tried in order (the TF variable name first, then the raw-dict / ``target/<k>`` names of
  round-1/2 files).  Raises ValueError when no tensor matched (the file is not a checkpoint of
  this model) and names the missing ones when only some matched.  Returns the number copied."""
  import torch
  found, missing = 0, []
  for name, (dst, keys) in targets.items():
    key = next((k for k in keys if k in arrays), None)
    if key is None:
      missing.append(name)
      continue
    dst.copy_(torch.as_tensor(arrays[key]).reshape(dst.shape))
    found += 1
  if not found:
    raise ValueError('%s: the checkpoint holds none of the expected tensors (%s ...)' % (what, ', '.join(
        k for _, ks in list(targets.values())[:2] for k in ks[:1])))
  if missing:
    print(' [!] %s: checkpoint lacks %s (kept as initialised)' % (what, ', '.join(missing)))
  return found


def load_checkpoint(path):
  with np.load(path, allow_pickle=False) as f:
    key = 'step' if 'step' in f.files else '__step__'     # (files of rounds 1-2)
    step = int(f[key])
    return {k: f[k] for k in f.files if k != key}, step

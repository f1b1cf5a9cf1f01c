"""History (history.py:3-27) on device: the frame stack is a u8 [L, 84, 84] device tensor pushed
by the K2 kernel (a3c_history_push); ``get`` / ``copy`` return float32 device tensors in the
reference's NHWC [84,84,L] (or NCHW [L,84,84]) order via a3c_history_get_f32."""
import numpy as np
import torch

from . import kernels as K


class History:
  def __init__(self, config, device='cuda'):
    self.cnn_format = config.cnn_format

    batch_size, history_length, screen_height, screen_width = \
        config.batch_size, config.history_length, config.screen_height, config.screen_width

    self.history = torch.zeros((1, history_length, screen_height, screen_width), dtype=torch.uint8, device=device)
    self._zero_mask = torch.ones(1, dtype=torch.uint8, device=device)

  @staticmethod
  def _u8(screen, device):
    if isinstance(screen, torch.Tensor):
      return screen.to(device=device, dtype=torch.uint8).reshape(1, *screen.shape[-2:]).contiguous()
    return torch.as_tensor(np.asarray(screen, dtype=np.uint8)).to(device).reshape(1, *np.shape(screen)[-2:])

  def add(self, screen):                      # history.py:13-15
    K.history_push(self.history, self._u8(screen, self.history.device))

  def reset(self):                            # history.py:17-18
    self.history.zero_()

  def get(self):                              # history.py:20-24
    return K.history_get(self.history, nhwc=self.cnn_format == 'NHWC')[0]

  def copy(self):                             # history.py:26-27
    return self.get().clone()

  def planes(self):
    """u8 [L,84,84] view (the layout the fused kernels take)."""
    return self.history[0]

"""Host-side pieces of the drop-in layer that need no GPU: flags/config (main.py:8-40,
config.py:52-66), BaseModel attribute copy + model_dir (base.py:13-41), checkpoint round trip,
TF-style initialisers, and the ValueError contract of Network (network.py:21,54)."""
import numpy as np
import pytest


def test_flags_and_config():
    import main
    import config as C
    f = main.parse_flags(['--env_name', 'Pong-v0', '--double_q', 'true', '--mode', 'agent', '--beta', '0.02'])
    assert f.env_name == 'Pong-v0' and f.double_q is True and f.mode == 'agent'
    cfg = C.get_config(f)
    assert cfg is C.M1 and cfg.env_name == 'Pong-v0' and cfg.double_q is True and cfg.beta == 0.02
    assert cfg.learning_rate == 0.0007 and cfg.target_q_update_step == 40000   # config.py defaults
    with pytest.raises(ValueError):
        C.get_config(main.parse_flags(['--model', 'm9']))


def test_base_model_attrs_and_model_dir():
    from src.base import BaseModel
    import config as C

    class Cfg(C.M1):
        env_name = 'Breakout-v0'
    m = BaseModel(Cfg, verbose=False)
    assert m.test_step == Cfg._test_step and m.discount == 0.99
    assert m.model_dir.startswith('Breakout-v0/') and m.model_dir.endswith('/')
    assert m.checkpoint_dir.startswith('checkpoints')


def test_checkpoint_roundtrip(tmp_path):
    import torch
    from src.base import load_checkpoint, save_checkpoint
    named = {'l1_w': torch.arange(12, dtype=torch.float32).reshape(2, 2, 3), 'q_b': np.ones(3, np.float32)}
    path = save_checkpoint(str(tmp_path / 'a' / 'm'), named, 42)
    arrays, step = load_checkpoint(path)
    assert step == 42 and np.array_equal(arrays['l1_w'], named['l1_w'].numpy())


def test_initializers():
    from src import ops
    w = ops.truncated_normal_initializer(0, 0.02, seed=1)([8, 8, 4, 16])
    assert w.dtype == np.float32 and np.abs(w).max() <= 0.04 + 1e-7 and abs(w.std() - 0.0176) < 2e-3
    x = ops.xavier_initializer(seed=2)([3, 3, 64, 64])
    lim = np.sqrt(6.0 / (2 * 9 * 64))
    assert np.abs(x).max() <= lim
    assert np.all(ops.constant_initializer(0.5)([3]) == 0.5)


def test_network_value_errors_before_device():
    from src.network import Network
    with pytest.raises(ValueError, match='unknown data_format'):
        Network(None, 'NCWH', 4, 84, 84, 6, DQN_type='nips')
    with pytest.raises(ValueError, match='Wrong DQN type'):
        Network(None, 'NHWC', 4, 84, 84, 6, DQN_type='')

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
    assert issubclass(cfg, C.M1) and cfg.env_name == 'Pong-v0' and cfg.double_q is True and cfg.beta == 0.02
    assert cfg.learning_rate == 0.0007 and cfg.target_q_update_step == 40000   # config.py defaults
    with pytest.raises(ValueError):
        C.get_config(main.parse_flags(['--model', 'm9']))
    # one call's flags do not leak into the next (main() runs several times in one test process)
    C.get_config(main.parse_flags(['--max_step', '14', '--n_step', '7']))
    fresh = C.get_config(main.parse_flags([]))
    assert fresh.max_step == C.M1.max_step != 14 and fresh.n_step == C.M1.n_step


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
    assert int(np.load(path)['step']) == 42           # the global step under its TF name


def test_checkpoint_tf_names_and_saver(tmp_path):
    """Keys follow the TF variable names of the reference graphs (agent.py:218-296 + ops.py,
    network.py:43-79) and TF1's RMSProp slot names; the Saver keeps max_to_keep checkpoints
    (agent.py:29) with an index, dropping the oldest and its rank files."""
    from src import checkpoint as C
    from src.kernels import param_names_shapes
    q = [C.tf_name(n, 'q') for n, _ in param_names_shapes(6, 'q')]
    assert q == ['prediction/l1/w', 'prediction/l1/biases', 'prediction/l2/w', 'prediction/l2/biases',
                 'prediction/l3/Matrix', 'prediction/l3/bias', 'prediction/q/Matrix', 'prediction/q/bias']
    assert [C.tf_target_name(n) for n in ('l1_w', 'l3_b', 'q_w')] == \
        ['target/target_l1/w', 'target/target_l3/bias', 'target/target_q/Matrix']
    a = [C.tf_name(n, 'a3c') for n, _ in param_names_shapes(6, 'a3c', lstm=True)]
    assert a == ['l1_conv/w', 'l1_conv/biases', 'l2_conv/w', 'l2_conv/biases', 'l4_linear/Matrix', 'l4_linear/bias',
                 'policy/linear/Matrix', 'policy/linear/bias', 'value/linear/Matrix', 'value/linear/bias',
                 'lstm/basic_lstm_cell/weights', 'lstm/basic_lstm_cell/biases']
    assert C.tf_name('l3_w', 'a3c', 'nature') == 'Nature_DQN/l3_conv/w'
    assert C.tf_name('p_b', 'a3c', 'nature') == 'policy/linear/bias'
    assert C.slot_names('l1_conv/w') == ('l1_conv/w/RMSProp', 'l1_conv/w/RMSProp_1')
    saver = C.Saver(str(tmp_path), max_to_keep=3)
    assert saver.latest() is None
    for step in (10, 20, 30, 40):
        saver.write({'world': np.array(2)}, step, rank=1)
        saver.save({'step': np.array(step), 'l1_conv/w': np.full(3, step, np.float32)}, step)
    assert saver.latest().endswith('model.ckpt-40.npz')
    assert [p.split('-')[-1] for p in saver.kept()] == ['20.npz', '30.npz', '40.npz']
    assert not (tmp_path / 'model.ckpt-10.npz').exists() and not (tmp_path / 'model.ckpt-10.rank1.npz').exists()
    assert (tmp_path / 'model.ckpt-20.rank1.npz').exists()
    got = C.load(saver.latest())
    assert int(got['step']) == 40 and got['l1_conv/w'][0] == 40


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


@pytest.mark.parametrize('argv,want', [
    ([], dict(lstm=False)),
    (['--lstm', 'true'], dict(lstm=True)),
    (['--algo', 'q', '--double_q', 'true'], dict(lstm=False, double_q=True)),
    (['--algo', 'q'], dict(lstm=False)),
    (['--dqn_type', 'nature'], dict(lstm=False, dqn_type='nature')),
])
def test_engine_mode_honours_reference_options(argv, want):
    """main.py --mode engine passes every reference option it supports into the Engine config:
    --lstm (config 5), --double_q (agent.py:176-184, implemented in the engine's TD target), --dqn_type
    nature (network.py:30-42, nature.hip)."""
    import main
    assert main.engine_options(main.parse_flags(['--mode', 'engine'] + argv)) == want


@pytest.mark.parametrize('argv,match', [
    (['--dueling', 'true'], 'dueling'),
    (['--algo', 'q', '--dueling', 'true'], 'dueling'),
    (['--dqn_type', 'nature', '--algo', 'q'], 'nature'),
    (['--dqn_type', 'nature', '--lstm', 'true'], 'nature'),
    (['--double_q', 'true'], 'Q-learning option'),
    (['--algo', 'q', '--lstm', 'true'], 'A3C policy head'),
])
def test_engine_mode_rejects_unsupported_options(argv, match):
    """... and rejects the ones the fused engine does not implement, before any device work, so a
    user asking for them never silently gets the vanilla network (agent.py:234-249 dueling,
    network.py:30-42 nature trunk)."""
    import main
    with pytest.raises(ValueError, match=match):
        main.main(['--mode', 'engine'] + argv)


def test_double_q_target_oracle():
    """oracle td_target_double (agent.py:176-184): the target net's value at the ONLINE net's
    argmax (first maximum on ties), which differs from max_a Q' when the nets disagree."""
    from oracle import ref_cpu as R
    qt = np.array([[1.0, 5.0, 2.0], [3.0, 3.0, 0.0], [0.0, 1.0, 9.0]], np.float32)
    qo = np.array([[9.0, 0.0, 0.0], [2.0, 2.0, 1.0], [0.0, 0.0, 7.0]], np.float32)
    r = np.array([1.0, 0.0, -1.0], np.float32)
    term = np.array([0, 0, 1], np.uint8)
    got = R.td_target_double(r, term, qt, qo, 0.5)
    np.testing.assert_array_equal(got, [1.0 + 0.5 * 1.0, 0.5 * 3.0, -1.0])
    assert not np.array_equal(got, R.td_target(r, term, qt, 0.5))

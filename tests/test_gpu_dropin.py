"""GPU parity of the Python drop-in layer (src/environment.py, src/ops.py, src/network.py,
src/agent.py, src/optim.py) against the oracle and torch fp64 references.

Bars: env state / rewards / terminals / screens bit-exact vs oracle/synthetic_env.py +
ref_cpu.screen; fp32 kernels vs fp64 references at rtol 1e-4 (forward), losses 1e-4 relative,
gradients 2e-2 relative-L2 per tensor (independent forward, ReLU-mask flips allowed)."""
import types

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
F = torch.nn.functional

from oracle import ref_cpu as R  # noqa: E402
from oracle.synthetic_env import GAMES as OGAMES, SyntheticAtari, pool_frame  # noqa: E402


def rel_l2(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def make_config(env_name='Breakout-v0', **kw):
    sys_cfg = __import__('config')
    cfg = type('Cfg', (sys_cfg.M1,), {})
    cfg.env_name = env_name
    cfg.cnn_format = 'NHWC'
    for k, v in kw.items():
        setattr(cfg, k, v)
    return cfg


# ------------------------------------------------------------------ environment.py
@pytest.mark.parametrize('game,repeat,training', [('Breakout-v0', 1, True), ('SpaceInvaders-v0', 3, True),
                                                  ('Breakout-v0', 2, False)])
def test_batched_env_matches_oracle(game, repeat, training):
    from src.environment import BatchedEnvironment
    E, nf, seed = 37, 64, 77
    cfg = make_config(game, action_repeat=repeat, random_start=30)
    env = BatchedEnvironment(cfg, num_envs=E, env_id_base=5, seed=seed, num_frames=nf)
    ref = SyntheticAtari(seed, E, nf, OGAMES[game]['action_size'], OGAMES[game]['start_lives'], 30, repeat, 5)
    for f in (0, 17, nf - 1):
        assert np.array_equal(env.frame_pool[f].cpu().numpy(), pool_frame(seed, f))
    env.new_random_game()
    ref.new_random_game()
    rng = np.random.default_rng(3)
    A = env.action_size
    for t in range(260):
        a = rng.integers(0, A, E).astype(np.int32)
        scr, rew, term = env.act(torch.as_tensor(a), is_training=training)
        fr, rr, tt = ref.act(a, is_training=training)
        torch.cuda.synchronize()
        assert np.array_equal(env._frame.cpu().numpy(), fr.astype(np.int32)), t
        assert np.array_equal(rew.cpu().numpy(), rr), t
        assert np.array_equal(term.cpu().numpy().astype(bool), tt), t
        assert np.array_equal(env.lives_all.cpu().numpy(), ref.lives), t
        if t % 64 == 0:
            want = np.stack([R.screen(pool_frame(seed, int(f))) for f in fr])
            assert np.array_equal(scr.cpu().numpy(), want), t
        if tt.any():
            m = torch.as_tensor(tt.astype(np.uint8)).cuda()
            env.new_random_game(m)
            ref.new_random_game(tt.copy())


def test_batched_env_matches_reference_act_rule(golden_dir):
    """The device env (a3c_env_*: the same act / new_random_game code the engine's head kernels
    inline) against the reference's own GymEnvironment driving the synthetic emulator's primitives
    (tests/golden/synth_env_golden.npz, environment.py:28-96 + agent.py:66-67): frame id, reward,
    terminal and lives after every call."""
    from src.environment import BatchedEnvironment
    g = np.load(f'{golden_dir}/synth_env_golden.npz')
    for i, (game, c) in enumerate(zip(g['games'], g['cases'])):
        seed, env_id, P, rep, rs, training, _ = (int(x) for x in c)
        cfg = make_config(str(game), action_repeat=rep, random_start=rs)
        env = BatchedEnvironment(cfg, num_envs=1, env_id_base=env_id, seed=seed, num_frames=P)
        tr = g[f'trace{i}']
        env.new_random_game()
        k = 0

        def check(row, r=None, t=None):
            torch.cuda.synchronize()
            assert int(env._frame.cpu()[0]) == int(row[1]), (i, k, row)
            assert int(env.lives_all.cpu()[0]) == int(row[4]), (i, k, row)
            if r is not None:
                assert float(r.cpu()[0]) == row[2] and int(t.cpu()[0]) == int(row[3]), (i, k, row)
        check(tr[0])
        k = 1
        for a in g[f'actions{i}']:
            _, r, t = env.act(torch.tensor([a], dtype=torch.int32), is_training=bool(training))
            assert tr[k, 0] == 1
            check(tr[k], r, t)
            k += 1
            if int(t.cpu()[0]):
                env.new_random_game(torch.ones(1, dtype=torch.uint8, device='cuda'))
                check(tr[k])
                k += 1
        assert k == len(tr)


def test_simple_env_and_single_env_wrappers():
    from src.environment import BatchedEnvironment, GymEnvironment, SimpleGymEnvironment, game_spec
    with pytest.raises(ValueError):
        game_spec('NoSuchGame-v0')
    cfg = make_config('Breakout-v0', random_seed=123)
    E, nf = 9, 32
    env = BatchedEnvironment(cfg, num_envs=E, seed=5, num_frames=nf)
    ref = SyntheticAtari(5, E, nf, 4, 5, 30, 1, 0)
    env.new_game()
    ref.new_game()
    for t in range(50):
        a = (np.arange(E) + t) % 4
        env.act(torch.as_tensor(a, dtype=torch.int32), simple=True)
        fr, rr, tt = ref.simple_act(a)
        assert np.array_equal(env._frame.cpu().numpy(), fr.astype(np.int32))
        assert np.array_equal(env.rewards.cpu().numpy(), rr)
    g = GymEnvironment(cfg)
    screen, r, a0, term = g.new_random_game()
    assert tuple(screen.shape) == (84, 84) and screen.dtype == torch.uint8
    assert g.action_size == 4 and g.lives == 5
    s2, r2, t2 = g.act(1)
    assert isinstance(r2, float) and isinstance(t2, bool)
    sg = SimpleGymEnvironment(cfg)
    sg.new_game()
    sg.act(0)


# ------------------------------------------------------------------ ops.py
@pytest.mark.parametrize('fmt', ['NHWC', 'NCHW'])
@pytest.mark.parametrize('shape', [(3, 84, 84, 4, 32, 8, 4), (2, 20, 20, 32, 64, 4, 2), (4, 9, 9, 64, 64, 3, 1),
                                   (2, 13, 11, 5, 7, 3, 2)])
def test_conv2d_matches_torch(fmt, shape):
    from src import ops
    N, H, W, C, OC, k, s = shape
    rng = np.random.default_rng(1)
    x = rng.standard_normal((N, H, W, C)).astype(np.float32)
    w = (rng.standard_normal((k, k, C, OC)) * 0.1).astype(np.float32)
    b = (rng.standard_normal(OC) * 0.1).astype(np.float32)
    xin = x if fmt == 'NHWC' else x.transpose(0, 3, 1, 2).copy()
    xd = torch.as_tensor(xin).cuda().requires_grad_(True)
    wd = torch.nn.Parameter(torch.as_tensor(w).cuda())
    bd = torch.nn.Parameter(torch.as_tensor(b).cuda())
    y, _, _ = ops.conv2d(xd, OC, [k, k], [s, s], data_format=fmt, w=wd, b=bd)
    gy = torch.as_tensor(rng.standard_normal(tuple(y.shape)).astype(np.float32)).cuda()
    (y * gy).sum().backward()
    # fp64 torch CPU reference
    xr = torch.as_tensor(x, dtype=torch.float64).permute(0, 3, 1, 2).requires_grad_(True)
    wr = torch.as_tensor(w, dtype=torch.float64).requires_grad_(True)
    br = torch.as_tensor(b, dtype=torch.float64).requires_grad_(True)
    yr = F.relu(F.conv2d(xr, wr.permute(3, 2, 0, 1), br, stride=s))
    if fmt == 'NHWC':
        yr = yr.permute(0, 2, 3, 1)
    (yr * gy.cpu().double()).sum().backward()
    np.testing.assert_allclose(y.detach().cpu().numpy(), yr.detach().numpy(), rtol=1e-4, atol=1e-5)
    dx_ref = xr.grad.numpy() if fmt == 'NCHW' else xr.grad.permute(0, 2, 3, 1).numpy()
    assert rel_l2(xd.grad.cpu().numpy(), dx_ref) < 1e-5
    assert rel_l2(wd.grad.cpu().numpy(), wr.grad.numpy()) < 1e-5
    assert rel_l2(bd.grad.cpu().numpy(), br.grad.numpy()) < 1e-5


def test_linear_matches_torch():
    from src import ops
    rng = np.random.default_rng(2)
    x = rng.standard_normal((7, 3, 5, 9)).astype(np.float32)
    xd = torch.as_tensor(x).cuda().requires_grad_(True)
    y, w, b = ops.linear(xd, 33, stddev=0.1, bias_start=0.25, activation_fn=ops.relu)
    assert tuple(w.shape) == (135, 33) and np.allclose(b.detach().cpu().numpy(), 0.25)
    gy = torch.as_tensor(rng.standard_normal((7, 33)).astype(np.float32)).cuda()
    (y * gy).sum().backward()
    xr = torch.as_tensor(x, dtype=torch.float64).reshape(7, -1).requires_grad_(True)
    wr = w.detach().cpu().double().requires_grad_(True)
    br = b.detach().cpu().double().requires_grad_(True)
    yr = F.relu(xr @ wr + br)
    (yr * gy.cpu().double()).sum().backward()
    np.testing.assert_allclose(y.detach().cpu().numpy(), yr.detach().numpy(), rtol=1e-4, atol=1e-5)
    assert rel_l2(xd.grad.cpu().numpy().reshape(7, -1), xr.grad.numpy()) < 1e-5
    assert rel_l2(w.grad.cpu().numpy(), wr.grad.numpy()) < 1e-5
    assert rel_l2(b.grad.cpu().numpy(), br.grad.numpy()) < 1e-5
    with pytest.raises(ValueError):
        ops.conv2d(xd, 4, [2, 2], [1, 1], data_format='NCWH')


# ------------------------------------------------------------------ network.py
def _net_params(net):
    return {k: v.detach().cpu().numpy().copy() for k, v in net.w.items()}


@pytest.mark.parametrize('dqn_type', ['nips', 'nature'])
def test_network_forward_loss_grads_match_oracle(dqn_type):
    from src.network import Network
    with pytest.raises(ValueError):
        Network(None, 'NCWH', 4, 84, 84, 6, DQN_type='nips')
    with pytest.raises(ValueError):
        Network(None, 'NHWC', 4, 84, 84, 6, DQN_type='dense')
    net = Network(None, 'NHWC', 4, 84, 84, 6, beta=0.01, DQN_type=dqn_type, seed=12)
    # non-zero biases so the test sees them
    rng = np.random.default_rng(4)
    for k, v in net.w.items():
        if k.endswith('_b'):
            v.copy_(torch.as_tensor(rng.standard_normal(tuple(v.shape)) * 0.05, dtype=torch.float32))
        else:
            v.mul_(4.0)
    p = _net_params(net)
    B = 6
    planes = rng.integers(0, 256, (B, 4, 84, 84), dtype=np.uint8)
    states = R.states_nhwc(planes)
    fwd = R.forward(p, states, 'a3c', dqn_type)
    out = net.forward(torch.as_tensor(planes).cuda())
    z = np.concatenate([out['policy_logits'].cpu().numpy(), out['value'].cpu().numpy()[:, None]], 1)
    np.testing.assert_allclose(z, fwd['z'], rtol=1e-4, atol=1e-5 * np.abs(fwd['z']).max())
    # float NHWC placeholder input (history.get() layout) gives the same values
    out2 = net.forward(torch.as_tensor(states.astype(np.float32)).cuda())
    assert torch.equal(out2['value'], out['value'])
    pi, logpi, H = R.softmax_stats(fwd['z'][:, :6])
    np.testing.assert_allclose(out['policy'].cpu().numpy(), pi, rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(out['policy_entropy'].cpu().numpy(), H, rtol=1e-4)
    actions = rng.integers(0, 6, B)
    Rt = rng.standard_normal(B)
    losses, dz = R.a3c_loss_and_dz(fwd['z'], actions, Rt, 0.01)
    g_ref = R.backward(p, fwd, dz, 'a3c', dqn_type)
    grads, loss = net.loss_backward(torch.as_tensor(planes).cuda(), actions, Rt.astype(np.float32))
    loss = loss.cpu().numpy()
    for i, key in enumerate(['policy', 'value', 'entropy', 'total']):
        assert abs(loss[i] - losses[key]) <= 1e-4 * max(abs(losses[key]), 1.0), key
    g = grads.cpu().numpy()
    for (name, shp), o, n in zip(net.names_shapes, net.offsets, net.sizes):
        assert rel_l2(g[o:o + n].reshape(shp), g_ref[name]) < 2e-2, name      # independent forward (ReLU flips)
    # and at 1e-4 against the oracle backward on the kernels' own activations (the same ReLU masks)
    fa = {k: v.detach().cpu().numpy().astype(np.float64) for k, v in net.last_forward.items() if v is not None}
    x0 = states.astype(np.float64) / 255.0
    zs = fa['z'][:, :7]
    if dqn_type == 'nature':
        same = dict(z=zs, h3=fa['l4'], flat=fa['l3'], acts=[x0, fa['l1'].reshape(B, 20, 20, 32),
                                                           fa['l2'].reshape(B, 9, 9, 64), fa['l3'].reshape(B, 7, 7, 64)])
    else:
        same = dict(z=zs, h3=fa['l3'], flat=fa['l2'], acts=[x0, fa['l1'].reshape(B, 20, 20, 16),
                                                           fa['l2'].reshape(B, 9, 9, 32)])
    _, dz_same = R.a3c_loss_and_dz(zs, actions, Rt, 0.01)
    g_same = R.backward(p, same, dz_same, 'a3c', dqn_type)
    for (name, shp), o, n in zip(net.names_shapes, net.offsets, net.sizes):
        assert rel_l2(g[o:o + n].reshape(shp), g_same[name]) < 1e-4, (name, rel_l2(g[o:o + n].reshape(shp), g_same[name]))
    acts = net.sample_action(torch.as_tensor(planes).cuda(), seed=1, step=3)
    assert acts.shape == (B,) and int(acts.min()) >= 0 and int(acts.max()) < 6


def test_network_nchw_nature_matches_torch():
    from src.network import Network
    net = Network(None, 'NCHW', 4, 84, 84, 4, beta=0.01, DQN_type='nature', seed=13)
    rng = np.random.default_rng(8)
    planes = rng.integers(0, 256, (3, 4, 84, 84), dtype=np.uint8)
    out = net.forward(torch.as_tensor(planes).cuda())
    T = {k: torch.as_tensor(v, dtype=torch.float64) for k, v in _net_params(net).items()}
    x = torch.as_tensor(planes, dtype=torch.float64) / 255.
    h = x
    for i, s in ((1, 4), (2, 2), (3, 1)):
        h = F.relu(F.conv2d(h, T['l%d_w' % i].permute(3, 2, 0, 1), T['l%d_b' % i], stride=s))
    h = F.relu(h.reshape(3, -1) @ T['l4_w'] + T['l4_b'])           # NCHW flatten (c,h,w)
    np.testing.assert_allclose(out['policy_logits'].cpu().numpy(), (h @ T['p_w'] + T['p_b']).numpy(),
                               rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(out['value'].cpu().numpy(), (h @ T['q_w'] + T['q_b'])[:, 0].numpy(),
                               rtol=1e-4, atol=1e-6)


def test_network_global_copy_and_apply(tmp_path):
    from src.network import Network
    from src.optim import RMSPropOptimizer
    opt = RMSPropOptimizer(7e-4, decay=0.99, momentum=0.0, epsilon=0.1, clip_norm=40.0)
    glob_net = Network(None, 'NHWC', 4, 84, 84, 6, beta=0.01, DQN_type='nips')
    local = Network(None, 'NHWC', 4, 84, 84, 6, beta=0.01, DQN_type='nips', global_network=glob_net,
                    global_optim=opt)
    assert not torch.equal(local.flat, glob_net.flat)
    local.copy_from_global()
    assert torch.equal(local.flat, glob_net.flat)
    rng = np.random.default_rng(5)
    planes = torch.as_tensor(rng.integers(0, 256, (5, 4, 84, 84), dtype=np.uint8)).cuda()
    grads, _ = local.loss_backward(planes, [0, 1, 2, 3, 4], [1.0, -1.0, 0.5, 0.0, 2.0])
    g = grads.cpu().numpy().copy()
    w0 = glob_net.flat.cpu().numpy().copy()
    local.apply_gradients(grads, lr=1e-3)
    w1 = glob_net.flat.cpu().numpy()
    for (name, shp), o, n in zip(local.names_shapes, local.offsets, local.sizes):
        w = w0[o:o + n].copy()
        ms, mom = np.ones(n, np.float32), np.zeros(n, np.float32)
        R.rmsprop_apply(w, ms, mom, R.clip_by_norm(g[o:o + n], 40.0), 1e-3, 0.99, 0.0, 0.1)
        np.testing.assert_allclose(w1[o:o + n], w, rtol=1e-6, atol=1e-7, err_msg=name)
    path = glob_net.save_model(None, str(tmp_path), step=7)
    other = Network(None, 'NHWC', 4, 84, 84, 6, DQN_type='nips')
    assert other.load_model(None, str(tmp_path))
    assert torch.equal(other.flat, glob_net.flat) and path.endswith('.npz')


# ------------------------------------------------------------------ agent.py
def _agent(tmp_path=None, **kw):
    from src.agent import Agent
    from src.environment import GymEnvironment
    from src.optim import RMSPropOptimizer
    cfg = make_config('Breakout-v0', **kw)
    env = GymEnvironment(cfg)
    return Agent(cfg, env, RMSPropOptimizer(None, decay=0.99, momentum=0, epsilon=0.1))


def test_agent_batch_update_matches_oracle():
    agent = _agent()
    rng = np.random.default_rng(6)
    with torch.no_grad():
        agent.params.mul_(3.0)
        agent.target_params.copy_(agent.params * 0.9)
    p = {k: v.detach().cpu().numpy().copy() for k, v in agent.w.items()}
    tp = {k: v.detach().cpu().numpy().copy() for k, v in agent.t_w.items()}
    B = 8
    planes = rng.integers(0, 256, (B + 1, 4, 84, 84), dtype=np.uint8)
    actions = rng.integers(0, 4, B)
    rewards = rng.choice([-1.0, 0.0, 1.0], B).astype(np.float32)
    terms = rng.random(B) < 0.3
    agent.batch_s_t = [torch.as_tensor(x).cuda() for x in planes]
    agent.batch_action, agent.batch_reward, agent.batch_terminal = list(actions), list(rewards), list(terms)
    agent.step, agent.total_loss, agent.total_q, agent.update_count = 1000, 0., 0., 0
    lr = agent.lr
    seen = {}
    lb = agent.net.loss_backward

    def capture(params, s_t, fwd, *a, **kw):          # the kernels' own activations and gradients
        grads, loss = lb(params, s_t, fwd, *a, **kw)
        seen.update(fwd={k: v.detach().cpu().numpy().astype(np.float64) for k, v in fwd.items() if v is not None},
                    grads=grads.detach().cpu().numpy().copy())
        return grads, loss
    agent.net.loss_backward = capture
    agent.batch_update(is_chief=True)
    # oracle
    q_next = R.forward(tp, R.states_nhwc(planes[1:]), 'q')['z']
    target = R.td_target(rewards, terms, q_next, 0.99)
    fwd = R.forward(p, R.states_nhwc(planes[:-1]), 'q')
    loss, dz = R.q_loss_and_dz(fwd['z'], actions, target)
    assert abs(agent.total_loss - loss) <= 1e-4 * abs(loss)
    g = R.backward(p, fwd, dz, 'q')
    for name, w in agent.w.items():
        ref = p[name].copy()
        ms, mom = np.ones_like(ref), np.zeros_like(ref)
        R.rmsprop_apply(ref, ms, mom, R.clip_by_norm(g[name].astype(np.float32), 40.0), lr, 0.99, 0.0, 0.1)
        step = w.detach().cpu().numpy() - p[name]
        assert rel_l2(step, ref - p[name]) < 2e-2, name   # independent fp64 forward (ReLU flips)
    # and at 1e-4 against the oracle backward on the kernels' own activations (the same ReLU masks),
    # then the applied step against TF ApplyRMSProp of the kernels' own clipped gradients at 1e-5
    fa = seen['fwd']
    x0 = R.states_nhwc(planes[:-1]).astype(np.float64) / 255.0
    zs = fa['z'][:, :fwd['z'].shape[1]]
    same = dict(z=zs, h3=fa['l3'], flat=fa['l2'], acts=[x0, fa['l1'].reshape(B, 20, 20, 16),
                                                       fa['l2'].reshape(B, 9, 9, 32)])
    _, dz_same = R.q_loss_and_dz(zs, actions, target)
    g_same = R.backward(p, same, dz_same, 'q')
    g_k = seen['grads']
    for (name, shp), o, n in zip(agent.names_shapes, agent.offsets, agent.sizes):
        e = rel_l2(g_k[o:o + n].reshape(shp), g_same[name])
        assert e < 1e-4, (name, e)
        ref = p[name].copy()
        ms, mom = np.ones_like(ref), np.zeros_like(ref)
        R.rmsprop_apply(ref, ms, mom, R.clip_by_norm(g_k[o:o + n].reshape(shp).astype(np.float32), 40.0),
                        lr, 0.99, 0.0, 0.1)
        step = agent.w[name].detach().cpu().numpy() - p[name]
        assert rel_l2(step, ref - p[name]) < 1e-5, name


def test_agent_train_loop_and_target_update(tmp_path):
    from src.agent import Supervisor
    agent = _agent(train_frequency=8, learn_start=8, target_q_update_step=50, max_step=240, _test_step=100)
    assert agent.test_step == 100
    sv = Supervisor(is_chief=True, logdir=str(tmp_path), agent=agent)
    p0 = agent.params.clone()
    agent.update_target_q_network()
    agent.train_with_summary(sv, True)
    assert agent.step_op == 240
    assert not torch.equal(agent.params, p0)
    lines = open(tmp_path / 'summary.jsonl').read().splitlines()
    assert len(lines) == 1                     # step 199 (summaries only after step 180, agent.py:117)
    path = agent.save(str(tmp_path / 'ckpt'))
    a2 = _agent()
    assert a2.load(path) == 240 and torch.equal(a2.params, agent.params)
    best = agent.play(sv, True, n_step=50, n_episode=2)
    assert best >= 0


def test_agent_double_q_and_dueling():
    agent = _agent(double_q=True)
    rng = np.random.default_rng(9)
    planes = rng.integers(0, 256, (5, 4, 84, 84), dtype=np.uint8)
    agent.batch_s_t = [torch.as_tensor(x).cuda() for x in planes]
    agent.batch_action, agent.batch_reward, agent.batch_terminal = [0, 1, 2, 3], [1.0, 0.0, -1.0, 0.0], \
        [False, True, False, False]
    agent.step, agent.total_loss, agent.total_q, agent.update_count = 10, 0., 0., 0
    p = {k: v.detach().cpu().numpy().copy() for k, v in agent.w.items()}
    tp = {k: v.detach().cpu().numpy().copy() for k, v in agent.t_w.items()}
    agent.batch_update(True)
    qn = R.forward(p, R.states_nhwc(planes[1:]), 'q')['z']
    qt = R.forward(tp, R.states_nhwc(planes[1:]), 'q')['z']
    sel = qt[np.arange(4), qn.argmax(1)]
    target = (1 - np.array([0, 1, 0, 0])) * 0.99 * sel + np.array([1.0, 0.0, -1.0, 0.0])
    fwd = R.forward(p, R.states_nhwc(planes[:-1]), 'q')
    loss, _ = R.q_loss_and_dz(fwd['z'], np.array([0, 1, 2, 3]), target)
    assert abs(agent.total_loss - loss) <= 1e-4 * abs(loss)
    duel = _agent(dueling=True)
    assert 'l3_adv_w' in duel.w and 'val_w_out' in duel.w
    pl = torch.as_tensor(planes[:3]).cuda()
    q = duel.q_values(pl).cpu().numpy()
    T = {k: torch.as_tensor(v.detach().cpu().numpy(), dtype=torch.float64) for k, v in duel.w.items()}
    x = torch.as_tensor(planes[:3], dtype=torch.float64) / 255.
    h = F.relu(F.conv2d(x, T['l1_w'].permute(3, 2, 0, 1), T['l1_b'], stride=4))
    h = F.relu(F.conv2d(h, T['l2_w'].permute(3, 2, 0, 1), T['l2_b'], stride=2)).permute(0, 2, 3, 1).reshape(3, -1)
    v = F.relu(h @ T['l3_val_w'] + T['l3_val_b']) @ T['val_w_out'] + T['val_w_b']
    a = F.relu(h @ T['l3_adv_w'] + T['l3_adv_b']) @ T['adv_w_out'] + T['adv_w_b']
    np.testing.assert_allclose(q, (v + a - a.mean(1, keepdim=True)).numpy(), rtol=1e-4, atol=1e-6)
    duel.batch_s_t = [torch.as_tensor(x).cuda() for x in planes]
    duel.batch_action, duel.batch_reward, duel.batch_terminal = [0, 1, 2, 3], [1.0, 0.0, -1.0, 0.0], [False] * 4
    duel.step, duel.total_loss, duel.total_q, duel.update_count = 10, 0., 0., 0
    duel.batch_update(True)
    assert duel.update_count == 1 and np.isfinite(duel.total_loss)


@pytest.mark.parametrize('update', ['overlap', 'sync', 'hogwild'])
def test_main_engine_mode_runs(tmp_path, update):
    """main.py --mode engine (the batched drop-in for main.py:58-94) in every update mode."""
    import main
    eng = main.main(['--mode', 'engine', '--env_name', 'Breakout-v0', '--num_envs', '32', '--num_frames', '256',
                     '--iterations', '6', '--log_every', '3', '--logdir', str(tmp_path), '--update', update])
    torch.cuda.synchronize()
    assert torch.isfinite(eng.params).all()
    lines = open(tmp_path / 'engine.jsonl').read().splitlines()
    assert len(lines) == 2


@pytest.mark.parametrize('update', ['sync', 'overlap'])
def test_main_engine_mode_host_envs(tmp_path, update):
    """main.py --mode engine --envs_on host: host-stepped envs feed the engine
    (overlap falls back to the synchronous engine); hogwild and a missing gym are refused."""
    import main
    eng = main.main(['--mode', 'engine', '--env_name', 'Pong-v0', '--num_envs', '16', '--num_frames', '64',
                     '--iterations', '4', '--log_every', '2', '--logdir', str(tmp_path), '--update', update,
                     '--envs_on', 'host', '--host_threads', '4'])
    torch.cuda.synchronize()
    assert eng.external_env and torch.isfinite(eng.params).all()
    assert int(eng.counters[1].item()) == 4 * 16 * 5
    assert len(open(tmp_path / 'engine.jsonl').read().splitlines()) == 2
    with pytest.raises(ValueError):
        main.main(['--mode', 'engine', '--envs_on', 'host', '--update', 'hogwild', '--num_envs', '4',
                   '--iterations', '1', '--logdir', str(tmp_path)])
    try:
        import gym  # noqa: F401
    except ImportError:
        with pytest.raises(RuntimeError):
            main.main(['--mode', 'engine', '--envs_on', 'gym', '--num_envs', '4', '--iterations', '1',
                       '--logdir', str(tmp_path)])


def test_main_engine_mode_initialises_params_and_stops_at_max_step(tmp_path):
    """main.py --mode engine starts from the reference initialisers (conv truncated_normal(0,
    0.02) agent.py:214, linear normal(0.02) ops.py:36-37, zero biases), not from whatever
    hipMalloc returned, and trains no further than max_step on each worker's own loop counter
    (agent.py:46,55: `for self.step in xrange(self.step, self.max_step)`; here every env is such a
    worker, stepping in lock-step)."""
    import main
    from src.kernels import param_names_shapes
    E, n = 16, 5
    eng = main.main(['--mode', 'engine', '--env_name', 'Pong-v0', '--num_envs', str(E), '--num_frames', '64',
                     '--iterations', '50', '--log_every', '100', '--logdir', str(tmp_path), '--update', 'sync',
                     '--max_step', str(3 * n - 1), '--random_seed', '7', '--resume', 'false'])
    torch.cuda.synchronize()
    assert int(eng.counters[1].item()) == 3 * E * n          # 3 rollouts of n reach max_step, then stop
    assert eng.worker_step == 3 * n
    flat = eng.params.cpu().numpy()
    ns = param_names_shapes(6, 'a3c')
    for (name, shp), off, size in zip(ns, eng.offsets, eng.sizes):
        v = flat[off:off + size]
        if name.endswith('_b'):
            assert np.abs(v).max() < 0.05, name              # zero-initialised, 3 small updates
        else:
            assert abs(float(v.std()) - 0.02) < 0.006, (name, float(v.std()))
            assert np.count_nonzero(v) == v.size
    # past max_step the schedule is clamped at 0 (agent.py:393-395 would turn negative)
    from src.engine import _view
    before = eng.params.clone()
    eng.iterate()
    torch.cuda.synchronize()
    assert _view(eng.sched_ptr, (2,), torch.float32)[0].item() == 0.0
    assert torch.equal(before, eng.params)

"""Cross-check the oracle's hand-written forward/backward (oracle/ref_cpu.py) against torch CPU
autograd in float64 -- an independent implementation of the same TF semantics:
conv2d VALID NHWC with [kh,kw,cin,cout] weights (ops.py:21-28), flatten in (h,w,c) order
(agent.py:231-232), linear x@W+b (ops.py:41), the A3C losses with the SURVEY §8 A11 fixes and
the Q-learning MSE (agent.py:310-314).  The TF reference itself cannot run here (no TF), so this
is what pins the network/loss arithmetic ("parity unpinned" against a reference execution)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import ref_cpu as R


def torch_forward(p, states, algo):
    x = torch.as_tensor(states, dtype=torch.float64).permute(0, 3, 1, 2) / 255.0    # NHWC -> NCHW
    T = {k: torch.as_tensor(v, dtype=torch.float64).requires_grad_(True) for k, v in p.items()}
    w1 = T['l1_w'].permute(3, 2, 0, 1)          # [kh,kw,cin,cout] -> [cout,cin,kh,kw]
    w2 = T['l2_w'].permute(3, 2, 0, 1)
    h = F.relu(F.conv2d(x, w1, T['l1_b'], stride=4))
    h = F.relu(F.conv2d(h, w2, T['l2_b'], stride=2))
    flat = h.permute(0, 2, 3, 1).reshape(h.shape[0], -1)     # (h,w,c) order
    fc = 'l4' if algo == 'a3c' else 'l3'
    h3 = F.relu(flat @ T[fc + '_w'] + T[fc + '_b'])
    if algo == 'a3c':
        z = torch.cat([h3 @ T['p_w'] + T['p_b'], h3 @ T['q_w'] + T['q_b']], dim=1)
    else:
        z = h3 @ T['q_w'] + T['q_b']
    return T, z


@pytest.mark.parametrize('algo,A,literal', [('a3c', 6, False), ('a3c', 4, True), ('q', 6, False)])
def test_oracle_backward_matches_torch_autograd(algo, A, literal):
    rng = np.random.default_rng(11)
    B = 5
    from make_goldens import frame_from_spec  # noqa: F401  (conftest path check)
    shapes = R.param_shapes(A, algo)
    p = R.init_params(shapes, seed=3, stddev=0.08)
    for k in p:
        if k.endswith('_b'):
            p[k] = (rng.standard_normal(p[k].shape) * 0.05).astype(np.float32)
    states = rng.integers(0, 256, (B, 84, 84, 4), dtype=np.uint8)
    actions = rng.integers(0, A, B)
    target = rng.standard_normal(B)
    fwd = R.forward(p, states, algo)
    T, z = torch_forward(p, states, algo)
    np.testing.assert_allclose(z.detach().numpy(), fwd['z'], rtol=1e-10, atol=1e-12)
    beta = 0.01
    if algo == 'a3c':
        losses, dz = R.a3c_loss_and_dz(fwd['z'], actions, target, beta, literal)
        logits, V = z[:, :A], z[:, A]
        logpi = F.log_softmax(logits, dim=1)
        pi = logpi.exp()
        H = -(pi * logpi).sum(1)
        adv = torch.as_tensor(target) - V
        lp_a = logpi[torch.arange(B), torch.as_tensor(actions)]
        pol = -(lp_a * (adv if literal else adv.detach())) - beta * H
        loss = (pol + 0.5 * adv * adv).sum()
        assert np.isclose(loss.item(), losses['total'], rtol=1e-12)
        assert np.isclose((-(lp_a * adv) - beta * H).sum().item(), losses['policy'], rtol=1e-12)
    else:
        l, dz = R.q_loss_and_dz(fwd['z'], actions, target)
        q_a = z[torch.arange(B), torch.as_tensor(actions)]
        loss = ((torch.as_tensor(target) - q_a) ** 2).mean()
        assert np.isclose(loss.item(), l, rtol=1e-12)
    loss.backward()
    g = R.backward(p, fwd, dz, algo)
    for k in p:
        np.testing.assert_allclose(g[k].reshape(p[k].shape), T[k].grad.numpy(), rtol=1e-9, atol=1e-12,
                                   err_msg=k)


def test_rmsprop_differs_from_torch_default_as_documented():
    """torch.optim.RMSprop (eps outside sqrt, square_avg init 0) is NOT TF's ApplyRMSProp: the
    oracle follows TF (rms init 1.0, eps inside sqrt) -- guard against silently swapping them."""
    w = np.array([0.5], np.float32)
    ms, mom = np.ones(1, np.float32), np.zeros(1, np.float32)
    R.rmsprop_apply(w, ms, mom, np.array([2.0], np.float32), 0.1, 0.99, 0.0, 0.1)
    tw = torch.tensor([0.5], requires_grad=True)
    opt = torch.optim.RMSprop([tw], lr=0.1, alpha=0.99, eps=0.1)
    tw.grad = torch.tensor([2.0])
    opt.step()
    assert not np.isclose(w[0], tw.item(), rtol=1e-3)
    exp = 0.5 - 0.1 * 2.0 / np.sqrt(1.0 + (4.0 - 1.0) * 0.01 + 0.1)
    assert np.isclose(w[0], exp, rtol=1e-6)


def test_lstm_oracle_matches_torch_autograd():
    """C5 LSTM head (build-defined, no reference code): the oracle's hand-written truncated BPTT
    (ref_cpu.lstm_a3c_backward) against torch autograd in float64 over an n-step sequence with
    in-rollout terminals (state zeroed after a terminal transition) and a nonzero carry-in."""
    rng = np.random.default_rng(5)
    n, E, A, U = 4, 3, 6, R.LSTM_UNITS
    p = R.init_params(R.param_shapes(A, 'a3c', lstm=True), seed=9, stddev=0.05)
    for k in p:
        if k.endswith('_b'):
            p[k] = (rng.standard_normal(p[k].shape) * 0.05).astype(np.float32)
    states = rng.integers(0, 256, (n * E, 84, 84, 4), dtype=np.uint8)
    terms = np.zeros((n, E), np.uint8)
    terms[1, 0] = 1
    terms[2, 2] = 1
    h0 = rng.standard_normal((E, U)) * 0.3
    c0 = rng.standard_normal((E, U)) * 0.3
    actions = rng.integers(0, A, n * E)
    target = rng.standard_normal(n * E)
    fwd = R.lstm_a3c_forward(p, states, n, h0, c0, terms)
    losses, dz = R.a3c_loss_and_dz(fwd['z'], actions, target, 0.01)
    g = R.lstm_a3c_backward(p, fwd, dz, terms)

    T, _ = torch_forward({k: v for k, v in p.items() if not k.startswith('lstm')}, states, 'a3c')
    for k in ('lstm_w', 'lstm_b'):
        T[k] = torch.as_tensor(p[k], dtype=torch.float64).requires_grad_(True)
    # recompute the trunk from the same leaves (torch_forward's z used h3 directly)
    x = torch.as_tensor(states, dtype=torch.float64).permute(0, 3, 1, 2) / 255.0
    h = F.relu(F.conv2d(x, T['l1_w'].permute(3, 2, 0, 1), T['l1_b'], stride=4))
    h = F.relu(F.conv2d(h, T['l2_w'].permute(3, 2, 0, 1), T['l2_b'], stride=2))
    h3 = F.relu(h.permute(0, 2, 3, 1).reshape(n * E, -1) @ T['l4_w'] + T['l4_b']).reshape(n, E, -1)
    hp, cp = torch.as_tensor(h0), torch.as_tensor(c0)
    hs = []
    for t in range(n):
        a = torch.cat([h3[t], hp], 1) @ T['lstm_w'] + T['lstm_b']
        i, j, f, o = a.split(U, dim=1)
        c = cp * torch.sigmoid(f + 1.0) + torch.sigmoid(i) * torch.tanh(j)
        hh = torch.tanh(c) * torch.sigmoid(o)
        hs.append(hh)
        keep = torch.as_tensor(1.0 - terms[t].astype(np.float64))[:, None]
        hp, cp = hh * keep, c * keep
    H = torch.cat(hs, 0)
    z = torch.cat([H @ T['p_w'] + T['p_b'], H @ T['q_w'] + T['q_b']], dim=1)
    np.testing.assert_allclose(z.detach().numpy(), fwd['z'], rtol=1e-10, atol=1e-12)
    logpi = F.log_softmax(z[:, :A], dim=1)
    pi = logpi.exp()
    Hent = -(pi * logpi).sum(1)
    adv = torch.as_tensor(target) - z[:, A]
    lp_a = logpi[torch.arange(n * E), torch.as_tensor(actions)]
    loss = (-(lp_a * adv.detach()) - 0.01 * Hent + 0.5 * adv * adv).sum()
    assert np.isclose(loss.item(), losses['total'], rtol=1e-12)
    loss.backward()
    for k in p:
        np.testing.assert_allclose(np.asarray(g[k]).reshape(p[k].shape), T[k].grad.numpy(), rtol=1e-9,
                                   atol=1e-12, err_msg=k)
    carry = fwd['lstm']['carry']
    np.testing.assert_allclose(carry[0], hp.detach().numpy(), rtol=1e-12, atol=1e-14)


def test_nature_oracle_matches_torch_autograd():
    """The nature trunk (network.py:30-42: conv 8x8/4 32, conv 4x4/2 64, conv 3x3/1 64, fc 3136 -> 512)
    in the oracle's hand-written forward / backward against torch autograd in float64, under the
    A3C losses -- what pins the engine's nature kernels (tests/test_gpu_nature.py compare them with
    this oracle)."""
    rng = np.random.default_rng(17)
    A, B, beta = 6, 3, 0.01
    shapes = R.param_shapes(A, 'a3c', dqn_type='nature')
    p = R.init_params(shapes, seed=5, stddev=0.05)
    for k in p:
        if k.endswith('_b'):
            p[k] = (rng.standard_normal(p[k].shape) * 0.05).astype(np.float32)
    states = rng.integers(0, 256, (B, 84, 84, 4), dtype=np.uint8)
    actions = rng.integers(0, A, B)
    target = rng.standard_normal(B)
    fwd = R.forward(p, states, 'a3c', dqn_type='nature')
    x = torch.as_tensor(states, dtype=torch.float64).permute(0, 3, 1, 2) / 255.0
    T = {k: torch.as_tensor(v, dtype=torch.float64).requires_grad_(True) for k, v in p.items()}
    h = x
    for name, s in (('l1', 4), ('l2', 2), ('l3', 1)):
        h = F.relu(F.conv2d(h, T[name + '_w'].permute(3, 2, 0, 1), T[name + '_b'], stride=s))
    flat = h.permute(0, 2, 3, 1).reshape(B, -1)               # (h, w, c) order: 7 x 7 x 64
    h4 = F.relu(flat @ T['l4_w'] + T['l4_b'])
    z = torch.cat([h4 @ T['p_w'] + T['p_b'], h4 @ T['q_w'] + T['q_b']], dim=1)
    np.testing.assert_allclose(z.detach().numpy(), fwd['z'], rtol=1e-10, atol=1e-12)
    losses, dz = R.a3c_loss_and_dz(fwd['z'], actions, target, beta, False)
    logpi = F.log_softmax(z[:, :A], dim=1)
    H = -(logpi.exp() * logpi).sum(1)
    adv = torch.as_tensor(target) - z[:, A]
    lp_a = logpi[torch.arange(B), torch.as_tensor(actions)]
    loss = (-(lp_a * adv.detach()) - beta * H + 0.5 * adv * adv).sum()
    assert np.isclose(loss.item(), losses['total'], rtol=1e-12)
    loss.backward()
    g = R.backward(p, fwd, dz, 'a3c', dqn_type='nature')
    for k in p:
        np.testing.assert_allclose(g[k].reshape(p[k].shape), T[k].grad.numpy(), rtol=1e-9, atol=1e-12,
                                   err_msg=k)

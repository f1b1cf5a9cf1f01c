"""numpy restatement of the reference's rollout + gradient path (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module; it is the checker, never the thing measured or shipped.

Each function cites the reference (``/root/reference``) file:line it restates.
Pinning status:
* ``luminance_u8``/``resize_bilinear_u8``/``screen`` and ``History``: pinned by golden
  vectors generated from the reference's own ``src/environment.py`` and
  ``src/history.py`` (tests/golden/make_goldens.py).
* network / loss / clip / RMSProp arithmetic: **parity unpinned** against a reference
  execution (TensorFlow 0.x is not installed and unpinned); cross-checked against torch
  CPU autograd (tests/test_oracle_autograd.py) and TF's documented op semantics.
"""
import math
import numpy as np

# --------------------------------------------------------------------------------------
# A1  Environment.screen  (environment.py:49-53)
# --------------------------------------------------------------------------------------

def luminance_u8(rgb):
    """environment.py:51-52: ``0.2126*R + 0.7152*G + 0.0722*B`` evaluated by numpy as
    u8 x python-float -> float64, left to right, then ``.astype(np.uint8)`` (truncation)."""
    rgb = np.asarray(rgb)
    r = rgb[..., 0].astype(np.float64)
    g = rgb[..., 1].astype(np.float64)
    b = rgb[..., 2].astype(np.float64)
    y = 0.2126 * r + 0.7152 * g + 0.0722 * b
    return y.astype(np.uint8)


PRECISION_BITS = 32 - 8 - 2   # Pillow Resample.c 8bpc fixed point


def pillow_bilinear_coeffs(in_size, out_size):
    """Coefficients of Pillow's separable BILINEAR resample (``precompute_coeffs`` +
    ``normalize_coeffs_8bpc``), which is what ``scipy.misc.imresize(y, dims)``
    (environment.py:5-8,99; scipy<1.3 -> ``PIL.Image.resize(size, BILINEAR)``) runs.
    Third-party algorithm pinned to Pillow 12.2.0 by the golden vectors.
    Returns (bounds[out,2] int32 = (xmin, count), kk[out, ksize] int32)."""
    support_f = 1.0                               # bilinear filter support
    scale = float(np.float32(in_size)) / out_size  # (double)(in1 - in0) / outSize
    filterscale = max(scale, 1.0)
    support = support_f * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int32)
    kk = np.zeros((out_size, ksize), np.int32)
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        ss = 1.0 / filterscale
        xmin = int(center - support + 0.5)        # C cast truncates toward zero
        if xmin < 0:
            xmin = 0
        xmax = int(center + support + 0.5)
        if xmax > in_size:
            xmax = in_size
        xmax -= xmin
        w = np.zeros(ksize, np.float64)
        ww = 0.0
        for x in range(xmax):
            t = abs((x + xmin - center + 0.5) * ss)
            w[x] = 1.0 - t if t < 1.0 else 0.0
            ww += w[x]
        if ww != 0.0:
            w[:xmax] = w[:xmax] / ww
        for x in range(ksize):
            v = w[x] * (1 << PRECISION_BITS)
            kk[xx, x] = int(-0.5 + v) if w[x] < 0 else int(0.5 + v)
        bounds[xx] = (xmin, xmax)
    return bounds, kk


def _clip8(acc):
    return np.clip(acc >> PRECISION_BITS, 0, 255).astype(np.uint8)


def resize_bilinear_u8(img, out_h, out_w):
    """Pillow ``ImagingResample`` two-pass (horizontal first into a u8 temp covering
    rows [ybox_first, ybox_last), then vertical), 8bpc fixed point: accumulator starts
    at 1<<(PRECISION_BITS-1), products u8*int32, ``clip8(acc >> 22)``."""
    img = np.asarray(img, np.uint8)
    in_h, in_w = img.shape
    hb, hk = pillow_bilinear_coeffs(in_w, out_w)
    vb, vk = pillow_bilinear_coeffs(in_h, out_h)
    y0 = int(vb[0, 0])
    y1 = int(vb[-1, 0] + vb[-1, 1])
    src = img[y0:y1].astype(np.int64)
    acc = np.full((y1 - y0, out_w), 1 << (PRECISION_BITS - 1), np.int64)
    for x in range(hk.shape[1]):
        idx = np.minimum(hb[:, 0] + x, in_w - 1)
        valid = x < hb[:, 1]
        acc += np.where(valid, src[:, idx] * hk[:, x].astype(np.int64), 0)
    tmp = _clip8(acc).astype(np.int64)
    acc = np.full((out_h, out_w), 1 << (PRECISION_BITS - 1), np.int64)
    for y in range(vk.shape[1]):
        idx = np.minimum(vb[:, 0] - y0 + y, tmp.shape[0] - 1)
        valid = (y < vb[:, 1])[:, None]
        acc += np.where(valid, tmp[idx, :] * vk[:, y].astype(np.int64)[:, None], 0)
    return _clip8(acc)


def screen(rgb, out_h=84, out_w=84):
    """environment.py:49-53 for one [H,W,3] frame or a batch [E,H,W,3]."""
    rgb = np.asarray(rgb, np.uint8)
    if rgb.ndim == 3:
        return resize_bilinear_u8(luminance_u8(rgb), out_h, out_w)
    return np.stack([screen(f, out_h, out_w) for f in rgb])


# --------------------------------------------------------------------------------------
# A3  History (history.py:3-27)
# --------------------------------------------------------------------------------------

class History:
    """history.py:3-27 restated (float32 [L,H,W] shift register)."""

    def __init__(self, history_length=4, screen_height=84, screen_width=84, cnn_format='NHWC'):
        self.cnn_format = cnn_format
        self.history = np.zeros([history_length, screen_height, screen_width], np.float32)

    def add(self, screen):            # history.py:13-15
        self.history[:-1] = self.history[1:]
        self.history[-1] = screen

    def reset(self):                  # history.py:17-18
        self.history *= 0

    def get(self):                    # history.py:20-24
        if self.cnn_format == 'NHWC':
            return np.transpose(self.history, (1, 2, 0))
        return self.history

    def copy(self):                   # history.py:26-27
        return self.get().copy()


# --------------------------------------------------------------------------------------
# A5 / A11  network trunk + heads (agent.py:217-254, network.py:43-79, ops.py:4-46)
# --------------------------------------------------------------------------------------

NIPS = dict(conv=[(16, 8, 4), (32, 4, 2)], fc=256)                    # network.py:43-52 / agent.py:226-251
NATURE = dict(conv=[(32, 8, 4), (64, 4, 2), (64, 3, 1)], fc=512)       # network.py:30-42


def trunk_spec(dqn_type='nips', history_length=4, h=84, w=84):
    spec = NIPS if dqn_type.lower() == 'nips' else NATURE
    layers = []
    cin, hh, ww = history_length, h, w
    for cout, k, s in spec['conv']:
        oh, ow = (hh - k) // s + 1, (ww - k) // s + 1
        layers.append(dict(cin=cin, cout=cout, k=k, s=s, ih=hh, iw=ww, oh=oh, ow=ow))
        cin, hh, ww = cout, oh, ow
    return layers, hh * ww * cin, spec['fc']


def param_shapes(action_size, algo='a3c', dqn_type='nips', history_length=4, lstm=False):
    """TF variable order/shapes (ops.py:21-24 conv ``w`` [kh,kw,cin,cout] + ``biases``;
    ops.py:36-39 linear ``Matrix`` [in,out] + ``bias``).  a3c: network.py names
    (l*_w/l*_b, p_w/p_b policy, q_w/q_b value); q: agent.py names (l*_w/l*_b, q_w/q_b)."""
    convs, flat, fc = trunk_spec(dqn_type, history_length)
    shapes = []
    for i, c in enumerate(convs):
        shapes.append((f'l{i+1}_w', (c['k'], c['k'], c['cin'], c['cout'])))
        shapes.append((f'l{i+1}_b', (c['cout'],)))
    fcname = 'l4' if algo == 'a3c' else 'l3'
    shapes.append((f'{fcname}_w', (flat, fc)))
    shapes.append((f'{fcname}_b', (fc,)))
    if algo == 'a3c':
        shapes += [('p_w', (fc, action_size)), ('p_b', (action_size,)),
                   ('q_w', (fc, 1)), ('q_b', (1,))]
    else:
        shapes += [('q_w', (fc, action_size)), ('q_b', (action_size,))]
    if lstm:
        shapes += lstm_param_shapes(LSTM_UNITS, fc)
    return shapes


def init_params(shapes, seed=123, stddev=0.02):
    """ops.py:21 conv weights truncated_normal(0, 0.02) (agent.py:214, network.py:10);
    ops.py:36-37 linear Matrix random_normal(stddev=0.02); biases zero (ops.py:24,38).
    The draws use numpy (TF's op RNG is not reproducible here)."""
    rng = np.random.default_rng(seed)
    out = {}
    for name, shp in shapes:
        if name.endswith('_b'):
            out[name] = np.zeros(shp, np.float32)
        elif len(shp) == 4:
            v = rng.standard_normal(shp)
            bad = np.abs(v) > 2.0
            while bad.any():
                v[bad] = rng.standard_normal(int(bad.sum()))
                bad = np.abs(v) > 2.0
            out[name] = (v * stddev).astype(np.float32)
        else:
            out[name] = (rng.standard_normal(shp) * stddev).astype(np.float32)
    return out


def _patches(x, k, s):
    """x [B,H,W,C] -> [B,OH,OW,k,k,C] VALID im2col view (ops.py:22 conv2d VALID, NHWC)."""
    B, H, W, C = x.shape
    oh, ow = (H - k) // s + 1, (W - k) // s + 1
    sb, sh, sw, sc = x.strides
    return np.lib.stride_tricks.as_strided(
        x, (B, oh, ow, k, k, C), (sb, sh * s, sw * s, sh, sw, sc), writeable=False)


def states_nhwc(planes):
    """[B,L,H,W] u8 frame planes (oldest first) -> [B,H,W,L] (history.py:20-22 NHWC)."""
    return np.ascontiguousarray(np.transpose(planes, (0, 2, 3, 1)))


def forward(params, states_u8, algo='a3c', dqn_type='nips', dtype=np.float64, keep=True):
    """Trunk + head forward.  ``states_u8`` is [B,84,84,4] NHWC (values 0..255).
    agent.py:226 / network.py:46 ``s_t / 255.``; conv2d+bias+relu (ops.py:22-28);
    flatten (h,w,c) (agent.py:231-232); linear relu (ops.py:41-44); head linear.
    Returns dict with 'z' [B, A(+1)] (a3c: logits then value) and saved activations."""
    convs, flat, fc = trunk_spec(dqn_type)
    x = states_u8.astype(dtype) / dtype(255.0)
    acts = [x]
    for i, c in enumerate(convs):
        w = params[f'l{i+1}_w'].astype(dtype)
        b = params[f'l{i+1}_b'].astype(dtype)
        p = _patches(x, c['k'], c['s'])
        B = x.shape[0]
        y = p.reshape(B * c['oh'] * c['ow'], -1) @ w.reshape(-1, c['cout']) + b
        x = np.maximum(y, 0).reshape(B, c['oh'], c['ow'], c['cout'])
        acts.append(x)
    h = x.reshape(x.shape[0], -1)
    fcname = 'l4' if algo == 'a3c' else 'l3'
    h3 = np.maximum(h @ params[f'{fcname}_w'].astype(dtype) + params[f'{fcname}_b'].astype(dtype), 0)
    if algo == 'a3c':
        logits = h3 @ params['p_w'].astype(dtype) + params['p_b'].astype(dtype)
        value = h3 @ params['q_w'].astype(dtype) + params['q_b'].astype(dtype)
        z = np.concatenate([logits, value], axis=1)
    else:
        z = h3 @ params['q_w'].astype(dtype) + params['q_b'].astype(dtype)
    out = dict(z=z, h3=h3, flat=h)
    if keep:
        out['acts'] = acts
    return out


def softmax_stats(logits):
    """network.py:60-69: pi = softmax, log pi = log(pi), H = -sum pi log pi.
    (log-softmax form: same value, no log(0) for underflowed pi.)"""
    m = logits.max(axis=1, keepdims=True)
    e = np.exp(logits - m)
    s = e.sum(axis=1, keepdims=True)
    pi = e / s
    logpi = (logits - m) - np.log(s)
    ent = -(pi * logpi).sum(axis=1)
    return pi, logpi, ent


def sample_categorical(pi32, u):
    """Build-defined ``batch_sample`` (network.py:4,72 -- missing in the reference):
    first j with fp32 cumsum(pi)[j] > u, else A-1."""
    pi32 = np.asarray(pi32, np.float32)
    A = pi32.shape[1]
    cdf = np.zeros(pi32.shape[0], np.float32)
    act = np.full(pi32.shape[0], A - 1, np.int32)
    done = np.zeros(pi32.shape[0], bool)
    for j in range(A):
        cdf = (cdf + pi32[:, j]).astype(np.float32)
        hit = (~done) & (cdf > u)
        act[hit] = j
        done |= hit
    return act


# --------------------------------------------------------------------------------------
# A7 / A11  returns, TD target, losses
# --------------------------------------------------------------------------------------

def nstep_returns(rewards, terminals, bootstrap_value, gamma=0.99):
    """assets/a3c.png Algorithm S3: R = 0 if terminal else V(s_t); for i = t-1..t_start:
    R <- r_i + gamma R.  Batched over envs [n,E], R reset at in-rollout terminals.
    Evaluated in float64 as the reference's numpy host code does (agent.py:188-190)."""
    n = rewards.shape[0]
    R = np.asarray(bootstrap_value, np.float64).copy()
    out = np.zeros(rewards.shape, np.float64)
    for i in range(n - 1, -1, -1):
        R = np.where(terminals[i], 0.0, R)
        R = rewards[i].astype(np.float64) + gamma * R
        out[i] = R
    return out


def td_target(reward, terminal, q_next, discount=0.99):
    """agent.py:186-190 in float64: (1 - term) * discount * max_a Q'(s') + reward."""
    terminal = np.asarray(terminal) + 0.
    return (1. - terminal) * discount * np.max(np.asarray(q_next, np.float64), axis=1) + \
        np.asarray(reward, np.float64)


def td_target_double(reward, terminal, q_next_target, q_next_online, discount=0.99):
    """agent.py:176-184 (double Q-learning) in float64: pred_action = argmax_a Q(s') of the online
    net (q_action = tf.argmax: the first maximum), then (1 - term) * discount * Q'(s', pred_action)
    + reward with the target net's Q'."""
    pred = np.argmax(np.asarray(q_next_online), axis=1)
    qt = np.asarray(q_next_target, np.float64)[np.arange(len(pred)), pred]
    terminal = np.asarray(terminal) + 0.
    return (1. - terminal) * discount * qt + np.asarray(reward, np.float64)


def a3c_loss_and_dz(z, actions, R, beta=0.01, literal_advantage_grad=False):
    """network.py:81-94 with the two bugs fixed: V squeezed to [N]
    and log pi(a) = log_softmax gathered at a.  Per-sample
    L = -log pi(a)*stopgrad(R-V) - beta*H + (R-V)^2/2; summed over the batch (TF
    compute_gradients of a vector loss == gradient of its sum).
    Returns (losses dict, dz [B, A+1])."""
    A = z.shape[1] - 1
    logits, V = z[:, :A], z[:, A]
    pi, logpi, H = softmax_stats(logits)
    B = z.shape[0]
    lp_a = logpi[np.arange(B), actions]
    adv = R - V
    policy_loss = -(lp_a * adv) - beta * H
    value_loss = 0.5 * adv * adv
    onehot = np.zeros_like(pi)
    onehot[np.arange(B), actions] = 1.0
    dlog = -adv[:, None] * (onehot - pi) + beta * pi * (logpi + H[:, None])
    dV = -adv + (lp_a if literal_advantage_grad else 0.0)
    dz = np.concatenate([dlog, dV[:, None]], axis=1)
    losses = dict(policy=policy_loss.sum(), value=value_loss.sum(), entropy=H.sum(),
                  total=(policy_loss + value_loss).sum())
    return losses, dz


def q_loss_and_dz(z, actions, target):
    """agent.py:306-314: loss = mean((target - Q(s)[a])^2); dL/dQ[a] = -2 delta / B."""
    B = z.shape[0]
    q_acted = z[np.arange(B), actions]
    delta = target - q_acted
    loss = np.mean(delta * delta)
    dz = np.zeros_like(z)
    dz[np.arange(B), actions] = -2.0 * delta / B
    return loss, dz


# --------------------------------------------------------------------------------------
# A9  backward (compute_gradients, agent.py:317)
# --------------------------------------------------------------------------------------

def backward(params, fwd, dz, algo='a3c', dqn_type='nips'):
    """Manual reverse pass of ``forward`` (conv1 gets weight grads only: the input
    placeholder needs no gradient).  Returns grads dict keyed like params."""
    convs, flat, fc = trunk_spec(dqn_type)
    dtype = fwd['z'].dtype
    g = {}
    h3 = fwd['h3']
    if algo == 'a3c':
        A = dz.shape[1] - 1
        g['p_w'] = h3.T @ dz[:, :A]
        g['p_b'] = dz[:, :A].sum(0)
        g['q_w'] = h3.T @ dz[:, A:]
        g['q_b'] = dz[:, A:].sum(0)
        dh3 = dz[:, :A] @ params['p_w'].astype(dtype).T + dz[:, A:] @ params['q_w'].astype(dtype).T
    else:
        g['q_w'] = h3.T @ dz
        g['q_b'] = dz.sum(0)
        dh3 = dz @ params['q_w'].astype(dtype).T
    dh3 = dh3 * (h3 > 0)
    return trunk_backward(params, fwd, dh3, g, algo, dqn_type)


def trunk_backward(params, fwd, dh3, g, algo='a3c', dqn_type='nips'):
    """Reverse pass from dL/d(fc pre-ReLU-masked output) ``dh3`` down through fc, conv2, conv1
    (shared by the feed-forward head and the LSTM head); fills and returns ``g``."""
    convs, flat, fc = trunk_spec(dqn_type)
    dtype = fwd['z'].dtype
    fcname = 'l4' if algo == 'a3c' else 'l3'
    g[f'{fcname}_w'] = fwd['flat'].T @ dh3
    g[f'{fcname}_b'] = dh3.sum(0)
    acts = fwd['acts']
    dx = (dh3 @ params[f'{fcname}_w'].astype(dtype).T).reshape(acts[-1].shape)
    dx = dx * (acts[-1] > 0)
    for i in range(len(convs) - 1, -1, -1):
        c = convs[i]
        xin = acts[i]
        B = xin.shape[0]
        p = _patches(xin, c['k'], c['s']).reshape(B * c['oh'] * c['ow'], -1)
        dy = dx.reshape(-1, c['cout'])
        g[f'l{i+1}_w'] = (p.T @ dy).reshape(c['k'], c['k'], c['cin'], c['cout'])
        g[f'l{i+1}_b'] = dy.sum(0)
        if i == 0:
            break
        w = params[f'l{i+1}_w'].astype(dtype).reshape(-1, c['cout'])
        dp = (dy @ w.T).reshape(B, c['oh'], c['ow'], c['k'], c['k'], c['cin'])
        dxin = np.zeros_like(xin)
        s = c['s']
        for kh in range(c['k']):
            for kw in range(c['k']):
                dxin[:, kh:kh + s * c['oh']:s, kw:kw + s * c['ow']:s, :] += dp[:, :, :, kh, kw, :]
        dx = dxin * (xin > 0)
    return g


# --------------------------------------------------------------------------------------
# A9 / A10  clip_by_norm + TF ApplyRMSProp (agent.py:316-321, main.py:63-65)
# --------------------------------------------------------------------------------------

def clip_by_norm(g, clip_norm=40.0):
    """tf.clip_by_norm (agent.py:319), TF 0.x form evaluated in float32:
    t * clip_norm * min(rsqrt(sum(t*t)), 1/clip_norm)."""
    g = np.asarray(g, np.float32)
    ss = np.float32(np.sum(g.astype(np.float64) ** 2))
    inv = np.float32(1.0) / np.sqrt(ss) if ss > 0 else np.float32(np.inf)
    return (g * np.float32(clip_norm)) * np.minimum(np.float32(inv), np.float32(1.0) / np.float32(clip_norm))


def rmsprop_apply(var, ms, mom, grad, lr, decay=0.99, momentum=0.0, epsilon=0.1):
    """TF ApplyRMSProp (main.py:64-65 RMSPropOptimizer(lr, decay=.99, momentum=0,
    epsilon=.1), applied by agent.py:321): ms += (g^2 - ms)(1 - rho);
    mom = mom*momentum + lr*g/sqrt(ms + eps); var -= mom.  The rms slot is
    initialised to 1.0 and mom to 0 (TF1 RMSPropOptimizer._create_slots).  In place."""
    f = np.float32
    ms += (grad * grad - ms) * (f(1.0) - f(decay))
    mom[...] = mom * f(momentum) + (grad * f(lr)) / np.sqrt(ms + f(epsilon))
    var -= mom


def learning_rate(step, max_step=80_000_000, learning_rate=0.0007):
    """agent.py:393-395.  The reference stops training at max_step (agent.py:46,55-57), where this
    is still > 0; past it the build clamps at 0 (a negative rate would make RMSProp ascend)."""
    return max(0.0, (max_step - step + 1.) / max_step * learning_rate)


def epsilon_schedule(step, ep_start=1., ep_end=0.1, ep_end_t=4_000_000, learn_start=32):
    """agent.py:142-144."""
    return ep_end + max(0., (ep_start - ep_end) * (ep_end_t - max(0., step - learn_start)) / ep_end_t)


# --------------------------------------------------------------------------------------
# C5  LSTM policy head (BASELINE config 5).  The reference has NO recurrent code (SURVEY §8(f)
# rank 4): this is a build-defined head, restated from TF1's ``BasicLSTMCell`` (tf.nn.rnn_cell,
# state_is_tuple, forget_bias=1.0; third-party, not in the reference) and the A3C-LSTM of the
# paper the reference implements (assets/a3c.png; Mnih et al. 2016: one 256-cell LSTM after
# the last hidden layer).  Parity unpinned against any reference execution; cross-checked
# against torch CPU autograd (tests/test_oracle_autograd.py).
#   gates a = [x, h_prev] @ W + b, W [256+U, 4U], columns (i, j, f, o)
#   c = c_prev * sigmoid(f + forget_bias) + sigmoid(i) * tanh(j);  h = tanh(c) * sigmoid(o)
# The recurrent state carried from step t to t+1 is zeroed when transition t was terminal
# (h_prev = h_t * (1 - term_t)).  Truncated BPTT over the n-step rollout: no gradient into the
# rollout's initial state.
# --------------------------------------------------------------------------------------
LSTM_UNITS = 256
FORGET_BIAS = 1.0


def lstm_param_shapes(units=LSTM_UNITS, fc=256):
    """flat order: appended after the a3c head (build-defined)."""
    return [('lstm_w', (fc + units, 4 * units)), ('lstm_b', (4 * units,))]


def _sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


def lstm_cell(x, h, c, W, b, forget_bias=FORGET_BIAS):
    """One BasicLSTMCell step; returns (h', c', gates) with gates = activated (i, j, f, o)."""
    dtype = x.dtype
    a = np.concatenate([x, h], axis=1) @ W.astype(dtype) + b.astype(dtype)
    U = h.shape[1]
    si = _sigmoid(a[:, :U])
    tj = np.tanh(a[:, U:2 * U])
    sf = _sigmoid(a[:, 2 * U:3 * U] + forget_bias)
    so = _sigmoid(a[:, 3 * U:])
    c2 = c * sf + si * tj
    h2 = np.tanh(c2) * so
    return h2, c2, np.concatenate([si, tj, sf, so], axis=1)


def lstm_forward_seq(params, x_seq, h0, c0, terms):
    """x_seq [n,E,256] (the fc ReLU outputs), (h0, c0) [E,U] the already-masked carry-in,
    terms [n,E].  Returns dict H, C (cell outputs per step), HP, CP (masked inputs per step),
    G (activated gates) and the carry-out (h, c) after masking by terms[n-1]."""
    n = x_seq.shape[0]
    W, b = params['lstm_w'], params['lstm_b']
    hp, cp = h0, c0
    H, C, HP, CP, G = [], [], [], [], []
    for t in range(n):
        HP.append(hp)
        CP.append(cp)
        h, c, g = lstm_cell(x_seq[t], hp, cp, W, b)
        H.append(h)
        C.append(c)
        G.append(g)
        keep = (1.0 - np.asarray(terms[t], np.float64))[:, None].astype(h.dtype)
        hp, cp = h * keep, c * keep
    return dict(H=np.stack(H), C=np.stack(C), HP=np.stack(HP), CP=np.stack(CP), G=np.stack(G),
                carry=(hp, cp))


def lstm_backward_seq(params, seq, x_seq, dH, terms):
    """Truncated BPTT of ``lstm_forward_seq``: dH [n,E,U] = dL/dh_t from the heads.  Returns
    (dX [n,E,256], dW, db)."""
    n, E, U = dH.shape
    W = params['lstm_w'].astype(dH.dtype)
    G, C, CP, HP = seq['G'], seq['C'], seq['CP'], seq['HP']
    dX = np.zeros(x_seq.shape, dH.dtype)
    dW = np.zeros(W.shape, dH.dtype)
    db = np.zeros(W.shape[1], dH.dtype)
    dh_next = np.zeros((E, U), dH.dtype)    # dL/d(masked h input of step t+1)
    dc_next = np.zeros((E, U), dH.dtype)
    for t in range(n - 1, -1, -1):
        keep = (1.0 - np.asarray(terms[t], np.float64))[:, None].astype(dH.dtype)
        dh = dH[t] + dh_next * keep
        i, j, f, o = (G[t][:, k * U:(k + 1) * U] for k in range(4))
        tc = np.tanh(C[t])
        dc = dc_next * keep + dh * o * (1.0 - tc * tc)
        da = np.concatenate([dc * j * i * (1.0 - i), dc * i * (1.0 - j * j),
                             dc * CP[t] * f * (1.0 - f), dh * tc * o * (1.0 - o)], axis=1)
        xh = np.concatenate([x_seq[t], HP[t]], axis=1)
        dW += xh.T @ da
        db += da.sum(0)
        dxh = da @ W.T
        dX[t] = dxh[:, :x_seq.shape[2]]
        dh_next = dxh[:, x_seq.shape[2]:]
        dc_next = dc * f
    return dX, dW, db


def lstm_a3c_forward(params, states_u8, n, h0, c0, terms, dtype=np.float64):
    """Trunk over the n*E states (b = t*E + e), the LSTM over the n steps, and the policy /
    value heads on h_t.  Returns the trunk dict of ``forward`` with z replaced by the LSTM
    head's z, plus 'lstm' (the sequence) and 'x_seq'."""
    fwd = forward(params, states_u8, 'a3c', dtype=dtype)
    E = states_u8.shape[0] // n
    x_seq = fwd['h3'].reshape(n, E, -1)
    seq = lstm_forward_seq(params, x_seq, h0.astype(dtype), c0.astype(dtype), terms)
    Hf = seq['H'].reshape(n * E, -1)
    logits = Hf @ params['p_w'].astype(dtype) + params['p_b'].astype(dtype)
    value = Hf @ params['q_w'].astype(dtype) + params['q_b'].astype(dtype)
    fwd['z'] = np.concatenate([logits, value], axis=1)
    fwd['lstm'] = seq
    fwd['x_seq'] = x_seq
    return fwd


def lstm_a3c_backward(params, fwd, dz, terms):
    """Heads on h_t, BPTT through the LSTM, then the ReLU-masked fc/conv trunk."""
    dtype = fwd['z'].dtype
    seq, x_seq = fwd['lstm'], fwd['x_seq']
    n, E, U = seq['H'].shape
    A = dz.shape[1] - 1
    Hf = seq['H'].reshape(n * E, U)
    g = {'p_w': Hf.T @ dz[:, :A], 'p_b': dz[:, :A].sum(0), 'q_w': Hf.T @ dz[:, A:], 'q_b': dz[:, A:].sum(0)}
    dH = dz[:, :A] @ params['p_w'].astype(dtype).T + dz[:, A:] @ params['q_w'].astype(dtype).T
    dX, g['lstm_w'], g['lstm_b'] = lstm_backward_seq(params, seq, x_seq, dH.reshape(n, E, U), terms)
    dh3 = dX.reshape(n * E, -1) * (fwd['h3'] > 0)
    return trunk_backward(params, fwd, dh3, g, 'a3c')

"""Torch-tensor front end of the C-ABI (include/a3c_hip.h).

Each function takes/returns device tensors, allocates outputs with torch (caller-owned memory
in the C-ABI's terms) and enqueues on the current torch stream.  Reference arithmetic each one
replaces is cited on the C-ABI declaration.
"""
import ctypes

import torch

from . import _lib
from ._lib import check, lib, ptr, stream_handle

IMG = 84
HIST = 4
FLAT = 2592
FC = 256
C1 = 400 * 16


def _dev(t, dtype, name):
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise ValueError(f'{name} must be a CUDA (HIP) tensor')
    if t.dtype != dtype:
        raise ValueError(f'{name} must be {dtype}, got {t.dtype}')
    if not t.is_contiguous():
        raise ValueError(f'{name} must be contiguous')
    return t


def preprocess(rgb, frame_idx=None, out_hw=(IMG, IMG), out=None):
    """Environment.screen (environment.py:49-53) for frames rgb [N,H,W,3] u8 (or a frame pool
    indexed by ``frame_idx`` [n] int32).  Returns [n,oh,ow] u8, bit-exact to the reference."""
    _dev(rgb, torch.uint8, 'rgb')
    if rgb.dim() == 3:
        rgb = rgb.unsqueeze(0)
    H, W = int(rgb.shape[1]), int(rgb.shape[2])
    n = int(rgb.shape[0]) if frame_idx is None else int(frame_idx.numel())
    if frame_idx is not None:
        _dev(frame_idx, torch.int32, 'frame_idx')
    oh, ow = out_hw
    if out is None:
        out = torch.empty((n, oh, ow), dtype=torch.uint8, device=rgb.device)
    check(lib().a3c_preprocess_u8(ptr(rgb), ptr(frame_idx), n, H, W, ptr(out), oh * ow, oh, ow,
                                  stream_handle()), 'a3c_preprocess_u8')
    return out


def luminance(rgb):
    """environment.py:51-52 alone: [...,3] u8 -> [...] u8 (exact integer form of the fp64 sum)."""
    _dev(rgb, torch.uint8, 'rgb')
    out = torch.empty(rgb.shape[:-1], dtype=torch.uint8, device=rgb.device)
    check(lib().a3c_luminance_u8(ptr(rgb), out.numel(), ptr(out), stream_handle()), 'a3c_luminance_u8')
    return out


def history_push(hist, screens, reset_mask=None):
    """History.add (+ History.reset when reset_mask) on [n,L,h,w] u8 histories, in place."""
    _dev(hist, torch.uint8, 'hist')
    _dev(screens, torch.uint8, 'screens')
    n, L = int(hist.shape[0]), int(hist.shape[1])
    hw = int(hist.shape[2] * hist.shape[3])
    if reset_mask is not None:
        _dev(reset_mask, torch.uint8, 'reset_mask')
    check(lib().a3c_history_push(ptr(hist), ptr(screens), ptr(reset_mask), n, L, hw, stream_handle()),
          'a3c_history_push')
    return hist


def history_get(hist, nhwc=True):
    """History.get (history.py:20-24): float32 [n,h,w,L] (NHWC) or [n,L,h,w]."""
    _dev(hist, torch.uint8, 'hist')
    n, L, h, w = (int(s) for s in hist.shape)
    shape = (n, h, w, L) if nhwc else (n, L, h, w)
    out = torch.empty(shape, dtype=torch.float32, device=hist.device)
    check(lib().a3c_history_get_f32(ptr(hist), n, L, h, w, 1 if nhwc else 0, ptr(out), stream_handle()),
          'a3c_history_get_f32')
    return out


def param_names_shapes(action_size, algo='a3c', lstm=False, dqn_type='nips'):
    """TF variable names/shapes in flat order (agent.py:226-252 q-net, network.py:47-79 a3c);
    lstm: the C5 LSTM head's gate matrix and bias appended (include/a3c_hip.h layout);
    dqn_type='nature': network.py:30-42's trunk (conv 32/64/64, fc 3136 -> 512) under A3C heads."""
    A = int(action_size)
    if str(dqn_type).lower() == 'nature':
        if algo != 'a3c' or lstm:
            raise ValueError('the nature trunk belongs to the A3C Network (network.py:30-42): a3c heads, no LSTM')
        return [('l1_w', (8, 8, 4, 32)), ('l1_b', (32,)), ('l2_w', (4, 4, 32, 64)), ('l2_b', (64,)),
                ('l3_w', (3, 3, 64, 64)), ('l3_b', (64,)), ('l4_w', (3136, 512)), ('l4_b', (512,)),
                ('p_w', (512, A)), ('p_b', (A,)), ('q_w', (512, 1)), ('q_b', (1,))]
    if str(dqn_type).lower() != 'nips':
        raise ValueError('Wrong DQN type: %s' % dqn_type)
    fc = 'l4' if algo == 'a3c' else 'l3'
    out = [('l1_w', (8, 8, 4, 16)), ('l1_b', (16,)), ('l2_w', (4, 4, 16, 32)), ('l2_b', (32,)),
           (fc + '_w', (FLAT, FC)), (fc + '_b', (FC,))]
    if algo == 'a3c':
        out += [('p_w', (FC, A)), ('p_b', (A,)), ('q_w', (FC, 1)), ('q_b', (1,))]
    else:
        out += [('q_w', (FC, A)), ('q_b', (A,))]
    if lstm:
        if algo != 'a3c':
            raise ValueError('the LSTM head is an a3c head')
        U = _lib.A3C_LSTM_UNITS
        out += [('lstm_w', (FC + U, 4 * U)), ('lstm_b', (4 * U,))]
    return out


def lstm_step(w, b, x, h_src, c_src, prev_terms=None, save=True):
    """One C5 LSTM cell step (a3c_lstm_step) for B envs: x [B,256], (h_src, c_src) [B,U] the previous
    step's outputs (zeroed where prev_terms [B] u8 is set).  Returns dict h, c (+ hp, cp, gates)."""
    B, U = int(x.shape[0]), _lib.A3C_LSTM_UNITS
    for t, nm in ((w, 'w'), (b, 'b'), (x, 'x'), (h_src, 'h_src'), (c_src, 'c_src')):
        _dev(t, torch.float32, nm)
    if prev_terms is not None:
        _dev(prev_terms, torch.uint8, 'prev_terms')
    new = lambda *s: torch.empty(s, dtype=torch.float32, device=x.device)  # noqa: E731
    out = dict(h=new(B, U), c=new(B, U))
    if save:
        out.update(hp=new(B, U), cp=new(B, U), gates=new(B, 4 * U))
    w_t = torch.empty((w.shape[1], w.shape[0]), dtype=torch.float32, device=x.device)
    check(lib().a3c_lstm_transpose(ptr(w), ptr(w_t), stream_handle()), 'a3c_lstm_transpose')
    check(lib().a3c_lstm_step(ptr(w_t), ptr(b), ptr(x), ptr(h_src), ptr(c_src), ptr(prev_terms), B,
                              ptr(out.get('hp')), ptr(out.get('cp')), ptr(out.get('gates')), ptr(out['h']),
                              ptr(out['c']), stream_handle()), 'a3c_lstm_step')
    return out


def lstm_bptt(w, x, hp, cp, gates, c, terms, dh):
    """Truncated BPTT (a3c_lstm_bptt) over [n,E,...] sequences; returns (dx masked by x > 0, dw, db)."""
    n, E = int(terms.shape[0]), int(terms.shape[1])
    for t, nm in ((w, 'w'), (x, 'x'), (hp, 'hp'), (cp, 'cp'), (gates, 'gates'), (c, 'c'), (dh, 'dh')):
        _dev(t, torch.float32, nm)
    _dev(terms, torch.uint8, 'terms')
    nb = _lib.c_i64()
    check(lib().a3c_lstm_workspace_bytes(n, E, ctypes.byref(nb)), 'a3c_lstm_workspace_bytes')
    ws = torch.empty(int(nb.value), dtype=torch.uint8, device=x.device)
    dx = torch.empty_like(x)
    dw = torch.empty_like(w)
    db = torch.empty(w.shape[-1], dtype=torch.float32, device=x.device)
    check(lib().a3c_lstm_bptt(ptr(w), n, E, ptr(x), ptr(hp), ptr(cp), ptr(gates), ptr(c), ptr(terms), ptr(dh),
                              ptr(dx), ptr(dw), ptr(db), ptr(ws), stream_handle()), 'a3c_lstm_bptt')
    return dx, dw, db


class NatureNet:
    """The nature trunk (network.py:30-42) + A3C heads on the nature.hip kernels: flat parameters
    in the C-ABI layout (include/a3c_hip.h), history_length 4."""

    def __init__(self, action_size):
        self.algo = 'a3c'
        self.A = int(action_size)
        self.desc = _lib.net_desc(self.A, 'a3c', dqn_type='nature')
        self.offsets, self.sizes, self.total = _lib.param_layout(self.desc)
        self.zs = _lib.z_stride(self.desc)
        self.names_shapes = param_names_shapes(self.A, 'a3c', dqn_type='nature')
        assert [int(torch.Size(s).numel()) for _, s in self.names_shapes] == self.sizes

    def workspace(self, B, device='cuda'):
        n = _lib.c_i64()
        check(lib().a3c_nature_workspace_bytes(ctypes.byref(self.desc), max(int(B), 1), ctypes.byref(n)),
              'a3c_nature_workspace_bytes')
        return torch.empty(int(n.value), dtype=torch.uint8, device=device)

    def forward(self, params, states, workspace=None):
        """states [B,4,84,84] u8 (oldest frame first).  Returns dict z/l1/l2/l3/l4."""
        _dev(params, torch.float32, 'params')
        _dev(states, torch.uint8, 'states')
        B = int(states.shape[0])
        dev = states.device
        out = dict(l1=torch.empty((B, 12800), dtype=torch.float32, device=dev),
                   l2=torch.empty((B, 5184), dtype=torch.float32, device=dev),
                   l3=torch.empty((B, 3136), dtype=torch.float32, device=dev),
                   l4=torch.empty((B, 512), dtype=torch.float32, device=dev),
                   z=torch.empty((B, self.zs), dtype=torch.float32, device=dev))
        ws = workspace if workspace is not None else self.workspace(B, dev)
        check(lib().a3c_nature_forward(ctypes.byref(self.desc), ptr(params), ptr(states), B, ptr(out['l1']),
                                       ptr(out['l2']), ptr(out['l3']), ptr(out['l4']), ptr(out['z']), ptr(ws),
                                       stream_handle()), 'a3c_nature_forward')
        return out

    def loss_backward(self, params, states, fwd, actions, target, beta=0.01, literal_adv=False, grads=None,
                      workspace=None):
        _dev(actions, torch.int32, 'actions')
        _dev(target, torch.float32, 'target')
        B = int(states.shape[0])
        dev = states.device
        if grads is None:
            grads = torch.zeros(self.total, dtype=torch.float32, device=dev)
        loss = torch.zeros(4, dtype=torch.float32, device=dev)
        ws = workspace if workspace is not None else self.workspace(B, dev)
        check(lib().a3c_nature_loss_backward(ctypes.byref(self.desc), ptr(params), ptr(states), B, ptr(fwd['l1']),
                                             ptr(fwd['l2']), ptr(fwd['l3']), ptr(fwd['l4']), ptr(fwd['z']),
                                             ptr(actions), ptr(target), float(beta), 1 if literal_adv else 0,
                                             ptr(grads), ptr(loss), ptr(ws), stream_handle()),
              'a3c_nature_loss_backward')
        return grads, loss


class Net:
    """Flat-parameter description of the NIPS trunk + head for ``algo`` in {'a3c','q'}."""

    def __init__(self, action_size, algo='a3c'):
        if algo not in ('a3c', 'q'):
            raise ValueError('Wrong algo: %s' % algo)
        self.algo = algo
        self.A = int(action_size)
        self.desc = _lib.net_desc(self.A, algo)
        self.offsets, self.sizes, self.total = _lib.param_layout(self.desc)
        self.zs = _lib.z_stride(self.desc)
        self.names_shapes = param_names_shapes(self.A, algo)
        assert [int(torch.Size(s).numel()) for _, s in self.names_shapes] == self.sizes

    def __repr__(self):
        return f'Net(algo={self.algo}, A={self.A}, params={self.total})'

    # flat <-> dict
    def flatten(self, params, device='cuda'):
        flat = torch.zeros(self.total, dtype=torch.float32, device=device)
        for (name, shp), off, n in zip(self.names_shapes, self.offsets, self.sizes):
            v = torch.as_tensor(params[name], dtype=torch.float32).reshape(-1)
            if v.numel() != n:
                raise ValueError(f'{name}: expected {n} values, got {v.numel()}')
            flat[off:off + n] = v.to(device)
        return flat

    def unflatten(self, flat):
        return {name: flat[off:off + n].reshape(shp)
                for (name, shp), off, n in zip(self.names_shapes, self.offsets, self.sizes)}

    def views(self, flat):
        return self.unflatten(flat)

    def workspace(self, B, device='cuda'):
        nbytes = _lib.workspace_bytes(self.desc, max(int(B), 1))
        return torch.empty(nbytes, dtype=torch.uint8, device=device)

    # -- forward (agent.py:217-254 / network.py:43-79) --------------------------------
    def forward(self, params, states, save_l1=True, workspace=None):
        """states [B,4,84,84] u8 (oldest frame first).  Returns dict z/l1/l2/l3."""
        _dev(params, torch.float32, 'params')
        _dev(states, torch.uint8, 'states')
        B = int(states.shape[0])
        dev = states.device
        l1 = torch.empty((B, C1), dtype=torch.float32, device=dev) if save_l1 else None
        l2 = torch.empty((B, FLAT), dtype=torch.float32, device=dev)
        l3 = torch.empty((B, FC), dtype=torch.float32, device=dev)
        z = torch.empty((B, self.zs), dtype=torch.float32, device=dev)
        ws = workspace if workspace is not None else self.workspace(B, dev)
        check(lib().a3c_forward(ctypes.byref(self.desc), ptr(params), ptr(states), B, ptr(l1), ptr(l2), ptr(l3),
                                ptr(z), ptr(ws), stream_handle()), 'a3c_forward')
        return dict(z=z, l1=l1, l2=l2, l3=l3)

    # -- K8/K9 loss + backward ----------------------------------------------------------
    def loss_backward(self, params, states, fwd, actions, target, beta=0.01, literal_adv=False,
                      grads=None, workspace=None):
        _dev(actions, torch.int32, 'actions')
        _dev(target, torch.float32, 'target')
        B = int(states.shape[0])
        dev = states.device
        if grads is None:
            grads = torch.zeros(self.total, dtype=torch.float32, device=dev)
        loss = torch.zeros(4, dtype=torch.float32, device=dev)
        ws = workspace if workspace is not None else self.workspace(B, dev)
        check(lib().a3c_loss_backward(ctypes.byref(self.desc), ptr(params), ptr(states), B, ptr(fwd['l1']),
                                      ptr(fwd['l2']), ptr(fwd['l3']), ptr(fwd['z']), ptr(actions), ptr(target),
                                      float(beta), 1 if literal_adv else 0, ptr(grads), ptr(loss), ptr(ws),
                                      stream_handle()), 'a3c_loss_backward')
        return grads, loss

    # -- K10/K11 clip + RMSProp -----------------------------------------------------------
    def _opt_ws(self, device):
        b = _lib.c_i64()
        check(lib().a3c_optim_workspace_bytes(self.total, ctypes.byref(b)), 'a3c_optim_workspace_bytes')
        return torch.empty(int(b.value), dtype=torch.uint8, device=device)

    def clip_rmsprop_apply(self, params, ms, mom, grads, lr, decay=0.99, momentum=0.0, epsilon=0.1,
                           clip=40.0, sumsq=None):
        ws = self._opt_ws(params.device)
        check(lib().a3c_clip_rmsprop_apply(ptr(params), ptr(ms), ptr(mom), ptr(grads), len(self.offsets),
                                           _lib.i64_array(self.offsets), _lib.i64_array(self.sizes), float(lr),
                                           float(decay), float(momentum), float(epsilon), float(clip), ptr(sumsq),
                                           ptr(ws), stream_handle()), 'a3c_clip_rmsprop_apply')

    def clip_grads(self, grads, clip=40.0, sumsq=None):
        ws = self._opt_ws(grads.device)
        check(lib().a3c_clip_grads(ptr(grads), len(self.offsets), _lib.i64_array(self.offsets),
                                   _lib.i64_array(self.sizes), float(clip), ptr(sumsq), ptr(ws), stream_handle()),
              'a3c_clip_grads')


def select_action(mode, z, A, seed, tau, eps=None, env_ids=None):
    """mode 0 categorical (network.py:65-72), 1 epsilon-greedy (agent.py:141-151)."""
    _dev(z, torch.float32, 'z')
    B, zs = int(z.shape[0]), int(z.shape[1])
    actions = torch.empty(B, dtype=torch.int32, device=z.device)
    check(lib().a3c_select_action(int(mode), ptr(z), B, zs, int(A), ptr(eps), int(seed) & (2 ** 64 - 1), int(tau),
                                  ptr(env_ids), ptr(actions), stream_handle()), 'a3c_select_action')
    return actions


def returns(rewards, terminals, bootstrap, gamma=0.99):
    """n-step returns [n,E] (assets/a3c.png) in float64 -> float32."""
    _dev(rewards, torch.float32, 'rewards')
    _dev(terminals, torch.uint8, 'terminals')
    _dev(bootstrap, torch.float32, 'bootstrap')
    n, E = int(rewards.shape[0]), int(rewards.shape[1])
    R = torch.empty((n, E), dtype=torch.float32, device=rewards.device)
    check(lib().a3c_returns(ptr(rewards), ptr(terminals), ptr(bootstrap), n, E, float(gamma), ptr(R),
                            stream_handle()), 'a3c_returns')
    return R


def td_target(rewards, terminals, q_next, A, discount=0.99):
    """agent.py:186-190."""
    B = int(rewards.shape[0])
    out = torch.empty(B, dtype=torch.float32, device=rewards.device)
    check(lib().a3c_td_target(ptr(rewards), ptr(terminals), ptr(q_next), B, int(A), int(q_next.shape[1]),
                              float(discount), ptr(out), stream_handle()), 'a3c_td_target')
    return out


def copy_params(dst, src):
    check(lib().a3c_copy_params(ptr(dst), ptr(src), int(src.numel()), stream_handle()), 'a3c_copy_params')

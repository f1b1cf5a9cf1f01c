"""ctypes binding of liba3c_hip.so (C-ABI declared in include/a3c_hip.h).

This is the only place the Python mirror of the reference API touches native code.  The
library is loaded after ``torch`` so both share torch's HIP runtime (same SONAME
``libamdhip64.so.7``): torch tensors provide device memory and ``torch.cuda`` streams are
valid ``hipStream_t`` handles here.  There is no CPU fallback: every op raises if the
library or a gfx950 device is missing.
"""
import ctypes
import os
import sys

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# A3C_LIB: alternative build of the same library (kernel A/B experiments, tools/ab.sh)
LIB_PATH = os.environ.get('A3C_LIB') or os.path.join(os.path.dirname(_HERE), 'lib', 'liba3c_hip.so')

A3C_ALGO_A3C = 0
A3C_ALGO_Q = 1
A3C_TRUNK_NIPS = 0
A3C_TRUNK_NATURE = 1
A3C_LSTM_UNITS = 256
MAX_TENSORS = 16

c_int, c_i64, c_u64, c_float, c_double, c_void_p = (ctypes.c_int, ctypes.c_int64, ctypes.c_uint64,
                                                    ctypes.c_float, ctypes.c_double, ctypes.c_void_p)


class NetDesc(ctypes.Structure):
    _fields_ = [('algo', c_int), ('trunk', c_int), ('action_size', c_int),
                ('history_length', c_int), ('screen_h', c_int), ('screen_w', c_int), ('lstm_units', c_int)]


class EngineConfig(ctypes.Structure):
    _fields_ = [('net', NetDesc), ('num_envs', c_int), ('n_step', c_int), ('env_id_base', c_int),
                ('world_size', c_int), ('start_lives', c_int), ('random_start', c_int),
                ('action_repeat', c_int), ('num_frames', c_int), ('use_graph', c_int),
                ('seed', c_u64), ('gamma', c_double), ('beta', c_float), ('learning_rate', c_float),
                ('max_step', c_i64), ('decay', c_float), ('momentum', c_float), ('epsilon', c_float),
                ('clip_norm', c_float), ('literal_adv', c_int), ('ep_start', c_float),
                ('ep_end', c_float), ('ep_end_t', c_i64), ('learn_start', c_i64),
                ('target_q_update_step', c_i64), ('discount', c_double), ('overlap', c_int),
                ('external_env', c_int), ('frame84', c_int), ('split_exchange', c_int),
                ('double_q', c_int)]


class EngineBuffers(ctypes.Structure):
    _fields_ = [('params', c_void_p), ('target_params', c_void_p), ('ms', c_void_p), ('mom', c_void_p),
                ('grads', c_void_p), ('n_params', c_i64), ('frame_ring', c_void_p), ('ring_slots', c_int),
                ('tau', c_void_p), ('global_step', c_void_p), ('actions', c_void_p), ('rewards', c_void_p),
                ('terminals', c_void_p), ('z', c_void_p), ('returns', c_void_p), ('loss', c_void_p),
                ('sumsq', c_void_p), ('act_l1', c_void_p), ('act_l2', c_void_p), ('act_l3', c_void_p),
                ('frame_pool', c_void_p), ('env_frame', c_void_p), ('env_lives', c_void_p),
                ('env_episode', c_void_p), ('env_step', c_void_p), ('env_len', c_void_p),
                ('zs', c_int), ('n_tensors', c_int), ('offsets', c_i64 * MAX_TENSORS),
                ('sizes', c_i64 * MAX_TENSORS), ('sched', c_void_p),
                ('lstm_h', c_void_p), ('lstm_c', c_void_p), ('lstm_hp', c_void_p), ('lstm_cp', c_void_p),
                ('lstm_gates', c_void_p), ('lstm_units', c_int), ('act_l4', c_void_p), ('trunk', c_int)]


# name -> (restype, argtypes)
SIGNATURES = {
    'a3c_version': (ctypes.c_char_p, []),
    'a3c_last_error': (ctypes.c_char_p, []),
    'a3c_device_ok': (c_int, []),
    'a3c_param_layout': (c_int, [ctypes.POINTER(NetDesc), ctypes.POINTER(c_int), ctypes.POINTER(c_i64),
                                 ctypes.POINTER(c_i64), ctypes.POINTER(c_i64)]),
    'a3c_workspace_bytes': (c_int, [ctypes.POINTER(NetDesc), c_i64, ctypes.POINTER(c_i64)]),
    'a3c_preprocess_u8': (c_int, [c_void_p, c_void_p, c_i64, c_int, c_int, c_void_p, c_i64, c_int, c_int,
                                  c_void_p]),
    'a3c_luminance_u8': (c_int, [c_void_p, c_i64, c_void_p, c_void_p]),
    'a3c_history_push': (c_int, [c_void_p, c_void_p, c_void_p, c_i64, c_int, c_i64, c_void_p]),
    'a3c_history_get_f32': (c_int, [c_void_p, c_i64, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    'a3c_z_stride': (c_int, [ctypes.POINTER(NetDesc)]),
    'a3c_forward': (c_int, [ctypes.POINTER(NetDesc), c_void_p, c_void_p, c_i64, c_void_p, c_void_p, c_void_p,
                            c_void_p, c_void_p, c_void_p]),
    'a3c_select_action': (c_int, [c_int, c_void_p, c_i64, c_int, c_int, c_void_p, c_u64, c_i64, c_void_p,
                                  c_void_p, c_void_p]),
    'a3c_returns': (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_i64, c_double, c_void_p, c_void_p]),
    'a3c_td_target': (c_int, [c_void_p, c_void_p, c_void_p, c_i64, c_int, c_int, c_double, c_void_p,
                              c_void_p]),
    'a3c_loss_backward': (c_int, [ctypes.POINTER(NetDesc), c_void_p, c_void_p, c_i64, c_void_p, c_void_p,
                                  c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_int, c_void_p,
                                  c_void_p, c_void_p, c_void_p]),
    'a3c_nature_workspace_bytes': (c_int, [ctypes.POINTER(NetDesc), c_i64, ctypes.POINTER(c_i64)]),
    'a3c_nature_forward': (c_int, [ctypes.POINTER(NetDesc), c_void_p, c_void_p, c_i64, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_void_p, c_void_p]),
    'a3c_nature_loss_backward': (c_int, [ctypes.POINTER(NetDesc), c_void_p, c_void_p, c_i64, c_void_p, c_void_p,
                                         c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_int, c_void_p,
                                         c_void_p, c_void_p, c_void_p]),
    'a3c_optim_workspace_bytes': (c_int, [c_i64, ctypes.POINTER(c_i64)]),
    'a3c_clip_grads': (c_int, [c_void_p, c_int, ctypes.POINTER(c_i64), ctypes.POINTER(c_i64), c_float,
                               c_void_p, c_void_p, c_void_p]),
    'a3c_clip_rmsprop_apply': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, ctypes.POINTER(c_i64),
                                       ctypes.POINTER(c_i64), c_float, c_float, c_float, c_float, c_float,
                                       c_void_p, c_void_p, c_void_p]),
    'a3c_conv2d_forward': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p] + [c_int] * 11 + [c_void_p]),
    'a3c_conv2d_backward': (c_int, [c_void_p] * 6 + [c_int] * 10 + [c_void_p]),
    'a3c_matmul': (c_int, [c_void_p, c_i64, c_i64, c_void_p, c_i64, c_i64, c_void_p, c_i64, c_int, c_int, c_int,
                           c_void_p, c_int, c_int, c_void_p]),
    'a3c_copy_params': (c_int, [c_void_p, c_void_p, c_i64, c_void_p]),
    'a3c_lstm_transpose': (c_int, [c_void_p, c_void_p, c_void_p]),
    'a3c_lstm_step': (c_int, [c_void_p] * 6 + [c_i64] + [c_void_p] * 6),
    'a3c_lstm_workspace_bytes': (c_int, [c_int, c_i64, ctypes.POINTER(c_i64)]),
    'a3c_lstm_bptt': (c_int, [c_void_p, c_int, c_i64] + [c_void_p] * 12),
    'a3c_env_create': (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_u64, c_int, ctypes.POINTER(c_void_p)]),
    'a3c_env_destroy': (c_int, [c_void_p]),
    'a3c_env_new_game': (c_int, [c_void_p, c_void_p, c_int, c_void_p]),
    'a3c_env_act': (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    'a3c_env_screen': (c_int, [c_void_p, c_void_p, c_i64, c_void_p]),
    'a3c_env_buffers': (c_int, [c_void_p] + [ctypes.POINTER(c_void_p)] * 7),
    'a3c_engine_config_default': (None, [ctypes.POINTER(EngineConfig)]),
    'a3c_engine_create': (c_int, [ctypes.POINTER(EngineConfig), ctypes.POINTER(c_void_p)]),
    'a3c_engine_destroy': (c_int, [c_void_p]),
    'a3c_engine_reset': (c_int, [c_void_p, c_void_p, c_void_p]),
    'a3c_engine_rollout_grad': (c_int, [c_void_p, c_void_p]),
    'a3c_engine_apply': (c_int, [c_void_p, c_void_p]),
    'a3c_engine_iterate': (c_int, [c_void_p, c_void_p]),
    'a3c_engine_span_stats': (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    'a3c_engine_span_steps': (c_int, [c_void_p, c_void_p, c_void_p]),
    'a3c_engine_span_raw': (c_int, [c_void_p, c_int, c_void_p, c_void_p]),
    'a3c_engine_get_buffers': (c_int, [c_void_p, ctypes.POINTER(EngineBuffers)]),
    'a3c_engine_slot_buffers': (c_int, [c_void_p, c_int, ctypes.POINTER(EngineBuffers)]),
    'a3c_engine_grad_ready': (c_int, [c_void_p]),
    'a3c_engine_advance': (c_int, [c_void_p, c_void_p]),
    'a3c_engine_set_step': (c_int, [c_void_p, c_i64, c_i64, c_void_p]),
    'a3c_engine_stats_accumulate': (c_int, [c_void_p, c_void_p]),
    'a3c_engine_stats_read': (c_int, [c_void_p, c_void_p, c_int, c_void_p]),
    'a3c_engine_state_bytes': (c_int, [c_void_p, ctypes.POINTER(c_i64)]),
    'a3c_engine_state_save': (c_int, [c_void_p, c_void_p, c_i64, c_void_p]),
    'a3c_engine_state_load': (c_int, [c_void_p, c_void_p, c_i64, c_void_p]),
    'a3c_engine_apply_shard': (c_int, [c_void_p, c_void_p, c_int, c_i64, c_i64, c_void_p, c_void_p]),
    'a3c_engine_apply_commit': (c_int, [c_void_p, c_void_p, c_void_p]),
    'a3c_engine_exchange_split': (c_int, [c_void_p, ctypes.POINTER(c_i64)]),
    'a3c_engine_wait_grad_head': (c_int, [c_void_p, c_void_p]),
    'a3c_engine_ext_begin': (c_int, [c_void_p, c_void_p, c_void_p]),
    'a3c_hostenv_create': (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_u64, c_int, c_int,
                                   ctypes.POINTER(c_void_p)]),
    'a3c_hostenv_destroy': (c_int, [c_void_p]),
    'a3c_hostenv_begin': (c_int, [c_void_p, c_void_p]),
    'a3c_hostenv_step': (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    'a3c_engine_ext_act': (c_int, [c_void_p, c_void_p, c_void_p]),
    'a3c_engine_ext_observe': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    'a3c_engine_ext_upload': (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p]),
    'a3c_hostenv_step_range': (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int]),
    'a3c_dev_alloc': (c_int, [c_i64, ctypes.POINTER(c_void_p)]),
    'a3c_dev_alloc_kind': (c_int, [c_i64, c_int, ctypes.POINTER(c_void_p)]),
    'a3c_dev_free': (c_int, [c_void_p]),
    'a3c_ipc_handle': (c_int, [c_void_p, c_void_p]),
    'a3c_ipc_open': (c_int, [c_void_p, ctypes.POINTER(c_void_p)]),
    'a3c_ipc_close': (c_int, [c_void_p]),
    'a3c_rmsprop_range': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_i64, c_void_p, c_float, c_float,
                                  c_float, c_float, c_void_p]),
    'a3c_engine_time_kernel': (c_int, [c_void_p, c_int, c_int, c_void_p, ctypes.POINTER(c_float)]),
}

# diagnostics an A/B build from an earlier commit may lack (every other symbol is required)
MEASUREMENT_ONLY = ('a3c_engine_span_steps', 'a3c_engine_span_raw')
# entry points an older build selected with A3C_LIB (A/B runs of earlier commits) may lack; any
# other missing symbol is an error, and each one skipped is named on stderr
OPTIONAL_IN_OLD_BUILDS = MEASUREMENT_ONLY + ('a3c_engine_exchange_split', 'a3c_engine_wait_grad_head',
                                             'a3c_dev_alloc_kind', 'a3c_engine_time_kernel', 'a3c_engine_set_step',
                                             'a3c_engine_stats_accumulate', 'a3c_engine_stats_read',
                                             'a3c_engine_state_bytes', 'a3c_engine_state_save',
                                             'a3c_engine_state_load')

KER_CONV12_FWD, KER_FC_FWD, KER_ENV_STEP, KER_CONV_BWD, KER_HEAD_SCREEN, KER_HEAD_SCREEN_CONV12, KER_FC_PART = 0, 1, 2, 3, 4, 5, 6
# nature trunk passes (include/a3c_hip.h A3C_KER_NAT_*)
KER_NAT = {'conv1_fwd': 7, 'conv2_fwd': 8, 'conv3_fwd': 9, 'fc_fwd': 10, 'conv3_dw': 11, 'conv3_dx': 12, 'conv2_dw': 13,
           'conv2_dx': 14, 'conv1_dw': 15}

_lib = None


def lib():
    """Load liba3c_hip.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f'{LIB_PATH} not built: run __graft_entry__.build() or make -C csrc')
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if not hasattr(L, name):
                if name in MEASUREMENT_ONLY:
                    continue
                if os.environ.get('A3C_LIB') and name in OPTIONAL_IN_OLD_BUILDS:
                    print(f'[a3c] {LIB_PATH} lacks {name} (older build): skipped', file=sys.stderr)
                    continue
                raise RuntimeError(f'{LIB_PATH} does not export {name}: rebuild it (make -C csrc)')
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


ERR_INVALID, ERR_STATE = 10001, 10002      # include/a3c_hip.h A3C_ERR_*; other codes are hipError_t


class A3CError(RuntimeError):
    """A failed C-ABI call; ``rc`` is its status (A3C_ERR_* or a hipError_t)."""

    def __init__(self, msg, rc):
        super().__init__(msg)
        self.rc = rc

    @property
    def device_fault(self):
        return self.rc not in (ERR_INVALID, ERR_STATE)


def check(rc, what=''):
    if rc != 0:
        msg = lib().a3c_last_error().decode(errors='replace')
        raise A3CError(f'{what} failed ({rc}): {msg}', rc)


def require_device():
    """Fail loudly (no CPU fallback) when the HIP path cannot run."""
    if not torch.cuda.is_available():
        raise RuntimeError('liba3c_hip requires a ROCm GPU (torch.cuda.is_available() is False)')
    if not lib().a3c_device_ok():
        raise RuntimeError('liba3c_hip is built for gfx950 (MI355X); no such device visible')


def ptr(t):
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def stream_handle(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def net_desc(action_size, algo='a3c', lstm=False, dqn_type='nips'):
    """lstm: the C5 LSTM head (a3c only; build-defined, the reference has no recurrent code);
    dqn_type: 'nips' (agent.py:226-251, network.py:43-52) or 'nature' (network.py:30-42, A3C heads)."""
    trunk = {'nips': A3C_TRUNK_NIPS, 'nature': A3C_TRUNK_NATURE}.get(str(dqn_type).lower())
    if trunk is None:
        raise ValueError('Wrong DQN type: %s' % dqn_type)                          # network.py:54
    return NetDesc(A3C_ALGO_A3C if algo == 'a3c' else A3C_ALGO_Q, trunk, int(action_size), 4, 84, 84,
                   A3C_LSTM_UNITS if lstm else 0)


def param_layout(desc):
    n = c_int()
    offs = (c_i64 * MAX_TENSORS)()
    sizes = (c_i64 * MAX_TENSORS)()
    total = c_i64()
    check(lib().a3c_param_layout(ctypes.byref(desc), ctypes.byref(n), offs, sizes, ctypes.byref(total)),
          'a3c_param_layout')
    return [int(offs[i]) for i in range(n.value)], [int(sizes[i]) for i in range(n.value)], int(total.value)


def z_stride(desc):
    return int(lib().a3c_z_stride(ctypes.byref(desc)))


def workspace_bytes(desc, B):
    b = c_i64()
    check(lib().a3c_workspace_bytes(ctypes.byref(desc), int(B), ctypes.byref(b)), 'a3c_workspace_bytes')
    return int(b.value)


def i64_array(vals):
    arr = (c_i64 * MAX_TENSORS)()
    for i, v in enumerate(vals):
        arr[i] = int(v)
    return arr

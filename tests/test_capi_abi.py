"""C-ABI checks that need no GPU: liba3c_hip.so loads, exports every function include/a3c_hip.h
declares, and the ctypes mirrors of the header's structs have the layout gcc gives them."""
import ctypes
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, 'include', 'a3c_hip.h')
SO = os.path.join(ROOT, 'async-rl-tensorflow_amd', 'lib', 'liba3c_hip.so')


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(a3c_[a-z0-9_]+)\s*\(', src)))


@pytest.fixture(scope='module')
def lib():
    if not os.path.exists(SO):
        pytest.skip('liba3c_hip.so not built (run __graft_entry__.build())')
    import torch  # noqa: F401  (share torch's HIP runtime, as the package does)
    return ctypes.CDLL(SO)


def test_header_declares_the_boundary():
    fns = declared_functions()
    for f in ('a3c_preprocess_u8', 'a3c_history_push', 'a3c_forward', 'a3c_select_action', 'a3c_returns',
              'a3c_td_target', 'a3c_loss_backward', 'a3c_clip_rmsprop_apply', 'a3c_copy_params',
              'a3c_engine_create', 'a3c_engine_rollout_grad', 'a3c_engine_apply', 'a3c_engine_iterate'):
        assert f in fns, f


def test_library_exports_every_declared_symbol(lib):
    missing = [f for f in declared_functions() if not hasattr(lib, f)]
    assert not missing, missing


def test_ctypes_bindings_cover_the_header():
    sys.path.insert(0, os.path.join(ROOT, 'async-rl-tensorflow_amd'))
    from src import _lib
    missing = [f for f in declared_functions() if f not in _lib.SIGNATURES]
    assert not missing, missing


def test_version_and_layout_without_gpu(lib):
    lib.a3c_version.restype = ctypes.c_char_p
    assert b'gfx950' in lib.a3c_version()
    sys.path.insert(0, os.path.join(ROOT, 'async-rl-tensorflow_amd'))
    from src import _lib
    offs, sizes, total = _lib.param_layout(_lib.net_desc(6, 'a3c'))
    assert sizes == [4096, 16, 8192, 32, 663552, 256, 1536, 6, 256, 1]
    assert sum(sizes) == 677943 and all(o % 64 == 0 for o in offs)
    offs, sizes, total = _lib.param_layout(_lib.net_desc(6, 'q'))
    assert sum(sizes) == 677686                         # 676,144 + 257*A
    assert _lib.z_stride(_lib.net_desc(6, 'a3c')) == 8
    # invalid descriptions are rejected with a status code, not a crash
    bad = _lib.net_desc(6, 'a3c')
    bad.trunk = 7
    assert lib.a3c_param_layout(ctypes.byref(bad), None, None, None, None) != 0


C_PROBE = r'''
#include <stdio.h>
#include <stddef.h>
#include "a3c_hip.h"
#define F(T, m) printf(#T "." #m " %zu\n", offsetof(T, m));
int main(void) {
  printf("a3c_net_desc %zu\n", sizeof(a3c_net_desc));
  printf("a3c_engine_config %zu\n", sizeof(a3c_engine_config));
  printf("a3c_engine_buffers %zu\n", sizeof(a3c_engine_buffers));
  F(a3c_engine_config, seed) F(a3c_engine_config, gamma) F(a3c_engine_config, max_step)
  F(a3c_engine_config, clip_norm) F(a3c_engine_config, ep_end_t) F(a3c_engine_config, discount) F(a3c_engine_config, overlap)
  F(a3c_engine_buffers, n_params) F(a3c_engine_buffers, ring_slots) F(a3c_engine_buffers, zs)
  F(a3c_engine_buffers, offsets) F(a3c_engine_buffers, sizes) F(a3c_engine_buffers, sched)
  return 0;
}
'''


def test_struct_layout_matches_gcc(tmp_path):
    src = tmp_path / 'probe.c'
    src.write_text(C_PROBE)
    exe = tmp_path / 'probe'
    subprocess.run(['gcc', '-std=c99', '-I', os.path.dirname(HEADER), str(src), '-o', str(exe)], check=True)
    got = dict(line.rsplit(' ', 1) for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                              check=True).stdout.splitlines())
    sys.path.insert(0, os.path.join(ROOT, 'async-rl-tensorflow_amd'))
    from src import _lib
    assert int(got['a3c_net_desc']) == ctypes.sizeof(_lib.NetDesc)
    assert int(got['a3c_engine_config']) == ctypes.sizeof(_lib.EngineConfig)
    assert int(got['a3c_engine_buffers']) == ctypes.sizeof(_lib.EngineBuffers)
    for key, val in got.items():
        if '.' in key:
            st, field = key.split('.')
            cls = {'a3c_engine_config': _lib.EngineConfig, 'a3c_engine_buffers': _lib.EngineBuffers}[st]
            assert getattr(cls, field).offset == int(val), key

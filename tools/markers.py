"""Unprofiled iteration timeline from the marker build (-DA3C_MARKERS): rollout start (0) / end (1),
backward start (2), apply end (3), s_memrealtime (100 MHz).  Per iteration (anchored at each
rollout start) prints the mean offsets of the other marks and the rollout / backward spans.
A3C_LIB=<marker build> python3 tools/markers.py [overlap|sync] [m2] [eager]"""
import ctypes
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'async-rl-tensorflow_amd'))
import numpy as np
import torch
from src import _lib
from src.engine import Engine
from src.initializers import init_params, flatten_host
from src.kernels import param_names_shapes

mode = sys.argv[1] if len(sys.argv) > 1 else 'overlap'
L = _lib.lib()
L.a3c_debug_marks.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = np.zeros(2 + 2 * 8192, dtype=np.uint64)
eng = Engine(num_envs=256, n_step=5, action_size=6, num_frames=16384, seed=123, overlap=mode == 'overlap',
             frame84=int('m2' in sys.argv[2:]), use_graph='eager' not in sys.argv[2:])
ns = param_names_shapes(6, 'a3c')
eng.reset(flatten_host(ns, eng.offsets, eng.params.numel(), init_params(ns, seed=123)))
for _ in range(20):
    eng.iterate()
L.a3c_debug_marks(buf.ctypes.data, 1)
N = 200
for _ in range(N):
    eng.iterate()
L.a3c_debug_marks(buf.ctypes.data, 0)
n = int(buf[0])
ev = buf[2:2 + 2 * n].reshape(-1, 2).astype(np.int64)
ev = ev[np.argsort(ev[:, 1], kind='stable')]
t0s = ev[ev[:, 0] == 0, 1]
rows = []
for a, b in zip(t0s[5:-2], t0s[6:-1]):
    seg = ev[(ev[:, 1] >= a) & (ev[:, 1] < b)]
    r = {'len': (b - a) / 100.0}
    for k in (1, 2, 3, 4, 5):
        s = seg[seg[:, 0] == k, 1]
        r[k] = (s[0] - a) / 100.0 if len(s) else np.nan
    rows.append(r)
lens = np.array([r['len'] for r in rows])
print('%s: %d iterations, mean %.1f us (min %.1f, max %.1f)' % (mode, len(rows), lens.mean(), lens.min(), lens.max()))
for k, nm in ((1, 'rollout end'), (2, 'backward start'), (4, 'conv bwd start'), (5, 'conv bwd end'), (3, 'apply end')):
    v = np.array([r[k] for r in rows])
    print('  %-15s at %7.1f us (median %.1f)' % (nm, np.nanmean(v), np.nanmedian(v)))
# raw marks of three iterations (id, us from the first rollout start shown)
a = t0s[len(t0s) // 2]
seg = ev[(ev[:, 1] >= a - 30000) & (ev[:, 1] < a + 3 * 30000)]
print('raw:', ' '.join('%d@%.1f' % (i, (t - a) / 100.0) for i, t in seg[:40]))

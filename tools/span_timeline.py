"""Unperturbed overlap-pipeline timeline from the kernels' own launch-span records (no marker
kernels): per iteration, the start / end of each fused rollout step (k_head_screen_conv12) and of
the concurrent backward's k_conv_bwd, relative to step 0's start, averaged over the last
iterations.  A3C_LIB selects a build.   python tools/span_timeline.py [iters] [extra engine kw]"""
import ctypes
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path[:0] = [ROOT, os.path.join(ROOT, 'async-rl-tensorflow_amd')]
import numpy as np
import torch
from src import _lib
from src.engine import Engine
from src.initializers import init_params, flatten_host
from src.kernels import param_names_shapes

K = int(sys.argv[1]) if len(sys.argv) > 1 else 300
n, E = 5, int(os.environ.get('TL_E', 256))
eng = Engine(num_envs=E, n_step=n, action_size=6, algo='a3c', start_lives=0, num_frames=16384, seed=123,
             overlap=True)
ns = param_names_shapes(6, 'a3c')
eng.reset(flatten_host(ns, eng.offsets, eng.params.numel(), init_params(ns, seed=123)))
for _ in range(20):
    eng.iterate()
torch.cuda.synchronize()
eng.span_stats(0, reset=True)
eng.span_stats(1, reset=True)
for _ in range(K):
    eng.iterate()
torch.cuda.synchronize()
L = _lib.lib()
raw = {}
tau = ctypes.c_int64()
for w in (0, 1):
    buf = np.zeros(2 * 1024, dtype=np.uint64)
    rc = L.a3c_engine_span_raw(eng._h, w, buf.ctypes.data, ctypes.byref(tau))
    assert rc == 0, _lib.lib().a3c_last_error()
    raw[w] = buf.reshape(1024, 2).astype(np.int64)
T_last = tau.value - n          # the last rollout's tau (its bootstrap head advanced the counter)
rows = []
for i in range(1, min(150, K - 2)):
    T = T_last - i * n
    st = [raw[1][(T + t + 1) % 1024] for t in range(n)]
    cb = raw[0][((T - n) // n) % 1024]      # the backward of the previous rollout runs beside it
    nxt = raw[1][(T + n + 1) % 1024]         # next rollout's step 0
    if any(s[0] == 0 for s in st) or nxt[0] == 0:
        continue
    t0 = st[0][0]
    cbv = [(cb[0] - t0) / 100.0, (cb[1] - t0) / 100.0] if cb[0] else [np.nan, np.nan]
    rows.append([v for s in st for v in ((s[0] - t0) / 100.0, (s[1] - t0) / 100.0)] +
                cbv + [(nxt[0] - t0) / 100.0])
a = np.array(rows)
m = np.nanmedian(a, axis=0)
out = {'iterations': len(rows),
       'steps_us': [[round(m[2 * t], 1), round(m[2 * t + 1], 1)] for t in range(n)],
       'step_len_us': [round(m[2 * t + 1] - m[2 * t], 1) for t in range(n)],
       'conv_bwd_us': [round(m[2 * n], 1), round(m[2 * n + 1], 1)],
       'next_step0_us': round(m[2 * n + 2], 1)}
print(json.dumps(out))
eng.close()

"""Per-workgroup CU occupancy of the overlap pipeline from a -DA3C_WGLOG build
(async-rl-tensorflow_amd/lib/var/wglog): every instrumented kernel's workgroups log (start, end,
XCC, HW_ID), so for each launch of one iteration this prints its dispatch skew and span, and for
the rollout kernel's late workgroups what else held their CU when the launch began.
    A3C_LIB=.../var/wglog/liba3c_hip.so python tools/wglog.py [iters] [--frames84]"""
import ctypes
import json
import os
import sys
from collections import Counter, defaultdict

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path[:0] = [ROOT, os.path.join(ROOT, 'async-rl-tensorflow_amd')]
import numpy as np
import torch
from src import _lib
from src.engine import Engine
from src.initializers import init_params, flatten_host
from src.kernels import param_names_shapes

KIND = {1: 'rollout_step', 2: 'fc_part', 3: 'conv12_fwd', 4: 'head_fwd', 5: 'gemm', 6: 'conv_bwd',
        7: 'head_bwd', 8: 'fold', 9: 'apply', 10: 'prep_fwd'}
args = [a for a in sys.argv[1:] if not a.startswith('--')]
K = int(args[0]) if args else 3
f84 = '--frames84' in sys.argv
eng = Engine(num_envs=256, n_step=5, action_size=6, algo='a3c', start_lives=0, num_frames=16384, seed=123,
             overlap=True, frame84=f84)
ns = param_names_shapes(6, 'a3c')
eng.reset(flatten_host(ns, eng.offsets, eng.params.numel(), init_params(ns, seed=123)))
L = _lib.lib()
fn = L.a3c_debug_wglog
fn.restype = ctypes.c_int64
fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
for _ in range(30):
    eng.iterate()
torch.cuda.synchronize()
size = fn(None, 1, 1)
for _ in range(K):
    eng.iterate()
torch.cuda.synchronize()
KINDS, MAXWG, RING = 16, 4096, 16
raw = np.zeros(size // 8, dtype=np.uint64)
fn(raw.ctypes.data, 0, 1)
cnt = raw[2:2 + KINDS * MAXWG // 2].view(np.uint32).reshape(KINDS, MAXWG)
ent = raw[2 + KINDS * MAXWG // 2:].reshape(KINDS, MAXWG, RING, 3)
kind_l, t0_l, t1_l, meta_l, seq_l = [], [], [], [], []
for k in range(KINDS):
    for b in np.nonzero(cnt[k])[0]:
        c = int(cnt[k][b])
        for q in range(max(0, c - RING), c):
            r = ent[k][b][q % RING]
            kind_l.append(k); t0_l.append(int(r[0])); t1_l.append(int(r[1])); meta_l.append(int(r[2]))
            seq_l.append(q)
kind = np.array(kind_l)
t0 = np.array(t0_l, dtype=np.int64)
t1 = np.array(t1_l, dtype=np.int64)
meta = np.array(meta_l, dtype=np.int64)
seq = np.array(seq_l)
n = len(kind)
xcc = (meta >> 32) & 15
hw = meta & 0xffffffff
cu = xcc * 256 + ((hw >> 8) & 0xff)          # CU_ID [11:8], SH_ID [12], SE_ID [15:13] within the XCC
base = t0.min()
t0 = (t0 - base) / 100.0
t1 = (t1 - base) / 100.0

# launches: per kind, consecutive workgroups whose spans overlap belong to one launch
launches = []
for k in sorted(set(kind)):
    idx = np.where(kind == k)[0]
    idx = idx[np.argsort(t0[idx])]
    cur, end = [], -1e18
    for i in idx:
        if cur and t0[i] > end:
            launches.append((k, cur))
            cur, end = [], -1e18
        cur.append(i)
        end = max(end, t1[i])
    if cur:
        launches.append((k, cur))
launches.sort(key=lambda kl: t0[kl[1]].min())

# one iteration: from the last-but-one conv12_fwd (rollout start) to the last one
starts = [t0[ix].min() for k, ix in launches if k == 3]
lo, hi = (starts[-2], starts[-1]) if len(starts) >= 2 else (0.0, 1e18)
rows = []
for k, ix in launches:
    ix = np.array(ix)
    s0 = t0[ix].min()
    if s0 < lo - 60 or s0 >= hi:
        continue
    per_cu = Counter(cu[ix])
    row = {'kernel': KIND.get(k, k), 'wgs': len(ix), 'start': round(s0 - lo, 1),
           'last_start': round(t0[ix].max() - lo, 1), 'end': round(t1[ix].max() - lo, 1),
           'wg_us_med': round(float(np.median(t1[ix] - t0[ix])), 1), 'cus': len(per_cu),
           'max_per_cu': max(per_cu.values())}
    if k == 1:   # late rollout workgroups: what held their CU at the launch's first start
        late = ix[t0[ix] > s0 + 2.0]
        held = Counter()
        for i in late:
            on = (cu == cu[i]) & (t0 < s0) & (t1 > s0) & (kind != 1)
            for kk in kind[on]:
                held[KIND.get(int(kk), kk)] += 1
        row['late_wgs'] = int(len(late))
        row['late_cu_held_by'] = dict(held)
    rows.append(row)
# co-residency extremes over the whole log
conc = defaultdict(int)
for k in (1, 6):
    ix = np.where(kind == k)[0]
    worst = 0
    for c in set(cu[ix]):
        iv = sorted((t0[i], t1[i]) for i in ix if cu[i] == c)
        ev = sorted([(a, 1) for a, b in iv] + [(b, -1) for a, b in iv])
        m = x = 0
        for _, d in ev:
            x += d
            m = max(m, x)
        worst = max(worst, m)
    conc[KIND[k]] = worst
print(json.dumps({'entries': int(n), 'iteration_us': round(hi - lo, 1), 'distinct_cus': int(len(set(cu))),
                  'max_concurrent_per_cu': conc}))
for r in rows:
    print(json.dumps(r))
eng.close()

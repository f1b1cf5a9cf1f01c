"""Diagnostic (not collected by pytest): localise engine ring mismatches vs the oracle."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'async-rl-tensorflow_amd')]

from oracle import ref_cpu as R  # noqa: E402
from oracle.synthetic_env import pool_frame  # noqa: E402
from src.engine import Engine  # noqa: E402
from src import kernels as K  # noqa: E402

E, n = 8, 5
eng = Engine(num_envs=E, n_step=n, action_size=6, num_frames=48, seed=131)
eng.reset(np.zeros(eng.params.numel(), np.float32))
torch.cuda.synchronize()
pool = eng.frame_pool.cpu().numpy()
bad_pool = [f for f in range(48) if not np.array_equal(pool[f], pool_frame(131, f))]
print('pool frames differing from oracle:', bad_pool[:10], len(bad_pool))
frames = eng.env_frame.cpu().numpy()
print('env frames', frames)
ring = eng.frame_ring.cpu().numpy()
scr_dev = K.preprocess(eng.frame_pool, frame_idx=torch.as_tensor(frames).cuda()).cpu().numpy()
for e in range(E):
    ref = R.screen(pool_frame(131, int(frames[e])))
    for c in range(4):
        d = ring[e, c] != ref
        if d.any():
            ys, xs = np.nonzero(d)
            print(f'env {e} slot {c}: {d.sum()} px differ, rows {ys.min()}..{ys.max()} cols {xs.min()}..{xs.max()}')
    print(f'env {e}: kernels.preprocess == oracle: {np.array_equal(scr_dev[e], ref)}; ring slot0 == preprocess: '
          f'{np.array_equal(ring[e, 0], scr_dev[e])}')

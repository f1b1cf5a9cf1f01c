"""PCIe H2D ceiling for the external-env path: pinned host -> HBM copy rate of one rollout step's
raw frames (E x 210x160x3 u8), whole and in chunks, on one stream (HIP events)."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'async-rl-tensorflow_amd')]

E = int(sys.argv[1]) if len(sys.argv) > 1 else 256
nbytes = E * 210 * 160 * 3
src = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
dst = torch.empty(nbytes, dtype=torch.uint8, device='cuda')
out = {}
for chunks in (1, 2, 8):
    cut = [nbytes * c // chunks for c in range(chunks + 1)]
    for _ in range(3):
        for a, b in zip(cut[:-1], cut[1:]):
            dst[a:b].copy_(src[a:b], non_blocking=True)
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 50
    t0.record()
    for _ in range(reps):
        for a, b in zip(cut[:-1], cut[1:]):
            dst[a:b].copy_(src[a:b], non_blocking=True)
    t1.record()
    torch.cuda.synchronize()
    ms = t0.elapsed_time(t1) / reps
    out[f'chunks{chunks}'] = {'ms_per_step_frames': round(ms, 4), 'GB_per_s': round(nbytes / ms / 1e6, 2)}
# host side alone: one step of E synthetic envs (a3c_hostenv, 16 threads) into the pinned buffer
from src.host_env import SyntheticHostEnvPool  # noqa: E402
pool = SyntheticHostEnvPool(E, 6, 0, num_frames=2048, seed=123, threads=16)
pool.begin()
acts = np.zeros(E, np.int32)
for _ in range(5):
    pool.step(acts)
t = time.perf_counter()
for _ in range(50):
    pool.step(acts)
out['host_step_ms'] = round((time.perf_counter() - t) / 50 * 1e3, 4)
pool.close()
print(json.dumps({'bytes_per_step': nbytes, 'envs': E, **out}))

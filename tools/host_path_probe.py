"""Where a rollout step of the external-env path (Engine.iterate_host) spends its wall time:
ext_act + stream sync (GPU forward, action D2H, and the tail of the previous step's H2D copy and
screen kernel), host stepping of each env range + its upload enqueue, observe enqueue."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'async-rl-tensorflow_amd')]
from src.engine import Engine  # noqa: E402
from src.host_env import SyntheticHostEnvPool  # noqa: E402

E, n, A = 256, 5, 6
chunks = int(sys.argv[1]) if len(sys.argv) > 1 else 2
eng = Engine(num_envs=E, n_step=n, action_size=A, start_lives=5, num_frames=1, seed=123, external_env=True)
eng.reset()
pool = SyntheticHostEnvPool(E, A, 5, num_frames=2048, seed=123, threads=16, upload_chunks=chunks)
for _ in range(5):
    eng.iterate_host(pool)
torch.cuda.synchronize()
acts = eng._ext_actions
stream = torch.cuda.current_stream()
bounds = [E * c // chunks for c in range(chunks + 1)]
acc = {'act_sync': 0.0, 'step_upload': 0.0, 'observe': 0.0, 'grad_apply_enqueue': 0.0}
iters = 100
t_all = time.perf_counter()
for _ in range(iters):
    for _ in range(n):
        t0 = time.perf_counter()
        eng.ext_act(acts)
        stream.synchronize()
        t1 = time.perf_counter()
        a = acts.numpy()
        for lo, hi in zip(bounds[:-1], bounds[1:]):
            pool.step_range(a, lo, hi)
            eng.ext_upload(pool.rgb, lo, hi)
        t2 = time.perf_counter()
        eng.ext_observe(None, pool.rewards, pool.terminals)
        t3 = time.perf_counter()
        acc['act_sync'] += t1 - t0
        acc['step_upload'] += t2 - t1
        acc['observe'] += t3 - t2
    t4 = time.perf_counter()
    eng.rollout_grad()
    eng.apply()
    acc['grad_apply_enqueue'] += time.perf_counter() - t4
torch.cuda.synchronize()
total = time.perf_counter() - t_all
out = {k: round(v / iters * 1e3, 4) for k, v in acc.items()}
out.update(chunks=chunks, ms_per_iteration=round(total / iters * 1e3, 4),
           env_steps_per_s=round(E * n * iters / total, 1))
print(json.dumps(out))

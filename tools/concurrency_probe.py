#!/usr/bin/env python3
"""Does the GPU overlap two independent engine iterations launched on two streams?
Prints env-steps/s for one engine alone and for two engines on two streams (graph mode)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'async-rl-tensorflow_amd')]
import torch  # noqa: E402
from src.engine import Engine  # noqa: E402


def run(engs, streams, iters=200):
    for _ in range(10):
        for e, s in zip(engs, streams):
            with torch.cuda.stream(s):
                e.iterate()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        for e, s in zip(engs, streams):
            with torch.cuda.stream(s):
                e.iterate()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return sum(e.E * e.n for e in engs) * iters / dt, dt / iters * 1e3


E = int(os.environ.get('E', '256'))
e1 = Engine(num_envs=E, n_step=5, action_size=6, num_frames=4096, seed=1)
e2 = Engine(num_envs=E, n_step=5, action_size=6, num_frames=4096, seed=2, env_id_base=E)
for e in (e1, e2):
    e.reset()
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
print('one engine     : %.0f env-steps/s  %.3f ms/iter' % run([e1], [s1]))
print('two engines/2s : %.0f env-steps/s  %.3f ms/iter(pair)' % run([e1, e2], [s1, s2]))
print('two engines/1s : %.0f env-steps/s  %.3f ms/iter(pair)' % run([e1, e2], [s1, s1]))

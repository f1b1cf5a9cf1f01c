"""Host enqueue cost vs device time per engine iteration: if the loop's enqueue time (before the
final synchronize) approaches the total, the GPU is starved by the host."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'async-rl-tensorflow_amd')]
import torch
from src.engine import Engine
for ov, ug in ((True, True), (False, True)):
    e = Engine(num_envs=256, n_step=5, action_size=6, num_frames=16384, overlap=ov, use_graph=ug)
    e.reset()
    torch.cuda.synchronize()
    for _ in range(10):
        e.iterate()
    torch.cuda.synchronize()
    for N in (20, 200):
        t0 = time.perf_counter()
        for _ in range(N):
            e.iterate()
        tm = time.perf_counter()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        print('overlap', ov, 'graph', ug, 'N', N, 'enqueue %.1f us/iter, total %.1f us/iter  %.0f env-steps/s'
              % ((tm - t0) / N * 1e6, (t1 - t0) / N * 1e6, 1280 * N / (t1 - t0)))
    e.close()

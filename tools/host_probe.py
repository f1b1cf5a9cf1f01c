import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'async-rl-tensorflow_amd')]
import torch
from src.engine import Engine
for ov, ug in ((False, True), (True, True), (True, False), (False, False)):
    for side in (False,):
        e = Engine(num_envs=256, n_step=5, action_size=6, num_frames=16384, overlap=ov, use_graph=ug)
        e.reset()
        st = torch.cuda.Stream() if side else torch.cuda.current_stream()
        torch.cuda.synchronize()
        with torch.cuda.stream(st):
            for _ in range(10):
                e.iterate()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(200):
                e.iterate()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
        print('overlap', ov, 'graph', ug, '%.1f us/iter  %.0f env-steps/s' % ((t1 - t0) / 200 * 1e6, 1280 * 200 / (t1 - t0)))
        e.close()

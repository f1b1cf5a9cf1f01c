"""Host enqueue cost vs device time per engine iteration: if the loop's enqueue time (before the
final synchronize) approaches the total, the GPU is starved by the host.  Eager and graph
launches, the fused single-GPU iterate and the split path a multi-GPU exchange takes
(rollout_grad, a stand-in exchange op on the gradient, apply)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'async-rl-tensorflow_amd')]
import torch
from src.engine import Engine
for ov in (True, False):
    for ug in (False, True):
        for split in (False, True):
            e = Engine(num_envs=256, n_step=5, action_size=6, num_frames=16384, overlap=ov, use_graph=ug)
            e.reset()

            def it():
                if not split:
                    e.iterate()
                    return
                e.rollout_grad()
                if e.grad_ready:
                    e.grads.mul_(1.0)          # stand-in for the exchange's collective on the gradient
                    e.apply()
            torch.cuda.synchronize()
            for _ in range(10):
                it()
            torch.cuda.synchronize()
            N = 200
            t0 = time.perf_counter()
            for _ in range(N):
                it()
            tm = time.perf_counter()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            print('overlap', ov, 'graph', ug, 'split', split, 'enqueue %.1f us/iter, total %.1f us/iter  %.0f env-steps/s'
                  % ((tm - t0) / N * 1e6, (t1 - t0) / N * 1e6, 1280 * N / (t1 - t0)), flush=True)
            e.close()

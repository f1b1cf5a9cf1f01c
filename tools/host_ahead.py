"""Is the host ahead of the GPU in the eager overlap pipeline?  Times each iterate() call on the
host (no synchronisation inside the timed loop) and the whole loop after a device sync.  If the
host only returns at the GPU's pace (per-call ~ iteration time) it is throttled by queue space;
per-call times well below the iteration time mean it runs ahead freely.

    python tools/host_ahead.py [iters]
"""
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path[:0] = [ROOT, os.path.join(ROOT, 'async-rl-tensorflow_amd')]
import numpy as np
import torch
from src.engine import Engine
from src.initializers import init_params, flatten_host
from src.kernels import param_names_shapes

K = int(sys.argv[1]) if len(sys.argv) > 1 else 400
eng = Engine(num_envs=256, n_step=5, action_size=6, algo='a3c', start_lives=0, num_frames=16384, seed=123,
             overlap=True)
ns = param_names_shapes(6, 'a3c')
eng.reset(flatten_host(ns, eng.offsets, eng.params.numel(), init_params(ns, seed=123)))
for _ in range(20):
    eng.iterate()
torch.cuda.synchronize()
out = {}
for rep in range(3):
    per = np.zeros(K)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        a = time.perf_counter()
        eng.iterate()
        per[i] = time.perf_counter() - a
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    out[f'rep{rep}'] = dict(host_loop_ms=round((t1 - t0) * 1e3, 3), total_ms=round((t2 - t0) * 1e3, 3),
                           gpu_us_per_iter=round((t2 - t0) / K * 1e6, 2),
                           host_us_per_call_p10_p50_p90=[round(float(np.percentile(per, q)) * 1e6, 1)
                                                         for q in (10, 50, 90)],
                           host_us_first10=[round(float(x) * 1e6, 1) for x in per[:10]])
print(json.dumps(out, indent=1))
eng.close()

"""Throughput probe for VERDICT r5 item 4 (two staggered env groups): can two 128-env overlap
pipelines, each on its own caller stream and its own rollout stream, outrun one 256-env
pipeline on one MI355X?  Two independent engines stand in for the two groups (each with its own
backward + apply of 640 rows instead of one shared backward of 1,280 -- so the probe is an upper
bound on the split's cost, not on its gain), started half an iteration apart.
    python tools/r6/two_groups_probe.py [seconds]"""
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..')
sys.path[:0] = [ROOT, os.path.join(ROOT, 'async-rl-tensorflow_amd')]
import torch  # noqa: E402
from src.engine import Engine  # noqa: E402
from src.initializers import init_params, flatten_host  # noqa: E402
from src.kernels import param_names_shapes  # noqa: E402

SECS = float(sys.argv[1]) if len(sys.argv) > 1 else 2.0
ns = param_names_shapes(6, 'a3c')


def make(E, base):
    e = Engine(num_envs=E, n_step=5, action_size=6, algo='a3c', start_lives=0, num_frames=16384, seed=123,
               env_id_base=base, overlap=True)
    e.reset(flatten_host(ns, e.offsets, e.params.numel(), init_params(ns, seed=123)))
    return e


def run(groups, stagger):
    engs = [make(E, base) for E, base in groups]
    streams = [torch.cuda.Stream() for _ in engs]
    for _ in range(10):
        for e, s in zip(engs, streams):
            with torch.cuda.stream(s):
                e.iterate()
    torch.cuda.synchronize()
    k = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < SECS or k < 20:
        for i, (e, s) in enumerate(zip(engs, streams)):
            with torch.cuda.stream(s):
                e.iterate()
            if stagger and i == 0 and k == 0:
                torch.cuda.synchronize()        # (first iteration only: offsets group B's start)
        k += 1
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    steps = sum(E for E, _ in groups) * 5 * k
    for e in engs:
        e.close()
    return dict(groups=[E for E, _ in groups], iters=k, us_per_iter=round(el / k * 1e6, 1),
                env_steps_per_s=round(steps / el, 1))


out = [run([(256, 0)], False), run([(128, 0)], False), run([(128, 0), (128, 128)], False),
       run([(128, 0), (128, 128)], True), run([(512, 0)], False), run([(256, 0), (256, 256)], False)]
for r in out:
    print(json.dumps(r), flush=True)

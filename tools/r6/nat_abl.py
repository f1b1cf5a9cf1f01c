"""Per-pass times of the nature trunk (a3c_engine_time_kernel) for the ablation builds of
tools/r6/nat_abl.sh (A3C_LIB selects the build).  Measurement only."""
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..')
sys.path[:0] = [ROOT, os.path.join(ROOT, 'async-rl-tensorflow_amd')]
import torch  # noqa: E402
from src import _lib  # noqa: E402
from src.engine import Engine  # noqa: E402
from src.initializers import init_params, flatten_host  # noqa: E402
from src.kernels import param_names_shapes  # noqa: E402

ns = param_names_shapes(6, 'a3c', dqn_type='nature')
eng = Engine(num_envs=256, n_step=5, action_size=6, num_frames=4096, seed=1, dqn_type='nature')
eng.reset(flatten_host(ns, eng.offsets, eng.params.numel(), init_params(ns, seed=1)))
for _ in range(3):
    eng.iterate()
torch.cuda.synchronize()
print(json.dumps({k: round(eng.time_kernel(v, 20) * 1e3, 1) for k, v in _lib.KER_NAT.items()}), flush=True)

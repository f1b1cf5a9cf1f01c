"""Isolated fc-forward time (a3c_engine_time_kernel KER_FC_FWD, engine buffers, 256 envs) of the
library A3C_LIB points at: python3 tools/fc_ab.py"""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'async-rl-tensorflow_amd'))
import torch
from src import _lib
from src.engine import Engine
from src.initializers import init_params, flatten_host
from src.kernels import param_names_shapes

kers = [int(k) for k in os.environ.get('AB_KERS', str(_lib.KER_FC_FWD)).split(',')]
overlap = bool(int(os.environ.get('AB_OVERLAP', '1')))
eng = Engine(num_envs=256, n_step=5, action_size=6, num_frames=4096, seed=123, overlap=overlap)
ns = param_names_shapes(6, 'a3c')
eng.reset(flatten_host(ns, eng.offsets, eng.params.numel(), init_params(ns, seed=123)))
for _ in range(4):
    eng.iterate()
torch.cuda.synchronize()
ref = eng.slot(0)['act_l3'][:256].clone()
out = []
for k in kers:
    ts = sorted(eng.time_kernel(k, 200) for _ in range(5))
    out.append('ker%d %.2f us (min %.2f)' % (k, 1e3 * ts[2], 1e3 * ts[0]))
print(os.environ.get('A3C_LIB', 'default'), ' '.join(out), flush=True)

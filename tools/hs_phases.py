"""Phase timestamps of one k_head_screen workgroup (debug build with -DHS_TIMES=<block>):
python3 tools/hs_phases.py  (A3C_LIB pointing at that build)."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'async-rl-tensorflow_amd'))
import torch
from src import _lib
from src.engine import Engine
from src.initializers import init_params, flatten_host
from src.kernels import param_names_shapes

E = int(os.environ.get('HS_E', 256))
eng = Engine(num_envs=E, n_step=5, action_size=6, algo='a3c', start_lives=0, num_frames=16384, seed=123,
             env_id_base=0, world_size=1, use_graph=True, overlap=bool(int(os.environ.get('HS_OVERLAP', '0'))))
ns = param_names_shapes(6, 'a3c')
eng.reset(flatten_host(ns, eng.offsets, eng.params.numel(), init_params(ns, seed=123)))
for _ in range(3):
    eng.iterate()
torch.cuda.synchronize()
KER = int(os.environ.get('HS_KER', _lib.KER_HEAD_SCREEN))   # 5: the fused head+screen+conv kernel
names = ['start', 'head_row', 'head_act', 'barrier1', 'first_load', 'lum_done', 'barrier2', 'hpass', 'vpass']
if KER == _lib.KER_HEAD_SCREEN_CONV12:
    names += ['(screen end)', 'conv_done', 'c1_start', 'c1_w0_done', 'c1_all_done', 'mid_start', 'mid_end', 'w2_loads_done', 'w1_env_done']
for rep in range(3):
    eng.time_kernel(KER, 1)
    torch.cuda.synchronize()
    z = eng.slot(0)['z'].reshape(-1)[:2 * len(names)].clone().view(torch.int64).cpu().tolist()
    t0 = z[0]
    print(' '.join('%s=%d' % (n, z[i] - t0) for i, n in enumerate(names)))

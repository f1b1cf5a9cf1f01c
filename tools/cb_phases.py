"""Per-phase time of k_conv_bwd (debug build with -DCB_PHASES:
make -C async-rl-tensorflow_amd/csrc OUT=../lib/var/cbp/liba3c_hip.so OBJDIR=../lib/var/cbp/obj EXTRA=-DCB_PHASES;
run with A3C_LIB pointing at it).  Wave 0 of every workgroup sums its phases over its samples
(s_memrealtime, 100 MHz): staging, (a) dW2, (b) dl1, dl1 bf16 split, (c) dW1, and the whole
workgroup; printed as the mean over workgroups in microseconds."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'async-rl-tensorflow_amd'))
import numpy as np
import torch
from src import _lib
from src.engine import Engine
from src.initializers import init_params, flatten_host
from src.kernels import param_names_shapes

NAMES = ['stage', 'a_dW2', 'b_dl1', 'split', 'c_dW1', 'total']
E = int(os.environ.get('CBP_E', 256))
for overlap in (False, True):
    eng = Engine(num_envs=E, n_step=5, action_size=6, algo='a3c', start_lives=0, num_frames=16384, seed=123,
                 env_id_base=0, world_size=1, use_graph=True, overlap=overlap)
    ns = param_names_shapes(6, 'a3c')
    eng.reset(flatten_host(ns, eng.offsets, eng.params.numel(), init_params(ns, seed=123)))
    for _ in range(4):
        eng.iterate()
    torch.cuda.synchronize()
    l1 = eng.slot(0)['act_l1']
    for rep in range(2):
        eng.time_kernel(_lib.KER_CONV_BWD, 1)
        torch.cuda.synchronize()
        a = l1.reshape(l1.shape[0], -1)[:, :12].contiguous().view(torch.int64).cpu().numpy()
        ok = (a >= 0).all(1) & (a < 10 ** 6).all(1) & (a[:, 5] > 0)
        a = a[ok] / 100.0
        print('overlap' if overlap else 'sync', f'wgs={len(a)}',
              ' '.join(f'{n}={v:.2f}' for n, v in zip(NAMES, a.mean(0))), f'total_max={a[:, 5].max():.2f}us')
    eng.close()

"""Per-workgroup start/end stamps of one launch of each hot engine kernel (debug build with
-DA3C_WG_TIMES: make -C async-rl-tensorflow_amd/csrc OUT=../lib/var/wgt/liba3c_hip.so
OBJDIR=../lib/var/wgt/obj EXTRA=-DA3C_WG_TIMES; run with A3C_LIB pointing at it).
Prints dispatch skew, per-workgroup duration and the launch span (s_memrealtime, 100 MHz)."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'async-rl-tensorflow_amd'))
import numpy as np
import torch
from src import _lib
from src.engine import Engine
from src.initializers import init_params, flatten_host
from src.kernels import param_names_shapes


def stamps(t):
    a = t.contiguous().view(torch.int64).cpu().numpy().reshape(-1, 2)
    ok = (a[:, 0] > 10 ** 8) & (a[:, 1] >= a[:, 0]) & (a[:, 1] - a[:, 0] < 10 ** 6)
    a = a[ok]
    if len(a) == 0:
        return a
    med = np.median(a[:, 0])
    return a[np.abs(a[:, 0] - med) < 10 ** 6]


def report(name, a):
    if len(a) == 0:
        print(f'{name:16s} no stamps')
        return
    t0 = a[:, 0].min()
    d = (a[:, 1] - a[:, 0]) / 100.0
    s = (a[:, 0] - t0) / 100.0
    print(f'{name:16s} wgs={len(a):4d} span={(a[:, 1].max() - t0) / 100:6.2f}us  start skew max={s.max():5.2f} '
          f'p50={np.median(s):5.2f}  dur mean={d.mean():6.2f} min={d.min():6.2f} p90={np.percentile(d, 90):6.2f} '
          f'max={d.max():6.2f}us')


for overlap in (False, True):
    E = int(os.environ.get('WGT_E', 256))
    eng = Engine(num_envs=E, n_step=5, action_size=6, algo='a3c', start_lives=0, num_frames=16384, seed=123,
                 env_id_base=0, world_size=1, use_graph=True, overlap=overlap)
    ns = param_names_shapes(6, 'a3c')
    eng.reset(flatten_host(ns, eng.offsets, eng.params.numel(), init_params(ns, seed=123)))
    for _ in range(4):
        eng.iterate()
    torch.cuda.synchronize()
    sl = eng.slot(0)
    print('overlap' if overlap else 'sync')
    for rep in range(2):
        eng.time_kernel(_lib.KER_CONV12_FWD, 1); torch.cuda.synchronize()
        report('conv12_fwd', stamps(sl['act_l2'][:E, :4]))
        eng.time_kernel(_lib.KER_FC_FWD, 1); torch.cuda.synchronize()
        report('fc_fwd', stamps(sl['act_l3'][:E].reshape(E // 16, 16, 16, 16)[:, 0, :, :4]))
        eng.time_kernel(_lib.KER_HEAD_SCREEN, 1); torch.cuda.synchronize()
        report('head_screen', stamps(sl['z'][0, :, :4]))
        eng.time_kernel(_lib.KER_CONV_BWD, 1); torch.cuda.synchronize()
        report('conv_bwd', stamps(sl['act_l1'][:, :4]))
    eng.close()

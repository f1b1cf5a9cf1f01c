"""Microbenchmark of K1 (Environment.screen) on a HBM-resident frame pool: band count sweep
(A3C_PRE_PARTS) vs a torch gather-copy of the same frames (achievable-bandwidth reference)."""
import os
import subprocess
import sys
import json

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'async-rl-tensorflow_amd')]


def run_one():
    import torch
    from src import kernels as K
    P, n = 16384, int(os.environ.get('NFR', '256'))
    pool = torch.randint(0, 256, (P, 210, 160, 3), dtype=torch.uint8, device='cuda')
    g = torch.Generator(device='cpu').manual_seed(0)
    idx = torch.randint(0, P, (n,), generator=g, dtype=torch.int32).cuda()
    out = torch.empty((n, 84, 84), dtype=torch.uint8, device='cuda')
    for _ in range(5):
        K.preprocess(pool, frame_idx=idx, out=out)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    it = 200
    s.record()
    for _ in range(it):
        K.preprocess(pool, frame_idx=idx, out=out)
    e.record()
    torch.cuda.synchronize()
    t_pre = s.elapsed_time(e) / it
    li = idx.long()
    dst = torch.empty((n, 210, 160, 3), dtype=torch.uint8, device='cuda')
    for _ in range(5):
        torch.index_select(pool, 0, li, out=dst)
    s.record()
    for _ in range(it):
        torch.index_select(pool, 0, li, out=dst)
    e.record()
    torch.cuda.synchronize()
    t_cp = s.elapsed_time(e) / it
    byts = n * (100800 + 7056)
    print(json.dumps(dict(rows=os.environ.get('A3C_PRE_ROWS', 'default'), n=n, pre_us=round(t_pre * 1e3, 2),
                          pre_GBs=round(byts / t_pre / 1e6, 1), gather_copy_us=round(t_cp * 1e3, 2),
                          copy_GBs=round(2 * n * 100800 / t_cp / 1e6, 1))), flush=True)


if __name__ == '__main__':
    if len(sys.argv) > 1 and sys.argv[1] == 'one':
        run_one()
    else:
        for parts in ['7', '12', '14', '21', '28', '42']:
            for nfr in ['256', '1024']:
                env = dict(os.environ, A3C_PRE_ROWS=parts, NFR=nfr)
                subprocess.run([sys.executable, __file__, 'one'], env=env, check=True, timeout=300)

"""CPU ps/worker restatement of the reference's distributed training (TEST INFRASTRUCTURE ONLY:
bench.py's cpu_baseline leg).

The reference (main.py:50-94) runs one parameter server holding the weights and the RMSProp
slots, plus W worker processes. Each worker repeatedly:
  * pulls the weights,
  * runs its rollout and its gradient,
  * clips the gradient per tensor (agent.py:316-319),
  * applies shared RMSProp on the PS without a lock (main.py:63-65, ``use_locking`` off).

Here the PS is a block of shared memory (params, ms, mom and the global step), and the workers
are processes that run oracle/engine_ref.py on their own env shard (env ids w*E ..). Each worker
snapshots the parameters at rollout start (theta' <- theta, network.py:96-107) and applies
its clipped gradient to the shared arrays in place, unlocked (Hogwild). numpy is pinned to one
thread per worker, so ``cores`` = W.

Workers are spawned processes. bench.py runs this leg before it initialises the GPU.
"""
import multiprocessing as mp
import os
import time

import numpy as np


def _names_shapes(A, algo, dqn_type='nips'):
    from . import ref_cpu as R
    return R.param_shapes(A, algo, dqn_type)


def _worker(wid, E, n, A, algo, lives, seed, seconds, shm_name, layout, start_evt, out_q, frame84=False,
            ready_q=None, dqn_type='nips'):
    os.environ['OMP_NUM_THREADS'] = '1'
    os.environ['OPENBLAS_NUM_THREADS'] = '1'
    os.environ['MKL_NUM_THREADS'] = '1'
    try:
        from threadpoolctl import threadpool_limits
        threadpool_limits(1)
    except Exception:   # pragma: no cover
        pass
    from multiprocessing import shared_memory
    from . import ref_cpu as R
    from .engine_ref import EngineRef
    shm = shared_memory.SharedMemory(name=shm_name)
    total = layout['total']
    buf = np.ndarray((3 * total + 2,), np.float32, buffer=shm.buf)
    P, MS, MOM = buf[:total], buf[total:2 * total], buf[2 * total:3 * total]

    def views(flat):
        return {k: flat[o:o + sz].reshape(shp) for k, (o, sz, shp) in layout['t'].items()}

    shared_p, shared_ms, shared_mom = views(P), views(MS), views(MOM)
    ref = EngineRef({k: v.copy() for k, v in shared_p.items()}, E, n, A, algo, lives, num_frames=16384,
                    seed=seed, env_id_base=wid * E, dtype=np.float32, frame84=frame84, dqn_type=dqn_type)
    ref.cache_screens = False
    ref.reset()
    if ready_q is not None:
        ready_q.put(wid)
    start_evt.wait()
    t0 = time.perf_counter()
    steps = 0
    iters = 0
    while time.perf_counter() - t0 < seconds:
        for k in ref.params:                           # theta' <- theta (pull from the PS)
            ref.params[k][...] = shared_p[k]
        out = ref.iterate()
        lr = ref.next_lr()                             # agent.py:393-395 at this worker's own step
        for k in shared_p:                             # unlocked shared RMSProp apply
            R.rmsprop_apply(shared_p[k], shared_ms[k], shared_mom[k], out['clipped'][k], lr,
                            ref.h['decay'], ref.h['momentum'], ref.h['epsilon'])
        ref.tau += n
        steps += E * n
        iters += 1
    el = time.perf_counter() - t0
    out_q.put((wid, steps, el, iters))
    shm.close()


def run(seconds=12.0, workers=1, envs_per_worker=8, n_step=5, action_size=6, algo='a3c', start_lives=0,
        seed=123, frame84=False, dqn_type='nips'):
    """Returns dict(value=env-steps/s over all workers, cores, iterations)."""
    from multiprocessing import shared_memory
    from . import ref_cpu as R
    ns = _names_shapes(action_size, algo, dqn_type)
    params = R.init_params(ns, seed=seed)
    layout = {'t': {}}
    off = 0
    for k, shp in ns:
        sz = int(np.prod(shp))
        layout['t'][k] = (off, sz, shp)
        off += sz
    layout['total'] = off
    shm = shared_memory.SharedMemory(create=True, size=(3 * off + 2) * 4)
    try:
        buf = np.ndarray((3 * off + 2,), np.float32, buffer=shm.buf)
        for k, shp in ns:
            o, sz, _ = layout['t'][k]
            buf[o:o + sz] = params[k].reshape(-1)
        buf[off:2 * off] = 1.0                         # TF1 rms slot init
        buf[2 * off:] = 0.0
        ctx = mp.get_context('spawn')
        start_evt = ctx.Event()
        out_q = ctx.Queue()
        ready_q = ctx.Queue()
        procs = [ctx.Process(target=_worker, args=(w, envs_per_worker, n_step, action_size, algo, start_lives,
                                                   seed, seconds, shm.name, layout, start_evt, out_q, frame84,
                                                   ready_q, dqn_type))
                 for w in range(workers)]
        for p in procs:
            p.start()
        for _ in procs:                # every worker built and reset: all start their clocks together
            ready_q.get(timeout=600)
        start_evt.set()
        res = [out_q.get(timeout=seconds + 600) for _ in procs]
        for p in procs:
            p.join(60)
        finite = bool(np.isfinite(buf[:off]).all())
    finally:
        shm.close()
        shm.unlink()
    steps = sum(r[1] for r in res)
    el = max(r[2] for r in res)
    return dict(value=steps / el, cores=workers, iterations=sum(r[3] for r in res), seconds=el, finite=finite)


if __name__ == '__main__':   # pragma: no cover
    import sys
    w = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    print(run(seconds=float(sys.argv[2]) if len(sys.argv) > 2 else 5.0, workers=w))

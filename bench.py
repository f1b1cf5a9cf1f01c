#!/usr/bin/env python3
"""Headline benchmark: env-steps/s of the A3C rollout + gradient path (BASELINE.json metric).

One "step" = one engine iteration on every GPU: E envs x n rollout steps (forward, categorical
draw, synthetic Atari step, Environment.screen preprocessing into the frame ring), bootstrap
forward, n-step returns, loss + backward, per-tensor clip, the RMSProp apply and, for N > 1, the
multi-GPU exchange: by default the partitioned parameter server (src/distributed.py PartitionedPS:
RCCL all-to-all of the per-worker-clipped gradients, each owned range stepped once per worker in
rank order, RCCL all-gather); `--exchange sum` is the plain SUM all-reduce baseline and
`--update hogwild` the collective-free IPC parameter server.  Inputs (the HBM-resident RGB frame
pool) are on the device before the timed region.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Rank 0 prints ONE JSON line (value = all GPUs' env-steps / max-over-ranks wall time), with the
dominant kernel's roofline (live in-graph launch spans, plus HIP-event timing of that kernel alone
on its live buffers) and the CPU baseline: oracle/ps_worker.py, the reference's ps/worker
algorithm restated in numpy (shared-memory PS, unlocked RMSProp workers) on host cores, bounded
sample.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'async-rl-tensorflow_amd'))
sys.path.insert(0, ROOT)

METRIC = json.load(open(os.path.join(ROOT, 'BASELINE.json')))['metric']
GAMES = {'Pong-v0': (6, 0), 'Breakout-v0': (4, 5), 'SpaceInvaders-v0': (6, 3)}

# algorithmic work per unit (DESIGN.md "Roofline"): FLOP per sample / bytes per env-step
CONV12_FWD_FLOP = 2 * 400 * 16 * 256 + 2 * 81 * 32 * 256            # 4,603,904
CONV_BWD_FLOP = 2 * 81 * 32 * 256 * 2 + 2 * 400 * 16 * 256          # 5,931,008
FC_FWD_FLOP = 2 * 2592 * 256                                        # 1,327,104
ENV_STEP_BYTES = 210 * 160 * 3 + 84 * 84                            # 107,856
# nature trunk (network.py:30-42), algorithmic FLOP per sample of each pass (nature.hip): the
# forward passes run once per rollout step and for the bootstrap state, the backward ones once
NAT_FLOP = {'conv1_fwd': 2 * 400 * 32 * 256, 'conv2_fwd': 2 * 81 * 64 * 512, 'conv3_fwd': 2 * 49 * 64 * 576,
            'fc_fwd': 2 * 3136 * 512, 'conv3_dw': 2 * 49 * 64 * 576, 'conv3_dx': 2 * 49 * 64 * 576,
            'conv2_dw': 2 * 81 * 64 * 512, 'conv2_dx': 2 * 81 * 64 * 512, 'conv1_dw': 2 * 400 * 32 * 256}
ENV_STEP_BYTES_84 = 84 * 84 + 84 * 84                               # 14,112 (--frames84: copy)
PEAK_FP32_TFLOPS = 157.3    # MI355X_MICROARCH.md: FP32 matrix peak (spec)
PEAK_HBM_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8 TB/s (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=200)
    ap.add_argument('--warmup', type=int, default=10)
    ap.add_argument('--envs', type=int, default=256, help='envs per GPU (BASELINE config 2: 256)')
    ap.add_argument('--n-step', type=int, default=5)
    ap.add_argument('--game', default='Pong-v0', choices=sorted(GAMES))
    ap.add_argument('--algo', default='a3c', choices=['a3c', 'q'])
    ap.add_argument('--env', default='device', choices=['device', 'host'],
                    help='device: the synthetic emulator runs on the GPU next to the net (default, HBM-resident '
                         'inputs); host: it runs on host threads (a3c_hostenv, stand-in for real ALE workers) '
                         'and every step moves the raw RGB frames over PCIe (PCIe-inclusive rate)')
    ap.add_argument('--host-threads', type=int, default=16)
    ap.add_argument('--host-chunks', type=int, default=2,
                    help='--env host: env ranges per rollout step; the H2D copy of one overlaps stepping the next')
    ap.add_argument('--dqn-type', default='nips', choices=['nips', 'nature'],
                    help="the A3C Network's trunk (network.py:30-54): nips 16/32/256 (the default, agent.py's "
                         "Q-net trunk too) or nature 32/64/64/512 (A3C heads, feed-forward)")
    ap.add_argument('--lstm', action='store_true',
                    help='C5 LSTM policy head (BASELINE config 5: SpaceInvaders-v0, 256-cell LSTM after the fc)')
    ap.add_argument('--frames', type=int, default=16384, help='HBM frame pool (16384 = 1.65 GB > L3)')
    ap.add_argument('--frames84', action='store_true',
                    help='measurement mode M2 (SURVEY 8(d)): the pool holds pre-sized 84x84 grey frames, the env '
                         'step copies one into the history ring (no Environment.screen); default M1: raw RGB')
    ap.add_argument('--graph', action='store_true',
                    help='capture each iteration into hipGraphs (default: eager launches, faster on MI355X: '
                         'a graph end costs ~13 us before the next packet on its stream)')
    ap.add_argument('--no-graph', action='store_true', help='(the default; kept for older command lines)')
    ap.add_argument('--update', default='overlap', choices=['overlap', 'sync', 'hogwild'],
                    help='overlap: rollout k overlaps backward+apply of rollout k-1 (stale-1 async A3C); '
                         'sync: rollout -> backward -> all-reduce -> apply; hogwild: unlocked pushes into a '
                         'sharded IPC parameter server, no collective (BASELINE config 4)')
    ap.add_argument('--hogwild-sync', action='store_true',
                    help='--update hogwild on a synchronous engine (push + pull after each rollout, no overlap); '
                         'default: the push of rollout k-1 and the pull overlap rollout k (staleness 1)')
    ap.add_argument('--hogwild-memory', default='fine', choices=['fine', 'coarse', 'uncached'],
                    help='--update hogwild: allocation kind of the IPC-shared shards (DESIGN §7 memory model)')
    ap.add_argument('--cpu-seconds', type=float, default=12.0)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--backend', default='nccl', choices=['nccl', 'gloo'],
                    help='process group backend for N > 1 (nccl = RCCL over xGMI; gloo only to rehearse the '
                         'multi-rank path with several ranks on one GPU)')
    ap.add_argument('--no-kernel-timing', action='store_true')
    ap.add_argument('--exchange', default='sequential', choices=['sequential', 'sum'],
                    help='N > 1 sync/overlap: sequential = partitioned PS (all-to-all, every worker\'s clipped '
                         'gradient its own RMSProp step in rank order, all-gather: the reference PS rule); '
                         'sum = one SUM all-reduce + one step (plain data parallel)')
    ap.add_argument('--min-seconds', type=float, default=2.0,
                    help='repeat the K-step timed window until at least this much time is measured (a short '
                         'K leaves a few ms of GPU time per window); value = median window rate, spread reported')
    ap.add_argument('--max-windows', type=int, default=100000,
                    help='upper bound on the window count (the default never binds before --min-seconds)')
    return ap.parse_args()


def host_cpu():
    """The box's host CPU as BASELINE.md asks it stated: model name, logical CPUs (nproc) and the
    CPUs this process may run on (a gpurun box gets a share of a larger host)."""
    model = None
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    model = line.split(':', 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        allowed = len(os.sched_getaffinity(0))
    except AttributeError:
        allowed = None
    quota = cgroup_cpu_quota()
    limit = min(x for x in (allowed, os.cpu_count(), quota['cpus'] if quota else None) if x)
    return dict(model=model, nproc=os.cpu_count(), affinity=allowed, cgroup=quota, cpu_limit=limit)


def cgroup_cpu_quota():
    """The CPU bandwidth limit of this process's cgroup, as CPUs (ceil(quota / period)), or None
    when unlimited: cgroup v2 `cpu.max`, else v1 `cpu.cfs_quota_us` / `cpu.cfs_period_us`."""
    import math
    rel = '/'
    try:
        with open('/proc/self/cgroup') as f:
            for line in f:
                parts = line.strip().split(':', 2)
                if len(parts) == 3 and (parts[0] == '0' or 'cpu' in parts[1].split(',')):
                    rel = parts[2]
                    if parts[0] == '0':
                        break
    except OSError:
        pass
    cands = [('/sys/fs/cgroup' + rel).rstrip('/') + '/cpu.max', '/sys/fs/cgroup/cpu.max']
    for path in cands:
        try:
            q, p = open(path).read().split()[:2]
        except (OSError, ValueError):
            continue
        if q == 'max':
            return dict(source=path, quota=None, period=int(p), cpus=None)
        return dict(source=path, quota=int(q), period=int(p), cpus=math.ceil(int(q) / int(p)))
    for base in (('/sys/fs/cgroup/cpu' + rel).rstrip('/'), '/sys/fs/cgroup/cpu', '/sys/fs/cgroup/cpu,cpuacct'):
        try:
            q = int(open(base + '/cpu.cfs_quota_us').read())
            p = int(open(base + '/cpu.cfs_period_us').read())
        except (OSError, ValueError):
            continue
        return dict(source=base, quota=None if q < 0 else q, period=p, cpus=None if q < 0 else math.ceil(q / p))
    return None


def cpu_baseline(seconds, game, algo, frame84=False, dqn_type='nips'):
    """The reference's ps/worker algorithm restated on the CPU (oracle/ps_worker.py: shared-memory
    PS, W worker processes with Hogwild RMSProp, one numpy thread each) on the same synthetic
    env: 1 ps / 1 worker (BASELINE config 1) and W = (the box's CPU limit) - 1 workers.  Runs
    before the GPU is initialised (the workers are spawned processes)."""
    from oracle import ps_worker
    A, lives = GAMES[game]
    n = 5 if algo == 'a3c' else 32
    host = host_cpu()
    # W = limit - 1 workers plus the PS process (nproc - 1 workers), where the limit is
    # the smallest of nproc, the affinity mask and the cgroup CPU quota -- the CPUs this process
    # can actually run on at once -- and of the pool's per-GPU CPU share: a gpurun box is one GPU's
    # share of a larger host (16 CPUs per GPU) that neither its affinity mask nor its cgroup states
    # (BENCH_CPU_SHARE overrides the per-GPU figure).  Every figure is recorded in host_cpu.
    import torch                        # device_count() does not initialise HIP on this image
    gpus = max(1, torch.cuda.device_count())
    per_gpu = int(os.environ.get('BENCH_CPU_SHARE', '16'))
    host['gpu_share'] = dict(visible_gpus=gpus, cpus_per_gpu=per_gpu, cpus=per_gpu * gpus)
    limit = min(host['cpu_limit'] or 2, per_gpu * gpus)
    W = max(1, limit - 1)
    host['limit_used'] = limit
    host['workers'] = W
    one = ps_worker.run(seconds=seconds / 2, workers=1, envs_per_worker=8, n_step=n, action_size=A, algo=algo,
                        start_lives=lives, frame84=frame84, dqn_type=dqn_type)
    many = ps_worker.run(seconds=seconds / 2, workers=W, envs_per_worker=8, n_step=n, action_size=A, algo=algo,
                         start_lives=lives, frame84=frame84, dqn_type=dqn_type) if W > 1 else one
    return dict(value=round(many['value'], 2), unit='env-steps/s', cores=W, kind='port',
                one_worker=round(one['value'], 2), host_cpu=host,
                sample=f'oracle/ps_worker.py ({algo} {dqn_type} ps/worker, shared-memory PS, unlocked RMSProp, numpy fp32, '
                       f'8 envs x n={n} per worker{", pre-sized 84x84 frames" if frame84 else ""}): {W} workers x {many["seconds"]:.1f} s = '
                       f'{many["iterations"]} iterations; 1 ps/1 worker: {one["value"]:.1f} env-steps/s')


CPU_FILE_ENV = 'BENCH_CPU_BASELINE_FILE'    # the spawning parent's CPU baseline, for rank 0's line


def spawn_ranks(args, cpu, cmd=None):
    """`bench.py --gpus N` (N > 1) started without a launcher: run N fresh child processes, one
    rank per GPU, with torch.distributed.run's environment contract (RANK, LOCAL_RANK, WORLD_SIZE,
    MASTER_ADDR=127.0.0.1, MASTER_PORT), the same arguments, and wait for them.  This parent never
    initialises the GPU (it only ran the CPU baseline, which rank 0 then puts in its line), so no
    process that touched the device is replaced or forked.  Reference: main.py:50-66 (one process
    per ps / worker task of the cluster).  cmd: the child command (default: this script with the
    same arguments; tests substitute a CPU-only child)."""
    import socket
    import subprocess
    import tempfile
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    fd, cpu_path = tempfile.mkstemp(prefix='bench_cpu_', suffix='.json')
    with os.fdopen(fd, 'w') as f:
        json.dump(cpu, f)
    procs = []
    try:
        for r in range(args.gpus):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                       LOCAL_WORLD_SIZE=str(args.gpus), GROUP_RANK='0', MASTER_ADDR='127.0.0.1',
                       MASTER_PORT=str(port), BENCH_LAUNCHER='bench.py spawn')
            env[CPU_FILE_ENV] = cpu_path
            procs.append(subprocess.Popen(cmd or [sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
        rc = 0
        pending = list(procs)
        while pending:                 # the first failing rank ends the job (as torch.distributed.run)
            for p in list(pending):
                code = p.poll()
                if code is None:
                    continue
                pending.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    for q in pending:
                        q.terminate()
            time.sleep(0.05)
        return rc
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        os.unlink(cpu_path)


def nature_roofline(eng, _lib, E, n, iter_ms, spans=None):
    """The nature trunk's passes (nature.hip), each timed alone with HIP events on the stream it is
    launched on (a3c_engine_time_kernel: forward passes over E states, backward passes over the
    last rollout's n E samples); the dominant one by time share of the iteration names the roofline
    (MFMA-bound: algorithmic FLOP per launch / its average launch duration, against the FP32 matrix
    peak).  The per-state conv kernel records its live launch spans over the timed region (spans:
    name -> (avg_us, max_us, launches)); when the roofline names it, the live average is its
    duration (as the rocprof trace sees it, beside the backward) and the isolated time is kept."""
    spans = spans or {}
    kernels = {}
    inside = []                        # passes that run inside conv2's launch (k_nat_conv23)
    for name, kid in _lib.KER_NAT.items():
        if name in ('conv1_fwd', 'conv3_fwd', 'conv2_dx'):
            try:
                ms = eng.time_kernel(kid, 10)
            except _lib.A3CError:
                inside.append(name)
                continue
        else:
            ms = eng.time_kernel(kid, 10)
        fwd = name.endswith('_fwd')
        B = E if fwd else n * E
        flop = NAT_FLOP[name] * B
        per_iter = n + 1 if fwd else 1
        kernels['nat_' + name] = dict(avg_ms=round(ms, 4), per_iter=per_iter, share=round(ms * per_iter / iter_ms, 3),
                                      bound='mfma', achieved=round(flop / (ms * 1e-3) / 1e12, 2), unit='TFLOP/s',
                                      flop_per_launch=flop)
    fin = [p for p in inside if p.endswith('_fwd')]
    if fin:                            # the conv2 launch is conv2 + conv3 (+ conv1) forward (k_nat_conv23)
        k = kernels.pop('nat_conv2_fwd')
        flop = sum(NAT_FLOP[p] for p in ['conv2_fwd'] + fin) * E
        key = 'nat_conv123_fwd' if 'conv1_fwd' in fin else 'nat_conv23_fwd'
        kernels[key] = dict(k, achieved=round(flop / (k['avg_ms'] * 1e-3) / 1e12, 2), flop_per_launch=flop)
    if 'conv2_dx' in inside:           # the conv3 dX launch is conv3 + conv2 dX (k_nat_dx32)
        k = kernels.pop('nat_conv3_dx')
        flop = (NAT_FLOP['conv3_dx'] + NAT_FLOP['conv2_dx']) * n * E
        kernels['nat_conv32_dx'] = dict(k, achieved=round(flop / (k['avg_ms'] * 1e-3) / 1e12, 2), flop_per_launch=flop)
    dom = max(kernels, key=lambda k: kernels[k]['avg_ms'] * kernels[k]['per_iter'])
    d = kernels[dom]
    traffic = None
    pmc = os.path.join(ROOT, 'profiles', 'pmc_hbm_bytes_nature.json')
    if os.path.exists(pmc):
        try:
            t = json.load(open(pmc))['hbm_bytes_per_launch'].get(dom)
            traffic = None if t is None else int(round(t))
        except Exception:
            traffic = None
    live = spans.get(dom)
    if live and live[2] > 0:
        d['live_avg_ms'] = round(live[0] * 1e-3, 4)
        d['live_launches'] = live[2]
        ach = round(d['flop_per_launch'] / (live[0] * 1e-6) / 1e12, 2)
        roofline = dict(kernel=dom, bound='mfma', achieved=ach, peak=PEAK_FP32_TFLOPS, unit='TFLOP/s',
                        frac=round(ach / PEAK_FP32_TFLOPS, 4), traffic=traffic,
                        timing='live: average in-graph launch span over the timed region (s_memrealtime, '
                               'a3c_engine_span_stats)',
                        avg_us=round(live[0], 2), isolated_us=round(d['avg_ms'] * 1e3, 2),
                        isolated_achieved=d['achieved'], isolated_frac=round(d['achieved'] / PEAK_FP32_TFLOPS, 4),
                        work_per_launch=d['flop_per_launch'], work_unit='FLOP')
        return roofline, kernels
    roofline = dict(kernel=dom, bound='mfma', achieved=d['achieved'], peak=PEAK_FP32_TFLOPS, unit='TFLOP/s',
                    frac=round(d['achieved'] / PEAK_FP32_TFLOPS, 4), traffic=traffic,
                    timing='isolated (HIP events on the launch stream, a3c_engine_time_kernel)',
                    avg_us=round(d['avg_ms'] * 1e3, 2), work_per_launch=d['flop_per_launch'], work_unit='FLOP')
    return roofline, kernels


def dist_record(args, torch, dist, local):
    """What the process group saw: backend, world size, launcher, every rank's device (index, name,
    PCI bus id) and the RCCL version torch was built against."""
    me = dict(rank=dist.get_rank(), local_rank=local, device=None, name='cpu', pci_bus_id=None, pci_device_id=None,
              hostname=os.uname().nodename)
    if torch.cuda.is_available():
        dev = torch.cuda.current_device()
        props = torch.cuda.get_device_properties(dev)
        me.update(device=dev, name=props.name, pci_bus_id=getattr(props, 'pci_bus_id', None),
                  pci_device_id=getattr(props, 'pci_device_id', None))
    ranks = [None] * dist.get_world_size()
    dist.all_gather_object(ranks, me)
    rccl = None
    try:
        v = torch.cuda.nccl.version()
        rccl = '.'.join(str(x) for x in v) if isinstance(v, tuple) else str(v)
    except Exception:           # gloo-only builds
        rccl = None
    return dict(backend=dist.get_backend(), world_size=dist.get_world_size(),
                launcher=os.environ.get('BENCH_LAUNCHER', 'torch.distributed.run'),
                rccl_version=rccl, ranks=ranks,
                distinct_devices=len({(r['hostname'], r['pci_bus_id'], r['device']) for r in ranks}))


def main():
    args = parse()
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world != args.gpus and world > 1:
        raise SystemExit(f'--gpus {args.gpus} but WORLD_SIZE={world}')
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        if os.environ.get(CPU_FILE_ENV):
            with open(os.environ[CPU_FILE_ENV]) as f:
                cpu = json.load(f)                  # measured by the spawning parent
        else:
            # rank 0, before any HIP initialisation (the workers are spawned processes); under a
            # launcher at N > 1 the other ranks wait in the rendezvous meanwhile
            cpu = cpu_baseline(args.cpu_seconds, args.game, args.algo, args.frames84, args.dqn_type)
    if world == 1 and args.gpus > 1:
        sys.exit(spawn_ranks(args, cpu))
    # stdout carries exactly the one JSON line: native libraries' chatter (gloo's connection
    # messages, runtime notices) goes to stderr
    sys.stdout.flush()
    line_out = os.fdopen(os.dup(1), 'w')
    os.dup2(2, 1)

    import numpy as np
    import torch
    import torch.distributed as dist
    ndev = torch.cuda.device_count()
    torch.cuda.set_device(local % max(ndev, 1))
    dist_rec = None
    if world > 1:
        if args.backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        else:
            dist.init_process_group('gloo')
        dist_rec = dist_record(args, torch, dist, local)

    from src import _lib
    from src.engine import Engine
    from src.initializers import init_params, flatten_host
    from src.kernels import param_names_shapes

    A, lives = GAMES[args.game]
    E, n = args.envs, args.n_step
    if args.lstm and args.algo != 'a3c':
        raise SystemExit('--lstm is an a3c head')
    nature = args.dqn_type == 'nature'
    if nature and (args.algo != 'a3c' or args.lstm or args.env != 'device'):
        raise SystemExit('--dqn-type nature: the A3C Network trunk (network.py:30-42) -- a3c, feed-forward head, '
                         'device envs')
    host = args.env == 'host'
    if host and args.update != 'sync':
        args.update = 'sync'              # host-stepped envs drive a synchronous engine
    if host and args.frames84:
        raise SystemExit('--frames84 is a device-env pool mode')
    eng = Engine(num_envs=E, n_step=n, action_size=A, algo=args.algo, start_lives=lives, num_frames=args.frames,
                 seed=123, env_id_base=rank * E, world_size=world, use_graph=args.graph and not args.no_graph,
                 overlap=args.update == 'overlap' or (args.update == 'hogwild' and not args.hogwild_sync),
                 lstm=args.lstm, external_env=host, frame84=int(args.frames84), dqn_type=args.dqn_type)
    hpool = None
    if host:
        from src.host_env import SyntheticHostEnvPool
        hpool = SyntheticHostEnvPool(E, A, lives, num_frames=min(args.frames, 2048), seed=123, env_id_base=rank * E,
                                     threads=args.host_threads, upload_chunks=args.host_chunks)
    ns = param_names_shapes(A, args.algo, lstm=args.lstm, dqn_type=args.dqn_type)
    params = flatten_host(ns, eng.offsets, eng.params.numel(), init_params(ns, seed=123))
    eng.reset(params)     # every rank starts from the same parameters
    torch.cuda.synchronize()

    ps = None
    if args.update == 'hogwild':
        from src.hogwild import HogwildPS
        ps = HogwildPS(eng.params, memory=args.hogwild_memory)

    def step():
        if hpool is not None:
            eng.iterate_host(hpool, exchange)
        elif ps is not None:
            eng.iterate_hogwild(ps)
        else:
            eng.iterate(exchange)

    exchange = None
    if world > 1 and args.update != 'hogwild':
        from src.distributed import GradExchange, PartitionedPS
        exchange = PartitionedPS(eng.params.numel()) if args.exchange == 'sequential' else GradExchange()

    def barrier():
        if world > 1:
            dist.barrier()

    def timed_window():
        # exactly K steps between a barrier + device sync on both sides; max over ranks
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        barrier()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device='cuda')
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    for _ in range(args.warmup):
        step()
    barrier()
    torch.cuda.synchronize()
    live = not host and not nature and (eng.overlap or args.update == 'sync')
    live_nat = nature and not host
    if live or live_nat:          # live launch spans of the dominant kernels, recorded in-graph
        eng.span_stats(0, reset=True)
        eng.span_stats(1, reset=True)
    # a short K-step window is a few ms of GPU time: repeat it until min_seconds are measured and
    # report the median window with the spread (every rank sees the same max-over-ranks window
    # times, so every rank stops at the same count)
    windows = [timed_window()]
    while sum(windows) < args.min_seconds and len(windows) < args.max_windows:
        windows.append(timed_window())
    el = float(np.median(windows))
    spans = {}
    if live_nat:                  # the nature trunk's per-state conv kernel (k_nat_conv23)
        spans['nat_conv123_fwd'] = eng.span_stats(1)
    if live:
        spans['k_conv_bwd'] = eng.span_stats(0)
        spans['k_head_screen_conv12'] = eng.span_stats(1)
        if eng.overlap and hasattr(_lib.lib(), 'a3c_engine_span_steps'):
            # per rollout step (the last step's launch also runs the bootstrap conv)
            spans['k_head_screen_conv12_by_step'] = eng.span_steps()
    loss = eng.loss.cpu().numpy().tolist()
    finite = bool(torch.isfinite(eng.params).all().item())

    roofline, kernels = None, {}
    if rank == 0 and not args.no_kernel_timing and nature:
        roofline, kernels = nature_roofline(eng, _lib, E, n, el / args.steps * 1e3, spans)
    elif rank == 0 and not args.no_kernel_timing and not host:
        # overlap mode fuses step t+1's conv1+conv2 into step t's head+screen kernel
        # (k_head_screen_conv12, engine.hip conv_fused): conv12 then runs once per rollout
        fused = eng.overlap and os.environ.get('A3C_FUSE_CONV', '1') != '0'
        step_bytes = ENV_STEP_BYTES_84 if args.frames84 else ENV_STEP_BYTES
        ms = {
            'k_conv12_fwd': eng.time_kernel(_lib.KER_CONV12_FWD, 20),
            'k_conv_bwd': eng.time_kernel(_lib.KER_CONV_BWD, 10),
            'k_fc_fwd': eng.time_kernel(_lib.KER_FC_FWD, 20),
        }
        count = {'k_conv12_fwd': 1 if fused else n + 1, 'k_conv_bwd': 1, 'k_fc_fwd': n + 1}
        work = {
            'k_conv12_fwd': ('mfma', CONV12_FWD_FLOP * E),
            'k_conv_bwd': ('mfma', CONV_BWD_FLOP * n * E),
            'k_fc_fwd': ('mfma', FC_FWD_FLOP * E),
        }
        if fused and os.environ.get('A3C_FC_SPLIT', '1') != '0' and not args.lstm:
            # every fc of the rollout (n steps + the bootstrap state) runs as K-slice partials
            # folded by the consuming head (k_fc_part): the single-pass k_fc_fwd is not launched
            ms['k_fc_part'] = eng.time_kernel(_lib.KER_FC_PART, 20)
            count['k_fc_part'] = n + 1
            work['k_fc_part'] = ('mfma', FC_FWD_FLOP * E)
            del ms['k_fc_fwd']
        if fused:
            ms['k_head_screen_conv12'] = eng.time_kernel(_lib.KER_HEAD_SCREEN_CONV12, 20)
            count['k_head_screen_conv12'] = n
            # two serial phases per workgroup: Environment.screen (HBM) then conv1+conv2 (MFMA);
            # roofline time = bytes / HBM peak + FLOP / FP32 MFMA peak
            work['k_head_screen_conv12'] = ('hbm+mfma', (step_bytes * E, CONV12_FWD_FLOP * E))
        else:
            ms['k_head_screen'] = eng.time_kernel(_lib.KER_HEAD_SCREEN, 20)
            count['k_head_screen'] = n
            work['k_head_screen'] = ('hbm', step_bytes * E)
        iter_ms = el / args.steps * 1e3
        # live = the average in-graph launch span over the timed region (contended in overlap
        # mode); avg_ms = the same kernel alone, back-to-back on the engine's buffers
        live_ms = {k: spans[k][0] * 1e-3 for k in spans if k in ms and spans[k][2] > 0}
        for k in ms:
            bound, w = work[k]
            kernels[k] = dict(avg_ms=round(ms[k], 4), per_iter=count[k],
                              share=round(live_ms.get(k, ms[k]) * count[k] / iter_ms, 3), bound=bound)
            if k in live_ms:
                kernels[k].update(live_avg_ms=round(live_ms[k], 4), live_launches=spans[k][2])
            if bound == 'hbm+mfma':
                byt, flop = w
                t_roof = byt / (PEAK_HBM_GBS * 1e9) + flop / (PEAK_FP32_TFLOPS * 1e12)
                kernels[k].update(achieved_gbs=round(byt / (ms[k] * 1e-3) / 1e9, 2),
                                  achieved_tflops=round(flop / (ms[k] * 1e-3) / 1e12, 2),
                                  achieved=round(t_roof / (ms[k] * 1e-3), 4), unit='fraction of roofline time')
            else:
                ach = w / (ms[k] * 1e-3) / (1e12 if bound == 'mfma' else 1e9)
                kernels[k].update(achieved=round(ach, 2), unit='TFLOP/s' if bound == 'mfma' else 'GB/s')
        if 'k_head_screen_conv12_by_step' in spans and 'k_head_screen_conv12' in kernels:
            kernels['k_head_screen_conv12']['live_us_by_step'] = spans['k_head_screen_conv12_by_step'][0]
        dom = max(ms, key=lambda k: live_ms.get(k, ms[k]) * count[k])
        bound, w = work[dom]
        t_dom = live_ms.get(dom, ms[dom])
        combined = None
        if bound == 'hbm+mfma':
            byt, flop = w
            combined = round((byt / PEAK_HBM_GBS / 1e9 + flop / PEAK_FP32_TFLOPS / 1e12) / (t_dom * 1e-3), 4)
        if bound == 'hbm+mfma':                  # report the phase that dominates its roofline time
            byt, flop = w
            bound, w = ('hbm', byt) if byt / PEAK_HBM_GBS / 1e9 >= flop / PEAK_FP32_TFLOPS / 1e12 else ('mfma', flop)
        dom_ach = round(w / (t_dom * 1e-3) / (1e12 if bound == 'mfma' else 1e9), 2)
        iso_ach = round(w / (ms[dom] * 1e-3) / (1e12 if bound == 'mfma' else 1e9), 2)
        peak = PEAK_FP32_TFLOPS if bound == 'mfma' else PEAK_HBM_GBS
        # HBM bytes per launch from the committed PMC passes (tools/profile_round.sh):
        # (2*FETCH_SIZE + WRITE_SIZE) KiB, gfx950 FETCH_SIZE correction per MI355X_MICROARCH.md
        traffic = None
        # (per frame mode: the committed passes of mode M1 and of mode M2)
        pmc = os.path.join(ROOT, 'profiles', 'pmc_hbm_bytes_m2.json' if args.frames84 else 'pmc_hbm_bytes.json')
        if os.path.exists(pmc):
            try:
                t = json.load(open(pmc))['hbm_bytes_per_launch'].get(dom)
                traffic = None if t is None else int(round(t))
            except Exception:
                traffic = None
        roofline = dict(kernel=dom, bound=bound, achieved=dom_ach, peak=peak,
                        unit='TFLOP/s' if bound == 'mfma' else 'GB/s',
                        frac=round(dom_ach / peak, 4), traffic=traffic,
                        timing=('live: average in-graph launch span over the timed region (s_memrealtime, '
                                'a3c_engine_span_stats)' if dom in live_ms else 'isolated (HIP events)'),
                        avg_us=round(t_dom * 1e3, 2), isolated_us=round(ms[dom] * 1e3, 2),
                        isolated_achieved=iso_ach,
                        work_per_launch=w, work_unit='FLOP' if bound == 'mfma' else 'B')
        if combined is not None:   # two serial phases: (bytes/HBM peak + FLOP/MFMA peak) / time
            roofline['frac_combined_hbm_mfma'] = combined

    if world > 1:
        dist.barrier()
    if rank == 0:
        steps_total = world * E * n * args.steps
        coll = 'RCCL' if args.backend == 'nccl' else 'gloo, host-staged'
        NETNAME = 'A3C' if args.algo == 'a3c' else 'one-step Q'
        line = {
            'metric': METRIC, 'value': round(steps_total / el, 1), 'unit': 'env-steps/s', 'n_gpus': world,
            'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(el / args.steps * 1e3, 4),
            'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': 'fp32',
            'data': (f'synthetic: HBM-resident hashed {"pre-sized 84x84 grey" if args.frames84 else "RGB 210x160x3"} '
                     f'frame pool ({args.frames} frames) stepped by the on-device synthetic Atari env; random-init '
                     f'{args.dqn_type.upper()} {NETNAME} conv net' if not host else
                     f'synthetic: host-stepped emulator ({args.host_threads} threads, a3c_hostenv) writing raw RGB '
                     f'210x160x3 frames into pinned buffers, PCIe H2D every step (PCIe-inclusive); random-init '
                     f'NIPS {NETNAME} conv net'),
            'config': {'workload': f'{args.game}, {E} envs batched per MI355X, n-step={n}, '
                                   f'{"A3C" if args.algo == "a3c" else "one-step Q"} conv net ({args.dqn_type} trunk'
                                   f'{" + 256-cell LSTM head" if args.lstm else ""})',
                       'frames': 'M2: pre-sized 84x84 (copy)' if args.frames84 else 'M1: raw RGB 210x160x3 + screen',
                       'game': args.game, 'trunk': args.dqn_type, 'head': 'lstm' if args.lstm else 'feed-forward', 'env': args.env, 'envs_per_gpu': E, 'n_step': n, 'action_size': A, 'algo': args.algo,
                       'env_steps_per_step': world * E * n,
                       'parallelism': (f'dp{world} hogwild: unlocked RMSProp pushes into {world} IPC-mapped HBM '
                                       f'shards ({dict(fine="fine-grained", coarse="coarse-grained", uncached="uncached")[args.hogwild_memory]}) '
                                       f'over xGMI, {"push + pull after each rollout" if args.hogwild_sync else "push of rollout k-1 + pull under rollout k (stale-1)"}, '
                                       f'no collective'
                                       if args.update == 'hogwild' else
                                       f'dp{world} partitioned PS: {coll} all-to-all of per-worker-clipped grads, '
                                       f'{world} sequential RMSProp steps per owned shard, {coll} all-gather'
                                       if args.exchange == 'sequential' else
                                       f'dp{world} all-reduce ({coll}) of per-worker-clipped grads, one summed step')
                       if world > 1 else 'dp1', 'hipgraph': args.graph and not args.no_graph,
                       # every A3C_* switch set in the environment (a release library reads only the
                       # documented ones, a3c_common.h A3C_KNOB; {} = the defaults)
                       'env_knobs': {k: v for k, v in sorted(os.environ.items()) if k.startswith('A3C_')},
                       'update': {'overlap': 'overlap: rollout k uses params after update k-2 (stale-1 async), '
                                             'backward+apply of k-1 concurrent with rollout k',
                                  'sync': 'synchronous: rollout -> backward -> apply',
                                  'hogwild': 'hogwild: sharded lock-free parameter server (reference PS semantics)' +
                                             ('' if args.hogwild_sync else ', overlapped with the next rollout (stale-1)')
                                  }[args.update]},
            'timing': {'windows': len(windows), 'steps_per_window': args.steps,
                       'timed_seconds': round(sum(windows), 3),
                       'window_ms': [round(w * 1e3, 3) for w in windows],
                       'value_spread': [round(steps_total / max(windows), 1), round(steps_total / min(windows), 1)],
                       'value_mean_over_windows': round(steps_total * len(windows) / sum(windows), 1)},
            'roofline': roofline, 'cpu_baseline': cpu, 'kernels': kernels, 'dist': dist_rec,
            'final_loss': loss, 'params_finite': finite,
        }
        print(json.dumps(line), file=line_out, flush=True)
    if ps is not None:
        ps.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()

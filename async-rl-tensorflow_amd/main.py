"""main.py:1-98 on MI355X.  Same flags; ``--job_name``/``--ps_hosts``/``--worker_hosts`` are
accepted but the TF ps/worker cluster is replaced by one process per GPU under torchrun
(torch.distributed, backend nccl = RCCL), see src/distributed.py.

  --mode agent   the reference's per-step Q-learning Agent loop (agent.py:52-139), one env per
                 process, drop-in API (src/agent.py);
  --mode engine  the batched MI355X actor-learner (num_envs envs per GPU, n-step rollout +
                 gradient + exchange + RMSProp per iteration, src/engine.py).

  python main.py --mode engine --env_name Pong-v0 --iterations 1000
  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 main.py --mode engine
"""
import argparse
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np    # noqa: E402
import torch          # noqa: E402


def str2bool(v):
  return str(v).lower() in ('1', 'true', 'yes', 'y', 't')


def parse_flags(argv=None):
  p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
  # Model
  p.add_argument('--model', default='m1')
  p.add_argument('--dueling', type=str2bool, default=False)
  p.add_argument('--double_q', type=str2bool, default=False)
  # Environment
  p.add_argument('--env_name', default='Breakout-v0')
  p.add_argument('--action_repeat', type=int, default=1)
  # Optimizer
  p.add_argument('--decay', type=float, default=0.99)
  p.add_argument('--epsilon', type=float, default=0.1)
  p.add_argument('--momentum', type=float, default=0.0)
  p.add_argument('--beta', type=float, default=0.01)
  # Distributed (accepted for compatibility; torchrun provides RANK/WORLD_SIZE)
  p.add_argument('--ps_hosts', default='0.0.0.0:2222')
  p.add_argument('--worker_hosts', default='0.0.0.0:2223,0.0.0.0:2224')
  p.add_argument('--job_name', default='')
  p.add_argument('--task_index', type=int, default=0)
  # Misc
  p.add_argument('--gpu_fraction', default='1/1')
  p.add_argument('--display', type=str2bool, default=False)
  p.add_argument('--is_train', type=str2bool, default=True)
  p.add_argument('--random_seed', type=int, default=123)
  # MI355X engine
  p.add_argument('--mode', choices=['agent', 'engine'], default='engine')
  p.add_argument('--algo', choices=['a3c', 'q'], default='a3c')
  p.add_argument('--n_step', type=int, default=5)
  p.add_argument('--num_envs', type=int, default=256)
  p.add_argument('--num_frames', type=int, default=16384)
  p.add_argument('--iterations', type=int, default=1000)
  p.add_argument('--envs_on', choices=['device', 'host', 'gym'], default='device',
                 help='engine mode: envs stepped on the GPU (synthetic), on host threads (C++ synthetic '
                      'emulator, frames over PCIe), or gym/ALE envs on the host (AtariEnv, needs gym)')
  p.add_argument('--host_threads', type=int, default=16)
  p.add_argument('--max_step', type=int, default=None)
  p.add_argument('--log_every', type=int, default=None,
                 help='engine mode: iterations between summaries (default: test_step env-steps per env, '
                      'agent.py:104)')
  p.add_argument('--save_model_secs', type=int, default=600, help='checkpoint period (main.py:80)')
  p.add_argument('--max_to_keep', type=int, default=30, help='checkpoints kept (agent.py:29)')
  p.add_argument('--checkpoint_dir', default=None, help='default: <logdir>/<model_dir> (main.py:75)')
  p.add_argument('--resume', type=str2bool, default=True,
                 help='restore the newest checkpoint of checkpoint_dir, as managed_session does (main.py:90)')
  p.add_argument('--update', choices=['overlap', 'sync', 'hogwild'], default='overlap',
                 help='engine mode: stale-1 overlapped A3C, synchronous exchange, or Hogwild sharded PS')
  p.add_argument('--exchange', choices=['sequential', 'sum'], default='sequential',
                 help='multi-GPU sync/overlap exchange: sequential = partitioned PS applying every '
                      "worker's clipped gradient as its own RMSProp step in rank order (the reference "
                      'PS semantics); sum = one all-reduce, one RMSProp step of the summed gradients')
  p.add_argument('--lstm', type=str2bool, default=False,
                 help='engine mode, a3c: the 256-cell LSTM policy head (BASELINE config 5, DESIGN §4b)')
  p.add_argument('--dqn_type', choices=['nips', 'nature'], default='nips',
                 help="conv trunk of network.py:30-50 (Network(DQN_type=...)): nips (fused kernels) or nature "
                      "(implicit-GEMM kernels, nature.hip; --algo a3c)")
  p.add_argument('--logdir', default='./logs')
  return p.parse_args(argv)


def engine_options(flags):
  """The reference options of --mode engine: each one either reaches the Engine or is rejected,
  so no option is silently dropped (agent.py:176-184 double-Q, :234-249 dueling, network.py:30-42
  nature trunk).  Returns the Engine keyword arguments the flags select."""
  if flags.dueling:
    raise ValueError('--dueling (agent.py:234-249) is not fused into the engine: use --mode agent')
  if flags.dqn_type == 'nature' and (flags.algo != 'a3c' or flags.lstm):
    raise ValueError('--dqn_type nature: the A3C Network trunk (network.py:30-42) runs with --algo a3c and the '
                     'feed-forward head (the Q-net of agent.py:226-252 is nips only)')
  if flags.double_q and flags.algo != 'q':
    raise ValueError('--double_q is a Q-learning option (agent.py:176-184): use it with --algo q')
  if flags.lstm and flags.algo != 'a3c':
    raise ValueError('--lstm is an A3C policy head: use it with --algo a3c')
  kw = dict(lstm=bool(flags.lstm))
  if flags.double_q:
    kw['double_q'] = True
  if flags.dqn_type == 'nature':
    kw['dqn_type'] = 'nature'
  return kw


def initial_params(eng, action_size, algo, seed):
  """Flat host parameters initialised as the reference does: conv weights
  truncated_normal(0, 0.02) (agent.py:214), linear weights normal(0.02) (ops.py:36-37),
  zero biases (ops.py:24,38-39)."""
  from src.initializers import flatten_host, init_params
  from src.kernels import param_names_shapes
  ns = param_names_shapes(action_size, algo, lstm=eng.lstm, dqn_type=eng.dqn_type)
  return flatten_host(ns, eng.offsets, eng.params.numel(), init_params(ns, seed=seed))


def make_host_pool(config, flags, E, A, lives, rank):
  """Host-stepped envs for the external-env engine: the C++ synthetic emulator
  (`host`), or E gym envs wrapped with the reference's Environment rules (`gym`,
  environment.py:14-96)."""
  from src.host_env import AtariEnv, HostEnvPool, SyntheticHostEnvPool
  if flags.envs_on == 'host':
    return SyntheticHostEnvPool(E, A, lives, num_frames=min(flags.num_frames, 2048), seed=flags.random_seed,
                                env_id_base=rank * E, random_start=config.random_start,
                                action_repeat=config.action_repeat, threads=flags.host_threads)
  try:
    import gym
  except ImportError as e:
    raise RuntimeError('--envs_on gym needs the gym package (with the Atari ROMs)') from e
  # one emulator seed and one no-op-start stream per env (the reference: one env and one `random`
  # per worker process, environment.py:37), so the pool's threads cannot reorder the draws
  envs = []
  for e in range(E):
    sid = flags.random_seed + rank * E + e
    envs.append(AtariEnv(gym.make(config.env_name), action_repeat=config.action_repeat,
                         random_start=config.random_start, rng=random.Random(sid), seed=sid))
  return HostEnvPool(envs, threads=flags.host_threads)


def _agree(flag, world):
  """Rank 0's decision on every rank (checkpoint times must match across the ranks)."""
  if world == 1:
    return bool(flag)
  import torch.distributed as dist
  t = torch.tensor([1 if flag else 0], dtype=torch.int32,
                   device='cuda' if dist.get_backend() == 'nccl' else 'cpu')
  dist.broadcast(t, src=0)
  return bool(t.item())


def run_engine(config, flags):
  from src import checkpoint as C
  from src import distributed as D
  from src.base import BaseModel
  from src.engine import Engine
  from src.environment import game_spec
  from src.kernels import param_names_shapes
  rank, world, local = D.init_from_env()
  torch.cuda.set_device(local)
  A, lives = game_spec(config.env_name)
  E = flags.num_envs
  net_kw = engine_options(flags)
  opts = dict(gamma=config.discount, discount=config.discount, beta=config.beta, learning_rate=config.learning_rate,
              max_step=config.max_step, decay=config.decay, momentum=config.momentum, epsilon=config.epsilon,
              clip_norm=config.clip_norm, literal_adv=int(config.literal_adv), ep_start=config.ep_start,
              ep_end=config.ep_end, ep_end_t=config.ep_end_t, learn_start=config.learn_start,
              target_q_update_step=config.target_q_update_step, random_start=config.random_start,
              action_repeat=config.action_repeat)
  host = flags.envs_on != 'device'
  if host and flags.update == 'hogwild':
    raise ValueError('--envs_on host/gym drives a synchronous engine; use --update sync or overlap')
  # hogwild overlaps the push / pull of rollout k-1 with rollout k (src/engine.py iterate_hogwild)
  overlap = flags.update in ('overlap', 'hogwild') and not host
  if flags.update == 'overlap' and not overlap and rank == 0:
    print('main.py: --update overlap needs device envs; running the synchronous engine',
          file=sys.stderr, flush=True)
  pool = make_host_pool(config, flags, E, A, lives, rank) if host else None
  eng = Engine(num_envs=E, n_step=flags.n_step, action_size=A, algo=flags.algo, start_lives=lives,
               num_frames=1 if host else flags.num_frames, seed=flags.random_seed, env_id_base=rank * E,
               world_size=world, overlap=overlap, external_env=host, **net_kw, **opts)
  ns = param_names_shapes(A, flags.algo, lstm=eng.lstm, dqn_type=eng.dqn_type)
  # checkpoints: <logdir>/<model_dir> as the Supervisor's logdir (main.py:75), Saver max_to_keep
  # (agent.py:29); restored at start as managed_session does (main.py:90)
  ckdir = flags.checkpoint_dir or os.path.join(flags.logdir, BaseModel(config, verbose=False).model_dir)
  saver = C.Saver(ckdir, max_to_keep=flags.max_to_keep)
  restored = C.restore_engine(saver, eng, ns, rank, world) if flags.resume else None
  if restored is None:
    eng.reset(initial_params(eng, A, flags.algo, flags.random_seed))
    D.broadcast_params(eng.params, src=0)
    if flags.algo == 'q':
      eng.target_params.copy_(eng.params)
    if overlap:
      eng.reset()    # keeps the broadcast parameters, re-takes the pipeline snapshots
  elif rank == 0:
    print(json.dumps({'restored': saver.latest(), 'global_step': restored}), flush=True)
  xch = None
  if world > 1:
    xch = D.PartitionedPS(eng.params.numel()) if flags.exchange == 'sequential' else D.GradExchange()
  ps = None
  if flags.update == 'hogwild':
    from src.hogwild import HogwildPS
    ps = HogwildPS(eng.params, decay=config.decay, momentum=config.momentum, epsilon=config.epsilon,
                   ms=eng.ms, mom=eng.mom)     # (restored slots, or the TF1 init after reset)
  # the reference's worker loop `for self.step in xrange(self.step, self.max_step)` (agent.py:46,55):
  # each worker -- here each env, all in lock-step -- takes env-steps up to max_step on its own
  # counter; one rollout is n of them, and the overlap pipeline applies one call later
  n = flags.n_step
  remaining = max(0, int(config.max_step) - eng.worker_step)
  iterations = min(flags.iterations, -(-remaining // n) + (1 if overlap else 0))
  test_step = int(getattr(config, 'test_step', getattr(config, '_test_step', 5000)))
  log_every = flags.log_every or max(1, test_step // n)
  torch.cuda.synchronize()
  t0 = time.time()
  last_save = t0
  log = None
  if rank == 0:
    os.makedirs(flags.logdir, exist_ok=True)
    log = open(os.path.join(flags.logdir, 'engine.jsonl'), 'a')
  for it in range(iterations):
    if ps is not None:
      eng.iterate_hogwild(ps)
    elif pool is not None:
      eng.iterate_host(pool, exchange=xch)
    else:
      eng.iterate(exchange=xch)
    if rank == 0:
      eng.stats_accumulate()       # train_with_summary's aggregates (agent.py:91-131), on device
    if (it + 1) % log_every == 0:
      if rank == 0:
        loss = eng.loss.tolist()
        st = eng.read_stats(reset=True)
        torch.cuda.synchronize()
        dt = time.time() - t0
        wstep = eng.worker_step
        rec = dict(iteration=it + 1, global_step=int(eng.counters[1].item()), worker_step=wstep,
                   env_steps_per_sec=(it + 1) * E * n * world / dt, **st,
                   learning_rate=max(0.0, (config.max_step - wstep + 1.) / config.max_step * config.learning_rate),
                   loss_policy=loss[0], loss_value=loss[1], entropy=loss[2], loss_total=loss[3],
                   mean_return=float(eng.returns.mean().item()))
        print(json.dumps(rec), flush=True)
        log.write(json.dumps(rec) + '\n')
      if _agree(rank == 0 and time.time() - last_save >= flags.save_model_secs, world):
        _sync_slots(eng, xch, ps)
        C.save_engine(saver, eng, ns, rank, world, barrier=_barrier(world))
        last_save = time.time()
  torch.cuda.synchronize()
  if iterations > 0:
    _sync_slots(eng, xch, ps)
    C.save_engine(saver, eng, ns, rank, world, barrier=_barrier(world))    # the final state
  if ps is not None:
    ps.close()
  if pool is not None:
    pool.close()
  if log:
    log.close()
  return eng


def _sync_slots(eng, xch, ps):
  """The RMSProp slots a sharded update keeps per owner (partitioned PS ranges, Hogwild shards)
  into the engine's full ms / mom before a checkpoint."""
  for x in (xch, ps):
    if hasattr(x, 'sync_slots'):
      x.sync_slots(eng)


def _barrier(world):
  if world == 1:
    return None
  import torch.distributed as dist
  return dist.barrier


def run_agent(config, flags):
  from src import distributed as D
  from src.agent import Agent, Supervisor
  from src.environment import GymEnvironment
  from src.optim import RMSPropOptimizer
  rank, world, local = D.init_from_env()
  torch.cuda.set_device(local)
  random.seed(flags.random_seed + rank)
  env = GymEnvironment(config)
  optimizer = RMSPropOptimizer(None, decay=0.99, momentum=0, epsilon=0.1)     # main.py:64-65
  agent = Agent(config, env, optimizer)
  agent.ep_end = random.sample([0.1, 0.01, 0.5], 1)[0]                        # main.py:68
  if world > 1:
    D.broadcast_params(agent.params, src=0)
  print(agent.model_dir)
  is_chief = rank == 0
  sv = Supervisor(is_chief=is_chief, logdir=os.path.join(flags.logdir, agent.model_dir), agent=agent)
  agent.update_target_q_network()
  if flags.is_train:
    (agent.train_with_summary if is_chief else agent.train)(sv, is_chief)
  else:
    agent.play(sv, is_chief)
  return agent


def main(argv=None):
  flags = parse_flags(argv)
  random.seed(flags.random_seed)
  np.random.seed(flags.random_seed)
  from config import get_config
  config = get_config(flags)
  config.cnn_format = 'NHWC'                       # main.py:45
  if flags.max_step is not None:
    config.max_step = flags.max_step
  config.algo, config.n_step, config.num_envs = flags.algo, flags.n_step, flags.num_envs
  if flags.mode == 'engine':
    engine_options(flags)             # reject unsupported reference options before any device work
    return run_engine(config, flags)
  return run_agent(config, flags)


if __name__ == '__main__':
  main()

"""Host-stepped envs feeding the engine (a3c_engine_ext_*, src/host_env.py).

With the synthetic emulator stepped on the HOST (oracle/synthetic_env.py one object per env, or the
C++ worker threads of a3c_hostenv_*, raw RGB frames through pinned buffers):
* the external-env engine is checked against the CPU replay oracle (oracle/engine_ref.py) directly,
  at the bar of tests/_engine_parity.py (frames, rewards, terminals bit-exact; returns, losses,
  gradients, parameters to fp tolerance), including the headline shape (256 envs) with chunked
  uploads;
* and it reproduces the device-env engine bit for bit (same actions, rewards, terminals, frame
  ring, losses and parameters).
The synthetic env's act / life-loss / no-op rule itself is pinned to the reference's own
GymEnvironment code by tests/golden/synth_env_golden.npz (tests/test_host_env.py)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')

from oracle.synthetic_env import SyntheticAtari, pool_frame  # noqa: E402
from _engine_parity import check_sync_vs_oracle  # noqa: E402


class HostSynthEnv:
    """One synthetic env on the host with the interface HostEnvPool steps (raw RGB frames)."""

    def __init__(self, seed, e, P, A, lives):
        self.seed = seed
        self.env = SyntheticAtari(seed, 1, P, A, lives, env_id_base=e)

    def _rgb(self):
        return pool_frame(self.seed, int(self.env.frame[0]))

    def new_random_game(self):
        self.env.new_random_game()
        return self._rgb(), 0, 0, bool(self.env.terminal[0])

    def act(self, action, is_training=True):
        _, r, t = self.env.act(np.array([action]), is_training=is_training)
        return self._rgb(), float(r[0]), bool(t[0])


def _pair(algo, A, E, n, lives, seed, P, lstm=False):
    from src.engine import Engine
    from src.initializers import init_params, flatten_host
    from src.kernels import param_names_shapes
    kw = dict(num_envs=E, n_step=n, action_size=A, algo=algo, start_lives=lives, seed=seed, lstm=lstm,
              learning_rate=2e-3)
    dev = Engine(num_frames=P, **kw)
    ext = Engine(num_frames=1, external_env=True, **kw)
    ns = param_names_shapes(A, algo, lstm=lstm)
    p = flatten_host(ns, dev.offsets, dev.params.numel(), init_params(ns, seed=seed, stddev=0.08))
    dev.reset(p)
    ext.reset(p)
    return dev, ext


@pytest.mark.parametrize('algo,A,E,n,lives,lstm', [('a3c', 6, 8, 5, 3, False), ('a3c', 4, 5, 3, 5, True),
                                                   ('q', 6, 4, 6, 3, False)])
def test_external_envs_equal_device_envs(algo, A, E, n, lives, lstm):
    from src.host_env import HostEnvPool
    seed, P = 900 + E, 40
    dev, ext = _pair(algo, A, E, n, lives, seed, P, lstm)
    pool = HostEnvPool([HostSynthEnv(seed, e, P, A, lives) for e in range(E)], threads=2)
    for it in range(4):
        dev.iterate()
        ext.iterate_host(pool)
        torch.cuda.synchronize()
        assert torch.equal(dev.actions, ext.actions), it
        assert torch.equal(dev.rewards, ext.rewards), it
        assert torch.equal(dev.terminals, ext.terminals), it
        assert torch.equal(dev.frame_ring, ext.frame_ring), it
        assert torch.equal(dev.counters, ext.counters), it
        torch.testing.assert_close(ext.loss, dev.loss, rtol=1e-6, atol=1e-6)
        torch.testing.assert_close(ext.params, dev.params, rtol=1e-6, atol=1e-7)
    pool.close()


@pytest.mark.parametrize('algo,A,E,n,lives,P,kind', [
    ('a3c', 6, 8, 5, 3, 40, 'py'), ('a3c', 4, 7, 3, 5, 40, 'py'), ('q', 6, 4, 6, 3, 40, 'py'),
    ('a3c', 6, 13, 5, 3, 64, 'cpp3'), ('a3c', 6, 256, 5, 0, 512, 'cpp2'), ('a3c', 4, 256, 5, 5, 512, 'cpp2')],
    ids=['a3c-py', 'breakout-py', 'q-py', 'a3c-cpp-3ranges', 'pong256-cpp-2ranges', 'breakout256-cpp-2ranges'])
def test_external_envs_match_oracle(algo, A, E, n, lives, P, kind):
    """The external-env engine (Engine.rollout_host + rollout_grad + apply) against EngineRef: the
    host envs are either Python objects (HostEnvPool of per-env oracle emulators) or the C++ worker
    threads stepping env ranges whose frames go up by a3c_engine_ext_upload while the next range
    steps (SyntheticHostEnvPool, `upload_chunks` ranges)."""
    from src.host_env import HostEnvPool, SyntheticHostEnvPool

    def pool(seed):
        if kind == 'py':
            return HostEnvPool([HostSynthEnv(seed, e, P, A, lives) for e in range(E)], threads=2)
        return SyntheticHostEnvPool(E, A, lives, num_frames=P, seed=seed, threads=4, upload_chunks=int(kind[-1]))
    check_sync_vs_oracle(algo, A, E, n, lives, iters=3, seed=500 + E, frames=P, host_pool=pool,
                         learning_rate=2e-3)


def test_external_env_call_order_enforced():
    from src.engine import Engine
    ext = Engine(num_envs=2, n_step=2, action_size=6, external_env=True, num_frames=1)
    ext.reset()
    acts = torch.zeros(2, dtype=torch.int32).pin_memory()
    with pytest.raises(RuntimeError):
        ext.ext_act(acts)                       # ext_begin first
    with pytest.raises(RuntimeError):
        ext.rollout_grad()                      # n steps first
    with pytest.raises(ValueError):
        ext.ext_act(torch.zeros(2, dtype=torch.int32))     # pageable host buffer
    with pytest.raises(RuntimeError):
        Engine(num_envs=2, n_step=2, action_size=6, external_env=True, overlap=True)


@pytest.mark.parametrize('chunks,E', [(1, 8), (3, 8), (4, 13), (13, 13), (2, 256)])   # 256: BASELINE config 2
def test_chunked_uploads_equal_device_envs(chunks, E):
    """The C++ host env stepped in env ranges, each range's frames sent by a3c_engine_ext_upload
    while the next is stepped (Engine.iterate_host), equals the device-env engine bit for bit."""
    from src.host_env import SyntheticHostEnvPool
    seed, P, A, n, lives = 321, 40, 6, 5, 3
    dev, ext = _pair('a3c', A, E, n, lives, seed, P)
    pool = SyntheticHostEnvPool(E, A, lives, num_frames=P, seed=seed, threads=3, upload_chunks=chunks)
    for it in range(4):
        dev.iterate()
        ext.iterate_host(pool)
        torch.cuda.synchronize()
        assert torch.equal(dev.actions, ext.actions), it
        assert torch.equal(dev.rewards, ext.rewards), it
        assert torch.equal(dev.terminals, ext.terminals), it
        assert torch.equal(dev.frame_ring, ext.frame_ring), it
        torch.testing.assert_close(ext.loss, dev.loss, rtol=1e-6, atol=1e-6)
        torch.testing.assert_close(ext.params, dev.params, rtol=1e-6, atol=1e-7)
    pool.close()


def test_ext_upload_checks():
    from src.engine import Engine
    ext = Engine(num_envs=3, n_step=2, action_size=6, external_env=True, num_frames=1)
    ext.reset()
    rgb = torch.zeros(3, 210, 160, 3, dtype=torch.uint8).pin_memory()
    with pytest.raises(RuntimeError):
        ext.ext_upload(rgb, 0, 3)               # ext_begin / ext_act first
    ext.ext_begin(rgb)
    ext.ext_act(torch.zeros(3, dtype=torch.int32).pin_memory())
    with pytest.raises(RuntimeError):
        ext.ext_upload(rgb, 2, 4)               # range outside [0, E]
    ext.ext_upload(rgb, 0, 2)
    r = torch.zeros(3, dtype=torch.float32).pin_memory()
    t = torch.zeros(3, dtype=torch.uint8).pin_memory()
    with pytest.raises(RuntimeError):
        ext.ext_observe(None, r, t)             # env 2's frame was never sent this step
    ext.ext_upload(rgb, 1, 3)                   # overlapping ranges: [0, 3) covered
    ext.ext_observe(None, r, t)
    with pytest.raises(RuntimeError):
        ext.ext_upload(rgb, 0, 3)               # observe closed the step: ext_act first
    ext.ext_act(torch.zeros(3, dtype=torch.int32).pin_memory())
    with pytest.raises(RuntimeError):
        ext.ext_act(torch.zeros(3, dtype=torch.int32).pin_memory())    # one observe per act
    ext.ext_observe(rgb, r, t)
    torch.cuda.synchronize()

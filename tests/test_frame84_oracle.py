"""Measurement mode M2 (pre-sized 84x84 frames) on the oracle side: the pre-sized pool
frame is the first 441 16-byte chunks of the same philox hash as the RGB frame (k_pool_fill with
frame_bytes = 7056), and the replay engine's history ring holds those frames unmodified."""
import numpy as np

from oracle.engine_ref import EngineRef
from oracle.ref_cpu import init_params
from oracle.synthetic_env import pool_frame, pool_frame84


def test_pool_frame84_is_the_hash_prefix():
    for seed, f in ((123, 0), (123, 17), (7, 4095)):
        a = pool_frame84(seed, f)
        assert a.shape == (84, 84) and a.dtype == np.uint8
        assert np.array_equal(a.reshape(-1), pool_frame(seed, f).reshape(-1)[:84 * 84])


def test_engine_ref_frame84_ring_holds_pool_frames():
    from oracle.ps_worker import _names_shapes
    ns = _names_shapes(6, 'a3c')
    ref = EngineRef(init_params(ns, seed=3), 4, 3, 6, 'a3c', 0, 64, seed=5, frame84=True)
    ref.reset()
    for c in range(4):
        for e in range(4):
            assert np.array_equal(ref.ring[e, c % ref.R], pool_frame84(5, ref.env.frame[e]))
    ref.iterate()
    for e in range(4):     # the newest screen is the post-act frame, copied as is
        assert np.array_equal(ref.ring[e, (ref.tau + 3) % ref.R], pool_frame84(5, ref.env.frame[e]))

"""Philox4x32-10 counter-based RNG, numpy restatement (TEST INFRASTRUCTURE ONLY).

The reference draws its randomness from Python's ``random`` module
(``agent.py:146-147`` epsilon coin / random action, ``environment.py:37`` no-op count,
``main.py:68`` ep_end choice) and TF's op RNG (``network.py:72`` ``batch_sample``,
missing).  Neither is reproducible across a batched GPU engine, so the build defines
its randomness as Philox4x32-10 (Salmon et al., SC'11) keyed by the run seed
(``main.py:35`` default 123) and counted by (step, env, purpose).  The HIP kernels
in ``csrc/philox.h`` implement the same function; this module replays it so the
oracle and the GPU agree bit for bit.
"""
import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint32(0x9E3779B9)
W1 = np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)

# purposes (counter word 3 unless stated) -- keep in sync with csrc/philox.h
P_ACTION = 1      # categorical sample / epsilon-greedy draws
P_STEP = 3        # synthetic env step (frame, reward, life loss)
P_RESET = 6       # synthetic env reset (episode length, first frame)
P_NOOP = 7        # random no-op count in new_random_game
P_POOL = 9        # frame pool bytes


def philox4x32(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10.  All counters are uint32 arrays (broadcastable);
    keys are python ints.  Returns four uint32 arrays."""
    c0 = np.asarray(c0, dtype=np.uint64) & MASK32
    c1 = np.asarray(c1, dtype=np.uint64) & MASK32
    c2 = np.asarray(c2, dtype=np.uint64) & MASK32
    c3 = np.asarray(c3, dtype=np.uint64) & MASK32
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    k0 = np.uint64(int(k0) & 0xFFFFFFFF)
    k1 = np.uint64(int(k1) & 0xFFFFFFFF)
    for r in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK32
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & MASK32, lo1, (hi0 ^ c3 ^ k1) & MASK32, lo0
        if r != 9:
            k0 = (k0 + np.uint64(W0)) & MASK32
            k1 = (k1 + np.uint64(W1)) & MASK32
    return (c0.astype(np.uint32), c1.astype(np.uint32),
            c2.astype(np.uint32), c3.astype(np.uint32))


def u01(x):
    """uint32 -> float32 uniform in [0,1): top 24 bits * 2^-24 (exact in fp32)."""
    return ((np.asarray(x, dtype=np.uint32) >> np.uint32(8)).astype(np.float32)
            * np.float32(1.0 / 16777216.0))


def seed_key(seed):
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    return seed & 0xFFFFFFFF, seed >> 32

"""Pin the CPU oracle to the reference's own outputs (tests/golden, made by
tests/golden/make_goldens.py from /root/reference/src/environment.py + history.py) and to
published known-answer vectors (Philox)."""
import hashlib
import os

import numpy as np
import pytest

from make_goldens import frame_from_spec
from oracle import philox as px
from oracle import ref_cpu as R


@pytest.fixture(scope='module')
def screen_golden(golden_dir):
    return np.load(os.path.join(golden_dir, 'screen_golden.npz'))


def test_screen_matches_reference(screen_golden):
    g = screen_golden
    for kind, seed, exp in zip(g['kinds'], g['seeds'], g['screens']):
        out = R.screen(frame_from_spec(str(kind), int(seed)))
        assert out.dtype == np.uint8 and out.shape == (84, 84)
        assert np.array_equal(out, exp), (kind, seed)


def test_resize_other_geometries_match_reference(screen_golden):
    g = screen_golden
    for i in range(len(g['extra_h'])):
        h, w, oh, ow, sd = (int(g['extra_' + k][i]) for k in ('h', 'w', 'oh', 'ow', 'seed'))
        out = R.resize_bilinear_u8(R.luminance_u8(frame_from_spec('noise', sd, h, w)), oh, ow)
        assert np.array_equal(out, g[f'extra_out{i}']), (h, w, oh, ow)


def test_full_luminance_table_matches_reference(screen_golden):
    """All 2^24 RGB values: fp64, left-to-right, truncating (environment.py:51-52)."""
    g = screen_golden
    rgb = np.arange(1 << 24, dtype=np.uint32)
    fr = np.stack([(rgb >> 16) & 255, (rgb >> 8) & 255, rgb & 255], -1).astype(np.uint8)
    lum = R.luminance_u8(fr)
    assert hashlib.sha256(lum.tobytes()).hexdigest() == str(g['lum_sha256'])
    assert np.array_equal(lum[g['lum_hard_idx']], g['lum_hard_val'])
    assert len(g['lum_hard_idx']) > 0          # a float32 evaluation would be wrong somewhere


def test_pillow_coefficients_shape():
    b, k = R.pillow_bilinear_coeffs(160, 84)
    assert k.shape == (84, 5)
    b, k = R.pillow_bilinear_coeffs(210, 84)
    assert k.shape == (84, 7)
    # each row of fixed-point weights sums to ~2^22
    assert np.all(np.abs(k.sum(1) - (1 << 22)) <= k.shape[1])


def test_history_matches_reference(golden_dir, screen_golden):
    hg = np.load(os.path.join(golden_dir, 'history_golden.npz'))
    seq = screen_golden['screens'][:7]
    for fmt in ('NHWC', 'NCHW'):
        h = R.History(cnn_format=fmt)
        gets = []
        for i, s in enumerate(seq):
            h.add(s)
            gets.append(h.get().copy())
            if i == 4:
                h.reset()
                gets.append(h.copy())
        assert np.array_equal(np.stack(gets), hg[f'gets_{fmt}'].astype(np.float32)), fmt


def test_philox_known_answers():
    """Random123 philox4x32-10 KAT vectors."""
    kat = [((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
           ((0xffffffff,) * 4, (0xffffffff, 0xffffffff), (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
           ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
            (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]
    for ctr, key, exp in kat:
        out = px.philox4x32(*ctr, *key)
        assert tuple(int(o) for o in out) == exp


def test_returns_and_td_target_semantics():
    rewards = np.array([[1, 0], [0, -1], [0, 1]], np.float32)
    terms = np.array([[0, 0], [1, 0], [0, 0]], np.uint8)
    boot = np.array([2.0, 3.0], np.float32)
    Rt = R.nstep_returns(rewards, terms, boot, 0.99)
    # env 0: terminal at i=1 cuts the bootstrap from i=2 onward
    assert np.isclose(Rt[2, 0], 0 + 0.99 * 2.0)
    assert np.isclose(Rt[1, 0], 0.0)
    assert np.isclose(Rt[0, 0], 1.0)
    assert np.isclose(Rt[0, 1], 0 + 0.99 * (-1 + 0.99 * (1 + 0.99 * 3.0)))
    t = R.td_target([1., 0.], [0, 1], [[0.5, 2.0], [7.0, 1.0]], 0.99)
    assert np.allclose(t, [1 + 0.99 * 2.0, 0.0])


def test_clip_by_norm_and_rmsprop_semantics():
    g = np.full(100, 10.0, np.float32)            # norm 100 > 40
    c = R.clip_by_norm(g, 40.0)
    assert np.isclose(np.linalg.norm(c), 40.0, rtol=1e-6)
    small = np.full(4, 0.1, np.float32)
    assert np.allclose(R.clip_by_norm(small, 40.0), small, rtol=1e-6)
    w = np.zeros(3, np.float32)
    ms = np.ones(3, np.float32)
    mom = np.zeros(3, np.float32)
    grad = np.array([1.0, -2.0, 0.0], np.float32)
    R.rmsprop_apply(w, ms, mom, grad, 0.001)
    exp_ms = 1 + (grad ** 2 - 1) * 0.01
    assert np.allclose(ms, exp_ms)
    assert np.allclose(w, -0.001 * grad / np.sqrt(exp_ms + 0.1))
    assert np.isclose(R.learning_rate(0), 0.0007 * (80_000_001 / 80_000_000))


def test_epsilon_schedule():
    assert R.epsilon_schedule(0) == 1.0
    assert np.isclose(R.epsilon_schedule(2_000_032), 0.55)
    assert R.epsilon_schedule(10 ** 9) == 0.1

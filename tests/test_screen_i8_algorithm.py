"""The integer-GEMM form of Pillow's BILINEAR resample that the screen kernels run on the int8
matrix cores (csrc/screen_atari.h, MfmaTab / resample_tile), restated in numpy and checked
against the oracle's Pillow resample (oracle/ref_cpu.py resize_bilinear_u8, pinned by the
reference's goldens) on random and extreme images -- the exactness argument, on the CPU:
  taps k = 65536 d2 + 256 d1 + d0 in balanced base-256 digits, bytes x' = x - 128,
  acc = ((32 + S2) * 256 + S1) * 256 - 128 delta + S0  (S_j = sum d_j x'),  out = 128 + (acc >> 22),
over 16x16 output tiles whose K = 64 source window starts at a 16-aligned offset, with the
source rows / columns past the image edge and the pad outputs as the kernel has them.
The GPU kernels themselves are checked bit for bit through the engine's frame ring
(tests/test_gpu_engine.py, tests/_engine_parity.py)."""
import numpy as np
import pytest

from oracle import ref_cpu as R

PB = 22
MT = 6          # 16-wide output tiles over 84 (+12 pad)


def tables(in_size, out_size):
    """MfmaTab::fill: B fragments [n-tile][digit 2,1,0][lane][16], window bases, corrections."""
    b, k = R.pillow_bilinear_coeffs(in_size, out_size)
    K = k.shape[1]
    B = np.zeros((MT, 3, 64, 16), np.int64)
    base = np.zeros(MT, np.int64)
    c0 = np.zeros(MT * 16, np.int64)
    for nt in range(MT):
        base[nt] = b[16 * nt, 0] // 16 * 16
        for n in range(16):
            o = 16 * nt + n
            if o < out_size:
                nz = np.nonzero(k[o])[0]
                assert b[o, 0] + nz.max() - base[nt] < 64       # the window covers every tap
                c0[o] = -128 * ((1 << PB) - int(k[o].sum()))
            for kk in range(64):
                t = base[nt] + kk - (b[o, 0] if o < out_size else 0)
                w = int(k[o, t]) if (o < out_size and 0 <= t < K) else 0
                d0 = ((w + 128) & 255) - 128
                w1 = (w - d0) // 256
                d1 = ((w1 + 128) & 255) - 128
                d2 = (w1 - d1) // 256
                assert -128 <= d2 <= 127 and 65536 * d2 + 256 * d1 + d0 == w
                lane, j = n + 16 * (kk >> 4), kk & 15
                B[nt, :, lane, j] = (d2, d1, d0)
    return B, base, c0


def bmat(frag):
    """[64 lanes][16] B fragment -> B[k = 16 (lane >> 4) + j][n = lane & 15]"""
    M = np.zeros((64, 16), np.int64)
    for lane in range(64):
        M[16 * (lane >> 4):16 * (lane >> 4) + 16, lane & 15] = frag[lane]
    return M


def tile(a_rows, Bt, c0):
    """resample_tile for 16 source rows of 64 bytes: C[m = row][n] output bytes"""
    xp = a_rows.astype(np.int64) - 128
    acc = np.full((16, 16), 32, np.int64) + xp @ bmat(Bt[0])
    acc = acc * 256 + xp @ bmat(Bt[1])
    acc = acc * 256 + c0[None, :] + xp @ bmat(Bt[2])
    assert np.abs(acc).max() < 2 ** 31
    return 128 + (acc >> 22)


HT = tables(160, 84)
VT = tables(210, 84)


def screen_resample_i8(gray):
    """hpass_mfma + vpass_mfma over a [210][160] luminance image (LDS images as the kernel has
    them: rows back to back, reads past a row run into the next, garbage times zero taps)."""
    HB, hbase, hc0 = HT
    VB, vbase, vc0 = VT
    flat = np.concatenate([gray.reshape(-1), np.full(256, 77, np.uint8)])   # (bytes past the end)
    tmpT = np.full((84, 224), 99, np.int64)
    for q in range(14 * MT):
        nt, mt = q % MT, q // MT
        rows = np.stack([flat[min(16 * mt + n, 209) * 160 + hbase[nt]:][:64] for n in range(16)])
        C = tile(rows, HB[nt], hc0[16 * nt:16 * nt + 16])
        for n in range(16):
            X = 16 * nt + n
            if X < 84:
                tmpT[X, 16 * mt:16 * mt + 16] = C[:, n]
    tflat = np.concatenate([tmpT.reshape(-1), np.full(256, 55, np.int64)])
    out = np.zeros((84, 84), np.int64)
    for q in range(MT * MT):
        nt, mt = q % MT, q // MT
        rows = np.stack([tflat[min(16 * mt + n, 83) * 224 + vbase[nt]:][:64] for n in range(16)])
        C = tile(rows, VB[nt], vc0[16 * nt:16 * nt + 16])
        for n in range(16):
            yy = 16 * nt + n
            for m in range(16):
                x = 16 * mt + m
                if yy < 84 and x < 84:
                    out[yy, x] = C[m, n]
    return out.astype(np.uint8)


@pytest.mark.parametrize('kind', ['random', 'zeros', 'ones', 'checker', 'stripes', 'ramp'])
def test_i8_resample_equals_pillow(kind):
    rng = np.random.default_rng(len(kind))
    g = {'random': lambda: rng.integers(0, 256, (210, 160)),
         'zeros': lambda: np.zeros((210, 160)),
         'ones': lambda: np.full((210, 160), 255),
         'checker': lambda: (np.indices((210, 160)).sum(0) % 2) * 255,
         'stripes': lambda: (np.arange(160)[None, :] % 3 == 0) * 255 + np.zeros((210, 1)),
         'ramp': lambda: np.add.outer(np.arange(210), np.arange(160)) % 256}[kind]().astype(np.uint8)
    np.testing.assert_array_equal(screen_resample_i8(g), R.resize_bilinear_u8(g, 84, 84))


def test_i8_resample_on_screen_goldens():
    """The reference's own screens (tests/golden/screen_golden.npz, made by running its
    environment.py), every spec: luminance by the oracle, both resampling passes in i8 form."""
    import os
    from make_goldens import frame_from_spec
    g = np.load(os.path.join(os.path.dirname(__file__), 'golden', 'screen_golden.npz'))
    for kind, seed, exp in zip(g['kinds'], g['seeds'], g['screens']):
        got = screen_resample_i8(R.luminance_u8(frame_from_spec(str(kind), int(seed))))
        np.testing.assert_array_equal(got, exp, err_msg=f'{kind} {seed}')

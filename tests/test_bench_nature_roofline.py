"""bench.py's nature roofline (CPU): the per-pass table attributes the work of the passes that run
inside another pass's launch (the per-state conv kernel k_nat_conv23 under conv2's id, the fused
dX kernel under conv3 dX's) to that launch, and names the launch with the largest share of the
iteration.  The engine here is a stand-in that answers a3c_engine_time_kernel as the library does
(an A3CError for a pass with no launch of its own)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class FakeEngine:
    def __init__(self, lib, times, inside):
        self.lib, self.times, self.inside = lib, times, inside

    def time_kernel(self, kid, iters):
        name = {v: k for k, v in self.lib.KER_NAT.items()}[kid]
        if name in self.inside:
            raise self.lib.A3CError('a3c_engine_time_kernel failed (-2): runs inside k_nat_conv23', -2)
        return self.times[name]


TIMES = {'conv1_fwd': 0.0156, 'conv2_fwd': 0.0369, 'conv3_fwd': 0.0210, 'fc_fwd': 0.0174,
         'conv3_dw': 0.062, 'conv3_dx': 0.085, 'conv2_dw': 0.088, 'conv2_dx': 0.106, 'conv1_dw': 0.095}


def _roof(inside):
    import bench
    from src import _lib
    eng = FakeEngine(_lib, TIMES, inside)
    return bench, bench.nature_roofline(eng, _lib, 256, 5, 0.776)


def test_fused_forward_is_one_entry_with_the_three_layers_work():
    bench, (roof, k) = _roof({'conv1_fwd', 'conv3_fwd'})
    assert 'nat_conv1_fwd' not in k and 'nat_conv2_fwd' not in k and 'nat_conv3_fwd' not in k
    e = k['nat_conv123_fwd']
    flop = (bench.NAT_FLOP['conv1_fwd'] + bench.NAT_FLOP['conv2_fwd'] + bench.NAT_FLOP['conv3_fwd']) * 256
    assert e['flop_per_launch'] == flop == 3961520128
    assert e['achieved'] == pytest.approx(flop / 0.0369e-3 / 1e12, rel=1e-3)
    assert e['per_iter'] == 6
    assert roof['kernel'] == 'nat_conv123_fwd'            # 6 x 36.9 us: the largest share
    assert roof['frac'] == pytest.approx(e['achieved'] / bench.PEAK_FP32_TFLOPS, rel=1e-3)


def test_fused_dx_is_one_entry():
    bench, (roof, k) = _roof({'conv2_dx'})
    e = k['nat_conv32_dx']
    assert 'nat_conv2_dx' not in k and 'nat_conv3_dx' not in k
    assert e['flop_per_launch'] == (bench.NAT_FLOP['conv3_dx'] + bench.NAT_FLOP['conv2_dx']) * 5 * 256
    assert e['per_iter'] == 1


def test_unfused_passes_keep_their_own_entries():
    bench, (roof, k) = _roof(set())
    assert set(k) == {'nat_' + n for n in TIMES}
    assert k['nat_conv2_fwd']['flop_per_launch'] == bench.NAT_FLOP['conv2_fwd'] * 256


def test_live_span_names_the_roofline_time():
    """With the per-state conv kernel's live spans (bench.py's timed region), the roofline takes the
    live average (what the rocprof trace sees beside the backward) and keeps the isolated time."""
    import bench
    from src import _lib
    eng = FakeEngine(_lib, TIMES, {'conv1_fwd', 'conv3_fwd'})
    roof, k = bench.nature_roofline(eng, _lib, 256, 5, 0.776, {'nat_conv123_fwd': (42.1, 60.0, 1200)})
    assert roof['kernel'] == 'nat_conv123_fwd' and roof['timing'].startswith('live')
    assert roof['avg_us'] == 42.1 and roof['isolated_us'] == pytest.approx(36.9)
    assert roof['frac'] == pytest.approx(3961520128 / 42.1e-6 / 1e12 / bench.PEAK_FP32_TFLOPS, rel=1e-3)
    assert k['nat_conv123_fwd']['live_launches'] == 1200

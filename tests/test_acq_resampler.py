"""Acquisition resampler, host side (no GPU): the library's firdes::low_pass / flowgraph design
(gnss_flowgraph.cc:1070-1113) against the oracle restatement, and the oracle FIR's streaming.

GNU Radio (firdes, fir_filter_ccf) and VOLK are not in the reference tree and not installed, so
these restatements are parity-unpinned against the reference itself: the product and the oracle
restate the published algorithm independently and must agree bit for bit; the filter's response
is checked against its design (DC gain 1, stop band, symmetry).
"""
import numpy as np
import pytest

from gnss_sim_receiver_amd import abi, engine
from oracle import oracle as O

DESIGNS = [(4000000, 2e6), (25000000, 2e6), (50000000, 2e6), (6250000, 2e6), (20000000, 10e6), (4092000, 2e6), (2000000, 2e6),
           (3000000, 2e6)]


@pytest.fixture(scope="module")
def lib(built):
    return abi.load()


@pytest.mark.parametrize("fs,opt", DESIGNS)
def test_design_matches_oracle(lib, fs, opt):
    d, taps = engine.acq_resampler_design(lib, fs, opt)
    d_o, taps_o = O.acq_resampler_design(fs, opt)
    assert d == d_o
    assert np.array_equal(taps, taps_o)
    if d > 1:
        assert fs % d == 0 and d <= fs / opt
        assert len(taps) % 2 == 1 and np.allclose(taps, taps[::-1], rtol=0, atol=1e-7)  # float window: symmetric to an ulp
        assert abs(float(np.sum(taps, dtype=np.float64)) - 1.0) < 1e-6
        # stop band: past the transition band the response is down ≥ 40 dB (Hamming design)
        f = np.linspace(0, fs / 2, 4001)
        H = np.abs(np.exp(-2j * np.pi * np.outer(f / fs, np.arange(len(taps)))) @ taps.astype(np.float64))
        fdec = fs / d
        assert H[f >= fdec / 2.1 + fdec / 2].max() < 10 ** (-40 / 20)
    else:
        assert len(taps) == 0


def test_firdes_counts_and_errors(lib):
    for fs, cut, tw in [(1e6, 1e5, 5e4), (25e6, 1.19e6, 1.25e6), (8e6, 3e6, 1e5)]:
        t = engine.firdes_low_pass(lib, 1.0, fs, cut, tw)
        n = int(53.0 * fs / (22.0 * tw))
        assert len(t) == (n if n % 2 else n + 1)
        assert np.array_equal(t, O.firdes_low_pass(1.0, fs, cut, tw))
    t2 = engine.firdes_low_pass(lib, 2.5, 1e6, 1e5, 5e4)
    assert abs(float(t2.astype(np.float64).sum()) - 2.5) < 1e-5
    for bad in [(1.0, 1e6, 6e5, 1e4), (1.0, 0.0, 1e5, 1e4), (1.0, 1e6, 1e5, 0.0), (1.0, 1e6, -1.0, 1e4)]:
        with pytest.raises(abi.GnssHipError):
            engine.firdes_low_pass(lib, *bad)


def test_oracle_fir_streaming_equals_one_shot(built):
    rng = np.random.default_rng(5)
    d, taps = O.acq_resampler_design(25000000, 2e6)
    x = (rng.standard_normal(20 * d * 37) + 1j * rng.standard_normal(20 * d * 37)).astype(np.complex64)
    one = O.FirDecimator(taps, d)(x)
    f = O.FirDecimator(taps, d)
    parts = [f(x[a:b]) for a, b in [(0, d), (d, 11 * d), (11 * d, 500 * d), (500 * d, len(x))]]
    assert np.array_equal(np.concatenate(parts), one)
    # against a double-precision convolution with zero history
    ref = np.convolve(x.astype(np.complex128), taps.astype(np.float64))[: len(x)][::d]
    assert np.max(np.abs(one - ref)) < 1e-5 * np.max(np.abs(ref))

"""trk_lane_kernel (trk_lane.hip) — the AVX engine's throughput form, one 16-lane row per channel —
forced on (GNSSHIP_TRK_LANE=1) for the configurations the latency-form tests cover, and held bit for
bit to the oracle loop: every record field (compare_exact) and, where traced, every tap on the
device's own arguments (trace_exact).  The cases cover the three systems' tap layouts (3 taps; E1's 5
taps + the data prompt), the N mod 16 tail of u_avx (:294-308: GPS at 25 Msps N = 25000 has 8 tail
samples, B1I at 4.092 Msps 12, E1 at 6.25 Msps 8), the ibyte format with the IF in the NCO (C5), the
extended-integration state 3, the renormalisation cadence over long epochs (E1 at 25 Msps,
N = 100000), several channels per wave in different states, and the fallback to trk_fast's
throughput form when a code is not ±1 (the sign-bit replica needs ±1 chips)."""
import numpy as np
import pytest

from gnss_sim_receiver_amd import abi, engine, signals
from oracle import trk as T

import test_gpu_c5_closed_loop as C5
import trk_scenarios as S
from test_gpu_trk import compare_exact, dev_conf
from test_gpu_trk_persist import run_pair

pytestmark = pytest.mark.gpu


@pytest.fixture
def lane(monkeypatch):
    monkeypatch.setenv("GNSSHIP_TRK_LANE", "1")


@pytest.mark.parametrize("system,fs,epochs", [("GPS", 4e6, 700), ("GAL", 25e6 / 4, 90), ("BDS", 4.092e6, 300), ("GPS", 25e6, 200),
                                              ("GAL", 25e6, 60)])
def test_lane_loop_matches_oracle(ctx, lane, system, fs, epochs):
    rec, rounds, ref = run_pair(ctx, system, fs, epochs, avx=True)
    assert ref["state"][-1] == 4
    compare_exact(rec[:, 1], ref, f"lane {system} {fs / 1e6:g} Msps")
    assert not np.any(rec[:, 0]["flags"])  # the idle channel (same wave) never ran


@pytest.mark.parametrize("system,epochs", [("GPS", 300), ("GAL", 60), ("BDS", 300)])
def test_lane_c5_ibyte_if(ctx, lane, system, epochs):
    C5.test_c5_channel_closed_loop_ibyte_if(ctx, system, epochs, True)


@pytest.mark.parametrize("system,fs,epochs,ext", [("GPS", 4e6, 500, 10), ("GAL", 25e6 / 4, 110, 4)])
def test_lane_extended_integration(ctx, lane, system, fs, epochs, ext):
    rec, rounds, ref = run_pair(ctx, system, fs, epochs, avx=True, extend_correlation_symbols=ext)
    st = ref["state"]
    assert np.sum(st == 3) >= 3 * (ext - 1) and np.sum(st == 4) >= 3
    compare_exact(rec[:, 1], ref, f"lane {system} x{ext}")


def test_lane_channels_in_different_states(ctx, lane):
    """Nine GPS channels (three waves' rows, one partly filled): three synchronised, three still in
    the pull-in (state 2), one that loses lock half way (noise only after 0.3 s), two idle — each
    row's records equal its own oracle loop."""
    fs, vl, epochs = 4e6, 4000, 600
    sats = signals.random_sky(8, seed=0x6E550021)
    for s in sats:
        s.bits = "1000101100110"
    k = T.conf("GPS", fs, vl, rotator_avx=1)
    first = int(11 * fs)
    x = signals.generate_if(fs, vl * (epochs + 4), sats[:6], seed=0x6E550022, start=first).astype(np.complex64)
    lost = signals.generate_if(fs, vl * (epochs + 4), sats[6:7], seed=0x6E550023, start=first).astype(np.complex64)
    cut = int(0.3 * fs)
    lost[cut:] = 0
    x = x + lost
    trk = engine.DllPllVemlTracking(ctx, dev_conf(k, "GPS"), 9)
    starts = {}
    for ch in range(9):
        if ch in (4, 8):
            continue  # idle rows
        s = sats[ch if ch < 4 else ch - 1]
        ctx.set_code(500 + ch, s.code)
        stamp = 0 if ch % 3 else first - int(2 * fs)  # a recent stamp keeps these channels in the pull-in
        delay = signals.acq_delay_samples(s, fs, stamp, first) + 0.2 * (ch % 3 - 1)
        trk.start(ch, 500 + ch, delay, s.doppler_hz + 3.0 * (ch % 4 - 1.5), stamp, first)
        starts[ch] = (s, delay, s.doppler_hz + 3.0 * (ch % 4 - 1.5), stamp)
    rec, rounds = trk.run(x, first, epochs)
    assert trk.last_engine() == abi.TRK_ENGINE_LANES
    trk.close()
    states = set()
    for ch, (s, delay, dop, stamp) in starts.items():
        ref = T.track(k, x, s.code, delay, dop, stamp, first, epochs, buffer_first=first)
        states |= set(np.unique(ref["state"]).tolist())
        compare_exact(rec[:, ch], ref, f"lane row ch{ch}")
    for ch in (4, 8):
        assert not np.any(rec[:, ch]["flags"])
    assert {2, 4} <= states


def test_non_binary_code_falls_back_to_trk_fast(lane):
    """A code with a chip other than ±1 cannot take the sign-bit replica: the AVX engine then runs
    trk_fast's throughput form (and stays exact)."""
    own = engine.Context(0)
    try:
        sat, k, x, stamp, first, delay, dop = S.sync("GPS", 4e6, 200, rotator_avx=1)
        code = sat.code.astype(np.float32) * np.float32(0.5)
        trk = engine.DllPllVemlTracking(own, dev_conf(k, "GPS"), 1)
        own.set_code(7, code)
        trk.start(0, 7, delay, dop, stamp, first)
        rec, rounds = trk.run(x, first, 200)
        assert trk.last_engine() in (abi.TRK_ENGINE_FAST_LATENCY, abi.TRK_ENGINE_FAST_THROUGHPUT)
        trk.close()
        ref = T.track(k, x, code, delay, dop, stamp, first, 200, buffer_first=first)
        compare_exact(rec[:, 0], ref, "non-binary code")
    finally:
        own.close()

"""The AVX tracking engine's throughput forms — with more channels than compute units the default
dispatch runs trk_lane_kernel (one 16-lane row per channel, trk_lane.hip), the kernel behind bench.py's
tracked_channels_sustained; trk_fast_kernel's throughput form (two workgroups per CU) is the fallback
for codes that are not ±1.  Both keep u_avx's accumulation order (volk_gnsssdr_32fc_32f_rotator_dot_
prod_32fc_xn.h:220-308), so a sample of channels out of a 1024-channel run is held bit for bit to the
oracle: every traced epoch's taps on the device's own arguments (trace_exact) and every record field
against the oracle loop (compare_exact).

Channels c take satellite c mod 32 of one sky (as the bench's sweep does); each channel starts at its
own code-delay and Doppler offset, so channels sharing a satellite run different loops."""
import concurrent.futures as cf

import numpy as np
import pytest

from gnss_sim_receiver_amd import abi, engine, signals
from oracle import trk as T

from test_gpu_c5_closed_loop import trace_exact
from test_gpu_trk import compare_exact, dev_conf

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("form", ["default", "trk_fast"])
def test_1024_avx_channels_default_dispatch_exact(ctx, form, monkeypatch):
    if form == "trk_fast":
        monkeypatch.setenv("GNSSHIP_TRK_LANE", "0")
    fs, vl, n_ch, epochs = 4e6, 4000, 1024, 700
    sats = signals.random_sky(32, seed=0x6E550012)
    for s in sats:
        s.bits = "1000101100110"  # navigation bits with the preamble: the channels bit-synchronise (state 4)
    k = T.conf("GPS", fs, vl, rotator_avx=1)
    first = int(11 * fs)  # acquisition stamped at sample 0: the 10 s pull-in is over (bench.py's sweep)
    x = signals.generate_if(fs, vl * (epochs + 4), sats, seed=0x6E550013, start=first)
    trk = engine.DllPllVemlTracking(ctx, dev_conf(k, "GPS"), n_ch)
    for i, s in enumerate(sats):
        ctx.set_code(400 + i, s.code)
    starts = []
    for ch in range(n_ch):
        s = sats[ch % 32]
        lap = ch // 32  # 0..31: the start offsets of the channels that share satellite ch mod 32
        delay = signals.acq_delay_samples(s, fs, 0, first) + 0.37 * ((lap * 7) % 5 - 2) / 2.0
        dop = s.doppler_hz + 2.5 * ((lap * 11) % 9 - 4)
        trk.start(ch, 400 + ch % 32, delay, dop, 0, first)
        starts.append((delay, dop))
    trk.set_trace(True)
    rec, rounds = trk.run(x, first, epochs)
    assert rounds == epochs
    want = abi.TRK_ENGINE_LANES if form == "default" else abi.TRK_ENGINE_FAST_THROUGHPUT
    assert trk.last_engine() == want, abi.TRK_ENGINE_NAMES[trk.last_engine()]
    tr = trk.trace(epochs)
    states = trk.states()
    trk.close()
    xf = x.astype(np.complex64)
    sample = [0, 33, 100, 257, 511, 700, 901, 1023]

    def oracle(ch):
        s = sats[ch % 32]
        return T.track(k, xf, s.code, starts[ch][0], starts[ch][1], 0, first, epochs, buffer_first=first)

    with cf.ThreadPoolExecutor(8) as ex:
        refs = dict(zip(sample, ex.map(oracle, sample)))
    n_traced = 0
    for ch, ref in refs.items():
        label = f"throughput form ch{ch}"
        n_traced += trace_exact(tr[:, ch], xf, first, sats[ch % 32].code, None, label)
        compare_exact(rec[:, ch], ref, label)
        assert np.count_nonzero(ref["state"] == 4) > 0, (label, "the sampled channel never reached state 4")
    assert n_traced >= 8 * 500
    assert np.mean(states >= 2) >= 0.95, np.bincount(states)


def test_512_avx_channels_25msps_default_dispatch_exact(ctx):
    """north_star's second rate: 512 GPS L1 C/A channels at 25 Msps (N = 25000 = 1562 u_avx iterations
    + an 8-sample serial tail, gps_l1_ca_dll_pll_tracking.cc:47) through the default dispatch — the
    lane form behind bench.py's tracked_channels_sustained_25msps.  Eight sampled channels bit for bit:
    traced taps on the device's own arguments and every record field against the oracle loop."""
    fs, vl, n_ch, epochs = 25e6, 25000, 512, 300
    sats = signals.random_sky(32, seed=0x6E550022)
    for s in sats:
        s.bits = "1000101100110"
    k = T.conf("GPS", fs, vl, rotator_avx=1)
    first = int(11 * fs)
    x = signals.generate_if_device(fs, vl * (epochs + 4), sats, seed=0x6E550023, start=first, device="cpu").numpy()
    trk = engine.DllPllVemlTracking(ctx, dev_conf(k, "GPS"), n_ch)
    for i, s in enumerate(sats):
        ctx.set_code(700 + i, s.code)
    starts = []
    for ch in range(n_ch):
        s = sats[ch % 32]
        lap = ch // 32
        delay = signals.acq_delay_samples(s, fs, 0, first) + 2.3 * ((lap * 7) % 5 - 2) / 2.0
        dop = s.doppler_hz + 2.5 * ((lap * 11) % 9 - 4)
        trk.start(ch, 700 + ch % 32, delay, dop, 0, first)
        starts.append((delay, dop))
    trk.set_trace(True)
    rec, rounds = trk.run(x, first, epochs)
    assert rounds == epochs
    assert trk.last_engine() == abi.TRK_ENGINE_LANES, abi.TRK_ENGINE_NAMES[trk.last_engine()]
    tr = trk.trace(epochs)
    states = trk.states()
    trk.close()
    xf = x.astype(np.complex64)
    sample = [0, 45, 130, 255, 256, 377, 480, 511]

    def oracle(ch):
        s = sats[ch % 32]
        return T.track(k, xf, s.code, starts[ch][0], starts[ch][1], 0, first, epochs, buffer_first=first)

    with cf.ThreadPoolExecutor(8) as ex:
        refs = dict(zip(sample, ex.map(oracle, sample)))
    for ch, ref in refs.items():
        label = f"25 Msps lane form ch{ch}"
        trace_exact(tr[:, ch], xf, first, sats[ch % 32].code, None, label)
        compare_exact(rec[:, ch], ref, label)
    assert np.mean(states >= 2) >= 0.95, np.bincount(states)

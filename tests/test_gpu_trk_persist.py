"""Persistent closed loop (trk_persist.hip: one workgroup per channel for a whole run) vs the oracle
loop (oracle/trk_oracle.c), for both volk_gnsssdr rotator variants the reference can dispatch
(generic, and u_avx/a_avx: volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn.h:155-316), and at the
north_star's 25 Msps rates (GPS L1 C/A N = 25000, Galileo E1 N = 100000 — C3/C4's sampling rate).

The AVX variant runs trk_fast.hip, which reproduces u_avx's products and accumulation order, glibc's
phasor trig and the loop's libm calls; the generic variant runs trk_persist.hip's serial pipeline,
which reproduces the generic rotator's phasor chain and its one serial float sum per tap component.
Both variants' records equal the oracle loop's (test_gpu_trk.compare_exact).
"""
import os

import numpy as np
import pytest

from gnss_sim_receiver_amd import abi, engine
from oracle import trk as T

import trk_scenarios as S
from test_gpu_trk import compare_exact, dev_conf

pytestmark = pytest.mark.gpu


def run_pair(ctx, system, fs, epochs, avx, n_ch=2, **kw):
    """One channel (index 1) synchronising to state 4 on the device and in the oracle (both rotator
    variants sum in the reference's own order and are compared with the plain oracle)."""
    sat, k, x, stamp, first, delay, dop = S.sync(system, fs, epochs, rotator_avx=1 if avx else 0, **kw)
    c = dev_conf(k, system)
    c.rotator = abi.ROTATOR_AVX if avx else abi.ROTATOR_GENERIC
    trk = engine.DllPllVemlTracking(ctx, c, n_ch)
    ctx.set_code(40, sat.code)
    if sat.code_data is not None:
        ctx.set_code(41, sat.code_data)
    trk.start(1, 40, delay, dop, stamp, first, data_code_id=41)
    rec, rounds = trk.run(x, first, epochs)
    trk.close()
    ref = T.track(k, x, sat.code, delay, dop, stamp, first, epochs, data_code=sat.code_data, buffer_first=first)
    return rec, rounds, ref


@pytest.mark.parametrize("system,fs,epochs", [("GPS", 4e6, 700), ("GAL", 25e6 / 4, 90), ("BDS", 4.092e6, 300)])
def test_avx_rotator_loop_matches_oracle(ctx, system, fs, epochs):
    rec, rounds, ref = run_pair(ctx, system, fs, epochs, avx=True)
    assert ref["state"][-1] == 4
    compare_exact(rec[:, 1], ref, f"{system} avx")
    assert not np.any(rec[:, 0]["flags"])  # the idle channel never ran


@pytest.mark.parametrize("avx", [False, True])
@pytest.mark.parametrize("system,epochs", [("GPS", 300), ("GAL", 90)])
def test_closed_loop_25msps_matches_oracle(ctx, system, epochs, avx):
    """The closed loop at 25 Msps: GPS L1 C/A N = 25000 (north_star's second rate) and Galileo E1
    N = 100000 with the data prompt (configs[3]'s per-channel epoch, dll_pll_veml_tracking.cc:1728-2094)."""
    rec, rounds, ref = run_pair(ctx, system, 25e6, epochs, avx=avx)
    assert ref["state"][-1] == 4
    compare_exact(rec[:, 1], ref, f"{system} 25 Msps avx={avx}")


def test_galileo_e1_50msps_avx_matches_oracle(ctx):
    """E1 at 50 Msps (configs[4]'s N = 200000) with the AVX rotator: 12500-step phasor chains, the
    phasor slots and the products in LDS rings (trk_fast.hip fast_plan)."""
    rec, rounds, ref = run_pair(ctx, "GAL", 50e6, 40, avx=True)
    compare_exact(rec[:, 1], ref, "GAL 50 Msps avx")


@pytest.mark.parametrize("lds_kib", [36, 64])
def test_fast_kernel_rings_match_oracle(ctx, lds_kib, monkeypatch):
    """The same GPS 4 Msps loop with the LDS budget cut (GNSSHIP_TRK_FAST_LDS) so that the product
    ring holds only a few of the epoch's eight groups (36 KiB: 2 groups, 64 KiB: 4, with
    back-pressure on the producers) — still equal to the oracle."""
    monkeypatch.setenv("GNSSHIP_TRK_FAST_LDS", str(lds_kib))
    own = engine.Context(0)  # only GPS codes: the LDS replica is sized by the context's longest code
    try:
        rec, rounds, ref = run_pair(own, "GPS", 4e6, 300, avx=True)
    finally:
        own.close()
    compare_exact(rec[:, 1], ref, f"GPS rings {lds_kib} KiB")


def test_fast_kernel_slot_ring_matches_oracle(ctx, monkeypatch):
    """GPS at 25 Msps (196 tasks per epoch) with a budget that forces the phasor slots into their
    64-task ring and the products into a 2-group ring."""
    monkeypatch.setenv("GNSSHIP_TRK_FAST_LDS", "40")
    own = engine.Context(0)
    try:
        rec, rounds, ref = run_pair(own, "GPS", 25e6, 120, avx=True)
    finally:
        own.close()
    compare_exact(rec[:, 1], ref, "GPS 25 Msps slot ring")


def test_persistent_loop_matches_round_based_loop(ctx):
    """The persistent kernel and the round-based step/correlate launches (GNSSHIP_TRK_ROUNDS=1)
    run the same loop code on the same generic-rotator correlations: records agree to the
    correlations' summation-order differences."""
    sat, k, x, stamp, first, delay, dop = S.sync("GPS", 4e6, 400)
    out = []
    for rounds_env in ("1", None):
        if rounds_env:
            os.environ["GNSSHIP_TRK_ROUNDS"] = rounds_env
        try:
            trk = engine.DllPllVemlTracking(ctx, dev_conf(k, "GPS"), 3)
        finally:
            os.environ.pop("GNSSHIP_TRK_ROUNDS", None)
        ctx.set_code(50, sat.code)
        trk.start(2, 50, delay, dop, stamp, first)
        rec, n = trk.run(x, first, 400)
        trk.close()
        out.append(rec[:, 2])
    a, b = out
    for f in ("sample_counter", "state", "flags", "prn_length_samples"):
        assert np.array_equal(a[f], b[f]), f
    np.testing.assert_allclose(a["carrier_doppler_hz"], b["carrier_doppler_hz"], rtol=0, atol=1e-3)
    np.testing.assert_allclose(a["rem_code_phase_chips"], b["rem_code_phase_chips"], rtol=0, atol=1e-6)


def test_many_channels_and_ragged_buffers(ctx):
    """64 channels, 2 runs over consecutive buffers: each channel resumes where the previous
    buffer left it (its next window straddles the boundary), as general_work's consume_each does."""
    fs, vl, n_ch = 4e6, 4000, 64
    from gnss_sim_receiver_amd import signals
    rng = np.random.default_rng(9)
    sats = [signals.Satellite(prn=1 + (i % 32), doppler_hz=float(rng.uniform(-4000, 4000)), code_delay_chips=float(rng.uniform(0, 1023)),
                              cn0_dbhz=48.0, carrier_phase_rad=float(rng.uniform(0, 6.28))) for i in range(n_ch)]
    k = T.conf("GPS", fs, vl)
    x = signals.generate_if(fs, vl * 130, sats[:8], seed=4)  # 8 real signals; the other channels track noise and lose lock
    trk = engine.DllPllVemlTracking(ctx, dev_conf(k, "GPS"), n_ch)
    starts = []
    for ch, s in enumerate(sats):
        delay = (s.code_delay_chips / s.code_freq()) * fs
        ctx.set_code(100 + ch, s.code)
        trk.start(ch, 100 + ch, delay, s.doppler_hz + 5.0, 0, 0)
        starts.append((delay, s.doppler_hz + 5.0))
    half = vl * 64 + 1234
    r1, n1 = trk.run(x[:half], 0, 200)
    r2, n2 = trk.run(x[half - vl - 100:], half - vl - 100, 200)
    trk.close()
    for ch in (0, 5, 7, 40):
        ref = T.track(k, x, sats[ch].code, starts[ch][0], starts[ch][1], 0, 0, 200)
        d = np.concatenate([r1[:, ch][(r1[:, ch]["flags"] & 8) == 8], r2[:, ch][(r2[:, ch]["flags"] & 8) == 8]])
        compare_exact(d[:len(ref)], ref[:len(d)], f"ch{ch}")


@pytest.mark.parametrize("avx", [False, True])
def test_telemetry_fault_forces_loss_of_lock(ctx, avx):
    """msg_handler_telemetry_to_trk (dll_pll_veml_tracking.cc:617-640): a telemetry fault between
    two runs sets the carrier lock-fail counter to 200000; the next epoch's lock check declares loss
    of lock — the same epoch, with the same record, as the oracle loop given the same event."""
    sat, k, x, stamp, first, delay, dop = S.sync("GPS", 4e6, 300, rotator_avx=1 if avx else 0)
    c = dev_conf(k, "GPS")
    c.rotator = abi.ROTATOR_AVX if avx else abi.ROTATOR_GENERIC
    trk = engine.DllPllVemlTracking(ctx, c, 1)
    ctx.set_code(60, sat.code)
    trk.start(0, 60, delay, dop, stamp, first)
    ref_ch = T.Channel(k, sat.code, delay, dop, stamp, first)
    r1, _ = trk.run(x, first, 120)
    o1 = ref_ch.run(x, first, 120)
    cmp = compare_exact
    cmp(r1[:, 0], o1, "before")
    trk.telemetry_event(0, 2)  # not a fault: ignored
    trk.telemetry_event(0, 1)
    ref_ch.telemetry_fault()
    r2, _ = trk.run(x, first, 20)
    o2 = ref_ch.run(x, first, 20)
    d = r2[:, 0][(r2[:, 0]["flags"] & 8) == 8]
    assert len(d) == len(o2) == 1 and (d["flags"][0] & 2) and (o2["flags"][0] & 2)
    cmp(r2[:, 0], o2, "fault epoch")
    assert trk.channel_state(0)[0] == 0
    trk.close()


def test_c4_share_8_e1_channels_closed_loop_matches_oracle(ctx):
    """configs[3] (C4)'s per-GPU share in closed loop: 8 Galileo E1 B/C channels (5 VEML pilot taps +
    the data prompt, N = 100000 at 25 Msps, AVX rotator) on one engine, eight satellites in one
    signal, 90 epochs each (synchronised to the CS25 pilot code, state 4), every channel against the
    plain oracle loop on the same signal: every traced channel-epoch's taps and data prompt equal the
    oracle correlator's on the device's own arguments, and the records equal the oracle loop's."""
    import concurrent.futures as cf

    from gnss_sim_receiver_amd import signals
    from test_gpu_c5_closed_loop import trace_exact

    fs, epochs = 25e6, 90
    prns = [1, 5, 12, 19, 24, 30, 33, 36]
    sats = [signals.Satellite(prn=p, doppler_hz=-3000.0 + 800.0 * i, code_delay_chips=150.3 + 417.0 * i, cn0_dbhz=50.0, system="GAL",
                              carrier_phase_rad=0.3 * i, **S.SYNC_PATTERNS["GAL"]) for i, p in enumerate(prns)]
    k = T.conf("GAL", fs, int(round(fs * T.SYSTEMS["GAL"][2])), pull_in_time_s=0, rotator_avx=1)
    first = int(fs)
    x = signals.generate_if(fs, int(round(fs)) // 4 + k.vector_length * (epochs + 3), sats, seed=0x6E550004, start=first)
    c = dev_conf(k, "GAL")
    c.rotator = abi.ROTATOR_AVX
    trk = engine.DllPllVemlTracking(ctx, c, len(sats))
    starts = []
    for ch, s in enumerate(sats):
        ctx.set_code(60 + 2 * ch, s.code)
        ctx.set_code(61 + 2 * ch, s.code_data)
        starts.append((S.acq_delay_for(s, fs, "GAL", 0, first) + 0.2, s.doppler_hz + 15.0))
        trk.start(ch, 60 + 2 * ch, starts[-1][0], starts[-1][1], 0, first, data_code_id=61 + 2 * ch, prn=s.prn)
    trk.set_trace(True)
    rec, rounds = trk.run(x, first, epochs)
    tr = trk.trace(epochs)
    trk.close()

    def oracle(ch):
        s = sats[ch]
        return T.track(k, x, s.code, starts[ch][0], starts[ch][1], 0, first, epochs, data_code=s.code_data, buffer_first=first, prn=s.prn)

    with cf.ThreadPoolExecutor(8) as ex:
        refs = list(ex.map(oracle, range(len(sats))))
    for ch, ref in enumerate(refs):
        assert ref["state"][-1] == 4, (ch, np.bincount(ref["state"]))
        label = f"C4 share channel {ch} (PRN {sats[ch].prn})"
        trace_exact(tr[:, ch], x, first, sats[ch].code, sats[ch].code_data, label)
        compare_exact(rec[:, ch], ref, label)


def test_c4_full_64_e1_channels_one_engine(ctx):
    """configs[3] (C4) at its BASELINE channel count on one GPU: 64 Galileo E1 B/C channels (PRNs 1-36,
    then PRNs re-used with their own Doppler / delay / phase) on one engine at 25 Msps,
    90 epochs.  Eight sampled channels bit for bit against the oracle (traced taps and records); all
    64 synchronised to the CS25 pilot code (state 4)."""
    import concurrent.futures as cf

    from gnss_sim_receiver_amd import signals
    from test_gpu_c5_closed_loop import if_on_device, trace_exact

    fs, epochs = 25e6, 90
    rng = np.random.default_rng(0x6E550007)
    prns = (list(range(1, 37)) * 2)[:64]
    sats = [signals.Satellite(prn=p, doppler_hz=float(rng.uniform(-4000, 4000)), code_delay_chips=float(rng.uniform(0, 4000)), cn0_dbhz=48.0,
                              system="GAL", carrier_phase_rad=float(rng.uniform(0, 6.28)), **S.SYNC_PATTERNS["GAL"]) for p in prns]
    k = T.conf("GAL", fs, int(round(fs * T.SYSTEMS["GAL"][2])), pull_in_time_s=0, rotator_avx=1)
    first = int(fs)
    x = if_on_device(fs, int(round(fs)) // 4 + k.vector_length * (epochs + 3), sats, seed=0x6E550007, start=first)
    c = dev_conf(k, "GAL")
    c.rotator = abi.ROTATOR_AVX
    trk = engine.DllPllVemlTracking(ctx, c, len(sats))
    starts = []
    for ch, s in enumerate(sats):
        ctx.set_code(400 + 2 * ch, s.code)
        ctx.set_code(401 + 2 * ch, s.code_data)
        starts.append((S.acq_delay_for(s, fs, "GAL", 0, first) + 0.2, s.doppler_hz + 15.0))
        trk.start(ch, 400 + 2 * ch, starts[-1][0], starts[-1][1], 0, first, data_code_id=401 + 2 * ch, prn=s.prn)
    trk.set_trace(True)
    rec, rounds = trk.run(x, first, epochs)
    tr = trk.trace(epochs)
    st = trk.states()
    trk.close()
    assert np.all(st == 4), np.bincount(st)
    sample = [0, 9, 18, 27, 36, 45, 54, 63]

    def oracle(ch):
        s = sats[ch]
        return T.track(k, x, s.code, starts[ch][0], starts[ch][1], 0, first, epochs, data_code=s.code_data, buffer_first=first, prn=s.prn)

    with cf.ThreadPoolExecutor(8) as ex:
        refs = list(ex.map(oracle, sample))
    for ch, ref in zip(sample, refs):
        label = f"C4 full channel {ch} (PRN {sats[ch].prn})"
        trace_exact(tr[:, ch], x, first, sats[ch].code, sats[ch].code_data, label)
        compare_exact(rec[:, ch], ref, label)

"""configs[4] (C5) in closed loop: GPS L1 C/A, Galileo E1 B/C and BeiDou B1I tracked from one 50 Msps
ibyte block whose IF is centred at 1568.259 MHz — +7.161 MHz for L1/E1, −7.161 MHz for B1I (SURVEY
§8d C5).  The reference removes each signal's IF ahead of the channels (InputFilter.IF,
conf/gnss-sdr_BDS_B3I_GPS_L1_CA_ibyte.conf:45-92); the engine fuses it into the correlator's carrier
NCO (gnsship_trk_conf::if_hz) and the oracle loop (oracle/trk_oracle.c, orc_trk_conf::if_hz) applies
the same term, so every epoch of dll_pll_veml_tracking::general_work (:1728-2094) is compared.

The int8 samples go to the device as they are (converted in the loads, no scaling, as IbyteToComplex,
ibyte_to_complex.cc:39) and to the oracle converted to float.

With the IF in the NCO the phase step is ≈ 0.9 rad per sample, and one ulp of phase_inc turns the
carrier by ≈ 3e-3 rad over 50000 samples: the phasors must be glibc's cosf / sinf exactly, which the
engine reproduces (glibc_sincosf.h).  Both engines then equal the oracle: the AVX engine
(trk_fast.hip) sums in u_avx's order, the generic engine (trk_persist.hip) keeps the generic rotator's
one serial float sum per tap component (volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn.h:66-98);
every traced epoch's taps equal the oracle correlator's on the same arguments, and every record
field equals the oracle loop's (test_gpu_trk.compare_exact).  compare_if (the IF loop's bounds for
two loops whose sums differ in order) is kept for callers that compare across variants.
"""
import concurrent.futures as cf

import numpy as np
import pytest

from gnss_sim_receiver_amd import abi, engine, signals
from oracle import trk as T

import trk_scenarios as S
from test_gpu_trk import compare_exact, dev_conf

pytestmark = pytest.mark.gpu
TOL = 1e-5


def compare_if(dev, ref, label, kick_frac=0.0, kick_scale=1.0):
    """test_gpu_trk.compare with the IF loop's Doppler / carrier-phase bounds (module docstring).
    kick_frac > 0 (long runs): up to that fraction of the epochs may exceed a bound, by at most
    kick_scale × the bound — the one-epoch discriminator kicks that the loops' ~1e-7 correlation
    sum differences occasionally cause (test_gpu_headline_pin.py), which the PLL then carries for a
    few epochs; epoch boundaries, states and flags stay exact either way."""
    d = dev[(dev["flags"] & 8) == 8]
    assert len(d) == len(ref), (label, len(d), len(ref))
    for f in ("sample_counter", "state", "prn_length_samples"):
        assert np.array_equal(d[f], ref[f]), (label, f, np.nonzero(d[f] != ref[f])[0][:5])
    assert np.array_equal(d["flags"] & 7, ref["flags"] & 7), label
    # Doppler 0.25 Hz; the DLL sees the same phase-step kicks: code frequency 5e-2 Hz (5e-8
    # relative); the code NCO integrates that frequency difference: 5e-2 Hz over a 4 ms E1 epoch is
    # 2e-4 chips; CN0 5e-2 dB; accumulated carrier phase 5e-2 rad
    for f, tol in (("carrier_doppler_hz", 0.25), ("code_freq_chips", 5e-2), ("rem_code_phase_chips", 2e-4), ("cn0_db_hz", 5e-2),
                   ("carrier_phase_rads", 5e-2)):
        err = np.abs(d[f] - ref[f])
        if kick_frac > 0.0:
            assert np.mean(err > tol) <= kick_frac and err.max() <= kick_scale * tol, (label, f, float(np.mean(err > tol)), float(err.max()))
        else:
            np.testing.assert_allclose(d[f], ref[f], rtol=0, atol=tol, err_msg=f"{label} {f}")


def check_trace(tr, xf, first, codes, data_code=None):
    """Each traced channel-epoch re-run on the oracle correlator with the device's own arguments:
    taps within 1e-5 of max(|ref|, ‖x‖₂) (the E1 long-integration scale, test_gpu_e1.py), the oracle
    summing its float products in double at N ≥ 1e5."""
    from gnss_sim_receiver_amd import abi as A
    from oracle import oracle as O
    tr = tr[tr["n_samples"] > 0]
    assert len(tr) > 0
    jobs = np.zeros(len(tr), A.JOB_DTYPE)
    jobs["sample_offset"] = tr["sample_counter"].astype(np.int64) - first
    jobs["n_samples"] = tr["n_samples"]
    jobs["n_taps"] = tr["n_taps"]
    jobs["flags"] = 0
    jobs["rem_carrier_phase_rad"] = tr["rem_carrier_phase_rad"]
    jobs["phase_step_rad"] = tr["phase_step_rad"]
    jobs["rem_code_phase_chips"] = tr["rem_code_phase_samples"]
    jobs["code_phase_step_chips"] = tr["code_phase_step_samples"]
    jobs["shifts_chips"][:, :5] = tr["shifts"]
    return jobs


def trace_errors(tr, xf, first, code, data_code, rotator_avx, long_n=None):
    """Worst per-tap relative error of the traced taps against the oracle correlator on the device's
    own arguments.  long_n (default: N ≥ 1e5) compares with the oracle's float products summed in
    double, scaled by max(|ref|, ‖x‖₂); otherwise with the reference's serial float sum, scaled by |ref|."""
    from gnss_sim_receiver_amd import abi as A
    from oracle import oracle as O
    tr = tr[tr["n_samples"] > 0]
    jobs = check_trace(tr, xf, first, [code])
    jobs["code_id"] = 0
    jobs["flags"] = A.JOB_ROTATOR_AVX if rotator_avx else 0
    if long_n is None:
        long_n = int(jobs["n_samples"][0]) >= 100000
    ref = O.corr_batch(xf, jobs, [code], n_threads=8, accum_f64=long_n)
    worst = 0.0
    for j in range(len(jobs)):
        t = int(jobs["n_taps"][j])
        o, n = int(jobs["sample_offset"][j]), int(jobs["n_samples"][j])
        scale = max(float(np.max(np.abs(ref[j, :t]))), float(np.linalg.norm(xf[o:o + n].astype(np.complex128))) if long_n else 0.0)
        got = tr["taps"][j, 0:2 * t:2] + 1j * tr["taps"][j, 1:2 * t:2]
        e = np.abs(got - ref[j, :t]) / np.maximum(np.abs(ref[j, :t]), scale if long_n else 1e-30)
        worst = max(worst, float(e.max()))
    if data_code is not None:
        dj = jobs.copy()
        dj["n_taps"] = 1
        dj["shifts_chips"] = 0.0
        dref = O.corr_batch(xf, dj, [data_code], n_threads=8, accum_f64=long_n)
        got = tr["data_prompt"][:, 0] + 1j * tr["data_prompt"][:, 1]
        for j in range(len(dj)):
            o, n = int(dj["sample_offset"][j]), int(dj["n_samples"][j])
            scale = max(abs(dref[j, 0]), float(np.linalg.norm(xf[o:o + n].astype(np.complex128))) if long_n else 0.0)
            worst = max(worst, abs(got[j] - dref[j, 0]) / max(scale, 1e-30))
    return worst


def trace_exact(tr, xf, first, code, data_code, label="", avx=True):
    """Each traced channel-epoch re-run on the oracle correlator of the engine's rotator variant (u_avx,
    or the generic serial one) with the device's own arguments: every tap (and the data prompt)
    equal, bit for bit."""
    from gnss_sim_receiver_amd import abi as A
    from oracle import oracle as O
    tr = tr[tr["n_samples"] > 0]
    jobs = check_trace(tr, xf, first, [code])
    jobs["code_id"] = 0
    jobs["flags"] = A.JOB_ROTATOR_AVX if avx else 0
    ref = O.corr_batch(xf, jobs, [code], n_threads=8).astype(np.complex64)
    t = int(jobs["n_taps"][0])
    got = (tr["taps"][:, 0:2 * t:2] + 1j * tr["taps"][:, 1:2 * t:2]).astype(np.complex64)
    bad = np.nonzero(np.any(got != ref[:, :t], axis=1))[0]
    assert len(bad) == 0, (label, "taps differ in", len(bad), "of", len(jobs), "epochs; first", int(bad[0]), got[bad[0]], ref[bad[0], :t])
    if data_code is not None:
        dj = jobs.copy()
        dj["n_taps"] = 1
        dj["shifts_chips"] = 0.0
        dref = O.corr_batch(xf, dj, [data_code], n_threads=8).astype(np.complex64)[:, 0]
        dgot = (tr["data_prompt"][:, 0] + 1j * tr["data_prompt"][:, 1]).astype(np.complex64)
        bad = np.nonzero(dgot != dref)[0]
        assert len(bad) == 0, (label, "data prompt differs in", len(bad), "epochs; first", int(bad[0]), dgot[bad[0]], dref[bad[0]])
    return len(jobs)


FS = 50e6
F_IF = 7.161e6
IF_OF = {"GPS": F_IF, "GAL": F_IF, "BDS": -F_IF}


@pytest.mark.parametrize("avx", [False, True])
@pytest.mark.parametrize("system,epochs", [("GPS", 300), ("GAL", 60), ("BDS", 300)])
def test_c5_channel_closed_loop_ibyte_if(ctx, system, epochs, avx):
    """One channel per system at 50 Msps, ibyte, IF fused into the NCO, both rotator variants."""
    sat, k, x, stamp, first, delay, dop = S.sync(system, FS, epochs, f_if_hz=IF_OF[system], rotator_avx=1 if avx else 0, cn0=48.0)
    raw = signals.to_ibyte(x)
    xf = raw.astype(np.float32).view(np.complex64)
    c = dev_conf(k, system)
    assert c.if_hz == IF_OF[system]
    trk = engine.DllPllVemlTracking(ctx, c, 1)
    ctx.set_code(90, sat.code)
    if sat.code_data is not None:
        ctx.set_code(91, sat.code_data)
    trk.start(0, 90, delay, dop, stamp, first, data_code_id=91, prn=sat.prn)
    trk.set_trace(True)
    rec, rounds = trk.run(raw, first, epochs)
    tr = trk.trace(epochs)[:, 0]
    trk.close()
    ref = T.track(k, xf, sat.code, delay, dop, stamp, first, epochs, data_code=sat.code_data, buffer_first=first, prn=sat.prn)
    assert len(ref) == epochs and ref["state"][-1] in (3, 4), np.bincount(ref["state"])
    # bit-exact, both variants: the taps on the device's own arguments (u_avx order, or the generic
    # rotator's one serial float sum per tap component), then every record field of the loop
    trace_exact(tr, xf, first, sat.code, sat.code_data, f"C5 {system} avx={avx}", avx=avx)
    compare_exact(rec[:, 0], ref, f"C5 {system} avx={avx}")
    # the IF is wiped off: the loop holds the signal's Doppler (± the narrow-loop walk), not Doppler + IF
    assert np.all(np.abs(ref[-20:]["carrier_doppler_hz"] - sat.doppler_hz) < 200.0)


def test_if_must_be_whole_hz(ctx):
    k = T.conf("GPS", FS, 50000)
    c = dev_conf(k, "GPS")
    c.if_hz = 7161000.5
    with pytest.raises(abi.GnssHipError):
        engine.DllPllVemlTracking(ctx, c, 1)


def c5_share_sky():
    """The per-GPU share of configs[4] (256 channels over 8 GPUs): 12 GPS + 12 Galileo E1 + 8 BeiDou B1I
    (B1I MEO PRNs, NH code), each channel its own satellite, navigation / secondary patterns on."""
    rng = np.random.default_rng(0x6E550005)
    sky = {}
    for system, prns in (("GPS", range(1, 13)), ("GAL", [1, 2, 3, 4, 5, 7, 8, 9, 11, 12, 13, 15]), ("BDS", range(6, 14))):
        sats = []
        for p in prns:
            sats.append(signals.Satellite(prn=int(p), doppler_hz=float(rng.uniform(-4000, 4000)), code_delay_chips=float(rng.uniform(0, 1000)),
                                          cn0_dbhz=47.0, system=system, carrier_phase_rad=float(rng.uniform(0, 6.28)),
                                          f_if_hz=IF_OF[system], **S.SYNC_PATTERNS[system]))
        sky[system] = sats
    return sky


def test_c5_share_engines_concurrent_match_oracle(ctx):
    """C5's per-GPU share in closed loop: three tracking engines (GPS N = 50000, E1 5 VEML + data prompt
    N = 200000, B1I N = 50000), each on its own context (stream) of the one GPU, launched together
    over the same 50 Msps ibyte block (gnsship_trk_launch / _collect) — every channel's records equal
    to the oracle loop's, every epoch."""
    sky = c5_share_sky()
    seconds = 0.3
    first = int(FS)
    n = int(seconds * FS) + 4 * 200000
    allsats = sky["GPS"] + sky["GAL"] + sky["BDS"]
    x = signals.generate_if_device(FS, n, allsats, seed=0x6E550005, start=first, device="cpu").numpy()  # torch on the host: the HIP runtime stays libgnsship's
    raw = signals.to_ibyte(x)
    xf = raw.astype(np.float32).view(np.complex64)
    del x
    ctxs = {s: engine.Context(0) for s in ("GPS", "GAL", "BDS")}
    dev = {}
    trks, confs = {}, {}
    for system, sats in sky.items():
        cx = ctxs[system]
        vl = int(round(FS * T.SYSTEMS[system][2]))
        k = T.conf(system, FS, vl, pull_in_time_s=0, if_hz=IF_OF[system], rotator_avx=1)
        confs[system] = k
        trk = engine.DllPllVemlTracking(cx, dev_conf(k, system), len(sats))
        for ch, s in enumerate(sats):
            cx.set_code(2 * ch, s.code)
            if s.code_data is not None:
                cx.set_code(2 * ch + 1, s.code_data)
            trk.start(ch, 2 * ch, S.acq_delay_for(s, FS, system, 0, first) + 0.2, s.doppler_hz + 15.0, 0, first, data_code_id=2 * ch + 1,
                      prn=s.prn)
        dev[system] = cx.upload(raw)
        trks[system] = trk
    rounds = {"GPS": int(seconds * 1000), "GAL": int(seconds * 250), "BDS": int(seconds * 1000)}
    for system, trk in trks.items():  # all three enqueued before any is waited for
        trk.launch_ptr(dev[system].ptr, abi.FMT_CI8, first, len(raw), rounds[system], records=True)
    got = {system: trk.collect() for system, trk in trks.items()}

    def oracle(args):
        system, ch = args
        s = sky[system][ch]
        return T.track(confs[system], xf, s.code, S.acq_delay_for(s, FS, system, 0, first) + 0.2, s.doppler_hz + 15.0, 0, first,
                       rounds[system], data_code=s.code_data, buffer_first=first, prn=s.prn)

    jobs = [(system, ch) for system in sky for ch in range(len(sky[system]))]
    with cf.ThreadPoolExecutor(8) as ex:
        refs = dict(zip(jobs, ex.map(oracle, jobs)))
    states = {}
    for (system, ch), ref in refs.items():
        rec, done = got[system]
        compare_exact(rec[:, ch], ref, f"{system} ch{ch}")
        states.setdefault(system, []).append(int(ref["state"][-1]))
    # GPS and B1I synchronise within the block (preamble / NH code), E1 on CS25 after 25 epochs
    assert all(st in (3, 4) for st in states["GAL"]) and all(st in (3, 4) for st in states["BDS"]), states
    for system in trks:
        trks[system].close()
        dev[system].free()
        ctxs[system].close()


def if_on_device(fs, n, sats, seed, start):
    """The IF model (signals.generate_if_device) evaluated on the GPU with torch, returned to the host:
    hundreds of satellites at 50 Msps take minutes on the host."""
    import torch
    x = signals.generate_if_device(fs, n, sats, seed=seed, start=start, device="cuda")
    out = x.cpu().numpy()
    del x
    torch.cuda.empty_cache()
    return out


def c5_full_sky():
    """configs[4] whole: 96 GPS + 96 Galileo E1 + 64 BeiDou B1I MEO channels, every channel its own
    signal (PRNs re-used with their own Doppler, delay and phase beyond each system's PRN count)."""
    rng = np.random.default_rng(0x6E550006)
    sky = {}
    for system, prns in (("GPS", (list(range(1, 33)) * 3)[:96]), ("GAL", (list(range(1, 37)) * 3)[:96]), ("BDS", (list(range(6, 59)) * 2)[:64])):
        sky[system] = [signals.Satellite(prn=int(p), doppler_hz=float(rng.uniform(-4000, 4000)), code_delay_chips=float(rng.uniform(0, 1000)),
                                         cn0_dbhz=47.0, system=system, carrier_phase_rad=float(rng.uniform(0, 6.28)), f_if_hz=IF_OF[system],
                                         **S.SYNC_PATTERNS[system]) for p in prns]
    return sky


def test_c5_full_256_channels_one_gpu(ctx):
    """configs[4] at its BASELINE channel count on one GPU (the 8-GPU split divides exactly this): three
    engines — 96 GPS (N = 50000), 96 E1 (5 VEML + data prompt, N = 200000), 64 B1I (N = 50000) — on three
    streams over one 50 Msps ibyte block with the IF in the NCO, launched together.  A sampled subset of
    channels of every system is checked bit for bit against the oracle (traced taps on the device's own
    arguments, and every record against the oracle loop); every channel's state is checked."""
    import concurrent.futures as cf
    sky = c5_full_sky()
    seconds = 0.3
    first = int(FS)
    n = int(seconds * FS) + 4 * 200000
    allsats = sky["GPS"] + sky["GAL"] + sky["BDS"]
    x = if_on_device(FS, n, allsats, seed=0x6E550006, start=first)
    raw = signals.to_ibyte(x)
    xf = raw.astype(np.float32).view(np.complex64)
    del x
    ctxs = {s: engine.Context(0) for s in ("GPS", "GAL", "BDS")}
    dev, trks, confs = {}, {}, {}
    start = {}
    for system, sats in sky.items():
        cx = ctxs[system]
        vl = int(round(FS * T.SYSTEMS[system][2]))
        k = T.conf(system, FS, vl, pull_in_time_s=0, if_hz=IF_OF[system], rotator_avx=1)
        confs[system] = k
        trk = engine.DllPllVemlTracking(cx, dev_conf(k, system), len(sats))
        for ch, s in enumerate(sats):
            cx.set_code(2 * ch, s.code)
            if s.code_data is not None:
                cx.set_code(2 * ch + 1, s.code_data)
            start[(system, ch)] = (S.acq_delay_for(s, FS, system, 0, first) + 0.2, s.doppler_hz + 15.0)
            trk.start(ch, 2 * ch, *start[(system, ch)], 0, first, data_code_id=2 * ch + 1, prn=s.prn)
        trk.set_trace(True)
        dev[system] = cx.upload(raw)
        trks[system] = trk
    rounds = {"GPS": int(seconds * 1000), "GAL": int(seconds * 250), "BDS": int(seconds * 1000)}
    for system, trk in trks.items():
        trk.launch_ptr(dev[system].ptr, abi.FMT_CI8, first, len(raw), rounds[system], records=True)
    got = {system: trk.collect() for system, trk in trks.items()}
    traces = {system: trk.trace(rounds[system]) for system, trk in trks.items()}
    states = {system: trk.states() for system, trk in trks.items()}
    for system in trks:
        trks[system].close()
        dev[system].free()
        ctxs[system].close()
    sample = [("GPS", c) for c in (0, 31, 50, 95)] + [("GAL", c) for c in (0, 35, 61, 95)] + [("BDS", c) for c in (0, 29, 63)]

    def oracle(args):
        system, ch = args
        s = sky[system][ch]
        return T.track(confs[system], xf, s.code, *start[(system, ch)], 0, first, rounds[system], data_code=s.code_data, buffer_first=first,
                       prn=s.prn)

    with cf.ThreadPoolExecutor(8) as ex:
        refs = dict(zip(sample, ex.map(oracle, sample)))
    for (system, ch), ref in refs.items():
        label = f"C5 full {system} ch{ch}"
        s = sky[system][ch]
        trace_exact(traces[system][:, ch], xf, first, s.code, s.code_data, label)
        compare_exact(got[system][0][:, ch], ref, label)
    for system, st in states.items():  # every channel still tracking; E1 and B1I synchronised (secondary / NH code)
        assert np.all(st >= 2), (system, np.bincount(st))
        if system != "GPS":
            assert np.mean(np.isin(st, (3, 4))) >= 0.9, (system, np.bincount(st))

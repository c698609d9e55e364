"""configs[4] (C5) in closed loop: GPS L1 C/A, Galileo E1 B/C and BeiDou B1I tracked from one 50 Msps
ibyte block whose IF is centred at 1568.259 MHz — +7.161 MHz for L1/E1, −7.161 MHz for B1I (SURVEY
§8d C5).  The reference removes each signal's IF ahead of the channels (InputFilter.IF,
conf/gnss-sdr_BDS_B3I_GPS_L1_CA_ibyte.conf:45-92); the engine fuses it into the correlator's carrier
NCO (gnsship_trk_conf::if_hz) and the oracle loop (oracle/trk_oracle.c, orc_trk_conf::if_hz) applies
the same term, so every epoch of dll_pll_veml_tracking::general_work (:1728-2094) is compared.

The int8 samples go to the device as they are (converted in the loads, no scaling, as IbyteToComplex,
ibyte_to_complex.cc:39) and to the oracle converted to float.  Tolerances: test_gpu_trk.compare
(exact epoch boundaries / states / flags, Doppler ≤ 2e-3 Hz, …).  E1 at N = 200000 is checked
against the oracle's double-accumulated sums with once-rounded trig (test_gpu_trk_persist.run_pair's
reasoning for N ≥ 1e5).  With the IF in the NCO the phase step is ≈ 0.9 rad per sample, where one ulp
of phase_inc (glibc's cosf/sinf are not correctly rounded; the device forms the phasors from
once-rounded double cos/sin) turns the phase by ≈ 3e-3 rad over 50000 samples: the oracle takes the
device's trig rounding here (cr_trig) at every N; test_oracle_trk.py bounds the loop's distance
between the two trig choices.
"""
import concurrent.futures as cf

import numpy as np
import pytest

from gnss_sim_receiver_amd import abi, engine, signals
from oracle import trk as T

import trk_scenarios as S
from test_gpu_trk import compare, dev_conf

pytestmark = pytest.mark.gpu
FS = 50e6
F_IF = 7.161e6
IF_OF = {"GPS": F_IF, "GAL": F_IF, "BDS": -F_IF}


@pytest.mark.parametrize("avx", [False, True])
@pytest.mark.parametrize("system,epochs", [("GPS", 300), ("GAL", 60), ("BDS", 300)])
def test_c5_channel_closed_loop_ibyte_if(ctx, system, epochs, avx):
    """One channel per system at 50 Msps, ibyte, IF fused into the NCO, both rotator variants."""
    long_n = 1 if system == "GAL" else 0
    sat, k, x, stamp, first, delay, dop = S.sync(system, FS, epochs, f_if_hz=IF_OF[system], rotator_avx=1 if avx else 0,
                                                 accum_f64=long_n, cr_trig=1, cn0=48.0)
    raw = signals.to_ibyte(x)
    xf = raw.astype(np.float32).view(np.complex64)
    c = dev_conf(k, system)
    assert c.if_hz == IF_OF[system]
    trk = engine.DllPllVemlTracking(ctx, c, 1)
    ctx.set_code(90, sat.code)
    if sat.code_data is not None:
        ctx.set_code(91, sat.code_data)
    trk.start(0, 90, delay, dop, stamp, first, data_code_id=91, prn=sat.prn)
    rec, rounds = trk.run(raw, first, epochs)
    trk.close()
    ref = T.track(k, xf, sat.code, delay, dop, stamp, first, epochs, data_code=sat.code_data, buffer_first=first, prn=sat.prn)
    assert len(ref) == epochs and ref["state"][-1] in (3, 4), np.bincount(ref["state"])
    compare(rec[:, 0], ref, f"C5 {system} avx={avx}")
    # the IF is wiped off: the loop holds the signal's Doppler (not Doppler + IF)
    tail = ref[-20:]
    assert np.all(np.abs(tail["carrier_doppler_hz"] - sat.doppler_hz) < 20.0)


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
    over the same 50 Msps ibyte block (gnsship_trk_launch / _collect) — every channel against the
    oracle loop, every epoch."""
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
        long_n = 1 if system == "GAL" else 0
        k = T.conf(system, FS, vl, pull_in_time_s=0, if_hz=IF_OF[system], rotator_avx=1, accum_f64=long_n, cr_trig=1)
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
        compare(rec[:, ch], ref, f"{system} ch{ch}")
        states.setdefault(system, []).append(int(ref["state"][-1]))
    # GPS and B1I synchronise within the block (preamble / NH code), E1 on CS25 after 25 epochs
    assert all(st in (3, 4) for st in states["GAL"]) and all(st in (3, 4) for st in states["BDS"]), states
    for system in trks:
        trks[system].close()
        dev[system].free()
        ctxs[system].close()

"""Galileo E1 tracking correlations on the GPU (SURVEY §8d C4 / C5 shapes) vs the oracle.

dll_pll_veml_tracking with track_pilot = true runs, per channel-epoch, a 5-tap VEML correlator
on the E1-C pilot replica (shifts ±vel, ±el, 0 in replica samples, 2 per chip; :472-513) and a
1-tap prompt correlator on the E1-B data replica with the same NCO (:526-532).  Both are jobs of
one batch here.  N = 100000 (4 ms at 25 Msps) and 200000 (50 Msps ibyte).
Generic-rotator jobs run in the reference's serial order (corr_serial.hip) and equal the plain
oracle bit for bit.  AVX jobs (tree sums over the 16 exact phasor lanes): at N ≥ 1e5 the reference's
serial float accumulation is itself ~1e-5 away from the exact sum of its own float products (a √N
random walk of half-ulps of the accumulator; measured up to 1.4e-5 here), so the 1e-5 per-tap
contract is applied against the oracle with the same float products accumulated in double (oracle
corr_batch(accum_f64=True)), and against the serial oracle the bound is 1e-5 plus that oracle's own
distance to the exact accumulation.  Errors are relative to max(|ref|, ‖x‖₂) (‖x‖₂ only matters for
a tap at the noise floor).
"""
import numpy as np
import pytest

from gnss_sim_receiver_amd import abi, engine, signals
from oracle import oracle as O

pytestmark = pytest.mark.gpu
TOL = 1e-5
VEML = [-0.5, -0.25, 0.0, 0.25, 0.5]  # Dll_Pll_Conf defaults (very_early_late 0.5, early_late 0.25 chips)


def e1_jobs(sats, fs, n_ep, vl):
    jobs, cl = [], []
    for k, s in enumerate(sats):
        cl += [s.code, s.code_data]
        pj = signals.truth_jobs(s, fs, n_ep, vl, [2 * x for x in VEML], 2 * k)  # pilot, shifts in replica samples
        dj = pj.copy()
        dj["code_id"] = 2 * k + 1
        dj["n_taps"] = 1
        dj["shifts_chips"] = 0.0
        jobs += [pj, dj]
    return np.concatenate(jobs), cl


def check(out, sig, jobs, codes):
    r32 = O.corr_batch(sig, jobs, codes, n_threads=8)
    r64 = O.corr_batch(sig, jobs, codes, n_threads=8, accum_f64=True)
    worst = 0.0
    for j in range(len(jobs)):
        t = jobs[j]["n_taps"]
        if jobs[j]["flags"] == 0:  # the generic rotator in the reference's serial order: bit for bit
            assert np.array_equal(out[j, :t], r32[j, :t]), (j, out[j, :t], r32[j, :t])
            assert np.all(out[j, t:] == 0)
            continue
        o, n = jobs[j]["sample_offset"], jobs[j]["n_samples"]
        scale = np.maximum(np.abs(r64[j, :t]), float(np.linalg.norm(sig[o:o + n].astype(np.complex128))))
        e64 = np.abs(out[j, :t] - r64[j, :t]) / scale
        serial = np.abs(r32[j, :t] - r64[j, :t]) / scale
        e32 = np.abs(out[j, :t] - r32[j, :t]) / scale
        assert np.all(e64 <= TOL), (j, e64)
        assert np.all(e32 <= TOL + serial), (j, e32, serial)
        assert np.all(out[j, t:] == 0)
        worst = max(worst, float(e64.max()))
    return worst


def test_c4_e1_pilot_veml_and_data_prompt(ctx):
    fs, vl, n_ep = 25e6, 100000, 2
    sats = signals.random_sky(8, seed=404, system="GAL", cn0=45.0, prns=[1, 5, 12, 19, 24, 30, 33, 36])
    sig = signals.generate_if(fs, vl * (n_ep + 2), sats, seed=44)
    jobs, cl = e1_jobs(sats, fs, n_ep, vl)
    rng = np.random.default_rng(1)
    jobs["rem_carrier_phase_rad"] += rng.uniform(-0.2, 0.2, len(jobs)).astype(np.float32)
    out = engine.correlate_host(ctx, sig, jobs, cl)
    check(out, sig, jobs, cl)
    # locked truth NCO: prompt pilot and data prompt carry the signal, sinBOC VE/VL taps are the
    # negative side peaks of the BOC(1,1) correlation (ACF(±0.5 chip) = −0.5)
    pil = out[jobs["n_taps"] == 5]
    assert np.median(np.abs(pil[:, 2]) / np.abs(pil[:, 1])) > 2.5  # ACF(0.25 chip) = 0.25 for BOC(1,1)
    assert np.all(np.real(pil[:, 0] * np.conj(pil[:, 2])) < 0)


def test_c5_e1_ibyte_50msps(ctx):
    fs, vl = 50e6, 200000
    sats = signals.random_sky(3, seed=505, system="GAL", cn0=48.0, prns=[2, 9, 21])
    for s in sats:
        s.f_if_hz = 7.161e6  # C5: IF centred at 1568.259 MHz
    x = signals.generate_if(fs, vl * 3, sats, seed=55)
    raw = signals.to_ibyte(x)
    as_float = raw.astype(np.float32).view(np.complex64)
    jobs, cl = e1_jobs(sats, fs, 1, vl)
    out = engine.correlate_host(ctx, raw, jobs, cl)
    check(out, as_float, jobs, cl)


@pytest.mark.parametrize("flags", [0, abi.JOB_ROTATOR_AVX])
def test_c5_hybrid_batch_one_launch(ctx, flags):
    """configs[4]'s per-GPU mix in ONE batched launch from the 50 Msps ibyte block: GPS L1 C/A
    E/P/L (N = 50000) and Galileo E1 5 VEML pilot taps + data prompt (N = 200000) at IF +7.161 MHz,
    BeiDou B1I E/P/L (N = 50000, 2046-chip code) at −7.161 MHz (the 1568.259 MHz centre, SURVEY §8d
    C5).  Each job against the oracle on the same int8 samples (converted without scaling, as
    IbyteToComplex, ibyte_to_complex.cc:39), for the generic and the AVX rotator variant (the AVX
    batch path continues all 16 phasor lanes bit-exactly)."""
    fs, f_if = 50e6, 7.161e6
    gps = signals.random_sky(3, seed=551, system="GPS", cn0=48.0, prns=[3, 11, 27])
    gal = signals.random_sky(2, seed=552, system="GAL", cn0=48.0, prns=[4, 19])
    bds = signals.random_sky(2, seed=553, system="BDS", cn0=48.0, prns=[7, 30])
    for s in gps + gal:
        s.f_if_hz = f_if
    for s in bds:
        s.f_if_hz = -f_if
    x = signals.generate_if(fs, 200000 * 3, gps + gal + bds, seed=56)
    raw = signals.to_ibyte(x)
    as_float = raw.astype(np.float32).view(np.complex64)
    jobs, cl = [], []
    for s in gps + bds:
        cl.append(s.code)
        jobs.append(signals.truth_jobs(s, fs, 4, 50000, [-0.25, 0.0, 0.25], len(cl) - 1))
    ej, ecl = e1_jobs(gal, fs, 1, 200000)
    ej["code_id"] += len(cl)
    cl += ecl
    jobs = np.concatenate(jobs + [ej])
    rng = np.random.default_rng(5)
    jobs["rem_carrier_phase_rad"] += rng.uniform(-0.3, 0.3, len(jobs)).astype(np.float32)
    jobs["flags"] = flags
    out = engine.correlate_host(ctx, raw, jobs, cl)
    worst = check(out, as_float, jobs, cl)
    assert worst <= TOL
    # the locked prompts carry the signal (GPS / B1I prompt >> early/late noise)
    epl = out[jobs["n_taps"] == 3]
    assert np.median(np.abs(epl[:, 1]) / np.abs(epl[:, 0])) > 1.2  # ACF(0.25 chip) = 0.75 of the prompt


def test_c5_share_32_channels_one_launch_avx(ctx):
    """The whole per-GPU share of configs[4] (256 channels / 8 GPUs = 12 GPS + 12 E1 (5 + 1 taps) + 8
    B1I) in one batched launch, 4 GPS / B1I epochs and one E1 epoch per channel, AVX rotator variant,
    50 Msps ibyte with ±7.161 MHz IF — every job against the oracle."""
    fs, f_if = 50e6, 7.161e6
    gps = signals.random_sky(12, seed=561, system="GPS", cn0=47.0)
    gal = signals.random_sky(12, seed=562, system="GAL", cn0=47.0, prns=list(range(1, 13)))
    bds = signals.random_sky(8, seed=563, system="BDS", cn0=47.0, prns=list(range(6, 14)))
    for s in gps + gal:
        s.f_if_hz = f_if
    for s in bds:
        s.f_if_hz = -f_if
    x = signals.generate_if_device(fs, 200000 * 3, gps + gal + bds, seed=57, device="cpu").numpy()
    raw = signals.to_ibyte(x)
    as_float = raw.astype(np.float32).view(np.complex64)
    jobs, cl = [], []
    for s in gps + bds:
        cl.append(s.code)
        jobs.append(signals.truth_jobs(s, fs, 4, 50000, [-0.25, 0.0, 0.25], len(cl) - 1))
    ej, ecl = e1_jobs(gal, fs, 1, 200000)
    ej["code_id"] += len(cl)
    cl += ecl
    jobs = np.concatenate(jobs + [ej])
    jobs["flags"] = abi.JOB_ROTATOR_AVX
    rng = np.random.default_rng(6)
    jobs["rem_carrier_phase_rad"] += rng.uniform(-0.3, 0.3, len(jobs)).astype(np.float32)
    assert len(jobs) == 4 * 20 + 24
    out = engine.correlate_host(ctx, raw, jobs, cl)
    assert check(out, as_float, jobs, cl) <= TOL

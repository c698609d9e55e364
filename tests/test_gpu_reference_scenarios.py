"""The reference's own acquisition / pull-in test scenarios, run through the HIP engine.

* gps_l1_ca_pcps_acquisition_gsoc2013_test.cc — ValidationOfResults (:204-263, :505-548): PRN 10 at
  44 dB-Hz, 750 Hz, 600 chips, noiseless, 4 Msps, pfa 0.001, doppler_max 10000 / step 250: PRN 10
  detected within 0.5 chip / 2/(3·T) Hz, PRN 20 (absent) rejected.  ValidationOfResultsProbabilities
  (:274-331, :600-640): four satellites at 44 dB-Hz with noise, 100 realizations — the reference only
  prints Pd / Pfa; here every realization's decision and estimate must equal the oracle's, and
  Pd / Pfa must sit where 14 dB post-correlation SNR against a pfa = 1e-3 CFAR threshold puts them
  (Pd ≈ 0.4-0.6, Pfa ≲ 0.01).  The reference's signal
  goes through an 11-tap FIR (its "−5 samples" correction); ours is unfiltered, so no correction.
* tracking_pull-in_test.cc — acquisition feeding tracking: every acquired satellite is handed to a
  tracking channel with the acquisition's Gnss_Synchro fields and must reach narrow tracking (state
  4) with the Doppler and code phase of the synthetic truth.
"""
import numpy as np
import pytest
from scipy.special import gammaincinv

from gnss_sim_receiver_amd import abi, codes, engine, signals
from oracle import oracle as O
from oracle import trk as T

pytestmark = pytest.mark.gpu

FS = 4000000
N = 4000


def threshold(pfa, n_bins, fft_size, dwells=1):
    """calculate_threshold (pcps_acquisition.cc:884-899)."""
    p = (1.0 - float(np.float32(pfa))) ** (1.0 / float(np.float32(fft_size * n_bins)))  # double pow of float operands
    return 2.0 * gammaincinv(2.0 * dwells, p)


def test_gsoc2013_validation_of_results(ctx):
    sat = signals.Satellite(prn=10, doppler_hz=750.0, code_delay_chips=600.0, cn0_dbhz=44.0)
    x = signals.generate_if(FS, N, [sat], seed=0, noise=False)
    acq = engine.PcpsAcquisition(ctx, FS, N, 10000, 250, 0, True, max_prns=2)
    acq.set_local_code(codes.gps_l1_ca_code_gen_complex_sampled(10, FS), 0)
    acq.set_local_code(codes.gps_l1_ca_code_gen_complex_sampled(20, FS), 1)
    (r10, r20), _ = acq.run(x, n_prns=2)
    thr = threshold(0.001, acq.n_bins, N)
    assert r10.test_statistic > thr
    delay_err_chips = abs(600.0 - r10.acq_delay_samples * 1023.0 / (FS * 1e-3))
    assert delay_err_chips < 0.5
    assert abs(750.0 - r10.doppler_hz) < 2.0 / (3.0 * 1e-3)
    assert r20.test_statistic < thr
    acq.close()


def test_gsoc2013_probabilities(ctx):
    sats = [signals.Satellite(prn=p, doppler_hz=d, code_delay_chips=c, cn0_dbhz=44.0)
            for p, d, c in [(10, 750.0, 600.0), (15, 1000.0, 100.0), (21, 2000.0, 200.0), (22, 3000.0, 300.0)]]
    acq = engine.PcpsAcquisition(ctx, FS, N, 10000, 250, 0, True, max_prns=2)
    acq.set_local_code(codes.gps_l1_ca_code_gen_complex_sampled(10, FS), 0)
    acq.set_local_code(codes.gps_l1_ca_code_gen_complex_sampled(20, FS), 1)
    thr = threshold(0.001, acq.n_bins, N)
    realizations = 100
    x = signals.generate_if(FS, N * realizations, sats, seed=2013)
    correct = detected_absent = 0
    c10 = codes.gps_l1_ca_code_gen_complex_sampled(10, FS)
    c20 = codes.gps_l1_ca_code_gen_complex_sampled(20, FS)
    for i in range(realizations):
        seg = x[i * N:(i + 1) * N]
        (r10, r20), _ = acq.run(seg, n_prns=2)
        for r, c in ((r10, c10), (r20, c20)):
            ref, _ = O.pcps_acquisition_core_ex(seg, c, FS, N, 10000, 250, 0, True)
            assert (r.doppler_index, r.code_index) == (ref.doppler_index, ref.code_index), i
            assert (r.test_statistic > thr) == (ref.test_statistic > thr) or abs(r.test_statistic - thr) < 1e-3 * thr, i
        # delay relative to the realization's first sample
        truth = np.mod(600.0 / sats[0].code_freq() * FS - i * N, N)
        derr = abs(np.mod(r10.acq_delay_samples - truth + N / 2, N) - N / 2) * 1023.0 / N
        if r10.test_statistic > thr and derr < 0.5 and abs(750.0 - r10.doppler_hz) < 2.0 / 3e-3:
            correct += 1
        detected_absent += r20.test_statistic > thr
    pd, pfa = correct / realizations, detected_absent / realizations
    print(f"Pd = {pd}, Pfa (absent) = {pfa}")
    assert 0.25 <= pd <= 0.8 and pfa <= 0.05
    acq.close()


def test_pull_in_acquisition_to_tracking(ctx):
    """Acquire four satellites on the first millisecond, start one tracking channel per detection
    with the acquisition's delay / Doppler / sample stamp, track 1.5 s: every channel leaves the
    pull-in transitory after pull_in_time_s (integer seconds since the stamp, :1748-1756), then
    bit-synchronises on the preamble, reaches state 4 and follows the truth."""
    rng = np.random.default_rng(4)
    prns = [3, 8, 17, 25]
    sats = [signals.Satellite(prn=p, doppler_hz=float(rng.uniform(-4000, 4000)), code_delay_chips=float(rng.uniform(0, 1023)),
                              cn0_dbhz=50.0, carrier_phase_rad=float(rng.uniform(0, 6.28)), bits="1000101100110") for p in prns]
    epochs = 1600
    x = signals.generate_if(FS, N * (epochs + 8), sats, seed=41)
    # doppler step 125 Hz: FLAGS_external_signal_acquisition_doppler_step_hz of the pull-in test
    # (tracking_tests_flags.h:31); a 250 Hz grid leaves errors the 35 Hz PLL does not pull in
    acq = engine.PcpsAcquisition(ctx, FS, N, 5000, 125, 0, True, max_prns=len(prns))
    for i, p in enumerate(prns):
        acq.set_local_code(codes.gps_l1_ca_code_gen_complex_sampled(p, FS), i)
    # dwell = the 5th millisecond (samplestamp 4N): the first one holds the satellites' first
    # navigation-bit edge (bit_transition_flag territory), which splits the coherent integration
    stamp = 4 * N
    res, _ = acq.run(x[stamp:stamp + N], n_prns=len(prns))
    thr = threshold(0.01, acq.n_bins, N)
    k = T.conf("GPS", FS, N, pull_in_time_s=0)
    c = abi.TrkConf.defaults(abi.SYS_GPS_L1CA, FS, N, pull_in_time_s=0, rotator=abi.ROTATOR_GENERIC)
    trk = engine.DllPllVemlTracking(ctx, c, len(prns))
    first = 6 * N  # tracking starts two code periods after the acquisition's dwell
    for ch, (s, r) in enumerate(zip(sats, res)):
        assert r.test_statistic > thr, (s.prn, r.test_statistic, thr)
        ctx.set_code(ch, s.code)
        assert abs(r.doppler_hz - s.doppler_hz) <= 125, (s.prn, r.doppler_hz, s.doppler_hz)
        trk.start(ch, ch, r.acq_delay_samples, float(r.doppler_hz), stamp, first, prn=s.prn)
    rec, rounds = trk.run(x[first:], first, epochs)
    for ch, s in enumerate(sats):
        d = rec[:, ch][(rec[:, ch]["flags"] & 8) != 0]
        assert d["state"][-1] == 4, (s.prn, np.bincount(d["state"]))
        tail = d[-100:]
        assert np.sqrt(np.mean((tail["carrier_doppler_hz"] - s.doppler_hz) ** 2)) < 3.0
        assert np.max(np.abs(S_code_err(s, tail))) < 0.05
    trk.close()
    acq.close()


def S_code_err(sat, rec):
    import trk_scenarios as S
    return S.code_tracking_error_chips(sat, FS, rec, "GPS")

"""PCPS acquisition parity on the GPU: libgnsship.so vs the oracle's acquisition_core restatement.

Contract: acquisition peak (Doppler bin, code index) bit-exact, hence Acq_delay_samples and
Acq_doppler_hz exact; test statistic / input power within float tolerance (FFT implementations
differ: FFTW3f in the reference, our LDS Stockham FFT here, complex128 pocketfft in the oracle).
"""
import os

import numpy as np
import pytest

from gnss_sim_receiver_amd import codes, engine, signals
from oracle import oracle as O

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
TIE = 1.0 + 1e-4  # peak / second-largest grid value below this: a near-tie the float FFTs may order differently


class ExactCount:
    """Counts the (bin, index) comparisons made exactly and the near-tie skips, so that a test
    cannot pass with zero exact comparisons."""

    def __init__(self):
        self.exact, self.ties = 0, []

    def check(self, r, ref, rgrid, label):
        flat = np.sort(rgrid.ravel())
        if flat[-1] / flat[-2] > TIE:
            assert (r.doppler_index, r.code_index) == (ref.doppler_index, ref.code_index), label
            assert r.acq_delay_samples == ref.acq_delay_samples, label
            self.exact += 1
            return True
        self.ties.append(label)
        return False


def test_golden_acquisition_cases(ctx):
    g = np.load(os.path.join(GOLD, "acq_cases.npz"))
    i = 0
    while f"a{i}_sig" in g.files:
        fs, prn, dmax, step, cfar = (int(v) for v in g[f"a{i}_conf"])
        n = int(fs / 1000)
        acq = engine.PcpsAcquisition(ctx, fs, n, dmax, step, 0, bool(cfar))
        acq.set_local_code(codes.gps_l1_ca_code_gen_complex_sampled(prn, fs))
        (r,), _ = acq.run(g[f"a{i}_sig"])
        exp_idx = g[f"a{i}_expect_idx"]
        exp_val = g[f"a{i}_expect_val"]
        assert [r.doppler_index, r.code_index, r.doppler_hz] == list(exp_idx), i
        assert r.acq_delay_samples == exp_val[3]
        np.testing.assert_allclose([r.peak, r.input_power, r.test_statistic], exp_val[:3], rtol=2e-4)
        acq.close()
        i += 1
    assert i >= 5


def test_grid_matches_oracle_grid(ctx):
    fs, n, dmax, step = 4000000, 4000, 5000, 500
    sat = signals.Satellite(prn=9, doppler_hz=1234.0, code_delay_chips=321.4, cn0_dbhz=44.0)
    sig = signals.generate_if(fs, n, [sat], seed=4)
    code = codes.gps_l1_ca_code_gen_complex_sampled(9, fs)
    acq = engine.PcpsAcquisition(ctx, fs, n, dmax, step, 0, True)
    acq.set_local_code(code)
    (r,), grid = acq.run(sig, want_grid=True)
    ref, rgrid = O.pcps_acquisition_core(sig, code, fs, dmax, step, 0, True)
    scale = rgrid.max()
    assert np.max(np.abs(grid[0] - rgrid)) / scale < 1e-5
    assert (r.doppler_index, r.code_index) == (ref.doppler_index, ref.code_index)
    acq.close()


def test_multi_prn_sweep_present_and_absent(ctx):
    """All-sky style: several PRNs searched in one call over a shared FFT(in ⊙ w_b)."""
    fs, n, dmax, step = 4000000, 4000, 5000, 250
    present = [signals.Satellite(prn=p, doppler_hz=d, code_delay_chips=c, cn0_dbhz=48.0)
               for p, d, c in [(3, -2100.0, 100.3), (11, 3333.0, 800.7), (19, 50.0, 512.2), (27, -4700.0, 1000.1)]]
    sig = signals.generate_if(fs, n, present, seed=77)
    prns = [3, 11, 19, 27, 1, 2, 5, 8]
    acq = engine.PcpsAcquisition(ctx, fs, n, dmax, step, 0, True, max_prns=len(prns))
    for k, p in enumerate(prns):
        acq.set_local_code(codes.gps_l1_ca_code_gen_complex_sampled(p, fs), k)
    res, _ = acq.run(sig, n_prns=len(prns))
    cnt = ExactCount()
    for k, p in enumerate(prns):
        ref, rgrid = O.pcps_acquisition_core(sig, codes.gps_l1_ca_code_gen_complex_sampled(p, fs), fs, dmax, step, 0, True)
        exact = cnt.check(res[k], ref, rgrid, p)
        assert exact or k >= 4, p  # every present PRN is compared exactly
        np.testing.assert_allclose(res[k].test_statistic, ref.test_statistic, rtol=2e-3)
    assert cnt.exact >= 4 and len(cnt.ties) <= 2, (cnt.exact, cnt.ties)
    # noise-only CFAR statistic ≈ 2·ln(cells) ≈ 25 for 80 × 4000 cells; present PRNs far above
    absent_max = max(res[k].test_statistic for k in range(4, 8))
    assert absent_max < 40
    assert min(res[k].test_statistic for k in range(4)) > 2 * absent_max
    acq.close()


@pytest.mark.parametrize("fmt", ["ci16", "ci8"])
def test_integer_input_formats(ctx, fmt):
    fs, n = 4000000, 4000
    sat = signals.Satellite(prn=5, doppler_hz=-1500.0, code_delay_chips=77.7, cn0_dbhz=50.0)
    x = signals.generate_if(fs, n, [sat], seed=8)
    raw = signals.to_ishort(x) if fmt == "ci16" else signals.to_ibyte(x)
    code = codes.gps_l1_ca_code_gen_complex_sampled(5, fs)
    acq = engine.PcpsAcquisition(ctx, fs, n, 5000, 250, 0, False)
    acq.set_local_code(code)
    (r,), _ = acq.run(raw)
    ref, _ = O.pcps_acquisition_core(raw.astype(np.float32).view(np.complex64), code, fs, 5000, 250, 0, False)
    assert (r.doppler_index, r.code_index) == (ref.doppler_index, ref.code_index)
    acq.close()


def test_noncoherent_dwells_accumulate(ctx):
    fs, n = 4000000, 4000
    sat = signals.Satellite(prn=14, doppler_hz=900.0, code_delay_chips=10.0, cn0_dbhz=40.0)
    x = signals.generate_if(fs, 2 * n, [sat], seed=12)
    code = codes.gps_l1_ca_code_gen_complex_sampled(14, fs)
    acq = engine.PcpsAcquisition(ctx, fs, n, 5000, 250, 0, True, max_dwells=2)
    acq.set_local_code(code)
    acq.run(x[:n])
    (r2,), grid = acq.run(x[n:], want_grid=True)
    w = O.doppler_wipeoff_grid(acq.n_bins, n, 5000, 250, 0, fs)
    g = O.acquisition_grid(x[:n], code, w) + O.acquisition_grid(x[n:], code, w)
    st = O.acquisition_statistic(g, 5000, 250, 0, True, 4, 4000.0, dwells=2)
    assert (r2.doppler_index, r2.code_index) == (st.doppler_index, st.code_index)
    np.testing.assert_allclose(r2.input_power, st.input_power, rtol=1e-3)
    acq.close()


def test_bad_configuration_rejected(ctx):
    from gnss_sim_receiver_amd import abi
    with pytest.raises(abi.GnssHipError):
        engine.PcpsAcquisition(ctx, 4000000, 4001, 5000, 250)  # 4001 = 4001 (prime) not 2^a3^b5^c
    acq = engine.PcpsAcquisition(ctx, 4000000, 4000, 5000, 250)
    with pytest.raises(abi.GnssHipError):
        acq.run(np.zeros(4000, np.complex64))  # no local code yet
    acq.close()


# ---- large transforms (four-step, N = P·M > 16384): SURVEY §8 C3, 25 Msps, 1 ms GPS code ----

def _acq_big_case(ctx, fs, n, prns, present, dmax, step, cfar, seed, want_grid=False):
    sig = signals.generate_if(fs, n, present, seed=seed)
    acq = engine.PcpsAcquisition(ctx, fs, n, dmax, step, 0, cfar, max_prns=len(prns))
    for k, p in enumerate(prns):
        acq.set_local_code(codes.gps_l1_ca_code_gen_complex_sampled(p, fs), k)
    res, grid = acq.run(sig, n_prns=len(prns), want_grid=want_grid)
    acq.close()
    return sig, res, grid


def test_c3_25msps_four_step_matches_oracle(ctx):
    fs, n, dmax, step = 25000000, 25000, 5000, 250
    present = [signals.Satellite(prn=p, doppler_hz=d, code_delay_chips=c, cn0_dbhz=46.0)
               for p, d, c in [(4, 1750.0, 211.3), (17, -3900.0, 999.9)]]
    prns = [4, 17, 30]
    sig, res, grid = _acq_big_case(ctx, fs, n, prns, present, dmax, step, True, seed=21, want_grid=True)
    for k, p in enumerate(prns):
        ref, rgrid = O.pcps_acquisition_core(sig, codes.gps_l1_ca_code_gen_complex_sampled(p, fs), fs, dmax, step, 0, True)
        # fp32 four-step vs complex128: grid within 1e-5 of the grid maximum
        assert np.max(np.abs(grid[k] - rgrid)) / rgrid.max() < 1e-5, p
        assert ExactCount().check(res[k], ref, rgrid, p) or k == 2, p  # the present PRNs exactly
        np.testing.assert_allclose(res[k].test_statistic, ref.test_statistic, rtol=2e-3)
    assert res[0].test_statistic > 2 * res[2].test_statistic  # noise-only CFAR ≈ 2·ln(10⁶ cells) ≈ 28


def test_c3_full_sweep_32_prns_baseline_signal(ctx):
    """BASELINE.md C3 as specified: 32 PRNs × 40 bins × 25000 points at 25 Msps, 10 PRNs present
    (signals.c3_sky, seed 0x6E550003), CFAR statistic.  Every PRN against the oracle; every present
    PRN's (bin, index) exactly; near-ties (noise-only PRNs whose two largest cells differ by < 1e-4)
    counted, not silently skipped."""
    fs, n, dmax, step = 25000000, 25000, 5000, 250
    present = signals.c3_sky()
    present_prns = {s.prn for s in present}
    prns = list(range(1, 33))
    sig, res, _ = _acq_big_case(ctx, fs, n, prns, present, dmax, step, True, seed=0x6E550003)
    cnt = ExactCount()
    for k, p in enumerate(prns):
        ref, rgrid = O.pcps_acquisition_core(sig, codes.gps_l1_ca_code_gen_complex_sampled(p, fs), fs, dmax, step, 0, True)
        exact = cnt.check(res[k], ref, rgrid, p)
        assert exact or p not in present_prns, p
        np.testing.assert_allclose(res[k].test_statistic, ref.test_statistic, rtol=2e-3)
    assert cnt.exact >= 28, (cnt.exact, cnt.ties)  # at most a few noise-only near-ties
    # detection at 45 dB-Hz with 1 ms coherent integration is marginal for the weakest satellites
    # (Doppler / code straddle losses): most present PRNs clear the noise-only maximum
    stat = np.array([r.test_statistic for r in res])
    absent = [stat[p - 1] for p in prns if p not in present_prns]
    above = sum(stat[p - 1] > max(absent) for p in present_prns)
    assert above >= 8 and np.median([stat[p - 1] for p in present_prns]) > 1.5 * np.median(absent), (sorted(present_prns), stat)


def test_four_step_forced_at_small_size_first_vs_second(ctx, monkeypatch):
    """The four-step path at N = 4000 (P = 16, M = 250) against the oracle, second-peak statistic."""
    monkeypatch.setenv("GNSSHIP_ACQ_FORCE_BIG", "1")
    fs, n = 4000000, 4000
    sat = signals.Satellite(prn=22, doppler_hz=-620.0, code_delay_chips=432.1, cn0_dbhz=47.0)
    sig, (r,), grid = _acq_big_case(ctx, fs, n, [22], [sat], 5000, 250, False, seed=5, want_grid=True)
    ref, rgrid = O.pcps_acquisition_core(sig, codes.gps_l1_ca_code_gen_complex_sampled(22, fs), fs, 5000, 250, 0, False)
    assert np.max(np.abs(grid[0] - rgrid)) / rgrid.max() < 1e-5
    assert (r.doppler_index, r.code_index) == (ref.doppler_index, ref.code_index)
    np.testing.assert_allclose([r.peak, r.input_power, r.test_statistic], [ref.peak, ref.input_power, ref.test_statistic],
                               rtol=2e-4)


@pytest.mark.parametrize("fmt", ["ci16", "ci8"])
def test_four_step_integer_formats(ctx, fmt):
    fs, n = 25000000, 25000
    sat = signals.Satellite(prn=9, doppler_hz=2250.0, code_delay_chips=600.2, cn0_dbhz=52.0)
    x = signals.generate_if(fs, n, [sat], seed=31)
    raw = signals.to_ishort(x) if fmt == "ci16" else signals.to_ibyte(x)
    code = codes.gps_l1_ca_code_gen_complex_sampled(9, fs)
    acq = engine.PcpsAcquisition(ctx, fs, n, 5000, 500, 0, True)
    acq.set_local_code(code)
    (r,), _ = acq.run(raw)
    ref, _ = O.pcps_acquisition_core(raw.astype(np.float32).view(np.complex64), code, fs, 5000, 500, 0, True)
    assert (r.doppler_index, r.code_index) == (ref.doppler_index, ref.code_index)
    np.testing.assert_allclose(r.test_statistic, ref.test_statistic, rtol=2e-3)
    acq.close()


def test_four_step_max_size_and_limit(ctx):
    from gnss_sim_receiver_amd import abi
    # 32768 = 32 × 1024: the largest four-step transform; a 1 ms code at 32.768 Msps
    fs, n = 32768000, 32768
    sat = signals.Satellite(prn=2, doppler_hz=-1000.0, code_delay_chips=55.5, cn0_dbhz=50.0)
    sig, (r,), grid = _acq_big_case(ctx, fs, n, [2], [sat], 2000, 500, True, seed=3, want_grid=True)
    ref, rgrid = O.pcps_acquisition_core(sig, codes.gps_l1_ca_code_gen_complex_sampled(2, fs), fs, 2000, 500, 0, True)
    assert np.max(np.abs(grid[0] - rgrid)) / rgrid.max() < 1e-5
    assert (r.doppler_index, r.code_index) == (ref.doppler_index, ref.code_index)
    with pytest.raises(abi.GnssHipError):
        engine.PcpsAcquisition(ctx, 40001000, 40001, 5000, 250)  # 13·17·181: no layout


# ---- huge transforms (N = P·M > 32768, column and row stages as separate kernels) ----------

def test_huge_forced_at_small_size_matches_oracle(ctx, monkeypatch):
    """The huge layout at N = 4000 (P = 4, M = 1000) against the oracle, both statistics."""
    monkeypatch.setenv("GNSSHIP_ACQ_FORCE_HUGE", "1")
    fs, n = 4000000, 4000
    sat = signals.Satellite(prn=14, doppler_hz=1380.0, code_delay_chips=702.6, cn0_dbhz=47.0)
    for cfar in (False, True):
        sig, (r,), grid = _acq_big_case(ctx, fs, n, [14], [sat], 5000, 250, cfar, seed=15, want_grid=True)
        ref, rgrid = O.pcps_acquisition_core(sig, codes.gps_l1_ca_code_gen_complex_sampled(14, fs), fs, 5000, 250, 0, cfar)
        assert np.max(np.abs(grid[0] - rgrid)) / rgrid.max() < 1e-5
        assert (r.doppler_index, r.code_index) == (ref.doppler_index, ref.code_index)
        np.testing.assert_allclose([r.peak, r.input_power, r.test_statistic], [ref.peak, ref.input_power, ref.test_statistic],
                                   rtol=2e-4)


def test_huge_gps_50msps_multi_prn(ctx):
    """1 ms GPS L1 C/A at 50 Msps (SURVEY §8d C5 rate): N = 50000 = 4 × 12500."""
    fs, n, dmax, step = 50000000, 50000, 2000, 500
    present = [signals.Satellite(prn=p, doppler_hz=d, code_delay_chips=c, cn0_dbhz=47.0) for p, d, c in [(6, 1200.0, 333.3), (21, -800.0, 40.9)]]
    prns = [6, 21, 2]
    sig, res, grid = _acq_big_case(ctx, fs, n, prns, present, dmax, step, True, seed=61, want_grid=True)
    for k, p in enumerate(prns):
        ref, rgrid = O.pcps_acquisition_core(sig, codes.gps_l1_ca_code_gen_complex_sampled(p, fs), fs, dmax, step, 0, True)
        assert np.max(np.abs(grid[k] - rgrid)) / rgrid.max() < 1e-5, p
        assert ExactCount().check(res[k], ref, rgrid, p) or k == 2, p  # the present PRNs exactly
        np.testing.assert_allclose(res[k].test_statistic, ref.test_statistic, rtol=2e-3)
    assert min(res[0].test_statistic, res[1].test_statistic) > 2 * res[2].test_statistic


@pytest.mark.parametrize("cboc", [False, True])
def test_huge_galileo_e1_25msps(ctx, cboc):
    """Galileo E1 acquisition (GalileoE1PcpsAmbiguousAcquisition: ms_per_code 4,
    galileo_e1_pcps_ambiguous_acquisition.cc:51): 4 ms at 25 Msps, N = 100000 = 8 × 12500, E1-B
    replica from galileo_e1_code_gen_complex_sampled, against the oracle core."""
    fs, n, dmax, step = 25000000, 100000, 1000, 250
    present = [signals.Satellite(prn=p, doppler_hz=d, code_delay_chips=c, cn0_dbhz=45.0, system="GAL")
               for p, d, c in [(11, 400.0, 2222.2), (30, -650.0, 7001.5)]]
    prns = [11, 30, 4]
    sig = signals.generate_if(fs, n, present, seed=91)
    acq = engine.PcpsAcquisition(ctx, fs, n, dmax, step, 0, False, max_prns=3, ms_per_code=4)
    lc = [codes.galileo_e1_code_gen_complex_sampled("1B", cboc, p, fs) for p in prns]
    for k in range(3):
        acq.set_local_code(lc[k], k)
    res, grid = acq.run(sig, n_prns=3, want_grid=True)
    acq.close()
    spc, spcode = int(np.ceil(np.float32(fs) / np.float32(1023000.0))), float(np.float32(np.float32(fs) * np.float32(0.001)) * 4)
    for k, p in enumerate(prns):
        ref, rgrid = O.pcps_acquisition_core(sig, lc[k], fs, dmax, step, 0, False, samples_per_chip=spc, samples_per_code=spcode)
        assert np.max(np.abs(grid[k] - rgrid)) / rgrid.max() < 1e-5, p
        flat = np.sort(rgrid.ravel())
        if flat[-1] / flat[-2] > TIE:
            assert (res[k].doppler_index, res[k].code_index) == (ref.doppler_index, ref.code_index), p
        else:
            assert k == 2, p  # only the absent PRN may be a near-tie
        np.testing.assert_allclose(res[k].test_statistic, ref.test_statistic, rtol=2e-3)
    # the present satellites are found at their code delay (sinBOC samples → IF samples)
    for k, s in enumerate(present):
        exp = (s.code_delay_chips / s.code_freq() * fs) % n
        assert min(abs(res[k].code_index - exp), n - abs(res[k].code_index - exp)) <= 2, (s.prn, res[k].code_index, exp)


def test_huge_galileo_e1_all_sky_prn_batches(ctx):
    """E1 all-sky as the bench runs it: 32 PRNs x 41 bins at N = 100000, so the inverse stage runs in
    several PRN batches (≈256 MiB of row scratch each) with 4-wave column workgroups.  Two runs give
    identical results, every statistic is finite, and two present PRNs and one absent PRN match the
    oracle core exactly (a regression test for a cross-wave reduction that read past its workgroup's
    waves)."""
    fs, n, dmax, step = 25000000, 100000, 5000, 250
    present_prns = [2, 9, 13, 21, 26, 31]
    sats = signals.random_sky(6, seed=0x6E550007, system="GAL", prns=present_prns)
    sig = signals.generate_if(fs, n, sats, seed=0x6E550007)
    acq = engine.PcpsAcquisition(ctx, fs, n, dmax, step, 0, False, max_prns=32, ms_per_code=4)
    lc = [codes.galileo_e1_code_gen_complex_sampled("1B", False, p, fs) for p in range(1, 33)]
    for k in range(32):
        acq.set_local_code(lc[k], k)
    dev = ctx.upload(np.ascontiguousarray(sig))
    res1, _ = acq.run(dev, n_prns=32)
    res2, _ = acq.run(dev, n_prns=32)
    acq.close()
    dev.free()
    assert b"".join(bytes(r) for r in res1) == b"".join(bytes(r) for r in res2)
    stat = np.array([r.test_statistic for r in res1])
    assert np.all(np.isfinite(stat)), stat
    assert min(stat[p - 1] for p in present_prns) > max(stat[k] for k in range(32) if k + 1 not in present_prns)
    spc, spcode = int(np.ceil(np.float32(fs) / np.float32(1023000.0))), float(np.float32(np.float32(fs) * np.float32(0.001)) * 4)
    ex = ExactCount()
    for p in (2, 26, 5):
        ref, rgrid = O.pcps_acquisition_core(sig, lc[p - 1], fs, dmax, step, 0, False, samples_per_chip=spc, samples_per_code=spcode)
        ex.check(res1[p - 1], ref, rgrid, p)
        np.testing.assert_allclose(res1[p - 1].test_statistic, ref.test_statistic, rtol=2e-3)
    assert ex.exact >= 2, ex.ties


def test_huge_limits(ctx):
    from gnss_sim_receiver_amd import abi
    with pytest.raises(abi.GnssHipError):
        engine.PcpsAcquisition(ctx, 600000000, 600000, 5000, 250)  # > 32 × 16384


# ---- acquisition variants: bit_transition_flag, sampled_ms != ms_per_code, make_2_steps

def _variant_case(ctx, fs, fft, consumed, bt, cfar, prn, seed, monkeypatch=None, force=None):
    if force:
        monkeypatch.setenv(force, "1")
    sat = signals.Satellite(prn=prn, doppler_hz=-1830.0, code_delay_chips=511.7, cn0_dbhz=47.0)
    sig = signals.generate_if(fs, fft, [sat], seed=seed)
    code = np.tile(codes.gps_l1_ca_code_gen_complex_sampled(prn, fs), 4)
    acq = engine.PcpsAcquisition(ctx, fs, fft, 5000, 250, 0, cfar, consumed_samples=consumed, bit_transition_flag=bt)
    acq.set_local_code(code)
    (r,), grid = acq.run(sig[:consumed or fft], want_grid=True)
    acq.close()
    ref, rgrid = O.pcps_acquisition_core_ex(sig, code, fs, fft, 5000, 250, 0, cfar, consumed=consumed or fft, bit_transition=bt)
    assert grid.shape[1:] == rgrid.shape
    assert np.max(np.abs(grid[0] - rgrid)) / rgrid.max() < 1e-5
    assert (r.doppler_index, r.code_index, r.doppler_hz) == (ref.doppler_index, ref.code_index, ref.doppler_hz)
    assert r.acq_delay_samples == ref.acq_delay_samples
    np.testing.assert_allclose([r.peak, r.input_power, r.test_statistic], [ref.peak, ref.input_power, ref.test_statistic], rtol=2e-4)


@pytest.mark.parametrize("cfar", [True, False])
def test_bit_transition_flag(ctx, cfar):
    """bit_transition_flag: 2 ms of input against [1 ms zeros | 1 ms code], grid rows = the second half
    of |IFFT|² (pcps_acquisition.cc:187-192, 663-664), first-vs-second window modulo d_fft_size."""
    _variant_case(ctx, 4000000, 8000, 0, True, cfar, 17, 41)


@pytest.mark.parametrize("cfar", [True, False])
def test_zero_padded_input_sampled_ms_ne_ms_per_code(ctx, cfar):
    """sampled_ms != ms_per_code: fft_size = 2 × consumed, input and code zero-padded (:84-91, :197-202, :612-619)."""
    _variant_case(ctx, 4000000, 8000, 4000, False, cfar, 23, 42)


def test_bit_transition_four_step_and_huge(ctx, monkeypatch):
    _variant_case(ctx, 25000000, 50000, 0, True, True, 9, 43)              # huge layout (4 × 12500)
    _variant_case(ctx, 8000000, 16000, 0, True, False, 9, 44, monkeypatch, "GNSSHIP_ACQ_FORCE_BIG")  # four-step (16 × 1000)


@pytest.mark.parametrize("cfar", [True, False])
def test_make_2_steps_narrow_grid(ctx, cfar):
    """make_2_steps: step-two grid of nb2 bins × step2 around the step-one Doppler (:305-312); its
    Doppler formula (:553-556) and, with CFAR, the step-one input power (:516-525)."""
    fs, n = 4000000, 4000
    sat = signals.Satellite(prn=3, doppler_hz=1130.0, code_delay_chips=300.3, cn0_dbhz=48.0)
    sig = signals.generate_if(fs, n, [sat], seed=45)
    code = codes.gps_l1_ca_code_gen_complex_sampled(3, fs)
    acq = engine.PcpsAcquisition(ctx, fs, n, 5000, 250, 0, cfar)
    acq.set_local_code(code)
    (r1,), _ = acq.run(sig)
    ref1, _ = O.pcps_acquisition_core(sig, code, fs, 5000, 250, 0, cfar)
    assert (r1.doppler_index, r1.code_index) == (ref1.doppler_index, ref1.code_index)
    acq.set_grid_step2(float(r1.doppler_hz), 62.5, 8, r1.input_power)
    assert acq.n_bins == 8
    (r2,), grid = acq.run(sig, want_grid=True)
    ref2, rgrid = O.pcps_acquisition_core_ex(sig, code, fs, n, 5000, 250, 0, cfar, step2=(float(r1.doppler_hz), 62.5, 8, r1.input_power))
    assert np.max(np.abs(grid[0] - rgrid)) / rgrid.max() < 1e-5
    assert (r2.doppler_index, r2.code_index, r2.doppler_hz) == (ref2.doppler_index, ref2.code_index, ref2.doppler_hz)
    np.testing.assert_allclose([r2.peak, r2.input_power, r2.test_statistic], [ref2.peak, ref2.input_power, ref2.test_statistic], rtol=2e-4)
    assert abs(r2.doppler_hz - 1130) <= 62.5  # the finer grid closes in on the true Doppler
    acq.set_grid(5000, 250, 0)  # back to step one
    (r3,), _ = acq.run(sig)
    assert (r3.doppler_index, r3.code_index, r3.doppler_hz) == (r1.doppler_index, r1.code_index, r1.doppler_hz)
    acq.close()

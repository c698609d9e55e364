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
    for k, p in enumerate(prns):
        ref, rgrid = O.pcps_acquisition_core(sig, codes.gps_l1_ca_code_gen_complex_sampled(p, fs), fs, dmax, step, 0, True)
        flat = np.sort(rgrid.ravel())
        if flat[-1] / flat[-2] > 1.0 + 1e-4:  # peak not a near-tie: must be exact
            assert (res[k].doppler_index, res[k].code_index) == (ref.doppler_index, ref.code_index), p
        np.testing.assert_allclose(res[k].test_statistic, ref.test_statistic, rtol=2e-3)
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

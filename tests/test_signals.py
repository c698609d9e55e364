"""The bench's on-device IF generator (signals.generate_if_device) evaluates generate_if's signal
model: noise-free blocks agree to float32 rounding for every signal feature (GPS nav bits, E1 pilot
secondary code + data, BeiDou NH code, IF offset, Doppler ramp).  Runs on the CPU with torch."""
import numpy as np
import pytest

from gnss_sim_receiver_amd import signals as S


@pytest.mark.parametrize("system,fs,kw", [
    ("GPS", 4e6, dict(bits="1000101100110")),
    ("GAL", 25e6, dict(secondary="0011100000001010110110010", bits="0110")),
    ("BDS", 50e6, dict(secondary="00000100110101001110", bits="0111", f_if_hz=-7.161e6)),
    ("GPS", 4e6, dict(doppler_rate_hz_s=300.0, f_if_hz=7.161e6)),
])
def test_device_generator_matches_numpy(system, fs, kw):
    sats = [S.Satellite(prn=p, doppler_hz=d, code_delay_chips=c, cn0_dbhz=60.0, system=system, carrier_phase_rad=0.7, **kw)
            for p, d, c in ((3, 1234.5, 100.25), (7, -3210.0, 17.75))]
    start = 123456
    a = S.generate_if(fs, 60000, sats, noise=False, start=start)
    b = S.generate_if_device(fs, 60000, sats, start=start, device="cpu", noise=False, block=25000).numpy()
    assert np.max(np.abs(a - b)) <= 1e-6 * np.max(np.abs(a))


def test_acq_delay_samples_is_the_next_code_start():
    sat = S.Satellite(prn=5, doppler_hz=2500.0, code_delay_chips=321.5)
    fs, first = 4e6, int(11 * 4e6)
    d = S.acq_delay_samples(sat, fs, 0, first)
    n0 = d  # relative to stamp 0: absolute sample of a code start, within one period after first
    assert first <= n0 < first + 4000
    assert abs(np.mod(sat.chip_phase(np.float64(n0), fs), 1023)) < 1e-6 or abs(np.mod(sat.chip_phase(np.float64(n0), fs), 1023) - 1023) < 1e-6

"""The CPU oracle against the reference's own outputs (CPU only).

* tests/golden/*.npz were produced by the reference's own code generators and generic volk_gnsssdr
  kernels compiled from /root/reference (oracle/_ref) — see tests/golden/make_golden.py.
* When oracle/_ref/libref.so is present (this container), the restatement is also compared live
  against it on fresh random cases.
"""
import ctypes
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")
REF_SO = os.path.join(os.path.dirname(os.path.dirname(__file__)), "oracle", "_ref", "libref.so")
f32p = ctypes.POINTER(ctypes.c_float)


def gold(name):
    return np.load(os.path.join(GOLD, name))


def test_codes_match_reference_tables(built):
    g = gold("codes_ref.npz")
    for k in range(32):
        assert (O.gps_l1_ca_code(k + 1) == g["gps"][k]).all(), k + 1
    for k in range(63):
        assert (O.beidou_b1i_code(k + 1) == g["b1i"][k]).all(), k + 1
    for key in g.files:
        if key.startswith("gps_sampled_"):
            fs, prn = map(int, key.split("_")[2:])
            assert (O.gps_l1_ca_code_sampled(prn, fs).imag == g[key]).all()
        if key.startswith("b1i_sampled_"):
            fs, prn = map(int, key.split("_")[2:])
            assert (O.beidou_b1i_code_sampled(prn, fs).real == g[key]).all()


def test_gps_prn1_first_chips_octal_1440(built):
    # IS-GPS-200 Table 3-Ia: first 10 chips of PRN 1 in octal = 1440
    bits = "".join("1" if c > 0 else "0" for c in O.gps_l1_ca_code(1)[:10])
    assert int(bits, 2) == 0o1440


def test_resampler_matches_reference(built):
    g = gold("resampler_ref.npz")
    codes = gold("codes_ref.npz")
    i = 0
    while f"rs{i}_out" in g.files:
        rem, step, L, n = g[f"rs{i}_args"]
        idx, kind = g[f"rs{i}_codeid"]
        code = (codes["gps"][idx] if kind == 0 else codes["b1i"][idx]).astype(np.float32)
        out = O.resampler(code, np.float32(rem), np.float32(step), g[f"rs{i}_shifts"], int(n))
        assert (out == g[f"rs{i}_out"]).all(), i
        i += 1
    assert i >= 7
    out = O.resampler(codes["gps"][9].astype(np.float32), 0.3, 0.25575, np.array([-0.5, 0, 0.5], np.float32), 4000,
                      high_dyn_rate=1e-9)
    assert (out == g["hd_out"]).all()


def test_sincos_wipeoff_matches_reference(built):
    g = gold("sincos_ref.npz")
    for i in range(3):
        fd, fs, n = g[f"w{i}_args"]
        w = O.doppler_wipeoff_grid(1, int(n), -int(fd), 1, 0, int(fs))[0]  # one bin at exactly fd
        assert (w == g[f"w{i}"]).all(), i


def test_index_max_first_of_ties(built):
    x = np.array([1, 5, 5, 2, 5], np.float32)
    assert O.lib().orc_index_max_generic(x.ctypes.data_as(f32p), 5) == 1


def test_corr_cases_reproduce(built):
    g = gold("corr_cases.npz")
    codes = gold("codes_ref.npz")
    for i in range(10):
        prn, n, rem_carr, carr_step, rem_code, code_step = g[f"c{i}_args"]
        out = O.multicorrelator(g[f"c{i}_sig"], codes["gps"][int(prn) - 1].astype(np.float32), g[f"c{i}_shifts"], rem_carr,
                                carr_step, rem_code, code_step)
        assert (out == g[f"c{i}_out"]).all(), i


def test_acquisition_cases_reproduce(built):
    g = gold("acq_cases.npz")
    i = 0
    while f"a{i}_sig" in g.files:
        fs, prn, dmax, step, cfar = g[f"a{i}_conf"]
        code = O.gps_l1_ca_code_sampled(int(prn), int(fs))
        r, _ = O.pcps_acquisition_core(g[f"a{i}_sig"], code, int(fs), int(dmax), int(step), 0, bool(cfar))
        assert [r.doppler_index, r.code_index, r.doppler_hz] == list(g[f"a{i}_expect_idx"]), i
        np.testing.assert_allclose([r.peak, r.input_power, r.test_statistic], g[f"a{i}_expect_val"][:3], rtol=1e-6)
        i += 1


@pytest.mark.skipif(not os.path.exists(REF_SO), reason="oracle/_ref not built (needs /root/reference)")
def test_oracle_vs_reference_build_random(built):
    R = ctypes.CDLL(REF_SO)
    R.ref_resampler_generic.argtypes = [f32p, f32p, ctypes.c_float, ctypes.c_float, f32p, ctypes.c_uint, ctypes.c_int, ctypes.c_uint]
    rng = np.random.default_rng(5)
    for trial in range(50):
        L = [1023, 2046, 8184][trial % 3]
        code = np.where(rng.random(L) > 0.5, 1.0, -1.0).astype(np.float32)
        n = int(rng.integers(1, 30000))
        sh = np.sort(rng.uniform(-2, 2, int(rng.integers(1, 8)))).astype(np.float32)
        rem = np.float32(rng.uniform(-3 * L, 3 * L))
        step = np.float32(rng.uniform(0.01, 2.0))
        o = np.zeros((len(sh), n), np.float32)
        R.ref_resampler_generic(o.ctypes.data_as(f32p), code.ctypes.data_as(f32p), rem, step, sh.ctypes.data_as(f32p), L, len(sh), n)
        assert (o == O.resampler(code, rem, step, sh, n)).all(), trial


@pytest.mark.skipif(not os.path.exists(REF_SO), reason="oracle/_ref not built (needs /root/reference)")
def test_oracle_hd_resampler_vs_reference_build_random(built):
    """High-dynamics resampler (…_high_dynamics_resampler_32f_xn.h:67-91): rate term with the
    32-bit unsigned n·n (lengths past 65536 included), taps 1.. as circular shifts of tap 0."""
    R = ctypes.CDLL(REF_SO)
    R.ref_high_dynamics_resampler_generic.argtypes = [f32p, f32p, ctypes.c_float, ctypes.c_float, ctypes.c_float, f32p, ctypes.c_uint,
                                                      ctypes.c_int, ctypes.c_uint]
    rng = np.random.default_rng(6)
    for trial in range(30):
        L = [1023, 2046, 8184][trial % 3]
        code = np.where(rng.random(L) > 0.5, 1.0, -1.0).astype(np.float32)
        n = int(rng.integers(1000, 80000))
        step = np.float32(rng.uniform(0.05, 1.5))
        sh = np.sort(rng.uniform(-2, 2, int(rng.integers(1, 6)))).astype(np.float32)
        rem = np.float32(rng.uniform(-3 * L, 3 * L))
        rate = np.float32(rng.uniform(-1e-9, 1e-9))
        o = np.zeros((len(sh), n), np.float32)
        R.ref_high_dynamics_resampler_generic(o.ctypes.data_as(f32p), code.ctypes.data_as(f32p), rem, step, rate,
                                              sh.ctypes.data_as(f32p), L, len(sh), n)
        assert (o == O.resampler(code, rem, step, sh, n, high_dyn_rate=rate)).all(), trial


def test_oracle_f64_accumulation_variant():
    """accum_f64 keeps the reference's float products and only changes the sum: equal to the
    serial generic sum within float rounding at N = 4000, and the serial sum's drift at 1e5 stays
    at the ~1e-5 level that motivates it (tests/test_gpu_e1.py)."""
    from gnss_sim_receiver_amd import signals
    sats = signals.random_sky(2, seed=8)
    for n, lo, hi in [(4000, 0.0, 5e-6), (100000, 1e-7, 5e-5)]:
        sig = signals.generate_if(4e6 if n == 4000 else 25e6, 2 * n + 8000, sats, seed=2)  # jobs start up to one code period in
        jobs = np.concatenate([signals.truth_jobs(s, 4e6 if n == 4000 else 25e6, 1, n, [-0.25, 0, 0.25], k)
                               for k, s in enumerate(sats)])
        codes = [s.code for s in sats]
        a = O.corr_batch(sig, jobs, codes)
        b = O.corr_batch(sig, jobs, codes, accum_f64=True)
        xn = np.linalg.norm(sig[:n].astype(np.complex128))
        d = np.max(np.abs(a[:, :3] - b[:, :3]) / np.maximum(np.abs(b[:, :3]), xn))
        assert lo <= d <= hi, (n, d)

"""Generate the committed golden fixtures under tests/golden/ (run in the build container only).

    python tests/golden/make_golden.py

Sources of truth:
  * oracle/_ref/libref.so — the REFERENCE's own code generators (gps_sdr_signal_replica.cc,
    beidou_b1i_signal_replica.cc) and generic volk_gnsssdr kernels (resampler, high-dynamics
    resampler, sincos, index_max), compiled from /root/reference by oracle/Makefile;
  * oracle/liboracle.so — the clean-room restatement, for the parts the reference tree cannot
    build here (rotator dot-product: its header needs the Mako-generated volk_gnsssdr.h) and the
    acquisition core (GNU Radio / FFTW absent).  Every value that the _ref library can produce is
    produced by it, and the script asserts that the restatement agrees bit-for-bit first.

The fixtures are data only (inputs + expected outputs); no reference source text is stored.
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402

f32p = ctypes.POINTER(ctypes.c_float)


def ref_lib():
    path = os.path.join(ROOT, "oracle", "_ref", "libref.so")
    if not os.path.exists(path):
        raise SystemExit("oracle/_ref/libref.so missing: run `make -C oracle ref` (needs /root/reference)")
    L = ctypes.CDLL(path)
    L.ref_gps_l1_ca_code_gen_float.argtypes = [f32p, ctypes.c_int32, ctypes.c_uint32]
    L.ref_gps_l1_ca_code_gen_complex_sampled.argtypes = [f32p, ctypes.c_uint32, ctypes.c_int32, ctypes.c_uint32]
    L.ref_gps_l1_ca_code_gen_complex_sampled.restype = ctypes.c_int
    L.ref_beidou_b1i_code_gen_float.argtypes = [f32p, ctypes.c_int32, ctypes.c_uint32]
    L.ref_beidou_b1i_code_gen_complex_sampled.argtypes = [f32p, ctypes.c_uint32, ctypes.c_int32, ctypes.c_uint32]
    L.ref_beidou_b1i_code_gen_complex_sampled.restype = ctypes.c_int
    L.ref_resampler_generic.argtypes = [f32p, f32p, ctypes.c_float, ctypes.c_float, f32p, ctypes.c_uint, ctypes.c_int, ctypes.c_uint]
    L.ref_high_dynamics_resampler_generic.argtypes = [f32p, f32p, ctypes.c_float, ctypes.c_float, ctypes.c_float, f32p, ctypes.c_uint,
                                                      ctypes.c_int, ctypes.c_uint]
    L.ref_sincos_generic.argtypes = [f32p, ctypes.c_float, f32p, ctypes.c_uint]
    L.ref_index_max_generic.argtypes = [f32p, ctypes.c_uint]
    L.ref_index_max_generic.restype = ctypes.c_uint
    return L


def p(a):
    return a.ctypes.data_as(f32p)


def synth(fs, n, prn, doppler, delay_samples, cn0, seed, code_fn=O.gps_l1_ca_code, chip_rate=1.023e6, L=1023, carrier=1575.42e6,
          phase=0.3):
    """Numpy IF: one satellite + unit-σ complex noise."""
    rng = np.random.Generator(np.random.PCG64(seed))
    code = code_fn(prn)
    nn = np.arange(n, dtype=np.float64)
    fcode = chip_rate * (1 + doppler / carrier)
    chips = np.floor((nn - delay_samples) / fs * fcode).astype(np.int64) % L
    amp = np.sqrt(2 * 10 ** (cn0 / 10) / fs)
    x = amp * code[chips] * np.exp(1j * (2 * np.pi * doppler * nn / fs + phase))
    x = x + rng.standard_normal(n) + 1j * rng.standard_normal(n)
    return x.astype(np.complex64)


def main():
    R = ref_lib()
    out = {}

    # ---------------------------------------------------------------- F1: code tables (reference)
    gps = np.zeros((32, 1023), np.float32)
    for k in range(32):
        R.ref_gps_l1_ca_code_gen_float(p(gps[k]), k + 1, 0)
        assert (gps[k] == O.gps_l1_ca_code(k + 1)).all()
    b1i = np.zeros((63, 2046), np.float32)
    for k in range(63):
        R.ref_beidou_b1i_code_gen_float(p(b1i[k]), k + 1, 0)
        assert (b1i[k] == O.beidou_b1i_code(k + 1)).all()
    sampled = {}
    for fs in (4000000, 25000000):
        for prn in (1, 7, 32):
            n = int(fs / 1000)
            buf = np.zeros(2 * n, np.float32)
            assert R.ref_gps_l1_ca_code_gen_complex_sampled(p(buf), prn, fs, 0) == n
            assert (buf == O.gps_l1_ca_code_sampled(prn, fs).view(np.float32)).all()
            sampled[f"gps_sampled_{fs}_{prn}"] = buf[1::2].astype(np.int8)  # code in the imaginary part
    for fs in (4000000, 50000000):
        prn = 11
        n = int(fs / 1000)
        buf = np.zeros(2 * n, np.float32)
        assert R.ref_beidou_b1i_code_gen_complex_sampled(p(buf), prn, fs, 0) == n
        assert (buf == O.beidou_b1i_code_sampled(prn, fs).view(np.float32)).all()
        sampled[f"b1i_sampled_{fs}_{prn}"] = buf[0::2].astype(np.int8)
    np.savez_compressed(os.path.join(HERE, "codes_ref.npz"), gps=gps.astype(np.int8), b1i=b1i.astype(np.int8), **sampled)

    # ------------------------------------------------ F4: resampler index edge cases (reference)
    rng = np.random.Generator(np.random.PCG64(0x6E550004))
    cases = []
    res = {}
    edge = [
        # (code, rem, step, shifts, n) — negative indices, wrap past L, chip-boundary ulps
        (gps[0], 0.0, 0.25575, [-0.5, 0.0, 0.5], 4000),
        (gps[1], 0.999999, 0.25575, [-0.25, 0.0, 0.25], 4000),
        (gps[2], -1022.7, 0.04092, [-0.5, -0.25, 0.0, 0.25, 0.5], 25000),
        (gps[3], 1022.9999, 0.25575, [-0.15, 0.0, 0.15], 8000),
        (gps[4], 3.0e-7, 1.023, [-0.5, 0.0, 0.5], 2046),
        (b1i[5], 0.5, 0.04092, [-0.25, 0.0, 0.25], 50000),
        (gps[6], 5000.25, 0.25575, [-0.5, 0.0, 0.5], 4000),
    ]
    for i, (code, rem, step, shifts, n) in enumerate(edge):
        sh = np.array(shifts, np.float32)
        o = np.zeros((len(sh), n), np.float32)
        R.ref_resampler_generic(p(o), p(np.ascontiguousarray(code)), rem, step, p(sh), len(code), len(sh), n)
        assert (o == O.resampler(code, rem, step, sh, n)).all()
        res[f"rs{i}_out"] = o.astype(np.int8)
        res[f"rs{i}_args"] = np.array([rem, step, len(code), n], np.float64)
        res[f"rs{i}_shifts"] = sh
        res[f"rs{i}_codeid"] = np.array([i, 0 if len(code) == 1023 else 1])
    # high-dynamics resampler (pinned for the oracle; device path rejects rates for now)
    sh = np.array([-0.5, 0.0, 0.5], np.float32)
    o = np.zeros((3, 4000), np.float32)
    R.ref_high_dynamics_resampler_generic(p(o), p(gps[9]), 0.3, 0.25575, 1e-9, p(sh), 1023, 3, 4000)
    assert (o == O.resampler(gps[9], 0.3, 0.25575, sh, 4000, high_dyn_rate=1e-9)).all()
    res["hd_out"] = o.astype(np.int8)
    np.savez_compressed(os.path.join(HERE, "resampler_ref.npz"), **res)

    # ---------------------------------------------------------- sincos wipeoff recurrence (ref)
    sc = {}
    for i, (fd, fs, n) in enumerate([(-10000, 4e6, 4000), (1730, 4e6, 4000), (4750, 25e6, 25000)]):
        step = np.float32(np.float32(2 * np.pi) * np.float32(fd) / np.float32(fs))
        buf = np.zeros(2 * n, np.float32)
        ph = np.zeros(1, np.float32)
        R.ref_sincos_generic(p(buf), -step, p(ph), n)
        ph2 = np.zeros(1, np.float32)
        buf2 = np.zeros(2 * n, np.float32)
        O.lib().orc_sincos_generic(p(buf2), -step, p(ph2), n)
        assert (buf == buf2).all() and ph[0] == ph2[0]
        sc[f"w{i}"] = buf.view(np.complex64)
        sc[f"w{i}_args"] = np.array([fd, fs, n], np.float64)
    np.savez_compressed(os.path.join(HERE, "sincos_ref.npz"), **sc)

    # ------------------------------------------------------------ F2: correlator cases (oracle)
    # Rotator dot-product restated (reference header unbuildable), fed by the pinned resampler.
    corr = {}
    specs = []
    rng = np.random.Generator(np.random.PCG64(0x6E550002))
    for i in range(10):
        fs, n, ntaps = [(4e6, 4000, 3), (4e6, 4000, 3), (4e6, 4000, 3), (4e6, 4000, 3), (4e6, 4000, 5), (4e6, 4001, 3),
                        (25e6, 25000, 3), (25e6, 25000, 5), (4e6, 3999, 1), (2.046e6, 2046, 3)][i]
        prn = int(rng.integers(1, 33))
        fd = float(rng.uniform(-5000, 5000))
        code_fn = O.gps_l1_ca_code
        sig = synth(fs, n + 64, prn, fd, float(rng.uniform(0, 40)), 45.0, seed=100 + i)
        shifts = {1: [0.0], 3: [-0.25, 0.0, 0.25], 5: [-0.5, -0.25, 0.0, 0.25, 0.5]}[ntaps]
        rem_carr = float(np.float32(rng.uniform(-np.pi, np.pi)))
        carr_step = float(np.float32(2 * np.pi * fd / fs))
        rem_code = float(np.float32(rng.uniform(-1.0, 1.0)))
        code_step = float(np.float32(1.023e6 * (1 + fd / 1575.42e6) / fs))
        x = sig[:n]
        out_ = O.multicorrelator(x, code_fn(prn), np.array(shifts, np.float32), rem_carr, carr_step, rem_code, code_step)
        corr[f"c{i}_sig"] = x
        corr[f"c{i}_args"] = np.array([prn, n, rem_carr, carr_step, rem_code, code_step], np.float64)
        corr[f"c{i}_shifts"] = np.array(shifts, np.float32)
        corr[f"c{i}_out"] = out_
    np.savez_compressed(os.path.join(HERE, "corr_cases.npz"), **corr)

    # ------------------------------------------------------------ F3: acquisition cases (oracle)
    acq = {}
    # C1 of BASELINE.md: PRN 7, fD 1730 Hz, delay 1234 samples, CN0 45, 4 Msps, dmax 10000, step 250 (80 bins)
    cases = [
        dict(fs=4000000, prn=7, fd=1730.0, delay=1234, cn0=45.0, dmax=10000, step=250, cfar=1, seed=0x6E550001),
        dict(fs=4000000, prn=7, fd=1730.0, delay=1234, cn0=45.0, dmax=10000, step=250, cfar=0, seed=0x6E550001),
        dict(fs=4000000, prn=23, fd=-3312.0, delay=17, cn0=47.0, dmax=5000, step=250, cfar=1, seed=0x6E550011),
        dict(fs=4000000, prn=3, fd=4102.0, delay=3990, cn0=46.0, dmax=5000, step=500, cfar=0, seed=0x6E550012),
        dict(fs=2048000, prn=12, fd=-777.0, delay=1000, cn0=48.0, dmax=6000, step=250, cfar=1, seed=0x6E550013),
    ]
    for i, c in enumerate(cases):
        n = int(c["fs"] / 1000)
        sig = synth(c["fs"], n, c["prn"], c["fd"], c["delay"], c["cn0"], c["seed"])
        code = O.gps_l1_ca_code_sampled(c["prn"], c["fs"])
        r, grid = O.pcps_acquisition_core(sig, code, c["fs"], c["dmax"], c["step"], 0, bool(c["cfar"]))
        r32, _ = O.pcps_acquisition_core(sig, code, c["fs"], c["dmax"], c["step"], 0, bool(c["cfar"]), fft_dtype=np.complex64)
        assert (r.doppler_index, r.code_index) == (r32.doppler_index, r32.code_index), "peak not stable between fp64/fp32 FFT"
        flat = np.sort(grid.ravel())
        acq[f"a{i}_sig"] = sig
        acq[f"a{i}_conf"] = np.array([c["fs"], c["prn"], c["dmax"], c["step"], c["cfar"]], np.int64)
        acq[f"a{i}_expect_idx"] = np.array([r.doppler_index, r.code_index, r.doppler_hz], np.int64)
        acq[f"a{i}_expect_val"] = np.array([r.peak, r.input_power, r.test_statistic, r.acq_delay_samples], np.float64)
        acq[f"a{i}_margin"] = np.array([flat[-1] / flat[-2]], np.float64)
        print(f"acq case {i}: bin {r.doppler_index} idx {r.code_index} fd {r.doppler_hz} stat {r.test_statistic:.3f} "
              f"margin {flat[-1] / flat[-2]:.4f}")
    np.savez_compressed(os.path.join(HERE, "acq_cases.npz"), **acq)
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == "__main__":
    main()

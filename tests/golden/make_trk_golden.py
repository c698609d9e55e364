"""Golden vectors for the tracking-loop oracle from the REFERENCE's own classes (build container).

    make -C oracle ref && python tests/golden/make_trk_golden.py

oracle/_ref/libref.so carries Tracking_FLL_PLL_filter (tracking_FLL_PLL_filter.cc) and
Exponential_Smoother (exponential_smoother.cc) compiled from /root/reference.  This script runs
them on seeded inputs and stores inputs + outputs in tests/golden/trk_ref.npz (data only).
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
f32p = ctypes.POINTER(ctypes.c_float)


def p(a):
    return a.ctypes.data_as(f32p)


def main():
    L = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libref.so"))
    L.ref_fll_pll_run.argtypes = [ctypes.c_float, ctypes.c_float, ctypes.c_int, ctypes.c_float, f32p, f32p, f32p, ctypes.c_int, f32p]
    L.ref_smoother_run.argtypes = [ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_int, f32p, ctypes.c_int, f32p]
    rng = np.random.default_rng(2024)
    out = {}
    n = 500
    for k, (fll, pll, order, dop) in enumerate([(35.0, 35.0, 3, 1234.5), (10.0, 15.0, 2, -3210.0), (35.0, 40.0, 3, 0.0)]):
        f = rng.normal(0, 2.0, n).astype(np.float32)
        ph = rng.normal(0, 0.05, n).astype(np.float32)
        T = np.full(n, 0.001 if k != 1 else 0.004, np.float32)
        if k == 0:
            f[:] = 0.0
        y = np.zeros(n, np.float32)
        L.ref_fll_pll_run(fll, pll, order, dop, p(f), p(ph), p(T), n, p(y))
        out[f"fp{k}_params"] = np.array([fll, pll, order, dop], np.float64)
        out[f"fp{k}_in"] = np.stack([f, ph, T])
        out[f"fp{k}_out"] = y
    for k, (alpha, mn, off, ns, mean) in enumerate([(0.002, 25.0, 12.0, 200, 44.0), (0.002, -1.0, 0.0, 25, 0.9),
                                                     (0.01, 25.0, 12.0, 50, 30.0)]):
        raw = (mean + rng.normal(0, 1.5, 700)).astype(np.float32)
        y = np.zeros(len(raw), np.float32)
        L.ref_smoother_run(alpha, mn, off, ns, p(raw), len(raw), p(y))
        out[f"sm{k}_params"] = np.array([alpha, mn, off, ns], np.float64)
        out[f"sm{k}_in"] = raw
        out[f"sm{k}_out"] = y
    np.savez_compressed(os.path.join(HERE, "trk_ref.npz"), **out)
    print("wrote trk_ref.npz")


if __name__ == "__main__":
    main()

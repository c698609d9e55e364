"""A/B of two builds of the acquisition engine, byte for byte: the C3 sweep (32 PRNs x 40 bins x
25000) and the C1-shape sweep (32 x 81 x 4000) with the grid returned, each build in its own
process (the library is chosen by GNSSHIP_LIB_PATH), results and timings compared.
    python scripts/acq_ab.py scripts/libgnsship_base.so gnss_sim_receiver_amd/libgnsship.so [--tolerant]
Either side may carry environment settings after a colon: lib.so:GNSSHIP_ACQ_GRAPH=0.
--tolerant: a different FFT factorisation (other rounding) passes when every PRN's Doppler and code
delay agree exactly; the test-statistic difference is reported."""
import hashlib
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_one(out):
    sys.path.insert(0, ROOT)
    from gnss_sim_receiver_amd import codes as C, engine, signals as S
    ctx = engine.Context(0)
    res = {}
    for tag, fs, n, dmax, sky, seed in (("c3", 25000000, 25000, 5000, S.c3_sky(), 0x6E550003),
                                        ("c1", 4000000, 4000, 10000, S.random_sky(32, seed=0x6E550002), 0x6E550002)):
        sig = S.generate_if(fs, n, sky, seed=seed)
        acq = engine.PcpsAcquisition(ctx, fs, n, dmax, 250, 0, True, max_prns=32)
        for k in range(32):
            acq.set_local_code(C.gps_l1_ca_code_gen_complex_sampled(k + 1, fs), k)
        dev = ctx.upload(np.ascontiguousarray(sig))
        r, grid = acq.run(dev, n_prns=32, want_grid=True)
        res[tag] = np.frombuffer(b"".join(bytes(x) for x in r), np.uint8)
        res[tag + "_grid"] = np.frombuffer(hashlib.sha256(np.ascontiguousarray(grid).tobytes()).digest(), np.uint8)
        acq.run(dev, n_prns=32)
        ctx.sync()
        t0 = time.perf_counter()
        for _ in range(20):
            acq.run(dev, n_prns=32)
        res[tag + "_ms"] = np.array((time.perf_counter() - t0) / 20 * 1e3)
        acq.close()
        dev.free()
    # Galileo E1 all-sky (huge layout, N = 100000), results only (the grid would be 512 MB)
    fs, n = 25000000, 100000
    sats = S.random_sky(6, seed=0x6E550007, system="GAL", prns=[2, 9, 13, 21, 26, 31])
    sig = S.generate_if(fs, n, sats, seed=0x6E550007)
    acq = engine.PcpsAcquisition(ctx, fs, n, 5000, 250, 0, False, max_prns=32, ms_per_code=4)
    for k in range(32):
        acq.set_local_code(C.galileo_e1_code_gen_complex_sampled("1B", False, k + 1, fs), k)
    dev = ctx.upload(np.ascontiguousarray(sig))
    r, _ = acq.run(dev, n_prns=32)
    res["e1"] = np.frombuffer(b"".join(bytes(x) for x in r), np.uint8)
    res["e1_grid"] = np.zeros(1, np.uint8)
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(5):
        acq.run(dev, n_prns=32)
    res["e1_ms"] = np.array((time.perf_counter() - t0) / 5 * 1e3)
    acq.close()
    dev.free()
    ctx.close()
    np.savez(out, **res)


TOLERANT = False


def main():
    sys.path.insert(0, ROOT)
    from gnss_sim_receiver_amd import abi  # noqa: F401 (result dtype)
    globals()["abi"] = abi
    if sys.argv[1] == "--one":
        run_one(sys.argv[2])
        return
    global TOLERANT
    TOLERANT = "--tolerant" in sys.argv
    libs = [x for x in sys.argv[1:] if not x.startswith("--")]
    outs = []
    for i, spec in enumerate(libs[:2]):
        lib, _, extra = spec.partition(":")  # lib.so[:ENV=value,ENV2=value]
        out = os.path.join(ROOT, "gpurun_out", f"acq_ab_{i}.npz")
        os.makedirs(os.path.dirname(out), exist_ok=True)
        env = dict(os.environ, GNSSHIP_LIB_PATH=os.path.abspath(lib))
        env.update(kv.split("=", 1) for kv in extra.split(",") if kv)
        subprocess.run([sys.executable, os.path.abspath(__file__), "--one", out], env=env, check=True, timeout=300)
        outs.append(np.load(out))
    a, b = outs
    ok = True
    for tag in ("c3", "c1", "e1"):
        same = a[tag].tobytes() == b[tag].tobytes()
        gsame = a[tag + "_grid"].tobytes() == b[tag + "_grid"].tobytes()
        ra, rb = (np.frombuffer(x[tag].tobytes(), np.dtype(abi.AcqResult)) for x in (a, b))
        cells = all(np.array_equal(ra[f], rb[f]) for f in ("doppler_hz", "acq_delay_samples"))
        rel = float(np.max(np.abs(ra["test_statistic"] - rb["test_statistic"]) / np.abs(rb["test_statistic"])))
        ok &= cells if TOLERANT else (same and gsame)
        bad = [k for k in range(len(ra)) if bytes(ra[k]) != bytes(rb[k])]
        for k in bad[:6]:
            print(f"  {tag} prn slot {k}: " + ", ".join(f"{f} {ra[f][k]} / {rb[f][k]}" for f in ("doppler_hz", "acq_delay_samples", "peak", "test_statistic")))
        print(f"{tag}: results identical {same}, grid identical {gsame}, peaks (Doppler, delay) identical {cells}, "
              f"test statistic max rel diff {rel:.2e}; sweep {float(a[tag + '_ms']):.3f} -> {float(b[tag + '_ms']):.3f} ms")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()

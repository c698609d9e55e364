"""Acquisition sweeps for profiling (rocprofv3): C3 (32 PRN x 40 bins x 25000, 25 Msps, BASELINE's
signal), the C1 shape (32 PRN x 40 bins x 4000, 4 Msps) and the Galileo E1 all-sky sweep (32 PRN x
41 bins x 100000, huge layout), `reps` each after a warm-up.
    python scripts/acq_probe.py [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from gnss_sim_receiver_amd import codes as C, engine, signals as S  # noqa: E402


def sweep(ctx, fs, n, sig, reps, e1=False):
    if e1:
        acq = engine.PcpsAcquisition(ctx, fs, n, 5000, 250, 0, False, max_prns=32, ms_per_code=4)
        for k in range(32):
            acq.set_local_code(C.galileo_e1_code_gen_complex_sampled("1B", False, k + 1, fs), k)
    else:
        acq = engine.PcpsAcquisition(ctx, fs, n, 5000, 250, 0, True, max_prns=32)
        for k in range(32):
            acq.set_local_code(C.gps_l1_ca_code_gen_complex_sampled(k + 1, fs), k)
    dev = ctx.upload(np.ascontiguousarray(sig[:n]))
    res, _ = acq.run(dev, n_prns=32)
    t0 = time.perf_counter()
    for _ in range(reps):
        res, _ = acq.run(dev, n_prns=32)
    dt = (time.perf_counter() - t0) / reps
    acq.close()
    dev.free()
    return dt, res


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    ctx = engine.Context(0)
    c3 = S.c3_sky()
    dt3, r3 = sweep(ctx, 25000000, 25000, S.generate_if(25000000, 25000, c3, seed=0x6E550003), reps)
    sky = S.random_sky(32, seed=0x6E550002)
    dt1, r1 = sweep(ctx, 4000000, 4000, S.generate_if(4000000, 4000, sky, seed=0x6E550002), reps)
    gal = S.random_sky(6, seed=0x6E550007, system="GAL", prns=[2, 9, 13, 21, 26, 31])
    dte, _ = sweep(ctx, 25000000, 100000, S.generate_if(25000000, 100000, gal, seed=0x6E550007), max(1, reps // 4), e1=True)
    print(f"E1 all-sky sweep {dte * 1e3:.3f} ms")
    present = sorted(s.prn for s in c3)
    top = sorted(range(32), key=lambda k: -r3[k].test_statistic)[:10]
    hits = len(set(k + 1 for k in top) & set(present))  # a sanity count only: parity is tests/test_gpu_acq.py
    print(f"C3 sweep {dt3 * 1e3:.3f} ms, C1-shape sweep {dt1 * 1e3:.3f} ms; present PRNs among the 10 largest C3 statistics: {hits}/10")
    ctx.close()


if __name__ == "__main__":
    main()

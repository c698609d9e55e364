"""Phase timeline of acq_search_big_kernel (C3: 32 PRN x 40 bins x 25000) from the profiling build.
    make prof && python scripts/acq_wg_profile.py
Stamps (wall_clock64, 100 MHz) per workgroup: 0 start, 1 round-1 inputs in LDS, 2 round-1 rows done,
3 round-1 gathered, 4/5/6 the same for round 2, 7 |y|^2 done, 8 max+sum reduced, 9 second peak."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("GNSSHIP_LIB_PATH", os.path.join(os.path.dirname(os.path.abspath(__file__)), "libgnsship_prof.so"))
import numpy as np  # noqa: E402

from gnss_sim_receiver_amd import abi, codes as C, engine, signals as S  # noqa: E402


def main():
    lib = abi.load()
    lib.gnsship_debug_acq_profile.argtypes = [ctypes.c_void_p]
    ctx = engine.Context(0)
    fs, n = 25000000, 25000
    sig = S.generate_if(fs, n, S.c3_sky(), seed=0x6E550003)
    acq = engine.PcpsAcquisition(ctx, fs, n, 5000, 250, 0, True, max_prns=32)
    for k in range(32):
        acq.set_local_code(C.gps_l1_ca_code_gen_complex_sampled(k + 1, fs), k)
    dev = ctx.upload(sig)
    acq.run(dev, n_prns=32)
    cells = 32 * acq.n_bins
    prof = engine.DeviceBuffer(ctx, cells * 16 * 8)
    prof.upload(np.zeros(cells * 16, np.uint64))
    lib.gnsship_debug_acq_profile(ctypes.c_void_p(prof.ptr))
    acq.run(dev, n_prns=32)
    ctx.sync()
    lib.gnsship_debug_acq_profile(ctypes.c_void_p(0))
    t = np.zeros(cells * 16, np.uint64)
    prof.download(t)
    t = t.reshape(cells, 16).astype(np.int64)
    names = ["round-1 loads", "round-1 rows", "round-1 gather", "round-2 loads", "round-2 rows", "round-2 gather", "col DFT + |y|^2",
             "max/sum reduce", "second peak"]
    print(f"cell wall median {np.median(t[:, 9] - t[:, 0]) / 100:.2f} us; span of the launch {(t[:, 9].max() - t[:, 0].min()) / 100:.1f} us")
    for k, nm in enumerate(names):
        d = (t[:, k + 1] - t[:, k]) / 100.0
        print(f"  {nm:18s} median {np.median(d):7.2f} us  p90 {np.percentile(d, 90):7.2f}")
    w = lambda a, b: np.median(t[:, b] - t[:, a]) / 100.0
    print(f"  per wave: wave 0 col DFT {w(6, 10):.2f} us, stats {w(10, 7):.2f}; wave 15 col DFT {w(6, 11):.2f}, stats {w(11, 12):.2f}; "
          f"wave 15 done -> reduced {w(12, 8):.2f}")
    ctx.close()


if __name__ == "__main__":
    main()

"""Workgroup phase timeline of corr_batch_kernel on the bench workload (C2: 12 000 jobs).

    make prof && GNSSHIP_LIB_PATH=scripts/libgnsship_prof.so python scripts/corr_wg_profile.py

Stamps (wall_clock64, 100 MHz) per workgroup: 0 entry, 1 code in LDS, 2/6 chunk 0/1 set up,
3/7 chunk 0/1 main loop done, 4 end (5: end of an anchor-prefetch workgroup).  Each stamp waits
for the wave's outstanding scalar and LDS operations (lgkmcnt), so a phase boundary lands after
the loads issued before it.  Prints phase-duration percentiles, the
workgroup lifetime, and how many workgroups were resident over the kernel."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from gnss_sim_receiver_amd import abi, engine, signals  # noqa: E402


def main():
    os.environ.setdefault("GNSSHIP_LIB_PATH", os.path.join(os.path.dirname(os.path.abspath(__file__)), "libgnsship_prof.so"))
    lib = abi.load()
    lib.gnsship_debug_corr_profile.argtypes = [ctypes.c_void_p]
    sats = signals.random_sky(bench.N_SATS, seed=bench.SEED)  # the bench's open-loop block
    n = bench.FS + 2 * bench.VL
    block = np.ascontiguousarray(signals.generate_if(bench.FS, n, sats, seed=bench.SEED))
    ctx = engine.Context(0)
    jobs, codes = bench.receiver_jobs(sats, 0, 1.0)
    for cid, c in enumerate(codes):
        ctx.set_code(cid, c)
    b = engine.CorrelatorBatch(ctx, len(jobs))
    b.set_jobs(jobs, n)
    b2 = engine.CorrelatorBatch(ctx, len(jobs))
    b2.set_jobs(jobs, n)
    dev = ctx.upload(block)
    grid = len(jobs) + 64
    prof = engine.DeviceBuffer(ctx, grid * 8 * 8)
    prof.upload(np.zeros(grid * 8, np.uint64))
    mode = sys.argv[1] if len(sys.argv) > 1 else "pipelined"
    for _ in range(3):
        b.launch_pipelined(dev.ptr, abi.FMT_CF32, b2)
        b2.launch_pipelined(dev.ptr, abi.FMT_CF32, b)
    ctx.sync()
    lib.gnsship_debug_corr_profile(ctypes.c_void_p(prof.ptr))
    if mode == "pipelined":
        b.launch_pipelined(dev.ptr, abi.FMT_CF32, b2)
    else:
        b.launch_ptr(dev.ptr, abi.FMT_CF32, abi.STAGE_CORRELATE)
    ctx.sync()
    lib.gnsship_debug_corr_profile(ctypes.c_void_p(0))
    t = np.zeros(grid * 8, np.uint64)
    prof.download(t)
    t = t.reshape(grid, 8).astype(np.int64)
    corr = t[(t[:, 4] > 0)]
    anc = t[(t[:, 5] > 0)]
    t0 = corr[:, 0].min()
    us = lambda v: v / 100.0  # noqa: E731  (100 MHz → µs)
    print(f"mode {mode}: {len(corr)} correlation WGs, {len(anc)} anchor WGs; kernel span {us(corr[:, 4].max() - t0):.1f} us")
    two = corr[corr[:, 6] > 0]  # items of two or more chunks: chunk 1 start (6) / main-loop end (7)
    one = corr[corr[:, 6] == 0]
    phases = [("code->LDS", corr, 0, 1), ("chunk0 start", corr, 1, 2), ("chunk0 loop", corr, 2, 3)]
    if len(two):
        phases += [("wave sums+c1 start", two, 3, 6), ("chunk1 loop", two, 6, 7), ("reduce+store", two, 7, 4)]
    if len(one):
        phases += [("reduce+store(1)", one, 3, 4)]
    for name, rows, a, b in phases:
        d = us(rows[:, b] - rows[:, a])
        print(f"  {name:19s} n {len(rows):5d} p10 {np.percentile(d, 10):6.2f}  p50 {np.percentile(d, 50):6.2f}  p90 {np.percentile(d, 90):6.2f} us")
    life = us(corr[:, 4] - corr[:, 0])
    print(f"  WG lifetime   p10 {np.percentile(life, 10):6.2f}  p50 {np.percentile(life, 50):6.2f}  p90 {np.percentile(life, 90):6.2f} us")
    if len(anc):
        print(f"  anchor WGs    start {us(anc[:, 0].min() - t0):.1f}..{us(anc[:, 0].max() - t0):.1f}  end {us(anc[:, 5].max() - t0):.1f} us")
    # residency over time
    edges = np.linspace(0, corr[:, 4].max() - t0, 21)
    act = [int(np.sum((corr[:, 0] - t0 <= e) & (corr[:, 4] - t0 > e))) for e in edges[:-1]]
    print("  resident correlation WGs at 5% steps:", act)
    starts = np.sort(us(corr[:, 0] - t0))
    print("  WG start times p0/p25/p50/p75/p100:", [round(float(np.percentile(starts, q)), 1) for q in (0, 25, 50, 75, 100)])


if __name__ == "__main__":
    main()

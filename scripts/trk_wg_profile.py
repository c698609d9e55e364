"""Epoch phase timeline of the persistent tracking kernel (trk_persist.hip), C2 workload.

    make prof && python scripts/trk_wg_profile.py [rotator 0|1] [channels] [sync]

Stamps (wall_clock64, 100 MHz) per channel-epoch: 0 epoch start, 1 job derived (thread 0),
2 replay done (wave 0), 3/4 wave 0 / wave 1 correlation done, 5 taps reduced, 6 loop update done;
inside the loop update 8 before lock_status, 9 after it, 10 after run_dll_pll, 11 after
update_tracking_vars, 12 after log_data (state 2 only).  `sync`: the satellites carry GPS
navigation bits and the acquisition is stamped pull_in_time_s before the block, so the channels
bit-synchronise and the profiled epochs run in state 4 (steady state), as in bench.py.
Inside the AVX replay (wave 0, lane 0): 13 start phasors and iteration 0 done, 14 task loop done,
15 tail published."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("GNSSHIP_LIB_PATH", os.path.join(os.path.dirname(os.path.abspath(__file__)), "libgnsship_prof.so"))
import numpy as np  # noqa: E402

from gnss_sim_receiver_amd import abi, engine, signals  # noqa: E402

EP = 64
SLOTS = 32


def main():
    rot = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    n_ch = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    state4 = len(sys.argv) > 3 and sys.argv[3] == "sync"
    fs, vl = 4e6, 4000
    lib = abi.load()
    lib.gnsship_debug_trk_profile.argtypes = [ctypes.c_void_p]
    ctx = engine.Context(0)
    sats = signals.random_sky(32, seed=0x6E550002)
    # sync: bench.py's steady state — GPS navigation bits (the preamble recurring every 260 ms),
    # tracking from 11 s after the acquisition stamp (pull_in_time_s elapsed), 0.5 s of pre-roll
    first = int(11 * fs) if state4 else 0
    if state4:
        for s in sats:
            s.bits = "1000101100110"
    pre = 500 if state4 else 4
    block = signals.generate_if(fs, (pre + EP + 4) * vl, sats, seed=1, start=first - 2 * vl)
    trk = engine.DllPllVemlTracking(ctx, abi.TrkConf.defaults(abi.SYS_GPS_L1CA, fs, vl, rotator=rot), n_ch)
    for i, s in enumerate(sats):
        ctx.set_code(300 + i, s.code)
    for ch in range(n_ch):
        s = sats[ch % 32]
        trk.start(ch, 300 + ch % 32, signals.acq_delay_samples(s, fs, 0, first), s.doppler_hz, 0, first)
    dev = ctx.upload(block)
    trk.run(dev, first - 2 * vl, pre, n_buffer_samples=len(block), records=False)
    prof = engine.DeviceBuffer(ctx, n_ch * EP * SLOTS * 8)
    prof.upload(np.zeros(n_ch * EP * SLOTS, np.uint64))
    lib.gnsship_debug_trk_profile(ctypes.c_void_p(prof.ptr))
    trk.run(dev, first - 2 * vl, EP, n_buffer_samples=len(block), records=False)
    ctx.sync()
    lib.gnsship_debug_trk_profile(ctypes.c_void_p(0))
    print("states:", sorted(set(trk.channel_state(ch)[0] for ch in range(n_ch))))
    t = np.zeros(n_ch * EP * SLOTS, np.uint64)
    prof.download(t)
    t = t.reshape(n_ch, EP, SLOTS).astype(np.int64)
    us = lambda v: v / 100.0  # noqa: E731
    names = ["derive", "->replay done", "->wave0 corr done", "->wave1 corr done", "->reduced", "->loop update",
             " update: to lock_status", " update: lock_status", " update: run_dll_pll", " update: tracking_vars",
             " update: log_data (st2)", " update: sync+rest (st2)", " update: rest (st4)",
             " replay: start phasors", " replay: task loop", " replay: tail + publish", "end -> next epoch",
             "->wave2 corr done", "->wave3 corr done", "->wave0 sums stored", "->wave1 sums stored", "->wave2 sums stored",
             "->wave3 sums stored"]
    refs = [(0, 1), (1, 2), (1, 3), (1, 4), (1, 5), (5, 6), (5, 8), (8, 9), (9, 10), (10, 11), (11, 12), (12, 6), (11, 6),
            (1, 13), (13, 14), (14, 15), (6, 32), (1, 16), (1, 17), (1, 18), (1, 19), (1, 20), (1, 21)]
    cyc = t[:, 1:-1, 7]
    loop_us = (t[:, 1:-1, 14] - t[:, 1:-1, 13]) / 100.0
    if (cyc > 0).any():
        print(f"replay task loop: {np.median(cyc):.0f} shader cycles, effective clock {np.median(cyc / loop_us) / 1e3:.2f} GHz")
    nxt = np.concatenate([t[:, 1:, 0:1], np.zeros((n_ch, 1, 1), np.int64)], axis=1)
    t = np.concatenate([t, nxt], axis=2)
    v = t[:, 1:-1, :]  # drop first/last epoch
    print(f"rotator {rot}, {n_ch} channels: epoch period {us(np.median(np.diff(t[:, :, 0], axis=1))):.2f} us (median)")
    for nm, (a, b) in zip(names, refs):
        ok = (v[:, :, a] > 0) & (v[:, :, b] > 0)
        if nm.endswith("(st4)"):
            ok &= v[:, :, 12] == 0
        if nm.endswith("(st2)"):
            ok &= v[:, :, 12] > 0
        if not ok.any():
            continue
        d = us(v[:, :, b] - v[:, :, a])[ok]
        print(f"  {nm:26s} median {np.median(d):7.2f} us  p90 {np.percentile(d, 90):7.2f}  (n={ok.sum()})")
    trk.close()
    ctx.close()


if __name__ == "__main__":
    main()

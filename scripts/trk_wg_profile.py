"""Epoch phase timeline of the persistent tracking kernel (trk_persist.hip), C2 workload.

    make prof && python scripts/trk_wg_profile.py [rotator 0|1] [channels] [sync]

Stamps (wall_clock64, 100 MHz) per channel-epoch: 0 epoch start, 1 job derived (thread 0),
2 replay done (wave 0), 3/4 wave 0 / wave 1 correlation done, 5 taps reduced, 6 loop update done;
inside the loop update 8 before lock_status, 9 after it, 10 after run_dll_pll, 11 after
update_tracking_vars, 12 after log_data (state 2 only).  `sync`: the satellites carry GPS
navigation bits and the acquisition is stamped pull_in_time_s before the block, so the channels
bit-synchronise and the profiled epochs run in state 4 (steady state)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("GNSSHIP_LIB_PATH", os.path.join(os.path.dirname(os.path.abspath(__file__)), "libgnsship_prof.so"))
import numpy as np  # noqa: E402

from gnss_sim_receiver_amd import abi, engine, signals  # noqa: E402

EP = 64


def main():
    rot = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    n_ch = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    state4 = len(sys.argv) > 3 and sys.argv[3] == "sync"
    fs, vl = 4e6, 4000
    lib = abi.load()
    lib.gnsship_debug_trk_profile.argtypes = [ctypes.c_void_p]
    ctx = engine.Context(0)
    sats = signals.random_sky(32, seed=0x6E550002)
    first = int(10 * fs) if state4 else 0  # acquisition stamped 10 s (pull_in_time_s) before the block
    if state4:
        for s in sats:
            s.bits = "10001011" + "0110100111010010" * 8  # GPS preamble + filler bits (bit sync, state 4)
    block = signals.generate_if(fs, int(fs * (0.4 if state4 else 0.1)) + 8000, sats, seed=1, start=first)
    trk = engine.DllPllVemlTracking(ctx, abi.TrkConf.defaults(abi.SYS_GPS_L1CA, fs, vl, rotator=rot), n_ch)
    for i, s in enumerate(sats):
        ctx.set_code(300 + i, s.code)
    for ch in range(n_ch):
        s = sats[ch % 32]
        # Acq_delay_samples of an acquisition stamped at sample 0 (the code start after `first`, with code Doppler)
        m = np.ceil(s.chip_phase(np.float64(first), fs) / s.code_len)
        n0 = (m * s.code_len + s.code_delay_chips) * fs / s.code_freq()
        delay = first + np.mod(n0 - first, 1e-3 * fs)
        trk.start(ch, 300 + ch % 32, delay, s.doppler_hz, 0, first)
    dev = ctx.upload(block)
    trk.run(dev, first, 300 if state4 else 4, n_buffer_samples=len(block), records=False)
    prof = engine.DeviceBuffer(ctx, n_ch * EP * 16 * 8)
    prof.upload(np.zeros(n_ch * EP * 16, np.uint64))
    lib.gnsship_debug_trk_profile(ctypes.c_void_p(prof.ptr))
    trk.run(dev, first, EP, n_buffer_samples=len(block), records=False)
    ctx.sync()
    lib.gnsship_debug_trk_profile(ctypes.c_void_p(0))
    print("states:", sorted(set(trk.channel_state(ch)[0] for ch in range(n_ch))))
    t = np.zeros(n_ch * EP * 16, np.uint64)
    prof.download(t)
    t = t.reshape(n_ch, EP, 16).astype(np.int64)
    us = lambda v: v / 100.0  # noqa: E731
    names = ["derive", "->replay done", "->wave0 corr done", "->wave1 corr done", "->reduced", "->loop update",
             " update: to lock_status", " update: lock_status", " update: run_dll_pll", " update: tracking_vars",
             " update: log_data (st2)", " update: sync+rest (st2)", " update: rest (st4)"]
    refs = [(0, 1), (1, 2), (1, 3), (1, 4), (1, 5), (5, 6), (5, 8), (8, 9), (9, 10), (10, 11), (11, 12), (12, 6), (11, 6)]
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

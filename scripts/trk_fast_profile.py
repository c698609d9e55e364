"""Epoch phase timeline of the fast AVX persistent tracking kernel (trk_fast.hip), C2 workload.

    make prof && python scripts/trk_fast_profile.py [channels]

Stamps (wall_clock64, 100 MHz) per channel-epoch, lane 0 of the stamping wave: 0 derive start (wave 1),
1 job published, 2 replay + tail done (wave 1), 3/4 producer waves 2/3 done, 5 accumulation done
(wave 0), 6 taps combined and stored, 7 loop update + records done; 8 lock_status start (wave 2),
9 run_dll_pll start, 10 its end, 11 update_tracking_vars end (wave 0).  The channels bit-synchronise
first (state 4, as in bench.py)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("GNSSHIP_LIB_PATH", os.path.join(os.path.dirname(os.path.abspath(__file__)), "libgnsship_prof.so"))
import numpy as np  # noqa: E402

from gnss_sim_receiver_amd import abi, engine, signals  # noqa: E402

EP = 16  # epochs 8-23 of the profiled launch (trk_fast.hip kFProfFirst)
RUN = 64  # epochs in the profiled launch
SLOTS = 88


def main():
    n_ch = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    fs = float(sys.argv[2]) if len(sys.argv) > 2 else 4e6
    vl = int(round(fs / 1000))
    lib = abi.load()
    lib.gnsship_debug_trk_fast_profile.argtypes = [ctypes.c_void_p]
    ctx = engine.Context(0)
    sats = signals.random_sky(32, seed=0x6E550002)
    first = int(11 * fs)
    for s in sats:
        s.bits = "1000101100110"
    pre = 500
    block = signals.generate_if(fs, (pre + RUN + 4) * vl, sats, seed=1, start=first - 2 * vl)
    trk = engine.DllPllVemlTracking(ctx, abi.TrkConf.defaults(abi.SYS_GPS_L1CA, fs, vl, rotator=abi.ROTATOR_AVX), n_ch)
    for i, s in enumerate(sats):
        ctx.set_code(300 + i, s.code)
    for ch in range(n_ch):
        s = sats[ch % 32]
        trk.start(ch, 300 + ch % 32, signals.acq_delay_samples(s, fs, 0, first), s.doppler_hz, 0, first)
    dev = ctx.upload(block)
    trk.run(dev, first - 2 * vl, pre, n_buffer_samples=len(block), records=False)
    prof = engine.DeviceBuffer(ctx, n_ch * EP * SLOTS * 8)
    prof.upload(np.zeros(n_ch * EP * SLOTS, np.uint64))
    lib.gnsship_debug_trk_fast_profile(ctypes.c_void_p(prof.ptr))
    ctx.event_record(0)
    trk.run(dev, first - 2 * vl, RUN, n_buffer_samples=len(block), records=False)
    ctx.event_record(1)
    ms = ctx.event_elapsed_ms(0, 1)
    lib.gnsship_debug_trk_fast_profile(ctypes.c_void_p(0))
    print("states:", sorted(set(trk.channel_state(ch)[0] for ch in range(n_ch))), f"launch {ms:.3f} ms for {RUN} epochs")
    t = np.zeros(n_ch * EP * SLOTS, np.uint64)
    prof.download(t)
    t = t.reshape(n_ch, EP, SLOTS).astype(np.int64)
    us = lambda v: v / 100.0  # noqa: E731
    nxt = np.concatenate([t[:, 1:, :], np.zeros((n_ch, 1, SLOTS), np.int64)], axis=1)
    t = np.concatenate([t, nxt], axis=2)  # slots SLOTS + k = the next epoch's slot k
    v = t[:, 1:-1, :]
    print(f"{n_ch} channels: epoch period {us(np.median(np.diff(t[:, :, 0], axis=1))):.2f} us (median)")
    rows = [("derive", 0, 1), ("derive -> replay done", 1, 2), ("derive -> producer 2 done", 1, 3), ("derive -> producer 3 done", 1, 4),
            ("derive -> accumulation done", 1, 5), ("replay done -> accumulation done", 2, 5), ("accumulation -> taps stored", 5, 6),
            ("taps stored -> loop done", 6, 7), ("  taps -> run_dll_pll", 6, 9), ("  run_dll_pll", 9, 10), ("  update_tracking_vars", 10, 11),
            ("  tracking_vars -> loop done", 11, 7), ("loop done -> next derive", 7, SLOTS), ("  taps -> epoch_pre done", 16, 17),
            ("  epoch_pre -> published", 17, 18), ("  published -> run_dll_pll", 18, 9), ("  lock_status (wave 2)", 8, 26),
            ("  tracking_vars -> lock seen", 11, 19), ("  lock seen -> epoch_post done", 19, 24), ("  epoch_finish", 24, 25),
            ("  epoch_finish -> loop done (records)", 25, 7), ("seed (tracking_vars) -> next derive start", 11, SLOTS), ("  tracking_vars -> seed published", 11, 33), ("  seed published -> next derive start", 33, SLOTS), ("derive: sincos", 0, 35), ("derive: chains", 35, 36), ("derive: dz + publish", 36, 1), ("  run_dll_pll: PLL discriminator", 9, 37), ("  run_dll_pll: carrier filter", 37, 38), ("  run_dll_pll: DLL discriminator", 38, 39), ("  run_dll_pll: code loop filter", 39, 40), ("  run_dll_pll: code freq", 40, 10),
            ("derive -> wave 0 starts accumulating", 1, 27), ("derive -> group 0 seen by wave 0", 1, 28), ("derive -> last group seen by wave 0", 1, 29),
            ("derive -> producer 2 has group 0's slots", 1, 30), ("derive -> producer 3 has its last group's slots", 1, 31),
            ("last group seen -> accumulation done", 29, 5),
            ("ctl: taps stored -> control reads taps", 6, 16), ("ctl: reads taps -> run_dll_pll", 16, 9),
            ("ctl: PLL discriminator", 9, 37), ("ctl: carrier filter + spec hook", 37, 32), ("ctl: spec -> DLL start", 32, 38),
            ("ctl: DLL discriminator", 38, 39), ("ctl: code filter + code freq", 39, 10), ("ctl: update_tracking_vars", 10, 11),
            ("ctl: consume + seed", 11, 33), ("ctl: taps stored -> seed published", 6, 33), ("ctl: spec published -> spec seen", 32, SLOTS + 0),
            ("cycle: spec seen -> replay end", 0, 34), ("cycle: replay end -> taps stored", 34, 6),
            ("cycle: taps stored -> spec published", 6, 32), ("cycle: spec published -> spec seen (next)", 32, SLOTS + 0),
            ("tail: replay end -> producer 1 has its last slots", 34, 31), ("tail: replay end -> group 6 ready", 34, 54),
            ("tail: replay end -> group 7 ready", 34, 55), ("tail: replay end -> group 6 seen", 34, 62), ("tail: replay end -> group 7 seen", 34, 63),
            ("tail: group 7 seen -> accumulation done", 63, 5), ("tail: replay end -> last group seen", 34, 29),
            ("tail: last group seen -> accumulation done", 29, 5), ("tail: accumulation done -> taps stored", 5, 6)]
    for nm, a, b in rows:
        ok = (v[:, :, a] > 0) & (v[:, :, b] > 0)
        if not ok.any():
            continue
        d = us(v[:, :, b] - v[:, :, a])[ok]
        print(f"  {nm:40s} median {np.median(d):7.2f} us  p90 {np.percentile(d, 90):7.2f}  (n={ok.sum()})")
    ok = (v[:, :, 28] > 0) & (v[:, :, 13] > 0)
    if ok.any():
        print(f"  {'replay only (after barrier B + job)':40s} median {np.median((v[:, :, 13] - v[:, :, 28])[ok]):8.0f} shader cycles")
    for nm, a, b, wa, wb in [("replay", 12, 13, 1, 2), ("loop update", 14, 15, 6, 7)]:
        ok = (v[:, :, a] > 0) & (v[:, :, b] > 0) & (v[:, :, wa] > 0) & (v[:, :, wb] > 0)
        if not ok.any():
            continue
        cyc = (v[:, :, b] - v[:, :, a])[ok].astype(np.float64)
        wall = us(v[:, :, wb] - v[:, :, wa])[ok]
        print(f"  {nm:40s} median {np.median(cyc):8.0f} shader cycles, clock {np.median(cyc / wall) / 1e3:.2f} GHz")
    for g in range(8):
        for nm, sl in (("ready (producer)", 48 + g), ("seen (accumulator)", 56 + g), ("added (accumulator)", 64 + g)):
            ok = (v[:, :, 1] > 0) & (v[:, :, sl] > 0)
            if ok.any():
                d = us(v[:, :, sl] - v[:, :, 1])[ok]
                print(f"  derive -> group {g} {nm:22s} median {np.median(d):7.2f} us  p90 {np.percentile(d, 90):7.2f}  (n={ok.sum()})")
    for nm, k in (("producer 0: ring waits", 41), ("producer 0: slot waits", 42), ("producer 0: whole production", 43),
                  ("producer 0: phase A (codes, sample loads issued)", 79), ("producer 0: phase B (products, stores, flag)", 80),
                  ("accumulator 0: flag waits", 44), ("accumulator 0: whole accumulation", 45), ("accumulator 1: flag waits", 46),
                  ("accumulator 1: whole accumulation", 47)):
        d = v[:, :, k]
        d = d[d > 0]
        if len(d):
            print(f"  {nm:40s} median {np.median(d):8.0f} shader cycles ({np.median(d) / 2.4e3:6.2f} us at 2.4 GHz)")
    vv = v[:, :, 78]
    if np.any(vv > 0):
        print(f"  speculative replay: {int(np.sum(vv == 1))} confirmed, {int(np.sum(vv == 2))} refuted of {int(np.sum(vv > 0))} epochs")
    roles = {0: "control", 1: "replay", 2: "producer"}
    for ch in range(min(n_ch, 4)):
        ids = [int(t[ch, 0, 72 + w]) for w in range(6)]
        print(f"  channel {ch} waves: " + ", ".join(f"w{w} {roles.get(h >> 32, h >> 32)} simd {(h >> 4) & 3}" for w, h in enumerate(ids)))
    for ch in range(min(n_ch, 4)):
        ids = [int(t[ch, 0, 20 + w]) for w in range(4)]
        print(f"  channel {ch} HW_ID per wave: " + ", ".join(f"w{w} simd {(h >> 4) & 3} slot {h & 15} cu {(h >> 8) & 15} se {(h >> 13) & 7}" for w, h in enumerate(ids)))
    trk.close()
    ctx.close()


if __name__ == "__main__":
    main()

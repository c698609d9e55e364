"""One point of bench.py's channel sweep as a stand-alone program (for rocprofv3 --pmc passes):
N channels of GPS L1 C/A at 4 Msps on the bench's file (seed 0x6E550002), the AVX rotator, pre-rolled
to state 4, then one timed launch of R epochs.

    python scripts/trk_sweep_point.py [channels=65536] [epochs=20] [records]

With `records` the timed launch writes every channel-epoch record (as bench.py's sweep does) and they
are collected to the host after the timing.  The line names the kernel the timed launch ran."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    import torch
    from gnss_sim_receiver_amd import abi, engine, signals
    fs, vl = 4000000, 4000
    sats = signals.random_sky(32, seed=0x6E550002)
    for s in sats:
        s.bits = "1000101100110"
    first = int(11.0 * fs)
    pre = 450
    x = signals.generate_if_device(fs, (pre + rounds + 8) * vl, sats, seed=0x6E550002, start=first - 2 * vl, device="cuda:0")
    torch.cuda.synchronize()
    ctx = engine.Context(0)
    conf = abi.TrkConf.defaults(abi.SYS_GPS_L1CA, fs, vl, rotator=abi.ROTATOR_AVX)
    trk = engine.DllPllVemlTracking(ctx, conf, n)
    for i, s in enumerate(sats):
        ctx.set_code(300 + i, s.code)
    for ch in range(n):
        s = sats[ch % 32]
        trk.start(ch, 300 + ch % 32, signals.acq_delay_samples(s, fs, 0, first), s.doppler_hz, 0, first, prn=s.prn)
    base = x.data_ptr()
    trk.run_ptr(base + 2 * vl * 8, abi.FMT_CF32, first, (pre + 2) * vl, pre + 4)
    lo = first + pre * vl
    ctx.sync()
    t0 = time.perf_counter()
    recs = "records" in sys.argv[3:]
    if recs:
        trk.launch_ptr(base + (lo - first + 2 * vl) * 8, abi.FMT_CF32, lo, (rounds + 2) * vl, rounds, records=True)
        ctx.sync()
        dt = time.perf_counter() - t0
        rec, done = trk.collect()
        n_rec = int(np.count_nonzero(rec[:done]["flags"] & 8))
    else:
        done = trk.run_ptr(base + (lo - first + 2 * vl) * 8, abi.FMT_CF32, lo, (rounds + 2) * vl, rounds)
        dt = time.perf_counter() - t0
        n_rec = 0
    eng = abi.TRK_ENGINE_NAMES.get(trk.last_engine())
    st = np.bincount(trk.states(), minlength=5).tolist()
    trk.close()
    ctx.close()
    print(f"channels {n}: {done} epochs in {dt * 1e3:.2f} ms -> {n * done / dt / 1e6:.2f} M channel-epochs/s, realtime x{done * 1e-3 / dt:.2f}, "
          f"states {st}, kernel {eng}, records {n_rec}", flush=True)


if __name__ == "__main__":
    main()

"""Closed-loop tracking run for profiling: 12 GPS channels, 200 epoch rounds (rocprofv3 target)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from gnss_sim_receiver_amd import abi, engine, signals  # noqa: E402


def main():
    n_ch = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    fs, vl = 4e6, 4000
    sats = signals.random_sky(32, seed=1)
    x = signals.generate_if(fs, vl * (rounds + 8), sats, seed=1)
    ctx = engine.Context(0)
    trk = engine.DllPllVemlTracking(ctx, abi.TrkConf.defaults(abi.SYS_GPS_L1CA, fs, vl, rotator=abi.ROTATOR_GENERIC), n_ch)
    for i, s in enumerate(sats):
        ctx.set_code(i, s.code)
    for ch in range(n_ch):
        s = sats[ch % 32]
        trk.start(ch, ch % 32, (s.code_delay_chips / s.code_freq()) * fs, s.doppler_hz, 0, 0)
    dev = ctx.upload(x)
    t0 = time.perf_counter()
    _, done = trk.run(dev, 0, rounds, n_buffer_samples=len(x), records=False)
    dt = time.perf_counter() - t0
    print(f"{n_ch} ch, {done} rounds, {dt / done * 1e6:.2f} us/round")
    trk.close()
    ctx.close()


if __name__ == "__main__":
    main()

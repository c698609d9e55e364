"""Closed-loop timing probe on the GPU: per-epoch time of gnsship_trk for a few engines/rotators."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gnss_sim_receiver_amd import abi, engine, signals  # noqa: E402


def run(ctx, system, fs, vl, n_ch, rounds, rotator, env=None, sats=None, block=None):
    if env:
        os.environ.update(env)
    try:
        conf = abi.TrkConf.defaults({"GPS": abi.SYS_GPS_L1CA, "GAL": abi.SYS_GAL_E1}[system], fs, vl, rotator=rotator)
        trk = engine.DllPllVemlTracking(ctx, conf, n_ch)
    finally:
        for k in (env or {}):
            os.environ.pop(k, None)
    for i, s in enumerate(sats):
        ctx.set_code(300 + 2 * i, s.code)
        if s.code_data is not None:
            ctx.set_code(301 + 2 * i, s.code_data)
    for ch in range(n_ch):
        i = ch % len(sats)
        s = sats[i]
        trk.start(ch, 300 + 2 * i, (s.code_delay_chips / s.code_freq()) * fs, s.doppler_hz, 0, 0, data_code_id=301 + 2 * i)
    dev = ctx.upload(block)
    trk.run(dev, 0, 2, n_buffer_samples=len(block), records=False)
    t0 = time.perf_counter()
    _, done = trk.run(dev, 0, rounds, n_buffer_samples=len(block), records=False)
    dt = time.perf_counter() - t0
    tracking = sum(1 for ch in range(n_ch) if trk.channel_state(ch)[0] in (2, 3, 4))
    trk.close()
    dev.free()
    print(f"{system} fs={fs/1e6:g}M N={vl} ch={n_ch} rot={rotator} env={env}: {done} rounds {dt*1e3:.2f} ms "
          f"-> {dt/done*1e6:.2f} us/epoch, realtime x{done*vl/fs/dt:.1f}, tracking {tracking}/{n_ch}", flush=True)


def main():
    ctx = engine.Context(0)
    fs = 4e6
    sats = signals.random_sky(32, seed=0x6E550002)
    block = signals.generate_if(fs, int(fs * 0.3) + 8000, sats, seed=1)
    for rot in (0, 1):
        run(ctx, "GPS", fs, 4000, 12, 250, rot, sats=sats, block=block)
    run(ctx, "GPS", fs, 4000, 12, 250, 0, env={"GNSSHIP_TRK_ROUNDS": "1"}, sats=sats, block=block)
    for n in (256, 1024, 4096, 16384):
        run(ctx, "GPS", fs, 4000, n, 100, 1, sats=sats, block=block)
    run(ctx, "GPS", fs, 4000, 4096, 100, 1, env={"GNSSHIP_TRK_THRU": "0"}, sats=sats, block=block)
    fs = 25e6
    gs = signals.random_sky(8, seed=3, system="GAL")
    b25 = signals.generate_if(fs, int(fs * 0.1) + 300000, gs, seed=2)
    for rot in (0, 1):
        run(ctx, "GAL", fs, 100000, 8, 20, rot, sats=gs, block=b25)
    ctx.close()


if __name__ == "__main__":
    main()

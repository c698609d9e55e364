"""trk_lane bring-up: one epoch of 4 GPS channels traced through trk_lane (GNSSHIP_TRK_LANE=1) and
trk_fast (=0) on the same state, with the oracle's u_avx taps on the traced arguments."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402


def main():
    from gnss_sim_receiver_amd import abi, engine, signals
    from oracle import oracle as O, trk as T
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
    from test_gpu_c5_closed_loop import check_trace
    fs, vl, n_ch, epochs = 4e6, 4000, 4, 2
    sats = signals.random_sky(32, seed=0x6E550012)
    k = T.conf("GPS", fs, vl, rotator_avx=1)
    first = int(11 * fs)
    x = signals.generate_if(fs, vl * (epochs + 4), sats, seed=0x6E550013, start=first)
    xf = x.astype(np.complex64)
    ctx = engine.Context(0)
    for i, s in enumerate(sats):
        ctx.set_code(400 + i, s.code)
    out = {}
    for mode in ("1", "0"):
        os.environ["GNSSHIP_TRK_LANE"] = mode
        from test_gpu_trk import dev_conf
        trk = engine.DllPllVemlTracking(ctx, dev_conf(k, "GPS"), n_ch)
        for ch in range(n_ch):
            s = sats[ch]
            trk.start(ch, 400 + ch, signals.acq_delay_samples(s, fs, 0, first), s.doppler_hz, 0, first)
        trk.set_trace(True)
        rec, rounds = trk.run(x, first, epochs)
        print("mode", mode, "engine", abi.TRK_ENGINE_NAMES[trk.last_engine()], "rounds", rounds)
        out[mode] = trk.trace(epochs)
        trk.close()
    for ch in range(n_ch):
        tr = out["1"][:, ch]
        tf = out["0"][:, ch]
        jobs = check_trace(tr[tr["n_samples"] > 0], xf, first, [sats[ch].code])
        jobs["code_id"] = 0
        jobs["flags"] = abi.JOB_ROTATOR_AVX
        ref = O.corr_batch(xf, jobs, [sats[ch].code], n_threads=8).astype(np.complex64)
        for e in range(1):
            print("ch", ch, "args lane", tr[e]["sample_counter"], tr[e]["rem_carrier_phase_rad"], tr[e]["phase_step_rad"], tr[e]["rem_code_phase_samples"],
                  tr[e]["code_phase_step_samples"], tr[e]["shifts"][:3])
            print("ch", ch, "args fast", tf[e]["sample_counter"], tf[e]["rem_carrier_phase_rad"], tf[e]["phase_step_rad"], tf[e]["rem_code_phase_samples"],
                  tf[e]["code_phase_step_samples"], tf[e]["shifts"][:3])
            print("  lane", tr[e]["taps"][:6])
            print("  fast", tf[e]["taps"][:6])
            print("  ref ", ref[e, :3].view(np.float32))
    ctx.close()


if __name__ == "__main__":
    main()

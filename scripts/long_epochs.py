"""bench.py's long-epoch closed-loop lines on their own (A/B of trk_fast builds via GNSSHIP_LIB_PATH):
GPS L1 C/A at 25 Msps (N = 25000, 12 channels), the Galileo E1 C4 share (N = 100000, 8 channels),
and with `c5` the C5 per-GPU share (12 GPS + 12 E1 + 8 B1I at 50 Msps ibyte).

    python scripts/long_epochs.py [c5]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch
    from gnss_sim_receiver_amd import abi, engine
    ctx = engine.Context(0)
    rot = abi.ROTATOR_AVX
    out = {"gps_25msps": bench.closed_loop_aux(ctx, torch, 0, "GPS", 25e6, 25000, bench.N_CH, 0.3, rot, bench.SEED + 11),
           "e1_25msps_c4_share": bench.closed_loop_aux(ctx, torch, 0, "GAL", 25e6, 100000, 8, 0.4, rot, bench.SEED + 12)}
    if "c5" in sys.argv[1:]:
        out["c5_share"] = bench.closed_loop_c5_share(torch, 0, rot)
    ctx.close()
    for k, v in out.items():
        print(k, json.dumps({f: v.get(f) for f in ("realtime_factor", "us_per_epoch_round", "channels_in_state_4") if f in v}))


if __name__ == "__main__":
    main()

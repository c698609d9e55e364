"""Debug aid: one GPS channel through the fast AVX persistent kernel vs trk_persist (GNSSHIP_TRK_FAST=0)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np  # noqa: E402

from gnss_sim_receiver_amd import abi, engine  # noqa: E402
import trk_scenarios as S  # noqa: E402
from test_gpu_trk import dev_conf  # noqa: E402

ctx = engine.Context(0)
sat, k, x, stamp, first, delay, dop = S.sync("GPS", 4e6, 50, rotator_avx=1)
c = dev_conf(k, "GPS")
for fast in ("1", "0"):
    os.environ["GNSSHIP_TRK_FAST"] = fast
    trk = engine.DllPllVemlTracking(ctx, c, 1)
    ctx.set_code(40, sat.code)
    trk.start(0, 40, delay, dop, stamp, first)
    trk.set_trace(True)
    rec, rounds = trk.run(x, first, 20)
    print("fast", fast, "rounds", rounds, "state", trk.channel_state(0))
    r = rec[:, 0]
    print(r[["sample_counter", "flags", "state", "carrier_doppler_hz", "prompt_i", "prompt_q"]][:6])
    tr = trk.trace(20)[:, 0]
    print(tr[["sample_counter", "n_samples", "rem_carrier_phase_rad", "phase_step_rad", "rem_code_phase_samples"]][:3])
    print(tr["taps"][:3])
    trk.close()

"""The headline workload pinned to the oracle (BASELINE configs[1] as bench.py runs it): 12 GPS L1 C/A
channels at 4 Msps gr_complex, the AVX rotator variant (volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn
u_avx, :155-316 — what volk dispatches on an x86 host with AVX), the bench's sky (32 satellites, seed
0x6E550002, the TLM preamble every 260 ms), channels started from an acquisition stamped 11 s before
the first sample (the 10 s pull-in over), run for 1100 epochs so that every channel spends ≥ 500
epochs in state 4 (bit-synchronised, dll_pll_veml_tracking.cc:1971-2028).

Two checks on the same run (the persistent fast kernel, trk_fast.hip), both bit-exact:
  * the correlator: every traced channel-epoch (gnsship_trk_set_trace: the arguments the device
    correlated with and its tap sums) re-run on oracle.corr_batch (the u_avx restatement) with the
    same arguments — every tap equal;
  * the loop: every channel's epoch records equal the oracle loop's (oracle/trk_oracle.c, the same
    AVX correlator, glibc trig, discriminators and CN0 log10f) — test_gpu_trk.compare_exact.
"""
import concurrent.futures as cf

import numpy as np
import pytest

from gnss_sim_receiver_amd import abi, engine, signals
from oracle import trk as T

from test_gpu_trk import compare_exact, dev_conf
from test_gpu_c5_closed_loop import trace_exact

pytestmark = pytest.mark.gpu

FS, VL, N_CH = 4e6, 4000, 12
SEED = 0x6E550002
EPOCHS = 1100
def test_headline_c2_avx_500_state4_epochs_match_oracle(ctx):
    sats = signals.random_sky(32, seed=SEED)
    for s in sats:
        s.bits = "1000101100110"
    first = int(11.0 * FS)
    lo = first - 2 * VL
    x = signals.generate_if(FS, (EPOCHS + 6) * VL, sats, seed=SEED, start=lo)
    k = T.conf("GPS", FS, VL, rotator_avx=1)
    c = dev_conf(k, "GPS")
    c.rotator = abi.ROTATOR_AVX
    trk = engine.DllPllVemlTracking(ctx, c, N_CH)
    delays = []
    for ch in range(N_CH):
        s = sats[ch]
        ctx.set_code(300 + ch, s.code)
        delays.append(signals.acq_delay_samples(s, FS, 0, first))
        trk.start(ch, 300 + ch, delays[-1], s.doppler_hz, 0, first, prn=s.prn)
    trk.set_trace(True)
    rec, rounds = trk.run(x, lo, EPOCHS)
    tr = trk.trace(EPOCHS)
    trk.close()

    def oracle_loop(ch):
        s = sats[ch]
        return T.track(k, x, s.code, delays[ch], s.doppler_hz, 0, first, EPOCHS, buffer_first=lo, prn=s.prn)

    with cf.ThreadPoolExecutor(8) as ex:
        refs = list(ex.map(oracle_loop, range(N_CH)))
    for ch in range(N_CH):
        ref = refs[ch]
        assert np.count_nonzero(ref["state"] == 4) >= 500, (ch, np.bincount(ref["state"]))
        compare_exact(rec[:, ch], ref, f"C2 channel {ch}")
    # the correlator on the device's own arguments, every channel-epoch, tap for tap
    n = 0
    for ch in range(N_CH):
        n += trace_exact(tr[:, ch], x, lo, sats[ch].code, None, f"C2 channel {ch}")
    assert n >= N_CH * 1000

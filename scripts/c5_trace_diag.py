"""Per-epoch correlator trace error of one C5 closed-loop channel (tests/test_gpu_c5_closed_loop.py),
device kernel vs the oracle correlator on the device's own arguments.

    python scripts/c5_trace_diag.py GAL 1      (GNSSHIP_TRK_FAST=0 selects trk_persist.hip)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

from gnss_sim_receiver_amd import abi, engine, signals  # noqa: E402
from oracle import oracle as O  # noqa: E402
import trk_scenarios as S  # noqa: E402
from test_gpu_trk import dev_conf  # noqa: E402
import test_gpu_c5_closed_loop as C  # noqa: E402


def main():
    system = sys.argv[1] if len(sys.argv) > 1 else "GAL"
    avx = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    epochs = 60 if system == "GAL" else 100
    sat, k, x, stamp, first, delay, dop = S.sync(system, C.FS, epochs, f_if_hz=C.IF_OF[system], rotator_avx=avx, accum_f64=1, cn0=48.0)
    raw = signals.to_ibyte(x)
    xf = raw.astype(np.float32).view(np.complex64)
    ctx = engine.Context(0)
    trk = engine.DllPllVemlTracking(ctx, dev_conf(k, system), 1)
    ctx.set_code(90, sat.code)
    if sat.code_data is not None:
        ctx.set_code(91, sat.code_data)
    trk.start(0, 90, delay, dop, stamp, first, data_code_id=91, prn=sat.prn)
    trk.set_trace(True)
    trk.run(xf if os.environ.get("DIAG_CF32") == "1" else raw, first, epochs)
    tr = trk.trace(epochs)[:, 0]
    trk.close()
    ctx.close()
    tr = tr[tr["n_samples"] > 0]
    jobs = C.check_trace(tr, xf, first, [sat.code])
    jobs["code_id"] = 0
    jobs["flags"] = (abi.JOB_ROTATOR_AVX if avx else 0) | 4
    long_n = int(jobs["n_samples"][0]) >= 100000
    # the same arguments through the batch correlator (corr_kernel.hip), data prompt excluded
    bj = jobs.copy()
    bj["flags"] = abi.JOB_ROTATOR_AVX if avx else 0
    ctx2 = engine.Context(0)
    bout = engine.correlate_host(ctx2, xf, bj, [sat.code])
    bout8 = engine.correlate_host(ctx2, raw, bj, [sat.code])
    print("batch cf32 vs batch ci8 max abs diff", float(np.max(np.abs(bout - bout8))))
    ctx2.close()
    bref = O.corr_batch(xf, jobs, [sat.code], n_threads=8, accum_f64=True)
    for j in range(len(jobs)):
        t = int(jobs["n_taps"][j])
        o, n = int(jobs["sample_offset"][j]), int(jobs["n_samples"][j])
        scale = max(float(np.max(np.abs(bref[j, :t]))), float(np.linalg.norm(xf[o:o + n].astype(np.complex128))))
        got = tr["taps"][j, 0:2 * t:2] + 1j * tr["taps"][j, 1:2 * t:2]
        if j < 3 or j in (5, 49):
            print(f"  epoch {j}: batch-vs-oracle {np.max(np.abs(bout[j, :t] - bref[j, :t])) / scale:.3e}  trace-vs-batch "
                  f"{np.max(np.abs(got - bout[j, :t])) / scale:.3e}  trace-vs-oracle {np.max(np.abs(got - bref[j, :t])) / scale:.3e}")
    for acc in ([False, True] if long_n else [False]):
        ref = O.corr_batch(xf, jobs, [sat.code], n_threads=8, accum_f64=acc)
        errs = []
        for j in range(len(jobs)):
            t = int(jobs["n_taps"][j])
            o, n = int(jobs["sample_offset"][j]), int(jobs["n_samples"][j])
            scale = max(float(np.max(np.abs(ref[j, :t]))), float(np.linalg.norm(xf[o:o + n].astype(np.complex128))))
            got = tr["taps"][j, 0:2 * t:2] + 1j * tr["taps"][j, 1:2 * t:2]
            errs.append(np.abs(got - ref[j, :t]) / scale)
        errs = np.array(errs)
        print(f"{system} avx={avx} kernel={'v1' if os.environ.get('GNSSHIP_TRK_FAST') == '0' else 'fast'} oracle accum_f64={acc}: "
              f"max {errs.max():.3e} median {np.median(errs):.3e}; worst epochs {np.argsort(errs.max(axis=1))[-5:]} per-tap max {errs.max(axis=0)}")


if __name__ == "__main__":
    main()

"""Device-resident tracking loop (gnsship_trk, HIP) vs the oracle loop (oracle/trk_oracle.c).

Same IF, same start_tracking arguments, every epoch compared.  Both rotator variants' persistent
engines (generic: trk_persist.hip's serial pipeline; AVX: trk_fast.hip / trk_lane.hip) sum in the
reference's own order with glibc's libm restated on the device, so their records are compared for
equality (compare_exact).  The round-based high-dynamics loop (trk_kernel.hip + corr_hd_kernel.hip,
tree sums) is held to `compare`'s tolerances: the loop is a contracting feedback system, so the
device/oracle differences stay at the size of their per-epoch inputs' differences:
  exact      sample_counter (every consume_each), state, flags, prn_length_samples
  ≤ 2e-3 Hz  carrier Doppler; ≤ 2e-3 chips/s code frequency; ≤ 1e-5 chips remnant code phase
  ≤ 5e-3 dB  CN0; prompt ≤ 1e-4·|P| (+1e-3); ≤ 1e-2 rad accumulated carrier phase.
"""
import numpy as np
import pytest

from gnss_sim_receiver_amd import abi, engine, signals
from oracle import trk as T

import trk_scenarios as S

pytestmark = pytest.mark.gpu
SYS = {"GPS": abi.SYS_GPS_L1CA, "GAL": abi.SYS_GAL_E1, "BDS": abi.SYS_BDS_B1I}
SHARED = ["fs_in", "carrier_lock_th", "pll_bw_hz", "dll_bw_hz", "fll_bw_hz", "early_late_space_chips", "very_early_late_space_chips",
          "slope", "spc", "y_intercept", "cn0_smoother_alpha", "carrier_lock_test_smoother_alpha", "pull_in_time_s",
          "bit_synchronization_time_limit_s", "vector_length", "pll_filter_order", "dll_filter_order", "cn0_samples",
          "cn0_smoother_samples", "carrier_lock_test_smoother_samples", "cn0_min", "max_code_lock_fail", "max_carrier_lock_fail",
          "carrier_aiding", "track_pilot", "extend_correlation_symbols", "pll_bw_narrow_hz", "dll_bw_narrow_hz",
          "early_late_space_narrow_chips", "very_early_late_space_narrow_chips", "enable_fll_pull_in", "enable_fll_steady_state",
          "high_dyn", "smoother_length"]


def dev_conf(k, system):
    c = abi.TrkConf.defaults(SYS[system], k.fs_in, k.vector_length)
    for f in SHARED:
        setattr(c, f, getattr(k, f))
    c.rotator = abi.ROTATOR_AVX if k.rotator_avx else abi.ROTATOR_GENERIC  # the oracle's variant, not the host's
    c.if_hz = k.if_hz
    if system == "GAL":
        c.track_pilot = k.track_pilot
    return c


def compare(dev, ref, label="", cn0_tol=5e-3):
    d = dev[(dev["flags"] & 8) == 8]
    assert len(d) == len(ref), (label, len(d), len(ref))
    for f in ("sample_counter", "state", "prn_length_samples"):
        assert np.array_equal(d[f], ref[f]), (label, f, np.nonzero(d[f] != ref[f])[0][:5])
    assert np.array_equal(d["flags"] & 7, ref["flags"] & 7), label
    np.testing.assert_allclose(d["carrier_doppler_hz"], ref["carrier_doppler_hz"], rtol=0, atol=2e-3, err_msg=label)
    np.testing.assert_allclose(d["code_freq_chips"], ref["code_freq_chips"], rtol=0, atol=2e-3, err_msg=label)
    np.testing.assert_allclose(d["rem_code_phase_chips"], ref["rem_code_phase_chips"], rtol=0, atol=1e-5, err_msg=label)
    np.testing.assert_allclose(d["cn0_db_hz"], ref["cn0_db_hz"], rtol=0, atol=cn0_tol, err_msg=label)
    np.testing.assert_allclose(d["carrier_phase_rads"], ref["carrier_phase_rads"], rtol=0, atol=1e-2, err_msg=label)
    pd = d["prompt_i"] + 1j * d["prompt_q"]
    pr = ref["prompt_i"] + 1j * ref["prompt_q"]
    assert np.all(np.abs(pd - pr) <= 1e-4 * np.abs(pr) + 1e-3), label


# The AVX-rotator engine (trk_fast.hip) is bit-exact to the oracle loop: the correlator sums in u_avx's
# order, the phasors are glibc's cosf / sinf (glibc_sincosf.h), the discriminators glibc's atanf /
# atan2f / hypotf (glibc_atanf.h, nco_math.h) and the CN0 estimate glibc's log10f (glibc_logf.h), so
# every record field is compared for equality.
EXACT_FIELDS = [f for f in abi.TRK_EPOCH_DTYPE.names if f not in ("pad", "flags")]


def compare_exact(dev, ref, label=""):
    d = dev[(dev["flags"] & 8) == 8]
    assert len(d) == len(ref), (label, len(d), len(ref))
    for f in EXACT_FIELDS:
        same = (d[f] == ref[f]) | (np.isnan(d[f]) & np.isnan(ref[f])) if d[f].dtype.kind == "f" else d[f] == ref[f]
        if not np.all(same):
            i = int(np.nonzero(~same)[0][0])
            raise AssertionError(f"{label}: {f} differs first at epoch {i} of {len(d)}: device {d[f][i]!r} oracle {ref[f][i]!r} "
                                 f"({int(np.count_nonzero(~same))} epochs differ)")
    assert np.array_equal(d["flags"] & 7, ref["flags"] & 7), label


def test_gps_pull_in_eight_channels(ctx):
    fs, epochs = 4e6, 300
    rng = np.random.default_rng(17)
    sats = [signals.Satellite(prn=p, doppler_hz=float(rng.uniform(-4000, 4000)), code_delay_chips=float(rng.uniform(0, 1023)),
                              cn0_dbhz=47.0, carrier_phase_rad=float(rng.uniform(0, 6.28))) for p in range(1, 9)]
    k = T.conf("GPS", fs, 4000)
    x = signals.generate_if(fs, 4000 * (epochs + 3), sats, seed=3)
    trk = engine.DllPllVemlTracking(ctx, dev_conf(k, "GPS"), len(sats))
    starts = []
    for ch, s in enumerate(sats):
        delay = (s.code_delay_chips / s.code_freq()) * fs + float(rng.uniform(-0.4, 0.4))
        dop = s.doppler_hz + float(rng.uniform(-30, 30))
        ctx.set_code(ch, s.code)
        trk.start(ch, ch, delay, dop, 0, 0)
        starts.append((delay, dop))
    rec, rounds = trk.run(x, 0, epochs)
    assert rounds == epochs
    for ch, s in enumerate(sats):
        ref = T.track(k, x, s.code, starts[ch][0], starts[ch][1], 0, 0, epochs)
        compare_exact(rec[:, ch], ref, f"ch{ch}")
    trk.close()


@pytest.mark.parametrize("system,fs,epochs", [("GPS", 4e6, 700), ("GAL", 25e6 / 4, 90), ("BDS", 4.092e6, 300)])
def test_sync_to_state_4_matches_oracle(ctx, system, fs, epochs):
    sat, k, x, stamp, first, delay, dop = S.sync(system, fs, epochs)
    trk = engine.DllPllVemlTracking(ctx, dev_conf(k, system), 2)
    ctx.set_code(20, sat.code)
    if sat.code_data is not None:
        ctx.set_code(21, sat.code_data)
    trk.start(1, 20, delay, dop, stamp, first, data_code_id=21)  # channel 0 left idle
    rec, rounds = trk.run(x, first, epochs)
    ref = T.track(k, x, sat.code, delay, dop, stamp, first, epochs, data_code=sat.code_data, buffer_first=first)
    assert ref["state"][-1] == 4
    compare_exact(rec[:, 1], ref, system)
    assert not np.any(rec[:, 0]["flags"])
    trk.close()


@pytest.mark.parametrize("system,fs,epochs,ext", [("GPS", 4e6, 600, 10), ("GPS", 4e6, 500, 20), ("GAL", 25e6 / 4, 110, 4),
                                                  ("BDS", 4.092e6, 400, 5)])
def test_extended_integration_state_3_matches_oracle(ctx, system, fs, epochs, ext):
    """extend_correlation_symbols > 1: after synchronisation the loop runs extend − 1 coherent
    integration epochs (state 3) per narrow-loop update (state 4), narrow taps and bandwidths
    (dll_pll_veml_tracking.cc:1890-1970)."""
    sat, k, x, stamp, first, delay, dop = S.sync(system, fs, epochs, extend_correlation_symbols=ext)
    trk = engine.DllPllVemlTracking(ctx, dev_conf(k, system), 1)
    ctx.set_code(30, sat.code)
    if sat.code_data is not None:
        ctx.set_code(31, sat.code_data)
    trk.start(0, 30, delay, dop, stamp, first, data_code_id=31)
    rec, rounds = trk.run(x, first, epochs)
    ref = T.track(k, x, sat.code, delay, dop, stamp, first, epochs, data_code=sat.code_data, buffer_first=first)
    st = ref["state"]
    assert np.sum(st == 3) >= 3 * (ext - 1) and np.sum(st == 4) >= 3
    compare_exact(rec[:, 0], ref, f"{system} x{ext}")
    trk.close()


@pytest.mark.parametrize("pull_in,steady", [(1, 0), (1, 1), (0, 1)])
def test_fll_assisted_loop_matches_oracle(ctx, pull_in, steady):
    """enable_fll_pull_in / enable_fll_steady_state (run_dll_pll :1080-1097): fll_diff_atan of
    consecutive prompts drives the carrier filter's FLL input (alone during the pull-in)."""
    sat, k, x, stamp, first, delay, dop = S.pull_in("GPS", 4e6, 46.0, -2600.0, 321.0, 60.0, 0.3, 400, pull_in_time_s=0,
                                                     enable_fll_pull_in=pull_in, enable_fll_steady_state=steady)
    if pull_in:
        k.pull_in_time_s = 1 if not steady else 0
    ctx.set_code(40, sat.code)
    trk = engine.DllPllVemlTracking(ctx, dev_conf(k, "GPS"), 1)
    trk.start(0, 40, delay, dop, stamp, first)
    rec, rounds = trk.run(x, 0, 400)
    ref = T.track(k, x, sat.code, delay, dop, stamp, first, 400)
    assert len(ref) > 100
    compare_exact(rec[:, 0], ref, f"fll {pull_in}{steady}")
    trk.close()


@pytest.mark.parametrize("system,fs,epochs,rate_hz_s,smoother", [("GPS", 4e6, 500, 40.0, 10), ("GPS", 4e6, 300, -25.0, 1),
                                                                  ("GAL", 25e6 / 4, 100, 30.0, 10), ("BDS", 4.092e6, 300, 20.0, 7)])
def test_high_dyn_loop_matches_oracle(ctx, system, fs, epochs, rate_hz_s, smoother):
    """high_dyn (dll_pll_veml_tracking.cc:1205-1255 with the high-dynamics correlator pair
    :530,536): the carrier / code NCO rates are the smoothed differences of the last
    2·smoother_length phase steps and drive the high-dynamics resampler and rotator (taps 1.. are
    circular shifts of tap 0).  A Doppler ramp of tens of Hz/s; every epoch compared.  (Not E1 with
    smoother_length 4: there the rate feedback amplifies a 1e-4 Hz start perturbation to 0.08 Hz
    in the oracle itself, so rounding-level device/oracle differences grow the same way.)"""
    sat, k, x, stamp, first, delay, dop = S.sync(system, fs, epochs, high_dyn=1, smoother_length=smoother, rate_hz_s=rate_hz_s)
    trk = engine.DllPllVemlTracking(ctx, dev_conf(k, system), 1)
    ctx.set_code(50, sat.code)
    if sat.code_data is not None:
        ctx.set_code(51, sat.code_data)
    trk.start(0, 50, delay, dop, stamp, first, data_code_id=51)
    rec, rounds = trk.run(x, first, epochs)
    ref = T.track(k, x, sat.code, delay, dop, stamp, first, epochs, data_code=sat.code_data, buffer_first=first)
    assert len(ref) == epochs and ref["state"][-1] in (2, 4)
    compare(rec[:, 0], ref, f"high_dyn {system}")
    trk.close()


@pytest.mark.parametrize("ext", [1, 5])
def test_bds_geo_matches_oracle(ctx, ext):
    """BeiDou B1I GEO satellite (start args PRN 3; start_tracking :765-781): D2 preamble bit sync at
    2 symbols per bit, no NH code, extend capped at 2 — next to a MEO channel (PRN 9) of the same
    engine, which keeps the NH-code profile and the configured extend."""
    fs, epochs = 4.092e6, 300
    sat, k, x, stamp, first, delay, dop = S.sync("BDS", fs, epochs, prn=3, extend_correlation_symbols=ext)
    meo, km, xm, _, _, delay_m, dop_m = S.sync("BDS", fs, epochs, prn=9, dop=-830.0, delay_chips=1500.6,
                                                  extend_correlation_symbols=ext, seed=6)
    c = dev_conf(km, "BDS")  # the engine's configuration: the MEO one (GEO settings come from the PRN)
    trk = engine.DllPllVemlTracking(ctx, c, 2)
    ctx.set_code(60, sat.code)
    ctx.set_code(61, meo.code)
    both = (x + xm).astype(np.complex64)
    trk.start(0, 60, delay, dop, stamp, first, prn=3)
    trk.start(1, 61, delay_m, dop_m, stamp, first, prn=9)
    rec, rounds = trk.run(both, first, epochs)
    ref = T.track(k, both, sat.code, delay, dop, stamp, first, epochs, buffer_first=first)
    ref_m = T.track(km, both, meo.code, delay_m, dop_m, stamp, first, epochs, buffer_first=first)
    assert ref["state"][-1] in (3, 4) and ref_m["state"][-1] in (3, 4)
    compare_exact(rec[:, 0], ref, f"geo x{ext}")
    compare_exact(rec[:, 1], ref_m, f"meo x{ext}")
    trk.close()


@pytest.mark.parametrize("system,fs,epochs,kw", [("GPS", 4e6, 400, {}), ("GAL", 25e6 / 4, 90, {}),
                                                 ("GPS", 4e6, 300, dict(high_dyn=1, smoother_length=5, rate_hz_s=30.0))])
def test_dump_records_match_oracle(ctx, tmp_path, system, fs, epochs, kw):
    """log_data records (dll_pll_veml_tracking.cc:1376-1466) from the device loop vs the oracle's:
    written on the same epochs, same stamps/PRN, values within the loop tolerances."""
    sat, k, x, stamp, first, delay, dop = S.sync(system, fs, epochs, **kw)
    trk = engine.DllPllVemlTracking(ctx, dev_conf(k, system), 1)
    ctx.set_code(70, sat.code)
    if sat.code_data is not None:
        ctx.set_code(71, sat.code_data)
    trk.start(0, 70, delay, dop, stamp, first, data_code_id=71, prn=sat.prn)
    rec, rounds, dump = trk.run(x, first, epochs, dump=True)
    ref, rdump = T.track(k, x, sat.code, delay, dop, stamp, first, epochs, data_code=sat.code_data, buffer_first=first, dump=True,
                         prn=sat.prn)
    ran = (rec[:, 0]["flags"] & 8) != 0
    d_rec, d_dump = rec[ran, 0], dump[ran, 0]
    assert np.array_equal(d_rec["flags"] & 16, ref["flags"] & 16)
    w = (ref["flags"] & 16) != 0
    a, b = d_dump[w], rdump[w]
    assert len(a) > 20
    for f in ("PRN_start_sample_count", "aux2", "PRN"):
        assert np.array_equal(a[f], b[f]), f
    tol = {"abs_VE": 1e-4, "abs_E": 1e-4, "abs_P": 1e-4, "abs_L": 1e-4, "abs_VL": 1e-4, "prompt_I": 1e-4, "prompt_Q": 1e-4}
    for f, rt in tol.items():
        np.testing.assert_allclose(a[f], b[f], rtol=rt, atol=1e-3, err_msg=f)
    for f, at in [("acc_carrier_phase_rad", 1e-2), ("carrier_doppler_hz", 2e-3),
                  ("code_freq_chips", 2e-3), ("carr_error_hz", 1e-3), ("carr_error_filt_hz", 2e-3), ("code_error_chips", 1e-4),
                  ("code_error_filt_chips", 1e-4), ("CN0_SNV_dB_Hz", 5e-3), ("carrier_lock_test", 1e-4), ("aux1", 1e-4),
                  # rates: differences of smoothed steps over ~smoother_length epochs amplify the
                  # ≤ 2e-3 Hz Doppler agreement to ~0.1-0.5 Hz/s
                  ("carrier_doppler_rate_hz", 0.5), ("code_freq_rate_chips", 0.5)]:
        np.testing.assert_allclose(a[f], b[f], rtol=1e-5, atol=at, err_msg=f)
    if kw.get("high_dyn"):
        assert np.any(a["carrier_doppler_rate_hz"] != 0)
    paths = engine.DllPllVemlTracking.write_dump_files(str(tmp_path / "trk_channel_"), rec, dump)
    data = np.fromfile(paths[0], abi.TRK_DUMP_DTYPE)
    assert np.array_equal(data, a)
    trk.close()


def test_high_dyn_smoother_length_bound(ctx):
    k = abi.TrkConf.defaults(abi.SYS_GPS_L1CA, 4e6, 4000, high_dyn=1, smoother_length=65)
    with pytest.raises(abi.GnssHipError):
        engine.DllPllVemlTracking(ctx, k, 1)


def test_buffers_in_pieces_and_channel_state(ctx):
    sat, k, x, stamp, first, delay, dop = S.pull_in("GPS", 4e6, 45.0, 2100.0, 50.5, -20.0, 0.3, 120)
    ctx.set_code(3, sat.code)
    trk = engine.DllPllVemlTracking(ctx, dev_conf(k, "GPS"), 1)
    trk.start(0, 3, delay, dop, stamp, first)
    a, ra = trk.run(x[:150000], 0, 120)
    st, nx = trk.channel_state(0)
    assert st == 2 and 0 < ra < 120
    b, rb = trk.run(x[nx:], nx, 120)
    got = np.concatenate([a[:ra, 0], b[:, 0]])
    ref = T.track(k, x, sat.code, delay, dop, stamp, first, 120)
    compare_exact(got[(got["flags"] & 8) == 8][:len(ref)], ref, "pieces")
    trk.close()


def test_loss_of_lock_matches_oracle(ctx):
    """Signal for 0.3 s then noise only (whose m2m4 estimate sits near 29 dB-Hz, hence cn0_min = 35):
    CN0 decays through the smoother below cn0_min and the
    code-lock fail counter passes max_code_lock_fail → state 0, flags & 2, no further epochs."""
    fs = 4e6
    sat, k, x, stamp, first, delay, dop = S.sync("GPS", fs, 1200, cn0=45.0, cn0_smoother_alpha=0.02, cn0_min=35)
    cut = int(0.3 * fs)
    noise = signals.generate_if(fs, len(x) - cut, [], seed=99, start=first + cut)
    x = np.concatenate([x[:cut], noise])
    ctx.set_code(5, sat.code)
    trk = engine.DllPllVemlTracking(ctx, dev_conf(k, "GPS"), 1)
    trk.start(0, 5, delay, dop, stamp, first)
    rec, rounds = trk.run(x, first, 1200)
    ref = T.track(k, x, sat.code, delay, dop, stamp, first, 1200, buffer_first=first)
    assert ref["flags"][-1] & 2 and len(ref) < 1200
    compare_exact(rec[:, 0], ref, "loss")
    assert rounds == len(ref)
    assert trk.channel_state(0)[0] == 0
    trk.close()


def test_bad_configuration_and_arguments(ctx):
    k = T.conf("GPS", 4e6, 4000)
    bad = dev_conf(k, "GPS")
    bad.cn0_samples = 100
    with pytest.raises(abi.GnssHipError):
        engine.DllPllVemlTracking(ctx, bad, 1)
    trk = engine.DllPllVemlTracking(ctx, dev_conf(k, "GPS"), 2)
    with pytest.raises(abi.GnssHipError):
        trk.start(2, 0, 0.0, 0.0, 0, 0)  # channel out of range
    with pytest.raises(abi.GnssHipError):
        trk.start(0, 999, 0.0, 0.0, 0, 0)  # code not in the bank
    trk.close()


def test_idle_channel_with_empty_code_slot():
    """Regression: a never-started channel's job points at code slot 0; in a fresh context that slot
    is empty.  Idle chunks must not touch the code bank (illegal address before the fix)."""
    with engine.Context(0) as fresh:
        sat, k, x, stamp, first, delay, dop = S.pull_in("GPS", 4e6, 48.0, 900.0, 20.0, 5.0, 0.1, 30)
        fresh.set_code(77, sat.code)
        trk = engine.DllPllVemlTracking(fresh, dev_conf(k, "GPS"), 3)
        trk.start(2, 77, delay, dop, stamp, first)
        rec, rounds = trk.run(x, 0, 30)
        assert rounds == 30
        assert not np.any(rec[:, 0]["flags"]) and not np.any(rec[:, 1]["flags"])
        compare_exact(rec[:, 2], T.track(k, x, sat.code, delay, dop, stamp, first, 30), "idle")
        trk.close()


def test_auto_rotator_with_unreproduced_preference_fails_create(tmp_path):
    """ROTATOR_AUTO (every binding's default) under a volk_gnsssdr preference entry the engine does
    not reproduce (generic_reload): gnsship_trk_create fails with E_INVAL and the dispatcher's detail,
    instead of running another rotator silently.  A child process, so the preference file
    is the one the library reads."""
    import os
    import subprocess
    import sys
    cfg = tmp_path / "cfg" / "volk_gnsssdr"
    cfg.mkdir(parents=True)
    (cfg / "volk_gnsssdr_config").write_text("volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn generic_reload generic_reload\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from gnss_sim_receiver_amd import abi, engine\n"
            "ctx = engine.Context(0)\n"
            "c = abi.TrkConf.defaults(abi.SYS_GPS_L1CA, 4e6, 4000)\n"
            "assert c.rotator == abi.ROTATOR_AUTO\n"
            "try:\n    engine.DllPllVemlTracking(ctx, c, 1)\n    print('CREATED')\n"
            "except abi.GnssHipError as e:\n    print('ERR', e)\n") % root
    env = {k: v for k, v in os.environ.items() if k not in ("VOLK_GENERIC",)}
    env["VOLK_CONFIGPATH"] = str(tmp_path / "cfg")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    last = out.stdout.strip().splitlines()[-1]
    assert last.startswith("ERR") and "E_INVAL" in last and "generic_reload" in last, last


def test_start_many_matches_start(ctx):
    """gnsship_trk_start_many (one upload, one scatter, one sync) starts channels exactly as
    gnsship_trk_start does: the runs' records are identical; a bad entry starts nothing."""
    sats = [S.sync("GPS", 4e6, 150, prn=p, dop=d, delay_chips=c, seed=p) for p, d, c in ((3, 900.0, 10.5), (9, -1500.0, 700.2), (17, 40.0, 333.3))]
    x = np.sum([s[2] for s in sats], axis=0).astype(np.complex64)
    k, first = sats[0][1], sats[0][4]
    starts = []
    for i, (sat, _, _, stamp, _, delay, dop) in enumerate(sats):
        ctx.set_code(90 + i, sat.code)
        starts.append((2 * i + 1, 90 + i, delay, dop, stamp, first))
    recs = []
    for many in (False, True):
        trk = engine.DllPllVemlTracking(ctx, dev_conf(k, "GPS"), 7)
        if many:
            trk.start_many(starts)
        else:
            for st in starts:
                trk.start(*st)
        rec, rounds = trk.run(x, first, 150)
        recs.append(rec)
        if many:
            with pytest.raises(abi.GnssHipError):  # a channel twice
                trk.start_many([(0, 90, 10.0, 0.0, 0, first), (0, 91, 10.0, 0.0, 0, first)])
            with pytest.raises(abi.GnssHipError):  # the second entry's code is not in the bank: nothing starts
                trk.start_many([(0, 90, 10.0, 0.0, 0, first), (2, 999, 10.0, 0.0, 0, first)])
            assert trk.channel_state(0)[0] == 0
        trk.close()
    assert np.array_equal(recs[0].view(np.uint8), recs[1].view(np.uint8))
    assert np.count_nonzero(recs[1][:, 1]["flags"] & 8) == 150

"""Multicorrelator parity on the GPU: libgnsship.so (HIP, gfx950) vs the generic-semantics oracle.

Contract (BASELINE.json north_star): per tap |out − ref| / |ref| ≤ 1e-5 against the reference's
generic volk_gnsssdr path (oracle), same synthetic input.  Generic-rotator jobs (no flag) run the
reference's own order (corr_serial.hip: one phasor chain, one serial float sum per tap component)
and are compared for equality; GNSSHIP_JOB_ROTATOR_TREE jobs (anchored tree sums, the pipelined
launch forms) and AVX batch jobs are held to the 1e-5 contract.
"""
import os

import numpy as np
import pytest

from gnss_sim_receiver_amd import abi, engine, signals
from oracle import oracle as O

pytestmark = pytest.mark.gpu
TOL = 1e-5
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def rel_err(out, ref):
    return np.max(np.abs(out - ref) / np.maximum(np.abs(ref), 1e-30))


def mk_job(offset, n, code_id, shifts, rem_carr, carr_step, rem_code, code_step):
    j = np.zeros(1, abi.JOB_DTYPE)[0]
    j["sample_offset"] = offset
    j["n_samples"] = n
    j["code_id"] = code_id
    j["n_taps"] = len(shifts)
    j["rem_carrier_phase_rad"] = rem_carr
    j["phase_step_rad"] = carr_step
    j["rem_code_phase_chips"] = rem_code
    j["code_phase_step_chips"] = code_step
    s = np.zeros(abi.MAX_TAPS, np.float32)
    s[: len(shifts)] = shifts
    j["shifts_chips"] = s
    return j


def test_golden_corr_cases(ctx):
    g = np.load(os.path.join(GOLD, "corr_cases.npz"))
    codes = np.load(os.path.join(GOLD, "codes_ref.npz"))["gps"].astype(np.float32)
    mc = engine.MultiCorrelatorRealCodes(ctx)
    mc.init(2 * 25000, 5)
    for i in range(10):
        prn, n, rem_carr, carr_step, rem_code, code_step = g[f"c{i}_args"]
        sh = g[f"c{i}_shifts"]
        mc2 = engine.MultiCorrelatorRealCodes(ctx, rotator=abi.ROTATOR_GENERIC)
        mc2.init(int(n), len(sh))
        mc2.set_local_code_and_taps(1023, codes[int(prn) - 1], sh)
        out = np.zeros(len(sh), np.complex64)
        mc2.set_input_output_vectors(out, g[f"c{i}_sig"])
        mc2.Carrier_wipeoff_multicorrelator_resampler(rem_carr, carr_step, 0.0, rem_code, code_step, 0.0, int(n))
        mc2.free()
        assert np.array_equal(out, g[f"c{i}_out"]), (i, rel_err(out, g[f"c{i}_out"]))  # bit for bit
    mc.free()


@pytest.mark.parametrize("fs,ntaps,system", [(4e6, 3, "GPS"), (25e6, 3, "GPS"), (25e6, 5, "GPS"), (4e6, 1, "GPS"),
                                             (2.046e6, 3, "BDS"), (50e6, 3, "BDS")])
def test_batch_vs_oracle(ctx, fs, ntaps, system):
    rng = np.random.default_rng(int(fs) + ntaps)
    sats = signals.random_sky(6, seed=int(fs) % 9973, system=system)
    vl = int(round(fs / 1000))
    n_ep = 3
    total = vl * (n_ep + 3)
    sig = signals.generate_if(fs, total, sats, seed=ntaps)
    shifts = {1: [0.0], 3: [-0.25, 0.0, 0.25], 5: [-0.5, -0.25, 0.0, 0.25, 0.5]}[ntaps]
    jobs = []
    cl = []
    for k, s in enumerate(sats):
        cl.append(s.code)
        jobs.append(signals.truth_jobs(s, fs, n_ep, vl, shifts, k))
    jobs = np.concatenate(jobs)
    # perturb NCO a bit so taps are not all at ideal alignment
    jobs["rem_carrier_phase_rad"] += rng.uniform(-0.3, 0.3, len(jobs)).astype(np.float32)
    out = engine.correlate_host(ctx, sig, jobs, cl)
    ref = O.corr_batch(sig, jobs, cl, n_threads=8)
    for j in range(len(jobs)):
        t = jobs[j]["n_taps"]
        assert np.array_equal(out[j, :t], ref[j, :t]), (j, rel_err(out[j, :t], ref[j, :t]), out[j, :t], ref[j, :t])
        assert np.all(out[j, t:] == 0)


@pytest.mark.parametrize("fmt", ["ci16", "ci8"])
def test_integer_formats(ctx, fmt):
    fs = 4e6
    sats = signals.random_sky(4, seed=3)
    sig = signals.generate_if(fs, 20000, sats, seed=9)
    raw = signals.to_ishort(sig) if fmt == "ci16" else signals.to_ibyte(sig)
    as_float = raw.astype(np.float32).view(np.complex64)  # the reference converts without scaling
    jobs = np.concatenate([signals.truth_jobs(s, fs, 2, 4000, [-0.25, 0, 0.25], k) for k, s in enumerate(sats)])
    cl = [s.code for s in sats]
    out = engine.correlate_host(ctx, raw, jobs, cl)
    ref = O.corr_batch(as_float, jobs, cl)
    assert np.array_equal(out[:, :3], ref[:, :3])


def test_edge_cases_index_wrap_and_lengths(ctx):
    """Zero length, one sample, ragged lengths, multi-chunk jobs, codes longer/shorter than the
    span, negative and > L code phases (resampler wrap), noise-only input."""
    rng = np.random.default_rng(11)
    sig = (rng.standard_normal(300000) + 1j * rng.standard_normal(300000)).astype(np.complex64)
    code = np.where(rng.random(1023) > 0.5, 1.0, -1.0).astype(np.float32)
    code2 = np.where(rng.random(8184) > 0.5, 1.0, -1.0).astype(np.float32)
    jobs = [
        mk_job(0, 0, 0, [0.0], 0.1, 0.01, 0.0, 0.25575),
        mk_job(5, 1, 0, [-0.5, 0, 0.5], 0.1, 0.01, 0.0, 0.25575),
        mk_job(7, 255, 0, [-0.5, 0, 0.5], -3.0, -0.02, 0.7, 0.25575),
        mk_job(11, 4097, 0, [-0.5, 0, 0.5], 2.0, 0.005, -1022.5, 0.25575),
        mk_job(13, 100000, 1, [-1.0, -0.5, 0, 0.5, 1.0], 0.5, 0.0123, 8000.25, 0.08184),
        mk_job(17, 12345, 0, [-2.0, -0.1, 0.1, 2.0, 3.0, 4.0, 5.0, -5.0], 1.0, 0.001, 3000.75, 1.023),
        mk_job(299000, 1000, 0, [0.0], 0.0, 0.0, 0.0, 0.25575),
    ]
    jobs = np.array(jobs, abi.JOB_DTYPE)
    out = engine.correlate_host(ctx, sig, jobs, [code, code2])
    ref = O.corr_batch(sig, jobs, [code, code2])
    assert np.all(out[0] == 0)
    for j in range(1, len(jobs)):  # the reference's serial order: bit for bit, noise-only taps included
        t = jobs[j]["n_taps"]
        assert np.array_equal(out[j, :t], ref[j, :t]), (j, out[j, :t], ref[j, :t])
    # the anchored tree form (GNSSHIP_JOB_ROTATOR_TREE) of the same jobs: 1e-5 of the accumulation
    # scale — noise-only taps can cancel to |ref| ≪ ||x||₂, where the reference's own serial float sum
    # carries ~n·2⁻²⁴·|partial sum| of rounding (the RMS of such a sum is ||x||₂)
    tj = jobs.copy()
    tj["flags"] = abi.JOB_ROTATOR_TREE
    tout = engine.correlate_host(ctx, sig, tj, [code, code2])
    assert np.all(tout[0] == 0)
    for j in range(1, len(jobs)):
        t = jobs[j]["n_taps"]
        n = jobs[j]["n_samples"]
        x = sig[jobs[j]["sample_offset"]: jobs[j]["sample_offset"] + n]
        scale = np.maximum(np.abs(ref[j, :t]), np.sqrt(np.sum(np.abs(x.astype(np.complex128)) ** 2)))
        e = np.max(np.abs(tout[j, :t] - ref[j, :t]) / scale)
        assert e <= TOL, (j, e)


def test_bounds_and_state_errors(ctx):
    code = np.ones(1023, np.float32)
    ctx.set_code(0, code)
    b = engine.CorrelatorBatch(ctx, 4)
    j = np.array([mk_job(100, 1000, 0, [0.0], 0, 0, 0, 0.25)], abi.JOB_DTYPE)
    with pytest.raises(abi.GnssHipError):
        b.set_jobs(j, 500)  # reads past the buffer
    j2 = np.array([mk_job(0, 10, 9999, [0.0], 0, 0, 0, 0.25)], abi.JOB_DTYPE)
    with pytest.raises(abi.GnssHipError):
        b.set_jobs(j2, 500)  # unset code id
    j3 = np.array([mk_job(0, 10, 0, [0.0] * 1, 0, 0, 0, 0.25)], abi.JOB_DTYPE)
    j3["n_taps"] = 9
    with pytest.raises(abi.GnssHipError):
        b.set_jobs(j3, 500)
    b.close()
    mc = engine.MultiCorrelatorRealCodes(ctx)
    mc.init(100, 3)
    out = np.zeros(3, np.complex64)
    mc.set_input_output_vectors(out, np.zeros(100, np.complex64))
    with pytest.raises(abi.GnssHipError):  # set_local_code_and_taps not called
        mc.Carrier_wipeoff_multicorrelator_resampler(0, 0, 0, 0, 0.25, 0, 100)
    mc.set_local_code_and_taps(1023, code, np.zeros(3, np.float32))
    with pytest.raises(abi.GnssHipError):  # longer than max_signal_length_samples
        mc.Carrier_wipeoff_multicorrelator_resampler(0, 0, 0, 0, 0.25, 0, 101)
    mc.free()


def test_device_resident_buffer_large_batch_properties(ctx):
    """Full C2 shape (12 channels × 1000 epochs at 4 Msps) on a device-resident 1 s buffer:
    prompt power is maximal at the truth alignment for every channel-epoch and E/L are symmetric
    (size-independent properties), plus exact oracle parity on a sampled subset."""
    fs, vl = 4e6, 4000
    sats = signals.random_sky(12, seed=0x6E550002)
    n_ep = 1000
    total = vl * (n_ep + 4)
    sig = signals.generate_if(fs, total, sats, seed=0x6E550002)
    jobs = np.concatenate([signals.truth_jobs(s, fs, n_ep, vl, [-0.25, 0.0, 0.25], k) for k, s in enumerate(sats)])
    cl = [s.code for s in sats]
    out = engine.correlate_host(ctx, sig, jobs, cl)
    p = np.abs(out[:, :3])
    assert np.mean(p[:, 1] > p[:, 0]) > 0.95 and np.mean(p[:, 1] > p[:, 2]) > 0.95
    pick = np.random.default_rng(0).choice(len(jobs), 64, replace=False)
    ref = O.corr_batch(sig, jobs[pick], cl, n_threads=8)
    assert np.array_equal(out[pick, :3], ref[:, :3])


def test_pipelined_pair_matches_plain_launches(ctx):
    """gnsship_batch_launch_pipelined: A, B, A, B with each launch replaying the other batch's
    anchors gives exactly the plain launch results (same kernels, same anchors), including after
    set_jobs invalidates a batch's prefetched anchors (anchored generic jobs: GNSSHIP_JOB_ROTATOR_TREE)."""
    fs = 4e6
    sats = signals.random_sky(6, seed=41)
    sig = signals.generate_if(fs, 4000 * 40, sats, seed=42)
    dev = ctx.upload(sig)
    ja = np.concatenate([signals.truth_jobs(s, fs, 12, 4000, [-0.25, 0.0, 0.25], k) for k, s in enumerate(sats[:3])])
    jb = np.concatenate([signals.truth_jobs(s, fs, 9, 4000, [-0.5, -0.25, 0.0, 0.25, 0.5], k + 3, first_epoch=20)
                         for k, s in enumerate(sats[3:])])
    ja["flags"] = abi.JOB_ROTATOR_TREE
    jb["flags"] = abi.JOB_ROTATOR_TREE
    for k, s in enumerate(sats):
        ctx.set_code(k, s.code)
    A, B = engine.CorrelatorBatch(ctx, len(ja)), engine.CorrelatorBatch(ctx, len(jb))
    A.set_jobs(ja, len(sig))
    B.set_jobs(jb, len(sig))
    A.launch_ptr(dev.ptr)
    ref_a = A.results()
    B.launch_ptr(dev.ptr)
    ref_b = B.results()
    for rnd in range(3):
        A.launch_pipelined(dev.ptr, next_batch=B)
        assert np.array_equal(A.results(), ref_a), rnd
        B.launch_pipelined(dev.ptr, next_batch=A)
        assert np.array_equal(B.results(), ref_b), rnd
    # new jobs for A: its prefetched anchors are stale and must be recomputed
    ja2 = ja.copy()
    ja2["rem_carrier_phase_rad"] += np.float32(0.7)
    A.set_jobs(ja2, len(sig))
    A.launch_pipelined(dev.ptr, next_batch=B)
    got = A.results()
    ref = O.corr_batch(sig, ja2, [s.code for s in sats], n_threads=8)
    for j in range(len(ja2)):
        assert rel_err(got[j, :3], ref[j, :3]) <= TOL
    with pytest.raises(abi.GnssHipError):
        A.launch_pipelined(dev.ptr, next_batch=A)
    A.close()
    B.close()
    dev.free()


def test_pipelined_ring_of_three_split_replay(ctx):
    """gnsship_batch_launch_pipelined2 over a ring A, B, C: each launch finishes the replay of the
    next batch and runs the first half (up to each job's middle renormalisation block) of the one
    after; the resumed second halves give bit-identical anchors, hence exactly the plain launch
    results.  Covers odd block counts (3001-sample jobs: 12 blocks; 1 and 2 blocks), a set_jobs
    between the two halves (full replay again) and invalid rings."""
    fs = 4e6
    sats = signals.random_sky(6, seed=51)
    sig = signals.generate_if(fs, 4000 * 30, sats, seed=52)
    dev = ctx.upload(sig)
    for k, s in enumerate(sats):
        ctx.set_code(k, s.code)
    ja = np.concatenate([signals.truth_jobs(s, fs, 10, 4000, [-0.25, 0.0, 0.25], k) for k, s in enumerate(sats[:2])])
    jb = np.concatenate([signals.truth_jobs(s, fs, 8, 3001, [-0.5, 0.0, 0.5], k + 2, first_epoch=5) for k, s in enumerate(sats[2:4])])
    jc = np.concatenate([signals.truth_jobs(s, fs, 6, 4000, [0.0], k + 4, first_epoch=3) for k, s in enumerate(sats[4:])])
    jc["n_samples"][::3] = 200   # one block
    jc["n_samples"][1::3] = 300  # two blocks
    for j in (ja, jb, jc):
        j["flags"] = abi.JOB_ROTATOR_TREE  # the anchored generic form (the plain generic jobs have no anchors)
    sets = [ja, jb, jc]
    batches = [engine.CorrelatorBatch(ctx, len(j)) for j in sets]
    refs = []
    for b, j in zip(batches, sets):
        b.set_jobs(j, len(sig))
        b.launch_ptr(dev.ptr)
        refs.append(b.results())
    for rnd in range(7):
        k = rnd % 3
        batches[k].launch_pipelined(dev.ptr, next_batch=batches[(k + 1) % 3], next2=batches[(k + 2) % 3])
        assert np.array_equal(batches[k].results(), refs[k]), rnd
    # C got its first half in the last launch (k = 0); new jobs for C discard it
    jc2 = jc.copy()
    jc2["rem_carrier_phase_rad"] += np.float32(0.4)
    batches[2].set_jobs(jc2, len(sig))
    batches[1].launch_pipelined(dev.ptr, next_batch=batches[2], next2=batches[0])
    batches[2].launch_pipelined(dev.ptr, next_batch=batches[0], next2=batches[1])
    ref = O.corr_batch(sig, jc2, [s.code for s in sats], n_threads=8)
    got = batches[2].results()
    for j in range(2, len(jc2), 3):  # the full-length jobs (the 1- and 2-block ones are checked bit-exactly above)
        assert rel_err(got[j, :1], ref[j, :1]) <= TOL
    for nb, n2 in ((batches[1], batches[1]), (batches[0], batches[1]), (batches[1], batches[0])):
        with pytest.raises(abi.GnssHipError):
            batches[0].launch_pipelined(dev.ptr, next_batch=nb, next2=n2)
    for b in batches:
        b.close()
    dev.free()


@pytest.mark.parametrize("fs,ntaps,system", [(4e6, 3, "GPS"), (25e6, 3, "GPS"), (25e6, 5, "GPS"), (50e6, 3, "BDS")])
def test_batch_avx_rotator_vs_oracle(ctx, fs, ntaps, system):
    """GNSSHIP_JOB_ROTATOR_AVX jobs (the variant volk_gnsssdr dispatches on AVX hosts,
    volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn.h:155-316) against the oracle's AVX restatement:
    N = 4000, 25000 (N mod 16 = 8: the serial tail), 50000; mixed with generic jobs in one batch."""
    rng = np.random.default_rng(int(fs) + 7 * ntaps)
    sats = signals.random_sky(6, seed=int(fs) % 7919, system=system)
    vl = int(round(fs / 1000))
    n_ep = 3
    sig = signals.generate_if(fs, vl * (n_ep + 3), sats, seed=ntaps + 11)
    shifts = {3: [-0.25, 0.0, 0.25], 5: [-0.5, -0.25, 0.0, 0.25, 0.5]}[ntaps]
    jobs = np.concatenate([signals.truth_jobs(s, fs, n_ep, vl, shifts, k) for k, s in enumerate(sats)])
    cl = [s.code for s in sats]
    jobs["rem_carrier_phase_rad"] += rng.uniform(-0.3, 0.3, len(jobs)).astype(np.float32)
    jobs["flags"][::3] = 0
    jobs["flags"][1::3] = abi.JOB_ROTATOR_AVX
    jobs["flags"][2::3] = abi.JOB_ROTATOR_AVX
    out = engine.correlate_host(ctx, sig, jobs, cl)
    ref = O.corr_batch(sig, jobs, cl, n_threads=8)
    for j in range(len(jobs)):
        t = jobs[j]["n_taps"]
        e = rel_err(out[j, :t], ref[j, :t])
        assert e <= TOL, (j, int(jobs[j]["flags"]), e)
    # the two variants really differ in the oracle (the flag reaches it) by less than the tolerance
    gen = jobs.copy()
    gen["flags"] = 0
    ref_gen = O.corr_batch(sig, gen, cl, n_threads=8)
    avx = jobs["flags"] == abi.JOB_ROTATOR_AVX
    assert not np.array_equal(ref[avx], ref_gen[avx])


@pytest.mark.parametrize("n", [7, 15, 16, 17, 255, 1023, 4096, 4104, 8200, 12345])
def test_batch_avx_rotator_lengths(ctx, n):
    """AVX-variant edge lengths: no whole iteration (N < 16: all tail), one iteration, tasks ending
    mid-chunk, the N mod 16 tail alone in a new 4096-sample chunk (4104 = 256·16 + 8), several chunks;
    50 Msps with a 7 MHz IF (large phase steps) beside a zero-IF job."""
    fs = 50e6
    sats = signals.random_sky(2, seed=n, system="GPS")
    sats[0].f_if_hz = 7.161e6
    sig = signals.generate_if(fs, 3 * 50000 + n + 64, sats, seed=n + 1)  # epochs start at code-period boundaries (≤ 2 ms)
    jobs = np.concatenate([signals.truth_jobs(s, fs, 2, n, [-0.25, 0.0, 0.25], k, first_epoch=0) for k, s in enumerate(sats)])
    jobs["flags"] = abi.JOB_ROTATOR_AVX
    cl = [s.code for s in sats]
    out = engine.correlate_host(ctx, sig, jobs, cl)
    ref = O.corr_batch(sig, jobs, cl, n_threads=4)
    for j in range(len(jobs)):
        assert rel_err(out[j, :3], ref[j, :3]) <= TOL, (n, j, rel_err(out[j, :3], ref[j, :3]))


def test_pipelined_ring_avx_jobs_match_plain_launches(ctx):
    """AVX-variant jobs through the pipelined ring (replay split at the middle task, resumed from the
    stored 16 phasors) give exactly the plain launch results; odd task counts and one-task jobs."""
    fs = 4e6
    sats = signals.random_sky(6, seed=61)
    sig = signals.generate_if(fs, 4000 * 30, sats, seed=62)
    dev = ctx.upload(sig)
    for k, s in enumerate(sats):
        ctx.set_code(k, s.code)
    ja = np.concatenate([signals.truth_jobs(s, fs, 10, 4000, [-0.25, 0.0, 0.25], k) for k, s in enumerate(sats[:2])])
    jb = np.concatenate([signals.truth_jobs(s, fs, 8, 3001, [-0.5, 0.0, 0.5], k + 2, first_epoch=5) for k, s in enumerate(sats[2:4])])
    jc = np.concatenate([signals.truth_jobs(s, fs, 6, 4000, [0.0], k + 4, first_epoch=3) for k, s in enumerate(sats[4:])])
    jc["n_samples"][::3] = 200
    jc["n_samples"][1::3] = 1300
    for j in (ja, jb, jc):
        j["flags"] = abi.JOB_ROTATOR_AVX
    sets = [ja, jb, jc]
    batches = [engine.CorrelatorBatch(ctx, len(j)) for j in sets]
    refs = []
    for b, j in zip(batches, sets):
        b.set_jobs(j, len(sig))
        b.launch_ptr(dev.ptr)
        refs.append(b.results())
    for rnd in range(7):
        k = rnd % 3
        batches[k].launch_pipelined(dev.ptr, next_batch=batches[(k + 1) % 3], next2=batches[(k + 2) % 3])
        assert np.array_equal(batches[k].results(), refs[k]), rnd
    for k, j in enumerate(sets):
        ref = O.corr_batch(sig, j, [s.code for s in sats], n_threads=8)
        for i in range(len(j)):
            t = j[i]["n_taps"]
            assert rel_err(refs[k][i, :t], ref[i, :t]) <= TOL, (k, i)
    for b in batches:
        b.close()
    dev.free()

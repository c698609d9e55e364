#!/usr/bin/env python3
"""Benchmark: IF Msamples/s processed & tracked channels sustained (BASELINE.json `metric`).

Headline (`value`): a D-second synthetic IF file processed with ALL C channels in
steady-state closed-loop tracking — BASELINE.json configs[1]: GPS L1 C/A, 12 channels, 4 Msps
gr_complex, one MI355X per rank.
  * the file: 32 GPS satellites (SURVEY §8d model, CN0 45 dB-Hz, seed 0x6E550002) with navigation
    bits (the TLM preamble recurring every 260 ms), generated on the GPU (signals.generate_if_device)
    and resident in HBM before the timed region;
  * the receiver: dll_pll_veml_tracking for 12 channels (channel c tracks satellite c), started from
    an acquisition stamped 11 s before the file's first sample (the reference's 10 s pull-in is over,
    dll_pll_veml_tracking.cc:1746-1752) and pre-rolled 0.5 s, so every channel is bit-synchronised
    (state 4) before the warm-up steps;
  * one step = the closed loop over the next D seconds of the file (every channel runs every epoch
    whose window lies in it: correlation + DLL/PLL update + lock detectors, on the device, one
    persistent launch — trk_fast.hip for the AVX rotator, trk_persist.hip for the generic one —
    whose epoch records (gnsship_trk_epoch, as the reference's per-epoch output) come back to the
    host inside the step), steps consecutive in the file.
  value = fs·D·steps ÷ max-over-ranks wall: the IF file's samples per second of the whole job.  At N
  ranks every rank tracks its own 12 channels of the same RCCL-broadcast file (weak scaling in
  channels: `channels_tracked` = 12·N, `channel_msamples_per_s` = 12·N·fs·D·steps ÷ wall beside it).
  The rotator variant is the one volk_gnsssdr dispatches on this host (gnsship_rotator_dispatch: AVX
  on x86 hosts with AVX), named in `config`.
tracked_channels_sustained: channel sweep (12 … 65536 channels on one GPU, the same file and loop)
  → the largest MEASURED channel count that ran at ≥ real time.

Auxiliary lines (never `value`): the generic-rotator closed loop, closed loops at 25 Msps (GPS and
the Galileo E1 C4 share), the C5 per-GPU share in closed loop (12 GPS + 12 E1 + 8 B1I engines
launched together at 50 Msps ibyte with the IF in the NCO), the open-loop batched correlator (round
1's headline, truth NCOs), PCPS acquisition sweeps (C1-shape, C3, E1), the open-loop C4/C5 legs, and
for N > 1 the streaming leg (the file broadcast block by block, double-buffered against tracking).
cpu_baseline: the oracle's closed loop (same loop, same rotator variant) with one thread per
channel (12) on the host's cores, on a bounded sample of the same file, rank 0 at N = 1 — for the
AVX variant its correlator is the AVX2 restatement (oracle/avx_port.c: u_avx's 16 phasor lanes in
two __m256 pairs, the resampler vectorised), the form the reference itself runs on such a host.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FS = 4_000_000
VL = 4000               # vector_length = round(fs / (chip_rate / code_length))  (gps_l1_ca_dll_pll_tracking.cc:47)
N_CH = 12               # channels per receiver (configs[1])
N_SATS = 32
SHIFTS = [-0.25, 0.0, 0.25]   # Dll_Pll_Conf early_late_space_chips = 0.25 (dll_pll_conf.h:50)
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
VALU_PEAK = 256 * 4 * 2.4e9 / 2.0  # wave64 VALU instructions/s: 256 CUs x 4 SIMDs, 2 cycles per wave64 op at 2.4 GHz
SEED = 0x6E550002
T_START_S = 11.0        # tracking starts this long after the acquisition stamp (pull_in_time_s = 10 elapsed)
PRE_ROLL_S = 0.5        # untimed: bit synchronisation (state 2 -> 4)
GPS_NAV = "1000101100110"  # 10001011 preamble + 5 bits: the sync pattern every 13 bits = 260 ms


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--seconds", type=float, default=1.0, help="IF seconds per step (D)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU baseline time budget (0 = skip)")
    ap.add_argument("--no-aux", action="store_true", help="headline only (no auxiliary lines)")
    ap.add_argument("--sharded-aux-only", action="store_true", help="of the auxiliary lines, only the multi-rank ones")
    ap.add_argument("--rotator", type=int, default=-1, help="-1 volk's dispatch on this host, 0 generic, 1 AVX")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_trk.json"),
                    help="rocprofv3 PMC summary of the headline kernel (HBM bytes, VALU instructions per launch)")
    return ap.parse_args()


# ---------------------------------------------------------------------------------------------------
# closed loop
def gps_sky(n=N_SATS, seed=SEED, fs=FS):
    from gnss_sim_receiver_amd import signals
    sats = signals.random_sky(n, seed=seed)
    for s in sats:
        s.bits = GPS_NAV
    return sats


class Receiver:
    """n_ch channels of dll_pll_veml_tracking on one engine, channel c tracking sats[c % len(sats)],
    started from truth acquisitions stamped at sample 0 with tracking from absolute sample `first`."""

    def __init__(self, ctx, system, fs, vl, sats, n_ch, first, rotator, code_base=300):
        from gnss_sim_receiver_amd import abi, engine, signals
        sysid = {"GPS": abi.SYS_GPS_L1CA, "GAL": abi.SYS_GAL_E1, "BDS": abi.SYS_BDS_B1I}[system]
        self.conf = abi.TrkConf.defaults(sysid, fs, vl, rotator=rotator)
        self.trk = engine.DllPllVemlTracking(ctx, self.conf, n_ch)
        self.n_ch, self.vl, self.fs = n_ch, vl, fs
        for i, s in enumerate(sats):
            ctx.set_code(code_base + 2 * i, s.code)
            if s.code_data is not None:
                ctx.set_code(code_base + 2 * i + 1, s.code_data)
        starts = []
        for ch in range(n_ch):
            i = ch % len(sats)
            s = sats[i]
            starts.append((ch, code_base + 2 * i, signals.acq_delay_samples(s, fs, 0, first), s.doppler_hz, 0, first,
                           code_base + 2 * i + 1, s.prn))
        self.trk.start_many(starts)  # one transaction (gnsship_trk_start_many)

    def run(self, dev_ptr, fmt, first, n):
        return self.trk.run_ptr(dev_ptr, fmt, first, n, 1 << 20)

    def run_records(self, dev_ptr, fmt, first, n, max_rounds):
        """The same run with the epoch records copied back (launch + collect on the engine's stream)."""
        self.trk.launch_ptr(dev_ptr, fmt, first, n, max_rounds, records=True)
        return self.trk.collect()

    def close(self):
        self.trk.close()


def rotator_name(r):
    return {0: "generic (volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn_generic)",
            1: "u_avx/a_avx (volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn.h:155-316)"}[r]


def closed_loop_steps(ctx, rx, dev_ptr, t0_abs, fs, step_s, n_steps, barrier=None, timed=True, period_s=0.001):
    """Run n_steps consecutive D-second segments of the file through the receiver.  Each segment is
    passed with a little slack on both sides (the channels' epoch windows straddle the boundaries;
    every channel consumes each sample once); max_rounds is sized to the segment (D ÷ code period +
    4) and every step's epoch records are copied to the host inside the timed region.  Returns
    (wall, kernel_ms list, records emitted)."""
    step_n = int(round(step_s * fs))
    slack = 2 * rx.vl
    max_rounds = int(round(step_s / period_s)) + 4
    kms = []
    n_rec = 0
    if barrier:
        barrier()
    t0 = time.perf_counter()
    for i in range(n_steps):
        lo = t0_abs + i * step_n - slack
        ctx.event_record(0)
        rec, done = rx.run_records(dev_ptr[0] + (lo - dev_ptr[1]) * 8, 0, lo, step_n + 2 * slack, max_rounds)
        ctx.event_record(1)
        n_rec += int(np.count_nonzero(rec[:done]["flags"] & 8))
        if timed:
            kms.append(ctx.event_elapsed_ms(0, 1))
    if barrier:
        barrier()
    return time.perf_counter() - t0, kms, n_rec


def headline(ctx, torch, args, rank, world, device, barrier):
    from gnss_sim_receiver_amd import abi, sharding, signals
    rot = args.rotator if args.rotator >= 0 else abi.rotator_dispatch()
    sats = gps_sky()
    first = int(T_START_S * FS)
    n_total = int(round((PRE_ROLL_S + (args.warmup + args.steps) * args.seconds) * FS)) + 4 * VL
    # the file, resident in HBM on every rank: rank 0 generates it, one RCCL broadcast fans it out
    if rank == 0:
        x = signals.generate_if_device(FS, n_total, sats, seed=SEED, start=first - 2 * VL, device=f"cuda:{device}")
    else:
        x = torch.empty(n_total, dtype=torch.complex64, device=f"cuda:{device}")
    fan_out(ctx, torch, x, world)
    base = (x.data_ptr(), first - 2 * VL)  # (device pointer, absolute index of x[0])
    chans = [(rank * N_CH + c) % N_SATS for c in range(N_CH)]
    rx = Receiver(ctx, "GPS", FS, VL, [sats[i] for i in chans], N_CH, first, rot)
    # pre-roll: bit synchronisation, then the warm-up steps
    pre_n = int(round(PRE_ROLL_S * FS))
    rx.run(base[0] + 2 * VL * 8, 0, first, pre_n + 2 * VL)
    st = rx.trk.states()
    closed_loop_steps(ctx, rx, base, first + pre_n, FS, args.seconds, args.warmup, timed=False)
    t_timed = first + pre_n + int(round(args.warmup * args.seconds * FS))
    wall, kms, n_rec = closed_loop_steps(ctx, rx, base, t_timed, FS, args.seconds, args.steps, barrier=barrier)
    st_end = rx.trk.states()
    wall = sharding.max_over_ranks(wall)
    rx.close()
    return dict(rotator=rot, wall=wall, kernel_ms=float(np.mean(kms)), states_pre=st, states_end=st_end, x=x, base=base, sats=sats,
                first=first, records=n_rec)


SWEEP_PRE = 450  # epochs: every channel bit-synchronised (state 4) before a sweep point's timed epochs


def sweep_file_25msps(torch, device, rounds=1000):
    """The 25 Msps sweep's file: the same 32-satellite GPS sky model (navigation bits with the
    preamble), long enough for the pre-roll and `rounds` timed epochs of N = 25000, resident in HBM."""
    from gnss_sim_receiver_amd import signals
    fs, vl = 25_000_000, 25000
    sats = gps_sky(seed=SEED + 25)
    first = int(T_START_S * fs)
    n = (SWEEP_PRE + rounds + 8) * vl
    x = signals.generate_if_device(fs, n, sats, seed=SEED + 25, start=first - 2 * vl, device=f"cuda:{device}")
    torch.cuda.synchronize()
    return dict(x=x, base=(x.data_ptr(), first - 2 * vl), first=first, sats=sats, fs=fs, vl=vl)


def sweep(ctx, h, rot, counts, rounds=1000, fs=FS, vl=VL):
    """Tracked channels sustained: channels c -> satellite c mod 32 on the same file, each point run
    for `rounds` epochs (1 s of signal) from the steady-state point of the file, every channel-epoch's
    record (the Gnss_Synchro the reference emits, dll_pll_veml_tracking.cc:2063-2091) copied to the
    host inside the timed region.  fs / vl: the file's rate and the GPS vector_length (4 Msps: 4000,
    the headline's file; 25 Msps: 25000, gps_l1_ca_dll_pll_tracking.cc:47)."""
    from gnss_sim_receiver_amd import abi
    out = []
    t_abs = h["first"]
    pre = SWEEP_PRE
    for n in counts:
        rx = Receiver(ctx, "GPS", fs, vl, h["sats"], n, t_abs, rot, code_base=2000)
        n_samp = rounds * vl + 4 * vl
        # untimed: the pre-roll, with records on and the timed run's round count, so the device record
        # buffer is sized here; the host record array is allocated and touched here too
        rx.trk.launch_ptr(h["base"][0] + (t_abs - h["base"][1]) * 8, 0, t_abs, (pre + 2) * vl, rounds + 4, records=True)
        rx.trk.collect()
        host = np.empty((rounds + 4, n), abi.TRK_EPOCH_DTYPE)
        host.view(np.uint8).fill(0)
        lo = t_abs + pre * vl
        ctx.event_record(2)
        t0 = time.perf_counter()
        rx.trk.launch_ptr(h["base"][0] + (lo - h["base"][1]) * 8, 0, lo, n_samp, rounds + 4, records=True)
        rec, done = rx.trk.collect(out=host)
        dt = time.perf_counter() - t0
        ctx.event_record(3)
        k_ms = ctx.event_elapsed_ms(2, 3)
        eng = rx.trk.last_engine()  # the kernel the timed launch ran (gnsship_trk_last_engine)
        n_rec = int(np.count_nonzero(rec[:done]["flags"] & 8))
        idx = np.linspace(0, n - 1, min(n, 64)).astype(int)
        tracking = float(np.mean([rx.trk.channel_state(int(c))[0] in (2, 3, 4) for c in idx]))
        rx.close()
        del rec, host
        cps = n_rec / dt
        out.append({"channels": n, "kernel": abi.TRK_ENGINE_NAMES.get(eng, str(eng)), "epochs": done, "epoch_records": n_rec, "record_bytes": n_rec * 96, "us_per_epoch_round": round(dt / done * 1e6, 2),
                    "kernel_us_per_round": round(k_ms * 1e3 / done, 2), "channel_epochs_per_s": round(cps, 0),
                    "realtime_factor": round(done * 1e-3 / dt, 2), "tracking_fraction_sampled": round(tracking, 3)})
    return out


def closed_loop_aux(ctx, torch, device, system, fs, vl, n_ch, seconds, rot, seed):
    """Closed loop at another rate / signal: n_ch channels, 0.5 s pre-roll (synchronisation), then `seconds` timed."""
    from gnss_sim_receiver_amd import signals
    if system == "GAL":
        prns = [1, 5, 12, 19, 24, 30, 33, 36, 2, 8, 11, 26][:n_ch] if n_ch <= 12 else (list(range(1, 37)) * 2)[:n_ch]
        sats = signals.random_sky(n_ch, seed=seed, system="GAL", prns=prns)
        for s in sats:
            s.secondary = "0011100000001010110110010"
            s.bits = "0110"
        period = 0.004
    else:
        sats = gps_sky(n_ch, seed=seed)
        period = 0.001
    first = int(T_START_S * fs)
    pre = int(0.5 * fs)
    n_total = pre + int(round(seconds * fs)) + 4 * vl
    x = signals.generate_if_device(fs, n_total, sats, seed=seed, start=first - 2 * vl, device=f"cuda:{device}")
    torch.cuda.synchronize()
    base = (x.data_ptr(), first - 2 * vl)
    rx = Receiver(ctx, system, fs, vl, sats, n_ch, first, rot, code_base=1500)
    rx.run(base[0] + 2 * vl * 8, 0, first, pre + 2 * vl)
    lo = first + pre - 2 * vl
    ctx.event_record(2)
    t0 = time.perf_counter()
    done = rx.run(base[0] + (lo - base[1]) * 8, 0, lo, int(round(seconds * fs)) + 4 * vl)
    dt = time.perf_counter() - t0
    ctx.event_record(3)
    st = rx.trk.states()
    rx.close()
    del x
    sig_s = done * period
    return {"config": f"{system} {'L1 C/A' if system == 'GPS' else 'E1 B/C (5 VEML pilot taps + data prompt)'}, {n_ch} ch, "
                      f"{fs / 1e6:g} Msps, N={vl}, closed DLL/PLL loop, rotator {rot}",
            "epochs": done, "ms_per_signal_second": round(dt / sig_s * 1e3, 3), "realtime_factor": round(sig_s / dt, 1),
            "us_per_epoch_round": round(dt / done * 1e6, 2), "if_msamples_per_s": round(sig_s * fs / dt / 1e6, 1),
            "channels_in_state_4": int(np.sum(st == 4))}


def closed_loop_c5_share(torch, device, rot, seconds=0.2, pre_s=0.6, full=False):
    """configs[4]'s per-GPU share in closed loop: 12 GPS L1 C/A + 12 Galileo E1 (5 VEML pilot taps +
    data prompt) + 8 BeiDou B1I channels, three tracking engines each on its own context (stream),
    launched together over one 50 Msps ibyte block whose IF is centred 7.161 MHz from L1/E1 (−7.161
    MHz for B1I), the IF removed in the tracking NCO (gnsship_trk_conf::if_hz).  0.6 s pre-roll
    (bit / secondary-code synchronisation), then `seconds` timed: launch all three, collect all three.
    full=True: the whole of configs[4] on this one GPU — 96 GPS + 96 E1 + 64 B1I channels, every
    channel its own signal (PRNs re-used with their own Doppler, delay and phase, as SURVEY §8d C4
    does beyond PRN 36)."""
    from gnss_sim_receiver_amd import abi, engine, signals as S
    fs, f_if = 50e6, 7.161e6
    if full:
        prn_sets = (("GPS", (list(range(1, 33)) * 3)[:96], 0.001, 50000), ("GAL", (list(range(1, 37)) * 3)[:96], 0.004, 200000),
                    ("BDS", (list(range(6, 59)) * 2)[:64], 0.001, 50000))
    else:
        prn_sets = (("GPS", range(1, 13), 0.001, 50000), ("GAL", [1, 2, 3, 4, 5, 7, 8, 9, 11, 12, 13, 15], 0.004, 200000),
                    ("BDS", range(6, 14), 0.001, 50000))
    rng = np.random.default_rng(0x6E550005)
    sky = {}
    for system, prns, _, _ in prn_sets:
        sats = []
        for p in prns:
            s = S.Satellite(prn=int(p), doppler_hz=float(rng.uniform(-4000, 4000)), code_delay_chips=float(rng.uniform(0, 1000)), cn0_dbhz=47.0,
                            system=system, carrier_phase_rad=float(rng.uniform(0, 6.28)), f_if_hz=-f_if if system == "BDS" else f_if)
            if system == "GPS":
                s.bits = GPS_NAV
            elif system == "GAL":
                s.secondary, s.bits = "0011100000001010110110010", "0110"
            else:
                s.secondary, s.bits = "00000100110101001110", "0111"  # the B1I NH code (Beidou_B1I.h:48)
            sats.append(s)
        sky[system] = sats
    first = int(T_START_S * fs)
    n = int(round((pre_s + seconds) * fs)) + 3 * 200000
    allsats = sky["GPS"] + sky["GAL"] + sky["BDS"]
    x = S.generate_if_device(fs, n, allsats, seed=0x6E550005, start=first, device=f"cuda:{device}")
    iq = torch.view_as_real(x).reshape(-1)
    raw = torch.clamp(torch.round(8.0 * iq), -127, 127).to(torch.int8)  # signals.to_ibyte on the device
    del x, iq
    torch.cuda.synchronize()
    ctxs, trks = {}, {}
    for system, prns, period, vl in prn_sets:
        cx = engine.Context(device)
        sysid = {"GPS": abi.SYS_GPS_L1CA, "GAL": abi.SYS_GAL_E1, "BDS": abi.SYS_BDS_B1I}[system]
        conf = abi.TrkConf.defaults(sysid, fs, vl, rotator=rot)
        conf.if_hz = -f_if if system == "BDS" else f_if
        trk = engine.DllPllVemlTracking(cx, conf, len(sky[system]))
        for ch, s in enumerate(sky[system]):
            cx.set_code(2 * ch, s.code)
            if s.code_data is not None:
                cx.set_code(2 * ch + 1, s.code_data)
            trk.start(ch, 2 * ch, S.acq_delay_samples(s, fs, 0, first), s.doppler_hz, 0, first, data_code_id=2 * ch + 1, prn=s.prn)
        ctxs[system], trks[system] = cx, trk
    pre_n = int(round(pre_s * fs))
    for system, _, period, vl in prn_sets:  # pre-roll, all three engines together (records on: the buffers are sized here)
        trks[system].launch_ptr(raw.data_ptr(), abi.FMT_CI8, first, pre_n, int(pre_s / period) + 4, records=True)
    for system in trks:
        trks[system].collect()
    st_pre = {k: np.bincount(t.states(), minlength=5).tolist() for k, t in trks.items()}
    lo = first + pre_n - 2 * 200000
    span = int(round(seconds * fs)) + 4 * 200000
    ptr = raw.data_ptr() + (lo - first) * 2
    t0 = time.perf_counter()
    for system, _, period, vl in prn_sets:
        trks[system].launch_ptr(ptr, abi.FMT_CI8, lo, span, int(seconds / period) + 8, records=True)
    got = {system: trks[system].collect() for system in trks}
    dt = time.perf_counter() - t0
    epochs = {k: int(v[1]) for k, v in got.items()}
    recs = {k: int(np.count_nonzero(v[0][:v[1]]["flags"] & 8)) for k, v in got.items()}
    st_end = {k: np.bincount(t.states(), minlength=5).tolist() for k, t in trks.items()}
    for k in trks:
        trks[k].close()
        ctxs[k].close()
    del raw
    sig_s = min(epochs["GPS"] * 0.001, epochs["GAL"] * 0.004, epochs["BDS"] * 0.001)
    chan_samples = sum(recs[k] * vl for k, _, _, vl in prn_sets)
    counts = "96 GPS L1 C/A + 96 Galileo E1 (5 VEML + data prompt) + 64 BeiDou B1I (configs[4] whole, one GPU)" if full else \
        "C5 per-GPU share, 12 GPS L1 C/A + 12 Galileo E1 (5 VEML + data prompt) + 8 BeiDou B1I"
    return {"config": counts + ", closed loop, 50 Msps ibyte, "
                      "IF +-7.161 MHz in the tracking NCO, three engines on three streams launched together, rotator " + rotator_name(rot),
            "signal_s": round(sig_s, 3), "wall_ms": round(dt * 1e3, 3), "realtime_factor": round(sig_s / dt, 1),
            "if_msamples_per_s": round(sig_s * fs / dt / 1e6, 1), "channel_msamples_per_s": round(chan_samples / dt / 1e6, 1),
            "epochs": epochs, "epoch_records": recs, "states_before": st_pre, "states_after": st_end}


def streaming_broadcast(ctx, torch, rank, world, device, barrier, h, seconds=1.0, blocks=6):
    """N > 1: the IF file reaches the ranks block by block while they track — rank 0 holds the file,
    each D-second block is gnsship_comm_broadcast (RCCL) into every rank's resident copy on a second
    context's stream while the 12 channels of each rank track the block before it (double-buffered:
    block k+1 in flight during block k's closed loop).  Whole-job IF samples/s including the fan-out."""
    from gnss_sim_receiver_amd import engine, sharding
    cx = engine.Context(device)
    try:
        comm, transport = engine.Comm.from_process_group(cx), "gnsship_comm_broadcast (RCCL) on its own stream, double-buffered"
    except Exception as e:  # e.g. the gloo rehearsal on one device: torch.distributed, block by block, not overlapped
        comm, transport = None, f"torch.distributed broadcast per block, not overlapped ({type(e).__name__})"
    step_n = int(round(seconds * FS))
    t0_abs = h["first"] + int(round(PRE_ROLL_S * FS))
    lo0 = t0_abs - 2 * VL
    n = blocks * step_n + 4 * VL
    buf = torch.zeros(n, dtype=torch.complex64, device=f"cuda:{device}")
    if rank == 0:  # the file, on rank 0 only
        src = h["x"]
        off = lo0 - h["base"][1]
        m = min(n, src.numel() - off)
        buf[:m].copy_(src[off:off + m])
    torch.cuda.synchronize()
    chans = [(rank * N_CH + c) % N_SATS for c in range(N_CH)]
    rx = Receiver(ctx, "GPS", FS, VL, [h["sats"][i] for i in chans], N_CH, h["first"], h["rotator"], code_base=1200)
    # channels pre-rolled to t0_abs on the resident copy (untimed)
    rx.run(h["base"][0] + 2 * VL * 8, 0, h["first"], int(round(PRE_ROLL_S * FS)) + 2 * VL)
    edges = [0] + [2 * VL + (k + 1) * step_n for k in range(blocks)]
    edges[-1] = n
    def bcast(lo, hi):
        if comm is not None:
            comm.broadcast(buf.data_ptr() + lo * 8, (hi - lo) * 8, 0)
        else:
            sharding.broadcast_block(buf[lo:hi], src=0)

    barrier()
    t0 = time.perf_counter()
    bcast(0, edges[1])
    cx.sync()
    n_rec = 0
    for k in range(blocks):
        if k + 1 < blocks:  # block k+1 on the comm stream while block k is tracked
            bcast(edges[k + 1], edges[k + 2])
        rec, done = rx.run_records(buf.data_ptr(), 0, lo0, edges[k + 1], int(seconds * 1000) + 4)
        n_rec += int(np.count_nonzero(rec[:done]["flags"] & 8))
        cx.sync()
        torch.cuda.synchronize()
    barrier()
    wall = sharding.max_over_ranks(time.perf_counter() - t0)
    st = np.bincount(rx.trk.states(), minlength=5).tolist()
    rx.close()
    if comm is not None:
        comm.close()
    cx.close()
    del buf
    return {"config": f"GPS L1 C/A, 12 channels per rank, 4 Msps; {blocks} blocks of {seconds} s broadcast from rank 0 while the "
                      "previous block is tracked", "transport": transport,
            "n_ranks": world, "wall_s": round(wall, 4), "if_msamples_per_s": round(blocks * step_n / wall / 1e6, 1),
            "realtime_factor": round(blocks * seconds / wall, 1), "epoch_records_rank0": n_rec, "states_rank0": st,
            "block_mbytes": round(step_n * 8 / 1e6, 1)}


# ---------------------------------------------------------------------------------------------------
# multi-GPU fan-out: the C ABI's RCCL communicator (gnsship_comm_*) when it could be
# created, else torch.distributed — the transport used is reported in the JSON line.
COMM = {"comm": None, "transport": "single rank"}


def fan_out(ctx, torch, x, world):
    """Broadcast the IF tensor x (device, any dtype) from rank 0 to every rank."""
    torch.cuda.synchronize()
    if world > 1:
        c = COMM["comm"]
        if c is not None:
            c.broadcast(x.data_ptr(), x.numel() * x.element_size(), 0)
            ctx.sync()
        else:
            from gnss_sim_receiver_amd import sharding
            sharding.broadcast_block(x, src=0)
            torch.cuda.synchronize()


def allgather_rows(ctx, torch, rows, world):
    """All-gather equal-shaped float64 row blocks → rank-ordered stack."""
    if world == 1:
        return rows
    c = COMM["comm"]
    if c is not None:
        send = ctx.upload(np.ascontiguousarray(rows, np.float64))
        from gnss_sim_receiver_amd import engine
        recv = engine.DeviceBuffer(ctx, rows.nbytes * world)
        c.allgather(send.ptr, recv.ptr, rows.nbytes)
        ctx.sync()
        out = recv.download(np.empty((world,) + rows.shape, np.float64))
        send.free()
        recv.free()
        return out.reshape(-1, rows.shape[1])
    import torch.distributed as dist
    t = torch.from_numpy(np.ascontiguousarray(rows, np.float64))
    if dist.get_backend() == "nccl":
        t = t.cuda()
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t)
    return torch.cat(outs).cpu().numpy()


C3_CN0 = 50.0  # dB-Hz of the C3 bench signal's ten present PRNs


def acq_c3_sharded(ctx, torch, rank, world, device, barrier, reps=20):
    """C3 (32 PRN x 40 bins x 25000 at 25 Msps, BASELINE's signal: 10 present, seed 0x6E550003) with
    the (PRN x bin) cells sharded by PRN over the ranks: the 25000-sample block fanned out from rank 0,
    every rank searches all bins of its PRNs in one launch, per-PRN results all-gathered.  Whole-job
    sweeps/s = reps / max-over-ranks wall."""
    from gnss_sim_receiver_amd import codes as C, engine, sharding, signals as S
    fs, n = 25000000, 25000
    c3 = S.c3_sky(cn0=C3_CN0)
    x = torch.empty(n, dtype=torch.complex64, device=f"cuda:{device}")
    if rank == 0:
        x.copy_(torch.from_numpy(S.generate_if(fs, n, c3, seed=0x6E550003)))
    fan_out(ctx, torch, x, world)
    mine = sharding.shard_prns(32, world, rank)
    acq = engine.PcpsAcquisition(ctx, fs, n, 5000, 250, 0, True, max_prns=len(mine))
    for j, k in enumerate(mine):
        acq.set_local_code(C.gps_l1_ca_code_gen_complex_sampled(k + 1, fs), j)
    dev = engine.DeviceBuffer.wrap(ctx, x.data_ptr(), n * 8)
    for _ in range(3):
        acq.run(dev, n_prns=len(mine))
    barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        res, _ = acq.run(dev, n_prns=len(mine))
    barrier()
    wall = sharding.max_over_ranks(time.perf_counter() - t0)
    rows = sharding.pad_rows(sharding.acq_rows(res, mine), -(-32 // world))
    merged = sharding.merge_acq_rows(allgather_rows(ctx, torch, rows, world))
    acq.close()
    present = sorted(s.prn for s in c3)
    stat = {k + 1: float(merged[k][6]) for k in merged}
    dt = wall / reps
    cells = 32 * 40
    absent_max = max(v for p, v in stat.items() if p not in present)
    return {"config": f"C3: 32 PRN (10 present at {C3_CN0:g} dB-Hz, seed 0x6E550003) x 40 bins, fft 25000 (four-step), 25 Msps; "
                      f"cells sharded by PRN over {world} rank(s), per-PRN results all-gathered",
            "signal_note": "at 45 dB-Hz a 1 ms coherent search is marginal over 1280 cells (post-correlation SNR 31.6 against a "
                           "noise-only maximum near 14x the mean); the present PRNs are set 5 dB stronger so the line shows detection",
            "present_detected": sum(stat[p] > absent_max for p in present),
            "n_ranks": world, "prns_per_rank": len(mine), "sweep_ms": round(dt * 1e3, 3), "sweeps_per_s": round(1 / dt, 1),
            "cells_per_s": round(cells / dt, 0), "algorithmic_GBps": round(cells * 20 * n / dt / 1e9, 1),
            "prns_present": present, "prns_reported": len(merged),
            "present_min_test_statistic": round(min(stat[p] for p in present), 2),
            "absent_max_test_statistic": round(absent_max, 2),
            "fanout": COMM["transport"]}


def c1_receiver(torch, device, seconds=15.0, cpu_seconds=1.0):
    """BASELINE configs[0] (C1): a 15-s 4 Msps gr_complex file with GPS PRN 7 (fD 1730 Hz, delay 1234
    samples) through the Channel role end to end — tools/gnsship_rx (include/gnsship_receiver.hpp:
    5 channels, 1 in acquisition, pfa 0.01, ±10 kHz / 250 Hz, pll 40 / dll 4 — conf/gnss-sdr_GPS_L1_
    gr_complex.conf) — timed as a process over the file; beside it the oracle restatement of the same
    receiver (oracle/receiver.py: numpy FFT acquisition, scalar-C tracking, one thread) on the first
    `cpu_seconds` of the same file."""
    import subprocess
    import tempfile
    from gnss_sim_receiver_amd import signals as S
    fs = 4000000
    sats = S.c1_sky()
    d = tempfile.mkdtemp(prefix="gnsship_c1_")
    path = os.path.join(d, "c1.dat")
    n = int(seconds * fs)
    x = S.generate_if_device(fs, n, sats, seed=0x6E550001, device=f"cuda:{device}")
    x.cpu().numpy().tofile(path)
    del x
    rx = os.path.join(ROOT, "tools", "gnsship_rx")
    t0 = time.perf_counter()
    out = subprocess.run([rx, "--file", path, "--fs", str(fs), "--channels", "5", "--in-acquisition", "1", "--events",
                          os.path.join(d, "ev.csv"), "--dump", os.path.join(d, "trk_ch_")], capture_output=True, text=True, timeout=600)
    wall = time.perf_counter() - t0
    if out.returncode != 0:
        raise RuntimeError(f"gnsship_rx failed: {out.stderr[-400:]}")
    summ = json.loads(out.stdout.strip().splitlines()[-1])
    ev = np.loadtxt(os.path.join(d, "ev.csv"), delimiter=",", skiprows=1, ndmin=2)
    pos = ev[ev[:, 2] == 1]
    res = {"config": f"C1 (configs[0]): GPS L1 C/A PRN 7, 4 Msps gr_complex file, {seconds:g} s (past the 10 s pull-in: bit sync, "
                     "state 4); 5 channels, 1 in acquisition, pfa 0.01, "
                     "dmax 10000 / step 250, pll 40 / dll 4 (conf/gnss-sdr_GPS_L1_gr_complex.conf) — tools/gnsship_rx end to end",
           "signal_s": summ["signal_s"], "process_wall_s": round(wall, 3), "receiver_wall_s": round(summ["wall_s"], 3),
           "init_s": round(summ["init_s"], 3), "file_read_s": round(summ["io_s"], 3),
           "realtime_factor": round(summ["signal_s"] / summ["wall_s"], 1),
           "acq_attempts": summ["acq_positive"] + summ["acq_negative"], "acq_positive": summ["acq_positive"],
           "prn7_acquired_at_s": round(float(pos[pos[:, 3] == 7][0, 0]) / fs, 4) if (pos[:, 3] == 7).any() else None,
           "prn7_doppler_hz": float(pos[pos[:, 3] == 7][0, 4]) if (pos[:, 3] == 7).any() else None,
           "channels": summ["channels"]}
    if cpu_seconds > 0:
        from oracle import receiver as R
        xs = np.fromfile(path, np.complex64, count=int(cpu_seconds * fs))
        t0 = time.perf_counter()
        orx = R.Receiver(R.ReceiverConf(channels=5, in_acquisition=1, rotator_avx=1, block_samples=fs // 10))
        orx.work(xs)
        dt = time.perf_counter() - t0
        res["cpu_baseline"] = {"kind": "port", "cores": 1, "sample": f"first {cpu_seconds} s of the same file",
                               "realtime_factor": round(cpu_seconds / dt, 2), "wall_s": round(dt, 3),
                               "note": "oracle/receiver.py: the same control logic, numpy (pocketfft) acquisition, scalar-C DLL/PLL"}
        res["gpu_vs_cpu"] = round(res["realtime_factor"] / res["cpu_baseline"]["realtime_factor"], 1)
    for f in os.listdir(d):
        os.remove(os.path.join(d, f))
    os.rmdir(d)
    return res


# ---------------------------------------------------------------------------------------------------
# CPU baseline: the oracle's closed loop, one thread per channel (ctypes releases the GIL)
def cpu_baseline(h, budget_s):
    """The oracle's closed loop on the host: 12 threads, one per channel of the workload, over a
    bounded sample of the same file.  Like the GPU leg, only steady-state epochs are timed: each
    thread first runs its channel through start_tracking and the pre-roll (bit synchronisation,
    state 4) untimed, snapshots the channel (the oracle's channel state is one plain C struct), then
    replays the next 500 epochs of the file from that snapshot again and again while the clock runs —
    no start_tracking, pull-in or state-2 epochs inside the timed region.  For the AVX variant two
    figures: the AVX restatement (oracle/avx_port.c — the arithmetic the reference's u_avx kernel runs
    on such a host; `value`) and the scalar restatement of the same loop (`scalar_port`)."""
    import ctypes
    from oracle import trk as T
    from gnss_sim_receiver_amd import signals
    import platform
    from oracle import oracle as O
    O.build()
    rot = h["rotator"]
    pre_ep, run_ep = int(round(PRE_ROLL_S * 1000)), 500
    # bounded sample of the same file: the pre-roll plus 500 steady-state epochs (host copy)
    n_s = (pre_ep + run_ep + 4) * VL
    x = h["x"][: n_s + 4 * VL].cpu().numpy()
    first, base_abs = h["first"], h["base"][1]
    threads = min(N_CH, len(os.sched_getaffinity(0)))  # one thread per channel of the workload
    k = T.conf("GPS", FS, VL, rotator_avx=1 if rot == 1 else 0)
    sats = h["sats"]
    states = [None] * threads

    def timed(simd_on, seconds):
        simd = O.set_simd(simd_on, fast=True)
        done_epochs = [0] * threads
        stop = [False]

        def worker(t):
            s = sats[t % N_CH]
            ch = T.Channel(k, s.code, signals.acq_delay_samples(s, FS, 0, first), s.doppler_hz, 0, first, fast=True)
            ch.run(x, base_abs, pre_ep)  # untimed: pull-in over, bit synchronisation
            states[t] = ch.state
            snap = ctypes.create_string_buffer(ch.buf.raw, len(ch.buf))
            while not stop[0]:
                ctypes.memmove(ch.buf, snap, len(ch.buf))  # back to the steady-state snapshot
                rec = ch.run(x, base_abs, run_ep)
                done_epochs[t] += len(rec)
                if len(rec) == 0:
                    break

        ths = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
        for th in ths:
            th.start()
        while any(st is None for st in states):  # the pre-rolls run before the clock starts
            time.sleep(0.01)
        t0 = time.perf_counter()
        time.sleep(seconds)
        stop[0] = True
        for th in ths:
            th.join()
        dt = time.perf_counter() - t0
        O.set_simd(False, fast=True)
        return simd, sum(done_epochs), dt

    simd, ep, dt = timed(rot == 1, budget_s * (0.6 if rot == 1 else 1.0))
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    chan_sps = ep * VL / dt
    out = {"value": round(chan_sps / N_CH / 1e6, 2), "unit": "Msamples/s",
           "cores": threads, "kind": "port",
           "sample": f"{ep} steady-state channel-epochs of the closed loop (oracle/trk_oracle.c, rotator {rot}, -O3 -march=native, "
                     f"correlator {'AVX restatement oracle/avx_port.c' if simd else 'scalar restatement'}): {threads} threads (one channel "
                     f"each) replay the {run_ep} epochs after the {pre_ep}-epoch untimed pre-roll from a state-{states[0]} snapshot for "
                     f"{dt:.1f} s (no start_tracking / pull-in / state-2 epochs timed); value = channel-samples/s ÷ {N_CH} channels, "
                     f"i.e. the IF rate at which this host would keep {N_CH} channels",
           "states_after_preroll": [int(v) for v in states],
           "channel_msamples_per_s": round(chan_sps / 1e6, 2),
           "channel_msamples_per_s_per_core": round(chan_sps / threads / 1e6, 1),
           "cpu_model": model, "machine": platform.machine(),
           "reference_avx_note": "SURVEY §6 measured the reference's own AVX correlator at 268 M channel-samples/s per core in "
                                 "the survey container; the AVX restatement runs the same 16-lane u_avx arithmetic"}
    if simd:
        states[:] = [None] * threads
        _, ep2, dt2 = timed(False, budget_s * 0.4)
        cs2 = ep2 * VL / dt2
        out["scalar_port"] = {"value": round(cs2 / N_CH / 1e6, 2), "unit": "Msamples/s", "cores": threads,
                              "channel_msamples_per_s_per_core": round(cs2 / threads / 1e6, 1),
                              "sample": f"{ep2} channel-epochs, same loop with the scalar correlator restatement, {dt2:.1f} s"}
    return out


def cpu_acq_c3(budget_s=8.0):
    """C3's all-sky PCPS sweep on the host (32 PRN x 40 bins, 25000-point FFTs at 25 Msps, the C3
    signal): pcps_acquisition's Doppler loop per PRN (wipe-off, FFT, ⊙ conj(code FFT), IFFT, |·|²,
    pcps_acquisition.cc:640-672) with scipy's single-precision pocketfft on all host threads (FFTW
    in the reference), then the oracle's CFAR statistic.  Whole sweeps/s over ~budget_s."""
    import scipy.fft as sf
    from gnss_sim_receiver_amd import codes as C, signals as S
    from oracle import oracle as O
    fs, n = 25000000, 25000
    workers = len(os.sched_getaffinity(0))
    x = S.generate_if(fs, n, S.c3_sky(cn0=C3_CN0), seed=0x6E550003).astype(np.complex64)
    nb = O.num_doppler_bins(5000, 250)
    w = O.doppler_wipeoff_grid(nb, n, 5000, 250, 0, fs)
    cf = [np.conj(sf.fft(C.gps_l1_ca_code_gen_complex_sampled(k + 1, fs)[:n].astype(np.complex64), workers=workers)) for k in range(32)]
    spc = int(np.ceil(np.float32(fs) / np.float32(1023000.0)))
    spcode = float(np.float32(np.float32(fs) * np.float32(0.001)))
    sweeps, t0 = 0, time.perf_counter()
    while True:
        stats = []
        for k in range(32):
            X = sf.fft(x[None, :] * w, axis=1, workers=workers)
            Y = sf.ifft(X * cf[k][None, :], axis=1, workers=workers) * n
            grid = (Y.real ** 2 + Y.imag ** 2).astype(np.float32)
            stats.append(O.acquisition_statistic(grid, 5000, 250, 0, True, spc, spcode).test_statistic)
        sweeps += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = (time.perf_counter() - t0) / sweeps
    return {"kind": "port", "cores": workers, "sweep_ms": round(dt * 1e3, 1), "sweeps_per_s": round(1 / dt, 2),
            "sample": f"{sweeps} whole C3 sweeps (32 PRN x {nb} bins x 25000-point complex64 FFT + IFFT) in {dt * sweeps:.1f} s, "
                      f"scipy.fft (pocketfft, single precision) on {workers} threads + oracle CFAR statistic"}


# ---------------------------------------------------------------------------------------------------
# round 1's open-loop legs (auxiliary)
N_RING = 3


def receiver_jobs(sats, rank: int, seconds: float):
    from gnss_sim_receiver_amd import signals
    n_ep = int(round(seconds * 1000))
    jobs, code_ids = [], {}
    for c in range(rank * N_CH, (rank + 1) * N_CH):
        s = sats[c % N_SATS]
        cid = code_ids.setdefault(s.prn, len(code_ids))
        jobs.append(signals.truth_jobs(s, FS, n_ep, VL, SHIFTS, cid))
    jobs = np.stack(jobs, axis=1).reshape(-1)
    codes = [None] * len(code_ids)
    for prn, cid in code_ids.items():
        codes[cid] = next(s.code for s in sats if s.prn == prn)
    return jobs, codes


def job_flags(rot):
    """Batch job flag for the rotator variant (GNSSHIP_JOB_ROTATOR_AVX when volk would dispatch AVX)."""
    from gnss_sim_receiver_amd import abi
    return abi.JOB_ROTATOR_AVX if rot == abi.ROTATOR_AVX else 0


def open_loop_correlator(ctx, torch, device, steps=20, rot=0):
    """Round 1's headline, kept as an auxiliary line: 12 000 channel-epochs of one second with
    synthetic-truth NCOs (no loop filters) as one batched launch, three receivers in a ring."""
    from gnss_sim_receiver_amd import abi, engine, signals
    sats = signals.random_sky(N_SATS, seed=SEED)
    n = FS + 2 * VL
    x = signals.generate_if_device(FS, n, sats, seed=SEED, device=f"cuda:{device}")
    torch.cuda.synchronize()
    batches = []
    for k in range(N_RING):
        jk, ck = receiver_jobs(sats, k, 1.0)
        jk["code_id"] += 32 * k
        jk["flags"] = job_flags(rot)
        for cid, c in enumerate(ck):
            ctx.set_code(32 * k + cid, c)
        b = engine.CorrelatorBatch(ctx, len(jk))
        b.set_jobs(jk, n)
        batches.append(b)
    for i in range(3):
        batches[i % 3].launch_pipelined(x.data_ptr(), abi.FMT_CF32, batches[(i + 1) % 3], batches[(i + 2) % 3])
    ctx.sync()
    ctx.event_record(4)
    t0 = time.perf_counter()
    for i in range(steps):
        batches[i % 3].launch_pipelined(x.data_ptr(), abi.FMT_CF32, batches[(i + 1) % 3], batches[(i + 2) % 3])
    ctx.event_record(5)
    ctx.sync()
    wall = time.perf_counter() - t0
    ms = ctx.event_elapsed_ms(4, 5) / steps
    # the same batches as separate stages (the pipelined launch runs the
    # replay lanes at raised priority beside the correlation, so its time depends on placement):
    # the replay alone, the correlation alone, and the plain launch (replay then correlation).
    split = {}
    for name, st in (("anchors_only", 1), ("correlate_only", 2), ("plain_launch", 3)):
        for i in range(3):
            batches[i % 3].launch_ptr(x.data_ptr(), abi.FMT_CF32, st)
        ctx.sync()
        ctx.event_record(4)
        for i in range(steps):
            batches[i % 3].launch_ptr(x.data_ptr(), abi.FMT_CF32, st)
        ctx.event_record(5)
        ctx.sync()
        split[name] = round(ctx.event_elapsed_ms(4, 5) / steps, 4)
    for b in batches:
        b.close()
    jobs = N_CH * 1000
    byts = jobs * (8 * VL + 3 * 8)
    return {"config": "12 GPS L1 C/A channels x 1000 epochs (1 s, 4 Msps), synthetic-truth NCOs, one batched launch per "
                      "receiver-second, 3 receivers in a ring (gnsship_batch_launch_pipelined2), rotator " + rotator_name(rot),
            "if_msamples_per_s": round(FS * steps / wall / 1e6, 1), "ms_per_launch": round(ms, 4),
            "split_ms_per_launch": split,
            "channel_msamples_per_s": round(jobs * VL / (ms * 1e-3) / 1e6, 1),
            "algorithmic_GBps": round(byts / (ms * 1e-3) / 1e9, 1)}


def acq_bench(ctx, fs, n, sig, label, present=None):
    """32-PRN all-sky PCPS sweep: 40 bins (±5 kHz / 250 Hz) × n-sample FFTs at fs."""
    from gnss_sim_receiver_amd import codes as C, engine
    acq = engine.PcpsAcquisition(ctx, fs, n, 5000, 250, 0, True, max_prns=32)
    for k in range(32):
        acq.set_local_code(C.gps_l1_ca_code_gen_complex_sampled(k + 1, fs), k)
    dev = ctx.upload(np.ascontiguousarray(sig[:n]))
    for _ in range(3):
        acq.run(dev, n_prns=32)
    reps = 20
    ctx.event_record(6)
    t0 = time.perf_counter()
    for _ in range(reps):
        res, _ = acq.run(dev, n_prns=32)
    dt = (time.perf_counter() - t0) / reps
    ctx.event_record(7)
    cells = 32 * acq.n_bins
    out = {"config": label, "sweep_ms": round(dt * 1e3, 3),
           "sweeps_per_s": round(1 / dt, 1), "cells_per_s": round(cells / dt, 0),
           "algorithmic_GBps": round(cells * 20 * n / dt / 1e9, 1)}
    if present is not None:
        stat = np.array([r.test_statistic for r in res])
        out["prns_present"] = sorted(present)
        out["present_min_test_statistic"] = round(float(min(stat[p - 1] for p in present)), 2)
        out["absent_max_test_statistic"] = round(float(max(stat[k] for k in range(32) if k + 1 not in present)), 2)
    acq.close()
    dev.free()
    return out


def acq_e1_bench(ctx, reps=20):
    from gnss_sim_receiver_amd import codes as C, engine, signals as S
    fs, n = 25000000, 100000
    sats = S.random_sky(6, seed=SEED + 7, system="GAL", prns=[2, 9, 13, 21, 26, 31])
    sig = S.generate_if(fs, n, sats, seed=SEED + 7)
    acq = engine.PcpsAcquisition(ctx, fs, n, 5000, 250, 0, False, max_prns=32, ms_per_code=4)
    for k in range(32):
        acq.set_local_code(C.galileo_e1_code_gen_complex_sampled("1B", False, k + 1, fs), k)
    dev = ctx.upload(np.ascontiguousarray(sig))
    for _ in range(3):
        acq.run(dev, n_prns=32)
    t0 = time.perf_counter()
    for _ in range(reps):
        res, _ = acq.run(dev, n_prns=32)
    dt = (time.perf_counter() - t0) / reps
    present = {s.prn for s in sats}
    stat = np.array([r.test_statistic for r in res])
    cells = 32 * acq.n_bins
    out = {"config": "Galileo E1: 32 PRN x 40 bins, fft 100000 (huge layout, 10 x 10000), 25 Msps, first-vs-second statistic",
           "sweep_ms": round(dt * 1e3, 3), "sweeps_per_s": round(1 / dt, 1), "cells_per_s": round(cells / dt, 0),
           "prns_present": sorted(present),
           "present_min_test_statistic": round(float(min(stat[p - 1] for p in present)), 2),
           "absent_max_test_statistic": round(float(max(stat[k] for k in range(32) if k + 1 not in present)), 2),
           "algorithmic_GBps": round(cells * 20 * n / dt / 1e9, 1)}
    acq.close()
    dev.free()
    return out


def e1_open_loop(ctx, seconds=0.2, reps=10, rot=0):
    from gnss_sim_receiver_amd import abi, engine, signals as S
    fs, vl, nch = 25e6, 100000, 8
    sats = S.random_sky(nch, seed=SEED + 4, system="GAL", prns=[1, 5, 12, 19, 24, 30, 33, 36])
    n_ep = int(round(seconds * 250))
    sig = S.generate_if(fs, vl * (n_ep + 2), sats, seed=SEED + 4)
    jobs = []
    for k, s in enumerate(sats):
        pj = S.truth_jobs(s, fs, n_ep, vl, [-1.0, -0.5, 0.0, 0.5, 1.0], 100 + 2 * k)
        dj = pj.copy()
        dj["code_id"] = 100 + 2 * k + 1
        dj["n_taps"] = 1
        dj["shifts_chips"] = 0.0
        jobs += [pj, dj]
        ctx.set_code(100 + 2 * k, s.code)
        ctx.set_code(100 + 2 * k + 1, s.code_data)
    jobs = np.concatenate(jobs)
    jobs["flags"] = job_flags(rot)
    dev = ctx.upload(sig)
    ring = []
    for _ in range(3):
        b = engine.CorrelatorBatch(ctx, len(jobs))
        b.set_jobs(jobs, len(sig))
        ring.append(b)
    for i in range(3):
        ring[i % 3].launch_pipelined(dev.ptr, abi.FMT_CF32, ring[(i + 1) % 3], ring[(i + 2) % 3])
    ctx.sync()
    ctx.event_record(4)
    for i in range(reps):
        ring[i % 3].launch_pipelined(dev.ptr, abi.FMT_CF32, ring[(i + 1) % 3], ring[(i + 2) % 3])
    ctx.event_record(5)
    ctx.sync()
    ms = ctx.event_elapsed_ms(4, 5) / reps
    for b in ring:
        b.close()
    dev.free()
    if_msps = n_ep * vl / (ms * 1e-3) / 1e6
    return {"config": "C4 per-GPU share, open loop (truth NCOs): Galileo E1, 8 ch, 25 Msps, N=100000, 5 pilot taps + 1 data tap, "
                      f"gr_complex, {seconds} s block, 3 batches in a ring, rotator " + rotator_name(rot),
            "ms_per_signal_second": round(ms / seconds, 4), "if_msamples_per_s": round(if_msps, 1),
            "realtime_factor": round(if_msps * 1e6 / fs, 1), "algorithmic_GBps": round(2 * nch * n_ep * vl * 8 / (ms * 1e-3) / 1e9, 1)}


def c5_open_loop(ctx, seconds=0.2, reps=6, rot=0):
    from gnss_sim_receiver_amd import abi, engine, signals as S
    fs, f_if = 50e6, 7.161e6
    sys_conf = (("GPS", 12, 50000, [-0.25, 0.0, 0.25], 1000), ("GAL", 12, 200000, [-1.0, -0.5, 0.0, 0.5, 1.0], 250),
                ("BDS", 8, 50000, [-0.25, 0.0, 0.25], 1000))
    receivers, present = [], []
    for k in range(N_RING):
        jobs = []
        cid = 600 + 100 * k
        for si, (system, nch, vl, shifts, rate) in enumerate(sys_conf):
            prns = [1 + ((k * nch + c) % (36 if system == "GAL" else 32)) for c in range(nch)]
            sats = S.random_sky(nch, seed=SEED + 50 + 10 * k + si, system=system, prns=prns)
            for s in sats:
                s.f_if_hz = -f_if if system == "BDS" else f_if
                n_ep = int(round(seconds * rate)) - 2
                jobs.append(S.truth_jobs(s, fs, n_ep, vl, shifts, cid))
                ctx.set_code(cid, s.code)
                if system == "GAL":
                    dj = jobs[-1].copy()
                    dj["code_id"], dj["n_taps"], dj["shifts_chips"] = cid + 1, 1, 0.0
                    jobs.append(dj)
                    ctx.set_code(cid + 1, s.code_data)
                    cid += 1
                cid += 1
            if k == 0:
                present += sats[:2]
        receivers.append(np.concatenate(jobs))
        receivers[-1]["flags"] = job_flags(rot)
    n = int(round(fs * seconds)) + 400000
    block = S.to_ibyte(S.generate_if(fs, n, present, seed=SEED + 5))
    dev = ctx.upload(block)
    batches = []
    for jk in receivers:
        b = engine.CorrelatorBatch(ctx, len(jk))
        b.set_jobs(jk, n)
        batches.append(b)
    for i in range(3):
        batches[i % 3].launch_pipelined(dev.ptr, abi.FMT_CI8, batches[(i + 1) % 3], batches[(i + 2) % 3])
    ctx.sync()
    ctx.event_record(4)
    for i in range(reps):
        batches[i % 3].launch_pipelined(dev.ptr, abi.FMT_CI8, batches[(i + 1) % 3], batches[(i + 2) % 3])
    ctx.event_record(5)
    ctx.sync()
    ms = ctx.event_elapsed_ms(4, 5) / reps
    chan_samples = int(np.sum(receivers[0]["n_samples"]))
    for b in batches:
        b.close()
    dev.free()
    span_s = seconds - 2 * 0.004
    rt = span_s / (ms * 1e-3)
    return {"config": "C5 per-GPU share, open loop (truth NCOs): 12 GPS L1 C/A + 12 Galileo E1 (5+1 taps) + 8 BeiDou B1I, "
                      f"50 Msps ibyte, {seconds} s block, 3 receivers in a ring, rotator " + rotator_name(rot),
            "ms_per_block": round(ms, 4), "realtime_factor": round(rt, 1),
            "if_msamples_per_s": round(fs * span_s / (ms * 1e-3) / 1e6, 1),
            "channel_msamples_per_s": round(chan_samples / (ms * 1e-3) / 1e6, 1),
            "algorithmic_GBps": round(chan_samples * 2 / (ms * 1e-3) / 1e9, 1)}


# ---------------------------------------------------------------------------------------------------
def guarded(fn, *a, **kw):
    """An auxiliary line: its failure is reported in its place, never loses the headline line."""
    try:
        return fn(*a, **kw)
    except Exception as e:  # noqa: BLE001 — reported in the JSON, and on stderr
        print(f"[bench] {getattr(fn, '__name__', fn)} failed: {type(e).__name__}: {e}", file=sys.stderr)
        return {"error": f"{type(e).__name__}: {e}"}


def main():
    args = parse()
    from gnss_sim_receiver_amd import engine, sharding
    import torch

    rank, world, local_rank = sharding.dist_env()
    if world != args.gpus and not (world == 1 and args.gpus == 1):
        if world == 1:
            raise SystemExit("--gpus N>1 must be launched with torch.distributed.run (one process per GPU)")
    device = local_rank
    if world > 1:
        import torch.distributed as dist
        # GNSSHIP_DIST_BACKEND=gloo rehearses the multi-rank flow on a one-GPU box (RCCL refuses two
        # ranks on one device); the production path is nccl (RCCL over xGMI).
        backend = os.environ.get("GNSSHIP_DIST_BACKEND", "nccl")
        device = local_rank % max(1, torch.cuda.device_count()) if backend != "nccl" else local_rank
        torch.cuda.set_device(device)
        dist.init_process_group(backend)
    ctx = engine.Context(device)
    if world > 1:
        try:
            COMM["comm"] = engine.Comm.from_process_group(ctx)
            COMM["transport"] = "gnsship_comm (RCCL, C ABI)"
        except Exception as e:  # reported, never silent: the data then travels over torch.distributed
            COMM["transport"] = f"torch.distributed ({type(e).__name__}: {e})"
            print(f"[bench] gnsship_comm unavailable, IF fan-out over torch.distributed: {e}", file=sys.stderr)

    def barrier():
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        ctx.sync()

    h = headline(ctx, torch, args, rank, world, device, barrier)
    wall = h["wall"]
    samples = args.steps * args.seconds * FS
    value = samples / wall / 1e6  # the file's samples per second of the whole job (every rank tracks the same file)
    k_ms = h["kernel_ms"]
    chan_epochs = N_CH * args.seconds * 1000
    bytes_launch = chan_epochs * (8 * VL + 8 * 3)          # s·N + 8·T_out per channel-epoch
    achieved = bytes_launch / (k_ms * 1e-3) / 1e9
    pmc = {}
    if os.path.exists(args.pmc):
        try:
            pmc = json.load(open(args.pmc))
        except Exception:
            pmc = {}
    valu = pmc.get("valu_insts_per_launch")
    traffic = pmc.get("hbm_bytes_per_launch")
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
            "kernel": ("trk_fast_kernel" if h["rotator"] == 1 else "trk_persist_kernel") + " (one launch per step)", "kernel_ms": round(k_ms, 4),
            "binding": "latency: per channel the epoch chain derive -> phasor replay (N/16 dependent complex products, AVX "
                       "variant) -> correlation tail -> reduction -> loop update; 12 channels occupy 12 of 256 CUs"}
    if valu:
        roof["valu"] = {"achieved": round(valu / (k_ms * 1e-3), 0), "peak": VALU_PEAK, "unit": "wave64 instr/s",
                        "frac": round(valu / (k_ms * 1e-3) / VALU_PEAK, 5), "source": os.path.relpath(args.pmc, ROOT)}
    result = {
        "metric": "IF Msamples/sec processed & tracked-channels sustained @1/2/4/8 GPU",
        "value": round(value, 1),
        "unit": "Msamples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (SURVEY §8d IF model, generated on the GPU, resident in HBM)",
        "config": {"workload": "GPS L1 C/A, 12 channels, 4 Msps gr_complex, closed-loop DLL/PLL steady-state tracking (configs[1])",
                   "channels_per_gpu": N_CH, "fs_sps": FS, "vector_length": VL, "taps": 3, "step_s": args.seconds,
                   "rotator": rotator_name(h["rotator"]), "tracking_states_before": np.bincount(h["states_pre"], minlength=5).tolist(),
                   "tracking_states_after": np.bincount(h["states_end"], minlength=5).tolist(),
                   "parallelism": f"channels sharded over {world} rank(s) (weak scaling); IF file RCCL-broadcast once, resident on every rank"},
        "realtime_factor": round(samples / FS / wall, 1),
        "us_per_epoch": round(wall / (args.steps * args.seconds * 1000) * 1e6, 2),
        "channels_tracked": world * N_CH,
        "channel_msamples_per_s": round(world * N_CH * samples / wall / 1e6, 1),
        "epoch_records_emitted": h["records"] * world,
        "roofline": roof,
    }
    result["config"]["fanout"] = COMM["transport"]
    if not args.no_aux:  # every rank: its PRN shard of the C3 sweep
        result["acquisition_c3"] = guarded(acq_c3_sharded, ctx, torch, rank, world, device, barrier)
        if rank == 0 and world == 1 and args.cpu_seconds > 0:
            c3 = result["acquisition_c3"]
            c3["cpu_baseline"] = guarded(cpu_acq_c3, min(8.0, args.cpu_seconds))
            if "sweeps_per_s" in c3 and "sweeps_per_s" in c3["cpu_baseline"]:
                c3["gpu_vs_cpu"] = round(c3["sweeps_per_s"] / c3["cpu_baseline"]["sweeps_per_s"], 1)
    if rank == 0 and not args.no_aux and not args.sharded_aux_only:
        counts = [12, 256, 1024, 4096, 16384, 65536, 98304, 131072, 163840]
        sw = sweep(ctx, h, h["rotator"], counts)
        rt = [r["channels"] for r in sw if r["realtime_factor"] >= 1.0]
        result["tracked_channels_sustained"] = max(rt) if rt else 0
        result["channel_sweep"] = sw
        result["tracked_channels_note"] = ("the largest channel count of the sweep measured at >= real time: 1 s of signal (1000 epochs) per "
                                           "point, every channel-epoch record copied to the host inside the timed run; each point names the "
                                           "kernel its timed launch ran (gnsship_trk_last_engine): with the AVX rotator, trk_fast_kernel's "
                                           "latency form up to one workgroup per CU, trk_lane_kernel above (one 16-lane row per channel, "
                                           "u_avx's own accumulation order, channels beyond the resident ones in successive workgroup generations)")
        # north_star's second rate: the same sweep on a 25 Msps file (N = 25000)
        f25 = guarded(sweep_file_25msps, torch, device)
        if "x" in f25:
            sw25 = guarded(sweep, ctx, f25, h["rotator"], [12, 1024, 4096, 8192, 16384, 24576, 28672, 32768], fs=f25["fs"], vl=f25["vl"])
            del f25
            torch.cuda.empty_cache()
            if isinstance(sw25, list):
                rt25 = [r["channels"] for r in sw25 if r["realtime_factor"] >= 1.0]
                result["tracked_channels_sustained_25msps"] = max(rt25) if rt25 else 0
                result["channel_sweep_25msps"] = sw25
            else:
                result["channel_sweep_25msps"] = sw25
        else:
            result["channel_sweep_25msps"] = f25
        if h["rotator"] != 0:
            g = Receiver(ctx, "GPS", FS, VL, [h["sats"][i] for i in range(N_CH)], N_CH, h["first"], 0, code_base=800)
            pre = int(round(PRE_ROLL_S * FS))
            g.run(h["base"][0] + 2 * VL * 8, 0, h["first"], pre + 2 * VL)
            gw, _, _ = closed_loop_steps(ctx, g, h["base"], h["first"] + pre, FS, args.seconds, min(args.steps, 5))
            g.close()
            result["closed_loop_generic_rotator"] = {"config": "as value, rotator " + rotator_name(0),
                                                      "if_msamples_per_s": round(min(args.steps, 5) * args.seconds * FS / gw / 1e6, 1),
                                                      "realtime_factor": round(min(args.steps, 5) * args.seconds / gw, 1)}
        result["closed_loop_gps_25msps"] = guarded(closed_loop_aux, ctx, torch, device, "GPS", 25e6, 25000, N_CH, 0.3, h["rotator"], SEED + 11)
        result["closed_loop_e1_25msps_c4_share"] = guarded(closed_loop_aux, ctx, torch, device, "GAL", 25e6, 100000, 8, 0.4, h["rotator"], SEED + 12)
        result["closed_loop_c5_share"] = guarded(closed_loop_c5_share, torch, device, h["rotator"])
        # the BASELINE channel counts of C4 and C5 whole, on this one GPU (the 8-GPU split divides them)
        result["closed_loop_c4_full_64_e1"] = guarded(closed_loop_aux, ctx, torch, device, "GAL", 25e6, 100000, 64, 0.4, h["rotator"], SEED + 14)
        result["closed_loop_c5_full_256"] = guarded(closed_loop_c5_share, torch, device, h["rotator"], full=True)
        if world == 1 and args.cpu_seconds > 0:
            result["cpu_baseline"] = guarded(cpu_baseline, h, args.cpu_seconds)
        result["open_loop_correlator"] = guarded(open_loop_correlator, ctx, torch, device, rot=h["rotator"])
        from gnss_sim_receiver_amd import signals as S
        sky = S.random_sky(N_SATS, seed=SEED)
        blk = S.generate_if(FS, VL, sky, seed=SEED)
        result["acquisition"] = guarded(acq_bench, ctx, FS, VL, blk, "32 PRN x 40 bins, fft 4000, 4 Msps")
        result["acquisition_e1"] = guarded(acq_e1_bench, ctx)
        if world == 1:
            result["c1_receiver"] = guarded(c1_receiver, torch, device, cpu_seconds=1.0 if args.cpu_seconds > 0 else 0.0)
        result["tracking_c4_e1_open_loop"] = guarded(e1_open_loop, ctx, rot=h["rotator"])
        result["tracking_c5_hybrid_open_loop"] = guarded(c5_open_loop, ctx, rot=h["rotator"])
    if world > 1 and not args.no_aux:
        result["streaming_broadcast"] = guarded(streaming_broadcast, ctx, torch, rank, world, device, barrier, h)
    del h
    # the line's key figures once more at its end (a reader of the line's tail sees them)
    def pick(key, field):
        v = result.get(key)
        return v.get(field) if isinstance(v, dict) else None
    result["summary"] = {"value_msps": result["value"], "us_per_epoch": result["us_per_epoch"], "roofline_frac": roof["frac"],
                         "cpu_baseline_msps": pick("cpu_baseline", "value"),
                         "tracked_channels_sustained": result.get("tracked_channels_sustained"),
                         "tracked_channels_sustained_25msps": result.get("tracked_channels_sustained_25msps"),
                         "gps_25msps_realtime": pick("closed_loop_gps_25msps", "realtime_factor"),
                         "e1_c4_share_realtime": pick("closed_loop_e1_25msps_c4_share", "realtime_factor"),
                         "c5_share_realtime": pick("closed_loop_c5_share", "realtime_factor"),
                         "generic_rotator_realtime": pick("closed_loop_generic_rotator", "realtime_factor"),
                         "c3_sweep_ms": pick("acquisition_c3", "sweep_ms"), "e1_sweep_ms": pick("acquisition_e1", "sweep_ms")}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if COMM["comm"] is not None:
        COMM["comm"].close()
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()

"""Thin Python handles over the C ABI, used by the tests, the bench and the smoke entry point.

The classes mirror the reference's engine objects one-to-one:

* :class:`MultiCorrelatorRealCodes` — ``Cpu_Multicorrelator_Real_Codes``
  (src/algorithms/tracking/libs/cpu_multicorrelator_real_codes.h:37-61): ``init``,
  ``set_local_code_and_taps``, ``set_input_output_vectors``,
  ``Carrier_wipeoff_multicorrelator_resampler``, ``free`` with the same argument meaning.
* :class:`CorrelatorBatch` — many (channel, epoch) correlations in one device launch.
* :class:`PcpsAcquisition` — ``pcps_acquisition::set_local_code`` / ``init`` / ``acquisition_core``.

All compute runs in ``libgnsship.so`` (HIP, gfx950).  These wrappers only move arguments.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import abi
from .abi import FMT_CF32, FMT_CI8, FMT_CI16, JOB_DTYPE, MAX_TAPS, check, fptr

_FMT_OF_DTYPE = {np.dtype(np.complex64): FMT_CF32, np.dtype(np.int16): FMT_CI16, np.dtype(np.int8): FMT_CI8}
_FMT_BYTES = {FMT_CF32: 8, FMT_CI16: 4, FMT_CI8: 2}


def sample_format(x: np.ndarray) -> int:
    """complex64 → CF32 (gr_complex); int16 [..., 2] interleaved → CI16; int8 interleaved → CI8."""
    try:
        return _FMT_OF_DTYPE[x.dtype]
    except KeyError as e:
        raise TypeError(f"unsupported IF sample dtype {x.dtype}") from e


def device_count() -> int:
    n = ctypes.c_int(0)
    rc = abi.load().gnsship_device_count(ctypes.byref(n))
    return n.value if rc == abi.OK else 0


class Context:
    """One HIP device, one stream, one code bank."""

    def __init__(self, device: int = 0):
        self.lib = abi.load()
        h = ctypes.c_void_p()
        check(self.lib.gnsship_ctx_create(device, ctypes.byref(h)), f"gnsship_ctx_create(device={device})")
        self.h = h
        self.device = device

    def close(self):
        if self.h:
            self.lib.gnsship_ctx_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sync(self):
        check(self.lib.gnsship_ctx_sync(self.h), "gnsship_ctx_sync", self.h)

    def stream(self) -> int:
        s = ctypes.c_void_p()
        check(self.lib.gnsship_ctx_stream(self.h, ctypes.byref(s)), "gnsship_ctx_stream", self.h)
        return s.value or 0

    def event_record(self, slot: int):
        check(self.lib.gnsship_ctx_event_record(self.h, slot), "gnsship_ctx_event_record", self.h)

    def event_elapsed_ms(self, a: int, b: int) -> float:
        ms = ctypes.c_float()
        check(self.lib.gnsship_ctx_event_elapsed_ms(self.h, a, b, ctypes.byref(ms)), "gnsship_ctx_event_elapsed_ms", self.h)
        return ms.value

    def set_code(self, code_id: int, code: np.ndarray):
        code = np.ascontiguousarray(code, np.float32)
        check(self.lib.gnsship_code_set(self.h, code_id, fptr(code), len(code)), "gnsship_code_set", self.h)

    def upload(self, host: np.ndarray) -> "DeviceBuffer":
        buf = DeviceBuffer(self, host.nbytes)
        buf.upload(host)
        return buf


class DeviceBuffer:
    """An HBM allocation owned by a context (the IF sample buffer lives in one)."""

    def __init__(self, ctx: Context, nbytes: int):
        self.ctx = ctx
        p = ctypes.c_void_p()
        check(ctx.lib.gnsship_dev_alloc(ctx.h, nbytes, ctypes.byref(p)), f"gnsship_dev_alloc({nbytes})", ctx.h)
        self.ptr = p.value
        self.nbytes = nbytes
        self.owned = True

    @classmethod
    def wrap(cls, ctx: Context, ptr: int, nbytes: int) -> "DeviceBuffer":
        """A non-owning view of device memory allocated elsewhere (e.g. a torch tensor's storage)."""
        b = cls.__new__(cls)
        b.ctx, b.ptr, b.nbytes, b.owned = ctx, ptr, nbytes, False
        return b

    def upload(self, host: np.ndarray, offset: int = 0):
        host = np.ascontiguousarray(host)
        assert offset + host.nbytes <= self.nbytes
        check(self.ctx.lib.gnsship_dev_upload(self.ctx.h, self.ptr + offset, host.ctypes.data, host.nbytes), "gnsship_dev_upload",
              self.ctx.h)

    def download(self, out: np.ndarray, offset: int = 0):
        assert offset + out.nbytes <= self.nbytes and out.flags.c_contiguous
        check(self.ctx.lib.gnsship_dev_download(self.ctx.h, out.ctypes.data, self.ptr + offset, out.nbytes), "gnsship_dev_download",
              self.ctx.h)
        return out

    def free(self):
        if self.ptr and self.owned:
            self.ctx.lib.gnsship_dev_free(self.ctx.h, self.ptr)
        self.ptr = None

    def __del__(self):
        try:
            if self.ptr and self.ctx.h:
                self.free()
        except Exception:
            pass


def comm_unique_id() -> bytes:
    """A fresh RCCL unique id (rank 0 makes it; the launcher's store carries it to the others)."""
    buf = ctypes.create_string_buffer(abi.COMM_ID_BYTES)
    check(abi.load().gnsship_comm_unique_id(buf), "gnsship_comm_unique_id")
    return buf.raw


class Comm:
    """gnsship_comm: one RCCL communicator per context, collectives on the context stream — the
    multi-GPU form of the flowgraph's conditioner → channels fan-out (gnss_flowgraph.cc:1127-1136)."""

    def __init__(self, ctx: Context, n_ranks: int, rank: int, uid: bytes):
        if len(uid) != abi.COMM_ID_BYTES:
            raise ValueError("RCCL unique id must be 128 bytes")
        self.ctx = ctx
        self.rank, self.n_ranks = rank, n_ranks
        h = ctypes.c_void_p()
        idbuf = ctypes.create_string_buffer(uid, abi.COMM_ID_BYTES)
        check(ctx.lib.gnsship_comm_create(ctx.h, n_ranks, rank, idbuf, ctypes.byref(h)), "gnsship_comm_create", ctx.h)
        self.h = h

    @classmethod
    def from_process_group(cls, ctx: Context):
        """Build the communicator over the ranks of the initialised torch.distributed group: rank 0's
        id travels through the group (any backend), then every rank joins."""
        import torch.distributed as dist
        rank, world = dist.get_rank(), dist.get_world_size()
        obj = [comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        return cls(ctx, world, rank, obj[0])

    def broadcast(self, dev_ptr: int, nbytes: int, root: int = 0):
        check(self.ctx.lib.gnsship_comm_broadcast(self.h, dev_ptr, nbytes, root), "gnsship_comm_broadcast", self.ctx.h)

    def allgather(self, dev_send: int, dev_recv: int, bytes_per_rank: int):
        check(self.ctx.lib.gnsship_comm_allgather(self.h, dev_send, dev_recv, bytes_per_rank), "gnsship_comm_allgather", self.ctx.h)

    def max_f64(self, values) -> np.ndarray:
        """Max over ranks of a few doubles (host in, host out; through a device buffer)."""
        v = np.ascontiguousarray(values, np.float64).reshape(-1)
        buf = self.ctx.upload(v)
        check(self.ctx.lib.gnsship_comm_allreduce_max_f64(self.h, buf.ptr, v.size), "gnsship_comm_allreduce_max_f64", self.ctx.h)
        self.ctx.sync()
        out = buf.download(np.empty_like(v))
        buf.free()
        return out

    def close(self):
        if self.h:
            self.ctx.lib.gnsship_comm_destroy(self.h)
            self.h = None


class MultiCorrelatorRealCodes:
    """Mirror of Cpu_Multicorrelator_Real_Codes (cpu_multicorrelator_real_codes.h:37-61).  rotator: the
    volk_gnsssdr rotator variant its Carrier_wipeoff_multicorrelator_resampler runs (abi.ROTATOR_*;
    default AUTO = what the reference's dispatcher picks on this host)."""

    def __init__(self, ctx: Context, rotator: int = abi.ROTATOR_AUTO):
        self.ctx = ctx
        self.rotator = rotator
        self.h = None
        self.n_correlators = 0
        self._out = None
        self._sig = None

    def init(self, max_signal_length_samples: int, n_correlators: int) -> bool:
        h = ctypes.c_void_p()
        check(self.ctx.lib.gnsship_corr_create(self.ctx.h, max_signal_length_samples, n_correlators, ctypes.byref(h)),
              "gnsship_corr_create", self.ctx.h)
        self.h = h
        self.n_correlators = n_correlators
        check(self.ctx.lib.gnsship_corr_set_rotator(self.h, self.rotator), "gnsship_corr_set_rotator", self.ctx.h)
        return True

    def set_high_dynamics_resampler(self, use: bool):
        check(self.ctx.lib.gnsship_corr_set_high_dynamics_resampler(self.h, int(use)), "set_high_dynamics_resampler", self.ctx.h)

    def set_local_code_and_taps(self, code_length_chips: int, local_code_in: np.ndarray, shifts_chips: np.ndarray) -> bool:
        code = np.ascontiguousarray(local_code_in[:code_length_chips], np.float32)
        shifts = np.ascontiguousarray(shifts_chips, np.float32)
        if len(shifts) < self.n_correlators:
            raise ValueError("need one shift per correlator")
        check(self.ctx.lib.gnsship_corr_set_local_code_and_taps(self.h, code_length_chips, fptr(code), fptr(shifts)),
              "gnsship_corr_set_local_code_and_taps", self.ctx.h)
        return True

    def set_input_output_vectors(self, corr_out: np.ndarray, sig_in: np.ndarray) -> bool:
        self._out = corr_out
        self._sig = sig_in
        return True

    def Carrier_wipeoff_multicorrelator_resampler(self, rem_carrier_phase_in_rad, phase_step_rad, phase_rate_step_rad,
                                                  rem_code_phase_chips, code_phase_step_chips, code_phase_rate_step_chips,
                                                  signal_length_samples) -> bool:
        sig = np.ascontiguousarray(self._sig)
        fmt = sample_format(sig)
        tmp = np.zeros(2 * self.n_correlators, np.float32)
        check(self.ctx.lib.gnsship_corr_run(self.h, sig.ctypes.data, fmt, 0, rem_carrier_phase_in_rad, phase_step_rad,
                                            phase_rate_step_rad, rem_code_phase_chips, code_phase_step_chips,
                                            code_phase_rate_step_chips, signal_length_samples, fptr(tmp)),
              "gnsship_corr_run", self.ctx.h)
        self._out[: self.n_correlators] = tmp.view(np.complex64)
        return True

    def free(self) -> bool:
        if self.h:
            self.ctx.lib.gnsship_corr_destroy(self.h)
            self.h = None
        return True

    def __del__(self):
        try:
            if self.h and self.ctx.h:
                self.free()
        except Exception:
            pass


class CorrelatorBatch:
    """Batched multicorrelator: every row of a JOB_DTYPE array is one channel-epoch."""

    def __init__(self, ctx: Context, max_jobs: int):
        self.ctx = ctx
        h = ctypes.c_void_p()
        check(ctx.lib.gnsship_batch_create(ctx.h, max_jobs, ctypes.byref(h)), "gnsship_batch_create", ctx.h)
        self.h = h
        self.n_jobs = 0

    def set_jobs(self, jobs: np.ndarray, n_buffer_samples: int):
        jobs = np.ascontiguousarray(jobs, JOB_DTYPE)
        check(self.ctx.lib.gnsship_batch_set_jobs(self.h, jobs.ctypes.data, len(jobs), n_buffer_samples), "gnsship_batch_set_jobs",
              self.ctx.h)
        self.n_jobs = len(jobs)

    def launch(self, samples: DeviceBuffer, fmt: int = FMT_CF32):
        check(self.ctx.lib.gnsship_batch_launch(self.h, samples.ptr, fmt), "gnsship_batch_launch", self.ctx.h)

    def launch_ptr(self, dev_ptr: int, fmt: int = FMT_CF32, stages: int = 3):
        check(self.ctx.lib.gnsship_batch_launch_stages(self.h, dev_ptr, fmt, stages), "gnsship_batch_launch_stages", self.ctx.h)

    def launch_pipelined(self, dev_ptr: int, fmt: int = FMT_CF32, next_batch: "CorrelatorBatch" = None,
                         next2: "CorrelatorBatch" = None):
        """Correlate this batch and, in the same launch, replay anchors of the batches after it
        (gnsship_batch_launch_pipelined2): all of `next_batch`'s remaining replay and the first half
        of `next2`'s.  Pairs alternate A, B, A, ...; rings of three A, B, C, A, ... (with next2)
        carry half a replay chain per batch per launch."""
        nh = next_batch.h if next_batch is not None else None
        n2 = next2.h if next2 is not None else None
        check(self.ctx.lib.gnsship_batch_launch_pipelined2(self.h, dev_ptr, fmt, nh, n2), "gnsship_batch_launch_pipelined2", self.ctx.h)

    def results(self) -> np.ndarray:
        out = np.zeros((self.n_jobs, 2 * MAX_TAPS), np.float32)
        check(self.ctx.lib.gnsship_batch_results(self.h, fptr(out)), "gnsship_batch_results", self.ctx.h)
        return out.view(np.complex64)

    def close(self):
        if self.h:
            self.ctx.lib.gnsship_batch_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            if self.h and self.ctx.h:
                self.close()
        except Exception:
            pass


def correlate_host(ctx: Context, samples: np.ndarray, jobs: np.ndarray, codes: list) -> np.ndarray:
    """Upload samples + codes, run one batch, return complex64[n_jobs, MAX_TAPS]."""
    fmt = sample_format(samples)
    for i, c in enumerate(codes):
        ctx.set_code(i, c)
    buf = ctx.upload(samples)
    n_samples = samples.nbytes // _FMT_BYTES[fmt]
    b = CorrelatorBatch(ctx, max(1, len(jobs)))
    try:
        b.set_jobs(jobs, n_samples)
        b.launch(buf, fmt)
        return b.results()
    finally:
        b.close()
        buf.free()


class PcpsAcquisition:
    """pcps_acquisition (pcps_acquisition.cc) over up to ``max_prns`` local codes at once."""

    def __init__(self, ctx: Context, fs_in: int, fft_size: int, doppler_max: int, doppler_step: int, doppler_center: int = 0,
                 use_cfar: bool = True, samples_per_chip: int = None, samples_per_code: float = None, max_prns: int = 1,
                 max_dwells: int = 1, chip_rate: float = 1023000.0, ms_per_code: int = 1, consumed_samples: int = 0,
                 bit_transition_flag: bool = False, resampler_ratio: float = 1.0, resampler_latency_samples: int = 0):
        self.ctx = ctx
        conf = abi.AcqConf()
        conf.fs_in = fs_in
        conf.fft_size = fft_size
        conf.doppler_max = doppler_max
        conf.doppler_step = doppler_step
        conf.doppler_center = doppler_center
        conf.max_dwells = max_dwells
        conf.use_cfar = int(use_cfar)
        # Acq_Conf::SetDerivedParams (acq_conf.cc:113-118), float arithmetic as in the reference
        spms = np.float32(np.float32(fs_in) * np.float32(0.001))
        conf.samples_per_chip = int(np.ceil(np.float32(fs_in) / np.float32(chip_rate))) if samples_per_chip is None else samples_per_chip
        conf.samples_per_code = float(np.float32(spms * np.float32(ms_per_code))) if samples_per_code is None else samples_per_code
        conf.max_prns = max_prns
        conf.consumed_samples = consumed_samples
        conf.bit_transition_flag = int(bit_transition_flag)
        conf.resampler_ratio = resampler_ratio
        conf.resampler_latency_samples = resampler_latency_samples
        self.conf = conf
        self.consumed = consumed_samples or fft_size
        self.code_len = fft_size // 2 if bit_transition_flag else self.consumed  # samples set_local_code reads
        self.row_len = fft_size // 2 if bit_transition_flag else fft_size       # grid row length
        h = ctypes.c_void_p()
        check(ctx.lib.gnsship_acq_create(ctx.h, ctypes.byref(conf), ctypes.byref(h)), "gnsship_acq_create", ctx.h)
        self.h = h
        nb = ctypes.c_int()
        check(ctx.lib.gnsship_acq_num_bins(self.h, ctypes.byref(nb)), "gnsship_acq_num_bins", ctx.h)
        self.n_bins = nb.value

    def set_grid(self, doppler_max: int, doppler_step: int, doppler_center: int = 0):
        check(self.ctx.lib.gnsship_acq_set_grid(self.h, doppler_max, doppler_step, doppler_center), "gnsship_acq_set_grid", self.ctx.h)
        nb = ctypes.c_int()
        check(self.ctx.lib.gnsship_acq_num_bins(self.h, ctypes.byref(nb)), "gnsship_acq_num_bins", self.ctx.h)
        self.n_bins = nb.value

    def set_grid_step2(self, doppler_center_step_two: float, doppler_step2: float, num_doppler_bins_step2: int,
                       step_one_input_power: float):
        """update_grid_doppler_wipeoffs_step2 (pcps_acquisition.cc:305-312): make_2_steps' narrow grid."""
        check(self.ctx.lib.gnsship_acq_set_grid_step2(self.h, doppler_center_step_two, doppler_step2, num_doppler_bins_step2,
                                                      step_one_input_power), "gnsship_acq_set_grid_step2", self.ctx.h)
        nb = ctypes.c_int()
        check(self.ctx.lib.gnsship_acq_num_bins(self.h, ctypes.byref(nb)), "gnsship_acq_num_bins", self.ctx.h)
        self.n_bins = nb.value

    def set_local_code(self, code: np.ndarray, prn_slot: int = 0):
        code = np.ascontiguousarray(code, np.complex64)
        if len(code) < self.code_len:
            raise ValueError(f"local code must have at least {self.code_len} samples")
        code = np.ascontiguousarray(code[: self.code_len])
        check(self.ctx.lib.gnsship_acq_set_local_code(self.h, prn_slot, fptr(code.view(np.float32))), "gnsship_acq_set_local_code",
              self.ctx.h)

    def run(self, sig, n_prns: int = 1, want_grid: bool = False, fmt: int = None):
        """sig: host ndarray (CF32/CI16/CI8) or DeviceBuffer (then pass fmt)."""
        res = (abi.AcqResult * n_prns)()
        grid = np.zeros((n_prns, self.n_bins, self.row_len), np.float32) if want_grid else None
        if isinstance(sig, DeviceBuffer):
            ptr, on_dev, f = sig.ptr, 1, FMT_CF32 if fmt is None else fmt
        else:
            sig = np.ascontiguousarray(sig)
            ptr, on_dev, f = sig.ctypes.data, 0, sample_format(sig)
        check(self.ctx.lib.gnsship_acq_run(self.h, ptr, f, on_dev, n_prns, res, fptr(grid) if want_grid else None),
              "gnsship_acq_run", self.ctx.h)
        return list(res), grid

    def close(self):
        if self.h:
            self.ctx.lib.gnsship_acq_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            if self.h and self.ctx.h:
                self.close()
        except Exception:
            pass


def firdes_low_pass(lib, gain: float, fs: float, cutoff: float, transition: float) -> np.ndarray:
    """gr::filter::firdes::low_pass (Hamming) as the library restates it."""
    n = ctypes.c_int()
    rc = lib.gnsship_firdes_low_pass(gain, fs, cutoff, transition, None, 0, ctypes.byref(n))
    if rc != abi.OK:
        raise abi.GnssHipError(rc, "gnsship_firdes_low_pass: bad arguments")
    taps = np.zeros(n.value, np.float32)
    check(lib.gnsship_firdes_low_pass(gain, fs, cutoff, transition, fptr(taps), len(taps), ctypes.byref(n)), "gnsship_firdes_low_pass")
    return taps


def acq_resampler_design(lib, fs_in: int, opt_acq_fs: float):
    """gnss_flowgraph.cc:1070-1113: (decimation, taps); decimation 1 and no taps when not needed."""
    d, n = ctypes.c_int(), ctypes.c_int()
    check(lib.gnsship_acq_resampler_design(fs_in, opt_acq_fs, ctypes.byref(d), None, 0, ctypes.byref(n)), "gnsship_acq_resampler_design")
    taps = np.zeros(n.value, np.float32)
    if n.value:
        check(lib.gnsship_acq_resampler_design(fs_in, opt_acq_fs, ctypes.byref(d), fptr(taps), len(taps), ctypes.byref(n)),
              "gnsship_acq_resampler_design")
    return d.value, taps


class AcqResampler:
    """The acquisition resampler FIR (fir_filter_ccf(decimation, taps)) over a sample stream."""

    def __init__(self, ctx: Context, taps: np.ndarray, decimation: int, max_in_samples: int):
        self.ctx = ctx
        self.taps = np.ascontiguousarray(taps, np.float32)
        self.decimation = decimation
        h = ctypes.c_void_p()
        check(ctx.lib.gnsship_acq_resampler_create(ctx.h, fptr(self.taps), len(self.taps), decimation, max_in_samples, ctypes.byref(h)),
              "gnsship_acq_resampler_create", ctx.h)
        self.h = h

    @property
    def latency(self) -> int:
        return (len(self.taps) - 1) // 2

    def run(self, x, fmt: int = None, on_device: bool = False, n_in: int = None):
        """Filter a host array (or a device pointer with on_device=True and n_in): returns the
        decimated complex64 samples (host arrays) or (device pointer, n_out)."""
        dev = ctypes.c_void_p()
        n_out = ctypes.c_int64()
        if on_device:
            check(self.ctx.lib.gnsship_acq_resampler_run(self.h, x, fmt, 1, n_in, None, ctypes.byref(dev), ctypes.byref(n_out)),
                  "gnsship_acq_resampler_run", self.ctx.h)
            return dev.value, n_out.value
        fmt = sample_format(x) if fmt is None else fmt
        n = len(x) if x.dtype == np.complex64 else len(x) // 2
        out = np.zeros(n // self.decimation, np.complex64)
        check(self.ctx.lib.gnsship_acq_resampler_run(self.h, x.ctypes.data, fmt, 0, n, fptr(out.view(np.float32)), ctypes.byref(dev),
                                                      ctypes.byref(n_out)), "gnsship_acq_resampler_run", self.ctx.h)
        return out

    def reset(self):
        check(self.ctx.lib.gnsship_acq_resampler_reset(self.h), "gnsship_acq_resampler_reset", self.ctx.h)

    def close(self):
        if self.h:
            self.ctx.lib.gnsship_acq_resampler_destroy(self.h)
            self.h = None


class DllPllVemlTracking:
    """dll_pll_veml_tracking (dll_pll_veml_tracking.cc) for up to ``max_channels`` channels, the
    per-epoch loop resident on the device: ``start_tracking`` → :meth:`start`, ``general_work``
    over an IF buffer → :meth:`run` (one record per channel-epoch, TRK_EPOCH_DTYPE)."""

    def __init__(self, ctx: Context, conf: "abi.TrkConf", max_channels: int):
        self.ctx = ctx
        self.conf = conf
        self.max_channels = max_channels
        h = ctypes.c_void_p()
        check(ctx.lib.gnsship_trk_create(ctx.h, ctypes.byref(conf), max_channels, ctypes.byref(h)), "gnsship_trk_create", ctx.h)
        self.h = h

    def start(self, channel: int, code_id: int, acq_delay_samples: float, acq_doppler_hz: float, acq_samplestamp: int,
              first_sample: int, data_code_id: int = -1, prn: int = 0):
        a = abi.TrkStartArgs(code_id=code_id, data_code_id=data_code_id, acq_delay_samples=acq_delay_samples,
                             acq_doppler_hz=acq_doppler_hz, acq_samplestamp_samples=acq_samplestamp, first_sample=first_sample,
                             prn=prn)
        check(self.ctx.lib.gnsship_trk_start(self.h, channel, ctypes.byref(a)), "gnsship_trk_start", self.ctx.h)

    def start_many(self, starts):
        """gnsship_trk_start_many: `starts` = [(channel, code_id, acq_delay_samples, acq_doppler_hz,
        acq_samplestamp, first_sample[, data_code_id[, prn]]), ...] in one transaction."""
        n = len(starts)
        if n == 0:
            return
        chans = (ctypes.c_int32 * n)()
        args = (abi.TrkStartArgs * n)()
        for i, st in enumerate(starts):
            ch, code_id, delay, dop, stamp, first = st[:6]
            data_code_id = st[6] if len(st) > 6 else -1
            prn = st[7] if len(st) > 7 else 0
            chans[i] = ch
            args[i] = abi.TrkStartArgs(code_id=code_id, data_code_id=data_code_id, acq_delay_samples=delay, acq_doppler_hz=dop,
                                       acq_samplestamp_samples=stamp, first_sample=first, prn=prn)
        check(self.ctx.lib.gnsship_trk_start_many(self.h, n, chans, args), "gnsship_trk_start_many", self.ctx.h)

    def stop(self, channel: int):
        check(self.ctx.lib.gnsship_trk_stop(self.h, channel), "gnsship_trk_stop", self.ctx.h)

    def telemetry_event(self, channel: int, tlm_event: int = 1):
        """msg_handler_telemetry_to_trk (dll_pll_veml_tracking.cc:617-640): event 1 = telemetry fault."""
        check(self.ctx.lib.gnsship_trk_telemetry_event(self.h, channel, tlm_event), "gnsship_trk_telemetry_event", self.ctx.h)

    def channel_state(self, channel: int):
        st, nx = ctypes.c_int(), ctypes.c_uint64()
        check(self.ctx.lib.gnsship_trk_channel_state(self.h, channel, ctypes.byref(st), ctypes.byref(nx)), "gnsship_trk_channel_state",
              self.ctx.h)
        return st.value, nx.value

    def run(self, sig, buffer_first_sample: int, max_rounds: int, fmt: int = None, n_buffer_samples: int = None,
            records: bool = True, dump: bool = False):
        """sig: host ndarray or DeviceBuffer (pass fmt and n_buffer_samples).  Returns (records
        [max_rounds, max_channels] or None, rounds_done), plus the log_data dump records
        [max_rounds, max_channels] (TRK_DUMP_DTYPE; valid where the record has flags & 16) when dump."""
        out = np.zeros((max_rounds, self.max_channels), abi.TRK_EPOCH_DTYPE) if records else None
        dmp = np.zeros((max_rounds, self.max_channels), abi.TRK_DUMP_DTYPE) if dump else None
        if dump and not records:
            raise ValueError("dump records need the epoch records (flags & 16 marks them)")
        if isinstance(sig, DeviceBuffer):
            ptr, on_dev, f = sig.ptr, 1, FMT_CF32 if fmt is None else fmt
            n = n_buffer_samples if n_buffer_samples is not None else sig.nbytes // _FMT_BYTES[f]
        else:
            sig = np.ascontiguousarray(sig)
            ptr, on_dev, f = sig.ctypes.data, 0, sample_format(sig)
            n = sig.nbytes // _FMT_BYTES[f]
        done = ctypes.c_int()
        check(self.ctx.lib.gnsship_trk_run_dump(self.h, ptr, f, on_dev, buffer_first_sample, n, max_rounds,
                                                out.ctypes.data if records else None, dmp.ctypes.data if dump else None,
                                                ctypes.byref(done)), "gnsship_trk_run_dump", self.ctx.h)
        return (out, done.value, dmp) if dump else (out, done.value)

    def run_ptr(self, dev_ptr: int, fmt: int, buffer_first_sample: int, n_buffer_samples: int, max_rounds: int) -> int:
        """general_work over a device IF buffer given as a raw pointer (e.g. a torch tensor's data_ptr,
        or an offset into one), no records: returns the rounds run."""
        done = ctypes.c_int()
        check(self.ctx.lib.gnsship_trk_run_dump(self.h, ctypes.c_void_p(dev_ptr), fmt, 1, buffer_first_sample, n_buffer_samples, max_rounds,
                                                None, None, ctypes.byref(done)), "gnsship_trk_run_dump", self.ctx.h)
        return done.value

    def launch_ptr(self, dev_ptr: int, fmt: int, buffer_first_sample: int, n_buffer_samples: int, max_rounds: int,
                   records: bool = False, dump: bool = False):
        """gnsship_trk_launch: enqueue the run on this engine's context stream and return at once
        (engines on other contexts of the same device run concurrently); :meth:`collect` waits."""
        check(self.ctx.lib.gnsship_trk_launch(self.h, ctypes.c_void_p(dev_ptr), fmt, buffer_first_sample, n_buffer_samples, max_rounds,
                                              int(records), int(dump)), "gnsship_trk_launch", self.ctx.h)
        self._pending = (max_rounds, records, dump)

    def collect(self, out: np.ndarray = None):
        """gnsship_trk_collect for the last launch_ptr: (records or None, rounds_done[, dump]).
        out: a caller's (max_rounds, max_channels) TRK_EPOCH_DTYPE array to fill (reused buffers)."""
        max_rounds, records, dump = self._pending
        if out is not None:
            if not records or out.dtype != abi.TRK_EPOCH_DTYPE or out.shape != (max_rounds, self.max_channels) or not out.flags.c_contiguous:
                raise ValueError("collect(out=): a C-contiguous (max_rounds, max_channels) TRK_EPOCH_DTYPE array, records launched")
        else:
            out = np.zeros((max_rounds, self.max_channels), abi.TRK_EPOCH_DTYPE) if records else None
        dmp = np.zeros((max_rounds, self.max_channels), abi.TRK_DUMP_DTYPE) if dump else None
        done = ctypes.c_int()
        check(self.ctx.lib.gnsship_trk_collect(self.h, out.ctypes.data if records else None, dmp.ctypes.data if dump else None,
                                               ctypes.byref(done)), "gnsship_trk_collect", self.ctx.h)
        return (out, done.value, dmp) if dump else (out, done.value)

    def set_trace(self, enable: bool = True):
        """gnsship_trk_set_trace: record every channel-epoch's correlator arguments and outputs."""
        check(self.ctx.lib.gnsship_trk_set_trace(self.h, int(enable)), "gnsship_trk_set_trace", self.ctx.h)

    def trace(self, max_rounds: int) -> np.ndarray:
        """The last run's trace, [max_rounds, max_channels] TRK_TRACE_DTYPE (max_rounds of that run)."""
        out = np.zeros((max_rounds, self.max_channels), abi.TRK_TRACE_DTYPE)
        check(self.ctx.lib.gnsship_trk_trace_records(self.h, out.ctypes.data, out.size), "gnsship_trk_trace_records", self.ctx.h)
        return out

    def last_engine(self) -> int:
        """gnsship_trk_last_engine: the kernel the last run / launch ran (abi.TRK_ENGINE_*)."""
        v = ctypes.c_int(0)
        check(self.ctx.lib.gnsship_trk_last_engine(self.h, ctypes.byref(v)), "gnsship_trk_last_engine", self.ctx.h)
        return v.value

    def states(self) -> np.ndarray:
        """Tracking state (0 idle/lost, 2, 3, 4) of every channel."""
        return np.array([self.channel_state(ch)[0] for ch in range(self.max_channels)], np.int32)

    @staticmethod
    def write_dump_files(prefix: str, records: np.ndarray, dumps: np.ndarray, append: bool = False) -> list:
        """The reference's per-channel tracking dump files (<prefix><channel>.dat, dll_pll_veml_tracking.cc:
        set_channel :1674-1700, log_data :1376-1466): the records log_data wrote, in round order."""
        paths = []
        for ch in range(records.shape[1]):
            sel = (records[:, ch]["flags"] & abi.TRK_FLAG_DUMP) != 0
            path = f"{prefix}{ch}.dat"
            with open(path, "ab" if append else "wb") as f:
                f.write(np.ascontiguousarray(dumps[sel, ch]).tobytes())
            paths.append(path)
        return paths

    def close(self):
        if self.h:
            self.ctx.lib.gnsship_trk_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            if self.h and self.ctx.h:
                self.close()
        except Exception:
            pass

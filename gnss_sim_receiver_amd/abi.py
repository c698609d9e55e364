"""ctypes binding of the C ABI (include/gnsship.h) exported by ``libgnsship.so``.

The library is built in-tree (``make`` / ``__graft_entry__.build()``) next to this file.  There is
no fallback: if the shared object is missing or does not export the declared symbols, importing
the engine raises — the product path never degrades to a CPU implementation.
"""
from __future__ import annotations

import ctypes
import os
import re

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
LIB_PATH = os.path.join(PKG_DIR, "libgnsship.so")
HEADER_PATH = os.path.join(REPO_DIR, "include", "gnsship.h")

OK, E_INVAL, E_NOMEM, E_DEVICE, E_STATE, E_RCCL = 0, -1, -2, -3, -4, -5
FMT_CF32, FMT_CI16, FMT_CI8 = 0, 1, 2
STAGE_ANCHORS, STAGE_CORRELATE = 1, 2
MAX_TAPS = 8
_ERRNAMES = {E_INVAL: "E_INVAL", E_NOMEM: "E_NOMEM", E_DEVICE: "E_DEVICE", E_STATE: "E_STATE", E_RCCL: "E_RCCL"}
COMM_ID_BYTES = 128

JOB_DTYPE = np.dtype(
    [
        ("sample_offset", "<i8"),
        ("n_samples", "<i4"),
        ("code_id", "<i4"),
        ("n_taps", "<i4"),
        ("flags", "<i4"),
        ("rem_carrier_phase_rad", "<f4"),
        ("phase_step_rad", "<f4"),
        ("phase_rate_step_rad", "<f4"),
        ("rem_code_phase_chips", "<f4"),
        ("code_phase_step_chips", "<f4"),
        ("code_phase_rate_step_chips", "<f4"),
        ("shifts_chips", "<f4", (MAX_TAPS,)),
    ]
)
assert JOB_DTYPE.itemsize == 80


class AcqConf(ctypes.Structure):
    """gnsship_acq_conf — the Acq_Conf fields acquisition_core reads (acq_conf.h:33-81)."""
    _fields_ = [
        ("fs_in", ctypes.c_int64),
        ("fft_size", ctypes.c_int32),
        ("doppler_max", ctypes.c_int32),
        ("doppler_step", ctypes.c_int32),
        ("doppler_center", ctypes.c_int32),
        ("max_dwells", ctypes.c_int32),
        ("use_cfar", ctypes.c_int32),
        ("samples_per_chip", ctypes.c_int32),
        ("samples_per_code", ctypes.c_float),
        ("max_prns", ctypes.c_int32),
        ("consumed_samples", ctypes.c_int32),
        ("bit_transition_flag", ctypes.c_int32),
        ("resampler_ratio", ctypes.c_float),
        ("resampler_latency_samples", ctypes.c_uint32),
    ]


class AcqResult(ctypes.Structure):
    """gnsship_acq_result — what acquisition_core writes (pcps_acquisition.cc:683-696)."""
    _fields_ = [
        ("doppler_index", ctypes.c_uint32),
        ("code_index", ctypes.c_uint32),
        ("doppler_hz", ctypes.c_int32),
        ("peak", ctypes.c_float),
        ("input_power", ctypes.c_float),
        ("test_statistic", ctypes.c_float),
        ("acq_delay_samples", ctypes.c_double),
    ]


SYS_GPS_L1CA, SYS_GAL_E1, SYS_BDS_B1I = 0, 1, 2
# gnsship_trk_last_engine (include/gnsship.h GNSSHIP_TRK_ENGINE_*)
TRK_ENGINE_NONE, TRK_ENGINE_FAST_LATENCY, TRK_ENGINE_FAST_THROUGHPUT, TRK_ENGINE_PERSIST, TRK_ENGINE_ROUNDS, TRK_ENGINE_LANES = 0, 1, 2, 3, 4, 5
TRK_ENGINE_NAMES = {0: "none", 1: "trk_fast_kernel (latency form)", 2: "trk_fast_kernel (throughput form)", 3: "trk_persist_kernel",
                    4: "round-based loop (trk_step_kernel + correlator)", 5: "trk_lane_kernel (throughput form, one 16-lane row per channel)"}
# rotator dot-product variant (include/gnsship.h GNSSHIP_ROTATOR_*, job flag bits GNSSHIP_JOB_*)
ROTATOR_GENERIC, ROTATOR_AVX, ROTATOR_AUTO = 0, 1, -1
JOB_HIGH_DYN, JOB_ROTATOR_AVX, JOB_ROTATOR_TREE = 1, 2, 4


class TrkConf(ctypes.Structure):
    """gnsship_trk_conf — Dll_Pll_Conf (dll_pll_conf.h:33-80), same names/units; defaults as there
    with the gnss_sdr_flags defaults for cn0_samples/cn0_min/max_*lock_fail/carrier_lock_th.  The
    rotator defaults to ROTATOR_AUTO in every binding (include/gnsship.h): the variant volk_gnsssdr
    dispatches on this host.  if_hz (ABI 2): carrier IF fused into the correlator NCO."""
    _fields_ = [
        ("fs_in", ctypes.c_double), ("carrier_lock_th", ctypes.c_double),
        ("pll_bw_hz", ctypes.c_float), ("dll_bw_hz", ctypes.c_float), ("fll_bw_hz", ctypes.c_float),
        ("early_late_space_chips", ctypes.c_float), ("very_early_late_space_chips", ctypes.c_float),
        ("slope", ctypes.c_float), ("spc", ctypes.c_float), ("y_intercept", ctypes.c_float),
        ("cn0_smoother_alpha", ctypes.c_float), ("carrier_lock_test_smoother_alpha", ctypes.c_float),
        ("pull_in_time_s", ctypes.c_uint32), ("bit_synchronization_time_limit_s", ctypes.c_uint32),
        ("vector_length", ctypes.c_uint32),
        ("pll_filter_order", ctypes.c_int32), ("dll_filter_order", ctypes.c_int32),
        ("cn0_samples", ctypes.c_int32), ("cn0_smoother_samples", ctypes.c_int32),
        ("carrier_lock_test_smoother_samples", ctypes.c_int32), ("cn0_min", ctypes.c_int32),
        ("max_code_lock_fail", ctypes.c_int32), ("max_carrier_lock_fail", ctypes.c_int32),
        ("carrier_aiding", ctypes.c_int32), ("track_pilot", ctypes.c_int32), ("system", ctypes.c_int32),
        ("extend_correlation_symbols", ctypes.c_int32), ("pll_bw_narrow_hz", ctypes.c_float), ("dll_bw_narrow_hz", ctypes.c_float),
        ("early_late_space_narrow_chips", ctypes.c_float), ("very_early_late_space_narrow_chips", ctypes.c_float),
        ("enable_fll_pull_in", ctypes.c_int32), ("enable_fll_steady_state", ctypes.c_int32),
        ("high_dyn", ctypes.c_int32), ("smoother_length", ctypes.c_uint32), ("rotator", ctypes.c_int32),
        ("reserved0", ctypes.c_int32), ("if_hz", ctypes.c_double),
    ]

    @classmethod
    def defaults(cls, system: int, fs_in: float, vector_length: int, **kw) -> "TrkConf":
        c = cls(fs_in=fs_in, carrier_lock_th=0.7, pll_bw_hz=35.0, dll_bw_hz=2.0, fll_bw_hz=35.0,
                early_late_space_chips=0.25, very_early_late_space_chips=0.5, slope=1.0, spc=0.5, y_intercept=1.0,
                cn0_smoother_alpha=0.002, carrier_lock_test_smoother_alpha=0.002, pull_in_time_s=10,
                bit_synchronization_time_limit_s=20, vector_length=vector_length, pll_filter_order=3, dll_filter_order=2,
                cn0_samples=20, cn0_smoother_samples=200, carrier_lock_test_smoother_samples=25, cn0_min=25,
                max_code_lock_fail=50, max_carrier_lock_fail=5000, carrier_aiding=1, track_pilot=1, system=system,
                extend_correlation_symbols=1, pll_bw_narrow_hz=5.0, dll_bw_narrow_hz=0.75, early_late_space_narrow_chips=0.15,
                very_early_late_space_narrow_chips=0.5, enable_fll_pull_in=0, enable_fll_steady_state=0,
                high_dyn=0, smoother_length=10, rotator=ROTATOR_AUTO, reserved0=0, if_hz=0.0)
        for k, v in kw.items():
            setattr(c, k, v)
        return c


class TrkStartArgs(ctypes.Structure):
    """gnsship_trk_start_args — the Gnss_Synchro fields start_tracking reads (:647-649)."""
    _fields_ = [("code_id", ctypes.c_int32), ("data_code_id", ctypes.c_int32), ("acq_delay_samples", ctypes.c_double),
                ("acq_doppler_hz", ctypes.c_double), ("acq_samplestamp_samples", ctypes.c_uint64), ("first_sample", ctypes.c_uint64),
                ("prn", ctypes.c_int32), ("reserved", ctypes.c_int32)]


TRK_EPOCH_DTYPE = np.dtype([
    ("sample_counter", "<u8"), ("prompt_i", "<f8"), ("prompt_q", "<f8"), ("code_phase_samples", "<f8"),
    ("carrier_phase_rads", "<f8"), ("carrier_doppler_hz", "<f8"), ("cn0_db_hz", "<f8"), ("carrier_lock_test", "<f4"),
    ("state", "<i4"), ("flags", "<i4"), ("pad", "<i4"), ("code_freq_chips", "<f8"), ("rem_code_phase_chips", "<f8"),
    ("rem_carr_phase_rad", "<f4"), ("prn_length_samples", "<i4"),
])
assert TRK_EPOCH_DTYPE.itemsize == 96

# gnsship_trk_dump_record = the record dll_pll_veml_tracking::log_data writes (:1376-1466), packed
TRK_DUMP_DTYPE = np.dtype([
    ("abs_VE", "<f4"), ("abs_E", "<f4"), ("abs_P", "<f4"), ("abs_L", "<f4"), ("abs_VL", "<f4"), ("prompt_I", "<f4"), ("prompt_Q", "<f4"),
    ("PRN_start_sample_count", "<u8"), ("acc_carrier_phase_rad", "<f4"), ("carrier_doppler_hz", "<f4"), ("carrier_doppler_rate_hz", "<f4"),
    ("code_freq_chips", "<f4"), ("code_freq_rate_chips", "<f4"), ("carr_error_hz", "<f4"), ("carr_error_filt_hz", "<f4"),
    ("code_error_chips", "<f4"), ("code_error_filt_chips", "<f4"), ("CN0_SNV_dB_Hz", "<f4"), ("carrier_lock_test", "<f4"),
    ("aux1", "<f4"), ("aux2", "<f8"), ("PRN", "<u4"),
])
assert TRK_DUMP_DTYPE.itemsize == 96
TRK_FLAG_DUMP = 16

# gnsship_trk_corr_trace: one channel-epoch's do_correlation_step arguments and outputs
TRK_TRACE_DTYPE = np.dtype([
    ("sample_counter", "<u8"), ("n_samples", "<i4"), ("n_taps", "<i4"), ("rem_carrier_phase_rad", "<f4"), ("phase_step_rad", "<f4"),
    ("rem_code_phase_samples", "<f4"), ("code_phase_step_samples", "<f4"), ("shifts", "<f4", (5,)), ("taps", "<f4", (10,)),
    ("data_prompt", "<f4", (2,)), ("pad", "<i4"),
])
assert TRK_TRACE_DTYPE.itemsize == 104


class GnssHipError(RuntimeError):
    def __init__(self, code: int, what: str):
        super().__init__(f"{what} failed: {_ERRNAMES.get(code, code)}")
        self.code = code


_vp = ctypes.c_void_p
_vpp = ctypes.POINTER(ctypes.c_void_p)
_f32p = ctypes.POINTER(ctypes.c_float)
_i = ctypes.c_int
_f = ctypes.c_float

_SIGNATURES = {
    "gnsship_abi_version": ([], _i),
    "gnsship_rotator_dispatch": ([ctypes.POINTER(_i)], _i),
    "gnsship_rotator_dispatch_detail": ([ctypes.c_char_p, _i], _i),
    "gnsship_device_count": ([ctypes.POINTER(_i)], _i),
    "gnsship_ctx_create": ([_i, _vpp], _i),
    "gnsship_ctx_destroy": ([_vp], _i),
    "gnsship_last_error": ([_vp], ctypes.c_char_p),
    "gnsship_ctx_sync": ([_vp], _i),
    "gnsship_ctx_stream": ([_vp, _vpp], _i),
    "gnsship_ctx_event_record": ([_vp, _i], _i),
    "gnsship_ctx_event_elapsed_ms": ([_vp, _i, _i, _f32p], _i),
    "gnsship_dev_alloc": ([_vp, ctypes.c_size_t, _vpp], _i),
    "gnsship_dev_free": ([_vp, _vp], _i),
    "gnsship_dev_upload": ([_vp, _vp, _vp, ctypes.c_size_t], _i),
    "gnsship_dev_download": ([_vp, _vp, _vp, ctypes.c_size_t], _i),
    "gnsship_code_set": ([_vp, _i, _f32p, _i], _i),
    "gnsship_code_count": ([_vp, ctypes.POINTER(_i)], _i),
    "gnsship_gps_l1_ca_code_gen_float": ([_f32p, ctypes.c_int32, ctypes.c_uint32], _i),
    "gnsship_gps_l1_ca_code_gen_complex_sampled": ([_f32p, ctypes.c_uint32, ctypes.c_int32, ctypes.c_uint32], _i),
    "gnsship_beidou_b1i_code_gen_float": ([_f32p, ctypes.c_int32, ctypes.c_uint32], _i),
    "gnsship_beidou_b1i_code_gen_complex_sampled": ([_f32p, ctypes.c_uint32, ctypes.c_int32, ctypes.c_uint32], _i),
    "gnsship_code_samples_per_code": ([ctypes.c_int32, ctypes.c_int32, ctypes.c_int32], _i),
    "gnsship_corr_create": ([_vp, _i, _i, _vpp], _i),
    "gnsship_corr_set_local_code_and_taps": ([_vp, _i, _f32p, _f32p], _i),
    "gnsship_corr_set_high_dynamics_resampler": ([_vp, _i], _i),
    "gnsship_corr_set_rotator": ([_vp, _i], _i),
    "gnsship_corr_run": ([_vp, _vp, _i, _i, _f, _f, _f, _f, _f, _f, _i, _f32p], _i),
    "gnsship_corr_destroy": ([_vp], _i),
    "gnsship_batch_create": ([_vp, _i, _vpp], _i),
    "gnsship_batch_set_jobs": ([_vp, _vp, _i, ctypes.c_int64], _i),
    "gnsship_batch_launch": ([_vp, _vp, _i], _i),
    "gnsship_batch_launch_stages": ([_vp, _vp, _i, _i], _i),
    "gnsship_batch_results": ([_vp, _f32p], _i),
    "gnsship_batch_results_device": ([_vp, _vpp], _i),
    "gnsship_batch_launch_pipelined": ([_vp, _vp, _i, _vp], _i),
    "gnsship_batch_launch_pipelined2": ([_vp, _vp, _i, _vp, _vp], _i),
    "gnsship_batch_destroy": ([_vp], _i),
    "gnsship_acq_create": ([_vp, ctypes.POINTER(AcqConf), _vpp], _i),
    "gnsship_acq_set_grid": ([_vp, _i, _i, _i], _i),
    "gnsship_acq_set_grid_step2": ([_vp, _f, _f, _i, _f], _i),
    "gnsship_acq_set_local_code": ([_vp, _i, _f32p], _i),
    "gnsship_acq_run": ([_vp, _vp, _i, _i, _i, ctypes.POINTER(AcqResult), _f32p], _i),
    "gnsship_acq_num_bins": ([_vp, ctypes.POINTER(_i)], _i),
    "gnsship_acq_reset_dwells": ([_vp], _i),
    "gnsship_acq_destroy": ([_vp], _i),
    "gnsship_firdes_low_pass": ([ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double, _f32p, _i, ctypes.POINTER(_i)], _i),
    "gnsship_acq_resampler_design": ([ctypes.c_int64, ctypes.c_double, ctypes.POINTER(_i), _f32p, _i, ctypes.POINTER(_i)], _i),
    "gnsship_acq_resampler_create": ([_vp, _f32p, _i, _i, ctypes.c_int64, _vpp], _i),
    "gnsship_acq_resampler_run": ([_vp, _vp, _i, _i, ctypes.c_int64, _f32p, _vpp, ctypes.POINTER(ctypes.c_int64)], _i),
    "gnsship_acq_resampler_reset": ([_vp], _i),
    "gnsship_acq_resampler_destroy": ([_vp], _i),
    "gnsship_trk_create": ([_vp, ctypes.POINTER(TrkConf), _i, _vpp], _i),
    "gnsship_trk_start": ([_vp, _i, ctypes.POINTER(TrkStartArgs)], _i),
    "gnsship_trk_start_many": ([_vp, _i, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(TrkStartArgs)], _i),
    "gnsship_trk_stop": ([_vp, _i], _i),
    "gnsship_trk_telemetry_event": ([_vp, _i, _i], _i),
    "gnsship_trk_run": ([_vp, _vp, _i, _i, ctypes.c_uint64, ctypes.c_int64, _i, _vp, ctypes.POINTER(_i)], _i),
    "gnsship_trk_run_dump": ([_vp, _vp, _i, _i, ctypes.c_uint64, ctypes.c_int64, _i, _vp, _vp, ctypes.POINTER(_i)], _i),
    "gnsship_trk_launch": ([_vp, _vp, _i, ctypes.c_uint64, ctypes.c_int64, _i, _i, _i], _i),
    "gnsship_trk_collect": ([_vp, _vp, _vp, ctypes.POINTER(_i)], _i),
    "gnsship_trk_set_trace": ([_vp, _i], _i),
    "gnsship_trk_trace_records": ([_vp, _vp, _i], _i),
    "gnsship_trk_channel_state": ([_vp, _i, ctypes.POINTER(_i), ctypes.POINTER(ctypes.c_uint64)], _i),
    "gnsship_trk_last_engine": ([_vp, ctypes.POINTER(_i)], _i),
    "gnsship_trk_destroy": ([_vp], _i),
    "gnsship_comm_unique_id": ([_vp], _i),
    "gnsship_comm_create": ([_vp, _i, _i, _vp, _vpp], _i),
    "gnsship_comm_rank": ([_vp, ctypes.POINTER(_i), ctypes.POINTER(_i)], _i),
    "gnsship_comm_broadcast": ([_vp, _vp, ctypes.c_size_t, _i], _i),
    "gnsship_comm_allgather": ([_vp, _vp, _vp, ctypes.c_size_t], _i),
    "gnsship_comm_allreduce_max_f64": ([_vp, _vp, ctypes.c_size_t], _i),
    "gnsship_comm_destroy": ([_vp], _i),
}


def declared_symbols(header: str = HEADER_PATH) -> list:
    """Every function name declared in include/gnsship.h."""
    text = open(header).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(gnsship_[a-z0-9_]+)\s*\(", text)))


_LIB = None


ABI_VERSION = 2  # GNSSHIP_ABI_VERSION of the header these bindings mirror


def load() -> ctypes.CDLL:
    """Load libgnsship.so (raises if it was not built — no fallback)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    # GNSSHIP_LIB_PATH: tooling only (scripts/corr_wg_profile.py loads the instrumented build)
    path = os.environ.get("GNSSHIP_LIB_PATH", LIB_PATH)
    if not os.path.exists(path):
        raise RuntimeError(f"{path} is missing: build it with `make` or __graft_entry__.build(); "
                           "the GNSS engine has no CPU fallback")
    lib = ctypes.CDLL(path)
    for name, (argtypes, restype) in _SIGNATURES.items():
        fn = getattr(lib, name)  # AttributeError if the symbol is not exported
        fn.argtypes = argtypes
        fn.restype = restype
    if lib.gnsship_abi_version() != ABI_VERSION:
        raise RuntimeError(f"{path}: ABI version {lib.gnsship_abi_version()}, these bindings need {ABI_VERSION} (rebuild with `make`)")
    _LIB = lib
    return lib


def check(rc: int, what: str, ctx=None) -> None:
    if rc != OK:
        msg = what
        if ctx is not None:
            detail = load().gnsship_last_error(ctx)
            if detail:
                msg = f"{what} ({detail.decode(errors='replace')})"
        raise GnssHipError(rc, msg)


def fptr(a: np.ndarray):
    return a.ctypes.data_as(_f32p)


def rotator_dispatch() -> int:
    """The volk_gnsssdr rotator variant the reference would run on this host (gnsship_rotator_dispatch):
    ROTATOR_GENERIC or ROTATOR_AVX.  Host-only: no device needed.  Raises for a preferences entry
    naming a variant the engine does not reproduce (the message says which)."""
    v = ctypes.c_int(-1)
    rc = load().gnsship_rotator_dispatch(ctypes.byref(v))
    if rc != OK:
        raise GnssHipError(rc, f"gnsship_rotator_dispatch ({rotator_dispatch_detail()})")
    return v.value


def rotator_dispatch_detail() -> str:
    buf = ctypes.create_string_buffer(512)
    load().gnsship_rotator_dispatch_detail(buf, 512)
    return buf.value.decode(errors="replace")

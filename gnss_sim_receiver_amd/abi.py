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

OK, E_INVAL, E_NOMEM, E_DEVICE, E_STATE = 0, -1, -2, -3, -4
FMT_CF32, FMT_CI16, FMT_CI8 = 0, 1, 2
STAGE_ANCHORS, STAGE_CORRELATE = 1, 2
MAX_TAPS = 8
_ERRNAMES = {E_INVAL: "E_INVAL", E_NOMEM: "E_NOMEM", E_DEVICE: "E_DEVICE", E_STATE: "E_STATE"}

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
    "gnsship_corr_run": ([_vp, _vp, _i, _i, _f, _f, _f, _f, _f, _f, _i, _f32p], _i),
    "gnsship_corr_destroy": ([_vp], _i),
    "gnsship_batch_create": ([_vp, _i, _vpp], _i),
    "gnsship_batch_set_jobs": ([_vp, _vp, _i, ctypes.c_int64], _i),
    "gnsship_batch_launch": ([_vp, _vp, _i], _i),
    "gnsship_batch_launch_stages": ([_vp, _vp, _i, _i], _i),
    "gnsship_batch_results": ([_vp, _f32p], _i),
    "gnsship_batch_results_device": ([_vp, _vpp], _i),
    "gnsship_batch_destroy": ([_vp], _i),
    "gnsship_acq_create": ([_vp, ctypes.POINTER(AcqConf), _vpp], _i),
    "gnsship_acq_set_grid": ([_vp, _i, _i, _i], _i),
    "gnsship_acq_set_local_code": ([_vp, _i, _f32p], _i),
    "gnsship_acq_run": ([_vp, _vp, _i, _i, _i, ctypes.POINTER(AcqResult), _f32p], _i),
    "gnsship_acq_num_bins": ([_vp, ctypes.POINTER(_i)], _i),
    "gnsship_acq_destroy": ([_vp], _i),
}


def declared_symbols(header: str = HEADER_PATH) -> list:
    """Every function name declared in include/gnsship.h."""
    text = open(header).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(gnsship_[a-z0-9_]+)\s*\(", text)))


_LIB = None


def load() -> ctypes.CDLL:
    """Load libgnsship.so (raises if it was not built — no fallback)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: build it with `make` or __graft_entry__.build(); "
                           "the GNSS engine has no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (argtypes, restype) in _SIGNATURES.items():
        fn = getattr(lib, name)  # AttributeError if the symbol is not exported
        fn.argtypes = argtypes
        fn.restype = restype
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

"""ctypes bindings of oracle/trk_oracle.c — the CPU restatement of the DLL/PLL tracking loop.

TEST INFRASTRUCTURE ONLY (checker for gnsship_trk_*).  The per-system signal constants below are
restated from the reference independently of the product (dll_pll_veml_tracking.cc:142-330 and
start_tracking :662-797; GPS_L1_CA.h:61-73, Galileo_E1.h:35-52, Beidou_B1I.h:35-48).
"""
from __future__ import annotations

import ctypes

import numpy as np

from .oracle import lib, _ptr

_f32p = ctypes.POINTER(ctypes.c_float)
TRK_MAX_SEC = 256


class OrcTrkConf(ctypes.Structure):
    _fields_ = [
        ("fs_in", ctypes.c_double), ("carrier_lock_th", ctypes.c_double), ("code_chip_rate", ctypes.c_double),
        ("signal_carrier_freq", ctypes.c_double), ("code_period", ctypes.c_double),
        ("pll_bw_hz", ctypes.c_float), ("dll_bw_hz", ctypes.c_float), ("fll_bw_hz", ctypes.c_float),
        ("early_late_space_chips", ctypes.c_float), ("very_early_late_space_chips", ctypes.c_float),
        ("slope", ctypes.c_float), ("spc", ctypes.c_float), ("y_intercept", ctypes.c_float),
        ("cn0_smoother_alpha", ctypes.c_float), ("carrier_lock_test_smoother_alpha", ctypes.c_float),
        ("pull_in_time_s", ctypes.c_uint32), ("bit_synchronization_time_limit_s", ctypes.c_uint32), ("vector_length", ctypes.c_uint32),
        ("pll_filter_order", ctypes.c_int32), ("dll_filter_order", ctypes.c_int32), ("cn0_samples", ctypes.c_int32),
        ("cn0_smoother_samples", ctypes.c_int32), ("carrier_lock_test_smoother_samples", ctypes.c_int32), ("cn0_min", ctypes.c_int32),
        ("max_code_lock_fail", ctypes.c_int32), ("max_carrier_lock_fail", ctypes.c_int32), ("carrier_aiding", ctypes.c_int32),
        ("track_pilot", ctypes.c_int32), ("veml", ctypes.c_int32),
        ("code_length_chips", ctypes.c_int32), ("code_samples_per_chip", ctypes.c_int32), ("symbols_per_bit", ctypes.c_int32),
        ("secondary", ctypes.c_int32), ("secondary_code_length", ctypes.c_int32), ("data_secondary_code_length", ctypes.c_int32),
        ("secondary_code", ctypes.c_char * (TRK_MAX_SEC + 1)), ("data_secondary_code", ctypes.c_char * (TRK_MAX_SEC + 1)),
        ("extend_correlation_symbols", ctypes.c_int32), ("pll_bw_narrow_hz", ctypes.c_float), ("dll_bw_narrow_hz", ctypes.c_float),
        ("early_late_space_narrow_chips", ctypes.c_float), ("very_early_late_space_narrow_chips", ctypes.c_float),
        ("enable_fll_pull_in", ctypes.c_int32), ("enable_fll_steady_state", ctypes.c_int32),
        ("high_dyn", ctypes.c_int32), ("smoother_length", ctypes.c_uint32), ("rotator_avx", ctypes.c_int32),
        ("accum_f64", ctypes.c_int32), ("pad_trig", ctypes.c_int32), ("pad_if", ctypes.c_int32), ("if_hz", ctypes.c_double),
    ]


EPOCH_DTYPE = np.dtype([
    ("sample_counter", "<u8"), ("prompt_i", "<f8"), ("prompt_q", "<f8"), ("code_phase_samples", "<f8"),
    ("carrier_phase_rads", "<f8"), ("carrier_doppler_hz", "<f8"), ("cn0_db_hz", "<f8"), ("carrier_lock_test", "<f4"),
    ("state", "<i4"), ("flags", "<i4"), ("pad", "<i4"), ("code_freq_chips", "<f8"), ("rem_code_phase_chips", "<f8"),
    ("rem_carr_phase_rad", "<f4"), ("prn_length_samples", "<i4"),
])

# log_data's record (dll_pll_veml_tracking.cc:1376-1466 = tracking_dump_reader.cc:26-47), packed
DUMP_DTYPE = np.dtype([
    ("abs_VE", "<f4"), ("abs_E", "<f4"), ("abs_P", "<f4"), ("abs_L", "<f4"), ("abs_VL", "<f4"), ("prompt_I", "<f4"), ("prompt_Q", "<f4"),
    ("PRN_start_sample_count", "<u8"), ("acc_carrier_phase_rad", "<f4"), ("carrier_doppler_hz", "<f4"), ("carrier_doppler_rate_hz", "<f4"),
    ("code_freq_chips", "<f4"), ("code_freq_rate_chips", "<f4"), ("carr_error_hz", "<f4"), ("carr_error_filt_hz", "<f4"),
    ("code_error_chips", "<f4"), ("code_error_filt_chips", "<f4"), ("CN0_SNV_dB_Hz", "<f4"), ("carrier_lock_test", "<f4"),
    ("aux1", "<f4"), ("aux2", "<f8"), ("PRN", "<u4"),
])
assert DUMP_DTYPE.itemsize == 96

GPS_PREAMBLE_SYMBOLS = "1" * 20 + "0" * 60 + "1" * 20 + "0" * 20 + "1" * 40  # GPS_L1_CA.h:73 (10001011 × 20)
E1C_SECONDARY = "0011100000001010110110010"                               # Galileo_E1.h:52
B1I_NH = "00000100110101001110"                                           # Beidou_B1I.h:48
B1I_GEO_PREAMBLE = "1111110000001100001100"                               # Beidou_B1I.h:49 (11100010010 × 2)


def is_bds_geo(prn: int) -> bool:
    """start_tracking's GEO test (dll_pll_veml_tracking.cc:766)."""
    return (0 < prn < 6) or prn > 58

SYSTEMS = {
    # system: chip rate, carrier, code period, code length, samples/chip, symbols/bit, veml, secondary, sec code, data sec
    "GPS": (1.023e6, 1575.42e6, 0.001, 1023, 1, 20, 0, 0, GPS_PREAMBLE_SYMBOLS, ""),
    "GAL": (1.023e6, 1575.42e6, 0.004, 4092, 2, 1, 1, 1, E1C_SECONDARY, ""),
    "BDS": (2.046e6, 1561.098e6, 0.001, 2046, 1, 20, 0, 1, B1I_NH, B1I_NH),
}


def conf(system: str, fs_in: float, vector_length: int, prn: int = 0, **kw) -> OrcTrkConf:
    """Dll_Pll_Conf defaults (dll_pll_conf.h:33-80 + gnss_sdr_flags.cc:48-57) plus the signal
    constants of `system`; keyword overrides for any field.  `prn`: a BeiDou GEO PRN applies
    start_tracking's GEO settings (:765-781) — D2 symbols (2 per bit), no NH code, the 22-symbol
    preamble as the bit-synchronisation pattern, extend_correlation_symbols capped at 2."""
    rate, fc, period, L, spc, spb, veml, sec, sec_code, dsec = SYSTEMS[system]
    track_pilot = kw.pop("track_pilot", 1) if system == "GAL" else 0
    if system == "GAL" and not track_pilot:
        sec, sec_code = 0, ""
    c = OrcTrkConf(fs_in=fs_in, carrier_lock_th=0.7, code_chip_rate=rate, signal_carrier_freq=fc, code_period=period,
                   pll_bw_hz=35.0, dll_bw_hz=2.0, fll_bw_hz=35.0, early_late_space_chips=0.25, very_early_late_space_chips=0.5,
                   slope=1.0, spc=0.5, y_intercept=1.0, cn0_smoother_alpha=0.002, carrier_lock_test_smoother_alpha=0.002,
                   pull_in_time_s=10, bit_synchronization_time_limit_s=20, vector_length=vector_length, pll_filter_order=3,
                   dll_filter_order=2, cn0_samples=20, cn0_smoother_samples=200, carrier_lock_test_smoother_samples=25, cn0_min=25,
                   max_code_lock_fail=50, max_carrier_lock_fail=5000, carrier_aiding=1, track_pilot=track_pilot, veml=veml,
                   code_length_chips=L, code_samples_per_chip=spc, symbols_per_bit=spb, secondary=sec,
                   secondary_code_length=len(sec_code), data_secondary_code_length=len(dsec),
                   secondary_code=sec_code.encode(), data_secondary_code=dsec.encode(),
                   extend_correlation_symbols=1, pll_bw_narrow_hz=5.0, dll_bw_narrow_hz=0.75, early_late_space_narrow_chips=0.15,
                   very_early_late_space_narrow_chips=0.5, enable_fll_pull_in=0, enable_fll_steady_state=0,
                   high_dyn=0, smoother_length=10)
    for k, v in kw.items():
        setattr(c, k, v)
    if system == "BDS" and is_bds_geo(prn):
        c.symbols_per_bit = 2
        c.secondary = 0
        c.secondary_code = B1I_GEO_PREAMBLE.encode()
        c.secondary_code_length = len(B1I_GEO_PREAMBLE)
        c.data_secondary_code_length = 0
        c.data_secondary_code = b""
        c.extend_correlation_symbols = min(c.extend_correlation_symbols, 2)
    return c


def _L(fast: bool = False):
    L = lib(fast)
    if getattr(L, "_trk_ready", False):
        return L
    vp = ctypes.c_void_p
    L.orc_lf_init.argtypes = [vp, ctypes.c_float, ctypes.c_float, ctypes.c_int, ctypes.c_int]
    L.orc_lf_initialize.argtypes = [vp, ctypes.c_float]
    L.orc_lf_apply.argtypes = [vp, ctypes.c_float]
    L.orc_lf_apply.restype = ctypes.c_float
    L.orc_fp_set_params.argtypes = [vp, ctypes.c_float, ctypes.c_float, ctypes.c_int]
    L.orc_fp_initialize.argtypes = [vp, ctypes.c_float]
    L.orc_fp_get_carrier_error.argtypes = [vp, ctypes.c_float, ctypes.c_float, ctypes.c_float]
    L.orc_fp_get_carrier_error.restype = ctypes.c_float
    L.orc_sm_init.argtypes = [vp, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_int]
    L.orc_sm_smooth.argtypes = [vp, ctypes.c_float]
    L.orc_sm_smooth.restype = ctypes.c_float
    L.orc_pll_cloop_two_quadrant_atan.argtypes = [ctypes.c_float, ctypes.c_float]
    L.orc_pll_cloop_two_quadrant_atan.restype = ctypes.c_double
    L.orc_dll_nc_e_minus_l_normalized.argtypes = [ctypes.c_float] * 7
    L.orc_dll_nc_e_minus_l_normalized.restype = ctypes.c_double
    L.orc_dll_nc_vemlp_normalized.argtypes = [_f32p, _f32p, _f32p, _f32p]
    L.orc_dll_nc_vemlp_normalized.restype = ctypes.c_double
    L.orc_cn0_m2m4_estimator.argtypes = [_f32p, ctypes.c_int, ctypes.c_float]
    L.orc_cn0_m2m4_estimator.restype = ctypes.c_float
    L.orc_carrier_lock_detector.argtypes = [_f32p, ctypes.c_int]
    L.orc_carrier_lock_detector.restype = ctypes.c_float
    L.orc_trk_start.argtypes = [ctypes.POINTER(OrcTrkConf), vp, ctypes.c_double, ctypes.c_double, ctypes.c_uint64, ctypes.c_uint64]
    L.orc_trk_run.argtypes = [ctypes.POINTER(OrcTrkConf), vp, _f32p, ctypes.c_uint64, ctypes.c_int64, _f32p, ctypes.c_int, _f32p, ctypes.c_int,
                              vp, vp]
    L.orc_trk_set_prn.argtypes = [vp, ctypes.c_uint32]
    L.orc_trk_telemetry_fault.argtypes = [vp]
    L.orc_trk_nitems_read.argtypes = [vp]
    L.orc_trk_nitems_read.restype = ctypes.c_uint64
    L.orc_trk_state.argtypes = [vp]
    for name in ("orc_trk_sizeof_channel", "orc_trk_sizeof_conf", "orc_trk_sizeof_epoch", "orc_trk_sizeof_dump", "orc_trk_sizeof_loop_filter",
                 "orc_trk_sizeof_fll_pll", "orc_trk_sizeof_smoother"):
        getattr(L, name).restype = ctypes.c_int
    assert L.orc_trk_sizeof_conf() == ctypes.sizeof(OrcTrkConf)
    assert L.orc_trk_sizeof_epoch() == EPOCH_DTYPE.itemsize
    assert L.orc_trk_sizeof_dump() == DUMP_DTYPE.itemsize
    L._trk_ready = True
    return L


class LoopFilter:
    """Tracking_loop_filter restatement (tracking_loop_filter.cc)."""

    def __init__(self, update_interval, noise_bandwidth, order, include_last_integrator=False):
        L = _L()
        self.buf = ctypes.create_string_buffer(L.orc_trk_sizeof_loop_filter())
        L.orc_lf_init(self.buf, update_interval, noise_bandwidth, order, int(include_last_integrator))

    def initialize(self, initial_output=0.0):
        _L().orc_lf_initialize(self.buf, initial_output)

    def apply(self, x):
        return _L().orc_lf_apply(self.buf, x)


class FllPllFilter:
    def __init__(self, fll_bw, pll_bw, order, acq_doppler):
        L = _L()
        self.buf = ctypes.create_string_buffer(L.orc_trk_sizeof_fll_pll())
        L.orc_fp_set_params(self.buf, fll_bw, pll_bw, order)
        L.orc_fp_initialize(self.buf, acq_doppler)

    def get_carrier_error(self, fll, pll, T):
        return _L().orc_fp_get_carrier_error(self.buf, fll, pll, T)


class Smoother:
    def __init__(self, alpha, min_value=25.0, offset=12.0, samples_for_init=200):
        L = _L()
        self.buf = ctypes.create_string_buffer(L.orc_trk_sizeof_smoother())
        L.orc_sm_init(self.buf, alpha, min_value, offset, samples_for_init)

    def smooth(self, raw):
        return _L().orc_sm_smooth(self.buf, raw)


def dll_nc_e_minus_l_normalized(E: complex, Lt: complex, spc=0.5, slope=1.0, y_intercept=1.0) -> float:
    return _L().orc_dll_nc_e_minus_l_normalized(E.real, E.imag, Lt.real, Lt.imag, spc, slope, y_intercept)


def pll_cloop_two_quadrant_atan(P: complex) -> float:
    return _L().orc_pll_cloop_two_quadrant_atan(P.real, P.imag)


def cn0_m2m4_estimator(prompt: np.ndarray, coh_time_s: float) -> float:
    p = np.ascontiguousarray(prompt, np.complex64)
    return _L().orc_cn0_m2m4_estimator(_ptr(p.view(np.float32)), len(p), coh_time_s)


def carrier_lock_detector(prompt: np.ndarray) -> float:
    p = np.ascontiguousarray(prompt, np.complex64)
    return _L().orc_carrier_lock_detector(_ptr(p.view(np.float32)), len(p))


class Channel:
    """One oracle channel: start_tracking, then run() over successive buffers."""

    def __init__(self, k: OrcTrkConf, code: np.ndarray, acq_delay_samples: float, acq_doppler_hz: float, acq_samplestamp: int,
                 first_sample: int, data_code: np.ndarray = None, prn: int = 0, fast: bool = False):
        """fast: the same source built at -O3 -march=native (liboracle_fast.so), for timing only."""
        self.fast = fast
        L = _L(fast)
        self.k = k
        self.buf = ctypes.create_string_buffer(L.orc_trk_sizeof_channel())
        self.code = np.ascontiguousarray(code, np.float32)
        self.data_code = np.ascontiguousarray(data_code, np.float32) if data_code is not None else None
        L.orc_trk_start(ctypes.byref(k), self.buf, acq_delay_samples, acq_doppler_hz, acq_samplestamp, first_sample)
        L.orc_trk_set_prn(self.buf, prn)

    def run(self, samples: np.ndarray, buffer_first: int, max_epochs: int, dump: bool = False):
        """EPOCH_DTYPE records (and, with dump=True, the per-epoch DUMP_DTYPE records; rows whose
        epoch has flags & 16 are the ones log_data writes)."""
        L = _L(self.fast)
        x = np.ascontiguousarray(samples, np.complex64)
        out = np.zeros(max_epochs, EPOCH_DTYPE)
        d = np.zeros(max_epochs, DUMP_DTYPE) if dump else None
        dc = self.data_code
        n = L.orc_trk_run(ctypes.byref(self.k), self.buf, _ptr(x.view(np.float32)), buffer_first, len(x), _ptr(self.code), len(self.code),
                          _ptr(dc) if dc is not None else None, max_epochs, out.ctypes.data, d.ctypes.data if dump else None)
        return (out[:n], d[:n]) if dump else out[:n]

    def telemetry_fault(self):
        """msg_handler_telemetry_to_trk with tlm_event 1 (dll_pll_veml_tracking.cc:617-640)."""
        _L(self.fast).orc_trk_telemetry_fault(self.buf)

    @property
    def state(self) -> int:
        return _L(self.fast).orc_trk_state(self.buf)

    @property
    def next_sample(self) -> int:
        return _L(self.fast).orc_trk_nitems_read(self.buf)


def track(k: OrcTrkConf, samples: np.ndarray, code: np.ndarray, acq_delay_samples: float, acq_doppler_hz: float, acq_samplestamp: int,
          first_sample: int, max_epochs: int, data_code: np.ndarray = None, buffer_first: int = 0, dump: bool = False, prn: int = 0):
    """start_tracking + general_work until max_epochs / loss of lock / end of `samples`
    (samples[i] = absolute sample buffer_first + i).  Returns EPOCH_DTYPE records (+ DUMP_DTYPE)."""
    ch = Channel(k, code, acq_delay_samples, acq_doppler_hz, acq_samplestamp, first_sample, data_code, prn)
    return ch.run(samples, buffer_first, max_epochs, dump)

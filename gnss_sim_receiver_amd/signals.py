"""Synthetic GNSS IF generator and truth-aligned correlator job builder.

    x[n] = Σ_k A_k · c_k(n) · d_k(n) · exp(j(2π(f_IF,k + fD_k)·n/fs + φ_k)) + w[n]

* w: complex Gaussian, σ = 1 per component (as signal_generator_c.cc:540-546);
* A_k = sqrt(2·10^(CN0_k/10) / fs), so that C/N0 = A² / (2σ²/fs);
* c_k: the PRN code clocked at chip_rate·(1 + fD/f_carrier) (code Doppler), delayed by τ_k chips;
* d_k: ±1 data bits (GPS 50 bps = 20 code periods per bit), off by default.

Formats: gr_complex = complex64; ibyte = round(8·x) clipped to ±127, int8 interleaved I,Q.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import codes as C
from .abi import JOB_DTYPE, MAX_TAPS

SYSTEMS = {
    # name: (chip_rate, code_len, carrier_hz, code generator)
    "GPS": (C.GPS_L1_CA_CODE_RATE_CPS, C.GPS_L1_CA_CODE_LENGTH_CHIPS, C.GPS_L1_FREQ_HZ, C.gps_l1_ca_code_gen_float),
    "BDS": (C.BEIDOU_B1I_CODE_RATE_CPS, C.BEIDOU_B1I_CODE_LENGTH_CHIPS, C.BEIDOU_B1I_FREQ_HZ, C.beidou_b1i_code_gen_float),
    # Galileo E1 in units of the sinBOC(1,1) replica (2 samples per chip, 8184 per 4 ms code):
    # the tracking code is the E1-C pilot (track_pilot = true), the data code E1-B
    # (dll_pll_veml_tracking.cc:684-697 with galileo_e1_code_gen_sinboc11_float).
    "GAL": (2.0 * C.GALILEO_E1_CODE_CHIP_RATE_CPS, 2 * C.GALILEO_E1_B_CODE_LENGTH_CHIPS, C.GALILEO_E1_FREQ_HZ,
            lambda prn: C.galileo_e1_code_gen_sinboc11_float("1C", prn)),
}
DATA_CODES = {"GAL": lambda prn: C.galileo_e1_code_gen_sinboc11_float("1B", prn)}


@dataclass
class Satellite:
    prn: int
    doppler_hz: float
    code_delay_chips: float
    carrier_phase_rad: float = 0.0
    cn0_dbhz: float = 45.0
    system: str = "GPS"
    data_bits: bool = False
    bit_seed: int = 0
    f_if_hz: float = 0.0
    code: np.ndarray = field(default=None, repr=False)
    code_data: np.ndarray = field(default=None, repr=False)  # E1-B data component (Galileo)
    # cyclic navigation-bit pattern ('0' → +1, '1' → −1): GPS / BDS one bit per 20 code periods,
    # Galileo one E1-B symbol per code period (250 sps)
    bits: str = None
    # cyclic secondary code, one chip per code period: E1-C CS25 on the Galileo pilot, the B1I NH
    # code on the BeiDou signal
    secondary: str = None
    # line-of-sight dynamics: the Doppler ramps at this rate from doppler_hz at sample 0
    doppler_rate_hz_s: float = 0.0
    # code periods per navigation bit when not the system default (BeiDou GEO D2: 2)
    symbols_per_bit: int = None

    def __post_init__(self):
        if self.code is None:
            self.code = SYSTEMS[self.system][3](self.prn)
        if self.code_data is None and self.system in DATA_CODES:
            self.code_data = DATA_CODES[self.system](self.prn)

    @property
    def chip_rate(self):
        return SYSTEMS[self.system][0]

    @property
    def code_len(self):
        return SYSTEMS[self.system][1]

    def code_freq(self):
        rate, _, fc, _ = SYSTEMS[self.system]
        return rate * (1.0 + self.doppler_hz / fc)

    def chip_phase(self, n: np.ndarray, fs: float) -> np.ndarray:
        """Received code phase [chips] at sample n (unwrapped)."""
        ph = n / fs * self.code_freq() - self.code_delay_chips
        if self.doppler_rate_hz_s:
            rate, _, fc, _ = SYSTEMS[self.system]
            ph = ph + 0.5 * rate * self.doppler_rate_hz_s / fc * (n / fs) ** 2
        return ph

    def carrier_phase(self, n: np.ndarray, fs: float) -> np.ndarray:
        ph = 2.0 * np.pi * (self.f_if_hz + self.doppler_hz) * (n / fs) + self.carrier_phase_rad
        if self.doppler_rate_hz_s:
            ph = ph + np.pi * self.doppler_rate_hz_s * (n / fs) ** 2
        return ph


def generate_if(fs: float, n_samples: int, sats: list, seed: int = 0, noise: bool = True, start: int = 0,
                block: int = 1 << 20) -> np.ndarray:
    """complex64[n_samples] of synthetic IF starting at absolute sample `start`."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out = np.empty(n_samples, np.complex64)
    for b0 in range(0, n_samples, block):
        b1 = min(n_samples, b0 + block)
        n = np.arange(start + b0, start + b1, dtype=np.float64)
        acc = np.zeros(b1 - b0, np.complex128)
        for s in sats:
            amp = np.sqrt(2.0 * 10.0 ** (s.cn0_dbhz / 10.0) / fs)
            ph = s.chip_phase(n, fs)
            chip = np.floor(ph).astype(np.int64)
            c = s.code[np.mod(chip, s.code_len)].astype(np.float64)
            period = np.floor_divide(chip, s.code_len)
            if s.secondary:
                sec = np.array([1.0 if b == "0" else -1.0 for b in s.secondary])
                c = c * sec[np.mod(period, len(sec))]
            data_sign = 1.0
            if s.bits:
                pat = np.array([1.0 if b == "0" else -1.0 for b in s.bits])
                per_bit = s.symbols_per_bit or (1 if s.code_data is not None else 20)
                data_sign = pat[np.mod(np.floor_divide(period, per_bit), len(pat))]
            if s.code_data is not None:  # Galileo E1 OS: (E1B − E1C)/√2 with sinBOC(1,1) subcarriers
                c = (data_sign * s.code_data[np.mod(chip, s.code_len)].astype(np.float64) - c) / np.sqrt(2.0)
            else:
                c = c * data_sign
            if s.data_bits:
                periods = np.floor_divide(chip, s.code_len)
                bit_idx = np.floor_divide(periods, 20)
                bits = np.where((np.bitwise_xor(bit_idx * 2654435761 + s.bit_seed, 0x5BD1E995) >> 7) & 1, -1.0, 1.0)
                c = c * bits
            acc += amp * c * np.exp(1j * s.carrier_phase(n, fs))
        if noise:
            acc += rng.standard_normal(b1 - b0) + 1j * rng.standard_normal(b1 - b0)
        out[b0:b1] = acc.astype(np.complex64)
    return out


def to_ibyte(x: np.ndarray, scale: float = 8.0) -> np.ndarray:
    """int8 interleaved I,Q: round(scale·x) clipped to ±127 (the C5 ibyte format)."""
    iq = np.empty(2 * len(x), np.float32)
    iq[0::2] = x.real
    iq[1::2] = x.imag
    return np.clip(np.rint(scale * iq), -127, 127).astype(np.int8)


def to_ishort(x: np.ndarray, scale: float = 256.0) -> np.ndarray:
    iq = np.empty(2 * len(x), np.float32)
    iq[0::2] = x.real
    iq[1::2] = x.imag
    return np.clip(np.rint(scale * iq), -32767, 32767).astype(np.int16)


def truth_jobs(sat: Satellite, fs: float, n_epochs: int, vector_length: int, shifts_chips, code_id: int,
               samples_per_chip: int = 1, first_epoch: int = 1) -> np.ndarray:
    """One correlator job per code period, NCO set from the synthetic truth (as a locked DLL/PLL
    would): epoch e starts at the first sample at or after the start of code period e, with
    rem_code = −(fractional chip at that sample) and rem_carr = carrier phase at that sample.
    Argument meaning/units follow dll_pll_veml_tracking::do_correlation_step (:1037-1048)."""
    jobs = np.zeros(n_epochs, JOB_DTYPE)
    L = sat.code_len
    fcode = sat.code_freq()
    for i in range(n_epochs):
        e = first_epoch + i
        # sample where the received code phase crosses e*L chips
        t_start = (e * L + sat.code_delay_chips) / fcode
        s = int(np.ceil(t_start * fs))
        chip = sat.chip_phase(np.float64(s), fs) - e * L
        carr = np.mod(sat.carrier_phase(np.float64(s), fs), 2 * np.pi)
        jobs[i]["sample_offset"] = s
        jobs[i]["n_samples"] = vector_length
        jobs[i]["code_id"] = code_id
        jobs[i]["n_taps"] = len(shifts_chips)
        jobs[i]["rem_carrier_phase_rad"] = np.float32(carr)
        jobs[i]["phase_step_rad"] = np.float32(2 * np.pi * (sat.f_if_hz + sat.doppler_hz) / fs)
        jobs[i]["rem_code_phase_chips"] = np.float32(-chip * samples_per_chip)
        jobs[i]["code_phase_step_chips"] = np.float32(fcode / fs * samples_per_chip)
        sh = np.zeros(MAX_TAPS, np.float32)
        sh[: len(shifts_chips)] = np.asarray(shifts_chips, np.float32) * samples_per_chip
        jobs[i]["shifts_chips"] = sh
    return jobs


def random_sky(n_sats: int, seed: int, system: str = "GPS", cn0: float = 45.0, prns=None, dmax: float = 5000.0):
    """Satellites with fD ~ U[±dmax], τ ~ U[0, L), φ ~ U[0, 2π)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    L = SYSTEMS[system][1]
    prns = list(range(1, n_sats + 1)) if prns is None else list(prns)
    return [Satellite(prn=p, doppler_hz=float(rng.uniform(-dmax, dmax)), code_delay_chips=float(rng.uniform(0, L)),
                      carrier_phase_rad=float(rng.uniform(0, 2 * np.pi)), cn0_dbhz=cn0, system=system) for p in prns]


def generate_if_device(fs: float, n_samples: int, sats: list, seed: int = 0, start: int = 0, device: str = "cuda",
                       block: int = 1 << 23, noise: bool = True):
    """generate_if's signal model evaluated on the GPU with torch (bench inputs of many seconds:
    ~100 M samples): returns a complex64 torch tensor on `device`.  Same x[n] as generate_if
    (phases in float64), but the noise comes from torch's generator, so the samples are not
    numpy's; the bench starts its channels from the same truth either way."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(int(seed))
    out = torch.empty(n_samples, dtype=torch.complex64, device=device)
    codes = {}
    for b0 in range(0, n_samples, block):
        b1 = min(n_samples, b0 + block)
        n = torch.arange(start + b0, start + b1, dtype=torch.float64, device=device)
        acc_re = torch.zeros(b1 - b0, dtype=torch.float64, device=device)
        acc_im = torch.zeros_like(acc_re)
        for s in sats:
            key = id(s)
            if key not in codes:
                codes[key] = (torch.as_tensor(np.asarray(s.code, np.float64), device=device),
                              None if s.code_data is None else torch.as_tensor(np.asarray(s.code_data, np.float64), device=device))
            code, code_d = codes[key]
            amp = float(np.sqrt(2.0 * 10.0 ** (s.cn0_dbhz / 10.0) / fs))
            rate, _, fc, _ = SYSTEMS[s.system]
            ph = n / fs * s.code_freq() - s.code_delay_chips
            if s.doppler_rate_hz_s:
                ph = ph + 0.5 * rate * s.doppler_rate_hz_s / fc * (n / fs) ** 2
            chip = torch.floor(ph).to(torch.int64)
            idx = torch.remainder(chip, s.code_len)
            c = code[idx]
            period = torch.div(chip, s.code_len, rounding_mode="floor")
            if s.secondary:
                sec = torch.as_tensor([1.0 if b == "0" else -1.0 for b in s.secondary], dtype=torch.float64, device=device)
                c = c * sec[torch.remainder(period, len(sec))]
            sign = 1.0
            if s.bits:
                pat = torch.as_tensor([1.0 if b == "0" else -1.0 for b in s.bits], dtype=torch.float64, device=device)
                per_bit = s.symbols_per_bit or (1 if code_d is not None else 20)
                sign = pat[torch.remainder(torch.div(period, per_bit, rounding_mode="floor"), len(pat))]
            if code_d is not None:
                c = (sign * code_d[idx] - c) / np.sqrt(2.0)
            else:
                c = c * sign
            cp = 2.0 * np.pi * (s.f_if_hz + s.doppler_hz) * (n / fs) + s.carrier_phase_rad
            if s.doppler_rate_hz_s:
                cp = cp + np.pi * s.doppler_rate_hz_s * (n / fs) ** 2
            acc_re += amp * c * torch.cos(cp)
            acc_im += amp * c * torch.sin(cp)
        if noise:
            acc_re += torch.randn(b1 - b0, generator=g, dtype=torch.float64, device=device)
            acc_im += torch.randn(b1 - b0, generator=g, dtype=torch.float64, device=device)
        out[b0:b1] = torch.complex(acc_re.to(torch.float32), acc_im.to(torch.float32))
    return out


def acq_delay_samples(sat: Satellite, fs: float, stamp: int, first: int) -> float:
    """Acq_delay_samples as an acquisition stamped at sample `stamp` reports it for a channel whose
    tracking starts at `first`: the first code start at or after `first` (with code Doppler),
    relative to the stamp modulo the nominal code period (pcps_acquisition.cc:693)."""
    m = np.ceil(sat.chip_phase(np.float64(first), fs) / sat.code_len)
    n0 = (m * sat.code_len + sat.code_delay_chips) * fs / sat.code_freq()
    rate, L, _, _ = SYSTEMS[sat.system]
    t_nom = L / rate * fs
    return (first - stamp) + float(np.mod(n0 - first, t_nom))


def c3_sky(cn0: float = 45.0):
    """a 32-PRN all-sky sweep at 25 Msps with 10 PRNs present (seed 0x6E550003);
    which 10 is drawn from the same seed."""
    seed = 0x6E550003
    rng = np.random.Generator(np.random.PCG64(seed))
    prns = sorted(int(p) for p in rng.choice(np.arange(1, 33), 10, replace=False))
    return random_sky(10, seed=seed, cn0=cn0, prns=prns)


def c1_sky(cn0: float = 45.0, extra=()):
    """BASELINE.md / SURVEY §8d C1: GPS PRN 7 at fD = 1730 Hz with its code delayed 1234 samples at
    4 Msps (315.6 chips), GPS navigation bits (the TLM preamble pattern, so bit synchronisation
    completes); `extra`: more satellites (prn, doppler_hz, delay_samples) for multi-channel runs."""
    fs = 4e6
    sats = []
    for prn, fd, delay in ((7, 1730.0, 1234.0),) + tuple(extra):
        s = Satellite(prn=prn, doppler_hz=fd, code_delay_chips=delay * 1.023e6 / fs, carrier_phase_rad=0.7, cn0_dbhz=cn0)
        s.bits = "1000101100110"
        sats.append(s)
    return sats

"""Synthetic tracking scenarios shared by the oracle (CPU) and device (GPU) loop tests."""
import numpy as np

from gnss_sim_receiver_amd import signals
from oracle import trk as T


def acq_delay_for(sat, fs, system, stamp, first):
    """Acq_delay_samples as a fresh acquisition would report it: the code start nearest after
    `first` (with code Doppler), relative to the stamp modulo the nominal code period."""
    m = np.ceil(sat.chip_phase(np.float64(first), fs) / sat.code_len)
    n0 = (m * sat.code_len + sat.code_delay_chips) * fs / sat.code_freq()
    t_nom = T.SYSTEMS[system][2] * fs
    return (first - stamp) + np.mod(n0 - first, t_nom)


def pull_in(system, fs, cn0, dop, delay_chips, dop_err, delay_err_samples, epochs, prn=7, seed=11, **conf_kw):
    """Acquisition at sample 0 with errors; tracking starts at sample 0 (pull-in transitory on)."""
    sat = signals.Satellite(prn=prn, doppler_hz=dop, code_delay_chips=delay_chips, cn0_dbhz=cn0, system=system, carrier_phase_rad=0.4)
    k = T.conf(system, fs, int(round(fs * T.SYSTEMS[system][2])), **conf_kw)
    x = signals.generate_if(fs, k.vector_length * (epochs + 3), [sat], seed=seed)
    delay = (sat.code_delay_chips / sat.code_freq()) * fs + delay_err_samples
    return sat, k, x, 0, 0, delay, dop + dop_err


SYNC_PATTERNS = {"GPS": dict(bits="1000101100110"), "GAL": dict(secondary=T.E1C_SECONDARY, bits="0110"),
                 "BDS": dict(secondary=T.B1I_NH, bits="0111"),
                 # GEO D2: the 11-bit preamble 11100010010 at 2 code periods per bit, no NH code
                 "BDS_GEO": dict(bits="111000100100110", symbols_per_bit=2)}


def sync(system, fs, epochs, prn=9, dop=1210.0, delay_chips=100.3, seed=5, cn0=50.0, rate_hz_s=0.0, f_if_hz=0.0, **conf_kw):
    """A signal carrying the pattern the block synchronises on (GPS navigation bits with the
    10001011 preamble, CS25 on the E1-C pilot, the B1I NH code), acquisition stamped one second
    before tracking starts so that pull_in_time_s = 0 ends the pull-in at once.  x[0] is absolute
    sample `first` = fs.  rate_hz_s: Doppler ramp (the acquisition reports the Doppler at `first`).
    f_if_hz: the signal sits at this IF in the buffer (C5's front end), the loop's conf carries it."""
    geo = system == "BDS" and T.is_bds_geo(prn)
    sat = signals.Satellite(prn=prn, doppler_hz=dop, code_delay_chips=delay_chips, cn0_dbhz=cn0, system=system, carrier_phase_rad=1.0,
                            doppler_rate_hz_s=rate_hz_s, f_if_hz=f_if_hz, **SYNC_PATTERNS["BDS_GEO" if geo else system])
    kw = dict(pull_in_time_s=0, if_hz=f_if_hz)
    kw.update(conf_kw)
    k = T.conf(system, fs, int(round(fs * T.SYSTEMS[system][2])), prn=prn, **kw)
    first = int(fs)
    x = signals.generate_if(fs, int(round(fs)) // 4 + k.vector_length * (epochs + 3), [sat], seed=seed, start=first)
    return sat, k, x, 0, first, acq_delay_for(sat, fs, system, 0, first) + 0.2, sat.doppler_hz + rate_hz_s + 15.0


def code_tracking_error_chips(sat, fs, rec, system):
    """Local replica phase at each epoch start (−rem_code_phase of the previous update, in chips)
    minus the received code phase there, wrapped to ±L/2 (chips of the ranging code)."""
    per_chip = 2.0 if system == "GAL" else 1.0  # GAL synthetic phase is in sinBOC replica samples
    L = sat.code_len / per_chip
    truth = np.array([sat.chip_phase(np.float64(s), fs) for s in rec["sample_counter"][1:]]) / per_chip
    local = -rec["rem_code_phase_chips"][:-1]
    return np.mod(local - truth + L / 2, L) - L / 2

"""Galileo E1 code tables (CPU): the ICD memory codes shipped as data, expanded like the reference.

galileo_e1_code_gen_int (galileo_e1_signal_replica.cc:30-58) maps each hex digit of
Galileo_E1.h:56/:760 MSB-first to four chips (0 → +1, 1 → −1); sinboc11_float (:98-108) writes
[c, −c] per chip.  The reference generator itself is not buildable here (gnss_signal_replica.cc
includes GNU Radio's fxpt_nco.h), so the tables are pinned by their hex heads below — the first
digits of E1-B PRN 1 ("F5D7…") and E1-C PRN 1 ("B393…") — and by code properties.
"""
import numpy as np

from gnss_sim_receiver_amd import codes as C


def hexchips(h):
    return np.array([1 - 2 * ((int(c, 16) >> s) & 1) for c in h for s in (3, 2, 1, 0)], np.int32)


def test_e1_hex_heads():
    assert np.array_equal(C.galileo_e1_code_gen_int("1B", 1)[:16], hexchips("F5D7"))
    assert np.array_equal(C.galileo_e1_code_gen_int("1C", 1)[:16], hexchips("B393"))


def test_e1_code_properties():
    for sig in ("1B", "1C"):
        codes = np.array([C.galileo_e1_code_gen_int(sig, p) for p in range(1, 51)]).astype(np.float64)
        assert codes.shape == (50, 4092) and set(np.unique(codes)) == {-1.0, 1.0}
        assert np.all(np.abs(codes.sum(axis=1)) <= 64)  # memory codes are balanced
        f = np.fft.fft(codes, axis=1)
        auto = np.abs(np.fft.ifft(f * np.conj(f), axis=1)).real
        assert np.allclose(auto[:, 0], 4092) and auto[:, 1:].max() < 300
        cross = np.abs(np.fft.ifft(f[0] * np.conj(f[1:]), axis=1))
        assert cross.max() < 300
    b = C.galileo_e1_code_gen_int("1B", 7)
    c = C.galileo_e1_code_gen_int("1C", 7)
    assert not np.array_equal(b, c)


def test_e1_sinboc_and_edges():
    s = C.galileo_e1_code_gen_sinboc11_float("1C", 11)
    c = C.galileo_e1_code_gen_int("1C", 11)
    assert s.dtype == np.float32 and len(s) == 8184
    assert np.array_equal(s[0::2], c) and np.array_equal(s[1::2], -c)
    assert not C.galileo_e1_code_gen_int("1B", 0).any() and not C.galileo_e1_code_gen_int("1B", 51).any()
    assert not C.galileo_e1_code_gen_int("5X", 3).any()
    sec = C.galileo_e1_c_secondary_code()
    assert len(sec) == 25 and np.array_equal(sec[:5], [1, 1, -1, -1, -1])  # "00111…" (Galileo_E1.h:52)

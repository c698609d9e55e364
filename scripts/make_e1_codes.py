"""Extract the Galileo E1-B / E1-C primary codes and the E1-C secondary code as DATA.

    python scripts/make_e1_codes.py   # build container only (/root/reference present)

The codes are the Galileo OS SIS ICD memory codes (4092 chips per PRN, 50 PRNs per component).
The reference ships them as hex strings in src/core/system_parameters/Galileo_E1.h:56 (E1-B) and
:760 (E1-C), with the 25-chip E1-C secondary code at :52.  Its generator
(galileo_e1_signal_replica.cc:30-58 → hex_to_binary_converter, gnss_signal_replica.cc:43) maps each
hex digit MSB-first to four chips, bit 0 → +1, bit 1 → −1.  That generator cannot be compiled here
(gnss_signal_replica.cc needs GNU Radio's fxpt_nco.h), so this script reads the header as text and
stores the chip BITS (np.packbits, 1 = chip −1) in gnss_sim_receiver_amd/data/galileo_e1_codes.npz.
"""
import hashlib
import os
import re

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = "/root/reference/src/core/system_parameters/Galileo_E1.h"
OUT = os.path.join(ROOT, "gnss_sim_receiver_amd", "data", "galileo_e1_codes.npz")


def table(text, name):
    m = re.search(name + r"\[[^\]]*\]\[[^\]]*\]\s*=\s*\{(.*?)\};", text, re.S)
    # a PRN row is a run of adjacent string literals (C concatenation) closed by a comma
    rows, cur = [], ""
    for lit, comma in re.findall(r'"([0-9A-F]*)"\s*(,?)', m.group(1)):
        cur += lit
        if comma:
            rows.append(cur)
            cur = ""
    if cur:
        rows.append(cur)
    assert len(rows) == 50 and all(len(r) == 1023 for r in rows), (name, len(rows))
    bits = np.array([[int(c, 16) >> s & 1 for c in r for s in (3, 2, 1, 0)] for r in rows], np.uint8)
    assert bits.shape == (50, 4092)
    return bits, hashlib.sha256("".join(rows).encode()).hexdigest()


def main():
    text = open(HDR).read()
    b, hb = table(text, "GALILEO_E1_B_PRIMARY_CODE")
    c, hc = table(text, "GALILEO_E1_C_PRIMARY_CODE")
    sec = re.search(r'GALILEO_E1_C_SECONDARY_CODE\[\d+\]\s*=\s*"([01]+)"', text).group(1)
    assert len(sec) == 25
    np.savez_compressed(OUT, e1b_bits=np.packbits(b, axis=1), e1c_bits=np.packbits(c, axis=1),
                        e1c_secondary_bits=np.array([int(x) for x in sec], np.uint8),
                        provenance=np.array(f"Galileo_E1.h hex tables; sha256(E1B hex)={hb}; sha256(E1C hex)={hc}"))
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()

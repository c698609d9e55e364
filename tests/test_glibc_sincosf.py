"""The device's libm restatements (gnss_sim_receiver_amd/csrc/glibc_sincosf.h, glibc_atanf.h, glibc_logf.h) against
this host's own glibc, bit for bit: the tracking engines' carrier phasors are the reference's
(cos rem, −sin rem) and exp(−j·step) (cpu_multicorrelator_real_codes.cc:115,123 → glibc cosf / sinf /
cexpf → __sincosf), the loop's discriminators its atanf / atan2f (tracking_discriminators.cc:
68-104), and the CN0 estimate its log10f (lock_detectors.cc:119, log10f → the ifunc'd FMA logf).  The headers are compiled for the host (tests/cpp/glibc_sincosf_check.cpp, -ffp-contract=off,
as the device objects are built) and compared with sinf / cosf / sincosf / atanf / atan2f on:
  * every float in [0.5, 1) (8.4 M: the C5 steps' binade) and in [2^-8, 2^-7) (the C2 steps' binade),
  * 5 M uniform in ±7 rad (rem_carr after fmod(·, 2π), IF folded in),
  * 5 M uniform over the C5 IF steps ±2π(7.161 MHz ± 5 kHz)/50 MHz and 3 M over C2's ±2π·5 kHz/4 MHz,
  * 5 M random bit patterns (the whole float line: the large-argument reduction, tiny and special values);
≥ 20 M arguments in all.  glibc picks its FMA build of sinf/cosf on FMA hosts (every AVX2 server,
the GPU box's EPYC included); the restatement is that build, so the test requires FMA.
(One-off exhaustive runs here: every float with |x| < 120 for sin/cos — 2.25e9 arguments — every float
for atanf / atan2f and every positive float for logf / log10f, 0 mismatches)"""
import math
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "glibc_sincosf_check.cpp")


# The headers restate glibc 2.35's float routines (the GPU box's and this container's glibc).  Later
# releases replaced some of them, so on another glibc the comparison says nothing about the headers.
RESTATED_GLIBC = "2.35"


def host_glibc():
    import ctypes

    fn = ctypes.CDLL(None).gnu_get_libc_version
    fn.restype = ctypes.c_char_p
    return fn().decode()


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    if host_glibc() != RESTATED_GLIBC:
        pytest.skip(f"host glibc {host_glibc()}: the device headers restate glibc {RESTATED_GLIBC}'s float libm")
    exe = str(tmp_path_factory.mktemp("gsc") / "glibc_sincosf_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-pthread", SRC, "-o", exe, "-lm"], check=True)
    if subprocess.run([exe, "fma"], capture_output=True, text=True, check=True).stdout.strip() != "1":
        pytest.skip("host without FMA: glibc runs its non-FMA sinf/cosf build, which the device does not restate")
    return exe


def run(exe, *args, fn=None):
    env = dict(os.environ)
    if fn:
        env["FN"] = fn
    out = subprocess.run([exe, *map(str, args)], capture_output=True, text=True, env=env, timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr
    n = int(out.stdout.split("checked")[-1].split()[0])
    return n


def f32_bits(x):
    import struct
    return struct.unpack("<I", struct.pack("<f", x))[0]


def test_sincosf_matches_host_glibc(checker):
    n = 0
    n += run(checker, "range", f32_bits(0.5), f32_bits(1.0))
    n += run(checker, "range", f32_bits(2.0 ** -8), f32_bits(2.0 ** -7))
    n += run(checker, "uniform", 5_000_000, 1, -7.0, 7.0)
    c5_lo, c5_hi = 2 * math.pi * (7.161e6 - 5e3) / 50e6, 2 * math.pi * (7.161e6 + 5e3) / 50e6
    n += run(checker, "uniform", 2_500_000, 2, c5_lo, c5_hi)
    n += run(checker, "uniform", 2_500_000, 3, -c5_hi, -c5_lo)
    c2 = 2 * math.pi * 5e3 / 4e6
    n += run(checker, "uniform", 3_000_000, 4, -c2, c2)
    n += run(checker, "random", 5_000_000, 5)
    assert n >= 20_000_000


def test_atanf_atan2f_match_host_glibc(checker):
    n = 0
    n += run(checker, "uniform", 5_000_000, 11, -4.0, 4.0, fn="atan")
    n += run(checker, "random", 5_000_000, 12, fn="atan")
    n += run(checker, "range", f32_bits(0.4375), f32_bits(2.4375), fn="atan")
    assert n >= 10_000_000


def test_logf_log10f_match_host_glibc(checker):
    n = 0
    n += run(checker, "uniform", 5_000_000, 21, 1e-3, 1e6, fn="log")  # SNR and coherent-time arguments
    n += run(checker, "random", 5_000_000, 22, fn="log")
    n += run(checker, "range", f32_bits(0.5), f32_bits(2.0), fn="log")
    assert n >= 10_000_000

"""gnsship_rotator_dispatch mirrors volk_gnsssdr's choice of rotator variant (volk_gnsssdr_rank_archs.c:
VOLK_GENERIC → generic; a preferences-file entry → that entry (volk_gnsssdr_prefs.c); otherwise the
best variant the CPU supports).  Host-only, no GPU; each case runs in a child process so that the
environment it sets up is the one the library reads."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = ("import sys; sys.path.insert(0, %r); from gnss_sim_receiver_amd import abi\n"
        "try:\n    print(abi.rotator_dispatch())\nexcept abi.GnssHipError as e:\n    print('ERR', e)\n"
        "print(abi.rotator_dispatch_detail())") % ROOT


def dispatch_full(env_extra, tmp_path):
    env = {k: v for k, v in os.environ.items() if k not in ("VOLK_GENERIC", "VOLK_CONFIGPATH")}
    env["HOME"] = str(tmp_path)
    env.update(env_extra)
    out = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    lines = out.stdout.strip().splitlines()
    return lines[-2], lines[-1]


def dispatch(env_extra, tmp_path):
    v, _ = dispatch_full(env_extra, tmp_path)
    return int(v)


def has_avx():
    with open("/proc/cpuinfo") as f:
        return any(" avx " in (" " + line.split(":", 1)[-1].strip() + " ") for line in f if line.startswith("flags"))


def test_default_follows_cpu(tmp_path):
    assert dispatch({}, tmp_path) == (1 if has_avx() else 0)


def test_volk_generic_env_forces_generic(tmp_path):
    assert dispatch({"VOLK_GENERIC": "1"}, tmp_path) == 0


@pytest.mark.parametrize("impl,expect", [("generic", 0), ("u_avx", 1)])
def test_preferences_file_entry(tmp_path, impl, expect):
    d = tmp_path / ".volk_gnsssdr"
    d.mkdir()
    (d / "volk_gnsssdr_config").write_text(
        "volk_gnsssdr_32f_xn_resampler_32f_xn generic generic\n"
        f"volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn {impl.replace('u_', 'a_')} {impl}\n")
    v, detail = dispatch_full({}, tmp_path)
    assert int(v) == expect
    assert "volk_gnsssdr_config" in detail and impl in detail


@pytest.mark.parametrize("impl_a,impl_u", [("generic_reload", "generic_reload"), ("a_sse3", "u_sse3"), ("a_avx", "generic")])
def test_preferences_entry_not_reproduced_is_an_error(tmp_path, impl_a, impl_u):
    """generic_reload renormalises after every 256 samples (a different recursion), SSE variants are
    not restated, and an aligned/unaligned pair naming different variants is ambiguous: reported, not
    mapped to the nearest variant."""
    d = tmp_path / ".volk_gnsssdr"
    d.mkdir()
    (d / "volk_gnsssdr_config").write_text(f"volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn {impl_a} {impl_u}\n")
    v, detail = dispatch_full({}, tmp_path)
    assert v.startswith("ERR") and impl_u in v
    assert "not a variant the engine reproduces" in detail


def test_configpath_takes_precedence(tmp_path):
    home = tmp_path / ".volk_gnsssdr"
    home.mkdir()
    (home / "volk_gnsssdr_config").write_text("volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn a_avx u_avx\n")
    cp = tmp_path / "cfg" / "volk_gnsssdr"
    cp.mkdir(parents=True)
    (cp / "volk_gnsssdr_config").write_text("volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn generic generic\n")
    assert dispatch({"VOLK_CONFIGPATH": str(tmp_path / "cfg")}, tmp_path) == 0

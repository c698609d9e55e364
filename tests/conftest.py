import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libgnsship.so on cuda:0)")


@pytest.fixture(scope="session", autouse=True)
def _torch_hip_first(request):
    """torch's HIP runtime is initialised before libgnsship's in every GPU run, whichever test comes
    first (a module that loads libgnsship before the `ctx` fixture did otherwise leave the context
    creation that follows with no device)."""
    if any(item.get_closest_marker("gpu") for item in request.session.items):
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    yield


@pytest.fixture(scope="session")
def built():
    """Make sure libgnsship.so and the oracle exist (gcc/hipcc cross-compile, no GPU needed)."""
    import subprocess
    lib = os.path.join(ROOT, "gnss_sim_receiver_amd", "libgnsship.so")
    orc = os.path.join(ROOT, "oracle", "liboracle.so")
    if not (os.path.exists(lib) and os.path.exists(orc)):
        subprocess.run(["make", "-s", "-C", ROOT, "all"], check=True)
    return True


@pytest.fixture(scope="session")
def ctx(built):
    # torch's HIP runtime (its own libamdhip64) is initialised before libgnsship's, as bench.py does:
    # initialised second it finds no device, and the tests that generate long IF records on the GPU
    # (test_gpu_c5_closed_loop.if_on_device) need it
    import torch
    if torch.cuda.is_available():
        torch.cuda.init()
    from gnss_sim_receiver_amd import engine
    c = engine.Context(0)
    yield c
    c.close()

"""gnss_sim_receiver_amd — MI355X-native GNSS acquisition + tracking correlator engine.

The compute lives in libgnsship.so (HIP kernels for gfx950 behind the C ABI of include/gnsship.h).
This package holds the Python handles over that ABI (engine, codes) and the synthetic IF
generator used by the tests and the benchmark.
"""
from . import abi  # noqa: F401

__version__ = "0.1.0"

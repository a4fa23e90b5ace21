"""TEST INFRASTRUCTURE ONLY -- ctypes binding of the CPU oracle (liboracle.so).

The oracle is the checker the GPU path is compared against; only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg import this package.
"""
from .py import OracleDecoder, lib, load, PAD_Y, PAD_C, plane_stride  # noqa: F401

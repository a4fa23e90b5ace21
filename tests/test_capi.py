"""The C-ABI library builds for gfx950, loads without a GPU and exports every
symbol the public headers declare (no compute calls here)."""
import ctypes
import os
import re

from thor_amd import lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = re.findall(r"\b([a-z_][a-z0-9_]*)\s*\(", txt)
    skip = {"if", "while", "for", "return", "sizeof"}
    return sorted({n for n in names if n not in skip and not n.startswith("__")})


def test_library_loads_and_exports_batched_api():
    lib = L.load()
    for name in _declared("thor_amd.h"):
        assert hasattr(lib, name), name
    for name in L.BATCHED_SYMBOLS:
        assert hasattr(lib, name), name
    # the reference's SIMD kernel surface (common/common_kernels.h:31-41, enc/enc_kernels.h:32-37)
    declared = _declared("thor_kernels.h")
    assert set(declared) == set(L.SIMD_SURFACE_SYMBOLS)
    for name in declared:
        assert hasattr(lib, name), name
    assert b"gfx950" in lib.thor_version()


def test_block_descriptor_layout_matches_header():
    from thor_amd.trace import BLOCK_DTYPE

    assert BLOCK_DTYPE.itemsize == 72
    assert BLOCK_DTYPE.fields["mv0"][1] == 20
    assert BLOCK_DTYPE.fields["coeff_off"][1] == 60


def test_build_intra_list_host_helper():
    import numpy as np
    from thor_amd.trace import BLOCK_DTYPE

    lib = L.load()
    b = np.zeros(5, BLOCK_DTYPE)
    b["mode"] = [0, 1, 2, 1, 4]
    out = np.zeros(5, np.uint32)
    n = lib.thor_build_intra_list(b.ctypes.data, 5, out.ctypes.data)
    assert n == 2 and out[:2].tolist() == [1, 3]

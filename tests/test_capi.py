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
    # the reference's block / frame reconstruction entry points
    declared = _declared("thor_l2.h")
    assert set(declared) == set(L.L2_SURFACE_SYMBOLS)
    for name in declared:
        assert hasattr(lib, name), name
    assert b"gfx950" in lib.thor_version()


def test_l2_struct_layouts_match_reference():
    """thor_ref_yuv_frame_t / thor_ref_deblock_data_t mirror yuv_frame_t and
    deblock_data_t (common/types.h:41-59, :127-135; 44-byte deblock_data_t,
    SURVEY.md sec. 8(a) a16)."""
    import ctypes as C

    class Mv(C.Structure):
        _fields_ = [("x", C.c_int16), ("y", C.c_int16)]

    class Ip(C.Structure):
        _fields_ = [("mv0", Mv), ("mv1", Mv), ("ref_idx0", C.c_uint32), ("ref_idx1", C.c_uint32),
                    ("bipred_flag", C.c_uint32)]

    class Dd(C.Structure):
        _fields_ = [("mode", C.c_int32), ("cbp_y", C.c_int32), ("cbp_u", C.c_int32), ("cbp_v", C.c_int32),
                    ("size", C.c_uint8), ("tb_split", C.c_uint8), ("pb_part", C.c_int32), ("inter_pred", Ip)]

    assert C.sizeof(Dd) == 44 and Dd.pb_part.offset == 20 and Dd.inter_pred.offset == 24


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


def test_build_tu_list_host_helper():
    """thor_build_tu_list: one 12-byte entry per coded TU (tb-split quarters in
    raster order, 8x8 chroma unsplit, chroma qp mapped), SKIP never listed."""
    import numpy as np
    from thor_amd.decoder import TU_DTYPE
    from thor_amd.trace import BLOCK_DTYPE

    assert TU_DTYPE.itemsize == 12
    lib = L.load()
    b = np.zeros(3, BLOCK_DTYPE)
    b[0] = 0
    b["mode"] = [0, 2, 1]
    b["coeff_mask"] = [7, 7, 1]
    b["size"] = [64, 16, 8]
    b["tb_split"] = [0, 1, 1]
    b["ypos"], b["xpos"] = [0, 64, 80], [0, 32, 48]
    b["qp"] = [40, 40, 20]
    b["coeff_off"] = [[0, 0, 0], [100, 400, 500], [900, 0, 0]]
    n = lib.thor_build_tu_list(b.ctypes.data, 3, None)
    out = np.zeros(n, TU_DTYPE)
    assert lib.thor_build_tu_list(b.ctypes.data, 3, out.ctypes.data) == n == 4 + 4 + 4 + 4
    # CU 1 (16x16, tb split): luma quarters 8x8 with q = 8 -> offsets 100 + 64 t
    assert out[:4]["coeff_off"].tolist() == [100, 164, 228, 292]
    assert [(int(t["y"]), int(t["x"])) for t in out[:4]] == [(64, 32), (64, 40), (72, 32), (72, 40)]
    assert out[4]["comp"] == 1 and out[4]["size"] == 4 and out[4]["qp"] == 36 and (out[4]["y"], out[4]["x"]) == (32, 16)
    # CU 2 (8x8 intra, tb split): four 4x4 luma TUs, q = 4
    assert out[12:]["coeff_off"].tolist() == [900, 916, 932, 948] and set(out[12:]["size"]) == {4}

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


def _slow_units_py(b, W, H):
    """numpy restatement of the multi-key half classification (recon.hip prep_body)
    -> the set of k_recon units (128x16 luma) holding such a half."""
    sbw, sbh = (W + 63) // 64, (H + 63) // 64
    np_ = (sbw + 1) // 2
    slow = set()
    for B in b:
        if B["mode"] == 1:
            continue
        sbx, sby = int(B["xpos"]) // 64, int(B["ypos"]) // 64
        if int(B["size"]) < 64:
            slow.add((sbx, sby, int(int(B["ypos"]) % 64 >= 32)))
            continue
        quarters = B["mode"] in (2, 3)
        bi = B["mode"] == 3 or (B["mode"] in (0, 4) and B["dir"] == 2)
        m0, m1 = B["mv0"].reshape(4, 2), B["mv1"].reshape(4, 2)
        for h in range(2):
            q0, q1 = (2 * h, 2 * h + 1) if quarters else (0, 0)
            same = (m0[q0] == m0[q1]).all() and (not bi or (m1[q0] == m1[q1]).all())
            if not same and int(B["ypos"]) + 32 * h < H:
                slow.add((sbx, sby, h))
    return sorted({(4 * sby + 2 * h + j) * np_ + sbx // 2 for (sbx, sby, h) in slow for j in range(2)})


def test_build_slow_list_host_helper():
    """thor_build_slow_list == the numpy restatement on hand-made CUs and on every
    frame of golden streams (the reference encoder's .bit, host-parsed)."""
    import numpy as np
    from thor_amd.bitstream import parse_stream
    from thor_amd.trace import BLOCK_DTYPE

    lib = L.load()

    def host(b, W, H):
        b = np.ascontiguousarray(b, dtype=BLOCK_DTYPE)
        n = lib.thor_build_slow_list(b.ctypes.data, len(b), W, H, None)
        out = np.zeros(max(n, 1), np.uint32)
        assert lib.thor_build_slow_list(b.ctypes.data, len(b), W, H, out.ctypes.data) == n
        return out[:n].tolist()

    b = np.zeros(4, BLOCK_DTYPE)
    b["mode"] = [2, 0, 1, 3]
    b["size"] = [64, 64, 32, 64]
    b["xpos"], b["ypos"] = [0, 64, 128, 192], [0, 0, 0, 64]
    b["mv0"][0] = [4, 0, 4, 0, 8, 0, 4, 0]  # INTER 64x64: quarters 2 and 3 differ -> half 1 multi-key
    b["mv0"][3][0] = 2  # BIPRED 64x64 at SB (3, 1): quarter 0 differs from 1 -> half 0
    got = host(b, 256, 128)
    assert got == _slow_units_py(b, 256, 128)
    assert got == [2 * 2 + 0, 3 * 2 + 0, (4 + 0) * 2 + 1, (4 + 1) * 2 + 1]
    assert host(b[:0], 256, 128) == []
    assert lib.thor_build_slow_list(None, 3, 256, 128, None) < 0
    for name in ("cif_high.bit", "hd_low.bit", "k4_med.bit", "cif_hdb.bit"):
        seq, frames = parse_stream(open(os.path.join(ROOT, "tests", "golden", name), "rb").read())
        for fr in frames:
            assert host(fr.blocks, seq.width, seq.height) == _slow_units_py(fr.blocks, seq.width, seq.height), name


def test_frame_image_matches_the_host_lists():
    """thor_frame_image: one 256-aligned host image of a parsed frame whose parts
    equal the parse output and the thor_build_* lists (the native form of
    GpuDecoder.upload's image)."""
    import ctypes as C

    import numpy as np
    from thor_amd.bitstream import split_chunks
    from thor_amd.decoder import TU_DTYPE
    from thor_amd.trace import BLOCK_DTYPE

    lib = L.load()
    for name in ("cif_high.bit", "k4_med.bit"):
        p = lib.thor_parser_create()
        try:
            for payload in split_chunks(open(os.path.join(ROOT, "tests", "golden", name), "rb").read()):
                out = L.ThorParsedFrame()
                buf = C.create_string_buffer(payload, len(payload))
                assert lib.thor_parse_frame(p, buf, len(payload), C.byref(out)) == 0
                lay = L.ThorFrameImage()
                assert lib.thor_frame_image(C.byref(out), None, 0, C.byref(lay)) == L.THOR_ERR_NOMEM
                img = np.zeros(lay.bytes, np.uint8)
                assert lib.thor_frame_image(C.byref(out), img.ctypes.data, img.nbytes, C.byref(lay)) == 0
                nb = out.nblocks
                blocks = np.frombuffer((C.c_uint8 * (nb * 72)).from_address(out.blocks), BLOCK_DTYPE).copy()
                assert img[lay.off_blocks:lay.off_blocks + nb * 72].tobytes() == blocks.tobytes()
                coeffs = np.frombuffer((C.c_int16 * out.ncoeffs).from_address(out.coeffs), np.int16)
                assert np.array_equal(img[lay.off_coeffs:lay.off_coeffs + 2 * out.ncoeffs].view(np.int16), coeffs)
                n = lib.thor_build_tu_list(blocks.ctypes.data, nb, None)
                tus = np.zeros(max(n, 1), TU_DTYPE)
                lib.thor_build_tu_list(blocks.ctypes.data, nb, tus.ctypes.data)
                assert lay.n_tu == n and img[lay.off_tus:lay.off_tus + 12 * n].tobytes() == tus[:n].tobytes()
                n = lib.thor_build_slow_list(blocks.ctypes.data, nb, out.seq.width, out.seq.height, None)
                sl = np.zeros(max(n, 1), np.uint32)
                lib.thor_build_slow_list(blocks.ctypes.data, nb, out.seq.width, out.seq.height, sl.ctypes.data)
                assert lay.n_slow == n and np.array_equal(img[lay.off_slow:lay.off_slow + 4 * n].view(np.uint32), sl[:n])
                if out.hdr.clpf_on:
                    assert lay.n_flags == out.nclpf and lay.n_clpf >= 0
                else:
                    assert lay.n_flags == 0 and lay.n_clpf == -1
                for off in (lay.off_blocks, lay.off_coeffs, lay.off_flags, lay.off_intra, lay.off_tus, lay.off_clpf,
                            lay.off_slow):
                    assert off % 256 == 0
        finally:
            lib.thor_parser_destroy(p)

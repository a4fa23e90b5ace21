"""The L2 entry points (include/thor_l2.h) on the GPU against the reference:
deblock_frame_y / _uv against the reference's own deblocking of seeded frames
with random CU tilings (tests/golden/l2_deblock.npz), make_top_and_left +
get_intra_prediction against the reference's intra vectors (kernels.npz),
dequantize / quantize against the reference's vectors, reconstruct_block
against its definition, tb-split neighbour gathers against the oracle."""
import ctypes as C
import os

import numpy as np
import pytest

from conftest import GOLD

pytestmark = pytest.mark.gpu
K = np.load(os.path.join(GOLD, "kernels.npz"))


def _lib():
    from thor_amd import lib as L

    lib = L.load()
    P, i = C.c_void_p, C.c_int
    lib.deblock_frame_y.argtypes = [P, P, i, i, C.c_uint8]
    lib.deblock_frame_uv.argtypes = [P, P, i, i, C.c_uint8]
    lib.make_top_and_left.argtypes = [P, P, P, P, i, P, i, i, i, i, i, i, i, i, i]
    lib.get_intra_prediction.argtypes = [P, P, C.c_uint8, i, i, i, P, i]
    lib.dequantize.argtypes = [P, P, i, i]
    lib.reconstruct_block.argtypes = [P, P, P, i, i]
    lib.quantize.argtypes = [P, P, i, i, i, i]
    lib.quantize.restype = i
    return lib


class Yuv(C.Structure):  # yuv_frame_t / thor_ref_yuv_frame_t
    _fields_ = [("y", C.c_void_p), ("u", C.c_void_p), ("v", C.c_void_p)] + \
        [(n, C.c_int) for n in ("width", "height", "stride_y", "stride_c", "offset_y", "offset_c", "pad_hor_y",
                                "pad_hor_c", "pad_ver_y", "pad_ver_c", "area_y", "area_c", "frame_num")]


@pytest.mark.parametrize("k", range(4))
def test_gpu_deblock_frame_vs_reference(k):
    lib = _lib()
    z = np.load(os.path.join(GOLD, "l2_deblock.npz"))
    w, h, qp, qpc = (int(v) for v in z["dims_%d" % k])
    # planes with strides wider than the frame, as the reference's frames have
    sy, sc = w + 48, w // 2 + 32
    Y = np.zeros((h, sy), np.uint8)
    U = np.zeros((h // 2, sc), np.uint8)
    V = np.zeros((h // 2, sc), np.uint8)
    Y[:, :w], U[:, :w // 2], V[:, :w // 2] = z["in_y_%d" % k], z["in_u_%d" % k], z["in_v_%d" % k]
    f = Yuv(Y.ctypes.data, U.ctypes.data, V.ctypes.data, w, h, sy, sc)
    dd = np.ascontiguousarray(z["dd_%d" % k])
    lib.deblock_frame_y(C.byref(f), dd.ctypes.data, w, h, qp)
    lib.deblock_frame_uv(C.byref(f), dd.ctypes.data, w, h, qpc)
    for nm, p, ww in (("y", Y, w), ("u", U, w // 2), ("v", V, w // 2)):
        want = z["out_%s_%d" % (nm, k)]
        assert np.array_equal(p[:, :ww], want), (k, nm, int((p[:, :ww] != want).sum()))
    assert not Y[:, w:].any() and not U[:, w // 2:].any()  # nothing outside the frame touched


def test_gpu_intra_neighbours_and_prediction_vs_reference():
    lib = _lib()
    frame = np.ascontiguousarray(K["intra_frame"])
    FW = frame.shape[1]
    left = (C.c_uint8 * 160)()
    top = (C.c_uint8 * 160)()
    tl = C.c_uint8()
    off = 0
    for size, ypos, xpos, ur, dl, mode in K["intra_meta"]:
        size, ypos, xpos = int(size), int(ypos), int(xpos)
        want = K["intra_out"][off:off + size * size].reshape(size, size)
        off += size * size
        lp, tp = C.addressof(left) + 1, C.addressof(top) + 1
        lib.make_top_and_left(lp, tp, C.addressof(tl), frame.ctypes.data + ypos * FW + xpos, FW, None, 0, 0, 0, ypos,
                              xpos, size, int(ur), int(dl), 0)
        got = np.zeros((size, size), np.uint8)
        lib.get_intra_prediction(lp, tp, tl.value, ypos, xpos, size, got.ctypes.data, int(mode))
        assert np.array_equal(got, want), (size, ypos, xpos, int(mode))


def test_gpu_make_top_and_left_tb_split_vs_oracle():
    """tb-split sub-TU gathers (rblock, (i, j) offsets; dec/decode_block.c:65):
    the GPU surface against the oracle's restatement on random positions."""
    from oracle.py import load

    lib, olib = _lib(), load()
    rng = np.random.default_rng(5)
    FW = 256
    frame = rng.integers(0, 256, (200, FW), np.uint8)
    for _ in range(300):
        size = int(rng.choice([8, 16, 32, 64]))
        h2 = size // 2
        ypos = int(rng.integers(0, 2)) * 64 + int(rng.integers(0, 64 // size)) * size
        xpos = int(rng.integers(0, 3)) * 64 + int(rng.integers(0, 64 // size)) * size
        i, j = int(rng.integers(0, 2)) * h2, int(rng.integers(0, 2)) * h2
        ur, dl = int(rng.integers(0, 2)), int(rng.integers(0, 2))
        base = frame.ctypes.data + ypos * FW + xpos
        outs = []
        for L in (lib, olib):
            left, top, tl = (C.c_uint8 * 160)(), (C.c_uint8 * 160)(), C.c_uint8()
            fn = L.make_top_and_left if L is lib else L.or_make_top_and_left
            fn(C.addressof(left) + 1, C.addressof(top) + 1, C.addressof(tl), base, FW, base + i * FW + j, FW, i, j,
               ypos, xpos, h2, ur, dl, 1)
            outs.append((bytes(left)[1:1 + 2 * h2], bytes(top)[1:1 + 2 * h2], tl.value))
        assert outs[0] == outs[1], (size, ypos, xpos, i, j, ur, dl)


@pytest.mark.parametrize("size", [4, 8, 16, 32, 64])
def test_gpu_dequantize_and_quantize_vs_reference(size):
    lib = _lib()
    din, dqp, dout = K["dq_%d_in" % size], K["dq_%d_qp" % size], K["dq_%d_out" % size]
    for c, qp, want in zip(din, dqp, dout):
        c = np.ascontiguousarray(c)
        got = np.zeros_like(c)
        lib.dequantize(c.ctypes.data, got.ctypes.data, int(qp), size)
        assert np.array_equal(got, want), (size, int(qp))
    q = min(size, 16)
    for c, qp, typ, want, cbp in zip(K["q_%d_in" % size], K["q_%d_qp" % size], K["q_%d_type" % size],
                                     K["q_%d_out" % size], K["q_%d_cbp" % size]):
        c = np.ascontiguousarray(c)
        got = np.full_like(c, 12345)
        r = lib.quantize(c.ctypes.data, got.ctypes.data, int(qp), size, int(typ), 0)
        assert r == int(cbp), (size, int(qp), int(typ))
        assert np.array_equal(got[:q, :q], want[:q, :q]), (size, int(qp), int(typ))
        assert (got.reshape(size, size)[q:, :] == 12345).all() if size > 16 else True  # outside q x q untouched


def test_gpu_reconstruct_block():
    lib = _lib()
    rng = np.random.default_rng(9)
    for size in (4, 8, 16, 32, 64):
        blk = rng.integers(-300, 300, (size, size)).astype(np.int16)
        pb = rng.integers(0, 256, (size, size)).astype(np.uint8)
        stride = size + 24
        rec = np.full((size, stride), 7, np.uint8)
        lib.reconstruct_block(blk.ctypes.data, pb.ctypes.data, rec.ctypes.data, size, stride)
        assert np.array_equal(rec[:, :size], np.clip(blk.astype(int) + pb, 0, 255).astype(np.uint8))
        assert (rec[:, size:] == 7).all()

"""Temporal-interpolation luma pyramid:
scale_frame_down2x2_simd chained over the levels interpolate_frames builds
(common/temporal_interp.c:977-1019) + pad_yuv_frame on each level.

CPU: the oracle restatement (or_scale_down2x2 + or_pad_plane) and the level
count helper against tests/golden/pyramid.npz (outputs of the reference's own
scale_frame_down2x2_simd, tools/make_pyramid_goldens.py).
GPU: thor_scale_pyramid through the C-ABI against the same goldens, and at 4K
/ 1080p against the oracle (bit-exact, every level including its padding)."""
import ctypes as C
import os

import numpy as np
import pytest

from conftest import GOLD

PAD = 32
GOLDEN = os.path.join(GOLD, "pyramid.npz")


def _cases():
    g = np.load(GOLDEN)
    k = 0
    while "in_%d" % k in g:
        w, h, n = (int(v) for v in g["dims_%d" % k])
        yield g["in_%d" % k], w, h, [g["lvl_%d_%d" % (k, l)] for l in range(1, n + 1)]
        k += 1


def _stride(w):
    return (w + 2 * PAD + 15) & ~15


def oracle_pyramid(img, n):
    """Padded levels (h_l + 64) x (w_l + 64) from the oracle (test infrastructure)."""
    from oracle import py as orc

    OL = orc.lib()
    h, w = img.shape
    prev, ps = np.ascontiguousarray(img), w
    prev_ptr = prev.ctypes.data
    out = []
    for l in range(1, n + 1):
        wl, hl = w >> l, h >> l
        s = _stride(wl)
        buf = np.zeros((hl + 2 * PAD) * s + 16, np.uint8)
        org = buf.ctypes.data + PAD * s + PAD
        OL.or_scale_down2x2(prev_ptr, ps, org, s, wl, hl)
        OL.or_pad_plane(org, s, wl, hl, PAD)
        out.append(buf[:(hl + 2 * PAD) * s].reshape(hl + 2 * PAD, s)[:, :wl + 2 * PAD].copy())
        prev, prev_ptr, ps = buf, org, s
    return out


def test_oracle_pyramid_vs_reference_goldens():
    for img, w, h, levels in _cases():
        got = oracle_pyramid(img, len(levels))
        for l, (a, b) in enumerate(zip(got, levels), 1):
            assert np.array_equal(a, b), "%dx%d level %d" % (w, h, l)


def test_level_count_matches_interpolate_frames():
    from thor_amd import lib as tl

    L = tl.load()
    for _, w, h, levels in _cases():
        assert L.thor_pyramid_levels(w, h) == len(levels)
    # temporal_interp.c:977 at the BASELINE sizes, and the degenerate ones
    assert L.thor_pyramid_levels(3840, 2160) == 3
    assert L.thor_pyramid_levels(1920, 1080) == 3
    assert L.thor_pyramid_levels(64, 64) == 1
    assert L.thor_pyramid_levels(63, 64) == 0
    assert L.thor_pyramid_levels(0, 10) == 0


def _gpu_pyramid(L, img, n):
    """Run thor_scale_pyramid on device copies; return the padded levels."""
    h, w = img.shape
    ss = (w + 15) & ~15
    src = np.zeros((h, ss), np.uint8)
    src[:, :w] = img
    bufs = []
    try:
        dsrc = L.thor_dev_alloc(src.nbytes)
        assert dsrc
        bufs.append(dsrc)
        assert L.thor_h2d(dsrc, src.ctypes.data, src.nbytes) == 0
        ptrs, strides, shapes = [], [], []
        for l in range(1, n + 1):
            wl, hl = w >> l, h >> l
            s = _stride(wl)
            nb = (hl + 2 * PAD) * s
            d = L.thor_dev_alloc(nb)
            assert d
            bufs.append(d)
            ptrs.append(d + PAD * s + PAD)
            strides.append(s)
            shapes.append((hl, wl, s, d, nb))
        parr = (C.c_void_p * 3)(*ptrs)
        sarr = (C.c_int * 3)(*strides)
        rc = L.thor_scale_pyramid(dsrc, ss, w, h, C.cast(parr, C.c_void_p), C.cast(sarr, C.c_void_p), n, None)
        assert rc == 0
        out = []
        for hl, wl, s, d, nb in shapes:
            host = np.empty(nb, np.uint8)
            assert L.thor_d2h(host.ctypes.data, d, nb) == 0
            out.append(host.reshape(hl + 2 * PAD, s)[:, :wl + 2 * PAD].copy())
        return out
    finally:
        for p in bufs:
            L.thor_dev_free(p)


@pytest.mark.gpu
def test_gpu_pyramid_vs_reference_goldens():
    from thor_amd import lib as tl

    L = tl.load()
    for img, w, h, levels in _cases():
        got = _gpu_pyramid(L, img, len(levels))
        for l, (a, b) in enumerate(zip(got, levels), 1):
            assert np.array_equal(a, b), "%dx%d level %d: %d bytes differ" % (w, h, l, int((a != b).sum()))


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,n", [(3840, 2160, 3), (1920, 1080, 3), (1928, 1088, 2), (88, 40, 3)])
def test_gpu_pyramid_vs_oracle(w, h, n):
    from thor_amd import lib as tl

    L = tl.load()
    rng = np.random.default_rng(w * 7 + h)
    img = rng.integers(0, 256, (h, w), dtype=np.uint8)
    got = _gpu_pyramid(L, img, n)
    want = oracle_pyramid(img, n)
    for l, (a, b) in enumerate(zip(got, want), 1):
        assert np.array_equal(a, b), "%dx%d level %d: %d bytes differ" % (w, h, l, int((a != b).sum()))


def test_scale_pyramid_rejects_bad_arguments():
    from thor_amd import lib as tl

    L = tl.load()
    parr = (C.c_void_p * 3)()
    sarr = (C.c_int * 3)(96, 64, 48)
    # argument checks run before any device call
    assert L.thor_scale_pyramid(None, 64, 64, 64, C.cast(parr, C.c_void_p), C.cast(sarr, C.c_void_p), 1, None) == -1
    assert L.thor_scale_pyramid(16, 64, 64, 64, C.cast(parr, C.c_void_p), C.cast(sarr, C.c_void_p), 4, None) == -1
    assert L.thor_scale_pyramid(16, 60, 64, 64, C.cast(parr, C.c_void_p), C.cast(sarr, C.c_void_p), 1, None) == -1
    assert L.thor_scale_pyramid(16, 64, 64, 64, C.cast(parr, C.c_void_p), C.cast(sarr, C.c_void_p), 0, None) == 0


@pytest.mark.gpu
def test_gpu_pyramid2_both_references_vs_oracle():
    """thor_scale_pyramid2: ref0 and ref1 of interpolate_frames in one pair of launches."""
    from thor_amd import lib as tl

    L = tl.load()
    w, h, n = 1928, 1088, 3
    rng = np.random.default_rng(99)
    imgs = [rng.integers(0, 256, (h, w), dtype=np.uint8) for _ in range(2)]
    ss = (w + 15) & ~15
    bufs = []
    try:
        srcs, lv, shapes = [], [], []
        for img in imgs:
            src = np.zeros((h, ss), np.uint8)
            src[:, :w] = img
            d = L.thor_dev_alloc(src.nbytes)
            assert d
            bufs.append(d)
            assert L.thor_h2d(d, src.ctypes.data, src.nbytes) == 0
            srcs.append(d)
            ptrs, shp = [], []
            for l in range(1, n + 1):
                wl, hl = w >> l, h >> l
                s = _stride(wl)
                nb = (hl + 2 * PAD) * s
                dl = L.thor_dev_alloc(nb)
                assert dl
                bufs.append(dl)
                ptrs.append(dl + PAD * s + PAD)
                shp.append((hl, wl, s, dl, nb))
            lv.append((C.c_void_p * 3)(*ptrs))
            shapes.append(shp)
        sarr = (C.c_int * 3)(*[_stride(w >> l) for l in range(1, n + 1)])
        rc = L.thor_scale_pyramid2(srcs[0], srcs[1], ss, w, h, C.cast(lv[0], C.c_void_p), C.cast(lv[1], C.c_void_p),
                                   C.cast(sarr, C.c_void_p), n, None)
        assert rc == 0
        for img, shp in zip(imgs, shapes):
            want = oracle_pyramid(img, n)
            for (hl, wl, s, dl, nb), b in zip(shp, want):
                host = np.empty(nb, np.uint8)
                assert L.thor_d2h(host.ctypes.data, dl, nb) == 0
                assert np.array_equal(host.reshape(hl + 2 * PAD, s)[:, :wl + 2 * PAD], b)
    finally:
        for p in bufs:
            L.thor_dev_free(p)

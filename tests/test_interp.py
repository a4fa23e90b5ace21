"""Temporal-interpolation compensation:
interpolate_comp + mot_comp_avg (common/temporal_interp.c:387-441,920-944).

CPU: the oracle (or_interp_comp) against tests/golden/interp.npz -- per-block
outputs of the reference's own mot_comp_avg (tools/make_interp_goldens.py;
chroma's scale_mv is restated in the generator, so chroma vectors are pinned
by restatement, the compensation by the reference).
GPU: thor_interp_comp through the C-ABI against the same goldens, and a 4K
luma + chroma field against the oracle.  Bit-exact."""
import ctypes as C
import os

import numpy as np
import pytest

from conftest import GOLD

GOLDEN = os.path.join(GOLD, "interp.npz")


def _cases():
    g = np.load(GOLDEN)
    k = 0
    while "dims_%d" % k in g:
        w, h, ratio, pos, wt0, wt1, bw, bh = (int(v) for v in g["dims_%d" % k])
        for comp in (0, 1):
            tag = "%d_%d" % (k, comp)
            yield dict(w=w, h=h, wt0=wt0, wt1=wt1, bw=bw, bh=bh, comp=comp, mv=g["mv_%d" % k],
                       r0=g["ref0_" + tag], r1=g["ref1_" + tag], out=g["out_" + tag])
        k += 1


def _geom(c):
    """(bs, pad, wP, hP, plane pad) as interpolate_frame derives them (:955-960)."""
    bs = 8 if c["comp"] == 0 else 4
    pad, wP, hP = 4, c["w"] + 4, c["h"] + 4
    if c["comp"]:
        wP, hP, pad = wP // 2, hP // 2, pad // 2
    return bs, pad, wP, hP, (96 if c["comp"] == 0 else 48)


def oracle_interp(c):
    from oracle import py as orc

    OL = orc.lib()
    bs, pad, wP, hP, pf = _geom(c)
    r0, r1 = np.ascontiguousarray(c["r0"]), np.ascontiguousarray(c["r1"])
    s0, s1 = r0.shape[1], r1.shape[1]
    so = c["out"].shape[1]
    o = np.zeros((c["bh"] * bs, so), np.uint8)
    mv0, mv1 = np.ascontiguousarray(c["mv"][0]), np.ascontiguousarray(c["mv"][1])
    OL.or_interp_comp(r0.ctypes.data + pf * s0 + pf, s0, r1.ctypes.data + pf * s1 + pf, s1, o.ctypes.data, so,
                      mv0.ctypes.data, mv1.ctypes.data, c["bw"], c["bh"], bs, wP, hP, pad, c["comp"], c["wt0"],
                      c["wt1"])
    return o


def test_oracle_interp_vs_reference_goldens():
    for c in _cases():
        got = oracle_interp(c)
        assert np.array_equal(got, c["out"]), "%dx%d comp %d" % (c["w"], c["h"], c["comp"])


def _gpu_interp(L, c):
    bs, pad, wP, hP, pf = _geom(c)
    bufs = []

    def put(a):
        a = np.ascontiguousarray(a)
        p = L.thor_dev_alloc(a.nbytes)
        assert p
        bufs.append(p)
        assert L.thor_h2d(p, a.ctypes.data, a.nbytes) == 0
        return p

    try:
        s0, s1 = c["r0"].shape[1], c["r1"].shape[1]
        d0, d1 = put(c["r0"]), put(c["r1"])
        m0, m1 = put(c["mv"][0]), put(c["mv"][1])
        so = c["out"].shape[1]
        o = np.zeros((c["bh"] * bs, so), np.uint8)
        do = put(o)
        rc = L.thor_interp_comp(d0 + pf * s0 + pf, s0, d1 + pf * s1 + pf, s1, do, so, m0, m1, c["bw"], c["bh"], bs,
                                wP, hP, pad, c["comp"], c["wt0"], c["wt1"], None)
        assert rc == 0
        assert L.thor_d2h(o.ctypes.data, do, o.nbytes) == 0
        return o
    finally:
        for p in bufs:
            L.thor_dev_free(p)


@pytest.mark.gpu
def test_gpu_interp_vs_reference_goldens():
    from thor_amd import lib as tl

    L = tl.load()
    for c in _cases():
        got = _gpu_interp(L, c)
        assert np.array_equal(got, c["out"]), "%dx%d comp %d: %d bytes differ" % (
            c["w"], c["h"], c["comp"], int((got != c["out"]).sum()))


@pytest.mark.gpu
@pytest.mark.parametrize("comp,pitch_pad", [(0, 0), (1, 0), (0, 1), (1, 3)])
def test_gpu_interp_4k_vs_oracle(comp, pitch_pad):
    """pitch_pad != 0: an output stride not a multiple of the block width
    takes the per-pixel kernel instead of the row-per-lane one."""
    from thor_amd import lib as tl

    L = tl.load()
    rng = np.random.default_rng(77 + comp)
    w, h = 3840, 2160
    pw, ph, pf = (w, h, 96) if comp == 0 else (w // 2, h // 2, 48)
    s = (pw + 2 * pf + 15) & ~15
    bw, bh = 2 * ((w + 15) // 16), 2 * ((h + 15) // 16)
    mv = rng.integers(-400, 401, (2, bh * bw, 2)).astype(np.int16)
    far = rng.random(bh * bw) < 0.03
    mv[1, far] = rng.integers(-5000, 5001, (int(far.sum()), 2))
    bs = 8 if comp == 0 else 4
    c = dict(w=w, h=h, wt0=3, wt1=1, bw=bw, bh=bh, comp=comp, mv=mv,
             r0=rng.integers(0, 256, (ph + 2 * pf, s), dtype=np.uint8),
             r1=rng.integers(0, 256, (ph + 2 * pf, s), dtype=np.uint8),
             out=np.zeros((bh * bs, ((bw * bs + 15) & ~15) + pitch_pad), np.uint8))
    got = _gpu_interp(L, c)
    want = oracle_interp(c)
    assert np.array_equal(got, want), "%d bytes differ" % int((got != want).sum())


class InterpPlane(C.Structure):  # thor_interp_plane_t
    _fields_ = [("p0", C.c_void_p), ("p1", C.c_void_p), ("out", C.c_void_p), ("s0", C.c_int32), ("s1", C.c_int32),
                ("so", C.c_int32)]


@pytest.mark.gpu
def test_gpu_interp_frame_one_launch_vs_reference_goldens():
    """thor_interp_frame (Y, U, V in one launch): Y against the luma golden,
    U and V (fed the same chroma references) against the chroma golden."""
    from thor_amd import lib as tl

    L = tl.load()
    cases = list(_cases())
    for cy, cc in zip(cases[0::2], cases[1::2]):
        bufs = []

        def put(a):
            a = np.ascontiguousarray(a)
            p = L.thor_dev_alloc(a.nbytes)
            assert p
            bufs.append(p)
            assert L.thor_h2d(p, a.ctypes.data, a.nbytes) == 0
            return p

        try:
            planes, outs = (InterpPlane * 3)(), []
            for k, c in enumerate((cy, cc, cc)):
                pf = 96 if k == 0 else 48
                s = c["r0"].shape[1]
                o = np.zeros_like(c["out"])
                d0, d1, do = put(c["r0"]), put(c["r1"]), put(o)
                planes[k] = InterpPlane(d0 + pf * s + pf, d1 + pf * s + pf, do, s, s, o.shape[1])
                outs.append((do, o))
            rc = L.thor_interp_frame(C.cast(planes, C.c_void_p), put(cy["mv"][0]), put(cy["mv"][1]), cy["bw"], cy["bh"],
                                     cy["w"], cy["h"], cy["wt0"], cy["wt1"], None)
            assert rc == 0
            for k, ((do, o), c) in enumerate(zip(outs, (cy, cc, cc))):
                assert L.thor_d2h(o.ctypes.data, do, o.nbytes) == 0
                assert np.array_equal(o, c["out"]), "%dx%d plane %d" % (c["w"], c["h"], k)
        finally:
            for p in bufs:
                L.thor_dev_free(p)

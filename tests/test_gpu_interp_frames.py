"""GPU parity of the temporal-interpolated reference (tme.hip + pyramid.hip +
interp.hip through the C-ABI thor_interpolate_frames): the interpolated frame
must equal the reference's own interpolate_frames (tests/golden/interp_frames.npz)
and every level's final vector field must equal the oracle's; then whole
-interp_ref 1 streams (BASELINE config 5's reference structure) decode from
their .bit bit-exactly, stage by stage, against the reference decoder."""
import ctypes as C
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLD

pytestmark = pytest.mark.gpu


def _dev(L, arr):
    p = L.thor_dev_alloc(arr.nbytes)
    assert p
    assert L.thor_h2d(p, arr.ctypes.data, arr.nbytes) == 0
    return p


def _planes(L, f, ptrs):
    return L.ThorYuvPlanes(ptrs[0] + f.oy, ptrs[1] + f.oc, ptrs[2] + f.oc, f.sy, f.sc)


@pytest.mark.parametrize("k", range(6))
def test_gpu_interpolate_frames_vs_reference(k):
    from oracle.py import PaddedFrame, interpolate_frames
    from test_interp_frames import refs
    from thor_amd import lib as L

    lib = L.load()
    z = np.load(os.path.join(GOLD, "interp_frames.npz"))
    (w, h, ratio, pos), r0, r1 = refs(z, k)
    want, fields = interpolate_frames(r0, r1, ratio, pos, levels=True)
    out = PaddedFrame(w, h)
    bufs = []
    try:
        p0 = [_dev(lib, a) for a in (r0.Y, r0.U, r0.V)]
        p1 = [_dev(lib, a) for a in (r1.Y, r1.U, r1.V)]
        po = [_dev(lib, a) for a in (out.Y, out.U, out.V)]
        bufs = p0 + p1 + po
        t = lib.thor_ti_create(w, h, 0)
        assert t
        try:
            a, b, o = _planes(L, r0, p0), _planes(L, r1, p1), _planes(L, out, po)
            assert lib.thor_interpolate_frames(t, C.byref(a), C.byref(b), 96, C.byref(o), ratio, pos, None) == 0
            for lv, (f0, f1) in enumerate(fields):
                g0, g1 = np.zeros_like(f0), np.zeros_like(f1)
                assert lib.thor_ti_read_fields(t, lv, g0.ctypes.data, g1.ctypes.data) == 0
                bad = np.argwhere(np.any(g1 != f1, axis=2))
                assert bad.size == 0, (k, lv, "mv1", bad[:5].tolist(), len(bad))
                assert np.array_equal(g0, f0), (k, lv, "mv0")
        finally:
            lib.thor_ti_destroy(t)
        for arr, p in zip((out.Y, out.U, out.V), po):
            assert lib.thor_d2h(arr.ctypes.data, p, arr.nbytes) == 0
        for c, g in zip("yuv", out.planes()):
            ref = z["out_%s_%d" % (c, k)]
            assert np.array_equal(g, ref), (k, c, int((g != ref).sum()))
        for g, o in zip(out.planes(), want.planes()):
            assert np.array_equal(g, o)
    finally:
        for p in bufs:
            lib.thor_dev_free(p)


def _md5(b):
    return hashlib.md5(b).hexdigest()


@pytest.mark.parametrize("name", ["cif_hdbi", "cif_hdbi_high", "k4_hdbi", "k4_hdbi_high"])
def test_gpu_decode_interp_ref_stream(name, streams):
    """.bit -> host parser -> GPU decode with the interpolated references built
    on the GPU (dec/decode_frame.c:91-109); CIF checked at every stage."""
    from thor_amd.bitstream import parse_stream
    from thor_amd.decoder import GpuDecoder

    meta = streams[name]
    seq, frames = parse_stream(open(os.path.join(GOLD, name + ".bit"), "rb").read())
    assert seq.interp_ref == 1 and sum(f.interp_ratio > 0 for f in frames) > 0
    stages = ((0, "pre_deblock"), (1, "post_deblock"), (2, "final")) if seq.width < 1000 else ((2, "final"),)
    dec = GpuDecoder(seq)
    try:
        out = {}
        for fr in frames:
            d = dec.upload(fr)
            for stage, key in stages:
                dec.set_stop_stage(stage)
                dec.decode(d)
                dec.sync()
                got = dec.read_i420(fr.frame_num)
                assert _md5(got) == meta["stage_md5"][fr.decode_order][key], (name, fr.decode_order, key,
                                                                              fr.interp_ratio)
            out[fr.frame_num] = got
        assert _md5(b"".join(out[k] for k in sorted(out))) == meta["dec_md5"]
    finally:
        dec.close()

#!/usr/bin/env python3
"""Golden vectors for the temporal-interpolation compensation stage (TEST INFRASTRUCTURE).

interpolate_comp (common/temporal_interp.c:920-944) is static, so the
generator replays its loop here and calls the reference's exported
mot_comp_avg (:387-441, SIMD build: block_avg_simd) from
oracle/_ref/libthor_ref.so for every block.  Luma is therefore fully the
reference's arithmetic; for chroma the per-block mv0 = scale_mv(mv1 >> 1,
-wt1, wt0) (:934-938, static scale_mv :66-91) is restated below and only the
compensation is the reference's.  Writes tests/golden/interp.npz.  Runs only
in the build container.
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "_ref", "libthor_ref.so")
OUT = os.path.join(ROOT, "tests", "golden", "interp.npz")

# (w, h, ratio, pos): alloc_mv_data weights (:120-126)
CASES = [(352, 288, 2, 1), (200, 120, 4, 1), (200, 120, 4, 3), (136, 72, 8, 3)]


class Mv(C.Structure):
    _fields_ = [("x", C.c_int16), ("y", C.c_int16)]


def scale_val(v, numer, denom):
    if denom == 0:
        return 0
    prod = v * numer
    if denom < 0:
        denom, prod = -denom, -prod
    return (prod + denom // 2) // denom if prod >= 0 else -((-prod + denom // 2) // denom)


def i16(v):
    return ((v + 32768) & 0xFFFF) - 32768


def plane(rng, w, h, pad):
    s = (w + 2 * pad + 15) & ~15
    buf = np.zeros((h + 2 * pad) * s + 64, np.uint8)
    off = (-buf.ctypes.data) % 16
    body = buf[off:off + (h + 2 * pad) * s].reshape(h + 2 * pad, s)
    yy, xx = np.mgrid[0:h, 0:w]
    img = ((xx * 7 + yy * 3) % 256 + rng.integers(-30, 31, (h, w))).clip(0, 255).astype(np.uint8)
    body[pad:pad + h, pad:pad + w] = img
    # edge replication (pad_yuv_frame)
    body[pad:pad + h, :pad] = img[:, :1]
    body[pad:pad + h, pad + w:pad + w + pad] = img[:, -1:]
    body[:pad, :w + 2 * pad] = body[pad, :w + 2 * pad]
    body[pad + h:, :w + 2 * pad] = body[pad + h - 1, :w + 2 * pad]
    return body, s


def main():
    if not os.path.exists(LIB):
        sys.exit("build oracle/_ref first (make -C oracle ref)")
    L = C.CDLL(LIB)
    C.c_int.in_dll(L, "use_simd").value = 1
    P, I = C.c_void_p, C.c_int
    L.mot_comp_avg.argtypes = [I, I, P, I, P, I, P, I, Mv, Mv, I, I, I, I, P]
    rng = np.random.default_rng(4242)
    out = {}
    for k, (w, h, ratio, pos) in enumerate(CASES):
        reversed_ = pos > ratio // 2
        wt0 = pos if reversed_ else ratio - pos
        wt1 = ratio - wt0
        wt = (C.c_int * 2)(wt0, wt1)
        bs = 8
        bw, bh = 2 * ((w + 15) // 16), 2 * ((h + 15) // 16)
        mv = rng.integers(-300, 301, (2, bh * bw, 2)).astype(np.int16)
        far = rng.random(bh * bw) < 0.08  # clamped / one-sided cases
        mv[0, far] = rng.integers(-3000, 3001, (int(far.sum()), 2))
        far1 = rng.random(bh * bw) < 0.05
        mv[1, far1] = rng.integers(-3000, 3001, (int(far1.sum()), 2))
        out["dims_%d" % k] = np.array([w, h, ratio, pos, wt0, wt1, bw, bh], np.int32)
        out["mv_%d" % k] = mv
        for comp, (pw, ph, pad_f) in enumerate([(w, h, 96), (w // 2, h // 2, 48)]):
            r0, s0 = plane(rng, pw, ph, pad_f)
            r1, s1 = plane(rng, pw, ph, pad_f)
            cb = bs if comp == 0 else bs // 2
            pad = bs // 2
            wP, hP = w + pad, h + pad
            if comp:
                wP, hP, pad = wP // 2, hP // 2, pad // 2
            so = (bw * cb + 15) & ~15
            o = np.zeros((bh * cb, so), np.uint8)
            p0 = r0.ctypes.data + pad_f * s0 + pad_f
            p1 = r1.ctypes.data + pad_f * s1 + pad_f
            for yp in range(bh):
                for xp in range(bw):
                    b = yp * bw + xp
                    m0 = (int(mv[0, b, 0]), int(mv[0, b, 1]))
                    m1 = (int(mv[1, b, 0]), int(mv[1, b, 1]))
                    if comp:
                        m1 = (m1[0] >> 1, m1[1] >> 1)
                        if -wt1 == wt0:
                            m0 = m1
                        elif wt1 == wt0:
                            m0 = (i16(-m1[0]), i16(-m1[1]))
                        else:
                            m0 = (i16(scale_val(m1[0], -wt1, wt0)), i16(scale_val(m1[1], -wt1, wt0)))
                    L.mot_comp_avg(xp * cb, yp * cb, p0, s0, p1, s1, o.ctypes.data, so, Mv(*m0), Mv(*m1), wP, hP,
                                   pad, cb, wt)
            tag = "%d_%d" % (k, comp)
            out["ref0_" + tag] = r0
            out["ref1_" + tag] = r1
            out["out_" + tag] = o
        print("case %d: %dx%d ratio %d pos %d, %dx%d blocks" % (k, w, h, ratio, pos, bw, bh))
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Golden vectors for the temporal-interpolation luma pyramid (TEST INFRASTRUCTURE).

Runs the reference itself -- oracle/_ref/libthor_ref.so, common/*.c compiled
from /root/reference by oracle/Makefile -- the way interpolate_frames does
(common/temporal_interp.c:987-1019): create_yuv_frame(in, w, h, 96, 96, 48, 48)
(a padded reference frame), then for each level create_yuv_frame(.., 32, 32,
16, 16) and scale_frame_down2x2_simd (:187-245, which pads the level with
pad_yuv_frame).  Records the level-0 luma and each level's luma including its
32-pixel margin into tests/golden/pyramid.npz.  Runs only in the build
container (the GPU box has no /root/reference).
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "_ref", "libthor_ref.so")
OUT = os.path.join(ROOT, "tests", "golden", "pyramid.npz")

# (width, height): CIF, a width whose levels are not multiples of 16 or 8, odd sizes,
# a one-level frame
CASES = [(352, 288), (360, 264), (200, 120), (202, 134), (136, 72)]
PAD = 32


class YuvFrame(C.Structure):  # yuv_frame_t, common/types.h:41-59
    _fields_ = [("y", C.POINTER(C.c_uint8)), ("u", C.POINTER(C.c_uint8)), ("v", C.POINTER(C.c_uint8))] + [
        (n, C.c_int) for n in ("width", "height", "stride_y", "stride_c", "offset_y", "offset_c", "pad_hor_y",
                               "pad_hor_c", "pad_ver_y", "pad_ver_c", "area_y", "area_c", "frame_num")
    ]


def levels_for(w, h):
    import math
    return max(0, min(4, int(math.log10(min(w, h)) / math.log10(2.0) - 4.0)) - 1)


def main():
    if not os.path.exists(LIB):
        sys.exit("build oracle/_ref first (make -C oracle ref)")
    L = C.CDLL(LIB)
    C.c_int.in_dll(L, "use_simd").value = 1
    FP = C.POINTER(YuvFrame)
    L.create_yuv_frame.argtypes = [FP, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
    L.pad_yuv_frame.argtypes = [FP]
    L.scale_frame_down2x2_simd.argtypes = [FP, FP]
    rng = np.random.default_rng(20261016)
    out = {}
    for k, (w, h) in enumerate(CASES):
        src = YuvFrame()
        L.create_yuv_frame(C.byref(src), w, h, 96, 96, 48, 48)
        # texture: smooth ramp + noise, with saturated runs to exercise rounding at 0/255
        yy, xx = np.mgrid[0:h, 0:w]
        img = (xx * 3 + yy * 5) % 256 + rng.integers(-40, 41, (h, w))
        img[rng.random((h, w)) < 0.05] = 255
        img[rng.random((h, w)) < 0.05] = 0
        img = np.clip(img, 0, 255).astype(np.uint8)
        base = C.addressof(src.y.contents)
        for r in range(h):
            C.memmove(base + r * src.stride_y, img[r].ctypes.data, w)
        L.pad_yuv_frame(C.byref(src))
        n = levels_for(w, h)
        prev = src
        out["in_%d" % k] = img
        out["dims_%d" % k] = np.array([w, h, n], np.int32)
        for l in range(1, n + 1):
            lv = YuvFrame()
            L.create_yuv_frame(C.byref(lv), w >> l, h >> l, PAD, PAD, 16, 16)
            L.scale_frame_down2x2_simd(C.byref(prev), C.byref(lv))
            wl, hl = w >> l, h >> l
            lb = C.addressof(lv.y.contents)
            plane = np.zeros((hl + 2 * PAD, wl + 2 * PAD), np.uint8)
            for r in range(-PAD, hl + PAD):
                C.memmove(plane[r + PAD].ctypes.data, lb + r * lv.stride_y - PAD, wl + 2 * PAD)
            out["lvl_%d_%d" % (k, l)] = plane
            prev = lv  # frames are leaked: a short-lived generator
        print("case %d: %dx%d, %d levels" % (k, w, h, n))
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()

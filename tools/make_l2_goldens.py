#!/usr/bin/env python3
"""Golden vectors for the frame-level L2 entry points (TEST INFRASTRUCTURE):
the reference's own deblock_frame_y / deblock_frame_uv (common/common_frame.c:
46-321, SIMD build, oracle/_ref/libthor_ref.so) on seeded synthetic frames with
random CU tilings (quadtree 64..8, random mode / cbp / vectors / tb_split /
pb_part per CU, stored per 4x4 cell as copy_deblock_data does,
dec/decode_block.c:122-156).  Writes tests/golden/l2_deblock.npz.  Build
container only."""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from make_interp_frames_goldens import Yuv, get, put  # noqa: E402
from thor_amd import synth  # noqa: E402

LIB = os.path.join(ROOT, "oracle", "_ref", "libthor_ref.so")
OUT = os.path.join(ROOT, "tests", "golden", "l2_deblock.npz")
# (w, h, qp, seed)
CASES = [(128, 96, 32, 1), (192, 128, 40, 2), (136, 72, 26, 3), (256, 128, 50, 4)]

DD = np.dtype([("mode", "<i4"), ("cbp", "<i4", (3,)), ("size", "u1"), ("tb_split", "u1"), ("pad", "u1", (2,)),
               ("pb_part", "<i4"), ("mv", "<i2", (4,)), ("ref_idx0", "<u4"), ("ref_idx1", "<u4"),
               ("bipred", "<u4")])
assert DD.itemsize == 44


def tiling(w, h, rng):
    dd = np.zeros((h // 4, w // 4), DD)

    def cu(y, x, s):
        if y >= h or x >= w:
            return
        if s > 8 and (rng.random() < 0.55 or y + s > h or x + s > w):
            for dy in (0, s // 2):
                for dx in (0, s // 2):
                    cu(y + dy, x + dx, s // 2)
            return
        mode = int(rng.choice([0, 1, 2, 3, 4], p=[0.3, 0.2, 0.3, 0.1, 0.1]))
        rec = dd[y // 4:(y + s) // 4, x // 4:(x + s) // 4]
        rec["mode"] = mode
        rec["cbp"] = rng.integers(0, 2, 3) if mode else 0
        rec["size"] = s
        rec["tb_split"] = int(rng.random() < 0.2) if mode else 0
        rec["pb_part"] = int(rng.integers(0, 4)) if mode == 2 else 0
        if mode != 1:
            for q in range(4):  # per-quarter vectors
                qy, qx = (q >> 1) * s // 8, (q & 1) * s // 8
                sub = rec[qy:qy + max(1, s // 8), qx:qx + max(1, s // 8)]
                sub["mv"] = rng.integers(-7, 8, 4)
        rec["bipred"] = 2 if mode == 3 else 0

    for y in range(0, h, 64):
        for x in range(0, w, 64):
            cu(y, x, 64)
    return dd


def main():
    if not os.path.exists(LIB):
        sys.exit("build oracle/_ref first (make -C oracle ref)")
    L = C.CDLL(LIB)
    C.c_int.in_dll(L, "use_simd").value = 1
    L.create_yuv_frame.argtypes = [C.c_void_p] + [C.c_int] * 6
    L.pad_yuv_frame.argtypes = [C.c_void_p]
    L.deblock_frame_y.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_uint8]
    L.deblock_frame_uv.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_uint8]
    chroma_qp = [min(q, 29) if q < 30 else [29, 30, 31, 32, 33, 33, 34, 34, 35, 35, 36, 36, 37, 37, 38, 39, 40, 41, 42,
                                           43, 44, 45][q - 30] for q in range(52)]
    out = {}
    for k, (w, h, qp, seed) in enumerate(CASES):
        rng = np.random.default_rng(seed)
        planes = synth.synth_frame(w, h, 1, seed)
        planes = [(p.astype(np.int16) + rng.integers(-12, 13, p.shape)).clip(0, 255).astype(np.uint8) for p in planes]
        dd = np.ascontiguousarray(tiling(w, h, rng))
        f = Yuv()
        L.create_yuv_frame(C.byref(f), w, h, 0, 0, 0, 0)
        put(L, f, planes)
        L.deblock_frame_y(C.byref(f), dd.ctypes.data, w, h, qp)
        L.deblock_frame_uv(C.byref(f), dd.ctypes.data, w, h, chroma_qp[qp])
        got = get(f, w, h)
        out["dims_%d" % k] = np.array([w, h, qp, chroma_qp[qp]], np.int32)
        out["dd_%d" % k] = dd.view(np.uint8).reshape(-1)
        for c, nm in enumerate("yuv"):
            out["in_%s_%d" % (nm, k)] = planes[c]
            out["out_%s_%d" % (nm, k)] = got[c]
        print("case %d: %dx%d qp %d, %d Y px changed" % (k, w, h, qp, int((got[0] != planes[0]).sum())))
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()

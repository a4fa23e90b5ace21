#!/usr/bin/env python3
"""Golden vectors for cost_calc (enc/encode_block.c:1218-1228) from the
reference itself (TEST INFRASTRUCTURE): random original / reconstructed
yuv_block_t pairs of every CU size, bit counts and lambdas (the encoder's
operating range plus values that hit the 2^30 clamp), through the reference's
own ssd_calc and cost_calc (oracle/_ref/libthor_ref.so, SIMD build).  Writes
tests/golden/cost.npz: per case the three SSDs, nbits, lambda and the cost.
Build container only."""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "_ref", "libthor_ref.so")
OUT = os.path.join(ROOT, "tests", "golden", "cost.npz")


class Blk(C.Structure):  # yuv_block_t, enc/mainenc.h:90-95
    _fields_ = [("y", C.c_uint8 * 4096), ("u", C.c_uint8 * 1024), ("v", C.c_uint8 * 1024)]


def main():
    if not os.path.exists(LIB):
        sys.exit("build oracle/_ref first (make -C oracle ref)")
    L = C.CDLL(LIB)
    C.c_int.in_dll(L, "use_simd").value = 1
    L.cost_calc.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_double]
    L.cost_calc.restype = C.c_uint32
    L.ssd_calc.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int]
    L.ssd_calc.restype = C.c_int
    rng = np.random.default_rng(2024)
    rows = []
    for k in range(2000):
        size = int(rng.choice([8, 16, 32, 64]))
        org, rec = Blk(), Blk()
        o = rng.integers(0, 256, 6144, dtype=np.uint8)
        amp = int(rng.choice([2, 8, 40, 255]))
        r = (o.astype(np.int32) + rng.integers(-amp, amp + 1, 6144)).clip(0, 255).astype(np.uint8)
        C.memmove(C.addressof(org), o.ctypes.data, 6144)
        C.memmove(C.addressof(rec), r.ctypes.data, 6144)
        nbits = int(rng.integers(0, 20000))
        qp = int(rng.integers(0, 52))
        lam = float(rng.choice([0.57, 0.8, 1.2, 3.0])) * 2 ** ((qp - 12) / 3.0)  # squared_lambda_QP scale
        if k % 50 == 0:
            lam *= 1e4  # the 2^30 clamp
        sy = L.ssd_calc(C.addressof(org), C.addressof(rec), size, size, size, size)
        su = L.ssd_calc(C.addressof(org) + 4096, C.addressof(rec) + 4096, size // 2, size // 2, size // 2, size // 2)
        sv = L.ssd_calc(C.addressof(org) + 5120, C.addressof(rec) + 5120, size // 2, size // 2, size // 2, size // 2)
        cost = L.cost_calc(C.byref(org), C.byref(rec), size, size, size, nbits, lam)
        rows.append((sy, su, sv, nbits, lam, cost))
    a = np.array(rows, dtype=np.float64)
    np.savez_compressed(OUT, ssd=a[:, :3].astype(np.uint32), nbits=a[:, 3].astype(np.int32), lam=a[:, 4],
                        cost=a[:, 5].astype(np.uint32))
    print("wrote", OUT, os.path.getsize(OUT), "bytes;", int((a[:, 5] == 2 ** 30).sum()), "clamped")


if __name__ == "__main__":
    main()

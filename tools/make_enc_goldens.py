#!/usr/bin/env python3
"""Golden vectors of the encoder transform-block chain, produced by the
reference's own functions (TEST INFRASTRUCTURE; runs only in the build
container, where oracle/_ref/libthor_ref.so is compiled from /root/reference).

Composes, exactly as encode_and_reconstruct_block_inter does per TU
(enc/encode_block.c:1481-1518), the reference's get_residual
(enc/encode_block.c:484), transform (common/transform.c:249, SIMD path),
quantize (enc/encode_block.c:75, rdoq 0), dequantize + inverse_transform
(common/common_block.c:132, common/transform.c:488), reconstruct_block
(common/common_block.c:148) and ssd_calc (enc/encode_block.c:783), with
`use_simd` = 1 (the default x86-64 build).  Writes tests/golden/enc_tu.npz:

  enc_meta  (n, 5) int32   size, qp, type (bit1 intra, bit0 chroma), fast, cbp
  enc_orig / enc_pred      (n, 64, 64) uint8 (top-left size x size used)
  enc_levels (n, 16, 16) int16  quantised q x q corner
  enc_rec    (n, 64, 64) uint8  reconstruction
  enc_ssd    (n,) uint32
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from make_kernel_goldens import LIB, aligned, ptr  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "enc_tu.npz")
P, I = C.c_void_p, C.c_int


def main():
    if not os.path.exists(LIB):
        sys.exit("build oracle/_ref first (make -C oracle ref)")
    L = C.CDLL(LIB)
    C.c_int.in_dll(L, "use_simd").value = 1
    L.get_residual.argtypes = [P, P, P, I, I]
    L.transform.argtypes = [P, P, I, I]
    L.quantize.argtypes = [P, P, I, I, I, I]
    L.quantize.restype = I
    L.dequantize.argtypes = [P, P, I, I]
    L.inverse_transform.argtypes = [P, P, I]
    L.reconstruct_block.argtypes = [P, P, P, I, I]
    L.ssd_calc.argtypes = [P, P, I, I, I, I]
    L.ssd_calc.restype = C.c_uint

    rng = np.random.default_rng(20261016)
    meta, origs, preds, levs, recs, ssds = [], [], [], [], [], []
    plan = [(4, 160), (8, 200), (16, 120), (32, 60), (64, 30)]
    for size, count in plan:
        for c in range(count):
            qp = int(rng.integers(0, 52))
            typ = int(rng.integers(0, 4))
            fast = int(rng.integers(0, 2)) if size >= 32 else 0
            kind = c % 4
            org = aligned((64, 64), np.uint8)
            pb = aligned((size, size), np.uint8)
            base = rng.integers(0, 256, (size, size))
            if kind == 0:  # prediction close to the original (typical residual)
                o = base
                p = np.clip(base + rng.integers(-12, 13, (size, size)), 0, 255)
            elif kind == 1:  # extreme residuals (+-255)
                o = rng.choice([0, 255], (size, size))
                p = 255 - o
            elif kind == 2:  # smooth gradient vs flat prediction
                o = np.clip(np.cumsum(rng.integers(-6, 7, (size, size)), axis=1) + 128, 0, 255)
                p = np.full((size, size), int(rng.integers(0, 256)))
            else:  # uncorrelated
                o = base
                p = rng.integers(0, 256, (size, size))
            org[:size, :size] = o
            pb[:] = p
            block = aligned((64, 64), np.int16)
            coeff = aligned((64, 64), np.int16)
            coeffq = aligned((64, 64), np.int16)
            rcoeff = aligned((64, 64), np.int16)
            rblock = aligned((64, 64), np.int16)
            rec = aligned((64, 64), np.uint8)
            L.get_residual(ptr(block), ptr(pb), ptr(org), size, 64)
            L.transform(ptr(block), ptr(coeff), size, fast)
            cbp = L.quantize(ptr(coeff), ptr(coeffq), qp, size, typ, 0)
            if cbp:
                L.dequantize(ptr(coeffq), ptr(rcoeff), qp, size)
                L.inverse_transform(ptr(rcoeff), ptr(rblock), size)
                L.reconstruct_block(ptr(rblock), ptr(pb), ptr(rec), size, 64)
            else:
                for i in range(size):
                    rec[i, :size] = pb[i]
            ssd = L.ssd_calc(ptr(org), ptr(rec), 64, 64, size, size)
            q = min(size, 16)
            lv = np.zeros((16, 16), np.int16)
            lv[:q, :q] = coeffq.reshape(-1)[: size * size].reshape(size, size)[:q, :q]
            meta.append((size, qp, typ, fast, cbp))
            p64 = np.zeros((64, 64), np.uint8)
            p64[:size, :size] = pb
            origs.append(np.array(org))
            preds.append(p64)
            levs.append(lv)
            recs.append(np.array(rec))
            ssds.append(ssd)
    np.savez_compressed(OUT, enc_meta=np.array(meta, np.int32), enc_orig=np.stack(origs), enc_pred=np.stack(preds),
                        enc_levels=np.stack(levs), enc_rec=np.stack(recs), enc_ssd=np.array(ssds, np.uint32))
    print("wrote", OUT, len(meta), "TUs")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Kernel-level golden vectors from the reference itself (TEST INFRASTRUCTURE).

Loads oracle/_ref/libthor_ref.so -- the reference's common/*.c + enc/*.c
compiled from /root/reference by oracle/Makefile -- sets its `use_simd`
global to 1 (the default x86-64 build is the SIMD path)
and records seeded inputs/outputs of the hot-path functions into
tests/golden/kernels.npz.  Runs only in the build container.

  transform        common/transform.c:249 (SIMD: common/common_kernels.c:2176)
  inverse_transform common/transform.c:488
  dequantize       common/common_block.c:132
  quantize         enc/encode_block.c:75 (rdoq 0)
  luma / chroma MC common/inter_prediction.c:72-180
  intra            common/intra_prediction.c:57-388 (make_top_and_left + get_intra_prediction)
  clpf_block       common/common_block.c:180
  sad / ssd / widesad / fasthalf / fastquarter / detect_clpf  enc/encode_block.c:497-797,3036
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "_ref", "libthor_ref.so")
OUT = os.path.join(ROOT, "tests", "golden", "kernels.npz")

P = C.c_void_p
I = C.c_int


def ptr(a):
    return a.ctypes.data


def aligned(shape, dtype, align=64):
    """numpy array whose data pointer is `align`-byte aligned (the reference's
    SIMD kernels use aligned 16-byte loads)."""
    n = int(np.prod(shape)) * np.dtype(dtype).itemsize
    raw = np.zeros(n + align, np.uint8)
    off = (-raw.ctypes.data) % align
    return raw[off:off + n].view(dtype).reshape(shape)


class Mv(C.Structure):
    _fields_ = [("x", C.c_int16), ("y", C.c_int16)]


def main():
    if not os.path.exists(LIB):
        sys.exit("build oracle/_ref first (make -C oracle ref)")
    L = C.CDLL(LIB)
    C.c_int.in_dll(L, "use_simd").value = 1
    L.transform.argtypes = [P, P, I, I]
    L.inverse_transform.argtypes = [P, P, I]
    L.dequantize.argtypes = [P, P, I, I]
    L.quantize.argtypes = [P, P, I, I, I, I]
    L.quantize.restype = I
    L.get_inter_prediction_luma.argtypes = [P, P, I, I, I, I, C.POINTER(Mv), I, I]
    L.get_inter_prediction_chroma.argtypes = [P, P, I, I, I, I, C.POINTER(Mv), I]
    L.make_top_and_left.argtypes = [P, P, P, P, I, P, I, I, I, I, I, I, I, I, I]
    L.get_intra_prediction.argtypes = [P, P, C.c_uint8, I, I, I, P, I]
    L.clpf_block.argtypes = [P, P, I, I, I, I, I, I, I]
    for n in ("sad_calc", "ssd_calc"):
        getattr(L, n).argtypes = [P, P, I, I, I, I]
        getattr(L, n).restype = C.c_uint
    L.widesad_calc.argtypes = [P, P, I, I, I, I, C.POINTER(C.c_int)]
    L.widesad_calc.restype = C.c_uint
    for n in ("sad_calc_fasthalf", "sad_calc_fastquarter"):
        getattr(L, n).argtypes = [P, P, I, I, I, I, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        getattr(L, n).restype = C.c_uint
    L.detect_clpf.argtypes = [P, P, I, I, I, I, I, I, C.POINTER(C.c_int), C.POINTER(C.c_int)]

    rng = np.random.default_rng(20261015)
    G = {}

    # ---- forward transform: random, smooth and adversarial residuals ----
    for N in (4, 8, 16, 32, 64):
        for fast in ((0, 1) if N >= 32 else (0,)):
            cases = {4: 200, 8: 400, 16: 120, 32: 40, 64: 16}[N]
            ins, outs = [], []
            for c in range(cases):
                kind = c % 4
                if kind == 0:
                    blk = rng.integers(-255, 256, (N, N))
                elif kind == 1:
                    blk = rng.choice([-255, 255], (N, N))
                elif kind == 2:  # checkerboard-ish extreme patterns
                    s = rng.choice([-255, 255])
                    blk = s * (((np.arange(N)[:, None] + np.arange(N)[None, :] * rng.integers(1, 4)) % 2) * 2 - 1)
                else:
                    blk = np.clip(np.cumsum(rng.integers(-20, 21, (N, N)), axis=1), -255, 255)
                b2 = aligned((N, N), np.int16)
                b2[:] = blk
                blk = b2
                co = aligned((N, N), np.int16)
                co[:] = 0x5A5A  # sentinel: untouched area must survive
                L.transform(ptr(blk), ptr(co), N, fast)
                ins.append(blk)
                outs.append(co)
            G["ftx_%d_%d_in" % (N, fast)] = np.stack(ins)
            G["ftx_%d_%d_out" % (N, fast)] = np.stack(outs)

    # ---- inverse transform and dequantize ----
    for N in (4, 8, 16, 32, 64):
        ins, outs = [], []
        q = min(N, 16)
        for c in range({4: 120, 8: 120, 16: 60, 32: 30, 64: 12}[N]):
            co = np.zeros((N, N), np.int16)
            amp = [300, 3000, 32767][c % 3]
            co[:q, :q] = rng.integers(-amp, amp + 1, (q, q))
            if c % 5 == 0:
                co[:q, :q][rng.random((q, q)) < 0.8] = 0
            c2 = aligned((N, N), np.int16)
            c2[:] = co
            co = c2
            out = aligned((N, N), np.int16)
            L.inverse_transform(ptr(co), ptr(out), N)
            ins.append(co)
            outs.append(out)
        G["itx_%d_in" % N] = np.stack(ins)
        G["itx_%d_out" % N] = np.stack(outs)
        dq_in, dq_qp, dq_out = [], [], []
        for c in range({4: 60, 8: 60, 16: 30, 32: 12, 64: 6}[N]):
            co = rng.integers(-2000, 2001, (N, N)).astype(np.int16)
            qp = int(rng.integers(0, 52))
            out = np.zeros((N, N), np.int16)
            L.dequantize(ptr(co), ptr(out), qp, N)
            dq_in.append(co)
            dq_qp.append(qp)
            dq_out.append(out)
        G["dq_%d_in" % N] = np.stack(dq_in)
        G["dq_%d_qp" % N] = np.array(dq_qp, np.int32)
        G["dq_%d_out" % N] = np.stack(dq_out)

    # ---- quantize (coefficients from real transforms of residuals) ----
    for N in (4, 8, 16, 32, 64):
        ins, qps, types, outs, cbps = [], [], [], [], []
        for c in range({4: 200, 8: 200, 16: 100, 32: 40, 64: 20}[N]):
            res = rng.integers(-60, 61, (N, N)).astype(np.int16) if c % 2 else \
                np.clip(np.cumsum(rng.integers(-8, 9, (N, N)), axis=0), -255, 255).astype(np.int16)
            r2 = aligned((N, N), np.int16)
            r2[:] = res
            res = r2
            co = aligned((N, N), np.int16)
            L.transform(ptr(res), ptr(co), N, int(N >= 32 and c % 3 == 0))
            qp = int(rng.integers(10, 52))
            t = int(c % 4)
            out = np.full((N, N), 0x1234, np.int16)
            cbp = L.quantize(ptr(co), ptr(out), qp, N, t, 0)
            ins.append(co)
            qps.append(qp)
            types.append(t)
            outs.append(out)
            cbps.append(cbp)
        G["q_%d_in" % N] = np.stack(ins)
        G["q_%d_qp" % N] = np.array(qps, np.int32)
        G["q_%d_type" % N] = np.array(types, np.int32)
        G["q_%d_out" % N] = np.stack(outs)
        G["q_%d_cbp" % N] = np.array(cbps, np.int32)

    # ---- motion compensation (one shared reference picture, flat outputs) ----
    S = 160
    mref = rng.integers(0, 256, (S, S), dtype=np.uint8)
    meta, outs = [], []
    for bipred in (0, 1):
        for (w, h) in ((4, 4), (8, 8), (16, 16), (32, 32), (64, 64), (8, 16), (24, 8), (64, 48)):
            for c in range(12):
                mvx, mvy = int(rng.integers(-40, 41)), int(rng.integers(-40, 41))
                sign = int(rng.integers(0, 2))
                # pstride 64 as in the decoder (pblock stride = CU size): the SIMD
                # kernels store whole 8-byte chunks past `width`
                out = aligned((h, 64), np.uint8)
                mv = Mv(mvx, mvy)
                L.get_inter_prediction_luma(ptr(out), ptr(mref) + 48 * S + 48, w, h, S, 64, C.byref(mv), sign, bipred)
                meta.append((0, bipred, w, h, mvx, mvy, sign))
                outs.append(out[:, :w].reshape(-1).copy())
    for (w, h) in ((2, 2), (4, 4), (8, 8), (16, 16), (32, 32), (4, 8), (12, 4)):
        for c in range(16):
            mvx, mvy = int(rng.integers(-60, 61)), int(rng.integers(-60, 61))
            sign = int(rng.integers(0, 2))
            out = aligned((h, 64), np.uint8)
            mv = Mv(mvx, mvy)
            L.get_inter_prediction_chroma(ptr(out), ptr(mref) + 48 * S + 48, w, h, S, 64, C.byref(mv), sign)
            meta.append((1, 0, w, h, mvx, mvy, sign))
            outs.append(out[:, :w].reshape(-1).copy())
    G["mc_meta"] = np.array(meta, np.int32)
    G["mc_ref"] = mref
    G["mc_out"] = np.concatenate(outs)

    # ---- intra prediction on a random reconstructed frame ----
    FW, FH = 192, 192
    meta, outs = [], []
    frame = rng.integers(0, 256, (FH, FW), dtype=np.uint8)
    left = (C.c_uint8 * 160)()
    top = (C.c_uint8 * 160)()
    tl = C.c_uint8()
    for c in range(400):
        size = int(rng.choice([4, 8, 16, 32, 64]))
        ypos = int(rng.integers(0, (FH - size) // size + 1)) * size
        xpos = int(rng.integers(0, (FW - size) // size + 1)) * size
        ur = int(rng.integers(0, 2)) if ypos > 0 and xpos + size < FW else 0
        dl = int(rng.integers(0, 2)) if xpos > 0 and ypos + size < FH else 0
        mode = int(rng.integers(0, 10))
        lp = C.cast(C.byref(left, 1), P).value
        tp = C.cast(C.byref(top, 1), P).value
        L.make_top_and_left(lp, tp, C.byref(tl), ptr(frame) + ypos * FW + xpos, FW, None, 0, 0, 0, ypos, xpos, size,
                            ur, dl, 0)
        out = np.zeros((64, 64), np.uint8)
        pb = np.zeros(size * size, np.uint8)
        L.get_intra_prediction(lp, tp, tl.value, ypos, xpos, size, ptr(pb), mode)
        out[:size, :size] = pb.reshape(size, size)
        meta.append((size, ypos, xpos, ur, dl, mode))
        outs.append(out)
    G["intra_frame"] = frame
    G["intra_meta"] = np.array(meta, np.int32)
    G["intra_out"] = np.concatenate([o[:m[0], :m[0]].reshape(-1) for o, m in zip(outs, meta)])

    # ---- encoder distortion kernels (shared pictures, per-case offsets) ----
    A = aligned((160, 160), np.uint8)
    B = aligned((160, 160), np.uint8)
    A[:] = rng.integers(0, 256, (160, 160), dtype=np.uint8)
    B[:] = np.clip(A.astype(int) + rng.integers(-30, 31, (160, 160)), 0, 255).astype(np.uint8)
    dist = []
    for c in range(300):
        w = int(rng.choice([8, 16, 32, 64]))
        h = w if c % 3 else int(rng.choice([8, 16, 32, 64]))
        oy, ox = 16 * int(rng.integers(1, (160 - 64 - 16) // 16)), 16 * int(rng.integers(1, (160 - 64 - 16) // 16))
        ap, bp = ptr(A) + oy * 160 + ox, ptr(B) + oy * 160 + ox
        sad = L.sad_calc(ap, bp, 160, 160, w, h)
        ssd = L.ssd_calc(ap, bp, 160, 160, w, h)
        x = C.c_int(0)
        y = C.c_int(0)
        wsad = L.widesad_calc(ap, bp, 160, 160, w, h, C.byref(x))
        wx = x.value
        x.value, y.value = 0, 0
        fh = L.sad_calc_fasthalf(ap, bp, 160, 160, w, h, C.byref(x), C.byref(y))
        fhx, fhy = x.value, y.value
        qx, qy = int(rng.integers(-1, 2)), int(rng.integers(-1, 2))
        x.value, y.value = qx, qy
        fq = L.sad_calc_fastquarter(ap, bp, 160, 160, w, h, C.byref(x), C.byref(y))
        dist.append((w, h, oy, ox, sad, ssd, wsad, wx, fh, fhx, fhy, qx, qy, fq, x.value, y.value))
    G["dist_meta"] = np.array(dist, np.int64)
    G["dist_a"] = np.array(A)
    G["dist_b"] = np.array(B)

    # ---- CLPF block + detect (shared pictures) ----
    fr = aligned((128, 128), np.uint8)
    fr[:] = rng.integers(0, 256, (128, 128), dtype=np.uint8)
    fr[32:96, 32:96] = np.clip(fr[32:96, 32:96] // 32 * 32 + 10, 0, 255)  # flat areas make deltas fire
    org = rng.integers(0, 256, (128, 128), dtype=np.uint8)
    cl, cout = [], []
    for c in range(200):
        size = 8 if c % 2 else 4
        sb = 64 if size == 8 else 32
        x0 = int(rng.integers(0, 128 // size)) * size
        y0 = int(rng.integers(0, 128 // size)) * size
        dst = aligned((sb, sb), np.uint8)
        L.clpf_block(ptr(fr), ptr(dst), 128, sb, x0, y0, size, 128, 128)
        left, topv = x0 & ~(sb - 1), y0 & ~(sb - 1)
        blk = dst[y0 - topv:y0 - topv + size, x0 - left:x0 - left + size].copy()
        s0, s1 = C.c_int(0), C.c_int(0)
        if size == 8:
            L.detect_clpf(ptr(fr), ptr(org), x0, y0, 128, 128, 128, 128, C.byref(s0), C.byref(s1))
        cl.append((size, x0, y0, s0.value, s1.value))
        cout.append(blk.reshape(-1))
    G["clpf_meta"] = np.array(cl, np.int64)
    G["clpf_src"] = np.array(fr)
    G["clpf_org"] = org
    G["clpf_out"] = np.concatenate(cout)

    np.savez_compressed(OUT, **G)
    print("wrote", OUT, os.path.getsize(OUT), "bytes,", len(G), "arrays")


if __name__ == "__main__":
    main()

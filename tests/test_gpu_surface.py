"""The reference's SIMD kernel surface (include/thor_kernels.h) executed on
the GPU, against the golden vectors recorded from the reference SIMD build
itself (tests/golden/kernels.npz) and, for shapes the goldens do not cover,
against the CPU oracle on seeded random inputs."""
import ctypes as C
import os

import numpy as np
import pytest

from conftest import GOLD

pytestmark = pytest.mark.gpu
K = np.load(os.path.join(GOLD, "kernels.npz"))


def ptr(a):
    return a.ctypes.data


@pytest.fixture(scope="module")
def g():
    from thor_amd import lib as L

    return L.load()


@pytest.mark.parametrize("N,fast", [(4, 0), (8, 0), (16, 0), (32, 0), (32, 1), (64, 0), (64, 1)])
def test_transform_simd_vs_reference(g, N, fast):
    """transform_simd (common/common_kernels.c:2176-2250), incl. the 8x8
    16-bit butterfly wrap cases and the untouched-area sentinel."""
    bad = []
    for k, (blk, want) in enumerate(zip(K["ftx_%d_%d_in" % (N, fast)], K["ftx_%d_%d_out" % (N, fast)])):
        blk = np.ascontiguousarray(blk)
        got = np.full((N, N), 0x5A5A, np.int16)
        g.transform_simd(ptr(blk), ptr(got), N, fast)
        if N == 64 and not fast:  # rows/cols 16..31 come from uninitialised scratch in the reference
            ok = np.array_equal(got[:16, :16], want[:16, :16]) and np.all(got[32:, :] == 0x5A5A) and np.all(
                got[:, 32:] == 0x5A5A)
        else:
            ok = np.array_equal(got, want)
        if not ok:
            bad.append(k)
    assert not bad, bad[:10]


@pytest.mark.parametrize("N", [4, 8, 16, 32, 64])
def test_inverse_transform_simd_vs_reference(g, N):
    bad = []
    for k, (co, want) in enumerate(zip(K["itx_%d_in" % N], K["itx_%d_out" % N])):
        co = np.ascontiguousarray(co)
        got = np.zeros((N, N), np.int16)
        g.inverse_transform_simd(ptr(co), ptr(got), N)
        if not np.array_equal(got, want):
            bad.append(k)
    assert not bad, bad[:10]


def test_distortion_kernels_vs_reference(g):
    """sad_calc_simd / ssd_calc_simd / widesad_calc_simd / sad_calc_fasthalf_simd /
    sad_calc_fastquarter_simd (enc/enc_kernels.c) against the reference's
    dispatching wrappers (enc/encode_block.c:497-797) on the recorded cases."""
    A, B = np.ascontiguousarray(K["dist_a"]), np.ascontiguousarray(K["dist_b"])
    S = A.shape[1]
    x, y = C.c_int(0), C.c_int(0)
    bad = []
    for row in K["dist_meta"]:
        w, h, oy, ox, sad, ssd, wsad, wx, fh, fhx, fhy, qx, qy, fq, fqx, fqy = (int(v) for v in row)
        ap, bp = ptr(A) + oy * S + ox, ptr(B) + oy * S + ox
        if g.sad_calc_simd(ap, bp, S, S, w, h) != sad:
            bad.append(("sad", w, h))
        if w == h and g.ssd_calc_simd(ap, bp, S, S, w) != ssd:
            bad.append(("ssd", w))
        if w == 16 and h == 16:  # widesad_calc dispatches to the SIMD kernel only for 16x16
            if g.widesad_calc_simd(ap, bp, S, S, w, h, C.byref(x)) != wsad or x.value != wx:
                bad.append(("wide", w, h))
        x.value, y.value = 0, 0
        if g.sad_calc_fasthalf_simd(ap, bp, S, S, w, h, C.byref(x), C.byref(y)) != fh or (x.value, y.value) != (fhx, fhy):
            bad.append(("half", w, h))
        x.value, y.value = qx, qy
        if g.sad_calc_fastquarter_simd(ap, bp, S, S, w, h, C.byref(x), C.byref(y)) != fq or (x.value, y.value) != (
                fqx, fqy):
            bad.append(("quarter", w, h, qx, qy))
    assert not bad, bad[:10]


def test_clpf_kernels_vs_reference(g):
    """clpf_block4 / clpf_block8 (common/common_kernels.c:2277-2356) and
    detect_clpf_simd (enc/enc_kernels.c:124-159)."""
    src = np.ascontiguousarray(K["clpf_src"])
    org = np.ascontiguousarray(K["clpf_org"])
    off = 0
    bad = []
    for size, x0, y0, s0, s1 in K["clpf_meta"]:
        size, x0, y0 = int(size), int(x0), int(y0)
        want = K["clpf_out"][off:off + size * size].reshape(size, size)
        off += size * size
        sb = 64 if size == 8 else 32
        dst = np.full((sb, sb), 7, np.uint8)
        (g.clpf_block8 if size == 8 else g.clpf_block4)(ptr(src), ptr(dst), 128, sb, x0, y0, 128, 128)
        l, t = x0 & ~(sb - 1), y0 & ~(sb - 1)
        got = dst[y0 - t:y0 - t + size, x0 - l:x0 - l + size]
        if not np.array_equal(got, want):
            bad.append(("clpf", size, x0, y0))
        untouched = dst.copy()
        untouched[y0 - t:y0 - t + size, x0 - l:x0 - l + size] = 7
        if np.any(untouched != 7):
            bad.append(("clpf-outside", size, x0, y0))
        if size == 8:
            a, b = C.c_int(5), C.c_int(9)  # detect_clpf accumulates
            g.detect_clpf_simd(ptr(src), ptr(org), x0, y0, 128, 128, 128, 128, C.byref(a), C.byref(b))
            if (a.value - 5, b.value - 9) != (s0, s1):
                bad.append(("detect", x0, y0, a.value - 5, b.value - 9, s0, s1))
    assert not bad, bad[:10]


def test_block_avg_and_unaligned_sad(g):
    """block_avg_simd (rounding average) and sad_calc_simd_unaligned
    (common/common_kernels.c:34-123), whose default case advances both
    pointers four rows per 16-column step (restated here in numpy)."""
    rng = np.random.default_rng(5)
    S = 200
    a = rng.integers(0, 256, (S, S), dtype=np.uint8)
    b = rng.integers(0, 256, (S, S), dtype=np.uint8)
    for w in (4, 8, 16, 32, 64):
        for h in (4, 8, 16, 32):
            p = np.zeros((h, 64), np.uint8)
            g.block_avg_simd(ptr(p), ptr(a) + 3 * S + 5, ptr(b) + 7 * S + 1, 64, S, S, w, h)
            want = (a[3:3 + h, 5:5 + w].astype(int) + b[7:7 + h, 1:1 + w] + 1) >> 1
            assert np.array_equal(p[:, :w], want), (w, h)
            if w > 8:
                rows = [4 * ((i // 4) * (w // 16) + j // 16) + i % 4 for i in range(h) for j in range(w)]
                cols = [j for i in range(h) for j in range(w)]
                sad = int(np.abs(a[rows, cols].astype(int) - b[rows, cols]).sum())
            else:
                sad = int(np.abs(a[:h, :w].astype(int) - b[:h, :w]).sum())
            assert g.sad_calc_simd_unaligned(ptr(a), ptr(b), S, S, w, h) == sad, (w, h)


def test_transform_simd_fuzz_vs_oracle(g):
    """Extra random residuals (all sizes / fast flags) against the oracle."""
    import oracle

    o = oracle.load()
    rng = np.random.default_rng(99)
    for N in (4, 8, 16, 32, 64):
        for fast in ((0, 1) if N >= 32 else (0,)):
            for _ in range(12):
                blk = rng.integers(-255, 256, (N, N)).astype(np.int16)
                got = np.zeros((N, N), np.int16)
                want = np.zeros((N, N), np.int16)
                g.transform_simd(ptr(blk), ptr(got), N, fast)
                o.or_transform(ptr(blk), ptr(want), N, fast)
                q = min(N, 16)
                assert np.array_equal(got[:q, :q], want[:q, :q]), (N, fast)

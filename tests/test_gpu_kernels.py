"""Kernel-level GPU parity: the per-block SIMD surface (executed on the GPU)
against the CPU oracle on seeded random inputs, every fractional position,
size and filter table."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _libs():
    import oracle
    from thor_amd import lib as L

    g = L.load()
    o = oracle.load()
    P, i = C.c_void_p, C.c_int
    g.get_inter_prediction_luma_simd.argtypes = [i, i, i, i, P, i, P, i, i]
    g.get_inter_prediction_chroma_simd.argtypes = [i, i, i, i, P, i, P, i]
    return g, o


@pytest.mark.parametrize("bipred", [0, 1])
def test_luma_mc_all_fracs(bipred):
    g, o = _libs()
    rng = np.random.default_rng(7 + bipred)
    bad = []
    for w, h in [(4, 4), (8, 8), (16, 16), (32, 32), (64, 64), (8, 24), (40, 16)]:
        for fy in range(4):
            for fx in range(4):
                if fx == 0 and fy == 0:
                    continue
                S = 128
                ref = rng.integers(0, 256, (S, S), dtype=np.uint8)
                org = 8 * S + 8
                out_g = np.zeros((h, w), np.uint8)
                out_o = np.zeros((h, w), np.uint8)
                ip = ref.ctypes.data + org
                g.get_inter_prediction_luma_simd(w, h, fx, fy, out_g.ctypes.data, w, ip, S, bipred)
                o.or_mc_luma(out_o.ctypes.data, w, ip, S, w, h, fx, fy, 0, bipred)
                if not np.array_equal(out_g, out_o):
                    d = np.argwhere(out_g != out_o)
                    bad.append((w, h, fx, fy, len(d), d[:3].tolist(), out_g[tuple(d[0])], out_o[tuple(d[0])]))
    assert not bad, bad[:8]


def test_chroma_mc_all_fracs():
    g, o = _libs()
    rng = np.random.default_rng(11)
    bad = []
    for w, h in [(2, 2), (4, 4), (8, 8), (16, 16), (32, 32), (4, 12), (20, 8)]:
        for fy in range(8):
            for fx in range(8):
                if fx == 0 and fy == 0:
                    continue
                S = 96
                ref = rng.integers(0, 256, (S, S), dtype=np.uint8)
                ip = ref.ctypes.data + 6 * S + 6
                out_g = np.zeros((h, w), np.uint8)
                out_o = np.zeros((h, w), np.uint8)
                g.get_inter_prediction_chroma_simd(w, h, fx, fy, out_g.ctypes.data, w, ip, S)
                o.or_mc_chroma(out_o.ctypes.data, w, ip, S, w, h, fx, fy, 0)
                if not np.array_equal(out_g, out_o):
                    bad.append((w, h, fx, fy, int((out_g != out_o).sum())))
    assert not bad, bad[:8]

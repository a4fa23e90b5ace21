"""Batched encoder transform-block chain (thor_enc_tu_batch) and cost_calc
(thor_enc_cost_batch) on the GPU, against the reference's own functions
composed per TU (tests/golden/enc_tu.npz, tools/make_enc_goldens.py) and
against the oracle (or_encode_tu) on a larger random batch."""
import ctypes as C
import os

import numpy as np
import pytest

from conftest import GOLD

pytestmark = pytest.mark.gpu

TU_DTYPE = np.dtype([("orig_off", "<i4"), ("pred_off", "<i4"), ("rec_off", "<i4"), ("coeff_off", "<i4"),
                     ("orig_stride", "<i4"), ("pred_stride", "<i4"), ("rec_stride", "<i4"), ("size", "u1"),
                     ("qp", "u1"), ("type", "u1"), ("fast", "u1")])
assert TU_DTYPE.itemsize == 32


class Dev:
    """Device buffers through the library's own C-ABI helpers (no torch)."""

    def __init__(self, L):
        self.L, self.bufs = L, []

    def put(self, arr):
        arr = np.ascontiguousarray(arr)
        p = self.L.thor_dev_alloc(max(arr.nbytes, 4))
        assert p
        self.bufs.append(p)
        assert self.L.thor_h2d(p, arr.ctypes.data, arr.nbytes) == 0
        return p

    def empty(self, nbytes):
        p = self.L.thor_dev_alloc(max(nbytes, 4))
        assert p
        self.bufs.append(p)
        return p

    def get(self, p, shape, dtype):
        out = np.empty(shape, dtype)
        assert self.L.thor_d2h(out.ctypes.data, p, out.nbytes) == 0
        return out

    def free(self):
        for p in self.bufs:
            self.L.thor_dev_free(p)


def run_batch(L, metas, origs, preds):
    """metas: list of (size, qp, type, fast); origs/preds: (n, 64, 64) u8."""
    n = len(metas)
    tus = np.zeros(n, TU_DTYPE)
    q = [min(m[0], 16) for m in metas]
    coff = np.concatenate([[0], np.cumsum([x * x for x in q])]).astype(np.int64)
    for k, (size, qp, typ, fast) in enumerate(metas):
        tus[k] = (k * 4096, k * 4096, k * 4096, coff[k], 64, 64, 64, size, qp, typ, fast)
    D = Dev(L)
    try:
        d_tus = D.put(tus)
        d_org = D.put(origs.astype(np.uint8))
        d_pred = D.put(preds.astype(np.uint8))
        d_rec = D.empty(n * 4096)
        d_cq = D.empty(int(coff[-1]) * 2)
        d_cbp = D.empty(n)
        d_ssd = D.empty(n * 4)
        assert L.thor_enc_tu_batch(d_tus, n, d_org, d_pred, d_rec, d_cq, d_cbp, d_ssd, None) == 0
        rec = D.get(d_rec, (n, 64, 64), np.uint8)
        cq = D.get(d_cq, (int(coff[-1]),), np.int16)
        cbp = D.get(d_cbp, (n,), np.uint8)
        ssd = D.get(d_ssd, (n,), np.uint32)
    finally:
        D.free()
    levels = [cq[coff[k]:coff[k + 1]].reshape(q[k], q[k]) for k in range(n)]
    return rec, levels, cbp, ssd


@pytest.fixture(scope="module")
def L():
    from thor_amd import lib

    return lib.load()


def test_enc_tu_batch_vs_reference_chain(L):
    E = np.load(os.path.join(GOLD, "enc_tu.npz"))
    meta = E["enc_meta"]
    rec, levels, cbp, ssd = run_batch(L, [tuple(int(v) for v in m[:4]) for m in meta], E["enc_orig"], E["enc_pred"])
    bad = []
    for k, (size, qp, typ, fast, want_cbp) in enumerate(meta):
        size = int(size)
        q = min(size, 16)
        if cbp[k] != want_cbp:
            bad.append(("cbp", k))
        if not np.array_equal(levels[k], E["enc_levels"][k][:q, :q]):
            bad.append(("levels", k, size, int(qp), int(typ), int(fast)))
        if not np.array_equal(rec[k][:size, :size], E["enc_rec"][k][:size, :size]):
            bad.append(("rec", k))
        if ssd[k] != E["enc_ssd"][k]:
            bad.append(("ssd", k))
    assert not bad, bad[:10]


def test_enc_tu_batch_fuzz_vs_oracle(L):
    import oracle

    o = oracle.load()
    rng = np.random.default_rng(4242)
    n = 600
    metas, origs, preds = [], np.zeros((n, 64, 64), np.uint8), np.zeros((n, 64, 64), np.uint8)
    for k in range(n):
        size = int(rng.choice([4, 8, 16, 32, 64]))
        metas.append((size, int(rng.integers(0, 52)), int(rng.integers(0, 4)), int(rng.integers(0, 2)) if size >= 32 else 0))
        spread = int(rng.choice([3, 20, 255]))
        base = rng.integers(0, 256, (64, 64))
        origs[k] = base
        preds[k] = np.clip(base + rng.integers(-spread, spread + 1, (64, 64)), 0, 255)
    rec, levels, cbp, ssd = run_batch(L, metas, origs, preds)
    bad = []
    for k, (size, qp, typ, fast) in enumerate(metas):
        q = min(size, 16)
        r = np.zeros((64, 64), np.uint8)
        lv = np.zeros(q * q, np.int16)
        s = C.c_uint32()
        org, pb = np.ascontiguousarray(origs[k]), np.ascontiguousarray(preds[k])
        c = o.or_encode_tu(org.ctypes.data, 64, pb.ctypes.data, 64, r.ctypes.data, 64, size, qp, typ, fast,
                           lv.ctypes.data, C.byref(s))
        if (c, s.value) != (cbp[k], ssd[k]) or not np.array_equal(lv.reshape(q, q), levels[k]) or not np.array_equal(
                r[:size, :size], rec[k][:size, :size]):
            bad.append((k, size, qp, typ, fast))
    assert not bad, bad[:10]


def test_enc_tu_batch_rejects_bad_descriptor(L):
    rec, levels, cbp, ssd = run_batch(L, [(12, 30, 0, 0), (8, 60, 0, 0), (8, 30, 0, 0)], np.zeros((3, 64, 64)),
                                      np.zeros((3, 64, 64)))
    assert cbp.tolist() == [255, 255, 0]


def test_enc_cost_batch(L):
    """cost_calc (enc/encode_block.c:1218-1228): SSD_Y+SSD_U+SSD_V +
    (int32)(lambda*nbits + 0.5), clamp 2^30; lambda in double without FMA."""
    rng = np.random.default_rng(3)
    ncu = 500
    counts = rng.integers(1, 13, ncu).astype(np.int32)
    first = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int32)
    ssd = rng.integers(0, 1 << 22, int(counts.sum())).astype(np.uint32)
    ssd[:40] = 1 << 27  # some candidates hit the 2^30 clamp
    nbits = rng.integers(0, 5000, ncu).astype(np.int32)
    lam = 0.57 * 2 ** (37 / 3.0 - 4)  # a representative lambda (coeff * squared_lambda_QP)
    D = Dev(L)
    try:
        p = [D.put(x) for x in (ssd, first, counts, nbits)]
        d_cost = D.empty(ncu * 4)
        assert L.thor_enc_cost_batch(p[0], p[1], p[2], p[3], lam, d_cost, ncu, None) == 0
        cost = D.get(d_cost, (ncu,), np.uint32)
    finally:
        D.free()
    for c in range(ncu):
        s = int(ssd[first[c]:first[c] + counts[c]].sum())
        v = s + int(np.int32(np.float64(lam) * np.float64(nbits[c]) + 0.5))
        v = min(v & 0xFFFFFFFF, 1 << 30) if v <= (1 << 30) else (1 << 30)
        assert cost[c] == v, c


def test_enc_cost_batch_vs_reference_cost_calc(L):
    """k_enc_cost against the reference's own cost_calc (tests/golden/cost.npz,
    tools/make_cost_goldens.py: ssd_calc + cost_calc of libthor_ref.so on
    random blocks of every CU size, the encoder's lambda range and the 2^30
    clamp): the three SSDs of each case as three TUs of one candidate."""
    import os

    from conftest import GOLD

    z = np.load(os.path.join(GOLD, "cost.npz"))
    ssd, nbits, lam, want = z["ssd"], z["nbits"], z["lam"], z["cost"]
    D = Dev(L)
    try:
        first, counts = np.zeros(1, np.int32), np.full(1, 3, np.int32)
        p_first, p_counts = D.put(first), D.put(counts)
        d_cost = D.empty(4)
        for i in range(len(want)):
            p_ssd, p_nb = D.put(np.ascontiguousarray(ssd[i])), D.put(nbits[i:i + 1])
            assert L.thor_enc_cost_batch(p_ssd, p_first, p_counts, p_nb, float(lam[i]), d_cost, 1, None) == 0
            got = D.get(d_cost, (1,), np.uint32)[0]
            assert got == want[i], (i, int(got), int(want[i]))
    finally:
        D.free()

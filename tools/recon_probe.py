#!/usr/bin/env python3
"""Diagnostic: k_recon phase timing from in-kernel s_memrealtime stamps (100 MHz)
on a stream's P frames.  Stamps: 0 start, 1 frame context loaded, 2 P0 (MC params), 4 first
window staged, 3 prediction done, 5 end; 7 = HW_ID | XCC_ID << 32."""
import ctypes as C, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from thor_amd.decoder import GpuDecoder
from thor_amd.trace import load_trace
from thor_amd import lib as L

name = sys.argv[1] if len(sys.argv) > 1 else "k4_low"
seq, frames = load_trace(os.path.join(ROOT, "tests/golden/%s.trc.z" % name))
dec = GpuDecoder(seq)
lib = L.load()
lib.thor_dec_debug_recon.argtypes = [C.c_void_p, C.c_void_p]
nsb = ((seq.width + 63) // 64) * ((seq.height + 63) // 64)
nwg = 8 * (((((seq.width + 63) // 64 + 1) // 2) * 4 * ((seq.height + 63) // 64) + 7) // 8)  # k_recon units
nbytes = nwg * 8 * 8
buf = lib.thor_dev_alloc(nbytes)
devs = [dec.upload(fr) for fr in frames]
for i, d in enumerate(devs):
    z = np.zeros(nbytes // 8, np.uint64)
    lib.thor_h2d(buf, z.ctypes.data, nbytes)
    lib.thor_dec_debug_recon(dec.h, buf if i > 0 else None)
    dec.decode(d)
    dec.sync()
    if i == 0:
        continue
    lib.thor_d2h(z.ctypes.data, buf, nbytes)
    raw = z.reshape(nwg, 8)
    ok = (raw[:, 5] > 0) & (raw[:, 3] > 0)
    t = raw[ok].astype(np.float64)
    hw = raw[ok, 7]
    t0 = t[:, 0].min()
    rel = (t[:, :7] - t0) / 100.0
    def q(v):
        return "p10 %5.2f p50 %5.2f p90 %5.2f max %5.2f" % (np.percentile(v, 10), np.median(v), np.percentile(v, 90), v.max())
    print("frame %d: waves %d span %.1f us" % (i, len(t), rel[:, 5].max()))
    print("   start      ", q(rel[:, 0]))
    print("   init  dur  ", q(rel[:, 1] - rel[:, 0]))
    print("   P0    dur  ", q(rel[:, 2] - rel[:, 1]))
    print("   stage dur  ", q(rel[:, 4] - rel[:, 2]))
    print("   filter     ", q(rel[:, 3] - rel[:, 4]))
    print("   store      ", q(rel[:, 5] - rel[:, 3]))
    print("   end        ", q(rel[:, 5]))
    cu = ((hw >> 8) & 15) | (((hw >> 12) & 1) << 4) | (((hw >> 13) & 3) << 5)
    simd = (hw >> 4) & 3
    xcc = (hw >> 32) & 15
    key = (xcc * 128 + cu) * 4 + simd
    cnt = np.bincount(key.astype(np.int64))
    cnt = cnt[cnt > 0]
    print("   waves per SIMD: distinct SIMDs %d  min %d max %d mean %.2f" % (len(cnt), cnt.min(), cnt.max(), cnt.mean()))
    # end time vs waves on the same SIMD
    per = {}
    for k, e in zip(key, rel[:, 5]):
        per.setdefault(int(k), []).append(e)
    load = np.array([len(per[int(k)]) for k in key])
    for n in sorted(set(load.tolist())):
        print("     simds with %d waves: end p50 %.2f max %.2f (%d waves)" % (n, np.median(rel[load == n, 5]), rel[load == n, 5].max(), (load == n).sum()))
    idx = np.nonzero(ok)[0]
    hsb = idx  # stamps are indexed by half SB
    sbw = (seq.width + 63) // 64
    st = rel[:, 4] - rel[:, 2]
    order = np.argsort(-st)[:12]
    print("   slowest staging: (stage us, sby, sbx, half, xcc, end)",
          [(round(st[k], 1), int(hsb[k] >> 1) // sbw, int(hsb[k] >> 1) % sbw, int(hsb[k] & 1), int(xcc[k]), round(rel[k, 5], 1)) for k in order])
    order = np.argsort(-rel[:, 5])[:12]
    print("   latest end: (end, sby, sbx, half, stage, filt)",
          [(round(rel[k, 5], 1), int(hsb[k] >> 1) // sbw, int(hsb[k] >> 1) % sbw, int(hsb[k] & 1), round(st[k], 1), round(rel[k, 3] - rel[k, 4], 1)) for k in order])
    late = rel[:, 5] > np.percentile(rel[:, 5], 95)
    print("   late 5%%: xcc histogram %s" % np.bincount(xcc[late].astype(np.int64), minlength=8).tolist())
    if i >= 2:
        break
lib.thor_dec_debug_recon(dec.h, None)

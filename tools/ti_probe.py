#!/usr/bin/env python3
"""Diagnostics of the interpolation search wavefront (k_ti_search, level 0):
per-step (ready, done) stamps of one 4K thor_interpolate_frames call ->
step compute time T, row start lag, and the hop latency between a step's
publication and its consumer's readiness.  GPU box only; prints JSON."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from thor_amd import lib as L
    from thor_amd import synth

    lib = L.load()
    lib.thor_ti_debug.argtypes = [C.c_void_p, C.c_void_p]
    w, h = 3840, 2160
    a, b = synth.synth_frame(w, h, 0, 6), synth.synth_frame(w, h, 2, 6)
    sy, sc = (w + 192 + 15) & ~15, (w // 2 + 96 + 15) & ~15

    def padded(planes):
        out = []
        for p, s, pad in zip(planes, (sy, sc, sc), (96, 48, 48)):
            ph, pw = p.shape
            full = np.zeros((ph + 2 * pad, s), np.uint8)
            full[:, :pw + 2 * pad] = np.pad(p, pad, mode="edge")
            d = lib.thor_dev_alloc(full.nbytes)
            lib.thor_h2d(d, full.ctypes.data, full.nbytes)
            out.append(d + pad * s + pad)
        return L.ThorYuvPlanes(out[0], out[1], out[2], sy, sc)

    ra, rb, ro = padded(a), padded(b), padded([np.zeros_like(p) for p in a])
    t = lib.thor_ti_create(w, h, 0)
    nrows, ncols = 135, 240
    dbg = lib.thor_dev_alloc(nrows * ncols * 16)
    L.check(lib.thor_interpolate_frames(t, C.byref(ra), C.byref(rb), 96, C.byref(ro), 2, 1, None), "warm")
    lib.thor_ti_debug(t, dbg)
    L.check(lib.thor_interpolate_frames(t, C.byref(ra), C.byref(rb), 96, C.byref(ro), 2, 1, None), "probe")
    L.check(lib.thor_ti_status(t), "status")
    st = np.zeros((nrows, ncols, 2), np.uint64)
    lib.thor_d2h(st.ctypes.data, dbg, st.nbytes)
    st = (st.astype(np.int64) - int(st[:, :, 0].min())) * 10  # 100 MHz ticks -> ns
    ready, done = st[:, :, 0], st[:, :, 1]
    T = (done - ready).ravel()
    # hop: consumer (r, c) ready minus producer (r-1, c+1) done
    hop = (ready[1:, :-1] - done[:-1, 1:]).ravel()
    own = (ready[:, 1:] - done[:, :-1]).ravel()  # gap after own previous step
    pct = lambda v: {p: int(np.percentile(v, p)) for p in (10, 50, 90, 99)}
    print(json.dumps({"span_ns": int(done.max()), "T_step_ns": pct(T), "hop_ns": pct(hop), "own_gap_ns": pct(own),
                      "row_start_ns": [int(x) for x in ready[::15, 0]], "row_end_ns": [int(x) for x in done[::15, -1]]}))


if __name__ == "__main__":
    main()

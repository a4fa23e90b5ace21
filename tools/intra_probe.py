#!/usr/bin/env python3
"""Diagnostic: time the 4K I-frame intra kernel per SB row (s_memtime stamps)
with and without the wavefront waits."""
import ctypes as C, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from thor_amd.decoder import GpuDecoder
from thor_amd.trace import load_trace
from thor_amd import lib as L

seq, frames = load_trace(os.path.join(ROOT, "tests/golden/k4_low.trc.z"))
dec = GpuDecoder(seq)
lib = L.load()
lib.thor_dec_debug_intra.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
nrows = (seq.height + 63) // 64
buf = lib.thor_dev_alloc(nrows * 3 * 128)
d0 = dec.upload(frames[0])
lib.thor_dec_set_timing(dec.h, 1)
ms = (C.c_double * 6)()
for flags in [int(v) for v in os.environ.get("PROBE_FLAGS", "0,1,5").split(",")]:
    lib.thor_dec_debug_intra(dec.h, buf, flags)
    lib.thor_dec_stage_ms(dec.h, ms, 6)
    dec.decode(d0)
    dec.sync()
    lib.thor_dec_stage_ms(dec.h, ms, 6)
    h = np.zeros(nrows * 3 * 16, np.uint64)
    lib.thor_d2h(h.ctypes.data, buf, nrows * 3 * 128)
    h = h.reshape(nrows * 3, 16).astype(np.float64)
    t0 = h[:, 0].min()
    print("flags", flags, "intra ms", round(ms[2], 3))
    for task in range(0, nrows * 3):
        r, c = divmod(task, 3)
        if r % 6 and r != nrows - 1:
            continue
        busy = h[task, 1] - h[task, 0]
        print("  row %2d comp %d busy %9.0f wait %9.0f cus %d tus %d | per TU: sb %.0f A %.0f C %.0f other %.0f" % (
            r, c, busy, h[task, 2], h[task, 3], h[task, 7], h[task, 4] / max(1, h[task, 7]),
            h[task, 5] / max(1, h[task, 7]), h[task, 6] / max(1, h[task, 7]),
            (busy - h[task, 4] - h[task, 5] - h[task, 6]) / max(1, h[task, 7])))
lib.thor_dec_debug_intra(dec.h, None, 0)

#!/usr/bin/env python3
"""Speed of the temporal-interpolated reference on the GPU (tme.hip):

  1. thor_interpolate_frames on a 4K synthetic pair (frames 0 and 2 of the
     seeded clip, ratio 2 pos 1 -- dec/decode_frame.c's symmetric B case),
     wall clock over N back-to-back calls on one stream;
  2. the 4K HDB16 interp_ref golden (tests/golden/k4_hdbi.bit) decoded from
     its .bit with per-stage GPU timing (stage 6 = the interpolation).

Prints one JSON line.  GPU box only."""
from __future__ import annotations

import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from thor_amd import lib as L
    from thor_amd import synth
    from thor_amd.bitstream import parse_stream
    from thor_amd.decoder import GpuDecoder

    lib = L.load()
    w, h = 3840, 2160
    a, b = synth.synth_frame(w, h, 0, 6), synth.synth_frame(w, h, 2, 6)
    sy, sc = (w + 192 + 15) & ~15, (w // 2 + 96 + 15) & ~15
    bufs = []

    def padded(planes):
        out = []
        for p, s, pad in zip(planes, (sy, sc, sc), (96, 48, 48)):
            ph, pw = p.shape
            img = np.pad(p, pad, mode="edge")
            full = np.zeros((ph + 2 * pad, s), np.uint8)
            full[:, :pw + 2 * pad] = img
            d = lib.thor_dev_alloc(full.nbytes)
            lib.thor_h2d(d, full.ctypes.data, full.nbytes)
            bufs.append(d)
            out.append(d + pad * s + pad)
        return L.ThorYuvPlanes(out[0], out[1], out[2], sy, sc)

    ra, rb, ro = padded(a), padded(b), padded([np.zeros_like(p) for p in a])
    t = lib.thor_ti_create(w, h, 0)
    n = int(os.environ.get("TI_ITERS", "20"))
    for _ in range(3):
        L.check(lib.thor_interpolate_frames(t, C.byref(ra), C.byref(rb), 96, C.byref(ro), 2, 1, None), "interp")
    L.check(lib.thor_ti_status(t), "status")
    t0 = time.perf_counter()
    for _ in range(n):
        lib.thor_interpolate_frames(t, C.byref(ra), C.byref(rb), 96, C.byref(ro), 2, 1, None)
    L.check(lib.thor_ti_status(t), "status")
    ms = (time.perf_counter() - t0) / n * 1e3
    lib.thor_ti_destroy(t)
    for d in bufs:
        lib.thor_dev_free(d)

    seq, frames = parse_stream(open(os.path.join(ROOT, "tests", "golden", "k4_hdbi.bit"), "rb").read())
    dec = GpuDecoder(seq)
    devs = [dec.upload(f) for f in frames]
    for d in devs:  # warm pass
        dec.decode(d)
    dec.sync()
    dec2 = GpuDecoder(seq)
    devs2 = [dec2.upload(f) for f in frames]
    lib.thor_dec_set_timing(dec2.h, 1)
    t0 = time.perf_counter()
    for d in devs2:
        dec2.decode(d)
    dec2.sync()
    wall = (time.perf_counter() - t0) * 1e3
    st = (C.c_double * 7)()
    lib.thor_dec_stage_ms(dec2.h, st, 7)
    names = ["prep", "inter", "intra", "deblock", "clpf", "pad", "interp"]
    ninterp = sum(f.interp_ratio > 0 for f in frames)
    res = {"interp_frame_4k_ms": round(ms, 3),
           "k4_hdbi_decode": {"frames": len(frames), "interp_frames": ninterp, "wall_ms": round(wall, 2),
                              "stage_ms": {k: round(v, 3) for k, v in zip(names, st)},
                              "interp_ms_per_frame": round(st[6] / max(ninterp, 1), 3)}}
    dec.close()
    dec2.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()

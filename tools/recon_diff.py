#!/usr/bin/env python3
"""Diagnostic (GPU box): decode a golden stream's trace pre-deblock (stop stage
0) on the GPU and on the oracle, frame by frame; print where they differ
(per plane: count, first positions, max |diff|, and the 64x32 half SBs hit).
  recon_diff.py [stream] [max_frames]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import OracleDecoder  # noqa: E402
from thor_amd.decoder import GpuDecoder  # noqa: E402
from thor_amd.trace import load_trace  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "cif_low"
nmax = int(sys.argv[2]) if len(sys.argv) > 2 else 4
seq, frames = load_trace(os.path.join(ROOT, "tests", "golden", name + ".trc.z"))
W, H = seq.width, seq.height
g = GpuDecoder(seq)
o = OracleDecoder(seq)
for k, fr in enumerate(frames[:nmax]):
    g.set_stop_stage(0)
    g.decode(g.upload(fr))
    got = np.frombuffer(g.read_i420(fr.frame_num), np.uint8)
    want = np.frombuffer(o.decode(fr, 0).i420(), np.uint8)
    offs = [(0, W, H, "Y"), (W * H, W // 2, H // 2, "U"), (W * H * 5 // 4, W // 2, H // 2, "V")]
    for off, w, h, nm in offs:
        a = got[off:off + w * h].reshape(h, w).astype(int)
        b = want[off:off + w * h].reshape(h, w).astype(int)
        d = np.argwhere(a != b)
        if len(d):
            sc = 1 if nm == "Y" else 2
            halves = sorted({(int(y) * sc // 32, int(x) * sc // 64) for y, x in d})
            if nm == "Y":  # the CU over the first differing pixels: its MV / fraction
                b = fr.blocks
                for y, x in d[:1]:
                    m = (b["ypos"] <= y) & (y < b["ypos"].astype(int) + b["size"]) & (b["xpos"] <= x) & (
                        x < b["xpos"].astype(int) + b["size"])
                    for r in b[m]:
                        print("   px (%d,%d) in CU at (%d,%d) size %d mode %d mv0 %s ref0 %d mv1 %s ref1 %d dir %d" % (
                            y, x, r["ypos"], r["xpos"], r["size"], r["mode"], r["mv0"][:2].tolist(), r["ref0"],
                            r["mv1"][:2].tolist(), r["ref1"], r["dir"]))
                print("   columns mod 4 of differing px:", np.bincount(d[:, 1] % 4, minlength=4).tolist(),
                      "diff values:", np.unique((a - b)[a != b])[:10].tolist())
            print("frame %d (%s) %s: %d px differ, max %d, first %s, halves(row32,col64) %s" % (
                k, "I" if fr.frame_type == 0 else "P/B", nm, len(d), int(np.abs(a - b).max()), d[:4].tolist(),
                halves[:8]))
    # keep both chains on the exact reference
    g.set_stop_stage(2)
    g.decode(g.upload(fr))
    o.push_reference(o.decode(fr, 2))
print("done")

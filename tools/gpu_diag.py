#!/usr/bin/env python3
"""GPU-vs-oracle diagnostic (test infrastructure): decode a trace on the GPU and
with the oracle, and for each frame/stage report mismatching pixels with the
CU that covers them.  Usage: python tools/gpu_diag.py <stream> [max_frames]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import OracleDecoder  # noqa: E402
from thor_amd.decoder import GpuDecoder  # noqa: E402
from thor_amd.trace import load_trace  # noqa: E402


def cu_at(blocks, y, x):
    for i, b in enumerate(blocks):
        if b["ypos"] <= y < b["ypos"] + b["size"] and b["xpos"] <= x < b["xpos"] + b["size"]:
            return i, b
    return -1, None


def main():
    name = sys.argv[1]
    nmax = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    seq, frames = load_trace(os.path.join(ROOT, "tests", "golden", name + ".trc.z"))
    frames = frames[:nmax]
    g = GpuDecoder(seq)
    o = OracleDecoder(seq)
    for fr in frames:
        dev = g.upload(fr)
        for stage in (0, 1, 2):
            g.set_stop_stage(stage)
            g.decode(dev)
            g.sync()
            gp = g.read(fr.frame_num)
            op = o.decode(fr, stage).planes()
            for pn, a, b in zip("YUV", gp, op):
                bad = np.argwhere(a != b)
                if len(bad):
                    print("frame %d stage %d plane %s: %d bad px" % (fr.decode_order, stage, pn, len(bad)))
                    for (y, x) in bad[:6]:
                        sc = 1 if pn == "Y" else 2
                        i, blk = cu_at(fr.blocks, y * sc, x * sc)
                        desc = {k: (blk[k].tolist() if hasattr(blk[k], "tolist") else blk[k]) for k in blk.dtype.names} if blk is not None else None
                        print("   (%d,%d) gpu=%d oracle=%d cu#%d %s" % (y, x, a[y, x], b[y, x], i, desc))
                    if stage == 0:
                        break
        o.push_reference(o.decode(fr, 2))
        print("frame %d done" % fr.decode_order, flush=True)
    g.close()


if __name__ == "__main__":
    main()

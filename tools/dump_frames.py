#!/usr/bin/env python3
"""Diagnostic: decode the first N frames of a stream on the GPU (stage 0 = pre-deblock)
and with the oracle; save both as npz under gpurun_out/ for offline comparison."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import OracleDecoder
from thor_amd.decoder import GpuDecoder
from thor_amd.trace import load_trace

name = sys.argv[1]
n = int(sys.argv[2])
stage = int(sys.argv[3]) if len(sys.argv) > 3 else 0
seq, frames = load_trace(os.path.join(ROOT, "tests", "golden", name + ".trc.z"))
g, o = GpuDecoder(seq), OracleDecoder(seq)
out = {}
for fr in frames[:n]:
    dev = g.upload(fr)
    g.set_stop_stage(stage)
    g.decode(dev)
    g.sync()
    gp = g.read(fr.frame_num)
    op = o.decode(fr, stage).planes()
    for pn, a, b in zip("YUV", gp, op):
        out["g%d%s" % (fr.decode_order, pn)] = a
        out["o%d%s" % (fr.decode_order, pn)] = b
    # continue from the exact reference: restore both to the final stage
    g.set_stop_stage(2)
    g.decode(dev)
    o.push_reference(o.decode(fr, 2))
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", "dump_%s.npz" % name), **out)
print("saved", len(out))

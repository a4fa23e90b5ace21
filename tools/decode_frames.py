#!/usr/bin/env python3
"""Profiling driver: reconstruct the first N frames of a golden stream once on
cuda:0 (no timing, no checks) so rocprofv3 sees exactly one dispatch per kernel
per frame.  Usage: decode_frames.py [stream] [nframes]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from thor_amd.decoder import GpuDecoder  # noqa: E402
from thor_amd.trace import load_trace  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "k4_low"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1
seq, frames = load_trace(os.path.join(ROOT, "tests", "golden", name + ".trc.z"))
dec = GpuDecoder(seq)
devs = [dec.upload(fr) for fr in frames[:n]]
for d in devs:
    dec.decode(d)
dec.sync()
dec.close()
print("decoded", len(devs), "frames of", name)

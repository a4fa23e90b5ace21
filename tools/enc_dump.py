#!/usr/bin/env python3
"""Encode a golden clip on the GPU and write the .bit (and optionally the
reconstruction of every frame) under gpurun_out/, for offline comparison
with the reference .bit / the host harness (tools/enc_host)."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from thor_amd import synth  # noqa: E402
from thor_amd.encoder import GpuEncoder, params_for  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("name")
    ap.add_argument("--frames", type=int, default=0)
    ap.add_argument("--recon", action="store_true")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out"))
    a = ap.parse_args()
    meta = json.load(open(os.path.join(ROOT, "tests", "golden", "streams.json")))[a.name]
    n = a.frames or meta["frames"]
    w, h = meta["width"], meta["height"]
    clip = synth.synth_frames(w, h, n, meta["seed"], workers=8)
    enc = GpuEncoder(params_for(meta["config"], w, h, n, meta["extra"]))
    enc.upload_sequence(clip)
    want = open(os.path.join(ROOT, "tests", "golden", a.name + ".bit"), "rb").read()
    os.makedirs(a.out, exist_ok=True)
    bits, rec = b"", []
    for i in range(enc.num_frames()):
        ch = enc.encode_next()
        o = len(bits)
        bits += ch
        same = want[o:o + len(ch)] == ch
        print("frame", i, "bytes", len(ch), "match" if same else "DIFF", flush=True)
        if a.recon:
            y = np.empty(w * h * 3 // 2, np.uint8)
            enc.lib.thor_enc_read_recon(enc.h, y.ctypes.data, y[w * h:].ctypes.data, y[w * h * 5 // 4:].ctypes.data)
            rec.append(y)
    open(os.path.join(a.out, a.name + "_gpu.bit"), "wb").write(bits)
    if rec:
        np.stack(rec).tofile(os.path.join(a.out, a.name + "_gpu_rec.yuv"))
    enc.close()


if __name__ == "__main__":
    main()

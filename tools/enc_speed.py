#!/usr/bin/env python3
"""Device encoder timing probe: code a golden clip with B concurrent contexts
(thor_enc_frames batches), check every stream's bits against the reference
.bit, report per-frame wall times."""
import argparse
import json
import os
import sys
import time


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from thor_amd import synth  # noqa: E402
from thor_amd.encoder import GpuEncoder, encode_batch, params_for  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--name", default="k4_low")
    ap.add_argument("--batch", type=int, nargs="+", default=[1, 8])
    ap.add_argument("--frames", type=int, default=0)
    ap.add_argument("--limit", type=int, default=0,
                    help="code only the first LIMIT coded frames of the plan (the GOP as for --frames)")
    a = ap.parse_args()
    meta = json.load(open(os.path.join(ROOT, "tests", "golden", "streams.json")))[a.name]
    n = a.frames or meta["frames"]
    w, h = meta["width"], meta["height"]
    frames = synth.synth_frames(w, h, n, meta["seed"], workers=8)  # before any GPU call (fork)
    want = open(os.path.join(ROOT, "tests", "golden", a.name + ".bit"), "rb").read()
    res = {}
    for B in a.batch:
        encs = [GpuEncoder(params_for(meta["config"], w, h, n, meta["extra"])) for _ in range(B)]
        for e in encs:
            e.upload_sequence(frames)
        out = [b""] * B
        t_frames = []
        for i in range(a.limit or n):
            t0 = time.perf_counter()
            ch = encode_batch(encs)
            t_frames.append(time.perf_counter() - t0)
            print("  frame %d: %.1f ms" % (i, 1e3 * t_frames[-1]), flush=True)  # progress (long speed-0 frames)
            for k in range(B):
                out[k] += ch[k]
        ok = all(o == want[:len(o)] for o in out) and len(out[0]) == len(want) if (
            n == meta["frames"] and not a.limit) else all(want.startswith(o) for o in out)
        tot = sum(t_frames)
        res[B] = dict(ok=ok, total_s=tot, frame_ms=[round(1000 * t, 2) for t in t_frames],
                      mpx_s=B * w * h * (a.limit or n) / tot / 1e6)
        print(a.name, "batch", B, json.dumps(res[B]), flush=True)
        for e in encs:
            e.close()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Device encoder cycle profile: builds libthor_amd_prof.so (-DTHOR_ENC_PROFILE:
s_memtime accounting per RD function, lane 0 of every wave) and codes a clip,
printing cycles and calls per category per frame type.  Diagnostic only.
  python tools/enc_profile.py --build      (in the build container)
  python tools/enc_profile.py --name k4_low --frames 2   (on the GPU box)"""
import argparse
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "thor_amd", "libthor_amd_prof.so")
CATS = ["wcoef", "wblock", "inter_comp", "intra_comp", "enc_block", "cost", "search_intra", "me", "mode",
        "es_check", "es_search", "commit", "mc_y", "mc_c", "fwd", "quant", "inv", "ipred", "topleft", "sad", "sb",
        "wait"]


def build():
    src = os.path.join(ROOT, "thor_amd", "csrc", "libthor_amd.hip")
    sys.path.insert(0, ROOT)
    from thor_amd.build import FLAGS, HIPCC  # the product's flags, plus the cycle accounting

    subprocess.run([HIPCC] + FLAGS + ["-w", "-DTHOR_ENC_PROFILE", "-o", LIB, src], check=True, cwd=os.path.dirname(src))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--name", default="k4_low")
    ap.add_argument("--frames", type=int, default=2)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--limit", type=int, default=0, help="code only the first LIMIT coded frames of the plan")
    a = ap.parse_args()
    if a.build:
        build()
        return
    os.environ["THOR_AMD_LIB"] = LIB
    sys.path.insert(0, ROOT)
    from thor_amd import lib as L, synth
    from thor_amd.encoder import GpuEncoder, encode_batch, params_for
    lib = L.load(LIB)
    lib.thor_enc_profile_buffer.argtypes = [C.c_void_p]
    meta = json.load(open(os.path.join(ROOT, "tests", "golden", "streams.json")))[a.name]
    w, h, n = meta["width"], meta["height"], a.frames
    frames = synth.synth_frames(w, h, n, meta["seed"], workers=8)
    encs = [GpuEncoder(params_for(meta["config"], w, h, n, meta["extra"])) for _ in range(a.batch)]
    for e in encs:
        e.upload_sequence(frames)
    buf = lib.thor_dev_alloc(2 * 8 * 64)
    lib.thor_enc_profile_buffer(buf)
    for i in range(a.limit or n):
        zero = np.zeros(128, np.uint64)
        lib.thor_h2d(buf, zero.ctypes.data, zero.nbytes)
        import time
        t0 = time.perf_counter()
        encode_batch(encs)
        dt = time.perf_counter() - t0
        out = np.zeros(128, np.uint64)
        lib.thor_d2h(out.ctypes.data, buf, out.nbytes)
        tot = out[2 * CATS.index("sb")]
        print("frame %d: %.1f ms, SB cycles total %.3g" % (i, dt * 1e3, tot))
        for k, c in enumerate(CATS):
            cyc, cnt = int(out[2 * k]), int(out[2 * k + 1])
            if cnt:
                print("  %-12s %6.2f%%  calls %9d  cycles/call %9.0f" % (c, 100.0 * cyc / max(tot, 1), cnt, cyc / cnt))
        sys.stdout.flush()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Device encoder decision trace (diagnostic only): builds libthor_amd_trace.so
(-DTHOR_ENC_TRACE, TE_TR records in enc_rd.h) and codes a golden clip,
writing the records of one frame to gpurun_out/<name>_f<frame>_dev.trc; the
host harness (tools/enc_host/enc_host_trace -trace_frame F -trace_out f)
writes the same records from the serial build.  `--compare a b` lines the two
up per superblock and prints the first differing record.
  python tools/enc_trace.py --build                      (build container)
  python tools/enc_trace.py --name cif_high --frames 4 --frame 3   (GPU box)
  python tools/enc_trace.py --compare host.trc dev.trc"""
import argparse
import json
import os
import subprocess
import sys
from collections import defaultdict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "thor_amd", "libthor_amd_trace.so")
KINDS = {1: "me", 2: "enc_block", 3: "cost", 4: "bipred", 5: "mode_dec", 6: "dqp", 7: "bip_org8", 8: "bip_mv",
         9: "me_int", 10: "pb", 11: "ref", 12: "pred_q"}


def build():
    src = os.path.join(ROOT, "thor_amd", "csrc", "libthor_amd.hip")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                    "-ffp-contract=off", "-DTHOR_ENC_TRACE", "-o", LIB, src], check=True, cwd=os.path.dirname(src))


def per_sb(recs):
    d = defaultdict(list)
    for r in recs:
        if r[1] == 13:  # device-only (exec mask)
            continue
        d[(int(r[2]) // 64, int(r[3]) // 64)].append(tuple(int(v) for v in r))
    return d


def compare(a, b):
    A = per_sb(np.fromfile(a, np.int32).reshape(-1, 8))
    B = per_sb(np.fromfile(b, np.int32).reshape(-1, 8))
    for key in sorted(set(A) & set(B)):
        x, y = A.get(key, []), B.get(key, [])
        for i, (p, q) in enumerate(zip(x, y)):
            if p != q:
                print("SB", key, "record", i, "of", len(x), len(y))
                for j in range(max(0, i - 6), min(i + 4, len(x), len(y))):
                    print("  %s %-9s %s | %s" % ("*" if x[j] != y[j] else " ", KINDS.get(x[j][1], x[j][1]), x[j][2:],
                                                 y[j][2:]))
                return 1
        if len(x) != len(y):
            print("SB", key, "record counts differ", len(x), len(y))
            return 1
    print("traces identical:", sum(len(v) for v in A.values()), "records")
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--compare", nargs=2)
    ap.add_argument("--name", default="cif_high")
    ap.add_argument("--frames", type=int, default=4)
    ap.add_argument("--frame", type=int, default=3)
    ap.add_argument("--sb-rows", type=int, default=1, help="keep the records of the first N SB rows (0: all)")
    a = ap.parse_args()
    if a.build:
        return build()
    if a.compare:
        return compare(*a.compare)
    os.environ["THOR_AMD_LIB"] = LIB
    sys.path.insert(0, ROOT)
    import ctypes as C

    from thor_amd import lib as L, synth
    from thor_amd.encoder import GpuEncoder, params_for

    meta = json.load(open(os.path.join(ROOT, "tests", "golden", "streams.json")))[a.name]
    w, h, n = meta["width"], meta["height"], a.frames
    clip = synth.synth_frames(w, h, n, meta["seed"], workers=8)
    lib = L.load(LIB)
    lib.thor_enc_trace_buffer.argtypes = [C.c_void_p, C.c_uint, C.c_int]
    cap = 1 << 22
    buf = lib.thor_dev_alloc(4 * (8 + 8 * cap))
    zero = np.zeros(8, np.int32)
    lib.thor_h2d(buf, zero.ctypes.data, zero.nbytes)
    lib.thor_enc_trace_buffer(buf, cap, a.frame)
    enc = GpuEncoder(params_for(meta["config"], w, h, n, meta["extra"]))
    enc.upload_sequence(clip)
    for _ in range(n):
        enc.encode_next()
    cnt = np.zeros(8, np.int32)
    lib.thor_d2h(cnt.ctypes.data, buf, cnt.nbytes)
    m = min(int(cnt[0]), cap)
    recs = np.zeros((m, 8), np.int32)
    lib.thor_d2h(recs.ctypes.data, buf + 32, recs.nbytes)
    keep = (recs[:, 2] < 64 * a.sb_rows) if a.sb_rows else np.ones(len(recs), bool)
    recs = recs[keep]  # gpurun returns at most 64 MiB
    out = os.path.join(ROOT, "gpurun_out", "%s_f%d_dev.trc" % (a.name, a.frame))
    os.makedirs(os.path.dirname(out), exist_ok=True)
    recs.tofile(out)
    print("records", int(cnt[0]), "->", out)


if __name__ == "__main__":
    sys.exit(main())

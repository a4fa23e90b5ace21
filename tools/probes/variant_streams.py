#!/usr/bin/env python3
"""Diagnostics: decode golden streams with a given build of the library
(argv[1]) and report the first frame/stage whose md5 differs from the
reference decoder's."""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from thor_amd import lib as L  # noqa: E402

L.load(os.path.abspath(sys.argv[1]))
from thor_amd.decoder import GpuDecoder  # noqa: E402
from thor_amd.trace import load_trace  # noqa: E402

meta = json.load(open(os.path.join(ROOT, "tests", "golden", "streams.json")))
for name in sys.argv[2:]:
    seq, frames = load_trace(os.path.join(ROOT, "tests", "golden", name + ".trc.z"))
    dec = GpuDecoder(seq)
    bad = None
    devs = [dec.upload(fr) for fr in frames]
    for fr, d in zip(frames, devs):
        dec.decode(d)
        dec.sync()
        got = hashlib.md5(dec.read_i420(fr.frame_num)).hexdigest()
        if got != meta[name]["stage_md5"][fr.decode_order]["final"]:
            bad = fr.decode_order
            break
    dec.close()
    print(os.path.basename(sys.argv[1]), name, "OK" if bad is None else "first bad frame %d" % bad,
          flush=True)

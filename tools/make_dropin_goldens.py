#!/usr/bin/env python3
"""Golden digests for the drop-in link test (TEST INFRASTRUCTURE; build
container only).

Encodes small seeded synthetic clips (thor_amd/synth.py) with the reference
Thorenc (oracle/_ref/Thorenc, compiled from /root/reference, SIMD path) and
records the bitstream and reconstruction md5s in tests/golden/dropin.json.
On the GPU box, tests/test_gpu_dropin.py runs oracle/_ref/thorenc_amd -- the
same reference encoder host C with common/common_kernels.c and
enc/enc_kernels.c replaced by libthor_amd.so, every SIMD-surface call
executing on the GPU -- on the same clip and must produce the identical
bitstream (so every RD decision, i.e. every RD cost, matched).
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from thor_amd import synth  # noqa: E402

REF = os.environ.get("THOR_REF", "/root/reference")
OREF = os.path.join(ROOT, "oracle", "_ref")
OUT = os.path.join(ROOT, "tests", "golden", "dropin.json")

# name, width, height, frames, config, extra flags, seed
CLIPS = [
    ("tiny_low", 128, 64, 3, "config_LDB_low_complexity.txt", [], 11),
    ("tiny_high", 128, 64, 2, "config_LDB_high_efficiency.txt", ["-qp", "22"], 12),
    ("tiny_med", 128, 64, 3, "config_LDB_medium_complexity.txt", [], 13),
]


def write_clip(path, w, h, n, seed):
    with open(path, "wb") as f:
        for t in range(n):
            for p in synth.synth_frame(w, h, t, seed):
                f.write(p.tobytes())


def config_flags(cfg_path):
    """The option values of a reference config file (`-flag value ; comment`
    lines, read_config_file enc/strings.c:64-122) as a flag list, minus the
    I/O and size options the command line sets."""
    flags = []
    for line in open(cfg_path):
        line = line.split(";")[0].split()
        if len(line) >= 2 and line[0].startswith("-") and line[0] not in ("-if", "-of", "-rf", "-stat", "-width",
                                                                          "-height", "-n"):
            flags += line[:2]
    return flags


def encoder_cmd(exe, flags, yuv, bit, rec, stat, w, h, n, extra):
    return [exe] + list(flags) + ["-if", yuv, "-of", bit, "-rf", rec, "-stat", stat, "-width", str(w), "-height",
                                  str(h), "-n", str(n)] + list(extra)


def main():
    res = {}
    with tempfile.TemporaryDirectory() as work:
        for name, w, h, n, cfg, extra, seed in CLIPS:
            yuv, bit, rec = (os.path.join(work, name + s) for s in (".yuv", ".bit", "_rec.yuv"))
            write_clip(yuv, w, h, n, seed)
            flags = config_flags(os.path.join(REF, cfg))
            subprocess.run(encoder_cmd(os.path.join(OREF, "Thorenc"), flags, yuv, bit, rec,
                                       os.path.join(work, "st.txt"), w, h, n, extra), check=True,
                           stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            dec = os.path.join(work, name + "_dec.yuv")
            subprocess.run([os.path.join(OREF, "Thordec"), bit, dec], check=True, stdout=subprocess.DEVNULL,
                           stderr=subprocess.DEVNULL)
            md5 = lambda p: hashlib.md5(open(p, "rb").read()).hexdigest()  # noqa: E731
            assert md5(rec) == md5(dec)
            res[name] = dict(width=w, height=h, frames=n, config=cfg, flags=flags, extra=extra, seed=seed,
                             yuv_md5=md5(yuv), bit_md5=md5(bit), rec_md5=md5(rec), bit_bytes=os.path.getsize(bit))
            print(name, res[name])
    json.dump(res, open(OUT, "w"), indent=1)


if __name__ == "__main__":
    main()

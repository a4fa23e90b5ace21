#!/usr/bin/env python3
"""Generate tests/golden/bench_clips.json (TEST INFRASTRUCTURE, build container only).

bench.py encodes and decodes K streams drawn from 8 distinct seeded 4K clips
(thor_amd/synth.py) with config_LDB_low_complexity; every stream's .bit must
equal the reference Thorenc's for its clip and every decoded sequence the
reference Thordec's.  This script runs the reference (oracle/_ref, built from
/root/reference by oracle/Makefile) on each clip and records the md5s:

  {"clips": [{"seed": s, "synth_md5": .., "bit_md5": .., "bit_bytes": .., "dec_md5": ..}, ...],
   "width": 3840, "height": 2160, "frames": 8, "config": "config_LDB_low_complexity.txt"}

Seed 6 is tests/golden/k4_low (its full trace and stage md5s are in streams.json).
Usage: python tools/make_bench_goldens.py
"""
from __future__ import annotations

import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile
from concurrent.futures import ProcessPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from thor_amd import configs, synth  # noqa: E402

REF = os.environ.get("THOR_REF", "/root/reference")
OREF = os.path.join(ROOT, "oracle", "_ref")
SEEDS = [6, 21, 22, 23, 24, 25, 26, 27]
W, H, N, CFG = 3840, 2160, 8, "config_LDB_low_complexity.txt"


def one(seed: int, work: str) -> dict:
    clip = synth.synth_frames(W, H, N, seed, workers=1)
    yuv = os.path.join(work, "%d.yuv" % seed)
    clip.tofile(yuv)
    bit, dec = os.path.join(work, "%d.bit" % seed), os.path.join(work, "%d_dec.yuv" % seed)
    subprocess.run([os.path.join(OREF, "Thorenc"), "-cf", os.path.join(REF, CFG), "-if", yuv, "-of", bit,
                    "-rf", os.path.join(work, "%d_rec.yuv" % seed), "-stat", os.path.join(work, "%d.stat" % seed)]
                   + configs.flags(CFG, W, H, N), check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    subprocess.run([os.path.join(OREF, "Thordec"), bit, dec], check=True, stdout=subprocess.DEVNULL,
                   stderr=subprocess.DEVNULL)
    b = open(bit, "rb").read()
    d = open(dec, "rb").read()
    assert d == open(os.path.join(work, "%d_rec.yuv" % seed), "rb").read(), "encoder recon != decoder output"
    for f in (yuv, bit, dec, os.path.join(work, "%d_rec.yuv" % seed)):
        os.remove(f)
    return {"seed": seed, "synth_md5": hashlib.md5(clip.tobytes()).hexdigest(), "bit_md5": hashlib.md5(b).hexdigest(),
            "bit_bytes": len(b), "dec_md5": hashlib.md5(d).hexdigest()}


def main():
    if not os.path.isdir(os.path.join(REF, "common")):
        sys.exit("reference sources not found at %s: goldens can only be generated in the build container" % REF)
    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    work = tempfile.mkdtemp(prefix="thor_bench_gold_")
    with ProcessPoolExecutor(4) as ex:
        clips = list(ex.map(one, SEEDS, [work] * len(SEEDS)))
    shutil.rmtree(work, ignore_errors=True)
    k4 = json.load(open(os.path.join(ROOT, "tests", "golden", "streams.json")))["k4_low"]
    assert clips[0]["bit_md5"] == k4["bit_md5"] and clips[0]["dec_md5"] == k4["dec_md5"], "seed 6 != k4_low"
    out = {"width": W, "height": H, "frames": N, "config": CFG, "extra": [], "clips": clips}
    json.dump(out, open(os.path.join(ROOT, "tests", "golden", "bench_clips.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ (TEST INFRASTRUCTURE).

Runs ONLY in the build container, where the reference sources exist: it builds
oracle/_ref (reference Thorenc/Thordec + the trace-recording decoder) with
oracle/Makefile, encodes seeded synthetic clips (thor_amd/synth.py) with the
reference encoder, decodes them with the reference decoder and records

  tests/golden/<name>.bit        the reference bitstream
  tests/golden/<name>.trc.z      per-frame block-descriptor trace (zlib)
  tests/golden/streams.json      per-frame md5 of the reference decoder's frame
                                 at three stages (pre-deblock, post-deblock,
                                 final), md5 of the decoded/reconstructed .yuv,
                                 synthetic-input md5, encode/decode commands

Nothing here reads the reference at test time; the GPU box only sees the
fixtures.  Usage:  python tools/make_goldens.py [--only name ...]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from thor_amd import synth  # noqa: E402

REF = os.environ.get("THOR_REF", "/root/reference")
OREF = os.path.join(ROOT, "oracle", "_ref")
GOLD = os.path.join(ROOT, "tests", "golden")

# name, width, height, frames, config, extra encoder flags, seed
STREAMS = [
    ("cif_low", 352, 288, 10, "config_LDB_low_complexity.txt", [], 1),
    ("cif_med", 352, 288, 10, "config_LDB_medium_complexity.txt", [], 2),
    ("cif_high", 352, 288, 10, "config_LDB_high_efficiency.txt", ["-qp", "22"], 3),
    ("cif_hdb", 352, 288, 17, "config_HDB16_low_complexity.txt", ["-interp_ref", "0"], 4),
    ("hd_low", 1920, 1080, 17, "config_LDB_low_complexity.txt", [], 5),
    ("k4_low", 3840, 2160, 8, "config_LDB_low_complexity.txt", [], 6),
    # round 2: BASELINE config 4 (bi-pred at 4K), a width = 8 mod 16 clip (enc/strings.c:437)
    ("k4_med", 3840, 2160, 8, "config_LDB_medium_complexity.txt", [], 7),
    ("w8_low", 360, 288, 6, "config_LDB_low_complexity.txt", [], 8),
    # BASELINE config 3 operating point at 1080p (3 frames: the reference needs ~75 s)
    ("hd_high", 1920, 1080, 3, "config_LDB_high_efficiency.txt", [], 9),
    # temporal-interpolated references (-interp_ref 1, the HDB16 configs' default): BASELINE config 5
    ("cif_hdbi", 352, 288, 17, "config_HDB16_low_complexity.txt", [], 10),
    ("cif_hdbi_high", 352, 288, 17, "config_HDB16_high_efficiency.txt", [], 11),
    ("k4_hdbi", 3840, 2160, 17, "config_HDB16_low_complexity.txt", [], 12),
    # round 3: BASELINE config 5 at its stated size and operating point (speed 0 B frames: joint bi-pred search)
    ("k4_hdbi_high", 3840, 2160, 17, "config_HDB16_high_efficiency.txt", [], 13),
]


def md5(b: bytes) -> str:
    return hashlib.md5(b).hexdigest()


def build_ref():
    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)


def make_stream(name, w, h, n, cfg, extra, seed, work):
    yuv = os.path.join(work, name + ".yuv")
    t0 = time.time()
    with open(yuv, "wb") as f:
        for t in range(n):
            for p in synth.synth_frame(w, h, t, seed):
                f.write(p.tobytes())
    with open(yuv, "rb") as f:
        in_md5 = md5(f.read())
    bit = os.path.join(work, name + ".bit")
    rec = os.path.join(work, name + "_rec.yuv")
    enc_cmd = [os.path.join(OREF, "Thorenc"), "-cf", os.path.join(REF, cfg), "-if", yuv, "-of", bit, "-rf", rec,
               "-stat", os.path.join(work, "stat.txt"), "-width", str(w), "-height", str(h), "-n", str(n)] + extra
    t1 = time.time()
    subprocess.run(enc_cmd, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    t_enc = time.time() - t1
    dump = os.path.join(work, name + "_dump")
    os.makedirs(dump, exist_ok=True)
    trc = os.path.join(work, name + ".trc")
    dec = os.path.join(work, name + "_dec.yuv")
    env = dict(os.environ, THOR_TRACE=trc, THOR_TRACE_DUMP=dump)
    subprocess.run([os.path.join(OREF, "thordec_trace"), bit, dec], check=True, env=env,
                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    t2 = time.time()
    subprocess.run([os.path.join(OREF, "Thordec"), bit, dec + ".plain"], check=True,
                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    t_dec = time.time() - t2
    rd = open(rec, "rb").read()
    dd = open(dec, "rb").read()
    assert dd == open(dec + ".plain", "rb").read(), "trace hooks changed the decoder output"
    assert rd == dd, "encoder recon != decoder output"
    frames = []
    k = 0
    while os.path.exists(os.path.join(dump, "f%03d_final.yuv" % k)):
        fr = {}
        for st in ("pre_deblock", "post_deblock", "final"):
            fr[st] = md5(open(os.path.join(dump, "f%03d_%s.yuv" % (k, st)), "rb").read())
        frames.append(fr)
        k += 1
    shutil.copy(bit, os.path.join(GOLD, name + ".bit"))
    with open(trc, "rb") as f:
        z = zlib.compress(f.read(), 9)
    with open(os.path.join(GOLD, name + ".trc.z"), "wb") as f:
        f.write(z)
    meta = dict(width=w, height=h, frames=n, config=cfg, extra=extra, seed=seed, synth_md5=in_md5,
                bit_bytes=os.path.getsize(bit), bit_md5=md5(open(bit, "rb").read()), dec_md5=md5(dd),
                stage_md5=frames, ref_encode_s=round(t_enc, 3), ref_decode_s=round(t_dec, 3),
                gen_s=round(t1 - t0, 1))
    print(name, {k: meta[k] for k in ("bit_bytes", "dec_md5", "ref_encode_s", "ref_decode_s")}, flush=True)
    return meta


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*")
    a = ap.parse_args()
    if not os.path.isdir(os.path.join(REF, "common")):
        sys.exit("reference sources not found at %s: goldens can only be generated in the build container" % REF)
    build_ref()
    os.makedirs(GOLD, exist_ok=True)
    jpath = os.path.join(GOLD, "streams.json")
    db = json.load(open(jpath)) if os.path.exists(jpath) else {}
    work = tempfile.mkdtemp(prefix="thor_gold_")
    try:
        for s in STREAMS:
            if a.only and s[0] not in a.only:
                continue
            db[s[0]] = make_stream(*s, work)
            json.dump(db, open(jpath, "w"), indent=1, sort_keys=True)
    finally:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()

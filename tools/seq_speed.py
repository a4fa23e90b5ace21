"""Encoder A/B at the bench's workload: K x 4K LDB-low 8-frame streams (the
bench clips, tests/golden/bench_clips.json), coded
  batch : frame by frame (thor_enc_frames_begin / _end pipelined, one launch
          per stage per frame index -- bench.py's encoder leg)
  seq   : every frame in ONE sequence launch (thor_enc_seq_*), inputs resident
  fetch : the same with the raw frames read from page-locked host memory by
          the launch itself (FETCH tasks)
Each stream's .bit md5 is checked against the reference Thorenc's.
Usage: python3 tools/seq_speed.py [K] [modes, comma separated; mode:KNOB=v sets THOR_SEQ_KNOB] [reps]"""
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

K = int(sys.argv[1]) if len(sys.argv) > 1 else 240
MODES = (sys.argv[2] if len(sys.argv) > 2 else "batch,seq,fetch").split(",")
REPS = int(sys.argv[3]) if len(sys.argv) > 3 else 2

from thor_amd import synth  # noqa: E402

bc = json.load(open(os.path.join(ROOT, "tests", "golden", "bench_clips.json")))
W, H, nf = bc["width"], bc["height"], bc["frames"]
clips = [synth.synth_frames(W, H, nf, c["seed"], workers=8) for c in bc["clips"]]  # before the GPU is touched
nclip = len(clips)
fsize = W * H * 3 // 2

import torch  # noqa: E402

from thor_amd import lib as L  # noqa: E402
from thor_amd.encoder import GpuEncoder, SeqLaunch, encode_batch_begin, encode_batch_end, params_for  # noqa: E402

lib = L.load()
lib.thor_enc_debug_stall(-1, 60000)  # a wedged launch gives up after 60 s
dev = torch.device("cuda", 0)
host = [torch.from_numpy(c.reshape(nf, fsize)).pin_memory() for c in clips]
inbuf = [torch.empty((nf, fsize), dtype=torch.uint8, device=dev) for _ in range(K)]
for k in range(K):
    inbuf[k].copy_(host[k % nclip])
torch.cuda.synchronize()
encs = []
for k in range(K):
    e = GpuEncoder(params_for(bc["config"], W, H, nf, bc["extra"]))
    e.use_device_sequence(inbuf[k].data_ptr(), nf)
    encs.append(e)
want = [c["bit_md5"] for c in bc["clips"]]


def check(bits):
    bad = [k for k in range(K) if hashlib.md5(bits[k]).hexdigest() != want[k % nclip]]
    return "bit-exact" if not bad else "MISMATCH streams %s" % bad[:8]


def rows_profile():
    import ctypes as C

    v = (C.c_longlong * 3)()
    lib.thor_enc_rows_profile(0, v)
    return {"rd_ms": round(v[0] / 1e5, 1), "wait_ms": round(v[1] / 1e5, 1), "sbs": v[2]}


def run_batch(nb=None):
    """every frame per frame batch; with nb, the rows profile of the first nb frames apart"""
    for e in encs:
        e.reset()
    rows_profile()
    bits = [[] for _ in range(K)]
    prof = {}
    encode_batch_begin(encs)
    for i in range(nf):
        if i + 1 < nf and i + 1 != nb:
            encode_batch_begin(encs)
        for k, ch in enumerate(encode_batch_end(encs)):
            bits[k].append(ch)
        if nb and i + 1 == nb:
            prof["first_%d" % nb] = rows_profile()
            if nb < nf:
                encode_batch_begin(encs)
    prof["rows_profile"] = rows_profile()
    return [b"".join(b) for b in bits], prof


def run_seq(fetch, pre=0, nseq=None):
    """pre frames per frame batch first, then nseq (default: the rest) in one
    sequence launch, then the rest per frame batch"""
    for e in encs:
        e.reset()
    from thor_amd.encoder import encode_batch

    head = [[] for _ in range(K)]
    for _ in range(pre):
        for k, ch in enumerate(encode_batch(encs)):
            head[k].append(ch)
    nseq = nseq or nf - pre
    if fetch:
        for b in inbuf:
            b.zero_()
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    s = SeqLaunch(encs, nseq, host=(lambda i, k: host[i % nclip][k].data_ptr()) if fetch else None)
    first = None
    tl = []
    while True:
        r = s.ready()
        d = int((r >= 0).sum())
        if first is None and d:
            first = time.perf_counter() - t0
        if not tl or tl[-1][1] != d:
            tl.append((round((time.perf_counter() - t0) * 1e3, 1), d))
        if d == K * nseq or time.perf_counter() - t0 > 120:  # (a wedged launch gives up after 60 s)
            break
        time.sleep(0.001)
    st = s.end()
    t_seq = time.perf_counter() - t0
    tail = [[] for _ in range(K)]
    for _ in range(nf - pre - nseq):
        for k, ch in enumerate(encode_batch(encs)):
            tail[k].append(ch)
    bits = [b"".join(head[k] + [s.chunk(k, f) for f in range(nseq)] + tail[k]) for k in range(K)]
    # frames final per 100 ms
    marks = [(t, d) for t, d in tl if d in (1, K, K * nseq // 2, K * nseq)]
    return bits, {"seq_ms": round(t_seq * 1e3, 1), "stats": st, "profile": s.profile, "env": {k: v for k, v in os.environ.items() if k.startswith("THOR_SEQ")}, "first_final_ms": round(first * 1e3, 1), "marks": marks[:8]}


for spec in MODES:
    # mode[:KNOB=v[:KNOB=v]]: THOR_SEQ_<KNOB> set for this mode's runs (read at each launch)
    m, *kv = spec.split(":")
    for k in [k for k in os.environ if k.startswith("THOR_SEQ_")]:
        del os.environ[k]
    for x in kv:
        k, v = x.split("=")
        os.environ["THOR_SEQ_" + k] = v
    for r in range(REPS):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if m.startswith("batch"):  # batch[/NB]: the first NB frames' profile apart
            bits, extra = run_batch(int(m.split("/")[1]) if "/" in m else None)
        else:  # seq / fetch [ /PRE / NSEQ ]: e.g. seq/1 = frame 0 per batch, frames 1-7 in one launch
            parts = m.split("/")
            bits, extra = run_seq(parts[0] == "fetch", int(parts[1]) if len(parts) > 1 else 0,
                                  int(parts[2]) if len(parts) > 2 else None)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"mode": spec, "streams": K, "rep": r, "ms": round(dt * 1e3, 1),
                          "enc_mpx_s": round(K * nf * W * H / dt / 1e6, 1), "check": check(bits), "extra": extra}),
              flush=True)
for e in encs:
    e.close()

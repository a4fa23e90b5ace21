#!/usr/bin/env python3
"""Profiling / timing driver for k_recon in its bench form: B contexts of a
golden stream decoded together (thor_dec_frames, one launch per stage for the
B frames), so every P-frame k_recon launch covers B 4K frames exactly as the
bench's roofline launch does.  Resident parse output (trace), no checks.

  recon_batch.py [stream] [B] [reps] [--time]

--time: hipEvents around each stage of the P launches (thor_dec_set_timing),
prints the average k_recon launch and its fraction of HBM."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from thor_amd import lib as L  # noqa: E402
from thor_amd.decoder import GpuDecoder, decode_batch  # noqa: E402
from thor_amd.trace import load_trace  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
name = args[0] if args else "k4_low"
B = int(args[1]) if len(args) > 1 else 8
reps = int(args[2]) if len(args) > 2 else 2
timing = "--time" in sys.argv
seq, frames = load_trace(os.path.join(ROOT, "tests", "golden", name + ".trc.z"))
# RB_EXTRA=N: N more (idle) decoder contexts allocated first -- the bench's memory footprint
extra = [GpuDecoder(seq, slots=10) for _ in range(int(os.environ.get("RB_EXTRA", "0")))]
decs = [GpuDecoder(seq, slots=10) for _ in range(B)]
for d in decs[1:]:
    d.set_stream(C.c_void_p(decs[0].stream()))
devs = [[d.upload(fr) for fr in frames] for d in decs]
lib = L.load()
nf = len(frames)
if timing:
    lib.thor_dec_set_timing(decs[0].h, 1)
    cap = 8 * nf * reps
    mk_stage, mk_ms = (C.c_int * cap)(), (C.c_double * cap)()
    lib.thor_dec_stage_marks(decs[0].h, mk_stage, mk_ms, cap)
for _ in range(reps):
    for i in range(nf):
        decode_batch(decs, [devs[k][i] for k in range(B)])
for d in decs:
    d.sync()
if timing:
    import bench

    nm = lib.thor_dec_stage_marks(decs[0].h, mk_stage, mk_ms, cap)
    per, cur = [], None
    for k in range(nm):
        if mk_stage[k] == 0:
            cur = [0.0] * 7
            per.append(cur)
        cur[mk_stage[k]] += mk_ms[k]
    pidx = [i for i, fr in enumerate(frames) if fr.frame_type != 0]
    rec = [per[r * nf + i][1] for r in range(reps) for i in pidx]
    alg = B * sum(bench.recon_alg_bytes(frames[i], seq.width, seq.height) for i in pidx) / len(pidx)
    us = 1e3 * sum(rec) / len(rec)
    print("k_recon P launch (%d frames): avg %.2f us min %.2f us  alg %.1f MB  %.1f GB/s  frac %.3f" % (
        B, us, 1e3 * min(rec), alg / 1e6, alg / us / 1e3, alg / us / 1e3 / 8000.0))
    prep = [per[r * nf + i][0] for r in range(reps) for i in pidx]
    pus = 1e3 * sum(prep) / len(prep)
    print("k_frame_prep P launch: avg %.2f us min %.2f max %.2f us;  path (prep + recon) %.2f us  frac %.3f" % (
        pus, 1e3 * min(prep), 1e3 * max(prep), pus + us, alg / (pus + us) / 1e3 / 8000.0))
for d in decs:
    d.close()
print("decoded %d x %d frames of %s" % (reps, nf, name))

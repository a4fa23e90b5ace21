#!/usr/bin/env python3
"""Benchmark: Thor encode + decode of a 4K LDB-low stream on MI355X.

Metric (BASELINE.json): Mpixels/s encode+decode, 4K (3840x2160)
config_LDB_low_complexity, bit-exact vs the reference.  Workload
(config.workload): 8 distinct seeded synthetic 8-frame 4K clips
(thor_amd/synth.py; no real clips or network; tests/golden/bench_clips.json
holds the reference encoder's and decoder's md5 for each).

One step, per GPU, for K independent streams (a server coding K clips;
stream k codes clip k mod 8):
  input   every stream's raw frames from pinned host memory to its HBM buffer
          (H2D on a copy stream, frame-major; the encoder's frame i waits for
          frame i's copies only);
  encode  every stream's 8 frames through the device-resident encoder
          (thor_enc_frames: WPP RD loop, loop filters, CLPF decision and bit
          packing on the GPU, one launch per stage for the K streams) -> the
          streams' .bit, each checked against the reference Thorenc's for its
          clip;
  decode  every .bit: host parse (thor_parse_frame, 16 threads) -> upload of
          the parse output -> batched GPU reconstruction (thor_dec_frames),
          each decoded sequence checked against the reference Thordec's.
The legs are frame-pipelined: the host parse, upload and GPU reconstruction
of frame i run while the GPU encodes frame i + 1.  value = K x W x H x frames
/ wall time of the step (input upload, both legs, host parse and the H2D of
its output all included).  One extra step runs the legs one after the other
to report their split (config.serial_*).

Reported beside it (not part of `value`): the single-stream enc+dec latency,
decode_only (the reconstruction of resident parse output, the round-1
figure), the k_recon roofline (the north-star 4K inter-reconstruction kernel,
hipEvents on its stream) and a few kernel legs.

N > 1: one process per GPU, each with its own K streams (no data-path
collective): scaling "weak"; `bench.py --gpus N` run directly starts the N
ranks itself (launch_ranks), under torch.distributed.run it is one of them.
The time is the max over ranks.  Prints one JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import ctypes as C
import hashlib
import json
import os
import shlex
import subprocess
import sys
import queue
import threading
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# one hardware queue per decoder group (HIP's default is 4 per process); must be
# set before the HIP runtime initialises
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

import numpy as np  # noqa: E402

METRIC = "Mpixels/s encode+decode, 4K LDB_low_complexity; bit-exact vs ref"
_T0 = time.perf_counter()


def progress(msg: str) -> None:
    """One progress line on stderr (stdout carries only the JSON line)."""
    if int(os.environ.get("RANK", "0")) == 0:
        print("[bench %7.1f s] %s" % (time.perf_counter() - _T0, msg), file=sys.stderr, flush=True)
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
STAGES = ["prep", "inter", "intra", "deblock", "clpf", "pad"]
HOST_THREADS = 16  # the GPU box's CPU share per GPU


def recon_alg_bytes(fr, width: int, height: int) -> float:
    """Algorithmic HBM bytes of one k_recon launch (the inter-reconstruction
    kernel) on frame `fr`: per inter-predicted luma px
    1.5 B reference read (4:2:0, chroma folded in; x2 bi-pred) + 1.5 B
    reconstruction write; + the int16 residual read where the CU component is
    coded (2 B per luma px for Y, 2 B per chroma px for U and V); + 72 B per
    inter CU descriptor; + one 4 B cell-map word per 8x8 luma unit of the
    frame.  Halo re-reads and LDS staging are not counted."""
    b = fr.blocks
    inter = b["mode"] != 1
    w = b["bwidth"].astype(np.float64)
    h = b["bheight"].astype(np.float64)
    px = np.where(b["mode"] == 0, w * h, b["size"].astype(np.float64) ** 2)
    bi = (b["mode"] == 3) | (((b["mode"] == 0) | (b["mode"] == 4)) & (b["dir"] == 2))
    total = float(np.sum((1.5 * px * np.where(bi, 2.0, 1.0) + 1.5 * px)[inter]))
    total += 72.0 * float(np.count_nonzero(inter))
    coded = inter & (b["mode"] != 0)
    for c in range(3):
        has = coded & ((b["coeff_mask"] >> c) & 1).astype(bool)
        total += 2.0 * float(np.sum((px if c == 0 else px / 4.0)[has]))
    total += 4.0 * (width * height / 64.0)
    return total


TU_DTYPE = np.dtype([("orig_off", "<i4"), ("pred_off", "<i4"), ("rec_off", "<i4"), ("coeff_off", "<i4"),
                     ("orig_stride", "<i4"), ("pred_stride", "<i4"), ("rec_stride", "<i4"), ("size", "u1"),
                     ("qp", "u1"), ("type", "u1"), ("fast", "u1")])


def encoder_leg(torch, lib, reps: int = 10):
    """Encoder-side transform-block chain (SURVEY.md sec. 8(a) a4-a6, a8-a12;
    BASELINE config 3: 1080p, config_LDB_high_efficiency => encoder_speed 0,
    fast transforms off, qp 32): the RD evaluation of one inter candidate per
    CU at every quadtree level (64, 32, 16, 8) over a whole 1080p frame --
    orig = synthetic frame 1, pred = frame 0 co-located -- residual -> forward
    T -> quantize -> dequant -> inverse T -> recon -> SSD per TU
    (thor_enc_tu_batch), then cost_calc per CU (thor_enc_cost_batch): the
    batched entry points of the encoder's TU chain.  The device-resident
    encoder (k_enc_rows) runs the same chain inline in its RD loop."""
    from thor_amd import synth

    W, H, qp = 1920, 1080, 32
    chroma_qp = [min(q, 29) if q < 30 else [29, 30, 31, 32, 33, 33, 34, 34, 35, 35, 36, 36, 37, 37, 38, 39, 40, 41, 42,
                                            43, 44, 45][q - 30] for q in range(52)]
    org = synth.synth_frame(W, H, 1, 3)
    prd = synth.synth_frame(W, H, 0, 3)
    planes = [np.concatenate([p.reshape(-1) for p in fr]) for fr in (org, prd)]
    offs = [0, W * H, W * H + (W // 2) * (H // 2)]
    tus, cu_first, cu_count = [], [], []
    coff = 0
    for S in (64, 32, 16, 8):
        for y in range(0, H - S + 1, S):
            for x in range(0, W - S + 1, S):
                cu_first.append(len(tus))
                for c in range(3):
                    n = S if c == 0 else S // 2
                    st = W if c == 0 else W // 2
                    yy, xx = (y, x) if c == 0 else (y // 2, x // 2)
                    o = offs[c] + yy * st + xx
                    q = min(n, 16)
                    tus.append((o, o, o, coff, st, st, st, n, qp if c == 0 else chroma_qp[qp], c != 0, 0))
                    coff += q * q
                cu_count.append(3)
    tus = np.array(tus, TU_DTYPE)
    ncu, ntu = len(cu_first), len(tus)
    dev = torch.device("cuda", torch.cuda.current_device())
    t_org = torch.from_numpy(planes[0]).to(dev)
    t_prd = torch.from_numpy(planes[1]).to(dev)
    t_rec = torch.empty_like(t_org)
    t_tus = torch.from_numpy(tus.view(np.uint8)).to(dev)
    t_cq = torch.empty(coff, dtype=torch.int16, device=dev)
    t_cbp = torch.empty(ntu, dtype=torch.uint8, device=dev)
    t_ssd = torch.empty(ntu, dtype=torch.int32, device=dev)
    t_first = torch.tensor(cu_first, dtype=torch.int32, device=dev)
    t_count = torch.tensor(cu_count, dtype=torch.int32, device=dev)
    t_bits = torch.full((ncu,), 100, dtype=torch.int32, device=dev)
    t_cost = torch.empty(ncu, dtype=torch.int32, device=dev)
    lam = 0.57 * 2 ** ((qp - 12) / 3.0)

    def run():
        rc = lib.thor_enc_tu_batch(t_tus.data_ptr(), ntu, t_org.data_ptr(), t_prd.data_ptr(), t_rec.data_ptr(),
                                   t_cq.data_ptr(), t_cbp.data_ptr(), t_ssd.data_ptr(), None)
        rc |= lib.thor_enc_cost_batch(t_ssd.data_ptr(), t_first.data_ptr(), t_count.data_ptr(), t_bits.data_ptr(),
                                      lam, t_cost.data_ptr(), ncu, None)
        assert rc == 0

    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    px = 4 * W * H  # luma px evaluated (one candidate per CU at 4 levels)
    q2 = sum(min(int(t), 16) ** 2 for t in tus["size"])
    alg = 4 * 3 * W * H * 1.5 + 2.0 * q2  # orig + pred + rec bytes (4:2:0) + levels
    return {"workload": "1080p, one inter candidate per CU at 64/32/16/8 over the whole frame, qp 32, "
                        "LDB_high_efficiency transform flags; %d TUs, %d CUs per pass" % (ntu, ncu),
            "ms_per_pass": round(ms, 4), "mpx_evaluated_s": round(px / ms / 1e3, 1),
            "cbp_fraction": round(float(t_cbp.float().mean().item()), 3),
            "alg_bytes": int(alg), "achieved_gb_s": round(alg / ms / 1e6, 1),
            "note": "RD candidate evaluation throughput of the encoder TU chain; not part of `value`"}


def config3_leg(torch, lib, streams: int = 128, nf: int = 2):
    """BASELINE config 3 -- 1080p config_LDB_high_efficiency, the full encoder
    RD loop on the GPU (encoder_speed 0: exact sub-pel ME, tb / pb split,
    4 references, delta-QP RD) -- as a throughput leg beside `value`: `streams`
    independent contexts coding the first `nf` frames (the I frame, then P) of
    the seeded 1080p clip tests/golden/hd_high was encoded from, one
    thor_enc_frames launch set per frame for all of them.  Every stream's .bit
    must equal the reference Thorenc's (tests/golden/hd_high.bit) byte for byte.
    The reference's own figure on this config (0.046 Mpx/s, one
    core, 17 frames) is quoted beside it, with 16 cores taken as 16x that."""
    from thor_amd import synth
    from thor_amd.encoder import GpuEncoder, encode_batch, params_for

    gold = os.path.join(ROOT, "tests", "golden")
    meta = json.load(open(os.path.join(gold, "streams.json")))["hd_high"]
    w, h = meta["width"], meta["height"]
    clip = synth.synth_frames(w, h, nf, meta["seed"], workers=1)  # serial: this process owns the GPU
    want = open(os.path.join(gold, "hd_high.bit"), "rb").read()
    encs = [GpuEncoder(params_for(meta["config"], w, h, nf, meta["extra"])) for _ in range(streams)]
    try:
        for e in encs:
            e.upload_sequence(clip)
        torch.cuda.synchronize()
        out = [b""] * streams
        frame_s = []
        for _ in range(nf):
            t0 = time.perf_counter()
            ch = encode_batch(encs)
            frame_s.append(time.perf_counter() - t0)
            for k in range(streams):
                out[k] += ch[k]
        ok = all(want.startswith(o) and len(o) > 0 for o in out) and len(set(out)) == 1
    finally:
        for e in encs:
            e.close()
    t = sum(frame_s)
    mpx = streams * w * h * nf / t / 1e6
    ref1 = 0.046  # BASELINE.md, config_LDB_high_efficiency 1080p x 17, SIMD build, one core
    return {"workload": "%d streams x %d frames of 1080p config_LDB_high_efficiency (I + P, encoder_speed 0), "
                        "encode only, thor_enc_frames batches" % (streams, nf),
            "mpx_s": round(mpx, 3), "seconds": round(t, 3), "frame_s": [round(x, 3) for x in frame_s],
            "bit_exact": ok, "reference_single_core_mpx_s": ref1, "reference_16_core_mpx_s": round(16 * ref1, 3),
            "x_16_reference_cores": round(mpx / (16 * ref1), 2)}


CFG5_CODED = (0, 16)  # the first two coded frames of the 17-frame HDB16 plan: the I frame and P frame 16


def config5_frames():
    """Display frames 0 and 16 of the seeded 4K clip tests/golden/k4_hdbi_high was encoded from (the only
    input the I frame and P frame 16 read); synthesised in worker processes before the GPU is touched."""
    from thor_amd import synth

    meta = json.load(open(os.path.join(ROOT, "tests", "golden", "streams.json")))["k4_hdbi_high"]
    import multiprocessing as mp

    pool = mp.get_context("fork").Pool(2)
    try:
        fr = pool.map(synth._i420, [(meta["width"], meta["height"], t, meta["seed"]) for t in CFG5_CODED])
    finally:
        pool.close()
        pool.join()
    return meta, fr


def config5_leg(torch, lib, cfg5, streams: int = 64):
    """BASELINE config 5 -- 4K config_HDB16_high_efficiency (hierarchical B, 16-frame sub-GOP, encoder_speed
    0, temporal-interpolated references, 4 references, tb / pb split, delta-QP RD) -- as a throughput leg
    beside `value`: `streams` independent contexts coding the first two coded frames of the 17-frame plan
    (the I frame, then P frame 16: the telescope + exact sub-pel motion search at its longest distance),
    one thor_enc_frames launch set per frame for all of them.  Every stream's bytes must equal the
    reference Thorenc's tests/golden/k4_hdbi_high.bit (its first two frame chunks).  The P-16 batch is
    latency bound (the superblock wavefront's critical path), so its time is also the single-stream time
    of that frame."""
    from thor_amd.encoder import GpuEncoder, encode_batch, params_for

    meta, fr = cfg5
    w, h, n = meta["width"], meta["height"], meta["frames"]
    fsize = w * h * 3 // 2
    want = open(os.path.join(ROOT, "tests", "golden", "k4_hdbi_high.bit"), "rb").read()
    seq = torch.zeros((n, fsize), dtype=torch.uint8, device="cuda")  # display order; only frames 0, 16 are read
    for t, x in zip(CFG5_CODED, fr):
        seq[t].copy_(torch.from_numpy(x))
    encs = [GpuEncoder(params_for(meta["config"], w, h, n, meta["extra"])) for _ in range(streams)]
    try:
        for e in encs:
            e.use_device_sequence(seq.data_ptr(), n)
        torch.cuda.synchronize()
        out = [b""] * streams
        frame_s = []
        for _ in CFG5_CODED:
            t0 = time.perf_counter()
            ch = encode_batch(encs)
            frame_s.append(time.perf_counter() - t0)
            progress("config-5 frame batch: %.1f s" % frame_s[-1])
            for k in range(streams):
                out[k] += ch[k]
        ok = all(want.startswith(o) and len(o) > 0 for o in out) and len(set(out)) == 1
    finally:
        for e in encs:
            e.close()
    t = sum(frame_s)
    mpx = streams * w * h * len(CFG5_CODED) / t / 1e6
    ref1 = 0.099  # config_HDB16_high_efficiency 1080p x 17, SIMD build, one core
    return {"workload": "%d streams x the first 2 coded frames (I, P 16) of 4K config_HDB16_high_efficiency "
                        "(encoder_speed 0, interpolated references), encode only, thor_enc_frames batches" % streams,
            "mpx_s": round(mpx, 3), "seconds": round(t, 3), "frame_s": [round(x, 3) for x in frame_s],
            "bit_exact": ok, "reference_single_core_mpx_s": ref1,
            "reference_note": "the reference's figure is 1080p x 17 frames (all its frame types) on one core; "
                              "per 4K frame that is 4 x 8.3 / 0.099 ~ 84 s",
            "x_16_reference_cores": round(mpx / (16 * ref1), 2)}


def pyramid_leg(torch, lib, reps: int = 50):
    """Temporal-interpolation luma pyramid (thor_scale_pyramid2, the chains of
    scale_frame_down2x2_simd calls of common/temporal_interp.c:1011-1019) on
    both 4K reference frames: 3 levels each + their 32-px padding.  Not part of
    `value`.  Algorithmic bytes: level 0 read once (W*H) + every level byte
    written once, padding included."""
    W, H, n = 3840, 2160, 3
    pad = 32
    dev = torch.device("cuda", torch.cuda.current_device())
    srcs = [torch.randint(0, 256, (H, W), dtype=torch.uint8, device=dev) for _ in range(2)]
    bufs, parrs, wr = [], [], 0
    strides = [((W >> l) + 2 * pad + 15) & ~15 for l in range(1, n + 1)]
    for _ in range(2):
        ptrs = []
        for l in range(1, n + 1):
            wl, hl, s = W >> l, H >> l, strides[l - 1]
            b = torch.empty((hl + 2 * pad) * s, dtype=torch.uint8, device=dev)
            bufs.append(b)
            ptrs.append(b.data_ptr() + pad * s + pad)
            wr += (hl + 2 * pad) * (wl + 2 * pad)
        parrs.append((C.c_void_p * 3)(*ptrs))
    sarr = (C.c_int * 3)(*strides)
    st = torch.cuda.current_stream().cuda_stream

    def run():
        assert lib.thor_scale_pyramid2(srcs[0].data_ptr(), srcs[1].data_ptr(), W, W, H,
                                       C.cast(parrs[0], C.c_void_p), C.cast(parrs[1], C.c_void_p),
                                       C.cast(sarr, C.c_void_p), n, st) == 0

    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    alg = 2 * W * H + wr
    return {"workload": "both 4K luma references of interpolate_frames -> 3 down-sampled, padded levels "
                        "each (thor_scale_pyramid2: k_down_pyramid + k_pad_pyramid, grid z = reference)",
            "us_per_pair": round(ms * 1e3, 2), "alg_bytes": int(alg), "achieved_gb_s": round(alg / ms / 1e6, 1),
            "note": "hipEvents on torch's current stream (the launches' stream); not part of `value`"}


def interp_leg(torch, lib, reps: int = 50):
    """Temporal-interpolation compensation (thor_interp_frame: interpolate_comp
    + mot_comp_avg, common/temporal_interp.c:387-441,920-944) of one 4K frame,
    Y + U + V, from a random 8x8-block MV field (±50 px).  Not part of
    `value`.  Algorithmic bytes: two reference reads + one write per pixel
    + the MV field (8 B per block, read by the luma and both chroma passes)."""
    W, H, pf, pfc = 3840, 2160, 96, 48
    dev = torch.device("cuda", torch.cuda.current_device())
    bw, bh = 2 * ((W + 15) // 16), 2 * ((H + 15) // 16)
    g = torch.Generator(device="cpu").manual_seed(5)
    mv = torch.randint(-400, 401, (2, bh * bw, 2), generator=g, dtype=torch.int16).to(dev)
    planes = []
    for (pw, ph, pad) in ((W, H, pf), (W // 2, H // 2, pfc), (W // 2, H // 2, pfc)):
        s = (pw + 2 * pad + 15) & ~15
        r0 = torch.randint(0, 256, ((ph + 2 * pad) * s,), dtype=torch.uint8, device=dev)
        r1 = torch.randint(0, 256, ((ph + 2 * pad) * s,), dtype=torch.uint8, device=dev)
        o = torch.empty((ph + 2 * pad) * s, dtype=torch.uint8, device=dev)
        org = pad * s + pad
        planes.append((r0.data_ptr() + org, r1.data_ptr() + org, o.data_ptr() + org, s, pw == W, (r0, r1, o)))
    st = torch.cuda.current_stream().cuda_stream

    class Plane(C.Structure):  # thor_interp_plane_t
        _fields_ = [("p0", C.c_void_p), ("p1", C.c_void_p), ("out", C.c_void_p), ("s0", C.c_int32),
                    ("s1", C.c_int32), ("so", C.c_int32)]

    desc = (Plane * 3)(*[Plane(p0, p1, po, s, s, s) for p0, p1, po, s, _, _ in planes])

    def run():
        assert lib.thor_interp_frame(C.cast(desc, C.c_void_p), mv[0].data_ptr(), mv[1].data_ptr(), bw, bh, W, H, 3, 1,
                                     st) == 0

    def timed():
        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    ms = timed()
    # a smooth field as real motion has: global pan (+13.4, -6.1 px) with +-1 px jitter per block
    pan = torch.tensor([107, -49], dtype=torch.int16)
    jit = torch.randint(-8, 9, (2, bh * bw, 2), generator=g, dtype=torch.int16)
    mv.copy_((pan + jit).to(dev))
    ms_smooth = timed()
    alg = 3 * W * H * 1.5 + 3 * 8 * bw * bh
    return {"workload": "4K frame (Y, U, V in one k_interp_frame launch), 8x8 luma blocks, random MVs",
            "us_per_frame": round(ms * 1e3, 2), "alg_bytes": int(alg), "achieved_gb_s": round(alg / ms / 1e6, 1),
            "smooth_field_us_per_frame": round(ms_smooth * 1e3, 2),
            "smooth_field_gb_s": round(alg / ms_smooth / 1e6, 1),
            "note": "hipEvents on torch's current stream (the launches' stream); not part of `value`"}


def interp_frames_leg(torch, lib, clip: np.ndarray, reps: int = 10):
    """The whole temporal-interpolated reference of BASELINE config 5
    (thor_interpolate_frames: both luma pyramids, motion_estimate_bi on every
    level, interpolate_frame; common/temporal_interp.c:972-1053) from frames 0
    and 2 of the 4K clip (ratio 2, pos 1: dec/decode_frame.c's symmetric B
    case), on torch's current stream.  Not part of `value`; the reference's own
    interpolate_frames takes 33.6 ms for the same pair on one core of the build
    container (profiles/r02c_interp_speed.json)."""
    W, H = 3840, 2160
    dev = torch.device("cuda", torch.cuda.current_device())
    keep = []

    def padded(fr):
        y = fr[:W * H].reshape(H, W)
        u = fr[W * H:W * H * 5 // 4].reshape(H // 2, W // 2)
        v = fr[W * H * 5 // 4:].reshape(H // 2, W // 2)
        ptrs, strides = [], []
        for p, pad in ((y, 96), (u, 48), (v, 48)):
            s = (p.shape[1] + 2 * pad + 15) & ~15
            full = np.zeros((p.shape[0] + 2 * pad, s), np.uint8)
            full[:, :p.shape[1] + 2 * pad] = np.pad(p, pad, mode="edge")
            t = torch.from_numpy(full).to(dev)
            keep.append(t)
            ptrs.append(t.data_ptr() + pad * s + pad)
            strides.append(s)
        return L_planes(ptrs[0], ptrs[1], ptrs[2], strides[0], strides[1])

    from thor_amd.lib import ThorYuvPlanes as L_planes

    ra, rb = padded(clip[0]), padded(clip[2])
    ro = padded(np.zeros_like(clip[0]))
    st = torch.cuda.current_stream().cuda_stream
    t = lib.thor_ti_create(W, H, torch.cuda.current_device())
    try:
        def run():
            assert lib.thor_interpolate_frames(t, C.byref(ra), C.byref(rb), 96, C.byref(ro), 2, 1, st) == 0

        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        assert lib.thor_ti_status(t) == 0
        ms = e0.elapsed_time(e1) / reps
    finally:
        lib.thor_ti_destroy(t)
    return {"workload": "4K interpolated reference from frames 0 and 2 of the clip (pyramid + motion search on "
                        "4 levels + compensation)", "ms_per_frame": round(ms, 3),
            "reference_cpu_ms_per_frame_1core": 33.6,
            "note": "hipEvents on torch's current stream; latency-bound (the search is a wavefront of step rows)"}


def cpu_baseline(bc, clips_meta, clips, procs: int = HOST_THREADS, budget_s: float = 8.0):
    """The reference encoder + decoder (oracle/_ref/Thorenc, Thordec: SIMD
    build, -O3) on the bench's clips and configuration: `procs` concurrent
    encode->decode pipelines on the host cores (one stream each, round-robin
    over the clips, each reading its YUV from a file as the reference does),
    plus one pipeline alone (1 core).  Every bitstream and decoded md5 is
    checked against tests/golden/bench_clips.json.  Returns None when the
    reference binaries are not present (they are built from /root/reference by
    oracle/Makefile)."""
    from thor_amd.configs import flags

    enc = os.path.join(ROOT, "oracle", "_ref", "Thorenc")
    dec = os.path.join(ROOT, "oracle", "_ref", "Thordec")
    if not (os.path.exists(enc) and os.path.exists(dec)):
        return None
    W, H, n = bc["width"], bc["height"], bc["frames"]
    px = W * H * n
    tmp = "/tmp/thor_bench_%d" % os.getpid()
    os.makedirs(tmp, exist_ok=True)
    for c, clip in enumerate(clips):
        clip.tofile(os.path.join(tmp, "in%d.yuv" % c))
    fl = flags(bc["config"], W, H, n, bc["extra"])

    def pipeline(k):
        c = k % len(clips)
        bit, out = os.path.join(tmp, "%d.bit" % k), os.path.join(tmp, "%d.yuv" % k)
        cmd = "%s -if %s -of %s %s >/dev/null 2>&1 && %s %s %s >/dev/null 2>&1" % (
            shlex.quote(enc), os.path.join(tmp, "in%d.yuv" % c), bit, " ".join(shlex.quote(f) for f in fl),
            shlex.quote(dec), bit, out)
        return subprocess.Popen(["/bin/sh", "-c", cmd])

    def check(k):
        c = clips_meta[k % len(clips)]
        return (hashlib.md5(open(os.path.join(tmp, "%d.bit" % k), "rb").read()).hexdigest() == c["bit_md5"] and
                hashlib.md5(open(os.path.join(tmp, "%d.yuv" % k), "rb").read()).hexdigest() == c["dec_md5"])

    try:
        # one pipeline alone, repeated within the budget
        runs, t1 = 0, 0.0
        while runs < 1 or (t1 < budget_s and runs < 5):
            t0 = time.perf_counter()
            assert pipeline(0).wait() == 0
            t1 += time.perf_counter() - t0
            runs += 1
        ok = check(0)
        one = px * runs / t1 / 1e6
        # `procs` pipelines at once on the host cores
        t0 = time.perf_counter()
        ps = [pipeline(k) for k in range(procs)]
        rcs = [p.wait() for p in ps]
        tp = time.perf_counter() - t0
        assert all(r == 0 for r in rcs), rcs
        for k in range(procs):
            ok &= check(k)
    finally:
        for f in os.listdir(tmp):
            os.remove(os.path.join(tmp, f))
        os.rmdir(tmp)
    return {"value": round(px * procs / tp / 1e6, 3), "unit": "Mpixels/s", "cores": procs, "kind": "reference",
            "sample": "reference Thorenc -> Thordec (SIMD build, -O3) on the bench's 4K 8-frame LDB-low clips: "
                      "%d concurrent single-threaded pipelines (one per host core of the GPU's share, round-robin "
                      "over %d clips), %.1f s wall; bitstream + decoded md5 %s" % (
                          procs, len(clips), tp, "ok" if ok else "MISMATCH"),
            "single_core_mpx_s": round(one, 3), "single_core_s_per_pass": round(t1 / runs, 3)}


ST_COUNT = 7  # capi.hip stage marks: prep, inter, intra, deblock, clpf, pad, interpolated reference


def roofline_pass(lib, decs, groups, devs, frames_of, seq, isteps):
    """Instrumented decode of group 0 alone (resident parse output): hipEvents
    around every stage of every batched launch on its stream -> the stage
    breakdown and the k_recon roofline (one launch = the group's B frames, one
    per member; frames_of[j]: member j's parsed frames)."""
    lead = decs[groups[0][0]]
    B = len(groups[0])
    nf = len(frames_of[0])
    from thor_amd.decoder import decode_batch

    lib.thor_dec_set_timing(lead.h, 1)
    cap = 8 * nf * (isteps + 1)
    mk_stage, mk_ms = (C.c_int * cap)(), (C.c_double * cap)()
    lib.thor_dec_stage_marks(lead.h, mk_stage, mk_ms, cap)
    for _ in range(isteps):
        for i in range(nf):
            decode_batch([decs[k] for k in groups[0]], [devs[k][i] for k in groups[0]])
    nm = lib.thor_dec_stage_marks(lead.h, mk_stage, mk_ms, cap)
    lib.thor_dec_set_timing(lead.h, 0)
    per_frame, cur = [], None
    for k in range(nm):  # a frame opens with its interpolated reference (6) or else its side-info stage (0)
        st = mk_stage[k]
        if cur is None or st == 6 or (st == 0 and not (cur[6] > 0 and sum(cur[:6]) == 0)):
            cur = [0.0] * ST_COUNT
            per_frame.append(cur)
        cur[st] += mk_ms[k]
    assert len(per_frame) == isteps * nf, (len(per_frame), isteps, nf)
    stage_ms = [sum(f[i] for f in per_frame) / isteps / B for i in range(ST_COUNT)]  # per stream pass
    frames = frames_of[0]
    pidx = [i for i, fr in enumerate(frames) if fr.frame_type != 0]  # the I frame has no inter pixels
    recon_ms = sum(per_frame[s * nf + i][1] for s in range(isteps) for i in pidx) / (isteps * len(pidx))
    prep_ms = sum(per_frame[s * nf + i][0] for s in range(isteps) for i in pidx) / (isteps * len(pidx))
    # per launch: the members' P frames of one frame index, averaged over the P frame indices
    alg = sum(recon_alg_bytes(fs[i], seq.width, seq.height) for fs in frames_of for i in pidx) / len(pidx)
    return stage_ms, recon_ms, alg, B, prep_ms


ROWS_STREAM = "k4_med"  # BASELINE config 4: 4K config_LDB_medium_complexity, SB rows sharded across the GPUs


def band_kernel_ms(lib, seq, frames, world: int, rank: int, reps: int = 3):
    """Per-frame stage times (ms: prep, inter, intra, deblock, clpf, pad,
    interp) of rank `rank`'s share of a `world`-way row split, run alone on
    this GPU: a boundary-mode context (the band's k_frame_prep cells and TUs,
    band k_recon, band intra chains, band-local deblock / CLPF, band pad) with
    no exchange -- the rows outside the band are not final, so nothing is
    checked; each kernel does exactly the band's work.  Also the wall time of
    the rank's kernels per frame (one stream, host enqueue included)."""
    from thor_amd.decoder import GpuDecoder
    from thor_amd.shard import band_of

    dec = GpuDecoder(seq)
    try:
        b0, b1 = band_of(seq.height, world, rank)
        dec.set_band(b0, b1)
        dec.set_band_local(True)
        dec.set_band_intra(True)
        dec.set_band_pad(True)
        devs = [dec.upload(fr) for fr in frames]

        def one():
            for d in devs:
                dec.begin(d)
                dec.intra()
                dec.end()
                dec.finish()

        one()
        dec.sync()
        t0 = time.perf_counter()
        for _ in range(reps):
            one()
        dec.sync()
        wall = (time.perf_counter() - t0) / (reps * len(frames)) * 1e3
        lib.thor_dec_set_timing(dec.h, 1)
        ms = (C.c_double * 7)()
        lib.thor_dec_stage_ms(dec.h, ms, 7)  # (clears)
        for _ in range(reps):
            one()
        lib.thor_dec_stage_ms(dec.h, ms, 7)
        lib.thor_dec_set_timing(dec.h, 0)
        return [ms[i] / (reps * len(frames)) for i in range(7)], wall
    finally:
        dec.close()


def rows_leg(torch, dist, rank: int, world: int, local: int, passes: int = 5):
    """The north star's row split at this run's N (BASELINE config 4): ONE 4K
    LDB-medium stream (tests/golden/k4_med.bit, the reference Thorenc's) decoded
    by all ranks together, its SB rows in balanced bands (thor_amd/shard.py
    boundary mode: band k_recon, band intra with edge rows from the band above,
    8-row deblocking halos, band-local deblock / CLPF / pad, MV-reach halo
    fetch of reference rows; point-to-point over RCCL, device buffers).
    Strong scaling: the same stream whatever N.  Every frame is put together
    from its band owners and md5-checked against the reference decoder after
    the warmup pass and after the timed passes.  Returns the `rows` object
    (rank 0) or None."""
    from thor_amd import lib as L
    from thor_amd.bitstream import parse_stream
    from thor_amd.decoder import GpuDecoder
    from thor_amd.shard import RowShard, band_of

    gold = os.path.join(ROOT, "tests", "golden")
    meta = json.load(open(os.path.join(gold, "streams.json")))[ROWS_STREAM]
    seq, frames = parse_stream(open(os.path.join(gold, ROWS_STREAM + ".bit"), "rb").read())
    own = dist is None
    if own:  # a one-rank group keeps the same code path
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ["MASTER_PORT"] = str(29600 + os.getpid() % 300)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", local))
    lib = L.load()
    dec = GpuDecoder(seq, device=local)
    dev = torch.device("cuda", local)
    try:
        sh = RowShard(dec, dist, seq.width, seq.height, device_exchange=True, band_local=True, halo=True,
                      boundary=True)
        devs = [dec.upload(fr) for fr in frames]

        def step():
            for d, fr in zip(devs, frames):
                sh.decode(d, fr.frame_num, fr)

        def check():
            got = {fr.frame_num: sh.assemble(fr.frame_num) for fr in frames}
            return hashlib.md5(b"".join(got[k] for k in sorted(got))).hexdigest() == meta["dec_md5"]

        step()
        torch.cuda.synchronize(local)
        ok = check()
        dist.barrier()
        torch.cuda.synchronize(local)
        t0 = time.perf_counter()
        for _ in range(passes):
            step()
        torch.cuda.synchronize(local)
        elapsed = time.perf_counter() - t0
        dist.barrier()
        ok &= check()
        # this rank's kernel time per stage: one more pass with stage events on the decoder's stream
        lib.thor_dec_set_timing(dec.h, 1)
        ms = (C.c_double * 7)()
        lib.thor_dec_stage_ms(dec.h, ms, 7)
        step()
        lib.thor_dec_stage_ms(dec.h, ms, 7)
        lib.thor_dec_set_timing(dec.h, 0)
        mine = torch.tensor([ms[i] / len(frames) for i in range(7)] + [float(sum(sh.boundary_bytes)),
                                                                         float(sum(sh.halo_bytes))],
                            dtype=torch.float64, device=dev)
        every = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(every, mine)
        t = torch.tensor([elapsed, 0.0 if ok else 1.0], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, ok = float(t[0].item()), t[1].item() == 0.0
        every = [e.cpu().tolist() for e in every]
    finally:
        dec.close()
        if own:
            dist.destroy_process_group()
    if rank != 0:
        return None
    nfr = len(frames) * passes
    px = seq.width * seq.height
    nbytes_frames = len(frames) * (passes + 2)  # the warmup, timed and stage passes
    out = {
        "workload": "BASELINE config 4: ONE 4K (3840x2160) config_LDB_medium_complexity stream (%s: %d frames, "
                    "the reference Thorenc's .bit), SB rows in balanced bands over %d rank(s), boundary exchange "
                    "over RCCL (thor_amd/shard.py): band k_recon + intra + deblock + CLPF + pad per rank, edge "
                    "rows + 8-row deblocking halos + MV-reach reference halos point to point" % (
                        ROWS_STREAM, len(frames), world),
        "n_ranks": world,
        "scaling": "strong",
        "passes": passes,
        "ms_per_frame": round(elapsed / nfr * 1e3, 4),
        "mpx_s": round(px * nfr / elapsed / 1e6, 2),
        "bit_exact": ok,
        "bit_exact_scope": "every frame assembled from its band owners == the reference Thordec (md5 of the "
                           "sequence), after the warmup pass and after the timed passes",
        "bands_sb_rows": [list(band_of(seq.height, world, r)) for r in range(world)],
        "per_rank_stage_ms_per_frame": [{k: round(v, 4) for k, v in zip(STAGES + ["interp"], e[:7])}
                                        for e in every],
        "per_rank_kernel_ms_per_frame": [round(sum(e[:7]), 4) for e in every],
        "per_rank_exchange_kb_per_frame": [round((e[7] + e[8]) / nbytes_frames / 1e3, 1) for e in every],
        "note": "ms_per_frame: wall clock of the timed passes, max over ranks, host parse excluded (resident "
                "parse output), the exchange and its host-side protocol included",
    }
    if world == 1:  # the 8-way split's per-rank kernel work, each rank's band run alone on this GPU
        per = [band_kernel_ms(lib, seq, frames, 8, r) for r in range(8)]
        whole, wall1 = band_kernel_ms(lib, seq, frames, 1, 0)
        t1, t8 = sum(whole), max(sum(p[0]) for p in per)
        out["split8_on_one_gpu"] = {
            "what": "each of the 8 ranks' bands decoded alone on this GPU (boundary-mode context, no exchange): "
                    "per-rank kernel ms per frame, against the whole frame in the same mode",
            "whole_frame_stage_ms": {k: round(v, 4) for k, v in zip(STAGES + ["interp"], whole)},
            "whole_frame_kernel_ms": round(t1, 4),
            "whole_frame_wall_ms": round(wall1, 4),
            "rank_stage_ms": [{k: round(v, 4) for k, v in zip(STAGES + ["interp"], p[0])} for p in per],
            "rank_kernel_ms": [round(sum(p[0]), 4) for p in per],
            "rank_wall_ms": [round(p[1], 4) for p in per],
            "kernel_speedup_bound": round(t1 / t8, 3) if t8 > 0 else None,
            "wall_speedup_bound": round(wall1 / max(p[1] for p in per), 3),
            "prep_ratio_max_rank_vs_whole": round(max(p[0][0] for p in per) / whole[0], 4) if whole[0] > 0 else None,
        }
    return out


ROWS_TIMEOUT_S = 240


def rows_guarded(a, torch, dist, rank, world, local, out):
    """rows_leg on every rank under a watchdog: the row split's collectives
    must not hang the streams measurement -- past ROWS_TIMEOUT_S rank 0 prints
    `out` with a rows error and every rank exits."""
    done = threading.Event()

    def fire():
        if done.is_set():
            return
        if rank == 0 and out is not None:
            out["rows"] = {"error": "the rows leg did not finish within %d s" % ROWS_TIMEOUT_S}
            print(json.dumps(out), flush=True)
        os._exit(0)

    tm = threading.Timer(ROWS_TIMEOUT_S, fire)
    tm.daemon = True
    tm.start()
    try:
        return rows_leg(torch, dist, rank, world, local, a.rows_passes)
    except Exception as e:  # noqa: BLE001 - reported in the JSON line
        progress("rows leg failed: %r" % (e,))
        return {"error": repr(e)[:400]} if rank == 0 else None
    finally:
        done.set()
        tm.cancel()


def launch_ranks(n: int) -> int:
    """bench.py --gpus N run directly (no torch.distributed.run): start N ranks
    of this script, one per GPU, before anything here touches a GPU, with the
    launcher's environment (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*); the
    children inherit stdout, so rank 0's JSON line is the output.  Returns the
    worst exit status."""
    port = str(29500 + os.getpid() % 1000)
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    return max(abs(rc) for rc in rcs)


def reduce_max(dist, device, x: float) -> float:
    """max over ranks (the slowest rank's time); identity without a group."""
    if dist is None:
        return x
    import torch

    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def launcher_selftest(a) -> None:
    """--launcher-selftest (CPU, gloo): the N-rank plumbing of a --gpus N run
    without a GPU -- rank spawn, process group, barrier, max-over-ranks time,
    min-over-ranks bit-exactness -- and rank 0's one JSON line."""
    import torch.distributed as dist

    rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dist.barrier()
    elapsed = reduce_max(dist, "cpu", 1.0 + rank)
    ok = -reduce_max(dist, "cpu", -1.0)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "n_gpus": world, "selftest": True, "max_elapsed": elapsed,
                          "bit_exact": ok == 1.0}), flush=True)
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--config3-streams", type=int, default=128,
                    help="streams of the BASELINE config-3 encoder leg (1080p LDB high efficiency)")
    ap.add_argument("--config5-streams", type=int, default=64,
                    help="streams of the BASELINE config-5 encoder leg (4K HDB16 high efficiency, I + P 16); 0: off")
    ap.add_argument("--drop-in", nargs="?", const="hd_low", default=None, metavar="STREAM",
                    help="time the reference decoder's host C on this library's per-call surface "
                         "(oracle/_ref/thordec_amd) beside the reference Thordec on a golden .bit (default hd_low)")
    ap.add_argument("--no-legs", action="store_true", help="skip the kernel legs reported beside `value`")
    ap.add_argument("--dec-slots", type=int, default=10,
                    help="reference ring slots per decoder context (LDB: up to 4 references + the current frame)")
    ap.add_argument("--streams", type=int, default=240, help="independent streams (encoder + decoder) per GPU")
    ap.add_argument("--enc-cu-exclude", type=int, default=0, metavar="N",
                    help="experiment: keep the encoder's kernels off N of every 32 CUs (hipExtStreamCreateWithCUMask), "
                         "so concurrent decode launches always find free CUs")
    ap.add_argument("--dec-priority", type=int, default=0,
                    help="1: decoder groups on high-priority HIP streams (their launches dispatch ahead of the "
                         "encoder's queued workgroups); 0: default priority")
    ap.add_argument("--clips", type=int, default=8, help="distinct seeded clips the streams are drawn from (<= 8)")
    ap.add_argument("--band-local", action="store_true",
                    help="--shard rows: each rank deblocks / CLPFs only its band, then a second all-gather of final rows")
    ap.add_argument("--halo", action="store_true",
                    help="--shard rows, band-local: no second all-gather; each rank fetches the reference rows its "
                         "band's vectors reach (MV-reach halo exchange, thor_amd/shard.py)")
    ap.add_argument("--boundary", action="store_true",
                    help="--shard rows with the halo exchange and no pre-deblock all-gather either: edge rows for "
                         "each band's intra chains from the band above, 8 deblocking halo rows either side")
    ap.add_argument("--shard", choices=["streams", "rows"], default="streams",
                    help="streams: independent enc+dec streams per GPU (default); rows: decode-only, ONE "
                         "stream's SB rows split across the ranks with an RCCL all-gather before intra/deblock")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC-derived HBM bytes per k_recon launch (default tools/traffic_latest.json, "
                         "copied from profiles/<tag>_traffic.json by tools/prof_summary.py)")
    ap.add_argument("--no-rows", action="store_true", help="skip the config-4 row-split leg (the `rows` object)")
    ap.add_argument("--rows-passes", type=int, default=5, help="timed passes of the row-split leg's 8-frame stream")
    ap.add_argument("--launcher-selftest", action="store_true", help=argparse.SUPPRESS)
    a = ap.parse_args()

    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:  # not under torch.distributed.run: be the launcher
        sys.exit(launch_ranks(a.gpus))
    if a.launcher_selftest:
        return launcher_selftest(a)
    if a.drop_in:
        return dropin_mode(a)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    gold = os.path.join(ROOT, "tests", "golden")
    bc = json.load(open(os.path.join(gold, "bench_clips.json")))
    W, H, nf = bc["width"], bc["height"], bc["frames"]
    clips_meta = bc["clips"][:max(1, min(a.clips, len(bc["clips"])))]
    nclip = len(clips_meta)

    clips = None
    cfg5 = None
    if a.shard == "streams" and world == 1 and not a.no_legs and a.config5_streams > 0:
        cfg5 = config5_frames()  # before anything touches the GPU (worker processes fork)
        progress("config-5 input synthesised")
    if a.shard == "streams":  # synthesise the inputs before anything touches the GPU (worker processes fork)
        from thor_amd import synth

        clips = []
        for cm in clips_meta:
            c = synth.synth_frames(W, H, nf, cm["seed"], workers=8)
            assert hashlib.md5(c.tobytes()).hexdigest() == cm["synth_md5"], "synthetic clip %d drifted" % cm["seed"]
            clips.append(c)
            progress("clip %d synthesised" % cm["seed"])

    import torch

    dist = None
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    if a.shard == "rows":
        return rows_mode(a, torch, dist, rank, world, local)

    from thor_amd import lib as L
    from thor_amd.bitstream import Parser, parse_stream
    from thor_amd.decoder import GpuDecoder, decode_batch
    from thor_amd.encoder import GpuEncoder, encode_batch, encode_batch_begin, encode_batch_end, params_for

    lib = L.load()
    dev = torch.device("cuda", local)
    K = max(1, min(a.streams, 512))  # THOR_ENC_MAX_BATCH
    clip_of = [k % nclip for k in range(K)]
    fsize = W * H * 3 // 2
    # the raw input: each clip in pinned host memory; each stream's frames in its own HBM buffer, filled by
    # H2D copies inside the timed region (a copy stream, frame-major, overlapped with encoding)
    host = [torch.from_numpy(c.reshape(nf, fsize)).pin_memory() for c in clips]
    inbuf = [torch.empty((nf, fsize), dtype=torch.uint8, device=dev) for _ in range(K)]
    copy_stream = torch.cuda.Stream(device=dev)
    encs = []
    for k in range(K):
        e = GpuEncoder(params_for(bc["config"], W, H, nf, bc["extra"]), device=local)
        e.use_device_sequence(inbuf[k].data_ptr(), nf)
        if a.enc_cu_exclude and k == 0:  # the batch runs on its first member's stream (one masked queue, not K)
            ncu = torch.cuda.get_device_properties(dev).multi_processor_count
            words = [0] * ((ncu + 31) // 32)
            for c in range(ncu):
                if c % 32 < 32 - a.enc_cu_exclude:
                    words[c // 32] |= 1 << (c % 32)
            e.set_cu_mask(words)
        encs.append(e)
    want_bit = [None] * nclip  # the reference Thorenc's .bit per clip: md5 in bench_clips.json
    seq, _ = parse_stream(open(os.path.join(gold, "k4_low.bit"), "rb").read())  # sequence header (all clips share it)
    decs = [GpuDecoder(seq, device=local, slots=a.dec_slots) for _ in range(K)]
    groups = [list(range(g, min(g + 8, K))) for g in range(0, K, 8)]  # THOR_MAX_BATCH contexts per launch
    dec_streams = []
    for gk in groups:  # a group's members enqueue on their leader's stream
        if a.dec_priority:  # the short decode launches ahead of the encoder's queued row workers
            ps = torch.cuda.Stream(device=dev, priority=-1)
            dec_streams.append(ps)
            decs[gk[0]].set_stream(C.c_void_p(ps.cuda_stream))
        for k in gk[1:]:
            decs[k].set_stream(C.c_void_p(decs[gk[0]].stream()))
    pools = [[{} for _ in range(nf)] for _ in range(K)]  # per stream and frame: re-used device buffers
    pool = ThreadPoolExecutor(HOST_THREADS)

    def upload_inputs(ks):
        """Enqueue every input frame of streams ks (frame-major) on the copy
        stream; returns one event per frame index (that frame of every stream
        resident)."""
        evs = []
        with torch.cuda.stream(copy_stream):
            for i in range(nf):
                for k in ks:
                    inbuf[k][i].copy_(host[clip_of[k]][i], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(copy_stream)
                evs.append(ev)
        return evs

    def enc_wait(ks, ev):  # the batch runs on its first member's stream: it waits for the frame's copies
        torch.cuda.ExternalStream(encs[ks[0]].stream(), device=dev).wait_event(ev)

    def encode(ks):
        for k in ks:
            encs[k].reset()
        evs = upload_inputs(ks)
        bits = [[] for _ in ks]
        fms = []
        for i in range(nf):
            t0 = time.perf_counter()
            enc_wait(ks, evs[i])
            for j, ch in enumerate(encode_batch([encs[k] for k in ks])):
                bits[j].append(ch)
            fms.append((time.perf_counter() - t0) * 1e3)
        return [b"".join(b) for b in bits], fms

    def decode(ks, bits):
        def host_leg(j):  # parse + upload of one stream (GIL released inside the C calls)
            k = ks[j]
            _, frames = parse_stream(bits[j])
            return [decs[k].upload(fr, pools[k][i]) for i, fr in enumerate(frames)]

        t0 = time.perf_counter()
        devs = list(pool.map(host_leg, range(len(ks))))
        dec_host_s[0] += time.perf_counter() - t0
        gs = [[j for j, k in enumerate(ks) if k in gk] for gk in groups]
        for i in range(nf):
            for g in gs:
                if g:
                    decode_batch([decs[ks[j]] for j in g], [devs[j][i] for j in g])
        for k in ks:
            decs[k].sync()
        return devs

    dec_host_s = [0.0]  # parse + upload share of t_dec (serial steps)
    pipe_tl = {}  # the last pipelined step's timeline (ms from its start)

    def step_pipe(ks):
        """One timed step: H2D of every stream's raw frames on a copy stream,
        frame-pipelined encode + decode (while the GPU codes frame i + 1 of
        every stream, a consumer thread parses frame i's chunks -- one parser
        per stream, 16 host threads --, uploads the parse output and enqueues
        its GPU reconstruction on the decoder streams).  Returns the wall time
        of everything complete, the .bit files and the device frames."""
        t0 = time.perf_counter()
        for k in ks:
            encs[k].reset()
        evs = upload_inputs(ks)
        pipe_tl.update(enc_done_ms=[0.0] * nf, dec_enq_ms=[0.0] * nf)
        parsers = [Parser() for _ in ks]
        bits = [[] for _ in ks]
        devs = [[None] * nf for _ in ks]
        gs = [[j for j, k in enumerate(ks) if k in gk] for gk in groups]
        q = queue.Queue()
        err = []

        def consumer():
            try:
                for i in range(nf):
                    chunks = q.get()
                    if chunks is None:
                        return

                    def host_leg(j):  # parse + one host image + one copy, native (GIL released)
                        return decs[ks[j]].upload_payload(parsers[j], chunks[j], pools[ks[j]][i])

                    ds = list(pool.map(host_leg, range(len(ks))))
                    for g in gs:
                        if g:
                            decode_batch([decs[ks[j]] for j in g], [ds[j] for j in g])
                    for j in range(len(ks)):
                        devs[j][i] = ds[j]
                    pipe_tl["dec_enq_ms"][i] = round((time.perf_counter() - t0) * 1e3, 1)
            except BaseException as e:  # re-raised by the caller
                err.append(e)

        th = threading.Thread(target=consumer)
        th.start()
        sent = 0
        E = [encs[k] for k in ks]

        def collect(i):  # frame i's chunks: to the .bit files and the decode consumer
            chunks = encode_batch_end(E)
            for j, ch in enumerate(chunks):
                bits[j].append(ch)
            q.put([ch[4:] for ch in chunks])  # payload after the 4-byte chunk length (dec/getbits.c:48-69)
            pipe_tl["enc_done_ms"][i] = round((time.perf_counter() - t0) * 1e3, 1)

        try:
            # frame i + 1 is enqueued before frame i is collected: the GPU codes the next frame while the
            # host reads the last one back (thor_enc_frames_begin / _end)
            for i in range(nf):
                enc_wait(ks, evs[i])
                encode_batch_begin(E)
                if i > 0:
                    collect(i - 1)
                    sent += 1
            collect(nf - 1)
            sent += 1
        finally:
            if sent < nf:
                q.put(None)
            th.join()
        pipe_tl["consumer_done_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
        for k in ks:
            decs[k].sync()
        t = time.perf_counter() - t0
        for pr in parsers:
            pr.close()
        if err:
            raise err[0]
        return t, [b"".join(b) for b in bits], devs

    def step(ks):
        t0 = time.perf_counter()
        bits, fms = encode(ks)
        t1 = time.perf_counter()
        devs = decode(ks, bits)
        t2 = time.perf_counter()
        return t1 - t0, t2 - t1, bits, devs, fms

    def bits_ok(ks, bits):
        """every stream's .bit == the reference Thorenc's for its clip (md5)"""
        ok = True
        for j, k in enumerate(ks):
            c = clip_of[k]
            if want_bit[c] is None:
                if hashlib.md5(bits[j]).hexdigest() != clips_meta[c]["bit_md5"]:
                    return False
                want_bit[c] = bits[j]
            ok &= bits[j] == want_bit[c]
        return ok

    def decoded_ok(ks):
        """every stream's decoded sequence == the reference Thordec's for its
        clip: the first stream of each clip by md5, the others byte for byte
        against it"""
        ref = {}
        ok = True
        for k in ks:
            got = b"".join(decs[k].read_i420(fr) for fr in range(nf))
            c = clip_of[k]
            if c not in ref:
                ok &= hashlib.md5(got).hexdigest() == clips_meta[c]["dec_md5"]
                ref[c] = got
            else:
                ok &= got == ref[c]
        return ok

    allk = list(range(K))
    progress("%d encoder + decoder contexts ready" % K)
    for _ in range(max(1, a.warmup)):
        _, bits, devs = step_pipe(allk)
        progress("warmup step done")
    bit_exact = bits_ok(allk, bits) and decoded_ok(allk)
    rf_early = None
    if os.environ.get("THOR_BENCH_RF_EARLY"):  # diagnostic: the roofline pass before the timed steps too
        _, rf_early, _, _, _ = roofline_pass(lib, decs, [groups[0]], devs, [parse_stream(bits[k])[1] for k in groups[0]],
                                          seq, 3)

    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(local)
    elapsed = 0.0
    for _ in range(a.steps):
        te, bits, devs = step_pipe(allk)
        elapsed += te
        progress("timed step: %.1f ms" % (te * 1e3))
        bit_exact &= bits_ok(allk, bits)
        bit_exact &= decoded_ok(allk)  # every timed step's decode checked too (outside the timed region)
    torch.cuda.synchronize(local)
    if dist is not None:
        dist.barrier()
    # the two legs one after the other (one untimed-for-value step): the split of the work
    dec_host_s[0] = 0.0
    t_enc, t_dec, bits, devs, fms = step(allk)
    progress("serial step done")
    bit_exact &= bits_ok(allk, bits)
    enc_frame_ms = fms
    dec_host_ms = dec_host_s[0] * 1e3
    elapsed = reduce_max(dist, dev, elapsed)
    bit_exact = -reduce_max(dist, dev, -1.0 if bit_exact else 0.0) == 1.0
    px_stream = W * H * nf
    value = world * K * px_stream * a.steps / elapsed / 1e6
    in_bytes = K * nf * fsize

    # ---- beside `value` ----
    # single-stream latency: stream 0 alone, encode (its input upload included) + decode
    lat = [step([0])[:2] for _ in range(2)]
    lat_enc, lat_dec = min(x[0] for x in lat), min(x[1] for x in lat)
    # decode_only: reconstruction of every stream's resident parse output (no parse, no upload)
    dsteps = 5
    for k in allk:
        decs[k].sync()
    t0 = time.perf_counter()
    for _ in range(dsteps):
        for i in range(nf):
            for gk in groups:
                decode_batch([decs[k] for k in gk], [devs[k][i] for k in gk])
    for k in allk:
        decs[k].sync()
    t_do = (time.perf_counter() - t0) / dsteps
    frames_of = [parse_stream(bits[k])[1] for k in groups[0]]
    progress("roofline pass")
    stage_ms, recon_ms, alg, B, prep_ms = roofline_pass(lib, decs, [groups[0]], devs, frames_of, seq, 3)
    achieved = alg / (recon_ms / 1e3) / 1e9 if recon_ms > 0 else 0.0
    path_ms = prep_ms + recon_ms
    path_achieved = alg / (path_ms / 1e3) / 1e9 if path_ms > 0 else 0.0
    traffic = None
    traffic_source = None
    tj = a.traffic_json or os.path.join(ROOT, "tools", "traffic_latest.json")
    if os.path.exists(tj):
        tjd = json.load(open(tj))
        traffic = tjd.get("recon_hbm_bytes_per_p_launch")
        # the PMC passes this static figure came from: their profile tag and the commit of the kernels measured
        traffic_source = {"file": os.path.relpath(tj, ROOT), "profile_tag": tjd.get("tag"),
                          "kernels_commit": tjd.get("commit"), "profile": tjd.get("profile")}

    out = None
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "Mpixels/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8/i16",
            "data": "synthetic: %d distinct seeded 4K clips (thor_amd/synth.py, seeds %s), streams round-robin over "
                    "them; every step uploads each stream's raw frames from pinned host memory inside the timed "
                    "region (H2D on a copy stream, overlapped with encoding); decoded frames stay in HBM"
                    % (nclip, [c["seed"] for c in clips_meta]),
            "bit_exact": bit_exact,
            "bit_exact_scope": "every stream of every timed step: .bit md5 == the reference Thorenc's for its clip, "
                               "decoded sequence == the reference Thordec's (tests/golden/bench_clips.json)",
            "config": {
                "workload": "encode + decode of 4K (3840x2160) 8-frame config_LDB_low_complexity streams: "
                            "raw frames host -> HBM, device-resident encoder (RD loop, loop filters, CLPF, bit "
                            "packing) -> .bit == reference Thorenc's; host parse -> upload -> GPU reconstruction "
                            "== reference Thordec's output",
                "frames": nf, "width": W, "height": H, "clips": nclip,
                "parallelism": "streams: %d GPU(s) x %d independent streams" % (world, K),
                "streams_per_gpu": K,
                "h2d_bytes_per_step": in_bytes,
                "pipelining": "frame-pipelined: the H2D of frame i + 1's raw input and the host parse + upload + "
                              "GPU reconstruction of frame i run while the GPU encodes frame i + 1 (value = wall "
                              "time of everything complete)",
                "pipe_timeline_last_step": pipe_tl,
                "serial_t_enc_ms": round(t_enc * 1e3, 2),
                "serial_t_dec_ms": round(t_dec * 1e3, 2),
                "serial_mpx_s": round(K * px_stream / (t_enc + t_dec) / 1e6, 2),
                "serial_note": "one extra step with the legs one after the other: upload + encode all frames, then "
                               "parse + upload + reconstruct (the split of the work; not `value`)",
                "t_dec_host_ms": round(dec_host_ms, 2),
                "t_dec_host_note": "host parse (thor_parse_frame) + upload of the parse output, %d threads, "
                                   "in the serial step" % HOST_THREADS,
                "enc_mpx_s": round(K * px_stream / t_enc / 1e6, 2),
                "dec_mpx_s": round(K * px_stream / t_dec / 1e6, 2),
                "enc_batch_frame_ms": [round(x, 2) for x in enc_frame_ms],
                "single_stream_enc_ms": round(lat_enc * 1e3, 2),
                "single_stream_dec_ms": round(lat_dec * 1e3, 2),
                "single_stream_mpx_s": round(px_stream / (lat_enc + lat_dec) / 1e6, 2),
                "decode_only_mpx_s": round(K * px_stream / t_do / 1e6, 1),
                "decode_only_note": "GPU reconstruction of the K streams' resident parse output (no parse, "
                                    "no upload): the round-1 headline",
                "stage_ms_per_stream_pass": {k: round(v, 4) for k, v in zip(STAGES + ["interp"], stage_ms)},
                "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
                "decoder_stream_priority": "high" if a.dec_priority else "default",
                "enc_cu_exclude_per_32": a.enc_cu_exclude,
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "k_recon",
                "achieved": round(achieved, 1),
                "peak": PEAK_HBM_GBS,
                "unit": "GB/s",
                "frac": round(achieved / PEAK_HBM_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_source,
                "alg_bytes_per_launch": round(alg),
                "avg_launch_us": round(recon_ms * 1e3, 2),
                **({"avg_launch_us_before_steps": round(rf_early * 1e3, 2)} if rf_early is not None else {}),
                "frames_per_launch": B,
                "path": {
                    "kernels": ["k_frame_prep", "k_recon"],
                    "achieved": round(path_achieved, 1),
                    "frac": round(path_achieved / PEAK_HBM_GBS, 4),
                    "avg_us": round(path_ms * 1e3, 2),
                    "prep_avg_launch_us": round(prep_ms * 1e3, 2),
                    "note": "the whole 4K inter-reconstruction path of a batched P launch: side info + MC words + "
                            "dequant + inverse transform of every coded TU (k_frame_prep), then MC + residual add "
                            "+ stores (k_recon); same algorithmic bytes over the sum of both kernels' launch "
                            "durations (hipEvents on the decode stream)",
                },
                "launches": "batched P-frame decode launches of group 0 alone (streams of clips 0..7, the inter "
                            "stage: one k_recon launch -- 128x16 units, the frames' multi-key units first); "
                            "hipEvents on its stream",
                "dominant_kernel_note": "by GPU time the step is k_enc_rows, the encoder's superblock worker: "
                                        "integer RD search with negligible HBM traffic and no MFMA work, latency "
                                        "bound inside the wave (DESIGN.md 3b), so neither roofline bounds it; this "
                                        "object is k_recon, the north star's inter-reconstruction kernel",
            },
        }
    if not a.no_rows:  # every rank: the north star's row split of ONE config-4 stream at this N
        progress("rows leg: config 4 over %d rank(s)" % world)
        rows = rows_guarded(a, torch, dist, rank, world, local, out)
        if rank == 0:
            out["rows"] = rows
    if rank == 0:
        if world == 1 and not a.no_legs:
            progress("legs")
            out["encoder_tu_chain"] = encoder_leg(torch, lib)
            out["temporal_pyramid"] = pyramid_leg(torch, lib)
            out["temporal_interp_comp"] = interp_leg(torch, lib)
            out["temporal_interp_frame"] = interp_frames_leg(torch, lib, clips[0])
            progress("config-3 leg")
            out["config3_encoder"] = config3_leg(torch, lib, a.config3_streams)
            progress("config-5 leg")
            if cfg5 is not None:
                out["config5_encoder"] = config5_leg(torch, lib, cfg5, a.config5_streams)
        if not a.no_cpu_baseline and world == 1:
            progress("CPU baseline")
            cb = cpu_baseline(bc, clips_meta, clips)
            if cb is not None:
                out["cpu_baseline"] = cb
        print(json.dumps(out), flush=True)
    pool.shutdown()
    for x in encs + decs:
        x.close()
    if dist is not None:
        dist.destroy_process_group()


def dropin_mode(a):
    """--drop-in: the reference decoder's own host C linked against this
    library's SIMD-surface / L2 entry points (oracle/_ref/thordec_amd: every
    per-block kernel call of dec/decode_block.c:48-453 and the frame deblock
    runs on the GPU, one small launch per call) timed beside the reference
    Thordec (SIMD build, one core) on the same .bit; both outputs md5-checked
    against the reference decoder's.  The per-call surface exists for drop-in
    compatibility; the batched decoder (thor_dec_frames) is the throughput API."""
    gold = os.path.join(ROOT, "tests", "golden")
    name = a.drop_in
    meta = json.load(open(os.path.join(gold, "streams.json")))[name]
    bit = os.path.join(gold, name + ".bit")
    out = {"metric": "Mpixels/s decode, %s (%dx%d x %d frames) through the reference decoder host C" % (
        name, meta["width"], meta["height"], meta["frames"]), "unit": "Mpixels/s", "higher_is_better": True}
    px = meta["width"] * meta["height"] * meta["frames"]
    import tempfile

    for key, exe in (("reference_thordec_simd_1core", "Thordec"), ("thordec_amd_gpu_surface", "thordec_amd")):
        path = os.path.join(ROOT, "oracle", "_ref", exe)
        if not os.path.exists(path):
            out[key] = None
            continue
        with tempfile.TemporaryDirectory() as td:
            dec = os.path.join(td, "dec.yuv")
            best = None
            for _ in range(a.steps):
                t0 = time.perf_counter()
                subprocess.run([path, bit, dec], check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
                dt = time.perf_counter() - t0
                best = dt if best is None else min(best, dt)
            ok = hashlib.md5(open(dec, "rb").read()).hexdigest() == meta["dec_md5"]
        out[key] = {"seconds": round(best, 3), "mpx_s": round(px / best / 1e6, 3), "bit_exact": ok}
    r, g = out.get("reference_thordec_simd_1core"), out.get("thordec_amd_gpu_surface")
    if r and g:
        out["gpu_surface_vs_reference"] = round(r["seconds"] / g["seconds"], 4)
    print(json.dumps(out), flush=True)


def rows_mode(a, torch, dist, rank, world, local):
    """--shard rows: one 4K stream, its SB rows split across the ranks
    (thor_amd/shard.py); strong scaling.  Each frame: band reconstruction,
    RCCL all-gather of the bands (device buffers, torch's stream), then the
    whole-frame intra / deblock / CLPF / pad on every rank."""
    from thor_amd.decoder import GpuDecoder
    from thor_amd.shard import RowShard
    from thor_amd.trace import load_trace

    if dist is None:  # a one-rank group keeps the same code path
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", local))
    gold = os.path.join(ROOT, "tests", "golden")
    meta = json.load(open(os.path.join(gold, "streams.json")))["k4_low"]
    seq, frames = load_trace(os.path.join(gold, "k4_low.trc.z"))
    dec = GpuDecoder(seq, device=local)
    devs = [dec.upload(fr) for fr in frames]
    sh = RowShard(dec, dist, seq.width, seq.height, device_exchange=True,
                  band_local=a.band_local or a.halo or a.boundary, halo=a.halo or a.boundary, boundary=a.boundary)

    def step():
        for d, fr in zip(devs, frames):
            sh.decode(d, fr.frame_num, fr)

    for _ in range(max(1, a.warmup)):
        step()
    torch.cuda.synchronize(local)
    # halo mode: no rank holds every row final -- each frame is put together from
    # its bands' owners (outside the timed region)
    got = {fr.frame_num: sh.assemble(fr.frame_num) if (a.halo or a.boundary) else dec.read_i420(fr.frame_num)
           for fr in frames}
    ok = hashlib.md5(b"".join(got[k] for k in sorted(got))).hexdigest() == meta["dec_md5"]
    dist.barrier()
    torch.cuda.synchronize(local)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize(local)
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    okt = torch.tensor([1 if ok else 0], device="cuda")
    dist.all_reduce(okt, op=dist.ReduceOp.MIN)
    elapsed, ok = float(t.item()), bool(okt.item())
    px_step = seq.width * seq.height * len(frames)
    if rank == 0:
        print(json.dumps({
            "metric": METRIC, "value": round(px_step * a.steps / elapsed / 1e6, 2), "unit": "Mpixels/s",
            "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 4), "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "u8/i16", "data": "synthetic (seeded clip) encoded by the reference Thorenc",
            "bit_exact": ok,
            "config": {"workload": "ONE 4K 8-frame LDB-low stream, SB rows sharded across %d GPU(s): band k_recon, %s" % (
                                   world, "band intra, boundary exchange (edge rows for the intra chains, 8-row "
                                   "deblocking halos; no all-gather), band-local deblock/CLPF, MV-reach halo exchange "
                                   "of reference rows" if a.boundary
                                   else "RCCL all-gather of pre-deblock bands, whole-frame intra, " + (
                                       "band-local deblock/CLPF, pad, MV-reach halo exchange of reference rows"
                                       if a.halo else "band-local deblock/CLPF + all-gather of final bands, pad"
                                       if a.band_local else "whole-frame deblock/CLPF/pad")),
                       "parallelism": "rows%d" % world, "frames": len(frames)},
        }), flush=True)
    dec.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

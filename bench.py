#!/usr/bin/env python3
"""Benchmark: Thor per-block reconstruction on MI355X.

Workload (config.workload): the reference's own 4K (3840x2160) 8-frame
config_LDB_low_complexity stream of a seeded synthetic clip
(tests/golden/k4_low.*).  One step = GPU reconstruction of the whole stream,
frame after frame as the decoder must (frame n+1 references frame n): per
frame, per-4x4 side info, inter MC + dequant + inverse transform +
reconstruction, intra, deblock Y/UV, CLPF and reference padding, all through
libthor_amd.so's C-ABI.  The parse output (block descriptors, coefficients,
intra list, CLPF flags) is resident in HBM before timing starts; bit parsing
is CPU work outside the hot path.  The decoded frames are checked bit-exact
against the reference decoder's md5s (every context) after warmup.

Per GPU, --streams K (default 24: 3 groups of 8, THOR_MAX_BATCH) independent decoder contexts each decode
their own copy of the stream on their own HIP stream, interleaved frame by
frame (a server decoding K streams): value = K x stream pixels / time.  The
single-stream latency of one pass is reported next to it
(config.single_stream_ms_per_pass).

N > 1: one process per GPU, each with its own K streams (independent
streams, no data-path collective): scaling "weak".

Prints one JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import ctypes as C
import hashlib
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# one hardware queue per decoder context (HIP's default is 4 per process);
# must be set before the HIP runtime initialises
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

import numpy as np  # noqa: E402

METRIC = "Mpixels/s encode+decode, 4K LDB_low_complexity; bit-exact vs ref"
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
STAGES = ["prep", "inter", "intra", "deblock", "clpf", "pad"]


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
    (thor_enc_tu_batch), then cost_calc per CU (thor_enc_cost_batch).  The
    serial RD search that would issue these batches is not on the GPU
    (SURVEY.md sec. 8(f) #4)."""
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


def cpu_baseline(meta, gold, budget_s: float = 20.0):
    """Reference decoder (oracle/_ref/Thordec, SIMD build, 1 thread) on the
    same .bit, repeated up to ~budget_s; falls back to the oracle port."""
    exe = os.path.join(ROOT, "oracle", "_ref", "Thordec")
    bit = os.path.join(gold, "k4_low.bit")
    px = meta["width"] * meta["height"] * meta["frames"]
    if os.path.exists(exe):
        out = "/tmp/thor_bench_dec_%d.yuv" % os.getpid()
        runs, t_tot = 0, 0.0
        while t_tot < budget_s and runs < 30:
            t0 = time.perf_counter()
            subprocess.run([exe, bit, out], check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            t_tot += time.perf_counter() - t0
            runs += 1
        ok = hashlib.md5(open(out, "rb").read()).hexdigest() == meta["dec_md5"]
        os.remove(out)
        return {"value": round(px * runs / t_tot / 1e6, 3), "unit": "Mpixels/s", "cores": 1, "kind": "reference",
                "sample": "reference Thordec (SIMD build, -O3, 1 thread) decoding the same 4K 8-frame .bit "
                          "%d times (bit parsing included); output md5 %s" % (runs, "ok" if ok else "MISMATCH")}
    from oracle import OracleDecoder
    from thor_amd.trace import load_trace

    seq, frames = load_trace(os.path.join(gold, "k4_low.trc.z"))
    t0 = time.perf_counter()
    dec = OracleDecoder(seq)
    for _ in dec.run(frames):
        pass
    dt = time.perf_counter() - t0
    return {"value": round(px / dt / 1e6, 3), "unit": "Mpixels/s", "cores": 1, "kind": "port",
            "sample": "oracle restatement (plain C, 1 thread), full 8-frame stream"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--streams", type=int, default=24, help="independent decoder contexts per GPU")
    ap.add_argument("--groups", type=int, default=3,
                    help="batches per frame slot (contexts of a group share one launch per stage)")
    ap.add_argument("--shard", choices=["streams", "rows"], default="streams",
                    help="streams: independent streams per GPU (default); rows: ONE stream's SB rows split "
                         "across the ranks with an RCCL all-gather of the bands before intra/deblock")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC-derived HBM bytes per k_recon launch (default tools/traffic_latest.json, "
                         "copied from profiles/<tag>_traffic.json by tools/prof_summary.py)")
    a = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch

    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)

    if a.shard == "rows":
        return rows_mode(a, torch, dist, rank, world, local)

    from thor_amd import lib as L
    from thor_amd.decoder import GpuDecoder, decode_batch
    from thor_amd.trace import load_trace

    gold = os.path.join(ROOT, "tests", "golden")
    meta = json.load(open(os.path.join(gold, "streams.json")))["k4_low"]
    seq, frames = load_trace(os.path.join(gold, "k4_low.trc.z"))
    # K decoder contexts per GPU, each decoding its own copy of the stream on its
    # own HIP stream (independent streams, as a server decodes many): the I
    # frame's intra chain occupies ~100 waves, so other streams' frames fill the
    # GPU meanwhile.  Context 0 alone gives the single-stream latency.
    K = max(1, a.streams)
    # each context enqueues on its own non-blocking HIP stream (created by
    # thor_dec_create, consecutively, so they spread over the hardware queues)
    decs, devs = [], []
    for k in range(K):
        dk = GpuDecoder(seq, device=local)
        decs.append(dk)
        devs.append([dk.upload(fr) for fr in frames])
    dec = decs[0]
    torch.cuda.synchronize(local)

    # Contexts are split into G groups; a group decodes its contexts' next frames
    # with one launch per stage (thor_dec_frames) on its leader's HIP stream.
    # Every context decodes the stream cyclically (frames 0..7, 0..7, ...) and
    # group g runs (8g/G) frames out of phase with group 0, so the groups' I
    # frames (the latency-bound intra chains) overlap other groups' P frames.
    nf = len(frames)
    G = max(1, min(a.groups, K))
    groups = [list(range(g, K, G)) for g in range(G)]
    gphase = [(g * nf) // G for g in range(G)]
    phase = [0] * K
    for g, ks in enumerate(groups):
        for k in ks:
            phase[k] = gphase[g]

    for gk in groups:  # a group's members enqueue on their leader's stream
        for k in gk[1:]:
            decs[k].set_stream(C.c_void_p(decs[gk[0]].stream()))

    def step(ks=None, gs=None):
        for i in range(nf):  # interleave the groups frame by frame
            if ks is not None:
                for k in ks:
                    decs[k].decode(devs[k][(phase[k] + i) % nf])
                continue
            for g in (range(G) if gs is None else gs):
                gk = groups[g]
                decode_batch([decs[k] for k in gk], [devs[k][(gphase[g] + i) % nf] for k in gk])

    def sync_all():
        for dk in decs:
            dk.sync()
        torch.cuda.synchronize(local)

    for k in range(K):  # one plain pass (every reference resident), then shift to the context's phase
        for i in range(nf + phase[k]):
            decs[k].decode(devs[k][i % nf])
    for _ in range(a.warmup):
        step()
    sync_all()

    # check bit-exactness of what every context produced
    bit_exact = True
    for dk in decs:
        got = {fr.frame_num: dk.read_i420(fr.frame_num) for fr in frames}
        yuv = b"".join(got[k] for k in sorted(got))
        bit_exact &= hashlib.md5(yuv).hexdigest() == meta["dec_md5"]

    lib = L.load()
    if dist is not None:
        dist.barrier()
    sync_all()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    sync_all()
    elapsed = time.perf_counter() - t0

    # single-stream latency of one pass over the stream (context 0 alone)
    lsteps = max(1, min(a.steps, 10))
    t1 = time.perf_counter()
    for _ in range(lsteps):
        step(ks=[0])
    sync_all()
    latency_ms = (time.perf_counter() - t1) / lsteps * 1e3

    # instrumented pass (not part of `value`): group 0 alone, hipEvents around
    # every stage of every batched launch on its stream, for the stage breakdown
    # and the roofline (one launch = the group's B frames)
    isteps = max(1, min(a.steps, 5))
    lead = decs[groups[0][0]]
    B = len(groups[0])
    lib.thor_dec_set_timing(lead.h, 1)
    cap = 8 * len(frames) * (isteps + 1)
    mk_stage, mk_ms = (C.c_int * cap)(), (C.c_double * cap)()
    lib.thor_dec_stage_marks(lead.h, mk_stage, mk_ms, cap)
    for _ in range(isteps):
        step(gs=[0])
    nm = lib.thor_dec_stage_marks(lead.h, mk_stage, mk_ms, cap)
    lib.thor_dec_set_timing(lead.h, 0)
    # attribute the marks to frames: every frame opens with its side-info stage (0)
    per_frame, cur = [], None
    for k in range(nm):
        if mk_stage[k] == 0:
            cur = [0.0] * 6
            per_frame.append(cur)
        cur[mk_stage[k]] += mk_ms[k]
    assert len(per_frame) == isteps * len(frames), (len(per_frame), isteps, len(frames))
    stage_ms = [sum(f[i] for f in per_frame) / isteps / B for i in range(6)]  # per stream pass
    # k_recon roofline over the P frames (the I frame has no inter pixels)
    pidx = [i for i, fr in enumerate(frames) if fr.frame_type != 0]
    recon_ms = sum(per_frame[s * len(frames) + i][1] for s in range(isteps) for i in pidx) / (isteps * len(pidx))
    alg = B * sum(recon_alg_bytes(frames[i], seq.width, seq.height) for i in pidx) / len(pidx)  # per launch
    if dist is not None:
        t = torch.tensor([elapsed], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        ok = torch.tensor([1 if bit_exact else 0], device="cuda")
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        bit_exact = bool(ok.item())

    px_step = seq.width * seq.height * len(frames)
    value = world * K * px_step * a.steps / elapsed / 1e6
    ms_per_step = elapsed / a.steps * 1e3

    achieved = alg / (recon_ms / 1e3) / 1e9 if recon_ms > 0 else 0.0
    traffic = None
    tj = a.traffic_json or os.path.join(ROOT, "tools", "traffic_latest.json")
    if os.path.exists(tj):
        traffic = json.load(open(tj)).get("recon_hbm_bytes_per_p_launch")

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "Mpixels/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8/i16",
            "data": "synthetic (seeded clip, thor_amd/synth.py) encoded by the reference Thorenc; "
                    "parse output resident in HBM",
            "bit_exact": bit_exact,
            "config": {
                "workload": "decode-side per-block reconstruction of the 4K (3840x2160) 8-frame "
                            "config_LDB_low_complexity reference stream: inter MC + dequant + inverse transform + "
                            "recon, intra, deblock, CLPF, padding (encode-side reconstruction not yet on GPU)",
                "frames": len(frames),
                "width": seq.width,
                "height": seq.height,
                "parallelism": "streams: %d GPU(s) x %d independent decoder contexts" % (world, K),
                "streams_per_gpu": K,
                "batch_groups": G,
                "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
                "single_stream_ms_per_pass": round(latency_ms, 4),
                "single_stream_mpx_s": round(px_step / latency_ms / 1e3, 1),
                "stage_ms_per_step": {k: round(v, 4) for k, v in zip(STAGES, stage_ms)},
                "stage_note": "per stream pass: hipEvent-bracketed batched stages of group 0 alone / frames per launch",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "k_recon",
                "achieved": round(achieved, 1),
                "peak": PEAK_HBM_GBS,
                "unit": "GB/s",
                "frac": round(achieved / PEAK_HBM_GBS, 4),
                "traffic": traffic,
                "alg_bytes_per_launch": round(alg),
                "avg_launch_us": round(recon_ms * 1e3, 2),
                "frames_per_launch": B,
                "launches": "batched P-frame launches of group 0 alone; hipEvents on its stream",
            },
        }
        if world == 1:
            out["encoder_tu_chain"] = encoder_leg(torch, lib)
            out["temporal_pyramid"] = pyramid_leg(torch, lib)
            out["temporal_interp_comp"] = interp_leg(torch, lib)
        if not a.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(meta, gold)
        print(json.dumps(out), flush=True)
    for dk in decs:
        dk.close()
    if dist is not None:
        dist.destroy_process_group()


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
    dec.set_stream(C.c_void_p(torch.cuda.current_stream(local).cuda_stream))
    devs = [dec.upload(fr) for fr in frames]
    sh = RowShard(dec, dist, seq.width, seq.height, device_exchange=True)

    def step():
        for d, fr in zip(devs, frames):
            sh.decode(d, fr.frame_num)

    for _ in range(max(1, a.warmup)):
        step()
    torch.cuda.synchronize(local)
    got = {fr.frame_num: dec.read_i420(fr.frame_num) for fr in frames}
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
            "config": {"workload": "ONE 4K 8-frame LDB-low stream, SB rows sharded across %d GPU(s): band k_recon, "
                                   "RCCL all-gather of pre-deblock bands, whole-frame intra/deblock/CLPF/pad" % world,
                       "parallelism": "rows%d" % world, "frames": len(frames)},
        }), flush=True)
    dec.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

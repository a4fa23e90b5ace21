"""GPU parity of the device-resident encoder (thor_enc_*, k_enc_rows): the
reference encoder's own bitstreams (tests/golden/<name>.bit, written by the
reference Thorenc from the seeded synthetic clips) must come out byte for
byte, frame by frame."""
import os
import time
import hashlib

import numpy as np
import pytest

from thor_amd import synth

pytestmark = pytest.mark.gpu


def _frames(b):
    out, o = [], 0
    while o < len(b):
        n = int.from_bytes(b[o:o + 4], "big")
        out.append(b[o:o + 4 + n])
        o += 4 + n
    return out


def _rd_frames(name):
    """The reference encoder's per-superblock RD costs for `name`
    (tests/golden/rd_costs.npz, tools/make_rd_goldens.py: -Wl,--wrap=process_block
    on the reference Thorenc), grouped per coded frame in coding order: int32
    rows (frame_num, size, ypos, xpos, qp, cost), one per top-level
    process_block call -- every delta-QP trial, then the final encode -- in
    raster SB order.  None when the stream has no RD golden."""
    z = np.load(os.path.join("tests", "golden", "rd_costs.npz"))
    if name not in z.files:
        return None
    r = z[name]
    order = []
    for f in r[:, 0]:
        if not order or order[-1] != f:
            order.append(int(f))
    return [r[r[:, 0] == f] for f in order]


def _check_rd(enc, want, i, name):
    """Coded frame i's per-SB RD costs (thor_enc_sb_costs) == the reference's."""
    if want is None or i >= len(want):
        return
    got = enc.sb_costs()
    w = want[i]
    assert got.size == len(w), (name, i, got.shape, len(w))
    bad = np.nonzero(got.reshape(-1) != w[:, 5])[0]
    assert bad.size == 0, (name, i, "first differing call (frame, size, y, x, qp, ref cost), device cost",
                           w[bad[0]].tolist(), int(got.reshape(-1)[bad[0]]), "of", bad.size)


def _input(meta, n):
    # serial: no fork from a process that has initialised the GPU
    return synth.synth_frames(meta["width"], meta["height"], n, meta["seed"], workers=1)


@pytest.mark.parametrize("name,nframes", [("cif_low", 10), ("w8_low", 6), ("cif_med", 10), ("hd_low", 17)])
def test_device_encoder_matches_reference_bitstream(name, nframes, streams):
    from thor_amd.encoder import GpuEncoder, params_for

    meta = streams[name]
    p = params_for(meta["config"], meta["width"], meta["height"], nframes, meta["extra"])
    enc = GpuEncoder(p)
    rd = _rd_frames(name)
    try:
        enc.upload_sequence(_input(meta, nframes))
        if rd is not None:
            enc.record_sb_costs()
        want = _frames(open("tests/golden/%s.bit" % name, "rb").read())
        for i in range(enc.num_frames()):
            got = enc.encode_next()
            assert got == want[i], (name, i, len(got), len(want[i]))
            _check_rd(enc, rd, i, name)
    finally:
        enc.close()


def test_batched_encoders_match_reference(streams):
    """thor_enc_frames: several streams' next frames in one launch per stage."""
    from thor_amd.encoder import GpuEncoder, encode_batch, params_for

    meta = streams["cif_low"]
    want = _frames(open("tests/golden/cif_low.bit", "rb").read())
    encs = []
    try:
        for _ in range(3):
            e = GpuEncoder(params_for(meta["config"], meta["width"], meta["height"], 10, meta["extra"]))
            e.upload_sequence(_input(meta, 10))
            encs.append(e)
        for i in range(10):
            for got in encode_batch(encs):
                assert got == want[i], i
    finally:
        for e in encs:
            e.close()


@pytest.mark.parametrize("name", ["cif_low", "cif_high", "hd_low", "k4_med", "w8_low"])
def test_gpu_decode_from_bitstream(name, streams):
    """The product decode path from a .bit: host parser (thor_parse_frame) ->
    device descriptors -> batched GPU reconstruction; the decoded sequence must
    match the reference decoder's output md5."""
    from thor_amd.bitstream import parse_stream
    from thor_amd.decoder import GpuDecoder

    meta = streams[name]
    seq, frames = parse_stream(open("tests/golden/%s.bit" % name, "rb").read())
    dec = GpuDecoder(seq)
    try:
        out = {}
        for fr in frames:
            dec.decode(dec.upload(fr))
            out[fr.frame_num] = dec.read_i420(fr.frame_num)
            assert hashlib.md5(out[fr.frame_num]).hexdigest() == meta["stage_md5"][fr.decode_order]["final"]
        assert hashlib.md5(b"".join(out[k] for k in sorted(out))).hexdigest() == meta["dec_md5"]
    finally:
        dec.close()


@pytest.mark.parametrize("name,nframes", [("cif_high", 4), ("k4_low", 8), ("k4_med", 3), ("hd_high", 2)])
def test_device_encoder_more_configs(name, nframes, streams):
    """LDB high-efficiency (speed 0: telescope + exact sub-pel ME, tb / pb split,
    4 references, delta-qp RD search; CIF at -qp 22 and 1080p at the config's
    qp 32) and 4K LDB-low / medium."""
    from thor_amd.encoder import GpuEncoder, params_for

    meta = streams[name]
    p = params_for(meta["config"], meta["width"], meta["height"], nframes, meta["extra"])
    enc = GpuEncoder(p)
    rd = _rd_frames(name)
    try:
        enc.upload_sequence(_input(meta, nframes))
        if rd is not None:  # per-SB RD costs == the reference's (every delta-QP trial and final encode)
            enc.record_sb_costs()
        want = _frames(open("tests/golden/%s.bit" % name, "rb").read())
        for i in range(enc.num_frames()):
            got = enc.encode_next()
            assert got == want[i], (name, i, len(got), len(want[i]))
            _check_rd(enc, rd, i, name)
    finally:
        enc.close()


@pytest.mark.parametrize("name", ["cif_hdb", "cif_hdbi", "cif_hdbi_high", "k4_hdbi"])
def test_device_encoder_hierarchical_b(name, streams):
    """Hierarchical B (HDB16, 16-frame sub-GOP, coding order != display order):
    cif_hdb without interpolated references; cif_hdbi / k4_hdbi (speed 2) and
    cif_hdbi_high (speed 0: the joint mv0 = -mv1 bi-pred search,
    enc/encode_block.c:2410-2426) with the temporal-interpolated reference
    built on the GPU per B frame (enc/mainenc.c:324-330) -- every frame of the
    reference Thorenc's .bit, byte for byte."""
    _encode_and_compare(name, streams[name]["frames"], streams)


def test_device_encoder_4k_hdb16_high_efficiency(streams):
    """BASELINE config 5 at its stated size and operating point: 4K
    config_HDB16_high_efficiency (speed 0, interpolated references, 4
    references, tb / pb split, delta-qp).  The first three coded frames of the
    17-frame plan -- the I frame, the P frame 16 and the B frame 8 (joint
    bi-pred search against the interpolated reference) -- byte-equal to the
    reference Thorenc's tests/golden/k4_hdbi_high.bit, every SB's RD costs
    equal to the reference's (rd_costs.npz).  Default-on since round 6: I 27.5 s,
    P 16 66.3 s, B 8 87.7 s on one stream, 189 s in all (profiles/r07t_cfg5_long.log);
    it replaces the I + P 16 test."""
    _encode_and_compare("k4_hdbi_high", streams["k4_hdbi_high"]["frames"], streams, limit=3)


def _encode_and_compare(name, nframes, streams, limit=None):
    from thor_amd.encoder import GpuEncoder, params_for

    meta = streams[name]
    p = params_for(meta["config"], meta["width"], meta["height"], nframes, meta["extra"])
    enc = GpuEncoder(p)
    rd = _rd_frames(name)
    try:
        enc.upload_sequence(_input(meta, nframes))
        if rd is not None:
            enc.record_sb_costs()
        want = _frames(open("tests/golden/%s.bit" % name, "rb").read())
        assert enc.num_frames() == len(want)
        for i in range(enc.num_frames() if limit is None else limit):
            t0 = time.perf_counter()
            got = enc.encode_next()
            print("%s frame %d: %d bytes, %.2f s" % (name, i, len(got), time.perf_counter() - t0),
                  flush=True)  # progress (long speed-0 clips)
            assert got == want[i], (name, i, len(got), len(want[i]))
            _check_rd(enc, rd, i, name)
    finally:
        enc.close()


def test_pipelined_batches_match_reference(streams):
    """thor_enc_frames_begin / _end: frame i + 1 of every context begun before
    frame i is ended (two batches in flight) -- the same bytes as the reference
    encoder; a third begin without an end is refused."""
    import ctypes as C

    from thor_amd import lib as L
    from thor_amd.encoder import GpuEncoder, encode_batch_begin, encode_batch_end, params_for

    meta = streams["cif_med"]
    want = _frames(open("tests/golden/cif_med.bit", "rb").read())
    encs = []
    try:
        for _ in range(3):
            e = GpuEncoder(params_for(meta["config"], meta["width"], meta["height"], 10, meta["extra"]))
            e.upload_sequence(_input(meta, 10))
            encs.append(e)
        got = [[] for _ in encs]
        encode_batch_begin(encs)
        for i in range(10):
            if i + 1 < 10:
                encode_batch_begin(encs)
                if i == 0:  # two in flight: a third is refused
                    n = len(encs)
                    hs = (C.c_void_p * n)(*[e.h for e in encs])
                    ptrs = (C.c_void_p * n)(*[e.next_input_ptr() for e in encs])
                    assert encs[0].lib.thor_enc_frames_begin(hs, n, ptrs, None) == L.THOR_ERR_ARG
            for k, ch in enumerate(encode_batch_end(encs)):
                got[k].append(ch)
        for k in range(len(encs)):
            assert got[k] == want[:10], k
    finally:
        for e in encs:
            e.close()


def test_encoder_reset_recodes_the_sequence(streams):
    """thor_enc_reset: the context codes its sequence again, same .bit."""
    from thor_amd.encoder import GpuEncoder, params_for

    meta = streams["cif_low"]
    want = _frames(open("tests/golden/cif_low.bit", "rb").read())
    enc = GpuEncoder(params_for(meta["config"], meta["width"], meta["height"], 4, meta["extra"]))
    try:
        enc.upload_sequence(_input(meta, 4))
        first = [enc.encode_next() for _ in range(3)]
        enc.reset()
        again = [enc.encode_next() for _ in range(4)]
        assert first == want[:3] and again == want[:4]
    finally:
        enc.close()


def test_wpp_wait_gives_up_once_per_wave(streams):
    """A superblock row that never reports progress (thor_enc_debug_stall) ends
    the launch in bounded time with an error -- each wave gives up waiting at
    most once (a per-SB give-up would cost the 30 SBs of a 1080p row 30 wait
    periods) -- and the context has not advanced: the same frame then codes
    normally, byte-equal to the reference."""
    import time

    from thor_amd.encoder import GpuEncoder, params_for

    meta = streams["hd_low"]
    enc = GpuEncoder(params_for(meta["config"], meta["width"], meta["height"], 2, meta["extra"]))
    lib = enc.lib
    try:
        enc.upload_sequence(_input(meta, 2))
        want = _frames(open("tests/golden/hd_low.bit", "rb").read())
        lib.thor_enc_debug_stall(3, 500)
        t0 = time.time()
        with pytest.raises(RuntimeError):
            enc.encode_next()
        dt = time.time() - t0
        lib.thor_enc_debug_stall(-1, 0)
        assert dt < 6.0, dt  # one 0.5 s wait per stalled wave, not one per superblock
        assert enc.encode_next() == want[0]
    finally:
        lib.thor_enc_debug_stall(-1, 0)
        enc.close()


def test_pipelined_batches_with_interpolated_references(streams):
    """thor_enc_frames_begin / _end on a stream whose B frames interpolate a
    reference from frames the previous batch is still filtering (HDB16 coding
    order 0, 16, 8, ...: frame 8 interpolates from frame 16), two contexts --
    the second on its own stream, so its interpolation must wait for the
    pending batch -- byte-equal to the reference encoder."""
    from thor_amd.encoder import GpuEncoder, encode_batch_begin, encode_batch_end, params_for

    name = "cif_hdbi"
    meta = streams[name]
    nf = meta["frames"]
    want = _frames(open("tests/golden/%s.bit" % name, "rb").read())
    encs = []
    try:
        for _ in range(2):
            e = GpuEncoder(params_for(meta["config"], meta["width"], meta["height"], nf, meta["extra"]))
            e.upload_sequence(_input(meta, nf))
            encs.append(e)
        n = encs[0].num_frames()
        got = [[] for _ in encs]
        encode_batch_begin(encs)
        for i in range(n):
            if i + 1 < n:
                encode_batch_begin(encs)
            for k, ch in enumerate(encode_batch_end(encs)):
                got[k].append(ch)
        for k in range(len(encs)):
            assert got[k] == want[:n], k
    finally:
        for e in encs:
            e.close()


def test_concurrent_enc_frames_calls_on_one_device(streams):
    """thor_enc_frames from two threads at once (the GIL is released inside the
    call): each call's begin and end run under one hold of the device pool's
    lock, so neither thread's end meets the other's batch -- both
    sequences byte-equal to the reference."""
    import threading

    from thor_amd.encoder import GpuEncoder, encode_batch, params_for

    meta = streams["cif_low"]
    want = _frames(open("tests/golden/cif_low.bit", "rb").read())
    groups = []
    try:
        for _ in range(2):
            g = []
            for _ in range(2):
                e = GpuEncoder(params_for(meta["config"], meta["width"], meta["height"], 10, meta["extra"]))
                e.upload_sequence(_input(meta, 10))
                g.append(e)
            groups.append(g)
        res, errs = [[] for _ in groups], []

        def run(j):
            try:
                for _ in range(10):
                    res[j].append(encode_batch(groups[j]))
            except Exception as ex:  # pragma: no cover - reported below
                errs.append(repr(ex))

        ts = [threading.Thread(target=run, args=(j,)) for j in range(len(groups))]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=100)
        assert not errs, errs
        for j in range(len(groups)):
            assert len(res[j]) == 10
            for i in range(10):
                assert res[j][i] == [want[i]] * len(groups[j]), (j, i)
    finally:
        for g in groups:
            for e in g:
                e.close()


def test_encoder_frame_wider_than_256_superblocks():
    """A 16 448 x 64 frame (257 SB columns): the SB scheduler's queue items code
    the SB column in 11 bits (8 bits spilled into the row field past
    256 columns, so workers coded the wrong SB or waited until the spin limit).
    The I frame must code without a device error, and its reconstruction must
    equal the oracle decoder's reconstruction of the .bit it wrote."""
    import ctypes as C

    from oracle import OracleDecoder
    from thor_amd.bitstream import parse_stream
    from thor_amd.encoder import GpuEncoder, params_for

    W, H = 16448, 64
    p = params_for("config_LDB_low_complexity.txt", W, H, 1)
    enc = GpuEncoder(p)
    try:
        enc.upload_sequence(synth.synth_frames(W, H, 1, 5, workers=1))
        bits = enc.encode_next()
        y = np.empty(W * H, np.uint8)
        u = np.empty(W * H // 4, np.uint8)
        v = np.empty(W * H // 4, np.uint8)
        assert enc.lib.thor_enc_read_recon(enc.h, y.ctypes.data, u.ctypes.data, v.ctypes.data) == 0
    finally:
        enc.close()
    seq, frames = parse_stream(bits)
    assert len(frames) == 1 and seq.width == W
    (fr, cur), = list(OracleDecoder(seq).run(frames))
    assert cur.i420() == y.tobytes() + u.tobytes() + v.tobytes()

"""GPU parity of the encoder's sequence launch (thor_enc_seq_*, k_enc_seq in
thor_amd/csrc/enc_seq.hip): every frame of several streams in ONE persistent
launch -- RD loop, loop filters, CLPF, padding and packing as tasks of the SB
scheduler, frame f + 1 of a stream starting once its frame f is a finished
reference -- must give the reference Thorenc's bitstreams (tests/golden/<name>.bit)
byte for byte, for every stream of the launch, whatever the mix."""
import ctypes as C

import numpy as np
import pytest

from thor_amd import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _bounded_waits():
    """A wedged launch gives up after 20 s (reported as a device error) instead
    of the 5-minute default."""
    from thor_amd import lib as L

    lib = L.load()
    lib.thor_enc_debug_stall(-1, 20000)
    yield
    lib.thor_enc_debug_stall(-1, 0)


def _frames(b):
    out, o = [], 0
    while o < len(b):
        n = int.from_bytes(b[o:o + 4], "big")
        out.append(b[o:o + 4 + n])
        o += 4 + n
    return out


def _golden(name):
    return _frames(open("tests/golden/%s.bit" % name, "rb").read())


def _encoders(streams, names, nframes):
    from thor_amd.encoder import GpuEncoder, params_for

    encs = []
    for name in names:
        meta = streams[name]
        p = params_for(meta["config"], meta["width"], meta["height"], nframes, meta["extra"])
        e = GpuEncoder(p)
        e.upload_sequence(synth.synth_frames(meta["width"], meta["height"], nframes, meta["seed"], workers=1))
        encs.append(e)
    return encs


@pytest.mark.parametrize("names,nframes", [
    (["cif_low"] * 3, 10),          # three copies of one stream
    (["cif_low", "cif_med"], 10),   # two configurations in one launch
    (["cif_high"], 4),              # delta-QP trials, speed 0 search
    (["w8_low"], 6),                # frame width not a multiple of 64 (partial SB column)
    (["hd_low", "hd_low"], 17),     # 1080p: partial SB row (H = 1080), 16 P frames
    (["k4_low", "k4_med"], 8),      # 4K LDB low + medium, the bench's geometry
])
def test_sequence_launch_matches_reference(streams, names, nframes):
    from thor_amd.encoder import SeqLaunch

    encs = _encoders(streams, names, nframes)
    try:
        s = SeqLaunch(encs)
        st = s.end()
        assert st["tasks"] > 0
        ready = s.ready()
        assert (ready >= 0).all(), ready
        for i, name in enumerate(names):
            want = _golden(name)
            for f in range(s.nf):
                got = s.chunk(i, f)
                assert got == want[f], (name, i, f, len(got), len(want[f]))
            # the last frame is also the context's thor_enc_frame_bytes chunk
            assert encs[i].chunk() == want[s.nf - 1]
    finally:
        for e in encs:
            e.close()


def test_sequence_launch_fetches_host_frames(streams):
    """Fetch mode: the launch copies each frame from page-locked host memory
    into HBM itself (FETCH tasks, one frame ahead of the RD loop); frames become
    final (thor_enc_seq_ready) while it runs, and the .bit is the reference's.
    (Page-locked memory from the HIP runtime the library uses, not torch's.)"""
    import time

    from thor_amd.encoder import GpuEncoder, SeqLaunch, params_for

    name, nframes, n = "k4_low", 8, 3
    meta = streams[name]
    W, H = meta["width"], meta["height"]
    fsize = W * H * 3 // 2
    frames = np.ascontiguousarray(synth.synth_frames(W, H, nframes, meta["seed"], workers=1)).reshape(nframes, fsize)
    hip = C.CDLL("libamdhip64.so")
    hip.hipHostMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
    hip.hipHostFree.argtypes = [C.c_void_p]
    pinned = C.c_void_p()
    assert hip.hipHostMalloc(C.byref(pinned), frames.nbytes, 0) == 0
    encs, devs = [], []
    try:
        C.memmove(pinned.value, frames.ctypes.data, frames.nbytes)
        for i in range(n):
            e = GpuEncoder(params_for(meta["config"], W, H, nframes, meta["extra"]))
            d = e.lib.thor_dev_alloc(frames.nbytes)
            assert d
            devs.append(d)
            e.use_device_sequence(d, nframes)
            encs.append(e)
        s = SeqLaunch(encs, host=lambda i, k: pinned.value + k * fsize)
        seen, t0 = 0, time.time()
        while seen < n * nframes and time.time() - t0 < 60:  # (a failed launch gives up after 20 s)
            seen = max(seen, int((s.ready() >= 0).sum()))
            time.sleep(0.001)
        s.end()
        assert seen == n * nframes
        want = _golden(name)
        back = np.empty_like(frames)
        for i in range(n):
            for f in range(nframes):
                assert s.chunk(i, f) == want[f], (i, f)
            assert encs[i].lib.thor_d2h(back.ctypes.data, devs[i], back.nbytes) == 0
            assert np.array_equal(back, frames), i  # the fetched inputs are the host frames
    finally:
        for e in encs:
            e.close()
        for d in devs:
            encs[0].lib.thor_dev_free(d)
        hip.hipHostFree(pinned)


def test_sequence_launch_then_frame_batches(streams):
    """A context coded part-way by a sequence launch continues with the
    per-frame batch (thor_enc_frames) and the other way round: the reference
    window, slots and cell state carry over."""
    from thor_amd.encoder import SeqLaunch, encode_batch

    name, nframes = "cif_med", 10
    encs = _encoders(streams, [name, name], nframes)
    want = _golden(name)
    try:
        got = [[], []]
        for f in range(3):  # frames 0-2 per frame
            for i, ch in enumerate(encode_batch(encs)):
                got[i].append(ch)
        s = SeqLaunch(encs, 4)  # frames 3-6 in one launch
        s.end()
        for i in range(2):
            got[i] += [s.chunk(i, f) for f in range(4)]
        for f in range(3):  # frames 7-9 per frame
            for i, ch in enumerate(encode_batch(encs)):
                got[i].append(ch)
        for i in range(2):
            assert got[i] == want[:nframes], i
    finally:
        for e in encs:
            e.close()


def test_sequence_launch_refusals(streams):
    """Interpolated-reference contexts are refused (thor_enc_frames codes
    them), and so is a second launch while one is in flight."""
    from thor_amd.encoder import GpuEncoder, SeqLaunch, params_for

    meta = streams["cif_hdbi"]
    e = GpuEncoder(params_for(meta["config"], meta["width"], meta["height"], 3, meta["extra"]))
    try:
        e.upload_sequence(synth.synth_frames(meta["width"], meta["height"], 3, meta["seed"], workers=1))
        hs = (C.c_void_p * 1)(e.h)
        ins = (C.c_void_p * 3)(*[e.seq_dev] * 3)
        assert e.lib.thor_enc_seq_begin(hs, 1, 3, ins, None, 0, 0) == -1
    finally:
        e.close()
    encs = _encoders(streams, ["cif_low"], 4)
    other = _encoders(streams, ["cif_low"], 4)
    try:
        s = SeqLaunch(encs)
        hs = (C.c_void_p * 1)(other[0].h)
        ins = (C.c_void_p * 4)(*[other[0].seq_dev] * 4)
        assert other[0].lib.thor_enc_seq_begin(hs, 1, 4, ins, None, 0, 0) == -1
        s.end()
        assert s.chunk(0, 3) == _golden("cif_low")[3]
    finally:
        for e in encs + other:
            e.close()

"""GPU parity of the device-resident encoder (thor_enc_*, k_enc_rows): the
reference encoder's own bitstreams (tests/golden/<name>.bit, written by the
reference Thorenc from the seeded synthetic clips) must come out byte for
byte, frame by frame."""
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


def _input(meta, n):
    w, h = meta["width"], meta["height"]
    return np.stack([np.concatenate([p.reshape(-1) for p in synth.synth_frame(w, h, t, meta["seed"])])
                     for t in range(n)])


@pytest.mark.parametrize("name,nframes", [("cif_low", 10), ("w8_low", 6), ("cif_med", 10), ("hd_low", 17)])
def test_device_encoder_matches_reference_bitstream(name, nframes, streams):
    from thor_amd.encoder import GpuEncoder, params_for

    meta = streams[name]
    p = params_for(meta["config"], meta["width"], meta["height"], nframes, meta["extra"])
    enc = GpuEncoder(p)
    try:
        enc.upload_sequence(_input(meta, nframes))
        want = _frames(open("tests/golden/%s.bit" % name, "rb").read())
        for i in range(enc.num_frames()):
            got = enc.encode_next()
            assert got == want[i], (name, i, len(got), len(want[i]))
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

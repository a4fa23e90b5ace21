"""The CPU oracle (oracle/thor_oracle.c) replays every committed reference
trace and must reproduce the reference decoder's frame at each stage
(pre-deblock, post-deblock, final) bit-exactly: this pins the oracle to the
reference (tests/golden/streams.json, written by tools/make_goldens.py)."""
import hashlib

import pytest

from conftest import trace_path
from oracle import OracleDecoder
from thor_amd.trace import load_trace

STREAMS = ["cif_low", "cif_med", "cif_high", "cif_hdb", "hd_low", "k4_low", "k4_med", "w8_low"]


@pytest.mark.parametrize("name", STREAMS)
def test_oracle_matches_reference_final(name, streams):
    meta = streams[name]
    seq, frames = load_trace(trace_path(name))
    assert (seq.width, seq.height) == (meta["width"], meta["height"])
    dec = OracleDecoder(seq)
    out = {}
    for fr, cur in dec.run(frames):
        assert hashlib.md5(cur.i420()).hexdigest() == meta["stage_md5"][fr.decode_order]["final"], fr.decode_order
        out[fr.frame_num] = cur.i420()
    # decoded .yuv is written in display order (dec/maindec.c:176-195)
    yuv = b"".join(out[k] for k in sorted(out))
    assert hashlib.md5(yuv).hexdigest() == meta["dec_md5"]


@pytest.mark.parametrize("name", ["cif_low", "cif_high", "cif_hdb"])
def test_oracle_matches_reference_stages(name, streams):
    meta = streams[name]
    seq, frames = load_trace(trace_path(name))
    dec = OracleDecoder(seq)
    for fr in frames:
        for stage, key in ((0, "pre_deblock"), (1, "post_deblock")):
            cur = dec.decode(fr, stage)
            assert hashlib.md5(cur.i420()).hexdigest() == meta["stage_md5"][fr.decode_order][key], (fr.decode_order, key)
        dec.push_reference(dec.decode(fr, 2))


@pytest.mark.parametrize("name", ["cif_hdbi", "cif_hdbi_high"])
def test_oracle_interp_ref_streams(name, streams):
    """Streams with temporal-interpolated references (-interp_ref 1): the frames
    come from the .bit through the host parser (which carries the interpolation
    header of dec/decode_frame.c:91-109; the parse itself is pinned to the
    reference's traces by tests/test_parser.py), the oracle builds each
    interpolated reference (oracle/thor_oracle_ti.c) and must reproduce the
    reference decoder at every stage."""
    import os

    from conftest import GOLD
    from thor_amd.bitstream import parse_stream

    meta = streams[name]
    seq, frames = parse_stream(open(os.path.join(GOLD, name + ".bit"), "rb").read())
    assert seq.interp_ref == 1 and any(f.interp_ratio for f in frames)
    dec = OracleDecoder(seq)
    out = {}
    for fr in frames:
        for stage, key in ((0, "pre_deblock"), (1, "post_deblock")):
            cur = dec.decode(fr, stage)
            assert hashlib.md5(cur.i420()).hexdigest() == meta["stage_md5"][fr.decode_order][key], (fr.decode_order, key)
        cur = dec.decode(fr, 2)
        assert hashlib.md5(cur.i420()).hexdigest() == meta["stage_md5"][fr.decode_order]["final"], fr.decode_order
        out[fr.frame_num] = cur.i420()
        dec.push_reference(cur)
    yuv = b"".join(out[k] for k in sorted(out))
    assert hashlib.md5(yuv).hexdigest() == meta["dec_md5"]

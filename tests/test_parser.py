"""The host .bit parser (thor_parse_frame, parse.hip) against the reference
decoder's own parse output: every committed reference bitstream must parse to
exactly the descriptors, coefficient pool and CLPF flags the reference
decoder's read_block produced (the committed traces, recorded through
oracle/ref_hooks/trace_dec.c).  CPU only: the parser is host code."""
import numpy as np
import pytest

from conftest import GOLD, trace_path
from thor_amd.trace import load_trace

STREAMS = ["cif_low", "cif_med", "cif_high", "cif_hdb", "hd_low", "k4_low", "k4_med", "w8_low", "hd_high", "cif_hdbi",
           "cif_hdbi_high", "k4_hdbi", "k4_hdbi_high"]
# fields the reference sets for every mode (pb_part / intra_mode only for
# INTER / INTRA: read_block leaves them stale otherwise, dec/read_bits.c:380, :582)
COMMON = ["ypos", "xpos", "size", "bwidth", "bheight", "mode", "tb_split", "dir", "qp", "cbp_y", "cbp_u", "cbp_v",
          "coeff_mask", "mv0", "mv1", "ref0", "ref1", "coeff_off"]


@pytest.mark.parametrize("name", STREAMS)
def test_parser_matches_reference_trace(name):
    import os

    from thor_amd.bitstream import parse_stream

    data = open(os.path.join(GOLD, name + ".bit"), "rb").read()
    seq, got = parse_stream(data)
    tseq, want = load_trace(trace_path(name))
    assert (seq.width, seq.height, seq.bipred, seq.deblocking, seq.clpf) == \
        (tseq.width, tseq.height, tseq.bipred, tseq.deblocking, tseq.clpf)
    assert len(got) == len(want)
    for g, w in zip(got, want):
        assert (g.frame_num, g.frame_type, g.qp, g.num_ref, g.clpf_on) == \
            (w.frame_num, w.frame_type, w.qp, w.num_ref, w.clpf_on), (name, w.decode_order)
        assert len(g.blocks) == len(w.blocks), (name, w.decode_order)
        for f in COMMON:
            bad = np.nonzero(np.any((g.blocks[f] != w.blocks[f]).reshape(len(w.blocks), -1), axis=1))[0]
            assert bad.size == 0, (name, w.decode_order, f, bad[:5])
        inter = w.blocks["mode"] == 2
        assert np.array_equal(g.blocks["pb_part"][inter], w.blocks["pb_part"][inter])
        intra = w.blocks["mode"] == 1
        assert np.array_equal(g.blocks["intra_mode"][intra], w.blocks["intra_mode"][intra])
        assert np.array_equal(g.coeffs, w.coeffs), (name, w.decode_order)
        if w.clpf_on:
            assert np.array_equal(g.clpf_flags, w.clpf_flags), (name, w.decode_order)


def test_parser_rejects_garbage():
    from thor_amd.bitstream import Parser

    p = Parser()
    try:
        with pytest.raises(ValueError):
            p.parse(b"\x00\x01")  # a zero-sized frame: width 0 in the sequence header
    finally:
        p.close()

"""The .bit container and the parse side of decoding.

A Thor .bit is a sequence of frame chunks: a 4-byte big-endian payload length
then the payload (enc/putbits.c:57-95, dec/getbits.c:48-69); the first payload
starts with the 44-bit sequence header.  `parse_stream` runs the library's
host parser (thor_parse_frame, parse.hip) over every chunk and yields
thor_amd.trace.Frame records -- the same descriptors the GPU decoder replays."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import lib as L
from .trace import BLOCK_DTYPE, Frame, SeqParams


def split_chunks(data: bytes):
    out, o = [], 0
    while o + 4 <= len(data):
        n = int.from_bytes(data[o:o + 4], "big")
        out.append(data[o + 4:o + 4 + n])
        o += 4 + n
    return out


class Parser:
    def __init__(self):
        self.lib = L.load()
        self.h = self.lib.thor_parser_create()

    def close(self):
        if self.h:
            self.lib.thor_parser_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def parse(self, payload: bytes) -> Frame:
        out = L.ThorParsedFrame()
        buf = C.create_string_buffer(payload, len(payload))
        rc = self.lib.thor_parse_frame(self.h, buf, len(payload), C.byref(out))
        if rc != 0:
            raise ValueError("thor_parse_frame failed (%d)" % rc)
        nb = out.nblocks
        blocks = np.frombuffer((C.c_uint8 * (nb * BLOCK_DTYPE.itemsize)).from_address(out.blocks),
                               BLOCK_DTYPE).copy() if nb else np.zeros(0, BLOCK_DTYPE)
        nc = out.ncoeffs
        coeffs = np.frombuffer((C.c_int16 * nc).from_address(out.coeffs), np.int16).copy() if nc else \
            np.zeros(0, np.int16)
        ncl = out.nclpf
        clpf = np.frombuffer((C.c_uint8 * ncl).from_address(out.clpf_flags), np.uint8).copy() if ncl else \
            np.zeros(0, np.uint8)
        h = out.hdr
        return Frame(out.decode_order, h.frame_num, h.frame_type, h.qp, out.num_ref, h.clpf_on, blocks, coeffs,
                     clpf if h.clpf_on else np.zeros(0, np.uint8), (h.interp_ref[0], h.interp_ref[1]),
                     h.interp_ratio, h.interp_pos)

    def seq(self) -> L.ThorSeq:
        s = L.ThorSeq()
        L.check(self.lib.thor_parser_seq(self.h, C.byref(s)), "thor_parser_seq")
        return s


def parse_stream(data: bytes):
    """(SeqParams-like thor_seq_t, [Frame]) of a whole .bit."""
    p = Parser()
    try:
        frames = [p.parse(c) for c in split_chunks(data)]
        s = p.seq()
        seq = SeqParams(s.width, s.height, 0, s.tb_split_enable, 0, s.interp_ref, 0, s.deblocking, s.clpf, 0, s.bipred)
        return seq, frames
    finally:
        p.close()

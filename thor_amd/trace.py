"""Per-frame block-descriptor traces: the parse-side output the GPU path replays.

A trace is what Thor's serial bit parser hands to reconstruction for each frame:
the frame header (dec/decode_frame.c:58-78), then, in decode order, one record per
decoded CU as `read_block` (dec/read_bits.c:221) leaves it in `block_info_dec_t`
(dec/maindec.h:47-57), plus the per-SB CLPF decisions read at
dec/decode_frame.c:130-133.  Traces are recorded from the reference decoder by
oracle/ref_hooks/trace_dec.c (test infrastructure) and committed as fixtures;
the product consumes them as plain descriptor arrays (include/thor_amd.h).

On-disk layout (little endian):
  "THTR" u32 version=1 u16 width u16 height u8 seq[12]
  repeated: "FRME" i32 decode_order i32 frame_num u8 frame_type u8 qp u8 num_ref
            u8 clpf_on u32 nblocks u32 nbytes u32 nclpf  <nbytes of blocks> <nclpf u8>
  block:    u16 ypos u16 xpos u8 size bwidth bheight mode intra_mode tb_split pb_part
            dir qp cbp_y cbp_u cbp_v coeff_mask pad[3]  i16 mv0[8] i16 mv1[8]
            i32 ref_frame0 i32 ref_frame1  [i16 Y size^2] [i16 U (size/2)^2] [i16 V ...]
Files may be zlib-compressed (suffix .z).
"""
from __future__ import annotations

import struct
import zlib
from dataclasses import dataclass, field

import numpy as np

# block_mode_t (common/types.h:83-90)
MODE_SKIP, MODE_INTRA, MODE_INTER, MODE_BIPRED, MODE_MERGE = 0, 1, 2, 3, 4
# frame_type_t (common/types.h:76-81)
I_FRAME, P_FRAME, B_FRAME = 0, 1, 2

# Descriptor record shared with the C-ABI (include/thor_amd.h: thor_block_t, 72 bytes)
BLOCK_DTYPE = np.dtype(
    [
        ("ypos", "<u2"), ("xpos", "<u2"),
        ("size", "u1"), ("bwidth", "u1"), ("bheight", "u1"), ("mode", "u1"),
        ("intra_mode", "u1"), ("tb_split", "u1"), ("pb_part", "u1"), ("dir", "u1"),
        ("qp", "u1"), ("cbp_y", "u1"), ("cbp_u", "u1"), ("cbp_v", "u1"),
        ("coeff_mask", "u1"), ("rsv", "u1", (3,)),
        ("mv0", "<i2", (8,)), ("mv1", "<i2", (8,)),
        ("ref0", "<i4"), ("ref1", "<i4"),
        ("coeff_off", "<u4", (3,)),
    ]
)
assert BLOCK_DTYPE.itemsize == 72


@dataclass
class SeqParams:
    width: int
    height: int
    pb_split: int
    tb_split_enable: int
    max_num_ref: int
    interp_ref: int
    max_delta_qp: int
    deblocking: int
    clpf: int
    use_block_contexts: int
    bipred: int


@dataclass
class Frame:
    decode_order: int
    frame_num: int
    frame_type: int
    qp: int
    num_ref: int
    clpf_on: int
    blocks: np.ndarray  # BLOCK_DTYPE
    coeffs: np.ndarray  # int16 compact coefficient pool
    clpf_flags: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint8))
    # temporal-interpolated reference (dec/decode_frame.c:91-109): the frame numbers of the
    # two interpolated references and interpolate_frames' (ratio, pos); ratio 0 = none
    interp_refs: tuple = (-1, -1)
    interp_ratio: int = 0
    interp_pos: int = 0

    def hdr_fields(self):
        """thor_frame_hdr_t's fields in order."""
        return (self.frame_num, self.frame_type, self.qp, self.clpf_on, self.interp_refs, self.interp_ratio,
                self.interp_pos)


def tu_layout(size: int, tb_split: int):
    """Compact coefficient-slot layout of one component of a CU.

    Only the low-frequency min(N,16)^2 corner of an NxN TU can be non-zero
    (forward transform common/transform.c:309-327 and quantize
    enc/encode_block.c:80-88 touch nothing else), so the pool keeps exactly
    those slots: one qsize^2 tile per TU, the four tb-split quarters
    consecutive in raster order (dec/decode_block.c:64-72,96-106).
    Returns (tu_size, n_tus, qsize)."""
    if tb_split:
        n = size // 2
        return n, 4, min(n, 16)
    return size, 1, min(size, 16)


def compact_coeffs(full: np.ndarray, size: int, tb_split: int) -> np.ndarray:
    """NxN reference layout (quarters consecutive when tb-split) -> compact slots."""
    n, ntu, q = tu_layout(size, tb_split)
    out = []
    for t in range(ntu):
        tu = full[t * n * n:(t + 1) * n * n].reshape(n, n)
        if np.any(tu[q:, :]) or np.any(tu[:, q:]):
            raise ValueError("non-zero coefficient outside the low-frequency corner")
        out.append(tu[:q, :q].reshape(-1))
    return np.concatenate(out)


def expand_coeffs(comp: np.ndarray, size: int, tb_split: int) -> np.ndarray:
    """Compact slots -> NxN reference layout."""
    n, ntu, q = tu_layout(size, tb_split)
    full = np.zeros(ntu * n * n, np.int16)
    for t in range(ntu):
        tu = np.zeros((n, n), np.int16)
        tu[:q, :q] = comp[t * q * q:(t + 1) * q * q].reshape(q, q)
        full[t * n * n:(t + 1) * n * n] = tu.reshape(-1)
    return full


def chroma_tb_split(size: int, tb_split: int) -> int:
    # dec/decode_block.c:449-450: chroma splits only when size > 8
    return int(bool(tb_split) and size > 8)


def _parse_frame(buf: memoryview, off: int, seq: SeqParams):
    if bytes(buf[off:off + 4]) != b"FRME":
        raise ValueError("bad frame magic at %d" % off)
    decode_order, frame_num = struct.unpack_from("<ii", buf, off + 4)
    ftype, qp, num_ref, clpf_on = struct.unpack_from("<BBBB", buf, off + 12)
    nblocks, nbytes, nclpf = struct.unpack_from("<III", buf, off + 16)
    p = off + 28
    end = p + nbytes
    blocks = np.zeros(nblocks, BLOCK_DTYPE)
    pool = []
    pool_len = 0
    for b in range(nblocks):
        (ypos, xpos, size, bw, bh, mode, imode, tbs, pbp, dr, bqp, cy, cu, cv, mask) = struct.unpack_from(
            "<HHBBBBBBBBBBBBB", buf, p)
        p += 20
        mvs = np.frombuffer(buf, "<i2", 16, p)
        p += 32
        r0, r1 = struct.unpack_from("<ii", buf, p)
        p += 8
        rec = blocks[b]
        rec["ypos"], rec["xpos"], rec["size"], rec["bwidth"], rec["bheight"] = ypos, xpos, size, bw, bh
        rec["mode"], rec["intra_mode"], rec["tb_split"], rec["pb_part"], rec["dir"] = mode, imode, tbs, pbp, dr
        rec["qp"], rec["cbp_y"], rec["cbp_u"], rec["cbp_v"] = bqp, cy, cu, cv
        rec["mv0"] = mvs[:8]
        rec["mv1"] = mvs[8:]
        rec["ref0"], rec["ref1"] = r0, r1
        offs = [0, 0, 0]
        cmask = 0
        for c in range(3):
            n = size if c == 0 else size // 2
            if mask & (1 << c):
                full = np.frombuffer(buf, "<i2", n * n, p).copy()
                p += 2 * n * n
                tbc = tbs if c == 0 else chroma_tb_split(size, tbs)
                comp = compact_coeffs(full, n, tbc)
                offs[c] = pool_len
                pool.append(comp)
                pool_len += comp.size
                cmask |= 1 << c
        rec["coeff_mask"] = cmask
        rec["coeff_off"] = offs
    if p != end:
        raise ValueError("block section length mismatch")
    flags = np.frombuffer(buf, np.uint8, nclpf, end).copy() if nclpf else np.zeros(0, np.uint8)
    coeffs = np.concatenate(pool).astype(np.int16) if pool else np.zeros(0, np.int16)
    fr = Frame(decode_order, frame_num, ftype, qp, num_ref, clpf_on, blocks, coeffs, flags)
    return fr, end + nclpf


def load_trace(path: str):
    with open(path, "rb") as f:
        data = f.read()
    if path.endswith(".z"):
        data = zlib.decompress(data)
    buf = memoryview(data)
    if bytes(buf[:4]) != b"THTR":
        raise ValueError("not a Thor trace")
    (version,) = struct.unpack_from("<I", buf, 4)
    if version != 1:
        raise ValueError("unsupported trace version %d" % version)
    w, h = struct.unpack_from("<HH", buf, 8)
    s = struct.unpack_from("<12B", buf, 12)
    seq = SeqParams(w, h, *s[:9])
    frames = []
    off = 24
    while off < len(buf):
        fr, off = _parse_frame(buf, off, seq)
        frames.append(fr)
    return seq, frames

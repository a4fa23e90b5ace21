"""TEST INFRASTRUCTURE ONLY -- ctypes binding of liboracle.so + a frame-replay
driver that restates the reference decoder's frame loop (dec/decode_frame.c:45-148,
dec/maindec.c:167-186) on CPU: reconstruct each frame from its descriptors,
deblock, CLPF, then keep it as a padded reference (create_reference_frame,
common/common_frame.c:464-483) in a sliding window of MAX_REF_FRAMES = 33
(common/global.h:69)."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PAD_Y, PAD_C = 96, 48  # PADDING_Y (common/global.h:63), chroma PADDING_Y/2 (dec/maindec.c:157)
MAX_REF_FRAMES = 33

_lib = None


def plane_stride(width: int, pad: int) -> int:
    # create_yuv_frame, common/common_frame.c:331-332
    return (width + 2 * pad + 15) & ~15


class ThorSeq(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("bipred", C.c_int32), ("deblocking", C.c_int32),
                ("clpf", C.c_int32), ("tb_split_enable", C.c_int32), ("interp_ref", C.c_int32)]


class ThorFrameHdr(C.Structure):
    _fields_ = [("frame_num", C.c_int32), ("frame_type", C.c_int32), ("qp", C.c_int32), ("clpf_on", C.c_int32),
                ("interp_ref", C.c_int32 * 2), ("interp_ratio", C.c_int32), ("interp_pos", C.c_int32)]


class OrFrame(C.Structure):
    _fields_ = [("y", C.c_void_p), ("u", C.c_void_p), ("v", C.c_void_p), ("stride_y", C.c_int),
                ("stride_c", C.c_int), ("frame_num", C.c_int)]


def load(build: bool = True):
    global _lib
    if _lib is not None:
        return _lib
    path = os.path.join(HERE, "liboracle.so")
    srcs = ("thor_oracle.c", "thor_oracle_ti.c", "thor_oracle.h")
    if build and (not os.path.exists(path) or
                  os.path.getmtime(path) < max(os.path.getmtime(os.path.join(HERE, f)) for f in srcs)):
        subprocess.run(["make", "-s", "-C", HERE, "liboracle.so"], check=True)
    _lib = C.CDLL(path)
    P = C.c_void_p
    i = C.c_int
    _lib.or_mc_luma.argtypes = [P, i, P, i, i, i, i, i, i, i]
    _lib.or_mc_chroma.argtypes = [P, i, P, i, i, i, i, i, i]
    _lib.or_dequantize.argtypes = [P, P, i, i]
    _lib.or_inverse_transform.argtypes = [P, P, i]
    _lib.or_transform.argtypes = [P, P, i, i]
    _lib.or_encode_tu.argtypes = [P, i, P, i, P, i, i, i, i, i, P, P]
    _lib.or_encode_tu.restype = i
    _lib.or_quantize.argtypes = [P, P, i, i, i]
    _lib.or_quantize.restype = i
    _lib.or_reconstruct_block.argtypes = [P, P, P, i, i]
    _lib.or_make_top_and_left.argtypes = [P, P, P, P, i, P, i, i, i, i, i, i, i, i, i]
    _lib.or_intra_pred.argtypes = [P, P, C.c_uint8, i, i, i, P, i]
    _lib.or_upright_available.argtypes = [i, i, i, i]
    _lib.or_downleft_available.argtypes = [i, i, i, i]
    _lib.or_clpf_block.argtypes = [P, P, i, i, i, i, i, i, i]
    _lib.or_sad.argtypes = [P, P, i, i, i, i]
    _lib.or_sad.restype = C.c_uint32
    _lib.or_ssd.argtypes = [P, P, i, i, i, i]
    _lib.or_ssd.restype = C.c_uint32
    _lib.or_decode_frame.argtypes = [C.POINTER(ThorSeq), C.POINTER(ThorFrameHdr), C.POINTER(OrFrame),
                                     C.POINTER(OrFrame), i, P, i, P, P, i]
    _lib.or_decode_frame.restype = i
    _lib.or_pad_frame.argtypes = [C.POINTER(OrFrame), i, i, i, i]
    _lib.or_scale_down2x2.argtypes = [P, i, P, i, i, i]
    _lib.or_pad_plane.argtypes = [P, i, i, i, i]
    _lib.or_interp_comp.argtypes = [P, i, P, i, P, i, P, P] + [i] * 9
    _lib.or_ti_levels.argtypes = [i, i]
    _lib.or_ti_levels.restype = i
    _lib.or_interpolate_frames.argtypes = [C.POINTER(OrFrame), C.POINTER(OrFrame), i, C.POINTER(OrFrame), i, i, i, i,
                                           P, P]
    _lib.or_interpolate_frames.restype = i
    return _lib


def lib():
    return load()


def ptr(a: np.ndarray) -> int:
    return a.ctypes.data


class PaddedFrame:
    """A padded I420 frame (pad 96 / 48) held as three numpy planes."""

    def __init__(self, width: int, height: int):
        self.w, self.h = width, height
        self.sy, self.sc = plane_stride(width, PAD_Y), plane_stride(width // 2, PAD_C)
        self.Y = np.zeros((height + 2 * PAD_Y) * self.sy + 64, np.uint8)
        self.U = np.zeros((height // 2 + 2 * PAD_C) * self.sc + 64, np.uint8)
        self.V = np.zeros_like(self.U)
        self.oy = PAD_Y * self.sy + PAD_Y
        self.oc = PAD_C * self.sc + PAD_C
        self.frame_num = -1

    def c(self) -> OrFrame:
        return OrFrame(ptr(self.Y) + self.oy, ptr(self.U) + self.oc, ptr(self.V) + self.oc, self.sy, self.sc,
                       self.frame_num)

    def planes(self):
        """Unpadded (Y, U, V) views."""
        y = self.Y[self.oy:self.oy + self.h * self.sy].reshape(self.h, self.sy)[:, :self.w]
        u = self.U[self.oc:self.oc + (self.h // 2) * self.sc].reshape(self.h // 2, self.sc)[:, :self.w // 2]
        v = self.V[self.oc:self.oc + (self.h // 2) * self.sc].reshape(self.h // 2, self.sc)[:, :self.w // 2]
        return y, u, v

    def i420(self) -> bytes:
        return b"".join(np.ascontiguousarray(p).tobytes() for p in self.planes())


def ti_block_grid(width: int, height: int, level: int):
    """alloc_mv_data's (bw, bh) at a pyramid level (common/temporal_interp.c:97-99)."""
    w, h = width >> level, height >> level
    return 2 * ((w + 15) // 16), 2 * ((h + 15) // 16)


def interpolate_frames(ref0: "PaddedFrame", ref1: "PaddedFrame", ratio: int, pos: int, levels: bool = False):
    """The oracle's interpolate_frames (thor_oracle_ti.c): the interpolated frame,
    padded (pad_yuv_frame, dec/decode_frame.c:107); with levels=True also the
    final (mv0, mv1) block-vector fields of every level, level 0 first."""
    L = load()
    w, h = ref0.w, ref0.h
    out = PaddedFrame(w, h)
    nl = L.or_ti_levels(w, h)
    fields = []
    p0 = (C.c_void_p * 4)()
    p1 = (C.c_void_p * 4)()
    for lv in range(max(nl, 0)):
        bw, bh = ti_block_grid(w, h, lv)
        f0, f1 = np.zeros((bh, bw, 2), np.int16), np.zeros((bh, bw, 2), np.int16)
        fields.append((f0, f1))
        p0[lv], p1[lv] = ptr(f0), ptr(f1)
    a, b, o = ref0.c(), ref1.c(), out.c()
    rc = L.or_interpolate_frames(C.byref(a), C.byref(b), PAD_Y, C.byref(o), w, h, ratio, pos,
                                 C.cast(p0, C.c_void_p), C.cast(p1, C.c_void_p))
    if rc != 0:
        raise RuntimeError("or_interpolate_frames failed: %d" % rc)
    L.or_pad_frame(C.byref(o), w, h, PAD_Y, PAD_C)
    return (out, fields) if levels else out


def padded_from_planes(y, u, v, frame_num: int = -1) -> "PaddedFrame":
    f = PaddedFrame(y.shape[1], y.shape[0])
    fy, fu, fv = f.planes()
    fy[:], fu[:], fv[:] = y, u, v
    f.frame_num = frame_num
    c = f.c()
    load().or_pad_frame(C.byref(c), f.w, f.h, PAD_Y, PAD_C)
    return f


class OracleDecoder:
    """Replays descriptor traces through the oracle, frame by frame."""

    def __init__(self, seq):
        self.lib = load()
        self.seq = seq
        self.cseq = ThorSeq(seq.width, seq.height, seq.bipred, seq.deblocking, seq.clpf, seq.tb_split_enable,
                            getattr(seq, "interp_ref", 0))
        self.refs: list[PaddedFrame] = []  # newest first, like decoder_info->ref[]

    def decode(self, fr, stop_stage: int = 2) -> PaddedFrame:
        cur = PaddedFrame(self.seq.width, self.seq.height)
        cur.frame_num = fr.frame_num
        ratio = getattr(fr, "interp_ratio", 0)
        refs = list(self.refs)
        if ratio > 0:  # the temporal-interpolated reference, named -2 by the blocks (dec/decode_frame.c:91-109)
            ra = [r for r in self.refs if r.frame_num == fr.interp_refs[0]]
            rb = [r for r in self.refs if r.frame_num == fr.interp_refs[1]]
            if not ra or not rb:
                raise RuntimeError("interpolated reference from a frame that is not resident")
            it = interpolate_frames(ra[0], rb[0], ratio, fr.interp_pos)
            it.frame_num = -2
            refs.append(it)
            self.last_interp = it
        hdr = ThorFrameHdr(fr.frame_num, fr.frame_type, fr.qp, fr.clpf_on,
                           (C.c_int32 * 2)(*getattr(fr, "interp_refs", (-1, -1))), ratio, getattr(fr, "interp_pos", 0))
        nref = len(refs)
        arr = (OrFrame * max(1, nref))(*[r.c() for r in refs])
        blocks = np.ascontiguousarray(fr.blocks)
        coeffs = np.ascontiguousarray(fr.coeffs) if fr.coeffs.size else np.zeros(1, np.int16)
        flags = np.ascontiguousarray(fr.clpf_flags) if fr.clpf_flags.size else np.zeros(1, np.uint8)
        cf = cur.c()
        rc = self.lib.or_decode_frame(C.byref(self.cseq), C.byref(hdr), C.byref(cf), arr, nref, ptr(blocks),
                                      len(blocks), ptr(coeffs), ptr(flags), stop_stage)
        if rc != 0:
            raise RuntimeError("or_decode_frame failed: %d" % rc)
        return cur

    def push_reference(self, cur: PaddedFrame):
        self.lib.or_pad_frame(C.byref(cur.c()), self.seq.width, self.seq.height, PAD_Y, PAD_C)
        self.refs.insert(0, cur)
        del self.refs[MAX_REF_FRAMES:]

    def run(self, frames, stop_stage: int = 2):
        """Decode every frame; yields (frame, PaddedFrame) in decode order."""
        for fr in frames:
            cur = self.decode(fr, stop_stage)
            yield fr, cur
            if stop_stage < 2:  # keep the reference chain exact: redo at full stage
                cur = self.decode(fr, 2)
            self.push_reference(cur)

"""Batched GPU decode driver: the restated frame loop of the reference decoder
(dec/maindec.c:167-186 -> dec/decode_frame.c:45-148) over parse-side
descriptors, with every reconstruction stage on the GPU through the C-ABI.

Typical use (a trace stands in for the serial CPU parser):

    seq, frames = trace.load_trace("stream.trc.z")
    dec = GpuDecoder(seq)
    dev = [dec.upload(fr) for fr in frames]     # inputs resident in HBM
    for d in dev: dec.decode(d)                 # enqueue, no host sync
    y, u, v = dec.read(frames[-1].frame_num)
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import lib as L
from .trace import BLOCK_DTYPE

# thor_tu_t (include/thor_amd.h): one coded transform block, 12 bytes
TU_DTYPE = np.dtype([("coeff_off", "<u4"), ("y", "<u2"), ("x", "<u2"), ("size", "u1"), ("comp", "u1"), ("qp", "u1"),
                     ("rsv", "u1")])


@dataclass
class DeviceFrame:
    hdr: L.ThorFrameHdr
    blocks: int  # device pointers
    nblocks: int
    coeffs: int
    clpf: int
    intra: int
    n_intra: int
    tus: int
    n_tu: int
    clpfl: int
    n_clpf: int
    slow: int
    n_slow: int
    nbytes: int  # bytes uploaded (descriptors + coefficients + flags + list)


class DeviceBuffer:
    def __init__(self, lib, nbytes: int):
        self.lib = lib
        self.nbytes = max(int(nbytes), 16)
        self.ptr = lib.thor_dev_alloc(self.nbytes)
        if not self.ptr:
            raise MemoryError("thor_dev_alloc(%d) failed" % self.nbytes)

    def upload(self, arr: np.ndarray):
        a = np.ascontiguousarray(arr)
        if a.nbytes:
            L.check(self.lib.thor_h2d(self.ptr, a.ctypes.data, a.nbytes), "thor_h2d")

    def free(self):
        if self.ptr:
            self.lib.thor_dev_free(self.ptr)
            self.ptr = None


MAX_SLOTS = 34  # MAX_REF_FRAMES (33, common/global.h:67) references + the frame being decoded


def ring_slots(frames, hold: int = 0) -> int:
    """Reference-ring slots a stream needs: 1 + the longest decode-order
    distance from a frame to a picture it predicts from (its blocks' ref0 /
    ref1 and the interpolated reference's two sources), or `hold` if more of
    the most recently decoded frames must stay readable.  The sequence header
    cannot bound this: it carries max_num_ref (dec/maindec.c:137) but a
    reference index reaches up to 32 pictures back (ref_array, 6 bits,
    dec/decode_frame.c:68; HDB16 uses 2 * sub_gop - 1 = 31 with max_num_ref 2,
    enc/mainenc.c:302), so the ring is sized from the parsed frame headers.
    The ring evicts the slot decoded longest ago (thor_dec_create)."""
    order = {}
    reach = 0
    for d, fr in enumerate(frames):
        refs = set()
        b = fr.blocks
        if len(b):
            refs.update(int(r) for r in np.unique(np.concatenate([b["ref0"], b["ref1"]])) if r >= 0)
        if getattr(fr, "interp_ratio", 0):
            refs.update(r for r in fr.interp_refs if r >= 0)
        for r in refs:
            if r not in order:
                raise ValueError("frame %d references frame %d, not decoded before it" % (fr.frame_num, r))
            reach = max(reach, d - order[r])
        order[fr.frame_num] = d
    n = max(reach + 1, hold, 2)
    if n > MAX_SLOTS:
        raise ValueError("stream reaches %d frames back, the ring holds at most %d" % (reach, MAX_SLOTS - 1))
    return n


class GpuDecoder:
    def __init__(self, seq, device: int = 0, slots: int = MAX_SLOTS):
        """slots: reference-ring size; ring_slots(frames) sizes it to a parsed
        stream (the default holds any stream the reference can produce)."""
        self.lib = L.load()
        if self.lib.thor_device_count() <= 0:
            raise RuntimeError("no HIP device visible: the GPU decode path has no CPU fallback")
        self.seq = seq
        cs = L.ThorSeq(seq.width, seq.height, seq.bipred, seq.deblocking, seq.clpf, seq.tb_split_enable,
                       getattr(seq, "interp_ref", 0))
        self.h = self.lib.thor_dec_create(C.byref(cs), device, slots)
        if not self.h:
            raise L.create_error("thor_dec_create")
        self._bufs = []
        self.use_slow_list = True  # False: every k_recon unit in planned order (same output; tests compare both)

    def close(self):
        for b in self._bufs:
            b.free()
        self._bufs = []
        if self.h:
            self.lib.thor_dec_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def _buf(self, arr: np.ndarray, pool=None, key=None) -> DeviceBuffer:
        if pool is not None:  # re-use the buffer `key` of `pool` when it is big enough
            b = pool.get(key)
            if b is None or b.nbytes < arr.nbytes:
                if b is not None:
                    b.free()
                    self._bufs.remove(b)
                b = DeviceBuffer(self.lib, arr.nbytes + (arr.nbytes >> 2))
                self._bufs.append(b)
                pool[key] = b
            b.upload(arr)
            return b
        b = DeviceBuffer(self.lib, arr.nbytes)
        b.upload(arr)
        self._bufs.append(b)
        return b

    def upload(self, fr, pool=None) -> DeviceFrame:
        """Upload frame `fr`'s parse output.  `pool` (a dict the caller keeps
        per in-flight frame) re-uses that frame slot's device buffers."""
        blocks = np.ascontiguousarray(fr.blocks, dtype=BLOCK_DTYPE)
        coeffs = np.ascontiguousarray(fr.coeffs, dtype=np.int16)
        flags = np.ascontiguousarray(fr.clpf_flags, dtype=np.uint8)
        n_intra = self.lib.thor_build_intra_list(blocks.ctypes.data, len(blocks), None)
        ilist = np.zeros(max(n_intra, 1), np.uint32)
        self.lib.thor_build_intra_list(blocks.ctypes.data, len(blocks), ilist.ctypes.data)
        n_tu = self.lib.thor_build_tu_list(blocks.ctypes.data, len(blocks), None)
        tlist = np.zeros(max(n_tu, 1), TU_DTYPE)
        self.lib.thor_build_tu_list(blocks.ctypes.data, len(blocks), tlist.ctypes.data)
        n_clpf = self.lib.thor_build_clpf_list(flags.ctypes.data, len(flags), None) if flags.size else 0
        clist = np.zeros(max(n_clpf, 1), np.uint32)
        if flags.size:
            self.lib.thor_build_clpf_list(flags.ctypes.data, len(flags), clist.ctypes.data)
        W, H = self.seq.width, self.seq.height
        n_slow = self.lib.thor_build_slow_list(blocks.ctypes.data, len(blocks), W, H, None)
        slist = np.zeros(max(n_slow, 1), np.uint32)
        self.lib.thor_build_slow_list(blocks.ctypes.data, len(blocks), W, H, slist.ctypes.data)
        # one host image, one device buffer, one copy (256-byte aligned parts)
        parts = [blocks, coeffs, flags, ilist, tlist, clist, slist]
        offs, o = [], 0
        for a in parts:
            offs.append(o)
            o += (a.nbytes + 255) & ~255
        img = np.zeros(max(o, 256), np.uint8)
        for a, off in zip(parts, offs):
            img[off:off + a.nbytes] = a.view(np.uint8).reshape(-1)
        base = self._buf(img, pool, 0).ptr
        bp, cp, fp, ip, tp, lp, sp = (base + off for off in offs)
        hdr = L.ThorFrameHdr(fr.frame_num, fr.frame_type, fr.qp, fr.clpf_on,
                             (C.c_int32 * 2)(*fr.interp_refs), fr.interp_ratio, fr.interp_pos)
        nbytes = blocks.nbytes + coeffs.nbytes + flags.nbytes + 4 * n_intra + TU_DTYPE.itemsize * n_tu + 4 * n_slow
        return DeviceFrame(hdr, bp, len(blocks), cp, fp if flags.size else 0, ip, n_intra, tp, n_tu, lp, n_clpf,
                           sp, n_slow, nbytes)

    def upload_payload(self, parser, payload: bytes, pool=None) -> DeviceFrame:
        """Parse one frame payload (parser: a thor_amd.bitstream.Parser of this
        stream) and upload its decoder input in one copy: the parse, the work
        lists and the host image all in native code (thor_parse_frame +
        thor_frame_image), no per-part numpy arrays."""
        out = L.ThorParsedFrame()
        buf = C.create_string_buffer(payload, len(payload))
        rc = self.lib.thor_parse_frame(parser.h, buf, len(payload), C.byref(out))
        if rc != 0:
            raise ValueError("thor_parse_frame failed (%d)" % rc)
        lay = L.ThorFrameImage()
        img = pool.get("img") if pool is not None else None
        rc = self.lib.thor_frame_image(C.byref(out), img.ctypes.data if img is not None else None,
                                       img.nbytes if img is not None else 0, C.byref(lay))
        if rc == L.THOR_ERR_NOMEM:
            img = np.empty(lay.bytes + (lay.bytes >> 2), np.uint8)
            if pool is not None:
                pool["img"] = img
            rc = self.lib.thor_frame_image(C.byref(out), img.ctypes.data, img.nbytes, C.byref(lay))
        L.check(rc, "thor_frame_image")
        base = self._buf(img[:lay.bytes], pool, 0).ptr
        h = out.hdr
        hdr = L.ThorFrameHdr(h.frame_num, h.frame_type, h.qp, h.clpf_on, (C.c_int32 * 2)(h.interp_ref[0], h.interp_ref[1]),
                             h.interp_ratio, h.interp_pos)
        return DeviceFrame(hdr, base + lay.off_blocks, lay.nblocks, base + lay.off_coeffs,
                           base + lay.off_flags if lay.n_flags else 0, base + lay.off_intra, lay.n_intra,
                           base + lay.off_tus, lay.n_tu, base + lay.off_clpf, lay.n_clpf, base + lay.off_slow,
                           lay.n_slow, int(lay.bytes))

    def decode(self, d: DeviceFrame):
        fi = self.frame_in(d)
        hs = (C.c_void_p * 1)(self.h)
        L.check(self.lib.thor_dec_frames(hs, 1, C.byref(d.hdr), C.byref(fi)), "thor_dec_frames")

    def frame_in(self, d: DeviceFrame) -> L.ThorFrameIn:
        return L.ThorFrameIn(d.blocks, d.nblocks, d.coeffs, d.clpf or None, d.intra, d.n_intra, d.tus, d.n_tu,
                             d.clpfl if d.clpf else None, d.n_clpf if d.clpf else -1,
                             d.slow if self.use_slow_list else None, d.n_slow)

    # ---- row-band sharding (thor_amd/shard.py) ----
    def set_band(self, sb_row0: int, sb_row1: int):
        L.check(self.lib.thor_dec_set_band(self.h, sb_row0, sb_row1), "thor_dec_set_band")

    def begin(self, d: DeviceFrame):
        fi = self.frame_in(d)
        L.check(self.lib.thor_dec_frame_begin(self.h, C.byref(d.hdr), C.byref(fi)), "thor_dec_frame_begin")

    def end(self):
        L.check(self.lib.thor_dec_frame_end(self.h), "thor_dec_frame_end")

    def set_band_local(self, on: bool):
        L.check(self.lib.thor_dec_set_band_local(self.h, 1 if on else 0), "thor_dec_set_band_local")

    def set_band_pad(self, on: bool):
        """thor_dec_set_band_pad: finish() pads only the band's rows (halo / boundary modes)."""
        L.check(self.lib.thor_dec_set_band_pad(self.h, 1 if on else 0), "thor_dec_set_band_pad")

    def set_band_intra(self, on: bool):
        L.check(self.lib.thor_dec_set_band_intra(self.h, 1 if on else 0), "thor_dec_set_band_intra")

    def intra(self):
        """The pending frame's intra stage now (band-local intra: the band's rows)."""
        L.check(self.lib.thor_dec_frame_intra(self.h), "thor_dec_frame_intra")

    def finish(self):
        L.check(self.lib.thor_dec_frame_finish(self.h), "thor_dec_frame_finish")

    def get_rows(self, frame_num: int, y0: int, nrows: int, dst_ptr):
        L.check(self.lib.thor_dec_get_rows(self.h, frame_num, y0, nrows, dst_ptr), "thor_dec_get_rows")

    def put_rows(self, frame_num: int, y0: int, nrows: int, src_ptr):
        L.check(self.lib.thor_dec_put_rows(self.h, frame_num, y0, nrows, src_ptr), "thor_dec_put_rows")

    def put_ref_rows(self, frame_num: int, y0: int, nrows: int, src_ptr):
        L.check(self.lib.thor_dec_put_ref_rows(self.h, frame_num, y0, nrows, src_ptr), "thor_dec_put_ref_rows")

    def pad_frame(self, frame_num: int):
        L.check(self.lib.thor_dec_pad_frame(self.h, frame_num), "thor_dec_pad_frame")

    def scratch(self, nbytes: int) -> int:
        return self._buf(np.zeros(max(nbytes, 16), np.uint8)).ptr

    def d2h(self, out: np.ndarray, ptr: int):
        self.sync()
        L.check(self.lib.thor_d2h(out.ctypes.data, ptr, out.nbytes), "thor_d2h")

    def h2d(self, ptr: int, arr: np.ndarray):
        a = np.ascontiguousarray(arr)
        L.check(self.lib.thor_h2d(ptr, a.ctypes.data, a.nbytes), "thor_h2d")

    def set_stop_stage(self, stage: int):
        L.check(self.lib.thor_dec_set_stop_stage(self.h, stage), "thor_dec_set_stop_stage")

    def set_stream(self, stream_ptr):
        L.check(self.lib.thor_dec_set_stream(self.h, stream_ptr), "thor_dec_set_stream")

    def stream(self):
        return self.lib.thor_dec_stream(self.h)

    def sync(self):
        L.check(self.lib.thor_dec_sync(self.h), "thor_dec_sync")

    def read(self, frame_num: int):
        W, H = self.seq.width, self.seq.height
        y = np.empty((H, W), np.uint8)
        u = np.empty((H // 2, W // 2), np.uint8)
        v = np.empty((H // 2, W // 2), np.uint8)
        L.check(self.lib.thor_dec_read_frame(self.h, frame_num, y.ctypes.data, u.ctypes.data, v.ctypes.data),
                "thor_dec_read_frame")
        return y, u, v

    def read_i420(self, frame_num: int) -> bytes:
        return b"".join(p.tobytes() for p in self.read(frame_num))

    def write(self, frame_num: int, y, u, v):
        y, u, v = (np.ascontiguousarray(p, dtype=np.uint8) for p in (y, u, v))
        L.check(self.lib.thor_dec_write_frame(self.h, frame_num, y.ctypes.data, u.ctypes.data, v.ctypes.data),
                "thor_dec_write_frame")


def decode_batch(decs, frames):
    """Decode frames[i] (a DeviceFrame of decs[i]) for every i with one launch
    per stage (thor_dec_frames); the contexts must be distinct."""
    n = len(decs)
    lib = decs[0].lib
    hs = (C.c_void_p * n)(*[d.h for d in decs])
    hdrs = (L.ThorFrameHdr * n)(*[f.hdr for f in frames])
    ins = (L.ThorFrameIn * n)(*[d.frame_in(f) for d, f in zip(decs, frames)])
    L.check(lib.thor_dec_frames(hs, n, hdrs, ins), "thor_dec_frames")

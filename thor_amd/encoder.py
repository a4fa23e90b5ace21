"""Host driver of the device-resident encoder (libthor_amd.so, thor_enc_*).

`GpuEncoder(params)` owns one encoder context: the reference's frame loop
(coding order, QP, references -- enc/mainenc.c) is planned inside the library;
each call codes the next frame on the GPU and returns its .bit chunk.  The
input sequence is uploaded to HBM once (`upload_sequence`) so that coding reads
only device memory.  No CPU fallback: without the library or a GPU, calls fail."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import lib as L
from .configs import flags as config_flags


def params_from_flags(flag_list) -> L.ThorEncParams:
    """thor_enc_params_t from `-flag value` pairs over the reference defaults
    (enc/strings.c:286-338)."""
    lib = L.load()
    p = L.ThorEncParams()
    lib.thor_enc_default_params(C.byref(p))
    it = list(flag_list)
    alias = {"-n": "num_frames", "-f": "frame_rate"}
    for k, v in zip(it[0::2], it[1::2]):
        name = alias.get(k, k.lstrip("-"))
        if not hasattr(p, name):
            raise KeyError("unknown encoder parameter %s" % k)
        cur = getattr(p, name)
        setattr(p, name, float(v) if isinstance(cur, float) else int(v))
    return p


def params_for(config: str, width: int, height: int, frames: int, extra=()) -> L.ThorEncParams:
    return params_from_flags(config_flags(config, width, height, frames, extra))


class GpuEncoder:
    def __init__(self, params: L.ThorEncParams, device: int = 0):
        self.lib = L.load()
        self.p = params
        if self.lib.thor_enc_check_params(C.byref(params)) != 0:
            raise ValueError("encoder parameters not supported")
        self.h = self.lib.thor_enc_create(C.byref(params), device)
        if not self.h:
            raise L.create_error("thor_enc_create")
        self.W, self.H = params.width, params.height
        self.fsize = self.W * self.H * 3 // 2
        self.seq_dev = None
        self.own_seq = False
        self.nin = 0

    def close(self):
        if self.h:
            self.lib.thor_enc_destroy(self.h)
            self.h = None
        if self.seq_dev and self.own_seq:
            self.lib.thor_dev_free(self.seq_dev)
        self.seq_dev = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def upload_sequence(self, frames: np.ndarray):
        """frames: uint8 array (n, W*H*3/2) of I420 input frames, display order."""
        a = np.ascontiguousarray(frames, dtype=np.uint8).reshape(-1, self.fsize)
        self.nin = a.shape[0]
        self.seq_dev = self.lib.thor_dev_alloc(a.nbytes)
        if not self.seq_dev:
            raise MemoryError("thor_dev_alloc")
        self.own_seq = True
        L.check(self.lib.thor_h2d(self.seq_dev, a.ctypes.data, a.nbytes), "thor_h2d")

    def use_device_sequence(self, ptr: int, nframes: int):
        """Read the input from `nframes` I420 frames the caller keeps (and
        fills) at DEVICE address `ptr`, frame k at ptr + k * W*H*3/2."""
        if self.seq_dev and self.own_seq:
            self.lib.thor_dev_free(self.seq_dev)
        self.seq_dev, self.own_seq, self.nin = ptr, False, nframes

    def reset(self):
        """Start the sequence again (thor_enc_reset): same input, same .bit."""
        L.check(self.lib.thor_enc_reset(self.h), "thor_enc_reset")

    def num_frames(self) -> int:
        return self.lib.thor_enc_num_frames(self.h)

    def next_input_ptr(self):
        k = self.lib.thor_enc_next_input(self.h)
        if k < 0:
            return None
        if k >= self.nin:
            raise IndexError("input frame %d not uploaded" % k)
        return self.seq_dev + k * self.fsize

    def set_cu_mask(self, words):
        """Restrict this context's kernels to the CUs whose bits are set
        (thor_enc_set_cu_mask; bit c % 32 of words[c // 32] = CU c)."""
        arr = (C.c_uint32 * len(words))(*words)
        L.check(self.lib.thor_enc_set_cu_mask(self.h, arr, len(words)), "thor_enc_set_cu_mask")

    def stream(self) -> int:
        """The context's HIP stream (thor_enc_stream): a batch runs on its first member's."""
        return self.lib.thor_enc_stream(self.h) or 0

    def encode_next(self) -> bytes:
        ptr = self.next_input_ptr()
        L.check(self.lib.thor_enc_frame(self.h, ptr, self.W), "thor_enc_frame")
        return self.chunk()

    def chunk(self) -> bytes:
        n = self.lib.thor_enc_frame_bytes(self.h, None, 0)
        buf = C.create_string_buffer(n)
        self.lib.thor_enc_frame_bytes(self.h, buf, n)
        return buf.raw

    def record_sb_costs(self, on: bool = True):
        """thor_enc_record_sb_costs: keep every superblock's top-level
        process_block costs (delta-QP trials, then the final encode)."""
        L.check(self.lib.thor_enc_record_sb_costs(self.h, 1 if on else 0), "thor_enc_record_sb_costs")

    def sb_costs(self) -> np.ndarray:
        """The last coded frame's per-SB costs: int32 (nsb, trials + 1), raster SB order."""
        per = C.c_int(0)
        n = self.lib.thor_enc_sb_costs(self.h, None, 0, C.byref(per))
        if n < 0:
            raise RuntimeError("thor_enc_sb_costs: %d" % n)
        out = np.empty(n, np.int32)
        got = self.lib.thor_enc_sb_costs(self.h, out.ctypes.data, n, C.byref(per))
        if got != n:
            raise RuntimeError("thor_enc_sb_costs: %d" % got)
        return out.reshape(-1, per.value)

    def encode_all(self) -> bytes:
        return b"".join(self.encode_next() for _ in range(self.num_frames()))


def encode_batch(encs):
    """Code the next frame of every encoder in `encs` with one launch per stage."""
    n = len(encs)
    lib = encs[0].lib
    hs = (C.c_void_p * n)(*[e.h for e in encs])
    ptrs = (C.c_void_p * n)(*[e.next_input_ptr() for e in encs])
    strides = (C.c_int * n)(*[e.W for e in encs])
    L.check(lib.thor_enc_frames(hs, n, ptrs, strides), "thor_enc_frames")
    return [e.chunk() for e in encs]


def encode_batch_begin(encs):
    """Enqueue the next frame of every encoder in `encs` (thor_enc_frames_begin):
    returns at once; encode_batch_end(encs) collects it.  The following frame
    may be begun before this one is ended (two batches in flight)."""
    n = len(encs)
    lib = encs[0].lib
    hs = (C.c_void_p * n)(*[e.h for e in encs])
    ptrs = (C.c_void_p * n)(*[e.next_input_ptr() for e in encs])
    strides = (C.c_int * n)(*[e.W for e in encs])
    L.check(lib.thor_enc_frames_begin(hs, n, ptrs, strides), "thor_enc_frames_begin")


def encode_batch_end(encs):
    """The oldest batch begun on `encs`: every encoder's coded frame (bytes)."""
    n = len(encs)
    lib = encs[0].lib
    hs = (C.c_void_p * n)(*[e.h for e in encs])
    L.check(lib.thor_enc_frames_end(hs, n), "thor_enc_frames_end")
    return [e.chunk() for e in encs]


class SeqLaunch:
    """One sequence launch (thor_enc_seq_begin): the next `nframes` frames of
    every encoder in `encs` in ONE persistent launch, frame f + 1 of a stream
    starting as soon as its frame f is a finished reference.  Inputs: each
    encoder's device sequence (upload_sequence / use_device_sequence), or, with
    `host`, page-locked host frames host(i, input_index) -> address that the
    launch itself copies into the device sequence (fetch mode)."""

    def __init__(self, encs, nframes=None, host=None, arena_bytes=0):
        self.encs = encs
        self.lib = encs[0].lib
        n = len(encs)
        if nframes is None:  # every frame each encoder has left
            nframes = min(self._left(e) for e in encs)
        self.n, self.nf = n, nframes
        ins, devs = [], []
        for i, e in enumerate(encs):
            for f in range(nframes):
                k = self.lib.thor_enc_plan_input(e.h, f)
                if k < 0 or k >= e.nin:
                    raise IndexError("input frame %d not available" % k)
                devs.append(e.seq_dev + k * e.fsize)
                ins.append(host(i, k) if host else e.seq_dev + k * e.fsize)
        hs = (C.c_void_p * n)(*[e.h for e in encs])
        self._ins = (C.c_void_p * len(ins))(*ins)
        self._devs = (C.c_void_p * len(devs))(*devs)
        L.check(self.lib.thor_enc_seq_begin(hs, n, nframes, self._ins, self._devs if host else None, 1 if host else 0,
                                            arena_bytes), "thor_enc_seq_begin")
        self.sizes = np.full(n * nframes, -1, np.int64)
        self.stats = None

    def _left(self, e):
        f = 0
        while self.lib.thor_enc_plan_input(e.h, f) >= 0:
            f += 1
        return f

    def ready(self) -> np.ndarray:
        """Chunk size per (encoder, frame) that is final, -1 otherwise (non-blocking)."""
        self.lib.thor_enc_seq_ready(self.encs[0].h, self.sizes.ctypes.data, self.sizes.size)
        return self.sizes.reshape(self.n, self.nf)

    def chunk(self, i: int, f: int) -> bytes:
        n = self.lib.thor_enc_seq_chunk(self.encs[0].h, i, f, None, 0)
        if n < 0:
            raise RuntimeError("thor_enc_seq_chunk(%d, %d): %d" % (i, f, n))
        buf = C.create_string_buffer(n)
        self.lib.thor_enc_seq_chunk(self.encs[0].h, i, f, buf, n)
        return buf.raw

    def end(self):
        st = (C.c_longlong * 4)()
        L.check(self.lib.thor_enc_seq_end(self.encs[0].h, st), "thor_enc_seq_end")
        self.stats = {"workers": st[0], "retired": st[1], "tasks": st[2], "arena_words": st[3]}
        pr = (C.c_longlong * 15)()
        self.lib.thor_enc_seq_profile(self.encs[0].h, pr, 15)
        names = ["rd", "fetch", "dbv", "dbh", "fin", "pack"]
        self.profile = {"task_ms": {k: round(pr[i] / 1e5, 1) for i, k in enumerate(names)},
                        "tasks": {k: pr[6 + i] for i, k in enumerate(names)},
                        "idle_ms": round(pr[12] / 1e5, 1), "claim_wait_ms": round(pr[13] / 1e5, 1),
                        "failed_claims": pr[14]}
        return self.stats


def encode_sequences(encs, nframes=None, host=None):
    """Every remaining frame (or `nframes`) of every encoder in one sequence
    launch; returns each encoder's .bit bytes for those frames."""
    s = SeqLaunch(encs, nframes, host)
    s.end()
    return [b"".join(s.chunk(i, f) for f in range(s.nf)) for i in range(s.n)]

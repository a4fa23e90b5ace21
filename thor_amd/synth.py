"""Seeded, integer-only synthetic camera-like YUV 4:2:0 generator.

The reference ships no test clips and its configs point at a
Windows path (config_LDB_low_complexity.txt:1), so every stream this repo uses
is encoded from frames produced here.  The recipe follows SURVEY.md sec. 8(d) /
BASELINE.md sec. 4: a multi-octave value-noise texture (cell sizes 64/16/4/1 px,
amplitudes 48/24/10/4), a sub-pel global pan of (+0.61, +1.37) px/frame, three
textured 224x160 objects moving at their own speeds, and temporal noise
(sigma ~3 on luma, ~1.2 on chroma).

Everything is integer arithmetic on numpy uint32/int64 (positions in 1/256 px),
so the output is bit-identical on every host; tests/golden/synth_md5.json pins it.
"""
from __future__ import annotations

import hashlib

import numpy as np

_PAN = (156, 351)  # 1/256 px per frame  (= +0.61, +1.37 px)
_OBJ_VEL = ((819, -282), (-614, 179), (333, 666))  # 1/256 px per frame
_OBJ_W, _OBJ_H = 224, 160


def _hash2(ix: np.ndarray, iy: np.ndarray, seed: int) -> np.ndarray:
    """32-bit integer hash of lattice coordinates (wrapping uint32 arithmetic)."""
    h = (ix.astype(np.uint32) * np.uint32(0x8DA6B343)) ^ (iy.astype(np.uint32) * np.uint32(0xD8163841))
    h ^= np.uint32((seed * 0x9E3779B1) & 0xFFFFFFFF)
    h ^= h >> np.uint32(15)
    h *= np.uint32(0x2C1B3C6D)
    h ^= h >> np.uint32(12)
    h *= np.uint32(0x297A2D39)
    h ^= h >> np.uint32(15)
    return h


def _value_noise(X: np.ndarray, Y: np.ndarray, cell_log2: int, seed: int) -> np.ndarray:
    """Bilinear value noise in [-128, 127]; X (cols) and Y (rows) in 1/256 px, 1-D."""
    sh = cell_log2 + 8
    cx = X >> sh
    cy = Y >> sh
    fx = ((X - (cx << sh)) >> cell_log2).astype(np.int64)  # 0..255
    fy = ((Y - (cy << sh)) >> cell_log2).astype(np.int64)
    x0, y0 = int(cx.min()), int(cy.min())
    gx = np.arange(x0, int(cx.max()) + 2, dtype=np.int64)
    gy = np.arange(y0, int(cy.max()) + 2, dtype=np.int64)
    lat = (_hash2(gx[None, :] & 0xFFFFFFFF, gy[:, None] & 0xFFFFFFFF, seed) >> np.uint32(24)).astype(np.int32) - 128
    ix = cx - x0
    iy = cy - y0
    # separable evaluation of the same exact sum (|value| < 2^23, int32 is exact):
    # lattice rows interpolated horizontally first, then the row pairs vertically
    fx32 = fx.astype(np.int32)[None, :]
    hrow = lat[:, ix] * (256 - fx32) + lat[:, ix + 1] * fx32
    fy32 = fy.astype(np.int32)[:, None]
    v = (hrow[iy] * (256 - fy32) + hrow[iy + 1] * fy32) >> 16
    return v.astype(np.int64)


def _texture(X, Y, seed, octaves):
    acc = None
    for k, (cell_log2, amp) in enumerate(octaves):
        v = (_value_noise(X, Y, cell_log2, seed * 7 + k) * amp) >> 7
        acc = v if acc is None else acc + v
    return acc


_LUMA_OCT = ((6, 48), (4, 24), (2, 10), (0, 4))
_CHROMA_OCT = ((5, 20), (3, 10), (1, 4))


def _temporal_noise(shape, seed, t, taps, span):
    rs = np.random.Generator(np.random.PCG64([seed, t, 0xC0DEC]))
    n = np.zeros(shape, dtype=np.int64)
    for _ in range(taps):
        n += rs.integers(-span, span + 1, size=shape, dtype=np.int64)
    return n


def _plane(width, height, t, seed, sub, octaves, noise_taps, noise_span, base):
    """One plane at subsampling `sub` (1 luma, 2 chroma)."""
    cols = np.arange(width, dtype=np.int64) * (256 * sub)
    rows = np.arange(height, dtype=np.int64) * (256 * sub)
    X = cols + t * _PAN[0]
    Y = rows + t * _PAN[1]
    img = base + _texture(X, Y, seed, octaves)
    full_w, full_h = width * sub, height * sub
    for o, (vx, vy) in enumerate(_OBJ_VEL):
        ox = (full_w * (o + 1)) // 4 - _OBJ_W // 2
        oy = (full_h * (o + 1)) // 4 - _OBJ_H // 2
        px = ox * 256 + t * vx  # object origin, 1/256 px (full-res units)
        py = oy * 256 + t * vy
        lx = cols - px  # local coords in 1/256 full-res px
        ly = rows - py
        inx = (lx >= 0) & (lx < _OBJ_W * 256)
        iny = (ly >= 0) & (ly < _OBJ_H * 256)
        if not inx.any() or not iny.any():
            continue
        # the object covers a rectangle: texture only that window
        c = np.flatnonzero(inx)
        r = np.flatnonzero(iny)
        c0, c1, r0, r1 = c[0], c[-1] + 1, r[0], r[-1] + 1
        img[r0:r1, c0:c1] = base + 16 * (o - 1) + _texture(lx[c0:c1] + (1 << 20), ly[r0:r1] + (1 << 20),
                                                           seed + 101 * (o + 1), octaves)
    img = img + _temporal_noise(img.shape, seed, t, noise_taps, noise_span)
    return np.clip(img, 0, 255).astype(np.uint8)


def synth_frame(width: int, height: int, t: int, seed: int = 1):
    """Return (Y, U, V) uint8 planes of frame t."""
    y = _plane(width, height, t, seed, 1, _LUMA_OCT, 3, 3, 128)
    u = _plane(width // 2, height // 2, t, seed + 1000, 2, _CHROMA_OCT, 2, 1, 120)
    v = _plane(width // 2, height // 2, t, seed + 2000, 2, _CHROMA_OCT, 2, 1, 136)
    return y, u, v


def _i420(args):
    return np.concatenate([p.reshape(-1) for p in synth_frame(*args)])


def synth_frames(width: int, height: int, frames: int, seed: int = 1, workers: int = 8) -> np.ndarray:
    """(frames, W*H*3/2) uint8 I420 array, frames generated in parallel
    processes (fork: call before the process initialises a GPU)."""
    args = [(width, height, t, seed) for t in range(frames)]
    if workers <= 1 or frames <= 1:
        return np.stack([_i420(a) for a in args])
    import multiprocessing as mp

    pool = mp.get_context("fork").Pool(min(workers, frames))
    try:
        out = np.stack(pool.map(_i420, args))
    finally:
        pool.close()  # workers exit on their own (the `with` block's terminate() SIGTERMs them, which
        pool.join()   # profilers log as aborts)
    return out


def synth_clip(width: int, height: int, frames: int, seed: int = 1) -> bytes:
    """Raw planar I420 bytes of `frames` frames."""
    out = []
    for t in range(frames):
        for p in synth_frame(width, height, t, seed):
            out.append(p.tobytes())
    return b"".join(out)


def clip_md5(width: int, height: int, frames: int, seed: int = 1) -> str:
    return hashlib.md5(synth_clip(width, height, frames, seed)).hexdigest()


if __name__ == "__main__":  # pragma: no cover
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, required=True)
    ap.add_argument("--height", type=int, required=True)
    ap.add_argument("--frames", type=int, required=True)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("out")
    a = ap.parse_args()
    with open(a.out, "wb") as f:
        for t in range(a.frames):
            for p in synth_frame(a.width, a.height, t, a.seed):
                f.write(p.tobytes())

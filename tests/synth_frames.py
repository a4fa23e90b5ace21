"""Test helper: random but well-formed parse output (block descriptors + compact
coefficients) for one P/B frame over given reference frames.

Used to drive the batched GPU path and the oracle with the same inputs at
every MC fraction, CU size 8..64, quadtree split pattern, mode (SKIP with
rectangular frame-edge clipping, MERGE, INTER with four quarter MVs, BIPRED,
bi-directional SKIP/MERGE), reference choice (past and future: the `sign`
negation), tb_split and qp -- cases the reference-encoded streams hit only
sparsely.  With INTRA in `modes`, intra CUs of every mode (DC, HOR, VER,
PLANAR and the six angular modes, common/intra_prediction.c:145-388) and size,
with and without tb-split, anywhere in the frame (so at every availability
pattern of the frame edges and of the quadtree).  The descriptor semantics follow block_info_dec_t as read by
read_block (dec/read_bits.c:221); see thor_amd/trace.py for the layout."""
from __future__ import annotations

import numpy as np

from thor_amd.trace import BLOCK_DTYPE, Frame, tu_layout, chroma_tb_split

SKIP, INTRA, INTER, BIPRED, MERGE = 0, 1, 2, 3, 4


def random_plane(rng, h, w):
    # blocky texture plus noise so the filters see real gradients
    base = rng.integers(0, 256, (h // 8 + 2, w // 8 + 2)).astype(np.float64)
    up = np.kron(base, np.ones((8, 8)))[:h, :w]
    return np.clip(up + rng.normal(0, 24, (h, w)), 0, 255).astype(np.uint8)


def random_frame(rng, W, H):
    return random_plane(rng, H, W), random_plane(rng, H // 2, W // 2), random_plane(rng, H // 2, W // 2)


def _leaves(rng, y, x, size, W, H, split_p):
    """Quadtree leaves in decode order (TL, BL, TR, BR: dec/decode_block.c:661-664).
    A CU that crosses the frame edge is split unless it becomes a SKIP
    rectangle (the only mode allowed to overhang, dec/decode_block.c:222-226)."""
    if y >= H or x >= W:
        return []
    inside = y + size <= H and x + size <= W
    if size > 8 and ((not inside and rng.random() < 0.7) or rng.random() < split_p):
        h = size // 2
        out = []
        for dy, dx in ((0, 0), (h, 0), (0, h), (h, h)):
            out += _leaves(rng, y + dy, x + dx, h, W, H, split_p)
        return out
    return [(y, x, size, inside)]


def synth_frame(rng, W, H, frame_num, ref_nums, coeff_p=0.0, split_p=0.35, mv_range=48,
                modes=(SKIP, MERGE, INTER, BIPRED), frame_type=1):
    blocks = []
    pool = []
    pool_len = 0
    for sby in range(0, H, 64):
        for sbx in range(0, W, 64):
            for (y, x, size, inside) in _leaves(rng, sby, sbx, 64, W, H, split_p):
                r = np.zeros(1, BLOCK_DTYPE)[0]
                r["ypos"], r["xpos"], r["size"] = y, x, size
                r["bwidth"], r["bheight"] = min(size, W - x), min(size, H - y)
                mode = SKIP if not inside else int(rng.choice(modes))
                r["mode"] = mode
                r["qp"] = int(rng.integers(18, 46))
                if mode == INTRA:
                    r["intra_mode"] = int(rng.integers(0, 10))
                q_mvs = 4 if mode in (INTER, BIPRED) else 1
                mv0 = rng.integers(-mv_range, mv_range + 1, (q_mvs, 2))
                mv1 = rng.integers(-mv_range, mv_range + 1, (q_mvs, 2))
                if q_mvs == 1:
                    mv0 = np.repeat(mv0, 4, 0)
                    mv1 = np.repeat(mv1, 4, 0)
                if mode == INTRA:
                    mv0[...] = 0
                    mv1[...] = 0
                r["mv0"] = mv0.reshape(-1)
                r["mv1"] = mv1.reshape(-1)
                r["ref0"] = int(rng.choice(ref_nums))
                bi = mode == BIPRED or (mode in (SKIP, MERGE) and rng.random() < 0.3)
                if mode == INTRA:
                    r["ref0"] = ref_nums[0]
                r["dir"] = 2 if (bi and mode != BIPRED) else 0
                r["ref1"] = int(rng.choice(ref_nums)) if bi else r["ref0"]
                cmask = 0
                offs = [0, 0, 0]
                if mode != SKIP and rng.random() < coeff_p:
                    tb = int(size > 8 and rng.random() < 0.4)
                    r["tb_split"] = tb
                    for c in range(3):
                        if rng.random() < 0.6:
                            n = size if c == 0 else size // 2
                            tbc = tb if c == 0 else chroma_tb_split(size, tb)
                            _, ntu, q = tu_layout(n, tbc)
                            comp = np.zeros(ntu * q * q, np.int16)
                            nz = rng.random(comp.size) < 0.3
                            comp[nz] = rng.integers(-40, 41, int(nz.sum()))
                            offs[c] = pool_len
                            pool.append(comp)
                            pool_len += comp.size
                            cmask |= 1 << c
                r["coeff_mask"] = cmask
                r["coeff_off"] = offs
                r["cbp_y"], r["cbp_u"], r["cbp_v"] = cmask & 1, (cmask >> 1) & 1, (cmask >> 2) & 1
                blocks.append(r)
    coeffs = np.concatenate(pool).astype(np.int16) if pool else np.zeros(0, np.int16)
    b = np.array(blocks, dtype=BLOCK_DTYPE)
    return Frame(0, frame_num, frame_type, int(rng.integers(22, 40)), len(ref_nums), 0, b, coeffs)

"""GPU parity on synthetic parse output: random quadtrees, modes, MVs at every
fraction (including the (2,2) centre and far out-of-frame displacements),
past / future references (the `sign` negation), bi-pred, tb_split, random
coefficients.  The batched HIP path through the C-ABI must reproduce the
oracle's reconstruction (stage 0) and deblocked frame (stage 1) bit-exactly."""
import numpy as np
import pytest

from synth_frames import random_frame, synth_frame
from thor_amd.trace import SeqParams

pytestmark = pytest.mark.gpu

CASES = [
    # W, H, bipred, frame_num, refs, coeff_p, split_p, mv_range
    (256, 128, 0, 2, [0, 1], 0.0, 0.35, 48),
    (256, 128, 1, 1, [0, 2], 0.0, 0.35, 48),
    (352, 136, 0, 2, [0, 1], 0.5, 0.6, 48),
    (352, 136, 1, 1, [0, 2], 0.5, 0.2, 300),
    (320, 192, 0, 5, [3, 4], 0.3, 0.0, 16),
    (320, 192, 1, 5, [3, 7], 0.3, 0.9, 64),
]


def _oracle_ref(odec, fnum, planes):
    from oracle.py import PaddedFrame

    pf = PaddedFrame(odec.seq.width, odec.seq.height)
    pf.frame_num = fnum
    y, u, v = pf.planes()
    y[...], u[...], v[...] = planes
    odec.push_reference(pf)


@pytest.mark.parametrize("case", range(len(CASES)))
@pytest.mark.parametrize("seed", [1, 2])
def test_recon_matches_oracle_on_synthetic_frames(case, seed):
    from oracle import OracleDecoder
    from thor_amd.decoder import GpuDecoder

    W, H, bipred, fnum, refs, coeff_p, split_p, mvr = CASES[case]
    rng = np.random.default_rng(1000 * case + seed)
    seq = SeqParams(W, H, 0, 1, 2, 0, 0, 1, 0, 1, bipred)
    gdec, odec = GpuDecoder(seq), OracleDecoder(seq)
    try:
        for r in refs:
            planes = random_frame(rng, W, H)
            gdec.write(r, *planes)
            _oracle_ref(odec, r, planes)
        fr = synth_frame(rng, W, H, fnum, refs, coeff_p=coeff_p, split_p=split_p, mv_range=mvr)
        dev = gdec.upload(fr)
        for stage in (0, 1):
            gdec.set_stop_stage(stage)
            gdec.decode(dev)
            gdec.sync()
            got = gdec.read(fnum)
            want = odec.decode(fr, stage).planes()
            for name, g, o in zip("YUV", got, want):
                bad = np.argwhere(g != o)
                assert bad.size == 0, (CASES[case], seed, stage, name, len(bad), bad[:4].tolist())
    finally:
        gdec.close()


INTRA_CASES = [
    # W, H, frame_type, modes, coeff_p, split_p
    (256, 128, 0, ("INTRA",), 0.7, 0.5),           # I frame: every CU intra, frame edges on all sides
    (352, 136, 1, ("SKIP", "INTRA", "INTER"), 0.6, 0.5),  # intra CUs among inter ones, ragged right/bottom
    (320, 192, 1, ("INTRA", "MERGE"), 0.3, 0.8),   # mostly 8x8 / 16x16 intra next to merges
]


@pytest.mark.parametrize("case", range(len(INTRA_CASES)))
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_intra_cus_match_oracle(case, seed):
    """k_intra's WPP chains on synthetic intra CUs: all ten modes, sizes 8..64,
    tb-split, every neighbour-availability pattern the quadtree and the frame
    edges produce (common/intra_prediction.c:57-388, common/common_block.c:100-129)."""
    import synth_frames as sf
    from oracle import OracleDecoder
    from thor_amd.decoder import GpuDecoder

    W, H, ftype, mnames, coeff_p, split_p = INTRA_CASES[case]
    modes = tuple(getattr(sf, m) for m in mnames)
    rng = np.random.default_rng(7000 + 10 * case + seed)
    seq = SeqParams(W, H, 0, 1, 2, 0, 0, 1, 0, 1, 0)
    gdec, odec = GpuDecoder(seq), OracleDecoder(seq)
    try:
        refs = [0]
        for r in refs:
            planes = random_frame(rng, W, H)
            gdec.write(r, *planes)
            _oracle_ref(odec, r, planes)
        fr = synth_frame(rng, W, H, 1, refs, coeff_p=coeff_p, split_p=split_p, modes=modes, frame_type=ftype)
        assert (fr.blocks["mode"] == sf.INTRA).any()
        dev = gdec.upload(fr)
        for stage in (0, 1):
            gdec.set_stop_stage(stage)
            gdec.decode(dev)
            gdec.sync()
            got = gdec.read(1)
            want = odec.decode(fr, stage).planes()
            for name, g, o in zip("YUV", got, want):
                bad = np.argwhere(g != o)
                assert bad.size == 0, (INTRA_CASES[case], seed, stage, name, len(bad), bad[:4].tolist())
    finally:
        gdec.close()

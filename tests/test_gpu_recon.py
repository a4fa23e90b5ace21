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

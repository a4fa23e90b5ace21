"""CPU: the synthetic parse-output generator makes frames the oracle accepts
(every CU inside the frame or a clipped SKIP, the quadtree tiles the frame)."""
import numpy as np

from synth_frames import random_frame, synth_frame


def test_synthetic_frames_tile_the_frame_and_decode_on_the_oracle():
    from oracle import OracleDecoder
    from oracle.py import PaddedFrame
    from thor_amd.trace import SeqParams

    rng = np.random.default_rng(5)
    W, H = 352, 136
    seq = SeqParams(W, H, 0, 1, 2, 0, 0, 1, 0, 1, 1)
    odec = OracleDecoder(seq)
    for r in (0, 2):
        pf = PaddedFrame(W, H)
        pf.frame_num = r
        y, u, v = pf.planes()
        y[...], u[...], v[...] = random_frame(rng, W, H)
        odec.push_reference(pf)
    fr = synth_frame(rng, W, H, 1, [0, 2], coeff_p=0.5)
    cover = np.zeros((H, W), np.int32)
    for b in fr.blocks:
        cover[b["ypos"]:b["ypos"] + b["bheight"], b["xpos"]:b["xpos"] + b["bwidth"]] += 1
    assert (cover == 1).all()
    odec.decode(fr, 1)


def test_synthetic_intra_frames_decode_on_the_oracle():
    """Intra CUs (all modes, tb-split, frame edges) in P and I frames decode on the oracle."""
    import synth_frames as sf
    from oracle import OracleDecoder
    from oracle.py import PaddedFrame
    from thor_amd.trace import SeqParams

    rng = np.random.default_rng(11)
    for W, H, ftype, modes in ((256, 128, 0, (sf.INTRA,)), (352, 136, 1, (sf.SKIP, sf.INTRA, sf.INTER))):
        seq = SeqParams(W, H, 0, 1, 2, 0, 0, 1, 0, 1, 0)
        odec = OracleDecoder(seq)
        pf = PaddedFrame(W, H)
        pf.frame_num = 0
        y, u, v = pf.planes()
        y[...], u[...], v[...] = random_frame(rng, W, H)
        odec.push_reference(pf)
        fr = synth_frame(rng, W, H, 1, [0], coeff_p=0.7, split_p=0.5, modes=modes, frame_type=ftype)
        assert (fr.blocks["mode"] == sf.INTRA).any()
        assert len(set(int(m) for m in fr.blocks["intra_mode"][fr.blocks["mode"] == sf.INTRA])) > 5
        odec.decode(fr, 1)

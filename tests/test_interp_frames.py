"""The oracle's interpolate_frames (oracle/thor_oracle_ti.c) against the
reference's own (tests/golden/interp_frames.npz, tools/make_interp_frames_goldens.py):
the whole temporal-interpolated reference -- luma pyramid, motion_estimate_bi
per level (common/temporal_interp.c:852-918) and interpolate_frame -- bit-exact."""
import os

import numpy as np
import pytest

from oracle.py import interpolate_frames, padded_from_planes
from thor_amd import synth

GOLD = os.path.join(os.path.dirname(__file__), "golden", "interp_frames.npz")


def cases():
    z = np.load(GOLD)
    k = 0
    while "dims_%d" % k in z:
        yield k, z
        k += 1


def refs(z, k):
    w, h, ratio, pos = (int(v) for v in z["dims_%d" % k])
    seed, is_synth = (int(v) for v in z["case_%d" % k])
    if is_synth:
        a, b = synth.synth_frame(w, h, 0, seed), synth.synth_frame(w, h, ratio, seed)
    else:
        a = [z["ref0_%s_%d" % (c, k)] for c in "yuv"]
        b = [z["ref1_%s_%d" % (c, k)] for c in "yuv"]
    return (w, h, ratio, pos), padded_from_planes(*a, 0), padded_from_planes(*b, ratio)


@pytest.mark.parametrize("k", range(6))
def test_oracle_interpolate_frames_vs_reference(k):
    z = np.load(GOLD)
    (w, h, ratio, pos), r0, r1 = refs(z, k)
    got = interpolate_frames(r0, r1, ratio, pos)
    for c, p in zip("yuv", got.planes()):
        want = z["out_%s_%d" % (c, k)]
        assert np.array_equal(p, want), (k, c, int((p != want).sum()))

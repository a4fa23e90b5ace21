"""cost_calc (enc/encode_block.c:1218-1228) as the device encoder and
k_enc_cost restate it -- SSD_Y + SSD_U + SSD_V + (int32)(lambda * nbits + 0.5)
in double without FMA, clamped to 2^30 -- against the reference's own
cost_calc outputs (tests/golden/cost.npz, tools/make_cost_goldens.py)."""
import os

import numpy as np

GOLD = os.path.join(os.path.dirname(__file__), "golden", "cost.npz")


def test_cost_formula_matches_reference():
    z = np.load(GOLD)
    np.seterr(invalid="ignore")  # (int32) of a clamp case's product overflows, as in C; the clamp decides
    for (sy, su, sv), nb, lam, want in zip(z["ssd"], z["nbits"], z["lam"], z["cost"]):
        v = (int(sy) + int(su) + int(sv) + int(np.int32(np.float64(lam) * np.float64(nb) + 0.5))) & 0xFFFFFFFF
        assert min(v, 1 << 30) == int(want)

"""The per-superblock RD-cost goldens (tests/golden/rd_costs.npz, recorded from
the reference Thorenc by tools/make_rd_goldens.py) against the reference's
superblock loop, on CPU: per coded frame one record per top-level
process_block call in raster SB order -- with delta QP every trial qp - d ..
qp + d, then the final encode at the trial QP with the first minimal cost
(enc/encode_frame.c:112-147) -- and the streams' geometry.  The device
encoder's costs are compared with these records in
tests/test_gpu_encoder_rd.py (thor_enc_sb_costs)."""
import json
import os

import numpy as np

from conftest import GOLD

# stream -> (max_delta_qp, delta_qp_step) of its config (config_LDB_high_efficiency / HDB16_high: 1, 1)
DQP = {"cif_low": 0, "k4_low": 0, "cif_high": 1, "hd_high": 1, "k4_hdbi_high": 1}


def test_rd_goldens_follow_the_reference_superblock_loop():
    z = np.load(os.path.join(GOLD, "rd_costs.npz"))
    meta = json.load(open(os.path.join(GOLD, "streams.json")))
    assert set(z.files) == set(DQP)
    for name in z.files:
        r = z[name]
        m = meta[name]
        nsbh, nsbv = (m["width"] + 63) // 64, (m["height"] + 63) // 64
        d = DQP[name]
        per = 2 * d + 2 if d else 1
        order = []
        for f in r[:, 0]:
            if not order or order[-1] != f:
                order.append(int(f))
        assert len(set(order)) == len(order), name  # each coded frame's records are contiguous
        for f in order:
            fr = r[r[:, 0] == f].reshape(nsbv * nsbh, per, 6)
            assert (fr[:, :, 1] == 64).all()
            k, l = np.divmod(np.arange(nsbv * nsbh), nsbh)
            assert (fr[:, :, 2] == 64 * k[:, None]).all() and (fr[:, :, 3] == 64 * l[:, None]).all(), (name, f)
            if d:
                qp = fr[:, 0, 4] + d
                assert (fr[:, :2 * d + 1, 4] == qp[:, None] + np.arange(-d, d + 1)[None, :]).all(), (name, f)
                best = np.argmin(fr[:, :2 * d + 1, 5], axis=1)  # first minimum: `cost < min_cost`
                assert (fr[:, -1, 4] == fr[np.arange(len(fr)), best, 4]).all(), (name, f)
        if name in ("k4_hdbi_high",):
            assert order == [0, 16], order  # the I frame and P frame 16 of the 17-frame HDB16 plan

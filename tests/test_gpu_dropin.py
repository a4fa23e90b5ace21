"""Drop-in boundary, end to end: the reference's own host C (Thorenc /
Thordec, compiled from the reference sources into oracle/_ref by
oracle/Makefile `dropin`) with common/common_kernels.c and
enc/enc_kernels.c replaced by libthor_amd.so, and the L2 entry points
(deblock_frame_y/uv, make_top_and_left, get_intra_prediction, dequantize,
reconstruct_block; include/thor_l2.h) bound to the library too.  Every
SIMD-surface call -- MC, forward/inverse transforms, SAD/SSD, fast sub-pel
search, CLPF -- and every one of those L2 calls executes on the GPU.  The encoder must produce the reference's bitstream
bit for bit (every RD decision, hence every RD cost, identical) and the
decoder the reference's output."""
import hashlib
import json
import os
import subprocess
import sys

import pytest

from conftest import GOLD, ROOT

pytestmark = pytest.mark.gpu
OREF = os.path.join(ROOT, "oracle", "_ref")
DROPIN = json.load(open(os.path.join(GOLD, "dropin.json")))


def md5(p):
    return hashlib.md5(open(p, "rb").read()).hexdigest()


def _exe(name):
    p = os.path.join(OREF, name)
    if not os.path.exists(p):
        pytest.fail("%s missing: build with `make -C oracle dropin` (the build container)" % p)
    return p


@pytest.mark.parametrize("name", sorted(DROPIN))
def test_reference_encoder_on_gpu_kernels(name, tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from make_dropin_goldens import encoder_cmd, write_clip

    c = DROPIN[name]
    yuv, bit, rec = (str(tmp_path / (name + s)) for s in (".yuv", ".bit", "_rec.yuv"))
    write_clip(yuv, c["width"], c["height"], c["frames"], c["seed"])
    assert md5(yuv) == c["yuv_md5"]
    cmd = encoder_cmd(_exe("thorenc_amd"), c["flags"], yuv, bit, rec, str(tmp_path / "st.txt"), c["width"],
                      c["height"], c["frames"], c["extra"])
    subprocess.run(cmd, check=True, timeout=100, stdout=subprocess.DEVNULL)
    assert md5(bit) == c["bit_md5"], "bitstream differs from the reference encoder's"
    assert md5(rec) == c["rec_md5"]
    dec = str(tmp_path / "dec.yuv")
    subprocess.run([_exe("thordec_amd"), bit, dec], check=True, timeout=60, stdout=subprocess.DEVNULL)
    assert md5(dec) == c["rec_md5"]


@pytest.mark.parametrize("stream", ["cif_low", "cif_high"])
def test_reference_decoder_on_gpu_kernels(stream, streams, tmp_path):
    dec = str(tmp_path / "dec.yuv")
    subprocess.run([_exe("thordec_amd"), os.path.join(GOLD, stream + ".bit"), dec], check=True, timeout=100,
                   stdout=subprocess.DEVNULL)
    assert md5(dec) == streams[stream]["dec_md5"]

"""CPU: the device encoder's RD source (thor_amd/csrc/enc_*.h) built for the
host as one lane (tools/enc_host, a debugging harness -- never the product
path) reproduces the reference Thorenc's .bit on the first frames of two
golden clips, including
hierarchical-B coding order and the temporal-interpolated reference (cif_hdbi;
the harness builds it with the oracle's interpolate_frames).  The GPU build of the same source is checked in
tests/test_gpu_encoder_rd.py; this test keeps the shared source honest on a
box without a GPU."""
import os
import subprocess

import pytest

from thor_amd import configs, synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "tools", "enc_host")


@pytest.fixture(scope="module")
def enc_host():
    r = subprocess.run(["make", "-s", "-C", HOST, "enc_host"], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip("host compiler unavailable: " + r.stderr[-200:])
    return os.path.join(HOST, "enc_host")


@pytest.mark.parametrize("name,nframes", [("cif_low", 3), ("w8_low", 2), ("cif_med", 2), ("cif_hdb", 17),
                                           ("cif_hdbi", 17)])
def test_host_build_of_the_rd_source_matches_reference(enc_host, streams, tmp_path, name, nframes):
    meta = streams[name]
    w, h = meta["width"], meta["height"]
    yuv = tmp_path / "in.yuv"
    synth.synth_frames(w, h, nframes, meta["seed"], workers=1).tofile(yuv)
    out = tmp_path / "out.bit"
    subprocess.run([enc_host, "-if", str(yuv), "-of", str(out)] +
                   configs.flags(meta["config"], w, h, nframes, meta["extra"]), check=True,
                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    got = out.read_bytes()
    want = open(os.path.join(ROOT, "tests", "golden", name + ".bit"), "rb").read()
    assert len(got) > 0 and want.startswith(got)

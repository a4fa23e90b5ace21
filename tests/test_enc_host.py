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


@pytest.mark.parametrize("name,nframes", [("cif_low", 3), ("cif_high", 2)])
def test_host_build_rd_costs_match_reference(enc_host, streams, tmp_path, name, nframes):
    """The per-superblock RD costs of the shared RD source (te_encode_sb's cost
    record: every delta-QP trial, then the final encode) == the reference
    encoder's process_block returns (tests/golden/rd_costs.npz, recorded with
    -Wl,--wrap=process_block), call by call.  cif_high: speed 0 with delta-QP
    trials (qp - 1, qp, qp + 1) per superblock."""
    import numpy as np

    meta = streams[name]
    w, h = meta["width"], meta["height"]
    yuv = tmp_path / "in.yuv"
    synth.synth_frames(w, h, nframes, meta["seed"], workers=1).tofile(yuv)
    rd = tmp_path / "costs.bin"
    subprocess.run([enc_host, "-if", str(yuv), "-of", str(tmp_path / "out.bit"), "-rdlog", str(rd)] +
                   configs.flags(meta["config"], w, h, nframes, meta["extra"]), check=True,
                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    got = np.fromfile(rd, dtype="<i4").reshape(-1, 6)
    want = np.load(os.path.join(ROOT, "tests", "golden", "rd_costs.npz"))[name][:len(got)]
    assert len(got) == len(want) and len(got) > 0
    assert (got[:, :4] == want[:, :4]).all()
    trial = got[:, 4] >= 0
    assert (got[trial, 4] == want[trial, 4]).all()
    bad = np.nonzero(got[:, 5] != want[:, 5])[0]
    assert bad.size == 0, ("first differing call", want[bad[0]].tolist(), int(got[bad[0], 5]))

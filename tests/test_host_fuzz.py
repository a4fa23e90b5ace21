"""CPU: the encoder's host control (thor_amd/csrc/enc_gop.h -- parameter
setter and checker, the GOP planner, header writers, early-skip thresholds)
and the decoder's host work lists (thor_amd/csrc/host_lists.h -- TU, intra and
CLPF lists) under AddressSanitizer and UndefinedBehaviorSanitizer
(tools/fuzz/host_fuzz.cpp, g++, nothing runs on a GPU), driven by a seeded
parameter and block-descriptor fuzz.  Every parameter set te_check_params
accepts must plan to frames the device encoder can code (QP range, reference
indices inside the 33-frame window, references already coded); the list
builders must agree between their counting and filling passes and fill
buffers of exactly the counted size."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FUZZ = os.path.join(ROOT, "tools", "fuzz")


@pytest.fixture(scope="module")
def harness():
    if shutil.which("g++") is None or shutil.which("make") is None:
        pytest.skip("g++ / make unavailable")
    r = subprocess.run(["make", "-s", "-C", FUZZ, "host_fuzz"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    return os.path.join(FUZZ, "host_fuzz")


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_host_fuzz(harness, seed):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([harness, "6000", str(seed)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert " 0 failures" in r.stdout, r.stdout
    accepted = int(r.stdout.split(",")[1].split()[0])
    assert accepted > 1000, r.stdout  # the fuzz reaches the planner, not only the checker


def test_check_params_follows_reference_rules():
    """check_parameters (enc/strings.c:431-479) through the C-ABI checker: the
    shipped configurations pass, each rule the reference enforces with
    fatalerror() is THOR_ERR_ARG here."""
    import ctypes as C

    from thor_amd import lib as L
    from thor_amd.configs import CONFIGS
    from thor_amd.encoder import params_for

    lib = L.load()
    for name in CONFIGS:
        assert lib.thor_enc_check_params(C.byref(params_for(name, 1920, 1080, 8))) == 0, name
    base = ("config_HDB16_high_efficiency.txt", 1920, 1080, 32)
    bad = [("-n", 0), ("-max_num_ref", 5), ("-max_delta_qp", 8), ("-HQperiod", 33),
           ("-num_reorder_pics", 2),  # dyadic coding needs num_reorder_pics + 1 a power of 2
           ("-intra_period", 24),     # not a multiple of the sub-GOP (16)
           ("-HQperiod", 24)]         # the sub-GOP must divide HQperiod
    for k, v in bad:
        assert lib.thor_enc_check_params(C.byref(params_for(*base, extra=(k, str(v))))) == L.THOR_ERR_ARG, k
    p = params_for("config_LDB_low_complexity.txt", 1920, 1080, 8, extra=("-num_reorder_pics", "1", "-max_num_ref", "1"))
    assert lib.thor_enc_check_params(C.byref(p)) == L.THOR_ERR_ARG  # reordering needs 2 references

"""CPU: the host .bit parser (thor_amd/csrc/parse.hip) under AddressSanitizer
and UndefinedBehaviorSanitizer (tools/fuzz: a host-only build, nothing runs on
a GPU) on every golden .bit intact and on seeded corruptions of it --
truncated frames, bit flips, overwritten byte runs, dropped / repeated /
swapped frames, a corrupt sequence header.  Every call must return THOR_OK or
a THOR_ERR_* code; any out-of-bounds access or undefined behaviour aborts the
harness (-fno-sanitize-recover)."""
import glob
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FUZZ = os.path.join(ROOT, "tools", "fuzz")


@pytest.fixture(scope="module")
def harness():
    if not os.path.exists("/opt/rocm/bin/hipcc") or shutil.which("make") is None:
        pytest.skip("hipcc / make unavailable")
    r = subprocess.run(["make", "-s", "-C", FUZZ, "parse_fuzz"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    return os.path.join(FUZZ, "parse_fuzz")


def _run(harness, iters, seed, files):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([harness, str(iters), str(seed)] + files, capture_output=True, text=True, timeout=600,
                       env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "0 unexpected return codes" in r.stdout, r.stdout


def test_parser_fuzz_small_streams(harness):
    files = sorted(f for f in glob.glob(os.path.join(ROOT, "tests", "golden", "*.bit"))
                   if not os.path.basename(f).startswith(("k4_", "hd_")))
    _run(harness, 60, 11, files)


def test_parser_fuzz_large_streams(harness):
    files = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "hd_*.bit")) +
                   glob.glob(os.path.join(ROOT, "tests", "golden", "k4_*.bit")))
    _run(harness, 3, 12, files)

# cif_hdbi_high encode time: HEAD library (var/lib_OLD.so) vs the working tree's.
set -o pipefail
cd /root/repo
O=gpurun_out/r04m
mkdir -p $O
T="tests/test_gpu_encoder_rd.py::test_device_encoder_hierarchical_b[cif_hdbi_high]"
THOR_AMD_LIB=var/lib_OLD.so timeout -k 10 400 python -u -m pytest -x -v --durations=3 --timeout 350 --timeout-method thread "$T" > $O/old.log 2>&1 || { echo OLD_FAIL; tail -30 $O/old.log; exit 1; }
grep -E "passed|failed|call" $O/old.log | tail -3
timeout -k 10 400 python -u -m pytest -x -v --durations=3 --timeout 350 --timeout-method thread "$T" > $O/new.log 2>&1 || { echo NEW_FAIL; tail -30 $O/new.log; exit 1; }
grep -E "passed|failed|call" $O/new.log | tail -3

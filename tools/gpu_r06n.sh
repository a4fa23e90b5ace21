# Round 6n: the full GPU suite + smoke at the final HEAD tree
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r06n
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 400 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log

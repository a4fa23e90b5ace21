# Round-3 closing evidence on the box: full GPU suite, smoke, the default bench, then the
# rocprofv3 kernel-trace + FETCH/WRITE PMC passes of the bench (tools/profile_round.sh).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 650 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread --durations 5 > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 200 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench.err; exit 1; }
cut -c1-400 gpurun_out/bench.json
bash tools/profile_round.sh || exit 1

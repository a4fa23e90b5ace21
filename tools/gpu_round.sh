set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1050 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
[ -n "$NO_BENCH" ] || timeout -k 10 200 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench.err; exit 1; }
[ -n "$NO_BENCH" ] || cat gpurun_out/bench.json

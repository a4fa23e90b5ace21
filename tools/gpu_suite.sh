# Round-end style GPU check on the box: the whole -m gpu suite, then smoke().
# Usage: bash tools/gpu_suite.sh TAG [pytest -k expression]
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
TAG=${1:-suite}
K=${2:-}
# heartbeat: the long speed-0 4K encoder tests run minutes per frame without output
( while sleep 30; do date +%T >> gpurun_out/${TAG}_heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --durations=15 --timeout 900 --timeout-method thread ${K:+-k "$K"} > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
grep -E "passed|failed" gpurun_out/${TAG}_pytest_gpu.log | tail -2
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -2 gpurun_out/${TAG}_smoke.log

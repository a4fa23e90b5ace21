# One long GPU test with its prints and a heartbeat (speed-0 4K encodes).
# Usage: bash tools/gpu_long.sh TAG TEST_NODEID [timeout_s]
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
TAG=$1; T=$2; TO=${3:-900}
( while sleep 30; do date +%T >> gpurun_out/${TAG}_heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
THOR_LONG_GPU_TESTS=1 timeout -k 10 $TO python -u -m pytest "$T" -x -v -s --timeout $((TO - 30)) --timeout-method thread > gpurun_out/${TAG}_long.log 2>&1 || { echo LONG_FAIL; tail -30 gpurun_out/${TAG}_long.log; exit 1; }
tail -5 gpurun_out/${TAG}_long.log

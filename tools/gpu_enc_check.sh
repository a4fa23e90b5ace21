# Encoder change check on the GPU box: the byte-exact device-encoder tests (all but the long
# 4K HDB16-high one), then the speed probe at 1 / 64 / 240 streams.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
TAG=${1:-ec}
( while sleep 30; do date +%T >> gpurun_out/${TAG}_heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 500 --timeout-method thread tests/test_gpu_encoder_rd.py tests/test_gpu_encoder.py -k "not 4k_hdb16_high" > gpurun_out/${TAG}_enc_pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/${TAG}_enc_pytest.log; exit 1; }
grep -E "passed|failed" gpurun_out/${TAG}_enc_pytest.log | tail -1
timeout -k 10 300 python3 tools/enc_speed.py --name k4_low --batch 1 64 240 2>&1 | tee gpurun_out/${TAG}_enc_speed.txt | grep -v "^frame"

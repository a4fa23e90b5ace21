set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_shard.py tests/test_gpu_streams.py > gpurun_out/r04i_pytest.log 2>&1 || { tail -40 gpurun_out/r04i_pytest.log; exit 1; }
grep -E "passed|failed" gpurun_out/r04i_pytest.log | tail -1
grep "boundary bytes" gpurun_out/r04i_pytest.log | head -12

# round 4: k_recon parity (streams, kernels, recon, shard) then A/B timing vs the HEAD library (var/lib_H.so)
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_streams.py tests/test_gpu_kernels.py tests/test_gpu_recon.py tests/test_gpu_shard.py > gpurun_out/r04a_pytest.log 2>&1 || { tail -40 gpurun_out/r04a_pytest.log; exit 1; }
tail -3 gpurun_out/r04a_pytest.log
VARS="${VARS:-A H A H}" PVARS="" bash tools/gpu_var.sh

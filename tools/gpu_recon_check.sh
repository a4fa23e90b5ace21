# k_recon change check on the GPU box: stream parity (every stage md5 vs the reference decoder),
# the kernel-level MC fuzz vs the oracle, the decode-from-bitstream and interpolated-reference
# streams, then the 8-frame launch timing.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
TAG=${1:-rc}
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_streams.py tests/test_gpu_kernels.py tests/test_gpu_recon.py tests/test_gpu_interp_frames.py tests/test_gpu_shard.py "tests/test_gpu_encoder_rd.py::test_gpu_decode_from_bitstream" > gpurun_out/${TAG}_pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
for S in ${STREAMS:-k4_low k4_med}; do
  echo "== $S"; timeout -k 10 120 python3 tools/recon_batch.py $S 8 10 --time || exit 1
done

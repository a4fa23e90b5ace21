# k_recon variant timing on the box: each variant library (var/lib_*.so, THOR_AMD_LIB) times the
# 8-frame 4K P launches of tools/recon_batch.py; then stream parity for the listed variants.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
for V in ${VARS:-A B B6 B7 B8}; do
  if [ $V = A ]; then LIBP=thor_amd/libthor_amd.so; else LIBP=var/lib_$V.so; fi
  for S in k4_low k4_med; do
    echo "== $V $S"; THOR_AMD_LIB=$LIBP timeout -k 10 120 python3 tools/recon_batch.py $S 8 10 --time > gpurun_out/var_time.log 2>&1 || { tail -8 gpurun_out/var_time.log; exit 1; }
    grep -E "avg" gpurun_out/var_time.log
  done
done
for V in ${PVARS-B B8}; do
  echo "== parity $V"
  THOR_AMD_LIB=var/lib_$V.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_streams.py tests/test_gpu_kernels.py > gpurun_out/var_${V}_pytest.log 2>&1 || { echo PYTEST_FAIL $V; tail -30 gpurun_out/var_${V}_pytest.log; exit 1; }
  tail -1 gpurun_out/var_${V}_pytest.log
done

# k_recon A/B: product library vs var/lib_NOAL.so (window chunks as 4-way-conflicting ds_write2_b32), then parity.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
for V in ${VARS:-NOAL A NOAL A}; do
  if [ $V = A ]; then LIBP=thor_amd/libthor_amd.so; else LIBP=var/lib_$V.so; fi
  for S in k4_low k4_med; do
    echo "== $V $S"; THOR_AMD_LIB=$LIBP timeout -k 10 120 python3 tools/recon_batch.py $S 8 10 --time > gpurun_out/var_time.log 2>&1 || { tail -8 gpurun_out/var_time.log; exit 1; }
    grep -E "avg" gpurun_out/var_time.log
  done
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_streams.py tests/test_gpu_recon.py > gpurun_out/r04q_pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/r04q_pytest.log; exit 1; }
tail -1 gpurun_out/r04q_pytest.log
if [ -n "$ENC_PROF" ]; then
  timeout -k 10 300 python3 tools/enc_profile.py --name k4_low --frames 1 --batch 1 > gpurun_out/r04q_enc_profile_b1.txt 2>&1 || { tail -20 gpurun_out/r04q_enc_profile_b1.txt; exit 1; }
  cat gpurun_out/r04q_enc_profile_b1.txt
fi

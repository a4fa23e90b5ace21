set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r07t
for v in cpw8 cpw16; do
  THOR_AMD_LIB=var/lib_$v.so timeout -k 10 120 python3 tools/recon_batch.py k4_low 8 10 --time > gpurun_out/r07t/recon_$v.txt 2>&1 || exit 1
  cat gpurun_out/r07t/recon_$v.txt
done
timeout -k 10 120 python3 tools/recon_batch.py k4_low 8 10 --time > gpurun_out/r07t/recon_cpw4.txt 2>&1 && cat gpurun_out/r07t/recon_cpw4.txt &&
THOR_LONG_GPU_TESTS=1 timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -s --timeout 650 --timeout-method thread -k "test_device_encoder_4k_hdb16_high_efficiency and not i_p16" > gpurun_out/r07t/cfg5_long.log 2>&1; rc=$?; tail -5 gpurun_out/r07t/cfg5_long.log; exit $rc

# Encoder A/B (240 streams of k4_low, I + P, bits checked): var/lib_PRE.so (HEAD) vs the working tree, then encoder parity tests.
set -o pipefail
cd /root/repo
O=gpurun_out/r04s
mkdir -p $O
for V in ${VARS:-PRE A PRE A}; do
  if [ $V = A ]; then LIBP=thor_amd/libthor_amd.so; else LIBP=var/lib_$V.so; fi
  THOR_AMD_LIB=$LIBP timeout -k 10 170 python3 tools/enc_speed.py --name k4_low --batch 240 --frames 2 > $O/enc_$V.txt 2>&1 || { tail -20 $O/enc_$V.txt; exit 1; }
  echo "$V $(tail -1 $O/enc_$V.txt)"
done
[ -n "$NO_TESTS" ] || timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_encoder_rd.py tests/test_gpu_encoder.py tests/test_gpu_dropin.py > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
[ -n "$NO_TESTS" ] || tail -1 $O/pytest.log

# Round 5f: k_recon without runtime divisions / tap-table address chains (decode parity + isolated timing),
# encoder A/B of the candidate-parallel ME (240 x 4K LDB-low I + P), config-5 I + P16 cycle profile
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r05f
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_streams.py tests/test_gpu_recon.py tests/test_synth_frames.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_dec.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest_dec.log; exit 1; }
tail -1 $OUT/pytest_dec.log
for s in k4_low k4_med k4_low; do timeout -k 10 120 python3 tools/recon_batch.py $s 8 10 --time > $OUT/time_$s.txt 2>&1 || { echo TIME_FAIL; tail $OUT/time_$s.txt; exit 1; }; cat $OUT/time_$s.txt; done
for V in PRE A PRE A; do
  if [ $V = A ]; then LIBP=thor_amd/libthor_amd.so; else LIBP=var/lib_$V.so; fi
  THOR_AMD_LIB=$LIBP timeout -k 10 170 python3 tools/enc_speed.py --name k4_low --batch 240 --frames 2 > $OUT/enc_$V.txt 2>&1 || { tail -20 $OUT/enc_$V.txt; exit 1; }
  echo "$V $(tail -1 $OUT/enc_$V.txt)"
done
timeout -k 10 400 python3 tools/enc_profile.py --name k4_hdbi_high --frames 17 --limit 2 > $OUT/cfg5_profile.txt 2>&1 || { tail -20 $OUT/cfg5_profile.txt; exit 1; }
cat $OUT/cfg5_profile.txt

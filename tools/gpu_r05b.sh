# Round 5b: encoder call-structure variants A/B (240 x 4K I + P), world-4 boundary shard test, config-5 I + P16 speed
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r05b
mkdir -p $OUT
for V in A B C D A B C D; do
  if [ $V = A ]; then LIBP=thor_amd/libthor_amd.so; else LIBP=var/lib_$V.so; fi
  THOR_AMD_LIB=$LIBP timeout -k 10 170 python3 tools/enc_speed.py --name k4_low --batch 240 --frames 2 > $OUT/enc_$V.txt 2>&1 || { tail -20 $OUT/enc_$V.txt; exit 1; }
  echo "$V $(tail -1 $OUT/enc_$V.txt)"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_shard.py -x -q -m gpu -k "boundary and k4_med" --timeout 200 --timeout-method thread > $OUT/pytest_shard.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest_shard.log; exit 1; }
tail -1 $OUT/pytest_shard.log
timeout -k 10 400 python3 tools/enc_speed.py --name k4_hdbi_high --batch 1 --frames 2 > $OUT/cfg5_b1.txt 2>&1 || { tail -20 $OUT/cfg5_b1.txt; exit 1; }
cat $OUT/cfg5_b1.txt

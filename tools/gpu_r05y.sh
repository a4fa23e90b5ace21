# Round 5y: each SB's original pixels and reference window pulled toward the L2 before its
# WPP wait (te_sb_prefetch): encoder parity, A/B vs no prefetch (NOPF2) on 240 x 4K, 8 frames
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r05y
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_encoder_rd.py tests/test_gpu_encoder.py -k "not hdb16 and not hierarchical" > $OUT/pytest_enc.log 2>&1 || { echo PYTEST_ENC_FAIL; tail -30 $OUT/pytest_enc.log; exit 1; }
tail -1 $OUT/pytest_enc.log
for V in NOPF2 A NOPF2 A; do
  if [ $V = A ]; then LIBP=thor_amd/libthor_amd.so; else LIBP=var/lib_$V.so; fi
  THOR_AMD_LIB=$LIBP timeout -k 10 170 python3 tools/enc_speed.py --name k4_low --batch 240 --frames 8 > $OUT/enc_$V.txt 2>&1 || { tail -20 $OUT/enc_$V.txt; exit 1; }
  echo "$V $(tail -1 $OUT/enc_$V.txt)"
done

# Round 6j: the 8x8 luma chain reuses the mode search's neighbour arrays and setup (LDS key): parity last, A/B vs HEAD (PRK), profile
# one worker per SB row): encoder parity incl. the stall / give-up and pipelined tests, A/B vs
# row workers (ROWS) on 240 x 4K x 8 frames, single-stream cycle profile (parity last: SB bit counts
# zeroed per batch, so a stalled launch packs nothing for the SBs it never coded)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r06j
mkdir -p $OUT
for V in PRK A PRK A; do
  if [ $V = A ]; then LIBP=thor_amd/libthor_amd.so; else LIBP=var/lib_$V.so; fi
  THOR_AMD_LIB=$LIBP timeout -k 10 170 python3 tools/enc_speed.py --name k4_low --batch 240 --frames 8 > $OUT/enc_$V.txt 2>&1 || { tail -20 $OUT/enc_$V.txt; exit 1; }
  echo "$V $(tail -1 $OUT/enc_$V.txt)"
done
timeout -k 10 300 python3 tools/enc_profile.py --name k4_low --frames 8 --limit 3 --batch 1 > $OUT/prof1.txt 2>&1 || { tail -20 $OUT/prof1.txt; exit 1; }
grep -E "frame|wait|sb " $OUT/prof1.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_encoder_rd.py tests/test_gpu_encoder.py -k "not hdb16 and not hierarchical" > $OUT/pytest_enc.log 2>&1 || { echo PYTEST_ENC_FAIL; tail -30 $OUT/pytest_enc.log; exit 1; }
tail -1 $OUT/pytest_enc.log

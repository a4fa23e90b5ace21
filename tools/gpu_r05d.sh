# Round 5d: candidate-parallel ME -- encoder parity (incl. config-5 I + P16), speed-0 timings
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r05d
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread tests/test_gpu_encoder_rd.py > $OUT/pytest_enc.log 2>&1 || { echo PYTEST_ENC_FAIL; tail -30 $OUT/pytest_enc.log; exit 1; }
grep -E "PASSED|FAILED|frame [0-9]+:|passed|failed" $OUT/pytest_enc.log | tail -40
timeout -k 10 300 python3 tools/enc_speed.py --name hd_high --batch 128 --frames 2 > $OUT/cfg3_b128.txt 2>&1 || { tail -20 $OUT/cfg3_b128.txt; exit 1; }
tail -1 $OUT/cfg3_b128.txt
timeout -k 10 170 python3 tools/enc_speed.py --name k4_low --batch 240 --frames 2 > $OUT/enc_k4low.txt 2>&1 || { tail -20 $OUT/enc_k4low.txt; exit 1; }
tail -1 $OUT/enc_k4low.txt

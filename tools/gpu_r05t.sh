# Round 5t: single-stream encoder cycle profile after the parallel coefficient coder (I + 2 P)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r05t
mkdir -p $OUT
timeout -k 10 300 python3 tools/enc_profile.py --name k4_low --frames 8 --limit 3 --batch 1 > $OUT/prof1.txt 2>&1 || { tail -20 $OUT/prof1.txt; exit 1; }
head -16 $OUT/prof1.txt

# Round 5o: encoder cycle profile, one stream and 16 streams, 4K LDB-low I + 2 P
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r05o
mkdir -p $OUT
timeout -k 10 300 python3 tools/enc_profile.py --name k4_low --frames 8 --limit 3 --batch 1 > $OUT/prof1.txt 2>&1 || { tail -20 $OUT/prof1.txt; exit 1; }
cat $OUT/prof1.txt
timeout -k 10 300 python3 tools/enc_speed.py --name k4_low --batch 1 --frames 8 > $OUT/speed1.txt 2>&1 || { tail -20 $OUT/speed1.txt; exit 1; }
tail -1 $OUT/speed1.txt

# Round 5n: encoder cycle profile at the bench's load (240 x 4K LDB-low, I + 2 P)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r05n
mkdir -p $OUT
timeout -k 10 400 python3 tools/enc_profile.py --name k4_low --frames 8 --limit 3 --batch 240 > $OUT/prof240.txt 2>&1 || { tail -20 $OUT/prof240.txt; exit 1; }
cat $OUT/prof240.txt

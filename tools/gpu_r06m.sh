# Round 6m: config-5 single-stream speed (4K HDB16 high efficiency, I + P16, one stream) at HEAD
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r06m
mkdir -p $OUT
timeout -k 10 600 python3 tools/enc_speed.py --name k4_hdbi_high --batch 1 --frames 17 --limit 2 > $OUT/cfg5_single.txt 2>&1 || { tail -20 $OUT/cfg5_single.txt; exit 1; }
tail -4 $OUT/cfg5_single.txt

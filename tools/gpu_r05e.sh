# Round 5e: A/B of the ME change on the 240-stream 4K LDB-low batch (I + P), config-5 I + P16 cycle profile
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r05e
mkdir -p $OUT
for V in PRE A PRE A; do
  if [ $V = A ]; then LIBP=thor_amd/libthor_amd.so; else LIBP=var/lib_$V.so; fi
  THOR_AMD_LIB=$LIBP timeout -k 10 170 python3 tools/enc_speed.py --name k4_low --batch 240 --frames 2 > $OUT/enc_$V.txt 2>&1 || { tail -20 $OUT/enc_$V.txt; exit 1; }
  echo "$V $(tail -1 $OUT/enc_$V.txt)"
done
timeout -k 10 400 python3 tools/enc_profile.py --name k4_hdbi_high --frames 17 --limit 2 > $OUT/cfg5_profile.txt 2>&1 || { tail -20 $OUT/cfg5_profile.txt; exit 1; }
cat $OUT/cfg5_profile.txt

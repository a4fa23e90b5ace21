# Round 5h: bisect the 4K I-frame slowdown: PRE (r05a) vs MESEQ (sequential device ME) vs MDI2 (two-loop
# I-frame mode decision) vs BOTH vs A (HEAD); 240 x 4K LDB-low I + P
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r05h
mkdir -p $OUT
for V in PRE MESEQ MDI2 BOTH A PRE MESEQ MDI2 BOTH A; do
  if [ $V = A ]; then LIBP=thor_amd/libthor_amd.so; else LIBP=var/lib_$V.so; fi
  THOR_AMD_LIB=$LIBP timeout -k 10 170 python3 tools/enc_speed.py --name k4_low --batch 240 --frames 2 > $OUT/enc_$V.txt 2>&1 || { tail -20 $OUT/enc_$V.txt; exit 1; }
  echo "$V $(tail -1 $OUT/enc_$V.txt)"
done

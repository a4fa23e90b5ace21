# Round 6c: one encoder worker per SIMD (WPE1: half the L2 working set of worker scratch and
# stacks; counters r06b: 43 % L2 miss rate on P frames at 240 streams) vs two (A)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r06c
mkdir -p $OUT
for V in WPE1 A WPE1 A; do
  if [ $V = A ]; then LIBP=thor_amd/libthor_amd.so; else LIBP=var/lib_$V.so; fi
  THOR_AMD_LIB=$LIBP timeout -k 10 170 python3 tools/enc_speed.py --name k4_low --batch 240 --frames 8 > $OUT/enc_$V.txt 2>&1 || { tail -20 $OUT/enc_$V.txt; exit 1; }
  echo "$V $(tail -1 $OUT/enc_$V.txt)"
done

# Round 5j: IPRA off (-mllvm -enable-ipra=false) vs HEAD vs PRE (r05a): 240 x 4K LDB-low I + P
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r05j
mkdir -p $OUT
for V in PRE A NOIPRA PRE A NOIPRA; do
  if [ $V = A ]; then LIBP=thor_amd/libthor_amd.so; else LIBP=var/lib_$V.so; fi
  THOR_AMD_LIB=$LIBP timeout -k 10 170 python3 tools/enc_speed.py --name k4_low --batch 240 --frames 2 > $OUT/enc_$V.txt 2>&1 || { tail -20 $OUT/enc_$V.txt; exit 1; }
  echo "$V $(tail -1 $OUT/enc_$V.txt)"
done

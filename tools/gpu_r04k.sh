# Encoder occupancy experiment: product lib (A) vs var/lib_E1 (pb / small levels in global)
# vs var/lib_E2 (the same at 2 waves per SIMD): 240 streams of k4_low, I + P frame, bits checked.
set -o pipefail
cd /root/repo
O=gpurun_out/r04k
mkdir -p $O
for V in ${VARS:-A E1 E2}; do
  if [ $V = A ]; then LIBP=thor_amd/libthor_amd.so; else LIBP=var/lib_$V.so; fi
  echo "== $V"
  THOR_AMD_LIB=$LIBP timeout -k 10 300 python3 tools/enc_speed.py --name k4_low --batch 240 --frames 2 > $O/enc_$V.txt 2>&1 || { tail -20 $O/enc_$V.txt; exit 1; }
  tail -2 $O/enc_$V.txt
done

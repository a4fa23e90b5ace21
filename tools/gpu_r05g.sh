# Round 5g: is the 4K I-frame slowdown of the ME build the scratch limit?  PRE / A with the default and a 4 GiB
# HSA_SCRATCH_SINGLE_LIMIT (240 x 4K LDB-low, I + P)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r05g
mkdir -p $OUT
for V in PRE A PREL AL PRE A PREL AL; do
  case $V in PRE|PREL) LIBP=var/lib_PRE.so;; *) LIBP=thor_amd/libthor_amd.so;; esac
  case $V in *L) LIM=4294967296;; *) LIM=;; esac
  HSA_SCRATCH_SINGLE_LIMIT=$LIM THOR_AMD_LIB=$LIBP timeout -k 10 170 python3 tools/enc_speed.py --name k4_low --batch 240 --frames 2 > $OUT/enc_$V.txt 2>&1 || { tail -20 $OUT/enc_$V.txt; exit 1; }
  echo "$V $(tail -1 $OUT/enc_$V.txt)"
done

# Round 5i: counters of the 240-stream 4K I frame, PRE (r05a) vs A (HEAD): instruction fetch, scratch, L2
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r05i
mkdir -p $OUT
for V in PRE A; do
  if [ $V = A ]; then LIBP=thor_amd/libthor_amd.so; else LIBP=$PWD/var/lib_$V.so; fi
  export THOR_AMD_LIB=$LIBP
  D="python3 tools/enc_speed.py --name k4_low --batch 240 --frames 1"
  timeout -s KILL 150 rocprofv3 --pmc SQ_IFETCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_VALU SQ_BUSY_CYCLES --kernel-trace -d $OUT/p1_$V -o run -- $D > $OUT/p1_$V.out 2> $OUT/p1_$V.err || { echo P1_FAIL; tail -20 $OUT/p1_$V.err; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --kernel-trace -d $OUT/p2_$V -o run -- $D > $OUT/p2_$V.out 2> $OUT/p2_$V.err || { echo P2_FAIL; tail -20 $OUT/p2_$V.err; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_SMEM SQ_IFETCH_LEVEL SQ_WAIT_INST_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_VMEM SQ_INSTS_LDS SQ_INSTS_FLAT --kernel-trace -d $OUT/p3_$V -o run -- $D > $OUT/p3_$V.out 2> $OUT/p3_$V.err || { echo P3_FAIL; tail -20 $OUT/p3_$V.err; exit 1; }
  echo "$V $(tail -1 $OUT/p1_$V.out)"
  python3 tools/sq_summary.py k_enc_rows $OUT/summary_$V.json $OUT/p1_$V $OUT/p2_$V $OUT/p3_$V && rm -rf $OUT/p1_$V $OUT/p2_$V $OUT/p3_$V
done

# Round 5c: config-5 (4K HDB16 high efficiency) I + P16 per-stage cycle profile (one stream) and at K streams;
# SQ counters of the 240-stream 4K I frame (VMEM writes after the call-frame cuts)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r05c
mkdir -p $OUT
timeout -k 10 400 python3 tools/enc_profile.py --name k4_hdbi_high --frames 17 --limit 2 > $OUT/cfg5_profile.txt 2>&1 || { tail -20 $OUT/cfg5_profile.txt; exit 1; }
cat $OUT/cfg5_profile.txt
timeout -k 10 400 python3 tools/enc_speed.py --name k4_hdbi_high --batch 32 --frames 17 --limit 2 > $OUT/cfg5_b32.txt 2>&1 || { tail -20 $OUT/cfg5_b32.txt; exit 1; }
tail -1 $OUT/cfg5_b32.txt
D="python3 tools/enc_speed.py --name k4_low --batch 240 --frames 1"
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS --kernel-trace -d $OUT/sq2 -o run -- $D > $OUT/sq2.out 2> $OUT/sq2.err || { echo SQ2_FAIL; tail -20 $OUT/sq2.err; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace -d $OUT/sq1 -o run -- $D > $OUT/sq1.out 2> $OUT/sq1.err || { echo SQ1_FAIL; tail -20 $OUT/sq1.err; exit 1; }
tail -1 $OUT/sq1.out
python3 tools/sq_summary.py k_enc_rows $OUT/summary.json $OUT/sq1 $OUT/sq2 && rm -rf $OUT/sq1 $OUT/sq2
cat $OUT/summary.json

# SQ counters of the encoder's I frame at the bench's load (240 streams of k4_low, two workers per SIMD).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r04u
mkdir -p $O
D="python3 tools/enc_speed.py --name k4_low --batch 240 --frames 1"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace -d $O/sq1 -o run -- $D > $O/sq1.out 2> $O/sq1.err || { echo SQ1_FAIL; tail -20 $O/sq1.err; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS --kernel-trace -d $O/sq2 -o run -- $D > $O/sq2.out 2> $O/sq2.err || { echo SQ2_FAIL; tail -20 $O/sq2.err; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INSTS_BRANCH SQ_INSTS_FLAT SQ_INST_CYCLES_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_IFETCH --kernel-trace -d $O/sq3 -o run -- $D > $O/sq3.out 2> $O/sq3.err || { echo SQ3_FAIL; tail -20 $O/sq3.err; exit 1; }
tail -1 $O/sq1.out
python3 tools/sq_summary.py k_enc_rows $O/summary.json $O/sq1 $O/sq2 $O/sq3 && rm -rf $O/sq1 $O/sq2 $O/sq3

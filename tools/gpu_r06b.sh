# Round 6b: SQ / SQC / TCC counters of the encoder's RD kernel at 240 x 4K streams, I then P
# frame batch (k_enc_rows per dispatch), to see what bounds the P frames at full occupancy
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r06b
mkdir -p $O
D="python3 tools/enc_speed.py --name k4_low --batch 240 --frames 2"
timeout -k 10 200 $D > $O/enc.txt 2>&1 || { tail -20 $O/enc.txt; exit 1; }
tail -1 $O/enc.txt
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace -d $O/sq1 -o run -- $D > /dev/null 2> $O/sq1.err || { echo SQ1_FAIL; tail -20 $O/sq1.err; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_IFETCH --kernel-trace -d $O/sq2 -o run -- $D > /dev/null 2> $O/sq2.err || { echo SQ2_FAIL; tail -20 $O/sq2.err; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $O/tcc -o run -- $D > /dev/null 2> $O/tcc.err || { echo TCC_FAIL; tail -20 $O/tcc.err; exit 1; }
python3 tools/sq_summary.py k_enc_rows $O/counters.json $O/sq1 $O/sq2 $O/tcc > /dev/null
timeout -s KILL 150 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_MISSES --kernel-trace -d $O/sqc -o run -- $D > /dev/null 2> $O/sqc.err || { echo SQC_FAIL; tail -5 $O/sqc.err; exit 0; }
python3 tools/sq_summary.py k_enc_rows $O/counters.json $O/sq1 $O/sq2 $O/tcc $O/sqc > /dev/null
python3 -c "import json; d=json.load(open('$O/counters.json'))['per_dispatch']; [print(k, ['%.4g' % x for x in v]) for k, v in sorted(d.items())]"

# Round-4 GPU pass: shard + streams parity (boundary exchange), the config-3
# encoder leg and the drop-in leg, then SQ counters of the encoder's I frame.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r04j
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_shard.py tests/test_gpu_streams.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
grep "boundary bytes" $O/pytest.log | head -12
timeout -k 10 300 python3 bench.py --drop-in hd_low > $O/dropin.json 2> $O/dropin.err || { tail -20 $O/dropin.err; exit 1; }
cat $O/dropin.json
timeout -k 10 300 python3 tools/enc_speed.py --name hd_low --batch 64 --frames 1 > $O/enc_i.txt 2>&1 || { tail -20 $O/enc_i.txt; exit 1; }
tail -3 $O/enc_i.txt
D="python3 tools/enc_speed.py --name hd_low --batch 64 --frames 1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace -d $O/sq1 -o run -- $D > /dev/null 2> $O/sq1.err || { echo SQ1_FAIL; tail -20 $O/sq1.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --kernel-trace -d $O/sq2 -o run -- $D > /dev/null 2> $O/sq2.err || { echo SQ2_FAIL; tail -20 $O/sq2.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM_RD SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_INSTS_FLAT SQ_INSTS_SMEM --kernel-trace -d $O/sq3 -o run -- $D > /dev/null 2> $O/sq3.err || echo SQ3_FAIL
find $O -name '*counter_collection.csv' | head
